"""Packed pipeline descriptors (am_pipe_submit_packed): automerge_amd.pipe.pack over the bench's
batches, and a numpy restatement of the device expansion (k_unpack_counts / k_unpack_write in
am_kernels.hip) that gives back the full am_chunk_desc / am_doc_desc arrays."""
import numpy as np


def _expand(clen, spans):
    off = np.concatenate([[0], np.cumsum(clen.astype(np.uint64))[:-1]]).astype(np.uint64)
    cnt = spans["chg_count"].astype(np.int64) + spans["has_base"].astype(np.int64)
    first = np.concatenate([[0], np.cumsum(cnt)[:-1]])
    base = np.where(spans["has_base"] != 0, first, -1)
    return off, base, first + spans["has_base"], spans["chg_count"]


def test_pack_round_trip():
    import bench
    import workload
    from automerge_amd import pipe
    from automerge_amd.batch import WANT_DIFF
    for gen in (workload.c4, workload.c2):
        arena, chunks, docs, _ = gen(7, 600, nthreads=2)
        docs = docs.copy()
        docs["flags"] |= WANT_DIFF
        for a, c, d in bench.split_batches(arena, chunks, docs, 250):
            k = pipe.pack(c, d)
            assert k is not None
            clen, spans = k
            assert clen.dtype == np.uint32 and spans.dtype == pipe.SPAN_DT and spans.itemsize == 8
            off, base, beg, cnt = _expand(clen, spans)
            assert (off == c["off"]).all() and (clen == c["len"]).all()
            assert (base == d["base_chunk"]).all() and (beg == d["chg_begin"]).all() and (cnt == d["chg_count"]).all()
            assert (spans["flags"] == d["flags"]).all()
            assert int(off[-1]) + int(clen[-1]) == len(a)


def test_pack_refuses_other_shapes():
    import workload
    from automerge_amd import pipe
    arena, chunks, docs, _ = workload.c4(0, 20, nthreads=1)
    c = chunks.copy()
    c["off"][3:] += 16  # a gap in the arena
    assert pipe.pack(c, docs) is None
    d = docs.copy()
    d["flags"][2] |= pipe.DOC_META
    assert pipe.pack(chunks, d) is None
    d = docs.copy()
    d["known_count"][1] = 1
    assert pipe.pack(chunks, d) is None
    d = docs[::-1].copy()  # documents out of chunk order
    assert pipe.pack(chunks, d) is None
