"""Pipelined batches (am_pipe_*): the same documents through the pipeline and through am_batch_*
give the same merged documents and patch logs; batches larger than the pipeline's capacities are
refused; documents that outgrow the output arenas report AM_U_CAPACITY instead of a truncated
result."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _parts(kind, first, n, batch, flags):
    import bench
    import workload
    arena, chunks, docs, _ = getattr(workload, kind)(first, n)
    docs = docs.copy()
    docs["flags"] |= flags
    return (arena, chunks, docs), bench.split_batches(arena, chunks, docs, batch)


@pytest.mark.parametrize("kind,packed", [("c4", False), ("c2", False), ("c4", True), ("c2", True)])
def test_pipeline_equals_batch_path(kind, packed):
    from automerge_amd import pipe
    from automerge_amd.batch import WANT_DIFF, Batch
    whole, parts = _parts(kind, 40, 2500, 700, WANT_DIFF)
    ref = Batch()
    ref.stage(*whole)
    ref.run()
    ref.sync()
    rr = ref.results()
    kinfo = ref.kernel_info()
    ws = int(ref.workspace_bytes())
    pl = pipe.Pipeline(max(len(p[0]) for p in parts), max(len(p[1]) for p in parts), 700, ws, 1 << 20, 4 << 20,
                       kinfo["k_doc_fast_lds_per_doc"], slots=2)
    outs = []
    for _ in range(2):  # the second pass reuses every slot
        keep = []
        for a, c, d in parts:
            s = pipe.Pinned(len(d) * pipe.SUMMARY_DT.itemsize)
            po, pp = pipe.Pinned(1 << 20), pipe.Pinned(4 << 20)
            if packed:
                cl, sp = pipe.pack(c, d)
                pa, pc, pd = pipe.pinned_copy(a), pipe.pinned_copy(cl), pipe.pinned_copy(sp)
                pl.submit_packed(pa.arr, pc.arr, pd.arr, s.view(pipe.SUMMARY_DT, len(d)), po.u8, pp.u8)
            else:
                pa, pc, pd = pipe.pinned_copy(a), pipe.pinned_copy(c), pipe.pinned_copy(d)
                pl.submit(pa.arr, pc.arr, pd.arr, s.view(pipe.SUMMARY_DT, len(d)), po.u8, pp.u8)
            keep.append((pa, pc, pd, s, po, pp, len(d)))
        pl.drain(len(parts))
        outs.append(keep)
    for keep in outs:
        i = 0
        for pa, pc, pd, s, po, pp, n in keep:
            sm = s.view(pipe.SUMMARY_DT, n)
            for j in range(n):
                assert int(sm[j]["status"]) == int(rr[i]["status"]) == 0
                o = bytes(po.u8[int(sm[j]["out_off"]):int(sm[j]["out_off"]) + int(sm[j]["out_len"])])
                assert o == ref.doc_output(i, rr[i]), i
                p = bytes(pp.u8[int(sm[j]["patch_off"]):int(sm[j]["patch_off"]) + int(sm[j]["patch_len"])])
                assert p == ref.doc_patch(i), i
                assert int(sm[j]["nqueued"]) == int(rr[i]["nqueued"])
                i += 1
        assert i == 2500
    ms_comp, ms_doc, nb = pl.times()
    assert nb == 2 * len(parts) and ms_comp > ms_doc > 0


def test_pipeline_capacities():
    from automerge_amd import _native as N
    from automerge_amd import pipe
    from automerge_amd.batch import WANT_DIFF, Batch
    _, parts = _parts("c4", 0, 300, 300, WANT_DIFF)
    a, c, d = parts[0]
    ref = Batch()
    ref.stage(a, c, d)
    kinfo = ref.kernel_info()
    ws = int(ref.workspace_bytes())
    # a batch above the capacities is refused
    small = pipe.Pipeline(len(a), len(c), 100, ws, 1 << 20, 1 << 20, kinfo["k_doc_fast_lds_per_doc"], slots=2)
    pa, pc, pd = pipe.pinned_copy(a), pipe.pinned_copy(c), pipe.pinned_copy(d)
    s = pipe.Pinned(len(d) * pipe.SUMMARY_DT.itemsize)
    po, pp = pipe.Pinned(1 << 20), pipe.Pinned(1 << 20)
    with pytest.raises(N.AutomergeError, match="capacities"):
        small.submit(pa.arr, pc.arr, pd.arr, s.view(pipe.SUMMARY_DT, len(d)), po.u8, pp.u8)
    # output arenas that hold only part of the batch: the rest report AM_U_CAPACITY
    tight = pipe.Pipeline(len(a), len(c), len(d), ws, 100 * 1024, 1 << 20, kinfo["k_doc_fast_lds_per_doc"], slots=2)
    sm = s.view(pipe.SUMMARY_DT, len(d))
    tight.submit(pa.arr, pc.arr, pd.arr, sm, po.u8, pp.u8)
    tight.drain(1)
    st = sm["status"]
    assert (st == 0).sum() > 50 and (st == 106).sum() > 50 and set(np.unique(st)) <= {0, 106}
    # too little workspace (half the scanned plans, no overflow room): the documents beyond it report
    # AM_U_CAPACITY, the others merge
    short = pipe.Pipeline(len(a), len(c), len(d), int(ref.workspace_plan()) // 2, 1 << 20, 1 << 20,
                          kinfo["k_doc_fast_lds_per_doc"], slots=2)
    short.submit(pa.arr, pc.arr, pd.arr, sm, po.u8, pp.u8)
    short.drain(1)
    st = sm["status"]
    assert (st == 0).sum() > 50 and (st == 106).sum() > 50
    # caller buffers smaller than the device arenas: the documents past them report AM_U_CAPACITY,
    # and every document reported as merged lies inside the buffers with the batch path's bytes
    roomy = pipe.Pipeline(len(a), len(c), len(d), ws, 1 << 20, 1 << 20, kinfo["k_doc_fast_lds_per_doc"], slots=2)
    small_out, small_patch = pipe.Pinned(64 * 1024), pipe.Pinned(24 * 1024)
    roomy.submit(pa.arr, pc.arr, pd.arr, sm, small_out.u8, small_patch.u8)
    roomy.drain(1)
    st = sm["status"]
    assert (st == 0).sum() > 20 and (st == 106).sum() > 20 and set(np.unique(st)) <= {0, 106}
    ref.run()
    ref.sync()
    res = ref.results()
    for i in np.flatnonzero(st == 0):
        o, n = int(sm["out_off"][i]), int(sm["out_len"][i])
        assert o + n <= 64 * 1024 and int(sm["patch_off"][i]) + int(sm["patch_len"][i]) <= 24 * 1024
        assert bytes(small_out.u8[o:o + n]) == ref.doc_output(int(i), res[i])


def test_packed_descriptors_that_lie():
    """A packed chunk length that disagrees with the arena shifts every later chunk: those documents
    fail their container checks (per-document errors, no out-of-bounds read), the earlier ones merge."""
    from automerge_amd import pipe
    from automerge_amd.batch import WANT_DIFF, Batch
    _, parts = _parts("c4", 0, 200, 200, WANT_DIFF)
    a, c, d = parts[0]
    ref = Batch()
    ref.stage(a, c, d)
    kinfo = ref.kernel_info()
    ws = int(ref.workspace_bytes())
    pl = pipe.Pipeline(len(a), len(c), len(d), ws, 1 << 20, 1 << 20, kinfo["k_doc_fast_lds_per_doc"], slots=2)
    cl, sp = pipe.pack(c, d)
    bad = 13 * 100 + 5  # a change chunk of document 100
    cl = cl.copy()
    cl[bad] += 7
    sp = sp.copy()
    sp["chg_count"][-1] += 50  # the last document names chunks past the batch
    s = pipe.Pinned(len(d) * pipe.SUMMARY_DT.itemsize)
    po, pp = pipe.Pinned(1 << 20), pipe.Pinned(1 << 20)
    sm = s.view(pipe.SUMMARY_DT, len(d))
    pa, pc, pd = pipe.pinned_copy(a), pipe.pinned_copy(cl), pipe.pinned_copy(sp)
    pl.submit_packed(pa.arr, pc.arr, pd.arr, sm, po.u8, pp.u8)
    pl.drain(1)
    st = sm["status"]
    assert (st[:100] == 0).all()
    assert (st[100:] != 0).all()


def test_pipeline_fast_kernel_fallback_uses_the_overflow():
    """Documents k_doc_fast gives up on (here: a change whose checksum is wrong) lose their compact
    workspace plan: k_rest re-plans them in the overflow room past the batch's plans, where k_doc
    reports their error exactly as the batch path does. Without overflow room they report
    AM_U_CAPACITY; every other document merges either way."""
    from automerge_amd import pipe
    from automerge_amd.batch import WANT_DIFF, Batch
    (a, c, d), _ = _parts("c4", 0, 300, 300, WANT_DIFF)
    a = a.copy()
    bad = [5, 77, 150, 299]
    for i in bad:  # the last byte of the document's second change: its SHA-256 no longer matches
        ch = c[int(d[i]["chg_begin"]) + 1]
        a[int(ch["off"]) + int(ch["len"]) - 1] ^= 0x5A
    ref = Batch()
    ref.stage(a, c, d)
    ref.run()
    ref.sync()
    rr = ref.results()
    assert all(int(rr[i]["status"]) != 0 for i in bad) and (rr["status"] != 0).sum() == len(bad)
    kinfo = ref.kernel_info()
    plan = int(ref.workspace_plan())
    assert plan < int(ref.workspace_bytes())  # the compact plans leave room for the overflow reserve
    pa, pc, pd = pipe.pinned_copy(a), pipe.pinned_copy(c), pipe.pinned_copy(d)
    for room, want_bad in ((plan // 8 + (8 << 20), None), (0, 106)):
        pl = pipe.Pipeline(len(a), len(c), len(d), plan + room, 1 << 20, 4 << 20, kinfo["k_doc_fast_lds_per_doc"], slots=2)
        s = pipe.Pinned(len(d) * pipe.SUMMARY_DT.itemsize)
        po, pp = pipe.Pinned(1 << 20), pipe.Pinned(4 << 20)
        sm = s.view(pipe.SUMMARY_DT, len(d))
        pl.submit(pa.arr, pc.arr, pd.arr, sm, po.u8, pp.u8)
        pl.drain(1)
        for j in range(len(d)):
            if j in bad:
                assert int(sm[j]["status"]) == (int(rr[j]["status"]) if want_bad is None else want_bad), j
                continue
            assert int(sm[j]["status"]) == 0, j
            o = bytes(po.u8[int(sm[j]["out_off"]):int(sm[j]["out_off"]) + int(sm[j]["out_len"])])
            assert o == ref.doc_output(j, rr[j]), j
