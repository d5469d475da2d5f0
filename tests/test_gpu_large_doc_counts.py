"""k_chunks counts the columns of a large document chunk (> 16 KB, at most two in a wave) one lane per
column, the six chains of dependent reads side by side (am_kernels.hip, the deferred counts); a wave
of three or more large documents keeps the lane-per-chunk count (rle_count_sum). The two must agree:
same counts (the merged bytes), same status and arguments for corrupted columns (the first failing
column in the order actor, depsNum, idCtr, succNum, keyStr, message, as counting them one after
another reports it). Inputs: 100k-op text histories saved by the oracle, their DEFLATEd columns
inflated by the engine's own stage (am_stage_document), checksums recomputed after each change."""
import random

import pytest

pytestmark = pytest.mark.gpu

# column ids counted by k_chunks (decodeDocumentHeader's column tables, columnar.js:1006-1038)
COUNTED = {"chg": (0x01, 0x40, 0x35), "ops": (0x23, 0x80, 0x15)}


def _columns(chunk):
    """[(table, column id, absolute offset, length)] of a saved (uncompressed) document chunk."""
    pos = [9]

    def u():
        v = sh = 0
        while True:
            b = chunk[pos[0]]
            pos[0] += 1
            v |= (b & 0x7F) << sh
            sh += 7
            if not b & 0x80:
                return v
    u()
    for _ in range(u()):
        n = u()  # (pos[0] += u() would read pos before u() moves it)
        pos[0] += n
    n = u()
    pos[0] += 32 * n
    tabs = []
    for t in ("chg", "ops"):
        tabs += [(t, u(), u()) for _ in range(u())]
    out, at = [], pos[0]
    for t, cid, n in tabs:
        out.append((t, cid, at, n))
        at += n
    return out


def _big_doc():
    import oracle_ffi as O
    import workload as W
    from automerge_amd import _native as N
    arena, chunks, docs, _ = W.text(21, 1, 1000, 100, 0)
    _, chg = W.doc_chunks(arena, chunks, docs, 0)
    d = O.Doc.init()
    d.apply(chg)
    from test_gpu_inflate import _rechecksum
    staged, _ = N.stage_document(d.save())  # keeps the checksum of the DEFLATEd form: recomputed
    assert len(staged) > 64 * 1024
    return _rechecksum(staged)


def _statuses(docs_bytes, copies):
    """Loads every document as the base of a batch document of its own, in a wave of its own (k_chunks:
    one thread per chunk, 64 chunks per wave): `copies` more copies of the first document follow it
    (copies = 2: three large documents in the wave, the lane-per-chunk count), then small documents
    (one change each) fill the wave."""
    import workload as W
    from automerge_amd.batch import Batch, pack
    a2, c2, d2, _ = W.c2(0, 64)
    fill = [(None, [W.doc_chunks(a2, c2, d2, i)[1][0]]) for i in range(64)]
    items, first = [], []
    for d in docs_bytes:
        first.append(len(items))
        items.append((d, []))
        items += [(docs_bytes[0], [])] * copies
        items += fill[:63 - copies]
    b = Batch()
    b.stage(*pack(items))
    b.run()
    b.sync()
    r = b.results()
    assert all(int(r[k]["status"]) == 0 for k in range(len(items)) if items[k][0] is None)
    return [(int(r[k]["status"]), int(r[k]["arg0"]), int(r[k]["arg1"]), int(r[k]["out_len"])) for k in first]


def test_large_document_counts_match_the_lane_per_chunk_count():
    from test_gpu_inflate import _rechecksum
    base = _big_doc()
    cols = [c for c in _columns(base) if c[1] in COUNTED[c[0]] and c[3] > 0]
    assert len(cols) >= 4
    rng = random.Random(7)
    docs = [base]
    for _ in range(24):
        t, cid, at, n = rng.choice(cols)
        c = bytearray(base)
        q = at + rng.randrange(n)
        c[q] = rng.choice([0x80 | c[q], c[q] ^ 0x40, 0x7F, 0xFF, 0x00])
        if rng.random() < 0.3:
            c[at + n - 1] |= 0x80  # an incomplete LEB128 at the column's end
        docs.append(_rechecksum(bytes(c)))
    side = _statuses(docs, 0)   # alone in their waves: the side-by-side column counts
    lane = _statuses(docs, 2)   # three large documents per wave: the lane-per-chunk count
    assert side[0][0] == 0 and side[0] == lane[0]
    assert side == lane
    assert sum(1 for s in side[1:] if s[0]) >= 8  # most corruptions fail the document
