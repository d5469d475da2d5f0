"""DEFLATE inflate on the GPU (automerge_amd/csrc/am_inflate.hip) against
zlib's raw inflate (the reference calls pako.inflateRaw, columnar.js:816 and :1064; inflate is
unambiguous, so any conforming decoder must return the same bytes).

Streams cover every block type: stored (level 0), fixed Huffman (Z_FIXED), dynamic Huffman (levels
1-9, Z_HUFFMAN_ONLY, Z_RLE), multi-block streams, back-references across the 32 KiB window, empty
input, plus malformed streams that must be rejected. The change-chunk path (type 2 chunks inflated
in the batch stage) is covered end to end by tests/test_gpu_text.py and tests/test_gpu_parity.py."""
import random
import zlib

import pytest

pytestmark = pytest.mark.gpu


def _deflate(data, level=6, strategy=zlib.Z_DEFAULT_STRATEGY, mem=8):
    c = zlib.compressobj(level, zlib.DEFLATED, -15, mem, strategy)
    return c.compress(data) + c.flush()


def _corpus(rng):
    out = [b"", b"a", bytes(range(256)), b"abc" * 1000]
    for n in (10, 100, 255, 256, 1000, 5000, 40000, 150000):
        text = bytes(rng.choice(b"abcdefghij      ") for _ in range(n))
        noise = bytes(rng.getrandbits(8) for _ in range(n))
        mixed = bytes(text[i] if (i // 64) % 3 else noise[i] for i in range(n))
        out += [text, noise, mixed]
    return out


def test_inflate_matches_zlib():
    from automerge_amd import _native as N
    rng = random.Random(1234)
    data, streams = [], []
    for d in _corpus(rng):
        for level, strat in [(6, zlib.Z_DEFAULT_STRATEGY), (0, zlib.Z_DEFAULT_STRATEGY), (1, zlib.Z_DEFAULT_STRATEGY),
                             (9, zlib.Z_DEFAULT_STRATEGY), (6, zlib.Z_FIXED), (6, zlib.Z_HUFFMAN_ONLY), (6, zlib.Z_RLE)]:
            data.append(d)
            streams.append(_deflate(d, level, strat))
    # a stream of many small blocks (sync flushes between pieces)
    c = zlib.compressobj(6, zlib.DEFLATED, -15)
    pieces = [bytes(rng.choice(b"xyz ") for _ in range(rng.randint(0, 300))) for _ in range(50)]
    s = b""
    for p in pieces:
        s += c.compress(p) + c.flush(zlib.Z_SYNC_FLUSH)
    s += c.flush()
    data.append(b"".join(pieces))
    streams.append(s)
    got = N.inflate_raw(streams)
    for i, (d, z, g) in enumerate(zip(data, streams, got)):
        assert zlib.decompress(z, -15) == d
        assert g == d, (i, len(d), None if g is None else len(g))


def test_inflate_rejects_malformed():
    from automerge_amd import _native as N
    good = _deflate(b"hello hello hello world" * 20)
    bad = [
        b"\x07",                            # block type 3 (reserved)
        good[: len(good) // 2],             # truncated
        b"\x01\x05\x00\x00\x00abc",         # stored block with LEN != ~NLEN
        b"\x01\x05\x00\xfa\xffab",          # stored block longer than the input
        bytes.fromhex("030200"),            # fixed block: a match at output position 0 (distance too far back)
    ]
    got = N.inflate_raw(bad + [good])
    assert got[:-1] == [None] * len(bad)
    assert got[-1] == zlib.decompress(good, -15)


def test_deflated_change_chunks_inflate_in_the_batch_stage():
    """Compressed change chunks (columnar.js:738 writes them for changes >= 256 B) go through the
    batch as they are: the stage inflates them on the GPU, the hashes and merged bytes equal the
    oracle's (which inflates with zlib)."""
    import oracle_ffi as O
    import workload as W
    from automerge_amd.batch import Batch
    arena, chunks, docs, _ = W.text(5, 6, 30, 60, 4)
    b = Batch()
    b.stage(arena, chunks, docs)
    ninf, nbytes, ms = b.inflate_info()
    nz = sum(1 for c in chunks if arena[int(c["off"]) + 8] == 2)
    assert nz > 100 and ninf == nz
    b.run()
    b.sync()
    r = b.results()
    hashes, _, _ = b.chunk_results()
    k = 0
    for i in range(len(docs)):
        _, chg = W.doc_chunks(arena, chunks, docs, i)
        ref = O.Doc.init()
        ref.apply(chg)
        assert int(r[i]["status"]) == 0
        assert b.doc_save(i) == ref.save()
        for c in chg:
            assert hashes[k].tobytes().hex() == O.change_meta(c)["hash"]
            k += 1


def test_stage_documents_batch_equals_per_document_stage():
    """am_stage_documents (one GPU checksum batch + one inflate batch for every DEFLATEd column of
    every document, inflateColumn columnar.js:1062-1068) stages each saved document exactly as
    am_stage_document does one at a time; a corrupted checksum fails that document only."""
    import oracle_ffi as O
    import workload as W
    from automerge_amd import _native as N
    arena, chunks, docs, _ = W.text(7, 5, 40, 30, 4)
    saved = []
    for i in range(len(docs)):
        _, chg = W.doc_chunks(arena, chunks, docs, i)
        d = O.Doc.init()
        d.apply(chg)
        saved.append(d.save())
    saved.append(O.Doc.init().save())
    one = [N.stage_document(s) for s in saved]
    assert sum(1 for s, (o, _) in zip(saved, one) if o != s) >= len(docs)  # columns were DEFLATEd
    assert N.stage_documents(saved) == one
    bad = bytearray(saved[1])
    bad[5] ^= 0xFF  # checksum byte
    with pytest.raises(N.AutomergeError):
        N.stage_documents([saved[0], bytes(bad), saved[2]])
    codes = (N.C.c_uint32 * 3)()
    msgs = (N.C.c_void_p * 3)()
    outs = (N.u8p * 3)()
    olens = (N.C.c_size_t * 3)()
    ver = (N.C.c_uint8 * 3)()
    datas = [saved[0], bytes(bad), saved[2]]
    nfail = N.lib.am_stage_documents(N.engine(), 3, (N.C.c_char_p * 3)(*datas), (N.C.c_size_t * 3)(*map(len, datas)),
                                     outs, olens, ver, codes, msgs)
    errs = N.batch_errors(3, codes, msgs)
    assert nfail == 1 and errs[0] is None and errs[2] is None and errs[1] is not None
    assert N.C.string_at(outs[0], olens[0]) == one[0][0] and N.C.string_at(outs[2], olens[2]) == one[2][0]
    for i in (0, 2):
        N.lib.am_free(outs[i])


def _first_deflated_column(chunk):
    """Offset of the first data byte of the first DEFLATEd column of a saved document chunk
    (decodeDocumentHeader, columnar.js:1006-1038)."""
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
    u()  # chunk length
    for _ in range(u()):  # actors
        n = u()
        pos[0] += n
    n = u()  # heads
    pos[0] += 32 * n
    cols = []
    for _ in range(2):
        for _ in range(u()):
            cols.append((u(), u()))
    at = pos[0]
    for cid, n in cols:
        if cid & 8 and n:
            return at
        at += n
    raise AssertionError("no DEFLATEd column")


def _rechecksum(chunk):
    """A container chunk with its checksum recomputed (columnar.js:659-686: SHA-256 of the bytes after
    the checksum, first 4 bytes)."""
    import hashlib
    c = bytearray(chunk)
    c[4:8] = hashlib.sha256(bytes(c[8:])).digest()[:4]
    return bytes(c)


def test_deflated_documents_load_in_the_batch_stage():
    """Saved documents with DEFLATEd columns (columnar.js:1052-1059) go into a batch as they are:
    the stage checks their checksum on the GPU and rebuilds them with every column inflated
    (inflateColumn, columnar.js:1062-1068), so Backend.load + applyChanges needs no host staging.
    Merged bytes and heads equal the oracle's and the host-staged path's; a wrong checksum fails its
    document with the checksum error, a column that does not inflate with AM_E_INFLATE."""
    import oracle_ffi as O
    import workload as W
    from automerge_amd import _native as N
    from automerge_amd.batch import Batch
    arena, chunks, docs, _ = W.text(11, 8, 60, 40, 4)
    items = []
    for i in range(len(docs)):
        _, chg = W.doc_chunks(arena, chunks, docs, i)
        d = O.Doc.init()
        d.apply(chg[:30])
        items.append((d.save(), chg[30:]))
    hs = [N.stage_document(s) for s, _ in items]  # the host stage: (chunk, checksum verified)
    staged = [h[0] for h in hs]
    assert sum(1 for (s, _), t in zip(items, staged) if s != t) >= len(docs) - 1  # DEFLATEd columns
    # a wrong checksum; a column that does not inflate (valid checksum)
    bad_sum = bytearray(items[2][0])
    bad_sum[5] ^= 0xFF
    raw = bytearray(items[3][0])
    raw[_first_deflated_column(raw)] = 0x07  # BFINAL + reserved block type 3: never a valid stream
    bad_z = _rechecksum(raw)
    cases = items + [(bytes(bad_sum), items[2][1]), (bad_z, items[3][1])]
    b = Batch()
    b.stage_docs(cases)
    ninf, _, _ = b.inflate_info()
    nzc = sum(1 for _, ch in cases for c in ch if c[8] == 2)
    assert ninf > nzc + len(docs)  # compressed changes + the documents' DEFLATEd columns
    b.run()
    b.sync()
    r = b.results()
    from automerge_amd.batch import pack
    ra, rc, rd = pack([(t, ch) for t, (_, ch) in zip(staged, items)])
    rc["flags"][rd["base_chunk"].astype(int)] = [1 if h[1] else 0 for h in hs]  # host-staged: checksum verified
    ref = Batch()
    ref.stage(ra, rc, rd)
    ref.run()
    ref.sync()
    rr = ref.results()
    for i, (s, ch) in enumerate(items):
        assert int(r[i]["status"]) == 0, (i, int(r[i]["status"]))
        want = O.Doc.load(s)
        want.apply(ch)
        assert b.doc_save(i) == want.save() == ref.doc_save(i), i
        assert b.doc_heads(i, int(r[i]["nheads"])) == want.heads(), i
        assert int(rr[i]["status"]) == 0
    AM_E_CHECKSUM, AM_E_INFLATE = 2, 35
    assert int(r[len(items)]["status"]) == AM_E_CHECKSUM
    assert int(r[len(items) + 1]["status"]) == AM_E_INFLATE
    with pytest.raises(N.AutomergeError, match="invalid deflate data"):
        N.stage_document(bad_z)


def _stage_both_forms(arena, chunks, docs):
    """Stages and runs one batch with the host form of the inflate stage and again with its
    device-side form (AM_ZSTAGE_DEV, AM_ZSTAGE_DEV_MIN are read per stage)."""
    import os
    from automerge_amd.batch import Batch
    out = []
    for dev in ("0", "1"):
        keep = {k: os.environ.get(k) for k in ("AM_ZSTAGE_DEV", "AM_ZSTAGE_DEV_MIN")}
        os.environ["AM_ZSTAGE_DEV"] = dev
        os.environ["AM_ZSTAGE_DEV_MIN"] = "0"
        try:
            b = Batch()
            b.stage(arena, chunks, docs)
            ninf, nbytes, _ = b.inflate_info()
            b.run()
            b.sync()
            r = b.results()
            h, st, cs = b.chunk_results()
            docs_out = [b.doc_output(i, r[i]) if int(r[i]["status"]) == 0 else None for i in range(len(docs))]
            out.append(((ninf, nbytes), r, h, st, cs, docs_out))
        finally:
            for k, v in keep.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
    return out


def test_device_side_stage_equals_host_stage():
    """A batch whose compressed chunks are all changes is staged by kernels (inflate_stage_dev:
    classification, stream table, layout and the re-wrapped headers on the device). It must stage
    exactly what the host form does -- inflated counts and bytes, every document's status and merged
    bytes, every chunk's hash, state and status -- including base documents (never a compressed
    change), a corrupted and a truncated compressed change, and a compressed change given as a base."""
    import oracle_ffi as O
    import workload as W
    from automerge_amd.batch import pack
    arena, chunks, docs, _ = W.text(11, 8, 40, 50, 4)
    items = [W.doc_chunks(arena, chunks, docs, i) for i in range(len(docs))]
    a4, c4, d4, _ = W.c4(3, 6)
    items += [W.doc_chunks(a4, c4, d4, i) for i in range(len(d4))]
    zi = [k for k, c in enumerate(items[0][1]) if c[8] == 2]
    assert len(zi) >= 3
    bad = [bytearray(c) for c in items[0][1]]
    mid = len(bad[zi[1]]) // 2
    for q in range(mid, mid + 6):
        bad[zi[1]][q] ^= 0x5A  # DEFLATE data corrupted
    items.append((None, [bytes(c) for c in bad]))
    trunc = list(items[1][1])
    z1 = [k for k, c in enumerate(trunc) if c[8] == 2][0]
    trunc[z1] = trunc[z1][:-3]  # the container's data runs past the chunk
    items.append((None, trunc))
    items.append((items[0][1][zi[0]], []))  # a compressed change as the base document
    arena2, chunks2, docs2 = pack(items)
    host, dev = _stage_both_forms(arena2, chunks2, docs2)
    assert host[0] == dev[0] and host[0][0] > 200
    for f in ("status", "err_change", "arg0", "arg1", "out_len", "nheads", "napplied", "nchanges", "max_op"):
        assert (host[1][f] == dev[1][f]).all(), f
    for k in (2, 3, 4):
        assert (host[k] == dev[k]).all(), k
    assert host[5] == dev[5]
    st = host[1]["status"]
    assert (st[:len(items) - 3] == 0).all() and (st[-3:] != 0).all(), st
