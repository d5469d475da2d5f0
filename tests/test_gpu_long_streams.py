"""k_doc's P4 decodes an op column of 256 values or more with a whole wave (decode_stream_wave,
am_doc_impl.h: a register window over the stream, records read by readlane, literal runs a window at a
time) and shorter ones a lane each (decode_stream, the RLEDecoder / DeltaDecoder / BooleanDecoder of
encoding.js:820-886, 1025-1030, 1171-1183). AM_DEC_LONG moves the threshold, so the same batch runs
through either decoder. They must agree on every input: the same merged bytes for valid documents, the
same status and arguments for corrupted ones (a stream with any error goes back to the lane decoder,
which reports the reference's first error). The valid merge also equals the oracle's.

Inputs: text histories saved by the oracle (a base of 2,900-4,900 ops, its DEFLATEd columns inflated by
the engine's own stage), loaded as the base of a batch document with the history's last change merged
into it; corrupted copies change bytes of one op column and recompute the checksum."""
import os
import random

import pytest

pytestmark = pytest.mark.gpu

LANES_ONLY = 1 << 30  # a threshold past every stream's length


def _base_and_change(seed, nchanges, cross):
    import oracle_ffi as O
    import workload as W
    from automerge_amd import _native as N
    from test_gpu_inflate import _rechecksum
    arena, chunks, docs, _ = W.text(seed, 1, nchanges, 100, cross)
    _, chg = W.doc_chunks(arena, chunks, docs, 0)
    d = O.Doc.init()
    d.apply(chg[:-1])
    staged, _ = N.stage_document(d.save())  # keeps the checksum of the DEFLATEd form: recomputed
    d.apply(chg[-1:])
    return _rechecksum(staged), chg[-1], d.save()


def _merge(items, dec_long):
    from automerge_amd.batch import Batch, pack
    os.environ["AM_DEC_LONG"] = str(dec_long)
    try:
        b = Batch()
        b.stage(*pack(items))
        b.run()
        b.sync()
        r = b.results()
        out = []
        for k in range(len(items)):
            st = int(r[k]["status"])
            out.append((st, int(r[k]["arg0"]), int(r[k]["arg1"]), b.doc_save(k) if st == 0 else None))
        return out
    finally:
        del os.environ["AM_DEC_LONG"]


@pytest.mark.parametrize("seed,nchanges,cross", [(21, 30, 0), (5, 50, 10)])
def test_wave_decoder_equals_lane_decoder_and_oracle(seed, nchanges, cross):
    base, last, want = _base_and_change(seed, nchanges, cross)
    wave = _merge([(base, [last])], 256)
    lanes = _merge([(base, [last])], LANES_ONLY)
    assert wave == lanes
    assert wave[0][0] == 0 and wave[0][3] == want


def test_wave_decoder_errors_equal_lane_decoder():
    from test_gpu_inflate import _rechecksum
    from test_gpu_large_doc_counts import _columns
    base, last, _ = _base_and_change(21, 30, 0)
    cols = [c for c in _columns(base) if c[0] == "ops" and c[3] > 8]
    assert len(cols) >= 6
    rng = random.Random(11)
    items = [(base, [last])]
    for _ in range(63):
        _, cid, at, n = rng.choice(cols)
        c = bytearray(base)
        for _ in range(rng.choice([1, 1, 2, 3])):
            q = at + rng.randrange(n)
            c[q] = rng.choice([0x80 | c[q], c[q] ^ 0x40, c[q] ^ 0x01, 0x7F, 0xFF, 0x00, 0x01, 0x02, c[q - 1]])
        if rng.random() < 0.2:
            c[at + n - 1] |= 0x80  # an incomplete LEB128 at the column's end
        items.append((_rechecksum(bytes(c)), [last]))
    wave = _merge(items, 256)
    lanes = _merge(items, LANES_ONLY)
    for k, (w, l) in enumerate(zip(wave, lanes)):
        assert w == l, k
    assert wave[0][0] == 0
    assert sum(1 for w in wave[1:] if w[0]) >= 8  # most corruptions fail the document


def test_every_stream_on_the_wave_decoder_matches_lanes(docs):
    """Every single-apply golden scenario (the reference's documents and changes: map keys, text,
    counters, malformed input) and a C4 / C2 sample through the general kernel (AM_FAST=0) with
    every column of one value or more on the wave decoder (AM_DEC_LONG=1), against all of them on
    lanes: identical results, merged bytes and heads."""
    import workload
    from automerge_amd.batch import Batch
    items = []
    for sc in docs:
        steps = sc["steps"]
        if len(steps) == 1 and steps[0]["op"] == "apply":
            items.append((None, [bytes.fromhex(c) for c in steps[0]["changes"]]))
        elif len(steps) == 2 and steps[0]["op"] == "load":
            items.append((bytes.fromhex(steps[0]["bytes"]), [bytes.fromhex(c) for c in steps[1]["changes"]]))
    for kind in ("c4", "c2"):
        arena, chunks, dd, _ = getattr(workload, kind)(9, 200)
        items += [workload.doc_chunks(arena, chunks, dd, i) for i in range(200)]
    assert len(items) > 600

    def run(dec_long):
        os.environ["AM_FAST"] = "0"
        os.environ["AM_DEC_LONG"] = str(dec_long)
        try:
            b = Batch()
            b.stage_docs(items)
            b.run()
            b.sync()
        finally:
            del os.environ["AM_FAST"], os.environ["AM_DEC_LONG"]
        r = b.results()
        outs = [b.doc_output(i, r[i]) if r[i]["status"] == 0 else b"" for i in range(len(items))]
        heads = [b.doc_heads(i, int(r[i]["nheads"])) if r[i]["status"] == 0 else [] for i in range(len(items))]
        return r, outs, heads

    rw, ow, hw = run(1)
    rl, ol, hl = run(LANES_ONLY)
    bad = []
    for i in range(len(items)):
        for k in ("status", "err_change", "arg0", "arg1", "napplied", "nqueued", "nheads", "nops", "nchanges", "max_op",
                  "out_len"):
            if rw[i][k] != rl[i][k]:
                bad.append((i, k, int(rw[i][k]), int(rl[i][k])))
        if ow[i] != ol[i]:
            bad.append((i, "bytes"))
        if hw[i] != hl[i]:
            bad.append((i, "heads"))
    assert not bad, bad[:10]
