#!/usr/bin/env python3
"""Per-phase k_doc cycle profile (probe build with -DAM_PHASE_CLOCK, see tools/build_probe.sh).

  AM_LIB_PATH=tools/clock/libam_clock.so python tools/phase_clock.py [--docs D]
Prints, for each k_doc phase, the average s_memtime cycles per sampled document (every 64th).
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
NAMES = ["P0 stage input", "P1 headers", "P2a lookups", "P2b plan (serial)", "P4 decode streams+ranks",
         "P4 gather+place", "P5a-c checks+id sort", "P5d-e preds+elements", "P5f RGA", "P5g row sort",
         "P5h succ merge", "P6 encode", "header+copy"]
FAST = ["F0 status+stage input", "F1 headers+hashes+refs", "F2 canon+actor table", "F3 base change rows",
        "F4 queue+deps+heads", "F5 op column decode", "F6 rows+entries+checks", "F7 id sort+key rank",
        "F8 preds+elements", "F9 RGA", "F10 doc order+succ", "F11 encode change cols", "F12 encode op cols",
        "F13 trailer+header+copy", "F14 patch (fast_diff)"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", type=int, default=65536)
    ap.add_argument("--streams", action="store_true",
                    help="print slots 16-31 as the wave-decoded streams' cycles by column (decode_stream_wave)")
    ap.add_argument("--text", type=int, default=0, help="C3 text histories of this many changes instead of C4")
    ap.add_argument("--patch", action="store_true", help="stage with AM_DOC_WANT_DIFF (the applyChanges patch)")
    ap.add_argument("--c5", action="store_true", help="C5 pairs merged: base + both sides' 10 changes (~100 rows)")
    ap.add_argument("--mid", action="store_true", help="mid-size documents (workload.mid: 48 changes, ~1,154 ops)")
    ap.add_argument("--handle", type=int, default=0,
                    help="the per-handle shape: load(save(text history of this many changes but the last)) + "
                         "applyChanges(the last change), with the applyChanges patch")
    args = ap.parse_args()
    import workload
    from automerge_amd import _native
    from automerge_amd.batch import WANT_DIFF, Batch
    lib = _native.lib
    f = lib.amx_phase_cycles
    f.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    if args.handle:
        from automerge_amd.batch import pack
        a0, c0, d0, _ = workload.text(0, args.docs, args.handle, 100, 0)
        hist = [workload.doc_chunks(a0, c0, d0, i)[1] for i in range(args.docs)]
        prep = Batch(device=0)
        prep.stage(*pack([(None, h[:-1]) for h in hist]))
        prep.run(); prep.sync()
        bases = [prep.doc_save(i) for i in range(args.docs)]
        arena, chunks, docs = pack([(b_, [h[-1]]) for b_, h in zip(bases, hist)], flags=WANT_DIFF)
        ops = 100 * args.docs
    elif args.mid:
        arena, chunks, docs, ops = workload.mid(0, args.docs)
    elif args.c5:
        arena, chunks, docs, ops = workload.c5(0, args.docs)
        docs = docs.copy()
    elif args.text:
        arena, chunks, docs, ops = workload.text(0, args.docs, args.text, 100, 10)
    else:
        arena, chunks, docs, ops = workload.c4(0, args.docs)
    if args.patch:
        docs["flags"] |= WANT_DIFF
    b = Batch(device=0)
    b.stage(arena, chunks, docs)
    b.run(); b.sync()
    buf = (ctypes.c_ulonglong * 48)()
    f(buf, 1)
    b.run(); b.sync()
    f(buf, 1)
    sampled = (args.docs + 63) // 64
    tot = 0
    for i, n in enumerate(NAMES):
        c = buf[i] / sampled
        tot += c
        print("%-26s %10.0f cycles/doc" % (n, c))
    print("%-26s %10.0f cycles/doc   k_doc stage ms: %s" % ("total", tot, b.stage_times()))
    if args.streams:
        cols = ["objActor", "objCtr", "keyActor", "keyCtr", "keyStr", "idActor", "idCtr", "insert", "action",
                "valLen", "chldActor", "chldCtr", "succNum", "succActor", "succCtr"]
        for j, c in enumerate(cols):
            print("wave stream %-10s %12d cycles" % (c, buf[16 + j]))
        print("streams handed back to the lane decoder: %d" % buf[31])
        print("last hand-back: reason %d at value %d, offset %d, column %d, count %d, state %d" % tuple(buf[32:38]))
        print("keyCtr: window loads %d, loop steps %d, sequential records %d, literal windows %d, values %d" % tuple(buf[40:45]))
        return
    # k_doc_fast: lane 0 of every 16th document
    sampled = (args.docs + 15) // 16
    tot = 0
    for i, n in enumerate(FAST):
        c = buf[16 + i] / sampled
        tot += c
        print("%-26s %10.0f cycles/doc" % (n, c))
    print("%-26s %10.0f cycles/doc (k_doc_fast)" % ("total", tot))


if __name__ == "__main__":
    main()
