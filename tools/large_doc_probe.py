#!/usr/bin/env python3
"""One batch of large or mid-size documents through the general kernels, for rocprofv3 --pmc passes
of glb_mode::k_doc and k_diff (tools/pmc_large.sh): C3-style text histories (--text, changes of 100
ops, load of nothing) or the mid workload (--mid), merged with the applyChanges patch (--diff).

  python tools/large_doc_probe.py --text 1000 --docs 64 [--diff]
  python tools/large_doc_probe.py --mid --docs 2048 [--diff]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--text", type=int, default=0)
    ap.add_argument("--mid", action="store_true")
    ap.add_argument("--docs", type=int, default=64)
    ap.add_argument("--diff", action="store_true")
    args = ap.parse_args()
    import workload as W
    from automerge_amd.batch import WANT_DIFF, Batch
    if args.mid:
        arena, chunks, docs, ops = W.mid(0, args.docs)
    else:
        arena, chunks, docs, ops = W.text(0, args.docs, args.text or 1000, 100, 10)
    docs = docs.copy()
    if args.diff:
        docs["flags"] |= WANT_DIFF
    b = Batch()
    b.stage(arena, chunks, docs)
    t0 = time.perf_counter()
    b.run()
    b.sync()
    dt = time.perf_counter() - t0
    r = b.results()
    print(json.dumps({"docs": len(docs), "ops": int(ops), "errors": int((r["status"] != 0).sum()), "run_s": dt,
                      "stage_ms": b.stage_times()}), flush=True)


if __name__ == "__main__":
    main()
