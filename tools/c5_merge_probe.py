#!/usr/bin/env python3
"""C5 pairs merged in one batch (base + both sides' 10 changes, ~100 rows: the general kernel) with
the applyChanges patch: k_doc stage time (k_doc + k_diff) per run, for A/B builds (AM_LIB_PATH).
  python tools/c5_merge_probe.py [--docs 65536] [--runs 3] [--no-patch]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", type=int, default=65536)
    ap.add_argument("--runs", type=int, default=3)
    ap.add_argument("--no-patch", action="store_true")
    a = ap.parse_args()
    import workload as W
    from automerge_amd.batch import WANT_DIFF, Batch
    arena, chunks, docs, ops = W.c5(0, a.docs)
    docs = docs.copy()
    if not a.no_patch:
        docs["flags"] |= WANT_DIFF
    b = Batch()
    b.stage(arena, chunks, docs)
    ms = []
    for _ in range(a.runs + 1):
        b.run()
        b.sync()
        ms.append(b.stage_times()[2])
    st = b.results()["status"]
    print(json.dumps({"lib": os.environ.get("AM_LIB_PATH", "default"), "docs": a.docs, "patch": not a.no_patch,
                      "k_doc_stage_ms": ms[1:], "errors": int((st != 0).sum()), "fast": int(b.fast_flags().sum())}), flush=True)


if __name__ == "__main__":
    main()
