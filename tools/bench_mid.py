#!/usr/bin/env python3
"""Mid-size documents (workload.mid: rounds of concurrent text / title edits by 4 actors, 200-2,000
ops per document) through one GPU batch per step from host memory: Backend.init() +
applyChanges(all changes) with the applyChanges patch (WANT_DIFF), the deflated changes inflated on
the device by the batch stage. Prints one JSON line: ops merged/s, the fraction of documents the
small-document kernel (k_doc_fast) merged, and per-kernel times.
  python tools/bench_mid.py [--docs N] [--steps K] [--actors A] [--rounds R] [--min-ops m] [--max-ops M]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", type=int, default=8192)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--actors", type=int, default=4)
    ap.add_argument("--rounds", type=int, default=12)
    ap.add_argument("--min-ops", type=int, default=8)
    ap.add_argument("--max-ops", type=int, default=40)
    ap.add_argument("--check", type=int, default=8)
    ap.add_argument("--flags", choices=["diff", "patch", "none"], default="diff",
                    help="diff: the applyChanges patch (default); patch: getPatch; none: merge only")
    a = ap.parse_args()
    import numpy as np
    import workload as W
    from automerge_amd.batch import WANT_DIFF, WANT_PATCH, Batch
    t0 = time.perf_counter()
    arena, chunks, docs, ops = W.mid(0, a.docs, a.actors, a.rounds, a.min_ops, a.max_ops)
    gen_s = time.perf_counter() - t0
    docs = docs.copy()
    docs["flags"] |= {"diff": WANT_DIFF, "patch": WANT_PATCH, "none": 0}[a.flags]
    b = Batch()
    rec = {}
    times = []
    for k in range(a.steps + 1):
        t0 = time.perf_counter()
        b.stage(arena, chunks, docs)
        b.run()
        b.sync()
        el = time.perf_counter() - t0
        if k:
            times.append(el)
    res = b.results()
    st = res["status"]
    fast = b.fast_flags()
    el = min(times)
    rec.update({"workload": "mid: %d docs, %d actors x %d rounds, %d-%d ops per change" % (a.docs, a.actors, a.rounds, a.min_ops,
                                                                                          a.max_ops),
                "flags": a.flags,
                "ops": ops, "ops_per_doc": ops / a.docs, "ms_per_step": el * 1e3, "ops_per_s": ops / el,
                "docs_per_s": a.docs / el, "errors": int((st != 0).sum()), "gen_s": gen_s,
                "fast_fraction": float(np.mean(fast)),
                "stage_times_ms": b.stage_times(), "inflate": b.inflate_info(), "workspace_bytes": int(b.workspace_bytes()),
                "kernel_info": b.kernel_info()})
    # the oracle on a few documents (outside the timing)
    import oracle_ffi as O
    for i in range(min(a.check, a.docs)):
        _, ch = W.doc_chunks(arena, chunks, docs, i)
        d = O.Doc.init()
        d.apply(ch)
        assert b.doc_save(i) == d.save(), "document %d differs from the oracle" % i
    rec["verified_docs"] = min(a.check, a.docs)
    # the oracle's own rate on one core over a bounded sample
    t0 = time.perf_counter()
    n = 0
    while time.perf_counter() - t0 < 5 and n < a.docs:
        _, ch = W.doc_chunks(arena, chunks, docs, n)
        d = O.Doc.init()
        d.apply(ch)
        d.save()
        n += 1
    rec["cpu_oracle_docs_per_s_1core"] = n / (time.perf_counter() - t0)
    rec["cpu_oracle_ops_per_s_1core"] = rec["cpu_oracle_docs_per_s_1core"] * ops / a.docs
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
