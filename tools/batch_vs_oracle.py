#!/usr/bin/env python3
"""Diagnosis: one Batch of C4 documents (the pipeline test's reference batch) against the oracle,
run `--reps` times; prints the documents whose merged bytes differ from the oracle's."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--first", type=int, default=40)
    ap.add_argument("--docs", type=int, default=2500)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--flags", default="diff")
    a = ap.parse_args()
    import workload as W
    import oracle_ffi as O
    from automerge_amd.batch import WANT_DIFF, WANT_PATCH, Batch
    arena, chunks, docs, _ = W.c4(a.first, a.docs)
    docs = docs.copy()
    docs["flags"] |= {"diff": WANT_DIFF, "patch": WANT_PATCH, "none": 0}[a.flags]
    want = []
    for i in range(a.docs):
        base, ch = W.doc_chunks(arena, chunks, docs, i)
        d = O.Doc.load(base)
        d.apply(ch)
        want.append(d.save())
    for rep in range(a.reps):
        b = Batch()
        b.stage(arena, chunks, docs)
        b.run()
        b.sync()
        r = b.results()
        fast = b.fast_flags()
        bad = []
        for i in range(a.docs):
            if int(r[i]["status"]) or b.doc_output(i, r[i]) != want[i]:
                bad.append((i, int(r[i]["status"]), bool(fast[i])))
        print(json.dumps({"rep": rep, "bad": len(bad), "first": bad[:10], "fast": int(fast.sum())}), flush=True)


if __name__ == "__main__":
    main()
