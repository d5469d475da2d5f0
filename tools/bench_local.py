#!/usr/bin/env python3
"""Per-call latency of Backend.applyLocalChange (backend/backend.js:54-91) on large text documents
(the reference's per-change cost on 10k- and 100k-op texts), through the engine's
per-handle C ABI (am_doc_apply_local_change: host encodeChange, then the document re-merged with
the new change on the GPU, applyChanges patch included).

The documents are C1-style text histories (workload.text, cross_every = 0: one actor pair typing
and deleting, 100 ops per change) loaded with applyChanges; each timed call inserts one character
into the text object, as Automerge.change(doc => doc.text.insertAt(0, 'x')) asks the backend.

  python tools/bench_local.py [--ops 10000 100000] [--calls 20]
  python tools/bench_local.py --dump DIR   # histories + requests for tools/cpu_reference_local.js
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

ACTOR = "0123456789abcdef0123456789abcdef"


def history(total_ops, per_change=100):
    import workload as W
    arena, chunks, docs, _ = W.text(0, 1, max(1, total_ops // per_change), per_change, 0)
    return W.doc_chunks(arena, chunks, docs, 0)[1]


def requests(obj, max_op, calls):
    out = []
    for k in range(calls):
        start = max_op + 1 + k
        out.append({"actor": ACTOR, "seq": k + 1, "startOp": start, "time": 0, "message": "", "deps": [],
                    "ops": [{"action": "set", "obj": obj, "elemId": "_head" if k == 0 else "%d@%s" % (start - 1, ACTOR),
                             "insert": True, "value": "x", "pred": []}]})
    return out


def text_object(patch):
    for key, vals in patch["diffs"]["props"].items():
        for v in vals.values():
            if isinstance(v, dict) and v.get("type") == "text":
                return v["objectId"]
    raise SystemExit("no text object in the document")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ops", type=int, nargs="+", default=[10000, 100000])
    ap.add_argument("--calls", type=int, default=20)
    ap.add_argument("--dump", default=None)
    args = ap.parse_args()
    if args.dump:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_ffi as O
        os.makedirs(args.dump, exist_ok=True)
        for n in args.ops:
            h = history(n)
            d = O.Doc.init()
            d.apply(h)
            p = d.patch()
            with open(os.path.join(args.dump, "hist_%d.bin" % n), "wb") as f:
                for c in h:
                    f.write(len(c).to_bytes(4, "little") + c)
            json.dump(requests(text_object(p), p["maxOp"], args.calls), open(os.path.join(args.dump, "req_%d.json" % n), "w"))
        return
    from automerge_amd import backend as B
    res = []
    for n in args.ops:
        h = history(n)
        st, _ = B.applyChanges(B.init(), h)
        p = B.getPatch(st)
        reqs = requests(text_object(p), p["maxOp"], args.calls + 2)
        ms = []
        for k, rq in enumerate(reqs):
            t0 = time.perf_counter()
            st, patch, _ = B.applyLocalChange(st, rq)
            dt = (time.perf_counter() - t0) * 1e3
            if k >= 2:  # the first calls build the actor's clock entry and warm the engine
                ms.append(dt)
            assert patch["diffs"]["objectId"] == "_root"
        ms.sort()
        # "ops": the history's size as requested (the reference side's label, tools/cpu_reference_local.js);
        # max_op: the document's maxOp (two actors that never meet: about half of it)
        res.append({"ops": n, "max_op": int(p["maxOp"]), "changes": len(h), "calls": len(ms),
                    "median_ms": ms[len(ms) // 2], "min_ms": ms[0], "max_ms": ms[-1]})
        print(json.dumps(res[-1]), flush=True)
    print(json.dumps({"what": "Backend.applyLocalChange per call (one inserted character) on text documents, "
                              "am_doc_apply_local_change: host encodeChange + GPU re-merge of the whole document "
                              "+ applyChanges patch + D2H", "results": res}), flush=True)


if __name__ == "__main__":
    main()
