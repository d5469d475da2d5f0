"""Throughput of the batched change history (k_history): computeHashGraph
(new.js:1879-1904) over the saved base documents of the C4 workload, many documents per call of
am_document_changes_batch. Prints a JSON line per document set: documents/s and changes/s of the whole call
(staging, H2D, k_chunks + k_history, D2H, host DEFLATE of the >= 256 B changes), at the C ABI and
through the Python host; the second set is the merged C4 documents (base + 12 concurrent
changes, saved). The reference under Node on one core is quoted from
profiles/cpu_reference_history.json (tools/cpu_reference_history.js, build container).

  python tools/bench_history.py [--docs N] [--reps R]
Under rocprofv3 --kernel-trace --stats the k_history row gives the kernel's own time.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", type=int, default=65536)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--merged", type=int, default=65536)
    args = ap.parse_args()
    import workload
    from automerge_amd import _native as N
    arena, chunks, docs, _ = workload.c4(0, args.docs)
    bases = []
    for i in range(args.docs):
        d = docs[i]
        k = int(d["base_chunk"])
        bases.append(bytes(arena[int(chunks[k]["off"]):int(chunks[k]["off"]) + int(chunks[k]["len"])]))
    out = [run(N, "C4 base documents (1 change each)", bases, args.reps)]
    # merged documents: each C4 document after its 12 concurrent changes, saved (13 changes, 4 actors)
    from automerge_amd.batch import Batch
    nm = min(args.docs, args.merged)
    b = Batch()
    b.stage(*_slice(arena, chunks, docs, nm))
    b.run()
    b.sync()
    merged = [b.doc_save(i) for i in range(nm)]
    out.append(run(N, "merged C4 documents (13 changes each, 4 actors)", merged, args.reps))
    try:
        ref = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "profiles",
                                          "cpu_reference_history.json")))
        out[0]["cpu_reference_node_docs_per_sec"] = ref["c4_base"]["docs_per_sec"]
        out[1]["cpu_reference_node_docs_per_sec"] = ref["c4_merged"]["docs_per_sec"]
    except (OSError, ValueError, KeyError):
        pass
    for o in out:
        print(json.dumps(o))


def _slice(arena, chunks, docs, n):
    d = docs[:n].copy()
    c1 = int(d["chg_begin"][-1] + d["chg_count"][-1])
    return arena, chunks[:c1].copy(), d


def run(N, what, docs, reps):
    res = N.document_changes_batch(docs[:64])  # warm-up (engine, code objects)
    assert not any(isinstance(r, Exception) for r in res)
    best = best_c = None
    for _ in range(reps):
        st = {}
        t0 = time.perf_counter()
        res = N.document_changes_batch(docs, stats=st)
        dt = time.perf_counter() - t0
        best = dt if best is None or dt < best else best
        best_c = st["c_seconds"] if best_c is None or st["c_seconds"] < best_c else best_c
    bad = [r for r in res if isinstance(r, Exception)]
    nchg = sum(len(r) for r in res if not isinstance(r, Exception))
    return {
        "what": "am_document_changes_batch over " + what, "docs": len(docs), "changes": nchg, "errors": len(bad),
        "seconds": best, "docs_per_sec": len(docs) / best, "changes_per_sec": nchg / best,
        "c_abi_seconds": best_c, "c_abi_docs_per_sec": len(docs) / best_c, "c_abi_changes_per_sec": nchg / best_c,
        "input_bytes": sum(len(x) for x in docs),
        "output_bytes": sum(len(c) for r in res if not isinstance(r, Exception) for c, _ in r),
    }

if __name__ == "__main__":
    main()
