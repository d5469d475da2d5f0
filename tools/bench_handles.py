#!/usr/bin/env python3
"""Batched per-handle calls on C4 documents at the C ABI (include/automerge_amd.h): am_doc_load_batch
of N saved base documents, then am_doc_apply_changes_batch of their 12 changes with patches (the
objectMeta-carrying applyChanges that Automerge.applyChanges / receiveSyncMessage reach), then a
second apply call on the same handles (the handles' objectMeta blobs restored). Prints docs/s per
call, the fraction k_doc_fast merged (am_engine_stats) and, with AM_SYNC_PROFILE=1, the stage times
of run_many on stderr. Outside the timing: patches and saved documents of a sample against the
general kernel (AM_FAST=0) and the oracle.
  python tools/bench_handles.py [--docs N] [--reps R]"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", type=int, default=200000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--split", type=int, default=6, help="changes in the first apply call (the rest in the second)")
    a = ap.parse_args()
    from automerge_amd import _native as N
    import workload
    arena, chunks, docs, _ = workload.c4(0, a.docs)
    n = a.docs
    get = lambda k: bytes(arena[int(chunks[k]["off"]):int(chunks[k]["off"]) + int(chunks[k]["len"])])  # noqa: E731
    bases = [get(int(docs[i]["base_chunk"])) for i in range(n)]
    chg = [[get(int(docs[i]["chg_begin"]) + j) for j in range(int(docs[i]["chg_count"]))] for i in range(n)]
    eng = N.engine(0)
    arr = (C.c_char_p * n)(*bases)
    lens = (C.c_size_t * n)(*[len(b) for b in bases])
    codes = np.zeros(n, np.uint32)

    def calls(parts):
        flat = [c for cl in parts for c in cl]
        carr = (C.c_char_p * len(flat))(*flat)
        clen = (C.c_size_t * len(flat))(*[len(c) for c in flat])
        off = np.zeros(n + 1, np.uint64)
        off[1:] = np.cumsum([len(cl) for cl in parts])
        return carr, clen, off, sum(len(c) for c in flat)

    first = calls([c[:a.split] for c in chg])
    second = calls([c[a.split:] for c in chg])
    res = {"workload": "C4 handles: load of %d saved base documents, then applyChanges with patches of %d + %d changes" %
                       (n, a.split, 12 - a.split), "docs": n}
    best = {"load": 1e9, "apply1": 1e9, "apply2": 1e9}
    stats = None
    for r in range(a.reps):
        handles = np.zeros(n, np.uint64)
        t0 = time.perf_counter()
        bad = N.lib.am_doc_load_batch(eng, n, arr, lens, handles.ctypes.data, codes.ctypes.data, None)
        best["load"] = min(best["load"], time.perf_counter() - t0)
        assert bad == 0, int(bad)
        N.engine_stats()
        pats = np.zeros(n, np.uint64)
        plen = np.zeros(n, np.uint64)
        for key, (carr, clen, off, _) in (("apply1", first), ("apply2", second)):
            t0 = time.perf_counter()
            bad = N.lib.am_doc_apply_changes_batch(n, handles.ctypes.data, off.ctypes.data, carr, clen, pats.ctypes.data,
                                                   plen.ctypes.data, None, codes.ctypes.data, None)
            best[key] = min(best[key], time.perf_counter() - t0)
            assert bad == 0, (int(bad), int(codes[codes != 0][0]))
            for p in pats:
                if p:
                    N.lib.am_free(C.c_void_p(int(p)))
        stats = N.engine_stats()
        if r < a.reps - 1:
            for h in handles:
                N.lib.am_doc_free(C.c_void_p(int(h)))
    res.update({"load_docs_per_s": n / best["load"], "apply1_docs_per_s": n / best["apply1"],
                "apply2_docs_per_s": n / best["apply2"], "apply1_s": best["apply1"], "apply2_s": best["apply2"],
                "ops_per_s_apply": n * 60 / (best["apply1"] + best["apply2"]),
                "fast_fraction": stats[1] / max(stats[0], 1), "per_handle_docs_counted": stats[0]})
    # the saved documents of a sample against the oracle
    import oracle_ffi as O
    checked = 0
    for i in range(0, n, max(1, n // 32)):
        o = O.Doc.load(bases[i])
        o.apply(chg[i])
        out, ln, err = N.u8p(), C.c_size_t(), N.Error()
        assert not N.lib.am_doc_save(C.c_void_p(int(handles[i])), C.byref(out), C.byref(ln), C.byref(err))
        assert N.take(out, ln.value) == o.save(), i
        checked += 1
    res["oracle_checked"] = checked
    print(json.dumps(res))


if __name__ == "__main__":
    main()
