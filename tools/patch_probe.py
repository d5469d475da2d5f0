#!/usr/bin/env python3
"""One applyChanges patch (WANT_DIFF) of C3-shaped text documents -- load(save(first half)) +
applyChanges(second half) -- or of mid documents, for timing the P8 replay (k_doc + k_diff stage
time). With AM_LIB_PATH=tools/dcheck/libam_dcheck.so the diagnostics build prints its per-section
cycle counts ([p8prof] lines).
  python tools/patch_probe.py [--docs 1] [--changes 1000] [--per-change 100] [--cross 10] [--runs 3]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", type=int, default=1)
    ap.add_argument("--changes", type=int, default=1000)
    ap.add_argument("--per-change", type=int, default=100)
    ap.add_argument("--cross", type=int, default=10)
    ap.add_argument("--runs", type=int, default=3)
    a = ap.parse_args()
    import workload as W
    from automerge_amd.batch import WANT_DIFF, Batch, pack
    arena, chunks, docs, _ = W.text(0, a.docs, a.changes, a.per_change, a.cross)
    hist = [W.doc_chunks(arena, chunks, docs, i)[1] for i in range(a.docs)]
    half = (1 + a.changes) // 2
    prep = Batch()
    prep.stage(*pack([(None, h[:half]) for h in hist]))
    prep.run()
    prep.sync()
    r = prep.results()
    assert (r["status"] == 0).all(), "preparation failed: %s" % {k: r[k][:4].tolist() for k in r.dtype.names} if hasattr(r, "dtype") else r
    bases = [prep.doc_save(i) for i in range(a.docs)]
    del prep
    b = Batch()
    b.stage(*pack([(bases[i], hist[i][half:]) for i in range(a.docs)], flags=WANT_DIFF))
    times = []
    for _ in range(a.runs):
        b.run()
        b.sync()
        times.append(b.stage_times()[2])
    st = b.results()["status"]
    print(json.dumps({"docs": a.docs, "ops_per_doc": 1 + a.changes * a.per_change, "k_doc_ms": times,
                      "statuses": sorted(set(int(x) for x in st))}), flush=True)


if __name__ == "__main__":
    main()
