#!/usr/bin/env python3
"""The host's share of a batched applyChanges (materializing the JS patch objects is
reported separately from the GPU step): C4 documents merged on the GPU with their applyChanges patch
(am_pipe_*, the bench's path), then the wire-form logs turned into patch objects by the Node host
(automerge_amd/js/backend.js materializePatch, tools/js_materialize.js) and by the Python host
(automerge_amd/patch.py). Prints one JSON line with microseconds per document for each host.

  python tools/js_materialize.py [--docs 65536]
"""
import argparse
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", type=int, default=65536)
    args = ap.parse_args()
    import workload
    from automerge_amd import patch as P
    from automerge_amd import pipe
    from automerge_amd.batch import WANT_DIFF, Batch
    D = args.docs
    arena, chunks, docs, _ = workload.c4(0, D)
    docs = docs.copy()
    docs["flags"] |= WANT_DIFF
    probe = Batch()
    probe.stage(arena, chunks, docs)
    ws = int(probe.workspace_bytes())
    kinfo = probe.kernel_info()
    del probe
    cap = D * 1024 + (1 << 20)
    pl = pipe.Pipeline(len(arena), len(chunks), D, ws + ws // 8 + (1 << 20), cap, cap, kinfo["k_doc_fast_lds_per_doc"], slots=2)
    summ = np.zeros(D, pipe.SUMMARY_DT)
    out = np.zeros(cap, np.uint8)
    pat = np.zeros(cap, np.uint8)
    pl.submit(arena, chunks, docs, summ, out, pat)
    pl.drain(1)
    assert (summ["status"] == 0).all()
    logs = [bytes(pat[int(s["patch_off"]):int(s["patch_off"]) + int(s["patch_len"])]) for s in summ]
    t0 = time.perf_counter()
    for log in logs:
        P.materialize(log, [], 0, 0)
    py_s = time.perf_counter() - t0
    rec = {"what": "materializing the applyChanges patch objects of C4 documents from the engine's wire-form logs "
                   "(host work, outside the GPU step)", "docs": D,
           "log_bytes_per_doc": sum(len(x) for x in logs) / D,
           "python": {"us_per_doc": 1e6 * py_s / D, "docs_per_s": D / py_s}}
    node = shutil.which("node")
    if node:
        with tempfile.NamedTemporaryFile(suffix=".bin", delete=False) as f:
            for log in logs:
                f.write(len(log).to_bytes(4, "little"))
                f.write(log)
            fn = f.name
        try:
            r = subprocess.run([node, os.path.join(ROOT, "tools", "js_materialize.js"), fn], capture_output=True, text=True,
                               timeout=300)
            rec["node"] = json.loads(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 else {"error": r.stderr[-500:]}
        finally:
            os.unlink(fn)
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
