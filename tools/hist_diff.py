"""Per-change diff of the GPU history (am_document_changes_batch) against a history_cases.json case:
writes gpurun_out/hist_diff.json with both change lists of every mismatching case."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from automerge_amd import _native as N  # noqa: E402

cases = json.load(open("tests/golden/history_cases.json"))
got = N.document_changes_batch([bytes.fromhex(c["doc"]) for c in cases])
out = []
for c, g in zip(cases, got):
    if isinstance(g, Exception):
        ok = c["direct_error"] == str(g)
        if not ok:
            out.append({"name": c["name"], "want_err": c["direct_error"], "got_err": str(g)})
        continue
    mine = [b.hex() for b, _ in g]
    if mine != c["direct"]:
        out.append({"name": c["name"], "want": c["direct"], "got": mine, "want_err": c["direct_error"]})
json.dump(out, open("gpurun_out/hist_diff.json", "w"))
print(len(out), "mismatching cases:", [o["name"] for o in out])
