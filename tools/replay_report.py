"""Prints every mismatch of the golden Backend logs (backend_log_*.json, newbackend_log.json) replayed
through automerge_amd.backend on the GPU (a diagnostic; the tests stop at the first)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import backend_log as L  # noqa: E402
import newbackend_log as NB  # noqa: E402
from automerge_amd import backend as B  # noqa: E402

files = sys.argv[1].split(",") if len(sys.argv) > 1 else L.FILES
for f in files:
    if f == "newbackend":
        calls, bad = NB.replay(B)
        scen = "-"
    else:
        calls, scen, bad = L.replay(B, [f], stop_at=1000)
    print("== %s: %s calls, %s scenarios, %d bad" % (f, calls, scen, len(bad)))
    for b in bad:
        print("   ", repr(b)[:700])
