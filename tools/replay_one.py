"""Replays one recorded backend-log scenario through the Python host and writes the first
mismatching call (expected and got, in full) to gpurun_out/replay_one.json.
  python tools/replay_one.py <file> <scenario name>"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import backend_log as L  # noqa: E402
from automerge_amd import backend as B  # noqa: E402

f, name = sys.argv[1], sys.argv[2]
sc = [s for s in L.load(f)["scenarios"] if s["name"] == name][0]
handles = {}
out = None
for i, e in enumerate(sc["log"]):
    try:
        res, err = getattr(B, e["fn"])(*L._args(e["fn"], L.decode(e["args"], handles))), None
    except Exception as x:  # noqa: BLE001
        res, err = None, str(x)
    if "error" in e or err is not None:
        if err != (e.get("error") or {}).get("message"):
            out = {"i": i, "fn": e["fn"], "args": e["args"], "want_err": e.get("error"), "got_err": err}
            break
        continue
    if not L.match(e["result"], res, handles):
        out = {"i": i, "fn": e["fn"], "args": e["args"], "want": e["result"], "got": L.canon(res)}
        break
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
json.dump(out, open(os.path.join(ROOT, "gpurun_out", "replay_one.json"), "w"), indent=1)
print("first mismatch:", None if out is None else (out["i"], out["fn"]))
