"""The Node host (automerge_amd/js/backend.js over the N-API addon am_napi.node) -- the drop-in
Backend module of BASELINE.json's north_star (backend/backend.js:8-197 surface)."""
import json
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ADDON = os.path.join(ROOT, "automerge_amd", "js", "am_napi.node")
node = shutil.which("node")
needs_node = pytest.mark.skipif(node is None or not os.path.exists(ADDON), reason="node or am_napi.node missing")


@needs_node
def test_js_backend_exports_and_no_cpu_fallback():
    """Every Backend export exists; without a HIP device the first call throws (no CPU path)."""
    script = ("const B=require(%r);" % os.path.join(ROOT, "automerge_amd", "js", "backend.js") +
              "const names=['init','clone','free','applyChanges','applyLocalChange','save','load','loadChanges',"
              "'getPatch','getHeads','getAllChanges','getChanges','getChangesAdded','getChangeByHash','getMissingDeps'];"
              "const missing=names.filter(n=>typeof B[n]!=='function');"
              "let err=null;try{B.init()}catch(e){err=e.constructor.name+': '+e.message}"
              "console.log(JSON.stringify({missing,err}))")
    env = dict(os.environ, HIP_VISIBLE_DEVICES="-1")  # hide any device: must fail loudly
    out = subprocess.run([node, "-e", script], capture_output=True, text=True, env=env, timeout=120)
    res = json.loads(out.stdout.strip().splitlines()[-1])
    assert res["missing"] == []
    assert res["err"] is not None and "no HIP device" in res["err"]


@needs_node
@pytest.mark.gpu
def test_js_backend_replays_golden_scenarios():
    out = subprocess.run([node, os.path.join(ROOT, "tests", "js", "backend_replay.js")], capture_output=True,
                         text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    res = json.loads(out.stdout.strip().splitlines()[-1])
    assert res["scenarios"] > 300
    assert res["applied"] > 300  # applyChanges patches compared with the reference's
    assert res["histDocs"] > 100  # getAllChanges(load(saved)) compared with the reference's
    assert res["nbad"] == 0, res["bad"]
    g = res["graph"]
    assert g["applied_equal_given"] and g["missing"] == [] and g["since_heads"] == 0
