"""The drop-in boundary on the GPU: every call of the 22 backend/index.js exports recorded from the
reference's own test files (sync_test.js, backend_test.js, test.js, text_test.js, table_test.js;
tests/golden/backend_log_*.json) replayed through the Python host and through the Node host --
patches, binary changes, saved documents, heads, hash-graph queries, sync messages and sync states,
handle identity and error class + message all compared with the reference's."""
import json
import os
import shutil
import subprocess

import pytest

import backend_log as L

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
node = shutil.which("node")


@pytest.mark.parametrize("name", L.FILES)
def test_python_host_replays_reference_backend_calls(name):
    from automerge_amd import backend as B
    calls, scenarios, bad = L.replay(B, [name])
    assert calls > 40 and scenarios > 10
    assert bad == []


@pytest.mark.skipif(node is None or not os.path.exists(os.path.join(ROOT, "automerge_amd", "js", "am_napi.node")),
                    reason="node or am_napi.node missing")
def test_node_host_replays_reference_backend_calls():
    out = subprocess.run([node, os.path.join(ROOT, "tests", "js", "backend_log_replay.js")], capture_output=True,
                         text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    res = json.loads(out.stdout.strip().splitlines()[-1])
    assert res["calls"] > 2500
    assert set(res["perFn"]) >= {"applyLocalChange", "generateSyncMessage", "receiveSyncMessage", "getChanges"}
    assert res["nbad"] == 0, res["bad"]
