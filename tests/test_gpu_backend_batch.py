"""The batched per-handle surface (am_doc_*_batch, include/automerge_amd.h; automerge_amd.backend
loadBatch / applyChangesBatch / loadChangesBatch / getPatchBatch / saveBatch): every golden scenario
replayed in lockstep, step k of all scenarios as ONE GPU batch, against the reference's recorded
results (tests/golden/docs.json, objmeta.json): patches, getPatch, save bytes, heads, pending
changes and error messages after every step. Loaded documents whose changes need the hash graph
(new.js:1826-1832) take the batched computeHashGraph and run again inside the call.
"""
import pytest

from test_gpu_apply_patch import _jsonable

pytestmark = pytest.mark.gpu


def _lockstep(scenarios, loadchanges_every=0):
    from automerge_amd import backend as B
    live = {i: None for i in range(len(scenarios))}  # scenario -> backend state
    napply = {i: 0 for i in live}
    done = set()
    bad, n = [], 0
    k = 0
    while len(done) < len(scenarios):
        loads, applies, loadch = [], [], []
        for i, sc in enumerate(scenarios):
            if i in done:
                continue
            if k >= len(sc["steps"]):
                done.add(i)
                continue
            st = sc["steps"][k]
            if st["op"] == "load":
                loads.append(i)
                continue
            if live[i] is None:
                live[i] = B.init()
            napply[i] += 1
            (loadch if loadchanges_every and napply[i] % loadchanges_every == 0 else applies).append(i)
        res = {}
        if loads:
            for i, r in zip(loads, B.loadBatch([bytes.fromhex(scenarios[i]["steps"][k]["bytes"]) for i in loads])):
                res[i] = (r, None) if isinstance(r, Exception) else (r, "load")
        chs = lambda i: [bytes.fromhex(c) for c in scenarios[i]["steps"][k]["changes"]]  # noqa: E731
        if applies:
            for i, r in zip(applies, B.applyChangesBatch([live[i] for i in applies], [chs(i) for i in applies])):
                res[i] = (r, None) if isinstance(r, Exception) else (r[0], _jsonable(r[1]))
        if loadch:
            for i, r in zip(loadch, B.loadChangesBatch([live[i] for i in loadch], [chs(i) for i in loadch])):
                res[i] = (r, None) if isinstance(r, Exception) else (r, "noop")
        ok = [i for i in sorted(res) if not isinstance(res[i][0], Exception)]
        saves = dict(zip(ok, B.saveBatch([res[i][0] for i in ok])))
        gps = dict(zip(ok, B.getPatchBatch([res[i][0] for i in ok])))
        for i in sorted(res):
            sc, exp = scenarios[i], scenarios[i]["results"][k]
            st, got = res[i]
            if isinstance(st, Exception):
                if "error" not in exp or str(st) != exp["error"]["message"]:
                    bad.append((sc["name"], k, "error", str(st)))
                done.add(i)
                continue
            if "error" in exp:
                bad.append((sc["name"], k, "missing error"))
                done.add(i)
                continue
            n += 1
            live[i] = st
            if isinstance(got, dict) and got != exp["patch"]:
                bad.append((sc["name"], k, "patch"))
            elif saves[i] != bytes.fromhex(exp["save"]) or B.getHeads(st) != exp["heads"]:
                bad.append((sc["name"], k, "save/heads"))
            elif B.pendingChanges(st) != exp["pending"]:
                bad.append((sc["name"], k, "pending"))
            elif _jsonable(gps[i]) != dict(exp["getPatch"], pendingChanges=exp["pending"]):
                bad.append((sc["name"], k, "getPatch"))
            else:
                continue
            done.add(i)
        k += 1
    return n, bad


@pytest.mark.parametrize("every", [0, 3])
def test_lockstep_batches_match_reference(docs, objmeta, every):
    n, bad = _lockstep(docs + objmeta, every)
    assert not bad, (n, len(bad), bad[:10])
    assert n > 1100


def test_batch_repeated_handle_is_sequential(objmeta):
    """A handle named twice in one applyChangesBatch behaves as two sequential calls: the first
    applies and freezes the handle, so the second raises the outdated-document error in its own slot
    (backend/util.js:1-10); when the first call fails, the handle is unchanged and the second call
    applies. The result of the first call stays usable and is not shared with another wrapper."""
    from automerge_amd import backend as B
    checked = 0
    for sc in objmeta[:40]:
        steps = [s for s in sc["steps"] if s["op"] == "apply"]
        if sc["steps"][0]["op"] != "apply" or len(steps) < 2:
            continue
        c0 = [bytes.fromhex(c) for c in steps[0]["changes"]]
        c1 = [bytes.fromhex(c) for c in steps[1]["changes"]]
        seq, p0 = B.applyChanges(B.init(), c0)
        h = B.init()
        r = B.applyChangesBatch([h, h], [c0, c1])
        assert not isinstance(r[0], Exception), r[0]
        assert isinstance(r[1], RuntimeError) and "outdated" in str(r[1]), r[1]
        assert _jsonable(r[0][1]) == _jsonable(p0), sc["name"]
        assert B.save(r[0][0]) == B.save(seq)
        # a failing first call leaves the handle usable: the second applies
        h = B.init()
        r = B.applyChangesBatch([h, h], [[b"\x85\x6f\x4a\x83\x00\x00\x00\x00\x01\x05abcde"], c0])
        assert isinstance(r[0], Exception) and not isinstance(r[1], Exception), r
        assert _jsonable(r[1][1]) == _jsonable(p0) and B.save(r[1][0]) == B.save(seq)
        checked += 1
    assert checked >= 10


def test_batch_errors_in_place(docs):
    """A batch mixing good and failing documents: each failure is the single call's error, in its
    place, and leaves its handle usable and unchanged; the others apply."""
    from automerge_amd import _native as N
    from automerge_amd import backend as B
    good = [sc for sc in docs if sc["steps"][0]["op"] == "apply" and "patch" in sc["results"][0]][:20]
    changes = [[bytes.fromhex(c) for c in sc["steps"][0]["changes"]] for sc in good]
    junk = [b"\x85\x6f\x4a\x83\x00\x00\x00\x00\x01\x05abcde"]
    lists = []
    for i, ch in enumerate(changes):
        lists.append(junk if i % 3 == 1 else ch)
    hs = [B.init() for _ in lists]
    r = B.applyChangesBatch(hs, lists)
    for i, x in enumerate(r):
        if i % 3 == 1:
            assert isinstance(x, N.AutomergeError), i
            with pytest.raises(N.AutomergeError) as e:
                B.applyChanges(B.init(), junk)
            assert str(x) == str(e.value)
            assert B.save(hs[i]) == B.save(B.init())  # unchanged, not frozen
        else:
            assert not isinstance(x, Exception), (i, x)
            assert _jsonable(x[1]) == good[i]["results"][0]["patch"]


def test_backend_logs_lockstep_through_batches():
    """Every recorded Backend call of the reference's own tests and randomized sync sessions
    (tests/golden/backend_log_*.json), replayed in lockstep: call k of every scenario at once, the
    calls of applyChanges / loadChanges / load / save / getPatch / generateSyncMessage /
    receiveSyncMessage each as ONE batched call (am_doc_*_batch, am_sync_generate,
    am_sync_receive_batch). Results, errors and handle identities equal the reference's."""
    import backend_log as L
    from automerge_amd import backend as B
    calls, batched, bad = L.replay_lockstep(B)
    assert not bad, (len(bad), bad[:5])
    assert calls > 7000 and batched > 3000, (calls, batched)


def test_node_backend_logs_lockstep_through_batches():
    """The same lockstep replay through the Node host's batched surface (automerge_amd/js/backend.js
    loadBatch / applyChangesBatch / loadChangesBatch / saveBatch / getPatchBatch /
    generateSyncMessages / receiveSyncMessages over the N-API addon), patches materialized lazily."""
    import json
    import os
    import shutil
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    node = shutil.which("node")
    if not node or not os.path.exists(os.path.join(root, "automerge_amd", "js", "am_napi.node")):
        pytest.skip("node or am_napi.node missing")
    out = subprocess.run([node, os.path.join(root, "tests", "js", "backend_log_replay.js"),
                          "sync,sync_random,objmeta,backend,test,text,table,errors", "--lockstep"],
                         capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    res = json.loads(out.stdout.strip().splitlines()[-1])
    assert res["nbad"] == 0, res["bad"]
    assert res["calls"] > 7000 and res["batched"] > 3000, res
