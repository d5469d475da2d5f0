"""objectMeta edge cases of the per-handle path (tests/golden/meta_edge.json, recorded from the
reference by tests/golden/gen/make_meta_edge.js):

* a root key with a make op and a concurrent counter `set` + `inc`: documentPatch's children
  snapshot keeps only the visible `set` / make ops (updatePatchProperty, new.js:919-926), so the
  visible inc row must not reach the blob k_doc_fast's patch writer leaves after load
  (am_doc_fast.h fast_diff); the next call edits inside the object and reads that snapshot back;
* a float counter increment: the reference adds it as JS does (new.js:958). The engine cannot
  write that patch (the call fails loudly, AM_U_INC_VALUE), but loadChanges of it commits, as
  the reference's does, with the snapshots the replay left, and later patches are the reference's.
"""
import pytest

pytestmark = pytest.mark.gpu


def _scen(name=None):
    from conftest import golden
    sc = golden("meta_edge.json")["scenarios"]
    return [s for s in sc if name is None or s["name"].startswith(name)]


def test_make_and_counter_on_one_key_per_handle():
    from test_gpu_apply_patch import _replay_handle
    from automerge_amd import _native as N
    n, bad = 0, []
    N.engine_stats()
    for sc in _scen("makecounter/"):
        for i, exp, got, saved, heads in _replay_handle(sc):
            n += 1
            if got != exp["patch"] or saved != exp["save"] or heads != exp["heads"]:
                bad.append((sc["name"], i, got))
                break
    st = N.engine_stats()
    assert n == 16  # apply steps (a load step yields nothing)
    assert st[1] >= 4, st  # the set-only calls after load take k_doc_fast's patch writer
    assert not bad, bad


def test_make_and_counter_on_one_key_batched():
    """The same histories through applyChangesBatch, every scenario's call k in one batch."""
    from test_gpu_apply_patch import _jsonable
    from automerge_amd import backend as B
    scen = _scen("makecounter/")
    hs = [None] * len(scen)
    for k in range(4):
        idx = [j for j, s in enumerate(scen) if k < len(s["steps"])]
        loads = [j for j in idx if scen[j]["steps"][k]["op"] == "load"]
        for j in loads:
            hs[j] = B.load(bytes.fromhex(scen[j]["steps"][k]["bytes"]))
        app = [j for j in idx if scen[j]["steps"][k]["op"] == "apply"]
        for j in app:
            if hs[j] is None:
                hs[j] = B.init()
        res = B.applyChangesBatch([hs[j] for j in app], [[bytes.fromhex(c) for c in scen[j]["steps"][k]["changes"]] for j in app])
        for j, r in zip(app, res):
            assert not isinstance(r, Exception), (scen[j]["name"], k, r)
            hs[j] = r[0]
            exp = scen[j]["results"][k]
            assert _jsonable(r[1]) == exp["patch"], (scen[j]["name"], k)
            assert B.save(hs[j]).hex() == exp["save"], (scen[j]["name"], k)


def test_float_increment_load_changes_commits():
    from test_gpu_apply_patch import _jsonable
    from automerge_amd import _native as N
    from automerge_amd import backend as B
    for sc in _scen("floatinc/"):
        st = B.init()
        for k, (step, exp) in enumerate(zip(sc["steps"], sc["results"])):
            changes = [bytes.fromhex(c) for c in step["changes"]]
            has_float = '"value": 6.5' in str(exp["patch"]).replace("'", '"')
            if has_float:
                # the patch call fails loudly and leaves the handle as it was ...
                with pytest.raises(N.AutomergeError, match="non-integer counter increment"):
                    B.applyChanges(B.clone(st), changes)
                # ... and loadChanges commits like the reference
                st = B.loadChanges(st, changes)
            else:
                st, patch = B.applyChanges(st, changes)
                assert _jsonable(patch) == exp["patch"], (sc["name"], k)
            assert B.save(st).hex() == exp["save"], (sc["name"], k)
            assert B.getHeads(st) == exp["heads"], (sc["name"], k)
