"""CPU oracle of the patch Backend.applyChanges returns (oracle/am_apply_patch_oracle.inc:
applyOps / mergeDocChangeOps / seekWithinBlock + incremental updatePatchProperty + setupPatches)
against the reference's own applyChanges patches for every apply step of every golden scenario
(tests/golden/docs.json, produced by the reference)."""
import oracle_ffi as O


def replay(sc):
    """Runs the scenario's steps through the oracle; yields (step index, expected result, got)."""
    doc = None
    for i, (step, exp) in enumerate(zip(sc["steps"], sc["results"])):
        if step["op"] == "load":
            doc = O.Doc.load(bytes.fromhex(step["bytes"]))
            continue
        if doc is None:
            doc = O.Doc.init()
        try:
            got = doc.apply_patch([bytes.fromhex(c) for c in step["changes"]])
        except O.OracleError as e:
            got = {"error": str(e)}
        yield i, exp, got


def test_apply_patch_matches_reference(docs):
    n, bad = 0, []
    for sc in docs:
        for i, exp, got in replay(sc):
            if "patch" not in exp:
                break
            n += 1
            if got != exp["patch"]:
                bad.append((sc["name"], i))
    assert n > 200
    assert not bad, (len(bad), bad[:10])


def test_apply_patch_objectmeta_across_calls(objmeta):
    """The children snapshots the reference's objectMeta carries from one applyChanges call to the
    next on the same handle (new.js:884-931, 1461-1528, 1812/1857): two to four actors create an
    object under one root key concurrently and the merged history arrives in several calls. A
    scenario stops at the first step the oracle does not restate (computeHashGraph of a loaded
    document); every step before it must match the reference's patch."""
    n, skipped, bad = 0, 0, []
    for sc in objmeta:
        for i, exp, got in replay(sc):
            if "patch" not in exp:
                break
            if "error" in got and "not restated by the oracle" in got["error"]:
                skipped += 1
                break
            n += 1
            if got != exp["patch"]:
                bad.append((sc["name"], i))
    assert n > 500 and skipped < n // 3, (n, skipped)
    assert not bad, (len(bad), bad[:10])
