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
