"""CPU oracle of Backend.getPatch() (oracle/am_patch_oracle.inc: documentPatch + updatePatchProperty
+ appendEdit/appendUpdate + decodeValue) against the reference's own getPatch output for every
step of every golden scenario (tests/golden/docs.json: getPatch(load(save(state))))."""
import oracle_ffi as O


def test_getpatch_matches_reference(docs):
    n, bad = 0, []
    for sc in docs:
        for i, res in enumerate(sc["results"]):
            if "getPatch" not in res or "save" not in res:
                continue
            got = O.Doc.load(bytes.fromhex(res["save"])).patch()
            n += 1
            if got != res["getPatch"]:
                bad.append((sc["name"], i))
    assert n > 400
    assert not bad, bad[:10]
