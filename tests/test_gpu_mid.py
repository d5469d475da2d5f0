"""Mid-size documents on the GPU (round-5 workload between C4's 62 ops and C3's 100k: 4-8 actors
editing a text and a title in rounds of concurrent changes, 50-2,000 ops per document, changes
>= 256 B deflated; workload/am_workload.cpp gen_mid). Every document runs through one batched
launch and is compared with tests/golden/mid.json, which the reference backend produced from the
same change bytes (tests/golden/gen/make_mid.py / make_mid.js): save() bytes, heads and getPatch()
of applyChanges(init(), all changes), and of load(save(first half)) + applyChanges(rest) with the
patch applyChanges returns."""
import json
import os

import pytest

from test_gpu_text import _jsonable, _run, jsha, sha

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
CASES = json.load(open(os.path.join(HERE, "golden", "mid.json")))


@pytest.mark.parametrize("build", ["glb4", "glb8", "glb16"])
@pytest.mark.parametrize("cs", CASES, ids=[c["name"] for c in CASES])
def test_mid_documents_match_reference(cs, build, monkeypatch):
    """The three builds of the global-mode k_doc must give the same documents and patches: four
    waves per SIMD, eight (AM_GLB8_MIN=0: every batch; by default batches of 1,024+ documents), and
    the 16-wave workgroup (AM_GLB16_MAX: by default batches of at most 8 documents)."""
    monkeypatch.setenv("AM_GLB16_MAX", "1000000" if build == "glb16" else "0")
    if build == "glb8":
        monkeypatch.setenv("AM_GLB8_MIN", "0")
    from automerge_amd import patch as P
    import workload as W
    from automerge_amd.batch import WANT_PATCH
    arena, chunks, docs, _ = W.mid(cs["first"], cs["n"], cs["nactors"], cs["rounds"], cs["min_ops"], cs["max_ops"])
    chg = [W.doc_chunks(arena, chunks, docs, i)[1] for i in range(cs["n"])]
    exp = cs["docs"]
    for c, e in zip(chg, exp):
        assert sha(b"".join(c)) == e["changes"] and len(c) == e["nchunks"]

    b, r = _run([(None, c) for c in chg], WANT_PATCH)
    for i, e in enumerate(exp):
        assert int(r[i]["status"]) == 0, (i, int(r[i]["status"]))
        assert sha(b.doc_save(i)) == e["full"]["save"], i
        heads = b.doc_heads(i, int(r[i]["nheads"]))
        assert heads == e["full"]["heads"], i
        assert jsha(_jsonable(P.materialize(b.doc_patch(i), heads, 0))) == e["full"]["getPatch"], i

    b, r = _run([(None, c[:e["split"]["half"]]) for c, e in zip(chg, exp)], 0)
    bases = []
    for i, e in enumerate(exp):
        assert int(r[i]["status"]) == 0, (i, int(r[i]["status"]))
        bases.append(b.doc_save(i))
        assert sha(bases[i]) == e["split"]["base"], i
    # load(base) + applyChanges(rest) through the batched per-handle calls: the split falls inside a
    # round, so the rest depends on changes that are not heads of the base and the loaded handles
    # compute their hash graph first (new.js:1826-1832)
    from automerge_amd import backend as B
    hs = B.loadBatch(bases)
    res = B.applyChangesBatch(hs, [c[e["split"]["half"]:] for c, e in zip(chg, exp)])
    pats = B.getPatchBatch([x[0] for x in res])
    for i, e in enumerate(exp):
        sp = e["split"]
        assert not isinstance(res[i], Exception), (i, res[i])
        st, patch = res[i]
        assert sha(B.save(st)) == sp["save"], i
        assert B.getHeads(st) == sp["heads"], i
        assert jsha(_jsonable(patch)) == sp["applyPatch"], i
        assert jsha(_jsonable(pats[i])) == sp["getPatch"], i
