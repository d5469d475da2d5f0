"""Text editing histories on the GPU (BASELINE configs[0], configs[2]):
long RGA histories with tombstones, two actors, deflated changes (host-staged, or inflated on the
device when the batch stages them raw). Every document runs through one batched launch and is
compared with tests/golden/text.json, which the reference backend produced from the same change
bytes (tests/golden/gen/make_text.js):

* full:  Backend.applyChanges(init(), all changes): save() bytes, heads, getPatch();
* split: base = save() of the first half (itself compared), then load(base) + applyChanges(rest):
         save() bytes, heads, getPatch() and the patch applyChanges returns.

The c3full case is configs[2]'s document size (100,001 ops, 1,001 changes per document)."""
import hashlib
import json
import os

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
CASES = json.load(open(os.path.join(HERE, "golden", "text.json")))


def sha(b):
    return hashlib.sha256(b).hexdigest()


def jsha(obj):
    return sha(json.dumps(obj, sort_keys=True, separators=(",", ":")).encode())


def _jsonable(x):
    if isinstance(x, (bytes, bytearray)):
        return {"__bytes": bytes(x).hex()}
    if isinstance(x, dict):
        return {k: _jsonable(v) for k, v in x.items()}
    if isinstance(x, list):
        return [_jsonable(v) for v in x]
    return x


def _run(docs, flags):
    from automerge_amd.batch import Batch
    b = Batch()
    b.stage_docs(docs, flags=flags)
    b.run()
    b.sync()
    return b, b.results()


@pytest.mark.parametrize("cs", CASES, ids=[c["name"] for c in CASES])
def test_text_history_matches_reference(cs):
    from automerge_amd import patch as P
    import workload as W
    from automerge_amd.batch import WANT_DIFF, WANT_PATCH
    arena, chunks, docs, _ = W.text(cs["first"], cs["n"], cs["nchanges"], cs["per_change"], cs["cross_every"])
    chg = [W.doc_chunks(arena, chunks, docs, i)[1] for i in range(cs["n"])]
    exp = cs["docs"]

    b, r = _run([(None, c) for c in chg], WANT_PATCH)
    for i, e in enumerate(exp):
        assert int(r[i]["status"]) == 0, (i, int(r[i]["status"]))
        assert sha(b.doc_save(i)) == e["full"]["save"], i
        heads = b.doc_heads(i, int(r[i]["nheads"]))
        assert heads == e["full"]["heads"], i
        assert jsha(_jsonable(P.materialize(b.doc_patch(i), heads, 0))) == e["full"]["getPatch"], i

    # base documents of the split (first half of every history) in one launch
    b, r = _run([(None, c[:e["split"]["half"]]) for c, e in zip(chg, exp)], 0)
    bases = []
    for i, e in enumerate(exp):
        assert int(r[i]["status"]) == 0, (i, int(r[i]["status"]))
        bases.append(b.doc_save(i))
        assert sha(bases[i]) == e["split"]["base"], i

    for flags in (WANT_PATCH, WANT_DIFF):
        b, r = _run([(base, c[e["split"]["half"]:]) for base, c, e in zip(bases, chg, exp)], flags)
        for i, e in enumerate(exp):
            sp = e["split"]
            assert int(r[i]["status"]) == 0, (i, int(r[i]["status"]))
            assert sha(b.doc_save(i)) == sp["save"], i
            heads = b.doc_heads(i, int(r[i]["nheads"]))
            assert heads == sp["heads"], i
            if flags == WANT_PATCH:
                got = P.materialize(b.doc_patch(i), heads, 0)
                assert jsha(_jsonable(got)) == sp["getPatch"], i
            else:
                got = P.materialize(b.doc_patch(i), heads, int(r[i]["nqueued"]), int(r[i]["max_op"]))
                assert jsha(_jsonable(got)) == sp["applyPatch"], i
