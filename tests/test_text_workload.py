"""Text editing histories (BASELINE configs[0] and configs[2] at test
sizes): the engine's generator (am_workload_text) against tests/golden/text.json, which the
reference backend produced from the same change bytes (tests/golden/gen/make_text.js), and the
CPU oracle against the reference's results. The GPU side is tests/test_gpu_text.py."""
import hashlib
import json
import os

import pytest

import oracle_ffi as O
import workload as W

HERE = os.path.dirname(os.path.abspath(__file__))
CASES = json.load(open(os.path.join(HERE, "golden", "text.json")))


def sha(b):
    return hashlib.sha256(b).hexdigest()


def jsha(obj):
    return sha(json.dumps(obj, sort_keys=True, separators=(",", ":")).encode())


def docs_of(cs):
    arena, chunks, docs, _ = W.text(cs["first"], cs["n"], cs["nchanges"], cs["per_change"], cs["cross_every"])
    return [W.doc_chunks(arena, chunks, docs, i)[1] for i in range(cs["n"])]


@pytest.mark.parametrize("cs", CASES, ids=[c["name"] for c in CASES])
def test_generator_pinned(cs):
    for chg, exp in zip(docs_of(cs), cs["docs"]):
        assert len(chg) == exp["nchunks"]
        assert sha(b"".join(chg)) == exp["changes"]
        assert sum(c[8] == 2 for c in chg) == exp["deflated"]


@pytest.mark.parametrize("cs", [c for c in CASES if c["n"] * c["nchanges"] * c["per_change"] <= 20000],
                         ids=lambda c: c["name"])
def test_oracle_text(cs):
    for chg, exp in zip(docs_of(cs), cs["docs"]):
        d = O.Doc.init()
        d.apply(chg)
        full = d.save()
        assert sha(full) == exp["full"]["save"]
        assert d.heads() == exp["full"]["heads"]
        assert jsha(d.patch()) == exp["full"]["getPatch"]
        sp = exp["split"]
        h = sp["half"]
        b = O.Doc.init()
        b.apply(chg[:h])
        base = b.save()
        assert sha(base) == sp["base"]
        d2 = O.Doc.load(base)
        patch = d2.apply_patch(chg[h:])
        assert sha(d2.save()) == sp["save"]
        assert d2.heads() == sp["heads"]
        assert jsha(d2.patch()) == sp["getPatch"]
        assert jsha(patch) == sp["applyPatch"]
