"""The bench's synthetic workload generator (automerge_amd/csrc/am_workload.cpp) reproduces the
bytes the reference's own encoder produced for the same seeded specification (CPU-only)."""
import hashlib

from conftest import golden


def sha(b):
    return hashlib.sha256(b).hexdigest()


def test_c4_generator_matches_reference_encoder():
    import workload
    w = golden("workload.json")["c4"]
    arena, chunks, docs, ops = workload.c4(0, len(w))
    assert ops == 60 * len(w)
    for i, v in enumerate(w):
        base, changes = workload.doc_chunks(arena, chunks, docs, i)
        assert sha(base) == v["base"], i
        assert [sha(c) for c in changes] == v["changes"], i


def test_c4_generator_is_deterministic_across_ranges():
    import workload
    a1, c1, d1, _ = workload.c4(100, 8, nthreads=1)
    a2, c2, d2, _ = workload.c4(96, 16, nthreads=4)
    for i in range(8):
        assert workload.doc_chunks(a1, c1, d1, i) == workload.doc_chunks(a2, c2, d2, i + 4)


def test_c4_oracle_merge_of_generated_docs():
    import oracle_ffi as O
    import workload
    w = golden("workload.json")["c4"]
    arena, chunks, docs, _ = workload.c4(0, 16)
    for i in range(16):
        base, changes = workload.doc_chunks(arena, chunks, docs, i)
        doc = O.Doc.load(base)
        doc.apply(changes)
        assert sha(doc.save()) == w[i]["merged"]
        assert doc.heads() == w[i]["heads"]


def test_c2_generator_matches_reference_encoder():
    import workload
    w = golden("workload.json")["c2"]
    arena, chunks, docs, ops = workload.c2(0, len(w))
    assert ops == 14 * len(w)
    for i, v in enumerate(w):
        base, changes = workload.doc_chunks(arena, chunks, docs, i)
        assert base is None
        assert [sha(c) for c in changes] == v["changes"], i


def test_c2_oracle_merge_and_getpatch_of_generated_docs():
    """init + applyChanges of the generated changes gives the reference's saved document, whose
    getPatch (documentPatch) the oracle reproduces."""
    import json
    import oracle_ffi as O
    import workload
    w = golden("workload.json")["c2"]
    arena, chunks, docs, _ = workload.c2(0, 16)
    for i in range(16):
        _, changes = workload.doc_chunks(arena, chunks, docs, i)
        doc = O.Doc.init()
        doc.apply(changes)
        saved = doc.save()
        assert sha(saved) == w[i]["doc_sha"]
        if w[i].get("getPatch"):
            assert O.Doc.load(saved).patch() == json.loads(json.dumps(w[i]["getPatch"]))
