"""Change history of saved documents (computeHashGraph new.js:1879-1904 =
decodeDocument + groupChangeOps + decodeDocumentChanges + encodeChange, columnar.js:876-981, 710),
batched on the GPU (k_history, am_document_changes_batch):
- against Backend.getAllChanges(Backend.load(saved)) as the reference returns it for every saved
  document of the golden scenarios and for text histories with deflated columns and deflated
  changes (tests/golden/history.json, tests/golden/gen/make_history.js);
- against concurrent multi-actor histories and the RangeErrors of groupChangeOps /
  decodeDocumentChanges on mutated documents (tests/golden/history_cases.json,
  tests/golden/gen/make_history_cases.js: decodeChanges + encodeChange run straight on the bytes,
  and getAllChanges after load where load accepts them)."""
import json
import os

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def _load(name):
    return json.load(open(os.path.join(HERE, "golden", name)))


def test_history_fixtures_shape():
    """The fixtures hold what the GPU tests below rely on: enough documents and changes, valid
    concurrent histories, and every history RangeError kind of columnar.js:876-981."""
    cases = _load("history.json")
    assert len(cases) > 300 and sum(len(c["changes"]) for c in cases) > 3000
    hc = _load("history_cases.json")
    for c in hc:
        assert (c["direct"] is None) != (c["direct_error"] is None), c["name"]
    errs = " | ".join(c["direct_error"] for c in hc if c["direct_error"])
    for kind in ("Expected seq = ", "maxOp must increase", "outside of allowed range", "No hash for index",
                 "Mismatched heads hashes", "Bad datatype for extra bytes", "document should not contain del"):
        assert kind in errs, kind
    assert sum(1 for c in hc if c["direct"] and c["name"].startswith("concurrent")) >= 7


@pytest.mark.gpu
def test_document_changes_match_reference():
    """All 359 documents in ONE batch (one workgroup per document)."""
    from automerge_amd import _native as N
    cases = _load("history.json")
    got = N.document_changes_batch([bytes.fromhex(c["doc"]) for c in cases])
    nchg = 0
    for i, (c, g) in enumerate(zip(cases, got)):
        assert not isinstance(g, Exception), (i, g)
        assert [b.hex() for b, _ in g] == c["changes"], i
        nchg += len(g)
    assert nchg > 3000


@pytest.mark.gpu
def test_document_changes_hashes_are_change_hashes():
    import oracle_ffi as O
    from automerge_amd import _native as N
    cases = _load("history.json")
    for c in cases[::25]:
        for b, h in N.document_changes(bytes.fromhex(c["doc"])):
            assert O.change_meta(b)["hash"] == h


@pytest.mark.gpu
def test_document_changes_cases():
    """Concurrent histories (parallel branches hash in the same round) and every RangeError of the
    history decode, batched; each document's result matches decodeChanges + encodeChange."""
    from automerge_amd import _native as N
    hc = _load("history_cases.json")
    got = N.document_changes_batch([bytes.fromhex(c["doc"]) for c in hc])
    for c, g in zip(hc, got):
        if c["direct_error"] is not None:
            assert isinstance(g, Exception), c["name"]
            assert str(g) == c["direct_error"], c["name"]
            assert g.kind == "RangeError", c["name"]
        else:
            assert not isinstance(g, Exception), (c["name"], g)
            assert [b.hex() for b, _ in g] == c["direct"], c["name"]


@pytest.mark.gpu
def test_document_changes_singly_equals_batched():
    """A document's history does not depend on the batch it runs in."""
    from automerge_amd import _native as N
    hc = _load("history_cases.json")
    docs = [bytes.fromhex(c["doc"]) for c in hc[:12]]
    batched = N.document_changes_batch(docs)
    for d, b in zip(docs, batched):
        s = N.document_changes_batch([d])[0]
        assert type(s) is type(b)
        if not isinstance(s, Exception):
            assert s == b


@pytest.mark.gpu
def test_get_all_changes_after_load_cases():
    """Backend.load + getAllChanges through the drop-in mirror where the reference's load accepts the
    document: the changes, or the RangeError getAllChanges throws."""
    from automerge_amd import backend as B
    from automerge_amd._native import AutomergeError
    for c in _load("history_cases.json"):
        if c["load_error"] is not None:
            continue
        st = B.load(bytes.fromhex(c["doc"]))
        if c["error"] is not None:
            with pytest.raises(AutomergeError) as ei:
                B.getAllChanges(st)
            assert str(ei.value) == c["error"], c["name"]
        else:
            assert [b.hex() for b in B.getAllChanges(st)] == c["changes"], c["name"]


@pytest.mark.gpu
def test_backend_get_all_changes_after_load():
    """Backend.load + getAllChanges / getChangeByHash through the drop-in mirror (the loaded state
    reconstructs its hash graph on first use, as computeHashGraph does)."""
    from automerge_amd import backend as B
    cases = json.load(open(os.path.join(HERE, "golden", "history.json")))
    for c in cases[::7]:
        st = B.load(bytes.fromhex(c["doc"]))
        got = [b.hex() for b in B.getAllChanges(st)]
        assert got == c["changes"]
        if got:
            from automerge_amd import _native as N
            h = N.document_changes(bytes.fromhex(c["doc"]))[-1][1]
            assert B.getChangeByHash(st, h).hex() == got[-1]


@pytest.mark.gpu
def test_apply_change_depending_on_history_of_loaded_document():
    """A change whose dependency is a non-head change of a loaded document: the loaded state only
    knows its heads, so applyChanges computes the hash graph and retries (new.js:1826-1832)."""
    import oracle_ffi as O
    from automerge_amd import backend as B
    import workload as W
    arena, chunks, docs, _ = W.text(3, 1, 6, 5, 0)  # two actors that never meet: B's deps = [change 0]
    _, chg = W.doc_chunks(arena, chunks, docs, 0)
    ref = O.Doc.init()
    ref.apply(chg[:2])                                # change 0 (A) + change 1 (A): heads = {change 1}
    base = ref.save()
    st = B.load(base)
    st, _ = B.applyChanges(st, [chg[2]])              # change 2 (B) depends on change 0 only
    # the oracle does not restate computeHashGraph; the reference's load(base) + applyChanges([c2])
    # saves the same bytes as init + apply([c0, c1]) + apply([c2]) (checked under Node when this
    # test was written)
    want = O.Doc.init()
    want.apply(chg[:2])
    want.apply([chg[2]])
    assert B.save(st) == want.save()
    assert B.getHeads(st) == want.heads()
    assert len(B.getAllChanges(st)) == 3


@pytest.mark.gpu
def test_backend_hash_graph_queries():
    """getChanges(haveDeps) / getChangesAdded / getMissingDeps of the Python mirror (new.js:1913-2020)
    on two concurrent chains, loaded from save() (history reconstructed) and freshly applied."""
    from automerge_amd import backend as B
    import workload as W
    arena, chunks, docs, _ = W.text(9, 1, 8, 4, 0)  # change 0, then A and B alternate, never meeting
    _, chg = W.doc_chunks(arena, chunks, docs, 0)
    hashes = B.changeHashes(chg)
    st, _ = B.applyChanges(B.init(), chg)
    loaded = B.load(B.save(st))
    for s in (st, loaded):
        assert B.getChanges(s, []) == B.getAllChanges(s)
        assert B.getChanges(s, B.getHeads(s)) == []
        assert B.getMissingDeps(s) == []
        # A's changes are 1, 3, 5, 7: everything except change 0 and A's chain is concurrent to A's head
        got = B.getChanges(s, [hashes[7]])
        assert sorted(B.changeHashes(got)) == sorted(hashes[k] for k in (2, 4, 6, 8))
    part, _ = B.applyChanges(B.init(), chg[:4])
    assert sorted(B.changeHashes(B.getChangesAdded(part, st))) == sorted(hashes[4:])
    q, _ = B.applyChanges(B.init(), [chg[0], chg[3]])  # change 3 waits for change 1
    assert B.getMissingDeps(q) == [hashes[1]]
