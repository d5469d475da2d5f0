"""Change history of a saved document (computeHashGraph new.js:1879-1904 =
decodeDocument + groupChangeOps + decodeDocumentChanges + encodeChange, columnar.js:876-981, 710):
am_document_changes against Backend.getAllChanges(Backend.load(saved)) as the reference returns it
for every saved document of the golden scenarios and for text histories with deflated columns and
deflated changes (tests/golden/history.json, tests/golden/gen/make_history.js). Host stage: runs
without a GPU."""
import json
import os

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def test_document_changes_match_reference():
    from automerge_amd import _native as N
    cases = json.load(open(os.path.join(HERE, "golden", "history.json")))
    assert len(cases) > 300
    nchg = 0
    for i, c in enumerate(cases):
        got = N.document_changes(bytes.fromhex(c["doc"]))
        assert [b.hex() for b, _ in got] == c["changes"], i
        nchg += len(got)
    assert nchg > 3000


def test_document_changes_hashes_are_change_hashes():
    import oracle_ffi as O
    from automerge_amd import _native as N
    cases = json.load(open(os.path.join(HERE, "golden", "history.json")))
    for c in cases[::25]:
        for b, h in N.document_changes(bytes.fromhex(c["doc"])):
            assert O.change_meta(b)["hash"] == h


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
