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
