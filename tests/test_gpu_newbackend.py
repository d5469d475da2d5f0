"""The reference's BackendDoc tests (test/new_backend_test.js: 40 cases, recorded by
tests/golden/gen/make_newbackend_log.js) replayed through automerge_amd.backend on the GPU: every
applyChanges patch and thrown error, and after every call the saved document bytes (which pin the op
columns checkColumns() asserts) and heads, as the reference produced them."""
import pytest

import newbackend_log as NB

pytestmark = pytest.mark.gpu


def test_new_backend_test_cases_replay_on_the_gpu():
    from automerge_amd import backend as B
    calls, bad = NB.replay(B)
    assert calls > 700
    assert bad == []
