"""Workspace bounds on the GPU: every kernel writes only inside the workspace plan k_bounds gave its
document. Round 5 found a 16-byte overrun of the applyChanges-patch scratch into the next
document's workspace on mid-size documents (an illegal address at 8,192 documents, fixed by sizing
the region with the function that binds it); these runs guard it with canary bytes after the
workspace (AM_DEBUG_WS_CANARY: filled with 0xA5 before the run, checked after it):

* >= 2,048 mid-size documents staged with WANT_DIFF (global-mode k_doc + k_diff);
* C5 document pairs staged with WANT_DIFF (LDS-mode k_doc + k_diff);
* a pipeline slot whose fast-kernel documents fall back into the overflow region (k_rest).
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

CANARY = 1 << 20


class _canary:
    def __enter__(self):
        self.old = os.environ.get("AM_DEBUG_WS_CANARY")
        os.environ["AM_DEBUG_WS_CANARY"] = str(CANARY)

    def __exit__(self, *a):
        if self.old is None:
            del os.environ["AM_DEBUG_WS_CANARY"]
        else:
            os.environ["AM_DEBUG_WS_CANARY"] = self.old


def _batch_canary(arena, chunks, docs):
    from automerge_amd import _native as N
    from automerge_amd.batch import Batch
    b = Batch()
    b.stage(arena, chunks, docs)
    with _canary():
        b.run()
    b.sync()
    return b, int(N.lib.am_batch_ws_canary(b._b, CANARY))


@pytest.mark.parametrize("kind,n", [("mid", 2048), ("c5", 4096)])
def test_patch_batches_stay_inside_their_workspace(kind, n):
    import workload as W
    from automerge_amd.batch import WANT_DIFF
    arena, chunks, docs, _ = getattr(W, kind)(0, n)
    docs = docs.copy()
    docs["flags"] |= WANT_DIFF
    b, off = _batch_canary(arena, chunks, docs)
    st = b.results()["status"]
    assert (st == 0).all(), np.unique(st, return_counts=True)
    assert off == -1, "a kernel wrote %d bytes past the batch workspace" % off


def test_pipeline_overflow_region_stays_inside_the_slot():
    from test_gpu_pipe import _parts
    from automerge_amd import _native as N
    from automerge_amd import pipe
    from automerge_amd.batch import WANT_DIFF, Batch
    (a, c, d), _ = _parts("c4", 0, 600, 600, WANT_DIFF)
    a = a.copy()
    bad = list(range(3, 600, 37))
    for i in bad:  # a wrong checksum: k_doc_fast gives up, k_rest re-plans the document in the overflow
        ch = c[int(d[i]["chg_begin"]) + 1]
        a[int(ch["off"]) + int(ch["len"]) - 1] ^= 0x5A
    ref = Batch()
    ref.stage(a, c, d)
    kinfo = ref.kernel_info()
    plan = int(ref.workspace_plan())
    pa, pc, pd = pipe.pinned_copy(a), pipe.pinned_copy(c), pipe.pinned_copy(d)
    with _canary():
        pl = pipe.Pipeline(len(a), len(c), len(d), plan + plan // 8 + (8 << 20), 1 << 20, 4 << 20,
                           kinfo["k_doc_fast_lds_per_doc"], slots=2)
    s = pipe.Pinned(len(d) * pipe.SUMMARY_DT.itemsize)
    po, pp = pipe.Pinned(1 << 20), pipe.Pinned(4 << 20)
    sm = s.view(pipe.SUMMARY_DT, len(d))
    for _ in range(3):
        pl.submit(pa.arr, pc.arr, pd.arr, sm, po.u8, pp.u8)
    pl.drain(3)
    assert all(int(sm[i]["status"]) != 0 for i in bad)
    assert (np.delete(sm["status"], bad) == 0).all()
    assert int(N.lib.am_pipe_ws_canary(pl._p)) == -1
