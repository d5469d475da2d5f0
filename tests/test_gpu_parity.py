"""Parity of the MI355X engine with the reference, on the GPU.

* every golden scenario (tests/golden/docs.json, produced by the reference JS backend) replayed
  through automerge_amd.backend: save() bytes, heads, pending count and error messages;
* the same scenarios packed into ONE batch launch;
* the C4 workload vectors (load + applyChanges of 12 concurrent changes);
* larger seeded batches checked against the CPU oracle (oracle/).
"""
import pytest

from conftest import golden
from docfmt import to_saved_form

pytestmark = pytest.mark.gpu


def replay(sc):
    from automerge_amd import _native as N
    from automerge_amd import backend as B
    st = None
    out = []
    for step in sc["steps"]:
        res = {}
        try:
            if step["op"] == "load":
                st = B.load(bytes.fromhex(step["bytes"]))
            else:
                if st is None:
                    st = B.init()
                st = B.loadChanges(st, [bytes.fromhex(c) for c in step["changes"]])
            res["save"] = B.save(st).hex()
            res["heads"] = B.getHeads(st)
            res["pending"] = B.pendingChanges(st)
        except N.AutomergeError as e:
            res["error"] = str(e)
            res["code"] = e.code
            out.append(res)
            break
        out.append(res)
    return out


def test_scenarios_per_document(docs):
    bad = []
    for sc in docs:
        got = replay(sc)
        for i, (exp, res) in enumerate(zip(sc["results"], got)):
            if "error" in exp:
                if res.get("error") != exp["error"]["message"]:
                    bad.append((sc["name"], i, "error", res.get("error"), exp["error"]["message"]))
                break
            if "error" in res:
                bad.append((sc["name"], i, "unexpected", res["error"]))
                break
            for k in ("heads", "pending", "save"):
                if res[k] != exp[k]:
                    bad.append((sc["name"], i, k))
                    break
    assert not bad, bad[:10]


def test_scenarios_one_batch(docs):
    """All single-apply scenarios (fresh and load+apply) merged by one launch."""
    from automerge_amd.batch import Batch
    items, expect = [], []
    for sc in docs:
        steps = sc["steps"]
        res = sc["results"]
        if len(steps) == 1 and steps[0]["op"] == "apply" and "error" not in res[0]:
            items.append((None, [bytes.fromhex(c) for c in steps[0]["changes"]]))
            expect.append(res[0])
        elif len(steps) == 2 and steps[0]["op"] == "load" and "error" not in res[-1]:
            items.append((bytes.fromhex(steps[0]["bytes"]), [bytes.fromhex(c) for c in steps[1]["changes"]]))
            expect.append(res[1])
    assert len(items) > 200
    b = Batch()
    b.stage_docs(items)
    b.run()
    b.sync()
    r = b.results()
    bad = []
    for i, exp in enumerate(expect):
        if r[i]["status"] != 0:
            bad.append((i, "status", int(r[i]["status"])))
            continue
        out = to_saved_form(b.doc_output(i, r[i]))
        if out.hex() != exp["save"]:
            bad.append((i, "save"))
        if b.doc_heads(i, int(r[i]["nheads"])) != exp["heads"]:
            bad.append((i, "heads"))
        if int(r[i]["nqueued"]) != exp["pending"]:
            bad.append((i, "pending"))
    assert not bad, bad[:10]


def test_workload_c4_vectors():
    from automerge_amd.batch import Batch
    w = golden("workload.json")["c4"]
    items = [(bytes.fromhex(v["baseBytes"]), [bytes.fromhex(c) for c in v["changeBytes"]]) for v in w if "baseBytes" in v]
    b = Batch()
    b.stage_docs(items)
    b.run()
    b.sync()
    r = b.results()
    for i, v in enumerate([v for v in w if "baseBytes" in v]):
        assert r[i]["status"] == 0
        assert r[i]["napplied"] == 12
        assert b.doc_output(i, r[i]).hex() == v["mergedBytes"]
        assert b.doc_heads(i, int(r[i]["nheads"])) == v["heads"]


def test_change_hashes():
    from automerge_amd import backend as B
    ch = golden("changes.json")
    good = [v for v in ch if not v.get("error")][:200]
    got = B.changeHashes([bytes.fromhex(v["bytes"]) for v in good])
    assert got == [v["hash"] for v in good]


def test_frozen_state():
    from automerge_amd import backend as B
    sc = [s for s in golden("docs.json")["scenarios"] if s["name"] == "concurrent-overwrite-order1"][0]
    s0 = B.init()
    s1, _ = B.applyChanges(s0, [bytes.fromhex(c) for c in sc["steps"][0]["changes"]])
    with pytest.raises(RuntimeError, match="outdated Automerge document"):
        B.save(s0)
    assert B.save(s1).hex() == sc["results"][0]["save"]


def _jsonable(x):
    if isinstance(x, (bytes, bytearray)):
        return {"__bytes": bytes(x).hex()}
    if isinstance(x, dict):
        return {k: _jsonable(v) for k, v in x.items()}
    if isinstance(x, list):
        return [_jsonable(v) for v in x]
    return x


def test_getpatch_per_step_matches_reference(docs):
    """Backend.getPatch() after every step (documentPatch on the GPU, k_doc phase P7) against the
    reference's getPatch of the same document state (tests/golden/docs.json)."""
    from automerge_amd import _native as N
    from automerge_amd import backend as B
    n, bad = 0, []
    for sc in docs:
        st = None
        for i, (step, exp) in enumerate(zip(sc["steps"], sc["results"])):
            if "error" in exp:
                break
            if step["op"] == "load":
                st = B.load(bytes.fromhex(step["bytes"]))
            else:
                if st is None:
                    st = B.init()
                st = B.loadChanges(st, [bytes.fromhex(c) for c in step["changes"]])
            want = dict(exp["getPatch"], pendingChanges=exp["pending"])
            try:
                got = _jsonable(B.getPatch(st))
            except N.AutomergeError as e:
                got = {"error": str(e)}
            n += 1
            if got != want:
                bad.append((sc["name"], i))
    assert n > 400
    assert not bad, bad[:10]


@pytest.mark.parametrize("kind,first,n", [("c4", 1000, 1500), ("c2", 77, 1500)])
def test_workload_batch_matches_oracle_and_digest(kind, first, n):
    """Seeded C4 / C2 batches (the bench's generator, am_workload.cpp): every merged document equals
    the CPU oracle's save(), and the device digest (am_batch_digest) equals the host restatement
    (shard.doc_digest) over the oracle's bytes."""
    import oracle_ffi as O
    from automerge_amd import shard
    import workload
    from automerge_amd.batch import Batch
    arena, chunks, docs, _ = getattr(workload, kind)(first, n)
    b = Batch()
    b.stage(arena, chunks, docs)
    b.run()
    b.sync()
    r = b.results()
    terms = []
    for i in range(n):
        base, changes = workload.doc_chunks(arena, chunks, docs, i)
        ref = O.Doc.load(base) if base else O.Doc.init()
        ref.apply(changes)
        want = ref.save()
        assert int(r[i]["status"]) == 0, (i, int(r[i]["status"]))
        assert b.doc_output(i, r[i]) == want, i
        terms.append(shard.doc_digest(first + i, 0, want))
    assert b.digest(first) == shard.combine(terms)


def test_fast_and_general_kernels_agree(docs):
    """Every single-apply golden scenario and a C4/C2 sample merged twice in one process: with the
    small-document kernel (k_doc_fast) and with it disabled (AM_FAST=0 at stage time, k_doc only).
    Outputs, heads and results must be identical, and the fast kernel must take the C4/C2 documents."""
    import os
    import workload
    from automerge_amd.batch import Batch
    items = []
    for sc in docs:
        steps = sc["steps"]
        if len(steps) == 1 and steps[0]["op"] == "apply":
            items.append((None, [bytes.fromhex(c) for c in steps[0]["changes"]]))
        elif len(steps) == 2 and steps[0]["op"] == "load":
            items.append((bytes.fromhex(steps[0]["bytes"]), [bytes.fromhex(c) for c in steps[1]["changes"]]))
    for kind in ("c4", "c2"):
        arena, chunks, dd, _ = getattr(workload, kind)(5, 300)
        items += [workload.doc_chunks(arena, chunks, dd, i) for i in range(300)]

    def run(fast):
        old = os.environ.get("AM_FAST")
        os.environ["AM_FAST"] = "1" if fast else "0"
        try:
            b = Batch()
            b.stage_docs(items)
        finally:
            if old is None:
                del os.environ["AM_FAST"]
            else:
                os.environ["AM_FAST"] = old
        b.run()
        b.sync()
        r = b.results()
        outs = [b.doc_output(i, r[i]) if r[i]["status"] == 0 else b"" for i in range(len(items))]
        heads = [b.doc_heads(i, int(r[i]["nheads"])) if r[i]["status"] == 0 else [] for i in range(len(items))]
        return r, outs, heads, b.fast_flags()

    rf, of, hf, flags = run(True)
    rg, og, hg, gflags = run(False)
    assert not gflags.any()
    nfast = int(flags.sum())
    assert flags[-600:].all(), "C4/C2 documents must take the fast kernel"
    bad = []
    for i in range(len(items)):
        for k in ("status", "err_change", "arg0", "arg1", "napplied", "nqueued", "nheads", "nops", "nchanges", "max_op",
                  "out_len"):
            if rf[i][k] != rg[i][k]:
                bad.append((i, k, int(rf[i][k]), int(rg[i][k]), bool(flags[i])))
        if of[i] != og[i]:
            bad.append((i, "bytes", bool(flags[i])))
        if hf[i] != hg[i]:
            bad.append((i, "heads", bool(flags[i])))
    assert not bad, (nfast, bad[:10])
    print("fast kernel merged %d of %d documents" % (nfast, len(items)))


def test_fast_kernel_split_launch_matches_single_launch():
    """AM_FAST_SPLIT (two k_doc_fast launches by LDS slice class: the documents whose slice fits the
    split first, with the smaller slice, then the rest) merges and patches every document exactly as
    one launch with the largest slice does, and the fast kernel still takes all of them."""
    import os
    import numpy as np
    import workload
    from automerge_amd import _native as N
    from automerge_amd.batch import WANT_DIFF, Batch
    items = []
    for kind in ("c4", "c2"):
        arena, chunks, dd, _ = getattr(workload, kind)(11, 400)
        items += [workload.doc_chunks(arena, chunks, dd, i) for i in range(400)]

    def run(split):
        b = Batch()
        b.stage_docs(items, flags=WANT_DIFF)
        sl = np.zeros(len(items), np.uint32)
        assert N.lib.am_batch_fast_slices(b._b, sl.ctypes.data) == 0
        old = os.environ.get("AM_FAST_SPLIT")
        if split is not None:
            os.environ["AM_FAST_SPLIT"] = str(split(sl))
        try:
            b.run()
            b.sync()
        finally:
            if old is None:
                os.environ.pop("AM_FAST_SPLIT", None)
            else:
                os.environ["AM_FAST_SPLIT"] = old
        r = b.results()
        outs = [b.doc_output(i, r[i]) for i in range(len(items))]
        pats = [b.doc_patch(i) for i in range(len(items))]
        return r, outs, pats, b.fast_flags(), sl

    r1, o1, p1, f1, sl = run(None)
    assert (sl > 0).all() and len(set(sl.tolist())) > 1
    r2, o2, p2, f2, _ = run(lambda s: int(np.median(s)) + 16)
    assert (r1["status"] == 0).all() and (r2["status"] == 0).all()
    assert f1.all() and f2.all()
    assert o1 == o2
    assert p1 == p2
