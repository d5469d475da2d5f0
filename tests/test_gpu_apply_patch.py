"""The patch Backend.applyChanges returns (new.js:1796-1871), replayed on the GPU
(k_doc phase P8, automerge_amd/csrc/am_diff.h) and materialized by automerge_amd/patch.py.

* every apply step of every golden scenario through automerge_amd.backend.applyChanges, against
  the reference's own patch (tests/golden/docs.json, produced by the reference);
* the same steps as ONE batch launch (base = the step's previous saved state, the form the per-
  document API hands the GPU), against the reference's patches;
* seeded C4 / C2 batches (the bench's generator) against the CPU oracle's applyChanges patch
  (oracle/am_apply_patch_oracle.inc, itself pinned by tests/test_apply_patch_oracle.py).
"""
import pytest

pytestmark = pytest.mark.gpu


def _jsonable(x):
    if isinstance(x, (bytes, bytearray)):
        return {"__bytes": bytes(x).hex()}
    if isinstance(x, dict):
        return {k: _jsonable(v) for k, v in x.items()}
    if isinstance(x, list):
        return [_jsonable(v) for v in x]
    return x


def test_apply_patch_per_step_matches_reference(docs):
    from automerge_amd import _native as N
    from automerge_amd import backend as B
    n, bad = 0, []
    for sc in docs:
        st = None
        for i, (step, exp) in enumerate(zip(sc["steps"], sc["results"])):
            if step["op"] == "load":
                st = B.load(bytes.fromhex(step["bytes"]))
                continue
            if st is None:
                st = B.init()
            try:
                st, patch = B.applyChanges(st, [bytes.fromhex(c) for c in step["changes"]])
                got = _jsonable(patch)
            except N.AutomergeError as e:
                got = {"error": str(e)}
            if "error" in exp:
                if got.get("error") != exp["error"]["message"]:
                    bad.append((sc["name"], i, "error", got.get("error")))
                break
            n += 1
            if got != exp["patch"]:
                bad.append((sc["name"], i, got.get("error")))
                break
    assert n > 300
    assert not bad, (len(bad), bad[:10])


def _replay_handle(sc, loadchanges_every=0):
    """One backend handle through the scenario's steps; yields (step, expected, got patch, saved hex,
    heads). With loadchanges_every = k, every k-th apply step goes through loadChanges (no patch;
    objectMeta moves on all the same, backend.js:116-121)."""
    from automerge_amd import _native as N
    from automerge_amd import backend as B
    st = None
    napply = 0
    for i, (step, exp) in enumerate(zip(sc["steps"], sc["results"])):
        if step["op"] == "load":
            st = B.load(bytes.fromhex(step["bytes"]))
            continue
        if st is None:
            st = B.init()
        napply += 1
        changes = [bytes.fromhex(c) for c in step["changes"]]
        try:
            if loadchanges_every and napply % loadchanges_every == 0:
                st, got = B.loadChanges(st, changes), None
            else:
                st, patch = B.applyChanges(st, changes)
                got = _jsonable(patch)
        except N.AutomergeError as e:
            got = {"error": str(e)}
        yield i, exp, got, (B.save(st).hex() if not (got and "error" in got) else None), \
            (B.getHeads(st) if not (got and "error" in got) else None)
        if got and "error" in got:
            return


@pytest.mark.parametrize("every", [0, 3])
def test_apply_patch_objectmeta_across_calls(objmeta, every):
    """objectMeta's children snapshots carried from call to call on one handle (new.js:884-931,
    1461-1528, 1812/1857): concurrent same-key makeMap / makeList / makeText from 2-4 actors with
    other-key edits, delivered in several calls (tests/golden/objmeta.json, recorded from the
    reference). Every patch, saved document and heads after every step match the reference's; with
    every=3 each third call is a loadChanges, which must move objectMeta on as well."""
    n, bad = 0, []
    for sc in objmeta:
        for i, exp, got, saved, heads in _replay_handle(sc, every):
            if "error" in exp:
                if not got or got.get("error") != exp["error"]["message"]:
                    bad.append((sc["name"], i, "error", got))
                break
            n += 1
            if got is not None and got != exp["patch"]:
                bad.append((sc["name"], i, "patch", (got or {}).get("error")))
                break
            if saved != exp["save"] or heads != exp["heads"]:
                bad.append((sc["name"], i, "save/heads"))
                break
    assert n > 600
    assert not bad, (len(bad), bad[:10])


def _steps(docs):
    """(base saved bytes | None, changes, expected patch) of every apply step whose previous state
    had no queued changes."""
    out = []
    for sc in docs:
        prev = None
        for step, exp in zip(sc["steps"], sc["results"]):
            if "error" in exp:
                break
            if step["op"] == "apply" and "patch" in exp and not (prev and prev.get("pending")):
                base = bytes.fromhex(prev["save"]) if prev else None
                out.append((base, [bytes.fromhex(c) for c in step["changes"]], exp))
            prev = exp
    return out


def test_apply_patch_one_batch_matches_reference(docs):
    from automerge_amd import patch as P
    from automerge_amd.batch import WANT_DIFF, Batch
    steps = _steps(docs)
    b = Batch()
    b.stage_docs([(base, ch) for base, ch, _ in steps], flags=WANT_DIFF)
    b.run()
    b.sync()
    res = b.results()
    bad = []
    for i, (_, _, exp) in enumerate(steps):
        assert int(res[i]["status"]) == 0, (i, int(res[i]["status"]))
        got = _jsonable(P.materialize(b.doc_patch(i), exp["heads"], exp["pending"], exp["patch"]["maxOp"]))
        if got != exp["patch"]:
            bad.append(i)
    assert len(steps) > 300
    assert not bad, (len(bad), bad[:10])


@pytest.mark.parametrize("kind,first,n", [("c4", 3000, 400), ("c2", 500, 400)])
def test_workload_apply_patch_matches_oracle(kind, first, n):
    import oracle_ffi as O
    from automerge_amd import patch as P
    import workload
    from automerge_amd.batch import WANT_DIFF, Batch
    arena, chunks, docs, _ = getattr(workload, kind)(first, n)
    docs = docs.copy()
    docs["flags"] |= WANT_DIFF
    b = Batch()
    b.stage(arena, chunks, docs)
    b.run()
    b.sync()
    r = b.results()
    for i in range(n):
        base, changes = workload.doc_chunks(arena, chunks, docs, i)
        ref = O.Doc.load(base) if base else O.Doc.init()
        want = ref.apply_patch(changes)
        assert int(r[i]["status"]) == 0, (i, int(r[i]["status"]))
        got = _jsonable(P.materialize(b.doc_patch(i), want["deps"], want["pendingChanges"], want["maxOp"]))
        assert got == want, i


def _first_steps(scenarios):
    """(base saved bytes | None, changes, expected) of the first apply step of each scenario (after
    init or load, objectMeta is documentPatch's, so the step stands alone as a batch document)."""
    out = []
    for sc in scenarios:
        prev = None
        for step, exp in zip(sc["steps"], sc["results"]):
            if step["op"] == "load":
                prev = exp
                continue
            if "patch" in exp and not (prev and prev.get("pending")):
                base = bytes.fromhex(prev["save"]) if prev else None
                out.append((base, [bytes.fromhex(c) for c in step["changes"]], exp, sc["name"]))
            break
    return out


def test_apply_patch_first_calls_one_batch(objmeta):
    """The first applyChanges of every objmeta scenario as one batch (k_doc_fast's wave-parallel
    patch writer where the shape allows, k_doc's replay otherwise) against the reference: concurrent
    same-key objects, one change over several root keys (the doc ops of an earlier key past the
    change's op are not in the patch, new.js:1125-1128, 1225-1230), concurrent counter increments
    in both actor orders (new.js:937-965)."""
    from automerge_amd import patch as P
    from automerge_amd.batch import WANT_DIFF, Batch
    steps = _first_steps(objmeta)
    b = Batch()
    b.stage_docs([(base, ch) for base, ch, _, _ in steps], flags=WANT_DIFF)
    b.run()
    b.sync()
    res = b.results()
    flags = b.fast_flags()
    bad, graph = [], 0
    for i, (_, _, exp, name) in enumerate(steps):
        if int(res[i]["status"]) == 100:  # AM_U_HASH_GRAPH: deps below the loaded heads (per-document path)
            graph += 1
            continue
        assert int(res[i]["status"]) == 0, (name, int(res[i]["status"]))
        got = _jsonable(P.materialize(b.doc_patch(i), exp["heads"], exp["pending"], exp["patch"]["maxOp"]))
        if got != exp["patch"]:
            bad.append((name, bool(flags[i])))
    fast_hand = [bool(flags[i]) for i, s in enumerate(steps) if s[3].startswith(("multikey/", "counter/"))]
    assert len(steps) - graph > 100 and sum(fast_hand) >= 4, (graph, fast_hand)
    assert not bad, (len(bad), bad[:10])


def test_fast_and_general_patch_writers_agree(docs, objmeta):
    """The wave-parallel patch writer of k_doc_fast (fast_diff, am_doc_fast.h) against k_doc's serial
    replay (am_diff.h): every golden apply step and seeded C4 / C2 documents staged with WANT_DIFF,
    once with the fast kernel and once without it (AM_FAST=0); the materialized patches must be
    equal, and the fast writer must take every C4 document (the bench's shape)."""
    import os
    from automerge_amd import patch as P
    import workload
    from automerge_amd.batch import WANT_DIFF, Batch
    items = [(base, ch) for base, ch, _ in _steps(docs)] + [(base, ch) for base, ch, _, _ in _first_steps(objmeta)]
    nc4 = 600
    for kind, first in (("c4", 11), ("c2", 7)):
        arena, chunks, dd, _ = getattr(workload, kind)(first, nc4)
        items += [workload.doc_chunks(arena, chunks, dd, i) for i in range(nc4)]

    def run(fast):
        old = os.environ.get("AM_FAST")
        os.environ["AM_FAST"] = "1" if fast else "0"
        try:
            b = Batch()
            b.stage_docs(items, flags=WANT_DIFF)
        finally:
            if old is None:
                del os.environ["AM_FAST"]
            else:
                os.environ["AM_FAST"] = old
        b.run()
        b.sync()
        r = b.results()
        pats = [_jsonable(P.materialize(b.doc_patch(i), [], 0, 0)) if r[i]["status"] == 0 else None
                for i in range(len(items))]
        outs = [b.doc_output(i, r[i]) if r[i]["status"] == 0 else b"" for i in range(len(items))]
        return r, pats, outs, b.fast_flags()

    rf, pf, of, flags = run(True)
    rg, pg, og, gflags = run(False)
    assert not gflags.any()
    assert flags[-2 * nc4:-nc4].all(), "every C4 document must take the fast patch writer"
    assert flags[-nc4:].all(), "every C2 document (counters) must take the fast patch writer"
    bad = [i for i in range(len(items)) if pf[i] != pg[i] or of[i] != og[i] or rf[i]["status"] != rg[i]["status"]]
    assert not bad, (int(flags.sum()), bad[:10])
    print("fast patch writer took %d of %d documents" % (int(flags.sum()), len(items)))


def test_fast_and_general_getpatch_writers_agree(docs, objmeta):
    """getPatch logs (documentPatch, new.js:1604-1635) from k_doc_fast's wave-parallel writer
    (fast_getpatch, am_doc_fast.h) against k_doc's serial patch_scan (P7, am_patch.h): every saved
    golden state and seeded C4 / C2 documents merged and staged with WANT_PATCH, once with the fast
    kernel and once without it (AM_FAST=0). Logs, merged documents and statuses must be equal, and
    the fast writer must take every C4 and C2 document."""
    import os
    from automerge_amd import patch as P
    import workload
    from automerge_amd.batch import WANT_PATCH, Batch
    items = []
    for sc in docs + objmeta:
        for res in sc["results"]:
            if "save" in res:
                items.append((bytes.fromhex(res["save"]), []))
    nw = 600
    for kind, first in (("c4", 21), ("c2", 9)):
        arena, chunks, dd, _ = getattr(workload, kind)(first, nw)
        items += [workload.doc_chunks(arena, chunks, dd, i) for i in range(nw)]

    def run(fast):
        old = os.environ.get("AM_FAST")
        os.environ["AM_FAST"] = "1" if fast else "0"
        try:
            b = Batch()
            b.stage_docs(items, flags=WANT_PATCH)
        finally:
            if old is None:
                del os.environ["AM_FAST"]
            else:
                os.environ["AM_FAST"] = old
        b.run()
        b.sync()
        r = b.results()
        pats = [_jsonable(P.materialize(b.doc_patch(i), [], 0)) if r[i]["status"] == 0 else None for i in range(len(items))]
        outs = [b.doc_output(i, r[i]) if r[i]["status"] == 0 else b"" for i in range(len(items))]
        return r, pats, outs, b.fast_flags()

    rf, pf, of, flags = run(True)
    rg, pg, og, gflags = run(False)
    assert not gflags.any()
    assert flags[-2 * nw:-nw].all(), "every C4 document must take the fast getPatch writer"
    assert flags[-nw:].all(), "every C2 document (counters) must take the fast getPatch writer"
    bad = [i for i in range(len(items)) if pf[i] != pg[i] or of[i] != og[i] or rf[i]["status"] != rg[i]["status"]]
    assert not bad, (int(flags.sum()), bad[:10])
    print("fast getPatch writer took %d of %d documents" % (int(flags.sum()), len(items)))


def test_meta_handles_take_the_fast_kernel():
    """Per-handle calls carry objectMeta (AM_DOC_META) and still run on k_doc_fast: C4 documents
    loaded as handles, their 12 changes applied in two applyChangesBatch calls (the first starts from
    documentPatch's snapshots, the second from the blob the first left). Patches, saved documents and
    heads equal the general kernel's (AM_FAST=0, whose replay is pinned to the reference), and most
    documents take the fast kernel."""
    import os
    import workload
    from automerge_amd import _native as N
    from automerge_amd import backend as B
    arena, chunks, docs, _ = workload.c4(100, 400)
    items = [workload.doc_chunks(arena, chunks, docs, i) for i in range(len(docs))]

    def run(fast):
        old = os.environ.get("AM_FAST")
        os.environ["AM_FAST"] = "1" if fast else "0"
        try:
            N.engine_stats()
            hs = B.loadBatch([base for base, _ in items])
            r1 = B.applyChangesBatch(hs, [ch[:6] for _, ch in items])
            r2 = B.applyChangesBatch([r[0] for r in r1], [ch[6:] for _, ch in items])
            st = N.engine_stats()
        finally:
            if old is None:
                del os.environ["AM_FAST"]
            else:
                os.environ["AM_FAST"] = old
        out = []
        for a, b in zip(r1, r2):
            assert not isinstance(a, Exception) and not isinstance(b, Exception), (a, b)
            out.append((_jsonable(a[1]), _jsonable(b[1]), B.save(b[0]).hex(), B.getHeads(b[0])))
        return out, st

    fast, st_fast = run(True)
    slow, st_slow = run(False)
    assert st_slow[1] == 0
    assert st_fast[0] >= 2 * len(items) and st_fast[1] >= 0.9 * 2 * len(items), st_fast
    bad = [i for i, (a, b) in enumerate(zip(fast, slow)) if a != b]
    assert not bad, (len(bad), bad[:10])
