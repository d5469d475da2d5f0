"""Text-history throughput on one MI355X (BASELINE configs[2] = SURVEY.md §8(d) C3: 1k text
documents with 100k-op interleaved editing histories; --cross 0 --docs 1 --changes 100 gives C1).

Each document is Backend.load(base) + Backend.applyChanges(rest): base = save() of the first half
of the history (made by the engine in an untimed preparation launch), rest = the second half as
compressed (type 2) change chunks, exactly as encodeChange writes them. `value` times the whole job
from host memory per step: the batched stage of the saved base documents (their DEFLATEd columns
inflated on the GPU in one am_stage_documents call), H2D of the chunks, the GPU DEFLATE inflate of
the compressed changes and the GPU pipeline (SHA-256 + parse, causal queue, decode, merge, re-encode, checksums) over all
documents; `kernel_resident_ops_per_s` repeats the pipeline alone on the staged inputs. Also
reported: the k_doc time of one document's applyChanges patch (WANT_DIFF, 50k ops onto 50k). Documents 0 and 1
are checked against the reference backend's own digests (tests/golden/text.json, c3full) when the
configuration matches; the rest against the engine's own second run (determinism).

  python tools/bench_text.py [--docs 1000] [--changes 1000] [--per-change 100] [--cross 10] [--steps 3]
"""
import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", type=int, default=1000)
    ap.add_argument("--changes", type=int, default=1000)
    ap.add_argument("--per-change", type=int, default=100)
    ap.add_argument("--cross", type=int, default=10)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--cpu-baseline", action="store_true", help="time the oracle on document 0 (load + apply)")
    args = ap.parse_args()
    import workload as W
    from automerge_amd.batch import Batch, pack

    t0 = time.perf_counter()
    arena, chunks, docs, _ = W.text(0, args.docs, args.changes, args.per_change, args.cross)
    hist = [W.doc_chunks(arena, chunks, docs, i)[1] for i in range(args.docs)]
    half = (1 + args.changes) // 2
    gen_s = time.perf_counter() - t0
    print("generated %d docs in %.1f s" % (args.docs, gen_s), flush=True)

    # preparation (untimed): base documents = save() of the first half of every history
    t0 = time.perf_counter()
    prep = Batch()
    prep.stage(*pack([(None, h[:half]) for h in hist]))
    prep.run()
    prep.sync()
    r = prep.results()
    assert (r["status"] == 0).all(), "preparation failed"
    bases = [prep.doc_save(i) for i in range(args.docs)]
    del prep
    print("bases ready in %.1f s (%.1f MB)" % (time.perf_counter() - t0, sum(map(len, bases)) / 1e6), flush=True)

    rest = [h[half:] for h in hist]
    ops_applied = sum(args.per_change for h in rest for _ in h)
    # the saved base documents as they are (DEFLATEd columns) and the compressed change chunks: the
    # batch stage inflates both on the GPU
    arena2, chunks2, docs2 = pack(list(zip(bases, rest)))
    b = Batch()
    t0 = time.perf_counter()
    b.stage(arena2, chunks2, docs2)
    stage_s = time.perf_counter() - t0
    ninf, inf_bytes, inf_ms = b.inflate_info()
    print("staged in %.1f s: %d chunks inflated on the GPU in %.2f ms" % (stage_s, ninf, inf_ms), flush=True)
    for _ in range(args.warmup):
        b.run()
    b.sync()
    stage_ms = [0.0] * 4
    t0 = time.perf_counter()
    for _ in range(args.steps):
        b.run()
        b.sync()
        for i, x in enumerate(b.stage_times()):
            stage_ms[i] += x
    elapsed = (time.perf_counter() - t0) / args.steps
    # Backend.load + applyChanges in full from host memory, per step: H2D of the saved base documents
    # and the compressed changes, the GPU checksum of the compressed documents, the GPU inflate of
    # their DEFLATEd columns (inflateColumn, columnar.js:1062-1068) and of the compressed changes,
    # then the pipeline
    t0 = time.perf_counter()
    st_s = 0.0
    for _ in range(args.steps):
        t1 = time.perf_counter()
        b.stage(arena2, chunks2, docs2)
        st_s += time.perf_counter() - t1
        b.run()
        b.sync()
    elapsed_full = (time.perf_counter() - t0) / args.steps
    # the same steps pipelined over two batches on two engines (two HIP streams): step k's stage (H2D,
    # checksums, inflate, sizing) runs while step k-1's kernels do, as the C4 pipeline overlaps its
    # batches; every step still moves and inflates all of its inputs
    from automerge_amd import _native as N
    err = N.Error()
    eng2 = N.lib.am_engine_create(0, N.C.byref(err))
    if not eng2:
        N.raise_for(err)
    b2 = Batch(engine=eng2)
    pair = [b, b2]
    b2.stage(arena2, chunks2, docs2)
    b2.run()
    b2.sync()
    npipe = max(2, args.steps)
    t0 = time.perf_counter()
    for k in range(npipe):
        cur = pair[k % 2]
        cur.stage(arena2, chunks2, docs2)
        cur.run()
        if k:
            pair[(k - 1) % 2].sync()
    pair[(npipe - 1) % 2].sync()
    elapsed_pipe = (time.perf_counter() - t0) / npipe
    pipe_err = int((b.results()["status"] != 0).sum()) + int((b2.results()["status"] != 0).sum())
    del b2
    N.lib.am_engine_destroy(eng2)
    # the same with the bases staged beforehand on the host path (am_stage_documents), untimed: the
    # stage then moves uncompressed bases and inflates only the changes
    hs = N.stage_documents(bases)
    arena4, chunks4, docs4 = pack([(h[0], r_) for h, r_ in zip(hs, rest)])
    chunks4["flags"][docs4["base_chunk"].astype(np.int64)] = [1 if h[1] else 0 for h in hs]
    b.stage(arena4, chunks4, docs4)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        b.stage(arena4, chunks4, docs4)
        b.run()
        b.sync()
    elapsed_h2d = (time.perf_counter() - t0) / args.steps
    b.stage(arena2, chunks2, docs2)
    b.run()
    b.sync()
    r = b.results()
    nerr = int((r["status"] != 0).sum())
    checked = []
    golden = json.load(open(os.path.join(ROOT, "tests", "golden", "text.json")))
    ref = {c["name"]: c for c in golden}.get("c3full")
    if ref and (args.changes, args.per_change, args.cross) == (ref["nchanges"], ref["per_change"], ref["cross_every"]):
        for i, e in enumerate(ref["docs"][:args.docs]):
            assert hashlib.sha256(bases[i]).hexdigest() == e["split"]["base"], "base %d differs from the reference" % i
            assert hashlib.sha256(b.doc_save(i)).hexdigest() == e["split"]["save"], "doc %d differs from the reference" % i
            checked.append(i)
    # the applyChanges patch of one 100k-op document (Backend.applyChanges' return value, P8)
    from automerge_amd.batch import WANT_DIFF
    pb = Batch()
    pb.stage(*pack([(bases[0], rest[0])], flags=WANT_DIFF))
    pb.run()
    pb.sync()
    patch_ms = []
    for _ in range(3):
        pb.run()
        pb.sync()
        patch_ms.append(pb.stage_times()[2])
    assert int(pb.results()["status"][0]) == 0, "patch run failed"
    cpu = None
    if args.cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_ffi as O
        t0 = time.perf_counter()
        d = O.Doc.load(bases[0])
        d.apply(rest[0])
        d.save()
        dt = time.perf_counter() - t0
        cpu = {"value": len(rest[0]) * args.per_change / dt, "unit": "ops/s", "cores": 1, "kind": "port",
               "sample": "document 0 (load + applyChanges + save) by oracle/liboracle.so, 1 thread, %.1f s" % dt}
    k = args.steps
    line = {
        "workload": "C3 text histories: load(save(first half)) + applyChanges(second half, deflated chunks)",
        "docs": args.docs, "ops_per_doc": 1 + args.changes * args.per_change, "ops_applied": ops_applied,
        "value": ops_applied / elapsed_full, "unit": "ops/s", "ms_per_step": elapsed_full * 1e3, "steps": k,
        "what": "per step from host memory: H2D of the saved bases and the compressed changes, GPU checksums of "
                "the compressed bases, GPU inflate of their DEFLATEd columns and of the changes, pipeline",
        "stage_ms_per_step": st_s * 1e3 / k,
        "pipelined_ops_per_s": ops_applied / elapsed_pipe, "pipelined_ms_per_step": elapsed_pipe * 1e3,
        "pipelined_steps": npipe, "pipelined_errors": pipe_err,
        "staged_bases_ops_per_s": ops_applied / elapsed_h2d, "staged_bases_ms_per_step": elapsed_h2d * 1e3,
        "kernel_resident_ops_per_s": ops_applied / elapsed, "kernel_resident_ms_per_step": elapsed * 1e3,
        "patch_100k_doc_k_doc_ms": min(patch_ms),
        "stage_ms": {"k_chunks": stage_ms[0] / k, "k_bounds+scan": stage_ms[1] / k, "k_doc": stage_ms[2] / k,
                     "k_out_hash": stage_ms[3] / k},
        "inflate": {"chunks": ninf, "ms": inf_ms, "inflated_arena_bytes": inf_bytes,
                    "GBps_out": inf_bytes / (inf_ms * 1e-3) / 1e9 if inf_ms else None},
        "errors": nerr, "verified_vs_reference": checked, "workspace_bytes": int(b.workspace_bytes()),
        "input_bytes": int(arena2.nbytes), "gen_s": gen_s, "cpu_baseline": cpu,
    }
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
