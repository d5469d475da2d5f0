#!/usr/bin/env python3
"""Batched Automerge.load (Backend.load + Backend.getPatch, src/automerge.js:52-55) on one MI355X:
saved C4 (or C2) documents -- the merged outputs of the bench's job -- loaded and given their
getPatch log (documentPatch, new.js:1604-1635, 2052-2060) in batches of 65,536, inputs resident in
HBM (am_pipe_run_resident with AM_DOC_WANT_PATCH, no change chunks). Prints one JSON line: documents
and visible ops per second, the document kernels' share, and a sample checked against the oracle's
getPatch (oracle/, pinned by the reference's getPatch fixtures).

  python tools/bench_getpatch.py [--workload c4|c2] [--docs 262144] [--steps 3] [--check 64]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", choices=["c4", "c2"], default="c4")
    ap.add_argument("--docs", type=int, default=1 << 18)
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--check", type=int, default=64)
    args = ap.parse_args()
    import torch
    import workload
    from automerge_amd import pipe
    from automerge_amd.batch import CHUNK_DT, DOC_DT, WANT_PATCH, Batch
    from bench import split_batches
    D = args.docs
    arena, chunks, docs, _ = getattr(workload, args.workload)(0, D)
    # 1. the saved documents: the job's merged outputs (pipeline from host memory)
    parts = split_batches(arena, chunks, docs, args.batch)
    probe = Batch()
    probe.stage(*max(parts, key=lambda p: len(p[0])))
    ws = int(probe.workspace_bytes())
    kinfo = probe.kernel_info()
    del probe
    ncap = max(len(p[2]) for p in parts)
    out_cap = ncap * 1024 + (1 << 20)
    pl = pipe.Pipeline(max(len(p[0]) for p in parts), max(len(p[1]) for p in parts), ncap, ws + ws // 8 + (1 << 20),
                       out_cap, 1 << 20, kinfo["k_doc_fast_lds_per_doc"], slots=3)
    saved = []
    for a, c, d in parts:
        summ = np.zeros(len(d), pipe.SUMMARY_DT)
        out = np.zeros(out_cap, np.uint8)
        pl.submit(a, c, d, summ, out, np.zeros(16, np.uint8))
        pl.drain(1)
        assert (summ["status"] == 0).all()
        for s in summ:
            saved.append(bytes(out[int(s["out_off"]):int(s["out_off"]) + int(s["out_len"])]))
    del pl
    # 2. load + getPatch batches: one base chunk per document, no changes
    lens = np.array([len(x) for x in saved], np.uint64)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    ga = np.frombuffer(b"".join(saved), np.uint8)
    gc = np.zeros(D, CHUNK_DT)
    gc["off"], gc["len"], gc["flags"] = offs, lens, 0
    gd = np.zeros(D, DOC_DT)
    gd["base_chunk"] = np.arange(D)
    gd["chg_begin"] = np.arange(D) + 1
    gd["chg_count"] = 0
    gd["flags"] = WANT_PATCH
    gparts = split_batches(ga, gc, gd, args.batch)
    probe = Batch()
    probe.stage(*max(gparts, key=lambda p: len(p[0])))
    ws = int(probe.workspace_bytes())
    kinfo = probe.kernel_info()
    del probe
    patch_cap = ncap * 4096 + (1 << 20)
    pl = pipe.Pipeline(max(len(p[0]) for p in gparts), max(len(p[1]) for p in gparts), ncap, ws + ws // 8 + (1 << 20),
                       out_cap, patch_cap, kinfo["k_doc_fast_lds_per_doc"], slots=2)
    dev = []
    for a, c, d in gparts:
        ta = torch.zeros(len(a) + 64, dtype=torch.uint8, device="cuda")
        ta[:len(a)].copy_(torch.from_numpy(np.ascontiguousarray(a)))
        tc = torch.from_numpy(np.ascontiguousarray(c).view(np.uint8)).cuda()
        td = torch.from_numpy(np.ascontiguousarray(d).view(np.uint8)).cuda()
        dev.append((len(a), len(c), len(d), ta, tc, td,
                    torch.zeros(len(d) * pipe.SUMMARY_DT.itemsize, dtype=torch.uint8, device="cuda"),
                    torch.empty(out_cap, dtype=torch.uint8, device="cuda"),
                    torch.empty(patch_cap, dtype=torch.uint8, device="cuda"),
                    torch.zeros(2, dtype=torch.int64, device="cuda")))
    torch.cuda.synchronize()

    def step():
        for na, nc, nd, ta, tc, td, ts, to, tp, tt in dev:
            pl.run_resident(ta.data_ptr(), na, tc.data_ptr(), nc, td.data_ptr(), nd, True, ts.data_ptr(), to.data_ptr(),
                            out_cap, tp.data_ptr(), patch_cap, tt.data_ptr())
        return pl.resident_sync()

    step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ms_c = ms_d = 0.0
    for _ in range(args.steps):
        a_, d_ = step()
        ms_c += a_
        ms_d += d_
    el = time.perf_counter() - t0
    # 3. checks (outside the timed region): every status, a sample against the oracle's getPatch
    import oracle_ffi as O
    from automerge_amd import patch as P
    summ = [x[6].cpu().numpy().view(pipe.SUMMARY_DT) for x in dev]
    tot = [x[9].cpu().numpy() for x in dev]
    pats = [x[8][:int(t[1])].cpu().numpy() for x, t in zip(dev, tot)]
    status = np.concatenate([s["status"] for s in summ])
    canon = lambda x: json.dumps(x, sort_keys=True, default=lambda v: bytes(v).hex())  # noqa: E731
    checked = 0
    for i in range(0, D, max(1, D // max(args.check, 1))):
        k, j = divmod(i, args.batch)
        s = summ[k][j]
        log = bytes(pats[k][int(s["patch_off"]):int(s["patch_off"]) + int(s["patch_len"])])
        want = O.Doc.load(saved[i]).patch()
        got = P.materialize(log, want["deps"], want["pendingChanges"])
        assert canon(got) == canon(want), "getPatch of document %d differs from the oracle" % i
        checked += 1
    ops = {"c4": 62, "c2": 14}[args.workload] * D
    print(json.dumps({
        "workload": "%s: Automerge.load = Backend.load + Backend.getPatch of %d saved documents (the job's merged "
                    "outputs), batches of %d, inputs resident in HBM" % (args.workload.upper(), D, args.batch),
        "docs_per_s": D * args.steps / el, "ops_per_s": ops * args.steps / el, "ms_per_step": el * 1000 / args.steps,
        "chain_ms_per_step": ms_c / args.steps, "doc_kernels_ms_per_step": ms_d / args.steps,
        "errors": int((status != 0).sum()), "patch_bytes": int(sum(int(t[1]) for t in tot)),
        "oracle_checked": checked,
        "note": "ops = the saved documents' op rows (C4: 2 base + 60 merged; C2: 14)"}), flush=True)


if __name__ == "__main__":
    main()
