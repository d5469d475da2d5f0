#!/usr/bin/env python3
"""bench.py -- batched load + applyChanges on MI355X (BASELINE.json metric), one process per GPU.

Workload: the 1M-document job. Document i is a saved base document (change 0:
makeList 'items' + 'title') that is loaded and merged with 12 concurrent changes from 4 actors (4
list inserts + 1 conflicting title set each): 13 changes, 60 ops merged, ~2.1 KB of input and a
~720 B merged document. Documents are sharded over the ranks by the first byte of their base
document's SHA-256 (the container checksum) mod N, so N GPUs split the same job (strong scaling).

A step is the whole job of a rank from host memory back to host memory, as a caller of the engine
sees it ("load + applyChanges (batched, H2D included)"): every batch of its shard goes
through am_pipe_submit_packed (include/automerge_amd.h) -- H2D of the encoded chunks and of 4 B per
chunk + 8 B per document of descriptors (the chunk / document tables are expanded on the device),
SHA-256 of every chunk, header parse, causal queue, column decode, merge (sort / RGA / succ),
canonical re-encode, checksum, the patch Backend.applyChanges returns (wire form of am_patch.h),
compaction, and D2H of the merged documents, patches and per-document summaries. Copies of batch
k+1 / k-1 overlap the kernels of batch k. This is `value`. The same chain with the inputs already in
HBM (am_pipe_run_resident) is reported beside it as `hbm_resident` and is never `value`.
Materializing the patches as JS objects is the host's job and is not timed here (tools/).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--docs D] [--batch B] [--slots S]
  python bench.py --mode resident [--workload c4|c2] --docs D   # value = the HBM-resident chain (not the contract)
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "ops merged/sec (batched load+applyChanges) + decode GB/s at 1/2/4/8 GPUs"
HBM_PEAK_GBPS = 8000.0  # MI355X spec (MI355X_MICROARCH.md)
CPU_REF_JSON = os.path.join(ROOT, "profiles", "cpu_reference_node.json")


def _oracle_sample(args):
    """load + applyChanges + save by the oracle of the workload's documents from index `first` on,
    generated here in blocks of 1024, for at most `seconds`; returns (documents done, seconds)."""
    wl, first, seconds = args
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_ffi as O
    import workload
    gen = workload.c4 if wl == "c4" else workload.c2
    n = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        arena, chunks, docs, _ = gen(first + n, 1024, nthreads=1)
        for i in range(len(docs)):
            base, changes = workload.doc_chunks(arena, chunks, docs, i)
            d = O.Doc.load(base) if base else O.Doc.init()
            d.apply(changes)
            d.save()
            n += 1
            if time.perf_counter() - t0 >= seconds:
                break
    return n, time.perf_counter() - t0


def _read(path):
    with open(path) as f:
        return f.read()


def bind_numa(local):
    """Binds this rank (and the CPU-baseline workers it forks) to the CPUs of its GPU's NUMA node,
    before any GPU call: the pinned staging arenas (hipHostMallocNumaUser, am_capi.hip) are then
    placed on the socket the GPU hangs off. HIP device `local` is the local-th GPU node of the KFD
    topology (after ROCR_VISIBLE_DEVICES / HIP_VISIBLE_DEVICES when they list indices); its PCI
    address gives the node (the DRM render node's device link when the topology is not readable).
    Returns what it found (reported in the bench line), never fails."""
    info = {"gpu": local, "numa_node": None, "bound": False}
    step = "kfd topology"
    try:
        bdf = None
        try:
            topo = "/sys/class/kfd/kfd/topology/nodes"
            gpus = []
            for n in sorted(os.listdir(topo), key=int):
                props = dict(ln.split(" ", 1) for ln in _read(os.path.join(topo, n, "properties")).splitlines() if " " in ln)
                if int(props.get("simd_count", "0")) > 0:
                    gpus.append(props)
            idx = local
            for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES"):
                vis = os.environ.get(var)
                if vis and all(x.strip().isdigit() for x in vis.split(",") if x.strip()):
                    idx = int([x for x in vis.split(",") if x.strip()][idx])
            loc, dom = int(gpus[idx]["location_id"]), int(gpus[idx].get("domain", "0"))
            bdf = "%04x:%02x:%02x.%x" % (dom, loc >> 8, (loc >> 3) & 31, loc & 7)
        except (OSError, ValueError, KeyError, IndexError) as e:
            info["kfd"] = "%s: %s" % (type(e).__name__, e)
        if bdf is None:
            # the render nodes the process can open, in minor order (one GPU per box: the visible one)
            step = "render nodes"
            rn = sorted((int(d[7:]), d) for d in os.listdir("/dev/dri") if d.startswith("renderD"))
            bdf = os.path.basename(os.path.realpath("/sys/class/drm/%s/device" % rn[local][1]))
        info["pci"] = bdf
        step = "pci numa_node"
        node = int(_read("/sys/bus/pci/devices/%s/numa_node" % bdf))
        info["numa_node"] = node
        if node < 0:
            return info
        step = "node cpulist"
        cpus = set()
        for part in _read("/sys/devices/system/node/node%d/cpulist" % node).strip().split(","):
            a, _, b = part.partition("-")
            cpus.update(range(int(a), int(b or a) + 1))
        mine = cpus & os.sched_getaffinity(0)
        step = "sched_setaffinity"
        if mine:
            os.sched_setaffinity(0, mine)
            info.update(bound=True, cpus=len(mine))
    except (OSError, ValueError, KeyError, IndexError) as e:
        info["why"] = "%s: %s: %s" % (step, type(e).__name__, e)
    return info


_PATCH_MODS = None


def _patch_part(args):
    """Sum of shard.patch_term over one slice of the engine's wire-form patch logs, in a CPU-baseline
    worker (forked before the GPU was touched): automerge_amd/patch.py and shard.py are loaded as
    plain files, so the worker never loads the HIP library."""
    global _PATCH_MODS
    ids, logs = args
    if _PATCH_MODS is None:
        import importlib.util

        def load(name):
            spec = importlib.util.spec_from_file_location("_am_" + name, os.path.join(ROOT, "automerge_amd", name + ".py"))
            m = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(m)
            return m
        _PATCH_MODS = load("patch"), load("shard")
    P, S = _PATCH_MODS
    t = 0
    for i, log in zip(ids, logs):
        if log:
            t += S.patch_term(int(i), P.materialize(log, [], 0, 0))
    return t & 0x7FFFFFFFFFFFFFFF


def patch_digest(pool, ids, summ_b, pats_b):
    """Digest of every document's applyChanges patch of this rank (shard.patch_term summed), from the
    wire-form logs the pipeline brought home; on the CPU-baseline workers when there are any."""
    from automerge_amd import shard
    jobs = []
    k0 = 0
    for s_, pb in zip(summ_b, pats_b):
        off = s_["patch_off"].astype(np.int64)
        ln = s_["patch_len"].astype(np.int64)
        ok = s_["status"] == 0
        raw = pb.tobytes() if len(pb) else b""
        logs = [raw[o:o + n] if good else b"" for o, n, good in zip(off.tolist(), ln.tolist(), ok.tolist())]
        for a in range(0, len(logs), 4096):
            jobs.append((ids[k0 + a:k0 + a + 4096].tolist(), logs[a:a + 4096]))
        k0 += len(logs)
    if pool is not None:
        return shard.combine(pool.map(_patch_part, jobs))
    return shard.combine(_patch_part(j) for j in jobs)


def cpu_pool(procs):
    """The worker processes of the all-cores CPU baseline, forked before this process touches the
    GPU or imports torch (a fork of a GPU-initialised process is not safe on this pool)."""
    import multiprocessing as mp
    return mp.get_context("fork").Pool(procs)


def cpu_baseline(pool, procs, wl, seconds=6.0, ops_per_doc=60):
    """The oracle (CPU restatement of the reference algorithm, oracle/) timed on the host over a
    bounded sample of the same workload: ops merged per second (load + applyChanges + save), on one
    core and on `procs` cores at once (one process each, disjoint documents)."""
    n1, t1 = _oracle_sample((wl, 0, seconds))
    res = pool.map(_oracle_sample, [(wl, k * 50000, seconds) for k in range(procs)])
    pool.close()
    pool.join()
    nall = sum(r[0] for r in res)
    tall = max(r[1] for r in res)
    name = wl.upper()
    return {"value": n1 * ops_per_doc / t1, "unit": "ops/s", "cores": 1, "kind": "port", "host_cpus": os.cpu_count(),
            "sample": "%d %s documents (load + applyChanges + save) by oracle/liboracle.so, 1 thread, %.1f s" % (n1, name, t1),
            "all_cores": {"value": nall * ops_per_doc / tall, "unit": "ops/s", "cores": procs,
                          "sample": "%d %s documents on %d processes at once, %.1f s" % (nall, name, procs, tall)}}


def pinned_digest(docs, field="digest"):
    """The digest of the whole C4 job of `docs` documents computed by the oracle in the build
    container (tools/pin_c4_digest.py -> tests/golden/c4_digest.json), or None. field: "digest" (the
    merged documents) or "patch_digest" (their applyChanges patches)."""
    try:
        rec = json.load(open(os.path.join(ROOT, "tests", "golden", "c4_digest.json")))
    except (OSError, ValueError):
        return None
    r = rec.get(str(docs))
    return int(r[field]) if r and field in r else None


def decode_alg_bytes(arena, chunks, docs, sample=256):
    """Algorithmic decode bytes of SURVEY 8(d) per document, over a sample: the encoded input read
    plus the SoA written -- 44 B per op row (11 u32 fields), 1 B insert flag, 8 B per pred/succ
    entry and the raw value bytes (the decode's rows and entries are the merged document's ops and
    succ entries: C4 has no deletions). Returns (input bytes, SoA bytes) per document."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_ffi as O
    import workload
    n = min(sample, len(docs))
    inb = soa = 0
    for i in range(n):
        base, changes = workload.doc_chunks(arena, chunks, docs, i)
        inb += (len(base) if base else 0) + sum(len(c) for c in changes)
        d = O.Doc.load(base) if base else O.Doc.init()
        d.apply(changes)
        e = O.export(d.save())
        soa += 45 * e["nops"] + 8 * e["nsucc"] + e["val_bytes"]
    return inb / n, soa / n


def kernel_source_digest():
    """Digest of the engine's kernel sources: profiles/traffic_k_doc.json (the PMC FETCH_SIZE /
    WRITE_SIZE passes, tools/gpu_traffic.sh + tools/traffic.py) is reported only for the sources it
    was measured on."""
    import hashlib
    h = hashlib.sha256()
    src = os.path.join(ROOT, "automerge_amd", "csrc")
    for name in sorted(os.listdir(src)):
        if name.endswith((".h", ".hip")):
            with open(os.path.join(src, name), "rb") as f:
                h.update(name.encode() + b"\0" + f.read())
    return h.hexdigest()[:16]


def measured_traffic(batch_docs):
    """profiles/traffic_k_doc.json when it was measured on these kernel sources and batch size."""
    try:
        rec = json.load(open(os.path.join(ROOT, "profiles", "traffic_k_doc.json")))
    except (OSError, ValueError):
        return None
    ok = rec.get("src_digest") == kernel_source_digest() and rec.get("batch_docs") == batch_docs
    return rec if ok else None


def cpu_reference():
    """The reference JS backend under Node (measured in the build container by
    tools/cpu_reference.js, which cannot run on the GPU box): per core and on all cores."""
    try:
        return json.load(open(CPU_REF_JSON))
    except (OSError, ValueError):
        return None


def split_batches(arena, chunks, docs, batch):
    """Per-batch (arena slice, rebased chunk descriptors, rebased document descriptors)."""
    import numpy as np
    out = []
    for lo in range(0, len(docs), batch):
        d = docs[lo:lo + batch].copy()
        c0 = int(d["chg_begin"][0]) - (1 if d["base_chunk"][0] >= 0 else 0)
        c1 = int(d["chg_begin"][-1] + d["chg_count"][-1])
        c = chunks[c0:c1].copy()
        a0 = int(c["off"][0])
        a1 = int(c["off"][-1] + c["len"][-1])
        c["off"] -= a0
        d["chg_begin"] -= c0
        d["base_chunk"] = np.where(d["base_chunk"] >= 0, d["base_chunk"] - c0, -1)
        out.append((arena[a0:a1], c, d))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--docs", type=int, default=1 << 20, help="documents of the whole job (sharded over the ranks)")
    ap.add_argument("--batch", type=int, default=0, help="documents per pipeline batch (0: auto)")
    ap.add_argument("--slots", type=int, default=3, help="batches in flight")
    ap.add_argument("--mode", choices=["pipe", "resident"], default="pipe",
                    help="pipe: from host memory back to host memory (the `value`); resident: inputs in HBM")
    ap.add_argument("--no-resident", action="store_true", help="pipe mode: skip the HBM-resident run reported beside it")
    ap.add_argument("--full-desc", action="store_true", help="pipe mode: send full chunk / document descriptors")
    ap.add_argument("--workload", choices=["c4", "c2"], default="c4")
    ap.add_argument("--no-patch", action="store_true", help="merge without the applyChanges patch")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--check", type=int, default=32, help="documents verified against the oracle (rank 0)")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    # AM_BENCH_DEVICE / AM_DIST_BACKEND=gloo: every rank on one GPU with a CPU exchange (the N>1
    # rehearsal of tests/test_gpu_bench_ranks.py; RCCL refuses two ranks on one device)
    local = int(os.environ.get("AM_BENCH_DEVICE", os.environ.get("LOCAL_RANK", "0")))
    # this rank on its GPU's NUMA node before anything touches the GPU (or forks)
    numa = bind_numa(local)
    # the CPU baseline's workers are forked now, before torch is imported or the GPU is touched
    procs = min(16, os.cpu_count() or 1)  # the GPU box's CPU share is 16 per GPU
    pool = cpu_pool(procs) if rank == 0 and not args.no_cpu_baseline else None
    backend = os.environ.get("AM_DIST_BACKEND", "nccl")
    import numpy as np
    import torch
    dist = None
    dist_info = {"world_size": 1, "backend": None}
    # AM_DIST_FORCE=1: the process group even for one rank (tests/test_gpu_bench_ranks.py runs the
    # nccl branch -- RCCL init, the device all-gather -- on a one-GPU box this way)
    if world > 1 or os.environ.get("AM_DIST_FORCE") == "1":
        import torch.distributed as dist
        if backend == "nccl":
            dist.init_process_group(backend="nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend=backend)
        dist_info = {"world_size": dist.get_world_size(), "backend": str(dist.get_backend()), "rank": dist.get_rank()}
    dist_info["numa"] = numa
    torch.cuda.set_device(local)
    xdev = "cuda" if backend == "nccl" else "cpu"

    from automerge_amd import shard
    from automerge_amd.batch import WANT_DIFF, Batch
    import workload

    t_gen = time.perf_counter()
    if args.workload == "c4":
        ids = workload.c4_shard(0, args.docs, world, rank)
        arena, chunks, docs, ops_rank = workload.c4_list(ids)
        per_doc = 60
    else:
        first, n = rank * (args.docs // world), args.docs // world
        ids = np.arange(first, first + n, dtype=np.uint64)
        arena, chunks, docs, ops_rank = workload.c2(first, n)
        per_doc = 14
    if not args.no_patch:
        docs["flags"] |= WANT_DIFF
    t_gen = time.perf_counter() - t_gen
    D = len(docs)

    def barrier():
        if dist is not None:
            dist.barrier()

    extra = {}
    from automerge_amd import pipe
    # 65536 documents per batch: big enough to fill the 256 CUs many times over (k_doc_fast: one
    # wave per document), small enough that one workspace serves every batch in turn
    batch = args.batch or max(16384, min(65536, -(-D // 4)))
    parts = split_batches(arena, chunks, docs, batch)
    # capacities from a representative batch (the largest one), staged the ordinary way
    probe = Batch(device=local)
    probe.stage(*max(parts, key=lambda p: len(p[0])))
    # the scanned plans (k_doc_fast's documents: compact ones), plus 1/8 + 64 MB of overflow room
    # for documents the fast kernel gives up on (each then takes k_doc's whole plan there)
    ws_need = int(probe.workspace_plan())
    kinfo = probe.kernel_info()
    del probe
    arena_cap = max(len(p[0]) for p in parts)
    ncap = max(len(p[2]) for p in parts)
    ccap = max(len(p[1]) for p in parts)
    out_cap = ncap * 1024 + (1 << 20)
    patch_cap = ncap * 1024 + (1 << 20) if not args.no_patch else (1 << 20)
    ws_slot = ws_need + ws_need // 8 + (64 << 20)
    pl = pipe.Pipeline(arena_cap, ccap, ncap, ws_slot, out_cap, patch_cap,
                       kinfo["k_doc_fast_lds_per_doc"], slots=args.slots, device=local)
    nb = len(parts)
    in_b = int(arena.nbytes)
    starts = np.cumsum([0] + [len(p[2]) for p in parts])
    packed = [None if args.full_desc else pipe.pack(c, d) for _, c, d in parts]
    desc_b = sum(int(k[0].nbytes + k[1].nbytes) if k is not None else int(c.nbytes + d.nbytes)
                 for k, (_, c, d) in zip(packed, parts))

    def run_pipe(steps, warmup):
        """The job from host memory back to host memory (am_pipe_submit_packed / drain)."""
        pin_in = []
        for (a, c, d), k in zip(parts, packed):
            desc = (pipe.pinned_copy(k[0]), pipe.pinned_copy(k[1])) if k is not None else (pipe.pinned_copy(c), pipe.pinned_copy(d))
            pin_in.append((pipe.pinned_copy(a), desc, k is not None))
        pin_out = []
        for a, c, d in parts:
            sb = pipe.Pinned(len(d) * pipe.SUMMARY_DT.itemsize)
            pin_out.append((sb, sb.view(pipe.SUMMARY_DT, len(d)), pipe.Pinned(out_cap), pipe.Pinned(patch_cap)))

        def step():
            for (pa, (p1, p2), is_packed), (_, summ, po, pp) in zip(pin_in, pin_out):
                if is_packed:
                    pl.submit_packed(pa.arr, p1.arr, p2.arr, summ, po.u8, pp.u8)
                else:
                    pl.submit(pa.arr, p1.arr, p2.arr, summ, po.u8, pp.u8)

        for _ in range(warmup):
            step()
        pl.drain(nb * warmup)
        pl.times()
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        # the steps stream through the pipeline back to back (a caller's stream of batches: the next
        # step's first H2D overlaps this step's last kernels and copies home); every batch of every
        # step is home when the clock stops
        for _ in range(steps):
            step()
        totals = pl.drain(nb * steps)[-nb:]
        torch.cuda.synchronize()
        barrier()
        el = time.perf_counter() - t0
        ms_c, ms_d, nt = pl.times()
        return el, totals, pin_out, ms_c / max(steps, 1), ms_d / max(nt, 1)

    def run_resident(steps, warmup):
        """Inputs resident in HBM (copied before the timed region); each step runs every batch of the
        shard through the whole chain (am_pipe_run_resident), outputs compacted in HBM."""
        dev = []
        for a, c, d in parts:
            ta = torch.zeros(len(a) + 64, dtype=torch.uint8, device="cuda")
            ta[:len(a)].copy_(torch.from_numpy(np.ascontiguousarray(a)))
            tc = torch.from_numpy(np.ascontiguousarray(c).view(np.uint8)).cuda()
            td = torch.from_numpy(np.ascontiguousarray(d).view(np.uint8)).cuda()
            ts = torch.zeros(len(d) * pipe.SUMMARY_DT.itemsize, dtype=torch.uint8, device="cuda")
            to = torch.empty(out_cap, dtype=torch.uint8, device="cuda")
            tp = torch.empty(patch_cap, dtype=torch.uint8, device="cuda")
            tt = torch.zeros(2, dtype=torch.int64, device="cuda")
            dev.append((len(a), len(c), len(d), ta, tc, td, ts, to, tp, tt))
        torch.cuda.synchronize()

        def step():
            for na, nc, nd, ta, tc, td, ts, to, tp, tt in dev:
                pl.run_resident(ta.data_ptr(), na, tc.data_ptr(), nc, td.data_ptr(), nd, not args.no_patch,
                                ts.data_ptr(), to.data_ptr(), out_cap, tp.data_ptr(), patch_cap, tt.data_ptr())
            return pl.resident_sync()

        for _ in range(warmup):
            step()
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ms_comp = ms_doc = 0.0
        for _ in range(steps):
            a_, d_ = step()
            ms_comp += a_
            ms_doc += d_
        torch.cuda.synchronize()
        barrier()
        el = time.perf_counter() - t0
        # results home (outside the timed region): summaries, merged documents, patch logs
        summ_b = [x[6].cpu().numpy().view(pipe.SUMMARY_DT) for x in dev]
        tot_b = [x[9].cpu().numpy() for x in dev]
        outs_b = [x[7][:int(t[0])].cpu().numpy() for x, t in zip(dev, tot_b)]
        pats_b = [x[8][:int(t[1])].cpu().numpy() for x, t in zip(dev, tot_b)]
        del dev
        return el, summ_b, outs_b, pats_b, [(int(t[0]), int(t[1])) for t in tot_b], ms_comp / steps, ms_doc / (steps * nb)

    def pcie_rates():
        """One 1 GB pinned H2D and D2H copy each (torch's copies, the link's plain rate)."""
        hb = torch.empty(min(in_b, 1 << 30), dtype=torch.uint8).pin_memory()
        db = torch.empty_like(hb, device="cuda")
        db.copy_(hb, non_blocking=True)
        torch.cuda.synchronize()
        e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        e0.record()
        db.copy_(hb, non_blocking=True)
        e1.record()
        hb.copy_(db, non_blocking=True)
        e2.record()
        torch.cuda.synchronize()
        return {"h2d": hb.numel() / (e0.elapsed_time(e1) * 1e-3) / 1e9, "d2h": hb.numel() / (e1.elapsed_time(e2) * 1e-3) / 1e9}

    extra["batches"] = nb
    extra["batch_docs"] = batch
    if args.mode == "pipe":
        elapsed, totals, pin_out, ms_comp, t_doc = run_pipe(args.steps, args.warmup)
        summ_b = [o[1] for o in pin_out]
        outs_b = [o[2].u8 for o in pin_out]
        pats_b = [o[3].u8 for o in pin_out]
        out_bytes = sum(t[0] for t in totals[:nb])
        patch_bytes = sum(t[1] for t in totals[:nb])
        extra["kernel_ms_per_step"] = ms_comp
        h2d = in_b + desc_b
        d2h = out_bytes + patch_bytes + D * pipe.SUMMARY_DT.itemsize
        rates = pcie_rates()
        e_h2d, e_home = pl.engines()
        extra["host_link"] = {
            "bytes_per_step_rank0": {"h2d": h2d, "d2h": d2h, "descriptors": desc_b,
                                     "packed_batches": sum(k is not None for k in packed)},
            "GBps_alone": rates, "sdma_engine_mask": {"h2d": e_h2d, "home": e_home},
            "h2d_ms": h2d / (rates["h2d"] * 1e9) * 1e3, "d2h_ms": d2h / (rates["d2h"] * 1e9) * 1e3,
            "ms_per_step_over_max_h2d_kernels": (elapsed * 1000.0 / args.steps) / max(h2d / (rates["h2d"] * 1e9) * 1e3, ms_comp)}
        if not args.no_resident:
            el_r, _, _, _, tot_r, msc_r, msd_r = run_resident(max(2, args.steps), 1)
            sr = max(2, args.steps)
            extra["hbm_resident"] = {
                "what": "the same chain with the inputs already in HBM (am_pipe_run_resident), outputs left in HBM; never `value`",
                "ops_per_s_rank0": ops_rank / (el_r / sr), "ms_per_step": el_r * 1000.0 / sr, "steps": sr,
                "kernel_ms_per_step": msc_r, "doc_kernel_ms_per_batch": msd_r}
    else:
        elapsed, summ_b, outs_b, pats_b, tot_b, ms_comp, t_doc = run_resident(args.steps, args.warmup)
        out_bytes = sum(t[0] for t in tot_b)
        patch_bytes = sum(t[1] for t in tot_b)
        extra["kernel_ms_per_step"] = ms_comp
    summ_all = np.concatenate(summ_b)
    statuses = summ_all["status"]
    alg_launch = (in_b + out_bytes + patch_bytes) / nb
    workspace = int(ws_slot)  # what one pipeline slot holds (plans + overflow room)
    # per-shard digest: container checksum, length and status of every merged document
    chk = []
    for s_, po in zip(summ_b, outs_b):
        off = s_["out_off"].astype(np.int64)
        ok_ = s_["status"] == 0
        offs = np.where(ok_, off, 0)
        b4 = [po[offs + j].astype(np.uint64) if len(po) else np.zeros(len(offs), np.uint64) for j in range(4, 8)]
        chk.append(np.where(ok_, b4[0] | (b4[1] << 8) | (b4[2] << 16) | (b4[3] << 24), 0))
    digest = shard.doc_digest_np(ids, statuses, summ_all["out_len"], np.concatenate(chk).astype(np.uint64))

    def check(i):
        k = int(np.searchsorted(starts, i, side="right") - 1)
        s_ = summ_b[k][i - starts[k]]
        o = bytes(outs_b[k][int(s_["out_off"]):int(s_["out_off"]) + int(s_["out_len"])])
        p_ = bytes(pats_b[k][int(s_["patch_off"]):int(s_["patch_off"]) + int(s_["patch_len"])])
        return o, (p_ if not args.no_patch else None)

    nerr = int((statuses != 0).sum())
    # every document's patch, materialized after the timed region (the reference's patch objects)
    t_pd = time.perf_counter()
    pdig = patch_digest(pool, ids, summ_b, pats_b) if not args.no_patch else 0
    t_pd = time.perf_counter() - t_pd
    tot, _ = shard.exchange(dist, [D, ops_rank, nerr, out_bytes, digest or 0, pdig], xdev)
    if dist is not None:  # rank -> GPU -> NUMA node of every rank, for the line (outside the timed region)
        allnuma = [None] * world
        dist.all_gather_object(allnuma, dict(numa, rank=rank))
        dist_info["numa"] = allnuma
    # correctness spot check against the oracle (outside the timed region): merged bytes and patch
    checked = 0
    if args.check and rank == 0:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_ffi as O
        from automerge_amd import patch as P
        canon = lambda x: json.dumps(x, sort_keys=True, default=lambda v: bytes(v).hex())
        for i in range(min(args.check, D)):
            base, changes = workload.doc_chunks(arena, chunks, docs, i)
            ref = O.Doc.load(base) if base else O.Doc.init()
            if args.no_patch:
                ref.apply(changes)  # apply_patch applies the changes too; without a patch apply them here
                want = None
            else:
                want = ref.apply_patch(changes)
            got, log = check(i)
            assert got == ref.save(), "document %d differs from the oracle" % i
            if log is not None:
                pat = P.materialize(log, want["deps"], want["pendingChanges"], want["maxOp"])
                assert canon(pat) == canon(want), "patch of document %d differs from the oracle" % i
            checked += 1
    if rank != 0:
        dist.destroy_process_group() if dist is not None else None
        return
    extra["dist"] = dist_info
    ms_per_step = elapsed * 1000.0 / args.steps
    value = tot[1] / (elapsed / args.steps)
    achieved = alg_launch / (t_doc * 1e-3) / 1e9 if t_doc else None
    tr = measured_traffic(extra.get("batch_docs")) if args.workload == "c4" and not args.no_patch else None
    if t_doc:
        # decode GB/s: algorithmic decode bytes of one launch (encoded input read + SoA
        # written, per document from an oracle-decoded sample) / the document kernel's time; the
        # kernel does the merge, encode and patch in the same time, so this is a lower bound
        din, dsoa = decode_alg_bytes(arena, chunks, docs)
        per_launch = (D / nb) * (din + dsoa)
        extra["decode_GBps"] = per_launch / (t_doc * 1e-3) / 1e9
        extra["decode_frac_of_hbm_peak"] = extra["decode_GBps"] / HBM_PEAK_GBPS
        extra["decode_bytes_per_doc"] = {"input": din, "soa": dsoa}
    if tr is not None and t_doc:
        extra["fetch_GBps"] = 2 * tr["fetch_size_kib"] * 1024 / (t_doc * 1e-3) / 1e9  # measured HBM reads (PMC)
    cpu = cpu_baseline(pool, procs, args.workload, ops_per_doc=per_doc) if pool is not None else None
    # the whole job against the oracle's digest of every document (tests/golden/c4_digest.json)
    want = pinned_digest(tot[0]) if args.workload == "c4" and digest is not None else None
    want_p = pinned_digest(tot[0], "patch_digest") if args.workload == "c4" and not args.no_patch else None
    if want is not None:
        extra["digest_pinned"] = {"expected": want, "match": tot[4] == want,
                                  "how": "oracle load + applyChanges + save of all %d documents (tools/pin_c4_digest.py)" % tot[0]}
        if want_p is not None:
            extra["digest_pinned"]["patches"] = {
                "expected": want_p, "got": tot[5], "match": tot[5] == want_p, "materialize_s_rank0": t_pd,
                "how": "every document's applyChanges patch materialized from the engine's wire form (automerge_amd/patch.py) "
                       "and hashed (shard.patch_term: clock + diffs), against the oracle's patches of all %d documents" % tot[0]}
    wl = {"c4": "C4 1M-document job: load base doc + applyChanges of 12 concurrent changes (4 actors x 3), 60 ops/doc",
          "c2": "C2: applyChanges of 3 changes (10 map/counter/string sets + 2 concurrent inc/overwrite), 14 ops/doc"}
    what = ("from host memory: H2D + merge + applyChanges patch + D2H (pipelined)" if args.mode == "pipe" else
            "inputs resident in HBM: merge + applyChanges patch + compaction in HBM (not the contract metric)")
    if args.no_patch:
        what = what.replace(" + applyChanges patch", "")
    line = {
        "metric": METRIC, "value": value, "unit": "ops/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": ms_per_step, "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (seeded %s generator, SURVEY.md 8(d); bytes pinned to the reference encoder)" % args.workload.upper(),
        "config": {"workload": wl[args.workload] + "; " + what, "total_docs": tot[0], "docs_rank0": D,
                   "ops_per_doc_merged": per_doc,
                   "sharding": "SHA-256(base doc)[0] mod N" if args.workload == "c4" else "ranges",
                   "parallelism": "doc-sharded dp%d" % world},
        "roofline": {"kernel": "k_doc_fast (+ k_doc for the rest)", "bound": "hbm", "achieved": achieved,
                     "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBPS if achieved else None,
                     "traffic": tr["traffic_bytes"] if tr else None, "alg_bytes_per_launch": alg_launch, "avg_ms": t_doc,
                     "limiter": "VALU issue of the one-wave-per-document merge (DESIGN.md 4); not HBM"},
        "errors": tot[2], "verified_docs": checked, "input_bytes_rank0": in_b, "output_bytes_rank0": out_bytes,
        "patch_bytes_rank0": patch_bytes, "workspace_bytes_per_batch": workspace,
        "workspace_bytes_per_doc": workspace / max(1, ncap), "gen_s": t_gen,
        "docs_per_sec": tot[0] / (elapsed / args.steps), "digest": tot[4], "patch_digest": tot[5],
        "cpu_baseline": cpu, "cpu_reference_node": cpu_reference(),
    }
    line.update(extra)
    print(json.dumps(line))
    if dist is not None:
        dist.destroy_process_group()
    if want is not None and tot[4] != want:
        sys.exit("bench: the job's digest %d differs from the oracle's %d" % (tot[4], want))
    if want_p is not None and tot[5] != want_p:
        sys.exit("bench: the job's patch digest %d differs from the oracle's %d" % (tot[5], want_p))


if __name__ == "__main__":
    main()
