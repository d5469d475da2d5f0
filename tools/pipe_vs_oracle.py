#!/usr/bin/env python3
"""Diagnosis of tests/test_gpu_pipe.py: the reference batch and the pipeline (2 passes, 2 slots)
both compared with the oracle; the reference batch is compared before and after the pipeline runs."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import bench
    import workload as W
    import oracle_ffi as O
    from automerge_amd import pipe
    from automerge_amd.batch import WANT_DIFF, Batch
    arena, chunks, docs, _ = W.c4(40, 2500)
    docs = docs.copy()
    docs["flags"] |= WANT_DIFF
    parts = bench.split_batches(arena, chunks, docs, 700)
    want = []
    for i in range(2500):
        base, ch = W.doc_chunks(arena, chunks, docs, i)
        d = O.Doc.load(base)
        d.apply(ch)
        want.append(d.save())
    ref = Batch()
    ref.stage(arena, chunks, docs)
    ref.run()
    ref.sync()
    rr = ref.results()
    bad0 = [i for i in range(2500) if ref.doc_output(i, rr[i]) != want[i]]
    kinfo = ref.kernel_info()
    ws = int(ref.workspace_bytes())
    pl = pipe.Pipeline(max(len(p[0]) for p in parts), max(len(p[1]) for p in parts), 700, ws, 1 << 20, 4 << 20,
                       kinfo["k_doc_fast_lds_per_doc"], slots=2)
    outs = []
    for _ in range(2):
        keep = []
        for a, c, d in parts:
            s = pipe.Pinned(len(d) * pipe.SUMMARY_DT.itemsize)
            po, pp = pipe.Pinned(1 << 20), pipe.Pinned(4 << 20)
            pa, pc, pd = pipe.pinned_copy(a), pipe.pinned_copy(c), pipe.pinned_copy(d)
            pl.submit(pa.arr, pc.arr, pd.arr, s.view(pipe.SUMMARY_DT, len(d)), po.u8, pp.u8)
            keep.append((pa, pc, pd, s, po, pp, len(d)))
        pl.drain(len(parts))
        outs.append(keep)
    bad1 = [i for i in range(2500) if ref.doc_output(i, rr[i]) != want[i]]
    badp = []
    for k, keep in enumerate(outs):
        i = 0
        for pa, pc, pd, s, po, pp, n in keep:
            sm = s.view(pipe.SUMMARY_DT, n)
            for j in range(n):
                o = bytes(po.u8[int(sm[j]["out_off"]):int(sm[j]["out_off"]) + int(sm[j]["out_len"])])
                if o != want[i]:
                    badp.append((k, i))
                i += 1
    print(json.dumps({"ref_before": bad0[:10], "ref_after": bad1[:10], "n_ref_after": len(bad1), "pipe_bad": badp[:10],
                      "n_pipe_bad": len(badp), "engines": pl.engines()}), flush=True)


if __name__ == "__main__":
    main()
