#!/usr/bin/env python3
"""Pins the digest of the whole C4 headline job (bench.py default: 1,048,576 documents) with the CPU
oracle, in the build container: every document is loaded, merged with its 12 changes and saved by
oracle/liboracle.so (test infrastructure, pinned to the reference by tests/test_oracle.py), and the
per-document terms of automerge_amd/shard.py doc_digest (index, container checksum, length, status)
are summed, and so are the terms of every document's applyChanges patch (shard.patch_term: SHA-256
of the canonical JSON of its clock and diffs, from the oracle's applyChanges patch, itself pinned to
the reference by tests/test_apply_patch_oracle.py). bench.py compares the two digests its pipeline
computes over every merged document and every patch log with the committed values
(tests/golden/c4_digest.json).

  python tools/pin_c4_digest.py [--docs 1048576] [--procs 8]
"""
import argparse
import json
import multiprocessing as mp
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
OUT = os.path.join(ROOT, "tests", "golden", "c4_digest.json")


def part(args):
    lo, hi = args
    import numpy as np
    import oracle_ffi as O
    import workload
    from automerge_amd import shard
    arena, chunks, docs, _ = workload.c4_list(np.arange(lo, hi, dtype=np.uint64), nthreads=1)
    chk = np.zeros(hi - lo, np.uint64)
    lens = np.zeros(hi - lo, np.uint64)
    status = np.zeros(hi - lo, np.uint64)
    pterms = 0
    for i in range(hi - lo):
        base, changes = workload.doc_chunks(arena, chunks, docs, i)
        try:
            d = O.Doc.load(base) if base else O.Doc.init()
            pat = d.apply_patch(changes)  # applies the changes and returns the applyChanges patch
            out = d.save()
        except O.OracleError:
            status[i] = 1
            continue
        chk[i] = int.from_bytes(out[4:8], "little")
        lens[i] = len(out)
        pterms += shard.patch_term(lo + i, pat)
    return (shard.doc_digest_np(np.arange(lo, hi, dtype=np.uint64), status, lens, chk), int((status != 0).sum()),
            pterms & 0x7FFFFFFFFFFFFFFF)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", type=int, default=1 << 20)
    ap.add_argument("--procs", type=int, default=min(8, os.cpu_count() or 1))
    args = ap.parse_args()
    from automerge_amd import shard
    step = 8192
    ranges = [(lo, min(lo + step, args.docs)) for lo in range(0, args.docs, step)]
    t0 = time.perf_counter()
    with mp.Pool(args.procs) as pool:
        res = pool.map(part, ranges)
    digest = shard.combine(r[0] for r in res)
    errors = sum(r[1] for r in res)
    rec = {"docs": args.docs, "digest": digest, "errors": errors, "patch_digest": shard.combine(r[2] for r in res),
           "how": "oracle/liboracle.so load + applyChanges + save of every C4 document (workload.c4_list), "
                  "shard.doc_digest terms summed mod 2^63; patch_digest: shard.patch_term of every document's "
                  "applyChanges patch (oracle), summed mod 2^63 (tools/pin_c4_digest.py)",
           "seconds": round(time.perf_counter() - t0, 1), "procs": args.procs}
    try:
        pinned = json.load(open(OUT))
    except (OSError, ValueError):
        pinned = {}
    pinned[str(args.docs)] = rec
    with open(OUT, "w") as f:
        json.dump(pinned, f, indent=1, sort_keys=True)
        f.write("\n")
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
