"""Batched sync on one MI355X (BASELINE configs[4] = SURVEY.md §8(d) C5): 100k document pairs, 10
change hashes per side since lastSync (uniform random 32 B, seeded). Side A's hashes build one
Bloom filter per pair (new BloomFilter(hashes), sync.js:38-110); side B's hashes are probed
against the peer filter (containsHash, :112-125); then getChangesToSend's selection (:246-306)
runs per pair over B's changes (a chain: change i depends on change i-1) against A's filter.

Each call is the C ABI end to end (host buffers in, H2D, kernel, D2H out), so the times are
PCIe-inclusive; the kernel times come from rocprofv3 (profiles/). A sample of pairs is checked
against the oracle (oracle/am_sync_oracle.c, pinned by the reference's Bloom vectors).

  python tools/bench_sync.py [--pairs 100000] [--per-side 10] [--reps 5]
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=100000)
    ap.add_argument("--per-side", type=int, default=10)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--check", type=int, default=200)
    args = ap.parse_args()
    from automerge_amd import _native as N
    P, K = args.pairs, args.per_side
    rng = np.random.default_rng(20240917)
    ha = rng.integers(0, 256, size=(P * K, 32), dtype=np.uint8)
    hb = rng.integers(0, 256, size=(P * K, 32), dtype=np.uint8)
    hoff = (np.arange(P + 1, dtype=np.uint64) * K)
    eng = N.engine(0)
    ha_b, hb_b = ha.tobytes(), hb.tobytes()  # the C ABI takes these as char*
    err = N.Error()
    fsize = int(N.lib.am_bloom_encoded_size(K))
    cap = fsize * P
    filt = np.zeros(cap + 1, np.uint8)
    foff = np.zeros(P + 1, np.uint64)
    pfilt = np.repeat(np.arange(P, dtype=np.uint32), K)
    contains = np.zeros(P * K, np.uint8)
    coff = hoff.copy()
    doff = np.zeros(P * K + 1, np.uint64)
    first = (np.arange(P * K) % K) == 0
    doff[1:] = np.cumsum(np.where(first, 0, 1)).astype(np.uint64)
    didx = (np.arange(P * K) % K - 1)[~first].astype(np.int32)
    pfoff = np.arange(P + 1, dtype=np.uint64)
    send = np.zeros(P * K, np.uint8)

    def build():
        if N.lib.am_bloom_build(eng, ha_b, hoff.ctypes.data, P, filt.ctypes.data, cap, foff.ctypes.data,
                                C.byref(err)):
            N.raise_for(err)

    def probe():
        if N.lib.am_bloom_probe(eng, filt.ctypes.data, foff.ctypes.data, P, hb_b, pfilt.ctypes.data, P * K,
                                contains.ctypes.data, C.byref(err)):
            N.raise_for(err)

    def select():
        if N.lib.am_sync_select(eng, P, coff.ctypes.data, hb_b, doff.ctypes.data, didx.ctypes.data,
                                pfoff.ctypes.data, filt.ctypes.data, foff.ctypes.data, send.ctypes.data, C.byref(err)):
            N.raise_for(err)

    times = {}
    for name, fn in (("build", build), ("probe", probe), ("select", select)):
        fn()
        t0 = time.perf_counter()
        for _ in range(args.reps):
            fn()
        times[name] = (time.perf_counter() - t0) / args.reps
    # oracle check on a sample of pairs (outside the timed region)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_ffi as O
    checked = 0
    for p in range(0, P, max(1, P // args.check)):
        f = O.bloom_build([bytes(ha[p * K + i]) for i in range(K)])
        assert bytes(filt[int(foff[p]):int(foff[p + 1])]) == f, p
        for i in range(K):
            assert bool(contains[p * K + i]) == O.bloom_contains(f, bytes(hb[p * K + i])), (p, i)
        checked += 1
    fp = float(contains.mean())
    line = {"workload": "C5: %d doc pairs, %d hashes per side" % (P, K), "pairs": P,
            "build": {"hashes_per_s": P * K / times["build"], "ms": times["build"] * 1e3},
            "probe": {"probes_per_s": P * K / times["probe"], "ms": times["probe"] * 1e3, "false_positive_rate": fp},
            "select": {"pairs_per_s": P / times["select"], "ms": times["select"] * 1e3,
                       "sent_fraction": float(send.mean())},
            "timing": "C ABI end to end (H2D + kernel + D2H), mean of %d calls" % args.reps,
            "verified_pairs": checked}
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
