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


def _ptrs(n):
    return np.zeros(max(n, 1), np.uint64)


def e2e(args):
    """The whole sync of P document pairs (sync.js:327-473 on both peers until neither has a
    message): every round is ONE am_sync_generate over all 2P documents and ONE
    am_sync_receive_batch over every delivered message (their changes applied in one batched
    applyChanges with patches). State blobs and messages stay engine-owned pointers between calls."""
    from automerge_amd import _native as N
    import workload
    P, K = args.pairs, args.per_side
    t0 = time.perf_counter()
    arena, chunks, docs, _ = workload.c5(0, P, K)
    gen_s = time.perf_counter() - t0
    eng = N.engine(0)
    base = [None] * P
    side = [[], []]
    for i in range(P):
        d = docs[i]
        b0 = int(d["base_chunk"])
        get = lambda k: bytes(arena[int(chunks[k]["off"]):int(chunks[k]["off"]) + int(chunks[k]["len"])])  # noqa: E731
        base[i] = get(b0)
        cb = int(d["chg_begin"])
        side[0].append([get(cb + j) for j in range(K)])
        side[1].append([get(cb + K + j) for j in range(K)])
    # setup (untimed): load every side's base and apply its own chain, batched
    n = 2 * P
    bufs = base + base
    arr = (C.c_char_p * n)(*bufs)
    lens = (C.c_size_t * n)(*[len(b) for b in bufs])
    handles = _ptrs(n)
    codes = np.zeros(n, np.uint32)
    t0 = time.perf_counter()
    bad = N.lib.am_doc_load_batch(eng, n, arr, lens, handles.ctypes.data, codes.ctypes.data, None)
    load_s = time.perf_counter() - t0
    assert bad == 0, int(bad)
    flat = [c for s in (0, 1) for i in range(P) for c in side[s][i]]
    carr = (C.c_char_p * len(flat))(*flat)
    clen = (C.c_size_t * len(flat))(*[len(c) for c in flat])
    off = np.arange(n + 1, dtype=np.uint64) * K
    t0 = time.perf_counter()
    bad = N.lib.am_doc_apply_changes_batch(n, handles.ctypes.data, off.ctypes.data, carr, clen, None, None, None,
                                           codes.ctypes.data, None)
    setup_apply_s = time.perf_counter() - t0
    assert bad == 0, int(bad)
    # resumed sync states (decodeSyncState of a persisted state, sync.js:217-225): sharedHeads = the
    # base's head, which is the one dependency of each side's first change (chunk header: magic,
    # checksum, type, uleb length, then uleb #deps + 32-byte hashes)
    keep = []
    st = _ptrs(n)
    stl = np.zeros(n, np.uint64)
    for i in range(n):
        c = side[0][i % P][0]
        o = 9
        while c[o] & 0x80:
            o += 1
        o += 1
        assert c[o] == 1, "a side's first change depends on the base head only"
        blob = b"\x53\x00\x01" + bytes(c[o + 1:o + 33]) + b"\x00\x00"
        keep.append(blob)
        st[i] = C.cast(C.c_char_p(blob), C.c_void_p).value
        stl[i] = len(blob)
    peer = np.concatenate([np.arange(P, n), np.arange(0, P)]).astype(np.int64)
    owned_states = False
    rounds, msgs_total, changes_bytes = 0, 0, 0
    t_gen = t_recv = 0.0
    t_start = time.perf_counter()
    while True:
        ost, ostl = _ptrs(n), np.zeros(n, np.uint64)
        msg, ml = _ptrs(n), np.zeros(n, np.uint64)
        t0 = time.perf_counter()
        bad = N.lib.am_sync_generate(n, handles.ctypes.data, st.ctypes.data, stl.ctypes.data, ost.ctypes.data,
                                     ostl.ctypes.data, msg.ctypes.data, ml.ctypes.data, codes.ctypes.data, None)
        t_gen += time.perf_counter() - t0
        assert bad == 0, int(bad)
        if owned_states:
            for p in st:
                N.lib.am_free(C.c_void_p(int(p)))
        st, stl, owned_states = ost, ostl, True
        senders = np.nonzero(msg)[0]
        if len(senders) == 0:
            break
        rounds += 1
        msgs_total += len(senders)
        changes_bytes += int(ml[senders].sum())
        recv = peer[senders]
        m = len(recv)
        rh, rs, rsl = handles[recv].copy(), st[recv].copy(), stl[recv].copy()
        mm, mml = msg[senders].copy(), ml[senders].copy()
        ost2, ostl2 = _ptrs(m), np.zeros(m, np.uint64)
        pat, pl = _ptrs(m), np.zeros(m, np.uint64)
        rc = np.zeros(m, np.uint32)
        t0 = time.perf_counter()
        bad = N.lib.am_sync_receive_batch(m, rh.ctypes.data, rs.ctypes.data, rsl.ctypes.data, mm.ctypes.data,
                                          mml.ctypes.data, ost2.ctypes.data, ostl2.ctypes.data, pat.ctypes.data,
                                          pl.ctypes.data, None, rc.ctypes.data, None)
        t_recv += time.perf_counter() - t0
        assert bad == 0, (int(bad), int(rc[rc != 0][0]) if bad else 0)
        for p in list(st[recv]) + list(mm) + list(pat[pat != 0]):
            N.lib.am_free(C.c_void_p(int(p)))
        st[recv], stl[recv] = ost2, ostl2
        assert rounds < 20, "sync did not converge"
    total_s = time.perf_counter() - t_start
    for p in st:
        N.lib.am_free(C.c_void_p(int(p)))
    # every pair converged: equal heads; a sample of documents equals the CPU oracle's merge
    hb = (C.c_uint8 * 64)()
    hb2 = (C.c_uint8 * 64)()
    for i in range(P):
        na = N.lib.am_doc_get_heads(C.c_void_p(int(handles[i])), hb, 2)
        nb = N.lib.am_doc_get_heads(C.c_void_p(int(handles[i + P])), hb2, 2)
        assert na == nb == 2 and bytes(hb) == bytes(hb2), i
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_ffi as O
    checked = 0
    for i in range(0, P, max(1, P // args.check)):
        for s_, first, second in ((i, 0, 1), (i + P, 1, 0)):
            o = O.Doc.load(base[i])
            o.apply(side[first][i])
            o.apply(side[second][i])
            out, ln = N.u8p(), C.c_size_t()
            err = N.Error()
            assert not N.lib.am_doc_save(C.c_void_p(int(handles[s_])), C.byref(out), C.byref(ln), C.byref(err))
            assert N.take(out, ln.value) == o.save(), (i, s_)
        checked += 1
    for h in handles:
        N.lib.am_doc_free(C.c_void_p(int(h)))
    return {"workload": "C5 end to end: %d document pairs, %d concurrent changes per side since the last sync" % (P, K),
            "pairs": P, "pairs_per_s": P / total_s, "seconds": total_s, "rounds": rounds, "messages": msgs_total,
            "message_bytes": changes_bytes, "generate_s": t_gen, "receive_s": t_recv,
            "setup": {"load_batch_docs_per_s": n / load_s, "apply_batch_docs_per_s": n / setup_apply_s,
                      "generator_s": gen_s},
            "timing": "am_sync_generate + am_sync_receive_batch wall clock (host + GPU), state blobs and messages "
                      "passed between calls as engine-owned buffers",
            "verified": {"pairs_converged": P, "oracle_checked_pairs": checked}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=100000)
    ap.add_argument("--per-side", type=int, default=10)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--check", type=int, default=200)
    ap.add_argument("--e2e", action="store_true", help="the whole sync of the pairs (generate/receive rounds)")
    ap.add_argument("--dump", help="write the C5 pairs (u32 length + bytes: base, side A's, side B's changes) to this "
                                   "file for tools/cpu_reference_sync.js, and exit")
    args = ap.parse_args()
    if args.dump:
        import struct
        import workload
        arena, chunks, docs, _ = workload.c5(0, args.pairs, args.per_side)
        with open(args.dump, "wb") as f:
            f.write(struct.pack("<II", args.pairs, args.per_side))
            for i in range(args.pairs):
                base, ch = workload.doc_chunks(arena, chunks, docs, i)
                for b in [base] + ch:
                    f.write(struct.pack("<I", len(b)) + b)
        return
    if args.e2e:
        print(json.dumps(e2e(args)), flush=True)
        return
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
