"""Synthetic workloads for bench.py and the tests: workload/libam_workload.so
(am_workload.cpp), a host-side generator kept out of the engine library."""
import ctypes as C
import os

import numpy as np

from automerge_amd.batch import CHUNK_DT, DOC_DT

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "libam_workload.so")
if not os.path.exists(_LIB):
    raise ImportError("workload: %s is missing; build it with `make -C workload` (or __graft_entry__.build())" % _LIB)
lib = C.CDLL(_LIB)
_P = C.c_void_p
for _name, _res, _args in (
        ("am_workload_c4", C.c_uint64, [C.c_uint64, C.c_uint32, _P, C.c_uint64, _P, _P, C.POINTER(C.c_uint64), C.c_int]),
        ("am_workload_c5", C.c_uint64, [C.c_uint64, C.c_uint32, C.c_uint32, _P, C.c_uint64, _P, _P, C.POINTER(C.c_uint64),
                                        C.c_int]),
        ("am_workload_c2", C.c_uint64, [C.c_uint64, C.c_uint32, _P, C.c_uint64, _P, _P, C.POINTER(C.c_uint64), C.c_int]),
        ("am_workload_text", C.c_uint64, [C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, _P, C.c_uint64, _P, _P,
                                          C.POINTER(C.c_uint64), C.c_int]),
        ("am_workload_mid", C.c_uint64, [C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, _P, C.c_uint64,
                                         _P, _P, C.POINTER(C.c_uint64), C.c_int]),
        ("am_workload_c4_shard", C.c_uint64, [C.c_uint64, C.c_uint64, C.c_uint32, C.c_uint32, _P, C.c_uint64, C.c_int]),
        ("am_workload_c4_list", C.c_uint64, [_P, C.c_uint32, _P, C.c_uint64, _P, _P, C.POINTER(C.c_uint64), C.c_int])):
    _f = getattr(lib, _name)
    _f.restype = _res
    _f.argtypes = _args



def c4(first, n, nthreads=None):
    """C4 documents [first, first+n): (arena, chunks, docs, ops_in_changes)."""
    nthreads = nthreads or min(16, os.cpu_count() or 1)
    ops = C.c_uint64()
    need = lib.am_workload_c4(first, n, None, 0, None, None, C.byref(ops), nthreads)
    arena = np.empty(need, np.uint8)
    chunks = np.empty(13 * n, CHUNK_DT)
    docs = np.empty(n, DOC_DT)
    got = lib.am_workload_c4(first, n, arena.ctypes.data, need, chunks.ctypes.data, docs.ctypes.data, C.byref(ops),
                               nthreads)
    assert got == need
    return arena, chunks, docs, int(ops.value)


def c2(first, n, nthreads=None):
    """C2 documents [first, first+n) (configs[1]): Backend.init() + 3 changes each; returns
    (arena, chunks, docs, ops_in_changes)."""
    nthreads = nthreads or min(16, os.cpu_count() or 1)
    ops = C.c_uint64()
    need = lib.am_workload_c2(first, n, None, 0, None, None, C.byref(ops), nthreads)
    arena = np.empty(need, np.uint8)
    chunks = np.empty(3 * n, CHUNK_DT)
    docs = np.empty(n, DOC_DT)
    got = lib.am_workload_c2(first, n, arena.ctypes.data, need, chunks.ctypes.data, docs.ctypes.data, C.byref(ops),
                               nthreads)
    assert got == need
    return arena, chunks, docs, int(ops.value)


def c5(first, n, per_side=10, nthreads=None):
    """C5 document pairs [first, first+n): (arena, chunks, docs, ops); pair i = the base chunk, side
    A's per_side changes, then side B's (chunk order)."""
    nthreads = nthreads or min(16, os.cpu_count() or 1)
    ops = C.c_uint64()
    need = lib.am_workload_c5(first, n, per_side, None, 0, None, None, C.byref(ops), nthreads)
    arena = np.empty(need, np.uint8)
    chunks = np.empty((1 + 2 * per_side) * n, CHUNK_DT)
    docs = np.empty(n, DOC_DT)
    got = lib.am_workload_c5(first, n, per_side, arena.ctypes.data, need, chunks.ctypes.data, docs.ctypes.data,
                             C.byref(ops), nthreads)
    assert got == need
    return arena, chunks, docs, int(ops.value)


def text(first, n, nchanges, per_change=100, cross_every=10, nthreads=None):
    """Text editing histories (C1: cross_every=0; C3: cross_every=10), documents [first, first+n):
    Backend.init() + (1 + nchanges) change chunks each, the ones >= 256 B deflated (type 2, as
    encodeChange writes them). Returns (arena, chunks, docs, ops)."""
    nthreads = nthreads or min(16, os.cpu_count() or 1)
    ops = C.c_uint64()
    need = lib.am_workload_text(first, n, nchanges, per_change, cross_every, None, 0, None, None, C.byref(ops),
                                  nthreads)
    arena = np.empty(need, np.uint8)
    chunks = np.empty((1 + nchanges) * n, CHUNK_DT)
    docs = np.empty(n, DOC_DT)
    got = lib.am_workload_text(first, n, nchanges, per_change, cross_every, arena.ctypes.data, need,
                                 chunks.ctypes.data, docs.ctypes.data, C.byref(ops), nthreads)
    assert got == need
    return arena, chunks, docs, int(ops.value)


def mid(first, n, nactors=4, rounds=12, min_ops=8, max_ops=40, nthreads=None):
    """Mid-size documents (am_workload.cpp gen_mid): Backend.init() + 1 + nactors * rounds change
    chunks each, rounds of concurrent text / title edits by nactors actors (200-2,000 ops per
    document with the defaults). Returns (arena, chunks, docs, ops)."""
    nthreads = nthreads or min(16, os.cpu_count() or 1)
    ops = C.c_uint64()
    args = (first, n, nactors, rounds, min_ops, max_ops)
    need = lib.am_workload_mid(*args, None, 0, None, None, C.byref(ops), nthreads)
    assert need, "workload.mid: bad parameters"
    arena = np.empty(need, np.uint8)
    chunks = np.empty((1 + nactors * rounds) * n, CHUNK_DT)
    docs = np.empty(n, DOC_DT)
    got = lib.am_workload_mid(*args, arena.ctypes.data, need, chunks.ctypes.data, docs.ctypes.data, C.byref(ops), nthreads)
    assert got == need
    return arena, chunks, docs, int(ops.value)


def c4_shard(first, n, world, rank, nthreads=None):
    """Indexes of the C4 documents [first, first+n) that rank `rank` of `world` merges: the base
    document's SHA-256 (container checksum) first byte mod world."""
    nthreads = nthreads or min(16, os.cpu_count() or 1)
    ids = np.empty(max(n // max(world, 1) * 2 + 64, 64), np.uint64)
    k = int(lib.am_workload_c4_shard(first, n, world, rank, ids.ctypes.data, len(ids), nthreads))
    if k > len(ids):
        ids = np.empty(k, np.uint64)
        k = int(lib.am_workload_c4_shard(first, n, world, rank, ids.ctypes.data, len(ids), nthreads))
    return ids[:k].copy()


def c4_list(ids, nthreads=None):
    """C4 documents with the given indexes: (arena, chunks, docs, ops_in_changes)."""
    nthreads = nthreads or min(16, os.cpu_count() or 1)
    ids = np.ascontiguousarray(ids, dtype=np.uint64)
    n = len(ids)
    ops = C.c_uint64()
    need = lib.am_workload_c4_list(ids.ctypes.data, n, None, 0, None, None, C.byref(ops), nthreads)
    arena = np.empty(need, np.uint8)
    chunks = np.empty(13 * n, CHUNK_DT)
    docs = np.empty(n, DOC_DT)
    got = lib.am_workload_c4_list(ids.ctypes.data, n, arena.ctypes.data, need, chunks.ctypes.data, docs.ctypes.data,
                                  C.byref(ops), nthreads)
    assert got == need
    return arena, chunks, docs, int(ops.value)


def doc_chunks(arena, chunks, docs, i):
    """(base bytes, [change bytes]) of document i (for checks)."""
    d = docs[i]
    get = lambda k: bytes(arena[int(chunks[k]["off"]):int(chunks[k]["off"]) + int(chunks[k]["len"])])
    base = get(int(d["base_chunk"])) if d["base_chunk"] >= 0 else None
    return base, [get(int(d["chg_begin"]) + j) for j in range(int(d["chg_count"]))]
