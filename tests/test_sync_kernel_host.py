"""The per-thread bodies of the sync kernels (am_sync.hip: bloom_build_one, bloom_test,
sync_select_one -- the exact code the GPU threads run) compiled for the host with
-DAM_SYNC_HOST_CHECK and checked against the reference's Bloom vectors (tests/golden/bloom.json)
and the CPU oracle. The GPU launches themselves are covered by tests/test_gpu_sync.py."""
import ctypes as C
import os
import random
import shutil
import subprocess

import pytest

import oracle_ffi as O
from conftest import golden

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, "tests", "_build")
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"


@pytest.fixture(scope="module")
def harness():
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not available")
    os.makedirs(BUILD, exist_ok=True)
    out = os.path.join(BUILD, "libsync_host.so")
    src = os.path.join(ROOT, "automerge_amd", "csrc", "am_sync.hip")
    subprocess.check_call([HIPCC, "-O2", "-std=c++17", "--offload-arch=gfx950", "-fPIC", "-shared", "-DAM_SYNC_HOST_CHECK",
                           src, "-o", out, "-L", os.path.join(ROOT, "automerge_amd"), "-lautomerge_amd",
                           "-Wl,-rpath," + os.path.join(ROOT, "automerge_amd")])
    L = C.CDLL(out)
    L.amx_bloom_build_one.argtypes = [C.c_char_p, C.c_uint64, C.c_char_p, C.c_int]
    L.amx_bloom_test.restype = C.c_uint8
    L.amx_bloom_test.argtypes = [C.c_char_p, C.c_uint64, C.c_char_p]
    L.amx_sync_select_one.restype = C.c_uint8
    L.amx_sync_select_one.argtypes = [C.c_void_p] * 8
    return L


def build(L, hashes, slot):
    n = len(hashes)
    if n == 0:
        return b""
    size = len(O.bloom_build(hashes))
    buf = C.create_string_buffer(size)
    L.amx_bloom_build_one(b"".join(hashes), n, buf, 1 if slot else 0)
    return buf.raw


def test_kernel_bloom_bodies_match_reference(harness):
    for v in golden("bloom.json"):
        hashes = [bytes.fromhex(h) for h in v["hashes"]]
        for slot in (True, False):
            assert build(harness, hashes, slot).hex() == v["bytes"]
        f = bytes.fromhex(v["bytes"])
        for h, c in zip(v["probes"], v["contains"]):
            assert harness.amx_bloom_test(f, len(f), bytes.fromhex(h)) == int(c)


def test_kernel_bloom_large_filters_match_oracle(harness):
    rnd = random.Random(11)
    for n in (51, 52, 200, 1000):  # around the 64-byte LDS slot limit, and far above it
        hashes = [rnd.randbytes(32) for _ in range(n)]
        ref = O.bloom_build(hashes)
        assert build(harness, hashes, True) == ref
        assert build(harness, hashes, False) == ref
        for _ in range(50):
            h = rnd.randbytes(32)
            assert harness.amx_bloom_test(ref, len(ref), h) == O.bloom_contains(ref, h)


def test_kernel_bloom_malformed(harness):
    f = O.bloom_build([bytes(range(32))])
    assert harness.amx_bloom_test(f[:-1], len(f) - 1, bytes(32)) == 4          # subarray
    assert harness.amx_bloom_test(b"\x80", 1, bytes(32)) == 3                  # incomplete
    assert harness.amx_bloom_test(b"\xff\xff\xff\xff\x7f", 5, bytes(32)) == 2  # out of range
    big = b"\x01\x0a\xff\xff\x03" + b"\xff" * 2                                  # numProbes 65535
    assert harness.amx_bloom_test(big, len(big), bytes(32)) == 5


def test_kernel_select_body_matches_oracle(harness):
    import numpy as np
    rnd = random.Random(3)
    for trial in range(200):
        n = rnd.randint(0, 12)
        hashes = [rnd.randbytes(32) for _ in range(n)]
        deps = [[rnd.randint(-1, i - 1) for _ in range(rnd.randint(0, 2))] if i else [] for i in range(n)]
        nf = rnd.randint(1, 3)
        filters = [O.bloom_build([h for h in hashes if rnd.random() < 0.6]) for _ in range(nf)]
        ref = O.sync_select(hashes, deps, filters)
        coff = np.array([0, n], dtype=np.uint64)
        doff = np.zeros(n + 1, dtype=np.uint64)
        for i, d in enumerate(deps):
            doff[i + 1] = doff[i] + len(d)
        didx = np.array([x for d in deps for x in d] or [0], dtype=np.int32)
        pfoff = np.array([0, nf], dtype=np.uint64)
        foff = np.zeros(nf + 1, dtype=np.uint64)
        for i, f in enumerate(filters):
            foff[i + 1] = foff[i] + len(f)
        fbuf = C.create_string_buffer(b"".join(filters) or b"\0")
        hbuf = C.create_string_buffer(b"".join(hashes) or b"\0")
        send = C.create_string_buffer(max(n, 1))
        st = harness.amx_sync_select_one(coff.ctypes.data, C.addressof(hbuf), doff.ctypes.data, didx.ctypes.data,
                                         pfoff.ctypes.data, C.addressof(fbuf), foff.ctypes.data, C.addressof(send))
        assert st == 0
        assert list(send.raw[:n]) == ref, (trial, deps)


def test_kernel_bloom_edge_vectors(harness):
    """numProbes 0 still tests one bit (getProbes returns [x], sync.js:95-100); malformed headers
    decode to the reference's RangeError kinds (tests/golden/bloom_edge.json)."""
    kinds = {"subarray exceeds buffer size": 4, "buffer ended with incomplete number": 3, "number out of range": 2}
    for v in golden("bloom_edge.json"):
        f = bytes.fromhex(v["bytes"])
        for i, h in enumerate(v["probes"]):
            got = harness.amx_bloom_test(f, len(f), bytes.fromhex(h))
            if v["error"]:
                assert got == kinds[v["error"]["message"]], v
            else:
                assert got == int(v["contains"][i]), (v["bytes"], i)
