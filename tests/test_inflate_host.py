"""The engine's raw DEFLATE decoder (automerge_amd/csrc/am_inflate_dec.h: the per-lane code of the
k_inflate_* kernels; both forms, the short-stream one and the long-stream
one with one-lookup tables) compiled for the host and checked against zlib's raw
inflate (the reference calls pako.inflateRaw, columnar.js:816 and :1064; inflate is unambiguous):
every block type, long and short back-references (distances below and above 16 bytes, overlapping
copies), streams starting at every alignment, and malformed streams that must be rejected. The same
corpus runs on the GPU in tests/test_gpu_inflate.py."""
import os
import random
import shutil
import struct
import subprocess
import zlib

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, "tests", "_build")


@pytest.fixture(scope="module")
def inflate_host():
    cxx = shutil.which("g++")
    if not cxx:
        pytest.skip("g++ not available")
    os.makedirs(BUILD, exist_ok=True)
    exe = os.path.join(BUILD, "inflate_host")
    subprocess.check_call([cxx, "-O2", "-std=c++17", "-Wall", "-Wno-unused-function",
                           os.path.join(ROOT, "tests", "native", "inflate_host.cpp"), "-o", exe])
    return exe


def _run(exe, streams, tmp):
    src, dst = os.path.join(tmp, "z.bin"), os.path.join(tmp, "o.bin")
    with open(src, "wb") as f:
        for z in streams:
            f.write(struct.pack("<I", len(z)) + z)
    subprocess.check_call([exe, src, dst])
    data = open(dst, "rb").read()
    out, off = [], 0
    while off < len(data):
        ok = data[off]
        (n,) = struct.unpack_from("<I", data, off + 1)
        out.append(data[off + 5:off + 5 + n] if ok else None)
        off += 5 + n
    # two results per stream: the short-stream decoder, then the long-stream one; they must agree
    short, long_ = out[0::2], out[1::2]
    assert short == long_, [i for i, (a, b) in enumerate(zip(short, long_)) if a != b][:10]
    return short


def _deflate(data, level=6, strategy=zlib.Z_DEFAULT_STRATEGY):
    c = zlib.compressobj(level, zlib.DEFLATED, -15, 8, strategy)
    return c.compress(data) + c.flush()


def _corpus(rng):
    out = [b"", b"a", bytes(range(256)), b"abc" * 1000, b"\x00" * 70000]
    for period in range(1, 40):  # every short distance, long overlapping copies
        pat = bytes(rng.getrandbits(8) for _ in range(period))
        out.append((pat * (3000 // period + 2))[:3000 + period])
    for n in (10, 100, 255, 256, 1000, 5000, 40000, 150000):
        text = bytes(rng.choice(b"abcdefghij      ") for _ in range(n))
        noise = bytes(rng.getrandbits(8) for _ in range(n))
        mixed = bytes(text[i] if (i // 64) % 3 else noise[i] for i in range(n))
        out += [text, noise, mixed]
    return out


def test_host_decoder_matches_zlib(inflate_host, tmp_path):
    rng = random.Random(77)
    data, streams = [], []
    for d in _corpus(rng):
        for level, strat in [(6, zlib.Z_DEFAULT_STRATEGY), (0, zlib.Z_DEFAULT_STRATEGY), (1, zlib.Z_DEFAULT_STRATEGY),
                             (9, zlib.Z_DEFAULT_STRATEGY), (6, zlib.Z_FIXED), (6, zlib.Z_HUFFMAN_ONLY), (6, zlib.Z_RLE)]:
            data.append(d)
            streams.append(_deflate(d, level, strat))
    c = zlib.compressobj(6, zlib.DEFLATED, -15)
    pieces = [bytes(rng.choice(b"xyz ") for _ in range(rng.randint(0, 300))) for _ in range(50)]
    s = b""
    for p in pieces:
        s += c.compress(p) + c.flush(zlib.Z_SYNC_FLUSH)
    s += c.flush()
    data.append(b"".join(pieces))
    streams.append(s)
    got = _run(inflate_host, streams, str(tmp_path))
    bad = [i for i, (d, g) in enumerate(zip(data, got)) if g != d]
    assert not bad, bad[:10]


def test_host_decoder_rejects_malformed(inflate_host, tmp_path):
    good = _deflate(b"hello hello hello world" * 20)
    bad = [
        b"\x07",                            # block type 3 (reserved)
        good[: len(good) // 2],             # truncated
        good[:-1],                          # truncated by one byte
        b"\x01\x05\x00\x00\x00abc",         # stored block with LEN != ~NLEN
        b"\x01\x05\x00\xfa\xffab",          # stored block longer than the input
        bytes.fromhex("030200"),            # fixed block: a match at output position 0 (distance too far back)
    ]
    rng = random.Random(5)
    for _ in range(200):  # random corruptions: whatever the decoder returns must be zlib's answer
        z = bytearray(_deflate(bytes(rng.choice(b"abcde") for _ in range(500))))
        z[rng.randrange(len(z))] ^= 1 << rng.randrange(8)
        bad.append(bytes(z))
    got = _run(inflate_host, bad + [good], str(tmp_path))
    assert got[:6] == [None] * 6
    for z, g in zip(bad[6:], got[6:-1]):
        try:
            want = zlib.decompress(z, -15)
        except zlib.error:
            want = None
        if want is not None and g is not None:
            assert g == want
        # zlib tolerates trailing garbage after the final block that the raw decoder also ignores;
        # a stream zlib rejects must never come back as data
        if want is None:
            assert g is None, z.hex()
    assert got[-1] == zlib.decompress(good, -15)
