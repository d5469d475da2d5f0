"""sync.js Bloom filters and change selection on the MI355X engine.

`BloomFilter` mirrors the reference class (sync.js:38-125): built from a list of hex hashes or
decoded from bytes, `.bytes`, `.containsHash(hash)`, with the same errors. The batched
functions are the C5 shape: thousands of filters or document pairs per launch.

    build_filters([[hash, ...], ...])        -> [bytes, ...]           (k_bloom_build)
    probe(filters, [(filter_index, hash)])   -> [bool, ...]            (k_bloom_probe)
    select_changes(pairs)                    -> [[send flags], ...]    (k_sync_select)

Hashes are 32-byte `bytes` (or 64-char hex strings). There is no CPU path: every call runs the
HIP kernels of am_sync.hip and fails loudly without a device.
"""
import ctypes as C

import numpy as np

from . import _native as N


def _hash_bytes(h):
    if isinstance(h, str):
        b = bytes.fromhex(h) if len(h) % 2 == 0 else b""
    else:
        b = bytes(h)
    if len(b) != 32:
        raise N.AutomergeError("Not a 256-bit hash: %s" % (h if isinstance(h, str) else bytes(h).hex()), kind="RangeError")
    return b


def build_filters(hash_lists, device=0):
    """new BloomFilter(hashes).bytes for every list (sync.js:38-47, 66-77)."""
    nf = len(hash_lists)
    hoff = np.zeros(nf + 1, dtype=np.uint64)
    for i, hs in enumerate(hash_lists):
        hoff[i + 1] = hoff[i] + len(hs)
    flat = b"".join(_hash_bytes(h) for hs in hash_lists for h in hs)
    total = sum(int(N.lib.am_bloom_encoded_size(len(hs))) for hs in hash_lists)
    out = C.create_string_buffer(max(total, 1))
    foff = np.zeros(nf + 1, dtype=np.uint64)
    err = N.Error()
    if nf and N.lib.am_bloom_build(N.engine(device), flat or b"\0", hoff.ctypes.data, nf, out, total, foff.ctypes.data,
                                   C.byref(err)):
        N.raise_for(err)
    raw = out.raw
    return [raw[int(foff[i]):int(foff[i + 1])] for i in range(nf)]


def _filter_arena(filters):
    foff = np.zeros(len(filters) + 1, dtype=np.uint64)
    for i, f in enumerate(filters):
        foff[i + 1] = foff[i] + len(f)
    return C.create_string_buffer(b"".join(bytes(f) for f in filters) or b"\0"), foff


def probe(filters, probes, device=0):
    """containsHash for each (filter_index, hash) (sync.js:112-125); malformed filters raise the
    RangeError their decode raises in the reference."""
    if not probes:
        return []
    fbuf, foff = _filter_arena(filters)
    pf = np.array([int(i) for i, _ in probes], dtype=np.uint32)
    ph = b"".join(_hash_bytes(h) for _, h in probes)
    out = C.create_string_buffer(len(probes))
    err = N.Error()
    if N.lib.am_bloom_probe(N.engine(device), fbuf, foff.ctypes.data, len(filters), ph, pf.ctypes.data, len(probes), out,
                            C.byref(err)):
        N.raise_for(err)
    return [b == 1 for b in out.raw]


def select_changes(pairs, device=0):
    """getChangesToSend selection for many document pairs (sync.js:246-306, `have` non-empty).
    pairs: list of (hashes, deps, filters): change hashes in getChanges order, deps[i] = indexes
    of change i's dependencies within the list (-1 = not in the list), the peer's encoded filters.
    Returns per pair the list of send flags (the caller adds explicitly needed changes)."""
    npairs = len(pairs)
    coff = np.zeros(npairs + 1, dtype=np.uint64)
    pfoff = np.zeros(npairs + 1, dtype=np.uint64)
    hashes, deps, filters = [], [], []
    for p, (hs, ds, fs) in enumerate(pairs):
        coff[p + 1] = coff[p] + len(hs)
        pfoff[p + 1] = pfoff[p] + len(fs)
        hashes += [_hash_bytes(h) for h in hs]
        deps += list(ds)
        filters += list(fs)
    nc = int(coff[-1])
    doff = np.zeros(nc + 1, dtype=np.uint64)
    for i, d in enumerate(deps):
        doff[i + 1] = doff[i] + len(d)
    didx = np.array([x for d in deps for x in d] or [0], dtype=np.int32)
    fbuf, foff = _filter_arena(filters)
    send = C.create_string_buffer(max(nc, 1))
    err = N.Error()
    if npairs and N.lib.am_sync_select(N.engine(device), npairs, coff.ctypes.data, b"".join(hashes) or b"\0",
                                       doff.ctypes.data, didx.ctypes.data, pfoff.ctypes.data, fbuf, foff.ctypes.data,
                                       send, C.byref(err)):
        N.raise_for(err)
    raw = send.raw
    return [list(raw[int(coff[p]):int(coff[p + 1])]) for p in range(npairs)]


class BloomFilter:
    """sync.js:38-125 on the engine: BloomFilter(list_of_hex_hashes) or BloomFilter(bytes)."""

    def __init__(self, arg, device=0):
        self.device = device
        if isinstance(arg, list):
            self._bytes = build_filters([arg], device)[0]
        elif isinstance(arg, (bytes, bytearray, memoryview)):
            self._bytes = bytes(arg)
            if self._bytes:  # decode now so malformed input raises here, as in the reference
                probe([self._bytes], [(0, bytes(32))], device)
        else:
            raise N.AutomergeError("invalid argument", kind="TypeError")

    @property
    def bytes(self):
        return self._bytes

    def containsHash(self, h):
        return probe([self._bytes], [(0, h)], self.device)[0]
