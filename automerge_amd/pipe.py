"""Pipelined batches (am_pipe_* in include/automerge_amd.h): a stream of batches of documents, each
Backend.load + Backend.applyChanges per document, from host memory back to host memory. The H2D
copy of the next batch and the D2H copy of the previous one overlap the kernels of the current one.

    p = Pipeline(arena_bytes, chunks, docs, ws_bytes, out_bytes, patch_bytes, fast_lds, slots=3)
    for arena, chunks, docs in batches:                            # pinned inputs (pinned_copy)
        p.submit(arena, chunks, docs, summary, out, patches)       # pinned outputs (Pinned views)
    totals = p.drain()                                             # every batch is home

The capacities are per batch (bench.py sizes them from one staged batch: Batch.workspace_bytes()
and the output lengths of a run, with headroom). A document whose merged chunk or patch log does
not fit the device arenas or the caller's `out` / `patches` reports AM_U_CAPACITY in its summary.

Each document's merged chunk is out[s.out_off : s.out_off + s.out_len] and its patch log (wire form,
automerge_amd/patch.py) patches[s.patch_off : s.patch_off + s.patch_len] for its summary s.
"""
import ctypes as C

import numpy as np

from . import _native as N
from .batch import CHUNK_DT, DOC_DT

DOC_META = 32  # AM_DOC_META: not accepted by a packed batch
# am_doc_span (am_pipe_submit_packed): change chunks, am_doc_desc flags, base-document bit
SPAN_DT = np.dtype([("chg_count", "<u4"), ("flags", "<u2"), ("has_base", "u1"), ("reserved", "u1")])
SUMMARY_DT = np.dtype([("status", "<u4"), ("nqueued", "<u4"), ("out_len", "<u4"), ("patch_len", "<u4"),
                       ("out_off", "<u8"), ("patch_off", "<u8")])
assert SUMMARY_DT.itemsize == C.sizeof(N.DocSummary)


def pack(chunks, docs):
    """(chunk_len, spans) of am_pipe_submit_packed for full descriptors whose chunks lie back to back
    from arena offset 0 and whose documents take consecutive chunks (base first), or None when the
    batch does not have that shape (then use submit)."""
    off = chunks["off"].astype(np.int64)
    ln = chunks["len"].astype(np.int64)
    if len(chunks) and (off[0] != 0 or np.any(off[1:] != off[:-1] + ln[:-1]) or np.any(chunks["flags"] != 0)):
        return None
    hb = docs["base_chunk"] >= 0
    cnt = docs["chg_count"].astype(np.int64)
    first = np.concatenate([[0], np.cumsum(hb.astype(np.int64) + cnt)[:-1]]) if len(docs) else np.zeros(0, np.int64)
    if (np.any(hb & (docs["base_chunk"] != first)) or np.any(docs["chg_begin"] != first + hb)
            or np.any(docs["known_count"] != 0) or np.any(docs["flags"] >= (1 << 16))
            or np.any(docs["flags"] & DOC_META)
            or (len(docs) and first[-1] + hb[-1] + cnt[-1] != len(chunks))):
        return None
    spans = np.zeros(len(docs), SPAN_DT)
    spans["chg_count"] = cnt
    spans["flags"] = docs["flags"]
    spans["has_base"] = hb
    return ln.astype(np.uint32), spans


class Pinned:
    """A numpy view of pinned host memory (am_host_alloc)."""

    def __init__(self, nbytes):
        self.nbytes = max(int(nbytes), 1)
        self.ptr = N.lib.am_host_alloc(self.nbytes)
        if not self.ptr:
            raise MemoryError("automerge_amd: pinned allocation of %d bytes failed" % self.nbytes)
        self.u8 = np.ctypeslib.as_array((C.c_uint8 * self.nbytes).from_address(self.ptr))

    def view(self, dtype, count=None, offset=0):
        dtype = np.dtype(dtype)
        if count is None:
            count = (self.nbytes - offset) // dtype.itemsize
        return self.u8[offset:offset + count * dtype.itemsize].view(dtype)

    def __del__(self):
        if getattr(self, "ptr", None):
            N.lib.am_host_free(self.ptr)
            self.ptr = None


def pinned_copy(arr):
    """A Pinned buffer holding a copy of a numpy array; `.arr` is the copy (keep the buffer alive)."""
    arr = np.ascontiguousarray(arr)
    p = Pinned(arr.nbytes)
    p.arr = p.view(arr.dtype, arr.size).reshape(arr.shape)
    p.arr[...] = arr
    return p


class Pipeline:
    def __init__(self, arena_bytes, chunks, docs, ws_bytes, out_bytes, patch_bytes, fast_lds, slots=3, device=0):
        self._eng = N.engine(device)
        self.caps = N.PipeCaps(int(arena_bytes), int(chunks), int(docs), int(ws_bytes), int(out_bytes), int(patch_bytes),
                               int(fast_lds), int(slots))
        err = N.Error()
        self._p = N.lib.am_pipe_create(self._eng, C.byref(self.caps), C.byref(err))
        if not self._p:
            N.raise_for(err)
        self._keep = {}

    def __del__(self):
        if getattr(self, "_p", None):
            N.lib.am_pipe_destroy(self._p)
            self._p = None

    def submit(self, arena, chunks, docs, summary, out, patches):
        """Enqueues one batch. All arrays should be pinned (pinned_copy / Pinned views) and must stay
        alive until drain()."""
        assert chunks.dtype == CHUNK_DT and docs.dtype == DOC_DT and summary.dtype == SUMMARY_DT
        assert len(summary) >= len(docs)
        t = C.c_uint64()
        err = N.Error()
        if N.lib.am_pipe_submit(self._p, arena.ctypes.data, arena.nbytes, chunks.ctypes.data, len(chunks), docs.ctypes.data,
                                len(docs), summary.ctypes.data, out.ctypes.data, out.nbytes, patches.ctypes.data,
                                patches.nbytes, C.byref(t), C.byref(err)):
            N.raise_for(err)
        self._keep[t.value] = (arena, chunks, docs, summary, out, patches)
        return t.value

    def submit_packed(self, arena, chunk_len, spans, summary, out, patches):
        """Enqueues one batch with packed descriptors (am_pipe_submit_packed): `arena` holds the chunks
        back to back in chunk order, `chunk_len` (u32) their lengths, `spans` (SPAN_DT) one entry per
        document whose chunks (base first when has_base) follow those of the previous document."""
        assert chunk_len.dtype == np.uint32 and spans.dtype == SPAN_DT and summary.dtype == SUMMARY_DT
        assert len(summary) >= len(spans)
        t = C.c_uint64()
        err = N.Error()
        if N.lib.am_pipe_submit_packed(self._p, arena.ctypes.data, arena.nbytes, chunk_len.ctypes.data, len(chunk_len),
                                       spans.ctypes.data, len(spans), summary.ctypes.data, out.ctypes.data, out.nbytes,
                                       patches.ctypes.data, patches.nbytes, C.byref(t), C.byref(err)):
            N.raise_for(err)
        self._keep[t.value] = (arena, chunk_len, spans, summary, out, patches)
        return t.value

    def engines(self):
        """SDMA engine masks of the host-link copies: (H2D, copies home); 0 = the runtime's choice."""
        m = (C.c_uint32 * 2)()
        N.lib.am_pipe_engines(self._p, m)
        return int(m[0]), int(m[1])

    def drain(self, nbatches=0):
        """Waits for every submitted batch; returns [(output bytes, patch bytes)] of the batches
        finalized since the last drain (in submission order)."""
        cap = max(int(nbatches), len(self._keep), 1)
        tot = (C.c_uint64 * (2 * cap))()
        err = N.Error()
        if N.lib.am_pipe_drain(self._p, tot, cap, C.byref(err)):
            N.raise_for(err)
        self._keep.clear()
        return [(int(tot[2 * i]), int(tot[2 * i + 1])) for i in range(cap)]

    def times(self):
        """(ms of the compute chains, ms of the document kernels, batches) retired since the last call."""
        ms = (C.c_float * 2)()
        n = C.c_uint32()
        N.lib.am_pipe_times(self._p, ms, C.byref(n))
        return float(ms[0]), float(ms[1]), int(n.value)

    def run_resident(self, d_arena, arena_len, d_chunks, nchunks, d_docs, ndocs, any_diff, d_summary, d_out, out_cap,
                     d_patches, patch_cap, d_totals):
        """One batch whose inputs are resident in device memory (device pointers as ints: the arena
        with 64 readable bytes past arena_len); outputs compacted into device buffers. Async."""
        err = N.Error()
        if N.lib.am_pipe_run_resident(self._p, d_arena, arena_len, d_chunks, nchunks, d_docs, ndocs, int(bool(any_diff)),
                                      d_summary, d_out, out_cap, d_patches, patch_cap, d_totals, C.byref(err)):
            N.raise_for(err)

    def resident_sync(self):
        """Waits for the resident batches; (ms of their chains, ms of their document kernels), summed."""
        ms = (C.c_float * 2)()
        err = N.Error()
        if N.lib.am_pipe_resident_sync(self._p, ms, C.byref(err)):
            N.raise_for(err)
        return float(ms[0]), float(ms[1])
