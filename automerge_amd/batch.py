"""Batched load + applyChanges over many documents per launch (am_batch_* in
include/automerge_amd.h). Each document is (optional base document bytes, list of change
buffers): Backend.load(base) followed by Backend.applyChanges(state, changes)."""
import ctypes as C

import numpy as np

from . import _native as N

CHUNK_DT = np.dtype([("off", "<u8"), ("len", "<u4"), ("flags", "<u4")])
DOC_DT = np.dtype([("base_chunk", "<i8"), ("chg_begin", "<u4"), ("chg_count", "<u4"), ("known_begin", "<u4"),
                   ("known_count", "<u4"), ("flags", "<u4"), ("meta_chunk", "<u4")])
RESULT_DT = np.dtype([("status", "<u4"), ("err_change", "<u4"), ("arg0", "<i8"), ("arg1", "<i8"),
                      ("arg_actor_off", "<u8"), ("arg_actor_len", "<u4"), ("napplied", "<u4"), ("nqueued", "<u4"),
                      ("nheads", "<u4"), ("nops", "<u4"), ("nchanges", "<u4"), ("max_op", "<i8"),
                      ("out_off", "<u8"), ("out_len", "<u8"), ("ws_off", "<u8"), ("ws_bytes", "<u8")])
assert CHUNK_DT.itemsize == C.sizeof(N.ChunkDesc)
assert DOC_DT.itemsize == C.sizeof(N.DocDesc)
assert RESULT_DT.itemsize == C.sizeof(N.DocResult)


WANT_PATCH = 2  # AM_DOC_WANT_PATCH: also write the getPatch() log of the merged document
WANT_DIFF = 4   # AM_DOC_WANT_DIFF: also write the patch applyChanges returns


def pack(docs, device=0, flags=0):
    """docs: iterable of (base_bytes | None, [change bytes]) -> (arena, chunks, docdescs).
    Compressed inputs go in as they are: the batch stage inflates compressed change chunks (type 2)
    and the DEFLATEd columns of base documents on the GPU (am_inflate.hip, am_capi.hip inflate_stage).
    flags: WANT_PATCH or WANT_DIFF for every document."""
    parts, chunks, descs = [], [], []
    off = 0
    for base, changes in docs:
        d = np.zeros((), DOC_DT)
        d["base_chunk"] = -1
        changes = [bytes(c) for c in changes]
        if base:
            base = bytes(base)
            d["base_chunk"] = len(chunks)
            chunks.append((off, len(base), 0))
            parts.append(base)
            off += len(base)
        d["chg_begin"] = len(chunks)
        d["chg_count"] = len(changes)
        d["flags"] = (0 if base else 1) | flags  # fresh documents have the full hash graph
        for c in changes:
            chunks.append((off, len(c), 0))
            parts.append(c)
            off += len(c)
        descs.append(d)
    arena = np.frombuffer(b"".join(parts), dtype=np.uint8) if parts else np.zeros(1, np.uint8)
    return arena, np.array(chunks, dtype=CHUNK_DT), np.array(descs, dtype=DOC_DT)


class Batch:
    def __init__(self, device=0, engine=None):
        """engine: an am_engine of one's own (N.lib.am_engine_create) -- its own HIP stream, so two
        batches on two engines overlap one's stage with the other's kernels; default the process's."""
        self._eng = engine if engine is not None else N.engine(device)
        self._b = N.lib.am_batch_create(self._eng)
        self.ndocs = 0
        self.nchunks = 0

    def __del__(self):
        if getattr(self, "_b", None):
            N.lib.am_batch_destroy(self._b)
            self._b = None

    def stage(self, arena, chunks, docs, known=None):
        arena = np.ascontiguousarray(arena, dtype=np.uint8)
        chunks = np.ascontiguousarray(chunks, dtype=CHUNK_DT)
        docs = np.ascontiguousarray(docs, dtype=DOC_DT)
        nk = 0 if known is None else len(known)
        err = N.Error()
        rc = N.lib.am_batch_stage(self._b, arena.ctypes.data, arena.nbytes, chunks.ctypes.data, len(chunks),
                                  docs.ctypes.data, len(docs), None if known is None else known.ctypes.data, nk,
                                  C.byref(err))
        if rc:
            N.raise_for(err)
        self.ndocs = len(docs)
        self.nchunks = len(chunks)
        self._keep = (arena, chunks, docs, known)

    def stage_docs(self, docs, flags=0):
        self.stage(*pack(docs, flags=flags))

    def run(self):
        if N.lib.am_batch_run(self._b):
            raise N.AutomergeError("automerge_amd: kernel launch failed")

    def sync(self):
        err = N.Error()
        if N.lib.am_batch_sync(self._b, C.byref(err)):
            N.raise_for(err)

    def results(self):
        out = np.zeros(self.ndocs, RESULT_DT)
        if self.ndocs and N.lib.am_batch_results(self._b, out.ctypes.data):
            raise N.AutomergeError("automerge_amd: result copy failed")
        return out

    def chunk_results(self):
        hashes = np.zeros((self.nchunks, 32), np.uint8)
        state = np.zeros(self.nchunks, np.int32)
        status = np.zeros(self.nchunks, np.uint32)
        if self.nchunks and N.lib.am_batch_chunk_results(self._b, hashes.ctypes.data, state.ctypes.data,
                                                         status.ctypes.data):
            raise N.AutomergeError("automerge_amd: result copy failed")
        return hashes, state, status

    def doc_output(self, i, res=None):
        n = C.c_uint64()
        cap = int(res["out_len"]) if res is not None else 1 << 24
        buf = (C.c_uint8 * max(cap, 1))()
        rc = N.lib.am_batch_doc_output(self._b, i, buf, cap, C.byref(n))
        if rc:
            raise N.AutomergeError("automerge_amd: output copy failed (%d)" % rc)
        return bytes(buf)[:n.value]

    def doc_save(self, i):
        """Backend.save() bytes of document i: the merged chunk with its columns of >= 256 bytes
        DEFLATEd (am_batch_doc_save)."""
        out = N.u8p()
        n = C.c_size_t()
        err = N.Error()
        if N.lib.am_batch_doc_save(self._b, i, C.byref(out), C.byref(n), C.byref(err)):
            N.raise_for(err)
        data = C.string_at(out, n.value)
        N.lib.am_free(out)
        return data

    def doc_heads(self, i, nheads):
        buf = (C.c_uint8 * (32 * max(nheads, 1)))()
        n = C.c_uint32()
        if N.lib.am_batch_doc_heads(self._b, i, buf, nheads, C.byref(n)):
            raise N.AutomergeError("automerge_amd: heads copy failed")
        raw = bytes(buf)
        return [raw[32 * k:32 * k + 32].hex() for k in range(min(n.value, nheads))]

    def doc_patch(self, i):
        """Patch log of document i (staged with WANT_PATCH or WANT_DIFF); automerge_amd.patch
        materializes it."""
        n = C.c_uint64()
        rc = N.lib.am_batch_doc_patch(self._b, i, None, 0, C.byref(n))
        if rc:
            raise N.AutomergeError("automerge_amd: no patch log for document %d (%d)" % (i, rc))
        buf = (C.c_uint8 * max(n.value, 1))()
        if N.lib.am_batch_doc_patch(self._b, i, buf, n.value, C.byref(n)):
            raise N.AutomergeError("automerge_amd: patch copy failed")
        return bytes(buf)[:n.value]

    def stage_times(self):
        ms = (C.c_float * 4)()
        if N.lib.am_batch_stage_times(self._b, ms):
            return None
        return list(ms)

    def digest(self, first_doc=0):
        """Device-side output digest (am_batch_digest; host restatement: shard.doc_digest)."""
        out = C.c_uint64()
        if N.lib.am_batch_digest(self._b, first_doc, C.byref(out)):
            raise N.AutomergeError("automerge_amd: digest failed")
        return int(out.value)

    def fast_flags(self):
        """Per document of the last run: True when k_doc_fast merged it."""
        out = np.zeros(self.ndocs, np.uint8)
        if self.ndocs and N.lib.am_batch_fast_flags(self._b, out.ctypes.data):
            raise N.AutomergeError("automerge_amd: flag copy failed")
        return out.astype(bool)

    def inflate_info(self):
        """(DEFLATE streams inflated on the GPU -- compressed change chunks and DEFLATEd document
        columns --, bytes of the rebuilt arena, ms of the two inflate passes) of the last stage."""
        n = C.c_uint64()
        nb = C.c_uint64()
        ms = C.c_float()
        N.lib.am_batch_inflate_info(self._b, C.byref(n), C.byref(nb), C.byref(ms))
        return int(n.value), int(nb.value), float(ms.value)

    def workspace_bytes(self):
        return N.lib.am_batch_workspace_bytes(self._b)

    def workspace_plan(self):
        """The scanned per-document plans (compact ones for k_doc_fast's documents), without the
        overflow reserve workspace_bytes() includes."""
        return N.lib.am_batch_workspace_plan(self._b)

    def kernel_info(self):
        """{k_doc LDS bytes, k_doc_fast LDS bytes per document, largest k_doc hot set} of the staged batch."""
        out = np.zeros(3, np.uint64)
        N.lib.am_batch_kernel_info(self._b, out.ctypes.data)
        return {"k_doc_lds": int(out[0]), "k_doc_fast_lds_per_doc": int(out[1]), "k_doc_max_hot": int(out[2])}
