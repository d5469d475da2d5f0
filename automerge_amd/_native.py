"""ctypes binding of libautomerge_amd.so (include/automerge_amd.h).

There is no CPU fallback: importing this module raises if the library is missing, and creating
an engine raises if no HIP device is visible.
"""
import ctypes as C
import os
import time

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("AM_LIB_PATH") or os.path.join(_HERE, "libautomerge_amd.so")

if not os.path.exists(LIB_PATH):
    raise ImportError(
        "automerge_amd: native library %s is missing; build it with "
        "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc, gfx950)" % LIB_PATH)

lib = C.CDLL(LIB_PATH)

u8p = C.POINTER(C.c_uint8)


class ChunkDesc(C.Structure):
    _fields_ = [("off", C.c_uint64), ("len", C.c_uint32), ("flags", C.c_uint32)]


class DocDesc(C.Structure):
    _fields_ = [("base_chunk", C.c_int64), ("chg_begin", C.c_uint32), ("chg_count", C.c_uint32),
                ("known_begin", C.c_uint32), ("known_count", C.c_uint32), ("flags", C.c_uint32),
                ("meta_chunk", C.c_uint32)]


class KnownHash(C.Structure):
    _fields_ = [("hash", C.c_uint8 * 32), ("index", C.c_int64)]


class DocResult(C.Structure):
    _fields_ = [("status", C.c_uint32), ("err_change", C.c_uint32), ("arg0", C.c_int64), ("arg1", C.c_int64),
                ("arg_actor_off", C.c_uint64), ("arg_actor_len", C.c_uint32), ("napplied", C.c_uint32),
                ("nqueued", C.c_uint32), ("nheads", C.c_uint32), ("nops", C.c_uint32), ("nchanges", C.c_uint32),
                ("max_op", C.c_int64), ("out_off", C.c_uint64), ("out_len", C.c_uint64), ("ws_off", C.c_uint64),
                ("ws_bytes", C.c_uint64)]


class DocSummary(C.Structure):
    _fields_ = [("status", C.c_uint32), ("nqueued", C.c_uint32), ("out_len", C.c_uint32), ("patch_len", C.c_uint32),
                ("out_off", C.c_uint64), ("patch_off", C.c_uint64)]


class CallInfo(C.Structure):
    _fields_ = [("max_op", C.c_int64), ("pending", C.c_uint32), ("nheads", C.c_uint32), ("heads", C.c_void_p)]

    def take(self):
        """(maxOp, heads hex list, pending); frees the heads."""
        raw = C.string_at(self.heads, 32 * self.nheads) if self.heads else b""
        if self.heads:
            lib.am_free(self.heads)
            self.heads = None
        return self.max_op, [raw[32 * i:32 * i + 32].hex() for i in range(len(raw) // 32)], self.pending


class PipeCaps(C.Structure):
    _fields_ = [("arena_bytes", C.c_uint64), ("chunks", C.c_uint32), ("docs", C.c_uint32), ("ws_bytes", C.c_uint64),
                ("out_bytes", C.c_uint64), ("patch_bytes", C.c_uint64), ("fast_lds", C.c_uint32), ("slots", C.c_uint32)]


class Span(C.Structure):
    _fields_ = [("off", C.c_uint64), ("len", C.c_uint64)]


class Error(C.Structure):
    _fields_ = [("code", C.c_uint32), ("is_type_error", C.c_int32), ("message", C.c_char * 8184)]


P = C.c_void_p
_sigs = {
    "am_version": (C.c_char_p, []),
    "am_engine_create": (P, [C.c_int, C.POINTER(Error)]),
    "am_engine_destroy": (None, [P]),
    "am_batch_create": (P, [P]),
    "am_batch_destroy": (None, [P]),
    "am_batch_stage": (C.c_int, [P, P, C.c_uint64, P, C.c_uint32, P, C.c_uint32, P, C.c_uint32, C.POINTER(Error)]),
    "am_batch_run": (C.c_int, [P]),
    "am_batch_sync": (C.c_int, [P, C.POINTER(Error)]),
    "am_batch_results": (C.c_int, [P, P]),
    "am_batch_chunk_results": (C.c_int, [P, P, P, P]),
    "am_batch_doc_output": (C.c_int, [P, C.c_uint32, P, C.c_uint64, C.POINTER(C.c_uint64)]),
    "am_document_changes": (C.c_int, [P, C.c_char_p, C.c_size_t, C.POINTER(u8p), C.POINTER(C.POINTER(C.c_uint64)),
                                      C.POINTER(u8p), C.POINTER(C.c_size_t), C.POINTER(Error)]),
    "am_document_changes_batch": (C.c_int, [P, C.POINTER(C.c_char_p), C.POINTER(C.c_size_t), C.c_size_t, P]),
    "am_doc_compute_hash_graph": (C.c_int, [P, C.POINTER(Error)]),
    "am_inflate_raw": (C.c_int, [P, C.POINTER(C.c_char_p), C.POINTER(C.c_size_t), C.c_size_t, C.POINTER(u8p),
                                 C.POINTER(C.c_size_t), P, C.POINTER(Error)]),
    "am_batch_inflate_info": (C.c_int, [P, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.POINTER(C.c_float)]),
    "am_batch_doc_save": (C.c_int, [P, C.c_uint32, C.POINTER(u8p), C.POINTER(C.c_size_t), C.POINTER(Error)]),
    "am_batch_doc_heads": (C.c_int, [P, C.c_uint32, P, C.c_uint32, C.POINTER(C.c_uint32)]),
    "am_batch_stage_times": (C.c_int, [P, C.POINTER(C.c_float)]),
    "am_batch_workspace_bytes": (C.c_uint64, [P]),
    "am_batch_workspace_plan": (C.c_uint64, [P]),
    "am_batch_kernel_info": (C.c_int, [P, P]),
    "am_batch_doc_plan": (C.c_int, [P, C.c_uint32, P]),
    "am_batch_fast_slices": (C.c_int, [P, P]),
    "am_batch_digest": (C.c_int, [P, C.c_uint64, C.POINTER(C.c_uint64)]),
    "am_batch_fast_flags": (C.c_int, [P, P]),
    "am_engine_stats": (C.c_int, [P, P]),
    "am_batch_ws_canary": (C.c_int64, [P, C.c_uint64]),
    "am_pipe_ws_canary": (C.c_int64, [P]),
    "am_batch_doc_layout": (C.c_int, [P, C.c_uint32, P, P, C.c_uint32]),
    "am_batch_doc_patch_raw": (C.c_int, [P, C.c_uint32, P]),
    "am_doc_init": (P, [P]),
    "am_doc_load": (P, [P, C.c_char_p, C.c_size_t, C.POINTER(Error)]),
    "am_doc_clone": (P, [P]),
    "am_doc_free": (None, [P]),
    "am_doc_apply_changes": (C.c_int, [P, C.POINTER(C.c_char_p), C.POINTER(C.c_size_t), C.c_size_t, C.POINTER(Error)]),
    "am_doc_apply_changes_patch": (C.c_int, [P, C.POINTER(C.c_char_p), C.POINTER(C.c_size_t), C.c_size_t, C.POINTER(u8p),
                                             C.POINTER(C.c_size_t), C.POINTER(Error)]),
    "am_doc_save": (C.c_int, [P, C.POINTER(u8p), C.POINTER(C.c_size_t), C.POINTER(Error)]),
    "am_doc_get_heads": (C.c_size_t, [P, P, C.c_size_t]),
    "am_doc_pending": (C.c_size_t, [P]),
    "am_doc_max_op": (C.c_int64, [P]),
    "am_doc_num_changes": (C.c_size_t, [P]),
    "am_doc_change": (C.c_int, [P, C.c_size_t, C.POINTER(u8p), C.POINTER(C.c_size_t), P]),
    "am_bloom_encoded_size": (C.c_uint64, [C.c_uint64]),
    "am_bloom_build": (C.c_int, [P, C.c_char_p, P, C.c_uint32, P, C.c_uint64, P, C.POINTER(Error)]),
    "am_bloom_probe": (C.c_int, [P, P, P, C.c_uint32, C.c_char_p, P, C.c_uint64, P, C.POINTER(Error)]),
    "am_sync_select": (C.c_int, [P, C.c_uint32, P, C.c_char_p, P, P, P, P, P, P, C.POINTER(Error)]),
    "am_doc_get_patch": (C.c_int, [P, C.POINTER(u8p), C.POINTER(C.c_size_t), C.POINTER(Error)]),
    "am_batch_doc_patch": (C.c_int, [P, C.c_uint32, P, C.c_uint64, C.POINTER(C.c_uint64)]),
    "am_doc_queued": (C.c_int, [P, C.c_size_t, C.POINTER(u8p), C.POINTER(C.c_size_t)]),
    "am_free": (None, [P]),
    "am_change_hashes": (C.c_int, [P, C.POINTER(C.c_char_p), C.POINTER(C.c_size_t), C.c_size_t, P, C.POINTER(Error)]),
    "am_stage_change": (C.c_int, [C.c_char_p, C.c_size_t, C.POINTER(u8p), C.POINTER(C.c_size_t), C.POINTER(Error)]),
    "am_stage_document": (C.c_int, [P, C.c_char_p, C.c_size_t, C.POINTER(u8p), C.POINTER(C.c_size_t),
                                    C.POINTER(C.c_int), C.POINTER(Error)]),
    "am_doc_get_changes": (C.c_int, [P, C.c_char_p, C.c_size_t, C.POINTER(C.POINTER(C.c_uint64)), C.POINTER(C.c_size_t),
                                     C.POINTER(Error)]),
    "am_doc_get_changes_added": (C.c_int, [P, P, C.POINTER(C.POINTER(C.c_uint64)), C.POINTER(C.c_size_t),
                                           C.POINTER(Error)]),
    "am_doc_change_index": (C.c_int64, [P, C.c_char_p]),
    "am_doc_get_missing_deps": (C.c_int, [P, C.c_char_p, C.c_size_t, C.POINTER(u8p), C.POINTER(C.c_size_t),
                                          C.POINTER(Error)]),
    "am_doc_clock": (C.c_int64, [P, C.c_char_p]),
    "am_doc_actor_hash": (C.c_int, [P, C.c_char_p, C.c_int64, P]),
    "am_doc_change_deps": (C.c_int, [P, C.c_size_t, C.POINTER(u8p), C.POINTER(C.c_size_t)]),
    "am_doc_engine": (P, [P]),
    "am_encode_change": (C.c_int, [C.c_char_p, C.c_size_t, C.POINTER(u8p), C.POINTER(C.c_size_t), P, C.POINTER(Error)]),
    "am_doc_apply_local_change": (C.c_int, [P, C.c_char_p, C.c_size_t, C.POINTER(u8p), C.POINTER(C.c_size_t),
                                            C.POINTER(u8p), C.POINTER(C.c_size_t), P, P, C.POINTER(C.c_int),
                                            C.POINTER(Error)]),
    "am_bloom_check": (C.c_int, [C.c_char_p, C.c_uint64, C.POINTER(Error)]),
    "am_sync_generate": (C.c_int, [C.c_size_t, P, P, P, P, P, P, P, P, P]),
    "am_sync_receive": (C.c_int, [P, C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t, C.POINTER(u8p),
                                  C.POINTER(C.c_size_t), C.POINTER(u8p), C.POINTER(C.c_size_t), C.POINTER(Error)]),
    "am_sync_receive_batch": (C.c_int, [C.c_size_t, P, P, P, P, P, P, P, P, P, P, P, P]),
    "am_sync_encode_message": (C.c_int, [C.c_char_p, C.c_size_t, C.POINTER(u8p), C.POINTER(C.c_size_t), C.POINTER(Error)]),
    "am_sync_decode_messages": (C.c_int, [C.c_size_t, P, P, C.POINTER(C.POINTER(Span)), P, P, P]),
    "am_sync_encode_state": (C.c_int, [C.c_char_p, C.c_size_t, C.POINTER(u8p), C.POINTER(C.c_size_t), C.POINTER(Error)]),
    "am_sync_decode_state": (C.c_int, [C.c_char_p, C.c_size_t, C.POINTER(u8p), C.POINTER(C.c_size_t), C.POINTER(Error)]),
    "am_doc_load_batch": (C.c_int, [P, C.c_size_t, P, P, P, P, P]),
    "am_stage_documents": (C.c_int, [P, C.c_size_t, P, P, P, P, P, P, P]),
    "am_doc_apply_changes_batch": (C.c_int, [C.c_size_t, P, P, P, P, P, P, P, P, P]),
    "am_doc_get_patch_batch": (C.c_int, [C.c_size_t, P, P, P, P, P, P]),
    "am_doc_save_batch": (C.c_int, [C.c_size_t, P, P, P, P, P]),
    "am_doc_compute_hash_graph_batch": (C.c_int, [C.c_size_t, P, P, P]),
    "am_doc_graph_ready": (C.c_int, [P]),
    "am_host_alloc": (P, [C.c_size_t]),
    "am_host_free": (None, [P]),
    "am_pipe_create": (P, [P, C.POINTER(PipeCaps), C.POINTER(Error)]),
    "am_pipe_destroy": (None, [P]),
    "am_pipe_submit": (C.c_int, [P, P, C.c_uint64, P, C.c_uint32, P, C.c_uint32, P, P, C.c_uint64, P, C.c_uint64,
                                 C.POINTER(C.c_uint64), C.POINTER(Error)]),
    "am_pipe_submit_packed": (C.c_int, [P, P, C.c_uint64, P, C.c_uint32, P, C.c_uint32, P, P, C.c_uint64, P,
                                        C.c_uint64, C.POINTER(C.c_uint64), C.POINTER(Error)]),
    "am_pipe_engines": (C.c_int, [P, C.POINTER(C.c_uint32)]),
    "am_pipe_drain": (C.c_int, [P, P, C.c_uint32, C.POINTER(Error)]),
    "am_pipe_times": (C.c_int, [P, C.POINTER(C.c_float), C.POINTER(C.c_uint32)]),
    "am_pipe_run_resident": (C.c_int, [P, P, C.c_uint64, P, C.c_uint32, P, C.c_uint32, C.c_int, P, P, C.c_uint64, P,
                                       C.c_uint64, P, C.POINTER(Error)]),
    "am_pipe_resident_sync": (C.c_int, [P, C.POINTER(C.c_float), C.POINTER(Error)]),
}
for _name, (_res, _args) in _sigs.items():
    _f = getattr(lib, _name)
    _f.restype = _res
    _f.argtypes = _args

EXPORTS = sorted(_sigs)

# status codes (include/automerge_amd.h)
CHG_DUP, CHG_QUEUED = -3, -2


class AutomergeError(Exception):
    """Error raised by the engine; `kind` is the reference's JS error class."""

    def __init__(self, message, code=0, kind="RangeError"):
        super().__init__(message)
        self.code = code
        self.kind = kind

    @property
    def unsupported(self):
        return self.code >= 100


def error_for(err):
    msg = err.message.decode("utf-8", "replace")
    return AutomergeError(msg, err.code, "TypeError" if err.is_type_error else "RangeError")


def raise_for(err):
    raise error_for(err)


def batch_errors(n, codes, msgs):
    """Per call of a batched per-handle call (include/automerge_amd.h): None, or its AutomergeError
    (bit 31 of the code: the reference throws a TypeError). Frees the messages."""
    out = [None] * n
    for i in range(n):
        if codes[i]:
            m = C.string_at(msgs[i]).decode("utf-8", "replace") if msgs[i] else ""
            c = int(codes[i])
            out[i] = AutomergeError(m, c & 0x7FFFFFFF, "TypeError" if c & 0x80000000 else "RangeError")
        if msgs[i]:
            lib.am_free(msgs[i])
    return out


_engines = {}


def engine(device=0):
    """Per-process engine for one HIP device (created on first use)."""
    if device not in _engines:
        err = Error()
        e = lib.am_engine_create(device, C.byref(err))
        if not e:
            raise_for(err)
        _engines[device] = e
    return _engines[device]


def engine_stats(device=0):
    """(documents of the per-handle calls, of them merged by k_doc_fast) since the last call."""
    out = (C.c_uint64 * 2)()
    lib.am_engine_stats(engine(device), out)
    return int(out[0]), int(out[1])


def buf_array(bufs):
    n = len(bufs)
    arr = (C.c_char_p * max(n, 1))(*[bytes(b) for b in bufs])
    lens = (C.c_size_t * max(n, 1))(*[len(b) for b in bufs])
    return arr, lens, n


def take(ptr, n):
    """bytes of a malloc'd engine result, then am_free."""
    b = C.string_at(ptr, n) if n else b""
    lib.am_free(ptr)
    return b


def stage_change(data):
    """Host DEFLATE stage for one change (inflates chunk type 2)."""
    if len(data) <= 8 or data[8] != 2:
        return bytes(data)
    out, n, err = u8p(), C.c_size_t(), Error()
    if lib.am_stage_change(bytes(data), len(data), C.byref(out), C.byref(n), C.byref(err)):
        raise_for(err)
    b = C.string_at(out, n.value)
    lib.am_free(out)
    return b


def stage_document(data, device=0):
    """Host DEFLATE stage for a document: returns (bytes, checksum_already_verified)."""
    out, n, v, err = u8p(), C.c_size_t(), C.c_int(), Error()
    if lib.am_stage_document(engine(device), bytes(data), len(data), C.byref(out), C.byref(n), C.byref(v),
                             C.byref(err)):
        raise_for(err)
    b = C.string_at(out, n.value)
    lib.am_free(out)
    return b, bool(v.value)


def stage_documents(datas, device=0):
    """stage_document over many documents in one call (am_stage_documents: one GPU checksum batch,
    one GPU inflate batch): a list of (bytes, checksum_already_verified); raises the first error."""
    datas = [bytes(d) for d in datas]
    n = len(datas)
    if n == 0:
        return []
    bufs = (C.c_char_p * n)(*datas)
    lens = (C.c_size_t * n)(*[len(d) for d in datas])
    outs = (u8p * n)()
    olens = (C.c_size_t * n)()
    ver = (C.c_uint8 * n)()
    codes = (C.c_uint32 * n)()
    msgs = (C.c_void_p * n)()
    lib.am_stage_documents(engine(device), n, bufs, lens, outs, olens, ver, codes, msgs)
    errs = batch_errors(n, codes, msgs)
    res = []
    for i in range(n):
        if outs[i]:
            res.append((C.string_at(outs[i], olens[i]), bool(ver[i])))
            lib.am_free(outs[i])
        else:
            res.append(None)
    for e in errs:
        if e is not None:
            raise e
    return res


def inflate_raw(buffers, device=0):
    """pako.inflateRaw over many buffers on the GPU (am_inflate_raw): a list of bytes, or None for a
    buffer that is not a valid raw DEFLATE stream."""
    n = len(buffers)
    if not n:
        return []
    arr = (C.c_char_p * n)(*[bytes(b) for b in buffers])
    lens = (C.c_size_t * n)(*[len(b) for b in buffers])
    outs = (u8p * n)()
    olens = (C.c_size_t * n)()
    ok = (C.c_uint8 * n)()
    err = Error()
    if lib.am_inflate_raw(engine(device), arr, lens, n, outs, olens, ok, C.byref(err)):
        raise_for(err)
    res = []
    for i in range(n):
        res.append(C.string_at(outs[i], olens[i]) if ok[i] else None)
        lib.am_free(outs[i])
    return res


class History(C.Structure):
    """am_history (include/automerge_amd.h): one document's reconstructed changes or its error."""
    _fields_ = [("changes", u8p), ("offs", C.POINTER(C.c_uint64)), ("hashes32", u8p), ("nchanges", C.c_size_t),
                ("err", Error)]


def document_changes_batch(docs, device=0, stats=None):
    """decodeChanges([doc]) re-encoded (computeHashGraph, new.js:1879-1904) for many saved documents
    in one GPU batch (k_history): per document [(change bytes, hash hex)], or the AutomergeError it
    raises."""
    n = len(docs)
    if n == 0:
        return []
    arr = (C.c_char_p * n)(*[bytes(d) for d in docs])
    lens = (C.c_size_t * n)(*[len(d) for d in docs])
    hs = (History * n)()
    eng = engine(device)
    t0 = time.perf_counter()
    lib.am_document_changes_batch(eng, arr, lens, n, hs)
    if stats is not None:
        stats["c_seconds"] = time.perf_counter() - t0
    res = []
    for h in hs:
        if h.err.code:
            res.append(error_for(h.err))
            continue
        nc = h.nchanges
        offs = h.offs[:nc + 1]  # one copy of each buffer, then slices
        buf = C.string_at(h.changes, offs[-1]) if nc and offs[-1] else b""
        hx = C.string_at(h.hashes32, 32 * nc).hex() if nc else ""
        res.append([(buf[offs[i]:offs[i + 1]], hx[64 * i:64 * i + 64]) for i in range(nc)])
        for p in (h.changes, h.offs, h.hashes32):
            lib.am_free(p)
    return res


def document_changes(doc, device=0):
    """decodeChanges([doc]) re-encoded (computeHashGraph, new.js:1879-1904): [(change bytes, hash hex)]
    of a saved document in its change order (am_document_changes_batch with one document)."""
    r = document_changes_batch([doc], device)[0]
    if isinstance(r, Exception):
        raise r
    return r
