"""ctypes binding of the CPU oracle (oracle/liboracle.so). Test infrastructure only."""
import ctypes as C
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_LIB_PATH = os.path.join(ROOT, "oracle", "liboracle.so")
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
        L = C.CDLL(_LIB_PATH)
        P, S, I64 = C.c_void_p, C.c_size_t, C.c_int64
        L.oc_leb_encode.argtypes = [C.c_int, I64, I64, I64, C.c_char_p]
        L.oc_leb_decode.argtypes = [C.c_int, C.c_char_p, S, C.POINTER(I64), C.POINTER(I64), C.POINTER(I64),
                                    C.POINTER(S), C.c_char_p, S]
        L.oc_col_encode.argtypes = [C.c_int, S, P, P, P, P, C.c_char_p, S, C.POINTER(S)]
        L.oc_col_decode.argtypes = [C.c_int, C.c_char_p, S, S, C.POINTER(S), P, P, P, S, P, C.c_char_p, S]
        L.oc_sha256.argtypes = [C.c_char_p, S, C.c_char_p]
        L.oc_change_meta.argtypes = [C.c_char_p, S, C.c_char_p, C.POINTER(I64), C.POINTER(I64), C.POINTER(I64),
                                     C.POINTER(I64), C.c_char_p, S]
        L.oc_doc_init.restype = P
        L.oc_doc_load.restype = P
        L.oc_doc_load.argtypes = [C.c_char_p, S, C.c_char_p, S]
        L.oc_doc_clone.restype = P
        L.oc_doc_clone.argtypes = [P]
        L.oc_doc_free.argtypes = [P]
        L.oc_doc_apply.argtypes = [P, C.POINTER(C.c_char_p), C.POINTER(S), S, C.c_char_p, S]
        L.oc_doc_save.restype = C.POINTER(C.c_uint8)
        L.oc_doc_save.argtypes = [P, C.POINTER(S)]
        L.oc_doc_heads.restype = S
        L.oc_doc_heads.argtypes = [P, C.c_char_p, S]
        L.oc_doc_pending.restype = S
        L.oc_doc_pending.argtypes = [P]
        L.oc_doc_num_ops.restype = S
        L.oc_doc_num_ops.argtypes = [P]
        L.oc_doc_max_op.restype = I64
        L.oc_doc_max_op.argtypes = [P]
        L.oc_free.argtypes = [P]
        L.oc_doc_patch.restype = C.c_void_p
        L.oc_doc_patch.argtypes = [P, C.c_char_p, S]
        L.oc_doc_apply_patch.restype = C.c_void_p
        L.oc_doc_apply_patch.argtypes = [P, C.POINTER(C.c_char_p), C.POINTER(S), S, C.c_char_p, S]
        L.oc_bloom_build.restype = S
        L.oc_bloom_build.argtypes = [C.c_char_p, S, C.c_char_p, S]
        L.oc_bloom_contains.restype = C.c_int
        L.oc_bloom_contains.argtypes = [C.c_char_p, S, C.c_char_p]
        L.oc_sync_select.argtypes = [S, C.c_char_p, P, P, S, C.POINTER(C.c_char_p), C.POINTER(S), C.c_char_p]
        _lib = L
    return _lib


class OracleError(Exception):
    def __init__(self, message, code=1):
        super().__init__(message)
        self.code = code


def leb_encode(fn, value=0, hi=0, lo=0):
    buf = C.create_string_buffer(16)
    n = lib().oc_leb_encode(fn, value, hi, lo, buf)
    return buf.raw[:n]


def leb_decode(fn, data):
    v, hi, lo, off = C.c_int64(), C.c_int64(), C.c_int64(), C.c_size_t()
    err = C.create_string_buffer(256)
    rc = lib().oc_leb_decode(fn, data, len(data), C.byref(v), C.byref(hi), C.byref(lo), C.byref(off), err, 256)
    if rc:
        return None, err.value.decode(), off.value
    if fn >= 4:
        return (hi.value, lo.value), None, off.value
    return v.value, None, off.value


COL_TYPES = {"uint": 0, "int": 1, "utf8": 2, "delta": 3, "bool": 4}


def col_encode(type_, values):
    t = COL_TYPES[type_]
    n = len(values)
    ints = (C.c_int64 * max(n, 1))()
    nulls = (C.c_uint8 * max(n, 1))()
    lens = (C.c_uint32 * max(n, 1))()
    strbuf = b""
    for i, v in enumerate(values):
        if v is None:
            nulls[i] = 1
        elif t == 2:
            b = v.encode("utf-8", "surrogatepass")
            lens[i] = len(b)
            strbuf += b
        else:
            ints[i] = int(v)
    sb = C.create_string_buffer(strbuf, max(len(strbuf), 1))
    cap = 64 + 32 * n + 2 * len(strbuf)
    out = C.create_string_buffer(cap)
    outlen = C.c_size_t()
    rc = lib().oc_col_encode(t, n, ints, nulls, sb, lens, out, cap, C.byref(outlen))
    assert rc == 0
    return out.raw[:outlen.value]


def col_decode(type_, data, maxn=4096):
    t = COL_TYPES[type_]
    ints = (C.c_int64 * maxn)()
    nulls = (C.c_uint8 * maxn)()
    lens = (C.c_uint32 * maxn)()
    strcap = 16 * len(data) + 64
    sb = C.create_string_buffer(strcap)
    n = C.c_size_t()
    err = C.create_string_buffer(256)
    rc = lib().oc_col_decode(t, data, len(data), maxn, C.byref(n), ints, nulls, sb, strcap, lens, err, 256)
    out, off = [], 0
    for i in range(n.value):
        if t == 2:
            if nulls[i]:
                out.append(None)
            else:
                out.append(sb.raw[off:off + lens[i]].decode("utf-8"))
                off += lens[i]
        elif t == 4:
            out.append(bool(ints[i]))
        else:
            out.append(None if nulls[i] else ints[i])
    return out, (err.value.decode() if rc else None)


def sha256(data):
    out = C.create_string_buffer(32)
    lib().oc_sha256(data, len(data), out)
    return out.raw


def change_meta(data):
    h = C.create_string_buffer(32)
    seq, start, nops, ndeps = C.c_int64(), C.c_int64(), C.c_int64(), C.c_int64()
    err = C.create_string_buffer(512)
    rc = lib().oc_change_meta(data, len(data), h, C.byref(seq), C.byref(start), C.byref(nops), C.byref(ndeps), err, 512)
    if rc:
        raise OracleError(err.value.decode())
    return {"hash": h.raw.hex(), "seq": seq.value, "startOp": start.value, "numOps": nops.value, "numDeps": ndeps.value}


class Doc:
    """Backend-state handle of the oracle (init/load/applyChanges/save/getHeads)."""

    def __init__(self, ptr):
        self._p = ptr

    @classmethod
    def init(cls):
        return cls(lib().oc_doc_init())

    @classmethod
    def load(cls, data):
        err = C.create_string_buffer(512)
        p = lib().oc_doc_load(data, len(data), err, 512)
        if not p:
            raise OracleError(err.value.decode())
        return cls(p)

    def clone(self):
        return Doc(lib().oc_doc_clone(self._p))

    def __del__(self):
        if getattr(self, "_p", None) and _lib is not None:
            _lib.oc_doc_free(self._p)
            self._p = None

    def apply(self, changes):
        n = len(changes)
        arr = (C.c_char_p * max(n, 1))(*changes)
        lens = (C.c_size_t * max(n, 1))(*[len(c) for c in changes])
        err = C.create_string_buffer(512)
        rc = lib().oc_doc_apply(self._p, arr, lens, n, err, 512)
        if rc:
            raise OracleError(err.value.decode(), rc)

    def apply_patch(self, changes):
        """Backend.applyChanges(doc, changes): applies and returns the patch as a dict."""
        import json
        n = len(changes)
        arr = (C.c_char_p * max(n, 1))(*changes)
        lens = (C.c_size_t * max(n, 1))(*[len(c) for c in changes])
        err = C.create_string_buffer(512)
        p = lib().oc_doc_apply_patch(self._p, arr, lens, n, err, 512)
        if not p:
            raise OracleError(err.value.decode())
        txt = C.string_at(p).decode("utf-8")
        lib().oc_free(p)
        return json.loads(txt)

    def patch(self):
        """Backend.getPatch(doc) as a dict (JSON from the C restatement)."""
        import json
        err = C.create_string_buffer(512)
        p = lib().oc_doc_patch(self._p, err, 512)
        if not p:
            raise OracleError(err.value.decode())
        txt = C.string_at(p).decode("utf-8")
        lib().oc_free(p)
        return json.loads(txt)

    def save(self):
        n = C.c_size_t()
        p = lib().oc_doc_save(self._p, C.byref(n))
        data = C.string_at(p, n.value)
        lib().oc_free(p)
        return data

    def heads(self):
        buf = C.create_string_buffer(32 * 256)
        n = lib().oc_doc_heads(self._p, buf, 256)
        return [buf.raw[32 * i:32 * i + 32].hex() for i in range(min(n, 256))]

    def pending(self):
        return lib().oc_doc_pending(self._p)

    def num_ops(self):
        return lib().oc_doc_num_ops(self._p)

    def max_op(self):
        return lib().oc_doc_max_op(self._p)


# ---- sync.js Bloom filter / change selection ----
def bloom_build(hashes):
    """new BloomFilter(hashes).bytes for a list of 32-byte hashes."""
    L = lib()
    flat = b"".join(hashes)
    n = L.oc_bloom_build(flat, len(hashes), None, 0)
    buf = C.create_string_buffer(max(n, 1))
    L.oc_bloom_build(flat, len(hashes), buf, n)
    return buf.raw[:n]


def bloom_contains(filt, h):
    return lib().oc_bloom_contains(bytes(filt), len(filt), bytes(h))


def sync_select(hashes, deps, filters):
    """Send mask of getChangesToSend: hashes (32 B each), deps[i] = indexes of change i's deps in
    the list (-1 = outside), filters = encoded Bloom filters."""
    import numpy as np
    n = len(hashes)
    off = np.zeros(n + 1, dtype=np.uint32)
    for i, d in enumerate(deps):
        off[i + 1] = off[i] + len(d)
    idx = np.array([x for d in deps for x in d] or [0], dtype=np.int32)
    fl = (C.c_char_p * max(len(filters), 1))(*[bytes(f) for f in filters])
    fn = (C.c_size_t * max(len(filters), 1))(*[len(f) for f in filters])
    out = C.create_string_buffer(max(n, 1))
    lib().oc_sync_select(n, b"".join(hashes), off.ctypes.data, idx.ctypes.data, len(filters), fl, fn, out)
    return list(out.raw[:n])


# ---- flat export of a saved document (oc_doc_export) ----
class _OcOp(C.Structure):
    _fields_ = [("obj_ctr", C.c_int64), ("key_ctr", C.c_int64), ("id_ctr", C.c_int64), ("action", C.c_int64),
                ("val_len", C.c_int64), ("obj_actor", C.c_int32), ("key_actor", C.c_int32), ("id_actor", C.c_int32),
                ("insert", C.c_int32), ("key_len", C.c_int32), ("val_n", C.c_uint32), ("nsucc", C.c_uint32),
                ("succ_off", C.c_uint32), ("key", C.c_void_p), ("val", C.c_void_p)]


class _OcExport(C.Structure):
    _fields_ = [("nops", C.c_size_t), ("ops", C.POINTER(_OcOp)), ("succ_ctr", C.c_void_p), ("succ_actor", C.c_void_p),
                ("nactors", C.c_size_t), ("actors", C.c_void_p), ("actor_lens", C.c_void_p), ("nchg", C.c_size_t),
                ("chg_actor", C.c_void_p), ("chg_seq", C.c_void_p), ("priv", C.c_void_p)]


def export(data):
    """Counts of a saved document's ops: {nops, nsucc, val_bytes, nchg} (oc_doc_export)."""
    L = lib()
    L.oc_doc_export.restype = C.POINTER(_OcExport)
    L.oc_doc_export.argtypes = [C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t]
    L.oc_export_free.argtypes = [C.POINTER(_OcExport)]
    err = C.create_string_buffer(256)
    e = L.oc_doc_export(bytes(data), len(data), err, 256)
    if not e:
        raise OracleError(err.value.decode(errors="replace"))
    x = e.contents
    out = {"nops": int(x.nops), "nchg": int(x.nchg),
           "nsucc": sum(int(x.ops[i].nsucc) for i in range(x.nops)),
           "val_bytes": sum(int(x.ops[i].val_n) for i in range(x.nops))}
    L.oc_export_free(e)
    return out
