"""Drop-in mirror of the reference Backend module (backend/backend.js, backend/index.js).

Same function names, argument meaning and error behaviour as the reference; every call runs the
MI355X pipeline of libautomerge_amd.so (there is no CPU path). A backend state is the reference's
`{state, heads, frozen}` wrapper: after applyChanges / loadChanges the old handle is frozen and
further use raises the reference's error (backend/util.js:1-10).
"""
import ctypes as C
import json
import re

from . import _native as N

_FROZEN_MSG = ("Attempting to use an outdated Automerge document that has already been updated. "
               "Please use the latest document state, or call Automerge.clone() if you really "
               "need to use this old document state.")


class BackendState:
    __slots__ = ("state", "heads", "frozen")

    def __init__(self, state, heads):
        self.state = state
        self.heads = heads
        self.frozen = False


class _Doc:
    """Owns an am_doc handle."""

    def __init__(self, ptr):
        self.ptr = ptr

    def __del__(self):
        if self.ptr:
            N.lib.am_doc_free(self.ptr)
            self.ptr = None

    def heads(self):
        n = N.lib.am_doc_get_heads(self.ptr, None, 0)
        buf = (C.c_uint8 * (32 * max(n, 1)))()
        N.lib.am_doc_get_heads(self.ptr, buf, n)
        raw = bytes(buf)
        return [raw[32 * i:32 * i + 32].hex() for i in range(n)]


def _backend_state(backend):
    # backendState() (backend/util.js:1-10)
    if backend.frozen:
        raise RuntimeError(_FROZEN_MSG)
    return backend.state


def init(device=0):
    """Backend.init() (backend/backend.js:8-10)."""
    d = _Doc(N.lib.am_doc_init(N.engine(device)))
    return BackendState(d, [])


def clone(backend):
    """Backend.clone() (backend/backend.js:12-14)."""
    s = _backend_state(backend)
    return BackendState(_Doc(N.lib.am_doc_clone(s.ptr)), backend.heads)


def free(backend):
    """Backend.free() (backend/backend.js:16-19)."""
    backend.state = None
    backend.frozen = True


def _apply(backend, changes, want_patch=False):
    s = _backend_state(backend)
    arr, lens, n = N.buf_array(changes)
    err = N.Error()
    blob = None
    if want_patch:
        out, nb = N.u8p(), C.c_size_t()
        if N.lib.am_doc_apply_changes_patch(s.ptr, arr, lens, n, C.byref(out), C.byref(nb), C.byref(err)):
            N.raise_for(err)
        blob = C.string_at(out, nb.value)
        N.lib.am_free(out)
    elif N.lib.am_doc_apply_changes(s.ptr, arr, lens, n, C.byref(err)):
        N.raise_for(err)
    backend.frozen = True
    return BackendState(s, s.heads()), blob


def applyChanges(backend, changes):
    """Backend.applyChanges() (backend/backend.js:27-32, new.js:1796-1871). Returns (state, patch):
    the patch's diffs are replayed on the GPU (k_doc phase P8, am_diff.h) and materialized by
    automerge_amd/patch.py into {maxOp, clock, deps, pendingChanges, diffs}."""
    from . import patch as P
    new, blob = _apply(backend, changes, want_patch=True)
    return new, P.materialize(blob, new.heads, pendingChanges(new), maxOp(new))


def loadChanges(backend, changes):
    """Backend.loadChanges() (backend/backend.js:115-120)."""
    return _apply(backend, changes)[0]


def load(data, device=0):
    """Backend.load() (backend/backend.js:104-107)."""
    err = N.Error()
    p = N.lib.am_doc_load(N.engine(device), bytes(data), len(data), C.byref(err))
    if not p:
        N.raise_for(err)
    d = _Doc(p)
    return BackendState(d, d.heads())


def save(backend):
    """Backend.save() (backend/backend.js:96-98)."""
    s = _backend_state(backend)
    out = N.u8p()
    n = C.c_size_t()
    err = N.Error()
    if N.lib.am_doc_save(s.ptr, C.byref(out), C.byref(n), C.byref(err)):
        N.raise_for(err)
    data = C.string_at(out, n.value)
    N.lib.am_free(out)
    return data


def getPatch(backend):
    """Backend.getPatch() (backend/backend.js:125-127, new.js:2052-2060): documentPatch runs on the
    GPU (k_doc phase P7); automerge_amd/patch.py turns its log into the reference patch object."""
    from . import patch as P
    s = _backend_state(backend)
    out, n, err = N.u8p(), C.c_size_t(), N.Error()
    if N.lib.am_doc_get_patch(s.ptr, C.byref(out), C.byref(n), C.byref(err)):
        N.raise_for(err)
    blob = C.string_at(out, n.value)
    N.lib.am_free(out)
    return P.materialize(blob, s.heads(), N.lib.am_doc_pending(s.ptr), N.lib.am_doc_max_op(s.ptr))


def getHeads(backend):
    """Backend.getHeads() (backend/backend.js:134-136)."""
    return backend.heads


def pendingChanges(backend):
    return N.lib.am_doc_pending(_backend_state(backend).ptr)


def maxOp(backend):
    return N.lib.am_doc_max_op(_backend_state(backend).ptr)


# ---- the same calls over many documents in one GPU batch (am_doc_*_batch, include/automerge_amd.h):
# per document the result the single call gives, or its error in its place ----
def _prepare(n, fn):
    """fn(i) for every item; an item whose fn raises (an outdated handle, a bad argument) gets that
    exception as its result. Returns (indexes that go to the engine, their values, results)."""
    idx, vals, out = [], [], [None] * n
    for i in range(n):
        try:
            v = fn(i)
        except (RuntimeError, TypeError, ValueError, N.AutomergeError) as e:
            out[i] = e
            continue
        idx.append(i)
        vals.append(v)
    return idx, vals, out


def _codes(n):
    return (C.c_uint32 * max(n, 1))(), (C.c_void_p * max(n, 1))()


def _take_all(bufs, lens, n):
    out = []
    for i in range(n):
        out.append(C.string_at(bufs[i], lens[i]) if bufs[i] else None)
        if bufs[i]:
            N.lib.am_free(bufs[i])
    return out


def loadBatch(datas, device=0):
    """Backend.load() of many documents in one GPU batch: [BackendState or AutomergeError]."""
    n = len(datas)
    bufs = [bytes(d) for d in datas]
    arr = (C.c_char_p * max(n, 1))(*bufs)
    lens = (C.c_size_t * max(n, 1))(*[len(b) for b in bufs])
    docs = (C.c_void_p * max(n, 1))()
    codes, msgs = _codes(n)
    N.lib.am_doc_load_batch(N.engine(device), n, arr, lens, docs, codes, msgs)
    errs = N.batch_errors(n, codes, msgs)
    out = []
    for i in range(n):
        if errs[i]:
            out.append(errs[i])
        else:
            d = _Doc(docs[i])
            out.append(BackendState(d, d.heads()))
    return out


def _rounds(backends, run):
    """Sequential semantics for a backend named more than once: `run(items)` takes the first
    occurrence of each backend; a later occurrence runs in a following round, where a handle its
    earlier call froze raises the outdated-document error (util.js:1-10) in its own slot, as the
    second of two sequential calls would, and a handle whose earlier call failed (unchanged, not
    frozen) is applied then. Returns the results in item order."""
    out = [None] * len(backends)
    pending = list(range(len(backends)))
    while pending:
        seen, now, later = set(), [], []
        for i in pending:
            (later if id(backends[i]) in seen else now).append(i)
            seen.add(id(backends[i]))
        for i, r in zip(now, run(now)):
            out[i] = r
        pending = later
    return out


def _apply_batch(backends, changes_lists, want_patch):
    return _rounds(backends, lambda items: _apply_once([backends[i] for i in items], [changes_lists[i] for i in items],
                                                       want_patch))


def _apply_once(backends, changes_lists, want_patch):
    from . import patch as P
    idx, states, out = _prepare(len(backends), lambda i: _backend_state(backends[i]))
    n = len(idx)
    ptrs = (C.c_void_p * max(n, 1))(*[s.ptr for s in states])
    lists = [[bytes(c) for c in changes_lists[i]] for i in idx]
    flat = [c for cl in lists for c in cl]
    off = [0]
    for cl in lists:
        off.append(off[-1] + len(cl))
    arr = (C.c_char_p * max(len(flat), 1))(*flat)
    lens = (C.c_size_t * max(len(flat), 1))(*[len(b) for b in flat])
    offs = (C.c_size_t * (n + 1))(*off)
    pats, plens = ((N.u8p * max(n, 1))(), (C.c_size_t * max(n, 1))()) if want_patch else (None, None)
    info = (N.CallInfo * max(n, 1))()
    codes, msgs = _codes(n)
    N.lib.am_doc_apply_changes_batch(n, ptrs, offs, arr, lens, pats, plens, info, codes, msgs)
    errs = N.batch_errors(n, codes, msgs)
    blobs = _take_all(pats, plens, n) if want_patch else [None] * n
    for k, i in enumerate(idx):
        if errs[k]:
            out[i] = errs[k]
            continue
        max_op, heads, pending = info[k].take()  # as of this call (a handle may appear again later)
        backends[i].frozen = True
        new = BackendState(states[k], heads)
        out[i] = (new, P.materialize(blobs[k], heads, pending, max_op)) if want_patch else new
    return out


def applyChangesBatch(backends, changes_lists):
    """Backend.applyChanges() of many documents in one GPU batch: [(state, patch) or error]."""
    return _apply_batch(backends, changes_lists, True)


def loadChangesBatch(backends, changes_lists):
    """Backend.loadChanges() of many documents in one GPU batch: [state or error]."""
    return _apply_batch(backends, changes_lists, False)


def saveBatch(backends):
    """Backend.save() of many documents (one GPU SHA-256 launch for their checksums)."""
    idx, states, out = _prepare(len(backends), lambda i: _backend_state(backends[i]))
    n = len(idx)
    ptrs = (C.c_void_p * max(n, 1))(*[s.ptr for s in states])
    bufs, lens = (N.u8p * max(n, 1))(), (C.c_size_t * max(n, 1))()
    codes, msgs = _codes(n)
    N.lib.am_doc_save_batch(n, ptrs, bufs, lens, codes, msgs)
    errs = N.batch_errors(n, codes, msgs)
    data = _take_all(bufs, lens, n)
    for k, i in enumerate(idx):
        out[i] = errs[k] or data[k]
    return out


def getPatchBatch(backends):
    """Backend.getPatch() of many documents in one GPU batch."""
    from . import patch as P
    idx, states, out = _prepare(len(backends), lambda i: _backend_state(backends[i]))
    n = len(idx)
    ptrs = (C.c_void_p * max(n, 1))(*[s.ptr for s in states])
    bufs, lens = (N.u8p * max(n, 1))(), (C.c_size_t * max(n, 1))()
    info = (N.CallInfo * max(n, 1))()
    codes, msgs = _codes(n)
    N.lib.am_doc_get_patch_batch(n, ptrs, bufs, lens, info, codes, msgs)
    errs = N.batch_errors(n, codes, msgs)
    data = _take_all(bufs, lens, n)
    for k, i in enumerate(idx):
        if errs[k]:
            out[i] = errs[k]
            continue
        max_op, heads, pending = info[k].take()
        out[i] = P.materialize(data[k], heads, pending, max_op)
    return out


def _hash_graph(s):
    # computeHashGraph (new.js:1879-1904) for a loaded document, once
    err = N.Error()
    if N.lib.am_doc_compute_hash_graph(s.ptr, C.byref(err)):
        N.raise_for(err)


def changeHashes(changes, device=0):
    """decodeChangeMeta(change, true).hash for each change (columnar.js:783), on the GPU."""
    arr, lens, n = N.buf_array(changes)
    out = (C.c_uint8 * (32 * max(n, 1)))()
    err = N.Error()
    if N.lib.am_change_hashes(N.engine(device), arr, lens, n, out, C.byref(err)):
        N.raise_for(err)
    raw = bytes(out)
    return [raw[32 * i:32 * i + 32].hex() for i in range(n)]


# ---- hash-graph queries (new.js:1913-2020): the traversals run in the engine (am_graph.cpp) ----
_HEX64 = re.compile(r"^[0-9a-f]{64}$")


def _flat_hashes(hashes):
    """One flat bytes of 32-byte hashes; a string that is not a hash travels as a sentinel the
    engine cannot know (0xff x 28 + its index), mapped back where a result or error names it."""
    out, odd = [], {}
    for i, h in enumerate(hashes):
        if isinstance(h, str) and _HEX64.match(h):
            out.append(bytes.fromhex(h))
        else:
            b = b"\xff" * 28 + i.to_bytes(4, "big")
            odd[b.hex()] = h
            out.append(b)
    return b"".join(out), odd


def _changes_at(s, idx, n):
    res = []
    for k in range(n):
        p, ln = N.u8p(), C.c_size_t()
        if N.lib.am_doc_change(s.ptr, idx[k], C.byref(p), C.byref(ln), None):
            raise N.AutomergeError("automerge_amd: change index out of range")
        res.append(C.string_at(p, ln.value))
    return res


def getChanges(backend, haveDeps):
    """Backend.getChanges() (backend/backend.js:150-156 -> BackendDoc.getChanges, new.js:1913-1966)."""
    if not isinstance(haveDeps, list):
        raise TypeError("Pass an array of hashes to Backend.getChanges()")
    s = _backend_state(backend)
    flat, odd = _flat_hashes(haveDeps)
    idx, n, err = C.POINTER(C.c_uint64)(), C.c_size_t(), N.Error()
    if N.lib.am_doc_get_changes(s.ptr, flat or None, len(haveDeps), C.byref(idx), C.byref(n), C.byref(err)):
        msg = err.message.decode("utf-8", "replace")
        for k, v in odd.items():
            msg = msg.replace(k, str(v))
        raise N.AutomergeError(msg, err.code, "TypeError" if err.is_type_error else "RangeError")
    try:
        return _changes_at(s, idx, n.value)
    finally:
        N.lib.am_free(idx)


def getAllChanges(backend):
    """Backend.getAllChanges() (backend/backend.js:142-144 -> getChanges(backend, []))."""
    return getChanges(backend, [])


def getChangesAdded(backend1, backend2):
    """Backend.getChangesAdded() (new.js:1971-1988): changes in backend2 that backend1 lacks."""
    s1, s2 = _backend_state(backend1), _backend_state(backend2)
    idx, n, err = C.POINTER(C.c_uint64)(), C.c_size_t(), N.Error()
    if N.lib.am_doc_get_changes_added(s1.ptr, s2.ptr, C.byref(idx), C.byref(n), C.byref(err)):
        N.raise_for(err)
    try:
        return _changes_at(s2, idx, n.value)
    finally:
        N.lib.am_free(idx)


def getChangeByHash(backend, hash_hex):
    """Backend.getChangeByHash() (backend/backend.js:166-168, new.js:1990-1993); None when unknown."""
    s = _backend_state(backend)
    if not (isinstance(hash_hex, str) and _HEX64.match(hash_hex)):
        return None
    i = N.lib.am_doc_change_index(s.ptr, bytes.fromhex(hash_hex))
    if i == -2:
        raise N.AutomergeError("automerge_amd: the document history could not be reconstructed")
    return None if i < 0 else _changes_at(s, [i], 1)[0]


def getMissingDeps(backend, heads=None):
    """Backend.getMissingDeps() (new.js:2005-2020)."""
    s = _backend_state(backend)
    heads = list(heads or [])
    flat, odd = _flat_hashes(heads)
    out, n, err = N.u8p(), C.c_size_t(), N.Error()
    if N.lib.am_doc_get_missing_deps(s.ptr, flat or None, len(heads), C.byref(out), C.byref(n), C.byref(err)):
        N.raise_for(err)
    raw = N.take(out, 32 * n.value)
    res = [odd.get(raw[i:i + 32].hex(), raw[i:i + 32].hex()) for i in range(0, len(raw), 32)]
    return sorted(res) if odd else res


# ---- applyLocalChange (backend.js:54-91): encodeChange + applyChanges(isLocal) in the engine ----
def _json_default(o):
    if isinstance(o, (bytes, bytearray, memoryview)):
        return {"__bytes": bytes(o).hex()}
    raise TypeError("not JSON serializable: %r" % (o,))


def _nonfinite(x):
    if isinstance(x, float) and (x != x or x in (float("inf"), float("-inf"))):
        return {"__f64": "NaN" if x != x else ("Infinity" if x > 0 else "-Infinity")}
    if isinstance(x, dict):
        return {k: _nonfinite(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [_nonfinite(v) for v in x]
    return x


def request_json(obj):
    """A change request / sync message as the JSON text the C ABI reads (include/automerge_amd.h)."""
    return json.dumps(_nonfinite(obj), default=_json_default, allow_nan=False).encode()


def encodeChange(change):
    """encodeChange (columnar.js:710-739) in the engine library (am_encode_change, host code)."""
    js = request_json(change)
    out, n, err = N.u8p(), C.c_size_t(), N.Error()
    if N.lib.am_encode_change(js, len(js), C.byref(out), C.byref(n), None, C.byref(err)):
        N.raise_for(err)
    return N.take(out, n.value)


def applyLocalChange(backend, change):
    """Backend.applyLocalChange() (backend/backend.js:54-91). Returns (state, patch, binaryChange);
    like the reference, the request's deps gain the local actor's previous change."""
    from . import patch as P
    s = _backend_state(backend)
    js = request_json(change)
    ch, cl, pa, pl = N.u8p(), C.c_size_t(), N.u8p(), C.c_size_t()
    nh, lh, has_last, err = (C.c_uint8 * 32)(), (C.c_uint8 * 32)(), C.c_int(), N.Error()
    rc = N.lib.am_doc_apply_local_change(s.ptr, js, len(js), C.byref(ch), C.byref(cl), C.byref(pa), C.byref(pl), nh,
                                         lh, C.byref(has_last), C.byref(err))
    if rc:
        if rc == 2:
            backend.frozen = True
        N.raise_for(err)
    if has_last.value:
        deps = {bytes(lh).hex(): True}
        for h in change["deps"]:
            deps[h] = True
        change["deps"] = sorted(deps)
    binary, log = N.take(ch, cl.value), N.take(pa, pl.value)
    backend.frozen = True
    new = BackendState(s, s.heads())
    patch = P.materialize(log, [h for h in new.heads if h != bytes(nh).hex()], N.lib.am_doc_pending(s.ptr),
                          N.lib.am_doc_max_op(s.ptr))
    patch["actor"] = change["actor"]
    patch["seq"] = change["seq"]
    return new, patch, binary


# ---- sync protocol (backend/sync.js) in the engine (am_sync_proto.cpp); SyncState dicts cross as
# the flat state blob of include/automerge_amd.h ----
def _checked_hash(h):
    if not isinstance(h, str):
        raise N.AutomergeError("value is not a string", kind="TypeError")
    if not re.match(r"^([0-9a-f][0-9a-f])*$", h):
        raise N.AutomergeError("value is not hexadecimal")
    if len(h) != 64:
        raise N.AutomergeError("heads hashes must be 256 bits", kind="TypeError")
    return bytes.fromhex(h)


def _uleb(v):
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        out.append(b | (0x80 if v else 0))
        if not v:
            return bytes(out)


def _pack_state(st):
    def hashes(lst):
        if not isinstance(lst, list):
            raise N.AutomergeError("hashes must be an array", kind="TypeError")
        return _uleb(len(lst)) + b"".join(_checked_hash(h) for h in lst)
    sent = st.get("sentHashes")
    keys = [k for k in sent if _HEX64.match(k)] if isinstance(sent, dict) else []
    flags = ((1 if st.get("theirHeads") is not None else 0) | (2 if st.get("theirNeed") is not None else 0) |
             (4 if st.get("theirHave") is not None else 0) | (8 if isinstance(sent, list) else 0))
    out = bytes([0x53, flags]) + hashes(st["sharedHeads"]) + hashes(st["lastSentHeads"])
    if flags & 1:
        out += hashes(st["theirHeads"])
    if flags & 2:
        out += hashes(st["theirNeed"])
    if flags & 4:
        out += _uleb(len(st["theirHave"]))
        for h in st["theirHave"]:
            b = bytes(h["bloom"])
            out += hashes(h["lastSync"]) + _uleb(len(b)) + b
    return out + _uleb(len(keys)) + b"".join(bytes.fromhex(k) for k in keys)


def _unpack_state(b):
    o = [2]

    def u():
        v = sh = 0
        while True:
            x = b[o[0]]
            o[0] += 1
            v |= (x & 0x7F) << sh
            sh += 7
            if not x & 0x80:
                return v

    def hashes():
        n = u()
        r = [b[o[0] + 32 * i:o[0] + 32 * i + 32].hex() for i in range(n)]
        o[0] += 32 * n
        return r
    flags = b[1]
    st = {"sharedHeads": hashes(), "lastSentHeads": hashes(), "theirHeads": None, "theirNeed": None, "theirHave": None}
    if flags & 1:
        st["theirHeads"] = hashes()
    if flags & 2:
        st["theirNeed"] = hashes()
    if flags & 4:
        st["theirHave"] = []
        for _ in range(u()):
            ls = hashes()
            ln = u()
            st["theirHave"].append({"lastSync": ls, "bloom": bytes(b[o[0]:o[0] + ln])})
            o[0] += ln
    sent = hashes()
    st["sentHashes"] = [] if flags & 8 else {h: True for h in sent}
    return st


def initSyncState():
    """initSyncState() (sync.js:308-317)."""
    return {"sharedHeads": [], "lastSentHeads": [], "theirHeads": None, "theirNeed": None, "theirHave": None,
            "sentHashes": {}}


def encodeSyncMessage(message):
    """encodeSyncMessage (sync.js:157-171)."""
    js = request_json(message)
    out, n, err = N.u8p(), C.c_size_t(), N.Error()
    if N.lib.am_sync_encode_message(js, len(js), C.byref(out), C.byref(n), C.byref(err)):
        N.raise_for(err)
    return N.take(out, n.value)


def decodeSyncMessages(messages):
    """decodeSyncMessage (sync.js:177-199) over many messages in one call (am_sync_decode_messages):
    a list of message dicts, or the AutomergeError of a malformed one in its place."""
    n = len(messages)
    bufs = [bytes(m) for m in messages]
    arr = (C.c_char_p * max(n, 1))(*bufs)
    lens = (C.c_size_t * max(n, 1))(*[len(b) for b in bufs])
    spans = C.POINTER(N.Span)()
    soff = (C.c_uint64 * (n + 1))()
    counts = (C.c_uint32 * (4 * max(n, 1)))()
    errs = (N.Error * max(n, 1))()
    N.lib.am_sync_decode_messages(n, arr, lens, C.byref(spans), soff, counts, errs)
    out = []
    for i, m in enumerate(bufs):
        if errs[i].code:
            e = errs[i]
            out.append(N.AutomergeError(e.message.decode("utf-8", "replace"), e.code,
                                        "TypeError" if e.is_type_error else "RangeError"))
            continue
        k = int(soff[i])

        def hl(sp):
            return [m[sp.off + 32 * j:sp.off + 32 * j + 32].hex() for j in range(sp.len)]
        msg = {"heads": hl(spans[k]), "need": hl(spans[k + 1]), "have": [], "changes": []}
        k += 2
        for _ in range(counts[4 * i + 2]):
            msg["have"].append({"lastSync": hl(spans[k]), "bloom": m[spans[k + 1].off:spans[k + 1].off + spans[k + 1].len]})
            k += 2
        for _ in range(counts[4 * i + 3]):
            msg["changes"].append(m[spans[k].off:spans[k].off + spans[k].len])
            k += 1
        out.append(msg)
    N.lib.am_free(spans)
    return out


def decodeSyncMessage(data):
    """decodeSyncMessage (sync.js:177-199)."""
    r = decodeSyncMessages([data])[0]
    if isinstance(r, Exception):
        raise r
    return r


def encodeSyncState(sync_state):
    """encodeSyncState (sync.js:206-211)."""
    blob = _pack_state({"sharedHeads": sync_state["sharedHeads"], "lastSentHeads": []})
    out, n, err = N.u8p(), C.c_size_t(), N.Error()
    if N.lib.am_sync_encode_state(blob, len(blob), C.byref(out), C.byref(n), C.byref(err)):
        N.raise_for(err)
    return N.take(out, n.value)


def decodeSyncState(data):
    """decodeSyncState (sync.js:217-225)."""
    out, n, err = N.u8p(), C.c_size_t(), N.Error()
    if N.lib.am_sync_decode_state(bytes(data), len(data), C.byref(out), C.byref(n), C.byref(err)):
        N.raise_for(err)
    return _unpack_state(N.take(out, n.value))


def generateSyncMessages(backends, sync_states):
    """generateSyncMessage for many documents in one call (am_sync_generate): their Bloom filters
    are built in one k_bloom_build launch and their change selections run in one k_sync_select
    launch. Returns [(state, message or None) or AutomergeError]."""
    def prep(i):
        if not backends[i]:
            raise N.AutomergeError("generateSyncMessage called with no Automerge document", kind="Error")
        if not sync_states[i]:
            raise N.AutomergeError("generateSyncMessage requires a syncState, which can be created with "
                                   "initSyncState()", kind="Error")
        return _backend_state(backends[i]), _pack_state(sync_states[i])
    idx, vals, res = _prepare(len(backends), prep)
    n = len(idx)
    ptrs = (C.c_void_p * max(n, 1))(*[v[0].ptr for v in vals])
    packed = [v[1] for v in vals]
    st = (C.c_char_p * max(n, 1))(*packed)
    sl = (C.c_size_t * max(n, 1))(*[len(p) for p in packed])
    ost, osl = (N.u8p * max(n, 1))(), (C.c_size_t * max(n, 1))()
    msg, ml = (N.u8p * max(n, 1))(), (C.c_size_t * max(n, 1))()
    codes, msgs = _codes(n)
    N.lib.am_sync_generate(n, ptrs, st, sl, ost, osl, msg, ml, codes, msgs)
    errs = N.batch_errors(n, codes, msgs)
    for k, i in enumerate(idx):
        if errs[k]:
            res[i] = errs[k]
            continue
        blob = N.take(ost[k], osl[k])
        m = N.take(msg[k], ml[k]) if msg[k] else None
        if m is None or blob == packed[k]:
            res[i] = (sync_states[i], m)
        else:
            nxt = _unpack_state(blob)
            res[i] = (dict(sync_states[i], lastSentHeads=nxt["lastSentHeads"], sentHashes=nxt["sentHashes"]), m)
    return res


def generateSyncMessage(backend, sync_state):
    """generateSyncMessage (sync.js:327-400): (syncState, message or None)."""
    if not backend:
        raise N.AutomergeError("generateSyncMessage called with no Automerge document", kind="Error")
    if not sync_state:
        raise N.AutomergeError("generateSyncMessage requires a syncState, which can be created with initSyncState()",
                               kind="Error")
    r = generateSyncMessages([backend], [sync_state])[0]
    if isinstance(r, Exception):
        raise r
    return r


def receiveSyncMessage(backend, old_sync_state, message):
    """receiveSyncMessage (sync.js:420-474): (backend, syncState, patch or None)."""
    from . import patch as P
    if not backend:
        raise N.AutomergeError("generateSyncMessage called with no Automerge document", kind="Error")
    if not old_sync_state:
        raise N.AutomergeError("generateSyncMessage requires a syncState, which can be created with initSyncState()",
                               kind="Error")
    msg = decodeSyncMessage(message)
    s = _backend_state(backend) if (msg["changes"] or msg["heads"]) else backend.state
    blob = _pack_state(old_sync_state)
    ost, osl, pa, pl, err = N.u8p(), C.c_size_t(), N.u8p(), C.c_size_t(), N.Error()
    rc = N.lib.am_sync_receive(s.ptr, blob, len(blob), bytes(message), len(message), C.byref(ost), C.byref(osl),
                               C.byref(pa), C.byref(pl), C.byref(err))
    if rc:
        if rc == 2:
            backend.frozen = True
        N.raise_for(err)
    st = _unpack_state(N.take(ost, osl.value))
    patch = None
    log = N.take(pa, pl.value) if pa else None
    if msg["changes"]:
        backend.frozen = True
        backend = BackendState(s, s.heads())
        patch = P.materialize(log, backend.heads, N.lib.am_doc_pending(s.ptr), N.lib.am_doc_max_op(s.ptr))
    sent = st["sentHashes"] if isinstance(st["sentHashes"], list) else old_sync_state.get("sentHashes")
    return backend, {"sharedHeads": st["sharedHeads"], "lastSentHeads": st["lastSentHeads"], "theirHave": msg["have"],
                     "theirHeads": msg["heads"], "theirNeed": msg["need"], "sentHashes": sent}, patch


def receiveSyncMessages(backends, old_sync_states, messages):
    """receiveSyncMessage for many documents in one call (am_sync_receive_batch): every message's
    changes go through ONE batched applyChanges. Returns [(backend, syncState, patch or None) or
    AutomergeError], each as receiveSyncMessage returns it (a backend named twice: as two
    sequential calls, _rounds)."""
    return _rounds(backends, lambda items: _receive_once([backends[i] for i in items], [old_sync_states[i] for i in items],
                                                         [messages[i] for i in items]))


def _receive_once(backends, old_sync_states, messages):
    from . import patch as P
    n = len(backends)
    decoded = [None] * n

    def prep(i):
        if not backends[i]:
            raise N.AutomergeError("generateSyncMessage called with no Automerge document", kind="Error")
        if not old_sync_states[i]:
            raise N.AutomergeError("generateSyncMessage requires a syncState, which can be created with "
                                   "initSyncState()", kind="Error")
        msg = decoded[i] = decodeSyncMessage(messages[i])
        s = _backend_state(backends[i]) if (msg["changes"] or msg["heads"]) else backends[i].state
        return s, _pack_state(old_sync_states[i]), bytes(messages[i])
    idx, vals, out = _prepare(n, prep)
    ptrs = [v[0] for v in vals]
    blobs = [v[1] for v in vals]
    mbufs = [v[2] for v in vals]
    m = len(idx)
    hp = (C.c_void_p * max(m, 1))(*[s.ptr for s in ptrs])
    sb = (C.c_char_p * max(m, 1))(*blobs)
    sl = (C.c_size_t * max(m, 1))(*[len(b) for b in blobs])
    mb = (C.c_char_p * max(m, 1))(*mbufs)
    mlen = (C.c_size_t * max(m, 1))(*[len(b) for b in mbufs])
    ost, osl = (N.u8p * max(m, 1))(), (C.c_size_t * max(m, 1))()
    pa, pl = (N.u8p * max(m, 1))(), (C.c_size_t * max(m, 1))()
    info = (N.CallInfo * max(m, 1))()
    codes, msgs = _codes(m)
    N.lib.am_sync_receive_batch(m, hp, sb, sl, mb, mlen, ost, osl, pa, pl, info, codes, msgs)
    errs = N.batch_errors(m, codes, msgs)
    states = _take_all(ost, osl, m)
    logs = _take_all(pa, pl, m)
    for k, i in enumerate(idx):
        msg, backend, s = decoded[i], backends[i], ptrs[k]
        if errs[k]:
            if errs[k].code & 0x40000000:  # the changes were applied before the error
                backend.frozen = True
            errs[k].code &= 0x3FFFFFFF
            out[i] = errs[k]
            continue
        st = _unpack_state(states[k])
        patch = None
        if msg["changes"]:
            max_op, heads, pending = info[k].take()
            backend.frozen = True
            backend = BackendState(s, heads)
            patch = P.materialize(logs[k], heads, pending, max_op)
        sent = st["sentHashes"] if isinstance(st["sentHashes"], list) else old_sync_states[i].get("sentHashes")
        out[i] = (backend, {"sharedHeads": st["sharedHeads"], "lastSentHeads": st["lastSentHeads"],
                            "theirHave": msg["have"], "theirHeads": msg["heads"], "theirNeed": msg["need"],
                            "sentHashes": sent}, patch)
    return out
