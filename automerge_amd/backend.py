"""Drop-in mirror of the reference Backend module (backend/backend.js, backend/index.js).

Same function names, argument meaning and error behaviour as the reference; every call runs the
MI355X pipeline of libautomerge_amd.so (there is no CPU path). A backend state is the reference's
`{state, heads, frozen}` wrapper: after applyChanges / loadChanges the old handle is frozen and
further use raises the reference's error (backend/util.js:1-10).
"""
import ctypes as C

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


def _hash_graph(s):
    # computeHashGraph (new.js:1879-1904) for a loaded document, once
    err = N.Error()
    if N.lib.am_doc_compute_hash_graph(s.ptr, C.byref(err)):
        N.raise_for(err)


def getAllChanges(backend):
    """Backend.getAllChanges() (backend/backend.js:142-144 -> getChanges(backend, [])): the whole
    history; a loaded document first reconstructs it from save() (computeHashGraph)."""
    s = _backend_state(backend)
    _hash_graph(s)
    out = []
    i = 0
    while True:
        p = N.u8p()
        n = C.c_size_t()
        if N.lib.am_doc_change(s.ptr, i, C.byref(p), C.byref(n), None):
            break
        out.append(C.string_at(p, n.value))
        i += 1
    return out


def getChangeByHash(backend, hash_hex):
    """Backend.getChangeByHash() (backend/backend.js:166-168)."""
    s = _backend_state(backend)
    _hash_graph(s)
    i = 0
    h = (C.c_uint8 * 32)()
    while True:
        p = N.u8p()
        n = C.c_size_t()
        if N.lib.am_doc_change(s.ptr, i, C.byref(p), C.byref(n), h):
            return None
        if bytes(h).hex() == hash_hex:
            return C.string_at(p, n.value)
        i += 1


def changeHashes(changes, device=0):
    """decodeChangeMeta(change, true).hash for each change (columnar.js:783), on the GPU."""
    arr, lens, n = N.buf_array(changes)
    out = (C.c_uint8 * (32 * max(n, 1)))()
    err = N.Error()
    if N.lib.am_change_hashes(N.engine(device), arr, lens, n, out, C.byref(err)):
        N.raise_for(err)
    raw = bytes(out)
    return [raw[32 * i:32 * i + 32].hex() for i in range(n)]


# ---- hash-graph queries (new.js:1913-2020), host traversals over the change history ----
def _uleb(b, o):
    v = sh = 0
    while True:
        c = b[o]
        o += 1
        v |= (c & 0x7F) << sh
        sh += 7
        if not c & 0x80:
            return v, o


def _change_deps(data):
    """deps (hex) of a binary change (decodeChangeMeta, columnar.js:783-793)."""
    b = N.stage_change(data)
    _, o = _uleb(b, 9)
    n, o = _uleb(b, o)
    return [b[o + 32 * i:o + 32 * i + 32].hex() for i in range(n)]


def _graph(s):
    _hash_graph(s)
    changes = []
    i = 0
    h = (C.c_uint8 * 32)()
    while True:
        p = N.u8p()
        n = C.c_size_t()
        if N.lib.am_doc_change(s.ptr, i, C.byref(p), C.byref(n), h):
            break
        changes.append((bytes(h).hex(), C.string_at(p, n.value)))
        i += 1
    index = {hh: k for k, (hh, _) in enumerate(changes)}
    deps_of = {hh: _change_deps(b) for hh, b in changes}
    dependents = {hh: [] for hh, _ in changes}
    for hh, _ in changes:
        for d in deps_of[hh]:
            dependents.setdefault(d, []).append(hh)
    return changes, index, deps_of, dependents


def getChanges(backend, haveDeps):
    """Backend.getChanges() (backend/backend.js:150-156 -> BackendDoc.getChanges, new.js:1913-1966)."""
    if not isinstance(haveDeps, list):
        raise TypeError("Pass an array of hashes to Backend.getChanges()")
    s = _backend_state(backend)
    changes, index, deps_of, dependents = _graph(s)
    if not haveDeps:
        return [b for _, b in changes]
    stack, seen, to_return = [], set(), []
    for h in haveDeps:
        seen.add(h)
        if h not in dependents:
            raise N.AutomergeError("hash not found: %s" % h, 0, "RangeError")
        stack += dependents[h]
    while stack:
        h = stack.pop()
        seen.add(h)
        to_return.append(h)
        if not all(d in seen for d in deps_of[h]):
            break
        stack += dependents[h]
    if not stack and all(h in seen for h in backend.heads):
        return [changes[index[h]][1] for h in to_return]
    stack, seen = list(haveDeps), set()
    while stack:
        h = stack.pop()
        if h not in seen:
            if h not in deps_of:
                raise N.AutomergeError("hash not found: %s" % h, 0, "RangeError")
            stack += deps_of[h]
            seen.add(h)
    return [b for h, b in changes if h not in seen]


def getChangesAdded(backend1, backend2):
    """Backend.getChangesAdded() (new.js:1971-1988): changes in backend2 that backend1 lacks."""
    _, other, _, _ = _graph(_backend_state(backend1))
    changes, index, deps_of, _ = _graph(_backend_state(backend2))
    stack, seen, to_return = list(backend2.heads), set(), []
    while stack:
        h = stack.pop()
        if h not in seen and h not in other:
            seen.add(h)
            to_return.append(h)
            stack += deps_of[h]
    return [changes[index[h]][1] for h in reversed(to_return)]


def getMissingDeps(backend, heads=None):
    """Backend.getMissingDeps() (new.js:2005-2020)."""
    s = _backend_state(backend)
    _, index, _, _ = _graph(s)
    all_deps, in_queue = set(heads or []), set()
    queued = []
    i = 0
    while True:
        p = N.u8p()
        n = C.c_size_t()
        if N.lib.am_doc_queued(s.ptr, i, C.byref(p), C.byref(n)):
            break
        queued.append(C.string_at(p, n.value))
        i += 1
    for b, h in zip(queued, changeHashes(queued) if queued else []):
        in_queue.add(h)
        all_deps.update(_change_deps(b))
    return sorted(h for h in all_deps if h not in index and h not in in_queue)
