"""Host stage of getPatch / applyChanges: turns the patch log written by the engine (wire form of
am_patch.h: PatchHdr2 + record stream; k_doc phases P7 / P8, k_doc_fast) into the reference's patch
object (new.js:2052-2060, 1862-1865; shapes in @types/automerge/index.d.ts:242-323). No merge logic
lives here: every decision (visible values, conflicts, counters, list indexes, multi-insert
coalescing, update pops) was made on the GPU; this is deserialization plus linking child object
patches by objectId.
"""
import struct

import numpy as np

HDR_DT = np.dtype([("magic", "<u4"), ("status", "<u4"), ("arg0", "<i8"), ("arg1", "<i8"), ("max_op", "<i8"),
                   ("nbytes", "<u8"), ("meta_bytes", "<u8")])
assert HDR_DT.itemsize == 48
MAGIC = 0x32504D41

PR_ACTOR, PR_CLOCK, PR_OBJ, PR_KEY, PR_PROP, PR_INSERT, PR_MULTI, PR_UPDATE, PR_REMOVE = range(1, 10)
(PV_NULL, PV_FALSE, PV_TRUE, PV_STR, PV_UINT, PV_INT, PV_F64, PV_COUNTER, PV_TIMESTAMP, PV_BYTES,
 PV_CHILD) = range(1, 12)
NAMED_DT = {PV_UINT: "uint", PV_INT: "int", PV_F64: "float64", PV_COUNTER: "counter", PV_TIMESTAMP: "timestamp"}
OBJ_TYPES = ("map", "list", "text", "table", None, None)  # 4: undefined (null action), 5: null (unknown even action)

# errors getPatch throws (am_patch.h PATCH_*)
PATCH_E_FLOAT_LEN, PATCH_E_UNKNOWN_COUNTER = 31, 32


def _f64(raw):
    return struct.unpack("<d", raw)[0]


class _Rd:
    __slots__ = ("b", "o")

    def __init__(self, b, o):
        self.b, self.o = b, o

    def u(self):
        v = sh = 0
        b = self.b
        while True:
            x = b[self.o]
            self.o += 1
            v |= (x & 0x7F) << sh
            sh += 7
            if x < 0x80:
                return v

    def s(self):
        v = sh = 0
        b = self.b
        while True:
            x = b[self.o]
            self.o += 1
            v |= (x & 0x7F) << sh
            sh += 7
            if x < 0x80:
                return v - (1 << sh) if x & 0x40 else v

    def raw(self, n):
        r = self.b[self.o:self.o + n]
        self.o += n
        return r

    def byte(self):
        x = self.b[self.o]
        self.o += 1
        return x


def header(blob):
    hdr = np.frombuffer(blob, dtype=HDR_DT, count=1)[0]
    if int(hdr["magic"]) != MAGIC:
        raise ValueError("not a patch log")
    return hdr


def actors_of(blob):
    """Actor ids (hex) of a log: its leading ACTOR records."""
    b = bytes(blob)
    r = _Rd(b, HDR_DT.itemsize)
    out = []
    while r.o < len(b) and b[r.o] == PR_ACTOR:
        r.o += 1
        out.append(r.raw(r.u()).hex())
    return out


def error_message(hdr, actors=None):
    st = int(hdr["status"])
    if st == PATCH_E_FLOAT_LEN:
        return "Invalid length for floating point number: %d" % int(hdr["arg0"])
    if st == PATCH_E_UNKNOWN_COUNTER:
        a = actors[int(hdr["arg1"])] if actors and 0 <= int(hdr["arg1"]) < len(actors) else "?"
        return "increment operation %d@%s for unknown counter" % (int(hdr["arg0"]), a)
    return "automerge_amd: getPatch not supported for this document (code %d)" % st


def materialize(blob, deps, pending_changes, max_op=None, js_bytes=bytes):
    """The getPatch() / applyChanges() result for a patch log. `deps` = heads (hex),
    `pending_changes` = queue length; max_op defaults to documentPatch's maxOp from the log.
    Raises AutomergeError with the reference's message when the log carries an error."""
    b = bytes(blob)
    hdr = header(b)
    if int(hdr["status"]):
        from ._native import AutomergeError
        raise AutomergeError(error_message(hdr, actors_of(b)), int(hdr["status"]), "RangeError")
    end = HDR_DT.itemsize + int(hdr["nbytes"])
    r = _Rd(b, HDR_DT.itemsize)
    actors, clock, nodes = [], {}, {}

    def opid(c, a):
        return "%d@%s" % (c, actors[a])

    def node(c, a, typ):
        k = (c, a)
        n = nodes.get(k)
        if n is None:
            t = OBJ_TYPES[typ]
            n = {"objectId": opid(c, a), "type": t}
            if t in ("list", "text"):
                n["edits"] = []
            else:
                n["props"] = {}
            nodes[k] = n
        return n

    def prim():
        """(vtag, datatype code, primitive value) of the VALUE at the cursor"""
        vt = r.byte()
        if vt == PV_NULL:
            return vt, 0, None
        if vt == PV_FALSE:
            return vt, 0, False
        if vt == PV_TRUE:
            return vt, 0, True
        if vt == PV_STR:
            return vt, 0, r.raw(r.u()).decode("utf-8", "replace")
        if vt == PV_UINT:
            return vt, 0, r.u()
        if vt in (PV_INT, PV_COUNTER, PV_TIMESTAMP):
            return vt, 0, r.s()
        if vt == PV_F64:
            return vt, 0, _f64(r.raw(8))
        if vt == PV_BYTES:
            dt = r.u()
            return vt, dt, js_bytes(r.raw(r.u()))
        if vt == PV_CHILD:
            c, a, t = r.u(), r.u(), r.u()
            return vt, t, (c, a)
        raise ValueError("bad value tag %d" % vt)

    def value():
        vt, dt, v = prim()
        if vt == PV_CHILD:
            return node(v[0], v[1], dt)
        out = {"type": "value", "value": v}
        if vt in NAMED_DT:
            out["datatype"] = NAMED_DT[vt]
        elif vt == PV_BYTES:
            out["datatype"] = dt
        return out

    root = {"objectId": "_root", "type": "map", "props": {}}
    cur, key = root, None
    while r.o < end:
        tag = r.byte()
        if tag == PR_ACTOR:
            actors.append(r.raw(r.u()).hex())
        elif tag == PR_CLOCK:
            a = r.u()
            clock[actors[a]] = r.u()
        elif tag == PR_OBJ:
            c, a, t = r.s(), r.s(), r.u()
            # getPatch logs announce an object in its parent first; applyChanges logs list the
            # object patches in objectMeta order, so a section may create its node
            cur = root if a < 0 else node(c, a, t)
        elif tag == PR_KEY:
            key = r.raw(r.u()).decode("utf-8", "replace")
            cur["props"][key] = {}
        elif tag == PR_PROP:
            c, a = r.u(), r.u()
            cur["props"][key][opid(c, a)] = value()
        elif tag == PR_INSERT:
            idx, ec, ea, oc, oa = r.u(), r.u(), r.u(), r.u(), r.u()
            cur["edits"].append({"action": "insert", "index": idx, "elemId": opid(ec, ea), "opId": opid(oc, oa),
                                 "value": value()})
        elif tag == PR_MULTI:
            idx, ec, ea, dt, n = r.u(), r.u(), r.u(), r.u(), r.u()
            e = {"action": "multi-insert", "index": idx, "elemId": opid(ec, ea)}
            if dt:
                e["datatype"] = NAMED_DT[PV_UINT + dt - 1] if dt < 100 else dt - 100
            e["values"] = [prim()[2] for _ in range(n)]
            cur["edits"].append(e)
        elif tag == PR_UPDATE:
            idx, oc, oa = r.u(), r.u(), r.u()
            cur["edits"].append({"action": "update", "index": idx, "opId": opid(oc, oa), "value": value()})
        elif tag == PR_REMOVE:
            idx = r.u()
            cur["edits"].append({"action": "remove", "index": idx, "count": r.u()})
        else:
            raise ValueError("bad record tag %d" % tag)
    return {"maxOp": int(hdr["max_op"]) if max_op is None else int(max_op), "clock": clock, "deps": list(deps),
            "pendingChanges": int(pending_changes), "diffs": root}
