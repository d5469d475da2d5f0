"""Host stage of getPatch: turns the binary patch log written by the engine (am_patch.h, phase P7
of k_doc) into the reference's patch object (new.js:2052-2060; shapes in
@types/automerge/index.d.ts:242-323). No merge logic lives here: every decision (visible values,
conflicts, counters, list indexes, multi-insert coalescing, update pops) was made on the GPU;
this is deserialization plus linking child object patches by objectId.

Layout: PatchHdr (64 B) | nrec PatchRec (64 B) | nmval PatchVal (32 B) | nheap bytes.
"""
import struct

import numpy as np

HDR_DT = np.dtype([("status", "<u4"), ("pad0", "<u4"), ("arg0", "<i8"), ("arg1", "<i8"), ("nrec", "<u8"),
                   ("nmval", "<u8"), ("nheap", "<u8"), ("max_op", "<i8"), ("pad1", "<u8")])
REC_DT = np.dtype([("tag", "<u4"), ("vtag", "<u4"), ("index", "<i8"), ("c1", "<i8"), ("c2", "<i8"), ("a1", "<i4"),
                   ("a2", "<i4"), ("v0", "<i8"), ("v1", "<i8"), ("dt", "<u4"), ("n", "<u4")])
VAL_DT = np.dtype([("vtag", "<u4"), ("dt", "<u4"), ("v0", "<i8"), ("v1", "<i8"), ("pad", "<i8")])
assert HDR_DT.itemsize == 64 and REC_DT.itemsize == 64 and VAL_DT.itemsize == 32

PR_ACTOR, PR_CLOCK, PR_OBJ, PR_KEY, PR_PROP, PR_INSERT, PR_MULTI, PR_UPDATE, PR_REMOVE = range(1, 10)
(PV_NULL, PV_FALSE, PV_TRUE, PV_STR, PV_UINT, PV_INT, PV_F64, PV_COUNTER, PV_TIMESTAMP, PV_BYTES,
 PV_CHILD) = range(1, 12)
NAMED_DT = {PV_UINT: "uint", PV_INT: "int", PV_F64: "float64", PV_COUNTER: "counter", PV_TIMESTAMP: "timestamp"}
OBJ_TYPES = ("map", "list", "text", "table")

# errors getPatch throws (am_patch.h PATCH_*)
PATCH_E_FLOAT_LEN, PATCH_E_UNKNOWN_COUNTER = 31, 32


def _f64(bits):
    return struct.unpack("<d", struct.pack("<q", int(bits)))[0]


def split(blob):
    """(header, records, values, heap) views of a patch log."""
    hdr = np.frombuffer(blob, dtype=HDR_DT, count=1)[0]
    nrec, nmval = int(hdr["nrec"]), int(hdr["nmval"])
    recs = np.frombuffer(blob, dtype=REC_DT, count=nrec, offset=64)
    off = 64 + 64 * nrec
    vals = np.frombuffer(blob, dtype=VAL_DT, count=nmval, offset=off)
    off += 32 * nmval
    heap = bytes(blob[off:off + int(hdr["nheap"])])
    return hdr, recs, vals, heap


def error_message(hdr, actors=None):
    st = int(hdr["status"])
    if st == PATCH_E_FLOAT_LEN:
        return "Invalid length for floating point number: %d" % int(hdr["arg0"])
    if st == PATCH_E_UNKNOWN_COUNTER:
        a = actors[int(hdr["arg1"])] if actors and 0 <= int(hdr["arg1"]) < len(actors) else "?"
        return "increment operation %d@%s for unknown counter" % (int(hdr["arg0"]), a)
    return "automerge_amd: getPatch not supported for this document (code %d)" % st


def materialize(blob, deps, pending_changes, max_op=None, js_bytes=bytes):
    """The getPatch() result for a patch log. `deps` = heads (hex), `pending_changes` = queue
    length; max_op defaults to documentPatch's maxOp from the log. Raises AutomergeError with the
    reference's message when the log carries an error."""
    hdr, recs, vals, heap = split(blob)
    actors, clock = [], {}
    # actor table first: needed for error messages too
    for r in recs:
        if r["tag"] != PR_ACTOR:
            break
        actors.append(heap[r["v0"]:r["v0"] + r["v1"]].hex())
    if int(hdr["status"]):
        from ._native import AutomergeError
        raise AutomergeError(error_message(hdr, actors), int(hdr["status"]), "RangeError")

    def opid(c, a):
        return "%d@%s" % (c, actors[a])

    nodes = {}

    def node(c, a, typ):
        k = (int(c), int(a))
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

    def prim(vtag, dt, v0, v1):
        if vtag == PV_NULL:
            return None
        if vtag == PV_FALSE:
            return False
        if vtag == PV_TRUE:
            return True
        if vtag == PV_STR:
            return heap[v0:v0 + v1].decode("utf-8", "replace")
        if vtag == PV_F64:
            return _f64(v0)
        if vtag == PV_BYTES:
            return js_bytes(heap[v0:v0 + v1])
        return int(v0)

    def value(vtag, dt, v0, v1):
        if vtag == PV_CHILD:
            return node(v0, v1, dt)
        out = {"type": "value", "value": prim(vtag, dt, v0, v1)}
        if vtag in NAMED_DT:
            out["datatype"] = NAMED_DT[vtag]
        elif vtag == PV_BYTES:
            out["datatype"] = int(dt)
        return out

    root = {"objectId": "_root", "type": "map", "props": {}}
    cur, key, mv = root, None, 0
    for r in recs[len(actors):]:
        tag = int(r["tag"])
        vt, dt, v0, v1 = int(r["vtag"]), int(r["dt"]), int(r["v0"]), int(r["v1"])
        if tag == PR_CLOCK:
            clock[actors[r["a1"]]] = int(r["index"])
        elif tag == PR_OBJ:
            a1 = int(r["a1"])
            # getPatch logs announce an object in its parent first; applyChanges logs list the
            # object patches in objectMeta order, so a section may create its node
            cur = root if a1 < 0 else node(r["c1"], a1, dt)
        elif tag == PR_KEY:
            key = heap[v0:v0 + v1].decode("utf-8", "replace")
            cur["props"][key] = {}
        elif tag == PR_PROP:
            cur["props"][key][opid(r["c2"], r["a2"])] = value(vt, dt, v0, v1)
        elif tag == PR_INSERT:
            cur["edits"].append({"action": "insert", "index": int(r["index"]), "elemId": opid(r["c1"], r["a1"]),
                                 "opId": opid(r["c2"], r["a2"]), "value": value(vt, dt, v0, v1)})
        elif tag == PR_MULTI:
            e = {"action": "multi-insert", "index": int(r["index"]), "elemId": opid(r["c1"], r["a1"])}
            if dt:
                e["datatype"] = NAMED_DT[PV_UINT + dt - 1] if dt < 100 else dt - 100
            n = int(r["n"])
            e["values"] = [prim(int(x["vtag"]), int(x["dt"]), int(x["v0"]), int(x["v1"])) for x in vals[mv:mv + n]]
            mv += n
            cur["edits"].append(e)
        elif tag == PR_UPDATE:
            cur["edits"].append({"action": "update", "index": int(r["index"]), "opId": opid(r["c2"], r["a2"]),
                                 "value": value(vt, dt, v0, v1)})
        elif tag == PR_REMOVE:
            cur["edits"].append({"action": "remove", "index": int(r["index"]), "count": int(r["n"])})
    return {"maxOp": int(hdr["max_op"]) if max_op is None else int(max_op), "clock": clock, "deps": list(deps),
            "pendingChanges": int(pending_changes), "diffs": root}
