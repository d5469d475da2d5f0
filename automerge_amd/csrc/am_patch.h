// am_patch.h -- Backend.getPatch() as a compact binary patch log.
//
// patch_scan() restates documentPatch (new.js:1604-1635) with updatePatchProperty for the whole
// document (new.js:884-1040, newBlock = null, oldSuccNum = succNum), appendEdit / appendUpdate
// (new.js:747-823) and decodeValue (columnar.js:300-329). It walks the ops in document order
// once and emits fixed-size records; every merge of list edits (multi-insert coalescing, update
// pops, remove counts) is resolved here at the tail of the log, so the host stage only turns
// records into objects (automerge_amd/patch.py, automerge_amd/js/backend.js).
//
// It is a template over the op source so that the same code runs on lane 0 of k_doc (rows in
// LDS, phase P7) and in the host check of tests/test_patch_kernel_host.py.
#pragma once
#include <stdint.h>

// Everything is force-inlined into the caller: on the device the op source and the scratch live in
// LDS, and inlining keeps that address space a compile-time fact (ds_* accesses, no flat casts).
#ifdef __HIPCC__
#define AM_PHD __host__ __device__ __attribute__((always_inline))
#else
#define AM_PHD __attribute__((always_inline))
#endif

// ---- working form of the log: nrec PatchRec, nmval PatchVal, nheap bytes (wire form below) ----
enum : uint32_t {
  PR_ACTOR = 1,   // actor id i: heap [v0, v0 + v1)
  PR_CLOCK = 2,   // clock[actor a1] = index
  PR_OBJ = 3,     // following records belong to object (c1, a1); a1 = -1: _root
  PR_KEY = 4,     // props[key] = {} with key = heap [v0, v0 + v1) -- current map key
  PR_PROP = 5,    // props[key][opId (c2, a2)] = value
  PR_INSERT = 6,  // {action: insert, index, elemId (c1, a1), opId (c2, a2), value}
  PR_MULTI = 7,   // {action: multi-insert, index, elemId (c1, a1), datatype dt, values: next n PatchVal}
  PR_UPDATE = 8,  // {action: update, index, opId (c2, a2), value}
  PR_REMOVE = 9,  // {action: remove, index, count: n}
};
// value tags (vtag): the {type: 'value', value, datatype} object, or a child object patch
enum : uint32_t {
  PV_NULL = 1, PV_FALSE, PV_TRUE,
  PV_STR,        // heap [v0, v0 + v1) as UTF-8 (TextDecoder: invalid -> U+FFFD)
  PV_UINT,       // v0, datatype 'uint'
  PV_INT,        // v0, datatype 'int'
  PV_F64,        // v0 = IEEE754 bits, datatype 'float64'
  PV_COUNTER,    // v0, datatype 'counter'
  PV_TIMESTAMP,  // v0, datatype 'timestamp'
  PV_BYTES,      // heap [v0, v0 + v1) as Uint8Array, datatype = dt (7 bytes, 0..2 / 10..15 unknown)
  PV_CHILD,      // child object patch: objectId (v0, actor v1), type dt (0 map 1 list 2 text 3 table
                 // 4 undefined 5 null)
};
// multi-insert datatype codes (dt of PR_MULTI): 0 none, else 1 + (vtag - PV_UINT) for named ones,
// 100 + n for a numeric datatype n
enum : uint32_t { PDT_NONE = 0 };

struct PatchRec {  // 64 bytes
  uint32_t tag, vtag;
  int64_t index;   // list index; remove: index; clock: seq
  int64_t c1, c2;  // counters of id1 (elemId / objectId) and id2 (opId)
  int32_t a1, a2;  // actor indexes of id1 / id2
  int64_t v0, v1;  // value payload
  uint32_t dt, n;  // datatype / child type; multi-insert value count or remove count
};
struct PatchVal {  // 32 bytes: a multi-insert value (the primitive only)
  uint32_t vtag, dt;
  int64_t v0, v1, pad;
};
struct PatchOut {
  PatchRec* rec;
  PatchVal* mval;
  uint8_t* heap;
  uint64_t nrec, nmval, nheap, cap_rec, cap_mval, cap_heap;
  uint32_t status;
  int64_t arg0, arg1;
};

// ---- wire form: what leaves the device and what the host stages read ----
// The fixed-size records above are the writers' working form (the scans pop and rewrite the tail
// of the log in place). The log handed to the host is PatchHdr2 followed by a byte stream of the
// same records, LEB128 fields and inline strings, 10-20x smaller than the working form:
//   ACTOR  uleb len, bytes               CLOCK  uleb actor, uleb seq
//   OBJ    sleb ctr, sleb actor, uleb type (root: -1, -1)
//   KEY    uleb len, bytes               PROP   uleb ctr, uleb actor, VALUE
//   INSERT uleb index, uleb elem ctr, uleb elem actor, uleb op ctr, uleb op actor, VALUE
//   MULTI  uleb index, uleb elem ctr, uleb elem actor, uleb datatype code, uleb n, n x VALUE
//   UPDATE uleb index, uleb op ctr, uleb op actor, VALUE
//   REMOVE uleb index, uleb count
//   VALUE  vtag byte, then: STR uleb len + bytes | UINT uleb | INT / COUNTER / TIMESTAMP sleb |
//          F64 8 bytes LE | BYTES uleb datatype, uleb len, bytes | CHILD uleb ctr, uleb actor,
//          uleb type | nothing for NULL / FALSE / TRUE
// Every record starts with its tag byte. Hosts: automerge_amd/patch.py, automerge_amd/js/backend.js.
#define AM_PATCH_MAGIC 0x32504d41u  // "AMP2"
struct PatchHdr2 {  // 48 bytes
  uint32_t magic;
  uint32_t status;    // 0 ok, else the AM_* code of the error the call throws
  int64_t arg0, arg1; // error arguments (counter increment: ctr, actor index)
  int64_t max_op;     // documentPatch's maxOp (getPatch logs)
  uint64_t nbytes;    // stream bytes after the header
  uint64_t meta_bytes;  // AM_DOC_META: bytes of the objectMeta blob after the stream (am_diff.h diff_meta_pack)
};

AM_PHD inline uint32_t pk_uleb_len(uint64_t v) {
  uint32_t n = 1;
  while (v >= 0x80) { v >>= 7; n++; }
  return n;
}
AM_PHD inline uint32_t pk_sleb_len(int64_t v) {
  uint32_t n = 1;
  while (!((v >= -64) && (v < 64))) { v >>= 7; n++; }
  return n;
}
AM_PHD inline uint8_t* pk_uleb(uint8_t* o, uint64_t v) {
  while (v >= 0x80) { *o++ = (uint8_t)(v | 0x80); v >>= 7; }
  *o++ = (uint8_t)v;
  return o;
}
AM_PHD inline uint8_t* pk_sleb(uint8_t* o, int64_t v) {
  for (;;) {
    const uint8_t b = (uint8_t)(v & 0x7f);
    v >>= 7;
    if ((v == 0 && !(b & 0x40)) || (v == -1 && (b & 0x40))) { *o++ = b; return o; }
    *o++ = (uint8_t)(b | 0x80);
  }
}
// bytes of a VALUE (vtag, dt, v0, v1; strings / bytes at heap + v0)
AM_PHD inline uint32_t pk_value_len(uint32_t vtag, uint32_t dt, int64_t v0, int64_t v1) {
  switch (vtag) {
    case PV_STR: return 1 + pk_uleb_len((uint64_t)v1) + (uint32_t)v1;
    case PV_UINT: return 1 + pk_uleb_len((uint64_t)v0);
    case PV_INT: case PV_COUNTER: case PV_TIMESTAMP: return 1 + pk_sleb_len(v0);
    case PV_F64: return 9;
    case PV_BYTES: return 1 + pk_uleb_len(dt) + pk_uleb_len((uint64_t)v1) + (uint32_t)v1;
    case PV_CHILD: return 1 + pk_uleb_len((uint64_t)v0) + pk_uleb_len((uint64_t)v1) + pk_uleb_len(dt);
    default: return 1;
  }
}
AM_PHD inline uint8_t* pk_value(uint8_t* o, uint32_t vtag, uint32_t dt, int64_t v0, int64_t v1, const uint8_t* bytes) {
  *o++ = (uint8_t)vtag;
  switch (vtag) {
    case PV_STR:
      o = pk_uleb(o, (uint64_t)v1);
      for (int64_t q = 0; q < v1; q++) *o++ = bytes[q];
      break;
    case PV_UINT: o = pk_uleb(o, (uint64_t)v0); break;
    case PV_INT: case PV_COUNTER: case PV_TIMESTAMP: o = pk_sleb(o, v0); break;
    case PV_F64:
      for (int q = 0; q < 8; q++) *o++ = (uint8_t)((uint64_t)v0 >> (8 * q));
      break;
    case PV_BYTES:
      o = pk_uleb(o, dt);
      o = pk_uleb(o, (uint64_t)v1);
      for (int64_t q = 0; q < v1; q++) *o++ = bytes[q];
      break;
    case PV_CHILD:
      o = pk_uleb(o, (uint64_t)v0);
      o = pk_uleb(o, (uint64_t)v1);
      o = pk_uleb(o, dt);
      break;
    default: break;
  }
  return o;
}
AM_PHD inline bool pv_has_bytes(uint32_t vtag) { return vtag == PV_STR || vtag == PV_BYTES; }

// Serializes a working-form log into its wire form at dst (capacity cap bytes, header included).
// Returns the total bytes, or 0 when cap is too small.
AM_PHD inline uint64_t patch_pack(const PatchOut& o, int64_t max_op, uint8_t* dst, uint64_t cap) {
  PatchHdr2 h;
  h.magic = AM_PATCH_MAGIC;
  h.status = o.status;
  h.arg0 = o.arg0;
  h.arg1 = o.arg1;
  h.max_op = max_op;
  h.meta_bytes = 0;
  uint64_t n = 0;
  if (!o.status) {
    uint64_t mv = 0;
    for (uint64_t k = 0; k < o.nrec; k++) {
      const PatchRec& r = o.rec[k];
      uint64_t b = 1;
      switch (r.tag) {
        case PR_ACTOR: case PR_KEY: b += pk_uleb_len((uint64_t)r.v1) + (uint64_t)r.v1; break;
        case PR_CLOCK: b += pk_uleb_len((uint64_t)r.a1) + pk_uleb_len((uint64_t)r.index); break;
        case PR_OBJ: b += pk_sleb_len(r.c1) + pk_sleb_len(r.a1) + pk_uleb_len(r.dt); break;
        case PR_PROP: b += pk_uleb_len((uint64_t)r.c2) + pk_uleb_len((uint64_t)r.a2) + pk_value_len(r.vtag, r.dt, r.v0, r.v1); break;
        case PR_INSERT:
          b += pk_uleb_len((uint64_t)r.index) + pk_uleb_len((uint64_t)r.c1) + pk_uleb_len((uint64_t)r.a1) +
               pk_uleb_len((uint64_t)r.c2) + pk_uleb_len((uint64_t)r.a2) + pk_value_len(r.vtag, r.dt, r.v0, r.v1);
          break;
        case PR_MULTI:
          b += pk_uleb_len((uint64_t)r.index) + pk_uleb_len((uint64_t)r.c1) + pk_uleb_len((uint64_t)r.a1) +
               pk_uleb_len(r.dt) + pk_uleb_len(r.n);
          for (uint32_t q = 0; q < r.n; q++) {
            const PatchVal& v = o.mval[mv + q];
            b += pk_value_len(v.vtag, v.dt, v.v0, v.v1);
          }
          mv += r.n;
          break;
        case PR_UPDATE:
          b += pk_uleb_len((uint64_t)r.index) + pk_uleb_len((uint64_t)r.c2) + pk_uleb_len((uint64_t)r.a2) +
               pk_value_len(r.vtag, r.dt, r.v0, r.v1);
          break;
        default: b += pk_uleb_len((uint64_t)r.index) + pk_uleb_len(r.n); break;  // PR_REMOVE
      }
      n += b;
    }
  }
  h.nbytes = n;
  if (sizeof(PatchHdr2) + n > cap) return 0;
  const uint8_t* hb = reinterpret_cast<const uint8_t*>(&h);
  for (uint32_t q = 0; q < sizeof(PatchHdr2); q++) dst[q] = hb[q];
  uint8_t* p = dst + sizeof(PatchHdr2);
  if (o.status) return sizeof(PatchHdr2);
  uint64_t mv = 0;
  for (uint64_t k = 0; k < o.nrec; k++) {
    const PatchRec& r = o.rec[k];
    *p++ = (uint8_t)r.tag;
    switch (r.tag) {
      case PR_ACTOR: case PR_KEY:
        p = pk_uleb(p, (uint64_t)r.v1);
        for (int64_t q = 0; q < r.v1; q++) *p++ = o.heap[r.v0 + q];
        break;
      case PR_CLOCK: p = pk_uleb(p, (uint64_t)r.a1); p = pk_uleb(p, (uint64_t)r.index); break;
      case PR_OBJ: p = pk_sleb(p, r.c1); p = pk_sleb(p, r.a1); p = pk_uleb(p, r.dt); break;
      case PR_PROP:
        p = pk_uleb(p, (uint64_t)r.c2); p = pk_uleb(p, (uint64_t)r.a2);
        p = pk_value(p, r.vtag, r.dt, r.v0, r.v1, pv_has_bytes(r.vtag) ? o.heap + r.v0 : nullptr);
        break;
      case PR_INSERT:
        p = pk_uleb(p, (uint64_t)r.index); p = pk_uleb(p, (uint64_t)r.c1); p = pk_uleb(p, (uint64_t)r.a1);
        p = pk_uleb(p, (uint64_t)r.c2); p = pk_uleb(p, (uint64_t)r.a2);
        p = pk_value(p, r.vtag, r.dt, r.v0, r.v1, pv_has_bytes(r.vtag) ? o.heap + r.v0 : nullptr);
        break;
      case PR_MULTI:
        p = pk_uleb(p, (uint64_t)r.index); p = pk_uleb(p, (uint64_t)r.c1); p = pk_uleb(p, (uint64_t)r.a1);
        p = pk_uleb(p, r.dt); p = pk_uleb(p, r.n);
        for (uint32_t q = 0; q < r.n; q++) {
          const PatchVal& v = o.mval[mv + q];
          p = pk_value(p, v.vtag, v.dt, v.v0, v.v1, pv_has_bytes(v.vtag) ? o.heap + v.v0 : nullptr);
        }
        mv += r.n;
        break;
      case PR_UPDATE:
        p = pk_uleb(p, (uint64_t)r.index); p = pk_uleb(p, (uint64_t)r.c2); p = pk_uleb(p, (uint64_t)r.a2);
        p = pk_value(p, r.vtag, r.dt, r.v0, r.v1, pv_has_bytes(r.vtag) ? o.heap + r.v0 : nullptr);
        break;
      default: p = pk_uleb(p, (uint64_t)r.index); p = pk_uleb(p, r.n); break;
    }
  }
  return sizeof(PatchHdr2) + n;
}

// errors of getPatch (mirrors include/automerge_amd.h codes; see am_common.h static_asserts)
#define PATCH_E_FLOAT_LEN 31u   // Invalid length for floating point number: arg0
#define PATCH_E_UNKNOWN_COUNTER 32u  // increment operation arg0@actor(arg1) for unknown counter
#define PATCH_U_CAPACITY 106u
#define PATCH_U_VALUE 105u
#define PATCH_U_INC_VALUE 107u  // a non-integer increment: the replay goes on, the patch value is unknown

// ---- value decode (decodeValue, columnar.js:300-329) ----
template <class Src>
AM_PHD inline bool patch_value(const Src& src, uint32_t i, PatchOut& o, uint32_t& vtag, uint32_t& dt, int64_t& v0, int64_t& v1) {
  const int64_t tag = src.val_len(i);  // null valLen reads as 0
  dt = 0;
  v0 = v1 = 0;
  if (tag == 0) { vtag = PV_NULL; return true; }
  if (tag == 1) { vtag = PV_FALSE; return true; }
  if (tag == 2) { vtag = PV_TRUE; return true; }
  const uint32_t len = (uint32_t)((uint64_t)tag >> 4);
  switch (tag & 15) {
    case 6: case 7: case 0: case 1: case 2: case 10: case 11: case 12: case 13: case 14: case 15: {
      if (o.nheap + len > o.cap_heap) { o.status = PATCH_U_CAPACITY; return false; }
      src.copy_value(i, o.heap + o.nheap);
      v0 = (int64_t)o.nheap;
      v1 = len;
      o.nheap += len;
      if ((tag & 15) == 6) vtag = PV_STR;
      else { vtag = PV_BYTES; dt = (uint32_t)(tag & 15); }
      return true;
    }
    case 5: {
      if (len != 8) { o.status = PATCH_E_FLOAT_LEN; o.arg0 = len; return false; }
      v0 = src.value_f64_bits(i);
      vtag = PV_F64;
      return true;
    }
    default: {
      int64_t x;
      if (!src.value_int(i, (tag & 15) == 3, x)) { o.status = PATCH_U_VALUE; return false; }
      v0 = x;
      vtag = (tag & 15) == 3 ? PV_UINT : (tag & 15) == 4 ? PV_INT : (tag & 15) == 8 ? PV_COUNTER : PV_TIMESTAMP;
      return true;
    }
  }
}

// JS typeof class of a value (multi-insert check): 0 object, 1 boolean, 2 string, 3 number
AM_PHD inline int pv_typeof(uint32_t vtag) {
  switch (vtag) {
    case PV_FALSE: case PV_TRUE: return 1;
    case PV_STR: return 2;
    case PV_UINT: case PV_INT: case PV_F64: case PV_COUNTER: case PV_TIMESTAMP: return 3;
    default: return 0;
  }
}
// datatype annotation code: 0 = none; named: 1 + vtag - PV_UINT; numeric n: 100 + n
AM_PHD inline uint32_t pv_dtcode(uint32_t vtag, uint32_t dt) {
  if (vtag >= PV_UINT && vtag <= PV_TIMESTAMP) return 1 + vtag - PV_UINT;
  if (vtag == PV_BYTES) return 100 + dt;
  return 0;
}
AM_PHD inline bool pv_dt_truthy(uint32_t code) { return code != 0 && code != 100; }
// object type of a make-like action (OBJECT_TYPE[ACTIONS[a]], new.js:886): 0 map 1 list 2 text
// 3 table, 4 undefined (null action), 5 null (an even action beyond ACTIONS); a = -1 for null
AM_PHD inline uint32_t pv_obj_type(int64_t a) {
  return a < 0 ? 4u : a == 2 ? 1u : a == 4 ? 2u : a == 6 ? 3u : a >= 8 ? 5u : 0u;
}

// ---- the scan ----
// Src interface (all indexes are positions in document order):
//   n(); obj_ctr(i) (-1 root), obj_actor(i) (-1 root); has_key(i) (key string not null);
//   key_eq(i, j); copy_key(i, dst) / key_len(i); key_ctr(i), key_actor(i); id_ctr(i), id_actor(i);
//   insert(i); action(i); val_len(i); copy_value(i, dst); value_int(i, is_uint, out);
//   value_f64_bits(i); nsucc(i); succ_ctr(i, k), succ_actor(i, k);
//   nactors(); actor_len(a); copy_actor(a, dst); nchg(); chg_actor(c); chg_seq(c)
// Scratch (caller-provided, sized by the op count n):
//   mk_ctr/mk_actor/mk_vis: make ops seen (objectMeta) and whether their object is reachable
//   cs_*: counter states of the current key group; cm_*: counterStates map (succ opId -> state)
struct PatchScratch {
  int64_t* mk_ctr; int32_t* mk_actor; uint8_t* mk_vis; uint32_t mk_cap;
  int64_t* cs_ctr; int32_t* cs_actor; int64_t* cs_val; int32_t* cs_left; uint32_t cs_cap;
  int64_t* cm_ctr; int32_t* cm_actor; int32_t* cm_state; uint32_t cm_cap;
};

AM_PHD inline bool patch_push(PatchOut& o, const PatchRec& r) {
  if (o.nrec >= o.cap_rec) { o.status = PATCH_U_CAPACITY; return false; }
  o.rec[o.nrec++] = r;
  return true;
}
AM_PHD inline bool patch_push_val(PatchOut& o, uint32_t vtag, uint32_t dt, int64_t v0, int64_t v1) {
  if (o.nmval >= o.cap_mval) { o.status = PATCH_U_CAPACITY; return false; }
  PatchVal& v = o.mval[o.nmval++];
  v.vtag = vtag; v.dt = dt; v.v0 = v0; v.v1 = v1; v.pad = 0;
  return true;
}

// appendEdit (new.js:747-782) on the tail of the current object's edits (records from rec0)
AM_PHD inline bool patch_append_edit(PatchOut& o, const PatchRec& ne, uint64_t rec0) {
  if (o.nrec > rec0) {
    PatchRec& last = o.rec[o.nrec - 1];
    if (last.tag == PR_INSERT && ne.tag == PR_INSERT && last.index == ne.index - 1 && last.vtag != PV_CHILD &&
        ne.vtag != PV_CHILD && last.c1 == last.c2 && last.a1 == last.a2 && ne.c1 == ne.c2 && ne.a1 == ne.a2 &&
        last.a1 == ne.a1 && last.c1 + 1 == ne.c1) {
      const uint32_t da = pv_dtcode(last.vtag, last.dt), db = pv_dtcode(ne.vtag, ne.dt);
      if (da == db && pv_typeof(last.vtag) == pv_typeof(ne.vtag)) {
        if (!patch_push_val(o, last.vtag, last.dt, last.v0, last.v1) || !patch_push_val(o, ne.vtag, ne.dt, ne.v0, ne.v1))
          return false;
        last.tag = PR_MULTI;
        last.n = 2;
        last.dt = pv_dt_truthy(db) ? db : 0;  // lastEdit.datatype set only when truthy
        return true;
      }
    }
    if (last.tag == PR_MULTI && ne.tag == PR_INSERT && last.index + (int64_t)last.n == ne.index && ne.vtag != PV_CHILD &&
        ne.c1 == ne.c2 && ne.a1 == ne.a2 && last.a1 == ne.a1 && last.c1 + (int64_t)last.n == ne.c1) {
      const uint32_t db = pv_dtcode(ne.vtag, ne.dt);
      const PatchVal& first = o.mval[o.nmval - last.n];  // this edit's values end the value array
      if (last.dt == db && pv_typeof(first.vtag) == pv_typeof(ne.vtag)) {
        if (!patch_push_val(o, ne.vtag, ne.dt, ne.v0, ne.v1)) return false;
        last.n++;
        return true;
      }
    }
    if (last.tag == PR_REMOVE && ne.tag == PR_REMOVE && last.index == ne.index) {
      last.n += ne.n;
      return true;
    }
  }
  return patch_push(o, ne);
}

// appendUpdate (new.js:797-823)
AM_PHD inline bool patch_append_update(PatchOut& o, int64_t index, int64_t ec, int32_t ea, int64_t oc, int32_t oa,
                                       uint32_t vtag, uint32_t dt, int64_t v0, int64_t v1, bool first, uint64_t rec0) {
  bool insert = false;
  if (first) {
    while (!insert && o.nrec > rec0) {
      PatchRec& last = o.rec[o.nrec - 1];
      if ((last.tag == PR_INSERT || last.tag == PR_UPDATE) && last.index == index) {
        insert = last.tag == PR_INSERT;
        o.nrec--;
      } else if (last.tag == PR_MULTI && last.index + (int64_t)last.n - 1 == index) {
        last.n--;
        o.nmval--;
        insert = true;
      } else {
        break;
      }
    }
  }
  PatchRec r = {};
  r.index = index;
  r.c2 = oc; r.a2 = oa;
  r.vtag = vtag; r.dt = dt; r.v0 = v0; r.v1 = v1;
  if (insert) { r.tag = PR_INSERT; r.c1 = ec; r.a1 = ea; }
  else r.tag = PR_UPDATE;
  return patch_append_edit(o, r, rec0);
}

template <class Src>
AM_PHD inline bool patch_scan(const Src& src, PatchOut& o, PatchScratch& w, int64_t& max_op) {
  o.nrec = o.nmval = o.nheap = 0;
  o.status = 0;
  max_op = 0;
  // actor table and clock
  for (uint32_t a = 0; a < src.nactors(); a++) {
    PatchRec r = {};
    r.tag = PR_ACTOR;
    const uint32_t l = src.actor_len(a);
    if (o.nheap + l > o.cap_heap) { o.status = PATCH_U_CAPACITY; return false; }
    src.copy_actor(a, o.heap + o.nheap);
    r.v0 = (int64_t)o.nheap;
    r.v1 = l;
    o.nheap += l;
    r.a1 = (int32_t)a;
    if (!patch_push(o, r)) return false;
  }
  for (uint32_t c = 0; c < src.nchg(); c++) {  // clock: last seq per actor, first-appearance order
    bool later = false;
    for (uint32_t d = c + 1; d < src.nchg() && !later; d++) later = src.chg_actor(d) == src.chg_actor(c);
    if (later) continue;
    PatchRec r = {};
    r.tag = PR_CLOCK;
    r.a1 = (int32_t)src.chg_actor(c);
    r.index = src.chg_seq(c);
    if (!patch_push(o, r)) return false;
  }
  const uint32_t N = src.n();
  uint32_t nmk = 0;
  int64_t last_oc = -2;
  int32_t last_oa = -2;
  bool reachable = false, is_list = false, elem_visible = false;
  int64_t list_index = 0;
  uint64_t obj_rec0 = 0;  // first record of the current object's section
  // current key group (propState[elemId])
  int32_t g_row = -1;  // first op of the group
  bool g_str = false;
  int64_t g_ec = 0;
  int32_t g_ea = 0;
  uint32_t g_action = 0;  // 0 none, 1 insert, 2 update, 3 remove
  uint32_t ncs = 0, ncm = 0;
  bool key_emitted = false;
  for (uint32_t i = 0; i < N; i++) {
    const int64_t oc = src.obj_ctr(i);
    const int32_t oa = src.obj_actor(i);
    if (oc != last_oc || oa != last_oa) {
      last_oc = oc; last_oa = oa;
      list_index = 0;
      elem_visible = false;
      g_row = -1;
      if (oa < 0) { reachable = true; is_list = false; }
      else {
        int32_t m = -1;
        for (uint32_t k = 0; k < nmk; k++) if (w.mk_ctr[k] == oc && w.mk_actor[k] == oa) m = (int32_t)k;
        if (m < 0) { o.status = PATCH_U_VALUE; return false; }  // objectMeta[objectId] undefined
        reachable = w.mk_vis[m] != 0;
        is_list = (w.mk_vis[m] & 6) != 0;  // bit 1 list, bit 2 text
      }
      if (reachable) {
        PatchRec r = {};
        r.tag = PR_OBJ;
        r.c1 = oc;
        r.a1 = oa;
        if (!patch_push(o, r)) return false;
        obj_rec0 = o.nrec;
      }
    }
    const uint32_t nsucc = src.nsucc(i);
    const bool ins = src.insert(i);
    if (ins && elem_visible) { elem_visible = false; list_index++; }
    if (nsucc == 0) elem_visible = true;
    const int64_t idc = src.id_ctr(i);
    const int32_t ida = src.id_actor(i);
    if (idc > max_op) max_op = idc;
    for (uint32_t k = 0; k < nsucc; k++) if (src.succ_ctr(i, k) > max_op) max_op = src.succ_ctr(i, k);
    const int64_t action = src.action(i);
    const bool has_key = src.has_key(i);
    if (has_key && src.key_len(i) == 0) { o.status = PATCH_U_VALUE; return false; }  // '' key (falsy in JS)
    const int64_t ec = ins ? idc : src.key_ctr(i);
    const int32_t ea = ins ? ida : src.key_actor(i);
    // make-like: `op[actionIdx] % 2 === 0` (new.js:894, 972), every even action and a null one
    const bool is_make = action < 0 || (action % 2) == 0;
    if (is_make) {  // objectMeta[opId]; reachable (visible make op of a reachable object) + type bits
      bool known = false;
      for (uint32_t k = 0; k < nmk && !known; k++) known = w.mk_ctr[k] == idc && w.mk_actor[k] == ida;
      if (!known) {
        if (nmk >= w.mk_cap) { o.status = PATCH_U_CAPACITY; return false; }
        w.mk_ctr[nmk] = idc;
        w.mk_actor[nmk] = ida;
        const uint8_t tbits = action == 2 ? 2 : action == 4 ? 4 : 0;
        w.mk_vis[nmk] = (reachable && nsucc == 0) ? (uint8_t)(1 | tbits) : 0;
        nmk++;
      }
    }
    // group = ops of one key / list element (adjacent in document order)
    bool same = false;
    if (g_row >= 0) {
      if (has_key) same = g_str && src.key_eq((uint32_t)g_row, i);
      else same = !g_str && g_ec == ec && g_ea == ea;
    }
    const bool first_op = !same;
    if (!same) {
      g_row = (int32_t)i; g_str = has_key; g_ec = ec; g_ea = ea;
      g_action = 0; ncs = 0; ncm = 0; key_emitted = false;
    }
    const bool overwritten = nsucc > 0;
    // patchKey / patchValue
    bool have_pv = false;
    uint32_t vtag = 0, vdt = 0;
    int64_t v0 = 0, v1 = 0, pk_c = 0;
    int32_t pk_a = 0;
    const int64_t tag = src.val_len(i);
    if (overwritten && action == 1 && (tag & 0x0f) == 8) {
      // set op creating a counter: its successors must all turn out to be increments
      if (ncs >= w.cs_cap) { o.status = PATCH_U_CAPACITY; return false; }
      int64_t cv;
      if (!src.value_int(i, false, cv)) { o.status = PATCH_U_VALUE; return false; }
      const uint32_t st = ncs++;
      w.cs_ctr[st] = idc; w.cs_actor[st] = ida; w.cs_val[st] = cv; w.cs_left[st] = 0;
      for (uint32_t k = 0; k < nsucc; k++) {
        const int64_t sc = src.succ_ctr(i, k);
        const int32_t sa = src.succ_actor(i, k);
        uint32_t q = 0;
        while (q < ncm && !(w.cm_ctr[q] == sc && w.cm_actor[q] == sa)) q++;
        if (q == ncm) {
          if (ncm >= w.cm_cap) { o.status = PATCH_U_CAPACITY; return false; }
          ncm++;
        }
        w.cm_ctr[q] = sc; w.cm_actor[q] = sa; w.cm_state[q] = (int32_t)st;
        bool dup = false;
        for (uint32_t j = 0; j < k; j++) dup = dup || (src.succ_ctr(i, j) == sc && src.succ_actor(i, j) == sa);
        if (!dup) w.cs_left[st]++;
      }
    } else if (action == 5) {  // inc
      uint32_t q = 0;
      while (q < ncm && !(w.cm_ctr[q] == idc && w.cm_actor[q] == ida)) q++;
      if (q == ncm) { o.status = PATCH_E_UNKNOWN_COUNTER; o.arg0 = idc; o.arg1 = ida; return false; }
      const int32_t st = w.cm_state[q];
      const uint32_t t15 = (uint32_t)(tag & 15);
      int64_t iv;
      if (tag < 16 || !(t15 == 3 || t15 == 4 || t15 == 8 || t15 == 9) || !src.value_int(i, t15 == 3, iv)) {
        o.status = PATCH_U_VALUE;  // non-integer increment (JS would concatenate / add a float)
        return false;
      }
      w.cs_val[st] += iv;
      w.cs_left[st]--;
      if (w.cs_left[st] == 0) {
        have_pv = true;
        vtag = PV_COUNTER;
        v0 = w.cs_val[st];
        pk_c = w.cs_ctr[st];
        pk_a = w.cs_actor[st];
      }
    } else if (!overwritten) {
      if (action == 1) {
        if (reachable && !patch_value(src, i, o, vtag, vdt, v0, v1)) return false;
        have_pv = true;
        pk_c = idc; pk_a = ida;
      } else if (is_make) {
        have_pv = true;
        vtag = PV_CHILD;
        vdt = pv_obj_type(action);
        v0 = idc; v1 = ida;
        pk_c = idc; pk_a = ida;
      }
    }
    if (!reachable) continue;  // unreachable object: its patch is not part of the result
    if (!has_key) {
      if (!is_list) { o.status = PATCH_U_VALUE; return false; }  // elemId key in a map object
      if (have_pv) {
        if (!g_action) {
          g_action = 1;
          PatchRec r = {};
          r.tag = PR_INSERT; r.vtag = vtag; r.dt = vdt; r.index = list_index;
          r.c1 = ec; r.a1 = ea; r.c2 = pk_c; r.a2 = pk_a; r.v0 = v0; r.v1 = v1;
          if (!patch_append_edit(o, r, obj_rec0)) return false;
        } else if (g_action == 3) {
          PatchRec* last = o.nrec > obj_rec0 ? &o.rec[o.nrec - 1] : nullptr;
          if (!last || last->tag != PR_REMOVE) { o.status = PATCH_U_VALUE; return false; }
          if (last->n > 1) last->n--; else o.nrec--;
          g_action = 2;
          if (!patch_append_update(o, list_index, ec, ea, pk_c, pk_a, vtag, vdt, v0, v1, true, obj_rec0)) return false;
        } else {
          if (!patch_append_update(o, list_index, ec, ea, pk_c, pk_a, vtag, vdt, v0, v1, false, obj_rec0)) return false;
        }
      } else if (nsucc == 0 && !g_action) {
        g_action = 3;
        PatchRec r = {};
        r.tag = PR_REMOVE; r.index = list_index; r.n = 1;
        if (!patch_append_edit(o, r, obj_rec0)) return false;
      }
    } else if (have_pv) {
      if (is_list) { o.status = PATCH_U_VALUE; return false; }  // string key in a list object
      if (first_op || !key_emitted) {
        PatchRec r = {};
        r.tag = PR_KEY;
        const uint32_t kl = src.key_len(i);
        if (o.nheap + kl > o.cap_heap) { o.status = PATCH_U_CAPACITY; return false; }
        src.copy_key(i, o.heap + o.nheap);
        r.v0 = (int64_t)o.nheap;
        r.v1 = kl;
        o.nheap += kl;
        if (!patch_push(o, r)) return false;
        key_emitted = true;
      }
      PatchRec r = {};
      r.tag = PR_PROP; r.vtag = vtag; r.dt = vdt; r.c2 = pk_c; r.a2 = pk_a; r.v0 = v0; r.v1 = v1;
      if (!patch_push(o, r)) return false;
    }
  }
  return true;
}
