// am_hist_dev.h -- k_history: the change history of saved documents, batched, one workgroup (one
// wave) per document: BackendDoc.computeHashGraph (new.js:1879-1904) over decodeChanges([doc]) =
// decodeDocument (columnar.js:1040) + groupChangeOps (:876-943) + decodeDocumentChanges (:945-981),
// every change re-encoded as encodeChange writes it (:710-739, encodeOps :380-440).
//
// Phases (per document; workspace in HBM, layout hist_layout in am_hist.h):
//   P1  lane 0: document header (parse_doc_hdr) and the actor table; lane per actor: its rank in
//       hex-string order
//   P2  lane per column: the 9 change columns and the 15 op columns (valRaw aside) into cells;
//       the first error in the reference's row-major decode order wins
//   P3  lane per row: op records, decode-phase checks; scans place the raw values and the succ
//       entries of every row
//   P4  succ targets by binary search over the rows sorted by id; an id no row has becomes one
//       re-created `del` (obj / key of the first op naming it, columnar.js:895-902)
//   P5  pred lists: every succ entry is a pred of its target, sorted as compareParsedOpIds
//   P6  change rows: decode checks, then the seq / maxOp rules of groupChangeOps; the del check;
//       every op -> its change (binary search on the author's maxOp)
//   P7  ops by (change, counter); opId contiguity
//   P8  lane per change: slot size, then the encodeChange body
//   P9  deps / extra-bytes checks, then the hashes level by level over the dependency DAG: every
//       change whose deps are hashed gets its sorted deps hashes, SHA-256 and checksum in the same
//       round (a linear history is one change per round; concurrent branches hash side by side);
//       then the heads check
// Errors carry the RangeError kind and arguments (HistResult); the host formats the text.
// Included by am_kernels.hip after the document kernels (uses parse_doc_hdr, ColDec, SHA-256).
#include "am_hist.h"

struct HChgD {          // change row (DOCUMENT_COLUMNS)
  int64_t seq, max_op, time, extra_tag;
  uint64_t msg_off, extra_off;  // arena offsets
  uint32_t actor, msg_len, ndeps, deps_off;
  uint32_t extra_len, op_begin, op_count, pred_count;
  uint64_t slot, slot_cap;      // output slot within the document's region, its bytes
  uint32_t body_at, body_len;   // body start within the slot, its length
  uint32_t deps_at, chunk_at;   // deps hashes position in the body, chunk start within the slot
};
struct HOpD {           // reconstructed op
  int64_t id_ctr, obj_ctr, elem_ctr, val_tag;
  int32_t id_actor, obj_actor, elem_actor, chg;
  uint64_t key_off, val_off;    // arena offsets (a re-created del: val_off = its creating succ entry)
  uint32_t key_len, val_len;    // key_len AM_NOSTR: list op (elem)
  uint32_t pred_begin, pred_count;
  uint8_t insert, is_del, pad0, pad1;
  uint32_t action;
};
struct HSucc {          // one succ entry of the document (a pred of the op it names)
  int64_t ctr;
  int32_t actor, owner;  // owner: doc row
  int32_t target;        // op index (row, or a re-created del)
  uint32_t pad;
};
static_assert(sizeof(HChgD) == AM_SZ_HCHG && sizeof(HOpD) == AM_SZ_HOP && sizeof(HSucc) == AM_SZ_HSUCC, "history records");

#ifdef __HIPCC__
namespace hist {

struct HKey { int64_t ctr; int32_t actor; int32_t row; };
struct HOrd { int64_t k0; int64_t k1; };

// decode type of each op column (DOC_OPS_COLUMNS, columnar.js:77-94)
__device__ __constant__ static const uint8_t kColDec[OC_NCOLS] = {
    DT_UINT, DT_UINT, DT_UINT, DT_DELTA, DT_UTF8, DT_UINT, DT_DELTA, DT_BOOL,
    DT_UINT, DT_UINT, DT_UINT, DT_UINT, DT_DELTA, DT_UINT, DT_UINT, DT_DELTA};

__device__ __forceinline__ void hfail(HistResult& r, uint32_t kind, int64_t a0 = 0, int64_t a1 = 0, int64_t a2 = 0, int64_t a3 = 0) {
  if (atomicCAS(&r.status, 0u, kind) == 0u) { r.a0 = a0; r.a1 = a1; r.a2 = a2; r.a3 = a3; }
}

// RLEEncoder state machine (encoding.js:558-783), one lane per change: uint, int (the caller
// passes deltas) or utf8 values (off << 20 | len into the arena); AM_NULL64 = null
struct REnc {
  uint8_t* o;
  uint32_t n;        // bytes written
  uint8_t kind;      // 0 uint, 1 int, 2 utf8
  uint8_t state;     // 0 empty, 1 lone value, 2 repetition, 3 literal, 4 nulls
  int64_t last;
  uint32_t cnt;      // repetition / null count, literal length (values in lit[])
  const uint8_t* A;
  int64_t* lit;
};
__device__ __forceinline__ void re_put_val(REnc& e, int64_t v) {
  if (e.kind == 0) e.n += (uint32_t)(put_uleb(e.o + e.n, (uint64_t)v) - (e.o + e.n));
  else if (e.kind == 1) e.n += (uint32_t)(put_sleb(e.o + e.n, v) - (e.o + e.n));
  else {
    const uint32_t len = (uint32_t)(v & 0xfffff);
    const uint64_t off = (uint64_t)v >> 20;
    e.n += (uint32_t)(put_uleb(e.o + e.n, len) - (e.o + e.n));
    for (uint32_t q = 0; q < len; q++) e.o[e.n + q] = e.A[off + q];
    e.n += len;
  }
}
__device__ __forceinline__ bool re_eq(const REnc& e, int64_t a, int64_t b) {
  if (e.kind != 2) return a == b;
  const uint32_t la = (uint32_t)(a & 0xfffff), lb = (uint32_t)(b & 0xfffff);
  if (la != lb) return false;
  const uint64_t oa = (uint64_t)a >> 20, ob = (uint64_t)b >> 20;
  for (uint32_t q = 0; q < la; q++) if (e.A[oa + q] != e.A[ob + q]) return false;
  return true;
}
__device__ __forceinline__ void re_flush(REnc& e) {
  if (e.state == 1) { e.n += (uint32_t)(put_sleb(e.o + e.n, -1) - (e.o + e.n)); re_put_val(e, e.last); }
  else if (e.state == 2) { e.n += (uint32_t)(put_sleb(e.o + e.n, (int64_t)e.cnt) - (e.o + e.n)); re_put_val(e, e.last); }
  else if (e.state == 3) {
    e.n += (uint32_t)(put_sleb(e.o + e.n, -(int64_t)e.cnt) - (e.o + e.n));
    for (uint32_t q = 0; q < e.cnt; q++) re_put_val(e, e.lit[q]);
  } else if (e.state == 4) {
    e.o[e.n++] = 0;
    e.n += (uint32_t)(put_uleb(e.o + e.n, e.cnt) - (e.o + e.n));
  }
  e.state = 0;
}
__device__ static void re_append(REnc& e, int64_t v) {
  const bool nul = v == AM_NULL64;
  if (e.state == 0) {
    if (nul) { e.state = 4; e.cnt = 1; } else { e.state = 1; e.last = v; }
  } else if (e.state == 1) {
    if (nul) { re_flush(e); e.state = 4; e.cnt = 1; }
    else if (re_eq(e, v, e.last)) { e.state = 2; e.cnt = 2; }
    else { e.state = 3; e.lit[0] = e.last; e.cnt = 1; e.last = v; }
  } else if (e.state == 2) {
    if (nul) { re_flush(e); e.state = 4; e.cnt = 1; }
    else if (re_eq(e, v, e.last)) e.cnt++;
    else { re_flush(e); e.state = 1; e.last = v; }
  } else if (e.state == 3) {
    if (nul) { e.lit[e.cnt++] = e.last; re_flush(e); e.state = 4; e.cnt = 1; }
    else if (re_eq(e, v, e.last)) { re_flush(e); e.state = 2; e.cnt = 2; }  // the literal ends before the run
    else { e.lit[e.cnt++] = e.last; e.last = v; }
  } else {
    if (nul) e.cnt++;
    else { re_flush(e); e.state = 1; e.last = v; }
  }
}
// finish (encoding.js:778-782): a literal keeps its pending last value; an all-null column is empty
__device__ __forceinline__ uint32_t re_finish(REnc& e) {
  if (e.state == 3) e.lit[e.cnt++] = e.last;
  if (e.state != 4 || e.n > 0) re_flush(e);
  return e.n;
}

// first (smallest key) error of a lane-parallel check
__device__ __forceinline__ void first_err(unsigned long long* key, uint64_t k) { atomicMin(key, (unsigned long long)k); }

__device__ static void hist_doc(const uint8_t* A, const am_chunk_desc& cd, const ChunkInfo& ci, const HistLayout& L,
                                uint8_t* ws, uint8_t* out, uint64_t out_cap, HistResult& R, HistChange* chout) {
  const uint32_t t = threadIdx.x, B = blockDim.x;
  __shared__ DocHdr dh;
  __shared__ uint32_t sh_ok, sh_nops, sh_prog[2];
  __shared__ unsigned long long sh_key;
  __shared__ uint32_t sh_code[OC_NCOLS + DC_NCOLS];
  __shared__ uint32_t stmp[65];
  const uint64_t NO = ci.nops, NS = ci.nents, NC = ci.nchg, ND = ci.ndeps, NA = ci.nactors;
  int64_t* C = reinterpret_cast<int64_t*>(ws + L.cells);  // [13][NO] row cells, then [2][NS] succ entries
  HChgD* chg = reinterpret_cast<HChgD*>(ws + L.chg);
  int64_t* depsv = reinterpret_cast<int64_t*>(ws + L.deps);
  HOpD* ops = reinterpret_cast<HOpD*>(ws + L.ops);
  HKey* idk = reinterpret_cast<HKey*>(ws + L.idk);
  HSucc* se = reinterpret_cast<HSucc*>(ws + L.sent);
  HOrd* ord = reinterpret_cast<HOrd*>(ws + L.ord);
  HOrd* pord = reinterpret_cast<HOrd*>(ws + L.pord);
  HOrd* ac = reinterpret_cast<HOrd*>(ws + L.actchg);
  uint64_t* aoff = reinterpret_cast<uint64_t*>(ws + L.aoff);
  uint32_t* alen = reinterpret_cast<uint32_t*>(ws + L.alen);
  uint32_t* arank = reinterpret_cast<uint32_t*>(ws + L.arank);
  uint64_t* slot = reinterpret_cast<uint64_t*>(ws + L.slot);
  uint32_t* stamp = reinterpret_cast<uint32_t*>(ws + L.mark);

  // ---- P1: header, actor table ----
  if (t == 0) {
    sh_ok = 1;
    if (ci.status) { hfail(R, HE_CODE, ci.status, ci.arg0); sh_ok = 0; }
    else if (ci.type != 0) { hfail(R, HE_CODE, AM_E_CHUNK_TYPE, ci.type); sh_ok = 0; }
    else {
      const uint32_t e = parse_doc_hdr(A + cd.off + ci.data_off, ci.data_len, cd.off + ci.data_off, dh);
      if (e) { hfail(R, HE_CODE, e); sh_ok = 0; }
      else if (dh.nunk) { hfail(R, HE_CODE, AM_U_UNKNOWN_COLUMN); sh_ok = 0; }
      else if (dh.ocol_len[OC_CHLD_ACTOR] || dh.ocol_len[OC_CHLD_CTR]) { hfail(R, HE_CODE, AM_U_VALUE); sh_ok = 0; }
      else if (NA > 0xffff || NO >= (1ull << 31) || NS >= (1ull << 31)) { hfail(R, HE_CODE, AM_U_VALUE); sh_ok = 0; }
      else {
        Rd r{A + dh.base + dh.actors_off, (uint64_t)1 << 40, 0};
        for (uint32_t i = 0; i < NA; i++) {
          int64_t l;
          rd_u53(r, l);
          aoff[i] = dh.base + dh.actors_off + r.off;
          alen[i] = (uint32_t)l;
          r.off += (uint64_t)l;
        }
      }
    }
    sh_key = ~0ull;
  }
  __syncthreads();
  if (!sh_ok) return;
  for (uint32_t i = t; i < NA; i += B) {
    uint32_t rk = 0;
    for (uint32_t j = 0; j < NA; j++) rk += actor_cmp_dev(A + aoff[j], alen[j], A + aoff[i], alen[i]) < 0;
    arank[i] = rk;
  }
  // ---- P2: columns (lane per column). decodeColumns reads row by row, changes first
  // (columnar.js:1042-1043): the error with the smallest (section, row, column) wins ----
  for (uint32_t col = t; col < OC_NCOLS + DC_NCOLS; col += B) {
    if (col < OC_NCOLS) {
      if (col == OC_VAL_RAW || col == OC_CHLD_ACTOR || col == OC_CHLD_CTR) continue;
      const uint32_t j = col < OC_VAL_RAW ? col : col - 3;  // cells slot: 0..9, then succNum 10 -> 12 below
      const uint32_t slotj = col == OC_GRP_NUM ? 12 : j;
      const uint64_t n = col < OC_GRP_ACTOR ? NO : NS;
      int64_t* dst = col < OC_GRP_ACTOR ? C + (uint64_t)slotj * NO : C + 13 * NO + (uint64_t)(col - OC_GRP_ACTOR) * NS;
      const uint8_t dt = kColDec[col];
      const uint64_t off = dh.base + dh.ocol_off[col];
      ColDec d;
      cd_init(d, dt, A + off, dh.ocol_len[col]);
      for (uint64_t i = 0; i < n; i++) {
        int64_t v;
        uint32_t e;
        if (dt == DT_BOOL) { bool b; e = cd_next_bool(d, b); v = b; }
        else {
          bool isnull;
          uint32_t l;
          int64_t x;
          e = cd_next(d, x, isnull, l);
          if (isnull) v = AM_NULL64;
          else if (dt == DT_UTF8) { v = (int64_t)((off + (uint64_t)x) << 20) | (int64_t)l; if (!e && l >= (1u << 20)) e = AM_U_VALUE; }
          else if (dt == DT_DELTA) v = (d.absolute += x);
          else v = x;
        }
        if (e) {
          sh_code[col] = e;
          // succ entries belong to rows; order them after the row fields (approximately row-major)
          first_err(&sh_key, (1ull << 62) | ((uint64_t)(col < OC_GRP_ACTOR ? i : NO) << 8) | col);
          break;
        }
        dst[i] = v;
      }
    } else {
      const uint32_t dc = col - OC_NCOLS;
      if (dc == DC_EXTRA_RAW) continue;
      const uint64_t off = dh.base + dh.ccol_off[dc];
      const uint8_t dt = (dc == DC_ACTOR || dc == DC_DEPS_NUM || dc == DC_EXTRA_LEN) ? DT_UINT : dc == DC_MESSAGE ? DT_UTF8 : DT_DELTA;
      ColDec d;
      cd_init(d, dt, A + off, dh.ccol_len[dc]);
      const uint64_t n = dc == DC_DEPS_INDEX ? ND : NC;
      for (uint64_t i = 0; i < n; i++) {
        bool isnull;
        uint32_t l;
        int64_t x, v;
        const uint32_t e = cd_next(d, x, isnull, l);
        if (e) {
          sh_code[col] = e;
          first_err(&sh_key, ((uint64_t)(dc == DC_DEPS_INDEX ? NC : i) << 8) | col);
          break;
        }
        if (isnull) v = AM_NULL64;
        else if (dt == DT_DELTA) v = (d.absolute += x);
        else v = x;
        if (dc == DC_DEPS_INDEX) { depsv[i] = v; continue; }
        HChgD& c = chg[i];
        switch (dc) {
          case DC_ACTOR: c.actor = (v == AM_NULL64 || v < 0 || v >= (int64_t)NA) ? 0xffffffffu : (uint32_t)v; break;
          case DC_SEQ: c.seq = v; break;
          case DC_MAXOP: c.max_op = v; break;
          case DC_TIME: c.time = v == AM_NULL64 ? 0 : v; break;
          case DC_MESSAGE: c.msg_off = isnull ? 0 : off + (uint64_t)x; c.msg_len = isnull ? 0 : l; break;
          case DC_DEPS_NUM: c.ndeps = (v == AM_NULL64 || v < 0) ? 0 : (uint32_t)v; break;
          default: c.extra_tag = v; break;  // DC_EXTRA_LEN
        }
      }
    }
  }
  __syncthreads();
  if (t == 0 && sh_key != ~0ull) hfail(R, HE_CODE, sh_code[sh_key & 0xff]);
  __syncthreads();
  if (R.status) return;
  // ---- P3: op records, decode-phase row checks; raw value offsets and succ entry starts ----
  uint32_t* tmpa = reinterpret_cast<uint32_t*>(ws + L.idk);  // 2 x NO u32 (idk is filled in P4)
  uint32_t* tmpb = tmpa + NO;
  for (uint64_t i = t; i < NO; i += B) {
    const int64_t* c = C + i;
    HOpD o;
    o.obj_actor = c[0] == AM_NULL64 ? -1 : (int32_t)c[0];
    o.obj_ctr = c[NO] == AM_NULL64 ? 0 : c[NO];
    o.elem_actor = c[2 * NO] == AM_NULL64 ? -1 : (int32_t)c[2 * NO];
    o.elem_ctr = c[3 * NO] == AM_NULL64 ? 0 : c[3 * NO];
    const int64_t ks = c[4 * NO];
    o.key_len = ks == AM_NULL64 ? AM_NOSTR : (uint32_t)(ks & 0xfffff);
    o.key_off = ks == AM_NULL64 ? 0 : (uint64_t)ks >> 20;
    o.id_actor = c[5 * NO] == AM_NULL64 ? -1 : (int32_t)c[5 * NO];
    o.id_ctr = c[6 * NO];
    o.insert = c[7 * NO] != 0;
    const int64_t act = c[8 * NO];
    o.action = act == AM_NULL64 ? 0xffffffffu : (uint32_t)act;
    o.val_tag = c[9 * NO] == AM_NULL64 ? 0 : c[9 * NO];
    o.val_len = (uint32_t)((uint64_t)o.val_tag >> 4);
    o.is_del = 0; o.chg = -1; o.pred_begin = 0; o.pred_count = 0; o.pad0 = o.pad1 = 0; o.val_off = 0;
    const int64_t sn = c[12 * NO];
    uint32_t e = 0;
    if (o.id_ctr == AM_NULL64 || c[5 * NO] == AM_NULL64 || c[5 * NO] < 0 || c[5 * NO] >= (int64_t)NA || act == AM_NULL64 ||
        (sn != AM_NULL64 && sn < 0) || (c[0] != AM_NULL64 && c[0] < 0) || (c[2 * NO] != AM_NULL64 && c[2 * NO] < 0))
      e = AM_U_VALUE;
    else if (o.obj_actor >= (int32_t)NA) e = AM_E_NO_ACTOR_INDEX;
    else if (o.key_len == AM_NOSTR && o.elem_actor >= (int32_t)NA) e = AM_E_NO_ACTOR_INDEX;
    if (e) first_err(&sh_key, (i << 8) | e);
    ops[i] = o;
    tmpa[i] = o.val_len;
    tmpb[i] = sn == AM_NULL64 ? 0u : (uint32_t)sn;
  }
  __syncthreads();
  if (t == 0 && sh_key != ~0ull) {
    const uint32_t e = (uint32_t)(sh_key & 0xff);
    const HOpD& o = ops[sh_key >> 8];
    hfail(R, HE_CODE, e, e == AM_E_NO_ACTOR_INDEX ? (o.obj_actor >= (int32_t)NA ? o.obj_actor : o.elem_actor) : 0);
  }
  __syncthreads();
  if (R.status) return;
  const uint32_t vtot = block_excl_scan(tmpa, (uint32_t)NO, stmp);
  const uint32_t stot = block_excl_scan(tmpb, (uint32_t)NO, stmp);
  if (t == 0) {
    if (vtot > dh.ocol_len[OC_VAL_RAW]) hfail(R, HE_CODE, AM_E_SUBARRAY);
    else if (stot != NS) hfail(R, HE_CODE, AM_U_VALUE);
  }
  __syncthreads();
  if (R.status) return;
  const uint64_t vr = dh.base + dh.ocol_off[OC_VAL_RAW];
  for (uint64_t i = t; i < NO; i += B) {
    ops[i].val_off = vr + tmpa[i];
    const uint32_t n = (i + 1 < NO ? tmpb[i + 1] : stot) - tmpb[i];
    for (uint32_t q = 0; q < n; q++) {
      const uint64_t k = tmpb[i] + q;
      const int64_t a = C[13 * NO + k], ctr = C[13 * NO + NS + k];
      if (a == AM_NULL64 || a < 0 || a >= (int64_t)NA || ctr == AM_NULL64) hfail(R, HE_CODE, AM_U_VALUE);
      se[k].ctr = ctr; se[k].actor = (int32_t)a; se[k].owner = (int32_t)i; se[k].target = -1; se[k].pad = 0;
    }
  }
  __syncthreads();
  if (R.status) return;
  // ---- P4: row id index, succ targets, re-created deletions ----
  const uint32_t PO = (uint32_t)hist_pow2(NO ? NO : 1);
  for (uint32_t i = t; i < PO; i += B) {
    HKey k;
    if (i < NO) { k.ctr = ops[i].id_ctr; k.actor = ops[i].id_actor; k.row = (int32_t)i; }
    else { k.ctr = INT64_MAX; k.actor = INT32_MAX; k.row = INT32_MAX; }
    idk[i] = k;
  }
  __syncthreads();
  block_bitonic_sort(idk, PO, [](const HKey& a, const HKey& b) {
    if (a.ctr != b.ctr) return a.ctr < b.ctr;
    if (a.actor != b.actor) return a.actor < b.actor;
    return a.row < b.row;
  });
  for (uint64_t k = t; k < NS; k += B) {
    uint32_t lo = 0, hi = (uint32_t)NO;
    while (lo < hi) {
      const uint32_t m = (lo + hi) >> 1;
      if (idk[m].ctr < se[k].ctr || (idk[m].ctr == se[k].ctr && idk[m].actor < se[k].actor)) lo = m + 1; else hi = m;
    }
    // a repeated id: the row first in document order (all rows of one id share one pred list in
    // groupChangeOps; such a change fails the opId check below whichever row holds it)
    se[k].target = (lo < NO && idk[lo].ctr == se[k].ctr && idk[lo].actor == se[k].actor) ? idk[lo].row : -1;
  }
  __syncthreads();
  // entries naming no row, by (id, entry): each id becomes one del, after the rows
  const uint32_t PS = (uint32_t)hist_pow2(NS ? NS : 1);
  for (uint32_t i = t; i < PS; i += B) {
    if (i < NS && se[i].target < 0) { ord[i].k0 = se[i].ctr; ord[i].k1 = ((int64_t)se[i].actor << 32) | (int64_t)i; }
    else { ord[i].k0 = INT64_MAX; ord[i].k1 = INT64_MAX; }
  }
  __syncthreads();
  block_bitonic_sort(ord, PS, [](const HOrd& a, const HOrd& b) {
    if (a.k0 != b.k0) return a.k0 < b.k0;
    return a.k1 < b.k1;
  });
  // group starts -> del index by a scan of the start flags
  uint32_t* dstart = reinterpret_cast<uint32_t*>(ws + L.pord);  // PS u32 (pord is filled in P5)
  for (uint32_t i = t; i < NS; i += B)
    dstart[i] = ord[i].k0 != INT64_MAX && (i == 0 || ord[i].k0 != ord[i - 1].k0 || (ord[i].k1 >> 32) != (ord[i - 1].k1 >> 32));
  __syncthreads();
  const uint32_t ndel = block_excl_scan(dstart, (uint32_t)NS, stmp);
  for (uint32_t i = t; i < NS; i += B) {
    if (ord[i].k0 == INT64_MAX) continue;
    const uint32_t e = (uint32_t)(ord[i].k1 & 0xffffffff);
    const bool start = (i + 1 < NS ? dstart[i + 1] : ndel) != dstart[i];
    const uint32_t di = start ? dstart[i] : dstart[i] - 1;  // exclusive scan: a start owns index dstart[i]
    se[e].target = (int32_t)(NO + di);
    if (start) {
      // the deletion groupChangeOps re-creates: obj / key of the first op that names it
      const HOpD& ow = ops[se[e].owner];
      HOpD d = ow;
      d.id_ctr = se[e].ctr;
      d.id_actor = se[e].actor;
      if (ow.key_len == AM_NOSTR) {
        d.elem_ctr = ow.insert ? ow.id_ctr : ow.elem_ctr;
        d.elem_actor = ow.insert ? ow.id_actor : ow.elem_actor;
      }
      d.insert = 0; d.action = 3; d.val_tag = 0; d.val_len = 0;
      d.val_off = e;  // creation order (Object.values(opsById), columnar.js:906-908)
      d.is_del = 1; d.chg = -1; d.pred_begin = 0; d.pred_count = 0;
      ops[NO + di] = d;
    }
  }
  if (t == 0) sh_nops = (uint32_t)(NO + ndel);
  __syncthreads();
  const uint32_t NOPS = sh_nops;
  // ---- P5: pred lists sorted by (target, counter, actor rank) = compareParsedOpIds ----
  for (uint32_t i = t; i < PS; i += B) {
    if (i < NS) {
      const HSucc& sc = se[i];
      const HOpD& ow = ops[sc.owner];
      pord[i].k0 = ((int64_t)sc.target << 32) | (int64_t)i;
      pord[i].k1 = ((int64_t)ow.id_ctr << 16) | (int64_t)arank[ow.id_actor];
    } else {
      pord[i].k0 = INT64_MAX;
      pord[i].k1 = INT64_MAX;
    }
  }
  __syncthreads();
  block_bitonic_sort(pord, PS, [](const HOrd& a, const HOrd& b) {
    if ((a.k0 >> 32) != (b.k0 >> 32)) return (a.k0 >> 32) < (b.k0 >> 32);
    if (a.k1 != b.k1) return a.k1 < b.k1;
    return a.k0 < b.k0;
  });
  for (uint32_t i = t; i < NS; i += B) {
    const int64_t tg = pord[i].k0 >> 32;
    if (i == 0 || (pord[i - 1].k0 >> 32) != tg) {
      uint32_t n = 1;
      while (i + n < NS && (pord[i + n].k0 >> 32) == tg) n++;
      ops[tg].pred_begin = i;
      ops[tg].pred_count = n;
    }
  }
  __syncthreads();
  // ---- P6: change rows. Decode checks, then groupChangeOps' seq / maxOp rules (:877-888) ----
  uint32_t* cda = reinterpret_cast<uint32_t*>(ws + L.slot);  // 2 x NC u32: deps / extra offsets
  uint32_t* cdb = cda + NC;
  for (uint64_t i = t; i < NC; i += B) {
    const HChgD& c = chg[i];
    if (c.actor == 0xffffffffu || c.seq == AM_NULL64 || c.max_op == AM_NULL64) first_err(&sh_key, i);
    cda[i] = c.ndeps;
    cdb[i] = c.extra_tag == AM_NULL64 ? 0u : (uint32_t)((uint64_t)c.extra_tag >> 4);
  }
  __syncthreads();
  const uint32_t dtot = block_excl_scan(cda, (uint32_t)NC, stmp);
  const uint32_t etot = block_excl_scan(cdb, (uint32_t)NC, stmp);
  if (t == 0) {
    if (sh_key != ~0ull || dtot > ND) hfail(R, HE_CODE, AM_U_VALUE);
    else if (etot > dh.ccol_len[DC_EXTRA_RAW]) hfail(R, HE_CODE, AM_E_SUBARRAY);
  }
  __syncthreads();
  if (R.status) return;
  const uint64_t er = dh.base + dh.ccol_off[DC_EXTRA_RAW];
  const uint32_t PC = (uint32_t)hist_pow2(NC ? NC : 1);
  for (uint32_t i = t; i < PC; i += B) {
    if (i < NC) {
      HChgD& c = chg[i];
      c.deps_off = cda[i];
      c.extra_off = er + cdb[i];
      c.extra_len = (uint32_t)(c.extra_tag == AM_NULL64 ? 0 : ((uint64_t)c.extra_tag >> 4));
      c.op_begin = 0; c.op_count = 0; c.pred_count = 0;
      ac[i].k0 = ((int64_t)c.actor << 32) | (int64_t)i;
      ac[i].k1 = (int64_t)i;
    } else {
      ac[i].k0 = INT64_MAX; ac[i].k1 = INT64_MAX;
    }
  }
  __syncthreads();
  // changes of each actor in document order: while every earlier change passed, a change's count
  // of earlier same-actor changes is its rank in its actor's group, so the first change (document
  // order) breaking seq = rank + 1 or the maxOp order is the one the sequential loop reports
  block_bitonic_sort(ac, PC, [](const HOrd& a, const HOrd& b) { return a.k0 < b.k0; });
  if (t == 0) sh_key = ~0ull;
  __syncthreads();
  for (uint32_t p = t; p < NC; p += B) {
    const uint32_t i = (uint32_t)ac[p].k1, a = chg[i].actor;
    uint32_t lo = 0, hi = p;  // first entry of the actor
    while (lo < hi) { const uint32_t m = (lo + hi) >> 1; if ((uint32_t)(ac[m].k0 >> 32) < a) lo = m + 1; else hi = m; }
    const int64_t rank = p - lo;
    const HChgD& c = chg[i];
    if (c.seq != rank + 1) first_err(&sh_key, ((uint64_t)i << 8) | HE_SEQ);
    else if (c.seq > 1 && chg[ac[p - 1].k1].max_op > c.max_op) first_err(&sh_key, ((uint64_t)i << 8) | HE_MAXOP);
  }
  __syncthreads();
  if (t == 0 && sh_key != ~0ull) {
    const uint32_t i = (uint32_t)(sh_key >> 8);
    if ((sh_key & 0xff) == HE_SEQ) {
      uint32_t p = 0;
      while ((uint32_t)ac[p].k1 != i) p++;
      uint32_t lo = p;
      while (lo > 0 && (uint32_t)(ac[lo - 1].k0 >> 32) == chg[i].actor) lo--;
      hfail(R, HE_SEQ, (int64_t)(p - lo) + 1, chg[i].seq);
    } else {
      hfail(R, HE_MAXOP);
    }
  }
  if (t == 0) sh_key = ~0ull;
  __syncthreads();
  if (R.status) return;
  // the ops loop (:889-905): a del among the rows
  for (uint64_t i = t; i < NO; i += B)
    if (ops[i].action == 3) first_err(&sh_key, i);
  __syncthreads();
  if (t == 0 && sh_key != ~0ull) hfail(R, HE_DEL);
  if (t == 0) sh_key = ~0ull;
  __syncthreads();
  if (R.status) return;
  // op -> its change: the first change of its actor with maxOp >= the op's counter (:910-925)
  for (uint32_t k = t; k < NOPS; k += B) {
    HOpD& o = ops[k];
    uint32_t lo = 0, hi = (uint32_t)NC;
    const int64_t key0 = (int64_t)o.id_actor << 32;
    while (lo < hi) {
      const uint32_t m = (lo + hi) >> 1;
      if (ac[m].k0 < key0) lo = m + 1; else hi = m;
    }
    uint32_t a_hi = lo, h = (uint32_t)NC;
    while (a_hi < h) {  // end of the actor's entries
      const uint32_t m = (a_hi + h) >> 1;
      if ((ac[m].k0 >> 32) <= o.id_actor) a_hi = m + 1; else h = m;
    }
    uint32_t l2 = lo, h2 = a_hi;
    while (l2 < h2) {
      const uint32_t m = (l2 + h2) >> 1;
      if (chg[ac[m].k1].max_op < o.id_ctr) l2 = m + 1; else h2 = m;
    }
    o.chg = l2 < a_hi ? (int32_t)ac[l2].k1 : -1;
    // the first op outside its actor's range: rows in document order, then the deletions in
    // creation order
    if (o.chg < 0) first_err(&sh_key, k < NO ? (uint64_t)k : (1ull << 40) + o.val_off);
  }
  __syncthreads();
  if (t == 0 && sh_key != ~0ull) {
    uint32_t k = 0;
    if (sh_key < (1ull << 40)) k = (uint32_t)sh_key;
    else for (k = (uint32_t)NO; k < NOPS && !(ops[k].chg < 0 && ops[k].val_off == sh_key - (1ull << 40)); k++) {}
    hfail(R, HE_RANGE, ops[k].id_ctr, ops[k].id_actor);
  }
  if (t == 0) sh_key = ~0ull;
  __syncthreads();
  if (R.status) return;
  // ---- P7: ops by (change, counter); opId contiguity (:929-940) ----
  const uint32_t PP = (uint32_t)hist_pow2(NOPS ? NOPS : 1);
  for (uint32_t i = t; i < PP; i += B) {
    if (i < NOPS) { ord[i].k0 = ((int64_t)ops[i].chg << 40) | (int64_t)i; ord[i].k1 = ops[i].id_ctr; }
    else { ord[i].k0 = INT64_MAX; ord[i].k1 = INT64_MAX; }
  }
  __syncthreads();
  block_bitonic_sort(ord, PP, [](const HOrd& a, const HOrd& b) {
    if ((a.k0 >> 40) != (b.k0 >> 40)) return (a.k0 >> 40) < (b.k0 >> 40);
    if (a.k1 != b.k1) return a.k1 < b.k1;
    return a.k0 < b.k0;
  });
  for (uint32_t i = t; i < NOPS; i += B) {
    const int64_t c = ord[i].k0 >> 40;
    if (i == 0 || (ord[i - 1].k0 >> 40) != c) {
      uint32_t n = 1;
      while (i + n < NOPS && (ord[i + n].k0 >> 40) == c) n++;
      chg[c].op_begin = i;
      chg[c].op_count = n;
    }
  }
  __syncthreads();
#define HOP(q) ops[ord[(q)].k0 & 0xffffffffffll]
#define HPRED_OWNER(p) ops[se[pord[(p)].k0 & 0xffffffff].owner]
  // ---- P8: lane per change: opId check, slot size ----
  for (uint64_t i = t; i < NC; i += B) {
    HChgD& c = chg[i];
    const int64_t start = c.max_op - (int64_t)c.op_count + 1;
    uint64_t np = 0, vb = 0, kb = 0, refb = alen[c.actor] + 5;
    for (uint32_t q = 0; q < c.op_count; q++) {
      const HOpD& o = HOP(c.op_begin + q);
      if (o.id_ctr != start + (int64_t)q || o.id_actor != (int32_t)c.actor) {
        first_err(&sh_key, (i << 24) | q);
        break;
      }
      np += o.pred_count;
      vb += o.val_len;
      if (o.key_len != AM_NOSTR) kb += o.key_len;
      if (o.obj_actor >= 0) refb += alen[o.obj_actor] + 5;
      if (o.key_len == AM_NOSTR && o.elem_actor >= 0) refb += alen[o.elem_actor] + 5;
      for (uint32_t p = 0; p < o.pred_count; p++) refb += alen[HPRED_OWNER(o.pred_begin + p).id_actor] + 5;
    }
    c.pred_count = (uint32_t)np;
    slot[i] = hist_slot_bound(c.op_count, np, c.ndeps, vb, kb, c.msg_len, c.extra_len, refb);
  }
  __syncthreads();
  if (t == 0 && sh_key != ~0ull) {
    const HChgD& c = chg[sh_key >> 24];
    const uint32_t q = (uint32_t)(sh_key & 0xffffff);
    const HOpD& o = HOP(c.op_begin + q);
    hfail(R, HE_OPID, c.max_op - (int64_t)c.op_count + 1 + q, c.actor, o.id_ctr, o.id_actor);
  }
  __syncthreads();
  if (R.status) return;
  // slots: exclusive scan of the bounds (u64, lane 0 over the 64 partial sums)
  {
    const uint64_t per = (NC + B - 1) / B, b0 = t * per, b1 = b0 + per < NC ? b0 + per : NC;
    uint64_t acc = 0;
    for (uint64_t i = b0; i < b1; i++) acc += slot[i];
    __shared__ uint64_t part[65];
    part[t] = acc;
    __syncthreads();
    if (t == 0) {
      uint64_t run = 0;
      for (uint32_t k = 0; k < B; k++) { const uint64_t x = part[k]; part[k] = run; run += x; }
      part[B] = run;
      if (run > out_cap) hfail(R, HE_CODE, AM_U_CAPACITY, (int64_t)run);
    }
    __syncthreads();
    uint64_t run = part[t];
    for (uint64_t i = b0; i < b1; i++) { chg[i].slot = run; chg[i].slot_cap = slot[i]; run += slot[i]; }
  }
  __syncthreads();
  if (R.status) return;
  // ---- P8b: lane per change: the encodeChange body (columnar.js:710-739) ----
  for (uint64_t i = t; i < NC; i += B) {
    HChgD& c = chg[i];
    uint8_t* S0 = out + c.slot;
    uint8_t* b = S0 + 16;  // body; the container header goes right before it
    uint32_t n = 0;
    // scratch at the slot's tail: literal values, then the change's other actors
    const uint64_t scr = (8ull * (c.op_count + c.pred_count + 2) + 4ull * (2 * c.op_count + c.pred_count + 2) + 15) & ~7ull;
    int64_t* lit = reinterpret_cast<int64_t*>(S0 + c.slot_cap - scr);
    int32_t* oth = reinterpret_cast<int32_t*>(lit + c.op_count + c.pred_count + 2);
    // other actors referenced by the change's ops, in string order (parseAllOpIds, :139-170)
    uint32_t no = 0;
    auto add = [&](int32_t a) {
      if (a < 0 || a == (int32_t)c.actor) return;
      for (uint32_t q = 0; q < no; q++) if (oth[q] == a) return;
      oth[no++] = a;
    };
    for (uint32_t q = 0; q < c.op_count; q++) {
      const HOpD& o = HOP(c.op_begin + q);
      add(o.obj_actor);
      if (o.key_len == AM_NOSTR) add(o.elem_actor);
      for (uint32_t p = 0; p < o.pred_count; p++) add(HPRED_OWNER(o.pred_begin + p).id_actor);
    }
    for (uint32_t x = 1; x < no; x++)
      for (uint32_t y = x; y > 0 && arank[oth[y]] < arank[oth[y - 1]]; y--) {
        const int32_t tt = oth[y]; oth[y] = oth[y - 1]; oth[y - 1] = tt;
      }
    auto num = [&](int32_t a) -> int64_t {
      if (a == (int32_t)c.actor) return 0;
      for (uint32_t q = 0; q < no; q++) if (oth[q] == a) return 1 + q;
      return 0;
    };
    // header: deps (hashes filled in P9), actor, seq, startOp, time, message, other actors
    n += (uint32_t)(put_uleb(b + n, c.ndeps) - (b + n));
    c.deps_at = n;
    n += 32 * c.ndeps;
    n += (uint32_t)(put_uleb(b + n, alen[c.actor]) - (b + n));
    for (uint32_t q = 0; q < alen[c.actor]; q++) b[n + q] = A[aoff[c.actor] + q];
    n += alen[c.actor];
    const int64_t start = c.max_op - (int64_t)c.op_count + 1;
    n += (uint32_t)(put_uleb(b + n, (uint64_t)c.seq) - (b + n));
    n += (uint32_t)(put_uleb(b + n, (uint64_t)start) - (b + n));
    n += (uint32_t)(put_sleb(b + n, c.time) - (b + n));
    n += (uint32_t)(put_uleb(b + n, c.msg_len) - (b + n));
    for (uint32_t q = 0; q < c.msg_len; q++) b[n + q] = A[c.msg_off + q];
    n += c.msg_len;
    n += (uint32_t)(put_uleb(b + n, no) - (b + n));
    for (uint32_t x = 0; x < no; x++) {
      n += (uint32_t)(put_uleb(b + n, alen[oth[x]]) - (b + n));
      for (uint32_t q = 0; q < alen[oth[x]]; q++) b[n + q] = A[aoff[oth[x]] + q];
      n += alen[oth[x]];
    }
    // columns (CHANGE_COLUMNS order), encoded after a gap for the column table
    constexpr uint8_t kIds[14] = {0x01, 0x02, 0x11, 0x13, 0x15, 0x34, 0x42, 0x56, 0x57, 0x61, 0x63, 0x70, 0x71, 0x73};
    const uint32_t tab_at = n, data0 = tab_at + 1 + 14 * 6;
    uint32_t cpos = data0;
    uint32_t clen[14];
    for (int k = 0; k < 14; k++) {
      const uint8_t id = kIds[k];
      uint8_t* o = b + cpos;
      uint32_t len = 0;
      if (id == 0x34) {  // insert: boolean runs, starting with false
        bool cur = false;
        uint64_t run = 0;
        for (uint32_t q = 0; q < c.op_count; q++) {
          const bool v = HOP(c.op_begin + q).insert != 0;
          if (v != cur) { len += (uint32_t)(put_uleb(o + len, run) - (o + len)); cur = v; run = 0; }
          run++;
        }
        if (c.op_count) len += (uint32_t)(put_uleb(o + len, run) - (o + len));
      } else if (id == 0x57) {  // valRaw
        for (uint32_t q = 0; q < c.op_count; q++) {
          const HOpD& op = HOP(c.op_begin + q);
          for (uint32_t x = 0; x < op.val_len; x++) o[len + x] = A[op.val_off + x];
          len += op.val_len;
        }
      } else if (id == 0x61 || id == 0x63) {
        len = 0;  // no link ops in a history (P1)
      } else {
        REnc e;
        e.o = o; e.n = 0; e.state = 0; e.cnt = 0; e.last = 0; e.A = A; e.lit = lit;
        e.kind = (id == 0x13 || id == 0x73) ? 1 : id == 0x15 ? 2 : 0;
        int64_t prev = 0;  // DeltaEncoder: the previous non-null value
        auto push = [&](int64_t v) {
          if (e.kind == 1 && v != AM_NULL64) { const int64_t d2 = v - prev; prev = v; v = d2; }
          re_append(e, v);
        };
        for (uint32_t q = 0; q < c.op_count; q++) {
          const HOpD& op = HOP(c.op_begin + q);
          const bool keyed = op.key_len != AM_NOSTR;
          switch (id) {
            case 0x01: push(op.obj_actor < 0 ? AM_NULL64 : num(op.obj_actor)); break;
            case 0x02: push(op.obj_actor < 0 ? AM_NULL64 : op.obj_ctr); break;
            case 0x11: push(keyed || op.elem_actor < 0 ? AM_NULL64 : num(op.elem_actor)); break;
            case 0x13: push(keyed ? AM_NULL64 : (op.elem_actor < 0 ? 0 : op.elem_ctr)); break;
            case 0x15: push(keyed ? (int64_t)((op.key_off << 20) | op.key_len) : AM_NULL64); break;
            case 0x42: push((int64_t)op.action); break;
            case 0x56: push(op.val_tag); break;
            case 0x70: push((int64_t)op.pred_count); break;
            case 0x71:
              for (uint32_t p = 0; p < op.pred_count; p++) push(num(HPRED_OWNER(op.pred_begin + p).id_actor));
              break;
            default:  // 0x73
              for (uint32_t p = 0; p < op.pred_count; p++) push(HPRED_OWNER(op.pred_begin + p).id_ctr);
              break;
          }
        }
        len = re_finish(e);
      }
      clen[k] = len;
      cpos += len;
    }
    // column table, then the columns moved up against it
    uint32_t ne = 0;
    for (int k = 0; k < 14; k++) ne += clen[k] != 0;
    uint32_t tp = tab_at;
    tp += (uint32_t)(put_uleb(b + tp, ne) - (b + tp));
    for (int k = 0; k < 14; k++)
      if (clen[k]) {
        tp += (uint32_t)(put_uleb(b + tp, kIds[k]) - (b + tp));
        tp += (uint32_t)(put_uleb(b + tp, clen[k]) - (b + tp));
      }
    const uint32_t dlen = cpos - data0;
    for (uint32_t q = 0; q < dlen; q++) b[tp + q] = b[data0 + q];
    n = tp + dlen;
    for (uint32_t q = 0; q < c.extra_len; q++) b[n + q] = A[c.extra_off + q];
    n += c.extra_len;
    c.body_len = n;
    // container header right before the body: magic, checksum (P9), type 1, body length
    const uint32_t hl = 9 + (uint32_t)uleb_len(n);
    c.chunk_at = 16 - hl;
    c.body_at = 16;
    uint8_t* h = S0 + c.chunk_at;
    h[0] = 0x85; h[1] = 0x6f; h[2] = 0x4a; h[3] = 0x83;
    h[8] = 1;
    put_uleb(h + 9, n);
    stamp[i] = 0;
  }
#undef HOP
#undef HPRED_OWNER
  __syncthreads();
  // ---- P9: decodeDocumentChanges (:945-981). Per change in order: a deps index with no hash
  // (not an earlier change), then the extra bytes' datatype ----
  for (uint64_t i = t; i < NC; i += B) {
    const HChgD& c = chg[i];
    bool bad = false;
    for (uint32_t k = 0; k < c.ndeps && !bad; k++) {
      const int64_t di = depsv[c.deps_off + k];
      bad = di == AM_NULL64 || di < 0 || (uint64_t)di >= i;
    }
    if (!bad && c.extra_tag != AM_NULL64 && (c.extra_tag & 0x0f) != 7) bad = true;
    if (bad) first_err(&sh_key, i);
  }
  __syncthreads();
  if (t == 0 && sh_key != ~0ull) {
    const uint64_t i = sh_key;
    const HChgD& c = chg[i];
    bool done = false;
    for (uint32_t k = 0; k < c.ndeps && !done; k++) {
      const int64_t di = depsv[c.deps_off + k];
      if (di == AM_NULL64 || di < 0 || (uint64_t)di >= i) { hfail(R, HE_NOHASH, di, (int64_t)i); done = true; }
    }
    if (!done) hfail(R, HE_EXTRA);
  }
  __syncthreads();
  if (R.status) return;
  // hashes, level by level: a change is hashed in the first round after all its deps were
  // (stamp = the round that hashed it; deps stamped in the current round are not ready yet, so a
  // round only reads hashes written before its barrier)
  for (uint32_t round = 1;; round++) {
    const uint32_t par = round & 1;
    if (t == 0) sh_prog[par] = 0;
    __syncthreads();
    for (uint64_t i = t; i < NC; i += B) {
      if (stamp[i]) continue;
      HChgD& c = chg[i];
      bool ready = true;
      for (uint32_t k = 0; k < c.ndeps && ready; k++) {
        const uint32_t s = stamp[depsv[c.deps_off + k]];
        ready = s != 0 && s < round;
      }
      if (!ready) continue;
      uint8_t* dp = out + c.slot + c.body_at + c.deps_at;
      for (uint32_t k = 0; k < c.ndeps; k++) {  // insertion into the sorted list (bytewise = hex order)
        const int64_t di = depsv[c.deps_off + k];
        chout[di].head = 0;
        const uint8_t* hh = chout[di].hash;
        uint32_t pos = k;
        while (pos > 0) {
          int cmp = 0;
          for (int q = 0; q < 32 && cmp == 0; q++) cmp = (int)dp[32 * (pos - 1) + q] - (int)hh[q];
          if (cmp <= 0) break;
          for (int q = 0; q < 32; q++) dp[32 * pos + q] = dp[32 * (pos - 1) + q];
          pos--;
        }
        for (int q = 0; q < 32; q++) dp[32 * pos + q] = hh[q];
      }
      uint8_t* ck = out + c.slot + c.chunk_at;
      uint8_t hash[32];
      sha256_dev(ck + 8, (uint64_t)(c.body_at - c.chunk_at - 8) + c.body_len, hash);
      for (int q = 0; q < 4; q++) ck[4 + q] = hash[q];
      HistChange& hc = chout[i];
      hc.off = c.slot + c.chunk_at;
      hc.len = (c.body_at - c.chunk_at) + c.body_len;
      hc.head = 1;
      for (int q = 0; q < 32; q++) hc.hash[q] = hash[q];
      stamp[i] = round;
      sh_prog[par] = 1;
    }
    __syncthreads();
    if (!sh_prog[par]) break;
  }
  // heads (:973-980): the changes no other change depends on, sorted, against the document's
  if (t == 0) {
    uint32_t nh = 0;
    for (uint64_t i = 0; i < NC; i++)
      if (chout[i].head) {
        uint32_t pos = nh++;
        while (pos > 0) {
          const uint8_t* a = chout[slot[pos - 1]].hash;
          const uint8_t* b = chout[i].hash;
          int cmp = 0;
          for (int q = 0; q < 32 && cmp == 0; q++) cmp = (int)a[q] - (int)b[q];
          if (cmp <= 0) break;
          slot[pos] = slot[pos - 1];
          pos--;
        }
        slot[pos] = i;
      }
    bool ok = nh == dh.nheads;
    for (uint32_t k = 0; k < nh && ok; k++) {
      const uint8_t* want = A + dh.base + dh.heads_off + 32 * k;
      for (int q = 0; q < 32 && ok; q++) ok = chout[slot[k]].hash[q] == want[q];
    }
    if (!ok) hfail(R, HE_HEADS);
    R.nchanges = (uint32_t)NC;
  }
}

}  // namespace hist

__global__ void __launch_bounds__(64) k_history(const uint8_t* __restrict__ arena, const am_chunk_desc* __restrict__ chunks,
                                                const ChunkInfo* __restrict__ info, const HistDesc* __restrict__ hd, uint32_t ndocs,
                                                uint8_t* __restrict__ ws, uint8_t* __restrict__ out, HistResult* __restrict__ res,
                                                HistChange* __restrict__ chg_out) {
  const uint32_t d = blockIdx.x;
  if (d >= ndocs) return;
  __shared__ HistResult R;
  const HistDesc h = hd[d];
  const ChunkInfo ci = info[h.chunk];
  const am_chunk_desc cd = chunks[h.chunk];
  if (threadIdx.x == 0) { R.status = 0; R.nchanges = 0; R.a0 = R.a1 = R.a2 = R.a3 = 0; }
  __syncthreads();
  const HistLayout L = hist_layout(ci.nops, ci.nents, ci.nchg, ci.ndeps, ci.nactors);
  hist::hist_doc(arena, cd, ci, L, ws + h.ws_off, out + h.out_off, h.out_cap, R, chg_out + h.chg_off);
  __syncthreads();
  if (threadIdx.x == 0) res[d] = R;
}
#endif
