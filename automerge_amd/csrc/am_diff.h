// am_diff.h -- the patch Backend.applyChanges returns as a patch log, written by
// lane 0 of k_doc (phase P8) after the parallel merge.
//
// Reference: applyChanges / applyOps / mergeDocChangeOps (new.js:1550-1597, 1304-1380,
// 1052-1290), seekWithinBlock (:50-192), updatePatchProperty (:884-1040), appendEdit /
// appendUpdate / convertInsertToUpdate (:747-869), setupPatches (:1461-1528), and the objectMeta
// that documentPatch leaves at load (:1604-1635, 1748).
//
// The reference merges the applied change ops into the document one applyOps call at a time.
// Here the merged document is already known (document order F from the parallel merge), and every
// intermediate document is F restricted to the rows present at that point: base rows, and change
// rows whose op precedes the current position in the applied op stream. A row's succ list at
// stream position p is likewise its final succ list restricted to the entries whose op precedes
// p. So the replay walks F under those filters -- the seek (with the reference's per-column
// decoder positions), the merge loop and updatePatchProperty -- and never rebuilds a document.
//
// The patch tree (objectMeta, object patches, props, edits) lives in index-linked pools; the
// object patches are written out at the end as PR_OBJ sections of the am_patch.h log (PR_OBJ
// carries the object type, so the host stage can create any object on first sight). Pools are
// sized from the row and entry counts; running out reports PATCH_U_CAPACITY, never a wrong patch.
#pragma once
#include "am_patch.h"
#if defined(__HIP_DEVICE_COMPILE__)
#include "am_wave.h"
#endif

// ---- pools ----
struct DVal { uint32_t vtag, dt; int64_t v0, v1; };  // a patch value as the log stores it
struct DObj {                                        // objectMeta entry + patches[objectId]
  int64_t ctr; int32_t actor; int32_t type;          // actor -1: _root; type 0 map 1 list 2 text 3 table
  int32_t parent;                                    // objectMeta.parentObj (DObj index), -1: none
  int32_t pk_row;                                    // the make op: its elemId is parentKey
  int32_t kids;                                      // children: first DKid
  int32_t has_patch;
  int32_t edit_tail;                                 // last DEdit of the object's edits, -1
  int32_t prop_head, prop_tail;                      // DProp list
  int32_t pad;
};
struct DKid { int32_t elem_row; int32_t head; int32_t n; int32_t next; };  // children[elemId]
struct DKV { int64_t ctr; int32_t actor; int32_t kind; int32_t ref; int32_t next; };  // 1: set row, 2: DObj
struct DProp { int32_t key_row; int32_t head, tail; int32_t next; };
struct DPE { int64_t ctr; int32_t actor; int32_t next; DVal v; };
struct DEdit {
  uint32_t action;  // PR_INSERT / PR_MULTI / PR_UPDATE / PR_REMOVE
  int32_t prev;
  int64_t index, ec, oc, count;
  int32_t ea, oa;
  DVal v;
  int32_t mv_tail;
  uint32_t nmv, mdt;
  int32_t pad;
};
struct DMV { DVal v; int32_t prev; int32_t pad; };
struct DPst { int32_t elem_row; int32_t vis_head, vis_tail; int32_t has_child; int32_t action; int32_t cs_head; int32_t cm_head; int32_t next; };
struct DVis { int32_t row; int32_t next; };
struct DCs { int64_t op_ctr; int64_t value; int32_t op_actor; int32_t nleft; int32_t next; int32_t pad; };
struct DCm { int64_t ctr; int32_t actor; int32_t state; int32_t next; int32_t pad; };

// a workgroup barrier in the wide replay (k_diff's workgroup is one wave: it orders the lanes'
// global writes before the next loop's reads)
#if defined(__HIP_DEVICE_COMPILE__)
#define DSYNC() do { if constexpr (Wide) __syncthreads(); } while (0)
#else
#define DSYNC() do { } while (0)
#endif

#define DIFF_NCAPS_MAX 24
struct DiffScratch {
  DObj* obj; uint32_t nobj, cap_obj;
  DKid* kid; uint32_t nkid, cap_kid;
  DKV* kv; uint32_t nkv, cap_kv;
  DProp* prop; uint32_t nprop, cap_prop;
  DPE* pe; uint32_t npe, cap_pe;
  DEdit* ed; uint32_t ned, cap_ed;
  DMV* mv; uint32_t nmv, cap_mv;
  DPst* pst; uint32_t npst, cap_pst;  // reset at each mergeDocChangeOps call
  DVis* vis; uint32_t nvis, cap_vis;
  DCs* cs; uint32_t ncs, cap_cs;
  DCm* cm; uint32_t ncm, cap_cm;
  int32_t* fpos;                      // row -> position in F (-1: deletion)
  int32_t* oids; uint32_t noid, cap_oid;  // objectIds (Set, insertion order)
  int32_t* tmp;                       // emission order of one object's edits / popped edits
  int32_t* cops; uint8_t* seen;       // changeOps (rows) and predSeen flags
  uint32_t* seen_off;
  uint32_t cap_cops, cap_seen;
  // O(log n) seek (Fenwick trees over F positions, see Diff::advance)
  int32_t* bitp;                      // present rows
  int32_t* bitv;                      // visible list elements (at their insert row)
  int32_t* nsc;                       // succ count of the row at F position f, as of the replay time
  int32_t* live;                      // element (insert-row F position): present rows with no succ
  int32_t* estart;                    // F position -> F position of its element's insert row, -1: map row
  int32_t* hash; uint32_t hmask;      // element id -> F position of its insert row (open addressing)
  uint32_t* ev_off; int32_t* ev;      // succ entries bucketed by the stream time of their op
#ifdef AM_DIFF_CHECK
  uint64_t dcap[DIFF_NCAPS_MAX];      // diagnostics build: the pool sizes, checked on every unchecked write
#endif
};

// sizes of the pools for R rows and E pred/succ entries (host and device agree)
#define DIFF_NCAPS 24
AM_PHD inline uint64_t diff_hash_cap(uint64_t R) {
  uint64_t h = 16;
  while (h < 2 * R + 2) h <<= 1;
  return h;
}
// pools with heuristic sizes (kv, pe, ed, mv, tmp) scale by `ps` (8 on a rerun after PATCH_U_CAPACITY)
AM_PHD inline void diff_caps(uint64_t R, uint64_t E, uint64_t caps[DIFF_NCAPS], uint64_t ps = 1) {
  caps[0] = R + 2;          // obj
  caps[1] = R + 2;          // kid
  caps[2] = ps * (4 * R + 64);     // kv
  caps[3] = R + 2;          // prop
  caps[4] = ps * (4 * R + 64);     // pe
  caps[5] = ps * (4 * R + 64);     // ed
  caps[6] = ps * (4 * R + 64);     // mv
  caps[7] = R + 2;          // pst
  caps[8] = 2 * R + 4;      // vis
  caps[9] = R + 2;          // cs
  caps[10] = E + 2;         // cm
  caps[11] = R + 2;         // fpos
  caps[12] = R + 2;         // oids
  caps[13] = ps * (8 * R + 128);   // tmp
  caps[14] = R + 2;         // cops (+ seen_off)
  caps[15] = E + 2;         // seen
  caps[16] = R + 2;         // bitp
  caps[17] = R + 2;         // bitv
  caps[18] = R + 2;         // nsc
  caps[19] = R + 2;         // live
  caps[20] = R + 2;         // estart
  caps[21] = diff_hash_cap(R);  // hash
  caps[22] = R + 2;         // ev_off
  caps[23] = E + 2;         // ev
}
// Binds the pools at p (16-byte aligned each) and returns their total bytes; the workspace layout
// sizes the region with the same function (diff_scratch_bytes), so the two can never disagree (they
// once rounded cops / seen_off as one pool and bound them as two: 16 bytes past the region).
AM_PHD inline uint64_t diff_scratch_bind(uint8_t* p, uint64_t R, uint64_t E, DiffScratch& w, uint64_t ps = 1) {
  uint64_t c[DIFF_NCAPS];
  diff_caps(R, E, c, ps);
  uint64_t o = 0;
  auto take = [&](uint64_t bytes) { uint8_t* at = p + o; o += (bytes + 15) & ~(uint64_t)15; return at; };
  w.obj = reinterpret_cast<DObj*>(take(c[0] * sizeof(DObj))); w.cap_obj = (uint32_t)c[0];
  w.kid = reinterpret_cast<DKid*>(take(c[1] * sizeof(DKid))); w.cap_kid = (uint32_t)c[1];
  w.kv = reinterpret_cast<DKV*>(take(c[2] * sizeof(DKV))); w.cap_kv = (uint32_t)c[2];
  w.prop = reinterpret_cast<DProp*>(take(c[3] * sizeof(DProp))); w.cap_prop = (uint32_t)c[3];
  w.pe = reinterpret_cast<DPE*>(take(c[4] * sizeof(DPE))); w.cap_pe = (uint32_t)c[4];
  w.ed = reinterpret_cast<DEdit*>(take(c[5] * sizeof(DEdit))); w.cap_ed = (uint32_t)c[5];
  w.mv = reinterpret_cast<DMV*>(take(c[6] * sizeof(DMV))); w.cap_mv = (uint32_t)c[6];
  w.pst = reinterpret_cast<DPst*>(take(c[7] * sizeof(DPst))); w.cap_pst = (uint32_t)c[7];
  w.vis = reinterpret_cast<DVis*>(take(c[8] * sizeof(DVis))); w.cap_vis = (uint32_t)c[8];
  w.cs = reinterpret_cast<DCs*>(take(c[9] * sizeof(DCs))); w.cap_cs = (uint32_t)c[9];
  w.cm = reinterpret_cast<DCm*>(take(c[10] * sizeof(DCm))); w.cap_cm = (uint32_t)c[10];
  w.fpos = reinterpret_cast<int32_t*>(take(c[11] * 4));
  w.oids = reinterpret_cast<int32_t*>(take(c[12] * 4)); w.cap_oid = (uint32_t)c[12];
  w.tmp = reinterpret_cast<int32_t*>(take(c[13] * 4));
  w.cops = reinterpret_cast<int32_t*>(take(c[14] * 4));
  w.seen_off = reinterpret_cast<uint32_t*>(take(c[14] * 4));
  w.cap_cops = (uint32_t)c[14];
  w.seen = take(c[15]);
  w.cap_seen = (uint32_t)c[15];
  w.bitp = reinterpret_cast<int32_t*>(take(c[16] * 4));
  w.bitv = reinterpret_cast<int32_t*>(take(c[17] * 4));
  w.nsc = reinterpret_cast<int32_t*>(take(c[18] * 4));
  w.live = reinterpret_cast<int32_t*>(take(c[19] * 4));
  w.estart = reinterpret_cast<int32_t*>(take(c[20] * 4));
  w.hash = reinterpret_cast<int32_t*>(take(c[21] * 4)); w.hmask = (uint32_t)c[21] - 1;
  w.ev_off = reinterpret_cast<uint32_t*>(take(c[22] * 4));
  w.ev = reinterpret_cast<int32_t*>(take(c[23] * 4));
#ifdef AM_DIFF_CHECK
  for (int i = 0; i < DIFF_NCAPS; i++) w.dcap[i] = c[i];
#endif
  w.nobj = w.nkid = w.nkv = w.nprop = w.npe = w.ned = w.nmv = w.npst = w.nvis = w.ncs = w.ncm = w.noid = 0;
  return o;
}
AM_PHD inline uint64_t diff_scratch_bytes(uint64_t R, uint64_t E, uint64_t ps = 1) {
  DiffScratch w;
  return diff_scratch_bind(nullptr, R, E, w, ps);
}

// ---- the replay ----
// Src interface (row indexes: base rows [0, nb()) in document order, then the applied change ops
// in application order, deletions included):
//   nb(); nrows(); nout(); frow(f); f_nsucc(f); f_succ_ctr(f, k); f_succ_actor(f, k);
//   f_succ_time(f, k) (-1: base entry, else the stream index of the succ op);
//   obj_ctr(i) / obj_actor(i) (-1: root); key_ctr(i) (-1: null) / key_actor(i) (-1: null);
//   has_key(i) (key string not null); key_len(i); key_cmp(i, j) (UTF-16 order); key_eq(i, j);
//   copy_key(i, dst); id_ctr(i); id_actor(i); insert(i); action(i); npred(i); pred_ctr(i, k);
//   pred_actor(i, k); rank(a); patch_value's val_len / copy_value / value_int / value_f64_bits;
//   nactors(); actor_len(a); copy_actor(a, dst); nchg(); chg_actor(c); chg_seq(c); npass();
//   pass_end(p) (stream index where pass p ends)
//
// Wide (k_diff): all 64 lanes of the wave run the replay's chain in lockstep -- every lane loads and
// stores the same addresses and takes the same branches, so the chain costs what one lane's does --
// and the steps that are scans or searches spread over the lanes: the presence sets below (a bit per
// F position instead of Fenwick trees: a prefix count or a k-th lookup is two rounds of independent
// loads and a wave scan, not log2(n) dependent loads), the per-row setup (fast_init, F positions,
// the documentPatch objectMeta pass), 64-way searches over F and the linear pool lookups. Serial
// (LDS-mode documents in k_doc, one lane of a larger workgroup): the same replay on Fenwick trees.
template <class Src, bool Wide = false>
struct Diff {
  const Src& s;
  DiffScratch& w;
  PatchOut& o;
  bool ok;
  uint32_t cur_t = 0;   // succ / row events of stream times < cur_t are in the trees
  int32_t ptotal = 0;   // present rows
  uint32_t nw = 0;      // wide presence sets: 64-bit words over F (the counts per 4096 positions follow)
  int64_t lo_oc = -3;   // fast_seek: the first F position of the last object sought
  int32_t lo_oa = -3, lo_f = 0;
#if defined(AM_DIFF_CHECK) && defined(__HIP_DEVICE_COMPILE__)
  // diagnostics build: cycles per replay section (apply_ops), printed for large documents
  uint64_t pacc[10] = {};
  uint64_t pt = 0;
#define DPT() pt = clock64()
#define DPA(k) do { const uint64_t t_ = clock64(); pacc[k] += t_ - pt; pt = t_; } while (0)
#else
#define DPT()
#define DPA(k)
#endif
  AM_PHD Diff(const Src& src, DiffScratch& ws, PatchOut& out) : s(src), w(ws), o(out), ok(true) {}

  // ---- replay state in Fenwick trees over F positions ----
  // The reference seeks by scanning the document (seekWithinBlock, new.js:50-192): the position
  // of an op is the number of present rows before it, and its list index the number of visible
  // elements before it in its object. Here both are prefix sums at the op's F position: `bitp`
  // counts present rows, `bitv` counts elements (at their insert row) with at least one present
  // row without a succ -- exactly the rows visit() counts. advance(W) applies, in stream order,
  // the rows and succ entries whose op precedes stream position W, so seek and the doc cursor
  // cost O(log n) instead of O(rows).
  AM_PHD static uint32_t lsb(uint32_t i) { return i & (~i + 1u); }
#ifdef AM_DIFF_CHECK
  // diagnostics build: an index outside pool `k` fails the replay with status 240 + k (arg0 = index,
  // arg1 = the pool's size) instead of writing past it
  AM_PHD bool dchk(int k, uint64_t i) {
    if (i < w.dcap[k]) return true;
    if (ok) { o.status = 240 + k; o.arg0 = (int64_t)i; o.arg1 = (int64_t)w.dcap[k]; ok = false; }
    return false;
  }
#define DCHK(k, i) if (!dchk(k, (uint64_t)(i))) return
#define DCHKF(k, i) if (!dchk(k, (uint64_t)(i))) return false
#else
#define DCHK(k, i)
#define DCHKF(k, i)
#endif
  AM_PHD void bit_add(int32_t* b, uint32_t i, int32_t v) {
    const uint32_t n = s.nout();
    DCHK(16, n);
    for (++i; i <= n; i += lsb(i)) b[i] += v;
  }
  AM_PHD int32_t bit_pre(const int32_t* b, uint32_t i) const {  // sum over F positions [0, i)
    int32_t r = 0;
    for (; i > 0; i -= lsb(i)) r += b[i];
    return r;
  }
  AM_PHD uint32_t bit_kth(const int32_t* b, int32_t k) const {  // F position of the k-th (1-based) counted one
    const uint32_t n = s.nout();
    uint32_t pos = 0, step = 1;
    while (step * 2 <= n) step *= 2;
    for (; step; step >>= 1)
      if (pos + step <= n && b[pos + step] < k) { pos += step; k -= b[pos]; }
    return pos;
  }
  // ---- presence sets: bitp (present rows), bitv (visible elements) over F positions ----
  // Wide layout in the same pool: nw 64-bit words, then one int32 count per 64 words (the pool's
  // R + 2 int32 always hold them: 8 * ceil(R / 64) + 4 * ceil(R / 4096) <= 4 * (R + 2)).
  AM_PHD void set_add(int32_t* b, uint32_t i, int32_t d) {
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (Wide) {
      DCHK(16, i >> 6 < nw ? 0 : ~0ull);
      uint64_t* wd = reinterpret_cast<uint64_t*>(b);
      const uint64_t bit = 1ull << (i & 63);
      wd[i >> 6] = d > 0 ? wd[i >> 6] | bit : wd[i >> 6] & ~bit;
      b[2 * nw + (i >> 12)] += d;
      return;
    }
#endif
    bit_add(b, i, d);
  }
  AM_PHD int32_t set_pre(const int32_t* b, uint32_t i) const {  // members at F positions [0, i)
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (Wide) {
      const uint64_t* wd = reinterpret_cast<const uint64_t*>(b);
      const int32_t* cn = b + 2 * nw;
      const uint32_t wi = i >> 6, si = wi >> 6, l = wave::lane_id();
      uint32_t acc = 0;
      for (uint32_t q = l; q < si; q += 64) acc += (uint32_t)cn[q];
      if ((si << 6) + l < wi) acc += (uint32_t)__popcll(wd[(si << 6) + l]);
      if ((i & 63) && l == 0) acc += (uint32_t)__popcll(wd[wi] & ((1ull << (i & 63)) - 1));
      return (int32_t)wave::sum_all(acc);
    }
#endif
    return bit_pre(b, i);
  }
  AM_PHD uint32_t set_kth(const int32_t* b, int32_t k) const {  // F position of the k-th (1-based) member
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (Wide) {
      const uint64_t* wd = reinterpret_cast<const uint64_t*>(b);
      const int32_t* cn = b + 2 * nw;
      const uint32_t l = wave::lane_id(), nsb = (nw + 63) >> 6;
      uint32_t sb = nsb ? nsb - 1 : 0;
      for (uint32_t base = 0; base < nsb; base += 64) {
        const uint32_t c = base + l < nsb ? (uint32_t)cn[base + l] : 0u;
        const uint32_t inc = wave::incl_add(c);
        const uint64_t m = __ballot(inc >= (uint32_t)k);
        if (m) {
          const uint32_t j = (uint32_t)__builtin_ctzll(m);
          sb = base + j;
          k -= (int32_t)wave::bcast(inc - c, (int)j);
          break;
        }
        k -= (int32_t)wave::bcast(inc, 63);
      }
      const uint32_t wq = (sb << 6) + l;
      const uint64_t x = wq < nw ? wd[wq] : 0ull;
      const uint32_t c = (uint32_t)__popcll(x);
      const uint32_t inc = wave::incl_add(c);
      const uint64_t m = __ballot(inc >= (uint32_t)k);
      const uint32_t j = m ? (uint32_t)__builtin_ctzll(m) : 63u;
      k -= (int32_t)wave::bcast(inc - c, (int)j);
      const uint64_t word = wave::bcast(x, (int)j);
      const uint64_t upto = l == 63 ? word : word & ((2ull << l) - 1);
      const uint64_t m2 = __ballot(((word >> l) & 1) && (int32_t)__popcll(upto) == k);
      return (((sb << 6) + j) << 6) + (m2 ? (uint32_t)__builtin_ctzll(m2) : 0u);
    }
#endif
    return bit_kth(b, k);
  }
  // first present F position >= f, or nout()
  AM_PHD int32_t next_present(int32_t f) const {
    if (f >= (int32_t)s.nout()) return (int32_t)s.nout();
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (Wide) {
      const uint64_t* wd = reinterpret_cast<const uint64_t*>(w.bitp);
      const uint32_t wi = (uint32_t)f >> 6, l = wave::lane_id();
      const uint64_t x = wd[wi] & (~0ull << (f & 63));
      if (x) return (int32_t)((wi << 6) + (uint32_t)__builtin_ctzll(x));
      for (uint32_t base = wi + 1; base < nw; base += 64) {
        const uint64_t y = base + l < nw ? wd[base + l] : 0ull;
        const uint64_t m = __ballot(y != 0);
        if (m) {
          const uint32_t j = (uint32_t)__builtin_ctzll(m);
          return (int32_t)(((base + j) << 6) + (uint32_t)__builtin_ctzll(wave::bcast(y, (int)j)));
        }
      }
      return (int32_t)s.nout();
    }
#endif
    const int32_t k = set_pre(w.bitp, (uint32_t)f);
    return k >= ptotal ? (int32_t)s.nout() : (int32_t)set_kth(w.bitp, k + 1);
  }
  // first index in [a, b) where pred is false (pred holds on a prefix of [a, b)); wide: 64 probes
  // per round
  template <class P>
  AM_PHD int32_t first_false(int32_t a, int32_t b, P pred) const {
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (Wide) {
      const int32_t l = (int32_t)wave::lane_id();
      while (a < b) {
        const int32_t step = (b - a + 63) / 64;
        const int32_t m = a + l * step;
        const uint64_t bal = __ballot(m < b && pred(m));
        const int32_t t = (int32_t)__popcll(bal);
        if (t == 0) return a;
        const int32_t nb = a + t * step < b ? a + t * step : b;
        a = a + (t - 1) * step + 1;
        b = nb;
      }
      return a;
    }
#endif
    while (a < b) {
      const int32_t m = (a + b) / 2;
      if (pred(m)) a = m + 1; else b = m;
    }
    return a;
  }
  AM_PHD uint32_t hslot(int64_t ctr, int32_t actor) const {
    uint64_t h = (uint64_t)ctr * 0x9E3779B97F4A7C15ull ^ ((uint64_t)(uint32_t)actor + 1u) * 0xC2B2AE3D27D4EB4Full;
    return (uint32_t)(h >> 32) & w.hmask;
  }
  AM_PHD int32_t elem_find(int64_t ctr, int32_t actor) const {  // F position of the insert row, -1
    for (uint32_t h = hslot(ctr, actor);; h = (h + 1) & w.hmask) {
      const int32_t f = w.hash[h];
      if (f < 0) return -1;
      const int32_t r = s.frow(f);
      if (s.id_ctr(r) == ctr && s.id_actor(r) == actor) return f;
    }
  }
  AM_PHD void elem_row_live(int32_t f, int32_t d) {
    DCHK(20, f);
    const int32_t e = w.estart[f];
    if (e < 0) return;
    DCHK(19, e);
    const int32_t before = w.live[e];
    w.live[e] = before + d;
    if (before == 0 && d > 0) set_add(w.bitv, (uint32_t)e, 1);
    else if (before > 0 && before + d == 0) set_add(w.bitv, (uint32_t)e, -1);
  }
  AM_PHD void fast_init() {
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (Wide) { fast_init_wide(); return; }
#endif
    const uint32_t n = s.nout(), nstream = s.nrows() - s.nb();
    DCHK(16, n);
    DCHK(18, n);
    DCHK(22, nstream);
    for (uint32_t i = 0; i <= n; i++) { w.bitp[i] = 0; w.bitv[i] = 0; }
    for (uint32_t h = 0; h <= w.hmask; h++) w.hash[h] = -1;
    for (uint32_t t = 0; t <= nstream; t++) w.ev_off[t] = 0;
    for (uint32_t f = 0; f < n; f++) {
      const int32_t r = s.frow((int32_t)f);
      w.nsc[f] = 0;
      w.live[f] = 0;
      if (s.has_key(r)) w.estart[f] = -1;
      else if (s.insert(r)) w.estart[f] = (int32_t)f;
      else w.estart[f] = f > 0 && w.estart[f - 1] >= 0 && s.obj_ctr(s.frow((int32_t)f - 1)) == s.obj_ctr(r) &&
                                 s.obj_actor(s.frow((int32_t)f - 1)) == s.obj_actor(r) ? w.estart[f - 1] : -1;
      if (!s.has_key(r) && s.insert(r)) {
        uint32_t h = hslot(s.id_ctr(r), s.id_actor(r));
        while (w.hash[h] >= 0) h = (h + 1) & w.hmask;
        w.hash[h] = (int32_t)f;
      }
      for (uint32_t k = 0; k < s.f_nsucc(f); k++) {
        const int64_t t = s.f_succ_time(f, k);
        if (t < 0) w.nsc[f]++;
        else if (t < (int64_t)nstream) w.ev_off[t + 1]++;
      }
    }
    for (uint32_t t = 0; t < nstream; t++) w.ev_off[t + 1] += w.ev_off[t];
    for (uint32_t f = 0; f < n; f++)  // bucket fill: ev_off[t] is the running cursor, restored below
      for (uint32_t k = 0; k < s.f_nsucc(f); k++) {
        const int64_t t = s.f_succ_time(f, k);
        if (t >= 0 && t < (int64_t)nstream) {
          DCHK(23, w.ev_off[t]);
          w.ev[w.ev_off[t]++] = (int32_t)f;
        }
      }
    for (uint32_t t = nstream; t > 0; t--) w.ev_off[t] = w.ev_off[t - 1];
    w.ev_off[0] = 0;
    ptotal = 0;
    for (uint32_t f = 0; f < n; f++)
      if (rtime(s.frow((int32_t)f)) < 0) {
        bit_add(w.bitp, f, 1);
        ptotal++;
        if (w.nsc[f] == 0) elem_row_live((int32_t)f, 1);
      }
    cur_t = 0;
  }
#if defined(__HIP_DEVICE_COMPILE__)
  // fast_init over the lanes: the same pools, rows 64 at a time (estart by a segmented scan, the
  // hash by CAS, the succ buckets by atomic counts then a scan, the presence words by ballots)
  __device__ void fast_init_wide() {
    const uint32_t n = s.nout(), nstream = s.nrows() - s.nb(), l = wave::lane_id();
    nw = (n + 63) >> 6;
    const uint32_t nsb = (nw + 63) >> 6;
    uint64_t* wp = reinterpret_cast<uint64_t*>(w.bitp);
    uint64_t* wv = reinterpret_cast<uint64_t*>(w.bitv);
    int32_t* cp = w.bitp + 2 * nw;
    int32_t* cv = w.bitv + 2 * nw;
    DCHK(22, nstream);
    for (uint32_t q = l; q < nsb; q += 64) { cp[q] = 0; cv[q] = 0; }
    for (uint32_t h = l; h <= w.hmask; h += 64) w.hash[h] = -1;
    for (uint32_t t = l; t <= nstream; t += 64) w.ev_off[t] = 0;
    for (uint32_t f = l; f < n; f += 64) w.live[f] = 0;
    __syncthreads();
    int32_t carry = -1;  // estart of the previous row
    int64_t coc = 0;
    int32_t coa = 0;
    ptotal = 0;
    for (uint32_t base = 0; base < n; base += 64) {
      const uint32_t f = base + l;
      const bool in = f < n;
      const int32_t r = in ? s.frow((int32_t)f) : 0;
      const bool hk = in && s.has_key(r), ins = in && s.insert(r);
      const int64_t oc = in ? s.obj_ctr(r) : 0;
      const int32_t oa = in ? s.obj_actor(r) : 0;
      const int64_t poc = wave::up1(oc, coc);
      const int32_t poa = wave::up1(oa, coa);
      // estart: -1 (map row, or a list row whose predecessor is in another object), f (insert
      // row), else the predecessor's: the last resetting row at or before this lane, or the carry
      const bool reset = !in || hk || ins || poc != oc || poa != oa;
      const int32_t v = in && !hk && ins ? (int32_t)f : -1;
      const uint64_t rm = __ballot(reset);
      const uint64_t upto = l == 63 ? rm : rm & ((2ull << l) - 1);
      const int32_t sv = __shfl(v, upto ? 63 - __builtin_clzll(upto) : 0);
      const int32_t es = upto ? sv : carry;
      uint32_t nsc = 0;
      if (in) {
        w.estart[f] = es;
        if (!hk && ins) {
          uint32_t h = hslot(s.id_ctr(r), s.id_actor(r));
          while (atomicCAS(&w.hash[h], -1, (int32_t)f) >= 0) h = (h + 1) & w.hmask;
        }
        for (uint32_t k = 0; k < s.f_nsucc(f); k++) {
          const int64_t t = s.f_succ_time(f, k);
          if (t < 0) nsc++;
          else if (t < (int64_t)nstream) atomicAdd(&w.ev_off[t + 1], 1u);
        }
        w.nsc[f] = (int32_t)nsc;
      }
      carry = wave::bcast(es, 63);
      coc = wave::bcast(oc, 63);
      coa = wave::bcast(oa, 63);
      const bool pres = in && rtime(r) < 0;
      const uint64_t word = __ballot(pres);
      wp[base >> 6] = word;
      const int32_t pc = (int32_t)__popcll(word);
      cp[base >> 12] += pc;
      ptotal += pc;
      if (pres && nsc == 0 && es >= 0) atomicAdd(&w.live[es], 1);
    }
    __syncthreads();
    for (uint32_t base = 0; base < n; base += 64) {
      const uint32_t f = base + l;
      const uint64_t word = __ballot(f < n && w.live[f] > 0);
      wv[base >> 6] = word;
      cv[base >> 12] += (int32_t)__popcll(word);
    }
    uint32_t run = 0;  // ev_off[t + 1] += ev_off[t]: bucket starts
    for (uint32_t base = 0; base <= nstream; base += 64) {
      const uint32_t t = base + l;
      const uint32_t inc = wave::incl_add(t <= nstream ? w.ev_off[t] : 0u) + run;
      if (t <= nstream) w.ev_off[t] = inc;
      run = wave::bcast(inc, 63);
    }
    __syncthreads();
    for (uint32_t f = l; f < n; f += 64)  // bucket fill (the order inside a bucket does not matter)
      for (uint32_t k = 0; k < s.f_nsucc(f); k++) {
        const int64_t t = s.f_succ_time(f, k);
        if (t >= 0 && t < (int64_t)nstream) w.ev[atomicAdd(&w.ev_off[t], 1u)] = (int32_t)f;
      }
    __syncthreads();
    for (uint32_t c = (nstream >> 6) + 1; c-- > 0;) {  // ev_off[t] = ev_off[t - 1], top chunk first
      const uint32_t t = (c << 6) + l;
      const uint32_t x = t >= 1 && t <= nstream ? w.ev_off[t - 1] : 0u;
      if (t <= nstream) w.ev_off[t] = x;
    }
    __syncthreads();
    cur_t = 0;
  }
#endif
  AM_PHD void advance(int64_t W) {
    const uint32_t nstream = s.nrows() - s.nb();
    while ((int64_t)cur_t < W && cur_t < nstream) {
      const uint32_t t = cur_t++;
      DCHK(11, srow(t));
      const int32_t f = w.fpos[srow(t)];
      if (f >= 0) {
        set_add(w.bitp, (uint32_t)f, 1);
        ptotal++;
        if (w.nsc[f] == 0) elem_row_live(f, 1);
      }
      for (uint32_t q = w.ev_off[t]; q < w.ev_off[t + 1]; q++) {
        const int32_t g = w.ev[q];
        if (w.nsc[g]++ == 0 && rtime(s.frow(g)) < (int64_t)t) elem_row_live(g, -1);
      }
    }
  }
  // seek of the op at stream row `first` from the trees: (skip, visible) as seek() computes them.
  // Returns false when the op has no F anchor (its element is unknown): seek() then decides.
  AM_PHD bool fast_seek(int32_t first, uint32_t& skip, int64_t& vis) {
    const int64_t q_oc = s.obj_ctr(first);
    const int32_t q_oa = s.obj_actor(first);
    const int32_t n = (int32_t)s.nout();
    // the object's first F position (F is fixed for the whole replay: kept for the last object)
    if (q_oc != lo_oc || q_oa != lo_oa) {
      lo_f = first_false(0, n, [&](int32_t m) {  // document order of objects: _root, then (ctr, actor)
        if (q_oa < 0 || q_oc < 0) return false;
        const int32_t r = s.frow(m);
        const int64_t oc = s.obj_ctr(r);
        const int32_t oa = s.obj_actor(r);
        if (oc < 0 || oa < 0) return true;
        return oc < q_oc || (oc == q_oc && act_lt(oa, q_oa));
      });
      lo_oc = q_oc;
      lo_oa = q_oa;
    }
    const int32_t lo = lo_f;
    int32_t target;
    if (s.has_key(first)) {
      const int32_t a = first_false(lo, n, [&](int32_t m) {
        const int32_t r = s.frow(m);
        return s.obj_ctr(r) == q_oc && s.obj_actor(r) == q_oa && s.has_key(r) && s.key_cmp(r, first) < 0;
      });
      skip = (uint32_t)set_pre(w.bitp, (uint32_t)a);
      vis = 0;
      return true;
    }
    if (s.insert(first)) {
      target = w.fpos[first];
    } else {
      if (!(s.key_ctr(first) > 0 && s.key_actor(first) >= 0)) return false;
      target = elem_find(s.key_ctr(first), s.key_actor(first));
    }
    if (target < 0) return false;
    skip = (uint32_t)set_pre(w.bitp, (uint32_t)target);
    vis = (int64_t)(set_pre(w.bitv, (uint32_t)target) - set_pre(w.bitv, (uint32_t)lo));
    return true;
  }

  AM_PHD bool fail(uint32_t st, int64_t a0 = 0, int64_t a1 = 0) {
    if (ok) { o.status = st; o.arg0 = a0; o.arg1 = a1; }
    ok = false;
    return false;
  }
  AM_PHD int64_t rtime(int32_t row) const { return row >= (int32_t)s.nb() ? (int64_t)row - s.nb() : -1; }
  // actor string order through the ranks; -1 (null / undefined) compares false
  AM_PHD bool act_lt(int32_t a, int32_t b) const { return a >= 0 && b >= 0 && s.rank(a) < s.rank(b); }
  // succ count of the row at F position f when the stream has reached position lim
  AM_PHD uint32_t nsucc_at(int32_t f, int64_t lim) const {
    uint32_t n = 0;
    for (uint32_t k = 0; k < s.f_nsucc(f); k++) n += s.f_succ_time(f, k) < lim ? 1u : 0u;
    return n;
  }
  // elemId of an op (new.js:888-890): the key string when truthy, else the element id
  AM_PHD bool elem_str(int32_t i) const { return s.has_key(i) && s.key_len(i) > 0; }
  AM_PHD int64_t elem_ctr(int32_t i) const { return s.insert(i) ? s.id_ctr(i) : s.key_ctr(i); }
  AM_PHD int32_t elem_actor(int32_t i) const { return s.insert(i) ? s.id_actor(i) : s.key_actor(i); }
  AM_PHD bool elem_eq(int32_t i, int32_t j) const {
    if (elem_str(i) != elem_str(j)) return false;
    if (elem_str(i)) return s.key_eq(i, j);
    return elem_ctr(i) == elem_ctr(j) && elem_actor(i) == elem_actor(j);
  }
  // make-like ops: `op[actionIdx] % 2 === 0` (new.js:894, 909, 923, 972) holds for every even action
  // and for a null action (null % 2 === 0); s.action() reads null as -1
  AM_PHD static bool is_make(int64_t a) { return a < 0 || a % 2 == 0; }
  // their object type (new.js:886, 924): OBJECT_TYPE[ACTIONS[a]] -- undefined (4) for a null action,
  // null (5) for an action beyond ACTIONS; 0 map 1 list 2 text 3 table
  AM_PHD static uint32_t obj_type_of_action(int64_t a) {
    return a < 0 ? 4u : a == 2 ? 1u : a == 4 ? 2u : a == 6 ? 3u : a >= 8 ? 5u : 0u;
  }

  // ---- objectMeta / patches ----
  AM_PHD int32_t obj_find(int64_t ctr, int32_t actor) const {
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (Wide) {
      const uint32_t l = wave::lane_id();
      for (uint32_t base = 0; base < w.nobj; base += 64) {
        const uint32_t k = base + l;
        const uint64_t m = __ballot(k < w.nobj && w.obj[k].ctr == ctr && w.obj[k].actor == actor);
        if (m) return (int32_t)(base + (uint32_t)__builtin_ctzll(m));
      }
      return -1;
    }
#endif
    for (uint32_t k = 0; k < w.nobj; k++) if (w.obj[k].ctr == ctr && w.obj[k].actor == actor) return (int32_t)k;
    return -1;
  }
  AM_PHD int32_t obj_new(int64_t ctr, int32_t actor, uint32_t type) {
    if (w.nobj >= w.cap_obj) { fail(PATCH_U_CAPACITY); return -1; }
    DObj& d = w.obj[w.nobj];
    d.ctr = ctr; d.actor = actor; d.type = (int32_t)type; d.parent = -1; d.pk_row = -1; d.kids = -1;
    d.has_patch = 0; d.edit_tail = -1; d.prop_head = d.prop_tail = -1; d.pad = 0;
    return (int32_t)w.nobj++;
  }
  AM_PHD int32_t kid_find(int32_t ob, int32_t row, bool create) {
    int32_t* link = &w.obj[ob].kids;
    while (*link >= 0) {
      if (elem_eq(w.kid[*link].elem_row, row)) return *link;
      link = &w.kid[*link].next;
    }
    if (!create) return -1;
    if (w.nkid >= w.cap_kid) { fail(PATCH_U_CAPACITY); return -1; }
    DKid& d = w.kid[w.nkid];
    d.elem_row = row; d.head = -1; d.n = 0; d.next = -1;
    *link = (int32_t)w.nkid;  // appended: JS object key order
    return (int32_t)w.nkid++;
  }
  // children[elemId][opId] = value (an existing opId keeps its position)
  AM_PHD bool kv_set(int32_t kd, int64_t ctr, int32_t actor, int32_t kind, int32_t ref) {
    int32_t* link = &w.kid[kd].head;
    while (*link >= 0) {
      DKV& e = w.kv[*link];
      if (e.ctr == ctr && e.actor == actor) { e.kind = kind; e.ref = ref; return true; }
      link = &e.next;
    }
    if (w.nkv >= w.cap_kv) return fail(PATCH_U_CAPACITY);
    DKV& e = w.kv[w.nkv];
    e.ctr = ctr; e.actor = actor; e.kind = kind; e.ref = ref; e.next = -1;
    *link = (int32_t)w.nkv++;
    w.kid[kd].n++;
    return true;
  }
  AM_PHD void patch_on(int32_t ob) { w.obj[ob].has_patch = 1; }
  AM_PHD DVal child_val(int32_t ob) const {
    DVal v;
    v.vtag = PV_CHILD; v.dt = (uint32_t)w.obj[ob].type; v.v0 = w.obj[ob].ctr; v.v1 = w.obj[ob].actor;
    return v;
  }
  AM_PHD bool row_val(int32_t row, DVal& v) {
    if (!patch_value(s, (uint32_t)row, o, v.vtag, v.dt, v.v0, v.v1)) {
      ok = false;
      return false;
    }
    return true;
  }

  // ---- edits (appendEdit / appendUpdate / convertInsertToUpdate, new.js:747-869) ----
  AM_PHD bool mv_push(DEdit& e, const DVal& v) {
    if (w.nmv >= w.cap_mv) return fail(PATCH_U_CAPACITY);
    DMV& m = w.mv[w.nmv];
    m.v = v; m.prev = e.mv_tail; m.pad = 0;
    e.mv_tail = (int32_t)w.nmv++;
    e.nmv++;
    return true;
  }
  AM_PHD const DVal& mv_first(const DEdit& e) const {
    int32_t k = e.mv_tail;
    for (uint32_t q = 1; q < e.nmv; q++) k = w.mv[k].prev;
    return w.mv[k].v;
  }
  AM_PHD bool edit_push(int32_t ob, const DEdit& ne) {
    if (w.ned >= w.cap_ed) return fail(PATCH_U_CAPACITY);
    DEdit& e = w.ed[w.ned];
    e = ne;
    e.prev = w.obj[ob].edit_tail;
    e.mv_tail = -1; e.nmv = 0;
    w.obj[ob].edit_tail = (int32_t)w.ned++;
    return true;
  }
  AM_PHD void edit_pop(int32_t ob) { w.obj[ob].edit_tail = w.ed[w.obj[ob].edit_tail].prev; }
  AM_PHD bool append_edit(int32_t ob, const DEdit& ne) {
    const int32_t lt = w.obj[ob].edit_tail;
    if (lt >= 0) {
      DEdit& last = w.ed[lt];
      if (last.action == PR_INSERT && ne.action == PR_INSERT && last.index == ne.index - 1 && last.v.vtag != PV_CHILD &&
          ne.v.vtag != PV_CHILD && last.ec == last.oc && last.ea == last.oa && ne.ec == ne.oc && ne.ea == ne.oa &&
          last.ea == ne.ea && last.ec + 1 == ne.ec) {
        const uint32_t da = pv_dtcode(last.v.vtag, last.v.dt), db = pv_dtcode(ne.v.vtag, ne.v.dt);
        if (da == db && pv_typeof(last.v.vtag) == pv_typeof(ne.v.vtag)) {
          const DVal first = last.v;
          last.action = PR_MULTI;
          last.mdt = pv_dt_truthy(db) ? db : 0;  // lastEdit.datatype set only when truthy
          last.mv_tail = -1; last.nmv = 0;
          return mv_push(last, first) && mv_push(last, ne.v);
        }
      }
      if (last.action == PR_MULTI && ne.action == PR_INSERT && last.index + (int64_t)last.nmv == ne.index &&
          ne.v.vtag != PV_CHILD && ne.ec == ne.oc && ne.ea == ne.oa && last.ea == ne.ea &&
          last.ec + (int64_t)last.nmv == ne.ec) {
        const uint32_t db = pv_dtcode(ne.v.vtag, ne.v.dt);
        if (last.mdt == db && pv_typeof(mv_first(last).vtag) == pv_typeof(ne.v.vtag)) return mv_push(last, ne.v);
      }
      if (last.action == PR_REMOVE && ne.action == PR_REMOVE && last.index == ne.index) {
        last.count += ne.count;
        return true;
      }
    }
    return edit_push(ob, ne);
  }
  AM_PHD bool append_update(int32_t ob, int64_t index, int64_t ec, int32_t ea, int64_t oc, int32_t oa, const DVal& v,
                            bool first) {
    bool ins = false;
    if (first) {
      while (!ins && w.obj[ob].edit_tail >= 0) {
        DEdit& last = w.ed[w.obj[ob].edit_tail];
        if ((last.action == PR_INSERT || last.action == PR_UPDATE) && last.index == index) {
          ins = last.action == PR_INSERT;
          edit_pop(ob);
        } else if (last.action == PR_MULTI && last.index + (int64_t)last.nmv - 1 == index) {
          last.mv_tail = w.mv[last.mv_tail].prev;  // values.pop()
          last.nmv--;
          ins = true;
        } else {
          break;
        }
      }
    }
    DEdit e = {};
    e.index = index; e.oc = oc; e.oa = oa; e.v = v;
    if (ins) { e.action = PR_INSERT; e.ec = ec; e.ea = ea; }
    else e.action = PR_UPDATE;
    return append_edit(ob, e);
  }
  AM_PHD bool convert_insert_to_update(int32_t ob, int64_t index, int64_t ec, int32_t ea) {
    // pop the suffix (updates, then the insert, at `index`) into tmp
    uint32_t nu = 0;
    while (w.obj[ob].edit_tail >= 0) {
      const int32_t k = w.obj[ob].edit_tail;
      const uint32_t act = w.ed[k].action;
      if (act == PR_INSERT || act == PR_UPDATE) {
        if (w.ed[k].index != index) return fail(PATCH_U_VALUE);  // 'last edit has unexpected index'
        DCHKF(13, nu);
        w.tmp[nu++] = k;
        edit_pop(ob);
        if (act == PR_INSERT) break;
      } else {
        return fail(PATCH_U_VALUE);  // 'last edit has unexpected action'
      }
    }
    for (uint32_t q = 0; q < nu; q++) {
      const DEdit u = w.ed[w.tmp[nu - 1 - q]];
      if (!append_update(ob, index, ec, ea, u.oc, u.oa, u.v, q == 0)) return false;
    }
    return true;
  }

  // ---- props (map objects) ----
  AM_PHD int32_t prop_get(int32_t ob, int32_t row, bool reset) {
    for (int32_t k = w.obj[ob].prop_head; k >= 0; k = w.prop[k].next)
      if (s.key_eq(w.prop[k].key_row, row)) {
        if (reset) w.prop[k].head = w.prop[k].tail = -1;
        return k;
      }
    if (w.nprop >= w.cap_prop) { fail(PATCH_U_CAPACITY); return -1; }
    DProp& p = w.prop[w.nprop];
    p.key_row = row; p.head = p.tail = -1; p.next = -1;
    if (w.obj[ob].prop_tail >= 0) w.prop[w.obj[ob].prop_tail].next = (int32_t)w.nprop;
    else w.obj[ob].prop_head = (int32_t)w.nprop;
    w.obj[ob].prop_tail = (int32_t)w.nprop;
    return (int32_t)w.nprop++;
  }
  // props[key][opId] = v; with `existed`, an existing opId is left alone and reported
  AM_PHD bool prop_set(int32_t pr, int64_t ctr, int32_t actor, const DVal& v, bool* existed = nullptr) {
    for (int32_t k = w.prop[pr].head; k >= 0; k = w.pe[k].next)
      if (w.pe[k].ctr == ctr && w.pe[k].actor == actor) {
        if (existed) { *existed = true; return true; }
        w.pe[k].v = v;
        return true;
      }
    if (existed) *existed = false;
    if (w.npe >= w.cap_pe) return fail(PATCH_U_CAPACITY);
    DPE& e = w.pe[w.npe];
    e.ctr = ctr; e.actor = actor; e.v = v; e.next = -1;
    if (w.prop[pr].tail >= 0) w.pe[w.prop[pr].tail].next = (int32_t)w.npe;
    else w.prop[pr].head = (int32_t)w.npe;
    w.prop[pr].tail = (int32_t)w.npe++;
    return true;
  }

  // ---- propState ----
  // propState[elemId]. In a whole-document scan (documentPatch) the rows of one key / element are
  // contiguous in document order, so only the last entry can match.
  AM_PHD int32_t pst_get(int32_t row, bool whole_doc) const {
    if (whole_doc) return w.npst && elem_eq(w.pst[w.npst - 1].elem_row, row) ? (int32_t)w.npst - 1 : -1;
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (Wide) {
      const uint32_t l = wave::lane_id();
      for (uint32_t base = 0; base < w.npst; base += 64) {
        const uint32_t k = base + l;
        const uint64_t m = __ballot(k < w.npst && elem_eq(w.pst[k].elem_row, row));
        if (m) return (int32_t)(base + (uint32_t)__builtin_ctzll(m));
      }
      return -1;
    }
#endif
    for (uint32_t k = 0; k < w.npst; k++) if (elem_eq(w.pst[k].elem_row, row)) return (int32_t)k;
    return -1;
  }

  // updatePatchProperty (new.js:884-1040). f: F position of a document op (its succ list as of
  // stream position lim), -1 for a change op (has_old = false, oldSuccNum undefined).
  AM_PHD bool update_property(int32_t ob, int32_t row, int32_t f, int64_t lim, int64_t list_index, bool has_old,
                              uint32_t old_succ, bool whole_doc) {
    const int64_t action = s.action(row);
    // an unknown odd action carries no value and no object (like link); a null or unknown even action
    // is make-like, its object of type undefined / null (emptyObjectPatch gives it props)
    const int64_t idc = s.id_ctr(row);
    const int32_t ida = s.id_actor(row);
    const uint32_t cur_succ = has_old ? nsucc_at(f, lim) : 0u;
    // a new make* op: objectMeta[opId] and children[elemId][opId] (new.js:894-897)
    if (is_make(action) && obj_find(idc, ida) < 0) {
      const int32_t nm = obj_new(idc, ida, obj_type_of_action(action));
      if (nm < 0) return false;
      w.obj[nm].parent = ob;
      w.obj[nm].pk_row = row;
      const int32_t kd = kid_find(ob, row, true);
      if (kd < 0 || !kv_set(kd, idc, ida, 2, nm)) return false;
    }
    int32_t ps = pst_get(row, whole_doc);
    const bool first_op = ps < 0;
    if (ps < 0) {
      if (w.npst >= w.cap_pst) return fail(PATCH_U_CAPACITY);
      DPst& p = w.pst[w.npst];
      p.elem_row = row; p.vis_head = p.vis_tail = -1; p.has_child = 0; p.action = 0; p.cs_head = -1; p.cm_head = -1; p.next = -1;
      ps = (int32_t)w.npst++;
    }
    const bool overwritten = has_old && cur_succ > 0;
    if (!overwritten) {
      if (w.nvis >= w.cap_vis) return fail(PATCH_U_CAPACITY);
      w.vis[w.nvis].row = row;
      w.vis[w.nvis].next = -1;
      if (w.pst[ps].vis_tail >= 0) w.vis[w.pst[ps].vis_tail].next = (int32_t)w.nvis;
      else w.pst[ps].vis_head = (int32_t)w.nvis;
      w.pst[ps].vis_tail = (int32_t)w.nvis++;
      if (is_make(action)) w.pst[ps].has_child = 1;
    }
    const int32_t prev = kid_find(ob, row, false);
    if (w.pst[ps].has_child || (prev >= 0 && w.kid[prev].n > 0)) {
      const int32_t kd = kid_find(ob, row, true);
      if (kd < 0) return false;
      w.kid[kd].head = -1;  // children[elemId] = values
      w.kid[kd].n = 0;
      for (int32_t v = w.pst[ps].vis_head; v >= 0; v = w.vis[v].next) {
        const int32_t vr = w.vis[v].row;
        const int64_t va = s.action(vr);
        if (va == 1) {
          if (!kv_set(kd, s.id_ctr(vr), s.id_actor(vr), 1, vr)) return false;
        } else if (is_make(va)) {
          const int32_t co = obj_find(s.id_ctr(vr), s.id_actor(vr));
          if (co < 0) return fail(PATCH_U_VALUE);
          if (!kv_set(kd, s.id_ctr(vr), s.id_actor(vr), 2, co)) return false;
        }
      }
    }
    if (whole_doc) return true;  // documentPatch at load: only objectMeta is kept
    // patchKey / patchValue (new.js:933-977)
    bool have_pv = false;
    DVal pv = {};
    int64_t pk_c = 0;
    int32_t pk_a = 0;
    const int64_t tag = s.val_len(row);
    if (overwritten && action == 1 && (tag & 0x0f) == 8) {
      if (w.ncs >= w.cap_cs) return fail(PATCH_U_CAPACITY);
      int64_t cv;
      if (!s.value_int((uint32_t)row, false, cv)) return fail(PATCH_U_VALUE);
      const int32_t st = (int32_t)w.ncs++;
      DCs& c = w.cs[st];
      c.op_ctr = idc; c.op_actor = ida; c.value = cv; c.nleft = 0; c.next = -1; c.pad = 0;
      for (uint32_t k = 0; k < s.f_nsucc(f); k++) {
        if (s.f_succ_time(f, k) >= lim) continue;
        const int64_t sc = s.f_succ_ctr(f, k);
        const int32_t sa = s.f_succ_actor(f, k);
        int32_t q = w.pst[ps].cm_head;
        while (q >= 0 && !(w.cm[q].ctr == sc && w.cm[q].actor == sa)) q = w.cm[q].next;
        if (q < 0) {
          if (w.ncm >= w.cap_cm) return fail(PATCH_U_CAPACITY);
          q = (int32_t)w.ncm++;
          w.cm[q].ctr = sc; w.cm[q].actor = sa; w.cm[q].next = w.pst[ps].cm_head; w.cm[q].pad = 0;
          w.pst[ps].cm_head = q;
          c.nleft++;
        } else if (w.cm[q].state != st) {
          c.nleft++;  // counterStates[succOp] rebound to this counter; counted once per counter
        }
        w.cm[q].state = st;
      }
    } else if (action == 5) {
      int32_t q = w.pst[ps].cm_head;
      while (q >= 0 && !(w.cm[q].ctr == idc && w.cm[q].actor == ida)) q = w.cm[q].next;
      if (q < 0) return fail(PATCH_E_UNKNOWN_COUNTER, idc, ida);
      DCs& c = w.cs[w.cm[q].state];
      const uint32_t t15 = (uint32_t)(tag & 15);
      int64_t iv;
      if (tag < 16 || !(t15 == 3 || t15 == 4 || t15 == 8 || t15 == 9) || !s.value_int((uint32_t)row, t15 == 3, iv)) {
        // JS adds it as it is (a float, or a string concatenation, new.js:958): the replay goes on --
        // objectMeta does not depend on the value -- and the call reports PATCH_U_INC_VALUE at the end
        inc_nonint = true;
        iv = 0;
      }
      c.value += iv;
      c.nleft--;  // delete counterState.succs[opId]
      if (c.nleft == 0) {
        have_pv = true;
        pv.vtag = PV_COUNTER; pv.dt = 0; pv.v0 = c.value; pv.v1 = 0;
        pk_c = c.op_ctr; pk_a = c.op_actor;
      }
    } else if (!overwritten) {
      if (action == 1) {
        if (!row_val(row, pv)) return false;
        have_pv = true;
        pk_c = idc; pk_a = ida;
      } else if (is_make(action)) {
        const int32_t co = obj_find(idc, ida);
        if (co < 0) return fail(PATCH_U_VALUE);
        patch_on(co);
        pv = child_val(co);
        have_pv = true;
        pk_c = idc; pk_a = ida;
      }
    }
    patch_on(ob);
    if (!s.has_key(row)) {
      // list / text object (new.js:983-1033); the patch of an object of type undefined / null has no
      // edits array (emptyObjectPatch, new.js:726-732), where the reference stops with a TypeError
      if (w.obj[ob].type >= 4) return fail(PATCH_U_VALUE);
      const int64_t ec = elem_ctr(row);
      const int32_t ea = elem_actor(row);
      if (has_old && old_succ == 0 && w.pst[ps].action == 1) {
        w.pst[ps].action = 2;
        if (!convert_insert_to_update(ob, list_index, ec, ea)) return false;
      }
      if (have_pv) {
        if (!w.pst[ps].action && !has_old) {
          w.pst[ps].action = 1;
          DEdit e = {};
          e.action = PR_INSERT; e.index = list_index; e.ec = ec; e.ea = ea; e.oc = pk_c; e.oa = pk_a; e.v = pv;
          return append_edit(ob, e);
        } else if (w.pst[ps].action == 3) {
          const int32_t lt = w.obj[ob].edit_tail;
          if (lt < 0 || w.ed[lt].action != PR_REMOVE) return fail(PATCH_U_VALUE);  // 'last edit has unexpected type'
          if (w.ed[lt].count > 1) w.ed[lt].count--;
          else edit_pop(ob);
          w.pst[ps].action = 2;
          return append_update(ob, list_index, ec, ea, pk_c, pk_a, pv, true);
        } else {
          const bool fst = !w.pst[ps].action;
          if (!w.pst[ps].action) w.pst[ps].action = 2;
          return append_update(ob, list_index, ec, ea, pk_c, pk_a, pv, fst);
        }
      } else if (has_old && old_succ == 0 && !w.pst[ps].action) {
        w.pst[ps].action = 3;
        DEdit e = {};
        e.action = PR_REMOVE; e.index = list_index; e.count = 1;
        return append_edit(ob, e);
      }
      return true;
    }
    // map / table object (new.js:1035-1039)
    const int32_t pr = prop_get(ob, row, first_op);
    if (pr < 0) return false;
    if (have_pv) return prop_set(pr, pk_c, pk_a, pv);
    return true;
  }

  // ---- seekWithinBlock over the rows present before stream position W (new.js:50-192) ----
  struct Cur { int32_t f; };
  AM_PHD void cur_norm(Cur& c, int64_t W) const {
    while (c.f < (int32_t)s.nout() && rtime(s.frow(c.f)) >= W) c.f++;
  }
  AM_PHD int32_t cur_read(Cur& c, int64_t W) const {  // row, or -1 past the end (readValue -> null)
    cur_norm(c, W);
    if (c.f >= (int32_t)s.nout()) return -1;
    return s.frow(c.f++);
  }
  AM_PHD bool cur_done(Cur& c, int64_t W) const {
    cur_norm(c, W);
    return c.f >= (int32_t)s.nout();
  }
  AM_PHD void cur_skip(Cur& c, uint32_t k, int64_t W) const {
    for (uint32_t q = 0; q < k; q++)
      if (cur_read(c, W) < 0) break;
  }
  // (row, current succ count) of the next present row
  AM_PHD int32_t cur_read_succ(Cur& c, int64_t W, int64_t& nsucc) const {
    cur_norm(c, W);
    if (c.f >= (int32_t)s.nout()) { nsucc = -1; return -1; }
    nsucc = (int64_t)nsucc_at(c.f, W);
    return s.frow(c.f++);
  }

  // The seek of an op with object (q_oc, q_oa), key row `qrow` (or element (q_kc, q_ka) when
  // key_row < 0), insert flag and id. Returns false for 'Reference element not found'.
  AM_PHD bool seek(int64_t q_oc, int32_t q_oa, int32_t qrow, int64_t q_kc, int32_t q_ka, bool q_ins, int64_t q_idc,
                   int32_t q_ida, int64_t W, uint32_t& skip, int64_t& vis) const {
    Cur objA{0}, objC{0}, keyS{0}, idA{0}, idC{0}, ins{0}, act{0}, succ{0};
    skip = 0;
    vis = 0;
    bool elem_visible = false;
    int64_t n_oc = -1;
    int32_t n_oa = -1;
    if (q_oc >= 0) {
      while (!cur_done(objC, W) || !cur_done(objA, W) || !cur_done(act, W)) {
        const int32_t a = cur_read(objC, W), b = cur_read(objA, W);
        n_oc = a >= 0 ? s.obj_ctr(a) : -1;
        n_oa = b >= 0 ? s.obj_actor(b) : -1;
        cur_read(act, W);
        if (n_oc < 0 || n_oa < 0 || n_oc < q_oc || (n_oc == q_oc && act_lt(n_oa, q_oa))) skip++;
        else break;
      }
    }
    if (n_oc != q_oc || n_oa != q_oa) return true;
    if (qrow >= 0 && s.has_key(qrow)) {
      cur_skip(keyS, skip, W);
      while (!cur_done(keyS, W)) {
        const int32_t a = cur_read(objA, W), b = cur_read(objC, W), k = cur_read(keyS, W);
        const int32_t noa = a >= 0 ? s.obj_actor(a) : -1;
        const int64_t noc = b >= 0 ? s.obj_ctr(b) : -1;
        if (s.has_key(k) && s.key_cmp(k, qrow) < 0 && noc == q_oc && noa == q_oa) skip++;
        else break;
      }
      return true;
    }
    cur_skip(idC, skip, W); cur_skip(idA, skip, W); cur_skip(ins, skip, W); cur_skip(succ, skip, W);
    int64_t n_idc = -1;
    int32_t n_ida = -1;
    bool n_ins = false;
    int64_t n_succ = -1;  // -1: null
    auto rd_id = [&]() {
      const int32_t a = cur_read(idC, W), b = cur_read(idA, W);
      n_idc = a >= 0 ? s.id_ctr(a) : -1;
      n_ida = b >= 0 ? s.id_actor(b) : -1;
    };
    auto rd_obj = [&]() {
      const int32_t a = cur_read(objC, W), b = cur_read(objA, W);
      n_oc = a >= 0 ? s.obj_ctr(a) : -1;
      n_oa = b >= 0 ? s.obj_actor(b) : -1;
    };
    auto rd_ins_succ = [&]() {
      const int32_t a = cur_read(ins, W);
      n_ins = a >= 0 ? s.insert(a) : false;
      cur_read_succ(succ, W, n_succ);
    };
    auto visit = [&]() {
      if (n_ins) elem_visible = false;
      if (n_succ == 0 && !elem_visible) { vis++; elem_visible = true; }
    };
    rd_id();
    rd_ins_succ();
    if (q_ins) {
      if (q_kc > 0 && q_ka >= 0) {
        skip++;
        while (!cur_done(idC, W) && !cur_done(idA, W) && (n_idc != q_kc || n_ida != q_ka)) {
          visit();
          rd_id();
          rd_obj();
          rd_ins_succ();
          if (n_oc == q_oc && n_oa == q_oa) skip++;
          else break;
        }
        if (n_oc != q_oc || n_oa != q_oa || n_idc != q_kc || n_ida != q_ka || !n_ins) return false;
        visit();
        if (cur_done(idC, W) || cur_done(idA, W)) return true;
        rd_id();
        rd_obj();
        rd_ins_succ();
      }
      for (;;) {
        const bool greater = n_idc >= 0 && (n_idc > q_idc || (n_idc == q_idc && act_lt(q_ida, n_ida)));
        if (!((!n_ins || greater) && n_oc == q_oc && n_oa == q_oa)) break;
        skip++;
        visit();
        if (!cur_done(idC, W) && !cur_done(idA, W)) {
          rd_id();
          rd_obj();
          rd_ins_succ();
        } else {
          break;
        }
      }
    } else if (q_kc > 0 && q_ka >= 0) {
      while ((!n_ins || n_idc != q_kc || n_ida != q_ka) && n_oc == q_oc && n_oa == q_oa) {
        skip++;
        visit();
        if (!cur_done(idC, W) && !cur_done(idA, W)) {
          rd_id();
          rd_obj();
          rd_ins_succ();
        } else {
          break;
        }
      }
      if (n_oc != q_oc || n_oa != q_oa || n_idc != q_kc || n_ida != q_ka || !n_ins) return false;
    }
    return true;
  }

  // ---- mergeDocChangeOps (new.js:1052-1290) for the window starting at stream index `pos` ----
  AM_PHD bool oid_add(int32_t ob) {
    for (uint32_t k = 0; k < w.noid; k++) if (w.oids[k] == ob) return true;
    if (w.noid >= w.cap_oid) return fail(PATCH_U_CAPACITY);
    w.oids[w.noid++] = ob;
    return true;
  }
  AM_PHD int32_t srow(uint32_t p) const { return (int32_t)(s.nb() + p); }  // stream index -> row

  AM_PHD bool apply_ops(uint32_t& pos, uint32_t pend) {
    const int64_t W = pos;  // rows present: time < W
    const int32_t first = srow(pos);
    const bool insert = s.insert(first);
    const int64_t f_oc = s.obj_ctr(first);
    const int32_t f_oa = s.obj_actor(first);
    uint32_t skip;
    int64_t visible;
    DPT();
    advance(W);
    DPA(0);
    if (!fast_seek(first, skip, visible) &&
        !seek(f_oc, f_oa, first, s.key_ctr(first), s.key_actor(first), insert, s.id_ctr(first), s.id_actor(first), W, skip,
              visible))
      return fail(PATCH_U_VALUE);  // Reference element not found (the merge reports it first)
    DPA(1);
    if (s.has_key(first)) visible = 0;
    int64_t list_index = visible;
    const int32_t ob = obj_find(f_oa < 0 ? -1 : f_oc, f_oa);
    if (ob < 0) return fail(PATCH_U_VALUE);  // objectMeta[objectId] undefined
    const int32_t author = s.id_actor(first);
    bool found_list_elem = false, elem_visible = false;
    w.npst = 0; w.nvis = 0; w.ncs = 0; w.ncm = 0;  // propState = {}
    // the first doc op: the present row after `skip` present rows
    Cur dc{(int32_t)skip < ptotal ? (int32_t)set_kth(w.bitp, (int32_t)skip + 1) : (int32_t)s.nout()};
    int32_t doc_f = dc.f < (int32_t)s.nout() ? dc.f : -1;  // F position of docOp, -1: null
    if (doc_f >= 0) dc.f++;
    uint32_t doc_old = doc_f >= 0 ? nsucc_at(doc_f, W) : 0u;
    uint32_t nc = 0, seen_top = 0;
    int32_t change_op = -1;
    bool have_lck = false;
    int32_t lck_row = -1;
    if (!oid_add(ob)) return false;
    DPA(2);
    for (;;) {
#if defined(AM_DIFF_CHECK) && defined(__HIP_DEVICE_COMPILE__)
      pacc[7]++;
#endif
      if (nc == 0) {
        found_list_elem = false;
        seen_top = 0;
        while (pos < pend) {
          const int32_t nx = srow(pos);
          if (!(s.id_actor(nx) == author && s.insert(nx) == insert && s.obj_ctr(nx) == f_oc && s.obj_actor(nx) == f_oa)) break;
          const int32_t last = nc > 0 ? w.cops[nc - 1] : -1;
          bool is_overwrite = false;
          for (uint32_t i = 0; i < s.npred(nx); i++)
            for (uint32_t k = 0; k < nc; k++)
              if (s.pred_actor(nx, i) == s.id_actor(w.cops[k]) && s.pred_ctr(nx, i) == s.id_ctr(w.cops[k])) is_overwrite = true;
          const int32_t dr0 = doc_f >= 0 ? s.frow(doc_f) : -1;
          bool take = false;
          if (nx == first) take = true;
          else if (insert && last >= 0 && !s.has_key(nx) && s.key_actor(nx) == s.id_actor(last) && s.key_ctr(nx) == s.id_ctr(last))
            take = true;
          else if (!insert && last >= 0 && s.has_key(nx) && s.has_key(last) && s.key_eq(nx, last) && !is_overwrite)
            take = true;
          else if (!insert && last >= 0 && !s.has_key(nx) && !s.has_key(last) && s.key_actor(nx) == s.key_actor(last) &&
                   s.key_ctr(nx) == s.key_ctr(last) && !is_overwrite)
            take = true;
          else if (!insert && last < 0 && !s.has_key(nx) && dr0 >= 0 && s.insert(dr0) && !s.has_key(dr0) &&
                   s.id_actor(dr0) == s.key_actor(nx) && s.id_ctr(dr0) == s.key_ctr(nx))
            take = true;
          else if (!insert && last < 0 && s.has_key(nx) && have_lck && s.key_cmp(lck_row, nx) < 0)
            take = true;
          if (!take) break;
          have_lck = s.has_key(nx);
          lck_row = nx;
          if (nc >= w.cap_cops || seen_top + s.npred(nx) > w.cap_seen) return fail(PATCH_U_CAPACITY);
          w.cops[nc] = nx;
          w.seen_off[nc] = seen_top;
          for (uint32_t k = 0; k < s.npred(nx); k++) w.seen[seen_top + k] = 0;
          seen_top += s.npred(nx);
          nc++;
          pos++;  // readNextChangeOp
        }
      }
      DPA(3);
      if (nc > 0) change_op = w.cops[0];
      const int32_t dr = doc_f >= 0 ? s.frow(doc_f) : -1;
      const bool in_obj = dr >= 0 && s.obj_actor(dr) == s.obj_actor(change_op) && s.obj_ctr(dr) == s.obj_ctr(change_op);
      const bool key_matches = dr >= 0 && s.has_key(dr) && s.has_key(change_op) && s.key_eq(dr, change_op);
      const bool elem_matches = dr >= 0 && !s.has_key(dr) && !s.has_key(change_op) &&
                                ((!s.insert(dr) && s.key_actor(dr) == s.key_actor(change_op) && s.key_ctr(dr) == s.key_ctr(change_op)) ||
                                 (s.insert(dr) && s.id_actor(dr) == s.key_actor(change_op) && s.id_ctr(dr) == s.key_ctr(change_op)));
      if (nc == 0 && !(in_obj && (key_matches || elem_matches))) break;
      bool take_doc = false;
      uint32_t take_chg = 0;
      if (insert || !in_obj || (!s.has_key(dr) && s.has_key(change_op)) ||
          (s.has_key(dr) && s.has_key(change_op) && s.key_cmp(change_op, dr) < 0)) {
        take_chg = nc;
        if (!in_obj && !found_list_elem && !s.has_key(change_op) && !s.insert(change_op))
          return fail(PATCH_U_VALUE);  // 'could not find list element with ID'
      } else if (key_matches || elem_matches || found_list_elem) {
        // the doc op gains every pulled op whose pred names it (its succ list as of `pos`)
        for (uint32_t oi = 0; oi < nc; oi++) {
          const int32_t op = w.cops[oi];
          for (uint32_t i = 0; i < s.npred(op); i++)
            if (s.pred_actor(op, i) == s.id_actor(dr) && s.pred_ctr(op, i) == s.id_ctr(dr)) {
              w.seen[w.seen_off[oi] + i] = 1;
              break;
            }
        }
        if (elem_matches) found_list_elem = true;
        if (found_list_elem && !elem_matches) {
          take_chg = nc;
        } else if (nc == 0 || s.id_ctr(dr) < s.id_ctr(change_op) ||
                   (s.id_ctr(dr) == s.id_ctr(change_op) && act_lt(s.id_actor(dr), author))) {
          take_doc = true;
          if (!update_property(ob, dr, doc_f, (int64_t)pos, list_index, true, doc_old, false)) return false;
          // a deletion whose preds have all been seen leaves no row (new.js:1205-1217)
          for (uint32_t i = nc; i-- > 0;) {
            const int32_t op = w.cops[i];
            bool deleted = true;
            for (uint32_t j = 0; j < s.npred(op); j++) if (!w.seen[w.seen_off[i] + j]) deleted = false;
            if (s.action(op) == 3 && deleted) {
              for (uint32_t k = i; k + 1 < nc; k++) { w.cops[k] = w.cops[k + 1]; w.seen_off[k] = w.seen_off[k + 1]; }
              nc--;
            }
          }
        } else if (s.id_ctr(dr) == s.id_ctr(change_op) && s.id_actor(dr) == author) {
          return fail(PATCH_U_VALUE);  // duplicate operation ID (the merge reports it first)
        } else {
          take_chg = 1;
        }
      } else {
        take_doc = true;
      }
      DPA(4);
      if (take_doc) {
        if (s.insert(dr) && elem_visible) { elem_visible = false; list_index++; }
        if (nsucc_at(doc_f, (int64_t)pos) == 0) elem_visible = true;
        dc.f = next_present(dc.f);
        doc_f = dc.f < (int32_t)s.nout() ? dc.f : -1;
        if (doc_f >= 0) { dc.f++; doc_old = nsucc_at(doc_f, W); }
      }
      DPA(5);
      if (take_chg > 0) {
        for (uint32_t i = 0; i < take_chg; i++) {
          const int32_t op = w.cops[i];
          for (uint32_t j = 0; j < s.npred(op); j++)
            if (!w.seen[w.seen_off[i] + j]) return fail(PATCH_U_VALUE);  // no matching operation for pred
          if (!update_property(ob, op, -1, (int64_t)pos, list_index, false, 0, false)) return false;
          if (s.insert(op)) { elem_visible = false; list_index++; }
          else elem_visible = true;
        }
        for (uint32_t k = 0; k + take_chg < nc; k++) { w.cops[k] = w.cops[k + take_chg]; w.seen_off[k] = w.seen_off[k + take_chg]; }
        nc -= take_chg;
      }
      DPA(6);
    }
    return true;
  }

  // ---- objectMeta after documentPatch of the base document (new.js:1604-1635) ----
  AM_PHD bool build_meta() {
    if (obj_new(-1, -1, 0) < 0) return false;
    int64_t last_oc = -2;
    int32_t last_oa = -2;
    bool elem_visible = false;
    int64_t list_index = 0;
    int32_t ob = 0;
    w.npst = 0; w.nvis = 0; w.ncs = 0; w.ncm = 0;
    const uint32_t nm = s.nmeta_rows();
#if defined(__HIP_DEVICE_COMPILE__)
    // wide: only the rows of key / element groups (runs of one key or element in one object) that
    // hold a make op reach update_property -- in whole-document mode it changes nothing for the rest
    // (no objectMeta entry, no children snapshot; propState is matched against its last entry only,
    // and a group never recurs in its object). Group starts go to cops, the make flags to tmp.
    if constexpr (Wide) {
      const uint32_t l = wave::lane_id();
      DCHKF(14, nm);
      for (uint32_t r = l; r < nm; r += 64) w.tmp[r] = 0;
      int32_t carry = 0;
      for (uint32_t base = 0; base < nm; base += 64) {
        const uint32_t r = base + l;
        const bool in = r < nm;
        const bool st = in && (r == 0 || s.obj_ctr((int32_t)r) != s.obj_ctr((int32_t)r - 1) ||
                               s.obj_actor((int32_t)r) != s.obj_actor((int32_t)r - 1) || !elem_eq((int32_t)r - 1, (int32_t)r));
        const uint64_t sm = __ballot(st || !in);
        const uint64_t upto = l == 63 ? sm : sm & ((2ull << l) - 1);
        const int32_t g = upto ? (int32_t)base + 63 - __builtin_clzll(upto) : carry;
        if (in) w.cops[r] = g;
        carry = wave::bcast(g, 63);
      }
      __syncthreads();
      for (uint32_t r = l; r < nm; r += 64)
        if (is_make(s.action((int32_t)r))) w.tmp[w.cops[r]] = 1;
      __syncthreads();
    }
#endif
    uint32_t mbase = 0;
    uint64_t mmask = 0;
    bool mset = false;
    auto next_row = [&](uint32_t i) -> uint32_t {  // the next row at or after i that update_property needs
#if defined(__HIP_DEVICE_COMPILE__)
      if constexpr (Wide) {
        while (i < nm) {
          if (!mset || i < mbase || i >= mbase + 64) {
            mset = true;
            mbase = i;
            const uint32_t r = i + wave::lane_id();
            mmask = __ballot(r < nm && w.tmp[w.cops[r]] != 0);
          }
          const uint64_t rest = mmask & (~0ull << (i - mbase));
          if (rest) return mbase + (uint32_t)__builtin_ctzll(rest);
          i = mbase + 64;
        }
        return nm;
      }
#endif
      return i;
    };
    for (uint32_t i = next_row(0); i < nm; i = next_row(i + 1)) {
      const int32_t r = (int32_t)i;
      const int64_t oc = s.obj_ctr(r);
      const int32_t oa = s.obj_actor(r);
      if (oc != last_oc || oa != last_oa) {
        last_oc = oc; last_oa = oa;
        w.npst = 0; w.nvis = 0; w.ncs = 0; w.ncm = 0;
        list_index = 0;
        elem_visible = false;
        ob = obj_find(oa < 0 ? -1 : oc, oa);
        if (ob < 0) return fail(PATCH_U_VALUE);
      }
      const int32_t f = w.fpos[r];
      if (f < 0) return fail(PATCH_U_VALUE);
      const uint32_t ns = nsucc_at(f, 0);
      if (s.insert(r) && elem_visible) { elem_visible = false; list_index++; }
      if (ns == 0) elem_visible = true;
      if (!update_property(ob, r, f, 0, list_index, true, ns, true)) return false;
    }
    return true;
  }

  // ---- setupPatches (new.js:1461-1528) ----
  AM_PHD bool setup_patches() {
    for (uint32_t oi = 0; oi < w.noid; oi++) {
      int32_t ob = w.oids[oi], child = -1;
      bool exists = false;
      for (;;) {
        int32_t kids = -1;
        bool has_children = false;
        if (child >= 0) {
          kids = kid_find(ob, w.obj[child].pk_row, false);
          if (kids < 0) return fail(PATCH_U_VALUE);
          has_children = w.kid[kids].n > 0;
        }
        patch_on(ob);
        if (child >= 0 && has_children) {
          if (w.obj[ob].type == 1 || w.obj[ob].type == 2) {
            for (int32_t e = w.obj[ob].edit_tail; e >= 0; e = w.ed[e].prev) {
              const DEdit& ed = w.ed[e];
              if (ed.action != PR_INSERT && ed.action != PR_UPDATE) continue;  // edit.opId
              for (int32_t k = w.kid[kids].head; k >= 0; k = w.kv[k].next)
                if (w.kv[k].ctr == ed.oc && w.kv[k].actor == ed.oa) exists = true;
            }
            if (!exists) {
              // seekToOp of an update of the element (parentKey) over the final document
              uint32_t skip;
              int64_t vis;
              const int32_t pk = w.obj[child].pk_row;
              if (!seek(w.obj[ob].ctr, w.obj[ob].actor, -1, elem_ctr(pk), elem_actor(pk), false, 0, -1,
                        (int64_t)s.nrows(), skip, vis))
                return fail(PATCH_U_VALUE);
              for (int32_t k = w.kid[kids].head; k >= 0; k = w.kv[k].next) {
                DVal v;
                if (w.kv[k].kind == 2) { patch_on(w.kv[k].ref); v = child_val(w.kv[k].ref); }
                else if (!row_val(w.kv[k].ref, v)) return false;
                DEdit e = {};
                e.action = PR_UPDATE; e.index = vis; e.oc = w.kv[k].ctr; e.oa = w.kv[k].actor; e.v = v;
                if (!append_edit(ob, e)) return false;
              }
            }
          } else {
            const int32_t pr = prop_get(ob, w.obj[child].pk_row, false);
            if (pr < 0) return false;
            for (int32_t k = w.kid[kids].head; k >= 0; k = w.kv[k].next) {
              DVal v;
              if (w.kv[k].kind == 2) { patch_on(w.kv[k].ref); v = child_val(w.kv[k].ref); }
              else if (!row_val(w.kv[k].ref, v)) return false;
              bool existed = false;
              if (!prop_set(pr, w.kv[k].ctr, w.kv[k].actor, v, &existed)) return false;
              if (existed) exists = true;
            }
          }
        }
        if (exists || w.obj[ob].parent < 0 || (child >= 0 && !has_children)) break;
        child = ob;
        ob = w.obj[ob].parent;
      }
    }
    return true;
  }

  // ---- the log ----
  AM_PHD bool emit() {
    for (uint32_t a = 0; a < s.nactors(); a++) {
      PatchRec r = {};
      r.tag = PR_ACTOR;
      const uint32_t l = s.actor_len(a);
      if (o.nheap + l > o.cap_heap) return fail(PATCH_U_CAPACITY);
      s.copy_actor(a, o.heap + o.nheap);
      r.v0 = (int64_t)o.nheap; r.v1 = l; r.a1 = (int32_t)a;
      o.nheap += l;
      if (!patch_push(o, r)) { ok = false; return false; }
    }
    for (uint32_t c = 0; c < s.nchg(); c++) {  // clock: last seq per actor, first-appearance order
      bool later = false;
      for (uint32_t d = c + 1; d < s.nchg() && !later; d++) later = s.chg_actor(d) == s.chg_actor(c);
      if (later) continue;
      PatchRec r = {};
      r.tag = PR_CLOCK; r.a1 = (int32_t)s.chg_actor(c); r.index = s.chg_seq(c);
      if (!patch_push(o, r)) { ok = false; return false; }
    }
    for (uint32_t ob = 0; ob < w.nobj; ob++) {
      const DObj& d = w.obj[ob];
      if (!d.has_patch) continue;
      PatchRec h = {};
      h.tag = PR_OBJ; h.c1 = d.ctr; h.a1 = d.actor; h.dt = (uint32_t)d.type;
      if (!patch_push(o, h)) { ok = false; return false; }
      for (int32_t p = d.prop_head; p >= 0; p = w.prop[p].next) {
        PatchRec k = {};
        k.tag = PR_KEY;
        const uint32_t kl = s.key_len(w.prop[p].key_row);
        if (o.nheap + kl > o.cap_heap) return fail(PATCH_U_CAPACITY);
        s.copy_key(w.prop[p].key_row, o.heap + o.nheap);
        k.v0 = (int64_t)o.nheap; k.v1 = kl;
        o.nheap += kl;
        if (!patch_push(o, k)) { ok = false; return false; }
        for (int32_t e = w.prop[p].head; e >= 0; e = w.pe[e].next) {
          PatchRec r = {};
          r.tag = PR_PROP; r.c2 = w.pe[e].ctr; r.a2 = w.pe[e].actor;
          r.vtag = w.pe[e].v.vtag; r.dt = w.pe[e].v.dt; r.v0 = w.pe[e].v.v0; r.v1 = w.pe[e].v.v1;
          if (!patch_push(o, r)) { ok = false; return false; }
        }
      }
      uint32_t ne = 0;
      for (int32_t e = d.edit_tail; e >= 0; e = w.ed[e].prev) {
        DCHKF(13, ne);
        w.tmp[ne++] = e;
      }
      for (uint32_t q = ne; q-- > 0;) {
        const DEdit& e = w.ed[w.tmp[q]];
        PatchRec r = {};
        r.tag = e.action; r.index = e.index;
        if (e.action == PR_REMOVE) {
          r.n = (uint32_t)e.count;
        } else if (e.action == PR_MULTI) {
          r.c1 = e.ec; r.a1 = e.ea; r.dt = e.mdt; r.n = e.nmv;
          uint32_t nv = 0;  // values, oldest first
          for (int32_t m = e.mv_tail; m >= 0 && nv < e.nmv; m = w.mv[m].prev) {
            DCHKF(13, ne + nv);
            w.tmp[ne + nv++] = m;
          }
          for (uint32_t k = nv; k-- > 0;) {
            const DVal& v = w.mv[w.tmp[ne + k]].v;
            if (!patch_push_val(o, v.vtag, v.dt, v.v0, v.v1)) { ok = false; return false; }
          }
        } else {
          r.c1 = e.ec; r.a1 = e.ea; r.c2 = e.oc; r.a2 = e.oa;
          r.vtag = e.v.vtag; r.dt = e.v.dt; r.v0 = e.v.v0; r.v1 = e.v.v1;
        }
        if (!patch_push(o, r)) { ok = false; return false; }
      }
    }
    return true;
  }

  // ---- objectMeta carried across calls on one handle (new.js:1812, 1857) ----
  // The reference keeps objectMeta per BackendDoc: documentPatch fills it at load (new.js:1748),
  // then every applyChanges call updates the children snapshots of the keys its
  // updatePatchProperty calls visit. A handle that has run a call hands its snapshots back in
  // (meta_restore); the objects themselves (parent, parentKey, type) follow from the make ops.
  AM_PHD bool build_objects() {
    if (obj_new(-1, -1, 0) < 0) return false;
    const uint32_t nm = s.nmeta_rows();
    for (uint32_t base = 0; base < nm; base += 64) {
      uint64_t mm = ~0ull;  // the chunk's make rows (wide: one ballot; serial: each row tested below)
#if defined(__HIP_DEVICE_COMPILE__)
      if constexpr (Wide) mm = __ballot(base + wave::lane_id() < nm && is_make(s.action((int32_t)(base + wave::lane_id()))));
#endif
      for (; mm; mm &= mm - 1) {
      const uint32_t i = base + (uint32_t)__builtin_ctzll(mm);
      if (i >= nm) break;
      const int32_t r = (int32_t)i;
      const int64_t a = s.action(r);
      if (!is_make(a)) continue;
      if (obj_find(s.id_ctr(r), s.id_actor(r)) >= 0) continue;
      const int32_t oa = s.obj_actor(r);
      const int32_t ob = obj_find(oa < 0 ? -1 : s.obj_ctr(r), oa);
      if (ob < 0) return fail(PATCH_U_VALUE);
      const int32_t no = obj_new(s.id_ctr(r), s.id_actor(r), obj_type_of_action(a));
      if (no < 0) return false;
      w.obj[no].parent = ob;
      w.obj[no].pk_row = r;
      }
    }
    return true;
  }
  AM_PHD static bool meta_uleb(const uint8_t* m, uint32_t len, uint32_t& off, uint32_t& v) {
    v = 0;
    for (uint32_t sh = 0; sh < 35; sh += 7) {
      if (off >= len) return false;
      const uint8_t b = m[off++];
      v |= (uint32_t)(b & 0x7f) << sh;
      if (!(b & 0x80)) return true;
    }
    return false;
  }
  // the blob of diff_meta_pack: "AMM1", uleb count, per key: uleb object (0 _root, else 1 + row of
  // its make op), uleb row of the key (its elemId), uleb n, n x uleb row of a visible op. Rows are
  // base rows: the document order of the call that wrote the blob.
  AM_PHD bool meta_restore(const uint8_t* m, uint32_t len) {
    if (len < 4 || m[0] != 'A' || m[1] != 'M' || m[2] != 'M' || m[3] != '1') return fail(PATCH_U_VALUE);
    uint32_t off = 4, nk;
    if (!meta_uleb(m, len, off, nk)) return fail(PATCH_U_VALUE);
    for (uint32_t k = 0; k < nk; k++) {
      uint32_t orow, erow, n;
      if (!meta_uleb(m, len, off, orow) || !meta_uleb(m, len, off, erow) || !meta_uleb(m, len, off, n) || erow >= s.nb() ||
          orow > s.nb())
        return fail(PATCH_U_VALUE);
      const int32_t ob = orow == 0 ? 0 : obj_find(s.id_ctr((int32_t)orow - 1), s.id_actor((int32_t)orow - 1));
      if (ob < 0) return fail(PATCH_U_VALUE);
      const int32_t kd = kid_find(ob, (int32_t)erow, true);
      if (kd < 0) return false;
      w.kid[kd].head = -1;
      w.kid[kd].n = 0;
      for (uint32_t q = 0; q < n; q++) {
        uint32_t vr;
        if (!meta_uleb(m, len, off, vr) || vr >= s.nb()) return fail(PATCH_U_VALUE);
        const int32_t r = (int32_t)vr;
        const int64_t a = s.action(r);
        if (a == 1) {
          if (!kv_set(kd, s.id_ctr(r), s.id_actor(r), 1, r)) return false;
        } else if (is_make(a)) {
          const int32_t co = obj_find(s.id_ctr(r), s.id_actor(r));
          if (co < 0) return fail(PATCH_U_VALUE);
          if (!kv_set(kd, s.id_ctr(r), s.id_actor(r), 2, co)) return false;
        } else {
          return fail(PATCH_U_VALUE);
        }
      }
    }
    return off == len || fail(PATCH_U_VALUE);
  }

  const uint8_t* meta_in = nullptr;  // the handle's snapshots, null: documentPatch's (load / init)
  uint32_t meta_len = 0;
  bool meta_mode = false;
  bool inc_nonint = false;  // a non-integer counter increment was met (its patch value is unknown)

  AM_PHD bool run() {
    DCHKF(11, s.nrows() ? s.nrows() - 1 : 0);
#if defined(AM_DIFF_CHECK) && defined(__HIP_DEVICE_COMPILE__)
    const uint64_t prof6 = clock64();
#endif
    uint32_t l0 = 0, step = 1;  // wide: the lanes split the per-row loops
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (Wide) { l0 = wave::lane_id(); step = 64; }
#endif
    for (uint32_t r = l0; r < s.nrows(); r += step) w.fpos[r] = -1;
    DSYNC();
    for (uint32_t f = l0; f < s.nout(); f += step) {
      DCHKF(11, s.frow((int32_t)f));
      w.fpos[s.frow((int32_t)f)] = (int32_t)f;
    }
    DSYNC();
#if defined(AM_DIFF_CHECK) && defined(__HIP_DEVICE_COMPILE__)
#define DPROF(k) prof[k] = clock64()
    uint64_t prof[7];
#else
#define DPROF(k)
#endif
    DPROF(0);
    if (meta_mode && meta_in) {
      if (!build_objects() || !meta_restore(meta_in, meta_len)) return false;
    } else if (!build_meta()) {
      return false;
    }
    DPROF(1);
    fast_init();
    if (!ok) return false;
    DPROF(2);
    uint32_t pos = 0, ncalls = 0;
    (void)ncalls;
    const uint32_t nstream = s.nrows() - s.nb();
    for (uint32_t p = 0; p < s.npass() && ok; p++) {
      const uint32_t pend = s.pass_end(p) < nstream ? s.pass_end(p) : nstream;
      while (pos < pend && ok) {
        ncalls++;
        if (!apply_ops(pos, pend)) return false;
      }
    }
    DPROF(3);
    if (!setup_patches()) return false;
    DPROF(4);
    const bool r = emit();
    if (r && ok && inc_nonint) o.status = PATCH_U_INC_VALUE;
    DPROF(5);
#if defined(AM_DIFF_CHECK) && defined(__HIP_DEVICE_COMPILE__)
    if (((s.nrows() > 1100 && s.nrows() < 1104) || s.nrows() > 20000) && (!Wide || wave::lane_id() == 0))
      printf("[p8prof] wide %d rows %u out %u stream %u merge-calls %u loops %llu: fpos %llu meta %llu init %llu ops %llu setup %llu emit %llu"
             " | advance %llu seek %llu start %llu pull %llu match+doc-upd %llu doc-next %llu chg-upd %llu cycles\n",
             (int)Wide, s.nrows(), s.nout(), nstream, ncalls, (unsigned long long)pacc[7], (unsigned long long)(prof[0] - prof6),
             (unsigned long long)(prof[1] - prof[0]), (unsigned long long)(prof[2] - prof[1]),
             (unsigned long long)(prof[3] - prof[2]), (unsigned long long)(prof[4] - prof[3]), (unsigned long long)(prof[5] - prof[4]),
             (unsigned long long)pacc[0], (unsigned long long)pacc[1], (unsigned long long)pacc[2], (unsigned long long)pacc[3],
             (unsigned long long)pacc[4], (unsigned long long)pacc[5], (unsigned long long)pacc[6]);
#endif
    return r;
  }
};

// meta: the call keeps objectMeta for its handle (restored from meta_in when given, documentPatch's
// otherwise); diff_meta_pack then writes what the call leaves.
template <bool Wide = false, class Src>
AM_PHD inline bool diff_scan(const Src& src, PatchOut& o, DiffScratch& w, bool meta = false, const uint8_t* meta_in = nullptr,
                             uint32_t meta_len = 0) {
  o.nrec = o.nmval = o.nheap = 0;
  o.status = 0;
  o.arg0 = o.arg1 = 0;
  Diff<Src, Wide> d(src, w, o);
  d.meta_mode = meta;
  d.meta_in = meta_in;
  d.meta_len = meta_len;
  return d.run();
}

// The children snapshots objectMeta holds after a successful diff_scan, as the blob meta_restore
// reads (rows = positions in this call's merged document order, the next call's base rows).
// Returns the bytes written, 0 when cap is too small or a snapshot names a row the merged document
// does not keep.
template <class Src>
AM_PHD inline uint64_t diff_meta_pack(const Src& s, const DiffScratch& w, uint8_t* dst, uint64_t cap) {
  uint64_t n = 4;
  bool ok = true;
  auto put = [&](uint64_t v) {
    const uint32_t l = pk_uleb_len(v);
    if (n + l > cap) { ok = false; return; }
    pk_uleb(dst + n, v);
    n += l;
  };
  auto frow = [&](int32_t row) -> uint64_t {
    const int32_t f = row >= 0 && (uint32_t)row < s.nrows() ? w.fpos[row] : -1;
    if (f < 0) ok = false;
    return f < 0 ? 0 : (uint64_t)f;
  };
  if (cap < 4) return 0;
  dst[0] = 'A'; dst[1] = 'M'; dst[2] = 'M'; dst[3] = '1';
  uint64_t nk = 0;
  for (uint32_t ob = 0; ob < w.nobj; ob++)
    for (int32_t k = w.obj[ob].kids; k >= 0; k = w.kid[k].next) nk++;
  put(nk);
  for (uint32_t ob = 0; ob < w.nobj && ok; ob++)
    for (int32_t k = w.obj[ob].kids; k >= 0 && ok; k = w.kid[k].next) {
      put(w.obj[ob].actor < 0 ? 0 : 1 + frow(w.obj[ob].pk_row));
      put(frow(w.kid[k].elem_row));
      put((uint64_t)w.kid[k].n);
      for (int32_t e = w.kid[k].head; e >= 0 && ok; e = w.kv[e].next)
        put(frow(w.kv[e].kind == 2 ? w.obj[w.kv[e].ref].pk_row : w.kv[e].ref));
    }
  return ok ? n : 0;
}
