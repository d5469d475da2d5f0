// am_doc_fast.h -- k_doc_fast: the merge of a small document with its op rows, changes, entries
// and columns held one per lane (one wave per document, one document per workgroup).
//
// This is the common case of Backend.load + Backend.applyChanges (backend/new.js:1550-1597,
// 1695-1871): every change of the call applies in list order during the first pass of the
// causal queue, and the document has at most 64 op rows, 64 pred/succ entries, 64 change rows,
// 64 actor references and 64 dependencies. Anything else -- a change that waits in the queue, a
// duplicate, any reference or range error, a value outside 31 bits, a getPatch request -- leaves
// fast_done[doc] = 0 and the document is merged by k_doc (am_doc_impl.h), which reports the
// reference's exact error. The sort keys are the ones k_doc sorts by (object, UTF-16 key |
// RGA position, opId; succ order of new.js:1173-1188) and the encoders produce the canonical
// RLE / delta / boolean forms of encoding.js:558-1207, so documents merged here are byte-for-byte
// the documents k_doc (and the reference) produce. tests/test_gpu_parity.py runs every golden
// scenario through both paths.
//
// Per document, everything lives in the wave's LDS slice and in registers:
//   input   the document's chunk bytes (16-byte loads of [span_lo, span_hi))
//   hashes  change hashes | base heads | host-known hashes, 32 B each (word compares)
//   refs    actor references: base actors, then every change's actor list
//   chg     parsed change headers
//   misc    small per-document tables (DocHdr, ranks, sort results, succ lists)
//   cells   decoded column values (4 B per value); reused as the output image afterwards
#pragma once

// Probe builds (-DAM_PHASE_CLOCK, tools/build_probe.sh): lane 0 of every 16th document adds the
// s_memtime delta of each phase to am_phase_cycles[16 + k]
#ifdef AM_PHASE_CLOCK
#define FPH(k)                                                                        \
  do {                                                                                \
    if (l == 0 && (doc & 15) == 0) {                                                  \
      const uint64_t now_ = clock64();                                                \
      atomicAdd(&am_phase_cycles[16 + (k)], (unsigned long long)(now_ - ph_last));    \
      ph_last = now_;                                                                 \
    }                                                                                 \
  } while (0)
#elif defined(FD_STOP)
// probe builds (tools/build_stop.sh): the kernel returns after phase FD_STOP, so PMC counters of
// the variants give the instructions of each phase
#define FPH(k)                   \
  do {                           \
    if ((k) == FD_STOP) return;  \
  } while (0)
#else
#define FPH(k) \
  do {         \
  } while (0)
#endif

#include "am_wave.h"

#define FD_MAX 64
#define FD_SPAN_MAX 8192
#define FD_LDS_CAP (24 * 1024)
// documents (waves) per workgroup: with one, the LDS slices pack per wave, so the occupancy is
// floor(160 KB / slice) waves per CU (C4, 11.2 KB: 14) instead of whole 4-document groups (12)
#ifndef FD_DOCS_PER_WG
#define FD_DOCS_PER_WG 1
#endif
#define FD_NULL ((int32_t)0x80000000)
#define FD_DIFF_SCRATCH 1216  // fast_diff's tables in the cells region
#define FD_REC_BYTES 1024     // FdRec's row words (key, objc, idc, vlen) at the end of the cells region

// misc region (byte offsets). Tables whose phases never overlap share a union slot:
//   U2: {CLOCK, FIRST} (actor table .. queue) | {SRCR, SRCE} (decode .. rows) | {CNTN} (succ)
// The 64-bit tables live in the cells region while it is free of decoded cells: the base heads' /
// known hashes' indexes (BHIDX, KIDX) before the decode, the sorted op ids (IDT) and the succ
// sort (NSORT, BENT) between the row gather and the encode; FdRec's row words at its end.
enum : uint32_t {
  FM_DH = 0,                      // DocHdrC (128 B)
  FM_U2 = 128,                    // 512 B union
  FM_CLOCK = FM_U2,               //   uint32 [64] base clock per doc actor
  FM_FIRST = FM_U2 + 256,         //   uint32 [64] first change authored by a canonical ref
  FM_SRCR = FM_U2,                //   int32 [64] row -> source marks
  FM_SRCE = FM_U2 + 256,          //   int32 [64] entry -> source marks
  FM_CNTN = FM_U2,                //   uint32 [64] new succs per target row
  FM_OUTC = FM_U2 + 512,          // int32 [64] output succ ctr
  FM_ROW0 = FM_OUTC + 256,        // uint8 [65] first row of each source (<= 64 rows)
  FM_ENT0 = FM_ROW0 + 80,         // uint8 [65] first entry of each source (<= 64 entries)
  FM_COLLEN = FM_ENT0 + 80,       // uint32 [32] encoded column lengths
  FM_OWN = FM_COLLEN + 128,       // uint8 [64] owner row of each entry
  FM_CANON = FM_OWN + 64,         // uint8 [64] canonical ref of each ref
  FM_RANKC = FM_CANON + 64,       // uint8 [64] rank of each canonical ref
  FM_DPC = FM_RANKC + 64,         // uint8 [64] doc actor index of each canonical ref
  FM_DP2REF = FM_DPC + 64,        // uint8 [64] doc actor index -> ref
  FM_RANKDP = FM_DP2REF + 64,     // uint8 [64] doc actor index -> rank
  FM_OPR = FM_RANKDP + 64,        // uint8 [64] row -> opId rank
  FM_FC = FM_OPR + 64,            // int8 [64] first child (RGA)
  FM_NS = FM_FC + 64,             // int8 [64] next sibling (RGA)
  FM_LON = FM_NS + 64,            // uint8 [64] first sorted new succ of each target row
  FM_DEPD = FM_LON + 64,          // uint8 [64] head candidate (change | base head, N + HB <= 64) is depended on
  FM_OUTA = FM_DEPD + 64,         // uint8 [64] output succ actor
  FM_DOWN = FM_OUTA + 64,         // uint8 [64] owner change of each dep slot
  FM_HSEL = FM_DOWN + 64,         // uint8 [64] hash-table slot of each sorted head
  FM_HIDX = FM_HSEL + 64,         // int32 [64] sorted heads' indexes
  FM_TOTAL = FM_HIDX + 256
};

struct FastLayout {
  uint32_t input, hashes, refs, misc, chg, cells, cells_cap, total, rw;
  uint32_t bk;      // BHIDX (int64 per base head), then KIDX (int64 per known hash), in the cells region
  uint32_t ob_cap;  // bytes of the cells region the output image / patch scratch may use (FdRec after)
};

// Per-document LDS slice of k_doc_fast (bytes, 16-aligned regions).
__host__ __device__ inline FastLayout fast_layout(const DocBounds& b, uint32_t nknown) {
  FastLayout F;
  uint32_t o = 0;
  auto take = [&](uint32_t n) { const uint32_t at = o; o += (n + 15) & ~15u; return at; };
  const uint32_t span = (uint32_t)(b.span_hi - b.span_lo);
  const uint32_t nbh = b.H - b.N, nrefs = (b.A - b.N) + b.AM;
  const uint32_t nht = b.N + nbh + nknown;
  F.input = take(span + 32);
  F.refs = take(8 * nrefs);  // (off, len) per ref
  F.misc = take(FM_TOTAL);
  F.chg = 0;  // change headers: read from k_chunks' slots in global memory
  const uint32_t nbc = b.C - b.N, nbd = b.D - b.ND;
  uint32_t cells = 4 * (13 * b.R + 2 * b.E);
  // until the op columns are decoded the cells region holds the hash table (changes | base heads |
  // known), then the refs' 32 B id words (actor table) and later the base change rows over them
  const uint32_t dcc = 8 * (9 * nbc + nbd), rwb = 32 * nrefs;
  const uint32_t bk = 32 * nht + (dcc > rwb ? dcc : rwb);
  const uint32_t early = bk + 8 * (nbh + nknown);
  if (early > cells) cells = early;
  if (cells < 1024) cells = 1024;  // IDT | NSORT, BENT
  // output image: header (actors, heads, column table) + columns + heads indexes + extra bytes
  // (a larger image fails the encoder's capacity check: the document then goes to k_doc). With a
  // patch requested, FdRec's row words take the last FD_REC_BYTES: the image gets the rest.
  const uint32_t out = 64 + 40 * b.A + 42 * b.H + 25 * 12 + span;
  if (out > cells) cells = out;
  if (b.P && cells < FD_DIFF_SCRATCH + FD_REC_BYTES) cells = FD_DIFF_SCRATCH + FD_REC_BYTES;
  F.cells = take(cells);
  F.cells_cap = cells;
  F.ob_cap = b.P ? cells - FD_REC_BYTES : cells;
  F.hashes = F.cells;
  F.rw = F.cells + 32 * nht;
  F.bk = F.cells + bk;
  F.total = o;
  return F;
}

__host__ __device__ inline bool fast_eligible(const DocBounds& b, const am_doc_desc& dd) {
  // getPatch logs: fast_getpatch; applyChanges patches: fast_diff (both fall back to k_doc)
  if (dd.flags & (AM_DOC_FIX_UTF8 | AM_DOC_PATCH_ROOM)) return false;
  if (b.B == 0 || doc_scattered(b) || b.UC) return false;
  if (dd.base_chunk < 0 && dd.chg_count == 0) return false;
  if (b.span_hi - b.span_lo > FD_SPAN_MAX) return false;
  if (b.R > FD_MAX || b.E > FD_MAX || b.C > FD_MAX || b.N > FD_MAX || b.D > FD_MAX || b.ND > FD_MAX || b.H > FD_MAX)
    return false;
  if (dd.known_count > FD_MAX || b.N + (b.H - b.N) + dd.known_count > 2 * FD_MAX) return false;
  if ((b.A - b.N) + b.AM > FD_MAX) return false;
  return fast_layout(b, dd.known_count).total <= FD_LDS_CAP;
}

namespace fastdoc {
using lds_mode::kEncKind;
using lds_mode::EK_U;
using lds_mode::EK_D;
using lds_mode::EK_S;
using lds_mode::EK_B;
using lds_mode::EK_W;

__device__ __forceinline__ uint32_t lane() { return threadIdx.x & 63; }
// a value every lane of the wave holds equally, moved to a scalar register (readfirstlane)
__device__ __forceinline__ uint32_t uni(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
// Orders this wave's LDS accesses (a wave's DS instructions execute in order; this stops the
// compiler from moving them across a cross-lane hand-off)
__device__ __forceinline__ void wsync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}
__device__ __forceinline__ uint64_t lt_mask() {
  const uint32_t l = lane();
  return l ? (~0ull >> (64 - l)) : 0ull;
}
__device__ __forceinline__ uint32_t ctz64(uint64_t m) { return m ? (uint32_t)__builtin_ctzll(m) : 64u; }
using wave::excl_add;
using wave::incl_max;
using wave::max_all;
using wave::sum_all;
using wave::sort64;
__device__ __forceinline__ bool words_eq(const uint32_t* a, const uint32_t* b) {
  const uint4 a0 = reinterpret_cast<const uint4*>(a)[0], a1 = reinterpret_cast<const uint4*>(a)[1];
  const uint4 b0 = reinterpret_cast<const uint4*>(b)[0], b1 = reinterpret_cast<const uint4*>(b)[1];
  return ((a0.x ^ b0.x) | (a0.y ^ b0.y) | (a0.z ^ b0.z) | (a0.w ^ b0.w) | (a1.x ^ b1.x) | (a1.y ^ b1.y) | (a1.z ^ b1.z) |
          (a1.w ^ b1.w)) == 0;
}
// 32 input bytes -> 8 little-endian words (hash compares; LDS bytes, any alignment)
__device__ __forceinline__ void load32(const uint8_t* p, uint32_t w[8]) {
#pragma unroll
  for (int k = 0; k < 8; k++)
    w[k] = (uint32_t)p[4 * k] | (uint32_t)p[4 * k + 1] << 8 | (uint32_t)p[4 * k + 2] << 16 | (uint32_t)p[4 * k + 3] << 24;
}
__device__ __forceinline__ uint64_t bswap64(uint64_t x) { return __builtin_bswap64(x); }

// ---- 32-bit column stream decoder (RLEDecoder / DeltaDecoder / BooleanDecoder,
// encoding.js:789-1207) specialised by column type at compile time. Every lane of a decode round
// runs the same type, so the wave executes one record state machine instead of the union of
// four. Anything the fast envelope does not cover -- a value outside 31 bits, a non-canonical
// record, a truncated stream -- only raises `bad`: the document then goes to k_doc, which
// reports the reference's exact error. ----
struct Dec32 {
  uint32_t off, end;  // byte offsets into the staged input
  int32_t count;      // values left in the current record
  int32_t last;       // repeated / last literal value (utf8: offset << 8 | length)
  int64_t abs;        // delta running value
  uint8_t state;      // 0 none, 1 repetition, 2 literal, 3 nulls
  bool has_last, last_null;
};
__device__ __forceinline__ void d32_init(Dec32& d, uint32_t off, uint32_t len) {
  d.off = off; d.end = off + len; d.count = 0; d.last = 0; d.abs = 0;
  d.state = 0; d.has_last = false; d.last_null = false;
}
// unsigned LEB128 < 2^31 (anything else is outside the envelope)
__device__ __forceinline__ uint32_t d32_uleb(const uint8_t* in, Dec32& d, bool& bad) {
  uint32_t v = 0;
  for (uint32_t sh = 0; sh < 35; sh += 7) {
    if (d.off >= d.end) { bad = true; return 0; }
    const uint32_t b = in[d.off++];
    v |= (b & 0x7f) << sh;
    if (!(b & 0x80)) {
      if (sh == 28 && (b & 0x78)) bad = true;  // >= 2^31
      if (b == 0 && sh) bad = true;            // over-long: let k_doc judge it
      return v;
    }
  }
  bad = true;
  return 0;
}
// signed LEB128 in (-2^31, 2^31)
__device__ __forceinline__ int32_t d32_sleb(const uint8_t* in, Dec32& d, bool& bad) {
  uint32_t v = 0;
  for (uint32_t sh = 0; sh < 35; sh += 7) {
    if (d.off >= d.end) { bad = true; return 0; }
    const uint32_t b = in[d.off++];
    v |= (b & 0x7f) << sh;
    if (!(b & 0x80)) {
      const uint32_t used = sh + 7;
      if (used < 32 && (b & 0x40)) v |= ~0u << used;
      if (sh == 28) {
        // the fifth byte carries bits 28..34: in range iff they all equal the sign bit
        if ((b & 0x78) != 0 && (b & 0x78) != 0x78) bad = true;
      }
      if ((int32_t)v == INT32_MIN) bad = true;
      return (int32_t)v;
    }
  }
  bad = true;
  return 0;
}
template <uint8_t T>
__device__ __forceinline__ int32_t d32_raw(const uint8_t* in, Dec32& d, bool& bad) {
  if constexpr (T == DT_UTF8) {
    const uint32_t len = d32_uleb(in, d, bad);
    const uint32_t at = d.off;
    if (len > 255 || d.off + len > d.end) { bad = true; return 0; }
    d.off += len;
    return (int32_t)((at << 8) | len);
  } else if constexpr (T == DT_UINT) {
    return (int32_t)d32_uleb(in, d, bad);
  } else {
    return d32_sleb(in, d, bad);
  }
}
template <uint8_t T>
__device__ __forceinline__ bool d32_eq(const uint8_t* in, int32_t a, int32_t b) {
  if constexpr (T == DT_UTF8) {
    const uint32_t al = (uint32_t)a & 255, bl = (uint32_t)b & 255;
    if (al != bl) return false;
    const uint32_t ao = (uint32_t)a >> 8, bo = (uint32_t)b >> 8;
    for (uint32_t q = 0; q < al; q++)
      if (in[ao + q] != in[bo + q]) return false;
    return true;
  } else {
    return a == b;
  }
}
// next value of an RLE stream: FD_NULL for nulls (and past the end, RLEDecoder.readValue)
template <uint8_t T>
__device__ __forceinline__ int32_t d32_next(const uint8_t* in, Dec32& d, bool& bad) {
  if (d.count == 0) {
    if (d.off == d.end) return FD_NULL;
    const int32_t c = d32_sleb(in, d, bad);
    if (c > 1) {
      const int32_t v = d32_raw<T>(in, d, bad);
      if ((d.state == 1 || d.state == 2) && d.has_last && !d.last_null && d32_eq<T>(in, v, d.last)) bad = true;
      d.state = 1; d.last = v; d.has_last = true; d.last_null = false; d.count = c;
    } else if (c < 0) {
      if (d.state == 2) bad = true;
      d.state = 2; d.count = -c;
    } else if (c == 0) {
      if (d.state == 3) bad = true;
      const uint32_t z = d32_uleb(in, d, bad);
      if (z == 0) bad = true;
      d.state = 3; d.has_last = true; d.last_null = true; d.count = (int32_t)z;
    } else {
      bad = true;  // a repetition of one
    }
    if (bad) { d.count = 0; d.off = d.end; return FD_NULL; }
  }
  d.count--;
  if (d.state == 2) {
    const int32_t v = d32_raw<T>(in, d, bad);
    if (d.has_last && !d.last_null && d32_eq<T>(in, v, d.last)) bad = true;
    d.last = v; d.has_last = true; d.last_null = false;
    return v;
  }
  return d.last_null ? FD_NULL : d.last;
}
// one op-column stream [off, off + len) -> n cells
template <uint8_t T>
__device__ __forceinline__ void d32_stream(const uint8_t* in, uint32_t off, uint32_t len, uint32_t n, int32_t* dst,
                                           bool& bad) {
  Dec32 d;
  d32_init(d, off, len);
  if constexpr (T == DT_BOOL) {
    bool cur = true, first = true;
    for (uint32_t i = 0; i < n; i++) {
      if (d.count == 0 && d.off == d.end) { dst[i] = 0; continue; }  // past the end: false
      while (d.count == 0) {
        const uint32_t c = d32_uleb(in, d, bad);
        cur = !cur;
        if (c == 0 && !first) bad = true;
        first = false;
        d.count = (int32_t)c;
        if (bad) break;
      }
      if (bad) return;
      d.count--;
      dst[i] = cur ? 1 : 0;
    }
  } else {
    for (uint32_t i = 0; i < n; i++) {
      const int32_t v = d32_next<T>(in, d, bad);
      if (bad) return;
      if (v == FD_NULL) { dst[i] = FD_NULL; continue; }
      if constexpr (T == DT_DELTA) {
        d.abs += v;
        if (d.abs <= -0x7fffffffLL || d.abs > 0x7fffffffLL) { bad = true; return; }
        dst[i] = (int32_t)d.abs;
      } else {
        dst[i] = v;
      }
    }
  }
}

// Canonical column encoder over the values of lanes [0, n) (one value per lane, wave-parallel):
// runs of equal adjacent values -> repetition / null / literal records (RLEEncoder,
// encoding.js:558-783), deltas against the previous non-null value (DeltaEncoder :932-951),
// alternating run counts (BooleanEncoder :1061-1135), concatenated raw bytes (valRaw). Writes
// the column at `out` and returns its length, or ~0u when it would exceed `cap`.
//   v: value (U / D / B), isnull; S: string bytes at in + soff (len slen), eqs = equal to the
//   previous lane's string; W: raw bytes at in + soff (len slen).
__device__ __forceinline__ uint32_t enc_col(uint8_t kind, uint32_t n, int64_t v, bool isnull, uint32_t soff, uint32_t slen, bool eqs,
                            const uint8_t* in, uint8_t* out, uint32_t cap) {
  if (n == 0) return 0;
  const uint32_t l = lane();
  const bool act = l < n;
  const bool nul = act && isnull && kind != EK_W && kind != EK_B;
  if (kind == EK_D) {
    const int32_t pi = incl_max(act && !nul ? (int32_t)l : -1);
    int32_t prev = wave::up1(pi, -1);
    if (l == 0) prev = -1;
    const int64_t pv = __shfl(v, prev < 0 ? 0 : prev, 64);
    if (act && !nul) v -= prev < 0 ? 0 : pv;
  }
  const int64_t pv = wave::up1(v, (int64_t)0);
  const int32_t pn = wave::up1((int32_t)nul, 0);
  bool same = false;
  if (act && l > 0 && kind != EK_W) {
    if (nul) same = pn != 0;
    else if (pn) same = false;
    else same = (kind == EK_S) ? eqs : (pv == v);
  }
  const bool st = act && !same;
  const uint64_t M = __ballot(st);
  const uint64_t above = l == 63 ? 0ull : (M >> (l + 1));
  const uint32_t rl = (above ? l + 1 + ctz64(above) : n) - l;
  uint32_t bytes = 0, gcnt = 0;
  bool gs = false;
  if (kind == EK_W) {
    bytes = act ? slen : 0;
  } else if (kind == EK_B) {
    bytes = st ? (uint32_t)uleb_len(rl) + ((l == 0 && v) ? 1u : 0u) : 0u;
  } else {
    if (!__any(act && !nul)) return 0;  // nulls only: nothing is written (RLEEncoder.finish)
    const bool single = st && !nul && rl == 1;
    const uint64_t SM = __ballot(single);
    gs = single && !(l > 0 && ((SM >> (l - 1)) & 1));
    gcnt = gs ? ctz64(~(SM >> l)) : 0;
    uint32_t vs = 0;
    if (kind == EK_U) vs = uleb_len((uint64_t)v);
    else if (kind == EK_D) vs = sleb_len(v);
    else vs = uleb_len(slen) + slen;
    if (st) {
      if (nul) bytes = 1 + uleb_len(rl);
      else if (rl >= 2) bytes = sleb_len((int64_t)rl) + vs;
      else bytes = vs + (gs ? (uint32_t)sleb_len(-(int64_t)gcnt) : 0u);
    }
  }
  uint32_t total;
  const uint32_t off = excl_add(bytes, total);
  if (total > cap) return ~0u;
  if (bytes) {
    uint8_t* o = out + off;
    if (kind == EK_W) {
      for (uint32_t q = 0; q < slen; q++) o[q] = in[soff + q];
    } else if (kind == EK_B) {
      if (l == 0 && v) *o++ = 0;
      put_uleb(o, rl);
    } else if (nul) {
      *o++ = 0;
      put_uleb(o, rl);
    } else {
      if (rl >= 2) o = put_sleb(o, (int64_t)rl);
      else if (gs) o = put_sleb(o, -(int64_t)gcnt);
      if (kind == EK_U) put_uleb(o, (uint64_t)v);
      else if (kind == EK_D) put_sleb(o, v);
      else {
        o = put_uleb(o, slen);
        for (uint32_t q = 0; q < slen; q++) o[q] = in[soff + q];
      }
    }
  }
  return total;
}

// LEB128 lengths in closed form (32-bit): ceil(significant bits / 7), bits / 7 as (x * 37) >> 8
__device__ __forceinline__ uint32_t uleb_len32(uint32_t v) { return ((32u - __clz(v | 1u) + 6u) * 37u) >> 8; }
__device__ __forceinline__ uint32_t sleb_len32(int32_t v) {
  return ((33u - __clz((uint32_t)(v ^ (v >> 31))) + 6u) * 37u) >> 8;
}
__device__ __forceinline__ uint8_t* put_uleb32(uint8_t* o, uint32_t v) {
  const uint32_t n = uleb_len32(v);
  for (uint32_t k = 0; k + 1 < n; k++) o[k] = (uint8_t)(((v >> (7 * k)) & 0x7f) | 0x80);
  o[n - 1] = (uint8_t)(v >> (7 * (n - 1)));
  return o + n;
}
__device__ __forceinline__ uint8_t* put_sleb32(uint8_t* o, int32_t v) {
  const uint32_t n = sleb_len32(v);
  for (uint32_t k = 0; k + 1 < n; k++) o[k] = (uint8_t)(((v >> (7 * k)) & 0x7f) | 0x80);
  o[n - 1] = (uint8_t)((v >> (7 * (n - 1))) & 0x7f);
  return o + n;
}
// enc_col for 31-bit values with the column kind fixed at compile time (op columns and every
// document change column but time). Unsigned / delta inputs must be >= 0 (else `bad`).
template <uint8_t K>
__device__ __forceinline__ uint32_t enc32(uint32_t n, int32_t v, bool isnull, uint32_t soff, uint32_t slen, bool eqs,
                                          const uint8_t* in, uint8_t* out, uint32_t cap, bool& bad) {
  if (n == 0) return 0;
  const uint32_t l = lane();
  const bool act = l < n;
  const bool nul = (K == EK_W || K == EK_B) ? false : (act && isnull);
  if constexpr (K == EK_U || K == EK_D) {
    if (act && !nul && v < 0) bad = true;
  }
  if constexpr (K != EK_W && K != EK_B) {
    if (!__any(act && !nul)) return 0;  // nulls only: nothing is written (RLEEncoder.finish)
  }
  if constexpr (K == EK_U || K == EK_S) {
    // one value n times: a single repetition (n >= 2) or literal (n == 1) record, written by lane 0
    const int32_t v0 = wave::bcast(v, 0);
    const bool differs = act && (nul || (K == EK_U ? v != v0 : (l > 0 && !eqs)));
    if (!__any(differs)) {
      const uint32_t sl0 = K == EK_S ? wave::bcast(slen, 0) : 0u;
      const uint32_t vs0 = K == EK_U ? uleb_len32((uint32_t)v0) : uleb_len32(sl0) + sl0;
      const uint32_t total = (n >= 2 ? sleb_len32((int32_t)n) : 1u) + vs0;
      if (total > cap) return ~0u;
      if (l == 0) {
        uint8_t* o = put_sleb32(out, n >= 2 ? (int32_t)n : -1);
        if constexpr (K == EK_U) put_uleb32(o, (uint32_t)v0);
        else {
          o = put_uleb32(o, sl0);
          for (uint32_t q = 0; q < sl0; q++) o[q] = in[soff + q];
        }
      }
      return total;
    }
  }
  if constexpr (K == EK_D) {
    const int32_t pi = incl_max(act && !nul ? (int32_t)l : -1);
    const int32_t prev = wave::up1(pi, -1);
    const int32_t pv = __shfl(v, prev < 0 ? 0 : prev, 64);
    if (act && !nul) v -= prev < 0 ? 0 : pv;
  }
  const int32_t pv = wave::up1(v, 0);
  const uint32_t pn = wave::up1((uint32_t)nul, 0u);
  bool same = false;
  if (K != EK_W && act && l > 0) {
    if (nul) same = pn != 0;
    else if (pn) same = false;
    else if constexpr (K == EK_S) same = eqs;
    else same = pv == v;
  }
  const bool st = act && !same;
  const uint64_t M = __ballot(st);
  const uint64_t above = l == 63 ? 0ull : (M >> (l + 1));
  const uint32_t rl = (above ? l + 1 + ctz64(above) : n) - l;
  uint32_t bytes = 0, gcnt = 0;
  bool gs = false;
  if constexpr (K == EK_W) {
    bytes = act ? slen : 0;
  } else if constexpr (K == EK_B) {
    bytes = st ? uleb_len32(rl) + ((l == 0 && v) ? 1u : 0u) : 0u;
  } else {
    const bool single = st && !nul && rl == 1;
    const uint64_t SM = __ballot(single);
    gs = single && !(l > 0 && ((SM >> (l - 1)) & 1));
    gcnt = gs ? ctz64(~(SM >> l)) : 0;
    uint32_t vs;
    if constexpr (K == EK_U) vs = uleb_len32((uint32_t)v);
    else if constexpr (K == EK_D) vs = sleb_len32(v);
    else vs = uleb_len32(slen) + slen;
    if (st) {
      if (nul) bytes = 1 + uleb_len32(rl);
      else if (rl >= 2) bytes = sleb_len32((int32_t)rl) + vs;
      else bytes = vs + (gs ? sleb_len32(-(int32_t)gcnt) : 0u);
    }
  }
  uint32_t total;
  const uint32_t off = excl_add(bytes, total);
  if (total > cap) return ~0u;
  if (bytes) {
    uint8_t* o = out + off;
    if constexpr (K == EK_W) {
      for (uint32_t q = 0; q < slen; q++) o[q] = in[soff + q];
    } else if constexpr (K == EK_B) {
      if (l == 0 && v) *o++ = 0;
      put_uleb32(o, rl);
    } else {
      if (nul) {
        *o++ = 0;
        put_uleb32(o, rl);
      } else {
        if (rl >= 2) o = put_sleb32(o, (int32_t)rl);
        else if (gs) o = put_sleb32(o, -(int32_t)gcnt);
        if constexpr (K == EK_U) put_uleb32(o, (uint32_t)v);
        else if constexpr (K == EK_D) put_sleb32(o, v);
        else {
          o = put_uleb32(o, slen);
          for (uint32_t q = 0; q < slen; q++) o[q] = in[soff + q];
        }
      }
    }
  }
  return total;
}
// enc32 for four narrow columns at once: each 16-lane DPP row encodes its own column (U or D kind,
// n <= 16 values, lane p of the row holds value p). Scans, neighbour moves and run searches stay
// inside the row (row_shr DPP, the row's 16 bits of a ballot). Returns the row's column length, or
// ~0u when it would exceed `cap`.
template <uint8_t K>
__device__ __forceinline__ uint32_t enc32r(uint32_t n, int32_t v, bool isnull, uint8_t* out, uint32_t cap, bool& bad) {
  static_assert(K == EK_U || K == EK_D, "row encoder: integer kinds");
  const uint32_t l = lane(), p = l & 15, rb = l & ~15u;
  const bool act = p < n;
  const bool nul = act && isnull;
  if (act && !nul && v < 0) bad = true;
  if constexpr (K == EK_D) {
    const int32_t I = INT32_MIN;
    int32_t pi = act && !nul ? (int32_t)p : -1;
    pi = max(pi, wave::dpp<wave::ROW_SHR1>(I, pi));
    pi = max(pi, wave::dpp<wave::ROW_SHR2>(I, pi));
    pi = max(pi, wave::dpp<wave::ROW_SHR4>(I, pi));
    pi = max(pi, wave::dpp<wave::ROW_SHR8>(I, pi));
    const int32_t prev = wave::dpp<wave::ROW_SHR1>(-1, pi);  // last non-null position before p
    const int32_t pv = __shfl(v, (int)(rb + (prev < 0 ? 0u : (uint32_t)prev)), 64);
    if (act && !nul) v -= prev < 0 ? 0 : pv;
  }
  const int32_t pv = wave::dpp<wave::ROW_SHR1>(0, v);
  const uint32_t pn = wave::dpp<wave::ROW_SHR1>(0u, (uint32_t)nul);
  bool same = false;
  if (act && p > 0) {
    if (nul) same = pn != 0;
    else if (pn) same = false;
    else same = pv == v;
  }
  const bool st = act && !same;
  const uint32_t rowm = (uint32_t)(__ballot(st) >> rb) & 0xffffu;
  const uint32_t above = rowm >> (p + 1);
  const uint32_t rl = (above ? p + 1 + (uint32_t)__builtin_ctz(above) : n) - p;
  const bool row_any = ((uint32_t)(__ballot(act && !nul) >> rb) & 0xffffu) != 0;
  const bool single = st && !nul && rl == 1;
  const uint32_t srow = (uint32_t)(__ballot(single) >> rb) & 0xffffu;
  const bool gs = single && !(p > 0 && ((srow >> (p - 1)) & 1));
  const uint32_t gcnt = gs ? (uint32_t)__builtin_ctz(~(srow >> p)) : 0u;
  const uint32_t vs = K == EK_U ? uleb_len32((uint32_t)v) : sleb_len32(v);
  uint32_t bytes = 0;
  if (st && row_any) {
    if (nul) bytes = 1 + uleb_len32(rl);
    else if (rl >= 2) bytes = sleb_len32((int32_t)rl) + vs;
    else bytes = vs + (gs ? sleb_len32(-(int32_t)gcnt) : 0u);
  }
  uint32_t x = bytes;
  x += wave::dpp<wave::ROW_SHR1>(0u, x);
  x += wave::dpp<wave::ROW_SHR2>(0u, x);
  x += wave::dpp<wave::ROW_SHR4>(0u, x);
  x += wave::dpp<wave::ROW_SHR8>(0u, x);
  const uint32_t total = (uint32_t)__shfl((int)x, (int)(rb + 15), 64);
  if (total > cap) return ~0u;
  if (bytes) {
    uint8_t* o = out + (x - bytes);
    if (nul) {
      *o++ = 0;
      put_uleb32(o, rl);
    } else {
      if (rl >= 2) o = put_sleb32(o, (int32_t)rl);
      else if (gs) o = put_sleb32(o, -(int32_t)gcnt);
      if constexpr (K == EK_U) put_uleb32(o, (uint32_t)v);
      else put_sleb32(o, v);
    }
  }
  return total;
}
__device__ __forceinline__ uint32_t enc32k(uint8_t kind, uint32_t n, int32_t v, bool isnull, uint32_t soff, uint32_t slen,
                                           bool eqs, const uint8_t* in, uint8_t* out, uint32_t cap, bool& bad) {
  switch (kind) {
    case EK_U: return enc32<EK_U>(n, v, isnull, soff, slen, eqs, in, out, cap, bad);
    case EK_D: return enc32<EK_D>(n, v, isnull, soff, slen, eqs, in, out, cap, bad);
    case EK_S: return enc32<EK_S>(n, v, isnull, soff, slen, eqs, in, out, cap, bad);
    case EK_B: return enc32<EK_B>(n, v, isnull, soff, slen, eqs, in, out, cap, bad);
    default: return enc32<EK_W>(n, v, isnull, soff, slen, eqs, in, out, cap, bad);
  }
}

// decodeValue (columnar.js:300-329) of a row's valLen / valRaw as the patch log carries it;
// strings and byte arrays point into the staged input (v0 = offset, v1 = length). false: the
// value raises an error (float length, integer range) -- k_doc reports it.
__device__ __forceinline__ bool fd_value(const uint8_t* in, int32_t vlen, uint32_t voff, uint32_t& vt, uint32_t& dt, int64_t& v0,
                                         int64_t& v1) {
  const uint32_t tag = vlen == FD_NULL ? 0u : (uint32_t)vlen;
  dt = 0;
  v0 = v1 = 0;
  if (tag <= 2) { vt = PV_NULL + tag; return true; }
  const uint32_t t = tag & 15, len = tag >> 4;
  if (t == 5) {
    if (len != 8) return false;
    uint64_t x = 0;
    for (int q = 0; q < 8; q++) x |= (uint64_t)in[voff + q] << (8 * q);
    v0 = (int64_t)x;
    vt = PV_F64;
    return true;
  }
  if (t == 3 || t == 4 || t == 8 || t == 9) {
    Rd rd{in + voff, len, 0};
    int64_t x;
    if ((t == 3 ? rd_u53(rd, x) : rd_i53(rd, x)) != AM_OK) return false;
    v0 = x;
    vt = t == 3 ? PV_UINT : t == 4 ? PV_INT : t == 8 ? PV_COUNTER : PV_TIMESTAMP;
    return true;
  }
  v0 = voff;
  v1 = len;
  vt = t == 6 ? PV_STR : PV_BYTES;
  dt = t == 6 ? 0u : t;
  return true;
}

// Row values of the merge that fast_diff reads back after the encode, in misc tables whose phases
// are over by then (U1, U2: opId sort .. succ merge; OWN .. DPC: refs .. entries; FC .. LON: RGA and
// succ merge; DEPD, DOWN: queue). FM_OPR (opId rank of each row) and FM_RANKDP stay as they are.
struct FdRec {
  uint32_t* key; int32_t* objc; int32_t* idc; int32_t* vlen;  // U1: 4 x 256 B
  uint16_t* voff;                                             // U2 + 0
  uint8_t *krow, *sck, *sok;                                  // U2 + 128 / 192 / 256 (by output position)
  int8_t* obja; uint8_t *ida, *krank;                         // U2 + 320 / 384 / 448
  uint32_t* bcs;                                              // OWN .. DPC (256 B): base change row -> seq
  int8_t* elem; uint8_t *act, *flags;                         // FC / NS / LON
  uint8_t *bca, *adp;                                         // DEPD: base change row -> actor; DOWN: change -> author
};
// U1: FD_REC_BYTES at the end of the cells region (after the output image / patch scratch)
__device__ __forceinline__ FdRec fd_rec(uint8_t* M, uint8_t* U1) {
  FdRec P;
  P.key = reinterpret_cast<uint32_t*>(U1);
  P.objc = reinterpret_cast<int32_t*>(U1 + 256);
  P.idc = reinterpret_cast<int32_t*>(U1 + 512);
  P.vlen = reinterpret_cast<int32_t*>(U1 + 768);
  P.voff = reinterpret_cast<uint16_t*>(M + FM_U2);
  P.krow = M + FM_U2 + 128; P.sck = M + FM_U2 + 192; P.sok = M + FM_U2 + 256;
  P.obja = reinterpret_cast<int8_t*>(M + FM_U2 + 320); P.ida = M + FM_U2 + 384; P.krank = M + FM_U2 + 448;
  P.bcs = reinterpret_cast<uint32_t*>(M + FM_OWN);
  P.elem = reinterpret_cast<int8_t*>(M + FM_FC); P.act = M + FM_NS; P.flags = M + FM_LON;
  P.bca = M + FM_DEPD; P.adp = M + FM_DOWN;
  return P;
}
static_assert(FM_CANON == FM_OWN + 64 && FM_RANKC == FM_CANON + 64 && FM_DPC == FM_RANKC + 64, "bcs spans OWN .. DPC");
static_assert(FM_U2 + 512 <= FM_OUTC, "U2 records");

// The patch Backend.applyChanges returns (new.js:1796-1871), written by the whole wave in wire form
// (am_patch.h) for the common shape of a batch of concurrent edits: every applied op is a `set` or
// an `inc` of a map key of the root object, or a `set` that inserts a list element into one
// list/text object whose make op is the only visible value of its root key. For that shape the
// serial replay of am_diff.h reduces to closed forms:
//   * props[key] comes from the last mergeDocChangeOps call over the key (each call resets it at the
//     key's first op, new.js:1037): the key's ops in opId order, except that when the call goes on
//     to a later key of the same change stream (new.js:1125-1128), the key's doc ops with an opId
//     above its last change op are taken without updatePatchProperty (new.js:1225-1230);
//   * of those ops a `set` without succ is a value; a counter `set` whose succs are all `inc` ops of
//     the key taken in that call is its value plus theirs (counterStates, new.js:937-965);
//   * an insert's index is the number of visible elements of the list that precede it in the
//     merged order and exist when it applies (base elements with a row without succ, earlier
//     inserts of the call): a popcount over row masks;
//   * appendEdit's multi-insert coalescing (new.js:747-782) joins an insert to the previous edit of
//     the list iff index, element counter and actor continue it with the same datatype and JS
//     type -- a segmented run over the insert lanes;
//   * setupPatches links the list to the root through its key (new.js:1461-1528).
// Anything else returns false before any result is committed and the document goes to k_doc,
// whose lane-0 replay covers every shape. Scratch: FD_DIFF_SCRATCH bytes at PS (the output image has
// left).
//
// objectMeta (AM_DOC_META, new.js:884-931, 1461-1528; am_diff.h meta_restore / diff_meta_pack): in this
// shape no call of updatePatchProperty rewrites a children snapshot -- a touched root key has only set /
// inc rows (a snapshot exists only for keys that have had a make op), a list element is a `set`, and
// the list's own key is not visited -- so the snapshots the call leaves are the ones it starts from,
// renumbered to the merged document order: the handle's blob (mblob), or documentPatch's of the base
// document when the handle has none (load / init: replayed per root key below). The closed form's
// link of the list to the root reads root.children[list key], which must then be exactly {make op};
// any other snapshot, a make op outside the root, or a snapshot of a touched key returns false.
__device__ __forceinline__ bool fast_diff(const uint8_t* IN, uint8_t* PS, uint32_t ps_cap, uint8_t* out, uint64_t out_cap,
                                          uint8_t* M, uint32_t R, uint32_t nb, uint32_t NOUT, uint32_t NA, uint32_t NC,
                                          uint32_t nbc, uint32_t N, const int32_t* OUTC, const uint8_t* OUTA, const uint32_t* RO,
                                          const ChgHdrC* chh, bool meta, const uint8_t* mblob, uint32_t mlen) {
  const FdRec P = fd_rec(M, PS + ps_cap);
  const uint32_t l = lane();
  const bool isrow_ = l < R;
  const int32_t r_key = isrow_ ? (int32_t)P.key[l] : FD_NULL, r_objc = isrow_ ? P.objc[l] : FD_NULL;
  const int32_t r_idc = isrow_ ? P.idc[l] : 0, r_vlen = isrow_ ? P.vlen[l] : FD_NULL;
  const uint32_t r_voff = isrow_ ? P.voff[l] : 0u;
  const int32_t r_obja = isrow_ ? P.obja[l] : -1, r_ida = isrow_ ? P.ida[l] : 0;
  const uint32_t r_krank = isrow_ ? P.krank[l] : 0u, r_opr = isrow_ ? M[FM_OPR + l] : 0u;
  const int32_t r_elem = isrow_ ? P.elem[l] : -1, r_act = isrow_ ? (int32_t)P.act[l] : 0;
  const uint32_t fl = isrow_ ? P.flags[l] : 0u;
  const bool r_chg = fl & 1, r_ins = (fl & 2) != 0, keyed = (fl & 4) != 0;
  const uint64_t r_objkey = (!isrow_ || r_objc == FD_NULL) ? 0ull
                                                          : (((uint64_t)(uint32_t)r_objc + 1) << 6) | (r_obja < 0 ? 0u : M[FM_RANKDP + r_obja]);
  const uint32_t k_row = l < NOUT ? P.krow[l] : 0u, sc_k = l < NOUT ? P.sck[l] : 0u, so_k = l < NOUT ? P.sok[l] : 0u;
  const uint32_t bc_actor = l < nbc ? P.bca[l] : 0u;
  const int64_t bc_seq = l < nbc ? (int64_t)P.bcs[l] : 0;
  const uint32_t a_dp = l < N ? P.adp[l] : 0u;
  const uint32_t a_off = l < NA ? RO[2 * M[FM_DP2REF + l]] : 0u, a_len = l < NA ? RO[2 * M[FM_DP2REF + l] + 1] : 0u;
  bool pbad = ps_cap < FD_DIFF_SCRATCH;
  if (__any(pbad)) return false;
  uint8_t* const POS = PS;        // row -> output position
  uint8_t* const SCR = PS + 64;   // row -> succ count in the merged document
  uint8_t* const EV = PS + 128;   // element (insert row) -> visible
  uint8_t* const TCH = PS + 192;  // key rank -> set / inc by a change op of the call
  uint32_t* const LASTC = reinterpret_cast<uint32_t*>(PS + 256);  // doc actor -> its last change row
  uint32_t* const LASTK = reinterpret_cast<uint32_t*>(PS + 512);  // key rank -> 1 + its last change row
  uint8_t* const CONT = PS + 768;  // key rank -> its last call goes on to a later key
  uint8_t* const LOPR = PS + 832;  // key rank -> opId rank of its last change op
  uint32_t* const COV = reinterpret_cast<uint32_t*>(PS + 896);  // row -> counter sets whose succ lists name it
  const bool isrow = l < R;
  EV[l] = 0;
  TCH[l] = 0;
  LASTC[l] = 0;
  LASTK[l] = 0;
  CONT[l] = 0;
  COV[l] = 0;
  wsync();
  if (l < NOUT) { POS[k_row] = (uint8_t)l; SCR[k_row] = (uint8_t)(sc_k > 255 ? 255 : sc_k); }
  const bool mod_root = r_chg && (r_act == 1 || r_act == 5) && keyed && r_objc == FD_NULL;
  const bool list_ins = r_chg && r_act == 1 && !keyed && r_ins;
  pbad |= r_chg && !(mod_root || list_ins);
  if (mod_root) {
    TCH[r_krank] = 1;
    atomicMax(&LASTK[r_krank], l + 1);
  }
  wsync();
  if (__any(pbad)) return false;
  // the call that holds a key's last change op goes on to the next change row (its stream successor)
  // when that row is by the same author, in the root, not an insert, with a greater key
  {
    const uint32_t nx = (l + 1) & 63;
    const int32_t n_ida = __shfl(r_ida, nx, 64), n_objc = __shfl(r_objc, nx, 64);
    const uint32_t n_kr = __shfl(r_krank, nx, 64);
    const int32_t n_chg = __shfl((int32_t)r_chg, nx, 64), n_ins = __shfl((int32_t)r_ins, nx, 64);
    const int32_t n_keyed = __shfl((int32_t)keyed, nx, 64);
    if (mod_root && LASTK[r_krank] == l + 1) {
      CONT[r_krank] = (l + 1 < R && n_chg && n_ida == r_ida && !n_ins && n_objc == FD_NULL && n_keyed && n_kr > r_krank) ? 1 : 0;
      LOPR[r_krank] = (uint8_t)r_opr;
    }
  }
  // visible elements: an element is visible while one of its rows has no succ (new.js:50-192)
  if (isrow && !r_chg && r_elem >= 0 && SCR[l] == 0) EV[r_elem] = 1;
  wsync();
  // the list object of the inserts: exactly one
  const uint64_t mli = __ballot(list_ins);
  const uint32_t f0 = mli ? ctz64(mli) : 0u;
  const uint64_t lkey = __shfl(r_objkey, f0, 64);
  const int32_t lc = __shfl(r_objc, f0, 64), la = __shfl(r_obja, f0, 64);
  pbad |= list_ins && r_objkey != lkey;
  // its make op M: a visible base row of a root key that no change touched, the key's only
  // visible value (objectMeta children of the root, new.js:894-930)
  const uint64_t mm = mli ? __ballot(isrow && r_idc == lc && r_ida == la) : 0ull;
  const uint32_t mrow = mm ? ctz64(mm) : 0u;
  const int32_t m_act = __shfl(r_act, mrow, 64), m_objc = __shfl(r_objc, mrow, 64), m_key = __shfl(r_key, mrow, 64);
  const uint32_t m_kr = __shfl(r_krank, mrow, 64);
  wsync();
  if (mli) {
    pbad |= l == 0 && (!mm || mrow >= nb || m_objc != FD_NULL || m_key == FD_NULL || (m_key & 255) == 0 ||
                       (m_act != 2 && m_act != 4) || SCR[mrow] != 0 || TCH[m_kr]);
    pbad |= isrow && r_objc == FD_NULL && keyed && r_krank == m_kr && l != mrow && SCR[l] == 0;
  }
  // the rows of a touched key are sets and increments (no child objects), keys non-empty
  const bool touched = isrow && keyed && r_objc == FD_NULL && TCH[r_krank];
  pbad |= touched && ((r_act != 1 && r_act != 5) || (r_key & 255) == 0);
  // ops of a touched key that its last call hands to updatePatchProperty
  const bool taken = touched && !(CONT[r_krank] && r_opr > LOPR[r_krank]);
  // objectMeta carried across calls: make ops only in the root (actions of ACTIONS or beyond, even)
  if (meta) pbad |= isrow && (r_act == 255 || ((r_act & 1) == 0 && (r_objc != FD_NULL || !keyed)));
  if (__any(pbad)) return false;

  // ---- counters (new.js:937-965): lane per succ entry of the merged document (entry q of output
  // position p = OWNE[q]); a counter set taken by its key's last call shows its value plus its
  // increments when every succ is an increment of the key that the call takes ----
  uint8_t* const OWNE = PS + 1152;  // succ entry -> output position of its owner
  const bool any_inc = __any(touched && r_act == 5);
  const uint32_t kr = k_row;        // output lane: its row
  const int32_t k_act = __shfl(r_act, kr, 64), k_vlen = __shfl(r_vlen, kr, 64);
  const int32_t k_touched = __shfl((int32_t)touched, kr, 64), k_taken = __shfl((int32_t)taken, kr, 64);
  const bool k_counter = l < NOUT && k_touched && k_taken && k_act == 1 && sc_k > 0 && k_vlen != FD_NULL && (k_vlen & 15) == 8;
  int64_t cnt_sum = 0;
  bool cnt_done = false;
  if (any_inc) {
    uint32_t nsucc_all;
    excl_add(l < NOUT ? sc_k : 0u, nsucc_all);
    if (l < NOUT)
      for (uint32_t j = 0; j < sc_k; j++) OWNE[so_k + j] = (uint8_t)l;
    wsync();
    const bool isent = l < nsucc_all;
    const uint32_t own = isent ? OWNE[l] : 0u;
    const int32_t ec = isent ? OUTC[l] : 0;
    const int32_t ea = isent ? (int32_t)OUTA[l] : -1;
    int32_t tgt = -1;  // the row with the entry's opId
    for (uint32_t j = 0; j < R; j++) {
      const int32_t jc = wave::bcast(r_idc, (int)j), ja = wave::bcast(r_ida, (int)j);
      if (isent && jc == ec && ja == ea) tgt = (int32_t)j;
    }
    pbad |= isent && tgt < 0;
    const uint32_t tu = tgt < 0 ? 0u : (uint32_t)tgt;
    const int32_t o_counter = __shfl((int32_t)k_counter, own, 64);
    const uint32_t o_kr = __shfl(r_krank, __shfl(kr, own, 64), 64);
    const int32_t t_act = __shfl(r_act, tu, 64), t_vlen = __shfl(r_vlen, tu, 64), t_taken = __shfl((int32_t)taken, tu, 64);
    const uint32_t t_kr = __shfl(r_krank, tu, 64), t_voff = __shfl(r_voff, tu, 64);
    const int32_t t_keyed = __shfl((int32_t)keyed, tu, 64), t_objc = __shfl(r_objc, tu, 64);
    const bool inc_of_key = isent && tgt >= 0 && t_act == 5 && t_keyed && t_objc == FD_NULL && t_kr == o_kr;
    if (isent && o_counter && inc_of_key) atomicAdd(&COV[tu], 1u);
    int64_t iv = 0;
    bool ok = isent && o_counter && inc_of_key && t_taken;
    if (ok) {
      uint32_t vt, dt;
      int64_t v1;
      const uint32_t t15 = t_vlen == FD_NULL ? 0u : ((uint32_t)t_vlen & 15);
      ok = (t15 == 3 || t15 == 4 || t15 == 8 || t15 == 9) && fd_value(IN, t_vlen, t_voff, vt, dt, iv, v1);
      pbad |= !ok;  // a non-integer increment (JS adds it as it is): k_doc replays it
    }
    // per counter owner: the sum of its increments, and whether any entry is not one (segmented
    // over the entry lanes of each owner)
    uint64_t owners = __ballot(k_counter);
    while (owners) {
      const uint32_t p = (uint32_t)__builtin_ctzll(owners);
      owners &= owners - 1;
      const bool mine = isent && own == p;
      int64_t sv = mine && ok ? iv : 0;
      uint32_t sb = mine && !ok ? 1u : 0u;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        sv += __shfl_xor(sv, o, 64);
        sb += __shfl_xor(sb, o, 64);
      }
      if (l == p) { cnt_sum = sv; cnt_done = sb == 0; }
    }
  }
  wsync();
  // every increment the last call takes is named by exactly one counter set of its key (else:
  // increment operation for unknown counter, or counterStates rebound -- k_doc replays it)
  pbad |= taken && r_act == 5 && COV[l] != 1;
  if (__any(pbad)) return false;

  // ---- record sizes; segments in stream order: actors, clock, root object, root keys, list ----
  // actors (PR_ACTOR)
  uint32_t tot;
  const uint32_t b_act = l < NA ? 1u + pk_uleb_len(a_len) + a_len : 0u;
  const uint32_t o_act = excl_add(b_act, tot);
  uint32_t base = tot;
  // clock (PR_CLOCK): each actor's last change row
  const uint32_t kc = l >= nbc ? l - nbc : 0u;
  const uint32_t kc_adp = __shfl(a_dp, kc & 63, 64);  // every lane takes part in the shuffle
  const uint32_t c_actor = l < nbc ? bc_actor : kc_adp;
  int64_t c_seq = bc_seq;  // change headers are in global memory: only rows that exist read one
  if (l >= nbc && kc < N) c_seq = chh[kc].seq;
  if (l < NC) atomicMax(&LASTC[c_actor], l);
  wsync();
  const bool c_emit = l < NC && LASTC[c_actor] == l;
  const uint32_t b_clk = c_emit ? 1u + pk_uleb_len(c_actor) + pk_uleb_len((uint64_t)c_seq) : 0u;
  const uint32_t o_clk = base + excl_add(b_clk, tot);
  base += tot;
  const uint32_t o_root = base;  // PR_OBJ _root: tag, sleb -1, sleb -1, uleb 0
  base += 4;
  // root keys (PR_KEY / PR_PROP), output lane p holds the row at position p
  const uint32_t r = k_row;
  const bool outl = l < NOUT;
  const int32_t k_objc = __shfl(r_objc, r, 64), k_key = __shfl(r_key, r, 64);
  const uint32_t k_kr = __shfl(r_krank, r, 64), k_voff = __shfl(r_voff, r, 64);
  const int32_t k_idc = __shfl(r_idc, r, 64), k_ida = __shfl(r_ida, r, 64);
  const bool k_keyed = outl && k_key != FD_NULL && k_objc == FD_NULL;
  const bool is_m = outl && mli && r == mrow;
  const bool k_tch = k_keyed && (TCH[k_kr] || (mli && k_kr == m_kr));
  const uint32_t p_kr = wave::up1(k_kr, ~0u);
  const bool p_tch = wave::up1((uint32_t)k_tch, 0u) != 0;
  const bool emit_key = k_tch && !(l > 0 && p_tch && p_kr == k_kr);
  // the list's make op (the only visible value of its untouched key); a set without succ, or a
  // counter completed by its increments, that the key's last call takes
  const bool emit_prop = is_m ? SCR[r] == 0
                              : k_tch && k_taken && ((k_act == 1 && SCR[r] == 0) || (k_counter && cnt_done));
  uint32_t pvt = 0, pdt = 0;
  int64_t pv0 = 0, pv1 = 0;
  if (emit_prop) {
    if (is_m) { pvt = PV_CHILD; pdt = m_act == 2 ? 1u : 2u; pv0 = lc; pv1 = la; }
    else {
      pbad |= !fd_value(IN, k_vlen, k_voff, pvt, pdt, pv0, pv1);
      if (k_counter) pv0 += cnt_sum;  // {type: 'value', datatype: 'counter', value} (new.js:962-963)
    }
  }
  const uint32_t klen = (uint32_t)k_key & 255;
  const uint32_t b_key = (emit_key ? 1u + pk_uleb_len(klen) + klen : 0u) +
                         (emit_prop ? 1u + pk_uleb_len((uint64_t)k_idc) + pk_uleb_len((uint64_t)k_ida) +
                                          pk_value_len(pvt, pdt, pv0, pv1)
                                    : 0u);
  const uint32_t o_key = base + excl_add(b_key, tot);
  base += tot;
  // the list object: PR_OBJ, then its edits in application order (lane = change row)
  const uint32_t o_lobj = base;
  const uint32_t ltype = m_act == 2 ? 1u : 2u;
  if (mli) base += 1 + pk_sleb_len(lc) + pk_sleb_len(la) + pk_uleb_len(ltype);
  // index: visible elements of the list before the insert's position that exist when it applies
  uint64_t below;  // rows at output positions < this lane's position (exclusive OR-scan)
  {
    uint64_t x = outl ? (1ull << r) : 0ull;
    uint64_t inc = x;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint64_t y = __shfl_up(inc, d, 64);
      if ((int)l >= d) inc |= y;
    }
    below = inc & ~x;
  }
  const uint64_t el_l = __ballot(isrow && r_elem == (int32_t)l && r_objkey == lkey);  // elements of the list
  const uint64_t vis_base = __ballot(isrow && l < nb && EV[l]);
  uint32_t ins_vt = 0, ins_dt = 0, dtc = 0;
  int64_t ins_v0 = 0, ins_v1 = 0;
  int64_t idx = 0;
  const uint64_t bl = __shfl(below, POS[l] & 63, 64);
  if (list_ins) {
    const uint64_t exist = (vis_base | (nb >= 64 ? 0ull : ~0ull << nb)) & lt_mask();  // visible base elements, earlier inserts
    idx = __popcll(el_l & exist & bl);
    pbad |= !fd_value(IN, r_vlen, r_voff, ins_vt, ins_dt, ins_v0, ins_v1);
    dtc = pv_dtcode(ins_vt, ins_dt);
    pbad |= dtc == 100;  // datatype 0 (falsy): appendEdit's chain rule differs; k_doc replays it
  }
  // appendEdit chain: previous insert of the call (same list), contiguous index / id, same types
  const uint64_t before = mli & lt_mask();
  const uint32_t prev = before ? 63u - (uint32_t)__clzll(before) : 0u;
  const int64_t p_idx = __shfl(idx, prev, 64);
  const int32_t p_idc = __shfl(r_idc, prev, 64), p_ida = __shfl(r_ida, prev, 64);
  const uint32_t p_dtc = __shfl(dtc, prev, 64), p_ty = __shfl((uint32_t)pv_typeof(ins_vt), prev, 64);
  const bool chain = list_ins && before && p_idx + 1 == idx && p_ida == r_ida && p_idc + 1 == r_idc && p_dtc == dtc &&
                     p_ty == (uint32_t)pv_typeof(ins_vt);
  const bool start = list_ins && !chain;
  const uint64_t smask = __ballot(start);
  const uint64_t above = l == 63 ? 0ull : (smask >> (l + 1)) << (l + 1);
  const uint32_t nxt = above ? ctz64(above) : 64u;
  const uint64_t span = (nxt >= 64 ? ~0ull : ((1ull << nxt) - 1)) & ~((1ull << l) - 1);
  const uint32_t run = start ? (uint32_t)__popcll(mli & span) : 0u;
  const uint32_t mdt = pv_dt_truthy(dtc) ? dtc : 0u;
  uint32_t b_ed = 0;
  if (list_ins) {
    if (start && run >= 2)
      b_ed = 1 + pk_uleb_len((uint64_t)idx) + pk_uleb_len((uint64_t)r_idc) + pk_uleb_len((uint64_t)r_ida) + pk_uleb_len(mdt) +
             pk_uleb_len(run);
    else if (start)
      b_ed = 1 + pk_uleb_len((uint64_t)idx) + 2 * (pk_uleb_len((uint64_t)r_idc) + pk_uleb_len((uint64_t)r_ida));
    b_ed += pk_value_len(ins_vt, ins_dt, ins_v0, ins_v1);
  }
  const uint32_t o_ed = base + excl_add(b_ed, tot);
  base += tot;
  pbad |= sizeof(PatchHdr2) + (uint64_t)base > out_cap;
  if (__any(pbad)) return false;

  // ---- objectMeta blob after the stream (lane 0; rows and positions < 64: one LEB128 byte each) ----
  uint32_t mbytes = 0;
  if (meta) {
    bool mok = true;
    if (l == 0) {
      uint8_t* const mo = out + sizeof(PatchHdr2) + base;
      const uint64_t mcap = out_cap - sizeof(PatchHdr2) - base;
      uint32_t w = 5, nk = 0;  // "AMM1", entry count, entries
      bool found_m = false;
      auto put = [&](uint32_t v) {
        if (v >= 128 || w >= mcap) { mok = false; return; }
        mo[w++] = (uint8_t)v;
      };
      auto root_key_row = [&](uint32_t row) { return row < R && P.objc[row] == FD_NULL && (P.flags[row] & 4) != 0; };
      if (mblob) {
        // the handle's snapshots (base rows = this call's base document order) renumbered
        uint32_t off = 0;
        auto get = [&](uint32_t& v) {
          v = 0;
          for (uint32_t sh = 0; sh < 35; sh += 7) {
            if (off >= mlen) { mok = false; return; }
            const uint8_t b8 = mblob[off++];
            v |= (uint32_t)(b8 & 0x7f) << sh;
            if (!(b8 & 0x80)) return;
          }
          mok = false;
        };
        uint32_t cnt = 0;
        mok = mlen >= 4 && mblob[0] == 'A' && mblob[1] == 'M' && mblob[2] == 'M' && mblob[3] == '1';
        off = 4;
        if (mok) get(cnt);
        for (uint32_t k = 0; mok && k < cnt; k++) {
          uint32_t orow = 0, erow = 0, n = 0;
          get(orow); get(erow); get(n);
          mok = mok && orow == 0 && erow < nb && root_key_row(erow) && !TCH[P.krank[erow]];
          if (!mok) break;
          const uint32_t kr_ = P.krank[erow];
          const bool is_mkey = mli && kr_ == m_kr;
          if (is_mkey && n != 1) mok = false;
          put(0); put(POS[erow]); put(n);
          for (uint32_t q = 0; mok && q < n; q++) {
            uint32_t vr = 0;
            get(vr);
            mok = mok && vr < nb && root_key_row(vr) && P.krank[vr] == kr_;
            if (mok) put(POS[vr]);
            if (is_mkey) mok = mok && n == 1 && vr == mrow;
          }
          found_m |= is_mkey;
          nk++;
        }
        mok = mok && off == mlen;
      } else {
        // documentPatch's snapshots of the base document (new.js:884-931 over each root key's rows in
        // document order): a make op joins the snapshot; the snapshot becomes the visible ops so far
        // once the key has a visible make op or a non-empty snapshot. Keys this call touches have no
        // make rows (above), so their (absent) snapshots are the base document's as well.
        uint32_t p = 0;
        while (mok && p < NOUT) {
          const uint32_t r0 = P.krow[p];
          if (!root_key_row(r0)) { p++; continue; }
          const uint32_t kr_ = P.krank[r0], p0 = p;
          bool exists = false, has_child = false;
          uint64_t snap = 0, vis = 0;
          for (; p < NOUT && root_key_row(P.krow[p]) && P.krank[P.krow[p]] == kr_; p++) {
            const uint32_t r = P.krow[p];
            const uint32_t a = P.act[r];
            const bool mk = (a & 1) == 0, visible = SCR[r] == 0;
            if (mk) { exists = true; snap |= 1ull << p; }
            // the snapshot keeps the visible 'set' and make ops only (new.js:919-926): a visible inc
            // or link row of the key is a visible op but never a child value
            if (visible) { if (a == 1 || mk) vis |= 1ull << p; has_child |= mk; }
            if (has_child || (exists && snap)) { snap = vis; exists = true; }
          }
          if (!exists) continue;
          const bool is_mkey = mli && kr_ == m_kr;
          if (is_mkey) mok = mok && snap == (1ull << POS[mrow]);
          found_m |= is_mkey;
          put(0); put(p0); put((uint32_t)__popcll(snap));
          for (uint64_t x = snap; x; x &= x - 1) put((uint32_t)__builtin_ctzll(x));
          nk++;
        }
      }
      mok = mok && (!mli || found_m) && nk < 128 && mcap >= 5;
      if (mok) {
        mo[0] = 'A'; mo[1] = 'M'; mo[2] = 'M'; mo[3] = '1'; mo[4] = (uint8_t)nk;
        mbytes = w;
      }
    }
    pbad |= !mok;
    mbytes = uni(__shfl(mbytes, 0, 64));
  }
  if (__any(pbad)) return false;

  // ---- write ----
  uint8_t* const o = out + sizeof(PatchHdr2);
  if (b_act) {
    uint8_t* p = o + o_act;
    *p++ = PR_ACTOR;
    p = pk_uleb(p, a_len);
    for (uint32_t q = 0; q < a_len; q++) p[q] = IN[a_off + q];
  }
  if (b_clk) {
    uint8_t* p = o + o_clk;
    *p++ = PR_CLOCK;
    p = pk_uleb(p, c_actor);
    pk_uleb(p, (uint64_t)c_seq);
  }
  if (l == 0) { o[o_root] = PR_OBJ; o[o_root + 1] = 0x7f; o[o_root + 2] = 0x7f; o[o_root + 3] = 0; }
  if (b_key) {
    uint8_t* p = o + o_key;
    if (emit_key) {
      *p++ = PR_KEY;
      p = pk_uleb(p, klen);
      const uint32_t ko = (uint32_t)k_key >> 8;
      for (uint32_t q = 0; q < klen; q++) *p++ = IN[ko + q];
    }
    if (emit_prop) {
      *p++ = PR_PROP;
      p = pk_uleb(p, (uint64_t)k_idc);
      p = pk_uleb(p, (uint64_t)k_ida);
      pk_value(p, pvt, pdt, pv0, pv1, pv_has_bytes(pvt) ? IN + pv0 : nullptr);
    }
  }
  if (mli && l == 0) {
    uint8_t* p = o + o_lobj;
    *p++ = PR_OBJ;
    p = pk_sleb(p, lc);
    p = pk_sleb(p, la);
    pk_uleb(p, ltype);
  }
  if (list_ins) {
    uint8_t* p = o + o_ed;
    if (start && run >= 2) {
      *p++ = PR_MULTI;
      p = pk_uleb(p, (uint64_t)idx);
      p = pk_uleb(p, (uint64_t)r_idc);
      p = pk_uleb(p, (uint64_t)r_ida);
      p = pk_uleb(p, mdt);
      p = pk_uleb(p, run);
    } else if (start) {
      *p++ = PR_INSERT;
      p = pk_uleb(p, (uint64_t)idx);
      p = pk_uleb(p, (uint64_t)r_idc);
      p = pk_uleb(p, (uint64_t)r_ida);
      p = pk_uleb(p, (uint64_t)r_idc);
      p = pk_uleb(p, (uint64_t)r_ida);
    }
    pk_value(p, ins_vt, ins_dt, ins_v0, ins_v1, pv_has_bytes(ins_vt) ? IN + ins_v0 : nullptr);
  }
  if (l == 0) {
    PatchHdr2 h;
    h.magic = AM_PATCH_MAGIC; h.status = 0; h.arg0 = 0; h.arg1 = 0; h.max_op = 0; h.nbytes = base; h.meta_bytes = mbytes;
    *reinterpret_cast<PatchHdr2*>(out) = h;
  }
  return true;
}

// Backend.getPatch (documentPatch, new.js:1604-1635, 2052-2060; patch_scan in am_patch.h) of the
// merged document, written by the whole wave in wire form for the common shape: every op of the root
// is a keyed `set`, `inc` or make op, every op of a child object is the insert (`set`) of its own list
// element, and every child object is made by a root op. For that shape documentPatch's single pass
// reduces to closed forms over the output positions (document order):
//   * a key's props are its ops without succ (values, child objects) plus each counter `set` whose
//     succs are all increments of the key, shown at its last increment with their sum
//     (counterStates, new.js:937-965); the key record comes with the key's first prop;
//   * a list's edits are its visible elements as inserts at their visible index, joined by
//     appendEdit's multi-insert rule (new.js:747-782) into runs of consecutive counters of one actor
//     with one datatype and JS type;
//   * a child object is in the patch iff its make op has no succ (objectMeta reachability).
// Anything else (deletes inside lists, nested objects, map children with ops, errors) returns false
// and k_doc writes the log (P7). Scratch: FD_DIFF_SCRATCH bytes at PS.
__device__ __forceinline__ bool fast_getpatch(const uint8_t* IN, uint8_t* PS, uint32_t ps_cap, uint8_t* out, uint64_t out_cap,
                                              uint8_t* M, uint32_t NOUT, uint32_t NSUCC, uint32_t NA, uint32_t NC, uint32_t nbc,
                                              uint32_t N, const int32_t* OUTC, const uint8_t* OUTA, const uint32_t* RO,
                                              const ChgHdrC* chh) {
  const FdRec P = fd_rec(M, PS + ps_cap);
  const uint32_t l = lane();
  const bool outl = l < NOUT;
  bool pbad = ps_cap < FD_DIFF_SCRATCH || NOUT > 64 || NSUCC > 64;
  if (__any(pbad)) return false;
  // the row at output position l and its values
  const uint32_t r = outl ? P.krow[l] : 0u, sc = outl ? P.sck[l] : 0u, so = outl ? P.sok[l] : 0u;
  const int32_t k_key = outl ? (int32_t)P.key[r] : FD_NULL, k_objc = outl ? P.objc[r] : FD_NULL;
  const int32_t k_idc = outl ? P.idc[r] : 0, k_vlen = outl ? P.vlen[r] : FD_NULL;
  const uint32_t k_voff = outl ? P.voff[r] : 0u;
  const int32_t k_obja = outl ? (int32_t)P.obja[r] : -1, k_ida = outl ? (int32_t)P.ida[r] : 0;
  const uint32_t k_kr = outl ? P.krank[r] : 0u;
  const int32_t k_act = outl ? (int32_t)P.act[r] : 0;
  const uint32_t fl = outl ? P.flags[r] : 0u;
  const bool k_ins = (fl & 2) != 0, k_keyed = (fl & 4) != 0;
  const bool root = outl && k_objc == FD_NULL;
  const bool child = outl && !root;
  const bool is_make = k_act == 0 || k_act == 2 || k_act == 4 || k_act == 6;
  // maxOp of documentPatch: ids and succ ids of every op
  int32_t mx = outl ? k_idc : 0;
  if (l < NSUCC && OUTC[l] > mx) mx = OUTC[l];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const int32_t y = __shfl_xor(mx, o, 64);
    mx = y > mx ? y : mx;
  }
  // object sections: first position of each object; a child object's make op (a root op)
  const int32_t p_objc = wave::up1(k_objc, (int32_t)0x7fffffff), p_obja = wave::up1(k_obja, (int32_t)-2);
  const bool first_obj = outl && (l == 0 || p_objc != k_objc || p_obja != k_obja);
  const uint64_t fom = __ballot(first_obj);
  const uint64_t le = l == 63 ? ~0ull : ((2ull << l) - 1);  // positions <= l
  const uint64_t fo_le = fom & le;
  const uint32_t ostart = fo_le ? 63u - (uint32_t)__clzll(fo_le) : 0u;
  int32_t mk = -1;
  for (uint32_t j = 0; j < NOUT; j++) {
    const int32_t jc = wave::bcast(k_idc, (int)j), ja = wave::bcast(k_ida, (int)j);
    if (child && jc == k_objc && ja == k_obja) mk = (int32_t)j;
  }
  const uint32_t mku = mk < 0 ? 0u : (uint32_t)mk;
  const int32_t m_act = __shfl(k_act, mku, 64);
  const uint32_t m_sc = __shfl(sc, mku, 64);
  const int32_t m_root = __shfl((int32_t)root, mku, 64);
  // a child object: made by a root list / text op; reachable iff that op has no succ
  pbad |= child && (mk < 0 || !m_root || (m_act != 2 && m_act != 4));
  const bool reach = root || (child && m_sc == 0);
  pbad |= root && (!k_keyed || (k_key & 255) == 0 || !(k_act == 1 || k_act == 5 || is_make));
  pbad |= child && reach && (!k_ins || k_keyed || k_act != 1);
  if (__any(pbad)) return false;

  // ---- counters: lane per succ entry; entry q belongs to the op at output position OWNE[q] ----
  uint8_t* const OWNE = PS;                                       // succ entry -> owner position
  uint8_t* const CAT = PS + 64;                                   // position -> 1 + counter completed here
  uint32_t* const COV = reinterpret_cast<uint32_t*>(PS + 128);    // position -> counter sets naming it
  CAT[l] = 0;
  COV[l] = 0;
  if (outl)
    for (uint32_t j = 0; j < sc; j++) OWNE[so + j] = (uint8_t)l;
  wsync();
  const bool counter = root && k_act == 1 && sc > 0 && k_vlen != FD_NULL && (k_vlen & 15) == 8;
  int64_t cnt_sum = 0;
  if (__any(counter) || __any(root && k_act == 5)) {
    const bool isent = l < NSUCC;
    const uint32_t own = isent ? OWNE[l] : 0u;
    const int32_t ec = isent ? OUTC[l] : 0, ea = isent ? (int32_t)OUTA[l] : -1;
    int32_t tgt = -1;  // the position of the op with the entry's opId
    for (uint32_t j = 0; j < NOUT; j++) {
      const int32_t jc = wave::bcast(k_idc, (int)j), ja = wave::bcast(k_ida, (int)j);
      if (isent && jc == ec && ja == ea) tgt = (int32_t)j;
    }
    const uint32_t tu = tgt < 0 ? 0u : (uint32_t)tgt;
    const int32_t o_counter = __shfl((int32_t)counter, own, 64);
    const uint32_t o_kr = __shfl(k_kr, own, 64);
    const int32_t t_act = __shfl(k_act, tu, 64), t_vlen = __shfl(k_vlen, tu, 64), t_root = __shfl((int32_t)root, tu, 64);
    const uint32_t t_kr = __shfl(k_kr, tu, 64), t_voff = __shfl(k_voff, tu, 64);
    const bool inc_of_key = isent && tgt >= 0 && t_act == 5 && t_root && t_kr == o_kr;
    if (isent && o_counter && inc_of_key) atomicAdd(&COV[tu], 1u);
    int64_t iv = 0;
    bool ok = isent && o_counter && inc_of_key;
    if (ok) {
      uint32_t vt, dt;
      int64_t v1;
      const uint32_t t15 = t_vlen == FD_NULL ? 0u : ((uint32_t)t_vlen & 15);
      ok = (t15 == 3 || t15 == 4 || t15 == 8 || t15 == 9) && fd_value(IN, t_vlen, t_voff, vt, dt, iv, v1);
      pbad |= isent && o_counter && inc_of_key && !ok;  // a non-integer increment: k_doc writes it
    }
    // per counter set: the sum of its increments, whether every succ is one, the last of them
    uint64_t owners = __ballot(counter);
    while (owners) {
      const uint32_t pw = (uint32_t)__builtin_ctzll(owners);
      owners &= owners - 1;
      const bool mine = isent && own == pw;
      int64_t sv = mine && ok ? iv : 0;
      uint32_t sb = mine && !ok ? 1u : 0u;
      int32_t last = mine ? tgt : -1;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        sv += __shfl_xor(sv, o, 64);
        sb += __shfl_xor(sb, o, 64);
        const int32_t y = __shfl_xor(last, o, 64);
        last = y > last ? y : last;
      }
      if (l == pw) cnt_sum = sv;
      if (l == 0 && sb == 0 && last >= 0) CAT[last] = (uint8_t)(pw + 1);
    }
  }
  wsync();
  // every increment is named by exactly one counter set of its key (else: increment operation for
  // unknown counter -- k_doc reports it)
  pbad |= root && k_act == 5 && COV[l] != 1;
  if (__any(pbad)) return false;

  // ---- props of the root (PR_KEY / PR_PROP) and edits of the lists, by output position ----
  const uint32_t cat = outl ? CAT[l] : 0u;
  const uint32_t cown = cat ? cat - 1 : 0u;
  const int64_t c_sum = __shfl(cnt_sum, cown, 64);
  const int32_t c_idc = __shfl(k_idc, cown, 64), c_ida = __shfl(k_ida, cown, 64);
  const int32_t c_vlen = __shfl(k_vlen, cown, 64);
  const uint32_t c_voff = __shfl(k_voff, cown, 64);
  bool have = false;
  uint32_t vt = 0, vdt = 0;
  int64_t v0 = 0, v1 = 0;
  int32_t pk_c = k_idc, pk_a = k_ida;
  if (root) {
    if (k_act == 5) {
      if (cat) {  // the counter completed by this increment (new.js:962-963)
        have = true;
        pbad |= !fd_value(IN, c_vlen, c_voff, vt, vdt, v0, v1);
        v0 += c_sum;
        pk_c = c_idc;
        pk_a = c_ida;
      }
    } else if (sc == 0) {
      have = true;
      if (k_act == 1) pbad |= !fd_value(IN, k_vlen, k_voff, vt, vdt, v0, v1);
      else { vt = PV_CHILD; vdt = pv_obj_type(k_act); v0 = k_idc; v1 = k_ida; }
    }
  }
  // key groups of the root: the key record precedes the group's first prop
  const uint32_t p_kr = wave::up1(k_kr, ~0u);
  const bool p_root = wave::up1((uint32_t)root, 0u) != 0;
  const bool gfirst = root && (l == 0 || !p_root || p_kr != k_kr);
  const uint64_t gm = __ballot(gfirst) & le;
  const uint32_t gs = gm ? 63u - (uint32_t)__clzll(gm) : 0u;
  const uint64_t hm = __ballot(have);
  const uint64_t before_l = le & ~(l == 63 ? 0ull : (1ull << l)) & ~((1ull << gs) - 1);  // positions [gs, l)
  const bool emit_key = have && (hm & before_l) == 0;
  // list elements: visible ones are inserts at their visible index
  const bool vis = child && reach && sc == 0;
  uint32_t ivt = 0, idt = 0, dtc = 0;
  int64_t iv0 = 0, iv1 = 0;
  if (vis) {
    pbad |= !fd_value(IN, k_vlen, k_voff, ivt, idt, iv0, iv1);
    dtc = pv_dtcode(ivt, idt);
    pbad |= dtc == 100;  // datatype 0 (falsy): appendEdit's chain rule differs; k_doc writes it
  }
  const uint64_t vm = __ballot(vis);
  const uint64_t ob = le & ~(l == 63 ? 0ull : (1ull << l)) & ~((1ull << ostart) - 1);  // positions [ostart, l)
  const int64_t idx = __popcll(vm & ob);
  const uint64_t pvm = vm & ob;
  const uint32_t prv = pvm ? 63u - (uint32_t)__clzll(pvm) : 0u;
  const int32_t q_idc = __shfl(k_idc, prv, 64), q_ida = __shfl(k_ida, prv, 64);
  const uint32_t q_dtc = __shfl(dtc, prv, 64), q_ty = __shfl((uint32_t)pv_typeof(ivt), prv, 64);
  const bool chain = vis && pvm && q_ida == k_ida && q_idc + 1 == k_idc && q_dtc == dtc && q_ty == (uint32_t)pv_typeof(ivt);
  const bool start = vis && !chain;
  const uint64_t smask = __ballot(start);
  const uint64_t above = l == 63 ? 0ull : (smask >> (l + 1)) << (l + 1);
  const uint32_t nxt = above ? ctz64(above) : 64u;
  const uint64_t span = (nxt >= 64 ? ~0ull : ((1ull << nxt) - 1)) & ~((1ull << l) - 1);
  const uint32_t run = start ? (uint32_t)__popcll(vm & span) : 0u;
  const uint32_t mdt = pv_dt_truthy(dtc) ? dtc : 0u;
  if (__any(pbad)) return false;

  // ---- record sizes: actors, clock, then the positions in document order ----
  const uint32_t a_off = l < NA ? RO[2 * M[FM_DP2REF + l]] : 0u, a_len = l < NA ? RO[2 * M[FM_DP2REF + l] + 1] : 0u;
  uint32_t tot;
  const uint32_t b_act = l < NA ? 1u + pk_uleb_len(a_len) + a_len : 0u;
  const uint32_t o_act = excl_add(b_act, tot);
  uint32_t base = tot;
  uint32_t* const LASTC = reinterpret_cast<uint32_t*>(PS + 384);  // doc actor -> its last change row
  LASTC[l] = 0;
  wsync();
  const uint32_t kc = l >= nbc ? l - nbc : 0u;
  const uint32_t kc_adp = __shfl(l < N ? (uint32_t)P.adp[l] : 0u, kc & 63, 64);
  const uint32_t c_actor = l < nbc ? (uint32_t)P.bca[l] : kc_adp;
  int64_t c_seq = l < nbc ? (int64_t)P.bcs[l] : 0;  // change headers are in global memory
  if (l >= nbc && kc < N) c_seq = chh[kc].seq;
  if (l < NC) atomicMax(&LASTC[c_actor], l);
  wsync();
  const bool c_emit = l < NC && LASTC[c_actor] == l;
  const uint32_t b_clk = c_emit ? 1u + pk_uleb_len(c_actor) + pk_uleb_len((uint64_t)c_seq) : 0u;
  const uint32_t o_clk = base + excl_add(b_clk, tot);
  base += tot;
  const bool obj_rec = first_obj && reach;
  const uint32_t b_obj = obj_rec ? (root ? 4u : 1u + pk_sleb_len(k_objc) + pk_sleb_len(k_obja) + 1u) : 0u;
  const uint32_t klen = (uint32_t)k_key & 255;
  uint32_t b_pos = b_obj;
  if (root && have)
    b_pos += (emit_key ? 1u + pk_uleb_len(klen) + klen : 0u) + 1u + pk_uleb_len((uint64_t)pk_c) + pk_uleb_len((uint64_t)pk_a) +
             pk_value_len(vt, vdt, v0, v1);
  if (vis) {
    if (start && run >= 2)
      b_pos += 1 + pk_uleb_len((uint64_t)idx) + pk_uleb_len((uint64_t)k_idc) + pk_uleb_len((uint64_t)k_ida) + pk_uleb_len(mdt) +
               pk_uleb_len(run);
    else if (start)
      b_pos += 1 + pk_uleb_len((uint64_t)idx) + 2 * (pk_uleb_len((uint64_t)k_idc) + pk_uleb_len((uint64_t)k_ida));
    b_pos += pk_value_len(ivt, idt, iv0, iv1);
  }
  const uint32_t o_pos = base + excl_add(b_pos, tot);
  base += tot;
  if (__any(sizeof(PatchHdr2) + (uint64_t)base > out_cap)) return false;

  // ---- write ----
  uint8_t* const o = out + sizeof(PatchHdr2);
  if (b_act) {
    uint8_t* p = o + o_act;
    *p++ = PR_ACTOR;
    p = pk_uleb(p, a_len);
    for (uint32_t q = 0; q < a_len; q++) p[q] = IN[a_off + q];
  }
  if (b_clk) {
    uint8_t* p = o + o_clk;
    *p++ = PR_CLOCK;
    p = pk_uleb(p, c_actor);
    pk_uleb(p, (uint64_t)c_seq);
  }
  if (b_pos) {
    uint8_t* p = o + o_pos;
    if (obj_rec) {  // PR_OBJ (documentPatch leaves its type field 0)
      *p++ = PR_OBJ;
      if (root) { *p++ = 0x7f; *p++ = 0x7f; }
      else { p = pk_sleb(p, k_objc); p = pk_sleb(p, k_obja); }
      *p++ = 0;
    }
    if (root && have) {
      if (emit_key) {
        *p++ = PR_KEY;
        p = pk_uleb(p, klen);
        const uint32_t ko = (uint32_t)k_key >> 8;
        for (uint32_t q = 0; q < klen; q++) *p++ = IN[ko + q];
      }
      *p++ = PR_PROP;
      p = pk_uleb(p, (uint64_t)pk_c);
      p = pk_uleb(p, (uint64_t)pk_a);
      pk_value(p, vt, vdt, v0, v1, pv_has_bytes(vt) ? IN + v0 : nullptr);
    }
    if (vis) {
      if (start && run >= 2) {
        *p++ = PR_MULTI;
        p = pk_uleb(p, (uint64_t)idx);
        p = pk_uleb(p, (uint64_t)k_idc);
        p = pk_uleb(p, (uint64_t)k_ida);
        p = pk_uleb(p, mdt);
        p = pk_uleb(p, run);
      } else if (start) {
        *p++ = PR_INSERT;
        p = pk_uleb(p, (uint64_t)idx);
        p = pk_uleb(p, (uint64_t)k_idc);
        p = pk_uleb(p, (uint64_t)k_ida);
        p = pk_uleb(p, (uint64_t)k_idc);
        p = pk_uleb(p, (uint64_t)k_ida);
      }
      pk_value(p, ivt, idt, iv0, iv1, pv_has_bytes(ivt) ? IN + iv0 : nullptr);
    }
  }
  if (l == 0) {
    PatchHdr2 h;
    h.magic = AM_PATCH_MAGIC; h.status = 0; h.arg0 = 0; h.arg1 = 0; h.max_op = mx; h.nbytes = base; h.meta_bytes = 0;
    *reinterpret_cast<PatchHdr2*>(out) = h;
  }
  return true;
}

}  // namespace fastdoc

// register budget for at least three waves per SIMD (<= 168 VGPRs; the kernel needs ~85 since its
// per-document values are scalar): the LDS slice decides the occupancy. Probe builds may ask for
// another count (-DAM_FAST_WAVES=n).
#ifndef AM_FAST_WAVES
#define AM_FAST_WAVES 3
#endif
#ifndef AM_FAST_WAVES_DIFF
#define AM_FAST_WAVES_DIFF AM_FAST_WAVES
#endif
#define FD_WAVES_ATTR __attribute__((amdgpu_waves_per_eu(kDiff ? AM_FAST_WAVES_DIFF : AM_FAST_WAVES, 8)))
// kDiff: the variant launched for batches that ask for applyChanges patches (it also merges the
// documents that do not); the other keeps the register budget of the plain merge.
template <bool kDiff>
__global__ void __launch_bounds__(64 * FD_DOCS_PER_WG) FD_WAVES_ATTR
    k_doc_fast(const uint8_t* __restrict__ arena, const am_chunk_desc* __restrict__ chunks, const am_doc_desc* __restrict__ docs,
               const am_known_hash* __restrict__ known, const ChunkInfo* __restrict__ info,
               const HdrSlot* __restrict__ hdr, const DocBounds* __restrict__ bounds, const uint64_t* __restrict__ ws_off, uint8_t* __restrict__ ws_base,
               uint64_t ws_cap, uint32_t lds_per_doc, uint32_t lds_floor, uint32_t ndocs, am_doc_result* __restrict__ results,
               int32_t* __restrict__ chg_state, uint8_t* __restrict__ fast_done) {
  using namespace fastdoc;
  const uint32_t l = lane();
  // wave-uniform by construction: readfirstlane tells the compiler, so the document's descriptors,
  // bounds and layout live in scalar registers and scalar loads fetch them
  const uint32_t doc = (uint32_t)__builtin_amdgcn_readfirstlane((int)(blockIdx.x * FD_DOCS_PER_WG + (threadIdx.x >> 6)));
  if (doc >= ndocs) return;
#ifdef AM_PHASE_CLOCK
  uint64_t ph_last = clock64();
#endif
  const am_doc_desc dd = docs[doc];
  const DocBounds b = bounds[doc];
  if (!fast_eligible(b, dd)) return;
  if (!(b.U & 4u)) return;  // not given the compact plan (AM_WS_COMPACT=0): k_doc merges it
  const FastLayout F = fast_layout(b, dd.known_count);
  if (F.total > lds_per_doc || F.total <= lds_floor) return;  // another launch's slice class (or k_doc's)
  const WsFast L = ws_fast(b);
  const uint64_t wso = ws_off[doc];
  if (wso + L.total > ws_cap) return;  // capacity error: reported by k_doc
  uint8_t* const wsg = ws_base + wso;
  uint8_t* const S = am_lds + uni(threadIdx.x >> 6) * lds_per_doc;
  uint8_t* const M = S + F.misc;
  const bool has_base = dd.base_chunk >= 0;
  const uint32_t N = dd.chg_count;
  bool bad = false;
#define FD_CHECK()          \
  do {                      \
    if (__any(bad)) return; \
  } while (0)

  // ---- chunk status (k_chunks) and per-change counts ----
  uint32_t c_nops = 0, c_nents = 0, c_ndeps = 0, c_nact = 0;
  if (l < N) {
    const ChunkInfo& ci = info[dd.chg_begin + l];
    bad |= ci.status != AM_OK || ci.type != 1;
    c_nops = ci.nops; c_nents = ci.nents; c_ndeps = ci.ndeps; c_nact = ci.nactors;
  }
  uint32_t nb = 0, nbe = 0, nbc = 0, nbd = 0;
  if (has_base) {
    const ChunkInfo& ci = info[dd.base_chunk];
    bad |= ci.status != AM_OK || ci.type != 0;
    nb = ci.nops; nbe = ci.nents; nbc = ci.nchg; nbd = ci.ndeps;
  }
  FD_CHECK();

  // ---- stage the input span (16-byte loads) ----
  const uint64_t a0 = b.span_lo & ~15ull;
  {
    const uint32_t nv = (uint32_t)((b.span_hi - a0 + 15) / 16);
    uint4* dst = reinterpret_cast<uint4*>(S + F.input);
    const uint4* src = reinterpret_cast<const uint4*>(arena + a0);
    for (uint32_t v = l; v < nv; v += 64) dst[v] = src[v];
  }
  const uint8_t* const IN = S + F.input;  // IN[off - a0] = arena[off]
  wsync();
  FPH(0);

  // ---- headers: the base document (lane 0) and one change per lane ----
  DocHdrC* dh = reinterpret_cast<DocHdrC*>(M + FM_DH);
  // the change headers parsed by k_chunks (compact slots) are read where they lie (global memory,
  // read a few times per change): their LDS copy would cost 128 B of every slice per change
  const ChgHdrC* const chh = reinterpret_cast<const ChgHdrC*>(hdr + dd.chg_begin);
  // the base document's header (8 x 16 B) into LDS
  {
    const uint4* src_b = reinterpret_cast<const uint4*>(hdr + (has_base ? dd.base_chunk : 0));
    if (has_base && l < 8) reinterpret_cast<uint4*>(dh)[l] = src_b[l];
    if (!has_base && l == 0) { dh->nactors = 0; dh->nheads = 0; dh->has_hidx = 0; dh->extra_len = 0; dh->base = 0; }
  }
  wsync();
  FD_CHECK();
  // header fields every lane reads: readfirstlane keeps them (and the loops they bound) scalar
  const uint32_t NB = uni(dh->nactors), HB = uni(dh->nheads), K = dd.known_count;
  const uint64_t dhb = ((uint64_t)uni((uint32_t)(dh->base >> 32)) << 32) | uni((uint32_t)dh->base);
  bad |= NB + N != b.A || HB + N != b.H;
  FD_CHECK();
  // base heads' changeIndexByHash indexes (new.js:1729-1739); -1 = unknown
  if (l == 0) {
    int64_t* bh = reinterpret_cast<int64_t*>(S + F.bk);
    if (dh->has_hidx) {
      Rd r{IN + (dhb + dh->hidx_off - a0), (uint64_t)1 << 40, 0};
      for (uint32_t h = 0; h < HB; h++) {
        int64_t v = -1;
        rd_u53(r, v);
        bh[h] = v;
      }
    } else {
      for (uint32_t h = 0; h < HB; h++) bh[h] = HB == 1 ? (int64_t)nbc - 1 : -1;
    }
  }

  // ---- hash table: changes [0, N) | base heads [N, N+HB) | known [N+HB, N+HB+K) ----
  uint32_t* HT = reinterpret_cast<uint32_t*>(S + F.hashes);
  if (l < N) {
    const uint4* h = reinterpret_cast<const uint4*>(info[dd.chg_begin + l].hash);
    reinterpret_cast<uint4*>(HT + 8 * l)[0] = h[0];
    reinterpret_cast<uint4*>(HT + 8 * l)[1] = h[1];
  }
  if (l < HB) {
    uint32_t w[8];
    load32(IN + (dhb + dh->heads_off + 32 * l - a0), w);
#pragma unroll
    for (int k = 0; k < 8; k++) HT[8 * (N + l) + k] = w[k];
  }
  if (l < K) {
    const am_known_hash& kh = known[dd.known_begin + l];
    uint32_t w[8];
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const uint8_t* p = kh.hash + 4 * k;
      w[k] = (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24;
    }
#pragma unroll
    for (int k = 0; k < 8; k++) HT[8 * (N + HB + l) + k] = w[k];
    reinterpret_cast<int64_t*>(S + F.bk + 8 * HB)[l] = kh.index;
  }

  // ---- actor references: base actors [0, NB), then each change's actor list ----
  uint32_t am_total;
  const uint32_t ambase = excl_add(l < N ? c_nact : 0u, am_total);
  const uint32_t NR = NB + am_total;
  bad |= NR > FD_MAX;
  FD_CHECK();
  uint32_t* RW = reinterpret_cast<uint32_t*>(S + F.rw);    // 8 words per ref (cells region, until the actor table)
  uint32_t* RO = reinterpret_cast<uint32_t*>(S + F.refs);  // (off - a0, len) per ref
  if (l == 0 && has_base) {
    Rd r{IN + (dhb + dh->actors_off - a0), (uint64_t)1 << 40, 0};
    for (uint32_t i = 0; i < NB; i++) {
      int64_t len = 0;
      bad |= rd_u53(r, len) != AM_OK;
      RO[2 * i] = (uint32_t)(dhb + dh->actors_off + r.off - a0);
      RO[2 * i + 1] = (uint32_t)len;
      r.off += (uint64_t)len;
    }
  }
  if (l < N) {
    const ChgHdrC& h = chh[l];
    const uint32_t r0 = NB + ambase;
    RO[2 * r0] = (uint32_t)(h.base + h.actor_off - a0);
    RO[2 * r0 + 1] = h.actor_len;
    Rd r{IN + (h.base + h.actors_off - a0), (uint64_t)1 << 40, 0};
    for (uint32_t k = 1; k < c_nact; k++) {
      int64_t len = 0;
      bad |= rd_u53(r, len) != AM_OK;
      RO[2 * (r0 + k)] = (uint32_t)(h.base + h.actors_off + r.off - a0);
      RO[2 * (r0 + k) + 1] = (uint32_t)len;
      r.off += (uint64_t)len;
    }
  }
  wsync();
  FD_CHECK();
  // padded big-endian words of each ref (ids up to 32 bytes)
  uint32_t r_len = 0;
  if (l < NR) {
    const uint32_t off = RO[2 * l];
    r_len = RO[2 * l + 1];
    bad |= r_len > 32;
#pragma unroll
    for (int k = 0; k < 8; k++) {
      uint32_t w = 0;
#pragma unroll
      for (int q = 0; q < 4; q++)
        if ((uint32_t)(4 * k + q) < r_len) w |= (uint32_t)IN[off + 4 * k + q] << (24 - 8 * q);
      RW[8 * l + k] = w;
    }
  }
  wsync();
  FD_CHECK();
  FPH(1);
  // canonical ref (first equal id) and rank of the canonical ids (hex order = bytewise, shorter
  // prefix first: actor_cmp_dev)
  uint8_t* CANON = M + FM_CANON;
  {
    uint32_t canon = l;
    if (l < NR) {
      for (uint32_t j = 0; j < NR; j++) {
        if (j >= l) break;
        if (RO[2 * j + 1] == r_len && words_eq(RW + 8 * j, RW + 8 * l)) { canon = j; break; }
      }
      CANON[l] = (uint8_t)canon;
    }
    wsync();
    uint32_t rank = 0;
    if (l < NR && canon == l) {
      for (uint32_t j = 0; j < NR; j++) {
        if (CANON[j] != j || j == l) continue;
        int c = 0;
        for (int k = 0; k < 8 && c == 0; k++) {
          const uint32_t a = RW[8 * j + k], bb = RW[8 * l + k];
          c = a < bb ? -1 : (a > bb ? 1 : 0);
        }
        if (c == 0) c = RO[2 * j + 1] < r_len ? -1 : 1;
        if (c < 0) rank++;
      }
      M[FM_RANKC + l] = (uint8_t)rank;
    }
  }
  // doc actor table: base actors, then new authors in application order (getActorTable,
  // new.js:1434-1451); every other actor of a change must already be in the table
  uint32_t* FIRST = reinterpret_cast<uint32_t*>(M + FM_FIRST);
  FIRST[l] = 0xffffffffu;
  wsync();
  uint32_t a_canon = 0;  // canonical ref of change l's author
  if (l < NB) bad |= CANON[l] != l;  // repeated base actor ids: k_doc decides
  if (l < N) {
    a_canon = CANON[NB + ambase];
    if (a_canon >= NB) atomicMin(&FIRST[a_canon], l);
  }
  wsync();
  const bool newauth = l < N && a_canon >= NB && FIRST[a_canon] == l;
  const uint64_t nam = __ballot(newauth);
  const uint32_t NA = NB + __popcll(nam);
  if (l < NB) { M[FM_DPC + l] = (uint8_t)l; M[FM_DP2REF + l] = (uint8_t)l; }
  if (newauth) {
    const uint32_t dp = NB + __popcll(nam & lt_mask());
    M[FM_DPC + a_canon] = (uint8_t)dp;
    M[FM_DP2REF + dp] = (uint8_t)(NB + ambase);
  }
  wsync();
  uint32_t a_dp = 0;  // doc actor index of change l's author
  if (l < N) {
    a_dp = a_canon < NB ? a_canon : M[FM_DPC + a_canon];
    for (uint32_t k = 1; k < c_nact; k++) {
      const uint32_t cr = CANON[NB + ambase + k];
      if (cr >= NB && !(FIRST[cr] <= l)) bad = true;  // actorId ... is not known to document
    }
  }
  if (l < NA) M[FM_RANKDP + l] = M[FM_RANKC + CANON[M[FM_DP2REF + l]]];
  wsync();
  FD_CHECK();
  const uint8_t* DPC = M + FM_DPC;
  const uint8_t* RANKDP = M + FM_RANKDP;

  FPH(2);
  // ---- base document change rows (DOCUMENT_COLUMNS, lane per column), then lane per row ----
  int64_t* DCC = reinterpret_cast<int64_t*>(S + F.rw);  // [9][nbc] (+ deps at [9*nbc]), after the hash table
  if (has_base && l < DC_NCOLS) {
    const uint32_t col = l;
    const uint64_t off = dhb + dh->ccol_off[col];
    const uint32_t len = dh->ccol_len[col];
    ColDec d;
    const uint8_t type = (col == DC_ACTOR || col == DC_DEPS_NUM || col == DC_EXTRA_LEN) ? DT_UINT
                         : col == DC_MESSAGE                                          ? DT_UTF8
                                                                                      : DT_INT;
    cd_init(d, type, IN + (off - a0), len);
    const uint32_t n = col == DC_DEPS_INDEX ? nbd : (col == DC_EXTRA_RAW ? 0u : nbc);
    int64_t* dst = col == DC_DEPS_INDEX ? DCC + 9 * nbc : DCC + col * nbc;
    for (uint32_t i = 0; i < n; i++) {
      int64_t v = 0;
      uint32_t e;
      if (type == DT_UTF8) {
        uint64_t so;
        uint32_t sl;
        e = cd_next_str(d, so, sl);
        v = sl == AM_NOSTR ? AM_NULL64 : (int64_t)(((off + so - a0) << 32) | sl);
        if (!e && sl != AM_NOSTR && !utf8_valid_dev(IN + (off + so - a0), sl)) bad = true;
      } else if (col == DC_SEQ || col == DC_MAXOP || col == DC_TIME || col == DC_DEPS_INDEX) {
        e = cd_next_delta(d, v);
      } else {
        e = cd_next_int(d, v);
      }
      if (e) { bad = true; break; }
      dst[i] = v;
    }
  }
  wsync();
  FD_CHECK();
  // base change row l: actor, seq, maxOp, time, message, deps, extra (readDocumentChanges)
  int64_t bc_seq = 0, bc_max = 0, bc_time = 0, bc_msg = AM_NULL64, bc_xlen = 7;
  uint32_t bc_actor = 0, bc_nd = 0, bc_xoff = 0, bc_xraw = 0;
  const int64_t bc_dep = l < nbd ? DCC[9 * nbc + l] : 0;  // base depsIndex value l (cells are reused below)
  {
    int64_t a = 0;
    if (l < nbc) {
      a = DCC[DC_ACTOR * nbc + l];
      bc_seq = DCC[DC_SEQ * nbc + l];
      bc_max = DCC[DC_MAXOP * nbc + l];
      bc_time = DCC[DC_TIME * nbc + l];
      bc_msg = DCC[DC_MESSAGE * nbc + l];
      const int64_t nd = DCC[DC_DEPS_NUM * nbc + l];
      bc_nd = nd == AM_NULL64 ? 0u : (uint32_t)nd;
      bc_xlen = DCC[DC_EXTRA_LEN * nbc + l];
      bc_xraw = bc_xlen == AM_NULL64 ? 0u : (uint32_t)((uint64_t)bc_xlen >> 4);
      bad |= a == AM_NULL64 || a < 0 || a >= (int64_t)NB || bc_seq == AM_NULL64 || nd > 64;
      bc_actor = (uint32_t)a;
    }
    uint32_t xt, dt;
    const uint32_t xo = excl_add(l < nbc ? bc_xraw : 0u, xt);
    excl_add(l < nbc ? bc_nd : 0u, dt);
    if (has_base) bad |= xt > dh->ccol_len[DC_EXTRA_RAW] || dt != nbd;
    bc_xoff = (uint32_t)(dhb + dh->ccol_off[DC_EXTRA_RAW] + xo - a0);
    // clock: seq must count 1, 2, ... per actor in row order (new.js:1654-1660)
    uint32_t before = 0;
    for (uint32_t j = 0; j < nbc; j++) {
      const uint32_t aj = wave::bcast(bc_actor, (int)j);
      if (j < l && aj == bc_actor) before++;
    }
    uint32_t* CLK = reinterpret_cast<uint32_t*>(M + FM_CLOCK);
    CLK[l] = 0;
    wsync();
    if (l < nbc) {
      bad |= bc_seq != (int64_t)before + 1;
      atomicMax(&CLK[bc_actor], (uint32_t)bc_seq);
    }
  }
  wsync();
  FD_CHECK();

  FPH(3);
  // ---- causal queue, first pass (applyChanges, new.js:1550-1597): every change must be new,
  // ready in list order and carry the next seq of its author ----
  uint32_t prior = 0;  // earlier changes of this call by the same author
  for (uint32_t j = 0; j < N; j++) prior += (wave::bcast(a_dp, (int)j) == a_dp && j < l) ? 1u : 0u;
  // hash t's first 8 bytes in lane t (t < N + HB + K): candidates are found by broadcasting the
  // prefixes (readlane, no LDS traffic); only a prefix hit compares the full 32 bytes
  const uint32_t NHT = N + HB + K;
  const uint64_t hpre = l < NHT ? (((uint64_t)HT[8 * l + 1] << 32) | HT[8 * l]) : ~0ull;
  {
    uint64_t hitmask = 0;  // (lane-local) earlier changes / heads / known hashes with an equal prefix
    for (uint32_t t = 0; t < NHT; t++) {
      const uint64_t pt = wave::bcast(hpre, (int)t);
      if (pt == hpre && t != l && !(t < N && t > l)) hitmask |= 1ull << t;
    }
    if (l < N) {
      uint32_t mine[8];
#pragma unroll
      for (int k = 0; k < 8; k++) mine[k] = HT[8 * l + k];
      while (hitmask) {
        const uint32_t t = (uint32_t)__builtin_ctzll(hitmask);
        hitmask &= hitmask - 1;
        if (words_eq(HT + 8 * t, mine)) { bad = true; break; }  // duplicate / already applied
      }
    }
  }
  if (l < N) {
    const uint32_t* CLK = reinterpret_cast<const uint32_t*>(M + FM_CLOCK);
    const int64_t expect = (int64_t)(a_dp < NB ? CLK[a_dp] : 0u) + prior + 1;
    bad |= chh[l].seq != expect;
  }
  uint32_t nd_total;
  const uint32_t dbase = excl_add(l < N ? c_ndeps : 0u, nd_total);
  bad |= nd_total != b.ND;
  uint8_t* DEPD = M + FM_DEPD;
  DEPD[l] = 0;
  if (l < N)
    for (uint32_t k = 0; k < c_ndeps; k++) M[FM_DOWN + dbase + k] = (uint8_t)l;
  wsync();
  FD_CHECK();
  // dependency q: a base head, a host-known change or an earlier change of this call
  int64_t dep_idx = 0;
  const uint32_t dep_c = l < nd_total ? M[FM_DOWN + l] : 0u;
  const uint32_t dep_b = __shfl(dbase, dep_c, 64);
  uint32_t w[8];
  uint64_t dpre = ~0ull;
  if (l < nd_total) {
    const ChgHdrC& h = chh[dep_c];
    load32(IN + (h.base + h.deps_off + 32 * (l - dep_b) - a0), w);
    dpre = ((uint64_t)w[1] << 32) | w[0];
  }
  uint64_t dmask = 0;  // hashes with the dependency's prefix
  for (uint32_t t = 0; t < NHT; t++)
    if (wave::bcast(hpre, (int)t) == dpre) dmask |= 1ull << t;
  if (l < nd_total) {
    const uint32_t c = dep_c;
    int32_t hit = -1;
    // base heads and host-known hashes first, then the changes of this call
    for (uint64_t m = dmask >> N; m && hit < 0; m &= m - 1) {
      const uint32_t t = N + (uint32_t)__builtin_ctzll(m);
      if (words_eq(HT + 8 * t, w)) hit = (int32_t)t;
    }
    if (hit >= 0) {
      dep_idx = hit < (int32_t)(N + HB) ? reinterpret_cast<const int64_t*>(S + F.bk)[hit - N]
                                        : reinterpret_cast<const int64_t*>(S + F.bk + 8 * HB)[hit - N - HB];
      if (dep_idx < 0) bad = true;
    } else {
      for (uint64_t m = dmask & (N < 64 ? (1ull << N) - 1 : ~0ull); m && hit < 0; m &= m - 1) {
        const uint32_t t = (uint32_t)__builtin_ctzll(m);
        if (words_eq(HT + 8 * t, w)) hit = (int32_t)t;
      }
      if (hit < 0 || (uint32_t)hit >= c) bad = true;  // missing or later: the change would wait
      dep_idx = (int64_t)nbc + hit;
    }
    if (hit >= 0 && hit < (int32_t)(N + HB)) DEPD[hit] = 1;
  }
  wsync();
  FD_CHECK();
  // heads: base heads and changes that nothing in this call depends on, sorted (new.js:1581-1593)
  uint32_t NH;
  {
    const uint32_t ncand = N + HB;
    const bool ishead = l < ncand && !DEPD[l];
    const uint64_t pre = l < ncand ? bswap64(((uint64_t)HT[8 * l + 1] << 32) | HT[8 * l]) : 0;
    uint32_t pos = 0;
    for (uint32_t y = 0; y < ncand; y++) {
      const uint64_t py = wave::bcast(pre, (int)y);
      const int32_t hy = wave::bcast((int32_t)ishead, (int)y);
      if (hy && y != l) {
        if (py < pre) pos++;
        else if (py == pre) bad = true;  // equal 8-byte prefixes: k_doc sorts full hashes
      }
    }
    NH = __popcll(__ballot(ishead));
    if (ishead) {
      const int64_t hidx = l < N ? (int64_t)nbc + l : reinterpret_cast<const int64_t*>(S + F.bk)[l - N];
      bad |= hidx < 0;
      reinterpret_cast<int32_t*>(M + FM_HIDX)[pos] = (int32_t)hidx;  // < nbc + N <= 128
      M[FM_HSEL + pos] = (uint8_t)l;
      uint4* hg = reinterpret_cast<uint4*>(wsg + L.heads + 32 * pos);
      hg[0] = reinterpret_cast<const uint4*>(HT + 8 * l)[0];
      hg[1] = reinterpret_cast<const uint4*>(HT + 8 * l)[1];
    }
  }
  FD_CHECK();

  FPH(4);
  // ---- op columns: lane per (source, column) stream into 4-byte cells (readOperation,
  // new.js:570-611) ----
  const uint32_t nsrc = (has_base ? 1u : 0u) + N;
  const uint32_t R = b.R, E = b.E;
  // source s: rows [row0, row0 + nr), entries [ent0, ent0 + ne)
  uint32_t s_nr = 0, s_ne = 0;
  {
    // lane s holds source s's counts
    const uint32_t c = has_base ? l - 1 : l;
    const uint32_t cnops = __shfl(c_nops, c & 63, 64), cnents = __shfl(c_nents, c & 63, 64);
    if (l < nsrc) {
      if (has_base && l == 0) { s_nr = nb; s_ne = nbe; }
      else { s_nr = cnops; s_ne = cnents; }
    }
  }
  uint32_t rtot, etot;
  const uint32_t s_row0 = excl_add(s_nr, rtot), s_ent0 = excl_add(s_ne, etot);
  bad |= rtot != R || etot != E || (l < nsrc && s_nr == 0 && s_ne != 0);
  uint8_t* ROW0 = M + FM_ROW0;  // values <= 64 in a document that stays here (else `bad` ends it below)
  uint8_t* ENT0 = M + FM_ENT0;
  ROW0[l] = (uint8_t)s_row0;
  ENT0[l] = (uint8_t)s_ent0;
  if (l == 0) { ROW0[64] = (uint8_t)rtot; ENT0[64] = (uint8_t)etot; }
  int32_t* SRCR = reinterpret_cast<int32_t*>(M + FM_SRCR);
  int32_t* SRCE = reinterpret_cast<int32_t*>(M + FM_SRCE);
  SRCR[l] = -1;
  SRCE[l] = -1;
  wsync();
  if (l < nsrc && s_nr) SRCR[s_row0] = (int32_t)l;
  if (l < nsrc && s_ne) SRCE[s_ent0] = (int32_t)l;
  FD_CHECK();
  int32_t* CELL = reinterpret_cast<int32_t*>(S + F.cells);
  // stream (source s, op column col) -> its cells: rows [ROW0[s], ROW0[s+1]) of cell column j
  // (j < 13), or entries [ENT0[s], ENT0[s+1]) of entry column j - 13
  auto stream = [&](uint32_t s, uint32_t col, uint32_t& off, uint32_t& len, uint32_t& n, int32_t*& dst) -> bool {
    const bool chg_src = !(has_base && s == 0);
    if (chg_src && (col == OC_ID_ACTOR || col == OC_ID_CTR)) return false;  // ids from the header
    const uint32_t c = has_base ? s - 1 : s;
    if (chg_src) {
      off = (uint32_t)(chh[c].base - a0) + chh[c].col_off[col];
      len = chh[c].col_len[col];
    } else {
      off = (uint32_t)(dhb - a0) + dh->ocol_off[col];
      len = dh->ocol_len[col];
    }
    const uint32_t j = col < OC_VAL_RAW ? col : col - 1;
    const uint32_t r0 = ROW0[s], e0 = ENT0[s];
    n = j < 13 ? ROW0[s + 1] - r0 : ENT0[s + 1] - e0;
    dst = j < 13 ? CELL + j * R + r0 : CELL + 13 * R + (j - 13) * E + e0;
    return true;
  };
  // type-uniform rounds: lanes take (source, column) pairs of one decoder type at a time
  {
    // the column lists as nibbles of one constant (a lane's column is a shift, not a table load)
    constexpr uint64_t kU = (uint64_t)OC_OBJ_ACTOR | (uint64_t)OC_OBJ_CTR << 4 | (uint64_t)OC_KEY_ACTOR << 8 |
                            (uint64_t)OC_ID_ACTOR << 12 | (uint64_t)OC_ACTION << 16 | (uint64_t)OC_VAL_LEN << 20 |
                            (uint64_t)OC_CHLD_ACTOR << 24 | (uint64_t)OC_GRP_NUM << 28 | (uint64_t)OC_GRP_ACTOR << 32;
    constexpr uint32_t kD = (uint32_t)OC_KEY_CTR | (uint32_t)OC_ID_CTR << 4 | (uint32_t)OC_CHLD_CTR << 8 |
                            (uint32_t)OC_GRP_CTR << 12;
    static_assert(OC_NCOLS <= 16, "op column ids fit a nibble");
    uint32_t off, len, n;
    int32_t* dst;
    for (uint32_t it = l; it < nsrc * 9; it += 64)
      if (stream(it / 9, (uint32_t)(kU >> (4 * (it % 9))) & 15u, off, len, n, dst))
        d32_stream<DT_UINT>(IN, off, len, n, dst, bad);
    for (uint32_t it = l; it < nsrc * 4; it += 64)
      if (stream(it >> 2, (kD >> (4 * (it & 3))) & 15u, off, len, n, dst)) d32_stream<DT_DELTA>(IN, off, len, n, dst, bad);
    for (uint32_t it = l; it < nsrc * 2; it += 64) {
      const uint32_t s2 = it >> 1;
      if (it & 1) { if (stream(s2, OC_INSERT, off, len, n, dst)) d32_stream<DT_BOOL>(IN, off, len, n, dst, bad); }
      else if (stream(s2, OC_KEY_STR, off, len, n, dst)) d32_stream<DT_UTF8>(IN, off, len, n, dst, bad);
    }
  }
  wsync();
  FD_CHECK();

  FPH(5);
  // ---- rows: lane per op row (gather_row) ----
  const int32_t r_src = incl_max(l < R ? SRCR[l] : -1);
  const bool isrow = l < R;
  const bool r_chg = isrow && !(has_base && r_src == 0);
  const uint32_t r_c = has_base ? (uint32_t)r_src - 1 : (uint32_t)r_src;  // change index of a change row
  const uint32_t r_q = isrow ? l - ROW0[r_src] : 0;
  // actor index of a change row maps through its change's actor list
  const uint32_t cnact = __shfl(c_nact, r_c & 63, 64), cab = __shfl(ambase, r_c & 63, 64);
  int64_t cstart = 0;
  if (r_chg) cstart = chh[r_c].start_op;
  const int32_t c_adp = (int32_t)__shfl(a_dp, r_c & 63, 64);
  auto mapact = [&](int32_t v) -> int32_t {
    if (v == FD_NULL) return -1;
    if (r_chg) {
      if (v < 0 || (uint32_t)v >= cnact) { bad = true; return 0; }
      return DPC[CANON[NB + cab + v]];
    }
    if (v < 0 || (uint32_t)v >= NB) { bad = true; return 0; }
    return v;
  };
  int32_t r_objc = FD_NULL, r_obja = -1, r_keyc = FD_NULL, r_keya = -1, r_key = FD_NULL, r_idc = 0, r_ida = 0;
  int32_t r_act = 0, r_vlen = FD_NULL, r_chc = FD_NULL, r_cha = -1, r_pcnt = 0;
  bool r_ins = false;
  if (isrow) {
    const int32_t* c = CELL + l;
    r_obja = mapact(c[0]);
    r_objc = c[R];
    r_keya = mapact(c[2 * R]);
    r_keyc = c[3 * R];
    r_key = c[4 * R];
    if (r_chg) { r_ida = c_adp; const int64_t x = cstart + r_q; bad |= x > 0x7fffffffLL; r_idc = (int32_t)x; }
    else { r_ida = mapact(c[5 * R]); r_idc = c[6 * R]; bad |= c[5 * R] == FD_NULL || r_idc == FD_NULL; }
    r_ins = c[7 * R] != 0;
    r_act = c[8 * R];
    r_vlen = c[9 * R];
    r_cha = mapact(c[10 * R]);
    r_chc = c[11 * R];
    r_pcnt = c[12 * R] == FD_NULL ? 0 : c[12 * R];
    bad |= r_act == FD_NULL || r_pcnt < 0 || (r_vlen != FD_NULL && r_vlen < 0);
    if (r_key != FD_NULL && !utf8_valid_dev(IN + ((uint32_t)r_key >> 8), (uint32_t)r_key & 255)) bad = true;
  }
  const bool r_del = r_chg && r_act == 3;
  const uint32_t r_vb = (isrow && r_vlen != FD_NULL) ? ((uint32_t)r_vlen >> 4) : 0u;
  uint32_t vtot, ptot;
  const uint32_t vsum = excl_add(r_vb, vtot);
  const uint32_t r_psoff = excl_add(isrow ? (uint32_t)r_pcnt : 0u, ptot);
  const uint32_t r_row0 = isrow ? ROW0[r_src] : 0;
  const uint32_t vsum0 = __shfl(vsum, r_row0 & 63, 64), psum0 = __shfl(r_psoff, r_row0 & 63, 64);
  uint32_t r_voff = 0;  // valRaw bytes of the row, relative to a0
  if (isrow) {
    uint64_t cbase = dhb;
    uint32_t coff, clen;
    if (r_chg) {
      cbase = chh[r_c].base;
      coff = chh[r_c].col_off[OC_VAL_RAW];
      clen = chh[r_c].col_len[OC_VAL_RAW];
    } else {
      coff = dh->ocol_off[OC_VAL_RAW];
      clen = dh->ocol_len[OC_VAL_RAW];
    }
    r_voff = (uint32_t)(cbase + coff - a0) + (vsum - vsum0);
    if (l + 1 == ROW0[r_src + 1] || l + 1 == R) {  // last row of its source
      bad |= (vsum - vsum0) + r_vb > clen;
      bad |= r_psoff + (uint32_t)r_pcnt - psum0 != ENT0[r_src + 1] - ENT0[r_src];
    }
  }
  bad |= ptot != E;
  // entries: lane per pred/succ entry
  const int32_t e_src = incl_max(l < E ? SRCE[l] : -1);
  const bool isent = l < E;
  const bool e_chg = isent && !(has_base && e_src == 0);
  int32_t e_ctr = 0, e_act = 0;
  {
    const uint32_t ec = has_base ? (uint32_t)e_src - 1 : (uint32_t)e_src;
    const uint32_t enact = __shfl(c_nact, ec & 63, 64), eab = __shfl(ambase, ec & 63, 64);
    if (isent) {
      const int32_t a = CELL[13 * R + l], ctr = CELL[13 * R + E + l];
      if (a == FD_NULL || ctr == FD_NULL) bad = true;
      else if (e_chg) {
        if (a < 0 || (uint32_t)a >= enact) bad = true;
        else e_act = DPC[CANON[NB + eab + a]];
      } else {
        if (a < 0 || (uint32_t)a >= NB) bad = true;
        else e_act = a;
      }
      e_ctr = ctr;
    }
  }
  // maxOp: base op ids and succ counters, applied changes' last op (new.js:1627-1630, 1749)
  int64_t maxop = 0;
  if (isrow && !r_chg) maxop = r_idc;
  if (isent && !e_chg && e_ctr > maxop) maxop = e_ctr;
  if (l < N && c_nops > 0) {
    const int64_t m = chh[l].start_op + (int64_t)c_nops - 1;
    if (m > maxop) maxop = m;
  }
  maxop = max_all(maxop);
  // per-op checks of change rows (readNextChangeOp new.js:715-723, mergeDocChangeOps shapes)
  if (r_chg) {
    bad |= (r_objc == FD_NULL) != (r_obja < 0);
    bad |= (r_keyc == FD_NULL && r_keya >= 0) || (r_keyc == 0 && r_keya >= 0) || (r_keyc != FD_NULL && r_keyc > 0 && r_keya < 0);
    bad |= r_del && (r_ins || r_pcnt == 0);
    bad |= r_ins && r_pcnt > 0;
    bad |= r_key == FD_NULL && !r_ins && r_keyc == FD_NULL;
  }
  if (isrow) bad |= r_idc < 0 || (r_objc != FD_NULL && r_objc < 0);
  FD_CHECK();

  FPH(6);
  // ---- opId order: (counter, actor rank) (new.js:1197-1224) ----
  const uint32_t r_rank = isrow ? RANKDP[r_ida] : 0;
  uint64_t* IDT = reinterpret_cast<uint64_t*>(S + F.cells);  // the decoded cells are in registers now
  uint32_t r_opr;
  {
    const uint64_t key = isrow ? ((uint64_t)(uint32_t)r_idc << 12) | (r_rank << 6) | l : ~0ull;
    const uint64_t s = sort64(key);
    const uint64_t prev = wave::up1(s, ~0ull);
    if (l > 0 && l < R && (prev >> 6) == (s >> 6)) bad = true;  // duplicate operation ID
    IDT[l] = s;
    if (l < R) M[FM_OPR + (s & 63)] = (uint8_t)l;
    wsync();
    r_opr = M[FM_OPR + l];
  }
  FD_CHECK();
  auto lookup = [&](int32_t ctr, uint32_t rank) -> int32_t {
    if (ctr < 0) return -1;
    const uint64_t want = ((uint64_t)(uint32_t)ctr << 6) | rank;
    uint32_t lo = 0, hi = R;
    while (lo < hi) {
      const uint32_t m = (lo + hi) >> 1;
      if ((IDT[m] >> 6) < want) lo = m + 1; else hi = m;
    }
    return (lo < R && (IDT[lo] >> 6) == want) ? (int32_t)(IDT[lo] & 63) : -1;
  };

  // ---- map keys: rank in UTF-16 order. Keys whose bytes stay below 0xEE compare in UTF-16
  // order exactly as bytes (only supplementary characters reorder against U+E000..U+FFFF) ----
  const bool keyed = isrow && r_key != FD_NULL;
  uint32_t r_krank = 0;
  {
    const uint32_t koff = keyed ? ((uint32_t)r_key >> 8) : 0, klen = keyed ? ((uint32_t)r_key & 255) : 0;
    uint64_t pre = 0;
    for (uint32_t q = 0; q < klen; q++) {
      const uint8_t c = IN[koff + q];
      if (c >= 0xee) bad = true;
      if (q < 8) pre |= (uint64_t)c << (56 - 8 * q);
    }
    uint64_t km = __ballot(keyed);
    while (km) {
      const uint32_t j = (uint32_t)__builtin_ctzll(km);
      km &= km - 1;
      const uint64_t pj = wave::bcast(pre, (int)j);
      const uint32_t kj = (uint32_t)wave::bcast(r_key, (int)j);
      if (!keyed || j == l) continue;
      bool less = pj < pre;
      if (pj == pre) {
        const uint32_t jo = kj >> 8, jl = kj & 255;
        uint32_t q = 8;
        while (q < jl && q < klen && IN[jo + q] == IN[koff + q]) q++;
        less = (q < jl && q < klen) ? IN[jo + q] < IN[koff + q] : jl < klen;
      }
      if (less) r_krank++;
    }
  }
  FD_CHECK();

  FPH(7);
  // ---- preds -> target rows (new.js:1173-1188, 1254-1258) ----
  uint8_t* OWN = M + FM_OWN;
  if (r_chg)
    for (int32_t q = 0; q < r_pcnt; q++) OWN[r_psoff + q] = (uint8_t)l;
  wsync();
  const bool e_new = isent && e_chg;
  int32_t e_tr = -1;
  uint32_t e_orank = 0, e_octr = 0;
  {
    const uint32_t o = e_new ? OWN[l] : 0;
    const int32_t o_objc = __shfl(r_objc, o, 64), o_obja = __shfl(r_obja, o, 64), o_key = __shfl(r_key, o, 64);
    const uint32_t o_kr = __shfl(r_krank, o, 64);
    const int32_t o_keyc = __shfl(r_keyc, o, 64), o_keya = __shfl(r_keya, o, 64), o_idc = __shfl(r_idc, o, 64);
    const uint32_t o_rank = __shfl(r_rank, o, 64);
    const int32_t tr = e_new ? lookup(e_ctr, RANKDP[e_act]) : -1;
    const uint32_t t = tr < 0 ? 0u : (uint32_t)tr;
    const int32_t t_objc = __shfl(r_objc, t, 64), t_obja = __shfl(r_obja, t, 64), t_key = __shfl(r_key, t, 64);
    const uint32_t t_kr = __shfl(r_krank, t, 64);
    const int32_t t_keyc = __shfl(r_keyc, t, 64), t_keya = __shfl(r_keya, t, 64), t_idc = __shfl(r_idc, t, 64);
    const int32_t t_ida = __shfl(r_ida, t, 64);
    const uint32_t t_rank = __shfl(r_rank, t, 64);
    const int32_t t_ins = __shfl((int32_t)r_ins, t, 64), t_del = __shfl((int32_t)r_del, t, 64);
    if (e_new) {
      bool ok = tr >= 0 && (uint32_t)tr < o && !t_del && t_objc == o_objc && t_obja == o_obja &&
                (t_idc < o_idc || (t_idc == o_idc && t_rank < o_rank));
      if (ok) {
        if (o_key != FD_NULL) ok = t_key != FD_NULL && t_kr == o_kr;
        else {
          const int32_t ec = t_ins ? t_idc : t_keyc, ea = t_ins ? t_ida : t_keya;
          ok = t_key == FD_NULL && ec == o_keyc && ea == o_keya;
        }
      }
      if (!ok) bad = true;
      e_tr = tr;
      e_orank = o_rank;
      e_octr = (uint32_t)o_idc;
    }
  }
  FD_CHECK();

  // ---- list elements: reference element of inserts, target element of updates ----
  int32_t r_parent = -1, r_elem = -1;
  {
    int32_t want_c = -1;
    uint32_t want_r = 0;
    const bool listop = isrow && r_key == FD_NULL && !r_del;
    if (listop && !(r_ins && (r_keyc == FD_NULL || r_keyc == 0 || r_keya < 0))) {
      if (r_keya >= 0) { want_c = r_keyc; want_r = RANKDP[r_keya]; }
    }
    const int32_t p = want_c >= 0 ? lookup(want_c, want_r) : -1;
    const uint32_t pu = p < 0 ? 0u : (uint32_t)p;
    const int32_t p_ins = __shfl((int32_t)r_ins, pu, 64), p_del = __shfl((int32_t)r_del, pu, 64);
    const int32_t p_objc = __shfl(r_objc, pu, 64), p_obja = __shfl(r_obja, pu, 64), p_key = __shfl(r_key, pu, 64);
    const int32_t p_idc = __shfl(r_idc, pu, 64);
    const uint32_t p_rank = __shfl(r_rank, pu, 64);
    if (listop) {
      if (r_ins) {
        r_elem = (int32_t)l;
        if (!(r_keyc == FD_NULL || r_keyc == 0 || r_keya < 0)) {
          const bool ok = p >= 0 && p_ins && !p_del && p_objc == r_objc && p_obja == r_obja && p_key == FD_NULL &&
                          (!r_chg || (uint32_t)p < l) && p_idc < r_idc;
          if (!ok) bad = true;
          r_parent = p;
        }
      } else {
        const bool ok = p >= 0 && p_ins && !p_del && p_objc == r_objc && p_obja == r_obja && p_key == FD_NULL &&
                        (!r_chg || (uint32_t)p < l) && (p_idc < r_idc || (p_idc == r_idc && p_rank < r_rank));
        if (!ok) bad = true;
        r_elem = p;
      }
    }
  }
  FD_CHECK();
  const uint64_t r_objkey = (!isrow || r_objc == FD_NULL) ? 0ull
                                                          : (((uint64_t)(uint32_t)r_objc + 1) << 6) | (r_obja < 0 ? 0u : RANKDP[r_obja]);

  FPH(8);
  // ---- RGA order: preorder of the reference-element tree, children by descending opId
  // (new.js:145-163); Euler tour + pointer jumping gives each element its suffix count ----
  int8_t* FC = reinterpret_cast<int8_t*>(M + FM_FC);
  int8_t* NS = reinterpret_cast<int8_t*>(M + FM_NS);
  FC[l] = -1;
  NS[l] = -1;
  wsync();
  const bool is_el = isrow && r_elem == (int32_t)l;
  {
    const uint64_t key = is_el ? (r_objkey << 19) | ((uint64_t)(r_parent + 1) << 12) | ((uint64_t)(63 - r_opr) << 6) | l : ~0ull;
    const uint64_t s = sort64(key);
    const uint64_t nx = wave::down1(s, ~0ull), pv = wave::up1(s, ~0ull);
    if (s != ~0ull) {
      const uint32_t row = (uint32_t)(s & 63);
      if (l < 63 && nx != ~0ull && (nx >> 12) == (s >> 12)) NS[row] = (int8_t)(nx & 63);
      const int32_t par = (int32_t)((s >> 12) & 127) - 1;
      if ((l == 0 || (pv >> 12) != (s >> 12)) && par >= 0) FC[par] = (int8_t)row;
    }
  }
  wsync();
  uint32_t r_suffix = 0;
  {
    const int32_t END = -1;
    int32_t n0 = END, n1 = END;
    uint32_t w0 = 0, w1 = 0;
    if (is_el) {
      n0 = FC[l] >= 0 ? 2 * FC[l] : (int32_t)(2 * l + 1);
      w0 = 1;
      n1 = NS[l] >= 0 ? 2 * NS[l] : (r_parent >= 0 ? 2 * r_parent + 1 : END);
    }
#pragma unroll 1
    for (int round = 0; round < 7; round++) {
      const uint32_t t0 = n0 < 0 ? 0u : (uint32_t)n0 >> 1, t1 = n1 < 0 ? 0u : (uint32_t)n1 >> 1;
      const int32_t a_n0 = __shfl(n0, t0, 64), a_n1 = __shfl(n1, t0, 64);
      const uint32_t a_w0 = __shfl(w0, t0, 64), a_w1 = __shfl(w1, t0, 64);
      const int32_t b_n0 = __shfl(n0, t1, 64), b_n1 = __shfl(n1, t1, 64);
      const uint32_t b_w0 = __shfl(w0, t1, 64), b_w1 = __shfl(w1, t1, 64);
      if (n0 != END) {
        const bool odd = n0 & 1;
        w0 += odd ? a_w1 : a_w0;
        n0 = odd ? a_n1 : a_n0;
      }
      if (n1 != END) {
        const bool odd = n1 & 1;
        w1 += odd ? b_w1 : b_w0;
        n1 = odd ? b_n1 : b_n0;
      }
    }
    bad |= n0 != END || n1 != END;  // chain longer than 128 nodes cannot happen; stay safe
    r_suffix = w0;
  }
  FD_CHECK();

  FPH(9);
  // ---- document order: object, then key (UTF-16) | list position, then opId ----
  const bool isout = isrow && !r_del;
  const uint32_t NOUT = __popcll(__ballot(isout));
  uint32_t k_row;  // row at output position l
  {
    const uint32_t esuf = __shfl(r_suffix, r_elem < 0 ? 0u : (uint32_t)r_elem, 64);
    const uint64_t k2 = keyed ? r_krank : (uint64_t)(64 - esuf);
    const uint64_t key = isout ? (r_objkey << 20) | ((uint64_t)(keyed ? 0 : 1) << 19) | (k2 << 12) | ((uint64_t)r_opr << 6) | l
                               : ~0ull;
    k_row = (uint32_t)(sort64(key) & 63);
  }

  // ---- succ lists: base succs merged with the new succs of each row (new.js:1173-1188) ----
  uint64_t* BENT = reinterpret_cast<uint64_t*>(S + F.cells + 512);
  uint64_t* NSORT = reinterpret_cast<uint64_t*>(S + F.cells);
  uint32_t* CNTN = reinterpret_cast<uint32_t*>(M + FM_CNTN);
  uint8_t* LON = M + FM_LON;
  CNTN[l] = 0;
  if (isent && !e_chg) BENT[l] = ((uint64_t)(uint32_t)e_ctr << 6) | RANKDP[e_act];
  wsync();
  {
    const uint64_t key = e_new ? ((uint64_t)e_tr << 37) | ((uint64_t)e_octr << 6) | e_orank : ~0ull;
    const uint64_t s = sort64(key);
    NSORT[l] = s;
    const uint64_t pv = wave::up1(s, ~0ull);
    if (s != ~0ull) {
      const uint32_t tg = (uint32_t)(s >> 37);
      if (l == 0 || (pv >> 37) != tg) LON[tg] = (uint8_t)l;
      atomicAdd(&CNTN[tg], 1u);
    }
  }
  wsync();
  int32_t* OUTC = reinterpret_cast<int32_t*>(M + FM_OUTC);
  uint8_t* OUTA = M + FM_OUTA;
  uint8_t* const RANK2DP = M + FM_CANON;  // canon table is dead: reuse as rank -> doc actor index
  wsync();
  if (l < NA) RANK2DP[RANKDP[l]] = (uint8_t)l;
  wsync();
  uint32_t NSUCC, sc_k, so_k;
  {
    const uint32_t r = k_row;
    const int32_t k_chg = __shfl((int32_t)r_chg, r, 64), k_pc = __shfl(r_pcnt, r, 64);
    const uint32_t k_pso = __shfl(r_psoff, r, 64);
    const bool out = l < NOUT;
    const uint32_t nold = (out && !k_chg) ? (uint32_t)k_pc : 0u;
    const uint32_t nnew = out ? CNTN[r] : 0u;
    sc_k = nold + nnew;
    so_k = excl_add(sc_k, NSUCC);
    if (out) {
      const uint32_t lo = nnew ? LON[r] : 0;
      uint32_t a = 0, b2 = 0, w = so_k;
      while (a < nold || b2 < nnew) {
        bool take_old;
        const uint64_t eo = a < nold ? BENT[k_pso + a] : 0, en = b2 < nnew ? NSORT[lo + b2] : 0;
        if (a >= nold) take_old = false;
        else if (b2 >= nnew) take_old = true;
        else {
          const uint64_t oc = eo >> 6, nc = (en >> 6) & 0x7fffffffull;
          take_old = oc < nc || (oc == nc && (eo & 63) < (en & 63));
        }
        if (take_old) { OUTC[w] = (int32_t)(eo >> 6); OUTA[w] = RANK2DP[eo & 63]; a++; }
        else { OUTC[w] = (int32_t)((en >> 6) & 0x7fffffffull); OUTA[w] = RANK2DP[en & 63]; b2++; }
        w++;
      }
    }
  }
  bad |= NSUCC > FD_MAX;
  wsync();
  FD_CHECK();
  // the row values fast_diff reads after the encode, parked in misc tables the merge is done with
  // (registers would stay live through the encode and spill)
  if (kDiff && b.P) {
    const FdRec P = fd_rec(M, S + F.cells + F.ob_cap);
    if (isrow) {
      P.key[l] = (uint32_t)r_key; P.objc[l] = r_objc; P.idc[l] = r_idc; P.vlen[l] = r_vlen;
      P.voff[l] = (uint16_t)r_voff; P.obja[l] = (int8_t)r_obja; P.ida[l] = (uint8_t)r_ida; P.krank[l] = (uint8_t)r_krank;
      P.elem[l] = (int8_t)r_elem; P.act[l] = (uint8_t)(r_act < 0 || r_act > 255 ? 255 : r_act);
      P.flags[l] = (uint8_t)((r_chg ? 1u : 0u) | (r_ins ? 2u : 0u) | (keyed ? 4u : 0u));
    }
    if (l < NOUT) { P.krow[l] = (uint8_t)k_row; P.sck[l] = (uint8_t)sc_k; P.sok[l] = (uint8_t)so_k; }
    if (l < nbc) { P.bca[l] = (uint8_t)bc_actor; P.bcs[l] = (uint32_t)bc_seq; }
    if (l < N) P.adp[l] = (uint8_t)a_dp;
    bad |= isrow && r_voff > 0xffff;
    bad |= l < nbc && (bc_seq < 0 || bc_seq > 0xffffffffLL);
  }
  wsync();
  FD_CHECK();

  FPH(10);
  // ---- canonical re-encode into the output image (cells are dead) ----
  uint8_t* const OB = S + F.cells;
  uint32_t* COLLEN = reinterpret_cast<uint32_t*>(M + FM_COLLEN);
  // header reserve: magic, checksum, type, body length, actors, heads, column tables
  uint32_t alen_sum;
  const uint32_t a_len = l < NA ? RO[2 * M[FM_DP2REF + l] + 1] : 0u;
  const uint32_t a_pos = excl_add(l < NA ? (uint32_t)uleb_len(a_len) + a_len : 0u, alen_sum);
  const uint32_t T0 = 9 + 10 + 10 + alen_sum + 10 + 32 * NH + 2 * (10 + 25 * 12);
  uint32_t cur = T0;
  const uint32_t NC = nbc + N, ND = nbd + nd_total;
  // change row l of the merged document: base rows then the applied changes (appendChange,
  // new.js:1680-1692)
  {
    const uint32_t c = l >= nbc ? l - nbc : 0;
    const uint32_t cs = c & 63;
    const ChgHdrC& h = chh[cs < N ? cs : 0];
    const uint32_t n_adp = __shfl(a_dp, cs, 64), n_nd = __shfl(c_ndeps, cs, 64), n_nops = __shfl(c_nops, cs, 64);
    const bool isnew = l >= nbc && l < NC;
    int64_t v_act = bc_actor, v_seq = bc_seq, v_max = bc_max, v_time = bc_time, v_xlen = bc_xlen;
    uint32_t v_nd = bc_nd, m_off = 0, m_len = 0, x_off = bc_xoff, x_len = bc_xraw;
    bool m_null = bc_msg == AM_NULL64;
    if (!m_null) { m_off = (uint32_t)((uint64_t)bc_msg >> 32); m_len = (uint32_t)(bc_msg & 0xffffffff); }
    if (isnew) {
      v_act = n_adp;
      v_seq = h.seq;
      v_max = h.start_op + (int64_t)n_nops - 1;
      v_time = h.time;
      m_null = false;
      m_off = (uint32_t)(h.base + h.msg_off - a0);
      m_len = h.msg_len;
      bad |= !utf8_valid_dev(IN + m_off, m_len);  // k_doc replaces invalid sequences (U+FFFD)
      v_nd = n_nd;
      v_xlen = (int64_t)(((uint64_t)(h.has_extra ? h.extra_len : 0u) << 4) | 7);
      x_off = (uint32_t)(h.base + h.extra_off - a0);
      x_len = h.has_extra ? h.extra_len : 0u;
    }
    // message equality with the previous row (S column run detection)
    const uint32_t pm_off = wave::up1(m_off, 0u), pm_len = wave::up1(m_len, 0u);
    bool meq = !m_null && l > 0 && pm_len == m_len;
    for (uint32_t q = 0; meq && q < m_len; q++) meq = IN[pm_off + q] == IN[m_off + q];
    const int64_t dep_new = __shfl(dep_idx, (l - nbd) & 63, 64);
    const int64_t v_deps = l < nbd ? bc_dep : dep_new;
    // 31-bit values go through enc32; time keeps the 64-bit encoder
    const bool act = l < NC;
    bad |= act && (v_act < 0 || v_act > 0x7fffffff || v_seq < 0 || v_seq > 0x7fffffff || v_max < 0 || v_max > 0x7fffffff ||
                   (v_xlen != AM_NULL64 && (v_xlen < 0 || v_xlen > 0x7fffffff)));
    bad |= l < ND && (v_deps < 0 || v_deps > 0x7fffffff);
    // narrow integer columns (NC <= 16 change rows): one 16-lane row each, four columns per encoder
    // pass (enc32r), staged at the end of the image region and copied into place below
    constexpr uint32_t kRowCap = 176;  // 16 values x (1 + 5 + 5) bytes
    const bool t31 = __all(!act || v_time == AM_NULL64 || (v_time >= 0 && v_time <= 0x7fffffff));
    const bool seg = NC <= 16 && F.ob_cap >= cur + 8 * kRowCap + 64;
    const uint32_t tbase = F.ob_cap - 8 * kRowCap;
    // encoded lengths of the staged rows U {actor, depsNum, extraLen} (lu) and D {seq, maxOp, time}
    // (ld), at lanes 0 / 16 / 32 of each (read back by readlane: an indexed local array of them was
    // private memory, 40 B per lane of scratch traffic)
    uint32_t lu = 0, ld = 0;
    if (seg) {
      const uint32_t g = l >> 4, p = l & 15;
      const int32_t a = __shfl((int32_t)v_act, (int)p, 64), nd = __shfl((int32_t)v_nd, (int)p, 64);
      const int32_t xl = __shfl((int32_t)v_xlen, (int)p, 64);
      const bool xn = __shfl((int32_t)(v_xlen == AM_NULL64), (int)p, 64) != 0;
      lu = enc32r<EK_U>(g < 3 ? NC : 0u, g == 0 ? a : g == 1 ? nd : xl, g == 2 && xn, OB + tbase + g * kRowCap,
                                       kRowCap, bad);
      const int32_t sq = __shfl((int32_t)v_seq, (int)p, 64), mx = __shfl((int32_t)v_max, (int)p, 64);
      const int32_t tm = __shfl((int32_t)v_time, (int)p, 64);
      const bool tn = __shfl((int32_t)(v_time == AM_NULL64), (int)p, 64) != 0;
      ld = enc32r<EK_D>(g < (t31 ? 3u : 2u) ? NC : 0u, g == 0 ? sq : g == 1 ? mx : tm, g == 2 && tn,
                                       OB + tbase + (4 + g) * kRowCap, kRowCap, bad);
    }
    const uint32_t cap_end = seg ? tbase : F.ob_cap;
#pragma unroll 1
    for (int col = 0; col < DC_NCOLS; col++) {
      uint32_t len;
      const int srow = !seg ? -1 : col == DC_ACTOR ? 0 : col == DC_DEPS_NUM ? 1 : col == DC_EXTRA_LEN ? 2 : col == DC_SEQ ? 4
                                 : col == DC_MAXOP ? 5 : (col == DC_TIME && t31) ? 6 : -1;
      if (srow >= 0) {
        len = srow < 4 ? wave::bcast(lu, 16 * srow) : wave::bcast(ld, 16 * (srow - 4));
        if (len == ~0u || cur + len > cap_end) { bad = true; break; }
        const uint8_t* src = OB + tbase + srow * kRowCap;
        for (uint32_t q = l; q < len; q += 64) OB[cur + q] = src[q];
      } else if (col == DC_TIME) {
        len = enc_col(EK_D, NC, v_time, v_time == AM_NULL64, 0, 0, false, IN, OB + cur, cap_end - cur);
      } else {
        int32_t v = 0;
        bool nul = false;
        uint32_t so = 0, sl = 0, n = NC;
        switch (col) {
          case DC_ACTOR: v = (int32_t)v_act; break;
          case DC_SEQ: v = (int32_t)v_seq; break;
          case DC_MAXOP: v = (int32_t)v_max; break;
          case DC_MESSAGE: nul = m_null; so = m_off; sl = m_len; break;
          case DC_DEPS_NUM: v = (int32_t)v_nd; break;
          case DC_DEPS_INDEX: v = (int32_t)v_deps; n = ND; break;
          case DC_EXTRA_LEN: nul = v_xlen == AM_NULL64; v = (int32_t)v_xlen; break;
          default: so = x_off; sl = x_len; break;
        }
        len = enc32k(kEncKind[OC_NCOLS + col], n, v, nul, so, sl, meq, IN, OB + cur, cap_end - cur, bad);
      }
      if (len == ~0u) { bad = true; break; }
      if (l == 0) COLLEN[OC_NCOLS + col] = len;
      cur += len;
    }
    wsync();  // the staged rows are read before the op columns overwrite the region
  }
  FPH(11);
  FD_CHECK();
  {
    const uint32_t r = k_row;
    const bool out = l < NOUT;
    const int32_t objc = __shfl(r_objc, r, 64), obja = __shfl(r_obja, r, 64), keyc = __shfl(r_keyc, r, 64);
    const int32_t keya = __shfl(r_keya, r, 64), key = __shfl(r_key, r, 64), idc = __shfl(r_idc, r, 64);
    const int32_t ida = __shfl(r_ida, r, 64), ins = __shfl((int32_t)r_ins, r, 64), act = __shfl(r_act, r, 64);
    const int32_t vlen = __shfl(r_vlen, r, 64), chc = __shfl(r_chc, r, 64), cha = __shfl(r_cha, r, 64);
    const uint32_t voff = __shfl(r_voff, r, 64), vb = __shfl(r_vb, r, 64), kr = __shfl(r_krank, r, 64);
    const uint32_t pkr = wave::up1(kr, ~0u);
    const uint32_t succ_a = OUTA[l], succ_c = (uint32_t)OUTC[l];
#pragma unroll 1
    for (int col = 0; col < OC_NCOLS; col++) {
      int32_t v = 0;
      bool nul = false;
      uint32_t so = 0, sl = 0, n = NOUT;
      switch (col) {
        case OC_OBJ_ACTOR: v = obja; nul = obja < 0; break;
        case OC_OBJ_CTR: v = objc; nul = objc == FD_NULL; break;
        case OC_KEY_ACTOR: v = keya; nul = keya < 0; break;
        case OC_KEY_CTR: v = keyc; nul = keyc == FD_NULL; break;
        case OC_KEY_STR: nul = key == FD_NULL; so = (uint32_t)key >> 8; sl = (uint32_t)key & 255; break;
        case OC_ID_ACTOR: v = ida; break;
        case OC_ID_CTR: v = idc; break;
        case OC_INSERT: v = ins; break;
        case OC_ACTION: v = act; break;
        case OC_VAL_LEN: v = vlen; nul = vlen == FD_NULL; break;
        case OC_VAL_RAW: so = voff; sl = vb; break;
        case OC_CHLD_ACTOR: v = cha; nul = cha < 0; break;
        case OC_CHLD_CTR: v = chc; nul = chc == FD_NULL; break;
        case OC_GRP_NUM: v = (int32_t)sc_k; break;
        case OC_GRP_ACTOR: v = (int32_t)succ_a; n = NSUCC; break;
        default: v = (int32_t)succ_c; n = NSUCC; break;
      }
      const bool eqs = col == OC_KEY_STR && key != FD_NULL && pkr == kr;
      const uint32_t len = enc32k(kEncKind[col], n, v, nul && out, so, sl, eqs, IN, OB + cur, F.ob_cap - cur, bad);
      if (len == ~0u) { bad = true; break; }
      if (l == 0) COLLEN[col] = len;
      cur += len;
    }
  }
  wsync();
  FD_CHECK();
  FPH(12);
  // trailer: heads indexes (all known here) and the base document's extra bytes
  const uint32_t cols_end = cur;
  const uint32_t xlen = has_base ? uni((uint32_t)dh->extra_len) : 0u;
  uint32_t hib = 0;
  {
    const int32_t* HIDX = reinterpret_cast<const int32_t*>(M + FM_HIDX);
    const uint32_t hb = l < NH ? (uint32_t)uleb_len((uint64_t)HIDX[l]) : 0u;
    const uint32_t ho = excl_add(hb, hib);
    if (cols_end + hib + xlen > F.ob_cap) bad = true;
    else {
      if (l < NH) put_uleb(OB + cols_end + ho, (uint64_t)HIDX[l]);
      for (uint32_t q = l; q < xlen; q += 64) OB[cols_end + hib + q] = IN[dhb + dh->extra_off - a0 + q];
    }
  }
  FD_CHECK();
  // header, written to end exactly at T0 (encodeDocumentHeader, columnar.js:983-1004). Column
  // table entries: lane e < 25 holds entry e (the 9 change columns, then the 16 op columns)
  const bool t_chg = l < DC_NCOLS, t_any = l < DC_NCOLS + OC_NCOLS;
  const uint32_t e_len = t_any ? COLLEN[t_chg ? OC_NCOLS + l : l - DC_NCOLS] : 0u;
  const uint32_t e_id = t_any ? (t_chg ? kDocChgColIds[l] : kDocOpColIds[l - DC_NCOLS]) : 0u;
  const uint32_t e_bytes = e_len ? uleb_len32(e_id) + uleb_len32(e_len) : 0u;
  uint32_t ctab, coltot;
  const uint32_t e_pos = excl_add(e_bytes, ctab);
  excl_add(e_len, coltot);
  const uint32_t nce = (uint32_t)__popcll(__ballot(t_chg && e_len)), noe = (uint32_t)__popcll(__ballot(!t_chg && e_len));
  const uint32_t pre_cols = uleb_len(NA) + alen_sum + uleb_len(NH) + 32 * NH + uleb_len(nce) + uleb_len(noe) + ctab;
  const uint64_t body = (uint64_t)pre_cols + coltot + hib + xlen;
  const uint32_t hs = 9 + uleb_len(body) + pre_cols;
  if (hs > T0) return;  // cannot happen (T0 bounds it); stay safe
  const uint32_t start = T0 - hs;
  {
    const uint32_t act0 = start + 9 + uleb_len(body) + uleb_len(NA);  // first actor record
    const uint32_t heads0 = act0 + alen_sum;
    if (l < NA) {
      uint8_t* o = put_uleb(OB + act0 + a_pos, a_len);
      const uint32_t src = RO[2 * M[FM_DP2REF + l]];
      for (uint32_t q = 0; q < a_len; q++) o[q] = IN[src + q];
    }
    const uint32_t hbytes0 = heads0 + uleb_len(NH);
    // head bytes from their sources (the hash table in the cells region is gone): a change of this
    // call (k_chunks' hash) or a base head (the base document's heads)
    for (uint32_t q = l; q < 32 * NH; q += 64) {
      const uint32_t t = M[FM_HSEL + (q >> 5)];
      OB[hbytes0 + q] = t < N ? info[dd.chg_begin + t].hash[q & 31] : IN[dhb + dh->heads_off + 32 * (t - N) + (q & 31) - a0];
    }
    if (l == 0) {
      uint8_t* o = OB + start;
      for (int k = 0; k < 4; k++) *o++ = kMagic[k];
      for (int k = 0; k < 4; k++) *o++ = 0;  // checksum: k_out_hash_ws
      *o++ = 0;                               // CHUNK_TYPE_DOCUMENT
      o = put_uleb(o, body);
      put_uleb(o, NA);
      o = put_uleb(OB + heads0, NH);
      o += 32 * NH;
      put_uleb(o, nce);
    }
    // [nce] change-column entries [noe] op-column entries
    const uint32_t tab0 = hbytes0 + 32 * NH + uleb_len(nce);
    if (e_len) {
      uint8_t* o = OB + tab0 + e_pos + (t_chg ? 0u : uleb_len(noe));
      o = put_uleb32(o, e_id);
      put_uleb32(o, e_len);
    }
    if (l == DC_NCOLS) put_uleb32(OB + tab0 + e_pos, noe);  // e_pos of the first op entry = end of the change entries
  }
  wsync();
  // copy the image [start, cols_end + hib + xlen) to the document's output slot, one dword per lane
  const uint32_t olen = cols_end + hib + xlen - start;
  if (olen > L.out_cap) return;
  {
    uint32_t* dst = reinterpret_cast<uint32_t*>(wsg + L.out);
    const uint8_t* src = OB + start;
    for (uint32_t q = 4 * l; q < olen; q += 256) {
      uint32_t w = 0;
#pragma unroll
      for (int k = 0; k < 4; k++) w |= (uint32_t)(q + k < olen ? src[q + k] : 0) << (8 * k);
      dst[q >> 2] = w;
    }
  }
  FPH(13);
  if (!kDiff && b.P) return;  // launched without the patch writers: k_doc writes the log
  if (kDiff && b.P == 2) {
    // AM_DOC_META: the handle's objectMeta blob (an AM_CHUNK_RAW chunk), or documentPatch's
    const bool meta = (dd.flags & AM_DOC_META) != 0;
    const uint8_t* mblob = nullptr;
    uint32_t mlen = 0;
    if (meta && dd.meta_chunk) {
      const am_chunk_desc mc = chunks[dd.meta_chunk - 1];
      mblob = arena + mc.off;
      mlen = mc.len;
    }
    if (!fast_diff(IN, S + F.cells, F.ob_cap, wsg + L.pwire, L.pwire_cap, M, R, nb, NOUT, NA, NC, nbc, N, OUTC, OUTA, RO, chh,
                   meta, mblob, mlen))
      return;  // outside the shapes fast_diff covers: k_doc replays the patch (am_diff.h)
  }
  if (kDiff && b.P == 1 && !fast_getpatch(IN, S + F.cells, F.ob_cap, wsg + L.pwire, L.pwire_cap, M, NOUT, NSUCC, NA, NC, nbc,
                                          N, OUTC, OUTA, RO, chh))
    return;  // outside the shapes fast_getpatch covers: k_doc writes the log (P7, am_patch.h)
  FPH(14);
  if (l < N) chg_state[dd.chg_begin + l] = (int32_t)l;
  if (l == 0) {
    am_doc_result r;
    r.status = AM_OK;
    r.err_change = 0xffffffffu;
    r.arg0 = r.arg1 = 0;
    r.arg_actor_off = 0;
    r.arg_actor_len = 0;
    r.napplied = N;
    r.nqueued = 0;
    r.nheads = NH;
    r.nops = NOUT;
    r.nchanges = NC;
    r.max_op = maxop;
    r.out_off = 0;
    r.out_len = olen;
    r.ws_off = wso;
    r.ws_bytes = L.total;
    results[doc] = r;
    fast_done[doc] = 1;
  }
#undef FD_CHECK
}
#undef FPH
