// am_kernels.hip -- MI355X (gfx950) kernels of the batched Automerge merge engine.
//
// Pipeline for a batch of independent documents (each = optional base document + the change
// list of one Backend.applyChanges call):
//   k_chunks   thread per chunk: SHA-256 (checksum + change hash), container and header parse,
//              per-chunk row/entry/string counts              columnar.js:635-765, 1006-1038
//   k_bounds   thread per document: workspace bounds          (sizing only)
//   k_scan*    exclusive scans (workspace offsets)
//   k_doc      one workgroup (one wave) per document, working set in LDS: causal queue + actor
//              table (new.js:1550-1597, 1434-1451), column decode into rows (encoding.js:789-1207),
//              merge as a data-parallel sort (object order, UTF-16 key order, RGA preorder via
//              Euler-tour list ranking, opId order; new.js:50-317, 1052-1290), succ lists,
//              canonical re-encode of every column and the document header (new.js:2025-2047,
//              columnar.js:983-1004)
//   k_out_hash_ws thread per document: container checksum of the merged document (columnar.js:659)
#include <hip/hip_runtime.h>
#include <atomic>
#include <cstdlib>
#include <cstring>

#include "am_dev_util.h"
#include "am_layout.h"
#include "am_wave.h"

// column ids in spec order
__device__ __constant__ static const uint8_t kChangeColIds[OC_NCOLS] = {0x01, 0x02, 0x11, 0x13, 0x15, 0x21, 0x23, 0x34,
                                                                      0x42, 0x56, 0x57, 0x61, 0x63, 0x70, 0x71, 0x73};
__device__ __constant__ static const uint8_t kDocOpColIds[OC_NCOLS] = {0x01, 0x02, 0x11, 0x13, 0x15, 0x21, 0x23, 0x34,
                                                                     0x42, 0x56, 0x57, 0x61, 0x63, 0x80, 0x81, 0x83};
__device__ __constant__ static const uint8_t kDocChgColIds[DC_NCOLS] = {0x01, 0x03, 0x13, 0x23, 0x35, 0x40, 0x43, 0x56, 0x57};

__device__ __constant__ static const uint8_t kMagic[4] = {0x85, 0x6f, 0x4a, 0x83};

// ------------------------------------------------------------------------------------------
// Header parsing (shared by k_chunks and k_doc). Offsets are relative to `base`, the arena
// offset of the chunk data, so headers stay compact (they live in LDS inside k_doc).
// ------------------------------------------------------------------------------------------
struct ChgHdr {              // decodeChangeHeader + column info (columnar.js:635-652, 741-765)
  uint64_t base;
  int64_t seq, start_op, time;
  uint32_t actor_off, actors_off, deps_off, msg_off, extra_off;
  uint32_t actor_len, nactors, ndeps, msg_len, extra_len, has_extra;
  uint32_t nunk;             // op columns outside CHANGE_COLUMNS
  uint32_t col_off[OC_NCOLS];
  uint32_t col_len[OC_NCOLS];
};
// compact forms (u16 offsets/lengths, chunk data < 64 KiB) kept per chunk in HdrSlot
struct alignas(16) ChgHdrC {
  uint64_t base;
  int64_t seq, start_op, time;
  uint16_t actor_off, actors_off, deps_off, msg_off, extra_off;
  uint16_t actor_len, nactors, ndeps, msg_len, extra_len, has_extra, pad;
  uint16_t col_off[OC_NCOLS];
  uint16_t col_len[OC_NCOLS];
};
struct alignas(16) DocHdrC {
  uint64_t base;
  uint16_t actors_off, heads_off, hidx_off, extra_off;
  uint16_t nactors, nheads, has_hidx, extra_len;
  uint16_t ccol_off[DC_NCOLS];
  uint16_t ccol_len[DC_NCOLS];
  uint16_t ocol_off[OC_NCOLS];
  uint16_t ocol_len[OC_NCOLS];
};
static_assert(sizeof(ChgHdrC) <= sizeof(HdrSlot) && sizeof(DocHdrC) <= sizeof(HdrSlot), "HdrSlot");
struct DocHdr {              // decodeDocumentHeader (columnar.js:1006-1038)
  uint64_t base;
  uint32_t actors_off, heads_off, hidx_off, extra_off;
  uint32_t nactors, nheads, has_hidx, extra_len;
  uint32_t nunk;             // op columns outside DOC_OPS_COLUMNS
  uint32_t ccol_off[DC_NCOLS];
  uint32_t ccol_len[DC_NCOLS];
  uint32_t ocol_off[OC_NCOLS];
  uint32_t ocol_len[OC_NCOLS];
};

// Column table (decodeColumnInfo, columnar.js:609) -> spec slots; the data follows in table
// order, i.e. ascending id order, so a second pass assigns offsets in spec order.
// NSPEC is a compile-time constant so the slot writes are predicated register moves rather than
// a dynamically indexed (scratch) array
// Column table (decodeColumnInfo, columnar.js:609) -> spec slots. The data follows in table
// order (ascending id), so each spec column's offset relative to the data start is the running
// sum of the lengths before it (`off`, made absolute by place_cols). Columns outside the spec (a
// future version's columns, new.js:1387-1425) are allowed among the op columns (`allow_unknown`):
// counted in `nunk`, their bytes skipped. Unknown ids in the pred / succ groups (7, 8) would change
// the group structure of the known columns and stay unsupported.
template <int NSPEC>
__device__ __forceinline__ uint32_t parse_cols(Rd& r, const uint8_t* spec, uint32_t* len, uint32_t* off, bool is_change,
                                               bool allow_unknown, uint64_t& total, uint32_t& nunk) {
  int64_t num;
  TRY(rd_u53(r, num));
  int64_t last = -1;
  uint64_t acc = 0;
  nunk = 0;
#pragma unroll
  for (int i = 0; i < NSPEC; i++) { len[i] = 0; off[i] = 0; }
  for (int64_t i = 0; i < num; i++) {
    int64_t id, l;
    TRY(rd_u53(r, id));
    TRY(rd_u53(r, l));
    if ((id & ~(int64_t)COL_DEFLATE) <= (last & ~(int64_t)COL_DEFLATE)) return AM_E_COL_ORDER;
    last = id;
    if (is_change && (id & COL_DEFLATE)) return AM_E_CHANGE_DEFLATED_COL;
    if (id & COL_DEFLATE) return AM_U_VALUE;  // the host stage inflates document columns
    if (l > 0x7fffffff) return AM_E_SUBARRAY;
    bool found = false;
#pragma unroll
    for (int j = 0; j < NSPEC; j++)
      if (spec[j] == id) { len[j] = (uint32_t)l; off[j] = (uint32_t)acc; found = true; }
    if (!found) {
      if (!allow_unknown || (id >> 4) == 7 || (id >> 4) == 8 || id > 0xffff) return AM_U_UNKNOWN_COLUMN;
      nunk++;
    }
    acc += (uint64_t)l;
  }
  total = acc;
  return AM_OK;
}
template <int NSPEC>
__device__ __forceinline__ uint32_t place_cols(Rd& r, uint32_t* off, uint64_t total) {
  const uint64_t at0 = r.off;
#pragma unroll
  for (int k = 0; k < NSPEC; k++) off[k] += (uint32_t)at0;
  uint64_t at;
  TRY(rd_raw(r, total, at));
  return AM_OK;
}
// Visits the unknown op columns of a change or document chunk body: f(id, offset in data, length).
template <typename F>
__device__ uint32_t visit_unknown_cols(const uint8_t* data, uint64_t n, bool is_doc, F f) {
  Rd r{data, n, 0};
  int64_t v, l;
  uint64_t at;
  if (!is_doc) {
    TRY(rd_u53(r, v)); TRY(rd_raw(r, (uint64_t)v * 32, at));
    TRY(rd_u53(r, v)); TRY(rd_raw(r, (uint64_t)v, at));
    TRY(rd_u53(r, v)); TRY(rd_u53(r, v)); TRY(rd_i53(r, v));
    TRY(rd_u53(r, v)); TRY(rd_raw(r, (uint64_t)v, at));
    TRY(rd_u53(r, v));
    for (int64_t i = 0; i < v; i++) { TRY(rd_u53(r, l)); TRY(rd_raw(r, (uint64_t)l, at)); }
  } else {
    TRY(rd_u53(r, v));
    for (int64_t i = 0; i < v; i++) { TRY(rd_u53(r, l)); TRY(rd_raw(r, (uint64_t)l, at)); }
    TRY(rd_u53(r, v)); TRY(rd_raw(r, (uint64_t)v * 32, at));
  }
  // (document: the change-column table comes first; its data precedes the op columns' data)
  uint64_t skip = 0;
  if (is_doc) {
    TRY(rd_u53(r, v));
    for (int64_t i = 0; i < v; i++) { int64_t id; TRY(rd_u53(r, id)); TRY(rd_u53(r, l)); skip += (uint64_t)l; }
  }
  int64_t num;
  TRY(rd_u53(r, num));
  const uint64_t tab = r.off;
  for (int64_t i = 0; i < num; i++) { int64_t id; TRY(rd_u53(r, id)); TRY(rd_u53(r, l)); }
  uint64_t pos = r.off + skip;
  r.off = tab;
  const uint8_t* spec = is_doc ? kDocOpColIds : kChangeColIds;
  for (int64_t i = 0; i < num; i++) {
    int64_t id;
    TRY(rd_u53(r, id)); TRY(rd_u53(r, l));
    bool known = false;
    for (int j = 0; j < OC_NCOLS; j++) known |= spec[j] == id;
    if (!known) f((uint32_t)id, pos, (uint32_t)l);
    pos += (uint64_t)l;
  }
  return AM_OK;
}

__device__ __forceinline__ uint32_t parse_change_hdr(const uint8_t* data, uint64_t n, uint64_t abs, ChgHdr& h) {
  Rd r{data, n, 0};
  int64_t v;
  uint64_t at;
  h.base = abs;
  TRY(rd_u53(r, v));
  h.ndeps = (uint32_t)v;
  TRY(rd_raw(r, (uint64_t)v * 32, at));
  h.deps_off = (uint32_t)at;
  TRY(rd_u53(r, v));
  TRY(rd_raw(r, (uint64_t)v, at));
  h.actor_off = (uint32_t)at;
  h.actor_len = (uint32_t)v;
  TRY(rd_u53(r, h.seq));
  TRY(rd_u53(r, h.start_op));
  TRY(rd_i53(r, h.time));
  TRY(rd_u53(r, v));
  TRY(rd_raw(r, (uint64_t)v, at));
  h.msg_off = (uint32_t)at;
  h.msg_len = (uint32_t)v;
  TRY(rd_u53(r, v));
  h.nactors = (uint32_t)v + 1;
  h.actors_off = (uint32_t)r.off;
  for (int64_t i = 0; i < v; i++) {
    int64_t l;
    TRY(rd_u53(r, l));
    TRY(rd_raw(r, (uint64_t)l, at));
  }
  uint64_t total;
  uint32_t nunk;
  TRY(parse_cols<OC_NCOLS>(r, kChangeColIds, h.col_len, h.col_off, true, true, total, nunk));
  TRY(place_cols<OC_NCOLS>(r, h.col_off, total));
  h.nunk = nunk;
  h.has_extra = r.off < r.n;
  h.extra_off = (uint32_t)r.off;
  h.extra_len = (uint32_t)(r.n - r.off);
  return AM_OK;
}

__device__ __forceinline__ uint32_t parse_doc_hdr(const uint8_t* data, uint64_t n, uint64_t abs, DocHdr& h) {
  Rd r{data, n, 0};
  int64_t v;
  uint64_t at;
  h.base = abs;
  TRY(rd_u53(r, v));
  h.nactors = (uint32_t)v;
  h.actors_off = (uint32_t)r.off;
  for (int64_t i = 0; i < v; i++) {
    int64_t l;
    TRY(rd_u53(r, l));
    TRY(rd_raw(r, (uint64_t)l, at));
  }
  TRY(rd_u53(r, v));
  h.nheads = (uint32_t)v;
  TRY(rd_raw(r, (uint64_t)v * 32, at));
  h.heads_off = (uint32_t)at;
  uint64_t ctot, otot;
  uint32_t cunk, nunk;
  TRY(parse_cols<DC_NCOLS>(r, kDocChgColIds, h.ccol_len, h.ccol_off, false, false, ctot, cunk));
  TRY(parse_cols<OC_NCOLS>(r, kDocOpColIds, h.ocol_len, h.ocol_off, false, true, otot, nunk));
  TRY(place_cols<DC_NCOLS>(r, h.ccol_off, ctot));
  TRY(place_cols<OC_NCOLS>(r, h.ocol_off, otot));
  h.nunk = nunk;
  h.has_hidx = r.off < r.n;
  h.hidx_off = (uint32_t)r.off;
  if (h.has_hidx) {
    for (uint32_t i = 0; i < h.nheads; i++) TRY(rd_u53(r, v));
  }
  h.extra_off = (uint32_t)r.off;
  h.extra_len = (uint32_t)(r.n - r.off);
  return AM_OK;
}

// unknown op columns: count and a bound on their values (every column holds a value per row, or,
// in an unknown column group, one per entry of that group: at most the sum of its cardinalities)
// (noinline, results by value: the caller's ChunkInfo stays in registers -- no scratch)
__device__ __noinline__ static uint64_t unknown_bound(const uint8_t* data, uint64_t n, bool is_doc, uint32_t nunk, uint32_t nrows) {
  uint64_t cards = 0;
  uint32_t st = AM_OK;
  uint32_t e = visit_unknown_cols(data, n, is_doc, [&](uint32_t id, uint64_t off, uint32_t l) {
    if ((id & 7) != 0 || st) return;
    uint64_t cnt, sum;
    st = rle_count_sum_i(data + off, l, false, cnt, sum, 0);
    cards += sum;
  });
  if (e) return (uint64_t)e << 32;
  if (st) return (uint64_t)st << 32;
  const uint64_t b = (uint64_t)(nunk + 1) * ((uint64_t)nrows + cards) + 2ull * nrows;
  if (b > 0x3fffffffull) return (uint64_t)AM_U_CAPACITY << 32;
  return b;
}

// ------------------------------------------------------------------------------------------
// k_chunks: one thread per chunk
// ------------------------------------------------------------------------------------------
// Per chunk: container header, SHA-256 (hash + checksum), change/document header parse into the
// compact slot, row/entry/string counts. `p` is the chunk start: a staged LDS copy or the arena.
__device__ __forceinline__ void chunk_body(const uint8_t* p, const am_chunk_desc cd, uint32_t i, ChunkInfo* __restrict__ info,
                                           HdrSlot* __restrict__ hdr, bool defer_counts, uint32_t* dcols) {
  ChunkInfo ci;
  uint32_t* hw = reinterpret_cast<uint32_t*>(ci.hash);
#pragma unroll
  for (int k = 0; k < 8; k++) hw[k] = 0;
  ci.status = AM_OK; ci.type = 0xff; ci.data_off = 0; ci.data_len = 0; ci.nops = 0; ci.nents = 0; ci.nchg = 0;
  ci.ndeps = 0; ci.nactors = 0; ci.strbytes = 0; ci.nheads = 0; ci.arg0 = 0; ci.nunk = 0;
  uint32_t st = AM_OK;
  do {
    if (cd.flags & AM_CHUNK_BADZ) { st = AM_E_INFLATE; break; }  // the batch stage could not inflate a column
    // decodeContainerHeader (columnar.js:688)
    if (cd.len < 4) { st = AM_E_SUBARRAY; break; }
    if (p[0] != kMagic[0] || p[1] != kMagic[1] || p[2] != kMagic[2] || p[3] != kMagic[3]) { st = AM_E_MAGIC; break; }
    if (cd.len < 9) { st = AM_E_SUBARRAY; break; }
    Rd r{p, cd.len, 8};
    ci.type = p[8];
    r.off = 9;
    int64_t len;
    if ((st = rd_u53(r, len))) break;
    uint64_t at;
    if ((st = rd_raw(r, (uint64_t)len, at))) break;
    ci.data_off = (uint32_t)at;
    ci.data_len = (uint32_t)len;
    // SHA-256: a change's hash, or a document's checksum -- unless the host stage has verified the
    // document already (its columns were inflated, am_stage_document): a document has no hash of
    // its own, so a verified one skips the single-lane pass over all its bytes
    if (!(ci.type == 0 && (cd.flags & 1))) {
      uint32_t h[8];
      sha256_words(p + 8, r.off - 8, h);
#pragma unroll
      for (int k = 0; k < 8; k++) hw[k] = __builtin_bswap32(h[k]);
      if (!(cd.flags & 1) && ((uint32_t)p[4] << 24 | (uint32_t)p[5] << 16 | (uint32_t)p[6] << 8 | p[7]) != h[0]) {
        st = AM_E_CHECKSUM;
        break;
      }
    }
    const uint8_t* data = p + at;
    if (ci.type == 1) {
      if (r.off != cd.len) { st = AM_E_CHANGE_TRAILING; break; }
      ChgHdr hh;
      if ((st = parse_change_hdr(data, len, cd.off + at, hh))) break;
      if (len < 65536) {
        ChgHdrC c;
        c.base = hh.base; c.seq = hh.seq; c.start_op = hh.start_op; c.time = hh.time;
        c.actor_off = hh.actor_off; c.actors_off = hh.actors_off; c.deps_off = hh.deps_off; c.msg_off = hh.msg_off;
        c.extra_off = hh.extra_off; c.actor_len = hh.actor_len; c.nactors = hh.nactors; c.ndeps = hh.ndeps;
        c.msg_len = hh.msg_len; c.extra_len = hh.extra_len; c.has_extra = hh.has_extra; c.pad = 0;
#pragma unroll
        for (int k = 0; k < OC_NCOLS; k++) { c.col_off[k] = hh.col_off[k]; c.col_len[k] = hh.col_len[k]; }
        *reinterpret_cast<ChgHdrC*>(hdr + i) = c;
      }
      ci.ndeps = hh.ndeps;
      ci.nactors = hh.nactors;
      uint64_t cnt, sum;
      // rows: values in the action column (new.js:701)
      if ((st = rle_count_sum_i(data + hh.col_off[OC_ACTION], hh.col_len[OC_ACTION], false, cnt, sum, 0))) break;
      ci.nops = (uint32_t)cnt;
      if ((st = rle_count_sum_i(data + hh.col_off[OC_GRP_NUM], hh.col_len[OC_GRP_NUM], false, cnt, sum, 0))) break;
      ci.nents = (uint32_t)sum;
      // key string bytes summed over rows (bounds the re-encoded keyStr column)
      uint64_t scnt, ssum;
      if ((st = rle_count_sum_i(data + hh.col_off[OC_KEY_STR], hh.col_len[OC_KEY_STR], true, scnt, ssum, 0))) break;
      ci.strbytes = (uint32_t)ssum + hh.msg_len;
      ci.nunk = hh.nunk;  // their value bound: k_bounds (unknown_bound)
    } else if (ci.type == 0) {
      if (r.off != cd.len) { st = AM_E_DOC_TRAILING; break; }
      DocHdr dh;
      if ((st = parse_doc_hdr(data, len, cd.off + at, dh))) break;
      if (len < 65536) {
        DocHdrC c;
        c.base = dh.base; c.actors_off = dh.actors_off; c.heads_off = dh.heads_off; c.hidx_off = dh.hidx_off;
        c.extra_off = dh.extra_off; c.nactors = dh.nactors; c.nheads = dh.nheads; c.has_hidx = dh.has_hidx;
        c.extra_len = dh.extra_len;
#pragma unroll
        for (int k = 0; k < DC_NCOLS; k++) { c.ccol_off[k] = dh.ccol_off[k]; c.ccol_len[k] = dh.ccol_len[k]; }
#pragma unroll
        for (int k = 0; k < OC_NCOLS; k++) { c.ocol_off[k] = dh.ocol_off[k]; c.ocol_len[k] = dh.ocol_len[k]; }
        *reinterpret_cast<DocHdrC*>(hdr + i) = c;
      }
      ci.nactors = dh.nactors;
      ci.nheads = dh.nheads;
      ci.nunk = dh.nunk;
      if (defer_counts) {  // a large document: the wave counts its columns together (k_chunks)
        const uint8_t kc[6] = {(uint8_t)DC_ACTOR, (uint8_t)DC_DEPS_NUM, (uint8_t)(OC_NCOLS + OC_ID_CTR), (uint8_t)(OC_NCOLS + OC_GRP_NUM),
                               (uint8_t)(OC_NCOLS + OC_KEY_STR), (uint8_t)DC_MESSAGE};
#pragma unroll
        for (int k = 0; k < 6; k++) {
          const uint32_t c = kc[k];
          dcols[2 * k] = (uint32_t)at + (c < OC_NCOLS ? dh.ccol_off[c] : dh.ocol_off[c - OC_NCOLS]);
          dcols[2 * k + 1] = c < OC_NCOLS ? dh.ccol_len[c] : dh.ocol_len[c - OC_NCOLS];
        }
        break;
      }
      uint64_t cnt, sum;
      if ((st = rle_count_sum_i(data + dh.ccol_off[DC_ACTOR], dh.ccol_len[DC_ACTOR], false, cnt, sum, 0))) break;
      ci.nchg = (uint32_t)cnt;
      if ((st = rle_count_sum_i(data + dh.ccol_off[DC_DEPS_NUM], dh.ccol_len[DC_DEPS_NUM], false, cnt, sum, 0))) break;
      ci.ndeps = (uint32_t)sum;
      // doc rows: values in the idCtr column (updateBlockMetadata, new.js:386)
      if ((st = rle_count_sum_i(data + dh.ocol_off[OC_ID_CTR], dh.ocol_len[OC_ID_CTR], false, cnt, sum, 0, true))) break;
      ci.nops = (uint32_t)cnt;
      if ((st = rle_count_sum_i(data + dh.ocol_off[OC_GRP_NUM], dh.ocol_len[OC_GRP_NUM], false, cnt, sum, 0))) break;
      ci.nents = (uint32_t)sum;
      uint64_t s1, s2;
      if ((st = rle_count_sum_i(data + dh.ocol_off[OC_KEY_STR], dh.ocol_len[OC_KEY_STR], true, cnt, s1, 0))) break;
      if ((st = rle_count_sum_i(data + dh.ccol_off[DC_MESSAGE], dh.ccol_len[DC_MESSAGE], true, cnt, s2, 0))) break;
      ci.strbytes = (uint32_t)(s1 + s2);
      ci.nunk = dh.nunk;
    } else {
      st = AM_E_CHUNK_TYPE;
      ci.arg0 = ci.type;
    }
  } while (0);
  ci.status = st;
  info[i] = ci;
}

#define KC_STAGE 12288  // bytes of LDS per wave for its 64 chunks
#define KC_BIG 16384     // a document chunk this large has its columns counted by the whole wave

// ---- counting of a large document's columns (k_chunks): the column parse of rle_count_sum with
// the LEB readers of leb_u64 / leb_i64 / rd_u53 / rd_i53 (same results and status codes) over a
// byte reader, one lane per column. ----
// One lane's reader over global memory with a 16-byte line in registers (arena-aligned loads: the
// arena is 16-aligned and carries >= 16 bytes of slack past its last chunk): each lane counts a
// column of its own, so a large document's columns are counted side by side
struct LineRd {
  const uint8_t* arena;
  uint64_t goff;  // chunk start (arena offset)
  uint64_t line;  // arena offset of the line held; ~0: none
  uint4 buf;
};
__device__ __forceinline__ uint8_t rd_byte(LineRd& r, uint64_t k) {
  const uint64_t a = r.goff + k, la = a & ~15ull;
  if (la != r.line) {
    r.buf = *reinterpret_cast<const uint4*>(r.arena + la);
    r.line = la;
  }
  const uint32_t q = (uint32_t)(a & 15);
  const uint32_t w = q < 8 ? (q < 4 ? r.buf.x : r.buf.y) : (q < 12 ? r.buf.z : r.buf.w);
  return (uint8_t)(w >> (8 * (q & 3)));
}
struct WinCur { uint64_t off, n; };  // a column: [off, off + n) of the chunk
template <class Rd_>
__device__ static uint32_t win_leb_u64(Rd_& w, WinCur& d, uint32_t& hi, uint32_t& lo) {
  uint32_t low = 0, high = 0;
  int shift = 0;
  while (d.off < d.n && shift <= 28) {
    const uint8_t b = rd_byte(w, d.off);
    low |= (uint32_t)(b & 0x7f) << shift;
    if (shift == 28) high = (b & 0x70) >> 4;
    shift += 7;
    d.off++;
    if (!(b & 0x80)) { hi = high; lo = low; return AM_OK; }
  }
  shift = 3;
  while (d.off < d.n) {
    const uint8_t b = rd_byte(w, d.off);
    if (shift == 31 && (b & 0xfe) != 0) return AM_E_LEB_RANGE;
    high |= (uint32_t)(b & 0x7f) << shift;
    shift += 7;
    d.off++;
    if (!(b & 0x80)) { hi = high; lo = low; return AM_OK; }
  }
  return AM_E_LEB_INCOMPLETE;
}
template <class Rd_>
__device__ static uint32_t win_leb_i64(Rd_& w, WinCur& d, int32_t& hi, uint32_t& lo) {
  uint32_t low = 0;
  int32_t high = 0;
  int shift = 0;
  while (d.off < d.n && shift <= 28) {
    const uint8_t b = rd_byte(w, d.off);
    low |= (uint32_t)(b & 0x7f) << shift;
    if (shift == 28) high = (b & 0x70) >> 4;
    shift += 7;
    d.off++;
    if (!(b & 0x80)) {
      if (b & 0x40) {
        if (shift < 32) low |= 0xffffffffu << shift;
        const int s2 = shift - 32 > 0 ? shift - 32 : 0;
        high |= (int32_t)(0xffffffffu << s2);
      }
      hi = high; lo = low;
      return AM_OK;
    }
  }
  shift = 3;
  while (d.off < d.n) {
    const uint8_t b = rd_byte(w, d.off);
    if (shift == 31 && b != 0 && b != 0x7f) return AM_E_LEB_RANGE;
    high |= (int32_t)((uint32_t)(b & 0x7f) << shift);
    shift += 7;
    d.off++;
    if (!(b & 0x80)) {
      if ((b & 0x40) && shift < 32) high |= (int32_t)(0xffffffffu << shift);
      hi = high; lo = low;
      return AM_OK;
    }
  }
  return AM_E_LEB_INCOMPLETE;
}
template <class Rd_>
__device__ __forceinline__ uint32_t win_u53(Rd_& w, WinCur& d, int64_t& v) {
  uint32_t hi, lo;
  TRY(win_leb_u64(w, d, hi, lo));
  if (hi > 0x1fffff) return AM_E_LEB_RANGE;
  v = (int64_t)hi * 4294967296LL + lo;
  return AM_OK;
}
template <class Rd_>
__device__ __forceinline__ uint32_t win_i53(Rd_& w, WinCur& d, int64_t& v) {
  int32_t hi;
  uint32_t lo;
  TRY(win_leb_i64(w, d, hi, lo));
  if (hi < -0x200000 || (hi == -0x200000 && lo == 0) || hi > 0x1fffff) return AM_E_LEB_RANGE;
  v = (int64_t)hi * 4294967296LL + lo;
  return AM_OK;
}
// rle_count_sum over the window (same record rules, same errors)
template <class Rd_>
__device__ __forceinline__ uint32_t win_count_sum(Rd_& w, uint64_t off, uint64_t n, bool is_str, bool is_signed, uint64_t& count, uint64_t& sum) {
  WinCur d{off, off + n};
  count = 0;
  sum = 0;
  while (d.off < d.n) {
    int64_t c;
    TRY(win_i53(w, d, c));
    if (c > 0) {
      int64_t v;
      if (is_str) {
        TRY(win_u53(w, d, v));
        if (d.off + (uint64_t)v > d.n) return AM_E_SUBARRAY;
        d.off += (uint64_t)v;
      } else if (is_signed) {
        TRY(win_i53(w, d, v));
        v = 0;
      } else {
        TRY(win_u53(w, d, v));
      }
      count += (uint64_t)c;
      sum += (uint64_t)c * (uint64_t)v;
    } else if (c < 0) {
      for (int64_t i = 0; i < -c; i++) {
        int64_t v;
        if (is_signed) { TRY(win_i53(w, d, v)); v = 0; } else { TRY(win_u53(w, d, v)); }
        if (is_str) {
          if (d.off + (uint64_t)v > d.n) return AM_E_SUBARRAY;
          d.off += (uint64_t)v;
        }
        sum += (uint64_t)v;
      }
      count += (uint64_t)(-c);
    } else {
      int64_t z;
      TRY(win_u53(w, d, z));
      count += (uint64_t)z;
    }
  }
  return AM_OK;
}
// k_chunks: thread per chunk. Each wave first stages the byte span of its 64 chunks (adjacent in
// the arena for staged batches) into LDS with 16-byte loads, so the SHA-256 rounds and the
// dependent LEB128 reads of the header parse hit LDS; a wave whose span does not fit reads the
// arena directly.
__global__ void __launch_bounds__(256) k_chunks(const uint8_t* __restrict__ arena, const am_chunk_desc* __restrict__ chunks,
                                                uint32_t nchunks, ChunkInfo* __restrict__ info,
                                                HdrSlot* __restrict__ hdr) {
  __shared__ __attribute__((aligned(16))) uint8_t stage[4][KC_STAGE + 16];
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t w = threadIdx.x >> 6, l = threadIdx.x & 63;
  bool valid = i < nchunks;
  am_chunk_desc cd;
  cd.off = 0; cd.len = 0; cd.flags = 0;
  if (valid) cd = chunks[i];
  // an objectMeta blob (AM_CHUNK_RAW) is not a container: no documents' chunk, nothing to parse
  if (valid && (cd.flags & AM_CHUNK_RAW)) {
    ChunkInfo& ci = info[i];
    ci.status = AM_OK; ci.type = 0xff; ci.nops = ci.nents = ci.nchg = ci.ndeps = ci.nactors = ci.strbytes = 0;
    ci.nheads = ci.nunk = 0; ci.arg0 = 0;
    valid = false;
    cd.off = 0; cd.len = 0; cd.flags = 0;
  }
  // span of the wave's chunks
  uint64_t lo = valid ? cd.off : ~0ull, hi = valid ? cd.off + cd.len : 0ull;
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) {
    const uint64_t a = __shfl_xor(lo, d, 64), b2 = __shfl_xor(hi, d, 64);
    lo = a < lo ? a : lo;
    hi = b2 > hi ? b2 : hi;
  }
  const uint64_t lo16 = lo & ~15ull;
  const bool staged = hi > lo && hi - lo16 <= KC_STAGE;
  if (staged) {
    const uint32_t nv = (uint32_t)((hi - lo16 + 15) >> 4);
    uint4* dst = reinterpret_cast<uint4*>(stage[w]);
    const uint4* src = reinterpret_cast<const uint4*>(arena + lo16);
    for (uint32_t v = l; v < nv; v += 64) dst[v] = src[v];
  }
  __syncthreads();
  // a large document: counted by the whole wave over an LDS window when the wave holds at most two
  // (one at a time, each ~3x faster than one lane's chain over global memory); a wave of many large
  // documents keeps one lane per document, their chains overlapping
  const bool large = valid && cd.len > KC_BIG && arena[cd.off + 8] == 0;
  const bool defer = large && __popcll(__ballot(large)) <= 2;
  uint32_t dcols[12];
#pragma unroll
  for (int k = 0; k < 12; k++) dcols[k] = 0;
  if (valid) {
    if (staged) chunk_body(stage[w] + (cd.off - lo16), cd, i, info, hdr, false, dcols);
    else chunk_body(arena + cd.off, cd, i, info, hdr, defer, dcols);
  }
  // the large documents of this wave (at most two): lanes 8j + k count column k of the j-th one, each
  // over its own line of global memory, so the six chains of dependent reads run side by side
  // (their chunk_body stopped before the counts when its header parse succeeded). The first failing
  // column in the order below gives the status, as counting them one after another would.
  uint64_t big = __ballot(defer && dcols[1] + dcols[3] + dcols[5] + dcols[7] + dcols[9] + dcols[11] + dcols[0] > 0);
  if (big) {
    const int j0 = __builtin_ctzll(big);
    const uint64_t rest = big & (big - 1);
    const int j1 = rest ? __builtin_ctzll(rest) : -1;
    const uint32_t grp = l >> 3, k = l & 7;
    const int j = grp == 0 ? j0 : grp == 1 ? j1 : -1;
    // every lane reads its document's column table entries (shuffles are wave-wide)
    const int js = j < 0 ? 0 : j;
    uint32_t o = 0, n = 0;
#pragma unroll
    for (int q = 0; q < 6; q++) {
      const uint32_t oq = __shfl(dcols[2 * q], js, 64), nq = __shfl(dcols[2 * q + 1], js, 64);
      if ((int)k == q) { o = oq; n = nq; }
    }
    const uint64_t goff = __shfl(cd.off, js, 64);
    uint64_t c = 0, sm = 0;
    uint32_t st = AM_OK;
    if (j >= 0 && k < 6) {
      LineRd rd{arena, goff, ~0ull, make_uint4(0, 0, 0, 0)};
      st = win_count_sum(rd, o, n, k >= 4, k == 2, c, sm);
    }
    // gather per document: lanes 8g .. 8g + 5
#pragma unroll
    for (int g = 0; g < 2; g++) {
      const int jg = g == 0 ? j0 : j1;
      if (jg < 0) continue;
      uint64_t v[6], w6[6];
      uint32_t e[6];
#pragma unroll
      for (int q = 0; q < 6; q++) {
        v[q] = __shfl(c, 8 * g + q, 64);
        w6[q] = __shfl(sm, 8 * g + q, 64);
        e[q] = __shfl(st, 8 * g + q, 64);
      }
      if ((int)l == jg) {
        uint32_t first = AM_OK;
#pragma unroll
        for (int q = 0; q < 6; q++)
          if (!first) first = e[q];
        ChunkInfo& ci = info[i];
        if (first) {
          ci.status = first;
        } else {
          ci.nchg = (uint32_t)v[0];
          ci.ndeps = (uint32_t)w6[1];
          ci.nops = (uint32_t)v[2];
          ci.nents = (uint32_t)w6[3];
          ci.strbytes = (uint32_t)(w6[4] + w6[5]);
        }
      }
    }
  }
}


// ------------------------------------------------------------------------------------------
// Exclusive scan of u64 (three kernels: per-block, block totals, add)
// ------------------------------------------------------------------------------------------
#define SCAN_T 256
__global__ void __launch_bounds__(SCAN_T) k_scan_blocks(const uint64_t* __restrict__ in, uint64_t* __restrict__ out,
                                                        uint64_t* __restrict__ block_sums, uint32_t n) {
  __shared__ uint64_t s[SCAN_T];
  uint32_t i = blockIdx.x * SCAN_T + threadIdx.x;
  uint64_t v = i < n ? in[i] : 0;
  s[threadIdx.x] = v;
  __syncthreads();
  for (uint32_t off = 1; off < SCAN_T; off <<= 1) {
    uint64_t x = threadIdx.x >= off ? s[threadIdx.x - off] : 0;
    __syncthreads();
    s[threadIdx.x] += x;
    __syncthreads();
  }
  if (i < n) out[i] = s[threadIdx.x] - v;
  if (threadIdx.x == SCAN_T - 1) block_sums[blockIdx.x] = s[SCAN_T - 1];
}
__global__ void __launch_bounds__(SCAN_T) k_scan_top(uint64_t* __restrict__ block_sums, uint32_t nblocks, uint64_t* __restrict__ total) {
  __shared__ uint64_t s[SCAN_T];
  uint64_t carry = 0;
  for (uint32_t base = 0; base < nblocks; base += SCAN_T) {
    uint32_t i = base + threadIdx.x;
    uint64_t v = i < nblocks ? block_sums[i] : 0;
    s[threadIdx.x] = v;
    __syncthreads();
    for (uint32_t off = 1; off < SCAN_T; off <<= 1) {
      uint64_t x = threadIdx.x >= off ? s[threadIdx.x - off] : 0;
      __syncthreads();
      s[threadIdx.x] += x;
      __syncthreads();
    }
    if (i < nblocks) block_sums[i] = carry + s[threadIdx.x] - v;
    uint64_t t = s[SCAN_T - 1];
    __syncthreads();
    carry += t;
  }
  if (threadIdx.x == 0) *total = carry;
}
__global__ void __launch_bounds__(SCAN_T) k_scan_add(uint64_t* __restrict__ out, const uint64_t* __restrict__ block_sums, uint32_t n) {
  uint32_t i = blockIdx.x * SCAN_T + threadIdx.x;
  if (i < n) out[i] += block_sums[blockIdx.x];
}

// ------------------------------------------------------------------------------------------
// k_doc: one workgroup (one wave) per document
// ------------------------------------------------------------------------------------------
#define DOC_T 64
#define DOC_T_GLB 256  // global-mode k_doc workgroup (4 waves per document)

struct IdKey { int64_t ctr; int32_t actor; int32_t row; };
struct ElemKey { int64_t obj_ctr; int64_t id_ctr; int32_t obj_rank; int32_t parent; int32_t id_rank; int32_t row; };
struct SortRec {
  int64_t obj_ctr; int64_t k1; int64_t id_ctr; uint64_t key_off;
  int32_t obj_rank; int32_t kind; int32_t id_rank; int32_t row; uint32_t key_len; uint32_t pad;
};
struct NewEnt { int64_t ctr; int32_t target; int32_t actor; int32_t rank; int32_t pad; };

// Optional per-phase cycle counters (probe builds only: -DAM_PHASE_CLOCK). Every 64th document
// adds the s_memtime delta of each phase; read back with amx_phase_cycles().
#ifdef AM_PHASE_CLOCK
__device__ unsigned long long am_phase_cycles[48];
#define PH(k)                                                                  \
  do {                                                                         \
    __syncthreads();                                                           \
    if (threadIdx.x == 0 && (blockIdx.x & 63) == 0) {                          \
      const uint64_t now_ = clock64();                                         \
      atomicAdd(&am_phase_cycles[k], (unsigned long long)(now_ - s.ph_last));  \
      s.ph_last = now_;                                                        \
    }                                                                          \
  } while (0)
#elif defined(AM_DIFF_CHECK)
// (AM_DEBUG_WS_CANARY runs of one document: the 16 bytes after its workspace hold 0xA5)
__device__ __forceinline__ bool dbg_canary_hit(const uint8_t* p) {
  for (int i = 0; i < 16; i++) if (p[i] != 0xA5) return true;
  return false;
}
// diagnostics build: at every phase marker thread 0 compares the document's shared bounds with the
// global copy and records the first phase after which they differ (s.dbg_phase; result status 280 + k)
#define PH(k)                                                                                            \
  do {                                                                                                   \
    __syncthreads();                                                                                     \
    if (threadIdx.x == 0 && s.dbg_phase == 0xffffu) {                                                    \
      const DocBounds gb_ = bounds[doc];                                                                 \
      if (gb_.R != s.b.R || gb_.E != s.b.E || gb_.P != s.b.P || gb_.N != s.b.N || gb_.C != s.b.C ||      \
          ws_layout(gb_).total != s.L.total || ws_layout(gb_).pwire != s.L.pwire)                        \
        s.dbg_phase = (k);                                                                               \
    }                                                                                                    \
    if (threadIdx.x == 0 && s.dbg_canary == 0xffffu && dbg_canary_hit(wsg + s.L.total))                 \
      s.dbg_canary = (k);                                                                                \
    __syncthreads();                                                                                     \
  } while (0)
#else
#define PH(k) \
  do {        \
  } while (0)
#endif

struct DocShared {
  DocHdr dh;
  DocBounds b;
  WsLayout L;
  uint8_t* ws;          // global workspace of this document (cold regions + hot mirror)
  uint8_t* hot;         // hot regions: LDS or the global mirror
  const uint8_t* A;     // arena view: A + arena_offset -> byte (staged in LDS when possible)
  uint32_t status, errchg;
  int64_t arg0, arg1;
  uint64_t arg_actor_off;
  uint32_t arg_actor_len;
  uint32_t has_base, nb, nbe, nbc, nbd;   // base rows / succ entries / change rows / deps
  uint32_t napplied, nqueued, nactors, nheads;
  uint32_t nrows, nents, nchg, ndeps;     // totals after planning
  uint32_t nout, nnew;
  uint32_t npass;                         // applyChanges passes that applied changes (P == 2)
  uint32_t pf_ok, pf_nheads;              // plan_fast: the closed form applies; heads collected
  unsigned long long pf_maxop;            // plan_fast: maxOp of the applied changes
  uint32_t nb_act;                        // values in the base document's action column: the ops
                                          // readNextDocOp sees (new.js:658-670), normally nb
  int64_t max_op;
  uint32_t col_len[OC_NCOLS + DC_NCOLS];
  uint32_t col_pos[OC_NCOLS + DC_NCOLS];
  uint64_t out_len;
  uint32_t* tmp;                          // block scans' scratch: blockDim.x + 1 entries (k_doc_one)
  uint64_t ph_last;
  uint32_t xs_used;                       // bytes of replaced strings after the staged input (b.U)
  uint32_t nunk_inst, nunk_ids;           // unknown op columns: instances, distinct output columns
#ifdef AM_DIFF_CHECK
  uint32_t dbg_phase, dbg_canary;
#endif
};

__device__ static void set_err(DocShared& s, uint32_t code, int64_t a0 = 0, int64_t a1 = 0, uint64_t actor_off = 0,
                               uint32_t actor_len = 0, uint32_t chg = 0xffffffffu) {
  if (atomicCAS(&s.status, 0u, code) == 0u) {
    s.arg0 = a0;
    s.arg1 = a1;
    s.arg_actor_off = actor_off;
    s.arg_actor_len = actor_len;
    s.errchg = chg;
  }
}

template <typename T>
__device__ __forceinline__ T* wsp(DocShared& s, uint64_t off) { return reinterpret_cast<T*>(s.ws + off); }

__device__ __forceinline__ bool hash_eq(const uint8_t* a, const uint8_t* b) {
  for (int i = 0; i < 32; i++) if (a[i] != b[i]) return false;
  return true;
}
__device__ __forceinline__ int hash_cmp(const uint8_t* a, const uint8_t* b) {
  for (int i = 0; i < 32; i++) if (a[i] != b[i]) return a[i] < b[i] ? -1 : 1;
  return 0;
}

// index of a base head in changeIndexByHash (new.js:1729-1739)
#include "am_patch.h"

// a document whose chunks are not adjacent in the arena has no input span (k_bounds): it runs in
// the global mode, reading the arena directly
__host__ __device__ inline bool doc_scattered(const DocBounds& b) { return b.span_hi == b.span_lo && b.B > 0; }

extern __shared__ __attribute__((aligned(16))) uint8_t am_lds[];

// k_doc's P4 decodes a stream of this many values or more with a whole wave (decode_stream_wave),
// the rest a lane each. AM_DEC_LONG (environment, read at every k_doc launch) moves the threshold:
// a value past every stream's length keeps them all on lanes (the tests compare the two decoders).
__device__ uint32_t am_dec_long = 256;
static void dec_long_sync() {
  static std::atomic<uint32_t> cur{256};
  const char* e = std::getenv("AM_DEC_LONG");
  const uint32_t v = e ? (uint32_t)std::strtoul(e, nullptr, 10) : 256u;
  if (v != cur.load()) {
    (void)hipDeviceSynchronize();
    (void)hipMemcpyToSymbol(HIP_SYMBOL(am_dec_long), &v, sizeof v);
    cur.store(v);
  }
}

#ifndef AM_LDS_DOC_T
#define AM_LDS_DOC_T DOC_T
#endif
#define K_DOC_WAVES_ATTR
namespace lds_mode {
constexpr bool kHotLds = true;
constexpr uint32_t kDocT = AM_LDS_DOC_T;  // the waves that share this document's LDS slice
#include "am_doc_impl.h"
}  // namespace lds_mode
#undef K_DOC_WAVES_ATTR
#ifndef AM_GLB_WAVES
#define AM_GLB_WAVES 4
#endif
namespace glb_mode {
constexpr bool kHotLds = false;
// four waves: large documents' sorts, scans and list ranking are latency-bound chains over global
// arrays; more lanes in flight per document (and more waves per SIMD) hide that latency
constexpr uint32_t kDocT = DOC_T_GLB;
#undef K_DOC_WAVES_ATTR
// four waves per SIMD (<= 128 VGPRs, the rest spills): four documents share a CU; measured on C3
// (1000 x 100k-op texts): 1 wave 1076 ms, 4 waves at 2 per SIMD 931 ms, at 4 per SIMD 783 ms
#define K_DOC_WAVES_ATTR __attribute__((amdgpu_waves_per_eu(AM_GLB_WAVES, 8)))
#include "am_doc_impl.h"
#undef K_DOC_WAVES_ATTR
}  // namespace glb_mode
// The same kernel at eight waves per SIMD (64 VGPRs, more of its state in scratch) for batches of many
// documents: their resident waves hide more of the global-memory latency than they lose to the
// spills (8,192 mid documents: k_doc 20.9 -> 17.4 ms; C3's 1,000 100k-op documents 208.5 / 209.9
// ms either way; one 100k-op document alone, the per-handle call, is 3% slower at eight:
// profiles/r6/r6t_ab_glb_waves.txt). Launched for batches of AM_GLB8_MIN documents or more
// (environment; default 1024).
static uint32_t glb8_min() {
  const char* e = std::getenv("AM_GLB8_MIN");
  return e ? (uint32_t)std::strtoul(e, nullptr, 10) : 1024u;
}
namespace glb8_mode {
constexpr bool kHotLds = false;
constexpr uint32_t kDocT = DOC_T_GLB;
#define K_DOC_WAVES_ATTR __attribute__((amdgpu_waves_per_eu(8, 8)))
#include "am_doc_impl.h"
#undef K_DOC_WAVES_ATTR
}  // namespace glb8_mode
// A batch of a few large documents (a per-handle call on one 100k-op text, say) leaves most of the
// GPU idle: each document gets a 16-wave workgroup, so its sorts, scans, gathers and list ranking
// run on four times the lanes (the column decode and encode keep their lane / wave per column).
// Launched for batches of at most AM_GLB16_MAX documents (environment; default 8).
#define DOC_T_GLB16 1024
static uint32_t glb16_max() {
  const char* e = std::getenv("AM_GLB16_MAX");
  return e ? (uint32_t)std::strtoul(e, nullptr, 10) : 8u;
}
namespace glb16_mode {
constexpr bool kHotLds = false;
constexpr uint32_t kDocT = DOC_T_GLB16;
#define K_DOC_WAVES_ATTR
#include "am_doc_impl.h"
#undef K_DOC_WAVES_ATTR
}  // namespace glb16_mode
// P8 of the global-mode documents (glb_mode::k_diff_one): one wave per document. Wide: all lanes run
// the replay (scans and searches spread over them: few, large documents); else lane 0 alone (many
// documents: the waves themselves fill the machine). The chain is dependent loads: resident waves hide
// their latency, but a register cap that spills puts scratch round trips into the chain itself.
// Measured (C5 pairs merged with their patch, 65,536 per batch / mid documents, 8,192): 8 waves per
// SIMD 236 ms / 29.3M ops/s, 6: 234 / 29.7M, 4: 207 / 34.8M, 3: 232 / 30.8M, 2: 278 / 26.3M
#ifndef AM_DIFF_WAVES
#define AM_DIFF_WAVES 4
#endif
template <bool Wide>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(AM_DIFF_WAVES, 8))) k_diff(const uint8_t* __restrict__ arena, const am_chunk_desc* __restrict__ chunks,
                                             const am_doc_desc* __restrict__ docs, const DocBounds* __restrict__ bounds,
                                             const uint64_t* __restrict__ ws_off, uint8_t* __restrict__ ws_base, uint32_t lds_bytes,
                                             const am_doc_result* __restrict__ results, const uint8_t* __restrict__ fast_done) {
  glb_mode::k_diff_one<Wide>(blockIdx.x, arena, chunks, docs, bounds, ws_off, ws_base, lds_bytes, results, fast_done);
}
#include "am_doc_fast.h"
#include "am_hist_dev.h"

void am_fast_slices_host(const DocBounds* db, const am_doc_desc* dd, uint32_t n, uint32_t* out) {
  for (uint32_t d = 0; d < n; d++) out[d] = fast_eligible(db[d], dd[d]) ? fast_layout(db[d], dd[d].known_count).total : 0u;
}

// ------------------------------------------------------------------------------------------
// k_bounds: one thread per document -> workspace bounds
// ------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_bounds(const uint8_t* __restrict__ arena, const am_doc_desc* __restrict__ docs, uint32_t ndocs,
                                                const am_chunk_desc* __restrict__ chunks, const ChunkInfo* __restrict__ info,
                                                DocBounds* __restrict__ bounds, uint64_t* __restrict__ ws_bytes,
                                                uint64_t* __restrict__ max_hot, bool compact, uint32_t fast_cap) {
  const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t h = 0, f = 0;  // k_doc hot set; k_doc_fast LDS slice (0: outside its envelope)
  uint64_t saved = 0;     // the whole plan of a document given the compact one (its overflow reserve)
  if (d < ndocs) {
  am_doc_desc dd = docs[d];
  DocBounds b;
  uint64_t R = 0, E = 0, C = 0, D = 0, A = 0, H = 0, S = 0, B = 0, AM = 0, ND = 0, UC = 0, UV = 0;
  uint64_t lo = ~0ull, hi = 0;
  if (dd.base_chunk >= 0) {
    const ChunkInfo& ci = info[dd.base_chunk];
    R += ci.nops; E += ci.nents; C += ci.nchg; D += ci.ndeps; A += ci.nactors; H += ci.nheads;
    S += ci.strbytes; B += chunks[dd.base_chunk].len;
    if (ci.nunk && !ci.status) {
      const uint64_t ub = unknown_bound(arena + chunks[dd.base_chunk].off + ci.data_off, ci.data_len, true, ci.nunk, ci.nops);
      UC += ci.nunk;
      // a malformed unknown column: a row-sized bound, k_doc's decode reports the error itself
      UV += (ub >> 32) ? (uint64_t)(ci.nunk + 3) * ci.nops : (uint32_t)ub;
    }
    lo = chunks[dd.base_chunk].off;
    hi = lo + chunks[dd.base_chunk].len;
  }
  for (uint32_t k = 0; k < dd.chg_count; k++) {
    const ChunkInfo& ci = info[dd.chg_begin + k];
    const am_chunk_desc cd = chunks[dd.chg_begin + k];
    R += ci.nops; E += ci.nents; C += 1; D += ci.ndeps; A += 1; H += 1; S += ci.strbytes;
    B += cd.len;
    if (ci.nunk && !ci.status) {
      const uint64_t ub = unknown_bound(arena + cd.off + ci.data_off, ci.data_len, false, ci.nunk, ci.nops);
      UC += ci.nunk;
      UV += (ub >> 32) ? (uint64_t)(ci.nunk + 3) * ci.nops : (uint32_t)ub;
    }
    AM += ci.nactors;
    ND += ci.ndeps;
    if (cd.off < lo) lo = cd.off;
    if (cd.off + cd.len > hi) hi = cd.off + cd.len;
  }
  if (hi < lo) lo = hi = 0;
  // chunks of one document are normally adjacent; a scattered document is not staged in LDS
  if (hi - lo > 2 * B + 64) hi = lo;
  const uint64_t cap = 0x3fffffffull;
  if (R > cap || E > cap || C > cap || D > cap || AM > cap || ND > cap || UV > cap) { R = E = C = D = AM = ND = UC = UV = 0; A = H = 0; S = B = 0; lo = hi = 0; }
  b.R = (uint32_t)R; b.E = (uint32_t)E; b.C = (uint32_t)C; b.D = (uint32_t)D; b.A = (uint32_t)A;
  b.H = (uint32_t)H; b.N = dd.chg_count; b.K = (uint32_t)(H + dd.known_count); b.AM = (uint32_t)AM;
  b.ND = (uint32_t)ND; b.S = S; b.B = B; b.span_lo = lo; b.span_hi = hi;
  b.P = (dd.flags & AM_DOC_WANT_PATCH) ? 1u : (dd.flags & AM_DOC_WANT_DIFF) ? 2u : 0u;
  b.U = ((dd.flags & AM_DOC_FIX_UTF8) ? 1u : 0u) | ((dd.flags & AM_DOC_PATCH_ROOM) ? 2u : 0u);
  b.UC = (uint32_t)UC; b.UV = (uint32_t)UV;
  WsLayout L = ws_layout(b);
  // a scattered document needs the global-mode launch: report a hot set above any LDS budget
  h = doc_scattered(b) ? (1ull << 40) : L.hot_total;
  if (fast_eligible(b, dd)) f = fast_layout(b, dd.known_count).total;
  uint64_t total = L.total;
  // k_doc_fast's document: its compact plan (k_rest re-plans it if the kernel gives up). A slice above
  // the launch's (a pipeline's fixed fast_lds) never runs there: it keeps the whole plan in the scan
  if (compact && f && f <= fast_cap) {
    b.U |= 4u;
    total = ws_layout(b).total;
    saved = L.total;
  }
  bounds[d] = b;
  ws_bytes[d] = total;
  }
  // max_hot[0]: largest k_doc hot working set; max_hot[1]: largest k_doc_fast LDS slice -- one
  // atomic per wave
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint64_t h2 = __shfl_xor(h, o, 64), f2 = __shfl_xor(f, o, 64);
    h = h2 > h ? h2 : h;
    f = f2 > f ? f2 : f;
    saved += __shfl_xor(saved, o, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    if (h) atomicMax(reinterpret_cast<unsigned long long*>(max_hot), (unsigned long long)h);
    if (f) atomicMax(reinterpret_cast<unsigned long long*>(max_hot + 1), (unsigned long long)f);
    if (saved) atomicAdd(reinterpret_cast<unsigned long long*>(max_hot + 2), (unsigned long long)saved);
  }
}


// ------------------------------------------------------------------------------------------
// k_compact: workgroup per document copies its merged chunk into the dense output arena
// k_out_hash: thread per document computes the container checksum (columnar.js:659-686)
// ------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_out_len(const am_doc_result* __restrict__ res, uint32_t ndocs, uint64_t* __restrict__ lens) {
  uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d < ndocs) lens[d] = res[d].out_len;
}
__global__ void __launch_bounds__(256) k_compact(const uint8_t* __restrict__ ws_base, am_doc_result* __restrict__ res,
                                                 const uint64_t* __restrict__ out_off, const DocBounds* __restrict__ bounds,
                                                 uint8_t* __restrict__ out) {
  const uint32_t d = blockIdx.x;
  const uint64_t len = res[d].out_len;
  if (threadIdx.x == 0) res[d].out_off = out_off[d];
  if (!len) return;
  const WsLayout L = ws_layout(bounds[d]);
  const uint8_t* src = ws_base + res[d].ws_off + L.out;
  uint8_t* dst = out + out_off[d];
  for (uint64_t q = threadIdx.x; q < len; q += blockDim.x) dst[q] = src[q];
}
__global__ void __launch_bounds__(256) k_out_hash(const am_doc_result* __restrict__ res, uint32_t ndocs, uint8_t* __restrict__ out) {
  uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= ndocs) return;
  const uint64_t len = res[d].out_len;
  if (!len) return;
  uint8_t* p = out + res[d].out_off;
  uint8_t h[32];
  sha256_dev(p + 8, len - 8, h);
  p[4] = h[0]; p[5] = h[1]; p[6] = h[2]; p[7] = h[3];
}
// standalone batched SHA-256 (used by the host stage for inflated inputs and by tests)
__global__ void __launch_bounds__(256) k_sha256(const uint8_t* __restrict__ arena, const am_chunk_desc* __restrict__ msgs,
                                                uint32_t n, uint8_t* __restrict__ out) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint8_t h[32];
  sha256_dev(arena + msgs[i].off, msgs[i].len, h);
  for (int k = 0; k < 32; k++) out[32 * i + k] = h[k];
}

// ------------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------------
#include "am_launch.h"

static_assert(sizeof(Row) == AM_SZ_ROW, "Row");
static_assert(sizeof(PatchRec) == 64 && sizeof(PatchVal) == 32 && sizeof(PatchHdr2) == 48, "patch log layout");
static_assert(PATCH_E_FLOAT_LEN == AM_E_FLOAT_LEN && PATCH_E_UNKNOWN_COUNTER == AM_E_UNKNOWN_COUNTER &&
              PATCH_U_CAPACITY == AM_U_CAPACITY && PATCH_U_VALUE == AM_U_VALUE, "patch status codes");
static_assert(sizeof(Ent) == AM_SZ_ENT, "Ent");
static_assert(sizeof(IdKey) == AM_SZ_IDKEY, "IdKey");
static_assert(sizeof(ElemKey) == AM_SZ_ELEMKEY, "ElemKey");
static_assert(sizeof(SortRec) == AM_SZ_SORTREC, "SortRec");
static_assert(sizeof(NewEnt) == AM_SZ_NEWENT, "NewEnt");
static_assert(sizeof(ChgRow) == AM_SZ_CHGROW, "ChgRow");
static_assert(sizeof(ActorRef) == AM_SZ_ACTORREF, "ActorRef");
static_assert(sizeof(ChgHdr) <= AM_SZ_CHGHDR, "ChgHdr");

size_t am_scan_tmp_elems(uint32_t n) { return (n + SCAN_T - 1) / SCAN_T + 1; }


void am_launch_chunks(const BatchDev& b, hipStream_t s) {
  if (!b.nchunks) return;
  hipLaunchKernelGGL(k_chunks, dim3((b.nchunks + 255) / 256), dim3(256), 0, s, b.arena, b.chunks, b.nchunks, b.info, b.hdr);
}
void am_launch_history(const uint8_t* arena, const am_chunk_desc* chunks, const ChunkInfo* info, const HistDesc* hd, uint32_t ndocs,
                       uint8_t* ws, uint8_t* out, HistResult* res, HistChange* chg_out, hipStream_t s) {
  if (!ndocs) return;
  hipLaunchKernelGGL(k_history, dim3(ndocs), dim3(64), 0, s, arena, chunks, info, hd, ndocs, ws, out, res, chg_out);
}
__global__ void __launch_bounds__(256) k_history_sizes(const HistResult* __restrict__ res, const HistDesc* __restrict__ hd, uint32_t ndocs,
                                                      const uint32_t* __restrict__ nchg, HistChange* __restrict__ chg,
                                                      uint64_t* __restrict__ sizes) {
  const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= ndocs) return;
  uint64_t acc = 0;
  if (res[d].status == HE_OK) {
    HistChange* c = chg + hd[d].chg_off;
    for (uint32_t k = 0; k < nchg[d]; k++) {
      const uint64_t src = c[k].off;
      c[k].off = acc | (src << 32);  // dense offset (low) | region offset (high): both < 4 GiB per document
      acc += c[k].len;
    }
  }
  sizes[d] = acc;
}
__global__ void __launch_bounds__(64) k_history_compact(const HistResult* __restrict__ res, const HistDesc* __restrict__ hd, uint32_t ndocs,
                                                        const uint32_t* __restrict__ nchg,
                                                        const HistChange* __restrict__ chg, const uint64_t* __restrict__ doc_off,
                                                        const uint8_t* __restrict__ out, uint8_t* __restrict__ dst) {
  const uint32_t d = blockIdx.x;
  if (d >= ndocs || res[d].status != HE_OK) return;  // only documents whose records k_history_sizes rewrote
  const HistDesc h = hd[d];
  uint8_t* o = dst + doc_off[d];
  for (uint32_t k = 0; k < nchg[d]; k++) {
    const HistChange c = chg[h.chg_off + k];
    const uint8_t* src = out + h.out_off + (c.off >> 32);
    uint8_t* q = o + (uint32_t)c.off;
    for (uint32_t i = threadIdx.x; i < c.len; i += 64) q[i] = src[i];
  }
}
void am_launch_history_sizes(const HistResult* res, const HistDesc* hd, uint32_t ndocs, const uint32_t* nchg, HistChange* chg,
                             uint64_t* sizes, hipStream_t s) {
  if (!ndocs) return;
  hipLaunchKernelGGL(k_history_sizes, dim3((ndocs + 255) / 256), dim3(256), 0, s, res, hd, ndocs, nchg, chg, sizes);
}
void am_launch_history_compact(const HistResult* res, const HistDesc* hd, uint32_t ndocs, const uint32_t* nchg, const HistChange* chg,
                               const uint64_t* doc_off, const uint8_t* out, uint8_t* dst, hipStream_t s) {
  if (!ndocs) return;
  hipLaunchKernelGGL(k_history_compact, dim3(ndocs), dim3(64), 0, s, res, hd, ndocs, nchg, chg, doc_off, out, dst);
}
void am_launch_bounds(const BatchDev& b, hipStream_t s) {
  if (!b.ndocs) return;
  (void)hipMemsetAsync(b.max_hot, 0, 4 * sizeof(uint64_t), s);
  hipLaunchKernelGGL(k_bounds, dim3((b.ndocs + 255) / 256), dim3(256), 0, s, b.arena, b.docs, b.ndocs, b.chunks, b.info, b.bounds,
                     b.ws_bytes, b.max_hot, b.compact, b.fast_cap);
  uint32_t nblk = (b.ndocs + SCAN_T - 1) / SCAN_T;
  hipLaunchKernelGGL(k_scan_blocks, dim3(nblk), dim3(SCAN_T), 0, s, b.ws_bytes, b.ws_off, b.scan_tmp, b.ndocs);
  hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(SCAN_T), 0, s, b.scan_tmp, nblk, b.ws_total);
  hipLaunchKernelGGL(k_scan_add, dim3(nblk), dim3(SCAN_T), 0, s, b.ws_off, b.scan_tmp, b.ndocs);
}
// the documents k_doc_fast left, as a list for k_doc's loop (rest[0] = count, zeroed beforehand).
// One that had the compact plan gets the whole plan, bump-allocated in the overflow region after
// the scanned workspaces ([*ws_total, ws_cap)); past its end k_doc reports AM_U_CAPACITY.
__global__ void __launch_bounds__(256) k_rest(const uint8_t* __restrict__ fast_done, uint32_t ndocs, uint32_t* __restrict__ rest,
                                              DocBounds* __restrict__ bounds, uint64_t* __restrict__ ws_off,
                                              const uint64_t* __restrict__ ws_total, uint64_t* __restrict__ ovf) {
  const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x, l = threadIdx.x & 63;
  const bool need = d < ndocs && !fast_done[d];
  if (need && (bounds[d].U & 4u)) {
    DocBounds b = bounds[d];
    b.U &= ~4u;
    const uint64_t t = ws_layout(b).total;
    const uint64_t o = atomicAdd(reinterpret_cast<unsigned long long*>(ovf), (unsigned long long)t);
    bounds[d] = b;
    ws_off[d] = *ws_total + o;
  }
  const uint64_t m = __ballot(need);
  uint32_t base = 0;
  if (l == 0 && m) base = atomicAdd(rest, (uint32_t)__popcll(m));
  base = __shfl(base, 0, 64);
  if (need) rest[1 + base + (uint32_t)__popcll(m & ((1ull << l) - 1))] = d;
}
#define K_DOC_LOOP_WG 2048  // workgroups of k_doc's loop over the documents k_doc_fast left

void am_launch_doc(const BatchDev& b, hipStream_t s) {
  if (!b.ndocs) return;
  // documents whose hot working set fits the LDS allocation run from LDS; the rest (if any)
  // from their global workspace
  // small documents first: k_doc_fast merges every document in its envelope (one wave each,
  // one per workgroup) and marks it; k_doc then takes the rest and exits at once for the marked
  const uint8_t* fd = nullptr;
  if (b.fast_lds && b.fast_done) {
    (void)hipMemsetAsync(b.fast_done, 0, b.ndocs, s);
    // AM_FAST_SPLIT=<bytes> (probe): documents whose slice fits that many bytes run in a first launch
    // with the smaller slice (more workgroups per CU), the others in a second with the largest
    const char* se = std::getenv("AM_FAST_SPLIT");
    const uint32_t split = se ? (uint32_t)std::strtoul(se, nullptr, 10) & ~15u : 0u;
    auto launch = [&](uint32_t slice, uint32_t floor) {
      hipLaunchKernelGGL(b.any_diff ? k_doc_fast<true> : k_doc_fast<false>, dim3((b.ndocs + FD_DOCS_PER_WG - 1) / FD_DOCS_PER_WG),
                         dim3(64 * FD_DOCS_PER_WG), FD_DOCS_PER_WG * slice, s, b.arena, b.chunks, b.docs, b.known, b.info, b.hdr,
                         b.bounds, b.ws_off, b.ws, b.ws_cap, slice, floor, b.ndocs, b.results, b.chg_state, b.fast_done);
    };
    if (split && split < b.fast_lds) {
      launch(split, 0);
      launch(b.fast_lds, split);
    } else {
      launch(b.fast_lds, 0);
    }
    fd = b.fast_done;
  }
  if (!b.fast_only) {
    // after k_doc_fast: k_doc loops over the list of what it left (a batch merged whole by the fast
    // kernel then costs a few microseconds here instead of one workgroup launch per document)
    const uint32_t* rest = fd && b.rest ? b.rest : nullptr;
    uint32_t grid = b.ndocs;
    if (rest) {
      (void)hipMemsetAsync(b.rest, 0, sizeof(uint32_t), s);
      (void)hipMemsetAsync(b.max_hot + 3, 0, sizeof(uint64_t), s);
      hipLaunchKernelGGL(k_rest, dim3((b.ndocs + 255) / 256), dim3(256), 0, s, fd, b.ndocs, b.rest, b.bounds, b.ws_off,
                         b.ws_total, b.max_hot + 3);
      grid = b.ndocs < K_DOC_LOOP_WG ? b.ndocs : K_DOC_LOOP_WG;
    }
    dec_long_sync();
    hipLaunchKernelGGL(lds_mode::k_doc, dim3(grid), dim3(AM_LDS_DOC_T), b.lds_bytes, s, b.arena, b.chunks, b.docs, b.known,
                       b.info, b.bounds, b.ws_off, b.ws, b.ws_cap, b.lds_bytes, b.results, b.chg_state, fd, rest);
    if (b.max_hot_host > b.lds_bytes)
      hipLaunchKernelGGL(b.ndocs <= glb16_max() ? glb16_mode::k_doc : b.ndocs >= glb8_min() ? glb8_mode::k_doc : glb_mode::k_doc, dim3(b.ndocs),
                         dim3(b.ndocs <= glb16_max() ? DOC_T_GLB16 : DOC_T_GLB), 0, s, b.arena, b.chunks, b.docs, b.known, b.info,
                         b.bounds, b.ws_off, b.ws, b.ws_cap, b.lds_bytes, b.results, b.chg_state, fd, nullptr);
    {
      if (b.any_diff) {
        // wide replay for batches of fewer documents than wave slots (AM_DIFF_MODE=wide|lane0 overrides)
        static const int mode = [] {
          const char* v = std::getenv("AM_DIFF_MODE");
          return !v ? 0 : std::strcmp(v, "wide") == 0 ? 1 : std::strcmp(v, "lane0") == 0 ? 2 : 0;
        }();
        const bool wide = mode == 1 || (mode == 0 && b.ndocs < 1024);
        if (wide)
          hipLaunchKernelGGL(k_diff<true>, dim3(b.ndocs), dim3(64), 0, s, b.arena, b.chunks, b.docs, b.bounds, b.ws_off, b.ws,
                             b.lds_bytes, b.results, fd);
        else
          hipLaunchKernelGGL(k_diff<false>, dim3(b.ndocs), dim3(64), 0, s, b.arena, b.chunks, b.docs, b.bounds, b.ws_off, b.ws,
                             b.lds_bytes, b.results, fd);
      }
    }
  }
}
__global__ void __launch_bounds__(256) k_out_hash_ws(am_doc_result* __restrict__ res, uint32_t ndocs, uint8_t* __restrict__ ws,
                                                     const DocBounds* __restrict__ bounds) {
  uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= ndocs) return;
  const uint64_t len = res[d].out_len;
  if (!len) return;
  const WsLayout L = ws_layout(bounds[d]);
  uint8_t* p = ws + res[d].ws_off + L.out;
  res[d].out_off = res[d].ws_off + L.out;
  uint8_t h[32];
  sha256_dev(p + 8, len - 8, h);
  p[4] = h[0]; p[5] = h[1]; p[6] = h[2]; p[7] = h[3];
}
__device__ __forceinline__ uint64_t mix64(uint64_t x) {
  x ^= x >> 30; x *= 0xbf58476d1ce4e5b9ull;
  x ^= x >> 27; x *= 0x94d049bb133111ebull;
  return x ^ (x >> 31);
}
// per-document output digest (am_batch_digest): thread per document, one atomic per workgroup
__global__ void __launch_bounds__(256) k_digest(const am_doc_result* __restrict__ res, uint32_t ndocs, const uint8_t* __restrict__ ws,
                                                uint64_t first, unsigned long long* __restrict__ out) {
  const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t v = 0;
  if (d < ndocs) {
    const am_doc_result r = res[d];
    uint32_t chk = 0;
    if (r.status == 0 && r.out_len >= 8) {
      const uint8_t* p = ws + r.out_off + 4;
      chk = (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24;
    }
    v = mix64(((first + d) << 32) | chk) + (r.status ? 0 : r.out_len) * 0x9E3779B97F4A7C15ull + r.status;
  }
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  __shared__ uint64_t part[4];
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(out, (unsigned long long)(part[0] + part[1] + part[2] + part[3]));
}
void am_launch_digest(const BatchDev& b, uint64_t first, uint64_t* d_out, hipStream_t s) {
  (void)hipMemsetAsync(d_out, 0, sizeof(uint64_t), s);
  if (b.ndocs)
    hipLaunchKernelGGL(k_digest, dim3((b.ndocs + 255) / 256), dim3(256), 0, s, b.results, b.ndocs, b.ws, first,
                       reinterpret_cast<unsigned long long*>(d_out));
}
void am_launch_out_hash(const BatchDev& b, hipStream_t s) {
  if (!b.ndocs) return;
  hipLaunchKernelGGL(k_out_hash_ws, dim3((b.ndocs + 255) / 256), dim3(256), 0, s, b.results, b.ndocs, b.ws, b.bounds);
}
// the 32-byte hashes of every chunk of a batch, densely (the batched per-handle calls copy home
// these instead of the whole ChunkInfo table)
__global__ void __launch_bounds__(256) k_chunk_hashes(const ChunkInfo* __restrict__ info, uint32_t n, uint32_t* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 8ull * n) return;
  out[i] = reinterpret_cast<const uint32_t*>(info[i >> 3].hash)[i & 7];
}
void am_launch_chunk_hashes(const ChunkInfo* info, uint32_t n, uint8_t* out32, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_chunk_hashes, dim3((unsigned)((8ull * n + 255) / 256)), dim3(256), 0, s, info, n,
                            reinterpret_cast<uint32_t*>(out32));
}
void am_launch_sha256(const uint8_t* arena, const am_chunk_desc* msgs, uint32_t n, uint8_t* out, hipStream_t s) {
  if (!n) return;
  hipLaunchKernelGGL(k_sha256, dim3((n + 255) / 256), dim3(256), 0, s, arena, msgs, n, out);
}

// ------------------------------------------------------------------------------------------
// Pipelined batches (am_pipe_*, am_capi.hip): the merged documents and patch logs of a batch are
// gathered into two dense arenas (16-byte slots) so that one D2H copy each brings them home.
// ------------------------------------------------------------------------------------------
void am_launch_scan(const uint64_t* in, uint64_t* out, uint64_t* tmp, uint32_t n, uint64_t* total, hipStream_t s) {
  if (!n) { (void)hipMemsetAsync(total, 0, sizeof(uint64_t), s); return; }
  const uint32_t nblk = (n + SCAN_T - 1) / SCAN_T;
  hipLaunchKernelGGL(k_scan_blocks, dim3(nblk), dim3(SCAN_T), 0, s, in, out, tmp, n);
  hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(SCAN_T), 0, s, tmp, nblk, total);
  hipLaunchKernelGGL(k_scan_add, dim3(nblk), dim3(SCAN_T), 0, s, out, tmp, n);
}
// Packed batch descriptors (am_pipe_submit_packed): 4 B per chunk and 8 B per document cross the
// host link; the chunk offsets and each document's first chunk are two exclusive scans on the device.
__global__ void __launch_bounds__(256) k_unpack_counts(const uint32_t* __restrict__ clen, uint32_t nchunks,
                                                       const am_doc_span* __restrict__ spans, uint32_t ndocs,
                                                       uint64_t* __restrict__ c64, uint64_t* __restrict__ d64) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < nchunks) c64[i] = clen[i];
  if (i < ndocs) d64[i] = (uint64_t)spans[i].chg_count + (spans[i].has_base ? 1u : 0u);
}
// A chunk that runs past the arena is cut at its end (k_chunks then reports the truncated container)
// and a document whose chunks run past the batch keeps those it has: a wrong descriptor becomes a
// per-document error, never an out-of-bounds read.
__global__ void __launch_bounds__(256) k_unpack_write(const uint32_t* __restrict__ clen, const uint64_t* __restrict__ coff,
                                                      uint32_t nchunks, uint64_t arena_len, const am_doc_span* __restrict__ spans,
                                                      const uint64_t* __restrict__ dbeg, uint32_t ndocs,
                                                      am_chunk_desc* __restrict__ chunks, am_doc_desc* __restrict__ docs) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < nchunks) {
    const uint64_t off = coff[i];
    am_chunk_desc c;
    c.off = off < arena_len ? off : arena_len;
    c.len = off >= arena_len ? 0u : (uint32_t)(clen[i] < arena_len - off ? clen[i] : arena_len - off);
    c.flags = 0;
    chunks[i] = c;
  }
  if (i < ndocs) {
    const am_doc_span sp = spans[i];
    const uint64_t b = dbeg[i];
    const uint32_t hb = sp.has_base ? 1u : 0u;
    am_doc_desc d;
    const uint64_t first = b < nchunks ? b : nchunks;
    d.base_chunk = hb && first < nchunks ? (int64_t)first : -1;
    d.chg_begin = (uint32_t)(first + hb < nchunks ? first + hb : nchunks);
    d.chg_count = (uint32_t)(d.chg_begin + (uint64_t)sp.chg_count <= nchunks ? sp.chg_count : nchunks - d.chg_begin);
    d.known_begin = d.known_count = 0;
    d.flags = sp.flags & ~(uint32_t)AM_DOC_META;
    d.meta_chunk = 0;
    docs[i] = d;
  }
}
void am_launch_unpack(const uint32_t* clen, uint32_t nchunks, uint64_t arena_len, const am_doc_span* spans, uint32_t ndocs,
                      uint64_t* c64, uint64_t* coff, uint64_t* ctmp, uint64_t* d64, uint64_t* dbeg, uint64_t* dtmp,
                      uint64_t* totals2, am_chunk_desc* chunks, am_doc_desc* docs, hipStream_t s) {
  const uint32_t n = nchunks > ndocs ? nchunks : ndocs;
  if (!n) return;
  hipLaunchKernelGGL(k_unpack_counts, dim3((n + 255) / 256), dim3(256), 0, s, clen, nchunks, spans, ndocs, c64, d64);
  am_launch_scan(c64, coff, ctmp, nchunks, totals2, s);
  am_launch_scan(d64, dbeg, dtmp, ndocs, totals2 + 1, s);
  hipLaunchKernelGGL(k_unpack_write, dim3((n + 255) / 256), dim3(256), 0, s, clen, coff, nchunks, arena_len, spans, dbeg, ndocs,
                     chunks, docs);
}
// per document: 16-byte-rounded lengths of its merged chunk and of its patch log (wire form)
__global__ void __launch_bounds__(256) k_pipe_lens(const am_doc_result* __restrict__ res, const DocBounds* __restrict__ bounds,
                                                   const uint8_t* __restrict__ ws, uint32_t ndocs, uint64_t* __restrict__ olen,
                                                   uint64_t* __restrict__ plen) {
  const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= ndocs) return;
  const am_doc_result r = res[d];
  uint64_t o = 0, p = 0;
  if (!r.status) {
    o = (r.out_len + 15) & ~15ull;
    const DocBounds b = bounds[d];
    if (b.P) {
      const WsLayout L = ws_layout(b);
      const PatchHdr2* h = reinterpret_cast<const PatchHdr2*>(ws + r.ws_off + L.pwire);
      // (AM_DOC_META: the objectMeta blob follows the stream)
      if (h->magic == AM_PATCH_MAGIC && sizeof(PatchHdr2) + h->nbytes + h->meta_bytes <= L.pwire_cap)
        p = (sizeof(PatchHdr2) + h->nbytes + h->meta_bytes + 15) & ~15ull;
    }
  }
  olen[d] = o;
  plen[d] = p;
}
// one wave per document: 16-byte copies of its chunk and its log into the dense arenas, and its
// summary (documents whose slot does not fit the arenas report AM_U_CAPACITY)
__global__ void __launch_bounds__(256) k_pipe_compact(const am_doc_result* __restrict__ res, const DocBounds* __restrict__ bounds,
                                                      const uint8_t* __restrict__ ws, uint32_t ndocs,
                                                      const uint64_t* __restrict__ olen, const uint64_t* __restrict__ ooff,
                                                      const uint64_t* __restrict__ plen, const uint64_t* __restrict__ poff,
                                                      uint8_t* __restrict__ dout, uint64_t out_cap, uint8_t* __restrict__ dpatch,
                                                      uint64_t patch_cap, am_doc_summary* __restrict__ summary) {
  // wave-uniform document index (readfirstlane): scalar loads of its result and offsets
  const uint32_t d = (uint32_t)__builtin_amdgcn_readfirstlane((int)(blockIdx.x * 4 + (threadIdx.x >> 6))), l = threadIdx.x & 63;
  if (d >= ndocs) return;
  const am_doc_result r = res[d];
  const uint64_t on = olen[d], oo = ooff[d], pn = plen[d], po = poff[d];
  const bool ofit = oo + on <= out_cap, pfit = po + pn <= patch_cap;
  const uint64_t nov = (on && ofit) ? on / 16 : 0, npv = (pn && pfit) ? pn / 16 : 0;
  const uint8_t* const pw = pn ? ws + r.ws_off + ws_layout(bounds[d]).pwire : ws;  // the document's patch log
  const uint4* osrc = reinterpret_cast<const uint4*>(ws + r.out_off);
  const uint4* psrc = reinterpret_cast<const uint4*>(pw);
  uint4* odst = reinterpret_cast<uint4*>(dout + oo);
  uint4* pdst = reinterpret_cast<uint4*>(dpatch + po);
  // the first 1 KB of the document and of its log loaded together, then stored (most documents
  // end there); the rest in 1 KB steps
  uint4 a = {0, 0, 0, 0}, c = {0, 0, 0, 0};
  if (l < nov) a = osrc[l];
  if (l < npv) c = psrc[l];
  if (l < nov) odst[l] = a;
  if (l < npv) pdst[l] = c;
  for (uint64_t q = l + 64; q < nov; q += 64) odst[q] = osrc[q];
  for (uint64_t q = l + 64; q < npv; q += 64) pdst[q] = psrc[q];
  if (l == 0) {
    am_doc_summary sm;
    sm.status = (!ofit || !pfit) && !r.status ? (uint32_t)AM_U_CAPACITY : r.status;
    sm.nqueued = r.nqueued;
    sm.out_len = sm.status ? 0u : (uint32_t)r.out_len;
    uint32_t pl = 0;
    if (!sm.status && pn) {
      const PatchHdr2* h = reinterpret_cast<const PatchHdr2*>(pw);
      pl = (uint32_t)(sizeof(PatchHdr2) + h->nbytes + h->meta_bytes);
    }
    sm.patch_len = pl;
    sm.out_off = oo;
    sm.patch_off = po;
    summary[d] = sm;
  }
}
void am_launch_pipe_compact(const BatchDev& b, uint64_t* olen, uint64_t* ooff, uint64_t* plen, uint64_t* poff, uint64_t* tmp,
                            uint64_t* totals, uint8_t* dout, uint64_t out_cap, uint8_t* dpatch, uint64_t patch_cap,
                            am_doc_summary* summary, hipStream_t s) {
  if (!b.ndocs) { (void)hipMemsetAsync(totals, 0, 2 * sizeof(uint64_t), s); return; }
  hipLaunchKernelGGL(k_pipe_lens, dim3((b.ndocs + 255) / 256), dim3(256), 0, s, b.results, b.bounds, b.ws, b.ndocs, olen, plen);
  am_launch_scan(olen, ooff, tmp, b.ndocs, totals, s);
  am_launch_scan(plen, poff, tmp, b.ndocs, totals + 1, s);
  hipLaunchKernelGGL(k_pipe_compact, dim3((b.ndocs + 3) / 4), dim3(256), 0, s, b.results, b.bounds, b.ws, b.ndocs, olen, ooff,
                     plen, poff, dout, out_cap, dpatch, patch_cap, summary);
}

// Copies home over the host link, written by a kernel of a few workgroups straight into mapped
// pinned host memory: the runtime's own device-to-host path runs as a full-width blit kernel that
// would take the CUs from the next batch's kernels for as long as the link is busy.
struct CopySeg { const uint4* src; uint4* dst; uint64_t n16; };
__global__ void __launch_bounds__(256) k_copy_home(CopySeg a, CopySeg b, CopySeg c) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (uint64_t i = t; i < a.n16; i += stride) a.dst[i] = a.src[i];
  for (uint64_t i = t; i < b.n16; i += stride) b.dst[i] = b.src[i];
  for (uint64_t i = t; i < c.n16; i += stride) c.dst[i] = c.src[i];
}
void am_launch_copy_home(const void* s0, void* d0, uint64_t n0, const void* s1, void* d1, uint64_t n1, const void* s2, void* d2,
                         uint64_t n2, uint32_t wgs, hipStream_t s) {
  CopySeg a{reinterpret_cast<const uint4*>(s0), reinterpret_cast<uint4*>(d0), n0 / 16};
  CopySeg b{reinterpret_cast<const uint4*>(s1), reinterpret_cast<uint4*>(d1), n1 / 16};
  CopySeg c{reinterpret_cast<const uint4*>(s2), reinterpret_cast<uint4*>(d2), n2 / 16};
  hipLaunchKernelGGL(k_copy_home, dim3(wgs), dim3(256), 0, s, a, b, c);
}

// Self-test of the DPP / permlane primitives (am_wave.h) on the device: one wave, the lane values
// in[64] -> 16 result rows of 64 lanes (tests/test_gpu_wave.py checks them against numpy)
__global__ void __launch_bounds__(64) k_wave_selftest(const uint64_t* __restrict__ in, uint64_t* __restrict__ out) {
  const uint32_t l = threadIdx.x;
  const uint64_t v = in[l];
  const uint32_t v32 = (uint32_t)v;
  uint32_t tot = 0;
  out[0 * 64 + l] = wave::incl_add(v32);
  out[1 * 64 + l] = wave::excl_add(v32, tot);
  out[2 * 64 + l] = tot;
  out[3 * 64 + l] = (uint64_t)(int64_t)wave::incl_max((int32_t)v32);
  out[4 * 64 + l] = (uint64_t)wave::max_all((int64_t)v);
  out[5 * 64 + l] = wave::xor_lane<1>(v);
  out[6 * 64 + l] = wave::xor_lane<2>(v);
  out[7 * 64 + l] = wave::xor_lane<4>(v);
  out[8 * 64 + l] = wave::xor_lane<8>(v);
  out[9 * 64 + l] = wave::xor_lane<16>(v);
  out[10 * 64 + l] = wave::xor_lane<32>(v);
  out[11 * 64 + l] = wave::sort64(v);
  out[12 * 64 + l] = wave::up1(v, 7ull);
  out[13 * 64 + l] = wave::down1(v, 9ull);
  out[14 * 64 + l] = wave::bcast(v, 37);
  out[15 * 64 + l] = wave::sum_all(v32);
}
extern "C" int amx_wave_selftest(const uint64_t* in_host, uint64_t* out_host) {
  uint64_t *din = nullptr, *dout = nullptr;
  if (hipMalloc(&din, 64 * 8) != hipSuccess) return 1;
  if (hipMalloc(&dout, 16 * 64 * 8) != hipSuccess) { (void)hipFree(din); return 1; }
  int rc = hipMemcpy(din, in_host, 64 * 8, hipMemcpyHostToDevice) != hipSuccess;
  if (!rc) {
    hipLaunchKernelGGL(k_wave_selftest, dim3(1), dim3(64), 0, 0, din, dout);
    rc = hipDeviceSynchronize() != hipSuccess || hipMemcpy(out_host, dout, 16 * 64 * 8, hipMemcpyDeviceToHost) != hipSuccess;
  }
  (void)hipFree(din);
  (void)hipFree(dout);
  return rc;
}

#ifdef AM_PHASE_CLOCK
extern "C" int amx_phase_cycles(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(am_phase_cycles), sizeof(unsigned long long) * 48) != hipSuccess) return -1;
  if (reset) {
    unsigned long long z[48] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(am_phase_cycles), z, sizeof(z)) != hipSuccess) return -1;
  }
  return 0;
}
#endif
