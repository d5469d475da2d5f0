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

#include "am_dev_util.h"
#include "am_layout.h"

// column ids in spec order
__device__ __constant__ static const uint8_t kChangeColIds[OC_NCOLS] = {0x01, 0x02, 0x11, 0x13, 0x15, 0x21, 0x23, 0x34,
                                                                      0x42, 0x56, 0x57, 0x61, 0x63, 0x70, 0x71, 0x73};
__device__ __constant__ static const uint8_t kDocOpColIds[OC_NCOLS] = {0x01, 0x02, 0x11, 0x13, 0x15, 0x21, 0x23, 0x34,
                                                                     0x42, 0x56, 0x57, 0x61, 0x63, 0x80, 0x81, 0x83};
__device__ __constant__ static const uint8_t kDocChgColIds[DC_NCOLS] = {0x01, 0x03, 0x13, 0x23, 0x35, 0x40, 0x43, 0x56, 0x57};

__device__ __constant__ static const uint8_t kMagic[4] = {0x85, 0x6f, 0x4a, 0x83};
// scratch slot of each output column that is delta-encoded (others unused)
__device__ __constant__ static const uint8_t kScratchSlot[OC_NCOLS + DC_NCOLS] = {
  0, 0, 0, 0, 0, 0, 1, 0, 0, 0, 0, 0, 2, 0, 0, 3, 0, 4, 5, 6, 0, 0, 7, 0, 0};

// ------------------------------------------------------------------------------------------
// Header parsing (shared by k_chunks and k_doc). Offsets are relative to `base`, the arena
// offset of the chunk data, so headers stay compact (they live in LDS inside k_doc).
// ------------------------------------------------------------------------------------------
struct ChgHdr {              // decodeChangeHeader + column info (columnar.js:635-652, 741-765)
  uint64_t base;
  int64_t seq, start_op, time;
  uint32_t actor_off, actors_off, deps_off, msg_off, extra_off;
  uint32_t actor_len, nactors, ndeps, msg_len, extra_len, has_extra;
  uint32_t col_off[OC_NCOLS];
  uint32_t col_len[OC_NCOLS];
};
struct DocHdr {              // decodeDocumentHeader (columnar.js:1006-1038)
  uint64_t base;
  uint32_t actors_off, heads_off, hidx_off, extra_off;
  uint32_t nactors, nheads, has_hidx, extra_len;
  uint32_t ccol_off[DC_NCOLS];
  uint32_t ccol_len[DC_NCOLS];
  uint32_t ocol_off[OC_NCOLS];
  uint32_t ocol_len[OC_NCOLS];
};

// Column table (decodeColumnInfo, columnar.js:609) -> spec slots; the data follows in table
// order, i.e. ascending id order, so a second pass assigns offsets in spec order.
__device__ static uint32_t parse_cols(Rd& r, const uint8_t* spec, int nspec, uint32_t* len, bool is_change) {
  int64_t num;
  TRY(rd_u53(r, num));
  int64_t last = -1;
  for (int i = 0; i < nspec; i++) len[i] = 0;
  for (int64_t i = 0; i < num; i++) {
    int64_t id, l;
    TRY(rd_u53(r, id));
    TRY(rd_u53(r, l));
    if ((id & ~(int64_t)COL_DEFLATE) <= (last & ~(int64_t)COL_DEFLATE)) return AM_E_COL_ORDER;
    last = id;
    if (is_change && (id & COL_DEFLATE)) return AM_E_CHANGE_DEFLATED_COL;
    if (id & COL_DEFLATE) return AM_U_VALUE;  // the host stage inflates document columns
    int k = -1;
    for (int j = 0; j < nspec; j++) if (spec[j] == id) k = j;
    if (k < 0) return AM_U_UNKNOWN_COLUMN;
    if (l > 0x7fffffff) return AM_E_SUBARRAY;
    len[k] = (uint32_t)l;
  }
  return AM_OK;
}
__device__ static uint32_t place_cols(Rd& r, int nspec, uint32_t* off, const uint32_t* len) {
  for (int k = 0; k < nspec; k++) {
    uint64_t at;
    TRY(rd_raw(r, len[k], at));
    off[k] = (uint32_t)at;
  }
  return AM_OK;
}

__device__ static uint32_t parse_change_hdr(const uint8_t* data, uint64_t n, uint64_t abs, ChgHdr& h) {
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
  TRY(parse_cols(r, kChangeColIds, OC_NCOLS, h.col_len, true));
  TRY(place_cols(r, OC_NCOLS, h.col_off, h.col_len));
  h.has_extra = r.off < r.n;
  h.extra_off = (uint32_t)r.off;
  h.extra_len = (uint32_t)(r.n - r.off);
  return AM_OK;
}

__device__ static uint32_t parse_doc_hdr(const uint8_t* data, uint64_t n, uint64_t abs, DocHdr& h) {
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
  TRY(parse_cols(r, kDocChgColIds, DC_NCOLS, h.ccol_len, false));
  TRY(parse_cols(r, kDocOpColIds, OC_NCOLS, h.ocol_len, false));
  TRY(place_cols(r, DC_NCOLS, h.ccol_off, h.ccol_len));
  TRY(place_cols(r, OC_NCOLS, h.ocol_off, h.ocol_len));
  h.has_hidx = r.off < r.n;
  h.hidx_off = (uint32_t)r.off;
  if (h.has_hidx) {
    for (uint32_t i = 0; i < h.nheads; i++) TRY(rd_u53(r, v));
  }
  h.extra_off = (uint32_t)r.off;
  h.extra_len = (uint32_t)(r.n - r.off);
  return AM_OK;
}

// ------------------------------------------------------------------------------------------
// k_chunks: one thread per chunk
// ------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_chunks(const uint8_t* __restrict__ arena, const am_chunk_desc* __restrict__ chunks,
                                                uint32_t nchunks, ChunkInfo* __restrict__ info) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nchunks) return;
  am_chunk_desc cd = chunks[i];
  const uint8_t* p = arena + cd.off;
  ChunkInfo ci;
  for (int k = 0; k < 32; k++) ci.hash[k] = 0;
  ci.status = AM_OK; ci.type = 0xff; ci.data_off = 0; ci.data_len = 0; ci.nops = 0; ci.nents = 0; ci.nchg = 0;
  ci.ndeps = 0; ci.nactors = 0; ci.strbytes = 0; ci.nheads = 0; ci.arg0 = 0;
  uint32_t st = AM_OK;
  do {
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
    uint8_t h[32];
    sha256_dev(p + 8, r.off - 8, h);
    for (int k = 0; k < 32; k++) ci.hash[k] = h[k];
    if (!(cd.flags & 1) && (h[0] != p[4] || h[1] != p[5] || h[2] != p[6] || h[3] != p[7])) { st = AM_E_CHECKSUM; break; }
    const uint8_t* data = p + at;
    if (ci.type == 1) {
      if (r.off != cd.len) { st = AM_E_CHANGE_TRAILING; break; }
      ChgHdr hh;
      if ((st = parse_change_hdr(data, len, cd.off + at, hh))) break;
      ci.ndeps = hh.ndeps;
      ci.nactors = hh.nactors;
      uint64_t cnt, sum;
      // rows: values in the action column (new.js:701)
      if ((st = rle_count_sum(data + hh.col_off[OC_ACTION], hh.col_len[OC_ACTION], false, cnt, sum, 0))) break;
      ci.nops = (uint32_t)cnt;
      if ((st = rle_count_sum(data + hh.col_off[OC_GRP_NUM], hh.col_len[OC_GRP_NUM], false, cnt, sum, 0))) break;
      ci.nents = (uint32_t)sum;
      // key string bytes summed over rows (bounds the re-encoded keyStr column)
      uint64_t scnt, ssum;
      if ((st = rle_count_sum(data + hh.col_off[OC_KEY_STR], hh.col_len[OC_KEY_STR], true, scnt, ssum, 0))) break;
      ci.strbytes = (uint32_t)ssum + hh.msg_len;
    } else if (ci.type == 0) {
      if (r.off != cd.len) { st = AM_E_DOC_TRAILING; break; }
      DocHdr dh;
      if ((st = parse_doc_hdr(data, len, cd.off + at, dh))) break;
      ci.nactors = dh.nactors;
      ci.nheads = dh.nheads;
      uint64_t cnt, sum;
      if ((st = rle_count_sum(data + dh.ccol_off[DC_ACTOR], dh.ccol_len[DC_ACTOR], false, cnt, sum, 0))) break;
      ci.nchg = (uint32_t)cnt;
      if ((st = rle_count_sum(data + dh.ccol_off[DC_DEPS_NUM], dh.ccol_len[DC_DEPS_NUM], false, cnt, sum, 0))) break;
      ci.ndeps = (uint32_t)sum;
      // doc rows: values in the idCtr column (updateBlockMetadata, new.js:386)
      if ((st = rle_count_sum(data + dh.ocol_off[OC_ID_CTR], dh.ocol_len[OC_ID_CTR], false, cnt, sum, 0, true))) break;
      ci.nops = (uint32_t)cnt;
      if ((st = rle_count_sum(data + dh.ocol_off[OC_GRP_NUM], dh.ocol_len[OC_GRP_NUM], false, cnt, sum, 0))) break;
      ci.nents = (uint32_t)sum;
      uint64_t s1, s2;
      if ((st = rle_count_sum(data + dh.ocol_off[OC_KEY_STR], dh.ocol_len[OC_KEY_STR], true, cnt, s1, 0))) break;
      if ((st = rle_count_sum(data + dh.ccol_off[DC_MESSAGE], dh.ccol_len[DC_MESSAGE], true, cnt, s2, 0))) break;
      ci.strbytes = (uint32_t)(s1 + s2);
    } else {
      st = AM_E_CHUNK_TYPE;
      ci.arg0 = ci.type;
    }
  } while (0);
  ci.status = st;
  info[i] = ci;
}

// ------------------------------------------------------------------------------------------
// k_bounds: one thread per document -> workspace bounds
// ------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_bounds(const am_doc_desc* __restrict__ docs, uint32_t ndocs,
                                                const am_chunk_desc* __restrict__ chunks, const ChunkInfo* __restrict__ info,
                                                DocBounds* __restrict__ bounds, uint64_t* __restrict__ ws_bytes) {
  uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= ndocs) return;
  am_doc_desc dd = docs[d];
  DocBounds b;
  uint64_t R = 0, E = 0, C = 0, D = 0, A = 0, H = 0, S = 0, B = 0, AM = 0, ND = 0;
  uint64_t lo = ~0ull, hi = 0;
  if (dd.base_chunk >= 0) {
    const ChunkInfo& ci = info[dd.base_chunk];
    R += ci.nops; E += ci.nents; C += ci.nchg; D += ci.ndeps; A += ci.nactors; H += ci.nheads;
    S += ci.strbytes; B += chunks[dd.base_chunk].len;
    lo = chunks[dd.base_chunk].off;
    hi = lo + chunks[dd.base_chunk].len;
  }
  for (uint32_t k = 0; k < dd.chg_count; k++) {
    const ChunkInfo& ci = info[dd.chg_begin + k];
    const am_chunk_desc cd = chunks[dd.chg_begin + k];
    R += ci.nops; E += ci.nents; C += 1; D += ci.ndeps; A += 1; H += 1; S += ci.strbytes;
    B += cd.len;
    AM += ci.nactors;
    ND += ci.ndeps;
    if (cd.off < lo) lo = cd.off;
    if (cd.off + cd.len > hi) hi = cd.off + cd.len;
  }
  if (hi < lo) lo = hi = 0;
  // chunks of one document are normally adjacent; a scattered document is not staged in LDS
  if (hi - lo > 2 * B + 64) hi = lo;
  const uint64_t cap = 0x3fffffffull;
  if (R > cap || E > cap || C > cap || D > cap || AM > cap || ND > cap) { R = E = C = D = AM = ND = 0; A = H = 0; S = B = 0; lo = hi = 0; }
  b.R = (uint32_t)R; b.E = (uint32_t)E; b.C = (uint32_t)C; b.D = (uint32_t)D; b.A = (uint32_t)A;
  b.H = (uint32_t)H; b.N = dd.chg_count; b.K = (uint32_t)(H + dd.known_count); b.AM = (uint32_t)AM;
  b.ND = (uint32_t)ND; b.S = S; b.B = B; b.span_lo = lo; b.span_hi = hi;
  WsLayout L = ws_layout(b);
  bounds[d] = b;
  ws_bytes[d] = L.total;
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

struct IdKey { int64_t ctr; int32_t actor; int32_t row; };
struct ElemKey { int64_t obj_ctr; int64_t id_ctr; int32_t obj_rank; int32_t parent; int32_t id_rank; int32_t row; };
struct SortRec {
  int64_t obj_ctr; int64_t k1; int64_t id_ctr; uint64_t key_off;
  int32_t obj_rank; int32_t kind; int32_t id_rank; int32_t row; uint32_t key_len; uint32_t pad;
};
struct NewEnt { int64_t ctr; int32_t target; int32_t actor; int32_t rank; int32_t pad; };

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
  int64_t max_op;
  uint32_t col_len[OC_NCOLS + DC_NCOLS];
  uint32_t col_pos[OC_NCOLS + DC_NCOLS];
  uint64_t out_len;
  uint32_t tmp[DOC_T + 1];
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
__device__ __forceinline__ T* hp(DocShared& s, uint64_t off) { return reinterpret_cast<T*>(s.hot + off); }
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
__device__ static int64_t base_head_index(DocShared& s, uint32_t h) {
  if (s.dh.has_hidx) {
    Rd r{s.A + s.dh.base + s.dh.hidx_off, (uint64_t)1 << 40, 0};
    int64_t v = -1;
    for (uint32_t i = 0; i <= h; i++) rd_u53(r, v);
    return v;
  }
  return s.dh.nheads == 1 ? (int64_t)s.nbc - 1 : -1;
}

// ---- P2a: lane-parallel lookups -- hashes, duplicates, canonical actors, dependency refs ----
// Canonical actor ids: base actors 0..NB-1, the author of change j (first occurrence) NB + j.
// Dependency refs: >= 0 change index (first occurrence of that hash in the list),
// <= -10: base head (-10 - h), -2: host-known hash, -1: missing.
__device__ static void plan_lookups(DocShared& s, const am_doc_desc& dd, const ChunkInfo* info, const am_known_hash* known) {
  const WsLayout& L = s.L;
  const uint32_t N = dd.chg_count, t = threadIdx.x, T = blockDim.x;
  const ChgHdr* ch = hp<ChgHdr>(s, L.chghdr);
  uint8_t* hashes = hp<uint8_t>(s, L.hashes);
  const uint8_t* A = s.A;
  const uint32_t NB = s.has_base ? s.dh.nactors : 0;
  for (uint32_t c = t; c < N; c += T) {
    const uint32_t* src = reinterpret_cast<const uint32_t*>(info[dd.chg_begin + c].hash);
    uint32_t* dst = reinterpret_cast<uint32_t*>(hashes + 32 * c);
    for (int k = 0; k < 8; k++) dst[k] = src[k];
  }
  __syncthreads();
  uint32_t* dup_of = hp<uint32_t>(s, L.dup_of);
  int64_t* self_idx = hp<int64_t>(s, L.self_idx);
  int32_t* aut = hp<int32_t>(s, L.aut);
  int32_t* can = hp<int32_t>(s, L.can);
  int32_t* dref = hp<int32_t>(s, L.dref);
  int64_t* dref_idx = hp<int64_t>(s, L.dref_idx);
  const uint32_t* ambase = hp<uint32_t>(s, L.ambase);
  const uint32_t* dbase = hp<uint32_t>(s, L.dbase);
  auto base_actor = [&](uint64_t off, uint32_t len) -> int32_t {
    if (!s.has_base) return -1;
    Rd r{A + s.dh.base + s.dh.actors_off, (uint64_t)1 << 40, 0};
    for (uint32_t i = 0; i < s.dh.nactors; i++) {
      int64_t l;
      rd_u53(r, l);
      if ((uint32_t)l == len && bytes_eq(r.p + r.off, A + off, len)) return (int32_t)i;
      r.off += (uint64_t)l;
    }
    return -1;
  };
  auto author_canon = [&](uint64_t off, uint32_t len, uint32_t upto) -> int32_t {
    int32_t a = base_actor(off, len);
    if (a >= 0) return a;
    for (uint32_t j = 0; j < upto; j++) {
      const ChgHdr& hj = ch[j];
      if (hj.actor_len == len && bytes_eq(A + hj.base + hj.actor_off, A + off, len)) return (int32_t)(NB + j);
    }
    return -1;
  };
  auto match_base = [&](const uint8_t* h, int32_t& ref, int64_t& idx) -> bool {
    if (s.has_base)
      for (uint32_t k = 0; k < s.dh.nheads; k++)
        if (hash_eq(A + s.dh.base + s.dh.heads_off + 32 * k, h)) { ref = -10 - (int32_t)k; idx = base_head_index(s, k); return true; }
    for (uint32_t k = 0; k < dd.known_count; k++)
      if (hash_eq(known[dd.known_begin + k].hash, h)) { ref = -2; idx = known[dd.known_begin + k].index; return true; }
    return false;
  };
  for (uint32_t c = t; c < N; c += T) {
    const ChgHdr& h = ch[c];
    const uint8_t* hc = hashes + 32 * c;
    uint32_t d = c;
    for (uint32_t j = 0; j < c; j++) if (hash_eq(hashes + 32 * j, hc)) { d = j; break; }
    dup_of[c] = d;
    int32_t ref;
    int64_t idx;
    self_idx[c] = match_base(hc, ref, idx) ? idx : (int64_t)-2;
    aut[c] = author_canon(h.base + h.actor_off, h.actor_len, c + 1);
    uint32_t am = ambase[c];
    can[am] = aut[c];
    Rd ar{A + h.base + h.actors_off, (uint64_t)1 << 40, 0};
    for (uint32_t k = 1; k < h.nactors; k++) {
      int64_t l;
      rd_u53(ar, l);
      can[am + k] = author_canon(h.base + h.actors_off + ar.off, (uint32_t)l, N);
      ar.off += (uint64_t)l;
    }
    for (uint32_t di = 0; di < h.ndeps; di++) {
      const uint8_t* dep = A + h.base + h.deps_off + 32 * di;
      int32_t r = -1;
      int64_t x = 0;
      if (!match_base(dep, r, x)) {
        for (uint32_t j = 0; j < N; j++) if (hash_eq(hashes + 32 * j, dep)) { r = (int32_t)j; break; }
      }
      dref[dbase[c] + di] = r;
      dref_idx[dbase[c] + di] = x;
    }
  }
}

// ---- P2b: causal queue, clock, actor table, heads (one lane; integer work only) ----
__device__ static void plan_doc(DocShared& s, const am_doc_desc& dd, const ChunkInfo* info, int32_t* chg_state) {
  const WsLayout& L = s.L;
  const uint8_t* A = s.A;
  ActorRef* actors = hp<ActorRef>(s, L.actors);
  int64_t* clock = hp<int64_t>(s, L.clock);
  int32_t* docpos = hp<int32_t>(s, L.docpos);
  uint8_t* heads = hp<uint8_t>(s, L.heads);
  int32_t* head_ref = hp<int32_t>(s, L.head_ref);
  ChgRow* chg = hp<ChgRow>(s, L.chg);
  int64_t* deps = hp<int64_t>(s, L.deps);
  const ChgHdr* ch = hp<ChgHdr>(s, L.chghdr);
  uint32_t* order = hp<uint32_t>(s, L.order);
  uint32_t* rowbase = hp<uint32_t>(s, L.rowbase);
  uint32_t* entbase = hp<uint32_t>(s, L.entbase);
  uint32_t* ambase_out = hp<uint32_t>(s, L.amb_out);  // per applied change, its amap base
  uint32_t* amap = hp<uint32_t>(s, L.amap);
  uint32_t* queue = hp<uint32_t>(s, L.queue);
  const uint8_t* hashes = hp<uint8_t>(s, L.hashes);
  const uint32_t* dup_of = hp<uint32_t>(s, L.dup_of);
  const int64_t* self_idx = hp<int64_t>(s, L.self_idx);
  const int32_t* aut = hp<int32_t>(s, L.aut);
  const int32_t* can = hp<int32_t>(s, L.can);
  const int32_t* dref = hp<int32_t>(s, L.dref);
  const int64_t* dref_idx = hp<int64_t>(s, L.dref_idx);
  const uint32_t* ambase = hp<uint32_t>(s, L.ambase);
  const uint32_t* dbase = hp<uint32_t>(s, L.dbase);
  int32_t* applied = hp<int32_t>(s, L.applied);  // applied index per change (first occurrence of its hash)
  const uint32_t N = dd.chg_count;
  const uint32_t NB = s.has_base ? s.dh.nactors : 0;

  // base actors + clock (readDocumentChanges, new.js:1645-1675)
  uint32_t na = 0;
  if (s.has_base) {
    Rd r{A + s.dh.base + s.dh.actors_off, (uint64_t)1 << 40, 0};
    for (uint32_t i = 0; i < NB; i++) {
      int64_t l;
      rd_u53(r, l);
      actors[na].off = s.dh.base + s.dh.actors_off + r.off;
      actors[na].len = (uint32_t)l;
      r.off += (uint64_t)l;
      docpos[na] = (int32_t)na;
      na++;
    }
  }
  for (uint32_t i = 0; i < NB + N; i++) clock[i] = 0;
  for (uint32_t j = 0; j < N; j++) { docpos[NB + j] = -1; applied[j] = -1; }
  for (uint32_t i = 0; i < s.nbc; i++) {
    int64_t a = chg[i].actor, seq = chg[i].seq;
    if (a == AM_NULL64 || a < 0 || a >= (int64_t)NB || seq == AM_NULL64) { set_err(s, AM_U_VALUE); return; }
    if (seq != 1 && seq != clock[a] + 1) {
      set_err(s, AM_E_DOC_SEQ, clock[a] == 0 ? AM_NULL64 : clock[a] + 1, seq, actors[a].off, actors[a].len);
      return;
    }
    clock[a] = seq;
  }
  uint32_t nheads = 0;
  if (s.has_base)
    for (uint32_t h = 0; h < s.dh.nheads; h++) head_ref[nheads++] = -10 - (int32_t)h;

  const bool have_graph = (dd.flags & 1) != 0;
  uint32_t nq = N;
  for (uint32_t i = 0; i < nq; i++) { queue[i] = i; chg_state[dd.chg_begin + i] = CHG_UNSEEN; }
  uint32_t nall = 0, nrow = s.nb, nent = s.nbe, nam = 0, ndep = s.nbd;
  int64_t max_op = 0;
  for (;;) {
    // one pass of applyChanges() (new.js:1550-1597)
    uint32_t ne = 0, na_pass = 0;
    for (uint32_t qi = 0; qi < nq; qi++) {
      const uint32_t c = queue[qi];
      const ChunkInfo& ci = info[dd.chg_begin + c];
      const ChgHdr& h = ch[c];
      const uint32_t j0 = dup_of[c];
      if (self_idx[c] != -2 || applied[j0] >= 0) { chg_state[dd.chg_begin + c] = CHG_DUP; continue; }
      bool ready = true;
      for (uint32_t di = 0; di < h.ndeps && ready; di++) {
        int32_t r = dref[dbase[c] + di];
        if (r >= 0) ready = applied[r] >= 0;
        else if (r == -1) ready = false;
        else ready = dref_idx[dbase[c] + di] != -1;
      }
      if (!ready) { queue[ne++] = c; continue; }
      const int32_t a = aut[c];
      const int64_t expected = clock[a] + 1;
      if (h.seq < expected) {
        if (have_graph) { set_err(s, AM_E_REUSE_SEQ, h.seq, 0, h.base + h.actor_off, h.actor_len, c); return; }
        set_err(s, AM_U_HASH_GRAPH);
        return;
      }
      if (h.seq > expected) { set_err(s, AM_E_SKIPPED_SEQ, expected, 0, h.base + h.actor_off, h.actor_len, c); return; }
      clock[a] = h.seq;
      if (docpos[a] < 0) {  // getActorTable appends a new author (new.js:1435-1441)
        docpos[a] = (int32_t)na;
        actors[na].off = h.base + h.actor_off;
        actors[na].len = h.actor_len;
        na++;
      }
      // actor table of the change's columns (getActorTable, new.js:1442-1450)
      ambase_out[nall] = nam;
      Rd ar{A + h.base + h.actors_off, (uint64_t)1 << 40, 0};
      for (uint32_t k = 0; k < h.nactors; k++) {
        int32_t x = can[ambase[c] + k];
        uint64_t aoff = h.base + h.actor_off;
        uint32_t alen = h.actor_len;
        if (k > 0) {
          int64_t l;
          rd_u53(ar, l);
          aoff = h.base + h.actors_off + ar.off;
          alen = (uint32_t)l;
          ar.off += (uint64_t)l;
        }
        if (x < 0 || docpos[x] < 0) { set_err(s, AM_E_UNKNOWN_ACTOR, 0, 0, aoff, alen, c); return; }
        amap[nam++] = (uint32_t)docpos[x];
      }
      // heads: drop the dependencies, add this change (new.js:1581-1583)
      for (uint32_t di = 0; di < h.ndeps; di++) {
        int32_t r = dref[dbase[c] + di];
        for (uint32_t q = 0; q < nheads; q++)
          if (head_ref[q] == r && r != -1 && r != -2) { head_ref[q] = head_ref[--nheads]; break; }
      }
      bool present = false;
      for (uint32_t q = 0; q < nheads; q++) present |= head_ref[q] == (int32_t)j0;
      if (!present) head_ref[nheads++] = (int32_t)j0;
      applied[j0] = (int32_t)nall;
      order[nall] = c;
      rowbase[nall] = nrow;
      entbase[nall] = nent;
      nrow += ci.nops;
      nent += ci.nents;
      // appendChange row (new.js:1680-1692)
      ChgRow& cr = chg[s.nbc + nall];
      cr.actor = docpos[a];
      cr.seq = h.seq;
      cr.max_op = h.start_op + (int64_t)ci.nops - 1;
      cr.time = h.time;
      cr.msg_off = h.base + h.msg_off;
      cr.msg_len = h.msg_len;
      cr.ndeps = h.ndeps;
      cr.deps_off = ndep;
      ndep += h.ndeps;
      cr.extra_len = h.has_extra ? (int64_t)(((uint64_t)h.extra_len << 4) | 7) : 7;
      cr.extra_off = h.base + h.extra_off;
      cr.extra_raw_len = h.has_extra ? h.extra_len : 0;
      if (ci.nops > 0 && cr.max_op > max_op) max_op = cr.max_op;
      chg_state[dd.chg_begin + c] = (int32_t)nall;
      nall++;
      na_pass++;
    }
    nq = ne;
    if (nq == 0) break;
    if (na_pass == 0) {
      if (have_graph) break;
      set_err(s, AM_U_HASH_GRAPH);  // BackendDoc.applyChanges would computeHashGraph() (new.js:1830)
      return;
    }
  }
  for (uint32_t i = 0; i < nq; i++) chg_state[dd.chg_begin + queue[i]] = CHG_QUEUED;
  // deps indexes of the appended change rows: changeIndexByHash[dep]
  for (uint32_t k = 0; k < nall; k++) {
    const uint32_t c = order[k];
    const ChgHdr& h = ch[c];
    ChgRow& cr = chg[s.nbc + k];
    for (uint32_t di = 0; di < h.ndeps; di++) {
      int32_t r = dref[dbase[c] + di];
      deps[cr.deps_off + di] = r >= 0 ? (int64_t)(s.nbc + applied[r]) : dref_idx[dbase[c] + di];
    }
  }
  // heads (sorted, new.js:1593) with their headsIndexes
  int64_t* hidx = hp<int64_t>(s, L.hidx);
  for (uint32_t q = 0; q < nheads; q++) {
    int32_t r = head_ref[q];
    const uint8_t* src = r >= 0 ? hashes + 32 * r : A + s.dh.base + s.dh.heads_off + 32 * (uint32_t)(-10 - r);
    for (int k = 0; k < 32; k++) heads[32 * q + k] = src[k];
    hidx[q] = r >= 0 ? (int64_t)(s.nbc + applied[r]) : base_head_index(s, (uint32_t)(-10 - r));
  }
  for (uint32_t a2 = 1; a2 < nheads; a2++)
    for (uint32_t b2 = a2; b2 > 0 && hash_cmp(heads + 32 * (b2 - 1), heads + 32 * b2) > 0; b2--) {
      for (int k = 0; k < 32; k++) { uint8_t tt = heads[32 * b2 + k]; heads[32 * b2 + k] = heads[32 * (b2 - 1) + k]; heads[32 * (b2 - 1) + k] = tt; }
      int64_t ti = hidx[b2]; hidx[b2] = hidx[b2 - 1]; hidx[b2 - 1] = ti;
    }
  if (nall > 0 || nq > 0)
    for (uint32_t q = 0; q < nheads; q++)
      if (hidx[q] < 0) { set_err(s, AM_U_HASH_GRAPH); return; }
  s.napplied = nall;
  s.nqueued = nq;
  s.nactors = na;
  s.nheads = nheads;
  s.nrows = nrow;
  s.nents = nent;
  s.nchg = s.nbc + nall;
  s.ndeps = ndep;
  s.max_op = max_op;
}

// ---- P4: column decode into rows; one (source, column) stream per lane ----
__device__ static void decode_item(DocShared& s, uint32_t item) {
  const WsLayout& L = s.L;
  const uint8_t* A = s.A;
  Row* rows = hp<Row>(s, L.rows);
  Ent* ents = hp<Ent>(s, L.ents);
  const uint32_t col = item % OC_NCOLS;
  const uint32_t src = item / OC_NCOLS;  // 0 = base (if any), then applied changes
  uint64_t off, roff = 0, rlen = 0;
  uint32_t len, nrows, nents, row0, ent0;
  const uint32_t* map = nullptr;
  uint32_t nmap = 0;
  bool is_change;
  int64_t start_op = 0;
  uint32_t self = 0, chg_local = 0xffffffffu;
  if (s.has_base && src == 0) {
    off = s.dh.base + s.dh.ocol_off[col];
    len = s.dh.ocol_len[col];
    roff = s.dh.base + s.dh.ocol_off[OC_VAL_RAW];
    rlen = s.dh.ocol_len[OC_VAL_RAW];
    nrows = s.nb; nents = s.nbe; row0 = 0; ent0 = 0;
    is_change = false;
  } else {
    const uint32_t k = src - (s.has_base ? 1 : 0);
    const uint32_t c = hp<uint32_t>(s, L.order)[k];
    const ChgHdr& h = hp<ChgHdr>(s, L.chghdr)[c];
    off = h.base + h.col_off[col];
    len = h.col_len[col];
    roff = h.base + h.col_off[OC_VAL_RAW];
    rlen = h.col_len[OC_VAL_RAW];
    row0 = hp<uint32_t>(s, L.rowbase)[k];
    ent0 = hp<uint32_t>(s, L.entbase)[k];
    uint32_t nextrow = (k + 1 < s.napplied) ? hp<uint32_t>(s, L.rowbase)[k + 1] : s.nrows;
    uint32_t nextent = (k + 1 < s.napplied) ? hp<uint32_t>(s, L.entbase)[k + 1] : s.nents;
    nrows = nextrow - row0;
    nents = nextent - ent0;
    map = hp<uint32_t>(s, L.amap) + hp<uint32_t>(s, L.amb_out)[k];
    nmap = h.nactors;
    self = map[0];
    start_op = h.start_op;
    is_change = true;
    chg_local = c;
  }
  ColDec d;
  uint32_t e = AM_OK;
  auto mapact = [&](int64_t v, int32_t& outv) -> uint32_t {
    if (v == AM_NULL64) { outv = -1; return AM_OK; }
    if (is_change) {
      if (v < 0 || v >= (int64_t)nmap) { set_err(s, AM_E_NO_ACTOR_INDEX, v, 0, 0, 0, chg_local); return AM_E_NO_ACTOR_INDEX; }
      outv = (int32_t)map[v];
    } else {
      if (v < 0 || v >= (int64_t)s.nactors) { set_err(s, AM_U_VALUE); return AM_U_VALUE; }
      outv = (int32_t)v;
    }
    return AM_OK;
  };
  switch (col) {
    case OC_OBJ_ACTOR: case OC_KEY_ACTOR: case OC_CHLD_ACTOR: {
      cd_init(d, DT_UINT, A + off, len);
      for (uint32_t i = 0; i < nrows; i++) {
        int64_t v;
        if ((e = cd_next_int(d, v))) break;
        int32_t a;
        if (mapact(v, a)) return;
        Row& r = rows[row0 + i];
        if (col == OC_OBJ_ACTOR) r.obj_actor = a; else if (col == OC_KEY_ACTOR) r.key_actor = a; else r.chld_actor = a;
      }
      break;
    }
    case OC_OBJ_CTR: case OC_KEY_CTR: case OC_CHLD_CTR: {
      cd_init(d, col == OC_OBJ_CTR ? DT_UINT : DT_INT, A + off, len);
      for (uint32_t i = 0; i < nrows; i++) {
        int64_t v;
        if ((e = (col == OC_OBJ_CTR) ? cd_next_int(d, v) : cd_next_delta(d, v))) break;
        Row& r = rows[row0 + i];
        if (col == OC_OBJ_CTR) r.obj_ctr = v; else if (col == OC_KEY_CTR) r.key_ctr = v; else r.chld_ctr = v;
      }
      break;
    }
    case OC_KEY_STR: {
      cd_init(d, DT_UTF8, A + off, len);
      for (uint32_t i = 0; i < nrows; i++) {
        uint64_t so;
        uint32_t sl;
        if ((e = cd_next_str(d, so, sl))) break;
        Row& r = rows[row0 + i];
        r.key_len = sl;
        r.key_off = (sl == AM_NOSTR) ? 0 : off + so;
        if (sl != AM_NOSTR && !utf8_valid_dev(A + off + so, sl)) { set_err(s, AM_U_UTF8); return; }
      }
      break;
    }
    case OC_ID_ACTOR: case OC_ID_CTR: {
      if (is_change) break;  // change ops get ids from the change header (new.js:708-709)
      cd_init(d, col == OC_ID_ACTOR ? DT_UINT : DT_INT, A + off, len);
      for (uint32_t i = 0; i < nrows; i++) {
        int64_t v;
        if (col == OC_ID_ACTOR) {
          if ((e = cd_next_int(d, v))) break;
          int32_t a;
          if (mapact(v, a)) return;
          rows[row0 + i].id_actor = a;
        } else {
          if ((e = cd_next_delta(d, v))) break;
          rows[row0 + i].id_ctr = v;
        }
      }
      break;
    }
    case OC_INSERT: {
      cd_init(d, DT_BOOL, A + off, len);
      for (uint32_t i = 0; i < nrows; i++) {
        bool v;
        if ((e = cd_next_bool(d, v))) break;
        rows[row0 + i].insert = v;
      }
      break;
    }
    case OC_ACTION: {
      cd_init(d, DT_UINT, A + off, len);
      for (uint32_t i = 0; i < nrows; i++) {
        int64_t v;
        if ((e = cd_next_int(d, v))) break;
        Row& r = rows[row0 + i];
        r.action = v;
        r.src_change = is_change;
        r.is_del = is_change && v == 3;
        if (is_change) { r.id_actor = (int32_t)self; r.id_ctr = start_op + i; }
      }
      break;
    }
    case OC_VAL_LEN: {
      // readOperation: VALUE_RAW reads valLen >>> 4 bytes (new.js:573-575, 601-604)
      cd_init(d, DT_UINT, A + off, len);
      uint64_t acc = 0;
      for (uint32_t i = 0; i < nrows; i++) {
        int64_t v;
        if ((e = cd_next_int(d, v))) break;
        Row& r = rows[row0 + i];
        r.val_len = v;
        uint64_t nb = (v == AM_NULL64) ? 0 : ((uint64_t)v >> 4);
        if (acc + nb > rlen) { e = AM_E_SUBARRAY; break; }
        r.val_off = roff + acc;
        acc += nb;
      }
      break;
    }
    case OC_VAL_RAW: break;
    case OC_GRP_NUM: {
      cd_init(d, DT_UINT, A + off, len);
      uint32_t acc = 0;
      for (uint32_t i = 0; i < nrows; i++) {
        int64_t v;
        if ((e = cd_next_int(d, v))) break;
        Row& r = rows[row0 + i];
        uint32_t cnt = (v == AM_NULL64) ? 0 : (uint32_t)v;
        r.ps_cnt = cnt;
        r.ps_off = ent0 + acc;
        acc += cnt;
      }
      if (!e && acc != nents) e = AM_U_VALUE;
      break;
    }
    case OC_GRP_ACTOR: case OC_GRP_CTR: {
      cd_init(d, col == OC_GRP_ACTOR ? DT_UINT : DT_INT, A + off, len);
      for (uint32_t j = 0; j < nents; j++) {
        int64_t v;
        if (col == OC_GRP_ACTOR) {
          if ((e = cd_next_int(d, v))) break;
          if (v == AM_NULL64) { set_err(s, AM_U_VALUE); return; }
          int32_t a;
          if (mapact(v, a)) return;
          ents[ent0 + j].actor = a;
        } else {
          if ((e = cd_next_delta(d, v))) break;
          if (v == AM_NULL64) { set_err(s, AM_U_VALUE); return; }
          ents[ent0 + j].ctr = v;
        }
        ents[ent0 + j].row = -1;
      }
      break;
    }
  }
  if (e) set_err(s, e, 0, 0, 0, 0, chg_local);
}

// base document change rows (DOCUMENT_COLUMNS), one column per lane
__device__ static void decode_base_chg_col(DocShared& s, uint32_t col) {
  ChgRow* chg = hp<ChgRow>(s, s.L.chg);
  int64_t* deps = hp<int64_t>(s, s.L.deps);
  const uint8_t* A = s.A;
  const uint64_t off = s.dh.base + s.dh.ccol_off[col];
  const uint32_t len = s.dh.ccol_len[col];
  const uint32_t n = s.nbc;
  ColDec d;
  uint32_t e = AM_OK;
  switch (col) {
    case DC_ACTOR: case DC_SEQ: case DC_MAXOP: case DC_TIME: case DC_EXTRA_LEN: {
      cd_init(d, (col == DC_ACTOR || col == DC_EXTRA_LEN) ? DT_UINT : DT_INT, A + off, len);
      uint64_t acc = 0;
      for (uint32_t i = 0; i < n; i++) {
        int64_t v;
        if ((e = (col == DC_ACTOR || col == DC_EXTRA_LEN) ? cd_next_int(d, v) : cd_next_delta(d, v))) break;
        ChgRow& r = chg[i];
        if (col == DC_ACTOR) r.actor = v;
        else if (col == DC_SEQ) r.seq = v;
        else if (col == DC_MAXOP) r.max_op = v;
        else if (col == DC_TIME) r.time = v;
        else {
          r.extra_len = v;
          uint64_t nb = (v == AM_NULL64) ? 0 : ((uint64_t)v >> 4);
          if (acc + nb > s.dh.ccol_len[DC_EXTRA_RAW]) { e = AM_E_SUBARRAY; break; }
          r.extra_off = s.dh.base + s.dh.ccol_off[DC_EXTRA_RAW] + acc;
          r.extra_raw_len = (uint32_t)nb;
          acc += nb;
        }
      }
      break;
    }
    case DC_MESSAGE: {
      cd_init(d, DT_UTF8, A + off, len);
      for (uint32_t i = 0; i < n; i++) {
        uint64_t so;
        uint32_t sl;
        if ((e = cd_next_str(d, so, sl))) break;
        chg[i].msg_len = sl;
        chg[i].msg_off = sl == AM_NOSTR ? 0 : off + so;
        if (sl != AM_NOSTR && !utf8_valid_dev(A + off + so, sl)) { set_err(s, AM_U_UTF8); return; }
      }
      break;
    }
    case DC_DEPS_NUM: {
      cd_init(d, DT_UINT, A + off, len);
      uint32_t acc = 0;
      for (uint32_t i = 0; i < n; i++) {
        int64_t v;
        if ((e = cd_next_int(d, v))) break;
        uint32_t c = v == AM_NULL64 ? 0 : (uint32_t)v;
        chg[i].ndeps = c;
        chg[i].deps_off = acc;
        acc += c;
      }
      break;
    }
    case DC_DEPS_INDEX: {
      cd_init(d, DT_INT, A + off, len);
      for (uint32_t j = 0; j < s.nbd; j++) {
        int64_t v;
        if ((e = cd_next_delta(d, v))) break;
        deps[j] = v;
      }
      break;
    }
    default: break;
  }
  if (e) set_err(s, e);
}

// ---- sequential canonical encoders (RLEEncoder/DeltaEncoder/BooleanEncoder, encoding.js:558-1135).
// Maximal runs; runs >= 2 -> repetition record; adjacent single values -> one literal record;
// null runs -> null record; an all-null column encodes to nothing. ----
template <typename Get>
__device__ static uint8_t* enc_rle_int(uint8_t* o, uint32_t n, Get get, bool sgn) {
  bool any = false;
  for (uint32_t i = 0; i < n && !any; i++) any = get(i) != AM_NULL64;
  if (!any) return o;
  uint32_t i = 0;
  int64_t vi = n ? get(0) : 0;
  while (i < n) {
    uint32_t j = i + 1;
    int64_t vj = 0;
    while (j < n && (vj = get(j)) == vi) j++;
    uint32_t run = j - i;
    if (vi == AM_NULL64) {
      o = put_sleb(o, 0);
      o = put_uleb(o, run);
    } else if (run >= 2) {
      o = put_sleb(o, (int64_t)run);
      o = sgn ? put_sleb(o, vi) : put_uleb(o, (uint64_t)vi);
    } else {
      // literal: consecutive single values until a repeat or a null
      uint32_t k = i;
      int64_t vk = vi;
      while (k < n) {
        if (vk == AM_NULL64) break;
        int64_t vn = (k + 1 < n) ? get(k + 1) : AM_NULL64;
        if (k + 1 < n && vn == vk) break;
        k++;
        vk = vn;
      }
      o = put_sleb(o, -(int64_t)(k - i));
      for (uint32_t t = i; t < k; t++) {
        int64_t v = get(t);
        o = sgn ? put_sleb(o, v) : put_uleb(o, (uint64_t)v);
      }
      j = k;
    }
    i = j;
    if (i < n) vi = get(i);
  }
  return o;
}
template <typename GetS>
__device__ static uint8_t* enc_rle_str(uint8_t* o, uint32_t n, const uint8_t* arena, GetS get) {
  // get(i, off, len): len == AM_NOSTR -> null
  bool any = false;
  for (uint32_t i = 0; i < n && !any; i++) { uint64_t so; uint32_t sl; get(i, so, sl); any = sl != AM_NOSTR; }
  if (!any) return o;
  auto eq = [&](uint64_t ao, uint32_t al, uint64_t bo, uint32_t bl) {
    if (al != bl) return false;
    if (al == AM_NOSTR) return true;
    return bytes_eq(arena + ao, arena + bo, al);
  };
  uint32_t i = 0;
  while (i < n) {
    uint64_t io; uint32_t il;
    get(i, io, il);
    uint32_t j = i + 1;
    for (; j < n; j++) { uint64_t jo; uint32_t jl; get(j, jo, jl); if (!eq(jo, jl, io, il)) break; }
    uint32_t run = j - i;
    if (il == AM_NOSTR) {
      o = put_sleb(o, 0);
      o = put_uleb(o, run);
    } else if (run >= 2) {
      o = put_sleb(o, (int64_t)run);
      o = put_uleb(o, il);
      for (uint32_t t = 0; t < il; t++) *o++ = arena[io + t];
    } else {
      uint32_t k = i;
      for (;;) {
        uint64_t ko; uint32_t kl;
        get(k, ko, kl);
        if (kl == AM_NOSTR) break;
        if (k + 1 < n) { uint64_t no; uint32_t nl; get(k + 1, no, nl); if (eq(no, nl, ko, kl)) break; }
        k++;
        if (k >= n) break;
      }
      o = put_sleb(o, -(int64_t)(k - i));
      for (uint32_t t = i; t < k; t++) {
        uint64_t to; uint32_t tl;
        get(t, to, tl);
        o = put_uleb(o, tl);
        for (uint32_t q = 0; q < tl; q++) *o++ = arena[to + q];
      }
      j = k;
    }
    i = j;
  }
  return o;
}
// Delta: materialised differences (nulls keep the running value), then signed RLE.
template <typename Get>
__device__ static uint8_t* enc_delta(uint8_t* o, uint32_t n, Get get, int64_t* scratch) {
  int64_t abs = 0;
  for (uint32_t i = 0; i < n; i++) {
    int64_t v = get(i);
    if (v == AM_NULL64) scratch[i] = AM_NULL64;
    else { scratch[i] = v - abs; abs = v; }
  }
  return enc_rle_int(o, n, [&](uint32_t i) { return scratch[i]; }, true);
}
template <typename GetB>
__device__ static uint8_t* enc_bool(uint8_t* o, uint32_t n, GetB get) {
  bool last = false;
  uint64_t count = 0;
  for (uint32_t i = 0; i < n; i++) {
    bool v = get(i);
    if (v == last) count++;
    else { o = put_uleb(o, count); last = v; count = 1; }
  }
  if (count > 0) o = put_uleb(o, count);
  return o;
}

__device__ __forceinline__ bool same_obj(const Row& a, const Row& b) {
  return a.obj_ctr == b.obj_ctr && a.obj_actor == b.obj_actor;
}

// binary search of (ctr, actor) in the id index; returns row or -1
__device__ static int32_t id_lookup(const IdKey* idk, uint32_t n, int64_t ctr, int32_t actor) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    uint32_t mid = (lo + hi) >> 1;
    const IdKey& k = idk[mid];
    if (k.ctr < ctr || (k.ctr == ctr && k.actor < actor)) lo = mid + 1; else hi = mid;
  }
  if (lo < n && idk[lo].ctr == ctr && idk[lo].actor == actor) return idk[lo].row;
  return -1;
}


__global__ void __launch_bounds__(DOC_T) k_doc(const uint8_t* __restrict__ arena, const am_chunk_desc* __restrict__ chunks,
                                               const am_doc_desc* __restrict__ docs, const am_known_hash* __restrict__ known,
                                               const ChunkInfo* __restrict__ info, const DocBounds* __restrict__ bounds,
                                               const uint64_t* __restrict__ ws_off, uint8_t* __restrict__ ws_base,
                                               uint64_t ws_cap, uint32_t lds_bytes, am_doc_result* __restrict__ results,
                                               int32_t* __restrict__ chg_state) {
  __shared__ DocShared s;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const uint32_t doc = blockIdx.x, t = threadIdx.x, T = blockDim.x;
  const am_doc_desc dd = docs[doc];
  if (t == 0) {
    s.b = bounds[doc];
    s.ws = ws_base + ws_off[doc];
    s.L = ws_layout(s.b);
    // hot working set in LDS when it fits, else in the document's global workspace
    s.hot = (s.L.hot_total <= lds_bytes) ? lds : s.ws;
    s.status = AM_OK; s.errchg = 0xffffffffu; s.arg0 = s.arg1 = 0; s.arg_actor_off = 0; s.arg_actor_len = 0;
    s.has_base = dd.base_chunk >= 0;
    s.nb = s.nbe = s.nbc = s.nbd = 0;
    s.napplied = s.nqueued = s.nactors = s.nheads = 0;
    s.nrows = s.nents = s.nchg = s.ndeps = s.nout = s.nnew = 0;
    s.max_op = 0;
    s.out_len = 0;
    if (ws_off[doc] + s.L.total > ws_cap) set_err(s, AM_U_CAPACITY);
    // chunk-level errors: the base document first (load), then changes in order (new.js:1798)
    if (s.has_base) {
      const ChunkInfo& ci = info[dd.base_chunk];
      if (ci.status) set_err(s, ci.status, ci.arg0);
      else if (ci.type != 0) set_err(s, AM_E_CHUNK_TYPE, ci.type);
      else { s.nb = ci.nops; s.nbe = ci.nents; s.nbc = ci.nchg; s.nbd = ci.ndeps; }
    }
    for (uint32_t k = 0; k < dd.chg_count && s.status == AM_OK; k++) {
      const ChunkInfo& ci = info[dd.chg_begin + k];
      if (ci.status) set_err(s, ci.status, ci.arg0, 0, 0, 0, k);
      else if (ci.type != 1) set_err(s, AM_E_CHUNK_TYPE, ci.type, 0, 0, 0, k);
    }
    if (s.b.R == 0 && s.b.N == 0 && !s.has_base && dd.chg_count) set_err(s, AM_U_CAPACITY);
  }
  __syncthreads();
  const WsLayout& L = s.L;
  if (s.status) goto done;
  // P0: stage the document's input bytes (base + changes, adjacent in the arena) into the hot
  // region with 16-byte coalesced loads; every later parse/decode reads them from there.
  {
    const uint64_t lo = s.b.span_lo, n = s.b.span_hi - s.b.span_lo;
    uint8_t* dst = s.hot + L.input;
    if (n) {
      const uint64_t head = (16 - (lo & 15)) & 15;  // bytes before the first 16-aligned source address
      for (uint64_t q = t; q < head && q < n; q += T) dst[q] = arena[lo + q];
      if (n > head) {
        const uint64_t nv = (n - head) / 16;
        // destination alignment follows the source phase: copy via 4-byte words when possible
        for (uint64_t v = t; v < nv; v += T) {
          const uint4 x = *reinterpret_cast<const uint4*>(arena + lo + head + 16 * v);
          uint8_t* o = dst + head + 16 * v;
          const uint8_t* xb = reinterpret_cast<const uint8_t*>(&x);
          for (int k = 0; k < 16; k++) o[k] = xb[k];
        }
        for (uint64_t q = head + 16 * nv + t; q < n; q += T) dst[q] = arena[lo + q];
      }
      if (t == 0) s.A = reinterpret_cast<const uint8_t*>(reinterpret_cast<uintptr_t>(dst) - lo);
    } else if (t == 0) {
      s.A = arena;
    }
  }
  __syncthreads();
  // P1: base document header, change headers (lane per change), base change rows (lane per column)
  if (t == 0 && s.has_base) {
    const ChunkInfo& ci = info[dd.base_chunk];
    const am_chunk_desc cd = chunks[dd.base_chunk];
    parse_doc_hdr(s.A + cd.off + ci.data_off, ci.data_len, cd.off + ci.data_off, s.dh);
  }
  if (t == 0 && !s.has_base) { s.dh.nactors = 0; s.dh.nheads = 0; s.dh.has_hidx = 0; s.dh.extra_len = 0; s.dh.base = 0; }
  for (uint32_t k = t; k < dd.chg_count; k += T) {
    const ChunkInfo& ci = info[dd.chg_begin + k];
    const am_chunk_desc cd = chunks[dd.chg_begin + k];
    ChgHdr& h = hp<ChgHdr>(s, L.chghdr)[k];
    parse_change_hdr(s.A + cd.off + ci.data_off, ci.data_len, cd.off + ci.data_off, h);
  }
  if (t == 0) {  // prefix offsets of the change actor lists and deps
    uint32_t am = 0, db = 0;
    for (uint32_t k = 0; k < dd.chg_count; k++) {
      hp<uint32_t>(s, L.ambase)[k] = am;
      hp<uint32_t>(s, L.dbase)[k] = db;
      am += info[dd.chg_begin + k].nactors;
      db += info[dd.chg_begin + k].ndeps;
    }
  }
  __syncthreads();
  if (s.has_base)
    for (uint32_t c = t; c < DC_NCOLS; c += T) decode_base_chg_col(s, c);
#if defined(AM_STOP_PHASE) && AM_STOP_PHASE == 1
  goto done;
#endif
  // P2: plan -- lane-parallel lookups, then the sequential causal queue on integers
  plan_lookups(s, dd, info, known);
  __syncthreads();
  if (s.status) goto done;
  if (t == 0) plan_doc(s, dd, info, chg_state);
  __syncthreads();
  if (s.status) goto done;
  {
    const uint8_t* A = s.A;
    Row* rows = hp<Row>(s, L.rows);
    Ent* ents = hp<Ent>(s, L.ents);
    ActorRef* actors = hp<ActorRef>(s, L.actors);
    const uint32_t R = s.nrows;
    // P4: decode rows
    for (uint32_t i = t; i < R; i += T) {
      Row& r = rows[i];
      r.obj_ctr = r.key_ctr = r.id_ctr = r.chld_ctr = r.action = r.val_len = AM_NULL64;
      r.obj_actor = r.key_actor = r.id_actor = r.chld_actor = -1;
      r.key_len = AM_NOSTR; r.key_off = 0; r.val_off = 0; r.ps_off = 0; r.ps_cnt = 0;
      r.insert = 0; r.is_del = 0; r.src_change = 0; r.flags = 0;
    }
    __syncthreads();
#if defined(AM_STOP_PHASE) && AM_STOP_PHASE == 2
    goto done;
#endif
    const uint32_t nsrc = (s.has_base ? 1 : 0) + s.napplied;
    for (uint32_t it = t; it < nsrc * OC_NCOLS; it += T) decode_item(s, it);
    // actor ranks (lexicographic order of the hex ids)
    for (uint32_t i = t; i < s.nactors; i += T) {
      uint32_t rank = 0;
      for (uint32_t j = 0; j < s.nactors; j++)
        if (actor_cmp_dev(A + actors[j].off, actors[j].len, A + actors[i].off, actors[i].len) < 0) rank++;
      actors[i].rank = rank;
    }
    __syncthreads();
    if (s.status) goto done;
#if defined(AM_STOP_PHASE) && AM_STOP_PHASE == 3
    goto done;
#endif

    // P5a: per-op checks of change rows (readNextChangeOp new.js:715-723; mergeDocChangeOps shapes)
    for (uint32_t i = t; i < R; i += T) {
      const Row& r = rows[i];
      if (r.id_ctr == AM_NULL64 || r.id_actor < 0) { set_err(s, AM_U_VALUE); continue; }
      if (!r.src_change) continue;
      if ((r.obj_ctr == AM_NULL64) != (r.obj_actor < 0)) { set_err(s, AM_E_MISMATCH_OBJ, r.obj_ctr, r.obj_actor); continue; }
      if ((r.key_ctr == AM_NULL64 && r.key_actor >= 0) || (r.key_ctr == 0 && r.key_actor >= 0) ||
          (r.key_ctr != AM_NULL64 && r.key_ctr > 0 && r.key_actor < 0)) {
        set_err(s, AM_E_MISMATCH_KEY, r.key_ctr, r.key_actor);
        continue;
      }
      if (r.action == AM_NULL64) { set_err(s, AM_U_VALUE); continue; }
      if (r.is_del && (r.insert || r.ps_cnt == 0)) { set_err(s, AM_U_DEL_SHAPE); continue; }
      if (r.insert && r.ps_cnt > 0) {
        const Ent& p = ents[r.ps_off];
        set_err(s, AM_E_PRED_NOT_FOUND, p.ctr, 0, actors[p.actor].off, actors[p.actor].len);
        continue;
      }
      if (r.key_len == AM_NOSTR && !r.insert && r.key_ctr == AM_NULL64) { set_err(s, AM_U_VALUE); continue; }
    }
    // P5c: id index sorted by (ctr, actor index)
    const uint32_t PR = pow2_ceil(R > 0 ? R : 1);
    IdKey* idk = hp<IdKey>(s, L.idk);
    for (uint32_t i = t; i < PR; i += T) {
      IdKey k;
      if (i < R) { k.ctr = rows[i].id_ctr; k.actor = rows[i].id_actor; k.row = (int32_t)i; }
      else { k.ctr = INT64_MAX; k.actor = INT32_MAX; k.row = INT32_MAX; }
      idk[i] = k;
    }
    __syncthreads();
    if (s.status) goto done;
    block_bitonic_sort(idk, PR, [](const IdKey& a, const IdKey& b) {
      if (a.ctr != b.ctr) return a.ctr < b.ctr;
      if (a.actor != b.actor) return a.actor < b.actor;
      return a.row < b.row;
    });
    for (uint32_t i = t + 1; i < R; i += T)
      if (idk[i].ctr == idk[i - 1].ctr && idk[i].actor == idk[i - 1].actor)
        set_err(s, AM_E_DUP_OPID, idk[i].ctr, 0, actors[idk[i].actor].off, actors[idk[i].actor].len);
    __syncthreads();
    if (s.status) goto done;

    auto id_less = [&](int64_t c1, int32_t a1, int64_t c2, int32_t a2) {
      if (c1 != c2) return c1 < c2;
      return actors[a1].rank < actors[a2].rank;
    };
    // P5d: resolve preds -> targets (new.js:1173-1188, 1254-1258)
    int32_t* elem_of = hp<int32_t>(s, L.elem_of);
    int32_t* parent = hp<int32_t>(s, L.parent);
    for (uint32_t i = t; i < R; i += T) {
      const Row& r = rows[i];
      elem_of[i] = -1;
      parent[i] = -1;
      if (!r.src_change || r.insert) continue;
      for (uint32_t q = 0; q < r.ps_cnt; q++) {
        Ent& p = ents[r.ps_off + q];
        int32_t tr = id_lookup(idk, R, p.ctr, p.actor);
        bool ok = tr >= 0 && (uint32_t)tr < i && !rows[tr].is_del;
        if (ok) {
          const Row& x = rows[tr];
          ok = same_obj(x, r) && id_less(x.id_ctr, x.id_actor, r.id_ctr, r.id_actor);
          if (ok) {
            if (r.key_len != AM_NOSTR) {
              ok = x.key_len == r.key_len && bytes_eq(A + x.key_off, A + r.key_off, r.key_len);
            } else {
              int64_t ec = x.insert ? x.id_ctr : x.key_ctr;
              int32_t ea = x.insert ? x.id_actor : x.key_actor;
              ok = x.key_len == AM_NOSTR && ec == r.key_ctr && ea == r.key_actor;
            }
          }
        }
        if (!ok) { set_err(s, AM_E_PRED_NOT_FOUND, p.ctr, 0, actors[p.actor].off, actors[p.actor].len); break; }
        p.row = tr;
      }
    }
    __syncthreads();
    if (s.status) goto done;
    // P5e: list elements: reference elements of inserts, target elements of updates
    for (uint32_t i = t; i < R; i += T) {
      const Row& r = rows[i];
      if (r.key_len != AM_NOSTR || r.is_del) continue;
      if (r.insert) {
        elem_of[i] = (int32_t)i;
        if (r.key_ctr == AM_NULL64 || r.key_ctr == 0 || r.key_actor < 0) { parent[i] = -1; continue; }
        int32_t p = id_lookup(idk, R, r.key_ctr, r.key_actor);
        bool ok = p >= 0 && rows[p].insert && !rows[p].is_del && same_obj(rows[p], r) && rows[p].key_len == AM_NOSTR &&
                  (!r.src_change || (uint32_t)p < i);
        if (!ok) {
          if (r.src_change) set_err(s, AM_E_REF_NOT_FOUND, r.key_ctr, 0, actors[r.key_actor].off, actors[r.key_actor].len);
          else set_err(s, AM_U_VALUE);
          continue;
        }
        if (!(rows[p].id_ctr < r.id_ctr)) { set_err(s, AM_U_NONCAUSAL); continue; }
        parent[i] = p;
      } else {
        int32_t e = (r.key_actor >= 0) ? id_lookup(idk, R, r.key_ctr, r.key_actor) : -1;
        bool ok = e >= 0 && rows[e].insert && !rows[e].is_del && same_obj(rows[e], r) && rows[e].key_len == AM_NOSTR &&
                  (!r.src_change || (uint32_t)e < i);
        if (!ok) {
          if (r.src_change) set_err(s, AM_E_ELEM_NOT_FOUND, r.key_ctr, 0, r.key_actor >= 0 ? actors[r.key_actor].off : 0,
                                    r.key_actor >= 0 ? actors[r.key_actor].len : 0);
          else set_err(s, AM_U_VALUE);
          continue;
        }
        if (!id_less(rows[e].id_ctr, rows[e].id_actor, r.id_ctr, r.id_actor)) { set_err(s, AM_U_NONCAUSAL); continue; }
        elem_of[i] = e;
      }
    }
    __syncthreads();
    if (s.status) goto done;

    // P5f: RGA order = preorder of the reference-element tree with children in descending opId
    // order (new.js:145-163). Euler tour + Wyllie list ranking (pointer jumping).
    uint32_t* scan = hp<uint32_t>(s, L.scan);
    for (uint32_t i = t; i < R; i += T) scan[i] = (elem_of[i] == (int32_t)i) ? 1u : 0u;
    __syncthreads();
    const uint32_t M = block_excl_scan(scan, R, s.tmp);
    const uint32_t PM = pow2_ceil(M > 0 ? M : 1);
    ElemKey* ek = hp<ElemKey>(s, L.elemk);
    for (uint32_t i = t; i < R; i += T)
      if (elem_of[i] == (int32_t)i) {
        const Row& r = rows[i];
        ElemKey k;
        k.obj_ctr = r.obj_ctr == AM_NULL64 ? -1 : r.obj_ctr;
        k.obj_rank = r.obj_actor < 0 ? -1 : (int32_t)actors[r.obj_actor].rank;
        k.parent = parent[i];
        k.id_ctr = r.id_ctr;
        k.id_rank = (int32_t)actors[r.id_actor].rank;
        k.row = (int32_t)i;
        ek[scan[i]] = k;
      }
    for (uint32_t i = M + t; i < PM; i += T) { ElemKey k; k.obj_ctr = INT64_MAX; k.row = -1; k.obj_rank = 0; k.parent = 0; k.id_ctr = 0; k.id_rank = 0; ek[i] = k; }
    __syncthreads();
    block_bitonic_sort(ek, PM, [](const ElemKey& a, const ElemKey& b) {
      if (a.obj_ctr != b.obj_ctr) return a.obj_ctr < b.obj_ctr;
      if (a.obj_rank != b.obj_rank) return a.obj_rank < b.obj_rank;
      if (a.parent != b.parent) return a.parent < b.parent;
      if (a.id_ctr != b.id_ctr) return a.id_ctr > b.id_ctr;  // children: descending opId
      return a.id_rank > b.id_rank;
    });
    int32_t* first_child = hp<int32_t>(s, L.first_child);
    int32_t* next_sib = hp<int32_t>(s, L.next_sib);
    for (uint32_t i = t; i < R; i += T) { first_child[i] = -1; next_sib[i] = -1; }
    __syncthreads();
    auto same_group = [&](const ElemKey& a, const ElemKey& b) {
      return a.obj_ctr == b.obj_ctr && a.obj_rank == b.obj_rank && a.parent == b.parent;
    };
    for (uint32_t i = t; i < M; i += T) {
      const ElemKey& k = ek[i];
      if (i + 1 < M && same_group(k, ek[i + 1])) next_sib[k.row] = ek[i + 1].row;
      if ((i == 0 || !same_group(ek[i - 1], k)) && k.parent >= 0) first_child[k.parent] = k.row;
    }
    __syncthreads();
    int32_t* nxtA = hp<int32_t>(s, L.tour_nxt);
    int32_t* nxtB = nxtA + 2 * R;
    int32_t* wA = hp<int32_t>(s, L.tour_w);
    int32_t* wB = wA + 2 * R;
    const int32_t END = -1;
    for (uint32_t i = t; i < R; i += T) {
      bool el = elem_of[i] == (int32_t)i;
      nxtA[2 * i] = el ? (first_child[i] >= 0 ? 2 * first_child[i] : (int32_t)(2 * i + 1)) : END;
      wA[2 * i] = el ? 1 : 0;
      nxtA[2 * i + 1] = el ? (next_sib[i] >= 0 ? 2 * next_sib[i] : (parent[i] >= 0 ? 2 * parent[i] + 1 : END)) : END;
      wA[2 * i + 1] = 0;
    }
    __syncthreads();
    for (uint32_t span = 1; span < 2 * R; span <<= 1) {
      for (uint32_t x = t; x < 2 * R; x += T) {
        int32_t nx = nxtA[x];
        if (nx != END) { wB[x] = wA[x] + wA[nx]; nxtB[x] = nxtA[nx]; }
        else { wB[x] = wA[x]; nxtB[x] = END; }
      }
      __syncthreads();
      int32_t* tp = nxtA; nxtA = nxtB; nxtB = tp;
      tp = wA; wA = wB; wB = tp;
    }
    // wA[2v] = number of elements from v to the end of its object's list (suffix count)
#if defined(AM_STOP_PHASE) && AM_STOP_PHASE == 4
    goto done;
#endif

    // P5g: document order: object, then key (UTF-16) | element position, then opId
    SortRec* sr = hp<SortRec>(s, L.sortrec);
    for (uint32_t i = t; i < R; i += T) scan[i] = rows[i].is_del ? 0u : 1u;
    __syncthreads();
    const uint32_t NOUT = block_excl_scan(scan, R, s.tmp);
    const uint32_t PO = pow2_ceil(NOUT > 0 ? NOUT : 1);
    for (uint32_t i = t; i < R; i += T) {
      const Row& r = rows[i];
      if (r.is_del) continue;
      SortRec k;
      k.obj_ctr = r.obj_ctr == AM_NULL64 ? -1 : r.obj_ctr;
      k.obj_rank = r.obj_actor < 0 ? -1 : (int32_t)actors[r.obj_actor].rank;
      k.kind = r.key_len != AM_NOSTR ? 0 : 1;
      k.k1 = k.kind ? -(int64_t)wA[2 * elem_of[i]] : 0;
      k.key_off = r.key_off;
      k.key_len = r.key_len;
      k.id_ctr = r.id_ctr;
      k.id_rank = (int32_t)actors[r.id_actor].rank;
      k.row = (int32_t)i;
      k.pad = 0;
      sr[scan[i]] = k;
    }
    for (uint32_t i = NOUT + t; i < PO; i += T) { SortRec k; k.row = -1; k.obj_ctr = INT64_MAX; k.obj_rank = 0; k.kind = 0; k.k1 = 0; k.key_off = 0; k.key_len = 0; k.id_ctr = 0; k.id_rank = 0; k.pad = 0; sr[i] = k; }
    __syncthreads();
    block_bitonic_sort(sr, PO, [A](const SortRec& a, const SortRec& b) {
      if ((a.row < 0) != (b.row < 0)) return b.row < 0;
      if (a.row < 0) return false;
      if (a.obj_ctr != b.obj_ctr) return a.obj_ctr < b.obj_ctr;
      if (a.obj_rank != b.obj_rank) return a.obj_rank < b.obj_rank;
      if (a.kind != b.kind) return a.kind < b.kind;
      if (a.kind == 0) {
        int c = utf16_cmp_dev(A + a.key_off, a.key_len, A + b.key_off, b.key_len);
        if (c) return c < 0;
      } else if (a.k1 != b.k1) {
        return a.k1 < b.k1;
      }
      if (a.id_ctr != b.id_ctr) return a.id_ctr < b.id_ctr;
      return a.id_rank < b.id_rank;
    });

    // P5h: succ lists = existing succ (base rows) merged with new succs from preds
    NewEnt* ne = hp<NewEnt>(s, L.newent);
    const uint32_t NNEW = s.nents - s.nbe;
    const uint32_t PN = pow2_ceil(NNEW > 0 ? NNEW : 1);
    for (uint32_t j = t; j < PN; j += T) {
      NewEnt x;
      x.target = j < NNEW ? ents[s.nbe + j].row : INT32_MAX;
      x.ctr = 0; x.actor = 0; x.rank = 0; x.pad = 0;
      ne[j] = x;
    }
    __syncthreads();
    // owning op id of each pred entry
    for (uint32_t i = t; i < R; i += T) {
      const Row& r = rows[i];
      if (!r.src_change) continue;
      for (uint32_t q = 0; q < r.ps_cnt; q++) {
        NewEnt& x = ne[r.ps_off + q - s.nbe];
        x.ctr = r.id_ctr;
        x.actor = r.id_actor;
        x.rank = (int32_t)actors[r.id_actor].rank;
      }
    }
    __syncthreads();
    block_bitonic_sort(ne, PN, [](const NewEnt& a, const NewEnt& b) {
      if (a.target != b.target) return a.target < b.target;
      if (a.ctr != b.ctr) return a.ctr < b.ctr;
      return a.rank < b.rank;
    });
    uint32_t* succ_cnt = hp<uint32_t>(s, L.succ_cnt);
    auto new_range = [&](int32_t row, uint32_t& lo_out) -> uint32_t {
      uint32_t lo = 0, hi = NNEW;
      while (lo < hi) { uint32_t m = (lo + hi) >> 1; if (ne[m].target < row) lo = m + 1; else hi = m; }
      uint32_t a = lo;
      hi = NNEW;
      while (lo < hi) { uint32_t m = (lo + hi) >> 1; if (ne[m].target <= row) lo = m + 1; else hi = m; }
      lo_out = a;
      return lo - a;
    };
    for (uint32_t i = t; i < NOUT; i += T) {
      const Row& r = rows[sr[i].row];
      uint32_t lo;
      succ_cnt[i] = (r.src_change ? 0 : r.ps_cnt) + new_range(sr[i].row, lo);
    }
    __syncthreads();
    const uint32_t NSUCC = block_excl_scan(succ_cnt, NOUT, s.tmp);
    Ent* outent = hp<Ent>(s, L.outent);
    for (uint32_t i = t; i < NOUT; i += T) {
      const int32_t ri = sr[i].row;
      const Row& r = rows[ri];
      uint32_t lo;
      uint32_t nn = new_range(ri, lo);
      uint32_t no = r.src_change ? 0 : r.ps_cnt;
      uint32_t a = 0, b2 = 0, w = succ_cnt[i];
      while (a < no || b2 < nn) {
        bool take_old;
        if (a >= no) take_old = false;
        else if (b2 >= nn) take_old = true;
        else {
          const Ent& eo = ents[r.ps_off + a];
          const NewEnt& en = ne[lo + b2];
          // insertion point: first existing succ that is not smaller (new.js:1178-1182)
          take_old = eo.ctr < en.ctr || (eo.ctr == en.ctr && (eo.actor >= 0 && (int32_t)actors[eo.actor].rank < en.rank));
        }
        Ent o;
        if (take_old) { o = ents[r.ps_off + a]; a++; }
        else { o.ctr = ne[lo + b2].ctr; o.actor = ne[lo + b2].actor; b2++; }
        o.row = ri;
        outent[w++] = o;
      }
    }
    if (t == 0) { s.nout = NOUT; s.nnew = NSUCC; }
    __syncthreads();
#if defined(AM_STOP_PHASE) && AM_STOP_PHASE == 5
    goto done;
#endif

    // P6: canonical re-encode, one column per lane (DOC_OPS_COLUMNS then DOCUMENT_COLUMNS)
    const ChgRow* chg = hp<ChgRow>(s, L.chg);
    const int64_t* depsv = hp<int64_t>(s, L.deps);
    const uint32_t NC = s.nchg;
    for (uint32_t c = t; c < OC_NCOLS + DC_NCOLS; c += T) {
      uint8_t* o0 = s.ws + L.colbuf[c];
      uint8_t* o = o0;
      int64_t* scratch = wsp<int64_t>(s, L.scratch) + (uint64_t)kScratchSlot[c] * L.scratch_stride;
      auto R_ = [&](uint32_t i) -> const Row& { return rows[sr[i].row]; };
      auto act = [](int32_t a) -> int64_t { return a < 0 ? AM_NULL64 : (int64_t)a; };
      switch (c) {
        case 0: o = enc_rle_int(o, NOUT, [&](uint32_t i) { return act(R_(i).obj_actor); }, false); break;
        case 1: o = enc_rle_int(o, NOUT, [&](uint32_t i) { return R_(i).obj_ctr; }, false); break;
        case 2: o = enc_rle_int(o, NOUT, [&](uint32_t i) { return act(R_(i).key_actor); }, false); break;
        case 3: o = enc_delta(o, NOUT, [&](uint32_t i) { return R_(i).key_ctr; }, scratch); break;
        case 4: o = enc_rle_str(o, NOUT, A, [&](uint32_t i, uint64_t& so, uint32_t& sl) { so = R_(i).key_off; sl = R_(i).key_len; }); break;
        case 5: o = enc_rle_int(o, NOUT, [&](uint32_t i) { return act(R_(i).id_actor); }, false); break;
        case 6: o = enc_delta(o, NOUT, [&](uint32_t i) { return R_(i).id_ctr; }, scratch); break;
        case 7: o = enc_bool(o, NOUT, [&](uint32_t i) { return R_(i).insert != 0; }); break;
        case 8: o = enc_rle_int(o, NOUT, [&](uint32_t i) { return R_(i).action; }, false); break;
        case 9: o = enc_rle_int(o, NOUT, [&](uint32_t i) { return R_(i).val_len; }, false); break;
        case 10:
          for (uint32_t i = 0; i < NOUT; i++) {
            const Row& r = R_(i);
            uint64_t nb = r.val_len == AM_NULL64 ? 0 : ((uint64_t)r.val_len >> 4);
            for (uint64_t q = 0; q < nb; q++) *o++ = A[r.val_off + q];
          }
          break;
        case 11: o = enc_rle_int(o, NOUT, [&](uint32_t i) { return act(R_(i).chld_actor); }, false); break;
        case 12: o = enc_delta(o, NOUT, [&](uint32_t i) { return R_(i).chld_ctr; }, scratch); break;
        case 13: o = enc_rle_int(o, NOUT, [&](uint32_t i) { return (int64_t)(i + 1 < NOUT ? succ_cnt[i + 1] : NSUCC) - succ_cnt[i]; }, false); break;
        case 14: o = enc_rle_int(o, NSUCC, [&](uint32_t i) { return act(outent[i].actor); }, false); break;
        case 15: o = enc_delta(o, NSUCC, [&](uint32_t i) { return outent[i].ctr; }, scratch); break;
        case 16 + DC_ACTOR: o = enc_rle_int(o, NC, [&](uint32_t i) { return chg[i].actor; }, false); break;
        case 16 + DC_SEQ: o = enc_delta(o, NC, [&](uint32_t i) { return chg[i].seq; }, scratch); break;
        case 16 + DC_MAXOP: o = enc_delta(o, NC, [&](uint32_t i) { return chg[i].max_op; }, scratch); break;
        case 16 + DC_TIME: o = enc_delta(o, NC, [&](uint32_t i) { return chg[i].time; }, scratch); break;
        case 16 + DC_MESSAGE: o = enc_rle_str(o, NC, A, [&](uint32_t i, uint64_t& so, uint32_t& sl) { so = chg[i].msg_off; sl = chg[i].msg_len; }); break;
        case 16 + DC_DEPS_NUM: o = enc_rle_int(o, NC, [&](uint32_t i) { return (int64_t)chg[i].ndeps; }, false); break;
        case 16 + DC_DEPS_INDEX: o = enc_delta(o, s.ndeps, [&](uint32_t i) { return depsv[i]; }, scratch); break;
        case 16 + DC_EXTRA_LEN: o = enc_rle_int(o, NC, [&](uint32_t i) { return chg[i].extra_len; }, false); break;
        case 16 + DC_EXTRA_RAW:
          for (uint32_t i = 0; i < NC; i++)
            for (uint32_t q = 0; q < chg[i].extra_raw_len; q++) *o++ = A[chg[i].extra_off + q];
          break;
      }
      s.col_len[c] = (uint32_t)(o - o0);
    }
    __syncthreads();
    // header + body assembly (encodeDocumentHeader, columnar.js:983-1004)
    uint8_t* out = s.ws + L.out;
    const uint8_t* heads = hp<uint8_t>(s, L.heads);
    const int64_t* hidx = hp<int64_t>(s, L.hidx);
    if (t == 0) {
      uint64_t body = uleb_len(s.nactors);
      for (uint32_t i = 0; i < s.nactors; i++) body += uleb_len(actors[i].len) + actors[i].len;
      body += uleb_len(s.nheads) + 32ull * s.nheads;
      uint32_t nce = 0, noe = 0;
      for (int c = 0; c < DC_NCOLS; c++) if (s.col_len[16 + c]) { nce++; body += uleb_len(kDocChgColIds[c]) + uleb_len(s.col_len[16 + c]) + s.col_len[16 + c]; }
      for (int c = 0; c < OC_NCOLS; c++) if (s.col_len[c]) { noe++; body += uleb_len(kDocOpColIds[c]) + uleb_len(s.col_len[c]) + s.col_len[c]; }
      body += uleb_len(nce) + uleb_len(noe);
      // headsIndexes only when every head index is known (loaded documents may lack them)
      bool write_hidx = true;
      for (uint32_t i = 0; i < s.nheads; i++) if (hidx[i] < 0) write_hidx = false;
      if (write_hidx)
        for (uint32_t i = 0; i < s.nheads; i++) body += uleb_len((uint64_t)hidx[i]);
      const uint32_t extra_len = s.has_base ? s.dh.extra_len : 0;
      body += extra_len;
      if (9 + 10 + body > L.out_cap) {
        set_err(s, AM_U_CAPACITY);
      } else {
        uint8_t* o = out;
        for (int k = 0; k < 4; k++) *o++ = kMagic[k];
        for (int k = 0; k < 4; k++) *o++ = 0;  // checksum, filled by k_out_hash_ws
        *o++ = 0;  // CHUNK_TYPE_DOCUMENT
        o = put_uleb(o, body);
        o = put_uleb(o, s.nactors);
        for (uint32_t i = 0; i < s.nactors; i++) {
          o = put_uleb(o, actors[i].len);
          for (uint32_t q = 0; q < actors[i].len; q++) *o++ = A[actors[i].off + q];
        }
        o = put_uleb(o, s.nheads);
        for (uint32_t i = 0; i < 32 * s.nheads; i++) *o++ = heads[i];
        o = put_uleb(o, nce);
        for (int c = 0; c < DC_NCOLS; c++) if (s.col_len[16 + c]) { o = put_uleb(o, kDocChgColIds[c]); o = put_uleb(o, s.col_len[16 + c]); }
        o = put_uleb(o, noe);
        for (int c = 0; c < OC_NCOLS; c++) if (s.col_len[c]) { o = put_uleb(o, kDocOpColIds[c]); o = put_uleb(o, s.col_len[c]); }
        uint64_t pos = (uint64_t)(o - out);
        // column data positions, in DOCUMENT_COLUMNS then DOC_OPS_COLUMNS order
        for (int c = 0; c < DC_NCOLS; c++) { s.col_pos[16 + c] = (uint32_t)pos; pos += s.col_len[16 + c]; }
        for (int c = 0; c < OC_NCOLS; c++) { s.col_pos[c] = (uint32_t)pos; pos += s.col_len[c]; }
        o = out + pos;
        if (write_hidx)
          for (uint32_t i = 0; i < s.nheads; i++) o = put_uleb(o, (uint64_t)hidx[i]);
        for (uint32_t q = 0; q < extra_len; q++) *o++ = A[s.dh.base + s.dh.extra_off + q];
        s.out_len = (uint64_t)(o - out);
      }
    }
    __syncthreads();
    if (s.status) goto done;
    for (uint32_t c = t; c < OC_NCOLS + DC_NCOLS; c += T) {
      const uint8_t* src = s.ws + L.colbuf[c];
      uint8_t* dst = out + s.col_pos[c];
      for (uint32_t q = 0; q < s.col_len[c]; q++) dst[q] = src[q];
    }
    // heads for the host (hot region may be LDS): mirror into the global workspace
    if (s.hot != s.ws)
      for (uint32_t q = t; q < 32 * s.nheads; q += T) s.ws[L.heads + q] = heads[q];
  }
done:
  __syncthreads();
  if (t == 0) {
    am_doc_result r;
    r.status = s.status;
    r.err_change = s.errchg;
    r.arg0 = s.arg0;
    r.arg1 = s.arg1;
    r.arg_actor_off = s.arg_actor_off;
    r.arg_actor_len = s.arg_actor_len;
    r.napplied = s.napplied;
    r.nqueued = s.nqueued;
    r.nheads = s.nheads;
    r.nops = s.nout;
    r.nchanges = s.nchg;
    r.max_op = s.max_op;
    r.out_off = 0;
    r.out_len = s.status ? 0 : s.out_len;
    r.ws_off = ws_off[doc];
    r.ws_bytes = s.L.total;
    results[doc] = r;
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
static_assert(sizeof(Ent) == AM_SZ_ENT, "Ent");
static_assert(sizeof(IdKey) == AM_SZ_IDKEY, "IdKey");
static_assert(sizeof(ElemKey) == AM_SZ_ELEMKEY, "ElemKey");
static_assert(sizeof(SortRec) == AM_SZ_SORTREC, "SortRec");
static_assert(sizeof(NewEnt) == AM_SZ_NEWENT, "NewEnt");
static_assert(sizeof(ChgRow) == AM_SZ_CHGROW, "ChgRow");
static_assert(sizeof(ActorRef) == AM_SZ_ACTORREF, "ActorRef");
static_assert(sizeof(ChgHdr) <= AM_SZ_CHGHDR, "ChgHdr");

size_t am_scan_tmp_elems(uint32_t n) { return (n + SCAN_T - 1) / SCAN_T + 1; }

__global__ void __launch_bounds__(256) k_max_hot(const DocBounds* __restrict__ bounds, uint32_t ndocs, uint64_t* __restrict__ max_hot) {
  uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= ndocs) return;
  WsLayout L = ws_layout(bounds[d]);
  atomicMax(reinterpret_cast<unsigned long long*>(max_hot), (unsigned long long)L.hot_total);
}

void am_launch_chunks(const BatchDev& b, hipStream_t s) {
  if (!b.nchunks) return;
  hipLaunchKernelGGL(k_chunks, dim3((b.nchunks + 255) / 256), dim3(256), 0, s, b.arena, b.chunks, b.nchunks, b.info);
}
void am_launch_bounds(const BatchDev& b, hipStream_t s) {
  if (!b.ndocs) return;
  (void)hipMemsetAsync(b.max_hot, 0, sizeof(uint64_t), s);
  hipLaunchKernelGGL(k_bounds, dim3((b.ndocs + 255) / 256), dim3(256), 0, s, b.docs, b.ndocs, b.chunks, b.info, b.bounds,
                     b.ws_bytes);
  hipLaunchKernelGGL(k_max_hot, dim3((b.ndocs + 255) / 256), dim3(256), 0, s, b.bounds, b.ndocs, b.max_hot);
  uint32_t nblk = (b.ndocs + SCAN_T - 1) / SCAN_T;
  hipLaunchKernelGGL(k_scan_blocks, dim3(nblk), dim3(SCAN_T), 0, s, b.ws_bytes, b.ws_off, b.scan_tmp, b.ndocs);
  hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(SCAN_T), 0, s, b.scan_tmp, nblk, b.ws_total);
  hipLaunchKernelGGL(k_scan_add, dim3(nblk), dim3(SCAN_T), 0, s, b.ws_off, b.scan_tmp, b.ndocs);
}
void am_launch_doc(const BatchDev& b, hipStream_t s) {
  if (!b.ndocs) return;
  hipLaunchKernelGGL(k_doc, dim3(b.ndocs), dim3(DOC_T), b.lds_bytes, s, b.arena, b.chunks, b.docs, b.known, b.info,
                     b.bounds, b.ws_off, b.ws, b.ws_cap, b.lds_bytes, b.results, b.chg_state);
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
void am_launch_out_hash(const BatchDev& b, hipStream_t s) {
  if (!b.ndocs) return;
  hipLaunchKernelGGL(k_out_hash_ws, dim3((b.ndocs + 255) / 256), dim3(256), 0, s, b.results, b.ndocs, b.ws, b.bounds);
}
void am_launch_sha256(const uint8_t* arena, const am_chunk_desc* msgs, uint32_t n, uint8_t* out, hipStream_t s) {
  if (!n) return;
  hipLaunchKernelGGL(k_sha256, dim3((n + 255) / 256), dim3(256), 0, s, arena, msgs, n, out);
}
