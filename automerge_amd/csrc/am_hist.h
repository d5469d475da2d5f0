// am_hist.h -- records shared by k_history (am_hist_dev.h) and its host stage (am_hist.hip): the
// per-document descriptor / result, the reconstructed-change record, the error kinds and the
// workspace layout. Plain structs, host and device.
#pragma once
#include <stdint.h>

#include "am_common.h"

enum : uint32_t {
  HE_OK = 0,
  HE_SEQ = 1,       // Expected seq = a0, got a1                          (columnar.js:880)
  HE_MAXOP = 2,     // maxOp must increase monotonically per actor        (:883)
  HE_RANGE = 3,     // Operation ID a0@actor(a1) outside of allowed range (:923)
  HE_OPID = 4,      // Expected opId a0@actor(a1), got a2@actor(a3)       (:935)
  HE_NOHASH = 5,    // No hash for index a0 while processing index a1     (:952)
  HE_HEADS = 6,     // Mismatched heads hashes (the host formats both lists) (:977)
  HE_EXTRA = 7,     // Bad datatype for extra bytes: 7                    (:961)
  HE_DEL = 8,       // document should not contain del operations         (:890)
  HE_CODE = 9,      // an AM_E_* / AM_U_* code in a0 (codec, container, shapes); AM_U_CAPACITY: a1 = bytes needed
};

struct HistDesc {
  uint32_t chunk;     // the document's chunk (am_chunk_desc / ChunkInfo index)
  uint32_t pad;
  uint64_t ws_off;    // workspace offset (hist_layout(...).total bytes)
  uint64_t out_off;   // change chunks region offset
  uint64_t out_cap;   // its bytes
  uint64_t chg_off;   // first HistChange of the document
};
struct HistResult {
  uint32_t status;    // HE_*
  uint32_t nchanges;
  int64_t a0, a1, a2, a3;
};
struct HistChange {   // one reconstructed change
  uint64_t off;       // chunk bytes: out[off, off + len) within the document's region
  uint32_t len;
  uint32_t head;      // 1: no later change depends on it (the actual heads)
  uint8_t hash[32];
};

struct HistLayout {
  uint64_t cells, chg, deps, ops, idk, sent, ord, pord, actchg, amax, acnt, aoff, alen, arank, slot, mark, total;
};

__host__ __device__ inline uint64_t hist_pow2(uint64_t n) {
  uint64_t p = 1;
  while (p < n) p <<= 1;
  return p;
}
// HChgD / HOpD / HSucc sizes (am_hist_dev.h asserts them)
#define AM_SZ_HCHG 112
#define AM_SZ_HOP 88
#define AM_SZ_HSUCC 24

// Per-document workspace from the chunk's counts (ChunkInfo: op rows NO, succ entries NS, change
// rows NC, depsIndex entries ND, actors NA)
__host__ __device__ inline HistLayout hist_layout(uint64_t NO, uint64_t NS, uint64_t NC, uint64_t ND, uint64_t NA) {
  HistLayout L;
  uint64_t o = 0;
  auto take = [&](uint64_t n) { const uint64_t at = o; o += (n + 15) & ~(uint64_t)15; return at; };
  const uint64_t NOPS = NO + NS;  // rows + at most one re-created deletion per succ entry
  L.cells = take((13 * NO + 2 * NS) * 8);
  L.chg = take(NC * AM_SZ_HCHG);
  L.deps = take(ND * 8);
  L.ops = take(NOPS * AM_SZ_HOP);
  L.idk = take(hist_pow2(NO ? NO : 1) * 16);
  L.sent = take(NS * AM_SZ_HSUCC);
  L.ord = take(hist_pow2(NOPS ? NOPS : 1) * 16);
  L.pord = take(hist_pow2(NS ? NS : 1) * 16);
  L.actchg = take(hist_pow2(NC ? NC : 1) * 16);
  L.amax = take((NA + 1) * 8);
  L.acnt = take((NA + 1) * 8);
  L.aoff = take((NA + 1) * 8);
  L.alen = take((NA + 1) * 4);
  L.arank = take((NA + 1) * 4);
  L.slot = take((NC + 1) * 8);
  L.mark = take((NC + 1) * 4);
  L.total = o;
  return L;
}
// Output slot of one change (8-aligned): container header room, the body -- header (deps hashes,
// author, seq/startOp/time, message, the other actors: at most one per actor reference `refb`),
// the column table and 14 columns (<= 11 bytes per RLE value plus a run header per column, key /
// value bytes), the extra bytes -- and the encoder's scratch at the slot's tail (literal values,
// the change's actor list).
__host__ __device__ inline uint64_t hist_slot_bound(uint64_t ops, uint64_t np, uint64_t nd, uint64_t vb, uint64_t kb, uint64_t msg,
                                                    uint64_t extra, uint64_t refb) {
  const uint64_t body = 16 + 160 + 14 * 24 + 32 * nd + 11 * 10 * ops + 11 * 2 * np + vb + kb + msg + extra + refb;
  const uint64_t scratch = 8 * (ops + np + 2) + 4 * (2 * ops + np + 2) + 16;
  return (body + scratch + 7) & ~(uint64_t)7;
}
// Host's first guess of a document's change-chunk bytes (actor ids up to 64 bytes); the kernel
// reports the exact need (HE_CODE / AM_U_CAPACITY, a1) when a document needs more.
__host__ __device__ inline uint64_t hist_out_guess(uint64_t NO, uint64_t NS, uint64_t NC, uint64_t ND, uint64_t B) {
  return NC * (16 + 160 + 14 * 24 + 64 + 24 + 16) + 32 * ND + (110 + 8 + 8 + 3 * 69) * (NO + NS) + (22 + 12 + 69) * NS + 2 * B + 64;
}
