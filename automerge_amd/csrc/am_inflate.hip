// am_inflate.hip -- DEFLATE decoding of compressed change chunks on the GPU.
//
// Reference: decodeChangeColumns / decodeChangeMeta inflate a chunk whose type byte is 2
// (columnar.js:742, 784) with inflateChange (:813-823): pako.inflateRaw (pako@2.0.3, raw DEFLATE,
// RFC 1951) of the container's chunk data, re-wrapped as magic + the ORIGINAL checksum + type 1 +
// uleb(length) + data. The checksum then verifies against the inflated chunk (k_chunks).
//
// Also the DEFLATEd columns of saved documents (inflateColumn, columnar.js:1062-1068): the batch
// stage rebuilds such a document in the new arena with its columns inflated (am_capi.hip
// inflate_stage), so Backend.load of a compressed document needs no host staging.
//
// One lane per raw DEFLATE stream (independent streams; C3 holds ~1M of them per GPU). A DEFLATE
// stream is bit-serial, so the parallelism is across streams, not within one; within a lane the
// decoder (am_inflate_dec.h) avoids what made it slow: it refills a 64-bit bit buffer one aligned
// word per 32 bits (not one global load per byte), decodes a Huffman code in one step from the code
// length limits held in registers (not a bit-at-a-time walk over LDS counts), and copies
// back-references in chunks of up to 16 bytes whose loads do not wait for one another. Each lane's
// symbol tables and a dynamic block's code lengths live in its own LDS slice. Two passes of the
// same decoder: pass 1 only counts the output bytes (no writes), the host then lays out the new
// arena, and pass 2 writes each stream's output at its place there (k_copy_segs moves everything
// else). Malformed streams (bad block type, over-subscribed / incomplete codes, distance too far
// back, truncated input, stored length mismatch) report failure; the chunk then stays as it is and
// k_chunks rejects it -- never a silently wrong chunk.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstdlib>

#include "am_common.h"
#include "am_launch.h"

#include "am_inflate_dec.h"

namespace {
using namespace amz;

// pass 1: zlen[s] = inflated length of raw DEFLATE stream s = ord[i], or 0xFFFFFFFF when it does not
// inflate. FAST: the long-stream form (one-lookup code tables, kSliceFast per lane)
// spw: streams per workgroup (one wave): lanes [0, spw) decode one stream each
template <bool FAST>
__global__ __launch_bounds__(kLanes) void k_inflate_size(const uint8_t* __restrict__ src, const am_zstream* __restrict__ zs,
                                                         const uint32_t* __restrict__ ord, uint32_t nz,
                                                         uint32_t* __restrict__ zlen, uint32_t spw) {
  extern __shared__ uint16_t lds_inf[];
  const uint32_t i = blockIdx.x * spw + threadIdx.x;
  if (threadIdx.x >= spw || i >= nz) return;
  const uint32_t s = ord[i];
  const am_zstream z = zs[s];
  const int64_t n =
      inflate_raw<false, FAST>(src + z.src, z.len, nullptr, 0xFFFFFFF0u, lds_inf + threadIdx.x * (FAST ? kSliceFast : kSlice));
  zlen[s] = n < 0 ? 0xFFFFFFFFu : (uint32_t)n;
}

// pass 2: stream s's zlen[s] bytes at dst + zs[s].dst (~0: the stream is not placed)
template <bool FAST>
__global__ __launch_bounds__(kLanes) void k_inflate_write(const uint8_t* __restrict__ src, const am_zstream* __restrict__ zs,
                                                          const uint32_t* __restrict__ ord, uint32_t nz,
                                                          const uint32_t* __restrict__ zlen, uint8_t* __restrict__ dst,
                                                          uint32_t spw) {
  extern __shared__ uint16_t lds_inf[];
  const uint32_t i = blockIdx.x * spw + threadIdx.x;
  if (threadIdx.x >= spw || i >= nz) return;
  const uint32_t s = ord[i];
  if (zlen[s] == 0xFFFFFFFFu) return;
  const am_zstream z = zs[s];
  if (z.dst == ~0ull) return;  // not placed: its chunk stays as it is
  if (z.hlen) {  // a compressed change re-wrapped: magic + original checksum + type 1 + uleb(length)
    uint8_t* h = dst + z.dst - 4 - z.hlen;
    h[0] = 0x85; h[1] = 0x6f; h[2] = 0x4a; h[3] = 0x83;
    for (uint32_t k = 0; k < z.hlen; k++) h[4 + k] = z.hdr[k];
  }
  inflate_raw<true, FAST>(src + z.src, z.len, dst + z.dst, zlen[s], lds_inf + threadIdx.x * (FAST ? kSliceFast : kSlice));
}

// byte ranges moved to the new arena (workgroup per segment): from the source arena or from the
// host-built header blob (the new container headers and column tables)
__global__ __launch_bounds__(256) void k_copy_segs(const uint8_t* __restrict__ src, const uint8_t* __restrict__ blob,
                                                   const am_seg* __restrict__ segs, uint32_t n, uint8_t* __restrict__ dst) {
  const uint32_t k = blockIdx.x;
  if (k >= n) return;
  const am_seg g = segs[k];
  const uint8_t* sp = (g.from ? blob : src) + g.src;
  uint8_t* dp = dst + g.dst;
  for (uint32_t q = threadIdx.x; q < g.len; q += blockDim.x) dp[q] = sp[q];
}

// ---- device-side stage of compressed change chunks (see am_launch.h) ----
constexpr uint32_t kLongZ = 1024;  // long streams: >= 1 KiB compressed (am_inflate_order)
constexpr uint32_t kZFail = 0xFFFFFFFFu;

__global__ __launch_bounds__(256) void k_zmark_bases(const am_doc_desc* __restrict__ docs, uint32_t ndocs, uint32_t nchunks,
                                                     uint8_t* __restrict__ isbase) {
  const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= ndocs) return;
  const int64_t c = docs[d].base_chunk;
  if (c >= 0 && (uint64_t)c < nchunks) isbase[c] = 1;  // a base chunk is never a compressed change
}
// unsigned LEB128 as the host stage reads a container length (HRd::u): false when the bytes run out
__device__ __forceinline__ bool z_uleb(const uint8_t* p, uint64_t n, uint64_t& off, uint64_t& v) {
  v = 0;
  int sh = 0;
  while (off < n) {
    const uint8_t b = p[off++];
    if (sh < 64) v |= (uint64_t)(b & 0x7f) << sh;
    sh += 7;
    if (!(b & 0x80)) return true;
  }
  return false;
}
// a compressed change: a container (magic, > 9 bytes, inside the arena) of type 2 whose data fits
__global__ __launch_bounds__(256) void k_zclass(const uint8_t* __restrict__ arena, uint64_t arena_len,
                                                const am_chunk_desc* __restrict__ chunks, uint32_t nchunks,
                                                const uint8_t* __restrict__ isbase, uint64_t* __restrict__ cnt,
                                                uint64_t* __restrict__ csrc, uint32_t* __restrict__ clen) {
  const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= nchunks) return;
  const am_chunk_desc k = chunks[c];
  uint64_t out = 0;
  if (!isbase[c] && !(k.flags & AM_CHUNK_RAW) && k.len > 9 && k.off + k.len <= arena_len) {
    const uint8_t* p = arena + k.off;
    if (p[0] == 0x85 && p[1] == 0x6f && p[2] == 0x4a && p[3] == 0x83 && p[8] == 2) {
      uint64_t off = 9, dl = 0;
      if (z_uleb(p, k.len, off, dl) && dl <= k.len - off) {
        csrc[c] = k.off + off;
        clen[c] = (uint32_t)dl;
        out = (dl >= kLongZ ? (1ull << 32) : 0ull) | 1ull;
      }
    }
  }
  cnt[c] = out;
}
__global__ __launch_bounds__(256) void k_zfill(const uint64_t* __restrict__ cnt, const uint64_t* __restrict__ z0, uint32_t nchunks,
                                               uint32_t nlong, const uint64_t* __restrict__ csrc, const uint32_t* __restrict__ clen,
                                               am_zstream* __restrict__ zs, uint32_t* __restrict__ ord, uint32_t* __restrict__ zid) {
  const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= nchunks) return;
  const uint64_t k = cnt[c];
  if (!k) { zid[c] = ~0u; return; }
  const uint32_t z = (uint32_t)z0[c], lb = (uint32_t)(z0[c] >> 32);
  am_zstream& o = zs[z];
  o.src = csrc[c];
  o.dst = ~0ull;
  o.len = clen[c];
  o.hlen = 0;
  ord[(k >> 32) ? lb : nlong + (z - lb)] = z;
  zid[c] = z;
}
__global__ __launch_bounds__(256) void k_zlayout(const uint8_t* __restrict__ arena, const am_chunk_desc* __restrict__ chunks,
                                                 uint32_t nchunks, const uint32_t* __restrict__ zid, const uint32_t* __restrict__ zlen,
                                                 am_zstream* __restrict__ zs, uint64_t* __restrict__ nl) {
  const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= nchunks) return;
  const am_chunk_desc k = chunks[c];
  const uint32_t z = zid[c];
  if (z == ~0u || zlen[z] == kZFail) { nl[c] = k.len; return; }
  // the header travels with the stream: the original checksum, type 1, uleb(inflated length)
  am_zstream& o = zs[z];
  const uint8_t* p = arena + k.off;
  o.hdr[0] = p[4]; o.hdr[1] = p[5]; o.hdr[2] = p[6]; o.hdr[3] = p[7];
  o.hdr[4] = 1;
  uint32_t q = 5;
  for (uint32_t v = zlen[z];;) {
    const uint8_t b = v & 0x7f;
    v >>= 7;
    o.hdr[q++] = b | (v ? 0x80 : 0);
    if (!v) break;
  }
  o.hlen = (uint8_t)q;
  nl[c] = 4ull + q + zlen[z];
}
// wave per chunk: its new descriptor, its stream's destination, or its bytes as they are
__global__ __launch_bounds__(256) void k_zplace(am_chunk_desc* __restrict__ chunks, uint32_t nchunks, const uint8_t* __restrict__ arena,
                                                const uint32_t* __restrict__ zid, const uint32_t* __restrict__ zlen,
                                                am_zstream* __restrict__ zs, const uint64_t* __restrict__ noff,
                                                const uint64_t* __restrict__ nl, uint8_t* __restrict__ dst) {
  const uint32_t c = blockIdx.x * 4 + (threadIdx.x >> 6), l = threadIdx.x & 63;
  if (c >= nchunks) return;
  const am_chunk_desc k = chunks[c];
  const uint32_t z = zid[c];
  const uint64_t at = noff[c];
  if (z != ~0u && zlen[z] != kZFail) {
    if (l == 0) zs[z].dst = at + 4 + zs[z].hlen;
  } else {
    const uint8_t* sp = arena + k.off;
    uint8_t* dp = dst + at;
    for (uint32_t q = l; q < k.len; q += 64) dp[q] = sp[q];
  }
  __builtin_amdgcn_wave_barrier();
  if (l == 0) chunks[c] = am_chunk_desc{at, (uint32_t)nl[c], k.flags};
}

}  // namespace

void am_launch_zstage_classify(const uint8_t* arena, uint64_t arena_len, const am_chunk_desc* chunks, uint32_t nchunks,
                               const am_doc_desc* docs, uint32_t ndocs, uint8_t* isbase, uint64_t* cnt, uint64_t* csrc,
                               uint32_t* clen, hipStream_t s) {
  if (!nchunks) return;
  (void)hipMemsetAsync(isbase, 0, nchunks, s);
  if (ndocs) k_zmark_bases<<<(ndocs + 255) / 256, 256, 0, s>>>(docs, ndocs, nchunks, isbase);
  k_zclass<<<(nchunks + 255) / 256, 256, 0, s>>>(arena, arena_len, chunks, nchunks, isbase, cnt, csrc, clen);
}
void am_launch_zstage_fill(const uint64_t* cnt, const uint64_t* z0, uint32_t nchunks, uint32_t nlong, const uint64_t* csrc,
                           const uint32_t* clen, am_zstream* zs, uint32_t* ord, uint32_t* zid, hipStream_t s) {
  if (nchunks) k_zfill<<<(nchunks + 255) / 256, 256, 0, s>>>(cnt, z0, nchunks, nlong, csrc, clen, zs, ord, zid);
}
void am_launch_zstage_layout(const uint8_t* arena, const am_chunk_desc* chunks, uint32_t nchunks, const uint32_t* zid,
                             const uint32_t* zlen, am_zstream* zs, uint64_t* nl, hipStream_t s) {
  if (nchunks) k_zlayout<<<(nchunks + 255) / 256, 256, 0, s>>>(arena, chunks, nchunks, zid, zlen, zs, nl);
}
void am_launch_zstage_place(am_chunk_desc* chunks, uint32_t nchunks, const uint8_t* arena, const uint32_t* zid,
                            const uint32_t* zlen, am_zstream* zs, const uint64_t* noff, const uint64_t* nl, uint8_t* dst,
                            hipStream_t s) {
  if (nchunks) k_zplace<<<(nchunks + 3) / 4, 256, 0, s>>>(chunks, nchunks, arena, zid, zlen, zs, noff, nl, dst);
}

static_assert(kLanes * kSliceFast * sizeof(uint16_t) <= 160 * 1024, "k_inflate LDS exceeds the gfx950 workgroup limit");
// ord[0, nlong): the long streams (largest first) for the FAST form; ord[nlong, nz): the rest.
// A long stream decodes in a wave of its own (AM_INFLATE_LONG_SPW streams per wave, default 1): its
// lane's dependent chain then runs without the other lanes' divergent paths, and many such waves
// per SIMD overlap their chains (64 long streams per wave held a CU's whole LDS for one wave); the
// short streams keep 64 per wave.
static uint32_t long_spw() {
  const char* e = std::getenv("AM_INFLATE_LONG_SPW");
  const uint32_t v = e ? (uint32_t)std::strtoul(e, nullptr, 10) : 1u;
  return v >= 1 && v <= (uint32_t)kLanes ? v : 1u;
}
void am_launch_inflate_size(const uint8_t* src, const am_zstream* zs, const uint32_t* ord, uint32_t nlong, uint32_t nz,
                            uint32_t* zlen, hipStream_t s) {
  if (nlong) {
    const uint32_t spw = long_spw();
    k_inflate_size<true><<<(nlong + spw - 1) / spw, kLanes, spw * kSliceFast * sizeof(uint16_t), s>>>(src, zs, ord, nlong, zlen, spw);
  }
  if (nz > nlong)
    k_inflate_size<false><<<(nz - nlong + kLanes - 1) / kLanes, kLanes, kLanes * kSlice * sizeof(uint16_t), s>>>(
        src, zs, ord + nlong, nz - nlong, zlen, (uint32_t)kLanes);
}
void am_launch_inflate_write(const uint8_t* src, const am_zstream* zs, const uint32_t* ord, uint32_t nlong, uint32_t nz,
                             const uint32_t* zlen, uint8_t* dst, hipStream_t s) {
  if (nlong) {
    const uint32_t spw = long_spw();
    k_inflate_write<true><<<(nlong + spw - 1) / spw, kLanes, spw * kSliceFast * sizeof(uint16_t), s>>>(src, zs, ord, nlong, zlen,
                                                                                                      dst, spw);
  }
  if (nz > nlong)
    k_inflate_write<false><<<(nz - nlong + kLanes - 1) / kLanes, kLanes, kLanes * kSlice * sizeof(uint16_t), s>>>(
        src, zs, ord + nlong, nz - nlong, zlen, dst, (uint32_t)kLanes);
}
// long streams (>= 1 KiB compressed) first, largest first, so each workgroup's lanes carry streams
// of similar length and the longest start at once; then the others in their order
uint32_t am_inflate_order(const am_zstream* zs, uint32_t nz, uint32_t* ord) {
  constexpr uint32_t kLong = kLongZ;
  uint32_t k = 0;
  for (uint32_t i = 0; i < nz; i++)
    if (zs[i].len >= kLong) ord[k++] = i;
  const uint32_t nlong = k;
  std::sort(ord, ord + nlong, [&](uint32_t a, uint32_t b) { return zs[a].len > zs[b].len; });
  for (uint32_t i = 0; i < nz; i++)
    if (zs[i].len < kLong) ord[k++] = i;
  return nlong;
}
void am_launch_copy_segs(const uint8_t* src, const uint8_t* blob, const am_seg* segs, uint32_t n, uint8_t* dst, hipStream_t s) {
  if (n) k_copy_segs<<<n, 256, 0, s>>>(src, blob, segs, n, dst);
}
