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

#include "am_common.h"
#include "am_launch.h"

#include "am_inflate_dec.h"

namespace {
using namespace amz;

// pass 1: zlen[s] = inflated length of raw DEFLATE stream s = ord[i], or 0xFFFFFFFF when it does not
// inflate. FAST: the long-stream form (one-lookup code tables, kSliceFast per lane)
template <bool FAST>
__global__ __launch_bounds__(kLanes) void k_inflate_size(const uint8_t* __restrict__ src, const am_zstream* __restrict__ zs,
                                                         const uint32_t* __restrict__ ord, uint32_t nz,
                                                         uint32_t* __restrict__ zlen) {
  extern __shared__ uint16_t lds_inf[];
  const uint32_t i = blockIdx.x * kLanes + threadIdx.x;
  if (i >= nz) return;
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
                                                          const uint32_t* __restrict__ zlen, uint8_t* __restrict__ dst) {
  extern __shared__ uint16_t lds_inf[];
  const uint32_t i = blockIdx.x * kLanes + threadIdx.x;
  if (i >= nz) return;
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

}  // namespace

static_assert(kLanes * kSliceFast * sizeof(uint16_t) <= 160 * 1024, "k_inflate LDS exceeds the gfx950 workgroup limit");
// ord[0, nlong): the long streams (largest first) for the FAST form; ord[nlong, nz): the rest
void am_launch_inflate_size(const uint8_t* src, const am_zstream* zs, const uint32_t* ord, uint32_t nlong, uint32_t nz,
                            uint32_t* zlen, hipStream_t s) {
  if (nlong)
    k_inflate_size<true><<<(nlong + kLanes - 1) / kLanes, kLanes, kLanes * kSliceFast * sizeof(uint16_t), s>>>(src, zs, ord, nlong,
                                                                                                             zlen);
  if (nz > nlong)
    k_inflate_size<false><<<(nz - nlong + kLanes - 1) / kLanes, kLanes, kLanes * kSlice * sizeof(uint16_t), s>>>(
        src, zs, ord + nlong, nz - nlong, zlen);
}
void am_launch_inflate_write(const uint8_t* src, const am_zstream* zs, const uint32_t* ord, uint32_t nlong, uint32_t nz,
                             const uint32_t* zlen, uint8_t* dst, hipStream_t s) {
  if (nlong)
    k_inflate_write<true><<<(nlong + kLanes - 1) / kLanes, kLanes, kLanes * kSliceFast * sizeof(uint16_t), s>>>(src, zs, ord, nlong,
                                                                                                              zlen, dst);
  if (nz > nlong)
    k_inflate_write<false><<<(nz - nlong + kLanes - 1) / kLanes, kLanes, kLanes * kSlice * sizeof(uint16_t), s>>>(
        src, zs, ord + nlong, nz - nlong, zlen, dst);
}
// long streams (>= 1 KiB compressed) first, largest first, so each workgroup's lanes carry streams
// of similar length and the longest start at once; then the others in their order
uint32_t am_inflate_order(const am_zstream* zs, uint32_t nz, uint32_t* ord) {
  constexpr uint32_t kLong = 1024;
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
