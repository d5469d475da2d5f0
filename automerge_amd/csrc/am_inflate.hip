// am_inflate.hip -- DEFLATE decoding of compressed change chunks on the GPU.
//
// Reference: decodeChangeColumns / decodeChangeMeta inflate a chunk whose type byte is 2
// (columnar.js:742, 784) with inflateChange (:813-823): pako.inflateRaw (pako@2.0.3, raw DEFLATE,
// RFC 1951) of the container's chunk data, re-wrapped as magic + the ORIGINAL checksum + type 1 +
// uleb(length) + data. The checksum then verifies against the inflated chunk (k_chunks).
//
// One lane per compressed chunk (independent streams; C3 holds ~1M of them per GPU). A DEFLATE
// stream is bit-serial, so the parallelism is across streams, not within one. Each lane keeps its
// canonical Huffman tables (count per code length + symbols in code order, the decoding method
// of RFC 1951 §3.2.2 -- the `puff` formulation) in its own LDS slice; a dynamic block's code
// lengths are staged in the same slice. Two passes of the same decoder: pass 1 only counts the
// output bytes (no writes), the host then lays out the new arena, and pass 2 writes the inflated
// chunk. Malformed streams (bad block type, over-subscribed / incomplete codes, distance too far
// back, truncated input, stored length mismatch) report failure; the chunk then stays type 2 and
// k_chunks rejects it -- never a silently wrong chunk.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "am_common.h"

namespace {

constexpr int kLanes = 64;
constexpr int kMaxBits = 15;
constexpr int kMaxLCodes = 286, kMaxDCodes = 30, kFixLCodes = 288;
// per-lane LDS slice (uint16 words): lencnt[16], lensym[288], distcnt[16], distsym[32], offs[16],
// lengths[320 bytes = 160 words]
constexpr int kLenCnt = 0, kLenSym = 16, kDistCnt = kLenSym + 288, kDistSym = kDistCnt + 16, kOffs = kDistSym + 32,
              kLengths = kOffs + 16, kSlice = kLengths + 160;

__constant__ uint16_t c_lbase[29] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31,
                                     35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
__constant__ uint8_t c_lext[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
__constant__ uint16_t c_dbase[30] = {1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129,
                                     193, 257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
__constant__ uint8_t c_dext[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
__constant__ uint8_t c_clorder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

struct Bits {
  const uint8_t* p;
  uint32_t n, pos;
  uint32_t buf;
  int cnt;
  bool err;
};

__device__ __forceinline__ uint32_t getbits(Bits& b, int need) {
  uint32_t v = b.buf;
  while (b.cnt < need) {
    uint32_t byte = 0;
    if (b.pos < b.n) byte = b.p[b.pos++];
    else b.err = true;
    v |= byte << b.cnt;
    b.cnt += 8;
  }
  b.buf = need < 32 ? v >> need : 0u;
  b.cnt -= need;
  return v & ((1u << need) - 1u);
}

// canonical decode, one bit at a time (RFC 1951 §3.2.2): -1 when no code matches
__device__ __forceinline__ int decode(Bits& b, const uint16_t* cnt, const uint16_t* sym) {
  int code = 0, first = 0, index = 0;
  for (int len = 1; len <= kMaxBits; len++) {
    code |= (int)getbits(b, 1);
    const int c = cnt[len];
    if (code - c < first) return sym[index + (code - first)];
    index += c;
    first += c;
    first <<= 1;
    code <<= 1;
  }
  return -1;
}

// table from code lengths; returns 0 complete, > 0 incomplete, < 0 over-subscribed
__device__ int construct(uint16_t* cnt, uint16_t* sym, uint16_t* offs, const uint8_t* lengths, int n) {
  for (int len = 0; len <= kMaxBits; len++) cnt[len] = 0;
  for (int s = 0; s < n; s++) cnt[lengths[s]]++;
  if (cnt[0] == n) return 0;
  int left = 1;
  for (int len = 1; len <= kMaxBits; len++) {
    left <<= 1;
    left -= cnt[len];
    if (left < 0) return left;
  }
  offs[1] = 0;
  for (int len = 1; len < kMaxBits; len++) offs[len + 1] = offs[len] + cnt[len];
  for (int s = 0; s < n; s++)
    if (lengths[s]) sym[offs[lengths[s]]++] = (uint16_t)s;
  return left;
}

// decodes literal/length + distance codes until end-of-block
template <bool WRITE>
__device__ bool codes(Bits& b, const uint16_t* T, uint8_t* out, uint64_t& outpos, uint64_t cap) {
  for (;;) {
    int sym = decode(b, T + kLenCnt, T + kLenSym);
    if (sym < 0 || b.err) return false;
    if (sym < 256) {
      if (outpos >= cap) return false;
      if (WRITE) out[outpos] = (uint8_t)sym;
      outpos++;
    } else if (sym == 256) {
      return true;
    } else {
      sym -= 257;
      if (sym >= 29) return false;
      const uint32_t len = c_lbase[sym] + getbits(b, c_lext[sym]);
      const int ds = decode(b, T + kDistCnt, T + kDistSym);
      if (ds < 0 || ds >= 30 || b.err) return false;
      const uint32_t dist = c_dbase[ds] + getbits(b, c_dext[ds]);
      if (dist > outpos || outpos + len > cap) return false;  // distance too far back
      if (WRITE)
        for (uint32_t k = 0; k < len; k++) out[outpos + k] = out[outpos - dist + k];
      outpos += len;
    }
  }
}

// inflates raw DEFLATE data [p, p + n); WRITE=false only counts. Returns the output length, or
// -1 on malformed input.
template <bool WRITE>
__device__ int64_t inflate_raw(const uint8_t* p, uint32_t n, uint8_t* out, uint64_t cap, uint16_t* T) {
  Bits b{p, n, 0, 0, 0, false};
  uint8_t* lengths = reinterpret_cast<uint8_t*>(T + kLengths);
  uint64_t outpos = 0;
  int last;
  do {
    last = (int)getbits(b, 1);
    const int type = (int)getbits(b, 2);
    if (b.err) return -1;
    if (type == 0) {  // stored
      b.buf = 0;
      b.cnt = 0;
      if (b.pos + 4 > b.n) return -1;
      const uint32_t len = p[b.pos] | (uint32_t)p[b.pos + 1] << 8;
      const uint32_t nlen = p[b.pos + 2] | (uint32_t)p[b.pos + 3] << 8;
      b.pos += 4;
      if (len != (~nlen & 0xffffu) || b.pos + len > b.n || outpos + len > cap) return -1;
      if (WRITE)
        for (uint32_t k = 0; k < len; k++) out[outpos + k] = p[b.pos + k];
      b.pos += len;
      outpos += len;
    } else if (type == 1) {  // fixed Huffman codes
      for (int s = 0; s < 144; s++) lengths[s] = 8;
      for (int s = 144; s < 256; s++) lengths[s] = 9;
      for (int s = 256; s < 280; s++) lengths[s] = 7;
      for (int s = 280; s < kFixLCodes; s++) lengths[s] = 8;
      construct(T + kLenCnt, T + kLenSym, T + kOffs, lengths, kFixLCodes);
      for (int s = 0; s < kMaxDCodes; s++) lengths[s] = 5;
      construct(T + kDistCnt, T + kDistSym, T + kOffs, lengths, kMaxDCodes);
      if (!codes<WRITE>(b, T, out, outpos, cap)) return -1;
    } else if (type == 2) {  // dynamic Huffman codes
      const int nlen = (int)getbits(b, 5) + 257, ndist = (int)getbits(b, 5) + 1, ncode = (int)getbits(b, 4) + 4;
      if (b.err || nlen > kMaxLCodes || ndist > kMaxDCodes) return -1;
      for (int k = 0; k < 19; k++) lengths[c_clorder[k]] = k < ncode ? (uint8_t)getbits(b, 3) : (uint8_t)0;
      // code-length code in the distance tables (free until the distance code is built)
      if (construct(T + kDistCnt, T + kDistSym, T + kOffs, lengths, 19) != 0) return -1;
      int idx = 0;
      while (idx < nlen + ndist) {
        int sym = decode(b, T + kDistCnt, T + kDistSym);
        if (sym < 0 || b.err) return -1;
        if (sym < 16) {
          lengths[idx++] = (uint8_t)sym;
        } else {
          int len = 0, rep;
          if (sym == 16) {
            if (idx == 0) return -1;
            len = lengths[idx - 1];
            rep = 3 + (int)getbits(b, 2);
          } else if (sym == 17) {
            rep = 3 + (int)getbits(b, 3);
          } else {
            rep = 11 + (int)getbits(b, 7);
          }
          if (idx + rep > nlen + ndist) return -1;
          while (rep--) lengths[idx++] = (uint8_t)len;
        }
      }
      if (lengths[256] == 0) return -1;  // no end-of-block code
      const int el = construct(T + kLenCnt, T + kLenSym, T + kOffs, lengths, nlen);
      if (el < 0 || (el > 0 && nlen != T[kLenCnt + 0] + T[kLenCnt + 1])) return -1;  // incomplete: one code only
      // distance code from lengths[nlen ..]: copy down first (construct reads lengths[0 .. ndist))
      for (int k = 0; k < ndist; k++) lengths[k] = lengths[nlen + k];
      const int ed = construct(T + kDistCnt, T + kDistSym, T + kOffs, lengths, ndist);
      if (ed < 0 || (ed > 0 && ndist != T[kDistCnt + 0] + T[kDistCnt + 1])) return -1;
      if (!codes<WRITE>(b, T, out, outpos, cap)) return -1;
    } else {
      return -1;
    }
  } while (!last);
  return (int64_t)outpos;
}

__device__ __forceinline__ uint32_t uleb_size(uint64_t v) {
  uint32_t n = 1;
  while (v >= 0x80) { v >>= 7; n++; }
  return n;
}

// container header of a type-2 chunk: magic, checksum, type, uleb chunk length (columnar.js:688-708)
__device__ bool zchunk(const uint8_t* p, uint32_t len, uint32_t& data_off, uint32_t& data_len) {
  if (len < 10 || p[0] != 0x85 || p[1] != 0x6f || p[2] != 0x4a || p[3] != 0x83 || p[8] != 2) return false;
  uint64_t v = 0;
  uint32_t o = 9;
  int sh = 0;
  for (;;) {
    if (o >= len || sh > 56) return false;
    const uint8_t c = p[o++];
    v |= (uint64_t)(c & 0x7f) << sh;
    sh += 7;
    if (!(c & 0x80)) break;
  }
  if (v > (uint64_t)(len - o)) return false;
  data_off = o;
  data_len = (uint32_t)v;
  return true;
}

// pass 1: zlen[i] = inflated data length of chunk zidx[i], or 0xFFFFFFFF when it does not inflate
__global__ __launch_bounds__(kLanes) void k_inflate_size(const uint8_t* __restrict__ arena,
                                                         const am_chunk_desc* __restrict__ chunks,
                                                         const uint32_t* __restrict__ zidx, uint32_t nz,
                                                         uint32_t* __restrict__ zlen) {
  extern __shared__ uint16_t lds_inf[];
  const uint32_t i = blockIdx.x * kLanes + threadIdx.x;
  if (i >= nz) return;
  const am_chunk_desc c = chunks[zidx[i]];
  const uint8_t* p = arena + c.off;
  uint32_t doff, dlen;
  int64_t n = -1;
  if (zchunk(p, c.len, doff, dlen))
    n = inflate_raw<false>(p + doff, dlen, nullptr, 0xFFFFFFF0u, lds_inf + threadIdx.x * kSlice);
  zlen[i] = n < 0 ? 0xFFFFFFFFu : (uint32_t)n;
}

// pass 2: the inflated chunk (magic + original checksum + type 1 + uleb(n) + data) at its new offset
__global__ __launch_bounds__(kLanes) void k_inflate_write(const uint8_t* __restrict__ arena,
                                                          const am_chunk_desc* __restrict__ chunks,
                                                          const am_chunk_desc* __restrict__ nchunks,
                                                          const uint32_t* __restrict__ zidx, uint32_t nz,
                                                          const uint32_t* __restrict__ zlen, uint8_t* __restrict__ dst) {
  extern __shared__ uint16_t lds_inf[];
  const uint32_t i = blockIdx.x * kLanes + threadIdx.x;
  if (i >= nz || zlen[i] == 0xFFFFFFFFu) return;
  const uint32_t ci = zidx[i];
  const am_chunk_desc c = chunks[ci];
  const uint8_t* p = arena + c.off;
  uint8_t* o = dst + nchunks[ci].off;
  uint32_t doff, dlen;
  if (!zchunk(p, c.len, doff, dlen)) return;
  const uint64_t n = zlen[i];
  for (int k = 0; k < 8; k++) o[k] = p[k];
  o[8] = 1;
  uint32_t q = 9;
  uint64_t v = n;
  do {
    const uint8_t byte = v & 0x7f;
    v >>= 7;
    o[q++] = byte | (v ? 0x80 : 0);
  } while (v);
  inflate_raw<true>(p + doff, dlen, o + q, n, lds_inf + threadIdx.x * kSlice);
}

// every chunk that is not re-inflated keeps its bytes at the new offset (workgroup per chunk)
__global__ __launch_bounds__(256) void k_copy_chunks(const uint8_t* __restrict__ src, const am_chunk_desc* __restrict__ chunks,
                                                     const am_chunk_desc* __restrict__ nchunks,
                                                     const uint8_t* __restrict__ inflated, uint32_t n, uint8_t* __restrict__ dst) {
  const uint32_t ci = blockIdx.x;
  if (ci >= n || inflated[ci]) return;
  const uint8_t* s = src + chunks[ci].off;
  uint8_t* d = dst + nchunks[ci].off;
  const uint32_t len = chunks[ci].len;
  for (uint32_t k = threadIdx.x; k < len; k += blockDim.x) d[k] = s[k];
}

}  // namespace

static_assert(kLanes * kSlice * sizeof(uint16_t) <= 160 * 1024, "k_inflate LDS exceeds the gfx950 workgroup limit");
void am_launch_inflate_size(const uint8_t* arena, const am_chunk_desc* chunks, const uint32_t* zidx, uint32_t nz,
                            uint32_t* zlen, hipStream_t s) {
  if (!nz) return;
  k_inflate_size<<<(nz + kLanes - 1) / kLanes, kLanes, kLanes * kSlice * sizeof(uint16_t), s>>>(arena, chunks, zidx, nz, zlen);
}

void am_launch_inflate_write(const uint8_t* arena, const am_chunk_desc* chunks, const am_chunk_desc* nchunks,
                             const uint32_t* zidx, uint32_t nz, const uint32_t* zlen, const uint8_t* inflated,
                             uint32_t n, uint8_t* dst, hipStream_t s) {
  if (n) k_copy_chunks<<<n, 256, 0, s>>>(arena, chunks, nchunks, inflated, n, dst);
  if (nz)
    k_inflate_write<<<(nz + kLanes - 1) / kLanes, kLanes, kLanes * kSlice * sizeof(uint16_t), s>>>(arena, chunks, nchunks,
                                                                                                 zidx, nz, zlen, dst);
}
