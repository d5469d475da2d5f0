// am_inflate_dec.h -- the raw DEFLATE decoder of am_inflate.hip (RFC 1951; pako.inflateRaw,
// columnar.js:816, 1064), one stream per lane. Kept in a header so the same code compiles for the
// host (tests/test_inflate_host.py checks it against zlib on the CPU; no GPU needed).
#pragma once
#include <stdint.h>

#ifndef __HIPCC__
#define __device__
#define __constant__
#define __forceinline__ inline
#include <algorithm>
using std::min;
#endif

#ifdef __clang__
#define AMZ_BREV32(x) __builtin_bitreverse32(x)
#else
static inline uint32_t AMZ_BREV32(uint32_t x) {
  x = ((x >> 1) & 0x55555555u) | ((x & 0x55555555u) << 1);
  x = ((x >> 2) & 0x33333333u) | ((x & 0x33333333u) << 2);
  x = ((x >> 4) & 0x0F0F0F0Fu) | ((x & 0x0F0F0F0Fu) << 4);
  x = ((x >> 8) & 0x00FF00FFu) | ((x & 0x00FF00FFu) << 8);
  return (x >> 16) | (x << 16);
}
#endif

namespace amz {

constexpr int kLanes = 64;
constexpr int kMaxBits = 15;
constexpr int kMaxLCodes = 286, kMaxDCodes = 30, kFixLCodes = 288;
// per-lane LDS slice (uint16 words): lencnt[16], lensym[288], distcnt[16], distsym[32], offs[16],
// lengths[320 bytes = 160 words]
constexpr int kLenCnt = 0, kLenSym = 16, kDistCnt = kLenSym + 288, kDistSym = kDistCnt + 16, kOffs = kDistSym + 32,
              kLengths = kOffs + 16, kSlice = kLengths + 160;
// long streams (the FAST decoder) also keep one-lookup tables of the codes up to kFastLBits /
// kFastDBits long: entry = symbol | length << 9 | 0x8000, 0 for a longer code (the register path)
constexpr int kFastLBits = 9, kFastDBits = 7;
constexpr int kFastL = kSlice, kFastD = kFastL + (1 << kFastLBits), kSliceFast = kFastD + (1 << kFastDBits);

__constant__ uint16_t c_lbase[29] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31,
                                     35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
__constant__ uint8_t c_lext[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
__constant__ uint16_t c_dbase[30] = {1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129,
                                     193, 257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
__constant__ uint8_t c_dext[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
__constant__ uint8_t c_clorder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// Bit reader: a 64-bit register buffer refilled one aligned 32-bit word at a time (one global load
// per 32 bits instead of one per byte, issued a refill ahead). `pos` counts the bits consumed; a
// stream that consumes more than its 8n bits is truncated (the words read past its end are never
// trusted). The arenas keep 64 bytes of slack after the last stream, so the look-ahead words are
// always readable.
struct Bits {
  const uint8_t* p;      // stream start
  const uint32_t* wp;    // the word after nw
  uint64_t buf;          // bits [0, cnt) valid
  uint32_t cnt;
  uint32_t nw;           // the next word, loaded one refill ahead (its latency hides behind 32 bits of decoding)
  uint64_t pos, nbits;   // bits consumed; 8 * stream bytes
};
__device__ __forceinline__ void bits_at(Bits& b, uint64_t byte) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(b.p + byte);
  const uint32_t* w = reinterpret_cast<const uint32_t*>(a & ~(uintptr_t)3);
  const uint32_t sh = (uint32_t)(a & 3) * 8;
  b.buf = (uint64_t)(w[0] >> sh);
  b.cnt = 32 - sh;
  b.nw = w[1];
  b.wp = w + 2;
  b.pos = 8 * byte;
}
__device__ __forceinline__ void refill(Bits& b) {
  if (b.cnt <= 32) {
    b.buf |= (uint64_t)b.nw << b.cnt;
    b.cnt += 32;
    b.nw = *b.wp++;
  }
}
__device__ __forceinline__ void drop(Bits& b, uint32_t k) {
  b.buf >>= k;
  b.cnt -= k;
  b.pos += k;
}
// k <= 24 bits (LSB first)
__device__ __forceinline__ uint32_t getbits(Bits& b, uint32_t k) {
  refill(b);
  const uint32_t v = (uint32_t)b.buf & ((1u << k) - 1u);
  drop(b, k);
  return v;
}

// A canonical Huffman code in registers for the decoder (RFC 1951 §3.2.2): lim[l] = the end of the
// codes of length <= l, left-justified to 15 bits (non-decreasing in l), cnt[l] = codes of length
// l. A code's length is the number of limits at or below the next 15 bits (+1), its symbol index
// the codes of shorter lengths plus its offset among those of its own length: no per-bit loop and
// no table walk, one LDS read (the symbol) per code.
struct Code {
  uint32_t lim[kMaxBits + 1], cnt[kMaxBits + 1];
};
__device__ __forceinline__ void code_regs(const uint16_t* cnt, Code& c) {
  uint32_t next = 0, prev = 0;
#pragma unroll
  for (int l = 1; l <= kMaxBits; l++) {
    next = (next + prev) << 1;  // first code of length l
    c.cnt[l] = cnt[l];
    prev = c.cnt[l];
    c.lim[l] = (next + prev) << (kMaxBits - l);
  }
}
// next symbol, or -1 when no code matches (an incomplete code)
__device__ __forceinline__ int decode(Bits& b, const Code& c, const uint16_t* sym) {
  refill(b);
  const uint32_t v = AMZ_BREV32((uint32_t)b.buf) >> (32 - kMaxBits);
  uint32_t L = 1, base = 0, idx = 0;
#pragma unroll
  for (int l = 1; l <= kMaxBits; l++) {
    const bool ge = v >= c.lim[l];
    L += ge ? 1u : 0u;
    base = ge ? c.lim[l] : base;
    idx += ge ? c.cnt[l] : 0u;
  }
  if (L > (uint32_t)kMaxBits) return -1;
  drop(b, L);
  return sym[idx + ((v - base) >> (kMaxBits - L))];
}

// the one-lookup table F of the codes of lengths[0, n) up to fbits long (after construct and
// code_regs; the offs scratch holds the next code per length while the symbols are placed)
__device__ void fast_table(uint16_t* F, int fbits, uint16_t* offs, const uint8_t* lengths, int n, const Code& c) {
  for (int k = 0; k < (1 << fbits); k++) F[k] = 0;
#pragma unroll
  for (int l = 1; l <= kMaxBits; l++) offs[l] = (uint16_t)((c.lim[l] >> (kMaxBits - l)) - c.cnt[l]);  // first code of length l
  for (int s = 0; s < n; s++) {
    const int len = lengths[s];
    if (len == 0 || len > fbits) continue;
    const uint32_t code = offs[len]++;
    const uint32_t r = AMZ_BREV32(code) >> (32 - len);  // the code as the bit stream delivers it
    const uint16_t e = (uint16_t)(s | (len << 9) | 0x8000);
    for (uint32_t k = r; k < (1u << fbits); k += 1u << len) F[k] = e;
  }
}
template <bool FAST>
__device__ __forceinline__ int decode_sym(Bits& b, const Code& c, const uint16_t* sym, const uint16_t* F, int fbits) {
  if constexpr (FAST) {
    refill(b);
    const uint32_t e = F[(uint32_t)b.buf & ((1u << fbits) - 1u)];
    if (e & 0x8000u) {
      drop(b, (e >> 9) & 15u);
      return (int)(e & 511u);
    }
  }
  return decode(b, c, sym);
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

// the back-reference out[pos - dist, pos - dist + len) -> out[pos, pos + len). Each chunk's source
// lies before its destination (chunk size <= the distance it copies from), so a chunk's loads are
// independent and wait for memory once; a short distance copies from the periodic pattern already
// written, at a multiple of the distance that reaches 16 bytes back.
__device__ __forceinline__ void lz_copy(uint8_t* out, uint64_t pos, uint32_t dist, uint32_t len) {
  uint32_t done = 0;
  while (done < len) {
    // bytes of the period-dist sequence available before the write position: dist + done
    // a multiple of dist within the dist + done bytes of the sequence already written, up to 16 back
    uint32_t back = dist;
    if (dist < 16) {
      uint32_t m = (dist + done) / dist;
      const uint32_t m16 = (16 + dist - 1) / dist;
      back = (m < m16 ? m : m16) * dist;
    }
    const uint32_t c = min(min(back, 16u), len - done);
    uint8_t t[16];
    const uint8_t* src = out + pos + done - back;
#pragma unroll
    for (int k = 0; k < 16; k++)
      if ((uint32_t)k < c) t[k] = src[k];
#pragma unroll
    for (int k = 0; k < 16; k++)
      if ((uint32_t)k < c) out[pos + done + k] = t[k];
    done += c;
  }
}

// decodes literal/length + distance codes until end-of-block
template <bool WRITE, bool FAST>
__device__ bool codes(Bits& b, const Code& lc, const Code& dc, const uint16_t* T, uint8_t* out, uint64_t& outpos, uint64_t cap) {
  for (;;) {
    int sym = decode_sym<FAST>(b, lc, T + kLenSym, T + kFastL, kFastLBits);
    if (sym < 0 || b.pos > b.nbits) return false;
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
      const int ds = decode_sym<FAST>(b, dc, T + kDistSym, T + kFastD, kFastDBits);
      if (ds < 0 || ds >= 30) return false;
      const uint32_t dist = c_dbase[ds] + getbits(b, c_dext[ds]);
      if (b.pos > b.nbits) return false;
      if (dist > outpos || outpos + len > cap) return false;  // distance too far back
      if (WRITE) lz_copy(out, outpos, dist, len);
      outpos += len;
    }
  }
}

// inflates raw DEFLATE data [p, p + n); WRITE=false only counts. Returns the output length, or
// -1 on malformed input. FAST: T is a kSliceFast slice and the codes go through the one-lookup
// tables (worth their construction on long streams).
template <bool WRITE, bool FAST = false>
__device__ int64_t inflate_raw(const uint8_t* p, uint32_t n, uint8_t* out, uint64_t cap, uint16_t* T) {
  Bits b;
  b.p = p;
  b.nbits = 8ull * n;
  bits_at(b, 0);
  uint8_t* lengths = reinterpret_cast<uint8_t*>(T + kLengths);
  uint64_t outpos = 0;
  Code lc, dc;
  int last;
  do {
    last = (int)getbits(b, 1);
    const int type = (int)getbits(b, 2);
    if (b.pos > b.nbits) return -1;
    if (type == 0) {  // stored: byte-aligned LEN, NLEN, then LEN raw bytes
      drop(b, (uint32_t)((8 - (b.pos & 7)) & 7));
      const uint64_t q = b.pos >> 3;
      if (q + 4 > n) return -1;
      const uint32_t len = p[q] | (uint32_t)p[q + 1] << 8;
      const uint32_t nlen = p[q + 2] | (uint32_t)p[q + 3] << 8;
      if (len != (~nlen & 0xffffu) || q + 4 + len > n || outpos + len > cap) return -1;
      if (WRITE)
        for (uint32_t k = 0; k < len; k++) out[outpos + k] = p[q + 4 + k];
      outpos += len;
      bits_at(b, q + 4 + len);
    } else if (type == 1) {  // fixed Huffman codes
      for (int s = 0; s < 144; s++) lengths[s] = 8;
      for (int s = 144; s < 256; s++) lengths[s] = 9;
      for (int s = 256; s < 280; s++) lengths[s] = 7;
      for (int s = 280; s < kFixLCodes; s++) lengths[s] = 8;
      construct(T + kLenCnt, T + kLenSym, T + kOffs, lengths, kFixLCodes);
      code_regs(T + kLenCnt, lc);
      if (FAST) fast_table(T + kFastL, kFastLBits, T + kOffs, lengths, kFixLCodes, lc);
      for (int s = 0; s < kMaxDCodes; s++) lengths[s] = 5;
      construct(T + kDistCnt, T + kDistSym, T + kOffs, lengths, kMaxDCodes);
      code_regs(T + kDistCnt, dc);
      if (FAST) fast_table(T + kFastD, kFastDBits, T + kOffs, lengths, kMaxDCodes, dc);
      if (!codes<WRITE, FAST>(b, lc, dc, T, out, outpos, cap)) return -1;
    } else if (type == 2) {  // dynamic Huffman codes
      const int nlen = (int)getbits(b, 5) + 257, ndist = (int)getbits(b, 5) + 1, ncode = (int)getbits(b, 4) + 4;
      if (b.pos > b.nbits || nlen > kMaxLCodes || ndist > kMaxDCodes) return -1;
      for (int k = 0; k < 19; k++) lengths[c_clorder[k]] = k < ncode ? (uint8_t)getbits(b, 3) : (uint8_t)0;
      // code-length code in the distance tables (free until the distance code is built)
      if (construct(T + kDistCnt, T + kDistSym, T + kOffs, lengths, 19) != 0) return -1;
      code_regs(T + kDistCnt, dc);
      int idx = 0;
      while (idx < nlen + ndist) {
        int sym = decode(b, dc, T + kDistSym);
        if (sym < 0 || b.pos > b.nbits) return -1;
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
      if (b.pos > b.nbits) return -1;
      if (lengths[256] == 0) return -1;  // no end-of-block code
      const int el = construct(T + kLenCnt, T + kLenSym, T + kOffs, lengths, nlen);
      if (el < 0 || (el > 0 && nlen != T[kLenCnt + 0] + T[kLenCnt + 1])) return -1;  // incomplete: one code only
      code_regs(T + kLenCnt, lc);
      if (FAST) fast_table(T + kFastL, kFastLBits, T + kOffs, lengths, nlen, lc);
      // distance code from lengths[nlen ..]: copy down first (construct reads lengths[0 .. ndist))
      for (int k = 0; k < ndist; k++) lengths[k] = lengths[nlen + k];
      const int ed = construct(T + kDistCnt, T + kDistSym, T + kOffs, lengths, ndist);
      if (ed < 0 || (ed > 0 && ndist != T[kDistCnt + 0] + T[kDistCnt + 1])) return -1;
      code_regs(T + kDistCnt, dc);
      if (FAST) fast_table(T + kFastD, kFastDBits, T + kOffs, lengths, ndist, dc);
      if (!codes<WRITE, FAST>(b, lc, dc, T, out, outpos, cap)) return -1;
    } else {
      return -1;
    }
  } while (!last);
  return b.pos > b.nbits ? -1 : (int64_t)outpos;
}


}  // namespace amz
