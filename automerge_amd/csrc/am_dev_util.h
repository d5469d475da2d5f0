// am_dev_util.h -- device-side primitives for the Automerge engine (gfx950, wave64).
//   SHA-256, LEB128 readers/writers with the reference's exact range checks, a sequential
//   column decoder (RLE/delta/boolean, encoding.js:789-1207) used one column per lane, and
//   block-level scan / bitonic sort helpers.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "am_common.h"

#define TRY(x) do { uint32_t _e = (x); if (_e) return _e; } while (0)

// ------------------------------------------------------------------------------------------
// SHA-256 (FIPS 180-4), one message per thread; bytes are read from global memory.
// ------------------------------------------------------------------------------------------
__device__ __constant__ static const uint32_t kSha256K[64] = {
  0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
  0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
  0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
  0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
  0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
  0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
  0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
  0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

__device__ __forceinline__ uint32_t rotr(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, n); }

__device__ __forceinline__ void sha256_compress(uint32_t h[8], uint32_t w[16]) {
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
#pragma unroll
  for (int i = 0; i < 64; i++) {
    uint32_t wi;
    if (i < 16) {
      wi = w[i];
    } else {
      uint32_t w15 = w[(i + 1) & 15], w2 = w[(i + 14) & 15];
      uint32_t s0 = rotr(w15, 7) ^ rotr(w15, 18) ^ (w15 >> 3);
      uint32_t s1 = rotr(w2, 17) ^ rotr(w2, 19) ^ (w2 >> 10);
      wi = w[i & 15] + s0 + w[(i + 9) & 15] + s1;
      w[i & 15] = wi;
    }
    uint32_t t1 = hh + (rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25)) + ((e & f) ^ (~e & g)) + kSha256K[i] + wi;
    uint32_t t2 = (rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
    hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

// Hash of p[0..len): message words come from aligned 32-bit loads funnel-shifted by the
// message's byte misalignment (v_alignbyte, shift in bytes), 17 loads per 64-byte block instead of 64 byte
// loads. Reads up to 4 bytes past the last message byte's word: every caller's buffer has slack
// (the arena and the staging slices carry >= 16 bytes of it).
__device__ __forceinline__ void sha256_words(const uint8_t* p, uint64_t len, uint32_t h[8]) {
  h[0] = 0x6a09e667; h[1] = 0xbb67ae85; h[2] = 0x3c6ef372; h[3] = 0xa54ff53a;
  h[4] = 0x510e527f; h[5] = 0x9b05688c; h[6] = 0x1f83d9ab; h[7] = 0x5be0cd19;
  const uint32_t sh = (uint32_t)((uintptr_t)p & 3);
  const uint32_t* w0 = reinterpret_cast<const uint32_t*>(p - sh);
  // little-endian word of message bytes [4k, 4k + 4)
  auto word_le = [&](uint64_t k) -> uint32_t {
    const uint32_t lo = w0[k], hi = w0[k + 1];
    return sh ? __builtin_amdgcn_alignbyte(hi, lo, sh) : lo;
  };
  uint32_t w[16];
  const uint64_t nfull = len / 64;
  for (uint64_t blk = 0; blk < nfull; blk++) {
    uint32_t lo = w0[16 * blk];
#pragma unroll
    for (int i = 0; i < 16; i++) {
      const uint32_t hi = w0[16 * blk + i + 1];
      w[i] = __builtin_bswap32(sh ? __builtin_amdgcn_alignbyte(hi, lo, sh) : lo);
      lo = hi;
    }
    sha256_compress(h, w);
  }
  const uint32_t rem = (uint32_t)(len - nfull * 64);
  const uint64_t kt = 16 * nfull;  // first word of the tail
  const int nblk = (rem + 9 <= 64) ? 1 : 2;
  const uint64_t bits = len * 8;
  for (int b = 0; b < nblk; b++) {
#pragma unroll
    for (int i = 0; i < 16; i++) {
      const uint32_t pos = 64 * b + 4 * i;  // tail byte position of this word
      uint32_t le = 0;
      if (pos < rem) {
        le = word_le(kt + 16 * b + i);
        const uint32_t cnt = rem - pos;
        if (cnt < 4) le = (le & ((1u << (8 * cnt)) - 1)) | (0x80u << (8 * cnt));
      } else if (pos == rem) {
        le = 0x80;
      }
      uint32_t be = __builtin_bswap32(le);
      if (b == nblk - 1 && i == 14) be = (uint32_t)(bits >> 32);
      if (b == nblk - 1 && i == 15) be = (uint32_t)bits;
      w[i] = be;
    }
    sha256_compress(h, w);
  }
}
__device__ static void sha256_dev(const uint8_t* p, uint64_t len, uint8_t out[32]) {
  uint32_t h[8];
  sha256_words(p, len, h);
#pragma unroll
  for (int k = 0; k < 8; k++) {
    out[4 * k] = h[k] >> 24; out[4 * k + 1] = h[k] >> 16; out[4 * k + 2] = h[k] >> 8; out[4 * k + 3] = h[k];
  }
}

// ------------------------------------------------------------------------------------------
// LEB128 (encoding.js:341-488): exact range checks of readUint53 / readInt53.
// ------------------------------------------------------------------------------------------
struct Rd {
  const uint8_t* p;
  uint64_t n;
  uint64_t off;
};

__device__ __forceinline__ uint32_t leb_u64(Rd& d, uint32_t& hi, uint32_t& lo) {
  uint32_t low = 0, high = 0;
  int shift = 0;
  while (d.off < d.n && shift <= 28) {
    uint8_t b = d.p[d.off];
    low |= (uint32_t)(b & 0x7f) << shift;
    if (shift == 28) high = (b & 0x70) >> 4;
    shift += 7;
    d.off++;
    if (!(b & 0x80)) { hi = high; lo = low; return AM_OK; }
  }
  shift = 3;
  while (d.off < d.n) {
    uint8_t b = d.p[d.off];
    if (shift == 31 && (b & 0xfe) != 0) return AM_E_LEB_RANGE;
    high |= (uint32_t)(b & 0x7f) << shift;
    shift += 7;
    d.off++;
    if (!(b & 0x80)) { hi = high; lo = low; return AM_OK; }
  }
  return AM_E_LEB_INCOMPLETE;
}
__device__ __forceinline__ uint32_t leb_i64(Rd& d, int32_t& hi, uint32_t& lo) {
  uint32_t low = 0;
  int32_t high = 0;
  int shift = 0;
  while (d.off < d.n && shift <= 28) {
    uint8_t b = d.p[d.off];
    low |= (uint32_t)(b & 0x7f) << shift;
    if (shift == 28) high = (b & 0x70) >> 4;
    shift += 7;
    d.off++;
    if (!(b & 0x80)) {
      if (b & 0x40) {
        if (shift < 32) low |= 0xffffffffu << shift;
        int s2 = shift - 32 > 0 ? shift - 32 : 0;
        high |= (int32_t)(0xffffffffu << s2);
      }
      hi = high; lo = low;
      return AM_OK;
    }
  }
  shift = 3;
  while (d.off < d.n) {
    uint8_t b = d.p[d.off];
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
__device__ __forceinline__ uint32_t rd_u53(Rd& d, int64_t& v) {
  // fast path: single byte
  if (d.off < d.n) {
    uint8_t b = d.p[d.off];
    if (!(b & 0x80)) { d.off++; v = b; return AM_OK; }
  }
  uint32_t hi, lo;
  TRY(leb_u64(d, hi, lo));
  if (hi > 0x1fffff) return AM_E_LEB_RANGE;
  v = (int64_t)hi * 4294967296LL + lo;
  return AM_OK;
}
__device__ __forceinline__ uint32_t rd_i53(Rd& d, int64_t& v) {
  if (d.off < d.n) {
    uint8_t b = d.p[d.off];
    if (!(b & 0x80)) { d.off++; v = (b & 0x40) ? (int64_t)b - 128 : (int64_t)b; return AM_OK; }
  }
  int32_t hi;
  uint32_t lo;
  TRY(leb_i64(d, hi, lo));
  if (hi < -0x200000 || (hi == -0x200000 && lo == 0) || hi > 0x1fffff) return AM_E_LEB_RANGE;
  v = (int64_t)hi * 4294967296LL + lo;
  return AM_OK;
}
__device__ __forceinline__ uint32_t rd_raw(Rd& d, uint64_t n, uint64_t& at) {
  if (d.off + n > d.n) return AM_E_SUBARRAY;
  at = d.off;
  d.off += n;
  return AM_OK;
}

// LEB128 writers: minimal unsigned / signed forms (encoding.js:97-226)
__device__ __forceinline__ int uleb_len(uint64_t v) {
  int n = 1;
  while (v >= 0x80) { v >>= 7; n++; }
  return n;
}
__device__ __forceinline__ int sleb_len(int64_t v) {
  int n = 1;
  for (;;) {
    uint8_t b = v & 0x7f;
    v >>= 7;
    if ((v == 0 && !(b & 0x40)) || (v == -1 && (b & 0x40))) return n;
    n++;
  }
}
__device__ __forceinline__ uint8_t* put_uleb(uint8_t* o, uint64_t v) {
  do { uint8_t b = v & 0x7f; v >>= 7; *o++ = b | (v ? 0x80 : 0); } while (v);
  return o;
}
__device__ __forceinline__ uint8_t* put_sleb(uint8_t* o, int64_t v) {
  for (;;) {
    uint8_t b = v & 0x7f;
    v >>= 7;
    if ((v == 0 && !(b & 0x40)) || (v == -1 && (b & 0x40))) { *o++ = b; return o; }
    *o++ = b | 0x80;
  }
}

// ------------------------------------------------------------------------------------------
// Sequential column decoder (one column stream per lane).
// RLEDecoder / DeltaDecoder / BooleanDecoder with the canonical-form checks of
// encoding.js:820-886, 1025-1030, 1171-1183.
// ------------------------------------------------------------------------------------------
enum : uint8_t { DT_UINT = 0, DT_INT = 1, DT_UTF8 = 2, DT_DELTA = 3, DT_BOOL = 4 };

struct ColDec {
  Rd r;
  int64_t count;
  int64_t last;         // last value (ints) or byte offset of last string
  int64_t absolute;     // delta running value
  uint32_t last_len;    // utf8
  uint8_t type, state;  // state: 0 undefined 1 repetition 2 literal 3 nulls
  uint8_t has_last, last_null;
  uint8_t blast, bfirst;
};

__device__ __forceinline__ void cd_init(ColDec& d, uint8_t type, const uint8_t* p, uint64_t n) {
  d.r.p = p; d.r.n = n; d.r.off = 0;
  d.count = 0; d.last = 0; d.absolute = 0; d.last_len = 0;
  d.type = type; d.state = 0; d.has_last = 0; d.last_null = 0;
  d.blast = 1; d.bfirst = 1;
}
__device__ __forceinline__ bool cd_done(const ColDec& d) { return d.count == 0 && d.r.off == d.r.n; }

__device__ __forceinline__ bool bytes_eq(const uint8_t* a, const uint8_t* b, uint32_t n) {
  for (uint32_t i = 0; i < n; i++) if (a[i] != b[i]) return false;
  return true;
}

// reads one raw value: ints -> v; utf8 -> v = offset of bytes, len
__device__ __forceinline__ uint32_t cd_raw(ColDec& d, int64_t& v, uint32_t& len) {
  if (d.type == DT_UTF8) {
    int64_t l;
    TRY(rd_u53(d.r, l));
    uint64_t at;
    TRY(rd_raw(d.r, (uint64_t)l, at));
    v = (int64_t)at;
    len = (uint32_t)l;
    return AM_OK;
  }
  if (d.type == DT_UINT) return rd_u53(d.r, v);
  return rd_i53(d.r, v);
}
__device__ __forceinline__ bool cd_eq(const ColDec& d, int64_t a, uint32_t alen, int64_t b, uint32_t blen) {
  if (d.type == DT_UTF8) return alen == blen && bytes_eq(d.r.p + a, d.r.p + b, alen);
  return a == b;
}
__device__ __forceinline__ uint32_t cd_record(ColDec& d) {
  TRY(rd_i53(d.r, d.count));
  if (d.count > 1) {
    int64_t v;
    uint32_t len = 0;
    TRY(cd_raw(d, v, len));
    if ((d.state == 1 || d.state == 2) && d.has_last && !d.last_null && cd_eq(d, v, len, d.last, d.last_len))
      return AM_E_RLE_SUCC_REP;
    d.state = 1;
    d.last = v; d.last_len = len; d.has_last = 1; d.last_null = 0;
  } else if (d.count == 1) {
    return AM_E_RLE_REP1;
  } else if (d.count < 0) {
    d.count = -d.count;
    if (d.state == 2) return AM_E_RLE_SUCC_LIT;
    d.state = 2;
  } else {
    if (d.state == 3) return AM_E_RLE_SUCC_NULL;
    TRY(rd_u53(d.r, d.count));
    if (d.count == 0) return AM_E_RLE_ZERO_NULL;
    d.has_last = 1; d.last_null = 1;
    d.state = 3;
  }
  return AM_OK;
}
// Next value of an RLE/delta integer column. isnull set for nulls (and when exhausted).
__device__ __forceinline__ uint32_t cd_next(ColDec& d, int64_t& v, bool& isnull, uint32_t& len) {
  if (cd_done(d)) { isnull = true; v = 0; len = 0; return AM_OK; }
  if (d.count == 0) TRY(cd_record(d));
  d.count--;
  int64_t val;
  uint32_t l = 0;
  bool nul;
  if (d.state == 2) {
    TRY(cd_raw(d, val, l));
    if (d.has_last && !d.last_null && cd_eq(d, val, l, d.last, d.last_len)) return AM_E_RLE_LIT_REP;
    d.last = val; d.last_len = l; d.has_last = 1; d.last_null = 0;
    nul = false;
  } else {
    nul = d.last_null;
    val = d.last;
    l = d.last_len;
  }
  isnull = nul;
  v = val;
  len = l;
  return AM_OK;
}
__device__ __forceinline__ uint32_t cd_next_int(ColDec& d, int64_t& v) {
  bool isnull;
  uint32_t len;
  TRY(cd_next(d, v, isnull, len));
  if (isnull) { v = AM_NULL64; return AM_OK; }
  return AM_OK;
}
// DeltaDecoder.readValue: nulls do not change the running value.
__device__ __forceinline__ uint32_t cd_next_delta(ColDec& d, int64_t& v) {
  bool isnull;
  uint32_t len;
  int64_t x;
  TRY(cd_next(d, x, isnull, len));
  if (isnull) { v = AM_NULL64; return AM_OK; }
  d.absolute += x;
  v = d.absolute;
  return AM_OK;
}
__device__ __forceinline__ uint32_t cd_next_str(ColDec& d, uint64_t& off, uint32_t& len) {
  bool isnull;
  int64_t x;
  uint32_t l;
  TRY(cd_next(d, x, isnull, l));
  if (isnull) { off = 0; len = AM_NOSTR; return AM_OK; }
  off = (uint64_t)x;
  len = l;
  return AM_OK;
}
__device__ __forceinline__ uint32_t cd_next_bool(ColDec& d, bool& v) {
  if (cd_done(d)) { v = false; return AM_OK; }
  while (d.count == 0) {
    TRY(rd_u53(d.r, d.count));
    d.blast = !d.blast;
    if (d.count == 0 && !d.bfirst) return AM_E_BOOL_ZERO_RUN;
    d.bfirst = 0;
  }
  d.count--;
  v = d.blast;
  return AM_OK;
}

// Counts values of an RLE uint column without materialising them; also sums the values
// (sum_shift applied) -- used to size rows, group entries and raw value bytes.
__device__ static uint32_t rle_count_sum(const uint8_t* p, uint64_t n, bool is_str, uint64_t& count, uint64_t& sum,
                                         int sum_shift, bool is_signed = false) {
  Rd r{p, n, 0};
  count = 0;
  sum = 0;
  while (r.off < r.n) {
    int64_t c;
    TRY(rd_i53(r, c));
    if (c > 0) {
      int64_t v;
      if (is_str) {
        TRY(rd_u53(r, v));
        uint64_t at;
        TRY(rd_raw(r, (uint64_t)v, at));
      } else if (is_signed) {
        TRY(rd_i53(r, v));
        v = 0;
      } else {
        TRY(rd_u53(r, v));
      }
      count += (uint64_t)c;
      sum += (uint64_t)c * ((uint64_t)v >> sum_shift);
    } else if (c < 0) {
      for (int64_t i = 0; i < -c; i++) {
        int64_t v;
        if (is_signed) { TRY(rd_i53(r, v)); v = 0; } else { TRY(rd_u53(r, v)); }
        if (is_str) {
          uint64_t at;
          TRY(rd_raw(r, (uint64_t)v, at));
        }
        sum += (uint64_t)v >> sum_shift;
      }
      count += (uint64_t)(-c);
    } else {
      int64_t z;
      TRY(rd_u53(r, z));
      count += (uint64_t)z;
    }
  }
  return AM_OK;
}

__device__ __forceinline__ uint32_t rle_count_sum_i(const uint8_t* p, uint64_t n, bool is_str, uint64_t& count, uint64_t& sum,
                                                int sum_shift, bool is_signed = false) {
  uint32_t st;
  [[clang::always_inline]] st = rle_count_sum(p, n, is_str, count, sum, sum_shift, is_signed);
  return st;
}

// UTF-8 well-formedness (WHATWG decoder would substitute U+FFFD otherwise)
__device__ __forceinline__ static bool utf8_valid_dev(const uint8_t* s, uint32_t n) {
  uint32_t i = 0;
  while (i < n) {
    uint8_t b = s[i];
    if (b < 0x80) { i++; continue; }
    int need;
    uint8_t lo = 0x80, hi = 0xbf;
    if (b >= 0xc2 && b <= 0xdf) need = 1;
    else if (b >= 0xe0 && b <= 0xef) { need = 2; if (b == 0xe0) lo = 0xa0; if (b == 0xed) hi = 0x9f; }
    else if (b >= 0xf0 && b <= 0xf4) { need = 3; if (b == 0xf0) lo = 0x90; if (b == 0xf4) hi = 0x8f; }
    else return false;
    for (int k = 1; k <= need; k++) {
      if (i + k >= n) return false;
      uint8_t c = s[i + k];
      if (c < lo || c > hi) return false;
      lo = 0x80; hi = 0xbf;
    }
    i += need + 1;
  }
  return true;
}
// TextDecoder('utf-8').decode + TextEncoder.encode (encoding.js:11-17): every maximal subpart of an
// ill-formed sequence becomes U+FFFD (EF BF BD), per the WHATWG UTF-8 decoder. Returns the output
// length; `out` null only measures.
__device__ static uint32_t utf8_sanitize_dev(const uint8_t* in, uint32_t n, uint8_t* out) {
  uint32_t o = 0, i = 0;
  while (i < n) {
    const uint8_t b = in[i];
    if (b < 0x80) { if (out) out[o] = b; o++; i++; continue; }
    uint32_t need;
    uint8_t lo = 0x80, hi = 0xbf;
    if (b >= 0xc2 && b <= 0xdf) need = 1;
    else if (b >= 0xe0 && b <= 0xef) { need = 2; if (b == 0xe0) lo = 0xa0; if (b == 0xed) hi = 0x9f; }
    else if (b >= 0xf0 && b <= 0xf4) { need = 3; if (b == 0xf0) lo = 0x90; if (b == 0xf4) hi = 0x8f; }
    else need = 0;
    uint32_t k = 1;
    if (need) {
      for (; k <= need; k++) {
        if (i + k >= n) break;
        const uint8_t c = in[i + k];
        if (c < lo || c > hi) break;
        lo = 0x80; hi = 0xbf;
      }
    }
    if (need && k > need) {
      if (out) for (uint32_t q = 0; q <= need; q++) out[o + q] = in[i + q];
      o += need + 1;
      i += need + 1;
    } else {  // the bytes read so far are one maximal subpart; the offending byte is read again
      if (out) { out[o] = 0xef; out[o + 1] = 0xbf; out[o + 2] = 0xbd; }
      o += 3;
      i += k;
    }
  }
  return o;
}
// JS string `<` on valid UTF-8: compares UTF-16 code units (new.js:84,1159).
__device__ __forceinline__ uint32_t utf8_cp(const uint8_t* s, uint32_t& i) {
  uint8_t b = s[i];
  if (b < 0x80) { i += 1; return b; }
  if (b < 0xe0) { uint32_t c = ((b & 0x1f) << 6) | (s[i + 1] & 0x3f); i += 2; return c; }
  if (b < 0xf0) { uint32_t c = ((b & 0x0f) << 12) | ((s[i + 1] & 0x3f) << 6) | (s[i + 2] & 0x3f); i += 3; return c; }
  uint32_t c = ((b & 0x07) << 18) | ((s[i + 1] & 0x3f) << 12) | ((s[i + 2] & 0x3f) << 6) | (s[i + 3] & 0x3f);
  i += 4;
  return c;
}
__device__ static int utf16_cmp_dev(const uint8_t* a, uint32_t an, const uint8_t* b, uint32_t bn) {
  uint32_t i = 0, j = 0, pa = 0, pb = 0;
  for (;;) {
    uint32_t ua, ub;
    if (pa) { ua = pa; pa = 0; }
    else if (i < an) {
      uint32_t cp = utf8_cp(a, i);
      if (cp >= 0x10000) { cp -= 0x10000; ua = 0xd800 + (cp >> 10); pa = 0xdc00 + (cp & 0x3ff); } else ua = cp;
    } else ua = 0xffffffffu;
    if (pb) { ub = pb; pb = 0; }
    else if (j < bn) {
      uint32_t cp = utf8_cp(b, j);
      if (cp >= 0x10000) { cp -= 0x10000; ub = 0xd800 + (cp >> 10); pb = 0xdc00 + (cp & 0x3ff); } else ub = cp;
    } else ub = 0xffffffffu;
    if (ua == 0xffffffffu && ub == 0xffffffffu) return 0;
    if (ua == 0xffffffffu) return -1;
    if (ub == 0xffffffffu) return 1;
    if (ua != ub) return ua < ub ? -1 : 1;
  }
}
// actor ids compare as hex strings == bytewise with shorter prefix first
__device__ __forceinline__ int actor_cmp_dev(const uint8_t* a, uint32_t an, const uint8_t* b, uint32_t bn) {
  uint32_t m = an < bn ? an : bn;
  for (uint32_t i = 0; i < m; i++) if (a[i] != b[i]) return a[i] < b[i] ? -1 : 1;
  return an < bn ? -1 : (an > bn ? 1 : 0);
}

// ------------------------------------------------------------------------------------------
// Block-level helpers (blockDim.x threads, any n; arrays live in global workspace)
// ------------------------------------------------------------------------------------------
// Exclusive scan of u32 counts in place; returns the total (to every thread).
__device__ static uint32_t block_excl_scan(uint32_t* a, uint32_t n, uint32_t* s_tmp /* >= blockDim+1 */) {
  uint32_t carry = 0;
  const uint32_t T = blockDim.x, t = threadIdx.x;
  for (uint32_t base = 0; base < n; base += T) {
    uint32_t i = base + t;
    uint32_t v = i < n ? a[i] : 0;
    s_tmp[t] = v;
    __syncthreads();
    for (uint32_t off = 1; off < T; off <<= 1) {
      uint32_t x = t >= off ? s_tmp[t - off] : 0;
      __syncthreads();
      s_tmp[t] += x;
      __syncthreads();
    }
    uint32_t incl = s_tmp[t];
    uint32_t tot = s_tmp[T - 1];
    if (i < n) a[i] = carry + incl - v;
    __syncthreads();
    carry += tot;
  }
  return carry;
}

// Stable LSD radix sort of n (key, val) pairs by the low `bits` bits of the keys, 8-bit digits, by
// the whole block (blockDim.x a multiple of 64, at most 64 * MaxW). k0 / v0 hold the input and on return
// the sorted pairs; k1 / v1 are scratch of n entries. Per digit: an LDS histogram, its exclusive
// scan, then tiles of blockDim.x pairs scattered in order -- a pair's place is its bucket's base,
// the same-digit pairs of earlier waves of the tile and its rank among its wave's same-digit lanes
// (eight ballots). A digit every key shares is skipped. O(n) per digit against bitonic's
// O(n log^2 n) compare-exchanges, for the large documents' id and document-order sorts.
template <uint32_t MaxW = 4>  // waves of the block (blockDim.x <= 64 * MaxW)
__device__ static void block_radix_sort(uint64_t* k0, uint32_t* v0, uint64_t* k1, uint32_t* v1, uint32_t n, uint32_t bits) {
  __shared__ uint32_t s_hist[256];
  __shared__ uint32_t s_wc[MaxW * 256];
  __shared__ uint32_t s_skip;
  const uint32_t T = blockDim.x, t = threadIdx.x, w = t >> 6, lane = t & 63, W = T >> 6;
  uint64_t* ka = k0;
  uint32_t* va = v0;
  uint64_t* kb = k1;
  uint32_t* vb = v1;
  for (uint32_t sh = 0; sh < bits; sh += 8) {
    for (uint32_t d = t; d < 256; d += T) s_hist[d] = 0;
    if (t == 0) s_skip = 0;
    __syncthreads();
    for (uint32_t i = t; i < n; i += T) atomicAdd(&s_hist[(uint32_t)(ka[i] >> sh) & 255u], 1u);
    __syncthreads();
    if (t == 0) {  // exclusive scan of the 256 buckets; one bucket holding every key: nothing to do
      uint32_t run = 0;
      for (uint32_t d = 0; d < 256; d++) {
        const uint32_t c = s_hist[d];
        if (c == n) s_skip = 1;
        s_hist[d] = run;
        run += c;
      }
    }
    __syncthreads();
    const bool skip = s_skip != 0;
    __syncthreads();  // every thread has read s_skip before the next pass resets it
    if (skip) continue;
    for (uint32_t b0 = 0; b0 < n; b0 += T) {
      const uint32_t i = b0 + t;
      const bool act = i < n;
      const uint64_t key = act ? ka[i] : 0;
      const uint32_t val = act ? va[i] : 0;
      const uint32_t dg = (uint32_t)(key >> sh) & 255u;
      uint64_t peers = __ballot(act);
#pragma unroll
      for (int bt = 0; bt < 8; bt++) {
        const uint64_t m = __ballot(act && ((dg >> bt) & 1u));
        peers &= ((dg >> bt) & 1u) ? m : ~m;
      }
      const uint32_t rank = (uint32_t)__popcll(peers & ((1ull << lane) - 1ull));
      for (uint32_t x = t; x < W * 256; x += T) s_wc[x] = 0;
      __syncthreads();
      if (act && rank == 0) s_wc[w * 256 + dg] = (uint32_t)__popcll(peers);
      __syncthreads();
      if (act) {
        uint32_t off = s_hist[dg] + rank;
        for (uint32_t q = 0; q < w; q++) off += s_wc[q * 256 + dg];
        kb[off] = key;
        vb[off] = val;
      }
      __syncthreads();
      for (uint32_t d = t; d < 256; d += T) {
        uint32_t c = 0;
        for (uint32_t q = 0; q < W; q++) c += s_wc[q * 256 + d];
        s_hist[d] += c;
      }
      __syncthreads();
    }
    uint64_t* tk = ka; ka = kb; kb = tk;
    uint32_t* tv = va; va = vb; vb = tv;
  }
  if (ka != k0) {  // an odd number of scatters: the result is in the scratch arrays
    for (uint32_t i = t; i < n; i += T) { k0[i] = ka[i]; v0[i] = va[i]; }
    __syncthreads();
  }
}

// Bitonic sort of a[0..P) (P power of two, padded with elements that compare as +inf).
template <typename T, typename Less>
__device__ static void block_bitonic_sort(T* a, uint32_t P, Less less) {
  // Each lane keeps kU compare-exchange pairs in flight (loads first, then the swaps): the pairs
  // of one step are disjoint, and for documents whose keys live in global memory the step is
  // latency-bound, so memory-level parallelism is what sets its speed.
  constexpr uint32_t kU = 4;
  const uint32_t B = blockDim.x;
  for (uint32_t k = 2; k <= P; k <<= 1) {
    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
      for (uint32_t i0 = threadIdx.x; i0 < P; i0 += kU * B) {
        T x[kU], y[kU];
        bool act[kU];
#pragma unroll
        for (uint32_t u = 0; u < kU; u++) {
          const uint32_t i = i0 + u * B, l = i ^ j;
          act[u] = i < P && l > i;
          if (act[u]) { x[u] = a[i]; y[u] = a[l]; }
        }
#pragma unroll
        for (uint32_t u = 0; u < kU; u++) {
          const uint32_t i = i0 + u * B, l = i ^ j;
          if (act[u]) {
            const bool asc = (i & k) == 0;
            const bool sw = asc ? less(y[u], x[u]) : less(x[u], y[u]);
            if (sw) { a[i] = y[u]; a[l] = x[u]; }
          }
        }
      }
      __syncthreads();
    }
  }
}

__host__ __device__ inline uint32_t pow2_ceil(uint32_t n) {
  uint32_t p = 1;
  while (p < n) p <<= 1;
  return p;
}

// ------------------------------------------------------------------------------------------
// Wave64 scans (the document workgroup is exactly one wave: blockDim.x == 64)
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t wave_incl_add(uint32_t v) {
  const uint32_t lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint32_t x = __shfl_up(v, d, 64);
    if (lane >= (uint32_t)d) v += x;
  }
  return v;
}
__device__ __forceinline__ int32_t wave_incl_max(int32_t v) {
  const uint32_t lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    int32_t x = __shfl_up(v, d, 64);
    if (lane >= (uint32_t)d && x > v) v = x;
  }
  return v;
}
// exclusive add-scan of a[0..n) in place (one wave); returns the total
__device__ static uint32_t wave_excl_scan_arr(uint32_t* a, uint32_t n) {
  uint32_t carry = 0;
  for (uint32_t base = 0; base < n; base += 64) {
    const uint32_t i = base + threadIdx.x;
    const uint32_t v = i < n ? a[i] : 0;
    const uint32_t inc = wave_incl_add(v);
    if (i < n) a[i] = carry + inc - v;
    carry += __shfl(inc, 63, 64);
  }
  return carry;
}
