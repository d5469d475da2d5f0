// am_host_codec.h -- host-side Automerge binary codecs shared by the host stages (the synthetic
// workload generator and the change-history reconstruction): SHA-256, LEB128, the canonical RLE /
// delta / boolean column encoders (encoding.js:97-278, 558-1207) and the container
// (columnar.js:659-686). Host code only; the GPU path has its own (am_dev_util.h).
#pragma once
#include <stdint.h>
#include <string.h>

#include <string>
#include <vector>

namespace {

// ---------------- SHA-256 (change hashes are part of the generated change headers) -------------
struct Sha {
  static uint32_t ror(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
  static void block(uint32_t h[8], const uint8_t* p) {
    static const uint32_t K[64] = {
        0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5, 0xd807aa98,
        0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174, 0xe49b69c1, 0xefbe4786,
        0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da, 0x983e5152, 0xa831c66d, 0xb00327c8,
        0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967, 0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13,
        0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85, 0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819,
        0xd6990624, 0xf40e3585, 0x106aa070, 0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a,
        0x5b9cca4f, 0x682e6ff3, 0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7,
        0xc67178f2};
    uint32_t w[64];
    for (int i = 0; i < 16; i++) w[i] = (uint32_t)p[4 * i] << 24 | (uint32_t)p[4 * i + 1] << 16 | (uint32_t)p[4 * i + 2] << 8 | p[4 * i + 3];
    for (int i = 16; i < 64; i++)
      w[i] = w[i - 16] + (ror(w[i - 15], 7) ^ ror(w[i - 15], 18) ^ (w[i - 15] >> 3)) + w[i - 7] +
             (ror(w[i - 2], 17) ^ ror(w[i - 2], 19) ^ (w[i - 2] >> 10));
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
    for (int i = 0; i < 64; i++) {
      uint32_t t1 = hh + (ror(e, 6) ^ ror(e, 11) ^ ror(e, 25)) + ((e & f) ^ (~e & g)) + K[i] + w[i];
      uint32_t t2 = (ror(a, 2) ^ ror(a, 13) ^ ror(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
      hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
  }
  static void hash(const uint8_t* data, size_t len, uint8_t out[32]) {
    uint32_t h[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    size_t i = 0;
    for (; i + 64 <= len; i += 64) block(h, data + i);
    uint8_t t[128] = {0};
    size_t rem = len - i;
    memcpy(t, data + i, rem);
    t[rem] = 0x80;
    size_t tl = rem + 9 <= 64 ? 64 : 128;
    uint64_t bits = (uint64_t)len * 8;
    for (int k = 0; k < 8; k++) t[tl - 1 - k] = (uint8_t)(bits >> (8 * k));
    block(h, t);
    if (tl == 128) block(h, t + 64);
    for (int k = 0; k < 8; k++) { out[4 * k] = h[k] >> 24; out[4 * k + 1] = h[k] >> 16; out[4 * k + 2] = h[k] >> 8; out[4 * k + 3] = h[k]; }
  }
};

using Bytes = std::vector<uint8_t>;
void pu(Bytes& o, uint64_t v) { do { uint8_t b = v & 0x7f; v >>= 7; o.push_back(b | (v ? 0x80 : 0)); } while (v); }
void ps(Bytes& o, int64_t v) {
  for (;;) {
    uint8_t b = v & 0x7f;
    v >>= 7;
    if ((v == 0 && !(b & 0x40)) || (v == -1 && (b & 0x40))) { o.push_back(b); return; }
    o.push_back(b | 0x80);
  }
}

// nullable value for the column encoders
struct V { bool null; int64_t i; std::string s; };
V N0() { return {true, 0, {}}; }
V I(int64_t x) { return {false, x, {}}; }
V S(const std::string& x) { return {false, 0, x}; }
bool eqv(const V& a, const V& b, bool str) { return a.null == b.null && (a.null || (str ? a.s == b.s : a.i == b.i)); }

// canonical RLE (RLEEncoder, encoding.js:558-783)
Bytes rle(const std::vector<V>& v, int type /*0 uint 1 int 2 utf8*/) {
  Bytes o;
  bool any = false;
  for (auto& x : v) any |= !x.null;
  if (!any) return o;
  auto put = [&](const V& x) {
    if (type == 2) { pu(o, x.s.size()); o.insert(o.end(), x.s.begin(), x.s.end()); }
    else if (type == 1) ps(o, x.i);
    else pu(o, (uint64_t)x.i);
  };
  size_t n = v.size(), i = 0;
  while (i < n) {
    size_t j = i + 1;
    while (j < n && eqv(v[j], v[i], type == 2)) j++;
    if (v[i].null) { ps(o, 0); pu(o, j - i); i = j; continue; }
    if (j - i >= 2) { ps(o, (int64_t)(j - i)); put(v[i]); i = j; continue; }
    size_t k = i;
    while (k < n && !v[k].null && (k + 1 >= n || !eqv(v[k + 1], v[k], type == 2))) k++;
    ps(o, -(int64_t)(k - i));
    for (size_t t = i; t < k; t++) put(v[t]);
    i = k;
  }
  return o;
}
Bytes delta(const std::vector<V>& v) {
  std::vector<V> d;
  int64_t abs = 0;
  for (auto& x : v) {
    if (x.null) d.push_back(N0());
    else { d.push_back(I(x.i - abs)); abs = x.i; }
  }
  return rle(d, 1);
}
Bytes boolean(const std::vector<bool>& v) {
  Bytes o;
  bool last = false;
  uint64_t c = 0;
  for (bool x : v) { if (x == last) c++; else { pu(o, c); last = x; c = 1; } }
  if (c) pu(o, c);
  return o;
}

Bytes container(uint8_t type, const Bytes& body, uint8_t hash_out[32]) {
  Bytes hb;
  hb.push_back(type);
  pu(hb, body.size());
  hb.insert(hb.end(), body.begin(), body.end());
  uint8_t h[32];
  Sha::hash(hb.data(), hb.size(), h);
  if (hash_out) memcpy(hash_out, h, 32);
  Bytes o = {0x85, 0x6f, 0x4a, 0x83, h[0], h[1], h[2], h[3]};
  o.insert(o.end(), hb.begin(), hb.end());
  return o;
}


}  // namespace
