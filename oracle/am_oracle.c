/*
 * am_oracle.c -- sequential CPU restatement of the reference backend hot path (plain C99 + zlib).
 *
 * TEST INFRASTRUCTURE ONLY (see am_oracle.h). It follows the reference's algorithm step by step:
 * every function cites the reference file:line it restates (paths relative to the reference repo).
 * Differences in *method* (not in result): the document is one flat op array instead of 600-op
 * blocks with Bloom filters (new.js:6-8, 227-421), which are not observable through the API.
 */
#include "am_oracle.h"

#include <setjmp.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>

/* ============================================================================================
 * Arena + error handling (one arena per API call; errors longjmp out and free the arena)
 * ============================================================================================ */
typedef struct ablock { struct ablock *next; } ablock;
typedef struct {
  ablock *blocks;
  jmp_buf jb;
  char msg[512];
  int code; /* 1 error, 2 unsupported */
} ctx_t;

static void *amalloc(ctx_t *c, size_t n) {
  ablock *b = (ablock *)malloc(sizeof(ablock) + (n ? n : 1));
  if (!b) { snprintf(c->msg, sizeof c->msg, "out of memory"); c->code = 1; longjmp(c->jb, 1); }
  b->next = c->blocks;
  c->blocks = b;
  return (void *)(b + 1);
}
static void *acalloc(ctx_t *c, size_t n) { void *p = amalloc(c, n); memset(p, 0, n); return p; }
static void afree_all(ctx_t *c) {
  while (c->blocks) { ablock *n = c->blocks->next; free(c->blocks); c->blocks = n; }
}
static void fail(ctx_t *c, const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(c->msg, sizeof c->msg, fmt, ap);
  va_end(ap);
  c->code = 1;
  longjmp(c->jb, 1);
}
static void unsupported(ctx_t *c, const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(c->msg, sizeof c->msg, fmt, ap);
  va_end(ap);
  c->code = 2;
  longjmp(c->jb, 1);
}

/* growable byte buffer (arena-backed) */
typedef struct { uint8_t *p; size_t n, cap; } bbuf;
static void bb_grow(ctx_t *c, bbuf *b, size_t need) {
  if (b->n + need <= b->cap) return;
  size_t nc = b->cap ? b->cap * 2 : 64;
  while (nc < b->n + need) nc *= 2;
  uint8_t *np = (uint8_t *)amalloc(c, nc);
  if (b->n) memcpy(np, b->p, b->n);
  b->p = np;
  b->cap = nc;
}
static void bb_byte(ctx_t *c, bbuf *b, uint8_t v) { bb_grow(c, b, 1); b->p[b->n++] = v; }
static void bb_raw(ctx_t *c, bbuf *b, const uint8_t *p, size_t n) {
  if (!n) return;
  bb_grow(c, b, n);
  memcpy(b->p + b->n, p, n);
  b->n += n;
}

/* ============================================================================================
 * SHA-256 (FIPS 180-4). The reference uses fast-sha256@1.3.0 (columnar.js:21); any SHA-256 is
 * bit-identical, pinned by the checksum bytes in columnar_test.js:17 and every fixture hash.
 * ============================================================================================ */
static const uint32_t K256[64] = {
  0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
  0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
  0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
  0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
  0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
  0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
  0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
  0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
#define ROR(x, n) (((x) >> (n)) | ((x) << (32 - (n))))
static void sha_block(uint32_t h[8], const uint8_t *p) {
  uint32_t w[64];
  for (int i = 0; i < 16; i++)
    w[i] = (uint32_t)p[4 * i] << 24 | (uint32_t)p[4 * i + 1] << 16 | (uint32_t)p[4 * i + 2] << 8 | p[4 * i + 3];
  for (int i = 16; i < 64; i++) {
    uint32_t s0 = ROR(w[i - 15], 7) ^ ROR(w[i - 15], 18) ^ (w[i - 15] >> 3);
    uint32_t s1 = ROR(w[i - 2], 17) ^ ROR(w[i - 2], 19) ^ (w[i - 2] >> 10);
    w[i] = w[i - 16] + s0 + w[i - 7] + s1;
  }
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
  for (int i = 0; i < 64; i++) {
    uint32_t t1 = hh + (ROR(e, 6) ^ ROR(e, 11) ^ ROR(e, 25)) + ((e & f) ^ (~e & g)) + K256[i] + w[i];
    uint32_t t2 = (ROR(a, 2) ^ ROR(a, 13) ^ ROR(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
    hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}
void oc_sha256(const uint8_t *data, size_t len, uint8_t out[32]) {
  uint32_t h[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  size_t i = 0;
  for (; i + 64 <= len; i += 64) sha_block(h, data + i);
  uint8_t tail[128];
  size_t rem = len - i;
  memcpy(tail, data + i, rem);
  tail[rem] = 0x80;
  size_t tl = (rem + 9 <= 64) ? 64 : 128;
  memset(tail + rem + 1, 0, tl - rem - 1);
  uint64_t bits = (uint64_t)len * 8;
  for (int k = 0; k < 8; k++) tail[tl - 1 - k] = (uint8_t)(bits >> (8 * k));
  sha_block(h, tail);
  if (tl == 128) sha_block(h, tail + 64);
  for (int k = 0; k < 8; k++) {
    out[4 * k] = h[k] >> 24; out[4 * k + 1] = h[k] >> 16; out[4 * k + 2] = h[k] >> 8; out[4 * k + 3] = h[k];
  }
}

/* ============================================================================================
 * LEB128 decoding with the reference's exact range checks (encoding.js:341-488)
 * ============================================================================================ */
typedef struct { const uint8_t *p; size_t n, off; } rd_t;

static const char *E_RANGE = "number out of range";
static const char *E_INCOMPLETE = "buffer ended with incomplete number";

/* Returns NULL on success, else an error message. Restates Decoder.readUint64 (encoding.js:416). */
static const char *leb_u64(rd_t *d, uint32_t *hi, uint32_t *lo) {
  uint32_t low = 0, high = 0;
  int shift = 0;
  while (d->off < d->n && shift <= 28) {
    uint8_t b = d->p[d->off];
    low |= (uint32_t)(b & 0x7f) << shift;
    if (shift == 28) high = (b & 0x70) >> 4;
    shift += 7;
    d->off++;
    if (!(b & 0x80)) { *hi = high; *lo = low; return NULL; }
  }
  shift = 3;
  while (d->off < d->n) {
    uint8_t b = d->p[d->off];
    if (shift == 31 && (b & 0xfe) != 0) return E_RANGE;
    high |= (uint32_t)(b & 0x7f) << shift;
    shift += 7;
    d->off++;
    if (!(b & 0x80)) { *hi = high; *lo = low; return NULL; }
  }
  return E_INCOMPLETE;
}
/* Restates Decoder.readInt64 (encoding.js:450); hi is a signed 32-bit half. */
static const char *leb_i64(rd_t *d, int32_t *hi, uint32_t *lo) {
  uint32_t low = 0;
  int32_t high = 0;
  int shift = 0;
  while (d->off < d->n && shift <= 28) {
    uint8_t b = d->p[d->off];
    low |= (uint32_t)(b & 0x7f) << shift;
    if (shift == 28) high = (b & 0x70) >> 4;
    shift += 7;
    d->off++;
    if (!(b & 0x80)) {
      if (b & 0x40) {
        if (shift < 32) low |= 0xffffffffu << shift;
        int s2 = shift - 32 > 0 ? shift - 32 : 0;
        high |= (int32_t)(0xffffffffu << s2);
      }
      *hi = high; *lo = low;
      return NULL;
    }
  }
  shift = 3;
  while (d->off < d->n) {
    uint8_t b = d->p[d->off];
    if (shift == 31 && b != 0 && b != 0x7f) return E_RANGE;
    high |= (int32_t)((uint32_t)(b & 0x7f) << shift);
    shift += 7;
    d->off++;
    if (!(b & 0x80)) {
      if ((b & 0x40) && shift < 32) high |= (int32_t)(0xffffffffu << shift);
      *hi = high; *lo = low;
      return NULL;
    }
  }
  return E_INCOMPLETE;
}
/* readUint53 (encoding.js:389) */
static const char *leb_u53(rd_t *d, int64_t *v) {
  uint32_t hi, lo;
  const char *e = leb_u64(d, &hi, &lo);
  if (e) return e;
  if (hi > 0x1fffff) return E_RANGE;
  *v = (int64_t)hi * 4294967296LL + lo;
  return NULL;
}
/* readInt53 (encoding.js:402) */
static const char *leb_i53(rd_t *d, int64_t *v) {
  int32_t hi;
  uint32_t lo;
  const char *e = leb_i64(d, &hi, &lo);
  if (e) return e;
  if (hi < -0x200000 || (hi == -0x200000 && lo == 0) || hi > 0x1fffff) return E_RANGE;
  *v = (int64_t)hi * 4294967296LL + lo;
  return NULL;
}
/* readUint32 (encoding.js:341) */
static const char *leb_u32(rd_t *d, int64_t *v) {
  uint32_t result = 0;
  int shift = 0;
  while (d->off < d->n) {
    uint8_t b = d->p[d->off];
    if (shift == 28 && (b & 0xf0) != 0) return E_RANGE;
    result |= (uint32_t)(b & 0x7f) << shift;
    shift += 7;
    d->off++;
    if (!(b & 0x80)) { *v = result; return NULL; }
  }
  return E_INCOMPLETE;
}
/* readInt32 (encoding.js:360) */
static const char *leb_i32(rd_t *d, int64_t *v) {
  int32_t result = 0;
  int shift = 0;
  while (d->off < d->n) {
    uint8_t b = d->p[d->off];
    if ((shift == 28 && (b & 0x80) != 0) || (shift == 28 && (b & 0x40) == 0 && (b & 0x38) != 0) ||
        (shift == 28 && (b & 0x40) != 0 && (b & 0x38) != 0x38))
      return E_RANGE;
    result |= (int32_t)((uint32_t)(b & 0x7f) << shift);
    shift += 7;
    d->off++;
    if (!(b & 0x80)) {
      if ((b & 0x40) == 0 || shift > 28) { *v = result; return NULL; }
      *v = result | (int32_t)(0xffffffffu << shift);
      return NULL;
    }
  }
  return E_INCOMPLETE;
}

static int64_t rd_u53(ctx_t *c, rd_t *d) {
  int64_t v;
  const char *e = leb_u53(d, &v);
  if (e) fail(c, "%s", e);
  return v;
}
static int64_t rd_i53(ctx_t *c, rd_t *d) {
  int64_t v;
  const char *e = leb_i53(d, &v);
  if (e) fail(c, "%s", e);
  return v;
}
static const uint8_t *rd_raw(ctx_t *c, rd_t *d, size_t n) {
  if (d->off + n > d->n || d->off + n < d->off) fail(c, "subarray exceeds buffer size");
  const uint8_t *p = d->p + d->off;
  d->off += n;
  return p;
}

/* ---- LEB128 encoding: minimal unsigned / signed forms (encoding.js:97-226) ---- */
static int leb_put_u(uint8_t *o, uint64_t v) {
  int n = 0;
  do { uint8_t b = v & 0x7f; v >>= 7; o[n++] = b | (v ? 0x80 : 0); } while (v);
  return n;
}
static int leb_put_s(uint8_t *o, int64_t v) {
  int n = 0;
  for (;;) {
    uint8_t b = v & 0x7f;
    v >>= 7; /* arithmetic shift */
    if ((v == 0 && !(b & 0x40)) || (v == -1 && (b & 0x40))) { o[n++] = b; return n; }
    o[n++] = b | 0x80;
  }
}
static void bb_u(ctx_t *c, bbuf *b, uint64_t v) { uint8_t t[10]; bb_raw(c, b, t, leb_put_u(t, v)); }
static void bb_s(ctx_t *c, bbuf *b, int64_t v) { uint8_t t[10]; bb_raw(c, b, t, leb_put_s(t, v)); }

/* ============================================================================================
 * UTF-8 canonicalisation. The reference decodes utf8 RLE values to JS strings with TextDecoder
 * (invalid sequences -> U+FFFD, encoding.js:15) and re-encodes them with TextEncoder, compares
 * them with === and orders map keys with JS `<` (UTF-16 code units, new.js:84,1159).
 * ============================================================================================ */
/* Decodes one code point per WHATWG UTF-8 decoder (maximal subpart replacement). */
static uint32_t utf8_next(const uint8_t *s, size_t n, size_t *i) {
  uint8_t b = s[*i];
  if (b < 0x80) { (*i)++; return b; }
  int need;
  uint32_t cp;
  uint8_t lo = 0x80, hi = 0xbf;
  if (b >= 0xc2 && b <= 0xdf) { need = 1; cp = b & 0x1f; }
  else if (b >= 0xe0 && b <= 0xef) { need = 2; cp = b & 0x0f; if (b == 0xe0) lo = 0xa0; if (b == 0xed) hi = 0x9f; }
  else if (b >= 0xf0 && b <= 0xf4) { need = 3; cp = b & 0x07; if (b == 0xf0) lo = 0x90; if (b == 0xf4) hi = 0x8f; }
  else { (*i)++; return 0xfffd; }
  size_t j = *i + 1;
  for (int k = 0; k < need; k++) {
    if (j >= n || s[j] < lo || s[j] > hi) { *i = j; return 0xfffd; }
    cp = (cp << 6) | (s[j] & 0x3f);
    lo = 0x80; hi = 0xbf;
    j++;
  }
  *i = j;
  return cp;
}
static int utf8_valid(const uint8_t *s, size_t n) {
  size_t i = 0;
  while (i < n) {
    size_t st = i;
    uint32_t cp = utf8_next(s, n, &i);
    if (cp == 0xfffd && !(i - st == 3 && s[st] == 0xef && s[st + 1] == 0xbf && s[st + 2] == 0xbd)) return 0;
  }
  return 1;
}
/* Returns canonical UTF-8 (arena copy only if it changes). */
static const uint8_t *utf8_canon(ctx_t *c, const uint8_t *s, uint32_t n, uint32_t *outn) {
  if (utf8_valid(s, n)) { *outn = n; return s; }
  uint8_t *o = (uint8_t *)amalloc(c, (size_t)n * 3 + 1);
  size_t i = 0, k = 0;
  while (i < n) {
    uint32_t cp = utf8_next(s, n, &i);
    if (cp < 0x80) o[k++] = cp;
    else if (cp < 0x800) { o[k++] = 0xc0 | (cp >> 6); o[k++] = 0x80 | (cp & 0x3f); }
    else if (cp < 0x10000) { o[k++] = 0xe0 | (cp >> 12); o[k++] = 0x80 | ((cp >> 6) & 0x3f); o[k++] = 0x80 | (cp & 0x3f); }
    else { o[k++] = 0xf0 | (cp >> 18); o[k++] = 0x80 | ((cp >> 12) & 0x3f); o[k++] = 0x80 | ((cp >> 6) & 0x3f); o[k++] = 0x80 | (cp & 0x3f); }
  }
  *outn = (uint32_t)k;
  return o;
}
/* JS string comparison (UTF-16 code units) of two UTF-8 byte strings. */
static int utf16_cmp(const uint8_t *a, size_t an, const uint8_t *b, size_t bn) {
  size_t i = 0, j = 0;
  uint32_t pa = 0, pb = 0; /* pending low surrogates */
  for (;;) {
    uint32_t ua, ub;
    if (pa) { ua = pa; pa = 0; }
    else if (i < an) {
      uint32_t cp = utf8_next(a, an, &i);
      if (cp >= 0x10000) { cp -= 0x10000; ua = 0xd800 + (cp >> 10); pa = 0xdc00 + (cp & 0x3ff); } else ua = cp;
    } else ua = 0xffffffffu;
    if (pb) { ub = pb; pb = 0; }
    else if (j < bn) {
      uint32_t cp = utf8_next(b, bn, &j);
      if (cp >= 0x10000) { cp -= 0x10000; ub = 0xd800 + (cp >> 10); pb = 0xdc00 + (cp & 0x3ff); } else ub = cp;
    } else ub = 0xffffffffu;
    if (ua == 0xffffffffu && ub == 0xffffffffu) return 0;
    if (ua == 0xffffffffu) return -1;
    if (ub == 0xffffffffu) return 1;
    if (ua != ub) return ua < ub ? -1 : 1;
  }
}

/* ============================================================================================
 * Column value model. A nullable integer (uint/int/delta/actor) or a nullable string.
 * ============================================================================================ */
typedef struct { int64_t v; uint8_t null; } nv;
typedef struct { const uint8_t *p; uint32_t n; uint8_t null; } ns;
static const nv NUL = {0, 1};
static nv NV(int64_t v) { nv r = {v, 0}; return r; }

/* RLE decoder restating RLEDecoder (encoding.js:789-920) incl. canonical checks. */
enum { T_UINT = 0, T_INT = 1, T_UTF8 = 2, T_DELTA = 3, T_BOOL = 4, T_RAW = 5 };
typedef struct {
  rd_t r;
  int type; /* T_UINT / T_INT / T_UTF8 (delta uses T_INT underneath) */
  int state; /* 0 undefined, 1 repetition, 2 literal, 3 nulls */
  int64_t count;
  nv last;
  ns lasts;
  int has_last;
  int64_t absolute; /* delta */
  int delta;
  /* boolean */
  int blast, bfirst;
} coldec;

static void cd_init(coldec *d, int coltype, const uint8_t *p, size_t n) {
  memset(d, 0, sizeof *d);
  d->r.p = p;
  d->r.n = n;
  d->type = coltype == T_DELTA ? T_INT : coltype;
  d->delta = coltype == T_DELTA;
  d->blast = 1;
  d->bfirst = 1;
}
static int cd_done(const coldec *d) { return d->count == 0 && d->r.off == d->r.n; }

static int ns_eq(ns a, ns b) { return a.n == b.n && (a.n == 0 || memcmp(a.p, b.p, a.n) == 0); }

static void cd_raw_value(ctx_t *c, coldec *d, nv *iv, ns *sv) {
  if (d->type == T_INT) *iv = NV(rd_i53(c, &d->r));
  else if (d->type == T_UINT) *iv = NV(rd_u53(c, &d->r));
  else {
    int64_t len = rd_u53(c, &d->r);
    const uint8_t *p = rd_raw(c, &d->r, (size_t)len);
    uint32_t cn;
    const uint8_t *cp = utf8_canon(c, p, (uint32_t)len, &cn);
    sv->p = cp; sv->n = cn; sv->null = 0;
  }
}
static int val_eq(const coldec *d, nv a, ns as, nv b, ns bs) {
  if (d->type == T_UTF8) return ns_eq(as, bs);
  return a.v == b.v;
}
/* readRecord (encoding.js:865) */
static void cd_record(ctx_t *c, coldec *d) {
  d->count = rd_i53(c, &d->r);
  if (d->count > 1) {
    nv v = NUL; ns s = {0, 0, 1};
    cd_raw_value(c, d, &v, &s);
    if ((d->state == 1 || d->state == 2) && d->has_last && val_eq(d, v, s, d->last, d->lasts))
      fail(c, "Successive repetitions with the same value are not allowed");
    d->state = 1;
    d->last = v; d->lasts = s; d->has_last = 1;
  } else if (d->count == 1) {
    fail(c, "Repetition count of 1 is not allowed, use a literal instead");
  } else if (d->count < 0) {
    d->count = -d->count;
    if (d->state == 2) fail(c, "Successive literals are not allowed");
    d->state = 2;
  } else {
    if (d->state == 3) fail(c, "Successive null runs are not allowed");
    d->count = rd_u53(c, &d->r);
    if (d->count == 0) fail(c, "Zero-length null runs are not allowed");
    d->last = NUL; d->lasts.null = 1; d->lasts.n = 0; d->has_last = 1;
    d->state = 3;
  }
}
/* readValue (encoding.js:820) for integer-typed RLE / delta columns */
static nv cd_int(ctx_t *c, coldec *d) {
  if (cd_done(d)) return NUL;
  if (d->count == 0) cd_record(c, d);
  d->count--;
  nv v;
  if (d->state == 2) {
    ns s = {0, 0, 1};
    cd_raw_value(c, d, &v, &s);
    if (d->has_last && !d->last.null && d->last.v == v.v) fail(c, "Repetition of values is not allowed in literal");
    d->last = v; d->has_last = 1;
  } else v = d->last;
  if (d->delta) { /* DeltaDecoder.readValue (encoding.js:1025) */
    if (v.null) return NUL;
    d->absolute += v.v;
    return NV(d->absolute);
  }
  return v;
}
static ns cd_str(ctx_t *c, coldec *d) {
  ns nulls = {0, 0, 1};
  if (cd_done(d)) return nulls;
  if (d->count == 0) cd_record(c, d);
  d->count--;
  if (d->state == 2) {
    nv dummy;
    ns s;
    cd_raw_value(c, d, &dummy, &s);
    if (d->has_last && !d->lasts.null && ns_eq(d->lasts, s)) fail(c, "Repetition of values is not allowed in literal");
    d->lasts = s; d->has_last = 1;
    return s;
  }
  return d->lasts;
}
/* BooleanDecoder.readValue (encoding.js:1171) */
static int cd_bool(ctx_t *c, coldec *d) {
  if (cd_done(d)) return 0;
  while (d->count == 0) {
    d->count = rd_u53(c, &d->r);
    d->blast = !d->blast;
    if (d->count == 0 && !d->bfirst) fail(c, "Zero-length runs are not allowed");
    d->bfirst = 0;
  }
  d->count--;
  return d->blast;
}

/* ---- canonical encoders (RLEEncoder/DeltaEncoder/BooleanEncoder state machines,
 *      encoding.js:558-783, 932-997, 1061-1135: maximal runs; runs >= 2 -> repetition record;
 *      adjacent length-1 runs -> one literal; nulls -> null record; all-null column -> empty) ---- */
static void enc_rle_int(ctx_t *c, bbuf *o, const nv *v, size_t n, int is_signed) {
  size_t nonnull = 0;
  for (size_t i = 0; i < n; i++) nonnull += !v[i].null;
  if (nonnull == 0) return; /* finish(): nothing written if only nulls (encoding.js:780) */
  size_t i = 0;
  while (i < n) {
    size_t j = i + 1;
    while (j < n && v[j].null == v[i].null && (v[i].null || v[j].v == v[i].v)) j++;
    size_t run = j - i;
    if (v[i].null) { bb_s(c, o, 0); bb_u(c, o, run); i = j; continue; }
    if (run >= 2) {
      bb_s(c, o, (int64_t)run);
      if (is_signed) bb_s(c, o, v[i].v); else bb_u(c, o, (uint64_t)v[i].v);
      i = j;
      continue;
    }
    /* literal: collect consecutive length-1 non-null runs */
    size_t k = i;
    while (k < n && !v[k].null && (k + 1 >= n || v[k + 1].null || v[k + 1].v != v[k].v)) k++;
    size_t lit = k - i;
    bb_s(c, o, -(int64_t)lit);
    for (size_t t = i; t < k; t++) { if (is_signed) bb_s(c, o, v[t].v); else bb_u(c, o, (uint64_t)v[t].v); }
    i = k;
  }
}
static void enc_rle_str(ctx_t *c, bbuf *o, const ns *v, size_t n) {
  size_t nonnull = 0;
  for (size_t i = 0; i < n; i++) nonnull += !v[i].null;
  if (nonnull == 0) return;
  size_t i = 0;
#define SEQ(a, b) ((a).null == (b).null && ((a).null || ns_eq(a, b)))
  while (i < n) {
    size_t j = i + 1;
    while (j < n && SEQ(v[j], v[i])) j++;
    size_t run = j - i;
    if (v[i].null) { bb_s(c, o, 0); bb_u(c, o, run); i = j; continue; }
    if (run >= 2) { bb_s(c, o, (int64_t)run); bb_u(c, o, v[i].n); bb_raw(c, o, v[i].p, v[i].n); i = j; continue; }
    size_t k = i;
    while (k < n && !v[k].null && (k + 1 >= n || v[k + 1].null || !ns_eq(v[k + 1], v[k]))) k++;
    bb_s(c, o, -(int64_t)(k - i));
    for (size_t t = i; t < k; t++) { bb_u(c, o, v[t].n); bb_raw(c, o, v[t].p, v[t].n); }
    i = k;
  }
#undef SEQ
}
static void enc_delta(ctx_t *c, bbuf *o, const nv *v, size_t n) {
  nv *d = (nv *)amalloc(c, sizeof(nv) * (n ? n : 1));
  int64_t abs = 0;
  for (size_t i = 0; i < n; i++) {
    if (v[i].null) d[i] = NUL;
    else { d[i] = NV(v[i].v - abs); abs = v[i].v; }
  }
  enc_rle_int(c, o, d, n, 1);
}
static void enc_bool(ctx_t *c, bbuf *o, const uint8_t *v, size_t n) {
  int last = 0;
  uint64_t count = 0;
  for (size_t i = 0; i < n; i++) {
    if (v[i] == last) count++;
    else { bb_u(c, o, count); last = v[i]; count = 1; }
  }
  if (count > 0) bb_u(c, o, count);
}

/* ============================================================================================
 * Column specs (columnar.js:35-94)
 * ============================================================================================ */
enum { CT_GROUP = 0, CT_ACTOR = 1, CT_INT_RLE = 2, CT_DELTA = 3, CT_BOOL = 4, CT_STR = 5, CT_VLEN = 6, CT_VRAW = 7 };
#define COL_DEFLATE 8
enum { /* column ids */
  C_OBJ_ACTOR = 0x01, C_OBJ_CTR = 0x02, C_KEY_ACTOR = 0x11, C_KEY_CTR = 0x13, C_KEY_STR = 0x15,
  C_ID_ACTOR = 0x21, C_ID_CTR = 0x23, C_INSERT = 0x34, C_ACTION = 0x42, C_VAL_LEN = 0x56, C_VAL_RAW = 0x57,
  C_CHLD_ACTOR = 0x61, C_CHLD_CTR = 0x63, C_PRED_NUM = 0x70, C_PRED_ACTOR = 0x71, C_PRED_CTR = 0x73,
  C_SUCC_NUM = 0x80, C_SUCC_ACTOR = 0x81, C_SUCC_CTR = 0x83
};
enum { /* document change columns */
  D_ACTOR = 0x01, D_SEQ = 0x03, D_MAXOP = 0x13, D_TIME = 0x23, D_MESSAGE = 0x35, D_DEPS_NUM = 0x40,
  D_DEPS_INDEX = 0x43, D_EXTRA_LEN = 0x56, D_EXTRA_RAW = 0x57
};
static const int CHANGE_COLS[] = {C_OBJ_ACTOR, C_OBJ_CTR, C_KEY_ACTOR, C_KEY_CTR, C_KEY_STR, C_ID_ACTOR, C_ID_CTR,
                                  C_INSERT, C_ACTION, C_VAL_LEN, C_VAL_RAW, C_CHLD_ACTOR, C_CHLD_CTR,
                                  C_PRED_NUM, C_PRED_ACTOR, C_PRED_CTR};
static const int DOC_OP_COLS[] = {C_OBJ_ACTOR, C_OBJ_CTR, C_KEY_ACTOR, C_KEY_CTR, C_KEY_STR, C_ID_ACTOR, C_ID_CTR,
                                  C_INSERT, C_ACTION, C_VAL_LEN, C_VAL_RAW, C_CHLD_ACTOR, C_CHLD_CTR,
                                  C_SUCC_NUM, C_SUCC_ACTOR, C_SUCC_CTR};
static const int DOC_CHG_COLS[] = {D_ACTOR, D_SEQ, D_MAXOP, D_TIME, D_MESSAGE, D_DEPS_NUM, D_DEPS_INDEX,
                                   D_EXTRA_LEN, D_EXTRA_RAW};

typedef struct { int id; const uint8_t *p; size_t n; } colbuf;

/* decodeColumnInfo (columnar.js:609) */
static int read_col_info(ctx_t *c, rd_t *d, colbuf **out) {
  int64_t num = rd_u53(c, d);
  colbuf *cols = (colbuf *)acalloc(c, sizeof(colbuf) * (size_t)(num ? num : 1));
  int64_t last = -1;
  for (int64_t i = 0; i < num; i++) {
    int64_t id = rd_u53(c, d), len = rd_u53(c, d);
    if ((id & ~(int64_t)COL_DEFLATE) <= (last & ~(int64_t)COL_DEFLATE)) fail(c, "Columns must be in ascending order");
    last = id;
    cols[i].id = (int)id;
    cols[i].n = (size_t)len;
  }
  *out = cols;
  return (int)num;
}
static const uint8_t *inflate_raw(ctx_t *c, const uint8_t *p, size_t n, size_t *outn) {
  size_t cap = n * 4 + 64;
  for (;;) {
    uint8_t *o = (uint8_t *)amalloc(c, cap);
    z_stream zs;
    memset(&zs, 0, sizeof zs);
    if (inflateInit2(&zs, -15) != Z_OK) fail(c, "inflate init failed");
    zs.next_in = (Bytef *)p; zs.avail_in = (uInt)n; zs.next_out = o; zs.avail_out = (uInt)cap;
    int r = inflate(&zs, Z_FINISH);
    size_t got = zs.total_out;
    inflateEnd(&zs);
    if (r == Z_STREAM_END) { *outn = got; return o; }
    if (r == Z_BUF_ERROR && zs.avail_out == 0) { cap *= 4; continue; }
    fail(c, "invalid deflate data");
  }
}
static const uint8_t *deflate_raw(ctx_t *c, const uint8_t *p, size_t n, size_t *outn) {
  z_stream zs;
  memset(&zs, 0, sizeof zs);
  if (deflateInit2(&zs, 6, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY) != Z_OK) fail(c, "deflate init failed");
  size_t cap = deflateBound(&zs, (uLong)n) + 16;
  uint8_t *o = (uint8_t *)amalloc(c, cap);
  zs.next_in = (Bytef *)p; zs.avail_in = (uInt)n; zs.next_out = o; zs.avail_out = (uInt)cap;
  if (deflate(&zs, Z_FINISH) != Z_STREAM_END) fail(c, "deflate failed");
  *outn = zs.total_out;
  deflateEnd(&zs);
  return o;
}

/* ============================================================================================
 * Containers (columnar.js:659-708) and changes (columnar.js:635-652, 741-765, 813-823)
 * ============================================================================================ */
static const uint8_t MAGIC[4] = {0x85, 0x6f, 0x4a, 0x83};

typedef struct {
  int type;
  const uint8_t *data; size_t n; /* chunk data */
  size_t end;                    /* offset just past the chunk in the input */
  uint8_t hash[32];
} chunk_t;

/* decodeContainerHeader (columnar.js:688) */
static void read_container(ctx_t *c, rd_t *d, int compute_hash, chunk_t *ch) {
  const uint8_t *m = rd_raw(c, d, 4);
  if (memcmp(m, MAGIC, 4) != 0) fail(c, "Data does not begin with magic bytes 85 6f 4a 83");
  const uint8_t *expect = rd_raw(c, d, 4);
  size_t hstart = d->off;
  if (d->off >= d->n) fail(c, "subarray exceeds buffer size"); /* readByte of undefined -> length read fails */
  ch->type = d->p[d->off++];
  int64_t len = rd_u53(c, d);
  ch->data = rd_raw(c, d, (size_t)len);
  ch->n = (size_t)len;
  ch->end = d->off;
  if (compute_hash) {
    oc_sha256(d->p + hstart, d->off - hstart, ch->hash);
    if (memcmp(ch->hash, expect, 4) != 0) fail(c, "checksum does not match data");
  }
}

typedef struct {
  uint8_t hash[32];
  const uint8_t *actor; uint32_t actor_len; /* actorIds[0] */
  int64_t seq, start_op, time;
  ns message;
  size_t ndeps; const uint8_t *deps; /* ndeps x 32 bytes */
  size_t nactors; const uint8_t **actors; uint32_t *actor_lens; /* incl. author at 0 */
  int ncols; colbuf *cols;
  const uint8_t *extra; size_t extra_n; int has_extra;
  const uint8_t *buffer; size_t buffer_n; /* as given by the caller */
  int64_t max_op; /* set when applied */
  size_t num_ops;
} change_t;

static void hex_actor(const uint8_t *p, uint32_t n, char *out) {
  static const char *H = "0123456789abcdef";
  for (uint32_t i = 0; i < n && i < 64; i++) { out[2 * i] = H[p[i] >> 4]; out[2 * i + 1] = H[p[i] & 15]; }
  out[2 * (n < 64 ? n : 64)] = 0;
}

/* decodeChangeColumns (columnar.js:741) */
static void decode_change(ctx_t *c, const uint8_t *buf, size_t n, change_t *ch) {
  memset(ch, 0, sizeof *ch);
  ch->buffer = buf;
  ch->buffer_n = n;
  const uint8_t *b = buf;
  size_t bn = n;
  if (n > 8 && buf[8] == 2) { /* inflateChange (columnar.js:813) */
    rd_t d0 = {buf, n, 0};
    chunk_t h0;
    read_container(c, &d0, 0, &h0);
    if (h0.type != 2) fail(c, "Unexpected chunk type: %d", h0.type);
    size_t dn;
    const uint8_t *dec = inflate_raw(c, h0.data, h0.n, &dn);
    bbuf o = {0};
    bb_raw(c, &o, buf, 8);
    bb_byte(c, &o, 1);
    bb_u(c, &o, dn);
    bb_raw(c, &o, dec, dn);
    b = o.p; bn = o.n;
  }
  rd_t d = {b, bn, 0};
  chunk_t h;
  read_container(c, &d, 1, &h);
  if (d.off != d.n) fail(c, "Encoded change has trailing data");
  if (h.type != 1) fail(c, "Unexpected chunk type: %d", h.type);
  memcpy(ch->hash, h.hash, 32);
  rd_t cd = {h.data, h.n, 0};
  /* decodeChangeHeader (columnar.js:635) */
  ch->ndeps = (size_t)rd_u53(c, &cd);
  ch->deps = rd_raw(c, &cd, ch->ndeps * 32);
  int64_t alen = rd_u53(c, &cd);
  ch->actor = rd_raw(c, &cd, (size_t)alen);
  ch->actor_len = (uint32_t)alen;
  ch->seq = rd_u53(c, &cd);
  ch->start_op = rd_u53(c, &cd);
  ch->time = rd_i53(c, &cd);
  int64_t mlen = rd_u53(c, &cd);
  const uint8_t *mp = rd_raw(c, &cd, (size_t)mlen);
  uint32_t mn;
  ch->message.p = utf8_canon(c, mp, (uint32_t)mlen, &mn);
  ch->message.n = mn;
  ch->message.null = 0;
  int64_t na = rd_u53(c, &cd);
  ch->nactors = (size_t)na + 1;
  ch->actors = (const uint8_t **)amalloc(c, sizeof(uint8_t *) * ch->nactors);
  ch->actor_lens = (uint32_t *)amalloc(c, sizeof(uint32_t) * ch->nactors);
  ch->actors[0] = ch->actor;
  ch->actor_lens[0] = ch->actor_len;
  for (int64_t i = 0; i < na; i++) {
    int64_t l = rd_u53(c, &cd);
    ch->actors[i + 1] = rd_raw(c, &cd, (size_t)l);
    ch->actor_lens[i + 1] = (uint32_t)l;
  }
  ch->ncols = read_col_info(c, &cd, &ch->cols);
  for (int i = 0; i < ch->ncols; i++) {
    if (ch->cols[i].id & COL_DEFLATE) fail(c, "change must not contain deflated columns");
    ch->cols[i].p = rd_raw(c, &cd, ch->cols[i].n);
  }
  if (cd.off < cd.n) {
    ch->has_extra = 1;
    ch->extra = cd.p + cd.off;
    ch->extra_n = cd.n - cd.off;
  }
}

/* ============================================================================================
 * Document state: flat op array in document order + change rows
 * ============================================================================================ */
typedef struct {
  nv obj_actor, obj_ctr, key_actor, key_ctr;
  ns key_str;
  nv id_actor, id_ctr;
  uint8_t insert;
  nv action, val_len;
  const uint8_t *val_raw; uint32_t val_raw_n;
  nv chld_actor, chld_ctr;
  uint32_t nsucc; nv *succ_actor; nv *succ_ctr; /* doc ops: succ; change ops: pred */
} op_t;

typedef struct {
  nv actor, seq, max_op, time;
  ns message;
  uint32_t ndeps; nv *deps_index;
  nv extra_len; const uint8_t *extra_raw; uint32_t extra_raw_n;
} chrow_t;

typedef struct { uint8_t h[32]; int64_t index; } hidx_t; /* changeIndexByHash entry */

struct oc_doc {
  uint8_t *state; size_t state_n;   /* internal doc chunk (no DEFLATE), NULL for an empty doc */
  uint8_t *binary; size_t binary_n; /* cached save() result (the loaded buffer, new.js:1712) */
  hidx_t *hidx; size_t nhidx;       /* changeIndexByHash */
  int have_hash_graph;              /* new.js:1697, 1752 */
  uint8_t **queue; size_t *queue_n; size_t nqueue; /* enqueued change buffers */
  size_t nops; int64_t max_op;
  size_t nchanges;
  /* objectMeta children carried across applyChanges calls (new.js:1812, 1857; see
   * am_apply_patch_oracle.inc): 0 = as documentPatch leaves them (load / init), 1 = pm[], 2 = not
   * tracked (after a patchless oc_doc_apply) */
  int meta_mode;
  struct pm_key *pm; size_t npm;
};
typedef struct { int64_t ctr, actor; int kind; } pm_val; /* children[elemId][opId]: 1 set op, 2 object */
typedef struct pm_key {
  int64_t octr, oactor;                                      /* the object (-1, -1: _root) */
  int is_str; uint8_t *key; uint32_t keyn; int64_t ec, ea;  /* elemId */
  size_t n; pm_val *v;
} pm_key;
static void pm_free(pm_key *pm, size_t n) {
  for (size_t i = 0; i < n; i++) { free(pm[i].key); free(pm[i].v); }
  free(pm);
}
static pm_key *pm_copy(const pm_key *pm, size_t n) {
  pm_key *d = (pm_key *)calloc(n + 1, sizeof(pm_key));
  for (size_t i = 0; i < n; i++) {
    d[i] = pm[i];
    d[i].key = (uint8_t *)malloc(pm[i].keyn + 1);
    if (pm[i].keyn) memcpy(d[i].key, pm[i].key, pm[i].keyn);
    d[i].v = (pm_val *)malloc(sizeof(pm_val) * (pm[i].n + 1));
    if (pm[i].n) memcpy(d[i].v, pm[i].v, sizeof(pm_val) * pm[i].n);
  }
  return d;
}

typedef struct {
  size_t nactors; const uint8_t **actors; uint32_t *actor_lens;
  size_t nheads; uint8_t *heads; /* 32 bytes each */
  size_t nheads_idx; int64_t *heads_idx;
  op_t *ops; size_t nops, capops;
  chrow_t *chg; size_t nchg, capchg;
  const uint8_t *extra; size_t extra_n;
} docst_t;

/* decodeDocumentHeader (columnar.js:1006) + column decode of both column sets */
static void decode_columns_generic(ctx_t *c, colbuf *cols, int ncols, const int *spec, int nspec, colbuf *bycol) {
  /* makeDecoders (columnar.js:553): spec columns get their buffers, missing ones are empty;
   * unknown columns are not supported by this restatement. */
  for (int i = 0; i < nspec; i++) { bycol[i].id = spec[i]; bycol[i].p = NULL; bycol[i].n = 0; }
  for (int i = 0; i < ncols; i++) {
    int k = -1;
    for (int j = 0; j < nspec; j++) if (spec[j] == cols[i].id) k = j;
    if (k < 0) unsupported(c, "unknown column id %d", cols[i].id);
    bycol[k] = cols[i];
  }
}

static void read_ops(ctx_t *c, colbuf *bycol, int is_doc, op_t **out, size_t *nout) {
  coldec d[16];
  static const int types[16] = {T_UINT, T_UINT, T_UINT, T_DELTA, T_UTF8, T_UINT, T_DELTA, T_BOOL, T_UINT,
                                T_UINT, T_RAW, T_UINT, T_DELTA, T_UINT, T_UINT, T_DELTA};
  for (int i = 0; i < 16; i++) cd_init(&d[i], types[i], bycol[i].p, bycol[i].n);
  size_t cap = 16, n = 0;
  op_t *ops = (op_t *)amalloc(c, sizeof(op_t) * cap);
  /* change: ops are read until the action column is done (new.js:701); doc: until idCtr is
   * done (new.js:386) -- both columns are complete in well-formed input */
  coldec *term = is_doc ? &d[6] : &d[8];
  while (!cd_done(term)) {
    if (n == cap) { op_t *np = (op_t *)amalloc(c, sizeof(op_t) * cap * 2); memcpy(np, ops, sizeof(op_t) * n); ops = np; cap *= 2; }
    op_t *o = &ops[n++];
    memset(o, 0, sizeof *o);
    o->obj_actor = cd_int(c, &d[0]);
    o->obj_ctr = cd_int(c, &d[1]);
    o->key_actor = cd_int(c, &d[2]);
    o->key_ctr = cd_int(c, &d[3]);
    o->key_str = cd_str(c, &d[4]);
    o->id_actor = cd_int(c, &d[5]);
    o->id_ctr = cd_int(c, &d[6]);
    o->insert = (uint8_t)cd_bool(c, &d[7]);
    o->action = cd_int(c, &d[8]);
    o->val_len = cd_int(c, &d[9]);
    /* readOperation (new.js:570): VALUE_RAW reads valLen >>> 4 bytes */
    uint32_t vl = o->val_len.null ? 0 : (uint32_t)((uint64_t)o->val_len.v >> 4);
    o->val_raw = rd_raw(c, &d[10].r, vl);
    o->val_raw_n = vl;
    o->chld_actor = cd_int(c, &d[11]);
    o->chld_ctr = cd_int(c, &d[12]);
    nv num = cd_int(c, &d[13]);
    o->nsucc = num.null ? 0 : (uint32_t)num.v;
    o->succ_actor = (nv *)amalloc(c, sizeof(nv) * (o->nsucc + 1));
    o->succ_ctr = (nv *)amalloc(c, sizeof(nv) * (o->nsucc + 1));
    for (uint32_t k = 0; k < o->nsucc; k++) o->succ_actor[k] = cd_int(c, &d[14]);
    for (uint32_t k = 0; k < o->nsucc; k++) o->succ_ctr[k] = cd_int(c, &d[15]);
  }
  *out = ops;
  *nout = n;
}

static void decode_doc(ctx_t *c, const uint8_t *buf, size_t n, docst_t *st) {
  memset(st, 0, sizeof *st);
  rd_t dd = {buf, n, 0};
  chunk_t h;
  read_container(c, &dd, 1, &h);
  if (dd.off != dd.n) fail(c, "Encoded document has trailing data");
  if (h.type != 0) fail(c, "Unexpected chunk type: %d", h.type);
  rd_t d = {h.data, h.n, 0};
  st->nactors = (size_t)rd_u53(c, &d);
  st->actors = (const uint8_t **)amalloc(c, sizeof(uint8_t *) * (st->nactors + 1));
  st->actor_lens = (uint32_t *)amalloc(c, sizeof(uint32_t) * (st->nactors + 1));
  for (size_t i = 0; i < st->nactors; i++) {
    int64_t l = rd_u53(c, &d);
    st->actors[i] = rd_raw(c, &d, (size_t)l);
    st->actor_lens[i] = (uint32_t)l;
  }
  st->nheads = (size_t)rd_u53(c, &d);
  st->heads = (uint8_t *)amalloc(c, 32 * st->nheads + 1);
  memcpy(st->heads, rd_raw(c, &d, 32 * st->nheads), 32 * st->nheads);
  colbuf *ccols, *ocols;
  int nc = read_col_info(c, &d, &ccols);
  int no = read_col_info(c, &d, &ocols);
  for (int i = 0; i < nc; i++) {
    ccols[i].p = rd_raw(c, &d, ccols[i].n);
    if (ccols[i].id & COL_DEFLATE) { ccols[i].p = inflate_raw(c, ccols[i].p, ccols[i].n, &ccols[i].n); ccols[i].id ^= COL_DEFLATE; }
  }
  for (int i = 0; i < no; i++) {
    ocols[i].p = rd_raw(c, &d, ocols[i].n);
    if (ocols[i].id & COL_DEFLATE) { ocols[i].p = inflate_raw(c, ocols[i].p, ocols[i].n, &ocols[i].n); ocols[i].id ^= COL_DEFLATE; }
  }
  st->heads_idx = (int64_t *)amalloc(c, sizeof(int64_t) * (st->nheads + 1));
  if (d.off < d.n) {
    for (size_t i = 0; i < st->nheads; i++) st->heads_idx[i] = rd_u53(c, &d);
    st->nheads_idx = st->nheads;
  }
  st->extra = d.p + d.off;
  st->extra_n = d.n - d.off;

  /* change rows (DOCUMENT_COLUMNS), read via the decoders as in readDocumentChanges */
  colbuf cb[9];
  decode_columns_generic(c, ccols, nc, DOC_CHG_COLS, 9, cb);
  coldec cd[9];
  static const int ct[9] = {T_UINT, T_DELTA, T_DELTA, T_DELTA, T_UTF8, T_UINT, T_DELTA, T_UINT, T_RAW};
  for (int i = 0; i < 9; i++) cd_init(&cd[i], ct[i], cb[i].p, cb[i].n);
  size_t cap = 8;
  st->chg = (chrow_t *)amalloc(c, sizeof(chrow_t) * cap);
  while (!cd_done(&cd[0])) { /* readDocumentChanges loops while the actor column has data (new.js:1657) */
    if (st->nchg == cap) { chrow_t *np = (chrow_t *)amalloc(c, sizeof(chrow_t) * cap * 2); memcpy(np, st->chg, sizeof(chrow_t) * st->nchg); st->chg = np; cap *= 2; }
    chrow_t *r = &st->chg[st->nchg++];
    r->actor = cd_int(c, &cd[0]);
    r->seq = cd_int(c, &cd[1]);
    r->max_op = cd_int(c, &cd[2]);
    r->time = cd_int(c, &cd[3]);
    r->message = cd_str(c, &cd[4]);
    nv dn = cd_int(c, &cd[5]);
    r->ndeps = dn.null ? 0 : (uint32_t)dn.v;
    r->deps_index = (nv *)amalloc(c, sizeof(nv) * (r->ndeps + 1));
    for (uint32_t k = 0; k < r->ndeps; k++) r->deps_index[k] = cd_int(c, &cd[6]);
    r->extra_len = cd_int(c, &cd[7]);
    uint32_t el = r->extra_len.null ? 0 : (uint32_t)((uint64_t)r->extra_len.v >> 4);
    r->extra_raw = rd_raw(c, &cd[8].r, el);
    r->extra_raw_n = el;
  }
  st->capchg = cap;

  colbuf ob[16];
  decode_columns_generic(c, ocols, no, DOC_OP_COLS, 16, ob);
  read_ops(c, ob, 1, &st->ops, &st->nops);
  st->capops = st->nops;
}

/* ---- actor helpers ---- */
static int actor_cmp(const uint8_t *a, uint32_t an, const uint8_t *b, uint32_t bn) {
  /* hex-string comparison == bytewise comparison with shorter-prefix-first */
  uint32_t m = an < bn ? an : bn;
  int r = m ? memcmp(a, b, m) : 0;
  if (r) return r < 0 ? -1 : 1;
  return an < bn ? -1 : (an > bn ? 1 : 0);
}
static int64_t actor_index(const docst_t *st, const uint8_t *a, uint32_t n) {
  for (size_t i = 0; i < st->nactors; i++)
    if (st->actor_lens[i] == n && (n == 0 || memcmp(st->actors[i], a, n) == 0)) return (int64_t)i;
  return -1;
}
/* compare opIds (counter, actorId) -- compareParsedOpIds (columnar.js:114) */
static int opid_cmp(const docst_t *st, int64_t c1, int64_t a1, int64_t c2, int64_t a2) {
  if (c1 != c2) return c1 < c2 ? -1 : 1;
  if (a1 == a2) return 0;
  return actor_cmp(st->actors[a1], st->actor_lens[a1], st->actors[a2], st->actor_lens[a2]);
}

/* ============================================================================================
 * Per-op merge. The reference seeks with seekToOp/seekWithinBlock (new.js:50-317) and merges with
 * mergeDocChangeOps (new.js:1052-1290); applied one op at a time this yields the same sequence:
 *   objects: root first, then by (counter, actorId)                    new.js:59-71
 *   map keys: JS string order, same-key ops in opId order               new.js:77-92, 1157-1224
 *   list insert: after the reference element, skip non-insert ops and
 *     insertions with a greater opId                                   new.js:106-163
 *   list update: after the element's ops with a smaller opId           new.js:165-190
 *   preds add the op to the matching op's sorted succ list; dels are not rows
 * ============================================================================================ */
static void ins_op(ctx_t *c, docst_t *st, size_t pos, const op_t *op) {
  if (st->nops == st->capops) {
    size_t nc = st->capops ? st->capops * 2 : 16;
    op_t *np = (op_t *)amalloc(c, sizeof(op_t) * nc);
    if (st->nops) memcpy(np, st->ops, sizeof(op_t) * st->nops);
    st->ops = np;
    st->capops = nc;
  }
  memmove(&st->ops[pos + 1], &st->ops[pos], sizeof(op_t) * (st->nops - pos));
  st->ops[pos] = *op;
  st->nops++;
}
static void add_succ(ctx_t *c, const docst_t *st, op_t *target, int64_t ctr, int64_t actor) {
  uint32_t j = 0;
  while (j < target->nsucc &&
         (target->succ_ctr[j].v < ctr ||
          (target->succ_ctr[j].v == ctr &&
           actor_cmp(st->actors[target->succ_actor[j].v], st->actor_lens[target->succ_actor[j].v],
                     st->actors[actor], st->actor_lens[actor]) < 0)))
    j++;
  nv *na = (nv *)amalloc(c, sizeof(nv) * (target->nsucc + 1));
  nv *nc = (nv *)amalloc(c, sizeof(nv) * (target->nsucc + 1));
  memcpy(na, target->succ_actor, sizeof(nv) * j);
  memcpy(nc, target->succ_ctr, sizeof(nv) * j);
  na[j] = NV(actor);
  nc[j] = NV(ctr);
  memcpy(na + j + 1, target->succ_actor + j, sizeof(nv) * (target->nsucc - j));
  memcpy(nc + j + 1, target->succ_ctr + j, sizeof(nv) * (target->nsucc - j));
  target->succ_actor = na;
  target->succ_ctr = nc;
  target->nsucc++;
}
static int same_obj(const op_t *a, const op_t *b) {
  return a->obj_actor.null == b->obj_actor.null && a->obj_ctr.null == b->obj_ctr.null &&
         (a->obj_actor.null || a->obj_actor.v == b->obj_actor.v) && (a->obj_ctr.null || a->obj_ctr.v == b->obj_ctr.v);
}
/* object order: null (root) first, then (ctr, actorId) -- seekWithinBlock (new.js:59-71) */
static int obj_before(const docst_t *st, const op_t *docop, const op_t *op) {
  if (op->obj_ctr.null) return 0;
  if (docop->obj_ctr.null || docop->obj_actor.null) return 1;
  return opid_cmp(st, docop->obj_ctr.v, docop->obj_actor.v, op->obj_ctr.v, op->obj_actor.v) < 0;
}

static void apply_op(ctx_t *c, docst_t *st, const op_t *op, int is_del) {
  size_t n = st->nops, i = 0;
  char ab[130];
  /* seek to the object's range */
  while (i < n && obj_before(st, &st->ops[i], op)) i++;
  size_t obj_start = i, obj_end = i;
  while (obj_end < n && same_obj(&st->ops[obj_end], op)) obj_end++;
  size_t pos, gstart, gend; /* insertion position and the key/element group [gstart, gend) */
  if (!op->key_str.null) {
    i = obj_start;
    while (i < obj_end && !st->ops[i].key_str.null &&
           utf16_cmp(st->ops[i].key_str.p, st->ops[i].key_str.n, op->key_str.p, op->key_str.n) < 0)
      i++;
    gstart = i;
    gend = i;
    while (gend < obj_end && !st->ops[gend].key_str.null && ns_eq(st->ops[gend].key_str, op->key_str)) gend++;
    pos = gstart;
    while (pos < gend && opid_cmp(st, st->ops[pos].id_ctr.v, st->ops[pos].id_actor.v, op->id_ctr.v, op->id_actor.v) < 0) pos++;
  } else if (op->insert) {
    if (op->key_ctr.null || op->key_ctr.v == 0 || op->key_actor.null) {
      i = obj_start;
    } else {
      i = obj_start;
      while (i < obj_end && !(st->ops[i].insert && st->ops[i].id_ctr.v == op->key_ctr.v && st->ops[i].id_actor.v == op->key_actor.v)) i++;
      if (i == obj_end) {
        hex_actor(st->actors[op->key_actor.v], st->actor_lens[op->key_actor.v], ab);
        fail(c, "Reference element not found: %lld@%s", (long long)op->key_ctr.v, ab);
      }
      i++;
    }
    while (i < obj_end && (!st->ops[i].insert ||
                           opid_cmp(st, st->ops[i].id_ctr.v, st->ops[i].id_actor.v, op->id_ctr.v, op->id_actor.v) > 0))
      i++;
    pos = gstart = gend = i;
  } else {
    /* update/delete of an existing list element */
    i = obj_start;
    while (i < obj_end && !(st->ops[i].insert && !op->key_ctr.null && !op->key_actor.null &&
                            st->ops[i].id_ctr.v == op->key_ctr.v && st->ops[i].id_actor.v == op->key_actor.v))
      i++;
    if (i == obj_end) {
      char kb[130] = "null";
      if (!op->key_actor.null) hex_actor(st->actors[op->key_actor.v], st->actor_lens[op->key_actor.v], kb);
      fail(c, "could not find list element with ID: %lld@%s", (long long)op->key_ctr.v, kb);
    }
    gstart = i;
    gend = i + 1;
    while (gend < obj_end && !st->ops[gend].insert) gend++;
    pos = gstart;
    while (pos < gend && opid_cmp(st, st->ops[pos].id_ctr.v, st->ops[pos].id_actor.v, op->id_ctr.v, op->id_actor.v) < 0) pos++;
  }
  /* duplicate id within the group (new.js:1219) */
  for (size_t k = gstart; k < gend; k++)
    if (st->ops[k].id_ctr.v == op->id_ctr.v && st->ops[k].id_actor.v == op->id_actor.v) {
      hex_actor(st->actors[op->id_actor.v], st->actor_lens[op->id_actor.v], ab);
      fail(c, "duplicate operation ID: %lld@%s", (long long)op->id_ctr.v, ab);
    }
  /* preds: must match ops of the same group that precede the insertion point (new.js:1173-1188,
   * 1254-1258); insertions never match (they take the change path first, new.js:1157) */
  for (uint32_t p = 0; p < op->nsucc; p++) {
    size_t k = gstart, found = 0;
    if (!op->insert) {
      for (; k < pos; k++)
        if (st->ops[k].id_ctr.v == op->succ_ctr[p].v && st->ops[k].id_actor.v == op->succ_actor[p].v) { found = 1; break; }
    }
    if (!found) {
      hex_actor(st->actors[op->succ_actor[p].v], st->actor_lens[op->succ_actor[p].v], ab);
      fail(c, "no matching operation for pred: %lld@%s", (long long)op->succ_ctr[p].v, ab);
    }
    add_succ(c, st, &st->ops[k], op->id_ctr.v, op->id_actor.v);
  }
  if (!is_del) {
    op_t row = *op;
    row.nsucc = 0;
    row.succ_actor = row.succ_ctr = NULL;
    ins_op(c, st, pos, &row);
  }
}

/* ============================================================================================
 * applyChanges (new.js:1550-1597 and BackendDoc.applyChanges new.js:1796-1871)
 * ============================================================================================ */
static int64_t hidx_get(const hidx_t *h, size_t n, const uint8_t *hash, int *found) {
  for (size_t i = 0; i < n; i++)
    if (memcmp(h[i].h, hash, 32) == 0) { *found = 1; return h[i].index; }
  *found = 0;
  return 0;
}

typedef struct { const uint8_t *a; uint32_t n; int64_t seq; } clock_t_;

static void encode_doc(ctx_t *c, const docst_t *st, int deflate, bbuf *out);

/* applyChanges patch replay (am_apply_patch_oracle.inc): set while oc_doc_apply_patch runs */
typedef struct apatch apatch;
static apatch *g_ap = NULL;
static void ap_pass(ctx_t *c, apatch *ap, change_t **applied, size_t na);

static void apply_changes(ctx_t *c, oc_doc *doc, docst_t *st, const uint8_t *const *bufs, const size_t *lens, size_t n) {
  /* decode all given changes first (new.js:1798), then append the old queue (new.js:1814) */
  size_t total = n + doc->nqueue;
  change_t *chs = (change_t *)acalloc(c, sizeof(change_t) * (total + 1));
  for (size_t i = 0; i < n; i++) {
    uint8_t *copy = (uint8_t *)amalloc(c, lens[i] + 1);
    memcpy(copy, bufs[i], lens[i]);
    decode_change(c, copy, lens[i], &chs[i]);
  }
  /* the queue's buffers are replaced at commit; the patch keeps pointers into the decoded bytes */
  for (size_t i = 0; i < doc->nqueue; i++) {
    uint8_t *copy = (uint8_t *)amalloc(c, doc->queue_n[i] + 1);
    memcpy(copy, doc->queue[i], doc->queue_n[i]);
    decode_change(c, copy, doc->queue_n[i], &chs[n + i]);
  }

  /* changeIndexByHash (mutable copy) */
  hidx_t *hidx = (hidx_t *)amalloc(c, sizeof(hidx_t) * (doc->nhidx + total + 1));
  memcpy(hidx, doc->hidx, sizeof(hidx_t) * doc->nhidx);
  size_t nh = doc->nhidx;
  /* clock from the document's change rows */
  clock_t_ *clock = (clock_t_ *)amalloc(c, sizeof(clock_t_) * (st->nactors + total + 1));
  size_t nclock = 0;
  for (size_t i = 0; i < st->nchg; i++) {
    int64_t a = st->chg[i].actor.v;
    size_t k = 0;
    while (k < nclock && !(clock[k].n == st->actor_lens[a] && memcmp(clock[k].a, st->actors[a], clock[k].n) == 0)) k++;
    if (k == nclock) { clock[k].a = st->actors[a]; clock[k].n = st->actor_lens[a]; nclock++; }
    clock[k].seq = st->chg[i].seq.v;
  }
  uint8_t *heads = (uint8_t *)amalloc(c, 32 * (st->nheads + total + 1));
  size_t nheads = st->nheads;
  memcpy(heads, st->heads, 32 * nheads);

  change_t **queue = (change_t **)amalloc(c, sizeof(change_t *) * (total + 1));
  for (size_t i = 0; i < total; i++) queue[i] = &chs[i];
  size_t nq = total;
  change_t **all_applied = (change_t **)amalloc(c, sizeof(change_t *) * (total + 1));
  size_t nall = 0;
  size_t base_changes = st->nchg;

  for (;;) {
    /* one pass of applyChanges() (new.js:1550) */
    change_t **applied = (change_t **)amalloc(c, sizeof(change_t *) * (nq + 1));
    change_t **enq = (change_t **)amalloc(c, sizeof(change_t *) * (nq + 1));
    size_t na = 0, ne = 0;
    uint8_t *hashes = (uint8_t *)amalloc(c, 32 * (nq + 1)); /* changeHashes of this pass */
    size_t nhs = 0;
    clock_t_ *clk = (clock_t_ *)amalloc(c, sizeof(clock_t_) * (nclock + nq + 1));
    memcpy(clk, clock, sizeof(clock_t_) * nclock);
    size_t nclk = nclock;
    uint8_t *hd = (uint8_t *)amalloc(c, 32 * (nheads + nq + 1));
    memcpy(hd, heads, 32 * nheads);
    size_t nhd = nheads;
    int reuse_abort = 0;
    for (size_t qi = 0; qi < nq && !reuse_abort; qi++) {
      change_t *ch = queue[qi];
      int f;
      hidx_get(hidx, nh, ch->hash, &f);
      int dup = f;
      for (size_t k = 0; k < nhs && !dup; k++) if (memcmp(hashes + 32 * k, ch->hash, 32) == 0) dup = 1;
      if (dup) continue;
      size_t k = 0;
      while (k < nclk && !(clk[k].n == ch->actor_len && memcmp(clk[k].a, ch->actor, ch->actor_len) == 0)) k++;
      int64_t expected = (k < nclk ? clk[k].seq : 0) + 1;
      int ready = 1;
      for (size_t di = 0; di < ch->ndeps; di++) {
        int fd;
        int64_t idx = hidx_get(hidx, nh, ch->deps + 32 * di, &fd);
        int inpass = 0;
        for (size_t t = 0; t < nhs; t++) if (memcmp(hashes + 32 * t, ch->deps + 32 * di, 32) == 0) inpass = 1;
        if ((!fd || idx == -1) && !inpass) ready = 0;
      }
      char ab[130];
      hex_actor(ch->actor, ch->actor_len, ab);
      if (!ready) {
        enq[ne++] = ch;
      } else if (ch->seq < expected) {
        if (doc->have_hash_graph) fail(c, "Reuse of sequence number %lld for actor %s", (long long)ch->seq, ab);
        reuse_abort = 1; /* return [[], decodedChanges] (new.js:1575) */
      } else if (ch->seq > expected) {
        fail(c, "Skipped sequence number %lld for actor %s", (long long)expected, ab);
      } else {
        if (k == nclk) { clk[k].a = ch->actor; clk[k].n = ch->actor_len; nclk++; }
        clk[k].seq = ch->seq;
        memcpy(hashes + 32 * nhs++, ch->hash, 32);
        for (size_t di = 0; di < ch->ndeps; di++) {
          for (size_t t = 0; t < nhd; t++)
            if (memcmp(hd + 32 * t, ch->deps + 32 * di, 32) == 0) { memmove(hd + 32 * t, hd + 32 * (t + 1), 32 * (nhd - t - 1)); nhd--; break; }
        }
        int present = 0;
        for (size_t t = 0; t < nhd; t++) if (memcmp(hd + 32 * t, ch->hash, 32) == 0) present = 1;
        if (!present) memcpy(hd + 32 * nhd++, ch->hash, 32);
        applied[na++] = ch;
      }
    }
    if (reuse_abort) { na = 0; ne = nq; memcpy(enq, queue, sizeof(change_t *) * nq); }
    if (na > 0 && g_ap) ap_pass(c, g_ap, applied, na);
    if (na > 0) {
      /* readNextChangeOp / applyOps over all ops of the applied changes (new.js:1589-1591) */
      for (size_t ai = 0; ai < na; ai++) {
        change_t *ch = applied[ai];
        char ab[130];
        /* getActorTable (new.js:1434) */
        int64_t self = actor_index(st, ch->actor, ch->actor_len);
        if (self < 0) {
          hex_actor(ch->actor, ch->actor_len, ab);
          if (ch->seq != 1) fail(c, "Seq %lld is the first change for actor %s", (long long)ch->seq, ab);
          const uint8_t **na_ = (const uint8_t **)amalloc(c, sizeof(uint8_t *) * (st->nactors + 1));
          uint32_t *nl_ = (uint32_t *)amalloc(c, sizeof(uint32_t) * (st->nactors + 1));
          memcpy(na_, st->actors, sizeof(uint8_t *) * st->nactors);
          memcpy(nl_, st->actor_lens, sizeof(uint32_t) * st->nactors);
          na_[st->nactors] = ch->actor;
          nl_[st->nactors] = ch->actor_len;
          st->actors = na_;
          st->actor_lens = nl_;
          self = (int64_t)st->nactors++;
        }
        int64_t *table = (int64_t *)amalloc(c, sizeof(int64_t) * ch->nactors);
        for (size_t t = 0; t < ch->nactors; t++) {
          table[t] = actor_index(st, ch->actors[t], ch->actor_lens[t]);
          if (table[t] < 0) {
            hex_actor(ch->actors[t], ch->actor_lens[t], ab);
            fail(c, "actorId %s is not known to document", ab);
          }
        }
        /* updateBlockColumns (new.js:1387): only the standard change columns are supported here */
        colbuf cb[16];
        decode_columns_generic(c, ch->cols, ch->ncols, CHANGE_COLS, 16, cb);
        op_t *ops;
        size_t nops;
        read_ops(c, cb, 0, &ops, &nops);
        ch->num_ops = nops;
        ch->max_op = ch->start_op - 1 + (int64_t)nops;
        for (size_t oi = 0; oi < nops; oi++) {
          op_t *o = &ops[oi];
          /* actor columns map through actorTable (new.js:588, 598) */
          nv *acts[3] = {&o->obj_actor, &o->key_actor, &o->chld_actor};
          for (int q = 0; q < 3; q++)
            if (!acts[q]->null) {
              if (acts[q]->v < 0 || (size_t)acts[q]->v >= ch->nactors) fail(c, "No actor index %lld", (long long)acts[q]->v);
              acts[q]->v = table[acts[q]->v];
            }
          for (uint32_t p = 0; p < o->nsucc; p++)
            if (!o->succ_actor[p].null) {
              if (o->succ_actor[p].v < 0 || (size_t)o->succ_actor[p].v >= ch->nactors) fail(c, "No actor index %lld", (long long)o->succ_actor[p].v);
              o->succ_actor[p].v = table[o->succ_actor[p].v];
            }
          o->id_actor = NV(self);
          o->id_ctr = NV(ch->start_op + (int64_t)oi);
          /* readNextChangeOp consistency checks (new.js:715-723) */
          if (o->obj_ctr.null != o->obj_actor.null)
            fail(c, "Mismatched object reference: (%s, %s)", o->obj_ctr.null ? "null" : "ctr", o->obj_actor.null ? "null" : "actor");
          if ((o->key_ctr.null && !o->key_actor.null) || (!o->key_ctr.null && o->key_ctr.v == 0 && !o->key_actor.null) ||
              (!o->key_ctr.null && o->key_ctr.v > 0 && o->key_actor.null))
            fail(c, "Mismatched operation key");
          if (o->action.null) unsupported(c, "null action");
          if (o->key_str.null && !o->insert && o->key_ctr.null) unsupported(c, "op without key");
          for (uint32_t p = 0; p < o->nsucc; p++)
            if (o->succ_ctr[p].null || o->succ_actor[p].null) unsupported(c, "null pred");
          apply_op(c, st, o, o->action.v == 3 /* del */);
        }
      }
      /* docState.heads = sorted heads (new.js:1593) */
      for (size_t a = 1; a < nhd; a++)
        for (size_t b = a; b > 0 && memcmp(hd + 32 * (b - 1), hd + 32 * b, 32) > 0; b--) {
          uint8_t t[32];
          memcpy(t, hd + 32 * b, 32); memcpy(hd + 32 * b, hd + 32 * (b - 1), 32); memcpy(hd + 32 * (b - 1), t, 32);
        }
      memcpy(heads, hd, 32 * nhd);
      nheads = nhd;
      memcpy(clock, clk, sizeof(clock_t_) * nclk);
      nclock = nclk;
    }
    /* new.js:1820-1833 */
    for (size_t ai = 0; ai < na; ai++) {
      memcpy(hidx[nh].h, applied[ai]->hash, 32);
      hidx[nh].index = (int64_t)(base_changes + nall + ai);
      nh++;
      all_applied[nall + ai] = applied[ai];
    }
    nall += na;
    memcpy(queue, enq, sizeof(change_t *) * ne);
    nq = ne;
    if (nq == 0) break;
    if (na == 0) {
      if (doc->have_hash_graph) break;
      unsupported(c, "computeHashGraph() of a loaded document is not restated by the oracle");
    }
  }

  /* commit: appendChange per applied change (new.js:1838-1850, 1680) */
  for (size_t ai = 0; ai < nall; ai++) {
    change_t *ch = all_applied[ai];
    if (st->nchg == st->capchg) {
      size_t ncap = st->capchg ? st->capchg * 2 : 8;
      chrow_t *np = (chrow_t *)amalloc(c, sizeof(chrow_t) * ncap);
      if (st->nchg) memcpy(np, st->chg, sizeof(chrow_t) * st->nchg);
      st->chg = np;
      st->capchg = ncap;
    }
    chrow_t *r = &st->chg[st->nchg++];
    memset(r, 0, sizeof *r);
    r->actor = NV(actor_index(st, ch->actor, ch->actor_len));
    r->seq = NV(ch->seq);
    r->max_op = NV(ch->max_op);
    r->time = NV(ch->time);
    r->message = ch->message;
    r->ndeps = (uint32_t)ch->ndeps;
    r->deps_index = (nv *)amalloc(c, sizeof(nv) * (ch->ndeps + 1));
    for (size_t di = 0; di < ch->ndeps; di++) {
      int f;
      int64_t idx = hidx_get(hidx, nh, ch->deps + 32 * di, &f);
      r->deps_index[di] = f ? NV(idx) : NUL;
    }
    r->extra_len = NV(ch->has_extra ? (int64_t)((ch->extra_n << 4) | 7) : 7);
    r->extra_raw = ch->extra;
    r->extra_raw_n = (uint32_t)ch->extra_n;
  }
  st->nheads = nheads;
  st->heads = heads;
  st->nheads_idx = nheads;
  st->heads_idx = (int64_t *)amalloc(c, sizeof(int64_t) * (nheads + 1));
  for (size_t i = 0; i < nheads; i++) {
    int f;
    st->heads_idx[i] = hidx_get(hidx, nh, heads + 32 * i, &f);
    if (!f || st->heads_idx[i] < 0) unsupported(c, "head without a change index");
  }

  /* persist the new state */
  bbuf enc = {0};
  encode_doc(c, st, 0, &enc);
  uint8_t *ns_ = (uint8_t *)malloc(enc.n);
  memcpy(ns_, enc.p, enc.n);
  hidx_t *nhx = (hidx_t *)malloc(sizeof(hidx_t) * (nh + 1));
  memcpy(nhx, hidx, sizeof(hidx_t) * nh);
  uint8_t **nqb = (uint8_t **)malloc(sizeof(uint8_t *) * (nq + 1));
  size_t *nql = (size_t *)malloc(sizeof(size_t) * (nq + 1));
  for (size_t i = 0; i < nq; i++) {
    nqb[i] = (uint8_t *)malloc(queue[i]->buffer_n + 1);
    memcpy(nqb[i], queue[i]->buffer, queue[i]->buffer_n);
    nql[i] = queue[i]->buffer_n;
  }
  for (size_t i = 0; i < doc->nqueue; i++) free(doc->queue[i]);
  free(doc->queue); free(doc->queue_n); free(doc->hidx); free(doc->state);
  free(doc->binary); doc->binary = NULL; doc->binary_n = 0; /* this.binaryDoc = null (new.js:1859) */
  doc->state = ns_; doc->state_n = enc.n;
  doc->hidx = nhx; doc->nhidx = nh;
  doc->queue = nqb; doc->queue_n = nql; doc->nqueue = nq;
  doc->nops = st->nops;
  doc->nchanges = st->nchg;
  int64_t mx = doc->max_op;
  for (size_t i = 0; i < nall; i++) if (all_applied[i]->num_ops && all_applied[i]->max_op > mx) mx = all_applied[i]->max_op;
  doc->max_op = mx;
}

/* ============================================================================================
 * save(): encodeDocumentHeader (columnar.js:983) over canonical column encodings
 * ============================================================================================ */
typedef struct { int id; bbuf b; } outcol;

static void put_col_info(ctx_t *c, bbuf *o, outcol *cols, int n) {
  int ne = 0;
  for (int i = 0; i < n; i++) ne += cols[i].b.n > 0;
  bb_u(c, o, (uint64_t)ne);
  for (int i = 0; i < n; i++)
    if (cols[i].b.n > 0) { bb_u(c, o, (uint64_t)cols[i].id); bb_u(c, o, cols[i].b.n); }
}
static void maybe_deflate(ctx_t *c, outcol *col) {
  /* deflateColumn (columnar.js:1052): DEFLATE_MIN_SIZE = 256 */
  if (col->b.n >= 256) {
    size_t dn;
    const uint8_t *d = deflate_raw(c, col->b.p, col->b.n, &dn);
    col->b.p = (uint8_t *)d;
    col->b.n = dn;
    col->b.cap = dn;
    col->id |= COL_DEFLATE;
  }
}

static void encode_doc(ctx_t *c, const docst_t *st, int deflate, bbuf *out) {
  size_t n = st->nops, m = st->nchg;
  outcol oc[16], cc[9];
  memset(oc, 0, sizeof oc);
  memset(cc, 0, sizeof cc);
  for (int i = 0; i < 16; i++) oc[i].id = DOC_OP_COLS[i];
  for (int i = 0; i < 9; i++) cc[i].id = DOC_CHG_COLS[i];
  nv *v = (nv *)amalloc(c, sizeof(nv) * (n + 1));
  size_t nsucc = 0;
  for (size_t i = 0; i < n; i++) nsucc += st->ops[i].nsucc;
  nv *sv = (nv *)amalloc(c, sizeof(nv) * (nsucc + 1));
#define COLI(idx, field, sgn) do { for (size_t i = 0; i < n; i++) v[i] = st->ops[i].field; enc_rle_int(c, &oc[idx].b, v, n, sgn); } while (0)
#define COLD(idx, field) do { for (size_t i = 0; i < n; i++) v[i] = st->ops[i].field; enc_delta(c, &oc[idx].b, v, n); } while (0)
  COLI(0, obj_actor, 0);
  COLI(1, obj_ctr, 0);
  COLI(2, key_actor, 0);
  COLD(3, key_ctr);
  {
    ns *s = (ns *)amalloc(c, sizeof(ns) * (n + 1));
    for (size_t i = 0; i < n; i++) s[i] = st->ops[i].key_str;
    enc_rle_str(c, &oc[4].b, s, n);
  }
  COLI(5, id_actor, 0);
  COLD(6, id_ctr);
  {
    uint8_t *b = (uint8_t *)amalloc(c, n + 1);
    for (size_t i = 0; i < n; i++) b[i] = st->ops[i].insert;
    enc_bool(c, &oc[7].b, b, n);
  }
  COLI(8, action, 0);
  COLI(9, val_len, 0);
  for (size_t i = 0; i < n; i++) bb_raw(c, &oc[10].b, st->ops[i].val_raw, st->ops[i].val_raw_n);
  COLI(11, chld_actor, 0);
  COLD(12, chld_ctr);
  for (size_t i = 0; i < n; i++) v[i] = NV(st->ops[i].nsucc);
  enc_rle_int(c, &oc[13].b, v, n, 0);
  size_t k = 0;
  for (size_t i = 0; i < n; i++) for (uint32_t j = 0; j < st->ops[i].nsucc; j++) sv[k++] = st->ops[i].succ_actor[j];
  enc_rle_int(c, &oc[14].b, sv, nsucc, 0);
  k = 0;
  for (size_t i = 0; i < n; i++) for (uint32_t j = 0; j < st->ops[i].nsucc; j++) sv[k++] = st->ops[i].succ_ctr[j];
  enc_delta(c, &oc[15].b, sv, nsucc);
#undef COLI
#undef COLD
  /* change columns */
  nv *cv = (nv *)amalloc(c, sizeof(nv) * (m + 1));
  size_t ndeps = 0;
  for (size_t i = 0; i < m; i++) ndeps += st->chg[i].ndeps;
  nv *dv = (nv *)amalloc(c, sizeof(nv) * (ndeps + 1));
#define CCOL(idx, field, kind) do { for (size_t i = 0; i < m; i++) cv[i] = st->chg[i].field; \
    if (kind) enc_delta(c, &cc[idx].b, cv, m); else enc_rle_int(c, &cc[idx].b, cv, m, 0); } while (0)
  CCOL(0, actor, 0);
  CCOL(1, seq, 1);
  CCOL(2, max_op, 1);
  CCOL(3, time, 1);
  {
    ns *s = (ns *)amalloc(c, sizeof(ns) * (m + 1));
    for (size_t i = 0; i < m; i++) s[i] = st->chg[i].message;
    enc_rle_str(c, &cc[4].b, s, m);
  }
  for (size_t i = 0; i < m; i++) cv[i] = NV(st->chg[i].ndeps);
  enc_rle_int(c, &cc[5].b, cv, m, 0);
  k = 0;
  for (size_t i = 0; i < m; i++) for (uint32_t j = 0; j < st->chg[i].ndeps; j++) dv[k++] = st->chg[i].deps_index[j];
  enc_delta(c, &cc[6].b, dv, ndeps);
  CCOL(7, extra_len, 0);
  for (size_t i = 0; i < m; i++) bb_raw(c, &cc[8].b, st->chg[i].extra_raw, st->chg[i].extra_raw_n);
#undef CCOL
  if (deflate) {
    for (int i = 0; i < 9; i++) maybe_deflate(c, &cc[i]);
    for (int i = 0; i < 16; i++) maybe_deflate(c, &oc[i]);
  }
  /* body */
  bbuf body = {0};
  bb_u(c, &body, st->nactors);
  for (size_t i = 0; i < st->nactors; i++) { bb_u(c, &body, st->actor_lens[i]); bb_raw(c, &body, st->actors[i], st->actor_lens[i]); }
  bb_u(c, &body, st->nheads);
  bb_raw(c, &body, st->heads, 32 * st->nheads);
  put_col_info(c, &body, cc, 9);
  put_col_info(c, &body, oc, 16);
  for (int i = 0; i < 9; i++) bb_raw(c, &body, cc[i].b.p, cc[i].b.n);
  for (int i = 0; i < 16; i++) bb_raw(c, &body, oc[i].b.p, oc[i].b.n);
  for (size_t i = 0; i < st->nheads_idx; i++) bb_u(c, &body, (uint64_t)st->heads_idx[i]);
  bb_raw(c, &body, st->extra, st->extra_n);
  /* encodeContainer (columnar.js:659) */
  bbuf hdr = {0};
  bb_byte(c, &hdr, 0);
  bb_u(c, &hdr, body.n);
  bbuf all = {0};
  bb_raw(c, &all, hdr.p, hdr.n);
  bb_raw(c, &all, body.p, body.n);
  uint8_t hash[32];
  oc_sha256(all.p, all.n, hash);
  bb_raw(c, out, MAGIC, 4);
  bb_raw(c, out, hash, 4);
  bb_raw(c, out, all.p, all.n);
}

/* ============================================================================================
 * Public API
 * ============================================================================================ */
#define CTX_BEGIN(cx) ctx_t cx; memset(&cx, 0, sizeof cx); if (setjmp(cx.jb))
static void set_err(const ctx_t *c, char *err, size_t cap) {
  if (err && cap) { strncpy(err, c->msg, cap - 1); err[cap - 1] = 0; }
}

oc_doc *oc_doc_init(void) {
  oc_doc *d = (oc_doc *)calloc(1, sizeof(oc_doc));
  d->have_hash_graph = 1;
  return d;
}

static void empty_state(docst_t *st) { memset(st, 0, sizeof *st); }

/* new BackendDoc(buffer) (new.js:1709-1750) */
oc_doc *oc_doc_load(const uint8_t *buf, size_t len, char *err, size_t errcap) {
  CTX_BEGIN(c) { set_err(&c, err, errcap); afree_all(&c); return NULL; }
  docst_t st;
  uint8_t *copy = (uint8_t *)amalloc(&c, len + 1);
  memcpy(copy, buf, len);
  decode_doc(&c, copy, len, &st);
  /* readDocumentChanges seq checks (new.js:1657-1668) + head actors */
  clock_t_ *clock = (clock_t_ *)amalloc(&c, sizeof(clock_t_) * (st.nactors + 1));
  size_t nclock = 0;
  for (size_t i = 0; i < st.nchg; i++) {
    int64_t a = st.chg[i].actor.v;
    if (st.chg[i].actor.null || a < 0 || (size_t)a >= st.nactors) unsupported(&c, "bad actor index in change columns");
    size_t k = 0;
    while (k < nclock && !(clock[k].n == st.actor_lens[a] && memcmp(clock[k].a, st.actors[a], clock[k].n) == 0)) k++;
    int64_t seq = st.chg[i].seq.v;
    if (seq != 1 && (k == nclock || seq != clock[k].seq + 1)) {
      char ab[130];
      hex_actor(st.actors[a], st.actor_lens[a], ab);
      if (k == nclock) fail(&c, "Expected seq NaN, got %lld for actor %s", (long long)seq, ab);
      fail(&c, "Expected seq %lld, got %lld for actor %s", (long long)(clock[k].seq + 1), (long long)seq, ab);
    }
    if (k == nclock) { clock[k].a = st.actors[a]; clock[k].n = st.actor_lens[a]; nclock++; }
    clock[k].seq = seq;
  }
  oc_doc *d = (oc_doc *)calloc(1, sizeof(oc_doc));
  d->have_hash_graph = 0;
  d->binary = (uint8_t *)malloc(len + 1);
  memcpy(d->binary, buf, len);
  d->binary_n = len;
  /* changeIndexByHash from heads (new.js:1729-1739) */
  d->hidx = (hidx_t *)malloc(sizeof(hidx_t) * (st.nheads + 1));
  d->nhidx = st.nheads;
  for (size_t i = 0; i < st.nheads; i++) {
    memcpy(d->hidx[i].h, st.heads + 32 * i, 32);
    if (st.nheads == st.nheads_idx) d->hidx[i].index = st.heads_idx[i];
    else if (st.nheads == 1) d->hidx[i].index = (int64_t)st.nchg - 1;
    else d->hidx[i].index = -1;
  }
  /* the internal state keeps headsIndexes consistent with changeIndexByHash */
  st.nheads_idx = st.nheads;
  st.heads_idx = (int64_t *)amalloc(&c, sizeof(int64_t) * (st.nheads + 1));
  for (size_t i = 0; i < st.nheads; i++) {
    st.heads_idx[i] = d->hidx[i].index;
    if (st.heads_idx[i] < 0) st.nheads_idx = 0; /* unknown indexes: keep only the hash map */
  }
  bbuf enc = {0};
  encode_doc(&c, &st, 0, &enc);
  d->state = (uint8_t *)malloc(enc.n);
  memcpy(d->state, enc.p, enc.n);
  d->state_n = enc.n;
  d->nops = st.nops;
  d->nchanges = st.nchg;
  int64_t mx = 0;
  for (size_t i = 0; i < st.nops; i++) {
    if (st.ops[i].id_ctr.v > mx) mx = st.ops[i].id_ctr.v;
    for (uint32_t j = 0; j < st.ops[i].nsucc; j++) if (st.ops[i].succ_ctr[j].v > mx) mx = st.ops[i].succ_ctr[j].v;
  }
  d->max_op = mx;
  afree_all(&c);
  return d;
}

oc_doc *oc_doc_clone(const oc_doc *s) {
  oc_doc *d = (oc_doc *)calloc(1, sizeof(oc_doc));
  *d = *s;
  if (s->state) { d->state = (uint8_t *)malloc(s->state_n); memcpy(d->state, s->state, s->state_n); }
  if (s->binary) { d->binary = (uint8_t *)malloc(s->binary_n); memcpy(d->binary, s->binary, s->binary_n); }
  d->hidx = (hidx_t *)malloc(sizeof(hidx_t) * (s->nhidx + 1));
  memcpy(d->hidx, s->hidx, sizeof(hidx_t) * s->nhidx);
  d->queue = (uint8_t **)malloc(sizeof(uint8_t *) * (s->nqueue + 1));
  d->queue_n = (size_t *)malloc(sizeof(size_t) * (s->nqueue + 1));
  for (size_t i = 0; i < s->nqueue; i++) {
    d->queue[i] = (uint8_t *)malloc(s->queue_n[i] + 1);
    memcpy(d->queue[i], s->queue[i], s->queue_n[i]);
    d->queue_n[i] = s->queue_n[i];
  }
  d->pm = s->npm ? pm_copy(s->pm, s->npm) : NULL;
  return d;
}

void oc_doc_free(oc_doc *d) {
  if (!d) return;
  for (size_t i = 0; i < d->nqueue; i++) free(d->queue[i]);
  free(d->queue); free(d->queue_n); free(d->hidx); free(d->state); free(d->binary);
  pm_free(d->pm, d->npm);
  free(d);
}

static void load_state(ctx_t *c, const oc_doc *doc, docst_t *st) {
  if (doc->state) decode_doc(c, doc->state, doc->state_n, st);
  else empty_state(st);
}

int oc_doc_apply(oc_doc *doc, const uint8_t *const *bufs, const size_t *lens, size_t n, char *err, size_t errcap) {
  CTX_BEGIN(c) { set_err(&c, err, errcap); int code = c.code; afree_all(&c); return code; }
  docst_t st;
  load_state(&c, doc, &st);
  apply_changes(&c, doc, &st, bufs, lens, n);
  doc->meta_mode = 2; /* the reference's objectMeta moved on too (updatePatchProperty runs in every applyChanges) */
  afree_all(&c);
  return 0;
}

uint8_t *oc_doc_save(oc_doc *doc, size_t *len) {
  if (doc->binary) {
    uint8_t *o = (uint8_t *)malloc(doc->binary_n + 1);
    memcpy(o, doc->binary, doc->binary_n);
    *len = doc->binary_n;
    return o;
  }
  CTX_BEGIN(c) { afree_all(&c); *len = 0; return NULL; }
  docst_t st;
  load_state(&c, doc, &st);
  bbuf enc = {0};
  encode_doc(&c, &st, 1, &enc);
  uint8_t *o = (uint8_t *)malloc(enc.n + 1);
  memcpy(o, enc.p, enc.n);
  *len = enc.n;
  afree_all(&c);
  return o;
}

size_t oc_doc_heads(const oc_doc *doc, uint8_t *out, size_t cap) {
  if (!doc->state) return 0;
  CTX_BEGIN(c) { afree_all(&c); return 0; }
  docst_t st;
  decode_doc(&c, doc->state, doc->state_n, &st);
  size_t n = st.nheads;
  memcpy(out, st.heads, 32 * (n < cap ? n : cap));
  afree_all(&c);
  return n;
}
size_t oc_doc_pending(const oc_doc *doc) { return doc->nqueue; }
size_t oc_doc_num_ops(const oc_doc *doc) { return doc->nops; }
int64_t oc_doc_max_op(const oc_doc *doc) { return doc->max_op; }
void oc_free(void *p) { free(p); }

/* ---- change meta (decodeChangeMeta, columnar.js:783) ---- */
int oc_change_meta(const uint8_t *buf, size_t len, uint8_t hash[32], int64_t *seq, int64_t *start_op,
                   int64_t *num_ops, int64_t *num_deps, char *err, size_t errcap) {
  CTX_BEGIN(c) { set_err(&c, err, errcap); afree_all(&c); return 1; }
  change_t ch;
  decode_change(&c, buf, len, &ch);
  memcpy(hash, ch.hash, 32);
  *seq = ch.seq;
  *start_op = ch.start_op;
  *num_deps = (int64_t)ch.ndeps;
  colbuf cb[16];
  decode_columns_generic(&c, ch.cols, ch.ncols, CHANGE_COLS, 16, cb);
  op_t *ops;
  size_t nops;
  read_ops(&c, cb, 0, &ops, &nops);
  *num_ops = (int64_t)nops;
  afree_all(&c);
  return 0;
}

/* ---- codec KAT entry points ---- */
int oc_leb_encode(int fn, int64_t value, int64_t hi, int64_t lo, uint8_t *out) {
  switch (fn) {
    case 0: case 2: return leb_put_u(out, (uint64_t)value);
    case 1: case 3: return leb_put_s(out, value);
    case 4: return leb_put_u(out, ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
    default: return leb_put_s(out, (int64_t)(((uint64_t)(uint32_t)(int32_t)hi << 32) | (uint32_t)lo));
  }
}
int oc_leb_decode(int fn, const uint8_t *buf, size_t len, int64_t *v, int64_t *hi, int64_t *lo, size_t *offset,
                  char *err, size_t errcap) {
  rd_t d = {buf, len, 0};
  const char *e = NULL;
  switch (fn) {
    case 0: e = leb_u32(&d, v); break;
    case 1: e = leb_i32(&d, v); break;
    case 2: e = leb_u53(&d, v); break;
    case 3: e = leb_i53(&d, v); break;
    case 4: { uint32_t h, l; e = leb_u64(&d, &h, &l); *hi = h; *lo = l; break; }
    default: { int32_t h; uint32_t l; e = leb_i64(&d, &h, &l); *hi = h; *lo = l; break; }
  }
  *offset = d.off;
  if (e) { if (err && errcap) { strncpy(err, e, errcap - 1); err[errcap - 1] = 0; } return 1; }
  return 0;
}

int oc_col_encode(int type, size_t n, const int64_t *ints, const uint8_t *nulls, const uint8_t *strbuf,
                  const uint32_t *strlens, uint8_t *out, size_t outcap, size_t *outlen) {
  CTX_BEGIN(c) { afree_all(&c); return 1; }
  bbuf o = {0};
  if (type == T_UTF8) {
    ns *s = (ns *)amalloc(&c, sizeof(ns) * (n + 1));
    size_t off = 0;
    for (size_t i = 0; i < n; i++) {
      s[i].null = nulls[i];
      s[i].p = strbuf + off;
      s[i].n = strlens[i];
      off += strlens[i];
    }
    enc_rle_str(&c, &o, s, n);
  } else if (type == T_BOOL) {
    uint8_t *b = (uint8_t *)amalloc(&c, n + 1);
    for (size_t i = 0; i < n; i++) b[i] = ints[i] != 0;
    enc_bool(&c, &o, b, n);
  } else {
    nv *v = (nv *)amalloc(&c, sizeof(nv) * (n + 1));
    for (size_t i = 0; i < n; i++) { v[i].v = ints[i]; v[i].null = nulls[i]; }
    if (type == T_DELTA) enc_delta(&c, &o, v, n);
    else enc_rle_int(&c, &o, v, n, type == T_INT);
  }
  int rc = o.n > outcap;
  if (!rc) memcpy(out, o.p, o.n);
  *outlen = o.n;
  afree_all(&c);
  return rc;
}

int oc_col_decode(int type, const uint8_t *buf, size_t len, size_t maxn, size_t *n, int64_t *ints, uint8_t *nulls,
                  uint8_t *strbuf, size_t strcap, uint32_t *strlens, char *err, size_t errcap) {
  volatile size_t k = 0, soff = 0;
  CTX_BEGIN(c) { *n = k; set_err(&c, err, errcap); afree_all(&c); return 1; }
  coldec d;
  cd_init(&d, type, buf, len);
  while (k < maxn && !cd_done(&d)) {
    if (type == T_UTF8) {
      ns s = cd_str(&c, &d);
      nulls[k] = s.null;
      strlens[k] = s.n;
      if (!s.null) { if (soff + s.n > strcap) fail(&c, "string buffer too small"); memcpy(strbuf + soff, s.p, s.n); soff += s.n; }
    } else if (type == T_BOOL) {
      ints[k] = cd_bool(&c, &d);
      nulls[k] = 0;
    } else {
      nv v = cd_int(&c, &d);
      ints[k] = v.v;
      nulls[k] = v.null;
    }
    k++;
  }
  *n = k;
  afree_all(&c);
  return 0;
}

#include "am_patch_oracle.inc"
#include "am_apply_patch_oracle.inc"
