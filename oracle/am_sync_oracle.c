/*
 * am_sync_oracle.c -- CPU restatement of the sync.js Bloom filter and change selection.
 *
 * TEST INFRASTRUCTURE ONLY (see am_oracle.h). Pinned by tests/golden/bloom.json, which the
 * reference produced (tests/golden/gen/make_fixtures.js bloomVectors).
 *
 *   oc_bloom_build     <- new BloomFilter(hashes).bytes      sync.js:38-47, 66-77, 90-110
 *   oc_bloom_contains  <- new BloomFilter(bytes).containsHash sync.js:48-59, 112-125
 *   oc_sync_select     <- getChangesToSend (have non-empty)   sync.js:246-306
 */
#include <stdlib.h>
#include <string.h>

#include "am_oracle.h"

#define BITS_PER_ENTRY 10
#define NUM_PROBES 7

static size_t put_uleb32(uint8_t *o, uint32_t v) {
  size_t n = 0;
  do {
    uint8_t b = v & 0x7f;
    v >>= 7;
    if (v) b |= 0x80;
    o[n++] = b;
  } while (v);
  return n;
}

/* Decoder.readUint32 (encoding.js:341-360): at most 5 bytes, value < 2^32 */
static int get_uleb32(const uint8_t *p, size_t len, size_t *pos, uint32_t *v) {
  uint64_t r = 0;
  int shift = 0;
  while (*pos < len) {
    uint8_t b = p[(*pos)++];
    if (shift == 28 && (b & 0xf0)) return -1; /* out of range */
    r |= (uint64_t)(b & 0x7f) << shift;
    shift += 7;
    if (!(b & 0x80)) {
      *v = (uint32_t)r;
      return 0;
    }
  }
  return -1; /* incomplete number */
}

/* getProbes (sync.js:90-104): three little-endian u32 from hash bytes 0..11, triple hashing */
static void probes(const uint8_t *h, uint64_t modulo, uint32_t nprobes, uint64_t *out) {
  uint64_t x = ((uint64_t)h[0] | (uint64_t)h[1] << 8 | (uint64_t)h[2] << 16 | (uint64_t)h[3] << 24) % modulo;
  uint64_t y = ((uint64_t)h[4] | (uint64_t)h[5] << 8 | (uint64_t)h[6] << 16 | (uint64_t)h[7] << 24) % modulo;
  uint64_t z = ((uint64_t)h[8] | (uint64_t)h[9] << 8 | (uint64_t)h[10] << 16 | (uint64_t)h[11] << 24) % modulo;
  out[0] = x;
  for (uint32_t i = 1; i < nprobes; i++) {
    x = (x + y) % modulo;
    y = (y + z) % modulo;
    out[i] = x;
  }
}

size_t oc_bloom_build(const uint8_t *hashes32, size_t n, uint8_t *out, size_t cap) {
  if (n == 0) return 0; /* numEntries 0 -> empty byte array */
  const size_t nbits = (n * BITS_PER_ENTRY + 7) / 8;
  uint8_t hdr[15];
  size_t hl = put_uleb32(hdr, (uint32_t)n);
  hl += put_uleb32(hdr + hl, BITS_PER_ENTRY);
  hl += put_uleb32(hdr + hl, NUM_PROBES);
  if (hl + nbits > cap) return hl + nbits;
  memcpy(out, hdr, hl);
  uint8_t *bits = out + hl;
  memset(bits, 0, nbits);
  uint64_t p[NUM_PROBES];
  for (size_t i = 0; i < n; i++) {
    probes(hashes32 + 32 * i, 8 * (uint64_t)nbits, NUM_PROBES, p);
    for (int k = 0; k < NUM_PROBES; k++) bits[p[k] >> 3] |= (uint8_t)(1u << (p[k] & 7));
  }
  return hl + nbits;
}

/* 1 contains, 0 not, -1 malformed filter */
int oc_bloom_contains(const uint8_t *f, size_t len, const uint8_t *hash32) {
  if (len == 0) return 0;
  size_t pos = 0;
  uint32_t ne, bpe, np;
  if (get_uleb32(f, len, &pos, &ne) || get_uleb32(f, len, &pos, &bpe) || get_uleb32(f, len, &pos, &np)) return -1;
  const uint64_t nbytes = ((uint64_t)ne * bpe + 7) / 8;
  if (pos + nbytes > len) return -1; /* readRawBytes: subarray exceeds buffer size */
  if (ne == 0) return 0;
  const uint64_t modulo = 8 * nbytes;
  if (modulo == 0) return 0;
  const uint8_t *bits = f + pos;
  uint64_t x = 0, y = 0, z = 0;
  {
    const uint8_t *h = hash32;
    x = ((uint64_t)h[0] | (uint64_t)h[1] << 8 | (uint64_t)h[2] << 16 | (uint64_t)h[3] << 24) % modulo;
    y = ((uint64_t)h[4] | (uint64_t)h[5] << 8 | (uint64_t)h[6] << 16 | (uint64_t)h[7] << 24) % modulo;
    z = ((uint64_t)h[8] | (uint64_t)h[9] << 8 | (uint64_t)h[10] << 16 | (uint64_t)h[11] << 24) % modulo;
  }
  /* getProbes returns [x] before its loop (sync.js:95-100): numProbes 0 still tests one bit */
  const uint32_t nprobe = np > 0 ? np : 1;
  for (uint32_t i = 0; i < nprobe; i++) {
    if (i) {
      x = (x + y) % modulo;
      y = (y + z) % modulo;
    }
    if (!(bits[x >> 3] & (1u << (x & 7)))) return 0;
  }
  return 1;
}

/* getChangesToSend with a non-empty `have` list, without the explicit `need` hashes (the caller
 * adds those): changes [0, n) in getChanges order, dep_idx[dep_off[i] .. dep_off[i+1]) = indexes
 * of change i's deps within the list (-1 = not in the list). send[i] = 1 when change i is absent
 * from every filter or (transitively) depends on such a change. */
void oc_sync_select(size_t n, const uint8_t *hashes32, const uint32_t *dep_off, const int32_t *dep_idx,
                    size_t nfilt, const uint8_t *const *filters, const size_t *flens, uint8_t *send) {
  for (size_t i = 0; i < n; i++) {
    int neg = 1;
    for (size_t f = 0; f < nfilt && neg; f++)
      if (oc_bloom_contains(filters[f], flens[f], hashes32 + 32 * i) == 1) neg = 0;
    send[i] = (uint8_t)neg;
  }
  /* dependents closure (sync.js:281-292): iterate to a fixed point */
  int changed = 1;
  while (changed) {
    changed = 0;
    for (size_t i = 0; i < n; i++) {
      if (send[i]) continue;
      for (uint32_t q = dep_off[i]; q < dep_off[i + 1]; q++) {
        const int32_t d = dep_idx[q];
        if (d >= 0 && send[d]) {
          send[i] = 1;
          changed = 1;
          break;
        }
      }
    }
  }
}
