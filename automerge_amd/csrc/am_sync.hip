// am_sync.hip -- batched sync.js Bloom filters and change selection.
//
//   k_bloom_build   <- new BloomFilter(hashes).bytes         sync.js:38-47, 66-77, 90-110
//   k_bloom_probe   <- new BloomFilter(bytes).containsHash   sync.js:48-59, 112-125
//   k_sync_select   <- getChangesToSend (have non-empty)      sync.js:246-306
//
// Integer/byte work, HBM-bound in principle (12 bytes read per hash + the filter bits), tiny
// per unit: one thread per filter / probe / document pair. The build keeps each filter's bits in
// an LDS slot (word-major, so the 64 lanes of a wave hit 64 different banks) when it fits 64 bytes
// (<= 51 entries; C5 has 10), else it updates the output bytes in place. The probe kernel bounds
// numProbes (a decoded filter may claim up to 2^32-1) so a malformed filter cannot stall a wave.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <vector>

#include "am_launch.h"

#define BLOOM_BITS_PER_ENTRY 10
#define BLOOM_PROBES 7
#define BLOOM_MAX_PROBES 4096
#define BLOOM_SLOT_WORDS 16  // 64-byte LDS slot per thread
#define SYNC_T 256

// probe outcome codes (kernel -> host)
enum : uint8_t { BP_NO = 0, BP_YES = 1, BP_RANGE = 2, BP_INCOMPLETE = 3, BP_SUBARRAY = 4, BP_TOO_MANY = 5, BP_INDEX = 6 };

__host__ __device__ static inline uint32_t uleb32_len(uint32_t v) {
  uint32_t n = 1;
  while (v >= 128) { v >>= 7; n++; }
  return n;
}
__host__ __device__ static inline uint64_t bloom_bits_bytes(uint64_t n) { return (n * BLOOM_BITS_PER_ENTRY + 7) / 8; }
__host__ __device__ static inline uint64_t bloom_size(uint64_t n) {
  return n ? uleb32_len((uint32_t)n) + uleb32_len(BLOOM_BITS_PER_ENTRY) + uleb32_len(BLOOM_PROBES) + bloom_bits_bytes(n) : 0;
}

// first probe and the two steps of the triple hashing (getProbes, sync.js:90-104)
struct Probe {
  uint64_t x, y, z, m;
  __host__ __device__ void init(const uint8_t* h, uint64_t modulo) {
    const uint32_t a = (uint32_t)h[0] | (uint32_t)h[1] << 8 | (uint32_t)h[2] << 16 | (uint32_t)h[3] << 24;
    const uint32_t b = (uint32_t)h[4] | (uint32_t)h[5] << 8 | (uint32_t)h[6] << 16 | (uint32_t)h[7] << 24;
    const uint32_t c = (uint32_t)h[8] | (uint32_t)h[9] << 8 | (uint32_t)h[10] << 16 | (uint32_t)h[11] << 24;
    m = modulo;
    if (modulo <= 0xffffffffull) {
      const uint32_t m32 = (uint32_t)modulo;
      x = a % m32; y = b % m32; z = c % m32;
    } else {
      x = a % modulo; y = b % modulo; z = c % modulo;
    }
  }
  // x, y, z < m: (x + y) % m without a division
  __host__ __device__ void step() {
    x += y; if (x >= m) x -= m;
    y += z; if (y >= m) y -= m;
  }
};

// One filter: header + bits. slot = this thread's 64-byte LDS slot (word w at slot[w * stride]),
// or nullptr to update the output bytes in place.
__host__ __device__ static void bloom_build_one(const uint8_t* hashes, uint64_t h0, uint64_t n, uint8_t* o, uint32_t* slot,
                                                uint32_t stride) {
  uint32_t hl = 0;
  for (uint32_t v = (uint32_t)n;;) {  // header: numEntries, numBitsPerEntry, numProbes (uleb32)
    const uint8_t b = v & 0x7f;
    v >>= 7;
    o[hl++] = v ? (b | 0x80) : b;
    if (!v) break;
  }
  o[hl++] = BLOOM_BITS_PER_ENTRY;
  o[hl++] = BLOOM_PROBES;
  uint8_t* bits = o + hl;
  const uint64_t nb = bloom_bits_bytes(n), modulo = 8 * nb;
  if (slot && nb <= 4 * BLOOM_SLOT_WORDS) {
    for (int w = 0; w < BLOOM_SLOT_WORDS; w++) slot[w * stride] = 0;
    for (uint64_t i = 0; i < n; i++) {
      Probe p;
      p.init(hashes + 32 * (h0 + i), modulo);
      for (int k = 0; k < BLOOM_PROBES; k++) {
        if (k) p.step();
        slot[(uint32_t)(p.x >> 5) * stride] |= 1u << (p.x & 31);  // byte x>>3, bit x&7 (little endian)
      }
    }
    for (uint64_t q = 0; q < nb; q++) bits[q] = (uint8_t)(slot[(uint32_t)(q >> 2) * stride] >> (8 * (q & 3)));
  } else {
    for (uint64_t q = 0; q < nb; q++) bits[q] = 0;
    for (uint64_t i = 0; i < n; i++) {
      Probe p;
      p.init(hashes + 32 * (h0 + i), modulo);
      for (int k = 0; k < BLOOM_PROBES; k++) {
        if (k) p.step();
        bits[p.x >> 3] |= (uint8_t)(1u << (p.x & 7));
      }
    }
  }
}

__global__ void __launch_bounds__(SYNC_T) k_bloom_build(const uint8_t* __restrict__ hashes, const uint64_t* __restrict__ hoff,
                                                       uint32_t nfilt, uint8_t* __restrict__ out,
                                                       const uint64_t* __restrict__ foff) {
  __shared__ uint32_t slot[BLOOM_SLOT_WORDS * SYNC_T];
  const uint32_t t = threadIdx.x;
  const uint32_t f = blockIdx.x * SYNC_T + t;
  if (f >= nfilt) return;
  const uint64_t h0 = hoff[f], n = hoff[f + 1] - h0;
  if (n == 0) return;  // numEntries 0 -> empty encoding
  bloom_build_one(hashes, h0, n, out + foff[f], slot + t, SYNC_T);
}

__host__ __device__ static inline uint8_t rd_uleb32(const uint8_t* p, uint64_t len, uint64_t& pos, uint32_t& v) {
  uint64_t r = 0;
  int shift = 0;
  while (pos < len) {
    const uint8_t b = p[pos++];
    if (shift == 28 && (b & 0xf0)) return BP_RANGE;
    r |= (uint64_t)(b & 0x7f) << shift;
    shift += 7;
    if (!(b & 0x80)) { v = (uint32_t)r; return BP_NO; }
  }
  return BP_INCOMPLETE;
}

// new BloomFilter(bytes) header decode (sync.js:47-58): BP_NO when well formed (or empty), else the
// error code; the filter's bits are at f + pos, nbytes long.
__host__ __device__ static uint8_t bloom_header(const uint8_t* f, uint64_t len, uint64_t& pos, uint32_t& ne, uint32_t& np,
                                                uint64_t& nbytes) {
  pos = 0; ne = 0; np = 0; nbytes = 0;
  if (len == 0) return BP_NO;
  uint32_t bpe;
  uint8_t e;
  if ((e = rd_uleb32(f, len, pos, ne)) || (e = rd_uleb32(f, len, pos, bpe)) || (e = rd_uleb32(f, len, pos, np))) return e;
  nbytes = ((uint64_t)ne * bpe + 7) / 8;
  if (pos + nbytes > len) return BP_SUBARRAY;
  return BP_NO;
}

// BloomFilter(bytes).containsHash(hash): BP_YES / BP_NO, or an error code for a malformed filter
__host__ __device__ static uint8_t bloom_test(const uint8_t* f, uint64_t len, const uint8_t* h) {
  uint64_t pos, nbytes;
  uint32_t ne, np;
  const uint8_t e = bloom_header(f, len, pos, ne, np, nbytes);
  if (e) return e;
  if (ne == 0 || nbytes == 0) return BP_NO;
  if (np > BLOOM_MAX_PROBES) return BP_TOO_MANY;
  const uint8_t* bits = f + pos;
  Probe p;
  p.init(h, 8 * nbytes);
  // getProbes always returns [x] before its loop (sync.js:95-100): numProbes 0 still tests one bit
  const uint32_t nprobe = np > 0 ? np : 1;
  for (uint32_t k = 0; k < nprobe; k++) {
    if (k) p.step();
    if (!(bits[p.x >> 3] & (1u << (p.x & 7)))) return BP_NO;
  }
  return BP_YES;
}

__global__ void __launch_bounds__(SYNC_T) k_bloom_probe(const uint8_t* __restrict__ filters, const uint64_t* __restrict__ foff,
                                                       uint32_t nfilt, const uint8_t* __restrict__ probes,
                                                       const uint32_t* __restrict__ pfilt, uint64_t nprobe,
                                                       uint8_t* __restrict__ contains) {
  const uint64_t i = (uint64_t)blockIdx.x * SYNC_T + threadIdx.x;
  if (i >= nprobe) return;
  const uint32_t f = pfilt[i];
  if (f >= nfilt) { contains[i] = BP_INDEX; return; }
  contains[i] = bloom_test(filters + foff[f], foff[f + 1] - foff[f], probes + 32 * i);
}

// One document pair: Bloom-negative changes, then their dependents to a fixed point (at most n
// passes; each pass that continues marks at least one more change). Returns the first filter
// decode error (BP_NO when none).
__host__ __device__ static uint8_t sync_select_one(uint32_t pr, const uint64_t* coff, const uint8_t* hashes,
                                                   const uint64_t* doff, const int32_t* didx, const uint64_t* pfoff,
                                                   const uint8_t* filters, const uint64_t* foff, uint8_t* send) {
  const uint64_t c0 = coff[pr], c1 = coff[pr + 1], f0 = pfoff[pr], f1 = pfoff[pr + 1];
  // every `have` filter is decoded before selection (sync.js:252-256): the first malformed one fails
  // the pair even when no change would probe it
  for (uint64_t f = f0; f < f1; f++) {
    uint64_t pos, nbytes;
    uint32_t ne, np;
    const uint8_t e = bloom_header(filters + foff[f], foff[f + 1] - foff[f], pos, ne, np, nbytes);
    if (e) {
      for (uint64_t c = c0; c < c1; c++) send[c] = 0;
      return e;
    }
  }
  uint8_t st = BP_NO;
  for (uint64_t c = c0; c < c1; c++) {
    uint8_t neg = 1;
    for (uint64_t f = f0; f < f1 && neg; f++) {
      const uint8_t r = bloom_test(filters + foff[f], foff[f + 1] - foff[f], hashes + 32 * c);
      if (r == BP_YES) neg = 0;
      else if (r != BP_NO && st == BP_NO) st = r;
    }
    send[c] = neg;
  }
  const uint64_t n = c1 - c0;
  for (uint64_t pass = 0; pass <= n; pass++) {
    bool changed = false;
    for (uint64_t c = c0; c < c1; c++) {
      if (send[c]) continue;
      for (uint64_t q = doff[c]; q < doff[c + 1]; q++) {
        const int32_t d = didx[q];
        if (d >= 0 && (uint64_t)d < n && send[c0 + d]) { send[c] = 1; changed = true; break; }
      }
    }
    if (!changed) break;
  }
  return st;
}

__global__ void __launch_bounds__(SYNC_T) k_sync_select(uint32_t npairs, const uint64_t* __restrict__ coff,
                                                       const uint8_t* __restrict__ hashes, const uint64_t* __restrict__ doff,
                                                       const int32_t* __restrict__ didx, const uint64_t* __restrict__ pfoff,
                                                       const uint8_t* __restrict__ filters, const uint64_t* __restrict__ foff,
                                                       uint8_t* __restrict__ send, uint8_t* __restrict__ status) {
  const uint32_t pr = blockIdx.x * SYNC_T + threadIdx.x;
  if (pr >= npairs) return;
  status[pr] = sync_select_one(pr, coff, hashes, doff, didx, pfoff, filters, foff, send);
}

#ifdef AM_SYNC_HOST_CHECK
// CPU harness hooks (tests/test_sync_kernel_host.py): the exact per-thread bodies of the kernels,
// run on the host. Built only into the test harness, never into libautomerge_amd.so.
extern "C" void amx_bloom_build_one(const uint8_t* hashes, uint64_t n, uint8_t* out, int use_slot) {
  uint32_t slot[BLOOM_SLOT_WORDS];
  bloom_build_one(hashes, 0, n, out, use_slot ? slot : nullptr, 1);
}
extern "C" uint8_t amx_bloom_test(const uint8_t* f, uint64_t len, const uint8_t* h) { return bloom_test(f, len, h); }
extern "C" uint8_t amx_sync_select_one(const uint64_t* coff, const uint8_t* hashes, const uint64_t* doff, const int32_t* didx,
                                      const uint64_t* pfoff, const uint8_t* filters, const uint64_t* foff, uint8_t* send) {
  return sync_select_one(0, coff, hashes, doff, didx, pfoff, filters, foff, send);
}
#endif

// ------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------
namespace {

// Device buffers of the engine's sync calls, kept between calls and grown on demand (a sync round
// calls these once per batch; a hipMalloc/hipFree pair per call would dominate small batches).
struct GBuf {
  uint8_t* p = nullptr;
  size_t cap = 0;
  bool ensure(size_t bytes) {
    if (bytes <= cap && p) return true;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    const size_t want = bytes + bytes / 4 + 256;
    if (hipMalloc(&p, want) != hipSuccess) { p = nullptr; return false; }
    cap = want;
    return true;
  }
  ~GBuf() { if (p) (void)hipFree(p); }
};
struct SyncCache {
  GBuf b[9];
};
template <typename T>
struct DBuf {  // view of one cached buffer of the engine
  T* p = nullptr;
  GBuf* g = nullptr;
  bool alloc(size_t n) {
    if (!g->ensure((n ? n : 1) * sizeof(T))) return false;
    p = reinterpret_cast<T*>(g->p);
    return true;
  }
};
SyncCache& sync_cache(am_engine* e) {
  void*& slot = am_engine_sync(e);
  if (!slot) slot = new SyncCache();
  return *static_cast<SyncCache*>(slot);
}

void fail(am_error* err, uint32_t code, const char* msg) {
  if (!err) return;
  err->code = code;
  err->is_type_error = 0;
  std::snprintf(err->message, sizeof(err->message), "%s", msg);
}

// RangeError text of BloomFilter(bytes) on a malformed filter (encoding.js readUint32 / readRawBytes)
bool probe_error(uint8_t r, am_error* err) {
  switch (r) {
    case BP_NO: case BP_YES: return false;
    case BP_RANGE: fail(err, AM_E_LEB_RANGE, "number out of range"); return true;
    case BP_INCOMPLETE: fail(err, AM_E_LEB_INCOMPLETE, "buffer ended with incomplete number"); return true;
    case BP_SUBARRAY: fail(err, AM_E_SUBARRAY, "subarray exceeds buffer size"); return true;
    case BP_TOO_MANY: fail(err, AM_U_VALUE, "automerge_amd: Bloom filter numProbes above 4096 is not supported"); return true;
    default: fail(err, AM_U_VALUE, "automerge_amd: probe names a filter index out of range"); return true;
  }
}

bool gpu_ok(am_error* err, hipError_t e, const char* what) {
  if (e == hipSuccess) return true;
  char m[256];
  std::snprintf(m, sizeof m, "automerge_amd: %s failed: %s", what, hipGetErrorString(e));
  fail(err, AM_U_CAPACITY, m);
  return false;
}
#define GPU(expr) do { if (!gpu_ok(err, (expr), #expr)) return 1; } while (0)

}  // namespace

void am_sync_cache_free(void* cache) { delete static_cast<SyncCache*>(cache); }

extern "C" uint64_t am_bloom_encoded_size(uint64_t nhashes) { return bloom_size(nhashes); }
// new BloomFilter(bytes) header check on the host (sync.js:47-58): 0 when well formed, else the
// RangeError the reference raises (the sync protocol decodes every `have` filter before it
// selects changes, sync.js:252-256)
extern "C" int am_bloom_check(const uint8_t* f, uint64_t len, am_error* err) {
  if (err) err->code = 0;
  uint64_t pos, nbytes;
  uint32_t ne, np;
  uint8_t e = bloom_header(f, len, pos, ne, np, nbytes);
  if (!e && ne && nbytes && np > BLOOM_MAX_PROBES) e = BP_TOO_MANY;
  return probe_error(e, err) ? 1 : 0;
}


void am_launch_bloom_build(const uint8_t* d_hashes, const uint64_t* d_hoff, uint32_t nfilt, uint8_t* d_out,
                           const uint64_t* d_foff, hipStream_t s) {
  if (nfilt) hipLaunchKernelGGL(k_bloom_build, dim3((nfilt + SYNC_T - 1) / SYNC_T), dim3(SYNC_T), 0, s, d_hashes, d_hoff, nfilt, d_out, d_foff);
}
void am_launch_bloom_probe(const uint8_t* d_filters, const uint64_t* d_foff, uint32_t nfilt, const uint8_t* d_probes,
                           const uint32_t* d_pfilt, uint64_t nprobe, uint8_t* d_contains, hipStream_t s) {
  if (nprobe)
    hipLaunchKernelGGL(k_bloom_probe, dim3((unsigned)((nprobe + SYNC_T - 1) / SYNC_T)), dim3(SYNC_T), 0, s, d_filters, d_foff,
                       nfilt, d_probes, d_pfilt, nprobe, d_contains);
}
void am_launch_sync_select(uint32_t npairs, const uint64_t* d_coff, const uint8_t* d_hashes, const uint64_t* d_doff,
                           const int32_t* d_didx, const uint64_t* d_pfoff, const uint8_t* d_filters, const uint64_t* d_foff,
                           uint8_t* d_send, uint8_t* d_status, hipStream_t s) {
  if (npairs)
    hipLaunchKernelGGL(k_sync_select, dim3((npairs + SYNC_T - 1) / SYNC_T), dim3(SYNC_T), 0, s, npairs, d_coff, d_hashes,
                       d_doff, d_didx, d_pfoff, d_filters, d_foff, d_send, d_status);
}

extern "C" int am_bloom_build(am_engine* eng, const uint8_t* hashes32, const uint64_t* hoff, uint32_t nfilt, uint8_t* out,
                              uint64_t cap, uint64_t* foff, am_error* err) {
  if (err) err->code = 0;
  foff[0] = 0;
  for (uint32_t f = 0; f < nfilt; f++) {
    if (hoff[f + 1] < hoff[f]) { fail(err, AM_U_VALUE, "automerge_amd: hash offsets must be non-decreasing"); return 1; }
    foff[f + 1] = foff[f] + bloom_size(hoff[f + 1] - hoff[f]);
  }
  const uint64_t total = foff[nfilt], nh = hoff[nfilt];
  if (total > cap) { fail(err, AM_U_CAPACITY, "automerge_amd: output buffer too small for the encoded filters"); return 1; }
  if (!nfilt || !total) return 0;
  GPU(hipSetDevice(am_engine_device(eng)));
  hipStream_t s = am_engine_stream(eng);
  SyncCache& K = sync_cache(eng);
  DBuf<uint8_t> dh{nullptr, &K.b[0]}, dout{nullptr, &K.b[1]};
  DBuf<uint64_t> dhoff{nullptr, &K.b[2]}, dfoff{nullptr, &K.b[3]};
  if (!dh.alloc(32 * nh) || !dout.alloc(total) || !dhoff.alloc(nfilt + 1) || !dfoff.alloc(nfilt + 1)) {
    fail(err, AM_U_CAPACITY, "automerge_amd: device allocation failed");
    return 1;
  }
  if (nh) GPU(hipMemcpyAsync(dh.p, hashes32, 32 * nh, hipMemcpyHostToDevice, s));
  GPU(hipMemcpyAsync(dhoff.p, hoff, 8 * (nfilt + 1), hipMemcpyHostToDevice, s));
  GPU(hipMemcpyAsync(dfoff.p, foff, 8 * (nfilt + 1), hipMemcpyHostToDevice, s));
  am_launch_bloom_build(dh.p, dhoff.p, nfilt, dout.p, dfoff.p, s);
  GPU(hipGetLastError());
  GPU(hipMemcpyAsync(out, dout.p, total, hipMemcpyDeviceToHost, s));
  GPU(hipStreamSynchronize(s));
  return 0;
}

extern "C" int am_bloom_probe(am_engine* eng, const uint8_t* filters, const uint64_t* foff, uint32_t nfilt,
                              const uint8_t* probes32, const uint32_t* pfilt, uint64_t nprobe, uint8_t* contains,
                              am_error* err) {
  if (err) err->code = 0;
  if (!nprobe) return 0;
  GPU(hipSetDevice(am_engine_device(eng)));
  hipStream_t s = am_engine_stream(eng);
  const uint64_t fbytes = foff[nfilt];
  SyncCache& K = sync_cache(eng);
  DBuf<uint8_t> df{nullptr, &K.b[0]}, dp{nullptr, &K.b[1]}, dc{nullptr, &K.b[2]};
  DBuf<uint64_t> dfo{nullptr, &K.b[3]};
  DBuf<uint32_t> dpf{nullptr, &K.b[4]};
  if (!df.alloc(fbytes) || !dp.alloc(32 * nprobe) || !dc.alloc(nprobe) || !dfo.alloc(nfilt + 1) || !dpf.alloc(nprobe)) {
    fail(err, AM_U_CAPACITY, "automerge_amd: device allocation failed");
    return 1;
  }
  if (fbytes) GPU(hipMemcpyAsync(df.p, filters, fbytes, hipMemcpyHostToDevice, s));
  GPU(hipMemcpyAsync(dfo.p, foff, 8 * (nfilt + 1), hipMemcpyHostToDevice, s));
  GPU(hipMemcpyAsync(dp.p, probes32, 32 * nprobe, hipMemcpyHostToDevice, s));
  GPU(hipMemcpyAsync(dpf.p, pfilt, 4 * nprobe, hipMemcpyHostToDevice, s));
  am_launch_bloom_probe(df.p, dfo.p, nfilt, dp.p, dpf.p, nprobe, dc.p, s);
  GPU(hipGetLastError());
  GPU(hipMemcpyAsync(contains, dc.p, nprobe, hipMemcpyDeviceToHost, s));
  GPU(hipStreamSynchronize(s));
  for (uint64_t i = 0; i < nprobe; i++)
    if (probe_error(contains[i], err)) return 1;
  return 0;
}

extern "C" int am_sync_select(am_engine* eng, uint32_t npairs, const uint64_t* coff, const uint8_t* hashes32,
                              const uint64_t* doff, const int32_t* didx, const uint64_t* pfoff, const uint8_t* filters,
                              const uint64_t* foff, uint8_t* send, am_error* err) {
  if (err) err->code = 0;
  if (!npairs) return 0;
  GPU(hipSetDevice(am_engine_device(eng)));
  hipStream_t s = am_engine_stream(eng);
  const uint64_t nc = coff[npairs], nd = doff[nc], nf = pfoff[npairs], fbytes = foff[nf];
  SyncCache& K = sync_cache(eng);
  DBuf<uint8_t> dh{nullptr, &K.b[0]}, dflt{nullptr, &K.b[1]}, dsend{nullptr, &K.b[2]}, dst{nullptr, &K.b[3]};
  DBuf<uint64_t> dcoff{nullptr, &K.b[4]}, ddoff{nullptr, &K.b[5]}, dpfoff{nullptr, &K.b[6]}, dfoff{nullptr, &K.b[7]};
  DBuf<int32_t> ddidx{nullptr, &K.b[8]};
  if (!dh.alloc(32 * nc) || !dflt.alloc(fbytes) || !dsend.alloc(nc) || !dst.alloc(npairs) || !dcoff.alloc(npairs + 1) ||
      !ddoff.alloc(nc + 1) || !dpfoff.alloc(npairs + 1) || !dfoff.alloc(nf + 1) || !ddidx.alloc(nd)) {
    fail(err, AM_U_CAPACITY, "automerge_amd: device allocation failed");
    return 1;
  }
  if (nc) GPU(hipMemcpyAsync(dh.p, hashes32, 32 * nc, hipMemcpyHostToDevice, s));
  if (fbytes) GPU(hipMemcpyAsync(dflt.p, filters, fbytes, hipMemcpyHostToDevice, s));
  if (nd) GPU(hipMemcpyAsync(ddidx.p, didx, 4 * nd, hipMemcpyHostToDevice, s));
  GPU(hipMemcpyAsync(dcoff.p, coff, 8 * (npairs + 1), hipMemcpyHostToDevice, s));
  GPU(hipMemcpyAsync(ddoff.p, doff, 8 * (nc + 1), hipMemcpyHostToDevice, s));
  GPU(hipMemcpyAsync(dpfoff.p, pfoff, 8 * (npairs + 1), hipMemcpyHostToDevice, s));
  GPU(hipMemcpyAsync(dfoff.p, foff, 8 * (nf + 1), hipMemcpyHostToDevice, s));
  am_launch_sync_select(npairs, dcoff.p, dh.p, ddoff.p, ddidx.p, dpfoff.p, dflt.p, dfoff.p, dsend.p, dst.p, s);
  GPU(hipGetLastError());
  std::vector<uint8_t> st(npairs);
  if (nc) GPU(hipMemcpyAsync(send, dsend.p, nc, hipMemcpyDeviceToHost, s));
  GPU(hipMemcpyAsync(st.data(), dst.p, npairs, hipMemcpyDeviceToHost, s));
  GPU(hipStreamSynchronize(s));
  for (uint32_t p = 0; p < npairs; p++)
    if (probe_error(st[p], err)) return 1;
  return 0;
}
