// am_capi.hip -- host side of libautomerge_amd.so: engine/batch management, the DEFLATE host stage,
// the per-document backend state (backend/backend.js semantics over the batch path) and error
// messages. All merge/codec/hash work runs in the kernels of am_kernels.hip; nothing here decodes
// op columns or merges operations. There is no CPU fallback: without a HIP device the entry points
// fail with an error.
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <zlib.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <memory>
#include <functional>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <unordered_set>
#include <vector>

#include "am_graph.h"
#include "am_launch.h"
#include "am_par.h"
#include "am_patch.h"

namespace {

struct Err {
  uint32_t code = 0;
  bool type_error = false;
  std::string msg;
};

void to_c(const Err& e, am_error* out) {
  if (!out) return;
  out->code = e.code;
  out->is_type_error = e.type_error ? 1 : 0;
  std::snprintf(out->message, sizeof(out->message), "%s", e.msg.c_str());
}

std::string hexs(const uint8_t* p, size_t n) {
  static const char* H = "0123456789abcdef";
  std::string s;
  s.reserve(2 * n);
  for (size_t i = 0; i < n; i++) { s += H[p[i] >> 4]; s += H[p[i] & 15]; }
  return s;
}

std::string fmt(const char* f, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, f);
  std::vsnprintf(buf, sizeof buf, f, ap);
  va_end(ap);
  return buf;
}

std::string numOrNull(int64_t v, bool is_actor) {
  if (is_actor ? v < 0 : v == AM_NULL64) return "null";
  return std::to_string(v);
}

// Reference error text for a status code (messages of encoding.js / columnar.js / new.js).
std::string message_for(uint32_t code, int64_t a0, int64_t a1, const std::string& actor) {
  switch (code) {
    case AM_E_MAGIC: return "Data does not begin with magic bytes 85 6f 4a 83";
    case AM_E_CHECKSUM: return "checksum does not match data";
    case AM_E_SUBARRAY: return "subarray exceeds buffer size";
    case AM_E_LEB_RANGE: return "number out of range";
    case AM_E_LEB_INCOMPLETE: return "buffer ended with incomplete number";
    case AM_E_CHUNK_TYPE: return fmt("Unexpected chunk type: %lld", (long long)a0);
    case AM_E_CHANGE_TRAILING: return "Encoded change has trailing data";
    case AM_E_DOC_TRAILING: return "Encoded document has trailing data";
    case AM_E_COL_ORDER: return "Columns must be in ascending order";
    case AM_E_CHANGE_DEFLATED_COL: return "change must not contain deflated columns";
    case AM_E_RLE_SUCC_REP: return "Successive repetitions with the same value are not allowed";
    case AM_E_RLE_REP1: return "Repetition count of 1 is not allowed, use a literal instead";
    case AM_E_RLE_SUCC_LIT: return "Successive literals are not allowed";
    case AM_E_RLE_SUCC_NULL: return "Successive null runs are not allowed";
    case AM_E_RLE_ZERO_NULL: return "Zero-length null runs are not allowed";
    case AM_E_RLE_LIT_REP: return "Repetition of values is not allowed in literal";
    case AM_E_BOOL_ZERO_RUN: return "Zero-length runs are not allowed";
    case AM_E_REUSE_SEQ: return fmt("Reuse of sequence number %lld for actor %s", (long long)a0, actor.c_str());
    case AM_E_SKIPPED_SEQ: return fmt("Skipped sequence number %lld for actor %s", (long long)a0, actor.c_str());
    case AM_E_FIRST_SEQ: return fmt("Seq %lld is the first change for actor %s", (long long)a0, actor.c_str());
    case AM_E_UNKNOWN_ACTOR: return fmt("actorId %s is not known to document", actor.c_str());
    case AM_E_NO_ACTOR_INDEX: return fmt("No actor index %lld", (long long)a0);
    case AM_E_MISMATCH_OBJ:
      return "Mismatched object reference: (" + numOrNull(a0, false) + ", " + numOrNull(a1, true) + ")";
    case AM_E_MISMATCH_KEY:
      return "Mismatched operation key: (" + numOrNull(a0, false) + ", " + numOrNull(a1, true) + ")";
    case AM_E_PRED_NOT_FOUND: return fmt("no matching operation for pred: %lld@%s", (long long)a0, actor.c_str());
    case AM_E_REF_NOT_FOUND: return fmt("Reference element not found: %lld@%s", (long long)a0, actor.c_str());
    case AM_E_ELEM_NOT_FOUND: return fmt("could not find list element with ID: %lld@%s", (long long)a0, actor.c_str());
    case AM_E_DUP_OPID: return fmt("duplicate operation ID: %lld@%s", (long long)a0, actor.c_str());
    case AM_E_DOC_SEQ:
      return "Expected seq " + (a0 == AM_NULL64 ? std::string("NaN") : std::to_string(a0)) + ", got " +
             std::to_string(a1) + " for actor " + actor;
    case AM_E_INFLATE: return "invalid deflate data";
    case AM_U_HASH_GRAPH: return "automerge_amd: unsupported: needs the change hash graph of a loaded document";
    case AM_U_UNKNOWN_COLUMN: return "automerge_amd: unsupported: column id outside the known column set";
    case AM_U_NONCAUSAL: return "automerge_amd: unsupported: operation ids violate causal (Lamport) order";
    case AM_U_UTF8: return "automerge_amd: unsupported: invalid UTF-8 in a key or message";
    case AM_U_DEL_SHAPE: return "automerge_amd: unsupported: del operation without pred or with insert";
    case AM_U_VALUE: return "automerge_amd: unsupported value shape in the input columns";
    case AM_U_CAPACITY: return "automerge_amd: workspace capacity exceeded";
    case AM_U_INC_VALUE: return "automerge_amd: unsupported: a non-integer counter increment in the patch";
    default: return fmt("automerge_amd: error %u", code);
  }
}

#define HIPCHECK(expr)                                                                    \
  do {                                                                                    \
    hipError_t _e = (expr);                                                               \
    if (_e != hipSuccess) {                                                               \
      std::fprintf(stderr, "automerge_amd: %s failed: %s\n", #expr, hipGetErrorString(_e)); \
      return false;                                                                       \
    }                                                                                     \
  } while (0)

template <typename T>
struct DevBuf {
  T* p = nullptr;
  size_t cap = 0;
  bool ensure(size_t n) {
    if (n <= cap && p) return true;
    if (p) { (void)hipFree(p); p = nullptr; cap = 0; }
    size_t bytes = (n ? n : 1) * sizeof(T);
    if (hipMalloc(&p, bytes) != hipSuccess) { p = nullptr; return false; }
    cap = n ? n : 1;
    return true;
  }
  ~DevBuf() { if (p) (void)hipFree(p); }
};

// ---- minimal host-side LEB128 / container handling for the DEFLATE stage ----
struct HRd {
  const uint8_t* p;
  size_t n, off;
  bool ok = true;
  uint64_t u() {
    uint64_t v = 0;
    int sh = 0;
    while (off < n) {
      uint8_t b = p[off++];
      if (sh < 64) v |= (uint64_t)(b & 0x7f) << sh;
      sh += 7;
      if (!(b & 0x80)) return v;
    }
    ok = false;
    return 0;
  }
  const uint8_t* raw(size_t k) {
    if (off + k > n) { ok = false; return p; }
    const uint8_t* r = p + off;
    off += k;
    return r;
  }
};
void put_u(std::vector<uint8_t>& o, uint64_t v) {
  do { uint8_t b = v & 0x7f; v >>= 7; o.push_back(b | (v ? 0x80 : 0)); } while (v);
}

bool zinflate(const uint8_t* p, size_t n, std::vector<uint8_t>& out) {
  size_t cap = n * 4 + 64;
  for (int attempt = 0; attempt < 16; attempt++) {
    out.resize(cap);
    z_stream zs;
    std::memset(&zs, 0, sizeof zs);
    if (inflateInit2(&zs, -15) != Z_OK) return false;
    zs.next_in = const_cast<Bytef*>(p);
    zs.avail_in = (uInt)n;
    zs.next_out = out.data();
    zs.avail_out = (uInt)cap;
    int r = inflate(&zs, Z_FINISH);
    size_t got = zs.total_out;
    inflateEnd(&zs);
    if (r == Z_STREAM_END) { out.resize(got); return true; }
    if (r == Z_BUF_ERROR && zs.avail_out == 0) { cap *= 4; continue; }
    return false;
  }
  return false;
}
// pako.deflateRaw defaults: level 6, memLevel 8, windowBits 15 (raw), default strategy
bool zdeflate(const uint8_t* p, size_t n, std::vector<uint8_t>& out) {
  z_stream zs;
  std::memset(&zs, 0, sizeof zs);
  if (deflateInit2(&zs, 6, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY) != Z_OK) return false;
  out.resize(deflateBound(&zs, (uLong)n) + 16);
  zs.next_in = const_cast<Bytef*>(p);
  zs.avail_in = (uInt)n;
  zs.next_out = out.data();
  zs.avail_out = (uInt)out.size();
  int r = deflate(&zs, Z_FINISH);
  size_t got = zs.total_out;
  deflateEnd(&zs);
  if (r != Z_STREAM_END) return false;
  out.resize(got);
  return true;
}

// AM_SYNC_PROFILE=1: stage wall times of the batched per-handle calls and the host stages on stderr
struct HostClock {
  bool on = std::getenv("AM_SYNC_PROFILE") != nullptr;
  std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
  std::string line;
  void mark(const char* what) {
    if (!on) return;
    const auto now = std::chrono::steady_clock::now();
    char b[64];
    std::snprintf(b, sizeof b, " %s=%.1fms", what, std::chrono::duration<double, std::milli>(now - t).count());
    line += b;
    t = now;
  }
  void print(const char* call, size_t n) {
    if (on) std::fprintf(stderr, "[am_batch] %s n=%zu%s\n", call, n, line.c_str());
  }
};

struct ColEnt { uint64_t id; std::vector<uint8_t> data; };
struct DocParts {
  std::vector<uint8_t> pre;  // actors + heads (verbatim)
  std::vector<ColEnt> ccols, ocols;
  std::vector<uint8_t> post; // headsIndexes + extra bytes (verbatim)
  uint32_t nheads = 0;
  const uint8_t* heads = nullptr;
};
// Splits a document chunk's data (decodeDocumentHeader layout, columnar.js:1006-1038).
bool split_doc(const uint8_t* data, size_t n, DocParts& d) {
  HRd r{data, n, 0};
  uint64_t na = r.u();
  for (uint64_t i = 0; i < na && r.ok; i++) r.raw(r.u());
  uint64_t nh = r.u();
  d.heads = r.raw(32 * nh);
  d.nheads = (uint32_t)nh;
  d.pre.assign(data, data + r.off);
  auto table = [&](std::vector<ColEnt>& cols) {
    uint64_t nc = r.u();
    for (uint64_t i = 0; i < nc && r.ok; i++) {
      ColEnt c;
      c.id = r.u();
      c.data.resize(r.u());
      cols.push_back(std::move(c));
    }
  };
  table(d.ccols);
  table(d.ocols);
  for (auto* cols : {&d.ccols, &d.ocols})
    for (auto& c : *cols) {
      const uint8_t* p = r.raw(c.data.size());
      if (!r.ok) return false;
      if (!c.data.empty()) std::memcpy(c.data.data(), p, c.data.size());
    }
  d.post.assign(data + r.off, data + n);
  return r.ok;
}
std::vector<uint8_t> join_doc(const DocParts& d) {
  std::vector<uint8_t> body(d.pre);
  for (auto* cols : {&d.ccols, &d.ocols}) {
    put_u(body, cols->size());
    for (auto& c : *cols) { put_u(body, c.id); put_u(body, c.data.size()); }
  }
  for (auto* cols : {&d.ccols, &d.ocols})
    for (auto& c : *cols) body.insert(body.end(), c.data.begin(), c.data.end());
  body.insert(body.end(), d.post.begin(), d.post.end());
  return body;
}

struct Container {
  uint8_t type = 0;
  size_t data_off = 0, data_len = 0, end = 0;
};
bool read_container(const uint8_t* p, size_t n, Container& c) {
  if (n < 9) return false;
  HRd r{p, n, 9};
  c.type = p[8];
  c.data_len = r.u();
  c.data_off = r.off;
  r.raw(c.data_len);
  c.end = r.off;
  return r.ok;
}
std::vector<uint8_t> make_chunk(const uint8_t checksum[4], uint8_t type, const std::vector<uint8_t>& data) {
  std::vector<uint8_t> o = {0x85, 0x6f, 0x4a, 0x83, checksum[0], checksum[1], checksum[2], checksum[3], type};
  put_u(o, data.size());
  o.insert(o.end(), data.begin(), data.end());
  return o;
}

}  // namespace

// =============================================================================================
// engine / batch
// =============================================================================================
// Pinned host memory follows the caller's NUMA policy (hipHostMallocNumaUser): a rank that bound
// itself to its GPU's NUMA node before its first GPU call (bench.py) gets its staging arenas on that
// node, the host-link copies then stay on the socket the GPU hangs off. AM_PINNED_NUMA=0: the
// runtime's default placement.
static unsigned pinned_flags() {
  static const unsigned f = [] {
    const char* v = std::getenv("AM_PINNED_NUMA");
    return (v && v[0] == '0') ? (unsigned)hipHostMallocDefault : (unsigned)hipHostMallocNumaUser;
  }();
  return f;
}
// pinned host memory (hipHostMalloc), grow-only (by at least half again)
template <class T>
struct PinBuf {
  T* p = nullptr;
  size_t cap = 0;
  bool ensure(size_t n) {
    if (n <= cap && p) return true;
    const size_t want = std::max<size_t>(n ? n : 1, cap + cap / 2);
    HostClock clk;
    if (p) { (void)hipHostFree(p); p = nullptr; cap = 0; }
    if (hipHostMalloc(reinterpret_cast<void**>(&p), want * sizeof(T), pinned_flags()) != hipSuccess) {
      p = nullptr;
      return false;
    }
    cap = want;
    clk.mark("alloc");
    clk.print("pinned", want * sizeof(T));
    return true;
  }
  ~PinBuf() { if (p) (void)hipHostFree(p); }
};
// device arenas the batched per-handle calls compact their outputs into (k_pipe_compact), and the
// pinned host buffers their input arena is packed into and their outputs come home in (no
// zero-filled std::vector per call, DMA-speed copies)
struct CollectBufs {
  DevBuf<uint64_t> olen, ooff, plen, poff, tmp, totals;
  DevBuf<am_doc_summary> summ;
  DevBuf<uint8_t> out, pat, hashes;
  PinBuf<uint8_t> h_arena, h_out, h_pat;
  PinBuf<am_doc_summary> h_summ;
};
struct am_engine {
  int device = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev[5] = {};
  am_batch* scratch = nullptr;  // batch reused by the per-document API
  void* hist = nullptr;         // device buffers of the history batches (am_hist.hip)
  void* sync = nullptr;         // device buffers of the Bloom / selection calls (am_sync.hip)
  CollectBufs* coll = nullptr;  // the batched per-handle calls
  uint64_t stat_docs = 0;       // documents of the per-handle calls (run_one / run_many) since the last am_engine_stats
  uint64_t stat_fast = 0;       // of those, merged by k_doc_fast
};

// A saved document's container and header as the host stage reads them (decodeDocumentHeader,
// columnar.js:1006-1038): offsets are chunk-relative; columns = the change columns, then the op
// columns, each with its id, length and data offset; [post, end) = headsIndexes + extra bytes.
struct DocLayout {
  uint64_t data_off = 0, end = 0, pre_end = 0, post = 0;
  uint32_t nc = 0;
  std::vector<uint64_t> id, len, off;
  bool deflated = false;
};
// The inflate stage's host tables and device buffers, kept by the batch between stages (a batch
// staged every step reuses their capacity: no page faults, no hipMalloc / hipFree per stage)
struct InflateScratch {
  std::vector<uint8_t> kind, hash, blob;
  std::vector<uint32_t> nzs, dat, z0, ord, zlen, nseg, s0, sha_of;
  std::vector<int64_t> base_of;
  std::vector<uint64_t> hoff;
  std::vector<DocLayout> lay;
  std::vector<am_zstream> zs;
  std::vector<am_chunk_desc> nc, sha;
  std::vector<std::vector<uint8_t>> dhdr;
  std::vector<std::vector<uint64_t>> dcl;
  std::vector<am_seg> seg;
  DevBuf<am_zstream> d_zs;
  DevBuf<uint32_t> d_zlen, d_ord;
  DevBuf<am_chunk_desc> d_sha;
  DevBuf<uint8_t> d_hash, d_arena, d_blob;  // d_arena: the rebuilt arena; swapped with the batch's
  DevBuf<am_seg> d_seg;
  // the device-side stage (inflate_stage_dev)
  DevBuf<uint8_t> d_isbase;
  DevBuf<uint64_t> d_cnt, d_z0, d_csrc, d_tmp, d_tot;
  DevBuf<uint32_t> d_clen, d_zid;
};

struct am_batch {
  am_engine* eng = nullptr;
  std::unique_ptr<InflateScratch> zscr;
  DevBuf<uint8_t> arena;
  DevBuf<am_chunk_desc> chunks;
  DevBuf<am_doc_desc> docs;
  DevBuf<am_known_hash> known;
  DevBuf<ChunkInfo> info;
  DevBuf<HdrSlot> hdr;
  DevBuf<DocBounds> bounds;
  DevBuf<uint64_t> ws_bytes, ws_off, scan_tmp, ws_total, max_hot;
  DevBuf<uint8_t> fast_done;
  DevBuf<uint32_t> rest;  // k_rest's list of what k_doc_fast left
  uint32_t fast_lds = 0;
  bool fast_only = false;
  bool any_diff = false;
  bool compact = false;       // k_doc_fast's documents get the compact workspace plan (ws_layout)
  uint32_t lds_bytes = 0;
  uint64_t max_hot_v = 0;
  DevBuf<uint8_t> ws;
  DevBuf<am_doc_result> results;
  DevBuf<int32_t> chg_state;
  uint32_t nchunks = 0, ndocs = 0;
  uint64_t ws_need = 0;       // workspace held: the scanned plans + the overflow reserve
  uint64_t ws_plan = 0;       // the scanned plans alone (compact plans for k_doc_fast's documents)
  uint32_t fast_cap = 0xffffffffu;  // compact plans only for fast slices up to this (a pipeline: its fast_lds)
  uint64_t ws_limit = 0;      // diagnostics (a pipeline under AM_DEBUG_WS_CANARY): the kernels' workspace size,
                              // canary bytes after it
  bool fresh = false;         // staged and not run since: the sizing pass's chunk info and plans stand
  bool timed = false;
  uint32_t inflated = 0;      // change chunks inflated on the GPU by the last stage
  float inflate_ms = 0.f;     // their two inflate passes (HIP events)
  bool inflate_ev = false;    // inflate_ms still to be read from the events (device-side stage)
  uint64_t inflated_bytes = 0;

  BatchDev dev() {
    BatchDev b;
    b.arena = arena.p; b.chunks = chunks.p; b.docs = docs.p; b.known = known.p; b.info = info.p; b.hdr = hdr.p; b.bounds = bounds.p;
    b.ws_bytes = ws_bytes.p; b.ws_off = ws_off.p; b.scan_tmp = scan_tmp.p; b.ws_total = ws_total.p; b.max_hot = max_hot.p; b.lds_bytes = lds_bytes; b.max_hot_host = max_hot_v; b.ws = ws.p;
    b.fast_lds = fast_lds; b.fast_done = fast_done.p; b.fast_only = fast_only; b.any_diff = any_diff; b.rest = rest.p;
    b.compact = compact; b.fast_cap = fast_cap;
    b.ws_cap = ws_limit ? ws_limit : ws.cap; b.results = results.p; b.chg_state = chg_state.p; b.nchunks = nchunks; b.ndocs = ndocs;
    return b;
  }
};

static bool set_device(am_engine* e) { return hipSetDevice(e->device) == hipSuccess; }

extern "C" const char* am_version(void) { return "automerge_amd 0.1 (gfx950)"; }

// accessors for the other translation units (am_launch.h)
hipStream_t am_engine_stream(am_engine* e) { return e->stream; }
int am_engine_device(am_engine* e) { return e->device; }
void*& am_engine_hist(am_engine* e) { return e->hist; }
void*& am_engine_sync(am_engine* e) { return e->sync; }

extern "C" am_engine* am_engine_create(int device, am_error* err) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= device || device < 0) {
    Err e{AM_U_CAPACITY, false, "automerge_amd: no HIP device available (MI355X required; no CPU fallback)"};
    to_c(e, err);
    return nullptr;
  }
  am_engine* eng = new am_engine();
  eng->device = device;
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&eng->stream, hipStreamNonBlocking) != hipSuccess) {
    delete eng;
    Err e{AM_U_CAPACITY, false, "automerge_amd: cannot create a HIP stream"};
    to_c(e, err);
    return nullptr;
  }
  for (auto& ev : eng->ev) (void)hipEventCreate(&ev);
  if (err) err->code = 0;
  return eng;
}

extern "C" void am_batch_destroy(am_batch* b) {
  if (!b) return;
  set_device(b->eng);
  delete b;
}

extern "C" void am_engine_destroy(am_engine* eng) {
  if (!eng) return;
  set_device(eng);
  am_batch_destroy(eng->scratch);
  am_hist_cache_free(eng->hist);
  am_sync_cache_free(eng->sync);
  delete eng->coll;
  for (auto& ev : eng->ev) (void)hipEventDestroy(ev);
  (void)hipStreamDestroy(eng->stream);
  delete eng;
}

extern "C" am_batch* am_batch_create(am_engine* eng) {
  am_batch* b = new am_batch();
  b->eng = eng;
  return b;
}

static bool doc_layout(const uint8_t* p, uint64_t n, DocLayout& L) {
  Container c;
  if (n < 9 || std::memcmp(p, "\x85\x6f\x4a\x83", 4) != 0 || !read_container(p, n, c) || c.type != 0) return false;
  HRd r{p, c.end, c.data_off};
  L.data_off = c.data_off;
  L.end = c.end;
  const uint64_t na = r.u();
  for (uint64_t i = 0; i < na && r.ok; i++) r.raw(r.u());
  const uint64_t nh = r.u();
  r.raw(32 * nh);
  if (!r.ok) return false;
  L.pre_end = r.off;
  for (int t = 0; t < 2 && r.ok; t++) {
    const uint64_t k = r.u();
    if (k > 4096) return false;
    if (t == 0) L.nc = (uint32_t)k;
    for (uint64_t i = 0; i < k && r.ok; i++) {
      L.id.push_back(r.u());
      L.len.push_back(r.u());
    }
  }
  for (size_t i = 0; i < L.id.size() && r.ok; i++) {
    L.off.push_back(r.off);
    r.raw(L.len[i]);
    L.deflated |= (L.id[i] & COL_DEFLATE) != 0;
  }
  L.post = r.off;
  return r.ok;
}

// The device-side form of the stage below for a batch whose compressed chunks are all changes (no
// saved document with DEFLATEd columns): the same classification, stream table, layout and
// headers, computed by kernels over the chunks (am_launch_zstage_*), so the host reads no chunk
// byte and waits twice for a total (the streams, the new arena's size). AM_ZSTAGE_DEV=0 keeps the
// host form; batches under AM_ZSTAGE_DEV_MIN chunks (default 1024) use it too.
static bool zstage_dev_on(uint32_t nchunks) {
  const char* e = std::getenv("AM_ZSTAGE_DEV");
  if (e && e[0] == '0') return false;
  const char* m = std::getenv("AM_ZSTAGE_DEV_MIN");
  return nchunks >= (m ? (uint32_t)std::strtoul(m, nullptr, 10) : 1024u);
}
static bool inflate_stage_dev(am_batch* b, uint64_t arena_len, uint32_t nchunks, uint32_t ndocs, HostClock& clk) {
  InflateScratch& X = *b->zscr;
  hipStream_t s = b->eng->stream;
  if (!X.d_isbase.ensure(nchunks) || !X.d_cnt.ensure(nchunks) || !X.d_z0.ensure(nchunks) || !X.d_csrc.ensure(nchunks) ||
      !X.d_clen.ensure(nchunks) || !X.d_zid.ensure(nchunks) || !X.d_tmp.ensure(am_scan_tmp_elems(nchunks)) || !X.d_tot.ensure(1))
    return false;
  am_launch_zstage_classify(b->arena.p, arena_len, b->chunks.p, nchunks, b->docs.p, ndocs, X.d_isbase.p, X.d_cnt.p,
                            X.d_csrc.p, X.d_clen.p, s);
  am_launch_scan(X.d_cnt.p, X.d_z0.p, X.d_tmp.p, nchunks, X.d_tot.p, s);
  uint64_t tot = 0;
  HIPCHECK(hipMemcpyAsync(&tot, X.d_tot.p, sizeof tot, hipMemcpyDeviceToHost, s));
  HIPCHECK(hipStreamSynchronize(s));
  HIPCHECK(hipGetLastError());
  const uint32_t nz = (uint32_t)tot, nlong = (uint32_t)(tot >> 32);
  clk.mark("classify");
  b->inflated = nz;
  b->inflate_ms = 0.f;
  b->inflate_ev = false;
  if (!nz) {
    clk.print("inflate_stage_dev", nchunks);
    return true;
  }
  if (!X.d_zs.ensure(nz) || !X.d_zlen.ensure(nz) || !X.d_ord.ensure(nz)) return false;
  am_launch_zstage_fill(X.d_cnt.p, X.d_z0.p, nchunks, nlong, X.d_csrc.p, X.d_clen.p, X.d_zs.p, X.d_ord.p, X.d_zid.p, s);
  (void)hipEventRecord(b->eng->ev[0], s);
  am_launch_inflate_size(b->arena.p, X.d_zs.p, X.d_ord.p, nlong, nz, X.d_zlen.p, s);
  (void)hipEventRecord(b->eng->ev[1], s);
  // new lengths (d_cnt) -> new offsets (d_z0)
  am_launch_zstage_layout(b->arena.p, b->chunks.p, nchunks, X.d_zid.p, X.d_zlen.p, X.d_zs.p, X.d_cnt.p, s);
  am_launch_scan(X.d_cnt.p, X.d_z0.p, X.d_tmp.p, nchunks, X.d_tot.p, s);
  HIPCHECK(hipMemcpyAsync(&tot, X.d_tot.p, sizeof tot, hipMemcpyDeviceToHost, s));
  HIPCHECK(hipStreamSynchronize(s));
  HIPCHECK(hipGetLastError());
  const uint64_t off = tot;
  clk.mark("size+layout");
  DevBuf<uint8_t>& d_arena = X.d_arena;
  if (!d_arena.ensure(off + 64)) return false;
  HIPCHECK(hipMemsetAsync(d_arena.p + off, 0, 64, s));
  (void)hipEventRecord(b->eng->ev[2], s);
  am_launch_zstage_place(b->chunks.p, nchunks, b->arena.p, X.d_zid.p, X.d_zlen.p, X.d_zs.p, X.d_z0.p, X.d_cnt.p, d_arena.p, s);
  am_launch_inflate_write(b->arena.p, X.d_zs.p, X.d_ord.p, nlong, nz, X.d_zlen.p, d_arena.p, s);
  (void)hipEventRecord(b->eng->ev[3], s);
  HIPCHECK(hipGetLastError());
  clk.mark("queued");
  char m[48];
  std::snprintf(m, sizeof m, " streams=%u long=%u", nz, nlong);
  clk.line += m;
  clk.print("inflate_stage_dev", nchunks);
  b->inflate_ev = true;  // read after the stage's next synchronisation
  b->inflated_bytes = off;
  std::swap(b->arena.p, d_arena.p);
  std::swap(b->arena.cap, d_arena.cap);
  return true;
}

// DEFLATE on the GPU in the batch stage (am_inflate.hip), so compressed inputs need no host staging:
//  * compressed change chunks (type 2, columnar.js:742/784 -> inflateChange :813): re-wrapped as
//    magic + the ORIGINAL checksum + type 1 + uleb(length) + inflated data (k_chunks then verifies
//    the checksum against the inflated chunk);
//  * saved documents with DEFLATEd columns (inflateColumn, columnar.js:1062-1068; Backend.load):
//    rebuilt with every column inflated and its column-table entry rewritten (deflate bit cleared,
//    new length), the ORIGINAL checksum kept and marked verified -- after a GPU SHA-256 of the
//    compressed chunk has checked it (a mismatch leaves the chunk as it is: k_chunks reports the
//    checksum error). A column that does not inflate fails the document (AM_E_INFLATE).
// Pass 1 sizes every stream, the host lays the chunks out again in index order (a document's
// chunks stay adjacent) with the new headers in a small blob, pass 2 writes the inflated streams in
// place and k_copy_segs moves everything else. Streams that do not inflate leave their chunk as
// it is (a type-2 change then fails in k_chunks).
static bool inflate_stage(am_batch* b, const uint8_t* arena, uint64_t arena_len, const am_chunk_desc* chunks,
                          uint32_t nchunks, const am_doc_desc* docs, uint32_t ndocs) {
  HostClock clk;
  b->inflate_ev = false;
  if (!b->zscr) b->zscr.reset(new InflateScratch());
  InflateScratch& X = *b->zscr;
  // per chunk: 0 as it is, 1 compressed change, 2 document with DEFLATEd columns, 4 a base chunk
  // as it is -- never taken for a compressed change: decodeDocumentHeader rejects its type before
  // anything inflates it (columnar.js:1011) -- (base chunks first, in parallel over the documents;
  // then every other chunk, in parallel over the chunks)
  std::vector<uint8_t>& kind = X.kind;
  std::vector<uint32_t>& nzs = X.nzs;  // streams of chunk c
  std::vector<uint32_t>& dat = X.dat;  // kind 2: the document (index into lay)
  std::vector<int64_t>& base_of = X.base_of;  // the base chunk of document d, for its first document only
  kind.assign(nchunks, 0);
  nzs.assign(nchunks + 1, 0);
  dat.assign(nchunks, 0);
  base_of.assign(ndocs, -1);
  for (uint32_t d = 0; d < ndocs; d++)
    if (docs[d].base_chunk >= 0 && (uint64_t)docs[d].base_chunk < nchunks && kind[docs[d].base_chunk] != 3) {
      kind[docs[d].base_chunk] = 3;  // a base chunk (never a compressed change)
      base_of[d] = docs[d].base_chunk;
    }
  auto container_ok = [&](uint32_t c) {
    const am_chunk_desc& k = chunks[c];
    return !(k.flags & AM_CHUNK_RAW) && k.len > 9 && k.off + k.len <= arena_len &&
           std::memcmp(arena + k.off, "\x85\x6f\x4a\x83", 4) == 0;
  };
  std::vector<DocLayout>& lay = X.lay;
  lay.resize(ndocs);
  for (uint32_t d = 0; d < ndocs; d++)
    if (base_of[d] >= 0) lay[d] = DocLayout{};
  am_par_for(ndocs, [&](size_t d) {
    if (base_of[d] < 0) return;
    const uint32_t c = (uint32_t)base_of[d];
    const am_chunk_desc& k = chunks[c];
    if (!container_ok(c) || arena[k.off + 8] != 0 || (k.flags & 1)) return;
    DocLayout& L = lay[d];
    if (!doc_layout(arena + k.off, k.len, L) || !L.deflated) { L = DocLayout{}; return; }
    uint32_t n = 0;
    for (uint64_t id : L.id) n += (id & COL_DEFLATE) ? 1u : 0u;
    nzs[c] = n;
    dat[c] = (uint32_t)d;
  });
  // base chunks that are not staged go to kind 4; staged ones to 2 (a base chunk shared by several
  // documents is staged once, through its first document)
  bool doc_z = false;
  for (uint32_t d = 0; d < ndocs; d++)
    if (base_of[d] >= 0 && kind[base_of[d]] == 3) {
      kind[base_of[d]] = nzs[base_of[d]] ? 2 : 4;
      doc_z |= kind[base_of[d]] == 2;
    }
  if (!doc_z && zstage_dev_on(nchunks)) return inflate_stage_dev(b, arena_len, nchunks, ndocs, clk);
  am_par_for(nchunks, [&](size_t c) {
    if (kind[c] || !container_ok((uint32_t)c)) return;
    const uint8_t* p = arena + chunks[c].off;
    if (p[8] != 2) return;
    Container ct;
    if (!read_container(p, chunks[c].len, ct)) return;
    kind[c] = 1;
    nzs[c] = 1;
  });
  // streams: exclusive scan of the counts, then each chunk fills its own
  std::vector<uint32_t>& z0 = X.z0;
  z0.resize(nchunks + 1);
  z0[0] = 0;
  for (uint32_t c = 0; c < nchunks; c++) z0[c + 1] = z0[c] + nzs[c];
  const uint32_t nz = z0[nchunks];
  b->inflated = nz;
  b->inflate_ms = 0.f;
  if (!nz) return true;
  std::vector<am_zstream>& zs = X.zs;
  zs.resize(nz);
  am_par_for(nchunks, [&](size_t c) {
    if (!nzs[c]) return;
    const am_chunk_desc& k = chunks[c];
    am_zstream z{};
    z.dst = ~0ull;  // set when placed
    if (kind[c] == 1) {
      Container ct;
      read_container(arena + k.off, k.len, ct);
      z.src = k.off + ct.data_off;
      z.len = (uint32_t)ct.data_len;
      zs[z0[c]] = z;
      return;
    }
    const DocLayout& L = lay[dat[c]];
    uint32_t q = z0[c];
    for (size_t i = 0; i < L.id.size(); i++)
      if (L.id[i] & COL_DEFLATE) {
        z.src = k.off + L.off[i];
        z.len = (uint32_t)L.len[i];
        zs[q++] = z;
      }
  });
  clk.mark("scan");
  hipStream_t s = b->eng->stream;
  DevBuf<am_zstream>& d_zs = X.d_zs;
  DevBuf<uint32_t>&d_zlen = X.d_zlen, &d_ord = X.d_ord;
  DevBuf<am_chunk_desc>& d_sha = X.d_sha;
  DevBuf<uint8_t>&d_hash = X.d_hash, &d_arena = X.d_arena, &d_blob = X.d_blob;
  DevBuf<am_seg>& d_seg = X.d_seg;
  if (!d_zs.ensure(nz) || !d_zlen.ensure(nz) || !d_ord.ensure(nz)) return false;
  std::vector<uint32_t>& ord = X.ord;
  ord.resize(nz);
  const uint32_t nlong = am_inflate_order(zs.data(), nz, ord.data());
  HIPCHECK(hipMemcpyAsync(d_zs.p, zs.data(), sizeof(am_zstream) * nz, hipMemcpyHostToDevice, s));
  HIPCHECK(hipMemcpyAsync(d_ord.p, ord.data(), 4ull * nz, hipMemcpyHostToDevice, s));
  (void)hipEventRecord(b->eng->ev[0], s);
  am_launch_inflate_size(b->arena.p, d_zs.p, d_ord.p, nlong, nz, d_zlen.p, s);
  HIPCHECK(hipGetLastError());  // sizes below come from this launch
  (void)hipEventRecord(b->eng->ev[1], s);
  // the compressed documents' checksums (SHA-256 of everything after the checksum, container end)
  std::vector<am_chunk_desc>& sha = X.sha;
  std::vector<uint32_t>& sha_of = X.sha_of;
  sha.clear();
  sha_of.assign(ndocs, 0);
  for (uint32_t d = 0; d < ndocs; d++)
    if (base_of[d] >= 0 && kind[base_of[d]] == 2 && dat[base_of[d]] == d) {
      sha_of[d] = (uint32_t)sha.size();
      sha.push_back({chunks[base_of[d]].off + 8, (uint32_t)(lay[d].end - 8), 0});
    }
  if (!sha.empty()) {
    if (!d_sha.ensure(sha.size()) || !d_hash.ensure(32 * sha.size())) return false;
    HIPCHECK(hipMemcpyAsync(d_sha.p, sha.data(), sizeof(am_chunk_desc) * sha.size(), hipMemcpyHostToDevice, s));
    am_launch_sha256(b->arena.p, d_sha.p, (uint32_t)sha.size(), d_hash.p, s);
  }
  std::vector<uint32_t>& zlen = X.zlen;
  std::vector<uint8_t>& hash = X.hash;
  zlen.resize(nz);
  hash.resize(32 * sha.size());
  HIPCHECK(hipMemcpyAsync(zlen.data(), d_zlen.p, 4ull * nz, hipMemcpyDeviceToHost, s));
  if (!sha.empty()) HIPCHECK(hipMemcpyAsync(hash.data(), d_hash.p, hash.size(), hipMemcpyDeviceToHost, s));
  HIPCHECK(hipStreamSynchronize(s));
  clk.mark("h2d+size+sha");
  // new layout in chunk-index order. Per chunk its new length and its copy segments (a staged
  // document's new header goes to its own blob, concatenated below); then a scan places the chunks
  std::vector<am_chunk_desc>& nc = X.nc;
  nc.assign(chunks, chunks + nchunks);
  std::vector<uint32_t>& nseg = X.nseg;
  nseg.assign(nchunks + 1, 0);
  std::vector<std::vector<uint8_t>>& dhdr = X.dhdr;  // staged documents' headers
  std::vector<std::vector<uint64_t>>& dcl = X.dcl;  // ... and their column lengths
  dhdr.resize(ndocs);
  dcl.resize(ndocs);
  am_par_for(nchunks, [&](size_t c) {
    const am_chunk_desc& k = chunks[c];
    const uint8_t* p = arena + k.off;
    if (kind[c] == 1 && zlen[z0[c]] != 0xFFFFFFFFu) {
      // the header travels with the stream (written by the inflate kernel): checksum, type 1, uleb
      am_zstream& z = zs[z0[c]];
      std::memcpy(z.hdr, p + 4, 4);
      z.hdr[4] = 1;
      uint32_t q = 5;
      for (uint64_t v = zlen[z0[c]];;) {
        const uint8_t byte = v & 0x7f;
        v >>= 7;
        z.hdr[q++] = byte | (v ? 0x80 : 0);
        if (!v) break;
      }
      z.hlen = (uint8_t)q;
      nc[c].len = (uint32_t)(4 + q + zlen[z0[c]]);
      return;
    }
    if (kind[c] == 2) {
      const uint32_t d = dat[c];
      const DocLayout& L = lay[d];
      bool inflated = true;
      for (uint32_t q = z0[c]; q < z0[c + 1]; q++) inflated &= zlen[q] != 0xFFFFFFFFu;
      if (std::memcmp(hash.data() + 32 * sha_of[d], p + 4, 4) != 0) {
        kind[c] = 0;  // checksum mismatch: the chunk stays as it is and k_chunks reports it
      } else if (!inflated) {
        kind[c] = 0;
        nc[c].flags |= AM_CHUNK_BADZ;  // the document fails with AM_E_INFLATE (k_chunks)
      } else {
        // body: actors + heads, the two column tables with the new lengths, columns, the rest
        std::vector<uint64_t>& clen = dcl[d];
        clen.resize(L.id.size());
        std::vector<uint8_t> tab;
        uint64_t cols = 0;
        uint32_t q = z0[c], ncopy = 0;
        for (size_t i = 0; i < L.id.size(); i++) {
          clen[i] = (L.id[i] & COL_DEFLATE) ? zlen[q++] : L.len[i];
          cols += clen[i];
          ncopy += (!(L.id[i] & COL_DEFLATE) && L.len[i]) ? 1u : 0u;
        }
        put_u(tab, L.nc);
        for (size_t i = 0; i < L.id.size(); i++) {
          if (i == L.nc) put_u(tab, L.id.size() - L.nc);
          put_u(tab, L.id[i] & ~(uint64_t)COL_DEFLATE);
          put_u(tab, clen[i]);
        }
        if (L.id.size() == L.nc) put_u(tab, 0);
        const uint64_t pre = L.pre_end - L.data_off;
        const uint64_t body = pre + tab.size() + cols + (L.end - L.post);
        std::vector<uint8_t>& h = dhdr[d];
        h.assign(p, p + 8);  // magic + the original checksum
        h.push_back(0);
        put_u(h, body);
        h.insert(h.end(), p + L.data_off, p + L.pre_end);
        h.insert(h.end(), tab.begin(), tab.end());
        nc[c].len = (uint32_t)(h.size() + cols + (L.end - L.post));
        nc[c].flags |= 1;  // the checksum was verified above, on the compressed chunk
        nseg[c] = 1 + ncopy + (L.end > L.post ? 1u : 0u);
        return;
      }
    }
    nseg[c] = 1;  // the chunk as it is
  });
  uint64_t off = 0;
  std::vector<uint32_t>& s0 = X.s0;
  std::vector<uint64_t>& hoff = X.hoff;
  s0.assign(nchunks + 1, 0);
  hoff.assign(ndocs, 0);
  uint64_t blob_len = 0;
  for (uint32_t c = 0; c < nchunks; c++) {
    nc[c].off = off;
    off += nc[c].len;
    s0[c + 1] = s0[c] + nseg[c];
    if (kind[c] == 2) {
      hoff[dat[c]] = blob_len;
      blob_len += dhdr[dat[c]].size();
    }
  }
  std::vector<uint8_t>& blob = X.blob;
  std::vector<am_seg>& seg = X.seg;
  blob.resize(blob_len);
  seg.resize(s0[nchunks]);
  am_par_for(nchunks, [&](size_t c) {
    const am_chunk_desc& k = chunks[c];
    if (kind[c] == 1 && zlen[z0[c]] != 0xFFFFFFFFu) {
      zs[z0[c]].dst = nc[c].off + 4 + zs[z0[c]].hlen;
      return;
    }
    uint32_t g = s0[c];
    if (kind[c] != 2) {
      seg[g] = {k.off, nc[c].off, k.len, 0};
      return;
    }
    const uint32_t d = dat[c];
    const DocLayout& L = lay[d];
    const std::vector<uint8_t>& h = dhdr[d];
    std::memcpy(blob.data() + hoff[d], h.data(), h.size());
    seg[g++] = {hoff[d], nc[c].off, (uint32_t)h.size(), 1};
    uint64_t at = nc[c].off + h.size();
    uint32_t q = z0[c];
    for (size_t i = 0; i < L.id.size(); i++) {
      if (L.id[i] & COL_DEFLATE) zs[q++].dst = at;
      else if (L.len[i]) seg[g++] = {k.off + L.off[i], at, (uint32_t)L.len[i], 0};
      at += dcl[d][i];
    }
    if (L.end > L.post) seg[g++] = {k.off + L.post, at, (uint32_t)(L.end - L.post), 0};
  });
  clk.mark("layout");
  if (!d_arena.ensure(off + 64) || !d_seg.ensure(seg.size()) || !d_blob.ensure(blob.size() + 1)) return false;
  HIPCHECK(hipMemcpyAsync(d_zs.p, zs.data(), sizeof(am_zstream) * nz, hipMemcpyHostToDevice, s));
  if (!seg.empty()) HIPCHECK(hipMemcpyAsync(d_seg.p, seg.data(), sizeof(am_seg) * seg.size(), hipMemcpyHostToDevice, s));
  if (!blob.empty()) HIPCHECK(hipMemcpyAsync(d_blob.p, blob.data(), blob.size(), hipMemcpyHostToDevice, s));
  HIPCHECK(hipMemsetAsync(d_arena.p + off, 0, 64, s));
  (void)hipEventRecord(b->eng->ev[2], s);
  am_launch_copy_segs(b->arena.p, d_blob.p, d_seg.p, (uint32_t)seg.size(), d_arena.p, s);
  am_launch_inflate_write(b->arena.p, d_zs.p, d_ord.p, nlong, nz, d_zlen.p, d_arena.p, s);
  (void)hipEventRecord(b->eng->ev[3], s);
  HIPCHECK(hipMemcpyAsync(b->chunks.p, nc.data(), sizeof(am_chunk_desc) * nchunks, hipMemcpyHostToDevice, s));
  HIPCHECK(hipStreamSynchronize(s));
  HIPCHECK(hipGetLastError());
  clk.mark("copy+write");
  char segs[48];
  std::snprintf(segs, sizeof segs, " streams=%u long=%u segs=%zu", nz, nlong, seg.size());
  clk.line += segs;
  clk.print("inflate_stage", nchunks);
  float ms1 = 0.f, ms2 = 0.f;
  (void)hipEventElapsedTime(&ms1, b->eng->ev[0], b->eng->ev[1]);
  (void)hipEventElapsedTime(&ms2, b->eng->ev[2], b->eng->ev[3]);
  b->inflate_ms = ms1 + ms2;
  b->inflated_bytes = off;
  std::swap(b->arena.p, d_arena.p);
  std::swap(b->arena.cap, d_arena.cap);
  return true;
}

// compact workspace plans for k_doc_fast's documents (AM_WS_COMPACT=0: every document gets k_doc's)
static bool ws_compact_on() {
  static const bool v = [] { const char* e = std::getenv("AM_WS_COMPACT"); return !(e && e[0] == '0'); }();
  return v;
}
// LDS budget of one k_doc workgroup (AM_LDS_BUDGET; AM_LDS_BUDGET_KB overrides it, for A/B runs).
// A batch that wants patches keeps 40 KB (measured on the C5 receive's batched apply, 200,000
// handles with their objectMeta: GPU 435 ms at 40 KB against 1,843 ms at 64 KB; a stateless C5
// batch prefers 64 KB, 177 against 207 ms per 65,536 -- the per-handle path is the one callers hit)
static uint32_t lds_budget(bool any_diff) {
  static const uint32_t v = [] {
    const char* e = std::getenv("AM_LDS_BUDGET_KB");
    const unsigned long k = e ? std::strtoul(e, nullptr, 10) : 0ul;
    return k >= 8 && k <= 160 ? (uint32_t)(k * 1024) : 0u;
  }();
  return v ? v : any_diff ? 40u * 1024 : (uint32_t)AM_LDS_BUDGET;
}

static bool stage_impl(am_batch* b, const uint8_t* arena, uint64_t arena_len, const am_chunk_desc* chunks, uint32_t nchunks,
                       const am_doc_desc* docs, uint32_t ndocs, const am_known_hash* known, uint32_t nknown) {
  am_engine* e = b->eng;
  if (!set_device(e)) return false;
  hipStream_t s = e->stream;
  // 64 bytes of slack: k_doc_fast stages whole 16-byte words of a document's span
  if (!b->arena.ensure(arena_len + 64) || !b->chunks.ensure(nchunks) || !b->docs.ensure(ndocs) || !b->known.ensure(nknown) ||
      !b->info.ensure(nchunks) || !b->hdr.ensure(nchunks) || !b->bounds.ensure(ndocs) || !b->ws_bytes.ensure(ndocs) || !b->ws_off.ensure(ndocs) ||
      !b->scan_tmp.ensure(am_scan_tmp_elems(ndocs)) || !b->ws_total.ensure(1) || !b->max_hot.ensure(4) ||
      !b->fast_done.ensure(ndocs) || !b->rest.ensure(ndocs + 1) || !b->results.ensure(ndocs) ||
      !b->chg_state.ensure(nchunks))
    return false;
  HostClock clk;
  if (arena_len) HIPCHECK(hipMemcpyAsync(b->arena.p, arena, arena_len, hipMemcpyHostToDevice, s));
  if (nchunks) HIPCHECK(hipMemcpyAsync(b->chunks.p, chunks, sizeof(am_chunk_desc) * nchunks, hipMemcpyHostToDevice, s));
  if (ndocs) HIPCHECK(hipMemcpyAsync(b->docs.p, docs, sizeof(am_doc_desc) * ndocs, hipMemcpyHostToDevice, s));
  if (nknown) HIPCHECK(hipMemcpyAsync(b->known.p, known, sizeof(am_known_hash) * nknown, hipMemcpyHostToDevice, s));
  b->nchunks = nchunks;
  b->ndocs = ndocs;
  b->any_diff = false;
  for (uint32_t d = 0; d < ndocs && !b->any_diff; d++) b->any_diff = (docs[d].flags & (AM_DOC_WANT_DIFF | AM_DOC_WANT_PATCH)) != 0;
  clk.mark("h2d-queued");
  if (!inflate_stage(b, arena, arena_len, chunks, nchunks, docs, ndocs)) return false;
  clk.mark("inflate-stage");
  // k_doc_fast (am_doc_fast.h) for the documents in its envelope; AM_FAST=0 turns it off
  const char* fe = std::getenv("AM_FAST");
  const bool fast_on = !(fe && fe[0] == '0');
  b->compact = fast_on && ws_compact_on();
  // sizing pass: chunk counts -> per-document workspace bounds -> total
  BatchDev d = b->dev();
  am_launch_chunks(d, s);
  am_launch_bounds(d, s);
  uint64_t total = 0, max_hot = 0, max_fast = 0, saved = 0;
  if (ndocs) HIPCHECK(hipMemcpyAsync(&total, b->ws_total.p, sizeof total, hipMemcpyDeviceToHost, s));
  if (ndocs) HIPCHECK(hipMemcpyAsync(&max_hot, b->max_hot.p, sizeof max_hot, hipMemcpyDeviceToHost, s));
  if (ndocs) HIPCHECK(hipMemcpyAsync(&max_fast, b->max_hot.p + 1, sizeof max_fast, hipMemcpyDeviceToHost, s));
  if (ndocs) HIPCHECK(hipMemcpyAsync(&saved, b->max_hot.p + 2, sizeof saved, hipMemcpyDeviceToHost, s));
  HIPCHECK(hipStreamSynchronize(s));
  HIPCHECK(hipGetLastError());
  if (b->inflate_ev) {
    float ms1 = 0.f, ms2 = 0.f;
    (void)hipEventElapsedTime(&ms1, e->ev[0], e->ev[1]);
    (void)hipEventElapsedTime(&ms2, e->ev[2], e->ev[3]);
    b->inflate_ms = ms1 + ms2;
    b->inflate_ev = false;
  }
  clk.mark("sizing");
  clk.print("stage", ndocs);
  // a batch reserves the whole plan of every compact document as overflow, so none of them can
  // run out of room if the fast kernel gives up on all of them (the pipe reserves a fraction)
  b->ws_plan = total;
  total += saved;
  b->ws_need = total;
  // dynamic LDS of the document workgroups: the largest hot working set, capped by the budget
  uint64_t lds = (max_hot + 15) & ~(uint64_t)15;
  if (lds > lds_budget(b->any_diff)) lds = lds_budget(b->any_diff);
  b->lds_bytes = (uint32_t)lds;
  b->max_hot_v = max_hot;
  b->fast_lds = fast_on ? (uint32_t)((max_fast + 15) & ~(uint64_t)15) : 0u;
  b->fast_only = false;
  if (!b->ws.ensure(total + 16)) return false;
  b->fresh = true;
  return true;
}

extern "C" int am_batch_stage(am_batch* b, const uint8_t* arena, uint64_t arena_len, const am_chunk_desc* chunks,
                              uint32_t nchunks, const am_doc_desc* docs, uint32_t ndocs, const am_known_hash* known,
                              uint32_t nknown, am_error* err) {
  if (!stage_impl(b, arena, arena_len, chunks, nchunks, docs, ndocs, known, nknown)) {
    to_c(Err{AM_U_CAPACITY, false, "automerge_amd: device allocation or copy failed"}, err);
    return 1;
  }
  if (err) err->code = 0;
  return 0;
}

extern "C" int am_batch_run(am_batch* b) {
  am_engine* e = b->eng;
  if (!set_device(e)) return 1;
  hipStream_t s = e->stream;
  BatchDev d = b->dev();
  // AM_DEBUG_SYNC=1 (diagnosis): synchronise after every stage and name the one that failed;
  // AM_DEBUG_WS_PAD=<bytes>: the kernels see the workspace that many bytes into a larger allocation
  static const bool dbg = std::getenv("AM_DEBUG_SYNC") != nullptr;
  static const uint64_t pad = [] { const char* v = std::getenv("AM_DEBUG_WS_PAD"); return v ? std::strtoull(v, nullptr, 10) & ~4095ull : 0ull; }();
  if (pad) {
    if (!b->ws.ensure(b->ws_need + pad + 16)) return 1;
    d.ws = b->ws.p + pad;
    d.ws_cap = b->ws.cap - pad;
  }
  // AM_DEBUG_WS_CANARY=<bytes>: the workspace is filled with 0xA5 and followed by that many canary
  // bytes; am_batch_ws_canary reports the first one a kernel wrote
  // (read per run: a test process turns it on for some batches only)
  const uint64_t canary = [] { const char* v = std::getenv("AM_DEBUG_WS_CANARY"); return v ? std::strtoull(v, nullptr, 10) : 0ull; }();
  if (canary) {
    if (!b->ws.ensure(b->ws_need + canary + 16)) return 1;
    (void)hipMemsetAsync(b->ws.p, 0xA5, b->ws_need + canary, s);
    d.ws = b->ws.p;  // (ensure may have moved it)
    d.ws_cap = b->ws_need;
  }
  auto check = [&](const char* what) {
    if (!dbg) return true;
    const hipError_t r = hipStreamSynchronize(s);
    if (r != hipSuccess) std::fprintf(stderr, "[am_debug] %s: %s (ndocs %u, ws %llu)\n", what, hipGetErrorString(r), b->ndocs,
                                      (unsigned long long)b->ws_need);
    return r == hipSuccess;
  };
  // the first run after a stage reuses the sizing pass's k_chunks / k_bounds results (nothing has
  // changed them; a run's k_rest re-plans bounds, so later runs redo both)
  const bool fresh = b->fresh;
  b->fresh = false;
  (void)hipEventRecord(e->ev[0], s);
  if (!fresh) am_launch_chunks(d, s);
  if (!check("k_chunks")) return 1;
  (void)hipEventRecord(e->ev[1], s);
  if (!fresh) am_launch_bounds(d, s);
  if (!check("k_bounds")) return 1;
  (void)hipEventRecord(e->ev[2], s);
  am_launch_doc(d, s);
  if (!check("k_doc_fast / k_doc")) return 1;
  (void)hipEventRecord(e->ev[3], s);
  am_launch_out_hash(d, s);
  if (!check("k_out_hash_ws")) return 1;
  (void)hipEventRecord(e->ev[4], s);
  b->timed = true;
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

// Diagnostics (AM_DEBUG_WS_CANARY): offset past the workspace end of the first canary byte a kernel
// changed, or -1
extern "C" int64_t am_batch_ws_canary(am_batch* b, uint64_t n) {
  std::vector<uint8_t> h(n);
  if (!set_device(b->eng) || hipMemcpy(h.data(), b->ws.p + b->ws_need, n, hipMemcpyDeviceToHost) != hipSuccess) return -2;
  for (uint64_t i = 0; i < n; i++)
    if (h[i] != 0xA5) return (int64_t)i;
  return -1;
}

extern "C" int am_batch_sync(am_batch* b, am_error* err) {
  if (!set_device(b->eng)) return 1;
  hipError_t r = hipStreamSynchronize(b->eng->stream);
  if (r != hipSuccess) {
    to_c(Err{AM_U_CAPACITY, false, std::string("automerge_amd: HIP error: ") + hipGetErrorString(r)}, err);
    return 1;
  }
  if (err) err->code = 0;
  return 0;
}

extern "C" int am_batch_results(am_batch* b, am_doc_result* out) {
  if (!set_device(b->eng) || !b->ndocs) return b->ndocs ? 1 : 0;
  return hipMemcpy(out, b->results.p, sizeof(am_doc_result) * b->ndocs, hipMemcpyDeviceToHost) == hipSuccess ? 0 : 1;
}

extern "C" int am_batch_chunk_results(am_batch* b, uint8_t* hashes32, int32_t* chg_state, uint32_t* status) {
  if (!set_device(b->eng)) return 1;
  if (!b->nchunks) return 0;
  std::vector<ChunkInfo> info(b->nchunks);
  if (hipMemcpy(info.data(), b->info.p, sizeof(ChunkInfo) * b->nchunks, hipMemcpyDeviceToHost) != hipSuccess) return 1;
  if (chg_state && hipMemcpy(chg_state, b->chg_state.p, sizeof(int32_t) * b->nchunks, hipMemcpyDeviceToHost) != hipSuccess)
    return 1;
  for (uint32_t i = 0; i < b->nchunks; i++) {
    if (hashes32) std::memcpy(hashes32 + 32 * i, info[i].hash, 32);
    if (status) status[i] = info[i].status;
  }
  return 0;
}

extern "C" int am_batch_doc_output(am_batch* b, uint32_t doc, uint8_t* dst, uint64_t cap, uint64_t* len) {
  if (!set_device(b->eng) || doc >= b->ndocs) return 1;
  am_doc_result r;
  if (hipMemcpy(&r, b->results.p + doc, sizeof r, hipMemcpyDeviceToHost) != hipSuccess) return 1;
  *len = r.out_len;
  if (!r.out_len) return 0;
  if (cap < r.out_len) return 2;
  return hipMemcpy(dst, b->ws.p + r.out_off, r.out_len, hipMemcpyDeviceToHost) == hipSuccess ? 0 : 1;
}

extern "C" int am_batch_doc_heads(am_batch* b, uint32_t doc, uint8_t* dst32, uint32_t cap, uint32_t* n) {
  if (!set_device(b->eng) || doc >= b->ndocs) return 1;
  am_doc_result r;
  DocBounds bd;
  if (hipMemcpy(&r, b->results.p + doc, sizeof r, hipMemcpyDeviceToHost) != hipSuccess) return 1;
  if (hipMemcpy(&bd, b->bounds.p + doc, sizeof bd, hipMemcpyDeviceToHost) != hipSuccess) return 1;
  *n = r.nheads;
  if (!r.nheads || r.status) return 0;
  WsLayout L = ws_layout(bd);
  uint32_t k = r.nheads < cap ? r.nheads : cap;
  return hipMemcpy(dst32, b->ws.p + r.ws_off + L.heads, 32ull * k, hipMemcpyDeviceToHost) == hipSuccess ? 0 : 1;
}

// Diagnostics: the first 48 bytes (PatchHdr2) of document doc's patch-log slot, as they are
extern "C" int am_batch_doc_patch_raw(am_batch* b, uint32_t doc, uint8_t* dst48) {
  if (!set_device(b->eng) || doc >= b->ndocs) return 1;
  am_doc_result r;
  DocBounds bd;
  if (hipMemcpy(&r, b->results.p + doc, sizeof r, hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(&bd, b->bounds.p + doc, sizeof bd, hipMemcpyDeviceToHost) != hipSuccess || !bd.P)
    return 1;
  const WsLayout L = ws_layout(bd);
  return hipMemcpy(dst48, b->ws.p + r.ws_off + L.pwire, 48, hipMemcpyDeviceToHost) == hipSuccess ? 0 : 1;
}

extern "C" int am_batch_doc_patch(am_batch* b, uint32_t doc, uint8_t* dst, uint64_t cap, uint64_t* len) {
  if (!set_device(b->eng) || doc >= b->ndocs) return 1;
  am_doc_result r;
  DocBounds bd;
  if (hipMemcpy(&r, b->results.p + doc, sizeof r, hipMemcpyDeviceToHost) != hipSuccess) return 1;
  if (hipMemcpy(&bd, b->bounds.p + doc, sizeof bd, hipMemcpyDeviceToHost) != hipSuccess) return 1;
  if (r.status) return 3;  // the document failed: there is no patch
  if (!bd.P) return 4;     // not staged with AM_DOC_WANT_PATCH / AM_DOC_WANT_DIFF
  const WsLayout L = ws_layout(bd);
  // the wire form (am_patch.h): PatchHdr2 + stream, written by the kernel that merged the document
  const uint8_t* base = b->ws.p + r.ws_off + L.pwire;
  PatchHdr2 h;
  if (hipMemcpy(&h, base, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return 1;
  // AM_DOC_META: the objectMeta blob follows the stream (PatchHdr2.meta_bytes)
  if (h.magic != AM_PATCH_MAGIC || sizeof h + h.nbytes + h.meta_bytes > L.pwire_cap) return 1;
  const uint64_t total = sizeof h + h.nbytes + h.meta_bytes;
  *len = total;
  if (cap == 0) return 0;
  if (cap < total) return 2;
  return hipMemcpy(dst, base, total, hipMemcpyDeviceToHost) == hipSuccess ? 0 : 1;
}

extern "C" int am_batch_stage_times(am_batch* b, float* ms4) {
  if (!b->timed) return 1;
  for (int i = 0; i < 4; i++) {
    if (hipEventElapsedTime(&ms4[i], b->eng->ev[i], b->eng->ev[i + 1]) != hipSuccess) return 1;
  }
  return 0;
}

extern "C" int am_batch_digest(am_batch* b, uint64_t first_doc, uint64_t* digest) {
  if (!set_device(b->eng) || !digest) return 1;
  DevBuf<uint64_t> d;
  if (!d.ensure(1)) return 1;
  hipStream_t s = b->eng->stream;
  am_launch_digest(b->dev(), first_doc, d.p, s);
  if (hipMemcpyAsync(digest, d.p, sizeof(uint64_t), hipMemcpyDeviceToHost, s) != hipSuccess) return 1;
  if (hipStreamSynchronize(s) != hipSuccess) return 1;
  *digest &= 0x7FFFFFFFFFFFFFFFull;
  return 0;
}

extern "C" int am_engine_stats(am_engine* e, uint64_t* out2) {
  out2[0] = e->stat_docs;
  out2[1] = e->stat_fast;
  e->stat_docs = e->stat_fast = 0;  // reset on read
  return 0;
}

extern "C" int am_batch_fast_flags(am_batch* b, uint8_t* flags) {
  if (!set_device(b->eng)) return 1;
  if (!b->ndocs) return 0;
  if (!b->fast_lds) { std::memset(flags, 0, b->ndocs); return 0; }
  return hipMemcpy(flags, b->fast_done.p, b->ndocs, hipMemcpyDeviceToHost) == hipSuccess ? 0 : 1;
}

extern "C" uint64_t am_batch_workspace_bytes(am_batch* b) { return b->ws_need; }
extern "C" uint64_t am_batch_workspace_plan(am_batch* b) { return b->ws_plan; }

// pako.inflateRaw over n independent buffers on the GPU (the kernels of the batch stage). outs[i]
// (malloc'd, am_free) / out_lens[i]; ok[i] = 0 when buffer i is not a valid raw DEFLATE stream.
extern "C" int am_inflate_raw(am_engine* eng, const uint8_t* const* bufs, const size_t* lens, size_t n, uint8_t** outs,
                              size_t* out_lens, uint8_t* ok, am_error* err) {
  auto fail = [&](const char* m) { to_c(Err{AM_U_CAPACITY, false, m}, err); return 1; };
  if (!set_device(eng)) return fail("automerge_amd: no device");
  hipStream_t s = eng->stream;
  HostClock clk;
  std::vector<uint8_t> arena;
  std::vector<am_zstream> zs(n);
  for (size_t i = 0; i < n; i++) {
    if (lens[i] > 0xFFFFFF00u) return fail("automerge_amd: buffer too large");
    zs[i] = {arena.size(), 0, (uint32_t)lens[i], 0};
    arena.insert(arena.end(), bufs[i], bufs[i] + lens[i]);
  }
  if (!n) return 0;
  DevBuf<uint8_t> d_arena, d_out;
  DevBuf<am_zstream> d_zs;
  DevBuf<uint32_t> d_zlen, d_ord;
  if (!d_arena.ensure(arena.size() + 64) || !d_zs.ensure(n) || !d_zlen.ensure(n) || !d_ord.ensure(n))
    return fail("automerge_amd: device allocation failed");
  std::vector<uint32_t> zlen(n), ord(n);
  const uint32_t nlong = am_inflate_order(zs.data(), (uint32_t)n, ord.data());
  bool okc = hipMemcpyAsync(d_arena.p, arena.data(), arena.size(), hipMemcpyHostToDevice, s) == hipSuccess &&
             hipMemcpyAsync(d_zs.p, zs.data(), sizeof(am_zstream) * n, hipMemcpyHostToDevice, s) == hipSuccess &&
             hipMemcpyAsync(d_ord.p, ord.data(), 4 * n, hipMemcpyHostToDevice, s) == hipSuccess;
  if (okc) {
    am_launch_inflate_size(d_arena.p, d_zs.p, d_ord.p, nlong, (uint32_t)n, d_zlen.p, s);
    okc = hipGetLastError() == hipSuccess && hipMemcpyAsync(zlen.data(), d_zlen.p, 4 * n, hipMemcpyDeviceToHost, s) == hipSuccess &&
          hipStreamSynchronize(s) == hipSuccess;
  }
  if (!okc) return fail("automerge_amd: inflate pass 1 failed");
  clk.mark("pack+h2d+size");
  uint64_t off = 0;
  for (size_t i = 0; i < n; i++) {
    zs[i].dst = off;
    off += zlen[i] == 0xFFFFFFFFu ? 0 : zlen[i];
  }
  if (!d_out.ensure(off + 64)) return fail("automerge_amd: device allocation failed");
  std::vector<uint8_t> out(off);
  okc = hipMemcpyAsync(d_zs.p, zs.data(), sizeof(am_zstream) * n, hipMemcpyHostToDevice, s) == hipSuccess;
  if (okc) {
    am_launch_inflate_write(d_arena.p, d_zs.p, d_ord.p, nlong, (uint32_t)n, d_zlen.p, d_out.p, s);
    okc = (off == 0 || hipMemcpyAsync(out.data(), d_out.p, off, hipMemcpyDeviceToHost, s) == hipSuccess) &&
          hipStreamSynchronize(s) == hipSuccess && hipGetLastError() == hipSuccess;
  }
  if (!okc) return fail("automerge_amd: inflate pass 2 failed");
  clk.mark("write+d2h");
  for (size_t i = 0; i < n; i++) {
    ok[i] = zlen[i] != 0xFFFFFFFFu;
    const size_t m = ok[i] ? zlen[i] : 0;
    outs[i] = (uint8_t*)std::malloc(m ? m : 1);
    if (m) std::memcpy(outs[i], out.data() + zs[i].dst, m);
    out_lens[i] = m;
  }
  clk.mark("outs");
  clk.print("inflate_raw", n);
  if (err) err->code = 0;
  return 0;
}

extern "C" int am_batch_inflate_info(am_batch* b, uint64_t* nchunks, uint64_t* arena_bytes, float* ms) {
  if (nchunks) *nchunks = b->inflated;
  if (arena_bytes) *arena_bytes = b->inflated_bytes;
  if (ms) *ms = b->inflate_ms;
  return 0;
}
// launch shape of the document kernels of the staged batch: [0] k_doc dynamic LDS bytes, [1] the
// k_doc_fast LDS slice per document (0: no document in its envelope), [2] largest k_doc hot set
extern "C" int am_batch_kernel_info(am_batch* b, uint64_t* out3) {
  out3[0] = b->lds_bytes;
  out3[1] = b->fast_lds;
  out3[2] = b->max_hot_v;
  return 0;
}

// workspace plan of document `doc` of the staged batch (diagnostics): [0] R, [1] E, [2] P,
// [3] hot working set, [4] workspace bytes, [5] its offset, [6] span_lo, [7] span_hi,
// [8] 1 when the document runs from LDS (k_doc lds_mode), [9] input bytes B
extern "C" int am_batch_doc_plan(am_batch* b, uint32_t doc, uint64_t* out10) {
  if (!set_device(b->eng) || doc >= b->ndocs) return 1;
  DocBounds db;
  uint64_t off = 0;
  if (hipMemcpy(&db, b->bounds.p + doc, sizeof db, hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(&off, b->ws_off.p + doc, sizeof off, hipMemcpyDeviceToHost) != hipSuccess)
    return 1;
  const WsLayout L = ws_layout(db);
  out10[0] = db.R; out10[1] = db.E; out10[2] = db.P; out10[3] = L.hot_total; out10[4] = L.total; out10[5] = off;
  out10[6] = db.span_lo; out10[7] = db.span_hi; out10[8] = (L.hot_total <= b->lds_bytes && !(db.span_hi == db.span_lo && db.B > 0)) ? 1 : 0;
  out10[9] = db.B;
  return 0;
}

// Diagnostics: the DocBounds of a staged document (96 bytes) and its WsLayout (all u64 fields, in
// declaration order); returns the number of u64 written to lay_out (cap permitting)
extern "C" int am_batch_doc_layout(am_batch* b, uint32_t doc, void* bounds_out, uint64_t* lay_out, uint32_t cap) {
  if (!set_device(b->eng) || doc >= b->ndocs) return -1;
  DocBounds db;
  if (hipMemcpy(&db, b->bounds.p + doc, sizeof db, hipMemcpyDeviceToHost) != hipSuccess) return -1;
  std::memcpy(bounds_out, &db, sizeof db);
  static_assert(sizeof(WsLayout) % 8 == 0, "WsLayout of u64");
  const WsLayout L = ws_layout(db);
  const uint32_t n = (uint32_t)(sizeof L / 8);
  std::memcpy(lay_out, &L, 8ull * (n < cap ? n : cap));
  return (int)n;
}

// k_doc_fast LDS slice of every document of the staged batch (diagnostics): out[doc] =
// fast_layout(...).total, 0 when the document is outside the fast kernel's envelope
extern "C" int am_batch_fast_slices(am_batch* b, uint32_t* out) {
  if (!set_device(b->eng)) return 1;
  std::vector<DocBounds> db(b->ndocs);
  std::vector<am_doc_desc> dd(b->ndocs);
  if (b->ndocs && (hipMemcpy(db.data(), b->bounds.p, sizeof(DocBounds) * b->ndocs, hipMemcpyDeviceToHost) != hipSuccess ||
                   hipMemcpy(dd.data(), b->docs.p, sizeof(am_doc_desc) * b->ndocs, hipMemcpyDeviceToHost) != hipSuccess))
    return 1;
  am_fast_slices_host(db.data(), dd.data(), b->ndocs, out);
  return 0;
}

// =============================================================================================
// pipelined batches (am_pipe_*): H2D of batch k+1 and D2H of batch k-1 overlap the kernels of k
// =============================================================================================
extern "C" void* am_host_alloc(size_t n) {
  void* p = nullptr;
  if (hipHostMalloc(&p, n ? n : 1, pinned_flags()) != hipSuccess) return nullptr;
  return p;
}
extern "C" void am_host_free(void* p) {
  if (p) (void)hipHostFree(p);
}

namespace {
struct PipeSlot {
  am_batch b;                                  // device inputs, workspace, results
  DevBuf<uint64_t> olen, ooff, plen, poff, tmp, totals;
  DevBuf<uint8_t> dout, dpatch;
  DevBuf<am_doc_summary> summ;
  DevBuf<uint32_t> clen;                       // packed descriptors (am_pipe_submit_packed) and their scans
  DevBuf<am_doc_span> spans;
  DevBuf<uint64_t> c64, coff, ctmp;
  uint64_t* h_totals = nullptr;                // pinned: the two arena sizes of the last run
  hipEvent_t ev_c0 = nullptr, ev_d0 = nullptr, ev_d1 = nullptr, ev_comp = nullptr, ev_in = nullptr, ev_out = nullptr;
  bool busy = false, finalized = false;
  uint64_t ticket = 0;
  am_doc_summary* h_summ = nullptr;
  uint8_t *h_out = nullptr, *h_patch = nullptr;
  uint64_t h_out_cap = 0, h_patch_cap = 0;
  hsa_signal_t home{};                         // SDMA copies home of the last batch (counts down to 0)
  bool home_sdma = false;                      // the copies home went to the SDMA engines
  hsa_signal_t insig{};                        // SDMA copies of the batch's inputs (engine mode)
  bool in_sdma = false;                        // some input segment went to an SDMA engine
  bool launched = false;                       // its compute chain is queued (pipe_launch)
  bool packed = false;                         // packed descriptors (am_pipe_submit_packed)
  uint64_t arena_len = 0;
};
}  // namespace

struct am_pipe {
  am_engine* eng = nullptr;
  hipStream_t s_in = nullptr, s_c = nullptr, s_out = nullptr;
  am_pipe_caps caps{};
  std::vector<PipeSlot*> slots;
  uint64_t next = 0;                           // ticket of the next submission
  std::vector<uint64_t> totals;                // per finalized batch since the last drain: out, patch bytes
  float ms_comp = 0.f, ms_doc = 0.f;           // kernel times of the drained batches
  uint32_t nms = 0;
  std::vector<hipEvent_t> rev;                 // resident batches: 4 events each (chain start, doc kernels, end)
  uint32_t nres = 0;                           // resident batches since the last am_pipe_resident_sync
  uint32_t eng_h2d = 0, eng_home = 0;          // SDMA engine masks of the host-link copies (0: runtime's choice)
  int eng_state = 0;                           // engine mode: 0 not chosen yet, 1 on, -1 off
  PipeSlot* pending = nullptr;                 // inputs queued, compute chain not yet (pipe_submit)
  PipeSlot* launched = nullptr;                // the slot whose chain was queued last
  hsa_agent_t gpu{}, host{};
  uint64_t canary = 0;                         // AM_DEBUG_WS_CANARY bytes after every slot's workspace
};

static bool sdma_wait(hsa_signal_t sig);

static void pipe_free(am_pipe* p) {
  if (!p) return;
  set_device(p->eng);
  for (PipeSlot* sl : p->slots) {
    for (hipEvent_t e : {sl->ev_c0, sl->ev_d0, sl->ev_d1, sl->ev_comp, sl->ev_in, sl->ev_out})
      if (e) (void)hipEventDestroy(e);
    if (sl->h_totals) (void)hipHostFree(sl->h_totals);
    if (sl->home.handle) (void)hsa_signal_destroy(sl->home);
    if (sl->insig.handle) (void)hsa_signal_destroy(sl->insig);
    delete sl;
  }
  for (hipStream_t s : {p->s_in, p->s_c, p->s_out})
    if (s) (void)hipStreamDestroy(s);
  for (hipEvent_t e : p->rev) (void)hipEventDestroy(e);
  delete p;
}

extern "C" void am_pipe_destroy(am_pipe* p) {
  if (!p) return;
  set_device(p->eng);
  (void)hipDeviceSynchronize();
  // SDMA copies of the engine mode are outside the HIP streams: wait for them before freeing
  for (PipeSlot* sl : p->slots) {
    if (sl->insig.handle) (void)sdma_wait(sl->insig);
    if (sl->home.handle) (void)sdma_wait(sl->home);
  }
  pipe_free(p);
}

extern "C" am_pipe* am_pipe_create(am_engine* eng, const am_pipe_caps* caps, am_error* err) {
  auto fail = [&](am_pipe* p, const char* m) -> am_pipe* {
    to_c(Err{AM_U_CAPACITY, false, m}, err);
    pipe_free(p);
    return nullptr;
  };
  if (!eng || !caps || caps->slots < 2 || !caps->docs) return fail(nullptr, "automerge_amd: bad pipeline capacities");
  if (!set_device(eng)) return fail(nullptr, "automerge_amd: no device");
  am_pipe* p = new am_pipe();
  p->eng = eng;
  p->caps = *caps;
  if (const char* v = std::getenv("AM_DEBUG_WS_CANARY")) p->canary = std::strtoull(v, nullptr, 10);
  for (hipStream_t* s : {&p->s_in, &p->s_c, &p->s_out})
    if (hipStreamCreateWithFlags(s, hipStreamNonBlocking) != hipSuccess) return fail(p, "automerge_amd: cannot create a HIP stream");
  const am_pipe_caps& c = *caps;
  for (uint32_t k = 0; k < c.slots; k++) {
    PipeSlot* sl = new PipeSlot();
    p->slots.push_back(sl);
    am_batch& b = sl->b;
    b.eng = eng;
    const bool ok =
        b.arena.ensure(c.arena_bytes + 64) && b.chunks.ensure(c.chunks) && b.docs.ensure(c.docs) && b.known.ensure(1) &&
        b.info.ensure(c.chunks) && b.hdr.ensure(c.chunks) && b.bounds.ensure(c.docs) && b.ws_bytes.ensure(c.docs) &&
        b.ws_off.ensure(c.docs) && b.scan_tmp.ensure(am_scan_tmp_elems(c.docs)) && b.ws_total.ensure(1) &&
        b.max_hot.ensure(4) && b.fast_done.ensure(c.docs) && b.rest.ensure(c.docs + 1) && b.results.ensure(c.docs) &&
        b.chg_state.ensure(c.chunks) &&
        b.ws.ensure(c.ws_bytes + 16) && sl->olen.ensure(c.docs) && sl->ooff.ensure(c.docs) && sl->plen.ensure(c.docs) &&
        sl->poff.ensure(c.docs) && sl->tmp.ensure(am_scan_tmp_elems(c.docs)) && sl->totals.ensure(2) &&
        sl->dout.ensure(c.out_bytes + 16) && sl->dpatch.ensure(c.patch_bytes + 16) && sl->summ.ensure(c.docs);
    if (!ok) return fail(p, "automerge_amd: device allocation failed (pipeline capacities too large)");
    if (hipHostMalloc(reinterpret_cast<void**>(&sl->h_totals), 2 * sizeof(uint64_t), hipHostMallocDefault) != hipSuccess)
      return fail(p, "automerge_amd: pinned allocation failed");
    for (hipEvent_t* e : {&sl->ev_c0, &sl->ev_d0, &sl->ev_d1, &sl->ev_comp, &sl->ev_in, &sl->ev_out})
      if (hipEventCreate(e) != hipSuccess) return fail(p, "automerge_amd: cannot create a HIP event");
    if (hsa_signal_create(0, 0, nullptr, &sl->home) != HSA_STATUS_SUCCESS) sl->home.handle = 0;
    if (hsa_signal_create(0, 0, nullptr, &sl->insig) != HSA_STATUS_SUCCESS) sl->insig.handle = 0;
    b.lds_bytes = lds_budget(false);   // k_doc takes what k_doc_fast leaves, in either mode (set per batch)
    b.compact = c.fast_lds != 0 && ws_compact_on();  // what the fast kernel gives up on takes the overflow
    b.max_hot_v = ~0ull;
    b.fast_lds = c.fast_lds;
    b.fast_cap = c.fast_lds;  // a slice above the pipe's fixed one keeps k_doc's whole plan in the scan
    if (p->canary) {  // AM_DEBUG_WS_CANARY: every slot's workspace is followed by canary bytes
      if (!b.ws.ensure(c.ws_bytes + 16 + p->canary) || hipMemset(b.ws.p, 0xA5, b.ws.cap) != hipSuccess)
        return fail(p, "automerge_amd: device allocation failed (workspace canary)");
      b.ws_limit = c.ws_bytes + 16;
    }
  }
  if (err) err->code = 0;
  return p;
}

// Diagnostics (a pipeline created under AM_DEBUG_WS_CANARY=<n>): offset past the workspace end of the
// first canary byte a kernel changed in any slot, -1 when none (call after am_pipe_drain)
extern "C" int64_t am_pipe_ws_canary(am_pipe* p) {
  if (!p || !p->canary || !set_device(p->eng)) return -2;
  std::vector<uint8_t> h(p->canary);
  for (PipeSlot* sl : p->slots) {
    if (hipMemcpy(h.data(), sl->b.ws.p + sl->b.ws_limit, p->canary, hipMemcpyDeviceToHost) != hipSuccess) return -2;
    for (uint64_t i = 0; i < p->canary; i++)
      if (h[i] != 0xA5) return (int64_t)i;
  }
  return -1;
}

// the D2H copies of a batch whose kernels have been enqueued: waits for its compute chain, then
// queues the copies of its summaries and arenas on the output stream
// The agent that owns an allocation (ROCr's pointer info); false for memory ROCr does not know
// (pageable host memory)
static bool hsa_owner(const void* ptr, hsa_agent_t& agent) {
  hsa_amd_pointer_info_t info;
  std::memset(&info, 0, sizeof info);
  info.size = sizeof info;
  if (!ptr || hsa_amd_pointer_info(ptr, &info, nullptr, nullptr, nullptr) != HSA_STATUS_SUCCESS) return false;
  if (info.type == HSA_EXT_POINTER_TYPE_UNKNOWN) return false;
  agent = info.agentOwner;
  return true;
}
// device view of a caller buffer in mapped pinned host memory (am_host_alloc), or null
static void* mapped(void* host) {
  void* d = nullptr;
  if (!host || hipHostGetDevicePointer(&d, host, 0) != hipSuccess) { (void)hipGetLastError(); return nullptr; }
  return d;
}

// Queues the copies home of a batch whose kernels have been enqueued, once its compute chain is
// done (the host needs the arena sizes). The copies go to the SDMA engines when the destinations
// are pinned: a device-to-host copy issued from the CUs (the runtime's blit kernel, or our own)
// keeps the L2's path to the host full for as long as the link is busy, and the next batch's
// kernels then wait on their own memory traffic (k_chunks ran 6x slower under it).
static bool pipe_finalize(am_pipe* p, PipeSlot* sl) {
  if (sl->finalized) return true;
  if (!sl->launched) return false;  // its chain is not queued: nothing to finalize (a caller's bug)
  if (hipEventSynchronize(sl->ev_comp) != hipSuccess) return false;
  const uint64_t to = sl->h_totals[0], tp = sl->h_totals[1];
  const uint32_t nd = sl->b.ndocs;
  const uint64_t ns = sizeof(am_doc_summary) * (uint64_t)nd;
  const uint64_t no = std::min<uint64_t>(std::min<uint64_t>(to, p->caps.out_bytes), sl->h_out_cap);
  const uint64_t np = std::min<uint64_t>(std::min<uint64_t>(tp, p->caps.patch_bytes), sl->h_patch_cap);
  struct { void* dst; const void* src; uint64_t n; } cp[3] = {{sl->h_summ, sl->summ.p, ns}, {sl->h_out, sl->dout.p, no},
                                                             {sl->h_patch, sl->dpatch.p, np}};
  hsa_agent_t gpu, host;
  // AM_HOME_SDMA=0: copies home through the HIP copy kernel / stream instead of the SDMA engines
  static const bool sdma_on = [] { const char* e = std::getenv("AM_HOME_SDMA"); return !(e && e[0] == '0'); }();
  bool sdma = sdma_on && sl->home.handle && hsa_owner(sl->summ.p, gpu);
  for (auto& c : cp) sdma = sdma && (!c.n || hsa_owner(c.dst, host));
  sl->home_sdma = false;
  if (sdma) {
    uint32_t n = 0;
    for (auto& c : cp) n += c.n ? 1 : 0;
    hsa_signal_store_screlease(sl->home, n);
    for (auto& c : cp) {
      if (!c.n) continue;
      // engine mode: the engine chosen for this direction, apart from the one the inputs use
      const hsa_status_t st =
          p->eng_state > 0 ? hsa_amd_memory_async_copy_on_engine(c.dst, host, c.src, gpu, c.n, 0, nullptr, sl->home,
                                                                 (hsa_amd_sdma_engine_id_t)p->eng_home, false)
                           : hsa_amd_memory_async_copy(c.dst, host, c.src, gpu, c.n, 0, nullptr, sl->home);
      if (st != HSA_STATUS_SUCCESS) {
        hsa_signal_subtract_screlease(sl->home, 1);  // this one is not in flight
        sdma = false;
      }
    }
    sl->home_sdma = true;
    if (!sdma) {  // a copy was refused: wait for the others, then copy everything the HIP way
      if (!sdma_wait(sl->home)) return false;
      sl->home_sdma = false;
    }
  }
  if (!sl->home_sdma) {
    void *ds = mapped(sl->h_summ), *dout = mapped(sl->h_out), *dpat = mapped(sl->h_patch);
    if (ds && (dout || !no) && (dpat || !np) && no % 16 == 0 && np % 16 == 0) {
      am_launch_copy_home(sl->summ.p, ds, ns, sl->dout.p, dout, no, sl->dpatch.p, dpat, np, 64, p->s_out);
    } else {
      for (auto& c : cp)
        if (c.n && hipMemcpyAsync(c.dst, c.src, c.n, hipMemcpyDeviceToHost, p->s_out) != hipSuccess) return false;
    }
    if (hipEventRecord(sl->ev_out, p->s_out) != hipSuccess) return false;
  }
  p->totals.push_back(to);
  p->totals.push_back(tp);
  sl->finalized = true;
  return true;
}

// Waits until the SDMA copies counted by `sig` are done; false when one reported an error (the
// runtime sets the signal negative, which EQ 0 would wait for forever)
static bool sdma_wait(hsa_signal_t sig) {
  const hsa_signal_value_t v = hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_BLOCKED);
  if (v < 0) {
    hsa_signal_store_screlease(sig, 0);
    return false;
  }
  return true;
}

// the copies home of a finalized batch are complete (host wait)
static bool pipe_wait_home(PipeSlot* sl) {
  if (sl->home_sdma) {
    sl->home_sdma = false;
    return sdma_wait(sl->home);
  }
  return hipEventSynchronize(sl->ev_out) == hipSuccess;
}

// A slot reused by a new batch: the previous batch's copies home are queued (finalize) and its
// kernel times are read (its compute chain is complete); the new batch's H2D waits for that compute
// chain on the device and its kernels wait for the copies home -- no host wait on the copies.
// wait_home: the host also waits for the copies (drain).
static bool pipe_retire(am_pipe* p, PipeSlot* sl, bool wait_home) {
  if (!sl->busy) return true;
  if (!pipe_finalize(p, sl)) return false;
  float a = 0.f, d = 0.f;
  (void)hipEventElapsedTime(&a, sl->ev_c0, sl->ev_comp);
  (void)hipEventElapsedTime(&d, sl->ev_d0, sl->ev_d1);
  p->ms_comp += a;
  p->ms_doc += d;
  p->nms++;
  if (wait_home || sl->home_sdma) {
    // SDMA copies are not ordered with the HIP streams: the host waits before the slot is reused
    if (!pipe_wait_home(sl)) return false;
  } else if (hipStreamWaitEvent(p->s_c, sl->ev_out, 0) != hipSuccess) {
    return false;
  }
  if (hipStreamWaitEvent(p->s_in, sl->ev_comp, 0) != hipSuccess) return false;
  sl->busy = false;
  return true;
}

// Engine mode (AM_PIPE_ENGINES, default on): the copies home go to an SDMA engine of their own
// (hsa_amd_memory_async_copy_on_engine), apart from the runtime's preferred H2D engine that the
// input copies use, so the two directions of the host link run at the same time; left to the
// runtime, both can land on one engine and the step becomes H2D + D2H (BENCH_r04: 42.8 + 21.9 ms;
// tools/copy_probe.hip measured 57 GB/s for both directions together on one engine, 97 on two).
// The engines are the first ones the runtime reports free, its preferred ones first. Any failure
// turns the mode off for the pipeline.
static void pipe_choose_engines(am_pipe* p, const void* pinned_src, const void* dev_dst) {
  if (p->eng_state) return;
  p->eng_state = -1;
  const char* e = std::getenv("AM_PIPE_ENGINES");
  if (e && e[0] == '0') return;
  hsa_agent_t gpu, host;
  if (!hsa_owner(dev_dst, gpu) || !hsa_owner(pinned_src, host)) return;
  uint32_t st_in = 0, st_out = 0, pf_in = 0, pf_out = 0;
  if (hsa_amd_memory_copy_engine_status(gpu, host, &st_in) != HSA_STATUS_SUCCESS ||
      hsa_amd_memory_copy_engine_status(host, gpu, &st_out) != HSA_STATUS_SUCCESS)
    return;
  (void)hsa_amd_memory_get_preferred_copy_engine(gpu, host, &pf_in);
  (void)hsa_amd_memory_get_preferred_copy_engine(host, gpu, &pf_out);
  // the inputs go through the runtime's copy path, which takes the preferred H2D engine: the copies
  // home take another one
  auto lowest = [](uint32_t m) { return m & (~m + 1); };
  uint32_t in = lowest(pf_in & st_in);
  if (!in) in = lowest(st_in);
  uint32_t out = lowest(pf_out & st_out & ~in);
  if (!out) out = lowest(st_out & ~in);
  if (!in || !out) return;
  p->gpu = gpu;
  p->host = host;
  p->eng_h2d = in;
  p->eng_home = out;
  p->eng_state = 1;
}

// H2D of one input segment of the slot's batch on the input stream, ordered after the slot's
// previous compute chain (pipe_retire) and handed to the compute stream by an event: the runtime's
// own copy path, which also makes the new bytes visible to the kernels that follow it. (An input
// copy on an engine of our own, outside the streams, left stale input lines visible to the next
// batch's kernels in tests/test_gpu_pipe.py; only the copies home, read by the host, take an
// engine of their own.)
static bool pipe_h2d(am_pipe* p, PipeSlot* sl, void* dst, const void* src, uint64_t n) {
  (void)sl;
  if (!n) return true;
  pipe_choose_engines(p, src, dst);
  return hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, p->s_in) == hipSuccess;
}
// The hand-over of the inputs to the compute stream: the engine copies are waited for on the host
// (the previous batch's kernels keep the GPU busy meanwhile; its copies home are queued right after)
static bool pipe_h2d_done(am_pipe* p, PipeSlot* sl) {
  if (sl->in_sdma) {
    sl->in_sdma = false;
    if (!sdma_wait(sl->insig)) return false;
  }
  return hipStreamWaitEvent(p->s_c, sl->ev_in, 0) == hipSuccess;
}
// after the last input segment of a batch: the input stream's event for its segments (recorded now,
// before a later batch's copies join the stream)
static bool pipe_h2d_issued(am_pipe* p, PipeSlot* sl) { return hipEventRecord(sl->ev_in, p->s_in) == hipSuccess; }
// the batch whose inputs are queued but whose chain is not (pipe_submit) gets its chain now
static bool pipe_flush_pending(am_pipe* p);

extern "C" int am_pipe_engines(am_pipe* p, uint32_t* out2) {
  out2[0] = p->eng_h2d;
  out2[1] = p->eng_home;
  return 0;
}

// The inputs of a submission: either full descriptors (am_pipe_submit) or packed ones
// (am_pipe_submit_packed, expanded on the device after the H2D)
struct PipeIn {
  const am_chunk_desc* chunks = nullptr;
  const am_doc_desc* docs = nullptr;
  const uint32_t* clen = nullptr;
  const am_doc_span* spans = nullptr;
};

// The compute chain of a slot whose inputs were queued by pipe_submit: waits for its H2D (engine
// mode: on the host), queues every kernel on the compute stream, then queues the copies home of the
// batch launched before it (its kernels are ahead on the stream).
static bool pipe_launch(am_pipe* p, PipeSlot* sl) {
  am_batch& b = sl->b;
  const am_pipe_caps& c = p->caps;
  if (!pipe_h2d_done(p, sl)) return false;
  BatchDev d = b.dev();
  d.ws_cap = c.ws_bytes;
  hipStream_t s = p->s_c;
  (void)hipEventRecord(sl->ev_c0, s);
  if (sl->packed)
    am_launch_unpack(sl->clen.p, b.nchunks, sl->arena_len, sl->spans.p, b.ndocs, sl->c64.p, sl->coff.p, sl->ctmp.p, sl->olen.p,
                     sl->ooff.p, sl->tmp.p, sl->totals.p, b.chunks.p, b.docs.p, s);
  am_launch_chunks(d, s);
  am_launch_bounds(d, s);
  (void)hipEventRecord(sl->ev_d0, s);
  am_launch_doc(d, s);
  (void)hipEventRecord(sl->ev_d1, s);
  am_launch_out_hash(d, s);
  // documents past the caller's buffers (or the device arenas) report AM_U_CAPACITY
  am_launch_pipe_compact(d, sl->olen.p, sl->ooff.p, sl->plen.p, sl->poff.p, sl->tmp.p, sl->totals.p, sl->dout.p,
                         std::min<uint64_t>(c.out_bytes, sl->h_out ? sl->h_out_cap : 0), sl->dpatch.p,
                         std::min<uint64_t>(c.patch_bytes, sl->h_patch ? sl->h_patch_cap : 0), sl->summ.p, s);
  if (hipMemcpyAsync(sl->h_totals, sl->totals.p, 2 * sizeof(uint64_t), hipMemcpyDeviceToHost, s) != hipSuccess) return false;
  if (hipEventRecord(sl->ev_comp, s) != hipSuccess || hipGetLastError() != hipSuccess) return false;
  sl->launched = true;
  PipeSlot* prev = p->launched;
  p->launched = sl;
  // (with two slots the previous batch's slot may already be retired and refilled by the next
  // submission: its new batch is not launched yet and must not be finalized)
  return !prev || !prev->busy || !prev->launched || prev->finalized || pipe_finalize(p, prev);
}

static bool pipe_flush_pending(am_pipe* p) {
  PipeSlot* pend = p->pending;
  p->pending = nullptr;
  return !pend || pipe_launch(p, pend);
}

// Queues batch `ticket`'s inputs, then the compute chain of the batch submitted before it: the
// input engine always holds the next batch's copy while the previous one is being waited for, so
// the host link never idles between batches.
static int pipe_submit(am_pipe* p, const uint8_t* arena, uint64_t arena_len, const PipeIn& in, uint32_t nchunks, uint32_t ndocs,
                       bool any_diff, am_doc_summary* summary, uint8_t* out, uint64_t out_cap, uint8_t* patches,
                       uint64_t patch_cap, uint64_t* ticket, am_error* err) {
  auto fail = [&](const char* m) { to_c(Err{AM_U_CAPACITY, false, m}, err); return 1; };
  if (!set_device(p->eng)) return fail("automerge_amd: no device");
  const am_pipe_caps& c = p->caps;
  if (arena_len > c.arena_bytes || nchunks > c.chunks || ndocs > c.docs)
    return fail("automerge_amd: batch exceeds the pipeline capacities");
  // resident batches run on slot 0's workspace without a ticket: they finish first
  if (p->nres) return fail("automerge_amd: resident batches in flight (am_pipe_resident_sync first)");
  PipeSlot* sl = p->slots[p->next % p->slots.size()];
  const bool packed = in.clen != nullptr;
  if (packed && !(sl->clen.ensure(c.chunks) && sl->spans.ensure(c.docs) && sl->c64.ensure(c.chunks) && sl->coff.ensure(c.chunks) &&
                  sl->ctmp.ensure(am_scan_tmp_elems(c.chunks))))
    return fail("automerge_amd: device allocation failed (packed descriptors)");
  if (sl == p->pending && !pipe_flush_pending(p)) return fail("automerge_amd: HIP error while launching a batch");
  if (!pipe_retire(p, sl, false)) return fail("automerge_amd: HIP error while retiring a batch");
  am_batch& b = sl->b;
  b.nchunks = nchunks;
  b.ndocs = ndocs;
  b.any_diff = any_diff;
  b.lds_bytes = lds_budget(any_diff);
  sl->packed = packed;
  sl->arena_len = arena_len;
  // inputs
  if (!pipe_h2d(p, sl, b.arena.p, arena, arena_len)) return fail("automerge_amd: H2D failed");
  if (packed) {
    if (!pipe_h2d(p, sl, sl->clen.p, in.clen, sizeof(uint32_t) * nchunks) ||
        !pipe_h2d(p, sl, sl->spans.p, in.spans, sizeof(am_doc_span) * ndocs))
      return fail("automerge_amd: H2D failed");
  } else if (!pipe_h2d(p, sl, b.chunks.p, in.chunks, sizeof(am_chunk_desc) * nchunks) ||
             !pipe_h2d(p, sl, b.docs.p, in.docs, sizeof(am_doc_desc) * ndocs)) {
    return fail("automerge_amd: H2D failed");
  }
  if (!pipe_h2d_issued(p, sl)) return fail("automerge_amd: stream ordering failed");
  sl->busy = true;
  sl->launched = false;
  sl->finalized = false;
  sl->ticket = p->next;
  sl->h_summ = summary;
  sl->h_out = out;
  sl->h_out_cap = out_cap;
  sl->h_patch = patches;
  sl->h_patch_cap = patch_cap;
  if (ticket) *ticket = p->next;
  p->next++;
  // the batch submitted before this one: its chain now (its inputs are on their way or there)
  PipeSlot* pend = p->pending;
  p->pending = sl;
  if (pend && !pipe_launch(p, pend)) return fail("automerge_amd: HIP error while launching a batch");
  if (err) err->code = 0;
  return 0;
}

extern "C" int am_pipe_submit(am_pipe* p, const uint8_t* arena, uint64_t arena_len, const am_chunk_desc* chunks,
                              uint32_t nchunks, const am_doc_desc* docs, uint32_t ndocs, am_doc_summary* summary,
                              uint8_t* out, uint64_t out_cap, uint8_t* patches, uint64_t patch_cap, uint64_t* ticket,
                              am_error* err) {
  PipeIn in;
  in.chunks = chunks;
  in.docs = docs;
  bool any_diff = false;
  for (uint32_t d = 0; d < ndocs && !any_diff; d++) any_diff = (docs[d].flags & (AM_DOC_WANT_DIFF | AM_DOC_WANT_PATCH)) != 0;
  return pipe_submit(p, arena, arena_len, in, nchunks, ndocs, any_diff, summary, out, out_cap, patches, patch_cap, ticket, err);
}

extern "C" int am_pipe_submit_packed(am_pipe* p, const uint8_t* arena, uint64_t arena_len, const uint32_t* chunk_len,
                                     uint32_t nchunks, const am_doc_span* docs, uint32_t ndocs, am_doc_summary* summary,
                                     uint8_t* out, uint64_t out_cap, uint8_t* patches, uint64_t patch_cap, uint64_t* ticket,
                                     am_error* err) {
  if ((nchunks && !chunk_len) || (ndocs && !docs)) {
    to_c(Err{AM_U_CAPACITY, false, "automerge_amd: missing packed descriptors"}, err);
    return 1;
  }
  PipeIn in;
  static const uint32_t none = 0;
  static const am_doc_span nospan{};
  in.clen = nchunks ? chunk_len : &none;
  in.spans = ndocs ? docs : &nospan;
  bool any_diff = false;
  for (uint32_t d = 0; d < ndocs && !any_diff; d++) any_diff = (docs[d].flags & (AM_DOC_WANT_DIFF | AM_DOC_WANT_PATCH)) != 0;
  return pipe_submit(p, arena, arena_len, in, nchunks, ndocs, any_diff, summary, out, out_cap, patches, patch_cap, ticket, err);
}

// One batch whose inputs are already resident in device memory: the whole chain of am_pipe_submit
// (k_chunks .. k_pipe_compact) on the pipeline's compute stream, with the merged documents, patch
// logs and summaries compacted into the caller's device buffers and the two arena totals written to
// d_totals; nothing crosses the host link and the host does not wait (hipStreamSynchronize /
// am_pipe_drain). Batches run back to back on one stream and share slot 0's workspace.
extern "C" int am_pipe_run_resident(am_pipe* p, const uint8_t* d_arena, uint64_t arena_len, const am_chunk_desc* d_chunks,
                                    uint32_t nchunks, const am_doc_desc* d_docs, uint32_t ndocs, int any_diff,
                                    am_doc_summary* d_summary, uint8_t* d_out, uint64_t out_cap, uint8_t* d_patches,
                                    uint64_t patch_cap, uint64_t* d_totals, am_error* err) {
  auto fail = [&](const char* m) { to_c(Err{AM_U_CAPACITY, false, m}, err); return 1; };
  if (!set_device(p->eng)) return fail("automerge_amd: no device");
  const am_pipe_caps& c = p->caps;
  if (arena_len > c.arena_bytes || nchunks > c.chunks || ndocs > c.docs)
    return fail("automerge_amd: batch exceeds the pipeline capacities");
  // 4 events per batch until am_pipe_resident_sync: a bounded number of batches between syncs
  if (p->nres >= 4096) return fail("automerge_amd: 4096 resident batches without am_pipe_resident_sync");
  if (!pipe_flush_pending(p)) return fail("automerge_amd: HIP error while launching a batch");
  PipeSlot* sl = p->slots[0];
  if (sl->busy && !pipe_retire(p, sl, true)) return fail("automerge_amd: HIP error while retiring a batch");
  am_batch& b = sl->b;
  b.nchunks = nchunks;
  b.ndocs = ndocs;
  b.any_diff = any_diff != 0;
  BatchDev d = b.dev();
  d.arena = d_arena;
  d.chunks = d_chunks;
  d.docs = d_docs;
  d.ws_cap = c.ws_bytes;
  while (p->rev.size() < 4ull * (p->nres + 1)) {
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) return fail("automerge_amd: cannot create a HIP event");
    p->rev.push_back(e);
  }
  hipEvent_t* ev = p->rev.data() + 4ull * p->nres++;
  hipStream_t s = p->s_c;
  (void)hipEventRecord(ev[0], s);
  am_launch_chunks(d, s);
  am_launch_bounds(d, s);
  (void)hipEventRecord(ev[1], s);
  am_launch_doc(d, s);
  (void)hipEventRecord(ev[2], s);
  am_launch_out_hash(d, s);
  am_launch_pipe_compact(d, sl->olen.p, sl->ooff.p, sl->plen.p, sl->poff.p, sl->tmp.p, d_totals, d_out, out_cap, d_patches,
                         patch_cap, d_summary, s);
  if (hipEventRecord(ev[3], s) != hipSuccess || hipGetLastError() != hipSuccess) return fail("automerge_amd: kernel launch failed");
  if (err) err->code = 0;
  return 0;
}

// Waits for the resident batches run since the last call; ms2 = their whole chains and their
// document kernels (k_doc_fast + k_doc), summed over the batches (HIP events on the compute stream).
extern "C" int am_pipe_resident_sync(am_pipe* p, float* ms2, am_error* err) {
  if (!set_device(p->eng) || hipStreamSynchronize(p->s_c) != hipSuccess) {
    to_c(Err{AM_U_CAPACITY, false, "automerge_amd: HIP error in a resident batch"}, err);
    return 1;
  }
  ms2[0] = ms2[1] = 0.f;
  for (uint32_t k = 0; k < p->nres; k++) {
    float a = 0.f, d = 0.f;
    (void)hipEventElapsedTime(&a, p->rev[4 * k], p->rev[4 * k + 3]);
    (void)hipEventElapsedTime(&d, p->rev[4 * k + 1], p->rev[4 * k + 2]);
    ms2[0] += a;
    ms2[1] += d;
  }
  p->nres = 0;
  if (err) err->code = 0;
  return 0;
}

extern "C" int am_pipe_drain(am_pipe* p, uint64_t* totals, uint32_t cap, am_error* err) {
  if (!set_device(p->eng)) { to_c(Err{AM_U_CAPACITY, false, "automerge_amd: no device"}, err); return 1; }
  if (!pipe_flush_pending(p)) {
    to_c(Err{AM_U_CAPACITY, false, "automerge_amd: HIP error while launching a batch"}, err);
    return 1;
  }
  const size_t S = p->slots.size();
  // in submission order
  for (uint64_t t = p->next >= S ? p->next - S : 0; t < p->next; t++) {
    PipeSlot* sl = p->slots[t % S];
    if (sl->busy && sl->ticket == t && !pipe_retire(p, sl, true)) {
      to_c(Err{AM_U_CAPACITY, false, "automerge_amd: HIP error while draining the pipeline"}, err);
      return 1;
    }
  }
  for (uint32_t i = 0; totals && i < cap && 2 * i + 1 < p->totals.size(); i++) {
    totals[2 * i] = p->totals[2 * i];
    totals[2 * i + 1] = p->totals[2 * i + 1];
  }
  p->totals.clear();
  if (err) err->code = 0;
  return 0;
}

extern "C" int am_pipe_times(am_pipe* p, float* ms2, uint32_t* n) {
  ms2[0] = p->ms_comp;
  ms2[1] = p->ms_doc;
  *n = p->nms;
  p->ms_comp = p->ms_doc = 0.f;  // reset on read
  p->nms = 0;
  return 0;
}

// =============================================================================================
// per-document backend state (backend/backend.js + BackendDoc over the batch path, n = 1)
// =============================================================================================
struct am_doc {
  am_engine* eng = nullptr;
  std::vector<uint8_t> state;   // merged document chunk, uncompressed columns (empty = Backend.init())
  std::vector<uint8_t> binary;  // save() cache: the loaded buffer until the first applyChanges (new.js:1712,1859)
  bool has_binary = false;
  bool have_hash_graph = true;  // new.js:1697,1752
  std::vector<std::vector<uint8_t>> changes;           // applied change buffers (this.changes)
  std::vector<std::array<uint8_t, 32>> hashes;         // their hashes
  std::vector<std::vector<uint8_t>> queue;             // enqueued change buffers (this.queue)
  std::vector<std::array<uint8_t, 32>> queue_hashes;   // their hashes
  std::vector<std::array<uint8_t, 32>> heads;
  std::vector<std::array<uint8_t, 32>> load_heads;     // changeIndexByHash of a loaded document without its graph
  HashGraph graph;                                     // over changes[0, graph.size()) (am_graph.h)
  // objectMeta's children snapshots as this handle's last applyChanges left them (am_diff.h
  // diff_meta_pack; new.js:1812, 1857); empty: documentPatch's of the state (load / init)
  std::vector<uint8_t> meta;
  int64_t max_op = 0;
  size_t nchanges = 0;
};

namespace {

am_batch* scratch_batch(am_engine* e) {
  if (!e->scratch) e->scratch = am_batch_create(e);
  return e->scratch;
}

// Host stage for one change buffer: DEFLATE-compressed changes (chunk type 2) are inflated into
// an uncompressed type-1 chunk that keeps the original checksum (inflateChange, columnar.js:813).
bool stage_change(const std::vector<uint8_t>& in, std::vector<uint8_t>& out, Err& err) {
  if (in.size() > 8 && in[8] == 2) {
    if (in.size() < 4 || std::memcmp(in.data(), "\x85\x6f\x4a\x83", 4) != 0) {
      err = {AM_E_MAGIC, false, message_for(AM_E_MAGIC, 0, 0, "")};
      return false;
    }
    Container c;
    if (!read_container(in.data(), in.size(), c)) {
      err = {AM_E_SUBARRAY, false, message_for(AM_E_SUBARRAY, 0, 0, "")};
      return false;
    }
    std::vector<uint8_t> dec;
    if (!zinflate(in.data() + c.data_off, c.data_len, dec)) {
      err = {AM_E_INFLATE, false, message_for(AM_E_INFLATE, 0, 0, "")};
      return false;
    }
    out = make_chunk(in.data() + 4, 1, dec);
    return true;
  }
  out = in;
  return true;
}

struct OneResult {
  am_doc_result r;
  std::vector<uint8_t> out;
  std::vector<int32_t> chg_state;
  std::vector<std::array<uint8_t, 32>> hashes;
  std::vector<std::array<uint8_t, 32>> heads;
  std::vector<uint8_t> patch;  // patch log (patch_mode: 1 getPatch, 2 the applyChanges patch)
  std::vector<uint8_t> meta;   // AM_DOC_META: the objectMeta blob the call leaves
};

// The objectMeta blob after a patch log's stream (AM_DOC_META) goes to res.meta; the log keeps
// header + stream.
void split_meta(OneResult& res) {
  res.meta.clear();
  if (res.patch.size() < sizeof(PatchHdr2)) return;
  PatchHdr2 h;
  std::memcpy(&h, res.patch.data(), sizeof h);
  if (h.meta_bytes && sizeof h + h.nbytes + h.meta_bytes == res.patch.size()) {
    res.meta.assign(res.patch.begin() + sizeof h + h.nbytes, res.patch.end());
    res.patch.resize(sizeof h + h.nbytes);
    h.meta_bytes = 0;
    std::memcpy(res.patch.data(), &h, sizeof h);
  }
}

// Runs one document (optional base chunk + change list) through the GPU pipeline.
// With `meta` (patch_mode 2): the handle's objectMeta snapshots go in (empty: documentPatch's) and
// res.meta receives what the call leaves.
bool run_one(am_engine* e, const std::vector<uint8_t>* base, bool base_verified, const std::vector<std::vector<uint8_t>>& chg,
             const std::vector<am_known_hash>& known, bool have_graph, OneResult& res, std::vector<uint8_t>& arena, Err& err,
             int patch_mode = 0, uint32_t extra_flags = 0, const std::vector<uint8_t>* meta = nullptr) {
  arena.clear();
  std::vector<am_chunk_desc> cds;
  am_doc_desc dd{};
  dd.base_chunk = -1;
  if (base && !base->empty()) {
    cds.push_back({arena.size(), (uint32_t)base->size(), base_verified ? 1u : 0u});
    arena.insert(arena.end(), base->begin(), base->end());
    dd.base_chunk = 0;
  }
  dd.chg_begin = (uint32_t)cds.size();
  dd.chg_count = (uint32_t)chg.size();
  for (auto& c : chg) {
    cds.push_back({arena.size(), (uint32_t)c.size(), 0});
    arena.insert(arena.end(), c.begin(), c.end());
  }
  dd.known_begin = 0;
  dd.known_count = (uint32_t)known.size();
  dd.flags = (have_graph ? 1u : 0u) | (patch_mode == 1 ? AM_DOC_WANT_PATCH : 0u) | (patch_mode == 2 ? AM_DOC_WANT_DIFF : 0u) |
             extra_flags;
  dd.meta_chunk = 0;
  if (meta && patch_mode == 2) {
    dd.flags |= AM_DOC_META;
    if (!meta->empty()) {
      dd.meta_chunk = (uint32_t)cds.size() + 1;
      cds.push_back({arena.size(), (uint32_t)meta->size(), AM_CHUNK_RAW});
      arena.insert(arena.end(), meta->begin(), meta->end());
    }
  }
  am_batch* b = scratch_batch(e);
  am_error ce;
  HostClock clk;
  clk.mark("pack");
  for (;;) {
    if (am_batch_stage(b, arena.data(), arena.size(), cds.data(), (uint32_t)cds.size(), &dd, 1, known.data(),
                       (uint32_t)known.size(), &ce) ||
        am_batch_run(b) || am_batch_sync(b, &ce) || am_batch_results(b, &res.r)) {
      err = {AM_U_CAPACITY, false, std::string("automerge_amd: GPU pipeline failed: ") + ce.message};
      return false;
    }
    // invalid UTF-8 in a key or message: run again with room for the U+FFFD replacements
    if (res.r.status != AM_U_UTF8 || (dd.flags & AM_DOC_FIX_UTF8)) break;
    dd.flags |= AM_DOC_FIX_UTF8;
  }
  clk.mark("stage+run+sync");
  if (clk.on) {
    float t[4] = {0, 0, 0, 0};
    am_batch_stage_times(b, t);
    char m[160];
    std::snprintf(m, sizeof m, " [k_chunks=%.2f bounds=%.2f doc=%.2f out_hash=%.2f ms; arena=%zu B]", t[0], t[1], t[2], t[3],
                  arena.size());
    clk.line += m;
  }
  {
    uint8_t f = 0;
    if (am_batch_fast_flags(b, &f) == 0) {
      e->stat_docs++;
      e->stat_fast += f;
    }
  }
  res.chg_state.assign(cds.size(), 0);
  std::vector<uint8_t> hs(32 * cds.size());
  std::vector<uint32_t> st(cds.size());
  if (!cds.empty() && am_batch_chunk_results(b, hs.data(), res.chg_state.data(), st.data())) {
    err = {AM_U_CAPACITY, false, "automerge_amd: result copy failed"};
    return false;
  }
  res.hashes.resize(cds.size());
  for (size_t i = 0; i < cds.size(); i++) std::memcpy(res.hashes[i].data(), hs.data() + 32 * i, 32);
  if (res.r.status) {
    std::string actor;
    if (res.r.arg_actor_len && res.r.arg_actor_off + res.r.arg_actor_len <= arena.size())
      actor = hexs(arena.data() + res.r.arg_actor_off, res.r.arg_actor_len);
    err = {res.r.status, false, message_for(res.r.status, res.r.arg0, res.r.arg1, actor)};
    return false;
  }
  res.out.resize(res.r.out_len);
  uint64_t len = 0;
  if (am_batch_doc_output(b, 0, res.out.data(), res.out.size(), &len)) {
    err = {AM_U_CAPACITY, false, "automerge_amd: output copy failed"};
    return false;
  }
  std::vector<uint8_t> hb(32 * (res.r.nheads + 1));
  uint32_t nh = 0;
  am_batch_doc_heads(b, 0, hb.data(), res.r.nheads, &nh);
  res.heads.resize(nh);
  for (uint32_t i = 0; i < nh; i++) std::memcpy(res.heads[i].data(), hb.data() + 32 * i, 32);
  if (patch_mode) {
    uint64_t plen = 0;
    if (am_batch_doc_patch(b, 0, nullptr, 0, &plen)) {
      err = {AM_U_CAPACITY, false, "automerge_amd: patch copy failed"};
      return false;
    }
    res.patch.resize(plen);
    if (am_batch_doc_patch(b, 0, res.patch.data(), plen, &plen)) {
      err = {AM_U_CAPACITY, false, "automerge_amd: patch copy failed"};
      return false;
    }
    split_meta(res);
  }
  clk.mark("results-home");
  clk.print("run_one", arena.size());
  return true;
}

// heads of a document chunk (decodeDocumentHeader: actors, then the sorted heads)
bool chunk_heads(const std::vector<uint8_t>& chunk, std::vector<std::array<uint8_t, 32>>& heads) {
  Container c;
  if (!read_container(chunk.data(), chunk.size(), c)) return false;
  HRd r{chunk.data() + c.data_off, c.data_len, 0};
  const uint64_t na = r.u();
  for (uint64_t i = 0; i < na && r.ok; i++) r.raw(r.u());
  const uint64_t nh = r.u();
  const uint8_t* h = r.raw(32 * nh);
  if (!r.ok) return false;
  heads.resize(nh);
  for (uint64_t i = 0; i < nh; i++) std::memcpy(heads[i].data(), h + 32 * i, 32);
  return true;
}

// Every document's merged chunk and patch log of the last run of batch b, densely in two host
// arenas (k_pipe_lens / k_pipe_compact: a sizing pass, then the copies; one D2H each).
bool batch_collect(am_batch* b, const am_doc_summary*& summ, const uint8_t*& out, const uint8_t*& pat) {
  am_engine* e = b->eng;
  if (!e->coll) e->coll = new CollectBufs();
  CollectBufs& c = *e->coll;
  const uint32_t nd = b->ndocs;
  if (!c.olen.ensure(nd) || !c.ooff.ensure(nd) || !c.plen.ensure(nd) || !c.poff.ensure(nd) ||
      !c.tmp.ensure(am_scan_tmp_elems(nd)) || !c.totals.ensure(2) || !c.summ.ensure(nd))
    return false;
  hipStream_t s = e->stream;
  BatchDev d = b->dev();
  uint64_t tot[2] = {0, 0};
  am_launch_pipe_compact(d, c.olen.p, c.ooff.p, c.plen.p, c.poff.p, c.tmp.p, c.totals.p, nullptr, 0, nullptr, 0, c.summ.p, s);
  if (hipMemcpyAsync(tot, c.totals.p, sizeof tot, hipMemcpyDeviceToHost, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
    return false;
  if (!c.out.ensure(tot[0] + 16) || !c.pat.ensure(tot[1] + 16)) return false;
  if (!c.h_summ.ensure(nd + 1) || !c.h_out.ensure(tot[0] + 16) || !c.h_pat.ensure(tot[1] + 16)) return false;
  am_launch_pipe_compact(d, c.olen.p, c.ooff.p, c.plen.p, c.poff.p, c.tmp.p, c.totals.p, c.out.p, tot[0], c.pat.p, tot[1],
                         c.summ.p, s);
  if (nd && hipMemcpyAsync(c.h_summ.p, c.summ.p, sizeof(am_doc_summary) * nd, hipMemcpyDeviceToHost, s) != hipSuccess) return false;
  if (tot[0] && hipMemcpyAsync(c.h_out.p, c.out.p, tot[0], hipMemcpyDeviceToHost, s) != hipSuccess) return false;
  if (tot[1] && hipMemcpyAsync(c.h_pat.p, c.pat.p, tot[1], hipMemcpyDeviceToHost, s) != hipSuccess) return false;
  summ = c.h_summ.p;
  out = c.h_out.p;
  pat = c.h_pat.p;
  return hipStreamSynchronize(s) == hipSuccess && hipGetLastError() == hipSuccess;
}

// One GPU batch for many documents (the batched per-handle calls): per document its base chunk
// and changes (adjacent in the arena), its known hashes and its objectMeta blob; per document the
// result run_one gives, or the error the document raised.
struct ManyJob {
  const std::vector<uint8_t>* base = nullptr;
  bool base_verified = false;
  const std::vector<std::vector<uint8_t>>* chg = nullptr;
  const std::vector<am_known_hash>* known = nullptr;
  bool have_graph = false;
  int patch_mode = 0;
  const std::vector<uint8_t>* meta = nullptr;  // patch_mode 2: the handle's objectMeta blob
};
struct ManyOut {
  OneResult res;
  Err err;
  bool ok = false;
};

bool run_many(am_engine* e, const std::vector<ManyJob>& jobs, std::vector<ManyOut>& outs, Err& err) {
  HostClock clk;
  const size_t n = jobs.size();
  outs.assign(n, ManyOut());
  if (!n) return true;
  // layout: per document its base and changes adjacent, then every objectMeta blob; offsets first,
  // then the copies on the host workers
  std::vector<uint64_t> aoff(n + 1), moff(n + 1);
  std::vector<uint32_t> c0(n + 1), kb(n + 1);
  std::vector<am_doc_desc> dds(n);
  c0[0] = 0;
  aoff[0] = 0;
  kb[0] = 0;
  for (size_t i = 0; i < n; i++) {
    const ManyJob& j = jobs[i];
    uint64_t bytes = (j.base ? j.base->size() : 0);
    uint32_t nc = (j.base && !j.base->empty()) ? 1u : 0u;
    if (j.chg)
      for (auto& c : *j.chg) bytes += c.size();
    nc += j.chg ? (uint32_t)j.chg->size() : 0u;
    aoff[i + 1] = aoff[i] + bytes;
    c0[i + 1] = c0[i] + nc;
    kb[i + 1] = kb[i] + (j.known ? (uint32_t)j.known->size() : 0u);
  }
  moff[0] = aoff[n];
  uint32_t nmeta = 0;
  for (size_t i = 0; i < n; i++) {
    const bool m = jobs[i].meta && jobs[i].patch_mode == 2 && !jobs[i].meta->empty();
    moff[i + 1] = moff[i] + (m ? jobs[i].meta->size() : 0);
    nmeta += m;
  }
  const uint32_t nchunks = c0[n] + nmeta;
  if (!e->coll) e->coll = new CollectBufs();
  std::vector<uint8_t> arena_v;  // pageable fallback when pinned memory is short
  uint8_t* arena = e->coll->h_arena.ensure(moff[n] + 16) ? e->coll->h_arena.p : (arena_v.resize(moff[n] + 16), arena_v.data());
  const uint64_t arena_len = moff[n];
  std::vector<am_chunk_desc> cds(nchunks);
  std::vector<am_known_hash> known(kb[n]);
  std::vector<uint32_t> mchunk(n, 0);
  for (uint32_t i = 0, k = c0[n]; i < n; i++)
    if (moff[i + 1] > moff[i]) mchunk[i] = k++;
  am_par_for(n, [&](size_t i) {
    const ManyJob& j = jobs[i];
    am_doc_desc dd{};
    dd.base_chunk = -1;
    uint64_t o = aoff[i];
    uint32_t c = c0[i];
    if (j.base && !j.base->empty()) {
      dd.base_chunk = (int64_t)c;
      cds[c++] = {o, (uint32_t)j.base->size(), j.base_verified ? 1u : 0u};
      std::memcpy(arena + o, j.base->data(), j.base->size());
      o += j.base->size();
    }
    dd.chg_begin = c;
    dd.chg_count = j.chg ? (uint32_t)j.chg->size() : 0u;
    if (j.chg)
      for (auto& ch : *j.chg) {
        cds[c++] = {o, (uint32_t)ch.size(), 0};
        if (!ch.empty()) std::memcpy(arena + o, ch.data(), ch.size());
        o += ch.size();
      }
    dd.known_begin = kb[i];
    dd.known_count = kb[i + 1] - kb[i];
    if (dd.known_count) std::memcpy(known.data() + kb[i], j.known->data(), sizeof(am_known_hash) * dd.known_count);
    dd.flags = (j.have_graph ? 1u : 0u) | (j.patch_mode == 1 ? AM_DOC_WANT_PATCH : 0u) | (j.patch_mode == 2 ? AM_DOC_WANT_DIFF : 0u);
    dd.meta_chunk = 0;
    if (j.meta && j.patch_mode == 2) {  // objectMeta blobs after every document's chunks
      dd.flags |= AM_DOC_META;
      if (moff[i + 1] > moff[i]) {
        dd.meta_chunk = mchunk[i] + 1;
        cds[mchunk[i]] = {moff[i], (uint32_t)j.meta->size(), AM_CHUNK_RAW};
        std::memcpy(arena + moff[i], j.meta->data(), j.meta->size());
      }
    }
    dds[i] = dd;
  });
  clk.mark("pack");
  am_batch* b = scratch_batch(e);
  am_error ce;
  if (am_batch_stage(b, arena, arena_len, cds.data(), nchunks, dds.data(), (uint32_t)n, known.data(),
                     (uint32_t)known.size(), &ce) ||
      am_batch_run(b) || am_batch_sync(b, &ce)) {
    err = {AM_U_CAPACITY, false, std::string("automerge_amd: GPU pipeline failed: ") + ce.message};
    return false;
  }
  clk.mark("gpu");
  std::vector<am_doc_result> rr(n);
  std::vector<uint8_t> hs(32ull * nchunks);
  std::vector<int32_t> cst(nchunks);
  const am_doc_summary* summ = nullptr;
  const uint8_t *out = nullptr, *pat = nullptr;
  bool ok = am_batch_results(b, rr.data()) == 0 && e->coll->hashes.ensure(32ull * nchunks + 16);
  if (ok && nchunks) {
    am_launch_chunk_hashes(b->info.p, nchunks, e->coll->hashes.p, e->stream);
    ok = hipMemcpyAsync(hs.data(), e->coll->hashes.p, hs.size(), hipMemcpyDeviceToHost, e->stream) == hipSuccess &&
         hipMemcpyAsync(cst.data(), b->chg_state.p, 4ull * nchunks, hipMemcpyDeviceToHost, e->stream) == hipSuccess &&
         hipStreamSynchronize(e->stream) == hipSuccess;
  }
  if (!ok || !batch_collect(b, summ, out, pat)) {
    err = {AM_U_CAPACITY, false, "automerge_amd: result copy failed"};
    return false;
  }
  {
    std::vector<uint8_t> fd(n);
    if (am_batch_fast_flags(b, fd.data()) == 0) {
      e->stat_docs += n;
      for (uint8_t f : fd) e->stat_fast += f;
    }
  }
  clk.mark("home");
  am_par_for(n, [&](size_t i) {
    ManyOut& o = outs[i];
    OneResult& res = o.res;
    res.r = rr[i];
    const uint32_t cb = c0[i], cn = c0[i + 1] - c0[i];
    res.chg_state.assign(cst.begin() + cb, cst.begin() + cb + cn);
    res.hashes.resize(cn);
    for (uint32_t k = 0; k < cn; k++) std::memcpy(res.hashes[k].data(), hs.data() + 32ull * (cb + k), 32);
    if (rr[i].status) {
      std::string actor;
      if (rr[i].arg_actor_len && rr[i].arg_actor_off + rr[i].arg_actor_len <= arena_len)
        actor = hexs(arena + rr[i].arg_actor_off, rr[i].arg_actor_len);
      o.err = {rr[i].status, false, message_for(rr[i].status, rr[i].arg0, rr[i].arg1, actor)};
      return;
    }
    const am_doc_summary& sm = summ[i];
    if (sm.status || sm.out_len != rr[i].out_len) {
      o.err = {AM_U_CAPACITY, false, "automerge_amd: output compaction failed"};
      return;
    }
    res.out.assign(out + sm.out_off, out + sm.out_off + sm.out_len);
    if (!chunk_heads(res.out, res.heads)) {
      o.err = {AM_U_VALUE, false, "automerge_amd: corrupt merged document"};
      return;
    }
    if (jobs[i].patch_mode) {
      res.patch.assign(pat + sm.patch_off, pat + sm.patch_off + sm.patch_len);
      split_meta(res);
    }
    o.ok = true;
  });
  clk.mark("unpack");
  clk.print("run_many", n);
  return true;
}

bool gpu_sha256(am_engine* e, const std::vector<const std::vector<uint8_t>*>& msgs, size_t skip,
                std::vector<std::array<uint8_t, 32>>& out) {
  std::vector<uint8_t> arena;
  std::vector<am_chunk_desc> d;
  for (auto* m : msgs) {
    size_t n = m->size() > skip ? m->size() - skip : 0;
    d.push_back({arena.size(), (uint32_t)n, 0});
    arena.insert(arena.end(), m->begin() + (m->size() > skip ? skip : m->size()), m->end());
  }
  if (!set_device(e)) return false;
  DevBuf<uint8_t> da;
  DevBuf<am_chunk_desc> dd;
  DevBuf<uint8_t> dout;
  // +16: sha256_words loads whole words past a message's last byte
  if (!da.ensure(arena.size() + 16) || !dd.ensure(d.size()) || !dout.ensure(32 * d.size())) return false;
  hipStream_t s = e->stream;
  if (!arena.empty()) HIPCHECK(hipMemcpyAsync(da.p, arena.data(), arena.size(), hipMemcpyHostToDevice, s));
  HIPCHECK(hipMemcpyAsync(dd.p, d.data(), sizeof(am_chunk_desc) * d.size(), hipMemcpyHostToDevice, s));
  am_launch_sha256(da.p, dd.p, (uint32_t)d.size(), dout.p, s);
  std::vector<uint8_t> h(32 * d.size());
  HIPCHECK(hipMemcpyAsync(h.data(), dout.p, h.size(), hipMemcpyDeviceToHost, s));
  HIPCHECK(hipStreamSynchronize(s));
  out.resize(d.size());
  for (size_t i = 0; i < d.size(); i++) std::memcpy(out[i].data(), h.data() + 32 * i, 32);
  return true;
}

// Host stage of Backend.load for documents with DEFLATE-compressed columns: the checksum of the
// original chunk is verified on the GPU, then the columns are inflated (inflateColumn,
// columnar.js:1062) into an uncompressed chunk marked as verified.
}  // namespace
extern "C" int am_inflate_raw(am_engine* eng, const uint8_t* const* bufs, const size_t* lens, size_t n, uint8_t** outs,
                              size_t* out_lens, uint8_t* ok, am_error* err);
namespace {

bool stage_doc(am_engine* e, const std::vector<uint8_t>& in, std::vector<uint8_t>& out, bool& verified, Err& err) {
  verified = false;
  Container c;
  if (in.size() < 4 || std::memcmp(in.data(), "\x85\x6f\x4a\x83", 4) != 0 || !read_container(in.data(), in.size(), c) ||
      c.type != 0) {
    out = in;  // let the GPU report the exact error
    return true;
  }
  DocParts parts;
  if (!split_doc(in.data() + c.data_off, c.data_len, parts)) { out = in; return true; }
  bool any = false;
  for (auto* cols : {&parts.ccols, &parts.ocols})
    for (auto& col : *cols) any |= (col.id & COL_DEFLATE) != 0;
  if (!any) { out = in; return true; }
  std::vector<uint8_t> whole(in.begin() + 8, in.begin() + c.end);
  std::vector<std::array<uint8_t, 32>> hh;
  if (!gpu_sha256(e, {&whole}, 0, hh)) { err = {AM_U_CAPACITY, false, "automerge_amd: GPU hash failed"}; return false; }
  if (std::memcmp(hh[0].data(), in.data() + 4, 4) != 0) {
    err = {AM_E_CHECKSUM, false, message_for(AM_E_CHECKSUM, 0, 0, "")};
    return false;
  }
  // the DEFLATEd columns (inflateColumn, columnar.js:1062-1068) inflate on the GPU in one batch
  std::vector<std::vector<uint8_t>*> zcol;
  std::vector<uint64_t*> zid;
  std::vector<const uint8_t*> zb;
  std::vector<size_t> zl;
  for (auto* cols : {&parts.ccols, &parts.ocols})
    for (auto& col : *cols)
      if (col.id & COL_DEFLATE) {
        zcol.push_back(&col.data);
        zid.push_back(&col.id);
        zb.push_back(col.data.data());
        zl.push_back(col.data.size());
      }
  const size_t nz = zb.size();
  std::vector<uint8_t*> zo(nz, nullptr);
  std::vector<size_t> zn(nz, 0);
  std::vector<uint8_t> zok(nz, 0);
  am_error ae;
  if (am_inflate_raw(e, zb.data(), zl.data(), nz, zo.data(), zn.data(), zok.data(), &ae)) {
    err = {AM_U_CAPACITY, false, ae.message};
    return false;
  }
  bool all_ok = true;
  for (size_t i = 0; i < nz; i++) {
    if (zok[i]) {
      zcol[i]->assign(zo[i], zo[i] + zn[i]);
      *zid[i] ^= COL_DEFLATE;
    } else {
      all_ok = false;
    }
    std::free(zo[i]);
  }
  if (!all_ok) { err = {AM_E_INFLATE, false, message_for(AM_E_INFLATE, 0, 0, "")}; return false; }
  out = make_chunk(in.data() + 4, 0, join_doc(parts));
  verified = true;
  return true;
}

// stage_doc over n documents with one GPU checksum batch and one inflate batch for every
// DEFLATEd column of every document (inflateColumn, columnar.js:1062-1068): out[i] is the staged
// chunk (the input itself when it has no compressed column), errs[i].code != 0 on failure.
void stage_docs(am_engine* e, size_t n, const uint8_t* const* data, const size_t* lens, std::vector<std::vector<uint8_t>>& out,
                std::vector<uint8_t>& verified, std::vector<Err>& errs) {
  HostClock clk;
  out.assign(n, {});
  verified.assign(n, 0);
  errs.assign(n, Err{});
  struct Zd {
    DocParts parts;
    uint64_t end = 0;
    bool z = false;
  };
  std::vector<Zd> zd(n);
  am_par_for(n, [&](size_t i) {
    const uint8_t* in = data[i];
    const size_t len = lens[i];
    Container c;
    Zd& z = zd[i];
    if (len < 4 || std::memcmp(in, "\x85\x6f\x4a\x83", 4) != 0 || !read_container(in, len, c) || c.type != 0 ||
        !split_doc(in + c.data_off, c.data_len, z.parts)) {
      out[i].assign(in, in + len);  // let the GPU report the exact error
      return;
    }
    for (auto* cols : {&z.parts.ccols, &z.parts.ocols})
      for (auto& col : *cols) z.z |= (col.id & COL_DEFLATE) != 0;
    if (!z.z) { out[i].assign(in, in + len); z.parts = DocParts{}; return; }
    z.end = c.end;
  });
  std::vector<size_t> zi;
  for (size_t i = 0; i < n; i++)
    if (zd[i].z) zi.push_back(i);
  if (zi.empty()) return;
  // checksums of the compressed chunks (one k_chunks-style SHA batch)
  std::vector<std::vector<uint8_t>> whole(zi.size());
  std::vector<const std::vector<uint8_t>*> wp(zi.size());
  for (size_t k = 0; k < zi.size(); k++) {
    whole[k].assign(data[zi[k]] + 8, data[zi[k]] + zd[zi[k]].end);
    wp[k] = &whole[k];
  }
  clk.mark("split");
  std::vector<std::array<uint8_t, 32>> hh;
  if (!gpu_sha256(e, wp, 0, hh)) {
    for (size_t i : zi) errs[i] = {AM_U_CAPACITY, false, "automerge_amd: GPU hash failed"};
    return;
  }
  clk.mark("sha");
  std::vector<std::vector<uint8_t>*> zcol;
  std::vector<uint64_t*> zid;
  std::vector<const uint8_t*> zb;
  std::vector<size_t> zl, zdoc;
  for (size_t k = 0; k < zi.size(); k++) {
    const size_t i = zi[k];
    if (std::memcmp(hh[k].data(), data[i] + 4, 4) != 0) {
      errs[i] = {AM_E_CHECKSUM, false, message_for(AM_E_CHECKSUM, 0, 0, "")};
      continue;
    }
    for (auto* cols : {&zd[i].parts.ccols, &zd[i].parts.ocols})
      for (auto& col : *cols)
        if (col.id & COL_DEFLATE) {
          zcol.push_back(&col.data);
          zid.push_back(&col.id);
          zb.push_back(col.data.data());
          zl.push_back(col.data.size());
          zdoc.push_back(i);
        }
  }
  const size_t nz = zb.size();
  std::vector<uint8_t*> zo(nz, nullptr);
  std::vector<size_t> zn(nz, 0);
  std::vector<uint8_t> zok(nz, 0);
  am_error ae;
  clk.mark("cols");
  if (nz && am_inflate_raw(e, zb.data(), zl.data(), nz, zo.data(), zn.data(), zok.data(), &ae)) {
    for (size_t i : zi)
      if (!errs[i].code) errs[i] = {AM_U_CAPACITY, false, ae.message};
    return;
  }
  for (size_t q = 0; q < nz; q++) {
    if (zok[q]) {
      zcol[q]->assign(zo[q], zo[q] + zn[q]);
      *zid[q] ^= COL_DEFLATE;
    } else if (!errs[zdoc[q]].code) {
      errs[zdoc[q]] = {AM_E_INFLATE, false, message_for(AM_E_INFLATE, 0, 0, "")};
    }
    std::free(zo[q]);
  }
  clk.mark("inflate");
  am_par_for(zi.size(), [&](size_t k) {
    const size_t i = zi[k];
    if (errs[i].code) return;
    out[i] = make_chunk(data[i] + 4, 0, join_doc(zd[i].parts));
    verified[i] = 1;
  });
  clk.mark("join");
  clk.print("stage_docs", n);
}

}  // namespace

bool am_stage_doc_chunk(am_engine* e, const std::vector<uint8_t>& in, std::vector<uint8_t>& out, bool& verified, am_error* err) {
  Err er;
  if (stage_doc(e, in, out, verified, er)) return true;
  to_c(er, err);
  return false;
}
void am_stage_doc_chunks(am_engine* e, size_t n, const uint8_t* const* data, const size_t* lens,
                         std::vector<std::vector<uint8_t>>& out, std::vector<uint8_t>& verified,
                         const std::function<am_error*(size_t)>& err_of) {
  std::vector<Err> E;
  stage_docs(e, n, data, lens, out, verified, E);
  for (size_t i = 0; i < n; i++)
    if (E[i].code) to_c(E[i], err_of(i));
}
std::string am_message_for(uint32_t code, int64_t a0, int64_t a1, const std::string& actor) { return message_for(code, a0, a1, actor); }

extern "C" am_doc* am_doc_init(am_engine* eng) {
  am_doc* d = new am_doc();
  d->eng = eng;
  return d;
}

extern "C" am_doc* am_doc_clone(const am_doc* s) { return new am_doc(*s); }
extern "C" void am_doc_free(am_doc* d) { delete d; }
extern "C" void am_free(void* p) { std::free(p); }

// Backend.load (backend/backend.js:104-107 -> new BackendDoc(buffer), new.js:1709-1750)
extern "C" am_doc* am_doc_load(am_engine* eng, const uint8_t* data, size_t len, am_error* err) {
  Err e;
  std::vector<uint8_t> in(data, data + len), staged, arena;
  bool verified = false;
  if (!stage_doc(eng, in, staged, verified, e)) { to_c(e, err); return nullptr; }
  OneResult res;
  if (!run_one(eng, &staged, verified, {}, {}, false, res, arena, e)) { to_c(e, err); return nullptr; }
  am_doc* d = new am_doc();
  d->eng = eng;
  d->state = std::move(res.out);
  d->binary = in;
  d->has_binary = true;
  d->have_hash_graph = false;
  d->heads = res.heads;
  d->load_heads = res.heads;
  d->nchanges = res.r.nchanges;
  // maxOp of a loaded document: the largest op counter in ids and succs (documentPatch,
  // new.js:1627-1630, 1749) -- reduced by k_doc over the base rows
  d->max_op = res.r.max_op;
  if (err) err->code = 0;
  return d;
}

// The error a patch log carries (getPatch or applyChanges: updatePatchProperty new.js:944,
// decodeValue columnar.js:318); false when the log is clean.
// actor id i of a wire-form log (its ACTOR records come first), hex
static std::string wire_actor(const std::vector<uint8_t>& log, int64_t want) {
  HRd r{log.data(), log.size(), sizeof(PatchHdr2)};
  for (int64_t i = 0; r.off < r.n && log[r.off] == PR_ACTOR; i++) {
    r.off++;
    const uint64_t l = r.u();
    const uint8_t* p = r.raw(l);
    if (!r.ok) break;
    if (i == want) return hexs(p, l);
  }
  return "?";
}

static bool patch_log_error(const std::vector<uint8_t>& log, Err& e) {
  PatchHdr2 h;
  if (log.size() < sizeof h) { e = Err{AM_U_CAPACITY, false, "automerge_amd: truncated patch log"}; return true; }
  std::memcpy(&h, log.data(), sizeof h);
  if (!h.status) return false;
  e = Err{h.status, false, ""};
  if (h.status == AM_E_FLOAT_LEN) {
    e.msg = fmt("Invalid length for floating point number: %lld", (long long)h.arg0);
  } else if (h.status == AM_E_UNKNOWN_COUNTER) {
    e.msg = fmt("increment operation %lld@%s for unknown counter", (long long)h.arg0, wire_actor(log, h.arg1).c_str());
  } else if (h.status == AM_U_INC_VALUE) {
    e.msg = am_message_for(AM_U_INC_VALUE, 0, 0, "");
  } else {
    e.msg = fmt("automerge_amd: the patch is not supported for this document (code %u)", h.status);
  }
  return true;
}

extern "C" int am_doc_compute_hash_graph(am_doc* d, am_error* err);

static int apply_finish(am_doc* d, std::vector<std::vector<uint8_t>>& orig, bool track, OneResult& res,
                        std::vector<uint8_t>* patch, am_error* err);

static int apply_changes(am_doc* d, const uint8_t* const* bufs, const size_t* lens, size_t n, std::vector<uint8_t>* patch,
                  am_error* err) {
  Err e;
  // decoded changes first, then the existing queue (new.js:1814)
  // compressed changes travel as they are: the batch stage inflates them on the GPU (am_inflate.hip)
  std::vector<std::vector<uint8_t>> orig;
  for (size_t i = 0; i < n; i++) orig.emplace_back(bufs[i], bufs[i] + lens[i]);
  for (auto& q : d->queue) orig.push_back(q);
  const std::vector<std::vector<uint8_t>>& staged = orig;
  // objectMeta moves on in every call, with or without a patch: loadChanges runs the same
  // BackendDoc.applyChanges (backend.js:116-121), whose updatePatchProperty calls refresh the
  // children snapshots and raise its errors. So every call replays the patch (P8) with the
  // handle's snapshots; loadChanges only drops the log.
  const bool track = true;
  const int pmode = 2;
  const std::vector<uint8_t>* meta = track ? &d->meta : nullptr;
  std::vector<am_known_hash> known;
  auto fill_known = [&]() {
    known.clear();
    if (!d->have_hash_graph) return;
    for (size_t i = 0; i < d->hashes.size(); i++) {
      am_known_hash k;
      std::memcpy(k.hash, d->hashes[i].data(), 32);
      k.index = (int64_t)i;
      known.push_back(k);
    }
  };
  HostClock clk;
  fill_known();
  OneResult res;
  std::vector<uint8_t> arena;
  clk.mark("prep");
  if (!run_one(d->eng, d->state.empty() ? nullptr : &d->state, true, staged, known, d->have_hash_graph, res, arena, e, pmode,
               0, meta)) {
    // a loaded document without its hash graph: compute it and run again (new.js:1826-1832)
    if (e.code != AM_U_HASH_GRAPH || d->have_hash_graph) { to_c(e, err); return 1; }
    if (am_doc_compute_hash_graph(d, err)) return 1;
    fill_known();
    e = Err{};
    if (!run_one(d->eng, &d->state, true, staged, known, true, res, arena, e, pmode, 0, meta)) {
      to_c(e, err);
      return 1;
    }
  }
  // a patch larger than the pools sized from the row counts: run again with 8x pools (the engine's
  // limit, not a reference error; the reference would return the patch)
  if (track && res.patch.size() >= sizeof(PatchHdr2)) {
    PatchHdr2 ph;
    std::memcpy(&ph, res.patch.data(), sizeof ph);
    if (ph.status == AM_U_CAPACITY && !run_one(d->eng, d->state.empty() ? nullptr : &d->state, true, staged, known,
                                               d->have_hash_graph, res, arena, e, 2, AM_DOC_PATCH_ROOM, meta)) {
      to_c(e, err);
      return 1;
    }
  }
  clk.mark("run_one");
  const int rc = apply_finish(d, orig, track, res, patch, err);
  clk.mark("finish");
  clk.print("apply_changes", d->state.size());
  return rc;
}

// The end of an applyChanges call whose GPU run succeeded: the patch's errors (an error in it throws
// before the document changes, new.js:1838; loadChanges throws the reference's errors too, and only
// loses objectMeta on an input the patch replay does not restate, AM_U_*), then the commit
// (new.js:1838-1860).
static int apply_finish(am_doc* d, std::vector<std::vector<uint8_t>>& orig, bool track, OneResult& res,
                        std::vector<uint8_t>* patch, am_error* err) {
  bool lost = false;
  if (track) {
    Err pe;
    if (patch_log_error(res.patch, pe)) {
      // loadChanges runs the same updatePatchProperty as applyChanges (backend.js:116-121), so what
      // the replay reports -- a reference error, or a shape it does not restate (the reference throws
      // there too, am_diff.h) -- fails the call either way and leaves the handle unchanged. Only the
      // engine's own pool limit lets a patchless call commit: its objectMeta is then resynchronised
      // to documentPatch's of the new state (as after save + load), never left unusable.
      if (patch || (pe.code != AM_U_CAPACITY && pe.code != AM_U_INC_VALUE)) { to_c(pe, err); return 1; }
      // AM_U_INC_VALUE: a non-integer counter increment, which the reference adds as JS does
      // (new.js:958); only the patch value depends on it, so a patchless call commits with the
      // snapshots the replay left
      lost = pe.code == AM_U_CAPACITY;
    }
    if (patch) patch->swap(res.patch);
  }
  // commit (new.js:1838-1860)
  const size_t base = d->state.empty() ? 0 : 1;
  std::vector<size_t> applied(res.r.napplied);
  std::vector<std::vector<uint8_t>> newq;
  std::vector<std::array<uint8_t, 32>> newqh;
  for (size_t i = 0; i < orig.size(); i++) {
    int32_t st = res.chg_state[base + i];
    if (st >= 0) applied[(size_t)st] = i;
    else if (st == CHG_QUEUED) { newq.push_back(orig[i]); newqh.push_back(res.hashes[base + i]); }
  }
  for (size_t k = 0; k < applied.size(); k++) {
    d->changes.push_back(std::move(orig[applied[k]]));
    d->hashes.push_back(res.hashes[base + applied[k]]);
  }
  d->queue = std::move(newq);
  d->queue_hashes = std::move(newqh);
  d->state = std::move(res.out);
  d->heads = res.heads;
  d->has_binary = false;
  d->binary.clear();
  d->nchanges = res.r.nchanges;
  if (res.r.max_op > d->max_op) d->max_op = res.r.max_op;
  if (track) {
    if (lost) d->meta.clear();  // documentPatch's snapshots of the new state
    else d->meta = std::move(res.meta);
  }
  if (err) err->code = 0;
  return 0;
}

// Backend.loadChanges (backend/backend.js:115-120): applyChanges without a patch
extern "C" int am_doc_apply_changes(am_doc* d, const uint8_t* const* bufs, const size_t* lens, size_t n, am_error* err) {
  return apply_changes(d, bufs, lens, n, nullptr, err);
}

// Backend.applyChanges (backend/backend.js:27-32 -> BackendDoc.applyChanges, new.js:1796-1871): the
// patch log of the call (k_doc phase P8, am_diff.h) in *out (malloc'd, am_free)
extern "C" int am_doc_apply_changes_patch(am_doc* d, const uint8_t* const* bufs, const size_t* lens, size_t n,
                                          uint8_t** out, size_t* len, am_error* err) {
  std::vector<uint8_t> log;
  if (apply_changes(d, bufs, lens, n, &log, err)) return 1;
  *out = static_cast<uint8_t*>(std::malloc(log.size() ? log.size() : 1));
  if (!*out) {
    to_c(Err{AM_U_CAPACITY, false, "automerge_amd: out of host memory"}, err);
    return 1;
  }
  std::memcpy(*out, log.data(), log.size());
  *len = log.size();
  return 0;
}

// save() bytes of a merged document chunk as k_doc writes it (columns uncompressed): DEFLATE of
// columns >= 256 bytes (deflateColumn, columnar.js:1052-1059, DEFLATE_MIN_SIZE :32) is the host
// stage; the container checksum of the compressed form is computed on the GPU.
// save_prepare: the bytes with the checksum still to fill in when *need_hash (the SHA-256 runs on
// the GPU, one launch for every document of a batched save).
static bool save_prepare(const std::vector<uint8_t>& state, std::vector<uint8_t>& bytes, bool& need_hash, Err& err) {
  need_hash = false;
  Container c;
  DocParts parts;
  if (!read_container(state.data(), state.size(), c) || !split_doc(state.data() + c.data_off, c.data_len, parts)) {
    err = {AM_U_VALUE, false, "automerge_amd: corrupt internal state"};
    return false;
  }
  bool any = false;
  for (auto* cols : {&parts.ccols, &parts.ocols})
    for (auto& col : *cols)
      if (col.data.size() >= 256) {
        std::vector<uint8_t> z;
        if (!zdeflate(col.data.data(), col.data.size(), z)) { err = {AM_U_VALUE, false, "deflate failed"}; return false; }
        col.data = std::move(z);
        col.id |= COL_DEFLATE;
        any = true;
      }
  if (!any) { bytes = state; return true; }
  std::vector<uint8_t> body = join_doc(parts);
  uint8_t zero[4] = {0, 0, 0, 0};
  bytes = make_chunk(zero, 0, body);
  need_hash = true;
  return true;
}

static bool save_bytes(am_engine* eng, const std::vector<uint8_t>& state, std::vector<uint8_t>& bytes, Err& err) {
  bool need = false;
  if (!save_prepare(state, bytes, need, err)) return false;
  if (!need) return true;
  std::vector<std::array<uint8_t, 32>> h;
  if (!gpu_sha256(eng, {&bytes}, 8, h)) { err = {AM_U_CAPACITY, false, "automerge_amd: GPU hash failed"}; return false; }
  std::memcpy(bytes.data() + 4, h[0].data(), 4);
  return true;
}

/* Backend.save() bytes of batch document `doc` (am_batch_doc_output + the DEFLATE stage). */
extern "C" int am_batch_doc_save(am_batch* b, uint32_t doc, uint8_t** out, size_t* len, am_error* err) {
  uint64_t n = 0;
  std::vector<uint8_t> raw;
  if (am_batch_doc_output(b, doc, nullptr, 0, &n) > 2) { to_c(Err{AM_U_CAPACITY, false, "automerge_amd: output copy failed"}, err); return 1; }
  raw.resize(n);
  if (n && am_batch_doc_output(b, doc, raw.data(), n, &n)) {
    to_c(Err{AM_U_CAPACITY, false, "automerge_amd: output copy failed"}, err);
    return 1;
  }
  if (!n) { to_c(Err{AM_U_VALUE, false, "automerge_amd: document has no output (failed status)"}, err); return 1; }
  std::vector<uint8_t> bytes;
  Err e;
  if (!save_bytes(b->eng, raw, bytes, e)) { to_c(e, err); return 1; }
  *out = (uint8_t*)std::malloc(bytes.size() ? bytes.size() : 1);
  if (!*out) { to_c(Err{AM_U_CAPACITY, false, "automerge_amd: out of host memory"}, err); return 1; }
  std::memcpy(*out, bytes.data(), bytes.size());
  *len = bytes.size();
  if (err) err->code = 0;
  return 0;
}

// Backend.save (new.js:2025-2047)
extern "C" int am_doc_save(am_doc* d, uint8_t** out, size_t* len, am_error* err) {
  std::vector<uint8_t> bytes;
  if (d->has_binary) {
    bytes = d->binary;
  } else if (d->state.empty()) {
    // Backend.init() saved: produce through the pipeline (no base, no changes)
    OneResult res;
    std::vector<uint8_t> arena;
    Err e;
    if (!run_one(d->eng, nullptr, false, {}, {}, true, res, arena, e)) { to_c(e, err); return 1; }
    bytes = res.out;
  } else {
    Err e;
    if (!save_bytes(d->eng, d->state, bytes, e)) { to_c(e, err); return 1; }
    d->binary = bytes;
    d->has_binary = true;
  }
  *out = (uint8_t*)std::malloc(bytes.size() ? bytes.size() : 1);
  if (!bytes.empty()) std::memcpy(*out, bytes.data(), bytes.size());
  *len = bytes.size();
  if (err) err->code = 0;
  return 0;
}

extern "C" size_t am_doc_get_heads(const am_doc* d, uint8_t* out32, size_t cap) {
  for (size_t i = 0; i < d->heads.size() && i < cap; i++) std::memcpy(out32 + 32 * i, d->heads[i].data(), 32);
  return d->heads.size();
}
extern "C" size_t am_doc_pending(const am_doc* d) { return d->queue.size(); }
extern "C" int64_t am_doc_max_op(const am_doc* d) { return d->max_op; }
extern "C" size_t am_doc_num_changes(const am_doc* d) { return d->nchanges; }
// computeHashGraph (new.js:1879-1904): the history decoded from the document (k_history, am_hist.hip)
extern "C" int am_doc_compute_hash_graph(am_doc* d, am_error* err) {
  if (err) err->code = 0;
  if (d->have_hash_graph) return 0;
  uint8_t *out = nullptr, *hs = nullptr;
  uint64_t* offs = nullptr;
  size_t n = 0;
  if (am_document_changes(d->eng, d->state.data(), d->state.size(), &out, &offs, &hs, &n, err)) return 1;
  d->changes.clear();
  d->hashes.clear();
  d->graph.clear();
  for (size_t i = 0; i < n; i++) {
    d->changes.emplace_back(out + offs[i], out + offs[i + 1]);
    std::array<uint8_t, 32> h;
    std::memcpy(h.data(), hs + 32 * i, 32);
    d->hashes.push_back(h);
  }
  std::free(out);
  std::free(offs);
  std::free(hs);
  d->have_hash_graph = true;
  return 0;
}

extern "C" int am_doc_change(const am_doc* d, size_t i, const uint8_t** data, size_t* len, uint8_t* hash32) {
  if (!d->have_hash_graph && am_doc_compute_hash_graph(const_cast<am_doc*>(d), nullptr)) return 2;
  if (i >= d->changes.size()) return 1;
  *data = d->changes[i].data();
  *len = d->changes[i].size();
  if (hash32) std::memcpy(hash32, d->hashes[i].data(), 32);
  return 0;
}

extern "C" int am_doc_get_patch(am_doc* d, uint8_t** out, size_t* len, am_error* err) {
  if (err) err->code = 0;
  std::vector<uint8_t> log;
  if (d->state.empty()) {  // Backend.init(): documentPatch of an empty document
    PatchHdr2 h{};
    h.magic = AM_PATCH_MAGIC;
    log.resize(sizeof h);
    std::memcpy(log.data(), &h, sizeof h);
  } else {
    OneResult res;
    std::vector<uint8_t> arena;
    Err e;
    if (!run_one(d->eng, &d->state, true, {}, {}, d->have_hash_graph, res, arena, e, true)) { to_c(e, err); return 1; }
    log.swap(res.patch);
  }
  Err pe;
  if (patch_log_error(log, pe)) {  // the RangeError getPatch throws (new.js:944, columnar.js:318)
    to_c(pe, err);
    return 1;
  }
  *out = static_cast<uint8_t*>(std::malloc(log.size()));
  if (!*out) {
    Err e{AM_U_CAPACITY, false, "automerge_amd: out of host memory"};
    to_c(e, err);
    return 1;
  }
  std::memcpy(*out, log.data(), log.size());
  *len = log.size();
  return 0;
}

// ---- the per-handle calls over many handles in one GPU batch ----
// Per call: codes[i] (0 = ok; bit 31 set when the reference throws a TypeError) and, when msgs is
// given, msgs[i] = the error text (malloc'd, am_free; nullptr for a call that succeeded).
static uint8_t* dup_bytes(const std::vector<uint8_t>& v) {
  uint8_t* p = static_cast<uint8_t*>(std::malloc(v.size() ? v.size() : 1));
  if (p && !v.empty()) std::memcpy(p, v.data(), v.size());
  return p;
}
static void call_info(const am_doc* d, am_call_info* info) {
  if (!info) return;
  info->max_op = d->max_op;
  info->pending = (uint32_t)d->queue.size();
  info->nheads = (uint32_t)d->heads.size();
  info->heads = static_cast<uint8_t*>(std::malloc(32 * (d->heads.size() ? d->heads.size() : 1)));
  if (info->heads)
    for (size_t k = 0; k < d->heads.size(); k++) std::memcpy(info->heads + 32 * k, d->heads[k].data(), 32);
}
static Err from_c(const am_error& e) { return Err{e.code, e.is_type_error != 0, e.message}; }
static int publish(const std::vector<Err>& E, uint32_t* codes, char** msgs) {
  int bad = 0;
  for (size_t i = 0; i < E.size(); i++) {
    codes[i] = E[i].code | (E[i].code && E[i].type_error ? 0x80000000u : 0u);
    if (msgs) {
      msgs[i] = nullptr;
      if (E[i].code) {
        msgs[i] = static_cast<char*>(std::malloc(E[i].msg.size() + 1));
        if (msgs[i]) std::memcpy(msgs[i], E[i].msg.c_str(), E[i].msg.size() + 1);
      }
    }
    bad += E[i].code != 0;
  }
  return bad;
}

// computeHashGraph (new.js:1879-1904) of the given loaded handles, k_history batches of 4096
static void hash_graphs(const std::vector<am_doc*>& ds, std::vector<Err>& E) {
  E.assign(ds.size(), Err{});
  const size_t G = 16384;  // am_history carries an am_error per document: bounded host memory (128 MiB)
  for (size_t g0 = 0; g0 < ds.size(); g0 += G) {
    const size_t g1 = std::min(ds.size(), g0 + G);
    std::vector<const uint8_t*> ptr;
    std::vector<size_t> len;
    for (size_t k = g0; k < g1; k++) { ptr.push_back(ds[k]->state.data()); len.push_back(ds[k]->state.size()); }
    std::vector<am_history> h(g1 - g0);
    am_document_changes_batch(ds[g0]->eng, ptr.data(), len.data(), g1 - g0, h.data());
    am_par_for(g1 - g0, [&](size_t kk) {  // each handle its own, on the host workers
      const size_t k = g0 + kk;
      am_doc* d = ds[k];
      am_history& x = h[k - g0];
      if (x.err.code) {
        E[k] = from_c(x.err);
      } else {
        d->changes.clear();
        d->hashes.clear();
        d->graph.clear();
        for (size_t i = 0; i < x.nchanges; i++) {
          d->changes.emplace_back(x.changes + x.offs[i], x.changes + x.offs[i + 1]);
          std::array<uint8_t, 32> hh;
          std::memcpy(hh.data(), x.hashes32 + 32 * i, 32);
          d->hashes.push_back(hh);
        }
        d->have_hash_graph = true;
      }
      std::free(x.changes);
      std::free(x.offs);
      std::free(x.hashes32);
    });
  }
}

static bool ensure_graph(am_doc* d, am_error* err);

// computeHashGraph of n handles (all of one engine): one k_history batch per 4096; then every
// handle's graph index is brought up to date on the host worker threads, so that the graph queries
// that follow (getChanges, getMissingDeps, getChangeByHash) only read it.
// A batch call that ran out of host memory (on the calling thread or a worker, am_par_for): every
// call of the batch reports it in its place instead of the process aborting
static int host_oom(size_t n, uint32_t* codes, char** msgs) {
  try {
    std::vector<Err> E(n, Err{AM_U_CAPACITY, false, "automerge_amd: out of host memory"});
    return publish(E, codes, msgs);
  } catch (const std::bad_alloc&) {
    for (size_t i = 0; i < n; i++) {
      codes[i] = AM_U_CAPACITY;
      msgs[i] = nullptr;
    }
    return (int)n;
  }
}

static int am_doc_compute_hash_graph_batch_impl(size_t n, am_doc* const* docs, uint32_t* codes, char** msgs) {
  std::vector<Err> E(n);
  std::vector<am_doc*> need;
  std::vector<size_t> at;
  std::unordered_set<am_doc*> seen;
  for (size_t i = 0; i < n; i++)
    if (!docs[i]->have_hash_graph && seen.insert(docs[i]).second) {
      if (docs[i]->eng != docs[0]->eng) {
        am_error tmp;
        if (am_doc_compute_hash_graph(docs[i], &tmp)) E[i] = from_c(tmp);
        continue;
      }
      need.push_back(docs[i]);
      at.push_back(i);
    }
  std::vector<Err> ge;
  hash_graphs(need, ge);
  for (size_t k = 0; k < at.size(); k++) E[at[k]] = ge[k];
  std::vector<am_doc*> idx;  // distinct handles whose graph exists
  std::unordered_set<am_doc*> seen2;
  for (size_t i = 0; i < n; i++)
    if (docs[i]->have_hash_graph && seen2.insert(docs[i]).second) idx.push_back(docs[i]);
  am_par_for(idx.size(), [&](size_t k) { (void)ensure_graph(idx[k], nullptr); });
  return publish(E, codes, msgs);
}
extern "C" int am_doc_compute_hash_graph_batch(size_t n, am_doc* const* docs, uint32_t* codes, char** msgs) {
  try {
    return am_doc_compute_hash_graph_batch_impl(n, docs, codes, msgs);
  } catch (const std::bad_alloc&) {
    return host_oom(n, codes, msgs);
  }
}

// Backend.load of n documents (backend.js:104-107) in one GPU batch: docs[i] = the handle, or
// nullptr with codes[i] / msgs[i] set. Returns the number that failed.
static int am_doc_load_batch_impl(am_engine* eng, size_t n, const uint8_t* const* data, const size_t* lens, am_doc** docs,
                                 uint32_t* codes, char** msgs) {
  std::vector<Err> E(n);
  std::vector<std::vector<uint8_t>> staged;
  std::vector<uint8_t> ver;
  stage_docs(eng, n, data, lens, staged, ver, E);
  std::vector<ManyJob> jobs;
  std::vector<size_t> at;
  for (size_t i = 0; i < n; i++) {
    docs[i] = nullptr;
    if (E[i].code) continue;
    ManyJob j;
    j.base = &staged[i];
    j.base_verified = ver[i] != 0;
    jobs.push_back(j);
    at.push_back(i);
  }
  std::vector<ManyOut> outs;
  Err e;
  if (!run_many(eng, jobs, outs, e)) {
    for (size_t i : at) E[i] = e;
    at.clear();
  }
  for (size_t k = 0; k < at.size(); k++) {
    const size_t i = at[k];
    if (!outs[k].ok) {
      if (outs[k].err.code == AM_U_UTF8) {  // room for the U+FFFD replacements: the single path
        am_error tmp;
        docs[i] = am_doc_load(eng, data[i], lens[i], &tmp);
        if (!docs[i]) E[i] = from_c(tmp);
      } else {
        E[i] = outs[k].err;
      }
      continue;
    }
    OneResult& res = outs[k].res;
    am_doc* d = new am_doc();
    d->eng = eng;
    d->state = std::move(res.out);
    d->binary.assign(data[i], data[i] + lens[i]);
    d->has_binary = true;
    d->have_hash_graph = false;
    d->heads = res.heads;
    d->load_heads = res.heads;
    d->nchanges = res.r.nchanges;
    d->max_op = res.r.max_op;
    docs[i] = d;
  }
  return publish(E, codes, msgs);
}
extern "C" int am_doc_load_batch(am_engine* eng, size_t n, const uint8_t* const* data, const size_t* lens, am_doc** docs,
                                 uint32_t* codes, char** msgs) {
  try {
    return am_doc_load_batch_impl(eng, n, data, lens, docs, codes, msgs);
  } catch (const std::bad_alloc&) {
    return host_oom(n, codes, msgs);
  }
}

// Backend.applyChanges / loadChanges (backend.js:27-32, 115-120) of n handles in one GPU batch:
// handle i gets the changes bufs[off[i] .. off[i+1]). patches != nullptr: applyChanges, patches[i]
// (malloc'd) / patch_lens[i] as am_doc_apply_changes_patch; otherwise loadChanges. A handle that
// appears more than once takes its later calls after the batch, in order; the handles whose call
// needs the hash graph (loaded documents, new.js:1826-1832) have it computed in one batch and run
// again. Returns the number of calls that failed (the handle unchanged).
static int am_doc_apply_changes_batch_impl(size_t n, am_doc* const* docs, const size_t* off, const uint8_t* const* bufs,
                                          const size_t* lens, uint8_t** patches, size_t* patch_lens, am_call_info* info,
                                          uint32_t* codes, char** msgs) {
  struct Call {
    size_t i;
    std::vector<std::vector<uint8_t>> orig;
    bool track;
    std::vector<am_known_hash> known;
  };
  std::vector<Err> E(n);
  std::vector<Call> calls;
  std::vector<size_t> single;  // calls taken one at a time after the batch, in call order
  std::unordered_set<am_doc*> seen;
  am_engine* eng = n ? docs[0]->eng : nullptr;
  auto known_of = [](am_doc* d, std::vector<am_known_hash>& known) {
    known.clear();
    if (!d->have_hash_graph) return;
    known.resize(d->hashes.size());
    for (size_t k = 0; k < d->hashes.size(); k++) {
      std::memcpy(known[k].hash, d->hashes[k].data(), 32);
      known[k].index = (int64_t)k;
    }
  };
  HostClock clk;
  for (size_t i = 0; i < n; i++) {
    if (patches) { patches[i] = nullptr; patch_lens[i] = 0; }
    if (info) info[i] = am_call_info{0, 0, 0, nullptr};
    am_doc* d = docs[i];
    const bool first = seen.insert(d).second;
    if (d->eng != eng || !first) { single.push_back(i); continue; }
    calls.emplace_back();
    calls.back().i = i;
  }
  am_par_for(calls.size(), [&](size_t k) {  // the calls' inputs, on the host workers (distinct handles)
    Call& c = calls[k];
    am_doc* d = docs[c.i];
    c.orig.reserve(off[c.i + 1] - off[c.i] + d->queue.size());
    for (size_t q = off[c.i]; q < off[c.i + 1]; q++) c.orig.emplace_back(bufs[q], bufs[q] + lens[q]);
    for (auto& q : d->queue) c.orig.push_back(q);
    c.track = true;
    known_of(d, c.known);
  });
  clk.mark("inputs");
  for (int round = 0; round < 2 && !calls.empty(); round++) {
    std::vector<ManyJob> jobs(calls.size());
    for (size_t k = 0; k < calls.size(); k++) {
      am_doc* d = docs[calls[k].i];
      ManyJob& j = jobs[k];
      j.base = d->state.empty() ? nullptr : &d->state;
      j.base_verified = true;  // the handle's state is the engine's own checksummed output
      j.chg = &calls[k].orig;
      j.known = &calls[k].known;
      j.have_graph = d->have_hash_graph;
      j.patch_mode = calls[k].track ? 2 : 0;
      j.meta = calls[k].track ? &d->meta : nullptr;
    }
    std::vector<ManyOut> outs;
    Err e;
    if (!run_many(eng, jobs, outs, e)) {
      for (auto& c : calls) E[c.i] = e;
      calls.clear();
      break;
    }
    clk.mark("run");
    std::vector<Call> graph;
    std::vector<uint8_t> commit(calls.size(), 0);
    for (size_t k = 0; k < calls.size(); k++) {
      Call& c = calls[k];
      am_doc* d = docs[c.i];
      ManyOut& o = outs[k];
      if (!o.ok) {
        if (o.err.code == AM_U_HASH_GRAPH && !d->have_hash_graph) graph.push_back(std::move(c));
        else if (o.err.code == AM_U_UTF8) single.push_back(c.i);
        else E[c.i] = o.err;
        continue;
      }
      if (c.track && o.res.patch.size() >= sizeof(PatchHdr2)) {
        PatchHdr2 ph;
        std::memcpy(&ph, o.res.patch.data(), sizeof ph);
        if (ph.status == AM_U_CAPACITY) { single.push_back(c.i); continue; }  // 8x pools: the single path
      }
      commit[k] = 1;
    }
    // the commits (new.js:1838-1860), each touching only its own handle, on the host workers
    am_par_for(calls.size(), [&](size_t k) {
      if (!commit[k]) return;
      Call& c = calls[k];
      am_doc* d = docs[c.i];
      std::vector<uint8_t> log;
      am_error tmp;
      if (apply_finish(d, c.orig, c.track, outs[k].res, patches ? &log : nullptr, &tmp)) {
        E[c.i] = from_c(tmp);
        return;
      }
      if (patches) {
        patches[c.i] = dup_bytes(log);
        patch_lens[c.i] = log.size();
      }
      call_info(d, info ? info + c.i : nullptr);
    });
    clk.mark("commit");
    am_reclaim(outs);
    if (graph.empty()) am_reclaim(calls);
    calls.clear();
    if (!graph.empty()) {
      std::vector<am_doc*> gd;
      for (auto& c : graph) gd.push_back(docs[c.i]);
      std::vector<Err> ge;
      hash_graphs(gd, ge);
      for (size_t k = 0; k < graph.size(); k++) {
        if (ge[k].code) { E[graph[k].i] = ge[k]; continue; }
        known_of(docs[graph[k].i], graph[k].known);
        calls.push_back(std::move(graph[k]));
      }
    }
  }
  for (auto& c : calls) single.push_back(c.i);
  std::sort(single.begin(), single.end());
  for (size_t i : single) {
    std::vector<uint8_t> log;
    am_error tmp;
    std::vector<const uint8_t*> b(bufs + off[i], bufs + off[i + 1]);
    std::vector<size_t> l(lens + off[i], lens + off[i + 1]);
    if (apply_changes(docs[i], b.data(), l.data(), b.size(), patches ? &log : nullptr, &tmp)) {
      E[i] = from_c(tmp);
      continue;
    }
    if (patches) {
      patches[i] = dup_bytes(log);
      patch_lens[i] = log.size();
    }
    call_info(docs[i], info ? info + i : nullptr);
  }
  clk.mark("single");
  clk.print("apply_changes_batch", n);
  return publish(E, codes, msgs);
}
extern "C" int am_doc_apply_changes_batch(size_t n, am_doc* const* docs, const size_t* off, const uint8_t* const* bufs,
                                          const size_t* lens, uint8_t** patches, size_t* patch_lens, am_call_info* info,
                                          uint32_t* codes, char** msgs) {
  try {
    return am_doc_apply_changes_batch_impl(n, docs, off, bufs, lens, patches, patch_lens, info, codes, msgs);
  } catch (const std::bad_alloc&) {
    return host_oom(n, codes, msgs);
  }
}

// Backend.getPatch (backend.js:125-127) of n handles in one GPU batch; out[i] malloc'd.
static int am_doc_get_patch_batch_impl(size_t n, am_doc* const* docs, uint8_t** out, size_t* lens, am_call_info* info,
                                      uint32_t* codes, char** msgs) {
  std::vector<Err> E(n);
  std::vector<ManyJob> jobs;
  std::vector<size_t> at, single;
  am_engine* eng = n ? docs[0]->eng : nullptr;
  for (size_t i = 0; i < n; i++) {
    out[i] = nullptr;
    lens[i] = 0;
    if (docs[i]->state.empty() || docs[i]->eng != eng) { single.push_back(i); continue; }
    ManyJob j;
    j.base = &docs[i]->state;
    j.base_verified = true;
    j.have_graph = docs[i]->have_hash_graph;
    j.patch_mode = 1;
    jobs.push_back(j);
    at.push_back(i);
  }
  std::vector<ManyOut> outs;
  Err e;
  if (!run_many(eng, jobs, outs, e)) {
    for (size_t i : at) E[i] = e;
    at.clear();
  }
  for (size_t k = 0; k < at.size(); k++) {
    const size_t i = at[k];
    if (!outs[k].ok) {
      if (outs[k].err.code == AM_U_UTF8) single.push_back(i);
      else E[i] = outs[k].err;
      continue;
    }
    if (patch_log_error(outs[k].res.patch, E[i])) continue;  // getPatch's RangeError (new.js:944)
    out[i] = dup_bytes(outs[k].res.patch);
    lens[i] = outs[k].res.patch.size();
  }
  for (size_t i : single) {
    am_error tmp;
    if (am_doc_get_patch(docs[i], out + i, lens + i, &tmp)) E[i] = from_c(tmp);
  }
  for (size_t i = 0; i < n && info; i++) {
    info[i] = am_call_info{0, 0, 0, nullptr};
    if (!E[i].code) call_info(docs[i], info + i);
  }
  return publish(E, codes, msgs);
}
extern "C" int am_doc_get_patch_batch(size_t n, am_doc* const* docs, uint8_t** out, size_t* lens, am_call_info* info,
                                      uint32_t* codes, char** msgs) {
  try {
    return am_doc_get_patch_batch_impl(n, docs, out, lens, info, codes, msgs);
  } catch (const std::bad_alloc&) {
    return host_oom(n, codes, msgs);
  }
}

// Backend.save (new.js:2025-2047) of n handles: the DEFLATE stage on the host, every checksum in one
// GPU SHA-256 launch; out[i] malloc'd.
static int am_doc_save_batch_impl(size_t n, am_doc* const* docs, uint8_t** out, size_t* lens, uint32_t* codes, char** msgs) {
  std::vector<Err> E(n);
  std::vector<std::vector<uint8_t>> bytes(n);
  std::vector<uint8_t> ready(n, 0);
  std::vector<const std::vector<uint8_t>*> hmsg;
  std::vector<size_t> hat;
  am_engine* eng = nullptr;
  for (size_t i = 0; i < n; i++) {
    out[i] = nullptr;
    lens[i] = 0;
    am_doc* d = docs[i];
    if (d->has_binary) { bytes[i] = d->binary; ready[i] = 1; continue; }
    if (d->state.empty() || (eng && d->eng != eng)) {
      am_error tmp;
      uint8_t* p = nullptr;
      size_t l = 0;
      if (am_doc_save(d, &p, &l, &tmp)) { E[i] = from_c(tmp); continue; }
      bytes[i].assign(p, p + l);
      std::free(p);
      ready[i] = 1;
      continue;
    }
    eng = d->eng;
    bool need = false;
    if (!save_prepare(d->state, bytes[i], need, E[i])) continue;
    if (need) { hmsg.push_back(&bytes[i]); hat.push_back(i); }
    else ready[i] = 1;
  }
  if (!hmsg.empty()) {
    std::vector<std::array<uint8_t, 32>> h;
    if (!gpu_sha256(eng, hmsg, 8, h)) {
      for (size_t i : hat) E[i] = Err{AM_U_CAPACITY, false, "automerge_amd: GPU hash failed"};
    } else {
      for (size_t k = 0; k < hat.size(); k++) { std::memcpy(bytes[hat[k]].data() + 4, h[k].data(), 4); ready[hat[k]] = 1; }
    }
  }
  for (size_t i = 0; i < n; i++) {
    if (!ready[i]) continue;
    am_doc* d = docs[i];
    if (!d->has_binary && !d->state.empty()) { d->binary = bytes[i]; d->has_binary = true; }
    out[i] = dup_bytes(bytes[i]);
    lens[i] = bytes[i].size();
  }
  return publish(E, codes, msgs);
}
extern "C" int am_doc_save_batch(size_t n, am_doc* const* docs, uint8_t** out, size_t* lens, uint32_t* codes, char** msgs) {
  try {
    return am_doc_save_batch_impl(n, docs, out, lens, codes, msgs);
  } catch (const std::bad_alloc&) {
    return host_oom(n, codes, msgs);
  }
}

extern "C" int am_doc_queued(const am_doc* d, size_t i, const uint8_t** data, size_t* len) {
  if (i >= d->queue.size()) return 1;
  *data = d->queue[i].data();
  *len = d->queue[i].size();
  return 0;
}

// ---- hash-graph queries of BackendDoc (new.js:1913-2020) over the graph kept with the document ----
static Hash32 h32(const uint8_t* p) {
  Hash32 h;
  std::memcpy(h.b, p, 32);
  return h;
}
// computeHashGraph on first use, then index the changes committed since
static bool ensure_graph(am_doc* d, am_error* err) {
  if (!d->have_hash_graph && am_doc_compute_hash_graph(d, err)) return false;
  for (size_t i = d->graph.size(); i < d->changes.size(); i++) {
    ChangeMeta m;
    if (!am_change_meta(d->changes[i].data(), d->changes[i].size(), m)) {
      to_c(Err{AM_U_VALUE, false, "automerge_amd: unreadable change header in the document history"}, err);
      return false;
    }
    d->graph.add(h32(d->hashes[i].data()), m);
  }
  if (err) err->code = 0;
  return true;
}
static std::vector<Hash32> heads_of(const am_doc* d) {
  std::vector<Hash32> h;
  for (auto& x : d->heads) h.push_back(h32(x.data()));
  return h;
}
static int out_indexes(const std::vector<size_t>& v, uint64_t** idx, size_t* n, am_error* err) {
  *n = v.size();
  *idx = static_cast<uint64_t*>(std::malloc(sizeof(uint64_t) * (v.size() ? v.size() : 1)));
  if (!*idx) { to_c(Err{AM_U_CAPACITY, false, "automerge_amd: out of host memory"}, err); return 1; }
  for (size_t i = 0; i < v.size(); i++) (*idx)[i] = v[i];
  if (err) err->code = 0;
  return 0;
}

extern "C" int am_doc_get_changes(am_doc* d, const uint8_t* have32, size_t nhave, uint64_t** idx, size_t* n, am_error* err) {
  if (!ensure_graph(d, err)) return 1;
  std::vector<Hash32> have;
  for (size_t i = 0; i < nhave; i++) have.push_back(h32(have32 + 32 * i));
  std::vector<size_t> out;
  Hash32 missing;
  if (!d->graph.changes_since(have, heads_of(d), out, missing)) {
    to_c(Err{AM_E_HISTORY, false, "hash not found: " + hexs(missing.b, 32)}, err);
    return 1;
  }
  return out_indexes(out, idx, n, err);
}

extern "C" int am_doc_get_changes_added(am_doc* d1, am_doc* d2, uint64_t** idx, size_t* n, am_error* err) {
  if (!ensure_graph(d2, err)) return 1;
  // d1's changeIndexByHash: every change once its graph exists, else the loaded heads and the
  // changes applied since the load (new.js:1729-1739, 1820-1822)
  std::function<bool(const Hash32&)> known;
  std::vector<Hash32> extra;
  if (d1->have_hash_graph) {
    if (!ensure_graph(d1, err)) return 1;
    known = [d1](const Hash32& h) { return d1->graph.find(h) >= 0; };
  } else {
    for (auto& x : d1->load_heads) extra.push_back(h32(x.data()));
    for (auto& x : d1->hashes) extra.push_back(h32(x.data()));
    known = [&extra](const Hash32& h) { return std::find(extra.begin(), extra.end(), h) != extra.end(); };
  }
  std::vector<size_t> out;
  d2->graph.added_since(known, heads_of(d2), out);
  return out_indexes(out, idx, n, err);
}

extern "C" int am_doc_graph_ready(const am_doc* d) { return d->have_hash_graph && d->graph.size() == d->changes.size(); }

extern "C" int64_t am_doc_change_index(am_doc* d, const uint8_t* hash32) {
  if (!ensure_graph(d, nullptr)) return -2;
  return d->graph.find(h32(hash32));
}

extern "C" int am_doc_get_missing_deps(am_doc* d, const uint8_t* heads32, size_t nheads, uint8_t** out32, size_t* n,
                                       am_error* err) {
  if (!ensure_graph(d, err)) return 1;
  std::vector<Hash32> all, inq;
  for (size_t i = 0; i < nheads; i++) all.push_back(h32(heads32 + 32 * i));
  for (size_t q = 0; q < d->queue.size(); q++) {
    inq.push_back(h32(d->queue_hashes[q].data()));
    ChangeMeta m;
    if (!am_change_meta(d->queue[q].data(), d->queue[q].size(), m)) {
      to_c(Err{AM_U_VALUE, false, "automerge_amd: unreadable queued change"}, err);
      return 1;
    }
    all.insert(all.end(), m.deps.begin(), m.deps.end());
  }
  std::vector<Hash32> missing;
  for (const Hash32& h : all)
    if (d->graph.find(h) < 0 && std::find(inq.begin(), inq.end(), h) == inq.end() &&
        std::find(missing.begin(), missing.end(), h) == missing.end())
      missing.push_back(h);
  std::sort(missing.begin(), missing.end());
  *n = missing.size();
  *out32 = static_cast<uint8_t*>(std::malloc(32 * (missing.size() ? missing.size() : 1)));
  if (!*out32) { to_c(Err{AM_U_CAPACITY, false, "automerge_amd: out of host memory"}, err); return 1; }
  for (size_t i = 0; i < missing.size(); i++) std::memcpy(*out32 + 32 * i, missing[i].b, 32);
  if (err) err->code = 0;
  return 0;
}

// clock[actor] (new.js:1857) and hashesByActor[actor][seq - 1] (new.js:1840-1841), read by
// applyLocalChange (backend.js:54-91); a loaded document computes its hash graph first
extern "C" int64_t am_doc_clock(am_doc* d, const char* actor_hex) {
  if (!ensure_graph(d, nullptr)) return -1;
  auto it = d->graph.clock.find(actor_hex);
  return it == d->graph.clock.end() ? 0 : it->second;
}
extern "C" int am_doc_actor_hash(am_doc* d, const char* actor_hex, int64_t seq, uint8_t* hash32) {
  if (!ensure_graph(d, nullptr)) return 2;
  auto it = d->graph.by_actor.find(actor_hex);
  if (it == d->graph.by_actor.end() || seq < 1 || (uint64_t)seq > it->second.size()) return 1;
  static const Hash32 zero{};
  const Hash32& h = it->second[(size_t)seq - 1];
  if (h == zero) return 1;  // a hole (the document misses that change)
  std::memcpy(hash32, h.b, 32);
  return 0;
}
extern "C" int am_doc_change_deps(am_doc* d, size_t i, const uint8_t** deps32, size_t* n) {
  if (!ensure_graph(d, nullptr) || i >= d->graph.meta.size()) return 1;
  const std::vector<Hash32>& v = d->graph.meta[i].deps;
  *deps32 = v.empty() ? nullptr : v[0].b;
  *n = v.size();
  return 0;
}
extern "C" am_engine* am_doc_engine(const am_doc* d) { return d->eng; }

extern "C" int am_change_hashes(am_engine* eng, const uint8_t* const* bufs, const size_t* lens, size_t n, uint8_t* out32,
                                am_error* err) {
  std::vector<std::vector<uint8_t>> staged(n);
  std::vector<const std::vector<uint8_t>*> ptrs;
  for (size_t i = 0; i < n; i++) {
    Err e;
    std::vector<uint8_t> in(bufs[i], bufs[i] + lens[i]);
    if (!stage_change(in, staged[i], e)) { to_c(e, err); return 1; }
    Container c;
    if (!read_container(staged[i].data(), staged[i].size(), c)) {
      to_c(Err{AM_E_SUBARRAY, false, message_for(AM_E_SUBARRAY, 0, 0, "")}, err);
      return 1;
    }
    staged[i].resize(c.end);
    ptrs.push_back(&staged[i]);
  }
  std::vector<std::array<uint8_t, 32>> h;
  if (!gpu_sha256(eng, ptrs, 8, h)) { to_c(Err{AM_U_CAPACITY, false, "automerge_amd: GPU hash failed"}, err); return 1; }
  for (size_t i = 0; i < n; i++) std::memcpy(out32 + 32 * i, h[i].data(), 32);
  if (err) err->code = 0;
  return 0;
}

// ---- host stage exposed for batch callers ----
extern "C" int am_stage_change(const uint8_t* in, size_t len, uint8_t** out, size_t* outlen, am_error* err) {
  Err e;
  std::vector<uint8_t> src(in, in + len), dst;
  if (!stage_change(src, dst, e)) { to_c(e, err); return 1; }
  *out = (uint8_t*)std::malloc(dst.size() ? dst.size() : 1);
  if (!dst.empty()) std::memcpy(*out, dst.data(), dst.size());
  *outlen = dst.size();
  if (err) err->code = 0;
  return 0;
}

// Host stage of Backend.load over n documents (am_stage_document batched): one GPU checksum batch
// and one GPU inflate batch for the DEFLATEd columns of all of them. outs[i] (malloc'd) = the staged
// chunk, verified[i] = 1 when its checksum was verified here; codes[i] / msgs[i] as in
// am_doc_load_batch. Returns the number that failed.
static int am_stage_documents_impl(am_engine* eng, size_t n, const uint8_t* const* data, const size_t* lens, uint8_t** outs,
                                  size_t* out_lens, uint8_t* verified, uint32_t* codes, char** msgs) {
  std::vector<std::vector<uint8_t>> st;
  std::vector<uint8_t> ver;
  std::vector<Err> E;
  stage_docs(eng, n, data, lens, st, ver, E);
  am_par_for(n, [&](size_t i) {
    outs[i] = nullptr;
    out_lens[i] = 0;
    verified[i] = ver[i];
    if (E[i].code) return;
    outs[i] = static_cast<uint8_t*>(std::malloc(st[i].size() ? st[i].size() : 1));
    std::memcpy(outs[i], st[i].data(), st[i].size());
    out_lens[i] = st[i].size();
  });
  return publish(E, codes, msgs);
}
extern "C" int am_stage_documents(am_engine* eng, size_t n, const uint8_t* const* data, const size_t* lens, uint8_t** outs,
                                  size_t* out_lens, uint8_t* verified, uint32_t* codes, char** msgs) {
  try {
    return am_stage_documents_impl(eng, n, data, lens, outs, out_lens, verified, codes, msgs);
  } catch (const std::bad_alloc&) {
    return host_oom(n, codes, msgs);
  }
}
extern "C" int am_stage_document(am_engine* eng, const uint8_t* in, size_t len, uint8_t** out, size_t* outlen,
                                 int* verified, am_error* err) {
  Err e;
  std::vector<uint8_t> src(in, in + len), dst;
  bool v = false;
  if (!stage_doc(eng, src, dst, v, e)) { to_c(e, err); return 1; }
  *out = (uint8_t*)std::malloc(dst.size() ? dst.size() : 1);
  if (!dst.empty()) std::memcpy(*out, dst.data(), dst.size());
  *outlen = dst.size();
  *verified = v ? 1 : 0;
  if (err) err->code = 0;
  return 0;
}
