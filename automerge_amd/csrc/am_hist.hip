// am_hist.hip -- the change history of saved documents, batched on the GPU:
// BackendDoc.computeHashGraph (new.js:1879-1904) = decodeChanges([doc]) (columnar.js:1040-1046,
// groupChangeOps :876-943, decodeDocumentChanges :945-981) with every change re-encoded by
// encodeChange (:710-739) and DEFLATEd when >= 256 bytes (deflateChange :798-808).
//
// Host stage around k_history (am_hist_dev.h): stage every document as Backend.load does (DEFLATEd
// columns inflated on the GPU, am_stage_doc_chunk), one arena, k_chunks (container, checksum,
// counts) -> the per-document workspace and output layout from the counts -> k_history (one
// workgroup per document) -> results, change records and change chunks back to the host, which
// deflates the large changes (zlib, as the save path does) and formats the reference's error text.
// A document whose change chunks outgrow the first guess of their size is run again with the
// exact size the kernel reports.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/automerge_amd.h"
#include "am_change_enc.h"
#include "am_launch.h"
#include "am_par.h"

namespace {

template <typename T>
struct DevArr {
  T* p = nullptr;
  size_t cap = 0;
  bool ensure(size_t n) {
    if (n <= cap && p) return true;
    if (p) { (void)hipFree(p); p = nullptr; cap = 0; }
    const size_t want = n + n / 4 + 64;  // headroom: batches of similar sizes reuse the buffer
    if (hipMalloc(&p, want * sizeof(T)) != hipSuccess) { p = nullptr; return false; }
    cap = want;
    return true;
  }
  ~DevArr() { if (p) (void)hipFree(p); }
};

std::string hexstr(const uint8_t* p, size_t n) {
  static const char* H = "0123456789abcdef";
  std::string s;
  s.reserve(2 * n);
  for (size_t i = 0; i < n; i++) { s += H[p[i] >> 4]; s += H[p[i] & 15]; }
  return s;
}

// actor ids and heads of a document chunk (decodeDocumentHeader, columnar.js:1006-1021), for the
// error text only (the kernel has validated the header when it reports a history error)
struct HdrText { std::vector<std::string> actors, heads; };
HdrText header_text(const uint8_t* d, size_t n) {
  HdrText h;
  size_t o = 9;
  auto u = [&](uint64_t& v) {
    v = 0;
    for (int sh = 0; o < n && sh < 64; sh += 7) {
      const uint8_t c = d[o++];
      v |= (uint64_t)(c & 0x7f) << sh;
      if (!(c & 0x80)) return true;
    }
    return false;
  };
  uint64_t len, na, nh;
  if (!u(len) || !u(na)) return h;
  for (uint64_t i = 0; i < na; i++) {
    uint64_t l;
    if (!u(l) || l > n - o) return h;
    h.actors.push_back(hexstr(d + o, l));
    o += l;
  }
  if (!u(nh)) return h;
  for (uint64_t i = 0; i < nh && o + 32 <= n; i++, o += 32) h.heads.push_back(hexstr(d + o, 32));
  return h;
}

struct DocRun {
  HistResult r{};
  std::vector<HistChange> ch;  // off = offset in `bytes`
  const uint8_t* bytes = nullptr;
  uint64_t cap = 0;            // the change-chunk region the kernel had
};

// device buffers kept by the engine between history batches (grown on demand)
struct HistCache {
  DevArr<uint8_t> arena, ws, out, dense;
  DevArr<am_chunk_desc> chunks;
  DevArr<ChunkInfo> info;
  DevArr<HdrSlot> hdr;
  DevArr<HistDesc> hd;
  DevArr<HistResult> res;
  DevArr<HistChange> chg;
  DevArr<uint32_t> nchg;
  DevArr<uint64_t> sizes, doff, scan_tmp;
  std::vector<uint8_t> host;   // dense change bytes of the last batch
};

#define HCHECK(expr)                                                                       \
  do {                                                                                     \
    if ((expr) != hipSuccess) { why = std::string("automerge_amd: ") + #expr + " failed"; return false; } \
  } while (0)
#define HALLOC(buf, n)                                                                     \
  do {                                                                                     \
    if (!(buf).ensure(n)) { why = "automerge_amd: device memory for the history batch"; return false; } \
  } while (0)

// A document chunk whose columns are stored as they are (no DEFLATEd column) goes to the GPU
// unchanged; false also for anything the header walk cannot read (Backend.load's staging reports it)
bool plain_columns(const uint8_t* p, size_t n) {
  size_t o = 9;
  auto u = [&](uint64_t& v) {
    v = 0;
    for (int sh = 0; o < n && sh < 64; sh += 7) {
      const uint8_t c = p[o++];
      v |= (uint64_t)(c & 0x7f) << sh;
      if (!(c & 0x80)) return true;
    }
    return false;
  };
  uint64_t len, na, nh, nc, id, cl;
  if (n < 10 || p[8] != 0 || !u(len) || !u(na)) return false;
  for (uint64_t i = 0; i < na; i++) {
    if (!u(cl) || cl > n - o) return false;
    o += cl;
  }
  if (!u(nh) || nh > (n - o) / 32) return false;
  o += 32 * nh;
  for (int part = 0; part < 2; part++) {
    if (!u(nc)) return false;
    for (uint64_t i = 0; i < nc; i++) {
      if (!u(id) || !u(cl)) return false;
      if (id & 8) return false;
    }
  }
  return true;
}

// k_chunks + k_history (+ the dense copy of the change chunks) over `docs` (staged chunks);
// caps[i] = change-chunk bytes (0: the guess)
bool run_history(am_engine* e, const std::vector<std::pair<const uint8_t*, size_t>>& docs, const std::vector<uint8_t>& verified,
                 const std::vector<uint64_t>& caps, std::vector<DocRun>& runs, std::string& why) {
  const uint32_t n = (uint32_t)docs.size();
  runs.assign(n, DocRun());
  if (!n) return true;
  HCHECK(hipSetDevice(am_engine_device(e)));
  hipStream_t s = am_engine_stream(e);
  void*& slot = am_engine_hist(e);
  if (!slot) slot = new HistCache();
  HistCache& K = *static_cast<HistCache*>(slot);
  std::vector<am_chunk_desc> cds(n);
  uint64_t asz = 0;
  for (uint32_t i = 0; i < n; i++) {
    cds[i] = {asz, (uint32_t)docs[i].second, verified[i] ? 1u : 0u};
    asz = (asz + docs[i].second + 15) & ~(uint64_t)15;
  }
  std::vector<uint8_t> arena(asz);
  for (uint32_t i = 0; i < n; i++) std::memcpy(arena.data() + cds[i].off, docs[i].first, docs[i].second);
  HALLOC(K.arena, asz + 16);
  HALLOC(K.chunks, n);
  HALLOC(K.info, n);
  HALLOC(K.hdr, n);
  HCHECK(hipMemcpyAsync(K.arena.p, arena.data(), asz, hipMemcpyHostToDevice, s));
  HCHECK(hipMemcpyAsync(K.chunks.p, cds.data(), sizeof(am_chunk_desc) * n, hipMemcpyHostToDevice, s));
  BatchDev bd{};
  bd.arena = K.arena.p;
  bd.chunks = K.chunks.p;
  bd.info = K.info.p;
  bd.hdr = K.hdr.p;
  bd.nchunks = n;
  am_launch_chunks(bd, s);
  std::vector<ChunkInfo> info(n);
  HCHECK(hipMemcpyAsync(info.data(), K.info.p, sizeof(ChunkInfo) * n, hipMemcpyDeviceToHost, s));
  HCHECK(hipStreamSynchronize(s));
  // layout: workspace, change-chunk regions and change records per document
  std::vector<HistDesc> hd;
  std::vector<uint32_t> which, nchg;  // hd index -> document, its change count
  uint64_t ws_tot = 0, out_tot = 0, chg_tot = 0;
  const uint64_t kDocLimit = 32ull << 30;  // one document's workspace + output
  for (uint32_t i = 0; i < n; i++) {
    const ChunkInfo& ci = info[i];
    const bool ok = ci.status == 0 && ci.type == 0;
    const HistLayout L = hist_layout(ok ? ci.nops : 0, ok ? ci.nents : 0, ok ? ci.nchg : 0, ok ? ci.ndeps : 0, ok ? ci.nactors : 0);
    const uint64_t cap = !ok ? 0 : caps[i] ? caps[i] : hist_out_guess(ci.nops, ci.nents, ci.nchg, ci.ndeps, cds[i].len);
    if (L.total + cap > kDocLimit) {
      runs[i].r.status = HE_CODE;
      runs[i].r.a0 = AM_U_CAPACITY;
      continue;
    }
    HistDesc h{};
    h.chunk = i;
    h.ws_off = ws_tot;
    h.out_off = out_tot;
    h.out_cap = cap;
    h.chg_off = chg_tot;
    ws_tot += (L.total + 255) & ~(uint64_t)255;
    out_tot += (cap + 255) & ~(uint64_t)255;
    chg_tot += ok ? ci.nchg : 0;
    runs[i].cap = cap;
    hd.push_back(h);
    which.push_back(i);
    nchg.push_back(ok ? ci.nchg : 0);
  }
  const uint32_t nd = (uint32_t)hd.size();
  if (!nd) return true;
  HALLOC(K.ws, ws_tot);
  HALLOC(K.out, out_tot + 16);
  HALLOC(K.hd, nd);
  HALLOC(K.res, nd);
  HALLOC(K.chg, chg_tot);
  HALLOC(K.nchg, nd);
  HALLOC(K.sizes, nd);
  HALLOC(K.doff, nd + 1);
  HALLOC(K.scan_tmp, am_scan_tmp_elems(nd));
  HCHECK(hipMemcpyAsync(K.hd.p, hd.data(), sizeof(HistDesc) * nd, hipMemcpyHostToDevice, s));
  HCHECK(hipMemcpyAsync(K.nchg.p, nchg.data(), sizeof(uint32_t) * nd, hipMemcpyHostToDevice, s));
  am_launch_history(K.arena.p, K.chunks.p, K.info.p, K.hd.p, nd, K.ws.p, K.out.p, K.res.p, K.chg.p, s);
  HCHECK(hipGetLastError());
  // the change chunks of the documents that succeeded, back to back (k_history_sizes rewrites the
  // records' offsets: dense offset in the low word)
  am_launch_history_sizes(K.res.p, K.hd.p, nd, K.nchg.p, K.chg.p, K.sizes.p, s);
  am_launch_scan(K.sizes.p, K.doff.p, K.scan_tmp.p, nd, K.doff.p + nd, s);
  std::vector<HistResult> res(nd);
  std::vector<HistChange> chs(chg_tot);
  std::vector<uint64_t> doff(nd + 1);
  HCHECK(hipMemcpyAsync(res.data(), K.res.p, sizeof(HistResult) * nd, hipMemcpyDeviceToHost, s));
  if (chg_tot) HCHECK(hipMemcpyAsync(chs.data(), K.chg.p, sizeof(HistChange) * chg_tot, hipMemcpyDeviceToHost, s));
  HCHECK(hipMemcpyAsync(doff.data(), K.doff.p, sizeof(uint64_t) * (nd + 1), hipMemcpyDeviceToHost, s));
  HCHECK(hipStreamSynchronize(s));
  const uint64_t dense = doff[nd];
  HALLOC(K.dense, dense);
  am_launch_history_compact(K.res.p, K.hd.p, nd, K.nchg.p, K.chg.p, K.doff.p, K.out.p, K.dense.p, s);
  K.host.resize(dense);
  if (dense) HCHECK(hipMemcpyAsync(K.host.data(), K.dense.p, dense, hipMemcpyDeviceToHost, s));
  HCHECK(hipStreamSynchronize(s));
  for (uint32_t k = 0; k < nd; k++) {
    DocRun& r = runs[which[k]];
    r.r = res[k];
    if (r.r.status == HE_OK || r.r.status == HE_HEADS) {
      r.ch.assign(chs.begin() + hd[k].chg_off, chs.begin() + hd[k].chg_off + nchg[k]);
      if (r.r.status == HE_OK)
        for (HistChange& c : r.ch) c.off = (uint32_t)c.off;
      r.bytes = K.host.data() + doff[k];
    }
  }
  return true;
}

std::string history_message(const DocRun& r, const uint8_t* doc, size_t len, uint32_t& code) {
  code = AM_E_HISTORY;
  const HistResult& x = r.r;
  auto actor = [&](int64_t a) {
    const HdrText h = header_text(doc, len);
    return a >= 0 && (size_t)a < h.actors.size() ? h.actors[a] : std::string("undefined");
  };
  char buf[256];
  switch (x.status) {
    case HE_SEQ:
      std::snprintf(buf, sizeof buf, "Expected seq = %lld, got %lld", (long long)x.a0, (long long)x.a1);
      return buf;
    case HE_MAXOP: return "maxOp must increase monotonically per actor";
    case HE_RANGE: return "Operation ID " + std::to_string(x.a0) + "@" + actor(x.a1) + " outside of allowed range";
    case HE_OPID:
      return "Expected opId " + std::to_string(x.a0) + "@" + actor(x.a1) + ", got " + std::to_string(x.a2) + "@" + actor(x.a3);
    case HE_NOHASH:
      return "No hash for index " + (x.a0 == AM_NULL64 ? std::string("null") : std::to_string(x.a0)) + " while processing index " +
             std::to_string(x.a1);
    case HE_EXTRA: return "Bad datatype for extra bytes: 7";
    case HE_DEL: return "document should not contain del operations";
    case HE_HEADS: {
      const HdrText h = header_text(doc, len);
      std::vector<std::string> got;
      for (auto& c : r.ch) if (c.head) got.push_back(hexstr(c.hash, 32));
      std::sort(got.begin(), got.end());
      std::string a, b;
      for (size_t i = 0; i < h.heads.size(); i++) a += (i ? ", " : "") + h.heads[i];
      for (size_t i = 0; i < got.size(); i++) b += (i ? ", " : "") + got[i];
      return "Mismatched heads hashes: expected " + a + ", got " + b;
    }
    default:
      code = (uint32_t)x.a0;
      return am_message_for(code, x.a1, 0, "");
  }
}

void set_err(am_error* e, uint32_t code, const std::string& m) {
  e->code = code;
  e->is_type_error = 0;
  std::snprintf(e->message, sizeof(e->message), "%s", m.c_str());
}

}  // namespace

void am_hist_cache_free(void* cache) { delete static_cast<HistCache*>(cache); }

extern "C" int am_document_changes_batch(am_engine* eng, const uint8_t* const* docs, const size_t* lens, size_t n, am_history* out) {
  for (size_t i = 0; i < n; i++) { std::memset(&out[i], 0, sizeof(am_history)); }
  // Backend.load's staging of every document: chunks with DEFLATEd columns are inflated (and their
  // checksum verified) first, the others go to the GPU as they are
  std::vector<std::vector<uint8_t>> staged(n);
  std::vector<std::pair<const uint8_t*, size_t>> src(n);
  std::vector<uint8_t> verified(n, 0);
  std::vector<uint32_t> live;
  // documents with DEFLATEd columns: one batched stage (GPU checksums + one inflate batch)
  std::vector<size_t> zi;
  std::vector<const uint8_t*> zp;
  std::vector<size_t> zl;
  std::vector<uint8_t> zbad(n, 0);
  for (size_t i = 0; i < n; i++)
    if (!plain_columns(docs[i], lens[i])) { zi.push_back(i); zp.push_back(docs[i]); zl.push_back(lens[i]); }
  if (!zi.empty()) {
    std::vector<std::vector<uint8_t>> zs;
    std::vector<uint8_t> zv;
    am_stage_doc_chunks(eng, zi.size(), zp.data(), zl.data(), zs, zv, [&](size_t k) {
      zbad[zi[k]] = 1;
      return &out[zi[k]].err;
    });
    for (size_t k = 0; k < zi.size(); k++) {
      staged[zi[k]] = std::move(zs[k]);
      verified[zi[k]] = zv[k];
    }
  }
  for (size_t i = 0; i < n; i++) {
    if (zbad[i]) continue;
    if (plain_columns(docs[i], lens[i])) src[i] = {docs[i], lens[i]};
    else src[i] = {staged[i].data(), staged[i].size()};
    live.push_back((uint32_t)i);
  }
  std::vector<DocRun> runs(n);
  std::vector<std::vector<uint8_t>> keep;  // the first pass's change bytes when a second pass runs
  std::string why;
  for (int pass = 0; pass < 2 && !live.empty(); pass++) {
    std::vector<std::pair<const uint8_t*, size_t>> ds;
    std::vector<uint8_t> vs;
    std::vector<uint64_t> caps;
    for (uint32_t i : live) {
      ds.push_back(src[i]);
      vs.push_back(verified[i]);
      caps.push_back(pass ? (uint64_t)runs[i].r.a1 : 0);
    }
    std::vector<DocRun> rr;
    if (!run_history(eng, ds, vs, caps, rr, why)) {
      for (uint32_t i : live) set_err(&out[i].err, AM_U_CAPACITY, why);
      return 1;
    }
    std::vector<uint32_t> again;
    for (size_t k = 0; k < live.size(); k++) {
      const uint32_t i = live[k];
      runs[i] = std::move(rr[k]);
      // change chunks larger than the first guess: once more with the size the kernel reported
      if (!pass && runs[i].r.status == HE_CODE && runs[i].r.a0 == AM_U_CAPACITY && (uint64_t)runs[i].r.a1 > runs[i].cap)
        again.push_back(i);
    }
    if (!pass && !again.empty()) {  // the cache's host buffer is reused by the second pass
      HistCache& K = *static_cast<HistCache*>(am_engine_hist(eng));
      keep.emplace_back(K.host);
      for (size_t i = 0; i < n; i++)
        if (runs[i].bytes) runs[i].bytes = keep.back().data() + (runs[i].bytes - K.host.data());
    }
    live.swap(again);
  }
  // per document on the host workers: each writes only its own out[i] (the change re-encode and
  // DEFLATE of large changes are the bulk of it)
  std::atomic<int> rc_any{0};
  am_par_for(n, [&](size_t i) {
    int rc = 0;
    struct Flag { std::atomic<int>& a; int& v; ~Flag() { if (v) a.store(1, std::memory_order_relaxed); } } flag{rc_any, rc};
    if (out[i].err.code) { rc = 1; return; }
    const DocRun& r = runs[i];
    if (r.r.status != HE_OK) {
      uint32_t code;
      const std::string m = history_message(r, src[i].first, src[i].second, code);
      set_err(&out[i].err, code ? code : AM_U_VALUE, m);
      rc = 1;
      return;
    }
    std::vector<Bytes> chs;
    size_t total = 0;
    for (const HistChange& c : r.ch) {
      chs.push_back(deflate_change(Bytes(r.bytes + c.off, r.bytes + c.off + c.len)));
      total += chs.back().size();
    }
    if (out[i].err.code) { rc = 1; return; }
    out[i].changes = (uint8_t*)std::malloc(total ? total : 1);
    out[i].offs = (uint64_t*)std::malloc(sizeof(uint64_t) * (chs.size() + 1));
    out[i].hashes32 = (uint8_t*)std::malloc(32 * (chs.size() ? chs.size() : 1));
    if (!out[i].changes || !out[i].offs || !out[i].hashes32) {
      std::free(out[i].changes); std::free(out[i].offs); std::free(out[i].hashes32);
      out[i].changes = nullptr; out[i].offs = nullptr; out[i].hashes32 = nullptr;
      set_err(&out[i].err, AM_U_CAPACITY, "automerge_amd: out of host memory");
      rc = 1;
      return;
    }
    size_t o = 0;
    for (size_t k = 0; k < chs.size(); k++) {
      out[i].offs[k] = o;
      if (!chs[k].empty()) std::memcpy(out[i].changes + o, chs[k].data(), chs[k].size());
      o += chs[k].size();
      std::memcpy(out[i].hashes32 + 32 * k, r.ch[k].hash, 32);
    }
    out[i].offs[chs.size()] = o;
    out[i].nchanges = chs.size();
  });
  return rc_any.load();
}

extern "C" int am_document_changes(am_engine* eng, const uint8_t* doc, size_t len, uint8_t** out, uint64_t** offs, uint8_t** hashes32,
                                   size_t* nchanges, am_error* err) {
  am_history h;
  const uint8_t* d[1] = {doc};
  const size_t l[1] = {len};
  const int rc = am_document_changes_batch(eng, d, l, 1, &h);
  if (rc || h.err.code) {
    if (err) *err = h.err;
    return 1;
  }
  *out = h.changes;
  *offs = h.offs;
  *hashes32 = h.hashes32;
  *nchanges = h.nchanges;
  if (err) err->code = 0;
  return 0;
}
