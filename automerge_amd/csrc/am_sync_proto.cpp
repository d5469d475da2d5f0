// am_sync_proto.cpp -- the sync protocol of backend/sync.js over engine documents (SURVEY.md §8
// a24/a25, C5). Host code; the Bloom filters and the change selection run in the HIP kernels of
// am_sync.hip (k_bloom_build, k_sync_select), batched over every document of a call.
//
//   am_sync_generate        <- generateSyncMessage   sync.js:327-400 (+ makeBloomFilter :234-238,
//                                                     getChangesToSend :246-306)
//   am_sync_receive         <- receiveSyncMessage    sync.js:420-474 (+ advanceHeads :408-413)
//   am_sync_encode_message  <- encodeSyncMessage     sync.js:157-171 (encodeHashes :130-139)
//   am_sync_decode_messages <- decodeSyncMessage     sync.js:177-199 (decodeHashes :145-151)
//   am_sync_encode_state    <- encodeSyncState       sync.js:206-211
//   am_sync_decode_state    <- decodeSyncState       sync.js:217-225
//
// The document side goes through the engine's own hash-graph queries (am_doc_get_changes,
// am_doc_get_missing_deps, am_doc_change_index) exactly where the reference calls Backend.*.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <map>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "../../include/automerge_amd.h"
#include "am_graph.h"
#include "am_json.h"
#include "am_par.h"

namespace {

using Hashes = std::vector<Hash32>;

struct SErr {
  bool type_error;
  std::string msg;
  uint32_t code = AM_E_LOCAL;
};
[[noreturn]] void range_error(const std::string& m, uint32_t code = AM_E_LOCAL) { throw SErr{false, m, code}; }
[[noreturn]] void type_error(const std::string& m) { throw SErr{true, m}; }

void to_err(const SErr& e, am_error* err) {
  if (!err) return;
  err->code = e.code;
  err->is_type_error = e.type_error ? 1 : 0;
  snprintf(err->message, sizeof(err->message), "%s", e.msg.c_str());
}
void from_am(const am_error& e) { throw SErr{e.is_type_error != 0, e.message, e.code}; }

// ---- Encoder / Decoder primitives (encoding.js) ----
void pu(std::vector<uint8_t>& o, uint64_t v) {
  do {
    uint8_t b = v & 0x7f;
    v >>= 7;
    o.push_back(b | (v ? 0x80 : 0));
  } while (v);
}

struct Dec {
  const uint8_t* p;
  size_t n, off = 0;
  int byte() {  // readByte: past the end reads `undefined`
    if (off >= n) { off++; return -1; }
    return p[off++];
  }
  uint32_t u32() {  // readUint32 (encoding.js:341-354)
    uint32_t r = 0;
    int shift = 0;
    while (off < n) {
      const uint8_t b = p[off];
      if (shift == 28 && (b & 0xf0)) range_error("number out of range", AM_E_LEB_RANGE);
      r |= (uint32_t)(b & 0x7f) << shift;
      shift += 7;
      off++;
      if (!(b & 0x80)) return r;
    }
    range_error("buffer ended with incomplete number", AM_E_LEB_INCOMPLETE);
  }
  uint64_t u53() {  // readUint53 over readUint64 (encoding.js:387-441)
    uint64_t r = 0;
    int shift = 0;
    while (off < n) {
      const uint8_t b = p[off];
      if (shift == 63 && (b & 0xfe)) range_error("number out of range", AM_E_LEB_RANGE);
      r |= (uint64_t)(b & 0x7f) << shift;
      shift += 7;
      off++;
      if (!(b & 0x80)) {
        if (r > 9007199254740991ull) range_error("number out of range", AM_E_LEB_RANGE);
        return r;
      }
    }
    range_error("buffer ended with incomplete number", AM_E_LEB_INCOMPLETE);
  }
  uint64_t raw(uint64_t k) {  // readRawBytes: offset of the bytes
    if (off > n || k > n - off) range_error("subarray exceeds buffer size", AM_E_SUBARRAY);
    const uint64_t o = off;
    off += k;
    return o;
  }
};

// ---- hashes ----
bool contains(const Hashes& v, const Hash32& h) { return std::find(v.begin(), v.end(), h) != v.end(); }
// encodeHashes (sync.js:130-139) of hashes already in binary form
void put_hashes(std::vector<uint8_t>& o, const Hashes& hs) {
  for (size_t i = 1; i < hs.size(); i++)
    if (!(hs[i - 1] < hs[i])) range_error("hashes must be sorted");
  pu(o, hs.size());
  for (const Hash32& h : hs) o.insert(o.end(), h.b, h.b + 32);
}
// decodeHashes (sync.js:145-151): offset of `count` contiguous hashes
Hashes get_hashes(Dec& d, uint64_t* off = nullptr, uint64_t* count = nullptr) {
  const uint32_t n = d.u32();
  Hashes v;
  if (off) *off = d.off;
  if (count) *count = n;
  for (uint32_t i = 0; i < n; i++) {
    Hash32 h;
    memcpy(h.b, d.p + d.raw(32), 32);
    v.push_back(h);
  }
  return v;
}

// ---- the state blob (include/automerge_amd.h) ----
struct Have {
  Hashes last_sync;
  std::vector<uint8_t> bloom;
};
struct State {
  Hashes shared_heads, last_sent_heads, their_heads, their_need, sent_hashes;
  bool has_their_heads = false, has_their_need = false, has_their_have = false, sent_is_array = false;
  std::vector<Have> their_have;
};
enum { F_HEADS = 1, F_NEED = 2, F_HAVE = 4, F_SENT_ARRAY = 8 };

Hashes blob_hashes(Dec& d) {
  const uint64_t n = d.u53();
  Hashes v;
  for (uint64_t i = 0; i < n; i++) {
    Hash32 h;
    memcpy(h.b, d.p + d.raw(32), 32);
    v.push_back(h);
  }
  return v;
}
State read_state(const uint8_t* p, size_t n) {
  Dec d{p, n};
  if (d.byte() != 0x53) type_error("automerge_amd: not a sync state blob");
  const int fl = d.byte();
  if (fl < 0) type_error("automerge_amd: truncated sync state blob");
  State s;
  s.has_their_heads = fl & F_HEADS;
  s.has_their_need = fl & F_NEED;
  s.has_their_have = fl & F_HAVE;
  s.sent_is_array = fl & F_SENT_ARRAY;
  s.shared_heads = blob_hashes(d);
  s.last_sent_heads = blob_hashes(d);
  if (s.has_their_heads) s.their_heads = blob_hashes(d);
  if (s.has_their_need) s.their_need = blob_hashes(d);
  if (s.has_their_have) {
    const uint64_t nh = d.u53();
    for (uint64_t i = 0; i < nh; i++) {
      Have h;
      h.last_sync = blob_hashes(d);
      const uint64_t bl = d.u53();
      const uint64_t o = d.raw(bl);
      h.bloom.assign(p + o, p + o + bl);
      s.their_have.push_back(std::move(h));
    }
  }
  s.sent_hashes = blob_hashes(d);
  return s;
}
void blob_put(std::vector<uint8_t>& o, const Hashes& hs) {
  pu(o, hs.size());
  for (const Hash32& h : hs) o.insert(o.end(), h.b, h.b + 32);
}
std::vector<uint8_t> write_state(const State& s) {
  std::vector<uint8_t> o{0x53, (uint8_t)((s.has_their_heads ? F_HEADS : 0) | (s.has_their_need ? F_NEED : 0) |
                                         (s.has_their_have ? F_HAVE : 0) | (s.sent_is_array ? F_SENT_ARRAY : 0))};
  blob_put(o, s.shared_heads);
  blob_put(o, s.last_sent_heads);
  if (s.has_their_heads) blob_put(o, s.their_heads);
  if (s.has_their_need) blob_put(o, s.their_need);
  if (s.has_their_have) {
    pu(o, s.their_have.size());
    for (const Have& h : s.their_have) {
      blob_put(o, h.last_sync);
      pu(o, h.bloom.size());
      o.insert(o.end(), h.bloom.begin(), h.bloom.end());
    }
  }
  blob_put(o, s.sent_hashes);
  return o;
}

// ---- messages ----
struct Msg {
  Hashes heads, need;
  std::vector<Have> have;
  std::vector<std::pair<const uint8_t*, size_t>> changes;
};
std::vector<uint8_t> encode_msg(const Msg& m) {  // encodeSyncMessage (sync.js:157-171)
  std::vector<uint8_t> o{0x42};
  put_hashes(o, m.heads);
  put_hashes(o, m.need);
  pu(o, m.have.size());
  for (const Have& h : m.have) {
    put_hashes(o, h.last_sync);
    pu(o, h.bloom.size());
    o.insert(o.end(), h.bloom.begin(), h.bloom.end());
  }
  pu(o, m.changes.size());
  for (auto& c : m.changes) {
    pu(o, c.second);
    o.insert(o.end(), c.first, c.first + c.second);
  }
  return o;
}
// decodeSyncMessage (sync.js:177-199); spans as documented in the header
Msg decode_msg(const uint8_t* p, size_t n, std::vector<am_span>* spans = nullptr, uint32_t* counts = nullptr) {
  Dec d{p, n};
  const int t = d.byte();
  if (t != 0x42) range_error("Unexpected message type: " + (t < 0 ? std::string("undefined") : std::to_string(t)));
  Msg m;
  uint64_t off, cnt;
  m.heads = get_hashes(d, &off, &cnt);
  if (spans) spans->push_back({off, cnt});
  m.need = get_hashes(d, &off, &cnt);
  if (spans) spans->push_back({off, cnt});
  const uint32_t nh = d.u32();
  for (uint32_t i = 0; i < nh; i++) {
    Have h;
    h.last_sync = get_hashes(d, &off, &cnt);
    if (spans) spans->push_back({off, cnt});
    const uint64_t bl = d.u53();
    const uint64_t bo = d.raw(bl);
    h.bloom.assign(p + bo, p + bo + bl);
    if (spans) spans->push_back({bo, bl});
    m.have.push_back(std::move(h));
  }
  const uint32_t nc = d.u32();
  for (uint32_t i = 0; i < nc; i++) {
    const uint64_t cl = d.u53();
    const uint64_t co = d.raw(cl);
    m.changes.push_back({p + co, (size_t)cl});
    if (spans) spans->push_back({co, cl});
  }
  if (counts) { counts[0] = (uint32_t)m.heads.size(); counts[1] = (uint32_t)m.need.size(); counts[2] = nh; counts[3] = nc; }
  return m;  // trailing bytes are ignored (extensions, sync.js:197)
}

// ---- document queries (Backend.* in the reference) ----
Hashes heads_of(am_doc* d) {
  const size_t n = am_doc_get_heads(d, nullptr, 0);
  Hashes h(n);
  std::vector<uint8_t> buf(32 * (n ? n : 1));
  am_doc_get_heads(d, buf.data(), n);
  for (size_t i = 0; i < n; i++) memcpy(h[i].b, buf.data() + 32 * i, 32);
  return h;
}
std::vector<size_t> get_changes(am_doc* d, const Hashes& have) {
  uint64_t* idx = nullptr;
  size_t n = 0;
  am_error e;
  if (am_doc_get_changes(d, have.empty() ? nullptr : have[0].b, have.size(), &idx, &n, &e)) from_am(e);
  std::vector<size_t> v(idx, idx + n);
  am_free(idx);
  return v;
}
Hashes missing_deps(am_doc* d, const Hashes& heads) {
  uint8_t* out = nullptr;
  size_t n = 0;
  am_error e;
  if (am_doc_get_missing_deps(d, heads.empty() ? nullptr : heads[0].b, heads.size(), &out, &n, &e)) from_am(e);
  Hashes v(n);
  for (size_t i = 0; i < n; i++) memcpy(v[i].b, out + 32 * i, 32);
  am_free(out);
  return v;
}
int64_t change_index(am_doc* d, const Hash32& h) {  // getChangeByHash: -1 when unknown
  const int64_t i = am_doc_change_index(d, h.b);
  if (i < -1) range_error("automerge_amd: the document history could not be reconstructed");
  return i;
}
struct ChangeRef {
  const uint8_t* data;
  size_t len;
  Hash32 hash;
};
ChangeRef change_at(am_doc* d, size_t i) {
  ChangeRef c;
  if (am_doc_change(d, i, &c.data, &c.len, c.hash.b)) range_error("automerge_amd: change index out of range");
  return c;
}
Hashes change_deps(am_doc* d, size_t i) {
  const uint8_t* p = nullptr;
  size_t n = 0;
  if (am_doc_change_deps(d, i, &p, &n)) range_error("automerge_amd: change index out of range");
  Hashes v(n);
  for (size_t k = 0; k < n; k++) memcpy(v[k].b, p + 32 * k, 32);
  return v;
}
bool same(const Hashes& a, const Hashes& b) { return a == b; }  // compareArrays (sync.js:319-321)

// one document of a generateSyncMessage call
struct Gen {
  am_doc* doc = nullptr;
  State st;
  bool failed = false;
  SErr err;
  Hashes our_heads, our_need;
  bool want_have = false;
  Hashes have_hashes;              // changes since sharedHeads (makeBloomFilter)
  std::vector<uint8_t> bloom;      // our filter
  bool reset = false;
  bool select = false;             // getChangesToSend runs
  bool select_gpu = false;         // ... with `have` filters (k_sync_select)
  std::vector<size_t> changes;     // getChanges(lastSync keys) (duplicates kept)
  Hashes change_hashes;
  std::vector<int32_t> didx;       // per change: index of each dep within `changes` (-1: outside)
  std::vector<uint64_t> doff;
  std::vector<uint8_t> send;       // k_sync_select result per change
  std::vector<size_t> to_send;     // final change indexes
  bool message = false;
  std::vector<uint8_t> out_msg;
};

// makeBloomFilter part 1 + the checks before the selection (host)
void gen_prepare(Gen& g) {
  State& s = g.st;
  g.our_heads = heads_of(g.doc);
  g.our_need = missing_deps(g.doc, s.has_their_heads ? s.their_heads : Hashes());
  if (!s.has_their_heads || std::all_of(g.our_need.begin(), g.our_need.end(), [&](const Hash32& h) { return contains(s.their_heads, h); })) {
    g.want_have = true;
    for (size_t i : get_changes(g.doc, s.shared_heads)) g.have_hashes.push_back(change_at(g.doc, i).hash);
  }
  if (s.has_their_have && !s.their_have.empty()) {
    for (const Hash32& h : s.their_have[0].last_sync)
      if (change_index(g.doc, h) < 0) { g.reset = true; return; }
  }
  if (!(s.has_their_have && s.has_their_need)) return;
  g.select = true;
  if (s.their_have.empty()) {  // need.map(getChangeByHash).filter(defined)
    for (const Hash32& h : s.their_need) {
      const int64_t i = change_index(g.doc, h);
      if (i >= 0) g.to_send.push_back((size_t)i);
    }
    return;
  }
  Hashes keys;
  for (const Have& h : s.their_have) {
    for (const Hash32& x : h.last_sync)
      if (!contains(keys, x)) keys.push_back(x);
    am_error e;
    if (am_bloom_check(h.bloom.data(), h.bloom.size(), &e)) from_am(e);
  }
  g.changes = get_changes(g.doc, keys);
  std::unordered_map<Hash32, int32_t, Hash32Hasher> pos;
  for (size_t c = 0; c < g.changes.size(); c++) {
    g.change_hashes.push_back(change_at(g.doc, g.changes[c]).hash);
    pos.emplace(g.change_hashes.back(), (int32_t)c);
  }
  g.doff.push_back(0);
  for (size_t c = 0; c < g.changes.size(); c++) {
    for (const Hash32& dep : change_deps(g.doc, g.changes[c])) {
      auto it = pos.find(dep);
      g.didx.push_back(it == pos.end() ? -1 : it->second);
    }
    g.doff.push_back(g.didx.size());
  }
  g.select_gpu = true;
}

// getChangesToSend after the selection (sync.js:288-305), then the rest of generateSyncMessage
void gen_finish(Gen& g) {
  State& s = g.st;
  if (g.reset) {
    Msg m;
    m.heads = g.our_heads;
    m.have.push_back(Have());
    g.out_msg = encode_msg(m);
    g.message = true;
    return;
  }
  if (g.select_gpu) {
    std::unordered_set<Hash32, Hash32Hasher> send, listed(g.change_hashes.begin(), g.change_hashes.end());
    for (size_t c = 0; c < g.changes.size(); c++)
      if (g.send[c]) send.insert(g.change_hashes[c]);
    for (const Hash32& h : s.their_need) {
      send.insert(h);
      if (!listed.count(h)) {
        const int64_t i = change_index(g.doc, h);
        if (i >= 0) g.to_send.push_back((size_t)i);
      }
    }
    for (size_t c = 0; c < g.changes.size(); c++)
      if (send.count(g.change_hashes[c])) g.to_send.push_back(g.changes[c]);
  }
  const bool heads_unchanged = same(g.our_heads, s.last_sent_heads);
  const bool heads_equal = s.has_their_heads && same(g.our_heads, s.their_heads);
  if (heads_unchanged && heads_equal && g.to_send.empty()) return;  // in sync: no message
  Msg m;
  m.heads = g.our_heads;
  m.need = g.our_need;
  if (g.want_have) {
    Have h;
    h.last_sync = s.shared_heads;
    h.bloom = g.bloom;
    m.have.push_back(std::move(h));
  }
  // membership through a hash set: a first sync of a long history sends every change
  std::unordered_set<Hash32, Hash32Hasher> sent(s.sent_hashes.begin(), s.sent_hashes.end());
  std::vector<Hash32> new_hashes;
  for (size_t i : g.to_send) {
    ChangeRef c = change_at(g.doc, i);
    if (sent.count(c.hash)) continue;
    m.changes.push_back({c.data, c.len});
    new_hashes.push_back(c.hash);
  }
  g.out_msg = encode_msg(m);
  g.message = true;
  if (!m.changes.empty()) {  // sentHashes = copyObject(sentHashes) + the hashes sent
    s.sent_is_array = false;
    for (const Hash32& h : new_hashes)
      if (sent.insert(h).second) s.sent_hashes.push_back(h);
  }
  s.last_sent_heads = g.our_heads;
}

// AM_SYNC_PROFILE=1: per-stage wall times of the batched sync calls on stderr
struct StageClock {
  bool on = getenv("AM_SYNC_PROFILE") != nullptr;
  std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
  std::string line;
  void mark(const char* what) {
    if (!on) return;
    const auto now = std::chrono::steady_clock::now();
    char b[64];
    snprintf(b, sizeof b, " %s=%.1fms", what, std::chrono::duration<double, std::milli>(now - t).count());
    line += b;
    t = now;
  }
  void print(const char* call, size_t n) {
    if (on) fprintf(stderr, "[am_sync] %s n=%zu%s\n", call, n, line.c_str());
  }
};

uint8_t* dup(const std::vector<uint8_t>& v) {
  uint8_t* p = (uint8_t*)malloc(v.size() ? v.size() : 1);
  if (p && !v.empty()) memcpy(p, v.data(), v.size());
  return p;
}

Hashes sorted_unique(Hashes v) {
  std::sort(v.begin(), v.end());
  v.erase(std::unique(v.begin(), v.end()), v.end());
  return v;
}

}  // namespace

extern "C" int am_sync_generate(size_t n, am_doc* const* docs, const uint8_t* const* states, const size_t* state_lens,
                                uint8_t** out_states, size_t* out_state_lens, uint8_t** msgs, size_t* msg_lens,
                                uint32_t* codes, char** errmsgs) {
  StageClock clk;
  std::vector<Gen> gs(n);
  {  // the hash graphs of loaded documents (computeHashGraph, new.js:1879-1904) in one batch
    std::vector<am_doc*> gd(docs, docs + n);
    std::vector<uint32_t> gc(n);
    if (n) am_doc_compute_hash_graph_batch(n, gd.data(), gc.data(), nullptr);  // errors resurface below
  }
  clk.mark("graphs");
  auto fail = [&](Gen& g, const SErr& e) {
    g.failed = true;
    g.err = e;
  };
  // the graph queries only read the (indexed) graphs: host workers over the documents; a document
  // whose graph is not ready (its history failed to decode) raises that error on this thread
  auto prepare = [&](size_t i) {
    gs[i].doc = docs[i];
    try {
      gs[i].st = read_state(states[i], state_lens[i]);
      gen_prepare(gs[i]);
    } catch (const SErr& e) {
      fail(gs[i], e);
    } catch (const std::bad_alloc&) {
      fail(gs[i], SErr{false, "automerge_amd: out of host memory", AM_U_CAPACITY});
    }
  };
  std::vector<uint8_t> ready(n);
  for (size_t i = 0; i < n; i++) ready[i] = am_doc_graph_ready(docs[i]) != 0;
  am_par_for(n, [&](size_t i) { if (ready[i]) prepare(i); });
  for (size_t i = 0; i < n; i++)
    if (!ready[i]) prepare(i);
  clk.mark("prepare");
  // the GPU stages, one launch per engine for all its documents
  std::vector<am_engine*> engines;
  for (auto& g : gs)
    if (!g.failed && std::find(engines.begin(), engines.end(), am_doc_engine(g.doc)) == engines.end())
      engines.push_back(am_doc_engine(g.doc));
  for (am_engine* eng : engines) {
    std::vector<Gen*> grp;
    for (auto& g : gs)
      if (!g.failed && am_doc_engine(g.doc) == eng) grp.push_back(&g);
    // Bloom filters of our changes since sharedHeads (k_bloom_build)
    std::vector<Gen*> bl;
    std::vector<uint8_t> flat;
    std::vector<uint64_t> hoff{0};
    for (Gen* g : grp)
      if (g->want_have) {
        bl.push_back(g);
        for (const Hash32& h : g->have_hashes) flat.insert(flat.end(), h.b, h.b + 32);
        hoff.push_back(hoff.back() + g->have_hashes.size());
      }
    if (!bl.empty()) {
      uint64_t total = 0;
      for (size_t f = 0; f < bl.size(); f++) total += am_bloom_encoded_size(hoff[f + 1] - hoff[f]);
      std::vector<uint8_t> out(total ? total : 1);
      std::vector<uint64_t> foff(bl.size() + 1);
      am_error e;
      if (am_bloom_build(eng, flat.empty() ? nullptr : flat.data(), hoff.data(), (uint32_t)bl.size(), out.data(), total,
                         foff.data(), &e)) {
        for (Gen* g : grp) fail(*g, SErr{false, e.message, e.code});
        continue;
      }
      for (size_t f = 0; f < bl.size(); f++) bl[f]->bloom.assign(out.begin() + foff[f], out.begin() + foff[f + 1]);
    }
    // change selection against the peer's filters (k_sync_select)
    std::vector<Gen*> sel;
    std::vector<uint64_t> coff{0}, doff{0}, pfoff{0}, foff{0};
    std::vector<uint8_t> hashes, filters;
    std::vector<int32_t> didx;
    for (Gen* g : grp)
      if (g->select_gpu && !g->reset) {
        sel.push_back(g);
        for (size_t c = 0; c < g->changes.size(); c++) {
          hashes.insert(hashes.end(), g->change_hashes[c].b, g->change_hashes[c].b + 32);
          for (uint64_t q = g->doff[c]; q < g->doff[c + 1]; q++) didx.push_back(g->didx[q]);
          doff.push_back(didx.size());
        }
        coff.push_back(coff.back() + g->changes.size());
        for (const Have& h : g->st.their_have) {
          filters.insert(filters.end(), h.bloom.begin(), h.bloom.end());
          foff.push_back(filters.size());
        }
        pfoff.push_back(foff.size() - 1);
      }
    if (!sel.empty()) {
      std::vector<uint8_t> send(coff.back() ? coff.back() : 1);
      am_error e;
      if (am_sync_select(eng, (uint32_t)sel.size(), coff.data(), hashes.empty() ? nullptr : hashes.data(), doff.data(),
                         didx.empty() ? nullptr : didx.data(), pfoff.data(), filters.empty() ? nullptr : filters.data(),
                         foff.data(), send.data(), &e)) {
        for (Gen* g : grp) fail(*g, SErr{false, e.message, e.code});
        continue;
      }
      for (size_t k = 0; k < sel.size(); k++) sel[k]->send.assign(send.begin() + coff[k], send.begin() + coff[k + 1]);
    }
  }
  clk.mark("gpu");
  auto finish = [&](size_t i) {
    Gen& g = gs[i];
    out_states[i] = nullptr;
    out_state_lens[i] = 0;
    msgs[i] = nullptr;
    msg_lens[i] = 0;
    if (!g.failed) {
      try {
        gen_finish(g);
        const std::vector<uint8_t> st = write_state(g.st);
        out_states[i] = dup(st);
        out_state_lens[i] = st.size();
        if (g.message) {
          msgs[i] = dup(g.out_msg);
          msg_lens[i] = g.out_msg.size();
        }
      } catch (const SErr& e) {
        fail(g, e);
      } catch (const std::bad_alloc&) {
        fail(g, SErr{false, "automerge_amd: out of host memory", AM_U_CAPACITY});
      }
    }
  };
  am_par_for(n, [&](size_t i) { if (ready[i]) finish(i); });
  for (size_t i = 0; i < n; i++)
    if (!ready[i]) finish(i);
  clk.mark("finish");
  int nfail = 0;
  for (size_t i = 0; i < n; i++) {
    Gen& g = gs[i];
    codes[i] = 0;
    if (errmsgs) errmsgs[i] = nullptr;
    if (g.failed) {
      codes[i] = (g.err.code ? g.err.code : (uint32_t)AM_E_LOCAL) | (g.err.type_error ? 0x80000000u : 0u);
      if (errmsgs) {
        errmsgs[i] = (char*)malloc(g.err.msg.size() + 1);
        if (errmsgs[i]) memcpy(errmsgs[i], g.err.msg.c_str(), g.err.msg.size() + 1);
      }
      nfail++;
    }
  }
  clk.mark("out");
  am_reclaim(gs);  // the per-document buffers, freed off the critical path
  clk.mark("free");
  clk.print("generate", n);
  return nfail;
}

namespace {
// receiveSyncMessage after the changes are applied (sync.js:430-473; advanceHeads :408-413)
std::vector<uint8_t> recv_finish(am_doc* d, State& s, const Msg& m, const Hashes& before) {
  if (!m.changes.empty()) {
    const Hashes after = heads_of(d);
    Hashes adv;
    for (const Hash32& h : after)
      if (!contains(before, h)) adv.push_back(h);
    for (const Hash32& h : s.shared_heads)
      if (contains(after, h)) adv.push_back(h);
    s.shared_heads = sorted_unique(adv);
  }
  if (m.changes.empty() && same(m.heads, before)) s.last_sent_heads = m.heads;
  Hashes known;
  for (const Hash32& h : m.heads)
    if (change_index(d, h) >= 0) known.push_back(h);
  if (known.size() == m.heads.size()) {
    s.shared_heads = m.heads;
    if (m.heads.empty()) {  // the peer lost its data: full resync
      s.last_sent_heads.clear();
      s.sent_hashes.clear();
      s.sent_is_array = true;
    }
  } else {
    known.insert(known.end(), s.shared_heads.begin(), s.shared_heads.end());
    s.shared_heads = sorted_unique(known);
  }
  s.has_their_have = s.has_their_heads = s.has_their_need = true;
  s.their_have = m.have;
  s.their_heads = m.heads;
  s.their_need = m.need;
  return write_state(s);
}
}  // namespace

extern "C" int am_sync_receive(am_doc* d, const uint8_t* state, size_t state_len, const uint8_t* msg, size_t msg_len,
                               uint8_t** out_state, size_t* out_state_len, uint8_t** patch, size_t* patch_len,
                               am_error* err) {
  *patch = nullptr;
  *patch_len = 0;
  bool applied = false;
  try {
    State s = read_state(state, state_len);
    Msg m = decode_msg(msg, msg_len);
    const Hashes before = heads_of(d);
    if (!m.changes.empty()) {
      std::vector<const uint8_t*> bufs;
      std::vector<size_t> lens;
      for (auto& c : m.changes) { bufs.push_back(c.first); lens.push_back(c.second); }
      am_error e;
      if (am_doc_apply_changes_patch(d, bufs.data(), lens.data(), bufs.size(), patch, patch_len, &e)) from_am(e);
      applied = true;
    }
    const std::vector<uint8_t> o = recv_finish(d, s, m, before);
    *out_state = dup(o);
    *out_state_len = o.size();
  } catch (const SErr& e) {
    to_err(e, err);
    if (*patch) { am_free(*patch); *patch = nullptr; *patch_len = 0; }
    return applied ? 2 : 1;
  } catch (const std::bad_alloc&) {
    to_err(SErr{false, "automerge_amd: out of host memory", AM_U_CAPACITY}, err);
    return applied ? 2 : 1;
  }
  if (err) err->code = 0;
  return 0;
}

// receiveSyncMessage of n (document, state, message) triples: the messages' changes applied to their
// documents in ONE batched applyChanges (am_doc_apply_changes_batch), the hash graphs the heads
// lookups need computed in one batch, then the state updates. codes[i]: 0, or the error (bit 31:
// TypeError; bit 30: the changes were applied before the error, as am_sync_receive's return 2).
extern "C" int am_sync_receive_batch(size_t n, am_doc* const* docs, const uint8_t* const* states, const size_t* state_lens,
                                     const uint8_t* const* msgs, const size_t* msg_lens, uint8_t** out_states,
                                     size_t* out_state_lens, uint8_t** patches, size_t* patch_lens, am_call_info* info,
                                     uint32_t* codes, char** errmsgs) {
  struct R {
    State s;
    Msg m;
    Hashes before;
    bool failed = false, applied = false, single = false;
    SErr err;
  };
  StageClock clk;
  std::vector<R> rs(n);
  std::unordered_set<am_doc*> seen;
  for (size_t i = 0; i < n; i++) {
    out_states[i] = nullptr;
    out_state_lens[i] = 0;
    patches[i] = nullptr;
    patch_lens[i] = 0;
    if (info) info[i] = am_call_info{0, 0, 0, nullptr};
    if (!seen.insert(docs[i]).second) rs[i].single = true;  // after the batch, in order
  }
  am_par_for(n, [&](size_t i) {
    R& r = rs[i];
    if (r.single) return;
    try {
      r.s = read_state(states[i], state_lens[i]);
      r.m = decode_msg(msgs[i], msg_lens[i]);
      r.before = heads_of(docs[i]);
    } catch (const SErr& e) {
      r.failed = true;
      r.err = e;
    } catch (const std::bad_alloc&) {
      r.failed = true;
      r.err = SErr{false, "automerge_amd: out of host memory", AM_U_CAPACITY};
    }
  });
  clk.mark("decode");
  // every message's changes: one batched applyChanges
  std::vector<size_t> at, off{0};
  std::vector<am_doc*> ad;
  std::vector<const uint8_t*> bufs;
  std::vector<size_t> lens;
  for (size_t i = 0; i < n; i++) {
    R& r = rs[i];
    if (r.single || r.failed || r.m.changes.empty()) continue;
    at.push_back(i);
    ad.push_back(docs[i]);
    for (auto& c : r.m.changes) { bufs.push_back(c.first); lens.push_back(c.second); }
    off.push_back(bufs.size());
  }
  if (!at.empty()) {
    std::vector<uint8_t*> pp(at.size());
    std::vector<size_t> pl(at.size());
    std::vector<uint32_t> cc(at.size());
    std::vector<char*> mm(at.size());
    std::vector<am_call_info> ci(at.size());
    am_doc_apply_changes_batch(at.size(), ad.data(), off.data(), bufs.data(), lens.data(), pp.data(), pl.data(),
                               info ? ci.data() : nullptr, cc.data(), mm.data());
    if (info)
      for (size_t k = 0; k < at.size(); k++) info[at[k]] = ci[k];
    for (size_t k = 0; k < at.size(); k++) {
      R& r = rs[at[k]];
      if (cc[k]) {
        r.failed = true;
        r.err = SErr{(cc[k] & 0x80000000u) != 0, mm[k] ? mm[k] : "", cc[k] & 0x7fffffffu};
      } else {
        r.applied = true;
        patches[at[k]] = pp[k];
        patch_lens[at[k]] = pl[k];
      }
      if (mm[k]) am_free(mm[k]);
    }
  }
  clk.mark("apply");
  // the hash graphs the heads lookups need (loaded documents), in one batch
  std::vector<am_doc*> gd;
  for (size_t i = 0; i < n; i++)
    if (!rs[i].single && !rs[i].failed && !rs[i].m.heads.empty()) gd.push_back(docs[i]);
  if (!gd.empty()) {
    std::vector<uint32_t> gc(gd.size());
    am_doc_compute_hash_graph_batch(gd.size(), gd.data(), gc.data(), nullptr);  // errors resurface below
  }
  clk.mark("graphs");
  // the state updates (graph reads only) on the host workers, for documents whose graph is ready
  std::vector<uint8_t> done(n, 0);
  am_par_for(n, [&](size_t i) {
    R& r = rs[i];
    if (r.single || r.failed || (!r.m.heads.empty() && !am_doc_graph_ready(docs[i]))) return;
    try {
      const std::vector<uint8_t> o = recv_finish(docs[i], r.s, r.m, r.before);
      out_states[i] = dup(o);
      out_state_lens[i] = o.size();
    } catch (const SErr& e) {
      r.failed = true;
      r.err = e;
    } catch (const std::bad_alloc&) {
      r.failed = true;
      r.err = SErr{false, "automerge_amd: out of host memory", AM_U_CAPACITY};
    }
    done[i] = 1;
  });
  clk.mark("finish");
  int nfail = 0;
  for (size_t i = 0; i < n; i++) {
    R& r = rs[i];
    std::string msg;
    uint32_t code = 0;
    if (r.single) {
      am_error e;
      const int rc = am_sync_receive(docs[i], states[i], state_lens[i], msgs[i], msg_lens[i], out_states + i,
                                     out_state_lens + i, patches + i, patch_lens + i, &e);
      if (!rc && info && patches[i]) {
        info[i].max_op = am_doc_max_op(docs[i]);
        info[i].pending = (uint32_t)am_doc_pending(docs[i]);
        info[i].nheads = (uint32_t)am_doc_get_heads(docs[i], nullptr, 0);
        info[i].heads = (uint8_t*)malloc(32 * (info[i].nheads ? info[i].nheads : 1));
        if (info[i].heads) am_doc_get_heads(docs[i], info[i].heads, info[i].nheads);
      }
      if (rc) {
        code = e.code | (e.is_type_error ? 0x80000000u : 0u) | (rc == 2 ? 0x40000000u : 0u);
        msg = e.message;
      }
    } else {
      if (!r.failed && !done[i]) {
        try {
          const std::vector<uint8_t> o = recv_finish(docs[i], r.s, r.m, r.before);
          out_states[i] = dup(o);
          out_state_lens[i] = o.size();
        } catch (const SErr& e) {
          r.failed = true;
          r.err = e;
        }
      }
      if (r.failed) {
        code = (r.err.code ? r.err.code : (uint32_t)AM_E_LOCAL) | (r.err.type_error ? 0x80000000u : 0u) | (r.applied ? 0x40000000u : 0u);
        msg = r.err.msg;
        if (patches[i]) { am_free(patches[i]); patches[i] = nullptr; patch_lens[i] = 0; }
        if (info && info[i].heads) { am_free(info[i].heads); info[i] = am_call_info{0, 0, 0, nullptr}; }
      }
    }
    codes[i] = code;
    if (errmsgs) {
      errmsgs[i] = nullptr;
      if (code) {
        errmsgs[i] = (char*)malloc(msg.size() + 1);
        if (errmsgs[i]) memcpy(errmsgs[i], msg.c_str(), msg.size() + 1);
      }
    }
    nfail += code != 0;
  }
  clk.mark("out");
  am_reclaim(rs);
  clk.mark("free");
  clk.print("receive", n);
  return nfail;
}

// encodeHashes (sync.js:130-139) of a JSON array of hex strings
static void json_hashes(std::vector<uint8_t>& o, const amjson::JV& v) {
  if (v.k != amjson::ARR) type_error("hashes must be an array");
  pu(o, v.a.size());
  for (size_t i = 0; i < v.a.size(); i++) {
    if (i > 0 && !(amjson::js_str(v.a[i - 1]) < amjson::js_str(v.a[i]))) range_error("hashes must be sorted");
    const amjson::JV& h = v.a[i];
    if (h.k != amjson::STR) type_error("value is not a string");
    if (h.s.size() % 2) range_error("value is not hexadecimal");
    std::vector<uint8_t> b;
    for (size_t k = 0; k < h.s.size(); k += 2) {
      int x = 0;
      for (int q = 0; q < 2; q++) {
        const char c = h.s[k + q];
        x <<= 4;
        if (c >= '0' && c <= '9') x |= c - '0';
        else if (c >= 'a' && c <= 'f') x |= c - 'a' + 10;
        else range_error("value is not hexadecimal");
      }
      b.push_back((uint8_t)x);
    }
    if (b.size() != 32) type_error("heads hashes must be 256 bits");
    o.insert(o.end(), b.begin(), b.end());
  }
}
static void json_prefixed(std::vector<uint8_t>& o, const amjson::JV& v) {  // appendPrefixedBytes
  if (v.k != amjson::BYTES) range_error("value is not an integer");
  pu(o, v.s.size());
  o.insert(o.end(), v.s.begin(), v.s.end());
}

extern "C" int am_sync_encode_message(const char* json, size_t len, uint8_t** out, size_t* out_len, am_error* err) {
  amjson::JV m;
  if (!amjson::parse(json, len, m)) {
    to_err(SErr{true, "automerge_amd: the sync message is not valid JSON"}, err);
    return 1;
  }
  try {
    std::vector<uint8_t> o{0x42};
    json_hashes(o, m["heads"]);
    json_hashes(o, m["need"]);
    const amjson::JV& have = m["have"];
    if (have.k != amjson::ARR) type_error("Cannot read property 'length' of " + amjson::js_str(have));
    pu(o, have.a.size());
    for (const amjson::JV& h : have.a) {
      json_hashes(o, h["lastSync"]);
      json_prefixed(o, h["bloom"]);
    }
    const amjson::JV& changes = m["changes"];
    if (changes.k != amjson::ARR) type_error("Cannot read property 'length' of " + amjson::js_str(changes));
    pu(o, changes.a.size());
    for (const amjson::JV& c : changes.a) json_prefixed(o, c);
    *out = dup(o);
    *out_len = o.size();
  } catch (const SErr& e) {
    to_err(e, err);
    return 1;
  }
  if (err) err->code = 0;
  return 0;
}

extern "C" int am_sync_decode_messages(size_t n, const uint8_t* const* msgs, const size_t* lens, am_span** spans,
                                       uint64_t* span_off, uint32_t* counts, am_error* errs) {
  std::vector<am_span> all;
  int nfail = 0;
  span_off[0] = 0;
  for (size_t i = 0; i < n; i++) {
    std::vector<am_span> sp;
    try {
      decode_msg(msgs[i], lens[i], &sp, counts + 4 * i);
      all.insert(all.end(), sp.begin(), sp.end());
      if (errs) errs[i].code = 0;
    } catch (const SErr& e) {
      to_err(e, errs ? &errs[i] : nullptr);
      memset(counts + 4 * i, 0, 4 * sizeof(uint32_t));
      nfail++;
    }
    span_off[i + 1] = all.size();
  }
  *spans = (am_span*)malloc(sizeof(am_span) * (all.empty() ? 1 : all.size()));
  if (!all.empty()) memcpy(*spans, all.data(), sizeof(am_span) * all.size());
  return nfail;
}

extern "C" int am_sync_encode_state(const uint8_t* state, size_t len, uint8_t** out, size_t* out_len, am_error* err) {
  try {
    const State s = read_state(state, len);
    std::vector<uint8_t> o{0x43};
    put_hashes(o, s.shared_heads);
    *out = dup(o);
    *out_len = o.size();
  } catch (const SErr& e) {
    to_err(e, err);
    return 1;
  }
  if (err) err->code = 0;
  return 0;
}

extern "C" int am_sync_decode_state(const uint8_t* bytes, size_t len, uint8_t** state, size_t* state_len, am_error* err) {
  try {
    Dec d{bytes, len};
    const int t = d.byte();
    if (t != 0x43) range_error("Unexpected record type: " + (t < 0 ? std::string("undefined") : std::to_string(t)));
    State s;  // initSyncState() + sharedHeads (sync.js:308-317)
    s.shared_heads = get_hashes(d);
    const std::vector<uint8_t> o = write_state(s);
    *state = dup(o);
    *state_len = o.size();
  } catch (const SErr& e) {
    to_err(e, err);
    return 1;
  }
  if (err) err->code = 0;
  return 0;
}
