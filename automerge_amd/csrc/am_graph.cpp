// am_graph.cpp -- change hash graph of a document (am_graph.h): header parse of change chunks and
// the hash-graph queries of BackendDoc (new.js:1913-2020). Host code.
#include "am_graph.h"

#include <zlib.h>

#include <algorithm>
#include <unordered_set>

namespace {

struct Cur {
  const uint8_t* p;
  size_t n, off;
  bool ok = true;
  uint64_t u() {
    uint64_t v = 0;
    for (int sh = 0; off < n; sh += 7) {
      const uint8_t b = p[off++];
      if (sh < 64) v |= (uint64_t)(b & 0x7f) << sh;
      if (!(b & 0x80)) return v;
    }
    ok = false;
    return 0;
  }
  const uint8_t* take(uint64_t k) {
    if (k > n - off) { ok = false; return p; }
    const uint8_t* r = p + off;
    off += k;
    return r;
  }
};

bool raw_inflate(const uint8_t* p, size_t n, std::vector<uint8_t>& out) {
  out.resize(n * 4 + 256);
  z_stream zs;
  memset(&zs, 0, sizeof zs);
  if (inflateInit2(&zs, -15) != Z_OK) return false;
  zs.next_in = const_cast<Bytef*>(p);
  zs.avail_in = (uInt)n;
  int r = Z_OK;
  while (r == Z_OK) {
    if (zs.total_out == out.size()) out.resize(out.size() * 2);
    zs.next_out = out.data() + zs.total_out;
    zs.avail_out = (uInt)(out.size() - zs.total_out);
    r = inflate(&zs, Z_FINISH);
    if (r == Z_BUF_ERROR && zs.avail_out == 0) r = Z_OK;
  }
  out.resize(zs.total_out);
  inflateEnd(&zs);
  return r == Z_STREAM_END;
}

const char* kHex = "0123456789abcdef";

}  // namespace

bool am_change_meta(const uint8_t* p, size_t n, ChangeMeta& m) {
  if (n < 10 || p[0] != 0x85 || p[1] != 0x6f || p[2] != 0x4a || p[3] != 0x83) return false;
  Cur c{p, n, 9};
  const uint64_t len = c.u();
  const uint8_t* body = c.take(len);
  if (!c.ok) return false;
  std::vector<uint8_t> inflated;
  if (p[8] == 2) {
    if (!raw_inflate(body, len, inflated)) return false;
    body = inflated.data();
  } else if (p[8] != 1) {
    return false;
  }
  Cur h{body, p[8] == 2 ? inflated.size() : (size_t)len, 0};
  const uint64_t nd = h.u();
  m.deps.clear();
  for (uint64_t i = 0; i < nd && h.ok; i++) {
    Hash32 d;
    const uint8_t* q = h.take(32);
    if (!h.ok) return false;
    memcpy(d.b, q, 32);
    m.deps.push_back(d);
  }
  const uint64_t al = h.u();
  const uint8_t* a = h.take(al);
  m.actor.clear();
  for (uint64_t i = 0; h.ok && i < al; i++) { m.actor += kHex[a[i] >> 4]; m.actor += kHex[a[i] & 15]; }
  m.seq = (int64_t)h.u();
  return h.ok;
}

void HashGraph::clear() {
  hashes.clear();
  meta.clear();
  index.clear();
  dependents.clear();
  by_actor.clear();
  clock.clear();
}

void HashGraph::add(const Hash32& h, const ChangeMeta& m) {
  index[h] = hashes.size();
  hashes.push_back(h);
  meta.push_back(m);
  dependents.emplace(h, std::vector<Hash32>());
  for (const Hash32& d : m.deps) dependents[d].push_back(h);
  std::vector<Hash32>& seqs = by_actor[m.actor];
  if (m.seq >= 1) {
    if ((size_t)m.seq > seqs.size()) seqs.resize((size_t)m.seq);
    seqs[(size_t)m.seq - 1] = h;
  }
  int64_t& c = clock[m.actor];
  if (m.seq > c) c = m.seq;
}

int64_t HashGraph::find(const Hash32& h) const {
  auto it = index.find(h);
  return it == index.end() ? -1 : (int64_t)it->second;
}

bool HashGraph::changes_since(const std::vector<Hash32>& have, const std::vector<Hash32>& heads, std::vector<size_t>& out,
                              Hash32& missing) const {
  out.clear();
  if (have.empty()) {
    for (size_t i = 0; i < hashes.size(); i++) out.push_back(i);
    return true;
  }
  // forward walk from `have` along dependents: complete when every change it meets has all its
  // dependencies already met and the walk reaches every head
  std::unordered_set<Hash32, Hash32Hasher> seen;
  std::vector<Hash32> todo;
  for (const Hash32& h : have) {
    seen.insert(h);
    auto it = dependents.find(h);
    if (it == dependents.end()) { missing = h; return false; }
    todo.insert(todo.end(), it->second.begin(), it->second.end());
  }
  std::vector<Hash32> found;
  while (!todo.empty()) {
    const Hash32 h = todo.back();
    todo.pop_back();
    seen.insert(h);
    found.push_back(h);
    const ChangeMeta& m = meta[index.at(h)];
    bool deps_met = true;
    for (const Hash32& d : m.deps) deps_met = deps_met && seen.count(d);
    if (!deps_met) break;
    const std::vector<Hash32>& next = dependents.at(h);
    todo.insert(todo.end(), next.begin(), next.end());
  }
  bool all_heads = true;
  for (const Hash32& h : heads) all_heads = all_heads && seen.count(h);
  if (todo.empty() && all_heads) {
    for (const Hash32& h : found) out.push_back(index.at(h));
    return true;
  }
  // otherwise: everything not reachable backwards from `have`, in history order
  seen.clear();
  todo = have;
  while (!todo.empty()) {
    const Hash32 h = todo.back();
    todo.pop_back();
    if (seen.count(h)) continue;
    auto it = index.find(h);
    if (it == index.end()) { missing = h; return false; }
    const std::vector<Hash32>& deps = meta[it->second].deps;
    todo.insert(todo.end(), deps.begin(), deps.end());
    seen.insert(h);
  }
  for (size_t i = 0; i < hashes.size(); i++)
    if (!seen.count(hashes[i])) out.push_back(i);
  return true;
}

void HashGraph::added_since(const std::function<bool(const Hash32&)>& known, const std::vector<Hash32>& heads,
                            std::vector<size_t>& out) const {
  out.clear();
  std::unordered_set<Hash32, Hash32Hasher> seen;
  std::vector<Hash32> todo = heads;
  std::vector<size_t> found;
  while (!todo.empty()) {
    const Hash32 h = todo.back();
    todo.pop_back();
    if (seen.count(h) || known(h)) continue;
    seen.insert(h);
    const size_t i = index.at(h);
    found.push_back(i);
    todo.insert(todo.end(), meta[i].deps.begin(), meta[i].deps.end());
  }
  out.assign(found.rbegin(), found.rend());
}
