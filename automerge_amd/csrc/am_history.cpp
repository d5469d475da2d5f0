// am_history.cpp -- change history of a saved document, host stage.
//
// Reference: computeHashGraph (new.js:1879-1904) = decodeChanges([save()]) -> decodeDocument
// (columnar.js:1040-1046): decodeDocumentHeader (:1006), the change and op columns
// (DOCUMENT_COLUMNS / DOC_OPS_COLUMNS :77-94), groupChangeOps (:876-943: succ lists turned back into
// pred lists, deletions re-created as `del` ops, every op assigned to its change by binary search
// on the author's maxOp, ops sorted by opId, startOp = maxOp - #ops + 1), decodeDocumentChanges
// (:945-981: deps from depsIndex, the hash of every change from its re-encoding, heads check),
// then encodeChange (:710-739, deflateChange when >= 256 B) of every change.
//
// The hash of change i needs the hashes of its deps, so the chain is sequential; it runs once per
// loaded document, on the host, next to the host DEFLATE stage. Values pass through as their
// (valLen, valRaw) bytes. Documents with unknown columns or link ops are reported (AM_U_*).
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <stdexcept>
#include <map>
#include <string>
#include <unordered_map>
#include <vector>

#include <zlib.h>

#include "../../include/automerge_amd.h"
#include "am_change_enc.h"

namespace {

struct HErr {
  uint32_t code = 0;
  std::string msg;
};

struct Rd {
  const uint8_t* p;
  size_t n, o = 0;
  bool bad = false;
  uint64_t u() {
    uint64_t v = 0;
    int sh = 0;
    for (;;) {
      if (o >= n) { bad = true; return 0; }
      const uint8_t c = p[o++];
      if (sh < 64) v |= (uint64_t)(c & 0x7f) << sh;
      sh += 7;
      if (!(c & 0x80)) return v;
      if (sh > 63) { bad = true; return 0; }
    }
  }
  int64_t s() {
    int64_t v = 0;
    int sh = 0;
    uint8_t c;
    do {
      if (o >= n) { bad = true; return 0; }
      c = p[o++];
      if (sh < 64) v |= (int64_t)(c & 0x7f) << sh;
      sh += 7;
      if (sh > 70) { bad = true; return 0; }
    } while (c & 0x80);
    if (sh < 64 && (c & 0x40)) v |= -((int64_t)1 << sh);
    return v;
  }
  const uint8_t* raw(size_t k) {
    if (k > n - o) { bad = true; return p; }
    const uint8_t* q = p + o;
    o += k;
    return q;
  }
  bool done() const { return o >= n; }
};

// one decoded column value: null, an integer, or a byte string (utf8 / actor hex)
struct Val { bool null = true; int64_t i = 0; std::string s; };

// RLE column (RLEDecoder, encoding.js:789-920) of uint / int / utf8 values
std::vector<Val> dec_rle(const std::vector<uint8_t>& b, int type, size_t count, bool& bad) {
  std::vector<Val> out;
  Rd r{b.data(), b.size()};
  while (!r.done() && !r.bad) {
    const int64_t n = r.s();
    // a run longer than the cap is malformed input, not an allocation request
    const uint64_t room = (1u << 30) - std::min<uint64_t>(out.size(), 1u << 30);
    if ((n > 0 && (uint64_t)n > room) || (n < 0 && (uint64_t)(-(n + 1)) + 1 > room)) { bad = true; break; }
    if (n > 0) {
      Val v;
      v.null = false;
      if (type == 2) { const uint64_t L = r.u(); const uint8_t* q = r.raw(L); v.s.assign((const char*)q, L); }
      else if (type == 1) v.i = r.s();
      else v.i = (int64_t)r.u();
      for (int64_t k = 0; k < n; k++) out.push_back(v);
    } else if (n < 0) {
      for (int64_t k = 0; k < -n; k++) {
        Val v;
        v.null = false;
        if (type == 2) { const uint64_t L = r.u(); const uint8_t* q = r.raw(L); v.s.assign((const char*)q, L); }
        else if (type == 1) v.i = r.s();
        else v.i = (int64_t)r.u();
        out.push_back(v);
      }
    } else {
      const uint64_t m = r.u();
      if (m > room) { bad = true; break; }
      for (uint64_t k = 0; k < m; k++) out.push_back(Val());
    }
    if (out.size() > (1u << 30)) { bad = true; break; }
  }
  bad |= r.bad;
  if (count > (1u << 30)) { bad = true; return out; }
  while (out.size() < count) out.push_back(Val());  // a missing / short column reads as nulls
  return out;
}
std::vector<Val> dec_delta(const std::vector<uint8_t>& b, size_t count, bool& bad) {
  std::vector<Val> v = dec_rle(b, 1, count, bad);
  int64_t run = 0;
  for (auto& x : v)
    if (!x.null) { run += x.i; x.i = run; }
  return v;
}
std::vector<bool> dec_bool(const std::vector<uint8_t>& b, size_t count, bool& bad) {
  std::vector<bool> out;
  Rd r{b.data(), b.size()};
  bool cur = false;
  while (!r.done() && !r.bad) {
    const uint64_t n = r.u();
    if (n > (1u << 30) - std::min<uint64_t>(out.size(), 1u << 30)) { bad = true; break; }
    for (uint64_t k = 0; k < n; k++) out.push_back(cur);
    cur = !cur;
  }
  bad |= r.bad;
  if (count > (1u << 30)) { bad = true; return out; }
  while (out.size() < count) out.push_back(false);
  return out;
}

bool inflate_col(const std::vector<uint8_t>& in, std::vector<uint8_t>& out) {
  z_stream zs;
  memset(&zs, 0, sizeof zs);
  if (inflateInit2(&zs, -15) != Z_OK) return false;
  out.assign(in.size() * 4 + 64, 0);
  zs.next_in = const_cast<uint8_t*>(in.data());
  zs.avail_in = (uInt)in.size();
  int rc;
  for (;;) {
    zs.next_out = out.data() + zs.total_out;
    zs.avail_out = (uInt)(out.size() - zs.total_out);
    rc = inflate(&zs, Z_FINISH);
    if (rc == Z_STREAM_END) break;
    if (rc != Z_OK && rc != Z_BUF_ERROR) break;
    out.resize(out.size() * 2);
  }
  out.resize(zs.total_out);
  inflateEnd(&zs);
  return rc == Z_STREAM_END;
}

struct Col { uint32_t id; std::vector<uint8_t> b; };

std::string hex(const uint8_t* p, size_t n) {
  static const char* H = "0123456789abcdef";
  std::string s;
  for (size_t i = 0; i < n; i++) { s += H[p[i] >> 4]; s += H[p[i] & 15]; }
  return s;
}

bool history(const uint8_t* doc, size_t len, std::vector<Bytes>& out, std::vector<std::vector<uint8_t>>& hashes, HErr& e) {
  auto fail = [&](uint32_t code, const std::string& m) { e.code = code; e.msg = m; return false; };
  Rd d{doc, len};
  const uint8_t* magic = d.raw(4);
  if (d.bad || memcmp(magic, "\x85\x6f\x4a\x83", 4) != 0) return fail(AM_E_MAGIC, "Data does not begin with magic bytes 85 6f 4a 83");
  d.raw(4);
  const uint8_t type = *d.raw(1);
  const uint64_t clen = d.u();
  const uint8_t* body = d.raw(clen);
  if (d.bad) return fail(AM_E_SUBARRAY, "subarray exceeds buffer size");
  if (type != 0) return fail(AM_E_CHUNK_TYPE, "Unexpected chunk type: " + std::to_string(type));
  Rd r{body, clen};
  std::vector<std::string> actors;
  const uint64_t na = r.u();
  for (uint64_t i = 0; i < na && !r.bad; i++) { const uint64_t L = r.u(); const uint8_t* q = r.raw(L); actors.push_back(hex(q, L)); }
  std::vector<std::string> heads;
  const uint64_t nh = r.u();
  for (uint64_t i = 0; i < nh && !r.bad; i++) heads.push_back(hex(r.raw(32), 32));
  std::vector<Col> cc, oc;
  for (auto* cols : {&cc, &oc}) {
    const uint64_t n = r.u();
    for (uint64_t i = 0; i < n && !r.bad; i++) {
      Col c;
      c.id = (uint32_t)r.u();
      const uint64_t l = r.u();
      if (l > len) { r.bad = true; break; }  // a column cannot be longer than the chunk
      c.b.resize(l);
      cols->push_back(std::move(c));
    }
  }
  for (auto* cols : {&cc, &oc})
    for (auto& c : *cols) {
      const uint8_t* q = r.raw(c.b.size());
      if (r.bad) return fail(AM_E_SUBARRAY, "subarray exceeds buffer size");
      memcpy(c.b.data(), q, c.b.size());
      if (c.id & 8) {
        std::vector<uint8_t> z;
        if (!inflate_col(c.b, z)) return fail(AM_E_SUBARRAY, "invalid deflate data");
        c.b.swap(z);
        c.id &= ~8u;
      }
    }
  if (r.bad) return fail(AM_E_SUBARRAY, "subarray exceeds buffer size");
  auto col = [](const std::vector<Col>& cs, uint32_t id) -> const std::vector<uint8_t>& {
    static const std::vector<uint8_t> empty;
    for (auto& c : cs) if (c.id == id) return c.b;
    return empty;
  };
  static const uint32_t kChg[] = {0x01, 0x03, 0x13, 0x23, 0x35, 0x40, 0x43, 0x56, 0x57};
  static const uint32_t kOps[] = {0x01, 0x02, 0x11, 0x13, 0x15, 0x21, 0x23, 0x34, 0x42, 0x56, 0x57, 0x61, 0x63, 0x80, 0x81, 0x83};
  for (auto& c : cc) if (std::find(std::begin(kChg), std::end(kChg), c.id) == std::end(kChg)) return fail(AM_U_UNKNOWN_COLUMN, "automerge_amd: unsupported: column id outside the known column set");
  for (auto& c : oc) if (std::find(std::begin(kOps), std::end(kOps), c.id) == std::end(kOps)) return fail(AM_U_UNKNOWN_COLUMN, "automerge_amd: unsupported: column id outside the known column set");
  bool bad = false;
  // change rows (DOCUMENT_COLUMNS); row count from the longest column
  auto c_actor = dec_rle(col(cc, 0x01), 0, 0, bad);
  const size_t NC = c_actor.size();
  auto c_seq = dec_delta(col(cc, 0x03), NC, bad), c_max = dec_delta(col(cc, 0x13), NC, bad), c_time = dec_delta(col(cc, 0x23), NC, bad);
  auto c_msg = dec_rle(col(cc, 0x35), 2, NC, bad), c_dn = dec_rle(col(cc, 0x40), 0, NC, bad);
  auto c_el = dec_rle(col(cc, 0x56), 0, NC, bad);
  std::vector<Val> c_di;
  {
    size_t nd = 0;
    for (size_t i = 0; i < NC; i++) nd += c_dn[i].null ? 0 : (size_t)c_dn[i].i;
    c_di = dec_delta(col(cc, 0x43), nd, bad);
  }
  const std::vector<uint8_t>& c_er = col(cc, 0x57);
  // op rows (DOC_OPS_COLUMNS)
  auto o_oa = dec_rle(col(oc, 0x01), 0, 0, bad);
  auto o_ic = dec_delta(col(oc, 0x23), 0, bad);
  const size_t NO = std::max(o_oa.size(), o_ic.size());
  o_oa.resize(std::max(o_oa.size(), NO));
  auto o_oc = dec_rle(col(oc, 0x02), 0, NO, bad), o_ka = dec_rle(col(oc, 0x11), 0, NO, bad);
  auto o_kc = dec_delta(col(oc, 0x13), NO, bad), o_ks = dec_rle(col(oc, 0x15), 2, NO, bad);
  auto o_ia = dec_rle(col(oc, 0x21), 0, NO, bad);
  auto o_ins = dec_bool(col(oc, 0x34), NO, bad);
  auto o_act = dec_rle(col(oc, 0x42), 0, NO, bad), o_vl = dec_rle(col(oc, 0x56), 0, NO, bad);
  auto o_sn = dec_rle(col(oc, 0x80), 0, NO, bad);
  if (!col(oc, 0x61).empty() || !col(oc, 0x63).empty()) return fail(AM_U_VALUE, "automerge_amd: unsupported: link operations in a document history");
  size_t ns = 0;
  for (size_t i = 0; i < NO; i++) ns += o_sn[i].null ? 0 : (size_t)o_sn[i].i;
  auto o_sa = dec_rle(col(oc, 0x81), 0, ns, bad), o_sc = dec_delta(col(oc, 0x83), ns, bad);
  if (bad) return fail(AM_E_LEB_INCOMPLETE, "buffer ended with incomplete number");
  auto actor_ok = [&](const Val& v) { return !v.null && v.i >= 0 && (uint64_t)v.i < actors.size(); };
  // groupChangeOps (columnar.js:876-943)
  std::vector<HOp> pool;
  pool.reserve(NO + ns);
  std::unordered_map<uint64_t, int> by_id;  // (ctr << 16 | actor) -> pool index
  auto key_of = [](int64_t ctr, int a) { return ((uint64_t)ctr << 16) | (uint64_t)(a & 0xffff); };
  if (actors.size() > 0xffff) return fail(AM_U_VALUE, "automerge_amd: too many actors");
  const std::vector<uint8_t>& vr = col(oc, 0x57);
  size_t vpos = 0, spos = 0;
  std::vector<int> doc_order, dels;
  for (size_t i = 0; i < NO; i++) {
    HOp op{};
    if (o_ic[i].null || !actor_ok(o_ia[i]) || o_act[i].null) return fail(AM_U_VALUE, "automerge_amd: unsupported value shape in the input columns");
    op.id_ctr = o_ic[i].i;
    op.id_actor = (int)o_ia[i].i;
    op.obj_actor = o_oa[i].null ? -1 : (int)o_oa[i].i;
    op.obj_ctr = o_oc[i].null ? 0 : o_oc[i].i;
    if (op.obj_actor >= (int)actors.size()) return fail(AM_E_NO_ACTOR_INDEX, "No actor index " + std::to_string(op.obj_actor));
    op.has_key = !o_ks[i].null;
    if (op.has_key) op.key = o_ks[i].s;
    else {
      op.elem_ctr = o_kc[i].null ? 0 : o_kc[i].i;
      op.elem_actor = o_ka[i].null ? -1 : (int)o_ka[i].i;
      if (op.elem_actor >= (int)actors.size()) return fail(AM_E_NO_ACTOR_INDEX, "No actor index " + std::to_string(op.elem_actor));
    }
    op.insert = o_ins[i];
    op.action = o_act[i].i;
    if (op.action == 3) return fail(AM_U_VALUE, "document should not contain del operations");
    op.val_len = o_vl[i].null ? 0 : o_vl[i].i;
    const size_t vn = (size_t)(op.val_len >> 4);
    if (vpos + vn > vr.size()) return fail(AM_E_SUBARRAY, "subarray exceeds buffer size");
    op.val_raw.assign((const char*)vr.data() + vpos, vn);
    vpos += vn;
    const uint64_t k = key_of(op.id_ctr, op.id_actor);
    auto it = by_id.find(k);
    int me;
    if (it != by_id.end()) {  // op.pred = opsById[op.id].pred (a succ seen earlier created the entry)
      HOp& prev = pool[it->second];
      op.pred = prev.pred;
      if (prev.action == 3) {  // replaces the placeholder del in place (opsById[op.id] = op)
        pool[it->second] = op;
        me = it->second;
        dels.erase(std::find(dels.begin(), dels.end(), me));
      } else {
        me = (int)pool.size();
        pool.push_back(op);
        it->second = me;
      }
    } else {
      me = (int)pool.size();
      pool.push_back(op);
      by_id[k] = me;
    }
    doc_order.push_back(me);
    const int64_t nsu = o_sn[i].null ? 0 : o_sn[i].i;
    for (int64_t q = 0; q < nsu; q++, spos++) {
      if (spos >= ns || !actor_ok(o_sa[spos]) || o_sc[spos].null) return fail(AM_U_VALUE, "automerge_amd: unsupported value shape in the input columns");
      const uint64_t sk = key_of(o_sc[spos].i, (int)o_sa[spos].i);
      auto st = by_id.find(sk);
      int si;
      if (st == by_id.end()) {
        HOp dl{};
        dl.id_ctr = o_sc[spos].i;
        dl.id_actor = (int)o_sa[spos].i;
        dl.obj_ctr = pool[me].obj_ctr;
        dl.obj_actor = pool[me].obj_actor;
        dl.has_key = pool[me].has_key;
        dl.key = pool[me].key;
        if (!dl.has_key) {
          dl.elem_ctr = pool[me].insert ? pool[me].id_ctr : pool[me].elem_ctr;
          dl.elem_actor = pool[me].insert ? pool[me].id_actor : pool[me].elem_actor;
        }
        dl.insert = false;
        dl.action = 3;
        dl.val_len = 0;
        si = (int)pool.size();
        pool.push_back(dl);
        by_id[sk] = si;
        dels.push_back(si);
      } else {
        si = st->second;
      }
      pool[si].pred.push_back({pool[me].id_ctr, pool[me].id_actor});
    }
  }
  // changes by actor, seq / maxOp checks (:877-888)
  std::vector<HChange> ch(NC);
  std::vector<std::vector<int>> by_actor(actors.size());
  size_t dpos = 0, epos = 0;
  for (size_t i = 0; i < NC; i++) {
    HChange& c = ch[i];
    if (!actor_ok(c_actor[i]) || c_seq[i].null || c_max[i].null) return fail(AM_U_VALUE, "automerge_amd: unsupported value shape in the input columns");
    c.actor = (int)c_actor[i].i;
    c.seq = c_seq[i].i;
    c.max_op = c_max[i].i;
    c.time = c_time[i].null ? 0 : c_time[i].i;
    c.message = c_msg[i].null ? std::string() : c_msg[i].s;
    const int64_t ndp = c_dn[i].null ? 0 : c_dn[i].i;
    for (int64_t q = 0; q < ndp; q++, dpos++) c.deps_idx.push_back(c_di[dpos].null ? -1 : c_di[dpos].i);
    const int64_t el = c_el[i].null ? 0 : c_el[i].i;
    if ((el & 0x0f) != 7 && !c_el[i].null) return fail(AM_E_HISTORY, "Bad datatype for extra bytes: 7");
    const size_t en = (size_t)(el >> 4);
    if (epos + en > c_er.size()) return fail(AM_E_SUBARRAY, "subarray exceeds buffer size");
    c.extra.assign((const char*)c_er.data() + epos, en);
    epos += en;
    auto& lst = by_actor[c.actor];
    if (c.seq != (int64_t)lst.size() + 1)
      return fail(AM_E_HISTORY, "Expected seq = " + std::to_string(lst.size() + 1) + ", got " + std::to_string(c.seq));
    if (c.seq > 1 && ch[lst[c.seq - 2]].max_op > c.max_op) return fail(AM_E_HISTORY, "maxOp must increase monotonically per actor");
    lst.push_back((int)i);
  }
  // ops (document order, then the re-created deletions in creation order) -> changes
  std::vector<int> all = doc_order;
  all.insert(all.end(), dels.begin(), dels.end());
  for (int k : all) {
    const HOp& op = pool[k];
    auto& lst = by_actor[op.id_actor];
    size_t lo = 0, hi = lst.size();
    while (lo < hi) {
      const size_t m = (lo + hi) / 2;
      if (ch[lst[m]].max_op < op.id_ctr) lo = m + 1; else hi = m;
    }
    if (lo >= lst.size())
      return fail(AM_E_HISTORY, "Operation ID " + std::to_string(op.id_ctr) + "@" + actors[op.id_actor] + " outside of allowed range");
    ch[lst[lo]].ops.push_back(k);
  }
  // decodeDocumentChanges (:945-981): deps, hashes in order, heads check
  std::map<std::string, bool> headset;
  out.clear();
  hashes.clear();
  for (size_t i = 0; i < NC; i++) {
    HChange& c = ch[i];
    std::sort(c.ops.begin(), c.ops.end(), [&](int a, int b) { return pool[a].id_ctr < pool[b].id_ctr; });
    const int64_t start = c.max_op - (int64_t)c.ops.size() + 1;
    for (size_t q = 0; q < c.ops.size(); q++)
      if (pool[c.ops[q]].id_ctr != start + (int64_t)q || pool[c.ops[q]].id_actor != c.actor)
        return fail(AM_E_HISTORY, "Expected opId " + std::to_string(start + (int64_t)q) + "@" + actors[c.actor] + ", got " +
                                      std::to_string(pool[c.ops[q]].id_ctr) + "@" + actors[pool[c.ops[q]].id_actor]);
    std::vector<std::vector<uint8_t>> deps;
    for (int64_t di : c.deps_idx) {
      if (di < 0 || (size_t)di >= i || ch[di].hash.empty())
        return fail(AM_E_HISTORY, "No hash for index " + std::to_string(di) + " while processing index " + std::to_string(i));
      deps.push_back(ch[di].hash);
      headset.erase(hex(ch[di].hash.data(), 32));
    }
    uint8_t h[32];
    Bytes b = encode(c, pool, actors, deps, start, h);
    c.hash.assign(h, h + 32);
    headset[hex(h, 32)] = true;
    out.push_back(deflate_change(std::move(b)));
    hashes.push_back(c.hash);
  }
  std::vector<std::string> actual;
  for (auto& kv : headset) actual.push_back(kv.first);
  std::vector<std::string> expect = heads;
  if (actual != expect) {
    std::string a, x;
    for (size_t i = 0; i < expect.size(); i++) x += (i ? ", " : "") + expect[i];
    for (size_t i = 0; i < actual.size(); i++) a += (i ? ", " : "") + actual[i];
    return fail(AM_E_HISTORY, "Mismatched heads hashes: expected " + x + ", got " + a);
  }
  return true;
}

}  // namespace

extern "C" int am_document_changes(const uint8_t* doc, size_t len, uint8_t** out, uint64_t** offs, uint8_t** hashes32,
                                   size_t* nchanges, am_error* err) {
  std::vector<Bytes> ch;
  std::vector<std::vector<uint8_t>> hs;
  HErr e;
  bool ok;
  try {
    ok = history(doc, len, ch, hs, e);
  } catch (const std::exception&) {  // allocation failure on hostile input: never across the C ABI
    ok = false;
    e.code = AM_U_CAPACITY;
    e.msg = "automerge_amd: document history exceeds the host memory limits";
  }
  if (!ok) {
    if (err) {
      err->code = e.code;
      err->is_type_error = 0;
      snprintf(err->message, sizeof(err->message), "%s", e.msg.c_str());
    }
    return 1;
  }
  size_t total = 0;
  for (auto& c : ch) total += c.size();
  *out = (uint8_t*)malloc(total ? total : 1);
  *offs = (uint64_t*)malloc(sizeof(uint64_t) * (ch.size() + 1));
  *hashes32 = (uint8_t*)malloc(32 * (ch.size() ? ch.size() : 1));
  if (!*out || !*offs || !*hashes32) {
    if (err) { err->code = AM_U_CAPACITY; snprintf(err->message, sizeof(err->message), "automerge_amd: out of host memory"); }
    return 1;
  }
  size_t o = 0;
  for (size_t i = 0; i < ch.size(); i++) {
    (*offs)[i] = o;
    if (!ch[i].empty()) memcpy(*out + o, ch[i].data(), ch[i].size());
    o += ch[i].size();
    memcpy(*hashes32 + 32 * i, hs[i].data(), 32);
  }
  (*offs)[ch.size()] = o;
  *nchanges = ch.size();
  if (err) err->code = 0;
  return 0;
}
