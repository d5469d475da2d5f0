// am_workload.cpp -- synthetic workloads of SURVEY.md §8(d) for bench.py (host-side data
// preparation, runs before any timed region; built as workload/libam_workload.so, outside the
// product library). Documents are generated from a seeded LCG
// (s = s*1664525 + 1013904223 mod 2^32, seed = document index) and encoded in the Automerge
// binary change format (columnar.js encodeChange/encodeContainer). The bytes are pinned by the
// SHA-256 digests in tests/golden/workload.json, which the reference's own encoder produced for
// the same specification (tests/golden/gen/make_fixtures.js: c4Doc, c2Doc).
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include <zlib.h>

#include "am_workload.h"
#include "../automerge_amd/csrc/am_host_codec.h"

namespace {

struct Actor { uint8_t b[16]; };
bool operator<(const Actor& a, const Actor& b) { return memcmp(a.b, b.b, 16) < 0; }
bool operator==(const Actor& a, const Actor& b) { return memcmp(a.b, b.b, 16) == 0; }

// one op of a generated change (only the shapes the workloads need)
struct Op {
  int obj;            // -1 root, else actor index (in `actors` of the document) with ctr obj_ctr
  int64_t obj_ctr;
  std::string key;    // map key (empty -> list op)
  int elem_actor;     // list: -1 = _head
  int64_t elem_ctr;
  bool insert;
  int action;         // 0 makeMap 1 set 2 makeList 5 inc ...
  int vtype;          // 0 null, 4 int, 6 utf8, 8 counter
  int64_t ival;
  std::string sval;
  std::vector<std::pair<int64_t, int>> pred;  // (ctr, doc actor index)
};

// encodeChange (columnar.js:710-739) for a change whose ops reference `doc_actors` indexes
Bytes encode_change(const std::vector<Actor>& doc_actors, int author, int64_t seq, int64_t start_op,
                    const std::vector<std::vector<uint8_t>>& deps_sorted, const std::vector<Op>& ops, uint8_t hash[32]) {
  // parseAllOpIds(single): author first, then the other referenced actors sorted
  std::vector<int> others;
  auto add = [&](int a) {
    if (a >= 0 && a != author && std::find(others.begin(), others.end(), a) == others.end()) others.push_back(a);
  };
  for (auto& op : ops) {
    if (op.obj >= 0) add(op.obj);
    if (op.elem_actor >= 0) add(op.elem_actor);
    for (auto& p : op.pred) add(p.second);
  }
  std::sort(others.begin(), others.end(), [&](int a, int b) { return doc_actors[a] < doc_actors[b]; });
  auto num = [&](int a) -> int64_t {
    if (a == author) return 0;
    return 1 + (std::find(others.begin(), others.end(), a) - others.begin());
  };
  std::vector<V> objA, objC, keyA, keyC, keyS, act, vlen, predN, predA, predC;
  std::vector<bool> ins;
  Bytes vraw;
  for (auto& op : ops) {
    if (op.obj < 0) { objA.push_back(N0()); objC.push_back(N0()); }
    else { objA.push_back(I(num(op.obj))); objC.push_back(I(op.obj_ctr)); }
    if (!op.key.empty()) { keyA.push_back(N0()); keyC.push_back(N0()); keyS.push_back(S(op.key)); }
    else if (op.elem_actor < 0) { keyA.push_back(N0()); keyC.push_back(I(0)); keyS.push_back(N0()); }
    else { keyA.push_back(I(num(op.elem_actor))); keyC.push_back(I(op.elem_ctr)); keyS.push_back(N0()); }
    ins.push_back(op.insert);
    act.push_back(I(op.action));
    if (op.vtype == 6) {
      vraw.insert(vraw.end(), op.sval.begin(), op.sval.end());
      vlen.push_back(I((int64_t)(op.sval.size() << 4) | 6));
    } else if (op.vtype == 4 || op.vtype == 8) {
      Bytes t;
      ps(t, op.ival);
      vraw.insert(vraw.end(), t.begin(), t.end());
      vlen.push_back(I((int64_t)(t.size() << 4) | op.vtype));
    } else {
      vlen.push_back(I(0));
    }
    auto pr = op.pred;
    std::sort(pr.begin(), pr.end(), [&](const std::pair<int64_t, int>& a, const std::pair<int64_t, int>& b) {
      if (a.first != b.first) return a.first < b.first;
      return doc_actors[a.second] < doc_actors[b.second];
    });
    predN.push_back(I((int64_t)pr.size()));
    for (auto& p : pr) { predA.push_back(I(num(p.second))); predC.push_back(I(p.first)); }
  }
  std::vector<V> chA(ops.size(), N0()), chC(ops.size(), N0());
  struct Col { int id; Bytes b; };
  std::vector<Col> cols = {{0x01, rle(objA, 0)}, {0x02, rle(objC, 0)}, {0x11, rle(keyA, 0)}, {0x13, delta(keyC)},
                           {0x15, rle(keyS, 2)}, {0x34, boolean(ins)}, {0x42, rle(act, 0)}, {0x56, rle(vlen, 0)},
                           {0x57, vraw},       {0x61, rle(chA, 0)}, {0x63, delta(chC)}, {0x70, rle(predN, 0)},
                           {0x71, rle(predA, 0)}, {0x73, delta(predC)}};
  Bytes body;
  pu(body, deps_sorted.size());
  for (auto& d : deps_sorted) body.insert(body.end(), d.begin(), d.end());
  pu(body, 16);
  body.insert(body.end(), doc_actors[author].b, doc_actors[author].b + 16);
  pu(body, (uint64_t)seq);
  pu(body, (uint64_t)start_op);
  ps(body, 0);   // time
  pu(body, 0);   // message ''
  pu(body, others.size());
  for (int a : others) { pu(body, 16); body.insert(body.end(), doc_actors[a].b, doc_actors[a].b + 16); }
  size_t ne = 0;
  for (auto& c : cols) ne += !c.b.empty();
  pu(body, ne);
  for (auto& c : cols) if (!c.b.empty()) { pu(body, c.id); pu(body, c.b.size()); }
  for (auto& c : cols) body.insert(body.end(), c.b.begin(), c.b.end());
  return container(1, body, hash);
}

uint32_t lcg(uint32_t& s) { s = s * 1664525u + 1013904223u; return s; }

void make_actors(uint32_t& s, int n, std::vector<Actor>& out) {
  while ((int)out.size() < n) {
    Actor a;
    for (int i = 0; i < 4; i++) {
      uint32_t x = lcg(s);
      a.b[4 * i] = x >> 24; a.b[4 * i + 1] = x >> 16; a.b[4 * i + 2] = x >> 8; a.b[4 * i + 3] = x;
    }
    if (std::find(out.begin(), out.end(), a) == out.end()) out.push_back(a);
  }
}

// Base document = save(loadChanges(init, [change0])) for the C4 first change: root 'items'
// (makeList, 1@a0) and 'title' = 'untitled' (2@a0). Encoded as BackendDoc.save() does.
Bytes c4_base_doc(const Actor& a0, const uint8_t h0[32], const Bytes& change0) {
  // change columns (DOCUMENT_COLUMNS): one row
  struct Col { int id; Bytes b; };
  std::vector<Col> cc = {{0x01, rle({I(0)}, 0)}, {0x03, delta({I(1)})}, {0x13, delta({I(2)})}, {0x23, delta({I(0)})},
                         {0x35, rle({S("")}, 2)}, {0x40, rle({I(0)}, 0)}, {0x43, {}}, {0x56, rle({I(7)}, 0)},
                         {0x57, {}}};
  std::vector<Col> oc = {{0x01, {}}, {0x02, {}}, {0x11, {}}, {0x13, {}},
                         {0x15, rle({S("items"), S("title")}, 2)}, {0x21, rle({I(0), I(0)}, 0)},
                         {0x23, delta({I(1), I(2)})}, {0x34, boolean({false, false})}, {0x42, rle({I(2), I(1)}, 0)},
                         {0x56, rle({I(0), I((8 << 4) | 6)}, 0)}, {0x57, Bytes{'u', 'n', 't', 'i', 't', 'l', 'e', 'd'}},
                         {0x61, {}}, {0x63, {}}, {0x80, rle({I(0), I(0)}, 0)}, {0x81, {}}, {0x83, {}}};
  Bytes body;
  pu(body, 1);
  pu(body, 16);
  body.insert(body.end(), a0.b, a0.b + 16);
  pu(body, 1);
  body.insert(body.end(), h0, h0 + 32);
  for (auto* cols : {&cc, &oc}) {
    size_t ne = 0;
    for (auto& c : *cols) ne += !c.b.empty();
    pu(body, ne);
    for (auto& c : *cols) if (!c.b.empty()) { pu(body, c.id); pu(body, c.b.size()); }
  }
  for (auto* cols : {&cc, &oc})
    for (auto& c : *cols) body.insert(body.end(), c.b.begin(), c.b.end());
  pu(body, 0);  // headsIndexes
  (void)change0;
  return container(0, body, nullptr);
}

struct DocOut {
  Bytes base;
  std::vector<Bytes> changes;
  uint64_t ops = 0;
};

// C4: 4 actors x 3 concurrent changes of 4 list inserts + 1 conflicting title set.
// The base document (change 0 saved) of document doc_index; s / actors / h0 continue the sequence.
Bytes c4_base_from(uint32_t& s, std::vector<Actor>& actors, uint8_t h0[32]) {
  make_actors(s, 4, actors);
  std::vector<Op> ops0 = {
      {-1, 0, "items", -1, 0, false, 2, 0, 0, "", {}},
      {-1, 0, "title", -1, 0, false, 1, 6, 0, "untitled", {}},
  };
  Bytes change0 = encode_change(actors, 0, 1, 1, {}, ops0, h0);
  return c4_base_doc(actors[0], h0, change0);
}
Bytes c4_base(uint32_t doc_index) {
  uint32_t s = doc_index;
  std::vector<Actor> actors;
  uint8_t h0[32];
  return c4_base_from(s, actors, h0);
}
void gen_c4(uint32_t doc_index, DocOut& out) {
  uint32_t s = doc_index;
  std::vector<Actor> actors;
  const int A0 = 0;
  uint8_t h0[32];
  out.base = c4_base_from(s, actors, h0);
  std::vector<std::vector<Bytes>> ch(4);
  for (int i = 0; i < 4; i++) {
    std::vector<uint8_t> last(h0, h0 + 32);
    int64_t last_title_ctr = 2;
    int last_title_actor = A0;
    std::vector<int64_t> own;
    int64_t seq_base = i == 0 ? 2 : 1;
    for (int j = 0; j < 3; j++) {
      int64_t start = 3 + 5 * j;
      std::vector<Op> ops;
      int ref_actor = -1;
      int64_t ref_ctr = 0;
      if (!own.empty()) {  // JS: (own.length === 0 || r() % 4 === 0) ? '_head' : own[r() % own.length]
        if (lcg(s) % 4 != 0) { ref_ctr = own[lcg(s) % own.size()]; ref_actor = i; }
      }
      for (int k = 0; k < 4; k++) {
        char c = (char)(97 + lcg(s) % 26);
        ops.push_back({A0, 1, "", ref_actor, ref_ctr, true, 1, 6, 0, std::string(1, c), {}});
        own.push_back(start + k);
        ref_actor = i;
        ref_ctr = start + k;
      }
      std::string title = "t" + std::to_string(i) + "." + std::to_string(j) + "." + std::to_string(lcg(s) % 1000);
      ops.push_back({-1, 0, "title", -1, 0, false, 1, 6, 0, title, {{last_title_ctr, last_title_actor}}});
      last_title_ctr = start + 4;
      last_title_actor = i;
      uint8_t h[32];
      Bytes b = encode_change(actors, i, seq_base + j, start, {last}, ops, h);
      last.assign(h, h + 32);
      ch[i].push_back(std::move(b));
    }
  }
  for (int j = 0; j < 3; j++)
    for (int i = 0; i < 4; i++) out.changes.push_back(ch[i][j]);
  out.ops = 60;
}

// C5 (SURVEY.md §8(d), configs[4]): one document pair = the C4 base document plus two concurrent
// chains of `per_side` changes (actor 1 for side A, actor 2 for side B; each change 4 list inserts
// + 1 conflicting title set, as C4's), so each side holds per_side changes the other lacks since
// their last sync (the base). changes = A's chain, then B's chain.
void gen_c5(uint32_t doc_index, uint32_t per_side, DocOut& out) {
  uint32_t s = doc_index ^ 0x5c5c5c5cu;
  std::vector<Actor> actors;
  uint8_t h0[32];
  out.base = c4_base_from(s, actors, h0);
  for (int i = 1; i <= 2; i++) {
    std::vector<uint8_t> last(h0, h0 + 32);
    int64_t last_title_ctr = 2;
    int last_title_actor = 0;
    std::vector<int64_t> own;
    for (uint32_t j = 0; j < per_side; j++) {
      const int64_t start = 3 + 5 * (int64_t)j;
      std::vector<Op> ops;
      int ref_actor = -1;
      int64_t ref_ctr = 0;
      if (!own.empty() && lcg(s) % 4 != 0) { ref_ctr = own[lcg(s) % own.size()]; ref_actor = i; }
      for (int k = 0; k < 4; k++) {
        const char c = (char)(97 + lcg(s) % 26);
        ops.push_back({0, 1, "", ref_actor, ref_ctr, true, 1, 6, 0, std::string(1, c), {}});
        own.push_back(start + k);
        ref_actor = i;
        ref_ctr = start + k;
      }
      std::string title = "s" + std::to_string(i) + "." + std::to_string(j) + "." + std::to_string(lcg(s) % 1000);
      ops.push_back({-1, 0, "title", -1, 0, false, 1, 6, 0, title, {{last_title_ctr, last_title_actor}}});
      last_title_ctr = start + 4;
      last_title_actor = i;
      uint8_t h[32];
      out.changes.push_back(encode_change(actors, i, 1 + (int64_t)j, start, {last}, ops, h));
      last.assign(h, h + 32);
    }
  }
  out.ops = 10ull * per_side;
}

// C2 (SURVEY.md §8(d), configs[1]): change 1 by actor 0 sets k0..k7 (int), a counter 'count' and a
// string 'name'; two concurrent changes (actors 1, 2) increment the counter and overwrite k1.
// JS generator: tests/golden/gen/make_fixtures.js c2Doc (same LCG call order).
void gen_c2(uint32_t doc_index, DocOut& out) {
  uint32_t s = doc_index;
  std::vector<Actor> actors;
  make_actors(s, 3, actors);
  std::vector<Op> ops;
  for (int k = 0; k < 8; k++)
    ops.push_back({-1, 0, "k" + std::to_string(k), -1, 0, false, 1, 4, (int64_t)(lcg(s) % 100000), "", {}});
  ops.push_back({-1, 0, "count", -1, 0, false, 1, 8, (int64_t)(lcg(s) % 100), "", {}});
  ops.push_back({-1, 0, "name", -1, 0, false, 1, 6, 0, "doc-" + std::to_string(doc_index), {}});
  uint8_t h1[32];
  out.changes.push_back(encode_change(actors, 0, 1, 1, {}, ops, h1));
  for (int i = 1; i <= 2; i++) {
    std::vector<Op> o2;
    o2.push_back({-1, 0, "count", -1, 0, false, 5, 4, (int64_t)(1 + lcg(s) % 9), "", {{9, 0}}});
    o2.push_back({-1, 0, "k1", -1, 0, false, 1, 4, (int64_t)(lcg(s) % 100000), "", {{2, 0}}});
    uint8_t h[32];
    out.changes.push_back(encode_change(actors, i, 1, 11, {std::vector<uint8_t>(h1, h1 + 32)}, o2, h));
  }
  out.ops = 14;
}

// deflateChange (columnar.js:798-808): chunks of >= DEFLATE_MIN_SIZE (256) bytes become type 2
// with the chunk data raw-DEFLATEd (pako.deflateRaw defaults = zlib level 6, memLevel 8, wbits
// -15); the magic bytes and the checksum of the uncompressed chunk are kept.
Bytes maybe_deflate(Bytes b) {
  if (b.size() < 256) return b;
  size_t p = 9;
  while (b[p] & 0x80) p++;
  p++;
  z_stream zs;
  memset(&zs, 0, sizeof zs);
  if (deflateInit2(&zs, 6, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY) != Z_OK) return b;
  Bytes z(deflateBound(&zs, b.size() - p) + 16);
  zs.next_in = b.data() + p;
  zs.avail_in = (uInt)(b.size() - p);
  zs.next_out = z.data();
  zs.avail_out = (uInt)z.size();
  const int r = deflate(&zs, Z_FINISH);
  const size_t zn = zs.total_out;
  deflateEnd(&zs);
  if (r != Z_STREAM_END) return b;
  Bytes o(b.begin(), b.begin() + 8);
  o.push_back(2);
  pu(o, zn);
  o.insert(o.end(), z.begin(), z.begin() + zn);
  return o;
}

// Text editing histories. Two actors A, B share one text object
// (change 0 by A: makeText at _root 'text' = 1@A). Changes alternate A, B, A, ... with
// `per_change` ops each. Every op is, with probability 1/5 (and a non-empty view), a delete of a
// random live element of the author's view (pred = [elemId]); otherwise an insert of one
// lowercase character. The first insert of a change goes after a random live element of the
// view (1/8: at the head), the following ones after the previous insert (typing).
// The author's view is its own changes plus the other actor's changes up to its last crossing:
// with cross_every > 0 each actor, at every cross_every-th change of its own, first absorbs all
// of the other's changes so far (deps = heads of the view; C3 "interleaved"); with
// cross_every == 0 the two actors never see each other (C1 "concurrent from the same base").
// startOp = 1 + the largest op counter in the view (Lamport). Changes >= 256 B are deflated.
// LCG call order per document (seed = doc index): make_actors(2); then per op one draw for
// del/insert, one for the delete's element, or (first insert of a change) one for head-or-not
// plus one for the element, then one for the character.
void gen_text(uint32_t doc_index, uint32_t nchanges, uint32_t per_change, uint32_t cross_every, DocOut& out) {
  uint32_t s = doc_index;
  std::vector<Actor> actors;
  make_actors(s, 2, actors);
  const int A0 = 0;
  uint8_t h0[32];
  out.changes.push_back(maybe_deflate(encode_change(actors, A0, 1, 1, {}, {{-1, 0, "text", -1, 0, false, 4, 0, 0, "", {}}}, h0)));
  struct Chg { std::vector<uint64_t> ins, del; int64_t last_op; std::vector<uint8_t> hash; };
  struct View {
    std::vector<uint64_t> live;                 // element ids (ctr << 1 | actor)
    std::unordered_map<uint64_t, uint32_t> at;  // element -> index in live
    std::vector<std::vector<uint8_t>> heads;
    int64_t maxop = 1;
    uint32_t absorbed = 0;                      // changes of the other actor in the view
    int64_t seq = 0;
    void add(uint64_t e) { at[e] = (uint32_t)live.size(); live.push_back(e); }
    void remove(uint64_t e) {
      auto it = at.find(e);
      if (it == at.end()) return;
      const uint32_t i = it->second;
      at.erase(it);
      const uint64_t last = live.back();
      live.pop_back();
      if (i < live.size()) { live[i] = last; at[last] = i; }
    }
  };
  View v[2];
  std::vector<Chg> hist[2];
  for (int a = 0; a < 2; a++) v[a].heads.push_back(std::vector<uint8_t>(h0, h0 + 32));
  v[0].seq = 1;
  for (uint32_t k = 1; k <= nchanges; k++) {
    const int a = (int)((k - 1) & 1), o = 1 - a;
    View& V = v[a];
    if (cross_every && (uint32_t)(hist[a].size() + 1) % cross_every == 0 && V.absorbed < hist[o].size()) {
      for (uint32_t j = V.absorbed; j < hist[o].size(); j++) {
        for (uint64_t e : hist[o][j].ins) V.add(e);
        for (uint64_t e : hist[o][j].del) V.remove(e);
        V.maxop = std::max(V.maxop, hist[o][j].last_op);
      }
      V.absorbed = (uint32_t)hist[o].size();
      // my last change is an ancestor of the other's latest iff the other absorbed all of mine
      std::vector<std::vector<uint8_t>> nh = {hist[o].back().hash};
      if (!(hist[a].empty() || v[o].absorbed == hist[a].size())) nh.push_back(hist[a].back().hash);
      V.heads = nh;
    }
    const int64_t start = V.maxop + 1;
    std::vector<Op> ops;
    Chg rec;
    bool have_ref = false;
    uint64_t ref = 0;
    for (uint32_t i = 0; i < per_change; i++) {
      const int64_t ctr = start + i;
      if (lcg(s) % 5 == 0 && !V.live.empty()) {
        const uint64_t e = V.live[lcg(s) % V.live.size()];
        ops.push_back({A0, 1, "", (int)(e & 1), (int64_t)(e >> 1), false, 3, 0, 0, "", {{(int64_t)(e >> 1), (int)(e & 1)}}});
        V.remove(e);
        rec.del.push_back(e);
      } else {
        if (!have_ref) {
          have_ref = true;
          if (lcg(s) % 8 == 0 || V.live.empty()) ref = 0;
          else ref = V.live[lcg(s) % V.live.size()];
        }
        const char c = (char)(97 + lcg(s) % 26);
        if (ref == 0) ops.push_back({A0, 1, "", -1, 0, true, 1, 6, 0, std::string(1, c), {}});
        else ops.push_back({A0, 1, "", (int)(ref & 1), (int64_t)(ref >> 1), true, 1, 6, 0, std::string(1, c), {}});
        const uint64_t e = ((uint64_t)ctr << 1) | (uint64_t)a;
        V.add(e);
        rec.ins.push_back(e);
        ref = e;
      }
    }
    std::vector<std::vector<uint8_t>> deps = V.heads;
    std::sort(deps.begin(), deps.end());
    uint8_t h[32];
    out.changes.push_back(maybe_deflate(encode_change(actors, a, ++V.seq, start, deps, ops, h)));
    rec.last_op = start + per_change - 1;
    rec.hash.assign(h, h + 32);
    V.maxop = rec.last_op;
    V.heads = {rec.hash};
    hist[a].push_back(std::move(rec));
  }
  out.ops = 1 + (uint64_t)nchanges * per_change;
}

// Mid-size documents (round-5 workload between C4's 62 and C3's 100k ops; VERDICT r4 Next 4):
// `nactors` actors edit one text and one title in `rounds` rounds of concurrent changes. Change 0
// (actor 0, seq 1): makeText at _root 'text' (1@A0), 'title' = 'mid' (2@A0). In round r every actor
// makes one change whose deps are all heads after round r-1 (change 0 for round 0): the round's
// changes are concurrent and the next round merges them. A change has min_ops + lcg % (max_ops -
// min_ops + 1) ops; each op is, by lcg % 20: 0-2 (with a live element in the view) a delete of a
// random live element; 3 a title set whose pred is every title op visible to the author; otherwise
// an insert of one lowercase character (the first insert of a change after a random live element,
// 1/8 at the head; the following ones after the previous insert). The author's view is the text
// after round r-1 plus its own ops of the change; startOp = 1 + the largest op counter of rounds
// < r. Changes >= 256 B are deflated as encodeChange writes them (columnar.js:738).
// LCG call order per document (seed = doc index ^ 0x6d1d0000): make_actors(nactors); per change
// one draw for the op count; per op one draw for the kind, one for a delete's element, (first
// insert) one for head-or-not plus one for the element, then one for the character; a title set
// draws one number for its value.
void gen_mid(uint32_t doc_index, uint32_t nactors, uint32_t rounds, uint32_t min_ops, uint32_t max_ops, DocOut& out) {
  uint32_t s = doc_index ^ 0x6d1d0000u;
  std::vector<Actor> actors;
  make_actors(s, (int)nactors, actors);
  uint8_t h0[32];
  out.changes.push_back(maybe_deflate(encode_change(
      actors, 0, 1, 1, {},
      {{-1, 0, "text", -1, 0, false, 4, 0, 0, "", {}}, {-1, 0, "title", -1, 0, false, 1, 6, 0, "mid", {}}}, h0)));
  uint64_t nops = 2;
  std::vector<uint64_t> live;                  // element ids (ctr << 8 | actor) after the last round
  std::vector<std::pair<int64_t, int>> title = {{2, 0}};  // visible title ops after the last round
  std::vector<std::vector<uint8_t>> heads = {std::vector<uint8_t>(h0, h0 + 32)};
  int64_t maxop = 2;
  std::vector<int64_t> seq(nactors, 0);
  seq[0] = 1;
  for (uint32_t r = 0; r < rounds; r++) {
    std::vector<uint64_t> ins_all, del_all;
    std::vector<std::pair<int64_t, int>> title_new, title_over;
    std::vector<std::vector<uint8_t>> round_heads;
    int64_t round_max = maxop;
    std::vector<std::vector<uint8_t>> deps = heads;
    std::sort(deps.begin(), deps.end());
    for (uint32_t a = 0; a < nactors; a++) {
      std::vector<uint64_t> view = live;  // the author's view: the text after round r-1 plus its own ops
      std::unordered_map<uint64_t, uint32_t> at;
      for (uint32_t i = 0; i < view.size(); i++) at[view[i]] = i;
      auto vremove = [&](uint64_t e) {
        auto it = at.find(e);
        if (it == at.end()) return;
        const uint32_t i = it->second;
        at.erase(it);
        const uint64_t last = view.back();
        view.pop_back();
        if (i < view.size()) { view[i] = last; at[last] = i; }
      };
      std::vector<std::pair<int64_t, int>> tvis = title;
      const uint32_t n = min_ops + lcg(s) % (max_ops - min_ops + 1);
      const int64_t start = maxop + 1;
      std::vector<Op> ops;
      bool have_ref = false;
      uint64_t ref = 0;
      for (uint32_t i = 0; i < n; i++) {
        const int64_t ctr = start + i;
        const uint32_t kind = lcg(s) % 20;
        if (kind < 3 && !view.empty()) {
          const uint64_t e = view[lcg(s) % view.size()];
          const int ea = (int)(e & 255);
          const int64_t ec = (int64_t)(e >> 8);
          ops.push_back({0, 1, "", ea, ec, false, 3, 0, 0, "", {{ec, ea}}});
          vremove(e);
          del_all.push_back(e);
        } else if (kind == 3) {
          const std::string t = "m" + std::to_string(a) + "." + std::to_string(lcg(s) % 10000);
          ops.push_back({-1, 0, "title", -1, 0, false, 1, 6, 0, t, tvis});
          for (auto& p : tvis) title_over.push_back(p);
          tvis = {{ctr, (int)a}};
        } else {
          if (!have_ref) {
            have_ref = true;
            if (lcg(s) % 8 == 0 || view.empty()) ref = ~0ull;
            else ref = view[lcg(s) % view.size()];
          }
          const char c = (char)(97 + lcg(s) % 26);
          if (ref == ~0ull) ops.push_back({0, 1, "", -1, 0, true, 1, 6, 0, std::string(1, c), {}});
          else ops.push_back({0, 1, "", (int)(ref & 255), (int64_t)(ref >> 8), true, 1, 6, 0, std::string(1, c), {}});
          const uint64_t e = ((uint64_t)ctr << 8) | a;
          at[e] = (uint32_t)view.size();
          view.push_back(e);
          ins_all.push_back(e);
          ref = e;
        }
      }
      if (!tvis.empty() && tvis.size() == 1 && tvis[0].second == (int)a && tvis[0].first >= start) title_new.push_back(tvis[0]);
      uint8_t h[32];
      out.changes.push_back(maybe_deflate(encode_change(actors, (int)a, ++seq[a], start, deps, ops, h)));
      round_heads.push_back(std::vector<uint8_t>(h, h + 32));
      round_max = std::max(round_max, start + (int64_t)n - 1);
      nops += n;
    }
    // the merged state after the round
    std::unordered_map<uint64_t, bool> gone;
    for (uint64_t e : del_all) gone[e] = true;
    std::vector<uint64_t> nl;
    for (uint64_t e : live) if (!gone.count(e)) nl.push_back(e);
    for (uint64_t e : ins_all) if (!gone.count(e)) nl.push_back(e);
    live.swap(nl);
    std::vector<std::pair<int64_t, int>> nt;
    for (auto& p : title)
      if (std::find(title_over.begin(), title_over.end(), p) == title_over.end()) nt.push_back(p);
    for (auto& p : title_new) nt.push_back(p);
    title.swap(nt);
    heads = round_heads;
    maxop = round_max;
  }
  out.ops = nops;
}

// Lays out documents [base?][changes...] back to back in the arena
uint64_t layout(std::vector<DocOut>& outs, uint8_t* arena, uint64_t cap, am_chunk_desc* chunks, am_doc_desc* docs,
                uint64_t* ops_out) {
  uint64_t total = 0, ops = 0;
  for (auto& o : outs) {
    total += o.base.size();
    for (auto& c : o.changes) total += c.size();
    ops += o.ops;
  }
  if (ops_out) *ops_out = ops;
  if (!arena || cap < total) return total;
  uint64_t off = 0;
  uint32_t ci = 0;
  for (size_t d = 0; d < outs.size(); d++) {
    DocOut& o = outs[d];
    docs[d].base_chunk = -1;
    if (!o.base.empty()) {
      docs[d].base_chunk = ci;
      chunks[ci++] = {off, (uint32_t)o.base.size(), 0};
      memcpy(arena + off, o.base.data(), o.base.size());
      off += o.base.size();
    }
    docs[d].chg_begin = ci;
    docs[d].chg_count = (uint32_t)o.changes.size();
    docs[d].known_begin = 0;
    docs[d].known_count = 0;
    docs[d].flags = o.base.empty() ? 1u : 0u;  // fresh documents have the full hash graph
    docs[d].meta_chunk = 0;
    for (auto& c : o.changes) {
      chunks[ci++] = {off, (uint32_t)c.size(), 0};
      memcpy(arena + off, c.data(), c.size());
      off += c.size();
    }
  }
  return total;
}

// Generated documents of the last size query, reused by the fill call that follows it
struct Cache {
  uint64_t key = ~0ull;
  std::vector<DocOut> outs;
};
Cache g_cache;

template <class Gen>
uint64_t generate_ids(Gen gen, uint64_t key, const uint64_t* ids, uint64_t first, uint32_t n, uint8_t* arena, uint64_t cap,
                      am_chunk_desc* chunks, am_doc_desc* docs, uint64_t* ops_out, int nthreads) {
  if (g_cache.key != key || g_cache.outs.size() != n) {
    std::vector<DocOut> outs(n);
    if (nthreads < 1) nthreads = 1;
    std::vector<std::thread> th;
    for (int t = 0; t < nthreads; t++)
      th.emplace_back([&, t]() {
        for (uint32_t d = t; d < n; d += nthreads) gen((uint32_t)(ids ? ids[d] : first + d), outs[d]);
      });
    for (auto& x : th) x.join();
    g_cache.outs.swap(outs);
    g_cache.key = key;
  }
  const uint64_t need = layout(g_cache.outs, arena, cap, chunks, docs, ops_out);
  if (arena && cap >= need) {  // filled: release
    g_cache.key = ~0ull;
    std::vector<DocOut>().swap(g_cache.outs);
  }
  return need;
}
uint64_t mix_key(uint64_t kind, uint64_t a, uint64_t b, uint64_t c) {
  uint64_t h = kind * 0x9E3779B97F4A7C15ull;
  for (uint64_t v : {a, b, c}) h = (h ^ v) * 0xff51afd7ed558ccdull + 0x632be59bd9b4e5f1ull;
  return h;
}
template <class Gen>
uint64_t generate(Gen gen, uint64_t kind, uint64_t first, uint32_t n, uint8_t* arena, uint64_t cap, am_chunk_desc* chunks,
                  am_doc_desc* docs, uint64_t* ops_out, int nthreads) {
  return generate_ids(gen, mix_key(kind, first, n, 0), nullptr, first, n, arena, cap, chunks, docs, ops_out, nthreads);
}

}  // namespace

extern "C" {

/* Generates C4 documents [first, first + n): each = base document (change 0 saved) + 12 change
 * chunks. Returns the number of bytes needed; fills the outputs when `arena` is non-NULL and
 * cap suffices. chunks: n * 13 entries; docs: n entries. ops_out: total ops in the changes. */
uint64_t am_workload_c4(uint64_t first, uint32_t n, uint8_t* arena, uint64_t cap, am_chunk_desc* chunks, am_doc_desc* docs,
                        uint64_t* ops_out, int nthreads) {
  return generate(gen_c4, 4, first, n, arena, cap, chunks, docs, ops_out, nthreads);
}

/* C2: documents [first, first + n), each = Backend.init() + 3 change chunks (no base chunk). */
uint64_t am_workload_c2(uint64_t first, uint32_t n, uint8_t* arena, uint64_t cap, am_chunk_desc* chunks, am_doc_desc* docs,
                        uint64_t* ops_out, int nthreads) {
  return generate(gen_c2, 2, first, n, arena, cap, chunks, docs, ops_out, nthreads);
}

/* C5 document pairs [first, first + n) (gen_c5 above): base chunk + 2 * per_side change chunks
 * each (side A's chain, then side B's). */
uint64_t am_workload_c5(uint64_t first, uint32_t n, uint32_t per_side, uint8_t* arena, uint64_t cap, am_chunk_desc* chunks,
                        am_doc_desc* docs, uint64_t* ops_out, int nthreads) {
  auto gen = [=](uint32_t d, DocOut& o) { gen_c5(d, per_side, o); };
  return generate(gen, mix_key(5, per_side, 0, 0), first, n, arena, cap, chunks, docs, ops_out, nthreads);
}

/* Text editing histories (gen_text above; C1: cross_every 0, C3: cross_every 10): documents
 * [first, first + n), each = Backend.init() + (1 + nchanges) change chunks, deflated when
 * >= 256 B as encodeChange does. */
uint64_t am_workload_text(uint64_t first, uint32_t n, uint32_t nchanges, uint32_t per_change, uint32_t cross_every,
                          uint8_t* arena, uint64_t cap, am_chunk_desc* chunks, am_doc_desc* docs, uint64_t* ops_out,
                          int nthreads) {
  auto gen = [=](uint32_t d, DocOut& o) { gen_text(d, nchanges, per_change, cross_every, o); };
  return generate(gen, mix_key(10, nchanges, per_change, cross_every), first, n, arena, cap, chunks, docs, ops_out, nthreads);
}

/* Document sharding of the C4 job: the documents of [first, first + n) whose
 * base document's SHA-256 (its container checksum, columnar.js:659-686) has first byte % world ==
 * rank, in index order. Writes up to cap indexes; returns how many belong to the shard. */
/* Mid-size documents (gen_mid above): Backend.init() + 1 + nactors * rounds change chunks each. */
uint64_t am_workload_mid(uint64_t first, uint32_t n, uint32_t nactors, uint32_t rounds, uint32_t min_ops, uint32_t max_ops,
                         uint8_t* arena, uint64_t cap, am_chunk_desc* chunks, am_doc_desc* docs, uint64_t* ops, int nthreads) {
  if (nactors < 1 || nactors > 200 || max_ops < min_ops || min_ops < 1) return 0;
  auto gen = [=](uint32_t d, DocOut& o) { gen_mid(d, nactors, rounds, min_ops, max_ops, o); };
  return generate(gen, mix_key(6, nactors * 1000003ull + rounds, min_ops, max_ops), first, n, arena, cap, chunks, docs, ops,
                  nthreads);
}

uint64_t am_workload_c4_shard(uint64_t first, uint64_t n, uint32_t world, uint32_t rank, uint64_t* ids, uint64_t cap,
                              int nthreads) {
  if (world == 0) return 0;
  if (nthreads < 1) nthreads = 1;
  std::vector<uint8_t> mine(n, 0);
  std::vector<std::thread> th;
  for (int t = 0; t < nthreads; t++)
    th.emplace_back([&, t]() {
      for (uint64_t d = t; d < n; d += nthreads) {
        const Bytes base = c4_base((uint32_t)(first + d));
        mine[d] = base.size() > 4 && base[4] % world == rank;
      }
    });
  for (auto& x : th) x.join();
  uint64_t k = 0;
  for (uint64_t d = 0; d < n; d++)
    if (mine[d]) {
      if (ids && k < cap) ids[k] = first + d;
      k++;
    }
  return k;
}

/* C4 documents with the given indexes (am_workload_c4 over a list, e.g. one shard). */
uint64_t am_workload_c4_list(const uint64_t* ids, uint32_t n, uint8_t* arena, uint64_t cap, am_chunk_desc* chunks,
                             am_doc_desc* docs, uint64_t* ops_out, int nthreads) {
  const uint64_t key = mix_key(40, n ? ids[0] : 0, n, n ? ids[n - 1] : 0);
  return generate_ids(gen_c4, key, ids, 0, n, arena, cap, chunks, docs, ops_out, nthreads);
}

}  // extern "C"
