// am_change_enc.h -- encodeChange (columnar.js:710-739) of one change given as ops with actor
// indexes, and deflateChange (:798-808). Shared by the history reconstruction (am_history.cpp,
// computeHashGraph) and the local-change encoder (am_local.cpp, applyLocalChange). Host code.
#pragma once
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#include <zlib.h>

#include "am_host_codec.h"

namespace {

struct OpId { int64_t ctr; int actor; };  // actor: index into the document's actor table
struct HOp {
  int64_t id_ctr; int id_actor;
  int64_t obj_ctr; int obj_actor;         // obj_actor -1: _root
  bool has_key; std::string key;          // map key
  int64_t elem_ctr; int elem_actor;       // list: elemId (elem_actor -1: _head)
  bool insert;
  int64_t action;
  int64_t val_len; std::string val_raw;
  std::vector<OpId> pred;
  int64_t child_ctr = 0; int child_actor = -1;  // chldActor / chldCtr (null when child_actor < 0)
  bool key_elem_actor = false;            // elem_actor names an actor although the op has a key
};
struct HChange {
  int actor; int64_t seq, max_op, time;
  std::string message;
  std::vector<int64_t> deps_idx;
  std::string extra;
  std::vector<int> ops;                   // indexes into the op pool
  std::vector<uint8_t> hash;
};

// encodeChange (columnar.js:710-739) of one reconstructed change
Bytes encode(const HChange& c, const std::vector<HOp>& pool, const std::vector<std::string>& actors,
             const std::vector<std::vector<uint8_t>>& deps, int64_t start_op, uint8_t hash[32]) {
  // parseAllOpIds(single): the author first, then every other referenced actor in string order
  std::vector<int> others;
  auto add = [&](int a) { if (a >= 0 && a != c.actor && std::find(others.begin(), others.end(), a) == others.end()) others.push_back(a); };
  for (int k : c.ops) {
    const HOp& op = pool[k];
    add(op.obj_actor);
    if (!op.has_key || op.key_elem_actor) add(op.elem_actor);
    add(op.child_actor);
    for (auto& p : op.pred) add(p.actor);
  }
  std::sort(others.begin(), others.end(), [&](int a, int b) { return actors[a] < actors[b]; });
  auto num = [&](int a) -> int64_t { return a == c.actor ? 0 : 1 + (std::find(others.begin(), others.end(), a) - others.begin()); };
  std::vector<V> objA, objC, keyA, keyC, keyS, act, vlen, predN, predA, predC, chA, chC;
  std::vector<bool> ins;
  Bytes vraw;
  for (int k : c.ops) {
    const HOp& op = pool[k];
    if (op.obj_actor < 0) { objA.push_back(N0()); objC.push_back(N0()); }
    else { objA.push_back(I(num(op.obj_actor))); objC.push_back(I(op.obj_ctr)); }
    if (op.has_key) { keyA.push_back(N0()); keyC.push_back(N0()); keyS.push_back(S(op.key)); }
    else if (op.elem_actor < 0) { keyA.push_back(N0()); keyC.push_back(I(0)); keyS.push_back(N0()); }
    else { keyA.push_back(I(num(op.elem_actor))); keyC.push_back(I(op.elem_ctr)); keyS.push_back(N0()); }
    ins.push_back(op.insert);
    act.push_back(I(op.action));
    vlen.push_back(I(op.val_len));
    vraw.insert(vraw.end(), op.val_raw.begin(), op.val_raw.end());
    if (op.child_actor >= 0 && op.child_ctr) { chA.push_back(I(num(op.child_actor))); chC.push_back(I(op.child_ctr)); }
    else { chA.push_back(N0()); chC.push_back(N0()); }
    std::vector<OpId> pr = op.pred;
    std::sort(pr.begin(), pr.end(), [&](const OpId& a, const OpId& b) {  // compareParsedOpIds
      if (a.ctr != b.ctr) return a.ctr < b.ctr;
      return actors[a.actor] < actors[b.actor];
    });
    predN.push_back(I((int64_t)pr.size()));
    for (auto& p : pr) { predA.push_back(I(num(p.actor))); predC.push_back(I(p.ctr)); }
  }
  struct C2 { int id; Bytes b; };
  std::vector<C2> cols = {{0x01, rle(objA, 0)}, {0x02, rle(objC, 0)}, {0x11, rle(keyA, 0)}, {0x13, delta(keyC)},
                          {0x15, rle(keyS, 2)}, {0x34, boolean(ins)}, {0x42, rle(act, 0)}, {0x56, rle(vlen, 0)},
                          {0x57, vraw},       {0x61, rle(chA, 0)}, {0x63, delta(chC)}, {0x70, rle(predN, 0)},
                          {0x71, rle(predA, 0)}, {0x73, delta(predC)}};
  Bytes body;
  std::vector<std::vector<uint8_t>> ds = deps;
  std::sort(ds.begin(), ds.end());
  pu(body, ds.size());
  for (auto& d : ds) body.insert(body.end(), d.begin(), d.end());
  auto hexbytes = [&](const std::string& h) {
    Bytes o;
    for (size_t i = 0; i + 1 < h.size(); i += 2) o.push_back((uint8_t)strtoul(h.substr(i, 2).c_str(), nullptr, 16));
    return o;
  };
  Bytes a0 = hexbytes(actors[c.actor]);
  pu(body, a0.size());
  body.insert(body.end(), a0.begin(), a0.end());
  pu(body, (uint64_t)c.seq);
  pu(body, (uint64_t)start_op);
  ps(body, c.time);
  pu(body, c.message.size());
  body.insert(body.end(), c.message.begin(), c.message.end());
  pu(body, others.size());
  for (int a : others) { Bytes ab = hexbytes(actors[a]); pu(body, ab.size()); body.insert(body.end(), ab.begin(), ab.end()); }
  size_t ne = 0;
  for (auto& x : cols) ne += !x.b.empty();
  pu(body, ne);
  for (auto& x : cols) if (!x.b.empty()) { pu(body, x.id); pu(body, x.b.size()); }
  for (auto& x : cols) body.insert(body.end(), x.b.begin(), x.b.end());
  body.insert(body.end(), c.extra.begin(), c.extra.end());
  return container(1, body, hash);
}

// deflateChange (columnar.js:798-808)
Bytes deflate_change(Bytes b) {
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

}  // namespace
