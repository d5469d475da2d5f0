// am_graph.h -- the change hash graph of a document (host side of libautomerge_amd.so).
//
// The reference keeps, per BackendDoc, changeIndexByHash / dependenciesByHash / dependentsByHash /
// hashesByActor / clock (new.js:1694-1707, filled by applyChanges :1838-1850 and computeHashGraph
// :1879-1904) and answers getChanges / getChangesAdded / getChangeByHash / getMissingDeps over them
// (new.js:1913-2020). HashGraph is the same index over a document's change list, kept next to the
// engine document (am_doc) and extended as changes are committed. The traversal orders are part
// of the contract (callers send the changes in that order), so the queries below follow the
// reference's stack discipline exactly, duplicates included.
#pragma once
#include <stdint.h>
#include <string.h>

#include <functional>
#include <string>
#include <unordered_map>
#include <vector>

struct Hash32 {
  uint8_t b[32];
  bool operator==(const Hash32& o) const { return memcmp(b, o.b, 32) == 0; }
  bool operator<(const Hash32& o) const { return memcmp(b, o.b, 32) < 0; }
};
struct Hash32Hasher {
  size_t operator()(const Hash32& h) const {
    uint64_t x;
    memcpy(&x, h.b, 8);
    return (size_t)x;
  }
};

// decodeChangeMeta (columnar.js:768-811) without the hash: author, seq and deps of a change chunk
// (DEFLATE-compressed chunks are inflated first)
struct ChangeMeta {
  std::string actor;  // hex
  int64_t seq = 0;
  std::vector<Hash32> deps;
};
bool am_change_meta(const uint8_t* p, size_t n, ChangeMeta& m);

class HashGraph {
 public:
  std::vector<Hash32> hashes;                               // change i (history order)
  std::vector<ChangeMeta> meta;
  std::unordered_map<Hash32, size_t, Hash32Hasher> index;   // changeIndexByHash
  // dependentsByHash: every committed change, and every hash a committed change depends on
  std::unordered_map<Hash32, std::vector<Hash32>, Hash32Hasher> dependents;
  std::unordered_map<std::string, std::vector<Hash32>> by_actor;  // hashesByActor (seq - 1 -> hash)
  std::unordered_map<std::string, int64_t> clock;

  void clear();
  void add(const Hash32& h, const ChangeMeta& m);  // commit (new.js:1838-1850)
  size_t size() const { return hashes.size(); }
  int64_t find(const Hash32& h) const;             // -1 when unknown
  // getChanges(haveDeps) (new.js:1913-1966): change indexes in the reference's order; false with
  // `missing` set to the unknown hash ("hash not found")
  bool changes_since(const std::vector<Hash32>& have, const std::vector<Hash32>& heads, std::vector<size_t>& out,
                     Hash32& missing) const;
  // getChangesAdded (new.js:1971-1988): indexes of this graph's changes the other document does not
  // index (`known`: the other's changeIndexByHash, which for a loaded document without its hash
  // graph holds only its heads and the changes applied since)
  void added_since(const std::function<bool(const Hash32&)>& known, const std::vector<Hash32>& heads,
                   std::vector<size_t>& out) const;
};
