// Host check of the engine's getPatch scan: runs patch_scan (automerge_amd/csrc/am_patch.h, the code
// lane 0 of k_doc runs in phase P7) over documents decoded by the CPU oracle, and writes the
// binary patch logs; tests/test_patch_kernel_host.py materializes them with automerge_amd/patch.py
// and compares with the reference's getPatch output. Test infrastructure only.
//   patch_host <in: [u32 len][doc bytes]...> <out: [u32 len][patch log]...>
#include <cstdio>
#include <cstring>
#include <vector>

#include "../../oracle/am_oracle.h"
#include "../../automerge_amd/csrc/am_patch.h"

struct ExportSrc {
  const oc_export* e;
  const oc_op& op(uint32_t i) const { return e->ops[i]; }
  uint32_t n() const { return (uint32_t)e->nops; }
  int64_t obj_ctr(uint32_t i) const { return op(i).obj_ctr; }
  int32_t obj_actor(uint32_t i) const { return op(i).obj_actor; }
  bool has_key(uint32_t i) const { return op(i).key_len >= 0; }
  uint32_t key_len(uint32_t i) const { return (uint32_t)op(i).key_len; }
  bool key_eq(uint32_t i, uint32_t j) const {
    return op(i).key_len == op(j).key_len && std::memcmp(op(i).key, op(j).key, key_len(i)) == 0;
  }
  void copy_key(uint32_t i, uint8_t* d) const { std::memcpy(d, op(i).key, key_len(i)); }
  int64_t key_ctr(uint32_t i) const { return op(i).key_ctr; }
  int32_t key_actor(uint32_t i) const { return op(i).key_actor; }
  int64_t id_ctr(uint32_t i) const { return op(i).id_ctr; }
  int32_t id_actor(uint32_t i) const { return op(i).id_actor; }
  bool insert(uint32_t i) const { return op(i).insert != 0; }
  int64_t action(uint32_t i) const { return op(i).action; }
  int64_t val_len(uint32_t i) const { return op(i).val_len; }
  void copy_value(uint32_t i, uint8_t* d) const { std::memcpy(d, op(i).val, op(i).val_n); }
  // Decoder.readUint53 / readInt53 over the whole value (encoding.js)
  bool value_int(uint32_t i, bool is_uint, int64_t& out) const {
    const uint8_t* p = op(i).val;
    const uint32_t n = op(i).val_n;
    uint64_t v = 0;
    int sh = 0;
    uint32_t k = 0;
    for (;;) {
      if (k >= n || sh > 56) return false;
      const uint8_t b = p[k++];
      v |= (uint64_t)(b & 0x7f) << sh;
      sh += 7;
      if (!(b & 0x80)) break;
    }
    if (!is_uint && sh < 64 && (p[k - 1] & 0x40)) v |= ~(uint64_t)0 << sh;
    out = (int64_t)v;
    if (is_uint ? v > 0x1fffffffffffffull : (out > 0x1fffffffffffffll || out < -0x1fffffffffffffll)) return false;
    return true;
  }
  int64_t value_f64_bits(uint32_t i) const {
    int64_t b;
    std::memcpy(&b, op(i).val, 8);
    return b;
  }
  uint32_t nsucc(uint32_t i) const { return op(i).nsucc; }
  int64_t succ_ctr(uint32_t i, uint32_t k) const { return e->succ_ctr[op(i).succ_off + k]; }
  int32_t succ_actor(uint32_t i, uint32_t k) const { return e->succ_actor[op(i).succ_off + k]; }
  uint32_t nactors() const { return (uint32_t)e->nactors; }
  uint32_t actor_len(uint32_t a) const { return e->actor_lens[a]; }
  void copy_actor(uint32_t a, uint8_t* d) const { std::memcpy(d, e->actors[a], e->actor_lens[a]); }
  uint32_t nchg() const { return (uint32_t)e->nchg; }
  int64_t chg_actor(uint32_t c) const { return e->chg_actor[c]; }
  int64_t chg_seq(uint32_t c) const { return e->chg_seq[c]; }
};

int main(int argc, char** argv) {
  if (argc != 3) return 2;
  FILE* in = std::fopen(argv[1], "rb");
  FILE* out = std::fopen(argv[2], "wb");
  if (!in || !out) return 2;
  uint32_t len;
  while (std::fread(&len, 4, 1, in) == 1) {
    std::vector<uint8_t> doc(len);
    if (len && std::fread(doc.data(), 1, len, in) != len) return 3;
    char err[256];
    oc_export* e = oc_doc_export(doc.data(), len, err, sizeof err);
    if (!e) { std::fprintf(stderr, "decode: %s\n", err); return 4; }
    ExportSrc src{e};
    const uint32_t n = src.n();
    uint64_t heap = 0, nsucc = 0;
    for (uint32_t i = 0; i < n; i++) {
      heap += (src.has_key(i) ? src.key_len(i) : 0) + e->ops[i].val_n;
      nsucc += src.nsucc(i);
    }
    for (uint32_t a = 0; a < src.nactors(); a++) heap += src.actor_len(a);
    std::vector<PatchRec> rec(3 * (size_t)n + src.nactors() + src.nchg() + 2);
    std::vector<PatchVal> mval(n + 1);
    std::vector<uint8_t> hp(heap + 1);
    std::vector<int64_t> mk_ctr(n + 1), cs_ctr(n + 1), cs_val(n + 1), cm_ctr(nsucc + 1);
    std::vector<int32_t> mk_actor(n + 1), cs_actor(n + 1), cs_left(n + 1), cm_actor(nsucc + 1), cm_state(nsucc + 1);
    std::vector<uint8_t> mk_vis(n + 1);
    PatchOut o = {rec.data(), mval.data(), hp.data(), 0, 0, 0, rec.size(), mval.size(), hp.size(), 0, 0, 0};
    PatchScratch w = {mk_ctr.data(), mk_actor.data(), mk_vis.data(), n + 1, cs_ctr.data(), cs_actor.data(),
                      cs_val.data(), cs_left.data(), n + 1, cm_ctr.data(), cm_actor.data(), cm_state.data(),
                      (uint32_t)nsucc + 1};
    int64_t max_op = 0;
    patch_scan(src, o, w, max_op);
    // the wire form the device hands to the host (am_patch.h patch_pack)
    std::vector<uint8_t> wire(64 + 64 * rec.size() + 32 * mval.size() + hp.size());
    const uint32_t total = (uint32_t)patch_pack(o, max_op, wire.data(), wire.size());
    if (!total) return 5;
    std::fwrite(&total, 4, 1, out);
    std::fwrite(wire.data(), 1, total, out);
    oc_export_free(e);
  }
  std::fclose(out);
  return 0;
}
