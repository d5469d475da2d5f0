/*
 * am_oracle.h -- CPU restatement of the reference Automerge backend hot path.
 *
 * TEST INFRASTRUCTURE ONLY. This library is the parity checker for the MI355X engine. Only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it; the product
 * (automerge_amd/, libautomerge_amd.so) never links or calls it.
 *
 * It restates, sequentially and in plain C, what the reference computes:
 *   - LEB128/RLE/delta/boolean codecs with their canonical-form checks   backend/encoding.js
 *   - chunk containers, SHA-256 checksums/hashes, change + document decode backend/columnar.js
 *   - applyChanges (causal queue, seq rules, actor table, per-op merge:
 *     object order, UTF-16 key order, RGA skip rule, succ lists) and save() backend/new.js
 * Parity is pinned by tests/golden/ (JSON fixtures), which were produced by running the reference itself
 * (tests/golden/gen/make_fixtures.js); see tests/test_oracle.py.
 */
#ifndef AM_ORACLE_H
#define AM_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- codec entry points (known-answer tests against tests/golden/codecs.json) ---- */
/* fn: 0 appendUint32 1 appendInt32 2 appendUint53 3 appendInt53 4 appendUint64 5 appendInt64.
 * For 4/5, (hi, lo) are the two 32-bit halves as in encoding.js. Returns bytes written. */
int oc_leb_encode(int fn, int64_t value, int64_t hi, int64_t lo, uint8_t *out);
/* fn: 0 readUint32 1 readInt32 2 readUint53 3 readInt53 4 readUint64 5 readInt64.
 * Returns 0 on success (value in *v, or halves in hi and lo for fn 4 and 5), else 1 with message in err. */
int oc_leb_decode(int fn, const uint8_t *buf, size_t len, int64_t *v, int64_t *hi, int64_t *lo,
                  size_t *offset, char *err, size_t errcap);

/* Column value vectors. type: 0 uint (RLE), 1 int (RLE), 2 utf8 (RLE), 3 delta, 4 boolean.
 * ints: values; nulls: 1 = null. For utf8: strbuf holds concatenated UTF-8, strlen lengths. */
int oc_col_encode(int type, size_t n, const int64_t *ints, const uint8_t *nulls,
                  const uint8_t *strbuf, const uint32_t *strlens, uint8_t *out, size_t outcap,
                  size_t *outlen);
/* Decodes up to maxn values. Returns 0 ok / 1 error (message in err; values decoded so far kept). */
int oc_col_decode(int type, const uint8_t *buf, size_t len, size_t maxn, size_t *n, int64_t *ints,
                  uint8_t *nulls, uint8_t *strbuf, size_t strcap, uint32_t *strlens, char *err,
                  size_t errcap);

void oc_sha256(const uint8_t *data, size_t len, uint8_t out[32]);

/* ---- change decode ---- */
/* Decodes a binary change (chunk type 1 or 2). On success fills the hash (32 bytes), seq,
 * startOp, numOps and the dependency count. Returns 0 ok, 1 error (message in err). */
int oc_change_meta(const uint8_t *buf, size_t len, uint8_t hash[32], int64_t *seq,
                   int64_t *start_op, int64_t *num_ops, int64_t *num_deps, char *err, size_t errcap);

/* ---- backend document (init / load / applyChanges / save / getHeads) ---- */
typedef struct oc_doc oc_doc;
oc_doc *oc_doc_init(void);
/* Backend.load(buf). Returns NULL on error (message in err). */
oc_doc *oc_doc_load(const uint8_t *buf, size_t len, char *err, size_t errcap);
oc_doc *oc_doc_clone(const oc_doc *doc);
void oc_doc_free(oc_doc *doc);
/* Backend.applyChanges(doc, changes): atomic -- on error the doc is unchanged.
 * Returns 0 ok, 1 error (message in err), 2 unsupported by the oracle (e.g. needs the
 * deferred hash graph of a loaded document). */
int oc_doc_apply(oc_doc *doc, const uint8_t *const *bufs, const size_t *lens, size_t n, char *err,
                 size_t errcap);
/* Backend.save(doc): returns a malloc'd buffer (caller frees with oc_free). */
uint8_t *oc_doc_save(oc_doc *doc, size_t *len);
/* Heads (sorted), 32 bytes each; returns the count (writes at most cap heads). */
size_t oc_doc_heads(const oc_doc *doc, uint8_t *out, size_t cap);
size_t oc_doc_pending(const oc_doc *doc);
size_t oc_doc_num_ops(const oc_doc *doc);
int64_t oc_doc_max_op(const oc_doc *doc);
void oc_free(void *p);

/* Backend.getPatch(doc) as JSON text (malloc'd, free with oc_free); NULL on error (message in err) */
char *oc_doc_patch(const oc_doc *doc, char *err, size_t errcap);
/* Backend.applyChanges(doc, changes): applies like oc_doc_apply and returns the patch the
 * reference returns (maxOp, clock, deps, pendingChanges, diffs) as JSON text (malloc'd, free with
 * oc_free); NULL on error (message in err). am_apply_patch_oracle.inc. */
char *oc_doc_apply_patch(oc_doc *doc, const uint8_t *const *bufs, const size_t *lens, size_t n, char *err,
                         size_t errcap);

/* Flat export of a decoded (saved) document: ops in document order -- for host checks of the
 * engine's patch scan. Nulls: obj/key ctr and actor -1, key_len -1, action -1, val_len 0. */
typedef struct {
  int64_t obj_ctr, key_ctr, id_ctr, action, val_len;
  int32_t obj_actor, key_actor, id_actor, insert;
  int32_t key_len;
  uint32_t val_n, nsucc, succ_off;
  const uint8_t *key, *val;
} oc_op;
typedef struct {
  size_t nops; oc_op *ops; int64_t *succ_ctr; int32_t *succ_actor;
  size_t nactors; const uint8_t **actors; uint32_t *actor_lens;
  size_t nchg; int64_t *chg_actor; int64_t *chg_seq;
  void *priv;
} oc_export;
oc_export *oc_doc_export(const uint8_t *buf, size_t len, char *err, size_t errcap);
void oc_export_free(oc_export *e);

/* ---- sync.js Bloom filter + change selection (am_sync_oracle.c) ---- */
/* new BloomFilter(hashes).bytes: returns the encoded length (0 for no hashes); writes when cap suffices */
size_t oc_bloom_build(const uint8_t *hashes32, size_t n, uint8_t *out, size_t cap);
/* new BloomFilter(bytes).containsHash(hash): 1 / 0, -1 for a malformed filter */
int oc_bloom_contains(const uint8_t *filter, size_t len, const uint8_t *hash32);
/* getChangesToSend selection mask (see am_sync_oracle.c) */
void oc_sync_select(size_t n, const uint8_t *hashes32, const uint32_t *dep_off, const int32_t *dep_idx,
                    size_t nfilt, const uint8_t *const *filters, const size_t *flens, uint8_t *send);

#ifdef __cplusplus
}
#endif
#endif
