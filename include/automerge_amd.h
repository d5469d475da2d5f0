/*
 * automerge_amd.h -- C ABI of libautomerge_amd.so, the MI355X batched merge engine for Automerge.
 *
 * Drop-in boundary. The reference backend is a JavaScript module whose 22 functions are selected
 * with Automerge.setDefaultBackend(module) (src/automerge.js:147-149; module shape
 * backend/index.js:1-8). This library replaces the hot path behind it:
 *   am_doc_load            <- Backend.load             backend/backend.js:104-107, new.js:1695-1768
 *   am_doc_apply_changes_patch <- Backend.applyChanges backend/backend.js:27-32,   new.js:1796-1871
 *   (loadChanges = am_doc_apply_changes without a patch)   backend/backend.js:115-120
 *   am_doc_save            <- Backend.save             backend/backend.js:96-98,   new.js:2025-2047
 *   am_doc_get_heads       <- Backend.getHeads         backend/backend.js:134-136
 *   am_doc_clone / _free   <- Backend.clone / free     backend/backend.js:12-19
 *   am_doc_get_patch       <- Backend.getPatch         backend/backend.js:125-127, new.js:2052-2060
 *   am_bloom_* / am_sync_select <- BloomFilter / getChangesToSend   sync.js:38-125, 246-306
 *   am_doc_change/_queued  <- this.changes / this.queue (getChanges & getMissingDeps, new.js:1913-2020)
 *   am_change_hashes       <- decodeChangeMeta(.., true).hash   columnar.js:783-793
 *   am_batch_*             batched load + applyChanges over thousands of documents per launch
 *                          (no reference counterpart: the reference processes one document per call)
 * Bindings: Node-API addon automerge_amd/js/am_napi.c (+ backend.js, the Backend module) and
 * Python ctypes (automerge_amd/_native.py); see INTEGRATION.md.
 * All entry points are synchronous and return 0 on success; errors carry the reference's
 * message text (see am_error).
 */
#ifndef AUTOMERGE_AMD_H
#define AUTOMERGE_AMD_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

// ---- status codes. 1..99 mirror the reference's thrown errors (message formatted on the host
// from code + args); >= 100 are inputs outside what this engine restates (reported, never
// silently mis-merged). ----
enum am_status {
  AM_OK = 0,
  AM_E_MAGIC = 1,           // Data does not begin with magic bytes 85 6f 4a 83
  AM_E_CHECKSUM,            // checksum does not match data
  AM_E_SUBARRAY,            // subarray exceeds buffer size
  AM_E_LEB_RANGE,           // number out of range
  AM_E_LEB_INCOMPLETE,      // buffer ended with incomplete number
  AM_E_CHUNK_TYPE,          // Unexpected chunk type: %a0
  AM_E_CHANGE_TRAILING,     // Encoded change has trailing data
  AM_E_DOC_TRAILING,        // Encoded document has trailing data
  AM_E_COL_ORDER,           // Columns must be in ascending order
  AM_E_CHANGE_DEFLATED_COL, // change must not contain deflated columns
  AM_E_RLE_SUCC_REP,        // Successive repetitions with the same value are not allowed
  AM_E_RLE_REP1,            // Repetition count of 1 is not allowed, use a literal instead
  AM_E_RLE_SUCC_LIT,        // Successive literals are not allowed
  AM_E_RLE_SUCC_NULL,       // Successive null runs are not allowed
  AM_E_RLE_ZERO_NULL,       // Zero-length null runs are not allowed
  AM_E_RLE_LIT_REP,         // Repetition of values is not allowed in literal
  AM_E_BOOL_ZERO_RUN,       // Zero-length runs are not allowed
  AM_E_REUSE_SEQ,           // Reuse of sequence number %a0 for actor %s
  AM_E_SKIPPED_SEQ,         // Skipped sequence number %a0 for actor %s
  AM_E_FIRST_SEQ,           // Seq %a0 is the first change for actor %s
  AM_E_UNKNOWN_ACTOR,       // actorId %s is not known to document
  AM_E_NO_ACTOR_INDEX,      // No actor index %a0
  AM_E_MISMATCH_OBJ,        // Mismatched object reference: (%a0, %a1)
  AM_E_MISMATCH_KEY,        // Mismatched operation key: (%a0, %a1)
  AM_E_PRED_NOT_FOUND,      // no matching operation for pred: %a0@%s
  AM_E_REF_NOT_FOUND,       // Reference element not found: %a0@%s
  AM_E_ELEM_NOT_FOUND,      // could not find list element with ID: %a0@%s
  AM_E_DUP_OPID,            // duplicate operation ID: %a0@%s
  AM_E_DOC_SEQ,             // Expected seq %a0, got %a1 for actor %s
  AM_E_LAST_REFERENCE_ERROR,
  AM_E_FLOAT_LEN = 31,      // Invalid length for floating point number: %a0 (getPatch)
  AM_E_UNKNOWN_COUNTER = 32,// increment operation %a0@%s for unknown counter (getPatch)
  AM_E_HISTORY = 33,        // RangeError of decodeDocument / groupChangeOps / decodeDocumentChanges (message as given)
  AM_E_LOCAL = 34,          // error of encodeChange / applyLocalChange / the sync functions (class + message as given)
  AM_E_INFLATE = 35,        // invalid deflate data (a DEFLATEd document column, inflateColumn columnar.js:1062)
  AM_U_HASH_GRAPH = 100,    // needs the deferred hash graph of a loaded document (new.js:1826-1832)
  AM_U_UNKNOWN_COLUMN,      // column id outside DOC_OPS_COLUMNS / CHANGE_COLUMNS (new.js:1387-1425)
  AM_U_NONCAUSAL,           // opId counters violate Lamport order (insert after a later element, ...)
  AM_U_UTF8,                // invalid UTF-8 in a key or message and the document was staged without
                            // AM_DOC_FIX_UTF8: stage it again with the flag (the per-document calls do)
  AM_U_DEL_SHAPE,           // del op without preds, or inserting del (reference keeps it as a row)
  AM_U_VALUE,               // null action / null pred / mixed map+list object / 2^31+ sizes
  AM_U_CAPACITY,            // workspace bound exceeded (internal)
  AM_U_INC_VALUE,           // a non-integer counter increment in an applyChanges patch (JS adds it as a
                            // float / string, new.js:958); loadChanges commits (the patch is dropped)
};

// ---- host -> device descriptors ----
typedef struct am_chunk_desc {      // one binary chunk in the input arena
  uint64_t off;
  uint32_t len;
  uint32_t flags;           // bit0: checksum already verified by the host stage (inflated input)
                            // bit1: AM_CHUNK_RAW -- not a container: a document's objectMeta blob
} am_chunk_desc;
#define AM_CHUNK_RAW 2u
#define AM_CHUNK_BADZ 4u          /* internal (set by the batch stage): a DEFLATEd column does not inflate */
typedef struct am_doc_desc {
  int64_t base_chunk;       // chunk index of the base document, -1 for Backend.init()
  uint32_t chg_begin, chg_count;   // change chunks [chg_begin, chg_begin + chg_count)
  uint32_t known_begin, known_count; // extra changeIndexByHash entries (hash, index)
  uint32_t flags;           // bit0: haveHashGraph (fresh doc, or host knows all change hashes)
                            // bit1: AM_DOC_WANT_PATCH -- also write the getPatch() log of the result
                            // bit2: AM_DOC_WANT_DIFF -- also write the patch applyChanges returns
                            // AM_DOC_META -- the handle keeps objectMeta across calls (below)
  uint32_t meta_chunk;      // with AM_DOC_META: 1 + index of the AM_CHUNK_RAW chunk holding the objectMeta
                            // children the handle's previous call left; 0: documentPatch's (load / init)
} am_doc_desc;
#define AM_DOC_WANT_PATCH 2u
#define AM_DOC_WANT_DIFF 4u
#define AM_DOC_PATCH_ROOM 16u /* 8x the applyChanges-patch pools (a rerun after a patch capacity report) */
#define AM_DOC_FIX_UTF8 8u   /* k_doc reserves room for U+FFFD replacements of invalid UTF-8 (encoding.js:15-17) */
/* With AM_DOC_WANT_DIFF: objectMeta as the reference carries it on one BackendDoc from call to call
 * (new.js:884-931 children snapshots, 1812/1857): the patch log's header field meta_bytes counts the
 * blob of snapshots this call leaves, stored after the log's stream; the next call of the same handle
 * passes it back through meta_chunk. The per-document calls (am_doc_*) do this themselves. */
#define AM_DOC_META 32u
typedef struct am_known_hash {      // changeIndexByHash entry supplied by the host
  uint8_t hash[32];
  int64_t index;
} am_known_hash;

// ---- per-document result (device -> host) ----
typedef struct am_doc_result {
  uint32_t status;          // AM_* code (0 = applied/loaded)
  uint32_t err_change;      // change index (within the doc) an error refers to, or ~0u
  int64_t arg0, arg1;       // error arguments
  uint64_t arg_actor_off;   // arena offset of the actor id an error names
  uint32_t arg_actor_len;
  uint32_t napplied;        // changes applied in this call
  uint32_t nqueued;         // changes left in the queue (pendingChanges)
  uint32_t nheads;
  uint32_t nops;            // op rows in the merged document
  uint32_t nchanges;        // change rows in the merged document
  int64_t max_op;           // this.maxOp of the result: max(base op ids / succ counters, applied changes)
  uint64_t out_off;         // merged document chunk (uncompressed columns) in the output arena
  uint64_t out_len;
  uint64_t ws_off, ws_bytes;
} am_doc_result;

// per change chunk outcome within its document
enum am_change_state { CHG_UNSEEN = -4, CHG_DUP = -3, CHG_QUEUED = -2, CHG_ERROR = -1 }; // >= 0: applied index


typedef struct am_error {
  uint32_t code;          /* AM_* status; 0 = ok */
  int32_t is_type_error;  /* the reference throws TypeError (else RangeError/Error) */
  char message[8184];     /* the reference's message text (heads lists of a history error run long) */
} am_error;

typedef struct am_engine am_engine;
typedef struct am_batch am_batch;
typedef struct am_doc am_doc;

/* ---- engine: one per GPU (HIP device ordinal), owns a HIP stream ---- */
am_engine *am_engine_create(int device, am_error *err);
void am_engine_destroy(am_engine *eng);
const char *am_version(void);

/* ---- batch: many documents resident in HBM ---- */
am_batch *am_batch_create(am_engine *eng);
void am_batch_destroy(am_batch *b);
/* Copies the input arena and descriptors to the device and sizes the per-document workspaces.
 * Chunks must be uncompressed (chunk type 0/1, no DEFLATE bit): am_stage_change / am_stage_document are the host stage. */
int am_batch_stage(am_batch *b, const uint8_t *arena, uint64_t arena_len, const am_chunk_desc *chunks,
                   uint32_t nchunks, const am_doc_desc *docs, uint32_t ndocs, const am_known_hash *known,
                   uint32_t nknown, am_error *err);
/* Enqueues the whole pipeline (hash/parse, plan, decode, merge, encode, checksum) on the engine
 * stream; inputs stay resident, so run may be repeated. am_batch_sync waits for completion. */
int am_batch_run(am_batch *b);
int am_batch_sync(am_batch *b, am_error *err);
/* Per-document results (ndocs entries) and per-change outcomes (nchunks entries: applied index,
 * or CHG_QUEUED / CHG_DUP), change hashes (32 bytes per chunk). */
int am_batch_results(am_batch *b, am_doc_result *out);
int am_batch_chunk_results(am_batch *b, uint8_t *hashes32, int32_t *chg_state, uint32_t *status);
/* Merged document chunk (uncompressed columns) of one document. */
int am_batch_doc_output(am_batch *b, uint32_t doc, uint8_t *dst, uint64_t cap, uint64_t *len);
/* DEFLATE-compressed change chunks (type 2) inflated on the GPU by the last am_batch_stage
 * (inflateChange, columnar.js:813-823): their number, the inflated arena bytes and the time of the
 * two inflate passes (ms, HIP events). */
int am_batch_inflate_info(am_batch *b, uint64_t *nchunks, uint64_t *arena_bytes, float *ms);
/* computeHashGraph (new.js:1879-1904) / decodeDocument (columnar.js:1040-1046, groupChangeOps :876-943,
 * decodeDocumentChanges :945-981) of n documents in one GPU batch (k_history, one workgroup per
 * document): the change history of each document chunk, every change re-encoded by encodeChange
 * (deflated when >= 256 B) in the document's change order. Per document: changes = the change
 * chunks back to back, offs[0..nchanges] their offsets, hashes32 their hashes (malloc'd, am_free),
 * or err.code != 0 with the reference's RangeError text (AM_E_HISTORY) or the codec error.
 * Returns nonzero when any document failed. */
typedef struct am_history {
  uint8_t *changes;
  uint64_t *offs;
  uint8_t *hashes32;
  size_t nchanges;
  am_error err;
} am_history;
int am_document_changes_batch(am_engine *eng, const uint8_t *const *docs, const size_t *lens, size_t n, am_history *out);
/* One document through am_document_changes_batch: *out = the changes back to back, (*offs)[0..n]
 * their offsets, *hashes32 their hashes (all malloc'd, am_free). */
int am_document_changes(am_engine *eng, const uint8_t *doc, size_t len, uint8_t **out, uint64_t **offs, uint8_t **hashes32,
                        size_t *nchanges, am_error *err);
/* Backend state of a loaded document: fills in its hash graph (new.js:1879-1904) so that
 * getAllChanges / getChanges / getChangeByHash see the whole history; no-op when it is known. */
int am_doc_compute_hash_graph(am_doc *d, am_error *err);
/* pako.inflateRaw (the call inside inflateChange / inflateColumn, columnar.js:816, 1064) over n
 * independent buffers on the GPU. outs[i] is malloc'd (am_free); ok[i] = 0 when buffer i is not a
 * valid raw DEFLATE stream. */
int am_inflate_raw(am_engine *eng, const uint8_t *const *bufs, const size_t *lens, size_t n, uint8_t **outs,
                   size_t *out_lens, uint8_t *ok, am_error *err);
/* Backend.save() bytes of one document (backend.js:96-98, new.js:2025-2047): the merged chunk with
 * columns >= 256 bytes DEFLATEd (deflateColumn, columnar.js:1052). *out is malloc'd (am_free). */
int am_batch_doc_save(am_batch *b, uint32_t doc, uint8_t **out, size_t *len, am_error *err);
int am_batch_doc_heads(am_batch *b, uint32_t doc, uint8_t *dst32, uint32_t cap, uint32_t *n);
/* Patch log of document `doc`: the getPatch() log (staged with AM_DOC_WANT_PATCH) or the patch
 * applyChanges returns (AM_DOC_WANT_DIFF, new.js:1862-1865): PatchHdr | records | values |
 * heap as described in automerge_amd/csrc/am_patch.h; materialized by automerge_amd/patch.py or
 * automerge_amd/js/backend.js. cap = 0 returns the size in *len. */
int am_batch_doc_patch(am_batch *b, uint32_t doc, uint8_t *dst, uint64_t cap, uint64_t *len);
/* Device time of each pipeline stage in the last run (ms): [chunks, bounds+scan, doc, out_hash]. */
int am_batch_stage_times(am_batch *b, float *ms4);
/* Order-independent digest of the batch's merged outputs, for the cross-rank exchange: the sum
 * mod 2^63 over documents d of mix64(((first_doc + d) << 32) | checksum32_le(output d)) +
 * out_len(d) * 0x9E3779B97F4A7C15 + status(d), where checksum32 = bytes 4..8 of the merged
 * container (columnar.js:659-686) and mix64 is the splitmix64 finalizer. Host restatement:
 * automerge_amd/shard.py doc_digest. */
int am_batch_digest(am_batch *b, uint64_t first_doc, uint64_t *digest);
/* Per document of the last run: 1 when the small-document kernel (k_doc_fast) merged it, 0 when
 * the general kernel did (documents outside its envelope, errors, getPatch requests). */
int am_batch_fast_flags(am_batch *b, uint8_t *flags);
/* Diagnostics of the batched per-handle calls since the last call (reset on read): out2[0] documents
 * run, out2[1] of them merged by the small-document kernel k_doc_fast. Not part of the reference
 * interface. */
int am_engine_stats(am_engine *e, uint64_t *out2);
/* Diagnostics (AM_DEBUG_WS_CANARY=<n> in the environment of am_batch_run): offset past the end of
 * the batch workspace of the first of n canary bytes a kernel wrote, -1 when none. */
int64_t am_batch_ws_canary(am_batch *b, uint64_t n);
/* Diagnostics: document doc's workspace bounds (96 bytes, the engine's DocBounds) and layout (u64
 * offsets; returns how many the layout has, writing at most cap). */
int am_batch_doc_layout(am_batch *b, uint32_t doc, void *bounds_out, uint64_t *lay_out, uint32_t cap);
/* Diagnostics: the raw 48-byte header of document doc's patch-log slot. */
int am_batch_doc_patch_raw(am_batch *b, uint32_t doc, uint8_t *dst48);
/* Device workspace the staged batch holds (for bench byte accounting): the scanned per-document
 * plans plus the overflow reserve (the whole plan of every document given k_doc_fast's compact plan,
 * in case the fast kernel gives up on it). */
uint64_t am_batch_workspace_bytes(am_batch *b);
/* The scanned per-document plans alone: what a pipeline slot needs before its overflow headroom. */
uint64_t am_batch_workspace_plan(am_batch *b);
/* Launch shape of the staged batch's document kernels: out3[0] = k_doc dynamic LDS bytes,
 * out3[1] = k_doc_fast LDS slice per document (0: none in its envelope), out3[2] = largest k_doc
 * hot working set. Not part of the reference interface (bench/profiling only). */
int am_batch_kernel_info(am_batch *b, uint64_t *out3);
/* Workspace plan of one staged document (diagnostics, not part of the reference interface):
 * R, E, P, hot set, workspace bytes, workspace offset, span_lo, span_hi, runs-from-LDS, input bytes. */
int am_batch_doc_plan(am_batch *b, uint32_t doc, uint64_t *out10);
/* Diagnostics: the k_doc_fast LDS slice of every staged document (0 = outside its envelope). */
int am_batch_fast_slices(am_batch *b, uint32_t *out);

/* ---- pipelined batches: the whole job from host memory to host memory ----
 * A stream of batches (each = many documents, one Backend.load + Backend.applyChanges per document,
 * as am_batch_*) runs through `slots` device buffer sets: the H2D copy of batch k+1 and the D2H
 * copy of batch k-1 overlap the kernels of batch k on separate HIP streams. Each batch's merged
 * documents and patch logs (documents staged with AM_DOC_WANT_DIFF) come back densely packed in
 * 16-byte slots, described by one am_doc_summary per document. Host buffers should come from
 * am_host_alloc (pinned) for the copies to be asynchronous.
 *   caps: per-batch capacities. ws_bytes: device workspace per batch (am_batch_workspace_plan of a
 *   representative batch, with headroom: the headroom past a batch's plans is the overflow region
 *   where a document the fast kernel gives up on gets k_doc's whole plan); fast_lds: k_doc_fast LDS slice per document
 *   (am_batch_kernel_info out3[1]; 0 disables the small-document kernel). Documents that exceed a
 *   capacity report AM_U_CAPACITY in their summary and can be rerun through am_batch_*.
 * Change chunks must be uncompressed (type 1): DEFLATEd ones go through am_batch_stage. */
typedef struct am_doc_summary {     /* 32 bytes per document */
  uint32_t status;                  /* AM_* code (0 = applied / loaded) */
  uint32_t nqueued;                 /* changes left in the queue (pendingChanges) */
  uint32_t out_len, patch_len;      /* merged document chunk (uncompressed columns) / patch log bytes */
  uint64_t out_off, patch_off;      /* their offsets in the batch's output arenas */
} am_doc_summary;
typedef struct am_pipe_caps {
  uint64_t arena_bytes;             /* input bytes per batch */
  uint32_t chunks, docs;            /* chunks / documents per batch */
  uint64_t ws_bytes;                /* device workspace per batch */
  uint64_t out_bytes, patch_bytes;  /* output arena capacities per batch */
  uint32_t fast_lds;                /* k_doc_fast LDS bytes per document (0: off) */
  uint32_t slots;                   /* batches in flight (>= 2) */
} am_pipe_caps;
typedef struct am_pipe am_pipe;
void *am_host_alloc(size_t n);      /* pinned host memory (hipHostMalloc) */
void am_host_free(void *p);
am_pipe *am_pipe_create(am_engine *eng, const am_pipe_caps *caps, am_error *err);
void am_pipe_destroy(am_pipe *p);
/* Enqueues batch `ticket` (returned in *ticket): H2D, the pipeline of am_batch_run, compaction and
 * D2H into summary[ndocs], out[..] and patches[..]. The output arenas hold min(out_cap, caps.out_bytes)
 * and min(patch_cap, caps.patch_bytes) bytes: a document whose chunk or log does not fit reports
 * AM_U_CAPACITY in its summary. Blocking: the submit queues the copies home of the previous batch,
 * which waits on the host for that batch's kernels (their output sizes); when every slot is in
 * flight it also waits for the oldest batch's copies home before reusing its slot. */
int am_pipe_submit(am_pipe *p, const uint8_t *arena, uint64_t arena_len, const am_chunk_desc *chunks, uint32_t nchunks,
                   const am_doc_desc *docs, uint32_t ndocs, am_doc_summary *summary, uint8_t *out, uint64_t out_cap,
                   uint8_t *patches, uint64_t patch_cap, uint64_t *ticket, am_error *err);
/* am_pipe_submit with packed descriptors: the arena holds the batch's chunks back to back in chunk
 * order and chunk_len[c] is the length of chunk c; a document's chunks are consecutive (its saved
 * base document first when has_base, then its chg_count change chunks), in document order. The
 * device derives the am_chunk_desc / am_doc_desc arrays (two scans), so the host link carries 4 B
 * per chunk and 8 B per document of descriptors instead of 16 and 32. Same outputs and semantics as
 * am_pipe_submit; AM_DOC_META is not accepted (no objectMeta chunks in a packed batch), and a
 * length that runs past the arena is cut there (that chunk then fails its container check). */
typedef struct am_doc_span {
  uint32_t chg_count;               /* change chunks of the document */
  uint16_t flags;                   /* am_doc_desc flags (AM_DOC_WANT_DIFF, AM_DOC_WANT_PATCH, ...) */
  uint8_t has_base;                 /* 1: the first chunk is a saved document (Backend.load), 0: Backend.init() */
  uint8_t reserved;
} am_doc_span;
int am_pipe_submit_packed(am_pipe *p, const uint8_t *arena, uint64_t arena_len, const uint32_t *chunk_len, uint32_t nchunks,
                          const am_doc_span *docs, uint32_t ndocs, am_doc_summary *summary, uint8_t *out, uint64_t out_cap,
                          uint8_t *patches, uint64_t patch_cap, uint64_t *ticket, am_error *err);
/* The SDMA engines the pipeline's host-link copies run on (bit k = HSA_AMD_SDMA_ENGINE_k): [0] the
 * H2D of the inputs, [1] the copies home; 0 = the runtime's choice / a copy kernel. */
int am_pipe_engines(am_pipe *p, uint32_t *out2);
/* Waits until every submitted batch is home. totals (optional, 2 per batch in submission order
 * since the last drain, up to cap batches): output / patch arena bytes. */
int am_pipe_drain(am_pipe *p, uint64_t *totals, uint32_t cap, am_error *err);
/* The same chain for a batch already resident in device memory (the bench's HBM-resident job):
 * d_arena (arena_len + 64 readable bytes), d_chunks, d_docs and the outputs are device pointers;
 * any_diff: some document asks for a patch log (AM_DOC_WANT_DIFF or AM_DOC_WANT_PATCH: the launch
 * then carries k_doc_fast's patch writers). Merged documents, patch logs and
 * summaries are compacted into d_out / d_patches / d_summary (layout of am_pipe_submit) and their
 * two arena totals into d_totals; nothing crosses the host link and the call does not wait.
 * am_pipe_resident_sync waits for the stream; ms2 = the chains / document kernels of the resident
 * batches since its last call, summed (HIP events). Resident batches share slot 0's workspace: at
 * most 4096 run between two syncs, and am_pipe_submit refuses work while any is unsynced. */
int am_pipe_run_resident(am_pipe *p, const uint8_t *d_arena, uint64_t arena_len, const am_chunk_desc *d_chunks,
                         uint32_t nchunks, const am_doc_desc *d_docs, uint32_t ndocs, int any_diff, am_doc_summary *d_summary,
                         uint8_t *d_out, uint64_t out_cap, uint8_t *d_patches, uint64_t patch_cap, uint64_t *d_totals,
                         am_error *err);
int am_pipe_resident_sync(am_pipe *p, float *ms2, am_error *err);
/* Device time (ms) of the batches retired since the last call (reset on read): [0] their whole
 * compute chains summed, [1] their document kernels (k_doc_fast + k_doc) summed; n = batches. */
int am_pipe_times(am_pipe *p, float *ms2, uint32_t *n);
/* Diagnostics: a pipeline created with AM_DEBUG_WS_CANARY=<n> in the environment follows every slot's
 * workspace with n canary bytes; after am_pipe_drain this returns the offset of the first one a
 * kernel wrote (any slot), -1 when none, -2 when the pipeline has no canary. */
int64_t am_pipe_ws_canary(am_pipe *p);

/* ---- per-document backend state (mirrors backend/backend.js over the batch path, n = 1) ---- */
am_doc *am_doc_init(am_engine *eng);
am_doc *am_doc_load(am_engine *eng, const uint8_t *data, size_t len, am_error *err);
am_doc *am_doc_clone(const am_doc *doc);
void am_doc_free(am_doc *doc);
/* Backend.loadChanges: applies without producing a patch */
int am_doc_apply_changes(am_doc *doc, const uint8_t *const *bufs, const size_t *lens, size_t n, am_error *err);
/* Backend.applyChanges (backend/backend.js:27-32, new.js:1796-1871): applies and returns the patch log
 * of the call (malloc'd, am_free; layout of am_batch_doc_patch). Its PR_CLOCK records are the clock;
 * maxOp / deps / pendingChanges come from am_doc_max_op / am_doc_get_heads / am_doc_pending. An error
 * the patch raises (unknown counter, float length) fails the call and leaves the document unchanged. */
int am_doc_apply_changes_patch(am_doc *doc, const uint8_t *const *bufs, const size_t *lens, size_t n,
                               uint8_t **patch, size_t *patch_len, am_error *err);
/* Returns a malloc'd buffer (release with am_free). DEFLATE of columns >= 256 bytes is the
 * host stage (columnar.js:1052-1057). */
int am_doc_save(am_doc *doc, uint8_t **out, size_t *len, am_error *err);
size_t am_doc_get_heads(const am_doc *doc, uint8_t *out32, size_t cap);
size_t am_doc_pending(const am_doc *doc);
int64_t am_doc_max_op(const am_doc *doc);
size_t am_doc_num_changes(const am_doc *doc);
/* i-th applied change buffer (as given by the caller) / its hash; for getChanges-style callers. */
int am_doc_change(const am_doc *doc, size_t i, const uint8_t **data, size_t *len, uint8_t *hash32);
/* Backend.getPatch(doc) (backend/backend.js:125-127, new.js:2052-2060): documentPatch over the
 * current document on the GPU; returns the patch log (malloc'd, am_free) -- see am_batch_doc_patch.
 * maxOp / deps / pendingChanges come from am_doc_max_op / am_doc_get_heads / am_doc_pending. */
int am_doc_get_patch(am_doc *doc, uint8_t **out, size_t *len, am_error *err);
/* i-th enqueued change (this.queue, new.js:1796-1871: changes waiting for missing deps), as given */
int am_doc_queued(const am_doc *doc, size_t i, const uint8_t **data, size_t *len);
/* ---- the per-document calls over n handles in ONE GPU batch (the batched backend surface) ----
 * Same semantics per handle as the single calls above, as if they ran in index order; a handle that
 * appears twice takes its later calls after the batch, in order. Per call: codes[i] (0 = ok; bit 31
 * set when the reference throws a TypeError) and, when msgs is non-null, msgs[i] = the error text
 * (malloc'd, am_free; nullptr when the call succeeded). Output buffers are malloc'd (am_free).
 * Each returns the number of calls that failed; a failed call leaves its handle unchanged.
 *   am_doc_load_batch          <- Backend.load           backend.js:104-107 (docs[i] = nullptr on error)
 *   am_doc_apply_changes_batch <- Backend.applyChanges   backend.js:27-32   (patches != nullptr)
 *                                 Backend.loadChanges    backend.js:115-120 (patches == nullptr)
 *     handle i gets the changes bufs[off[i] .. off[i+1]); loaded handles whose changes need the
 *     hash graph (new.js:1826-1832) have it computed together in one batch and run again.
 *     info (optional): per call, the handle's maxOp / heads / pending right after that call.
 *   am_doc_get_patch_batch     <- Backend.getPatch       backend.js:125-127
 *   am_doc_save_batch          <- Backend.save           backend.js:96-98 (one SHA-256 launch)
 *   am_doc_compute_hash_graph_batch <- computeHashGraph  new.js:1879-1904 */
/* What a patch is materialized with (maxOp, deps = heads, pendingChanges), taken right after call i:
 * heads is malloc'd (am_free), 32 x nheads bytes. */
typedef struct am_call_info {
  int64_t max_op;
  uint32_t pending;
  uint32_t nheads;
  uint8_t *heads;
} am_call_info;
int am_doc_load_batch(am_engine *eng, size_t n, const uint8_t *const *data, const size_t *lens, am_doc **docs,
                      uint32_t *codes, char **msgs);
int am_doc_apply_changes_batch(size_t n, am_doc *const *docs, const size_t *off, const uint8_t *const *bufs,
                               const size_t *lens, uint8_t **patches, size_t *patch_lens, am_call_info *info,
                               uint32_t *codes, char **msgs);
int am_doc_get_patch_batch(size_t n, am_doc *const *docs, uint8_t **out, size_t *lens, am_call_info *info, uint32_t *codes,
                           char **msgs);
int am_doc_save_batch(size_t n, am_doc *const *docs, uint8_t **out, size_t *lens, uint32_t *codes, char **msgs);
int am_doc_compute_hash_graph_batch(size_t n, am_doc *const *docs, uint32_t *codes, char **msgs);
/* 1 when the document's hash graph is computed and indexed: its graph queries then only read it
 * (safe from several host threads at once). */
int am_doc_graph_ready(const am_doc *doc);
/* ---- hash-graph queries (BackendDoc, new.js:1913-2020); the graph of a loaded document is
 * computed on first use (computeHashGraph, new.js:1879-1904). Change indexes refer to
 * am_doc_change; arrays are malloc'd (am_free). ----
 * am_doc_get_changes       <- getChanges(haveDeps)        new.js:1913-1966 ("hash not found: <hex>")
 * am_doc_get_changes_added <- getChangesAdded(doc1, doc2) new.js:1971-1988 (indexes into doc2)
 * am_doc_change_index      <- getChangeByHash             new.js:1990-1993 (-1: unknown, -2: error)
 * am_doc_get_missing_deps  <- getMissingDeps(heads)       new.js:2005-2020 (sorted hashes) */
int am_doc_get_changes(am_doc *doc, const uint8_t *have32, size_t nhave, uint64_t **idx, size_t *n, am_error *err);
int am_doc_get_changes_added(am_doc *doc1, am_doc *doc2, uint64_t **idx, size_t *n, am_error *err);
int64_t am_doc_change_index(am_doc *doc, const uint8_t *hash32);
int am_doc_get_missing_deps(am_doc *doc, const uint8_t *heads32, size_t nheads, uint8_t **out32, size_t *n, am_error *err);
/* ---- per-actor state of a document (read by applyLocalChange) ----
 * am_doc_clock       <- state.clock[actor]                 new.js:1857 (0: no entry; -1: error)
 * am_doc_actor_hash  <- state.hashesByActor[actor][seq-1]  new.js:1840-1841 (0 ok, 1 unknown)
 * am_doc_change_deps <- dependenciesByHash of change i      new.js:1843 (pointer valid until the next call)
 * am_doc_engine      -- the engine a document runs on */
int64_t am_doc_clock(am_doc *doc, const char *actor_hex);
int am_doc_actor_hash(am_doc *doc, const char *actor_hex, int64_t seq, uint8_t *hash32);
int am_doc_change_deps(am_doc *doc, size_t i, const uint8_t **deps32, size_t *n);
am_engine *am_doc_engine(const am_doc *doc);

/* ---- local changes ----
 * Requests are the frontend's change objects as JSON text; a Uint8Array travels as
 * {"__bytes":"<hex>"} and a non-finite number as {"__f64":"NaN"|"Infinity"|"-Infinity"}.
 * am_encode_change          <- encodeChange(change)               columnar.js:710-739
 *     out: the binary change (DEFLATE'd when >= 256 B, malloc'd); hash32: its hash
 * am_doc_apply_local_change <- Backend.applyLocalChange(backend, change)  backend.js:54-91
 *     out: the binary change, the patch log (wire form, am_patch.h), new_hash32 = the hash the
 *     patch's deps omit, last_hash32 (*has_last) = the local actor's previous change that joined
 *     the request's deps. Returns 0; 1 on an error before the document changed; 2 on the error
 *     the reference raises after applying (the caller's handle must be treated as updated). */
int am_encode_change(const char *json, size_t len, uint8_t **out, size_t *out_len, uint8_t *hash32, am_error *err);
int am_doc_apply_local_change(am_doc *doc, const char *json, size_t len, uint8_t **change, size_t *change_len,
                              uint8_t **patch, size_t *patch_len, uint8_t *new_hash32, uint8_t *last_hash32,
                              int *has_last, am_error *err);

/* ---- sync protocol (backend/sync.js) ----
 * A SyncState object {sharedHeads, lastSentHeads, theirHeads, theirNeed, theirHave, sentHashes}
 * (sync.js:262-271) crosses the ABI in this flat form ("state blob"):
 *   u8 0x53 | u8 flags (1 theirHeads, 2 theirNeed, 4 theirHave present; 8 sentHashes is the empty
 *   array receiveSyncMessage resets it to) | H sharedHeads | H lastSentHeads | [H theirHeads]
 *   | [H theirNeed] | [uleb n, n x (H lastSync, uleb len, bloom bytes)] | H sentHashes
 * where H = uleb count + count x 32-byte hash (sentHashes in insertion order).
 * am_sync_generate       <- generateSyncMessage(backend, state)  sync.js:327-400, for n documents
 *     at once: their Bloom filters are built in one k_bloom_build launch and their change
 *     selections run in one k_sync_select launch; loaded documents get their hash graphs in one
 *     batch. Per document: out state blob, message (NULL when none is due) and codes[i] / errmsgs[i]
 *     as the batched per-handle calls; returns the number of documents that failed.
 * am_sync_receive        <- receiveSyncMessage(backend, state, msg) sync.js:420-473; *patch is the
 *     applyChanges patch log when the message carried changes (else NULL). Returns 0, 1 (error,
 *     document unchanged) or 2 (error after the changes were applied).
 * am_sync_encode_message <- encodeSyncMessage(message)  sync.js:157-171 (message as JSON)
 * am_sync_decode_messages<- decodeSyncMessage(bytes)    sync.js:177-199, n messages: spans of
 *     message i are spans[span_off[i] .. span_off[i+1]): heads (off, count), need (off, count),
 *     per have: lastSync (off, count) and bloom (off, len), per change (off, len); offsets into
 *     the message, counts[4i..4i+3] = heads, need, have, changes. Returns the number failed.
 * am_sync_encode_state   <- encodeSyncState(state)      sync.js:206-211 (from a state blob)
 * am_sync_decode_state   <- decodeSyncState(bytes)      sync.js:217-225 (to a state blob) */
typedef struct { uint64_t off, len; } am_span;
int am_bloom_check(const uint8_t *filter, uint64_t len, am_error *err);
int am_sync_generate(size_t n, am_doc *const *docs, const uint8_t *const *states, const size_t *state_lens,
                     uint8_t **out_states, size_t *out_state_lens, uint8_t **msgs, size_t *msg_lens, uint32_t *codes,
                     char **errmsgs);
int am_sync_receive(am_doc *doc, const uint8_t *state, size_t state_len, const uint8_t *msg, size_t msg_len,
                    uint8_t **out_state, size_t *out_state_len, uint8_t **patch, size_t *patch_len, am_error *err);
/* receiveSyncMessage of n (document, state, message) triples in one call: every message's changes
 * go through ONE am_doc_apply_changes_batch, the hash graphs the heads lookups need are computed in
 * one batch (am_doc_compute_hash_graph_batch), then each state is updated as am_sync_receive does.
 * Outputs per triple as am_sync_receive (malloc'd, am_free), info (optional) as
 * am_doc_apply_changes_batch for the triples that applied changes; codes[i] = 0 or the error code with
 * bit 31 set for a TypeError and bit 30 set when the changes were applied before the error (the
 * single call's return 2); errmsgs (optional) as the batched per-handle calls. A document named
 * twice takes its later triples after the batch, in order. Returns the number that failed. */
int am_sync_receive_batch(size_t n, am_doc *const *docs, const uint8_t *const *states, const size_t *state_lens,
                          const uint8_t *const *msgs, const size_t *msg_lens, uint8_t **out_states, size_t *out_state_lens,
                          uint8_t **patches, size_t *patch_lens, am_call_info *info, uint32_t *codes, char **errmsgs);
int am_sync_encode_message(const char *json, size_t len, uint8_t **out, size_t *out_len, am_error *err);
int am_sync_decode_messages(size_t n, const uint8_t *const *msgs, const size_t *lens, am_span **spans,
                            uint64_t *span_off, uint32_t *counts, am_error *errs);
int am_sync_encode_state(const uint8_t *state, size_t len, uint8_t **out, size_t *out_len, am_error *err);
int am_sync_decode_state(const uint8_t *bytes, size_t len, uint8_t **state, size_t *state_len, am_error *err);

void am_free(void *p);

/* ---- host stage for batch callers (DEFLATE, columnar.js:798-823, 1052-1067) ----
 * am_stage_change: a DEFLATE-compressed change (chunk type 2) becomes an uncompressed type-1 chunk
 *   keeping its checksum (which covers the uncompressed form); other chunks are copied.
 * am_stage_document: a document with DEFLATE-compressed columns has its checksum verified on the
 *   GPU and its columns inflated; *verified = 1 means the result must be staged with
 *   am_chunk_desc.flags bit0 set (checksum already checked). Outputs are malloc'd (am_free). */
int am_stage_change(const uint8_t *in, size_t len, uint8_t **out, size_t *outlen, am_error *err);
int am_stage_document(am_engine *eng, const uint8_t *in, size_t len, uint8_t **out, size_t *outlen, int *verified,
                      am_error *err);
/* am_stage_document over n documents in one call (reference: load -> inflateColumn,
 * backend/columnar.js:1062-1068, for every document): one GPU checksum batch and one GPU inflate
 * batch for the DEFLATEd columns of all of them. outs[i] (free with am_free) / out_lens[i] = the
 * staged chunk, verified[i] = 1 when its checksum was verified here, codes[i] / msgs[i] as in
 * am_doc_load_batch. Returns the number of documents that failed. */
int am_stage_documents(am_engine *eng, size_t n, const uint8_t *const *data, const size_t *lens, uint8_t **outs,
                       size_t *out_lens, uint8_t *verified, uint32_t *codes, char **msgs);

/* ---- utilities ---- */
/* Change hash (SHA-256 of the uncompressed chunk) of each change, computed on the GPU. */
int am_change_hashes(am_engine *eng, const uint8_t *const *bufs, const size_t *lens, size_t n, uint8_t *out32,
                     am_error *err);

/* ---- sync.js Bloom filters and change selection, batched ----
 * am_bloom_build      <- new BloomFilter(hashes).bytes            sync.js:38-47, 66-77, 90-110
 *   Filter f holds hashes [hoff[f], hoff[f+1]) of hashes32 (32 bytes each). The encoded filters
 *   are written back to back into out; foff (nfilt + 1 entries) receives their offsets. A filter
 *   with no hashes encodes to 0 bytes. am_bloom_encoded_size(n) = size of one filter of n hashes.
 * am_bloom_probe      <- new BloomFilter(bytes).containsHash(h)   sync.js:48-59, 112-125
 *   Probe i tests hash probes32[i] against filter pfilt[i] (filters/foff as produced above or
 *   received from peers); contains[i] = 1 / 0. A malformed filter fails with the RangeError text
 *   of its decode (number out of range / incomplete number / subarray exceeds buffer size).
 * am_sync_select      <- getChangesToSend with non-empty `have`   sync.js:246-306
 *   For pair p: changes [coff[p], coff[p+1]) (hashes32, in getChanges order), change c's deps
 *   didx[doff[c] .. doff[c+1]) as indexes within the pair's list (-1 = not in the list), the
 *   pair's filters [pfoff[p], pfoff[p+1]) of filters/foff. send[c] = 1 for changes absent from
 *   every filter and their transitive dependents; the caller appends the explicit `need` hashes. */
uint64_t am_bloom_encoded_size(uint64_t nhashes);
int am_bloom_build(am_engine *eng, const uint8_t *hashes32, const uint64_t *hoff, uint32_t nfilt, uint8_t *out,
                   uint64_t cap, uint64_t *foff, am_error *err);
int am_bloom_probe(am_engine *eng, const uint8_t *filters, const uint64_t *foff, uint32_t nfilt, const uint8_t *probes32,
                   const uint32_t *pfilt, uint64_t nprobe, uint8_t *contains, am_error *err);
int am_sync_select(am_engine *eng, uint32_t npairs, const uint64_t *coff, const uint8_t *hashes32, const uint64_t *doff,
                   const int32_t *didx, const uint64_t *pfoff, const uint8_t *filters, const uint64_t *foff,
                   uint8_t *send, am_error *err);

#ifdef __cplusplus
}
#endif
#endif
