// am_launch.h -- host-side launchers of the kernels in am_kernels.hip.
#pragma once
#include <hip/hip_runtime.h>

#include "am_common.h"
#include "am_layout.h"
#include "am_hist.h"

#include <string>
#include <functional>
#include <vector>

struct BatchDev {
  const uint8_t* arena;
  const am_chunk_desc* chunks;
  const am_doc_desc* docs;
  const am_known_hash* known;
  ChunkInfo* info;
  HdrSlot* hdr;            // per chunk: compact parsed header (k_chunks)
  DocBounds* bounds;
  uint64_t* ws_bytes;      // per doc
  uint64_t* ws_off;        // per doc (exclusive scan)
  uint64_t* scan_tmp;      // block sums
  uint64_t* ws_total;      // 1 value
  uint64_t* max_hot;       // 4 values: largest hot set, largest fast slice, the whole plans of the compact documents,
                           // the overflow region's bump counter (k_rest)
  uint32_t lds_bytes;      // dynamic LDS per document workgroup
  uint64_t max_hot_host;   // host copy of *max_hot
  uint32_t fast_lds;       // k_doc_fast LDS slice per document (0: no document in its envelope / disabled)
  uint8_t* fast_done;      // per doc: 1 = merged by k_doc_fast
  uint32_t* rest;          // [0] = count, [1..]: the documents k_doc_fast left (k_rest)
  bool fast_only;          // every document is in the fast envelope: skip the k_doc launches
  bool any_diff;           // some document asks for its applyChanges patch (k_doc_fast<true>)
  bool compact;            // k_bounds gives k_doc_fast's documents the compact plan (ws_layout, U bit 2)
  uint32_t fast_cap;       // ... only those whose fast slice fits the launch's (a pipeline's fixed fast_lds;
                           // a batch sizes its launch from the largest slice, so every one fits)
  uint8_t* ws;
  uint64_t ws_cap;
  am_doc_result* results;
  int32_t* chg_state;      // per chunk
  uint32_t nchunks, ndocs;
};

void am_launch_chunks(const BatchDev& b, hipStream_t s);
// diagnostics: k_doc_fast LDS slice per document (0: outside its envelope)
void am_fast_slices_host(const DocBounds* db, const am_doc_desc* dd, uint32_t n, uint32_t* out);
void am_launch_chunk_hashes(const ChunkInfo* info, uint32_t n, uint8_t* out32, hipStream_t s);
void am_launch_bounds(const BatchDev& b, hipStream_t s);   // k_bounds + scan of ws bytes
void am_launch_doc(const BatchDev& b, hipStream_t s);
void am_launch_out_hash(const BatchDev& b, hipStream_t s);
void am_launch_digest(const BatchDev& b, uint64_t first, uint64_t* d_out, hipStream_t s);
void am_launch_sha256(const uint8_t* arena, const am_chunk_desc* msgs, uint32_t n, uint8_t* out, hipStream_t s);
size_t am_scan_tmp_elems(uint32_t n);
void am_launch_scan(const uint64_t* in, uint64_t* out, uint64_t* tmp, uint32_t n, uint64_t* total, hipStream_t s);
// packed batch descriptors (am_pipe_submit_packed) expanded into am_chunk_desc / am_doc_desc;
// c64/coff/ctmp: chunk scan buffers, d64/dbeg/dtmp: document scan buffers, totals2: 2 scratch u64
void am_launch_unpack(const uint32_t* clen, uint32_t nchunks, uint64_t arena_len, const am_doc_span* spans, uint32_t ndocs,
                      uint64_t* c64, uint64_t* coff, uint64_t* ctmp, uint64_t* d64, uint64_t* dbeg, uint64_t* dtmp,
                      uint64_t* totals2, am_chunk_desc* chunks, am_doc_desc* docs, hipStream_t s);
// pipelined batches: dense arenas of merged documents / patch logs + per-document summaries;
// totals[0..1] = bytes of the two arenas
void am_launch_pipe_compact(const BatchDev& b, uint64_t* olen, uint64_t* ooff, uint64_t* plen, uint64_t* poff, uint64_t* tmp,
                            uint64_t* totals, uint8_t* dout, uint64_t out_cap, uint8_t* dpatch, uint64_t patch_cap,
                            am_doc_summary* summary, hipStream_t s);
// 16-byte copies of three segments (sizes multiples of 16) by a grid of `wgs` workgroups; the
// destinations are device pointers of mapped pinned host memory
void am_launch_copy_home(const void* s0, void* d0, uint64_t n0, const void* s1, void* d1, uint64_t n1, const void* s2, void* d2,
                         uint64_t n2, uint32_t wgs, hipStream_t s);
// DEFLATE on the GPU (am_inflate.hip): raw streams [src, src + len) of a source arena; pass 1 sizes
// them, pass 2 writes stream i's output at dst + zs[i].dst; k_copy_segs moves byte ranges from the
// source arena (from = 0) or a header blob (from = 1) to the new arena
struct am_zstream {
  uint64_t src, dst;
  uint32_t len;
  uint8_t hlen;     // > 0: a chunk header goes before the output: magic + hdr[0, hlen) (checksum, type, uleb)
  uint8_t hdr[11];
};
struct am_seg {
  uint64_t src, dst;
  uint32_t len, from;
};
// ord: the launch order (am_inflate_order): ord[0, nlong) are the long streams, largest first, decoded
// with one-lookup code tables; ord[nlong, nz) the rest
void am_launch_inflate_size(const uint8_t* src, const am_zstream* zs, const uint32_t* ord, uint32_t nlong, uint32_t nz,
                            uint32_t* zlen, hipStream_t s);
void am_launch_inflate_write(const uint8_t* src, const am_zstream* zs, const uint32_t* ord, uint32_t nlong, uint32_t nz,
                             const uint32_t* zlen, uint8_t* dst, hipStream_t s);
// the launch order of am_launch_inflate_*; returns nlong
uint32_t am_inflate_order(const am_zstream* zs, uint32_t nz, uint32_t* ord);
void am_launch_copy_segs(const uint8_t* src, const uint8_t* blob, const am_seg* segs, uint32_t n, uint8_t* dst, hipStream_t s);
// The device-side stage of a batch whose compressed chunks are all changes (no DEFLATEd base
// document): the classification, stream table, layout and header rewrite of inflate_stage's host
// code as kernels over the chunks.
//  classify: cnt[c] = 0, or (long << 32 | 1) for a compressed change (csrc / clen: its stream)
//  fill:     z0 = exclusive scan of cnt, nlong = its long total: the stream table, the launch order
//            (long streams first) and zid[c] (the chunk's stream, or ~0u)
//  layout:   nl[c] = the chunk's new length; the headers of the inflated chunks into zs
//  place:    new descriptors in place, the streams' destinations, every other chunk copied to dst
void am_launch_zstage_classify(const uint8_t* arena, uint64_t arena_len, const am_chunk_desc* chunks, uint32_t nchunks,
                               const am_doc_desc* docs, uint32_t ndocs, uint8_t* isbase, uint64_t* cnt, uint64_t* csrc,
                               uint32_t* clen, hipStream_t s);
void am_launch_zstage_fill(const uint64_t* cnt, const uint64_t* z0, uint32_t nchunks, uint32_t nlong, const uint64_t* csrc,
                           const uint32_t* clen, am_zstream* zs, uint32_t* ord, uint32_t* zid, hipStream_t s);
void am_launch_zstage_layout(const uint8_t* arena, const am_chunk_desc* chunks, uint32_t nchunks, const uint32_t* zid,
                             const uint32_t* zlen, am_zstream* zs, uint64_t* nl, hipStream_t s);
void am_launch_zstage_place(am_chunk_desc* chunks, uint32_t nchunks, const uint8_t* arena, const uint32_t* zid,
                            const uint32_t* zlen, am_zstream* zs, const uint64_t* noff, const uint64_t* nl, uint8_t* dst,
                            hipStream_t s);

// engine internals shared with am_sync.hip
struct am_engine;
hipStream_t am_engine_stream(am_engine* e);
int am_engine_device(am_engine* e);
void am_launch_bloom_build(const uint8_t* d_hashes, const uint64_t* d_hoff, uint32_t nfilt, uint8_t* d_out,
                           const uint64_t* d_foff, hipStream_t s);
void am_launch_bloom_probe(const uint8_t* d_filters, const uint64_t* d_foff, uint32_t nfilt, const uint8_t* d_probes,
                           const uint32_t* d_pfilt, uint64_t nprobe, uint8_t* d_contains, hipStream_t s);
void am_launch_sync_select(uint32_t npairs, const uint64_t* d_coff, const uint8_t* d_hashes, const uint64_t* d_doff,
                           const int32_t* d_didx, const uint64_t* d_pfoff, const uint8_t* d_filters, const uint64_t* d_foff,
                           uint8_t* d_send, uint8_t* d_status, hipStream_t s);

// k_history (am_hist_dev.h): one workgroup per document of the change history
void am_launch_history(const uint8_t* arena, const am_chunk_desc* chunks, const ChunkInfo* info, const HistDesc* hd, uint32_t ndocs,
                       uint8_t* ws, uint8_t* out, HistResult* res, HistChange* chg_out, hipStream_t s);
// per-document change bytes of the history batch (thread per document over its change records:
// offsets within the document, its total), then the dense copy (workgroup per document) to
// dst + doc_off[d] (an exclusive scan of the totals)
void am_launch_history_sizes(const HistResult* res, const HistDesc* hd, uint32_t ndocs, const uint32_t* nchg, HistChange* chg,
                             uint64_t* sizes, hipStream_t s);
void am_launch_history_compact(const HistResult* res, const HistDesc* hd, uint32_t ndocs, const uint32_t* nchg, const HistChange* chg,
                               const uint64_t* doc_off, const uint8_t* out, uint8_t* dst, hipStream_t s);
// the engine's history buffers (am_hist.hip), freed with the engine
void*& am_engine_hist(am_engine* e);
void am_hist_cache_free(void* cache);
void*& am_engine_sync(am_engine* e);
void am_sync_cache_free(void* cache);
// host stages of am_capi.hip shared with am_hist.hip: Backend.load's staging of a document chunk
// (DEFLATEd columns inflated, checksum verified), the reference error text of an AM_* code
bool am_stage_doc_chunk(am_engine* e, const std::vector<uint8_t>& in, std::vector<uint8_t>& out, bool& verified, am_error* err);
// am_stage_doc_chunk over n documents: one GPU checksum batch and one inflate batch; err_of(i)
// receives document i's error (out[i] is then empty)
void am_stage_doc_chunks(am_engine* e, size_t n, const uint8_t* const* data, const size_t* lens,
                         std::vector<std::vector<uint8_t>>& out, std::vector<uint8_t>& verified,
                         const std::function<am_error*(size_t)>& err_of);
std::string am_message_for(uint32_t code, int64_t a0, int64_t a1, const std::string& actor);
