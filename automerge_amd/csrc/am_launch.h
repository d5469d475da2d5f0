// am_launch.h -- host-side launchers of the kernels in am_kernels.hip.
#pragma once
#include <hip/hip_runtime.h>

#include "am_common.h"
#include "am_layout.h"

struct BatchDev {
  const uint8_t* arena;
  const am_chunk_desc* chunks;
  const am_doc_desc* docs;
  const am_known_hash* known;
  ChunkInfo* info;
  DocBounds* bounds;
  uint64_t* ws_bytes;      // per doc
  uint64_t* ws_off;        // per doc (exclusive scan)
  uint64_t* scan_tmp;      // block sums
  uint64_t* ws_total;      // 1 value
  uint64_t* max_hot;       // 1 value: largest hot working set of the batch
  uint32_t lds_bytes;      // dynamic LDS per document workgroup
  uint64_t max_hot_host;   // host copy of *max_hot
  uint8_t* ws;
  uint64_t ws_cap;
  am_doc_result* results;
  int32_t* chg_state;      // per chunk
  uint32_t nchunks, ndocs;
};

void am_launch_chunks(const BatchDev& b, hipStream_t s);
void am_launch_bounds(const BatchDev& b, hipStream_t s);   // k_bounds + scan of ws bytes
void am_launch_doc(const BatchDev& b, hipStream_t s);
void am_launch_out_hash(const BatchDev& b, hipStream_t s);
void am_launch_sha256(const uint8_t* arena, const am_chunk_desc* msgs, uint32_t n, uint8_t* out, hipStream_t s);
size_t am_scan_tmp_elems(uint32_t n);
