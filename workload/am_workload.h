/*
 * am_workload.h -- synthetic workloads of SURVEY.md section 8(d) (bench.py input preparation, host
 * side). Built as workload/libam_workload.so; not part of the product library.
 */
#ifndef AM_WORKLOAD_H
#define AM_WORKLOAD_H
#include "../include/automerge_amd.h"

#ifdef __cplusplus
extern "C" {
#endif
/* C4: document i = base document (change 0 saved) + 12 concurrent changes (4 actors x 3), seeded
 * by i. Returns the arena bytes needed; fills arena/chunks (13 per doc)/docs when arena != NULL
 * and cap suffices. ops_out receives the number of ops in the 12 changes of all documents. */
uint64_t am_workload_c4(uint64_t first_doc, uint32_t ndocs, uint8_t *arena, uint64_t cap, am_chunk_desc *chunks,
                        am_doc_desc *docs, uint64_t *ops_out, int nthreads);
/* C2 (configs[1]): document i = Backend.init() + 3 changes (10 map/counter/string sets by actor 0;
 * two concurrent changes incrementing the counter and overwriting k1), 3 chunks per document. */
uint64_t am_workload_c2(uint64_t first_doc, uint32_t ndocs, uint8_t *arena, uint64_t cap, am_chunk_desc *chunks,
                        am_doc_desc *docs, uint64_t *ops_out, int nthreads);
/* C5 (configs[4]): document pair i = the C4 base + per_side changes by actor 1 (side A) and
 * per_side concurrent changes by actor 2 (side B); 1 + 2 * per_side chunks per pair. */
uint64_t am_workload_c5(uint64_t first_doc, uint32_t ndocs, uint32_t per_side, uint8_t *arena, uint64_t cap,
                        am_chunk_desc *chunks, am_doc_desc *docs, uint64_t *ops_out, int nthreads);
/* Text editing histories (C1: cross_every 0, two actors concurrent from the same base; C3:
 * cross_every 10, interleaved): document i = Backend.init() + 1 + nchanges change chunks (change 0
 * = makeText), per_change ops each (1/5 deletes of live elements, otherwise one-character
 * inserts), chunks >= 256 B deflated as encodeChange does (columnar.js:738). */
uint64_t am_workload_text(uint64_t first_doc, uint32_t ndocs, uint32_t nchanges, uint32_t per_change,
                          uint32_t cross_every, uint8_t *arena, uint64_t cap, am_chunk_desc *chunks,
                          am_doc_desc *docs, uint64_t *ops_out, int nthreads);
/* Mid-size documents (gen_mid): Backend.init() + 1 + nactors * rounds change chunks; nactors actors
 * edit one text and the title in rounds of concurrent changes of min_ops..max_ops ops. */
uint64_t am_workload_mid(uint64_t first, uint32_t n, uint32_t nactors, uint32_t rounds, uint32_t min_ops, uint32_t max_ops,
                         uint8_t *arena, uint64_t cap, am_chunk_desc *chunks, am_doc_desc *docs, uint64_t *ops, int nthreads);
/* Shard of the C4 job: indexes in [first, first + n) whose base document's checksum byte 0
 * (SHA-256 of the chunk) % world == rank. */
uint64_t am_workload_c4_shard(uint64_t first, uint64_t n, uint32_t world, uint32_t rank, uint64_t *ids, uint64_t cap,
                              int nthreads);
uint64_t am_workload_c4_list(const uint64_t *ids, uint32_t n, uint8_t *arena, uint64_t cap, am_chunk_desc *chunks,
                             am_doc_desc *docs, uint64_t *ops_out, int nthreads);
#ifdef __cplusplus
}
#endif
#endif
