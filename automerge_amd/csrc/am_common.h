// am_common.h -- data layout shared by the HIP kernels and the host side of libautomerge_amd.
//
// A *batch* is a set of independent documents resident in HBM. Each document is
//   (optional base document chunk) + (list of change chunks passed to applyChanges)
// which is exactly Backend.load(base) followed by Backend.applyChanges(state, changes)
// (reference: backend/backend.js:27-32, 104-107; backend/new.js:1695-1871).
#pragma once
#include <stdint.h>

#define AM_NULL64 ((int64_t)0x8000000000000000LL)
#define AM_NULL32 (-1)
#define AM_NOSTR 0xFFFFFFFFu

// ---- column ids (columnar.js:56-94) ----
enum : int {
  CT_GROUP = 0, CT_ACTOR = 1, CT_INT_RLE = 2, CT_DELTA = 3, CT_BOOL = 4, CT_STR = 5, CT_VLEN = 6, CT_VRAW = 7,
  COL_DEFLATE = 8
};
// op columns, index order = CHANGE_COLUMNS / DOC_OPS_COLUMNS order (pred* / succ* share 13..15)
enum : int {
  OC_OBJ_ACTOR = 0, OC_OBJ_CTR, OC_KEY_ACTOR, OC_KEY_CTR, OC_KEY_STR, OC_ID_ACTOR, OC_ID_CTR, OC_INSERT,
  OC_ACTION, OC_VAL_LEN, OC_VAL_RAW, OC_CHLD_ACTOR, OC_CHLD_CTR, OC_GRP_NUM, OC_GRP_ACTOR, OC_GRP_CTR, OC_NCOLS
};
// document change columns (DOCUMENT_COLUMNS)
enum : int {
  DC_ACTOR = 0, DC_SEQ, DC_MAXOP, DC_TIME, DC_MESSAGE, DC_DEPS_NUM, DC_DEPS_INDEX, DC_EXTRA_LEN, DC_EXTRA_RAW, DC_NCOLS
};

#include "../../include/automerge_amd.h"

// ---- per-chunk summary written by k_chunks (96 bytes) ----
// Compact parsed header of one chunk (128 B slot per chunk, written by k_chunks when the chunk
// data is shorter than 64 KiB; read by k_doc_fast instead of re-parsing). Typed views:
// ChgHdrC / DocHdrC in am_kernels.hip.
struct alignas(16) HdrSlot {
  uint8_t b[128];
};

struct ChunkInfo {
  uint8_t hash[32];
  uint32_t status;          // AM_* code
  uint32_t type;            // chunk type byte
  uint32_t data_off;        // chunk data offset relative to the chunk start
  uint32_t data_len;
  uint32_t nops;            // op rows (change: values in action column; doc: in idCtr column)
  uint32_t nents;           // pred entries (change) / succ entries (doc)
  uint32_t nchg;            // doc: change rows
  uint32_t ndeps;           // change: deps; doc: depsIndex entries
  uint32_t nactors;         // actor ids in the header (change: incl. author)
  uint32_t strbytes;        // bytes of key strings over all rows (+ messages)
  uint32_t nheads;          // doc: heads
  uint32_t nunk;            // op columns outside the known column set (new.js:1387-1425)
  int64_t arg0;             // error argument
};

// ---- device-side working rows (one per op) ----
struct Row {                // 96 bytes
  int64_t obj_ctr, key_ctr, id_ctr, chld_ctr, action, val_len;  // AM_NULL64 = null
  uint64_t val_off;         // arena offset of the raw value bytes
  uint64_t key_off;         // arena offset of the key string bytes
  int32_t obj_actor, key_actor, id_actor, chld_actor;            // doc actor index, -1 = null
  uint32_t key_len;         // AM_NOSTR = null key string
  uint32_t ps_off, ps_cnt;  // pred (change rows) / succ (doc rows) entries
  uint8_t insert, is_del, src_change, flags;
};
struct Ent {                // pred/succ entry
  int64_t ctr;
  int32_t actor;
  int32_t row;              // resolved target row (preds) / owning row
};
struct ChgRow {             // one row of the document's change columns (new.js:1680-1692)
  int64_t actor, seq, max_op, time;  // AM_NULL64 = null
  uint64_t msg_off;
  uint32_t msg_len;         // AM_NOSTR = null
  uint32_t ndeps;
  uint32_t deps_off;        // into the doc's deps array
  uint32_t extra_len_hi;
  int64_t extra_len;        // AM_NULL64 = null
  uint64_t extra_off;
  uint32_t extra_raw_len;
  uint32_t pad;
};
struct ActorRef { uint64_t off; uint32_t len; uint32_t rank; };
