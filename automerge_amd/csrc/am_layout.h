// am_layout.h -- per-document workspace layout (host + device). Every region is bounded from
// the per-chunk counts of k_chunks, so one exclusive scan sizes the whole batch.
//
// Two parts:
//   hot  -- everything the merge touches repeatedly (rows, sort keys, Euler tour, plan tables,
//           the document's input bytes). Placed in LDS when it fits the per-workgroup budget
//           (the common case for small documents), else in the global workspace.
//   cold -- streaming buffers written once (encoded columns, delta scratch, merged document).
#pragma once
#include <stdint.h>

#include "am_common.h"
#include "am_diff.h"

#ifndef __HIPCC__
#define AM_HD
#else
#define AM_HD __host__ __device__
#endif

// LDS budget of one document workgroup (bytes of dynamic shared memory). 64 KB: a C5 pair merged
// (~100 rows, a 40-64 KB hot set) runs in LDS mode, 1.7x faster than global mode (2 workgroups
// per CU against 4 four-wave ones; gfx950 has 160 KB of LDS per CU)
#define AM_LDS_BUDGET (64 * 1024)

struct DocBounds {
  uint32_t R;   // op rows (base + every change in the list)
  uint32_t E;   // pred/succ entries
  uint32_t C;   // document change rows
  uint32_t D;   // depsIndex entries
  uint32_t A;   // actor table
  uint32_t H;   // heads
  uint32_t N;   // changes in the list
  uint32_t K;   // changeIndexByHash entries
  uint32_t AM;  // actor-map entries (sum of change actor lists)
  uint32_t ND;  // sum of change deps (plan)
  uint32_t P;   // 1: write the getPatch() log (AM_DOC_WANT_PATCH); 2: the applyChanges patch (AM_DOC_WANT_DIFF)
  uint32_t U;   // bit0: invalid UTF-8 keys / messages are replaced (AM_DOC_FIX_UTF8): room for 3 bytes per input
                // byte; bit1: 8x applyChanges-patch pools (AM_DOC_PATCH_ROOM); bit2: k_doc_fast's compact
                // plan (ws_layout below; k_rest re-plans a document the fast kernel gives up on)
  uint32_t UC;  // instances of unknown op columns over the document's chunks (new.js:1387-1425)
  uint32_t UV;  // bound on their values
  uint64_t S;   // key + message string bytes over all rows
  uint64_t B;   // input bytes (base + changes)
  uint64_t span_lo, span_hi;  // arena byte span covering the document's chunks
};

struct WsLayout {
  // hot (offsets relative to the hot base). Regions after `u0` form a union: the decode cells
  // (dead once rows are built), the merge arrays (idk .. tour_w) and the encode scratch (used
  // after the merge) share the same bytes.
  uint64_t rows, ents, sortrec, scan, succ_cnt, outent, chg, deps, actors, clock, heads, hidx, chghdr, order, rowbase,
      entbase, ambase, amap, queue, enq, applied, amb_out, hashes, dup_of, self_idx, aut, can, dbase, dref, dref_idx,
      docpos, head_ref, input;
  uint64_t u0, idk, elemk, newent, elem_of, parent, first_child, next_sib, tour_nxt, tour_w;
  uint64_t cells;             // decode: (13 R + 2 E) int64 values
  uint64_t enc, enc_n;        // encode: V, W (int64) and S, RS, RB, RG (u32), enc_n entries each
  uint64_t pscr;              // getPatch scratch (PatchScratch arrays, after the encode)
  uint64_t hot_total;
  // cold (offsets relative to the document's global workspace, after the hot mirror)
  uint64_t out, out_cap, total;
  uint64_t patch, patch_nrec, patch_nmval, patch_heap;  // patch log, working form (when P)
  uint64_t pwire, pwire_cap;  // the same log in wire form (PatchHdr2 + stream, am_patch.h)
  uint64_t etime, passend, dscr;  // applyChanges patch (P == 2): succ-entry times, pass ends, replay pools
  uint64_t enc_x;             // encode scratch of waves 1..3 of a large document (0: wave 0 encodes alone)
  uint64_t djob;              // P == 2, global mode: the counts k_doc leaves for k_diff (8 x u32)
  uint64_t colbuf[OC_NCOLS + DC_NCOLS];
  // unknown op columns (UC > 0): instance table, decoded values, per-(source, column) instance
  // map, the output columns' ids / lengths / positions, per-row group offsets, encoded output
  uint64_t unk_inst, unk_cells, unk_map, unk_ids, unk_rowoff, unk_out, unk_out_cap;
};

#define AM_SZ_UNKINST 48

AM_HD inline uint32_t am_pow2(uint32_t n) {
  uint32_t p = 1;
  while (p < n) p <<= 1;
  return p;
}

// sizes of the device structs (kept in sync by static_asserts in am_kernels.hip)
#define AM_SZ_ROW 96
#define AM_SZ_ENT 16
#define AM_SZ_IDKEY 16
#define AM_SZ_ELEMKEY 32
#define AM_SZ_SORTREC 56
#define AM_SZ_NEWENT 24
#define AM_SZ_CHGROW 80
#define AM_SZ_ACTORREF 16
#define AM_SZ_CHGHDR 224

// k_doc_fast's plan (DocBounds.U bit 2): the heads, the output image and the patch's wire form --
// all the fast kernel writes to global memory. An image or a patch larger than these caps makes the
// fast kernel give up on the document (as any other miss does); k_rest then gives it the whole plan
// (ws_layout below) in the overflow region after the batch's workspaces. Its own small struct: the
// fast kernel reads only these, and the whole WsLayout there costs private (scratch) memory.
struct WsFast {
  uint64_t heads, out, out_cap, pwire, pwire_cap, total;
};
AM_HD inline WsFast ws_fast(const DocBounds& b) {
  WsFast F;
  const uint64_t span = b.span_hi - b.span_lo;
  auto r16 = [](uint64_t v) { return (v + 15) & ~(uint64_t)15; };
  F.heads = 0;
  F.out_cap = 64 + 40 * (uint64_t)b.A + 42 * (uint64_t)b.H + 300 + span + 10 * (uint64_t)b.R;
  F.out = r16((uint64_t)b.H * 32);
  F.pwire_cap = b.P ? 48 + 512 + 2 * b.B + 32 * ((uint64_t)b.R + b.A + b.C + b.H) : 0;
  F.pwire = F.out + r16(F.out_cap);
  F.total = F.pwire + (b.P ? r16(F.pwire_cap) : 0);
  return F;
}

AM_HD inline WsLayout ws_layout(const DocBounds& b) {
  WsLayout L;
  uint64_t o = 0;
  auto take = [&](uint64_t bytes) { uint64_t at = o; o += (bytes + 15) & ~(uint64_t)15; return at; };
  if (b.U & 4) {
    const WsFast F = ws_fast(b);
    L = WsLayout{};
    L.heads = F.heads;
    L.out = F.out; L.out_cap = F.out_cap;
    L.pwire = b.P ? F.pwire : 0; L.pwire_cap = F.pwire_cap;
    L.total = F.total;
    return L;
  }
  const uint64_t R = b.R, E = b.E, C = b.C, D = b.D, N = b.N;
  const uint64_t PR = am_pow2(b.R ? b.R : 1), PE = am_pow2(b.E ? b.E : 1);
  L.rows = take(R * AM_SZ_ROW);
  L.ents = take(E * AM_SZ_ENT);
  L.sortrec = take(PR * AM_SZ_SORTREC);
  L.scan = take(R * 4);
  L.succ_cnt = take(R * 4);
  L.outent = take(E * AM_SZ_ENT);
  L.chg = take(C * AM_SZ_CHGROW);
  L.deps = take(D * 8);
  L.actors = take((uint64_t)b.A * AM_SZ_ACTORREF);
  L.clock = take((uint64_t)(b.A + N) * 8);
  L.heads = take((uint64_t)b.H * 32);
  L.hidx = take((uint64_t)b.H * 8);
  L.chghdr = take(N * AM_SZ_CHGHDR);
  L.order = take(N * 4);
  L.rowbase = take(N * 4);
  L.entbase = take(N * 4);
  L.ambase = take(N * 4);
  L.amap = take((uint64_t)b.AM * 4);
  L.queue = take(N * 4);
  L.enq = take(N * 4);
  L.applied = take(N * 4);
  L.amb_out = take(N * 4);
  L.hashes = take(N * 32);
  L.dup_of = take(N * 4);
  L.self_idx = take(N * 8);
  L.aut = take(N * 4);
  L.can = take((uint64_t)b.AM * 4);
  L.dbase = take(N * 4);
  L.dref = take((uint64_t)b.ND * 4);
  L.dref_idx = take((uint64_t)b.ND * 8);
  L.docpos = take((uint64_t)(b.A + N) * 4);
  L.head_ref = take((uint64_t)b.H * 4);
  L.input = take((b.span_hi - b.span_lo) + ((b.U & 1) ? 3 * b.S + 64 : 0));
  // union region
  L.u0 = o;
  L.idk = take(PR * AM_SZ_IDKEY);
  L.elemk = take(PR * AM_SZ_ELEMKEY);
  L.newent = take(PE * AM_SZ_NEWENT);
  L.elem_of = take(R * 4);
  L.parent = take(R * 4);
  L.first_child = take(R * 4);
  L.next_sib = take(R * 4);
  L.tour_nxt = take(4 * R * 4);
  L.tour_w = take(4 * R * 4);
  uint64_t uend = o;
  L.cells = L.u0;
  const uint64_t cells_end = L.u0 + (((13 * R + 2 * E) * 8 + 15) & ~(uint64_t)15);
  if (cells_end > uend) uend = cells_end;
  uint64_t nm = R;
  if (b.UV > nm) nm = b.UV;
  if (E > nm) nm = E;
  if (C > nm) nm = C;
  if (D > nm) nm = D;
  nm = (nm + 3) & ~(uint64_t)3;
  L.enc = L.u0;
  L.enc_n = nm;
  const uint64_t enc_end = L.u0 + 32 * nm;
  if (enc_end > uend) uend = enc_end;
  // getPatch scratch: make ops (8+4+1 B) and counter states (8+4+8+4 B) per row, counter map
  // (8+4+4 B) per succ entry
  L.pscr = L.u0;
  const uint64_t pscr_end = L.u0 + (b.P == 1 ? 13 * (R + 1) + 24 * (R + 1) + 16 * (E + 1) + 16 * 10 : 0);
  if (pscr_end > uend) uend = pscr_end;
  // every region (and every document's workspace, placed by an exclusive scan of L.total) starts
  // 16-byte aligned: the global-mode hot set takes 64-bit atomics and the copies move 16-byte words
  o = (uend + 15) & ~(uint64_t)15;
  L.hot_total = o;
  // column buffers: a value costs at most 8 LEB bytes plus 2 bytes of RLE headers
  uint64_t cap = 0;
  for (int c = 0; c < OC_NCOLS + DC_NCOLS; c++) {
    uint64_t bound;
    if (c == OC_KEY_STR) bound = 10 * R + b.S;
    else if (c == OC_VAL_RAW) bound = b.B;
    else if (c == OC_INSERT) bound = 10 * (R + 1);
    else if (c == OC_GRP_ACTOR || c == OC_GRP_CTR) bound = 10 * E;
    else if (c < OC_NCOLS) bound = 10 * R;
    else if (c == OC_NCOLS + DC_MESSAGE) bound = 10 * C + b.S;
    else if (c == OC_NCOLS + DC_DEPS_INDEX) bound = 10 * D;
    else if (c == OC_NCOLS + DC_EXTRA_RAW) bound = b.B;
    else bound = 10 * C;
    bound += 16;
    L.colbuf[c] = take(bound);
    cap += bound;
  }
  // unknown op columns: a value costs at most 8 LEB bytes plus 2 bytes of RLE headers; raw bytes
  // come from the input
  const uint64_t UC = b.UC;
  L.unk_out_cap = UC ? UC * (10 * (R + b.UV) + 16 + 20) + b.B : 0;
  L.unk_out = UC ? take(L.unk_out_cap) : 0;
  cap += L.unk_out_cap;
  // document: header + actor ids + heads + column table + data + headsIndexes + extra bytes
  cap += 64 + 10 * (uint64_t)b.A + b.B + 42 * (uint64_t)b.H + 25 * 20 + b.B;
  L.out_cap = cap;
  L.out = take(cap);
  if (b.P == 1) {
    L.patch_nrec = 3 * R + b.A + C + 2;
    L.patch_nmval = R + 1;
    L.patch_heap = b.S + 2 * b.B + 16;
    L.patch = take(64 + 64 * L.patch_nrec + 32 * L.patch_nmval + L.patch_heap);
  } else if (b.P == 2) {
    // actors + clock + one section per object + keys + prop entries / edits (am_diff.h pools)
    const uint64_t ps = (b.U & 2) ? 8 : 1;
    L.patch_nrec = b.A + C + 2 + 2 * (R + 2) + ps * (8 * R + 128);
    L.patch_nmval = ps * (4 * R + 64);
    L.patch_heap = b.S + 2 * b.B + 16;
    L.patch = take(64 + 64 * L.patch_nrec + 32 * L.patch_nmval + L.patch_heap);
  } else {
    L.patch = L.patch_nrec = L.patch_nmval = L.patch_heap = 0;
  }
  // a packed record never exceeds its working-form size (am_patch.h patch_pack)
  L.pwire_cap = b.P ? 64 + 64 * L.patch_nrec + 32 * L.patch_nmval + L.patch_heap : 0;
  L.pwire = b.P ? take(L.pwire_cap) : 0;
  if (b.P == 2) {
    L.etime = take(4 * (E + 1));
    L.passend = take(4 * (N + 1));
    L.dscr = take(diff_scratch_bytes(R, E, (b.U & 2) ? 8 : 1));
    L.djob = take(32);
  } else {
    L.etime = L.passend = L.dscr = L.djob = 0;
  }
  // large documents: waves 1..3 of the global-mode workgroup encode columns of their own (P6)
  L.enc_x = nm >= 1024 ? take(3 * 32 * nm) : 0;
  if (UC) {
    L.unk_inst = take(UC * AM_SZ_UNKINST);
    L.unk_cells = take(((uint64_t)b.UV + 2 * R + 2) * 8);
    L.unk_map = take((N + 1) * UC * 4);
    L.unk_ids = take(UC * 16);
    L.unk_rowoff = take((R + 1) * 4);
  } else {
    L.unk_inst = L.unk_cells = L.unk_map = L.unk_ids = L.unk_rowoff = 0;
  }
  L.total = o;
  return L;
}
