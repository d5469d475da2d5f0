// am_unknown.h -- op columns outside DOC_OPS_COLUMNS / CHANGE_COLUMNS (columns of a future format
// version). The reference carries them through a merge unchanged: updateBlockColumns adds a
// change's unknown columns to the document (new.js:1387-1425), readOperation reads a value per op
// from every column -- or, for a column in the group of a GROUP_CARD column, as many values as that
// column says, and for a VALUE_RAW column the bytes its VALUE_LEN column announces -- remapping
// ACTOR_ID values through the change's actor table (new.js:570-611), and appendOperation writes
// them back, blanks for an op whose source lacks the column (new.js:618-655; null, false for
// BOOLEAN, 0 for VALUE_LEN and GROUP_CARD, no bytes for VALUE_RAW).
//
// Here: lane 0 collects every unknown column of every source (the base document, then the applied
// changes) into an instance table and decodes its values (rare input, so sequential); after the
// merge every distinct column is re-encoded over the rows in document order by the whole wave
// (encode_column), and the document assembly interleaves them with the known columns by id.
// Included by am_doc_impl.h inside its namespace (no include guard, like am_doc_impl.h).

struct UnkInst {
  uint32_t id, src, len, type;  // column id, source index, byte length, id & 7
  uint64_t off;                 // arena offset of the column bytes
  uint32_t cells, count;        // decoded values: unk_cells[cells .. cells + count)
  uint32_t member, card;        // 1: values per group entry; instance of the group's GROUP_CARD column
  uint32_t pre, uidx;           // card columns: per-row exclusive prefix at unk_cells[pre ..]; output column
};
static_assert(sizeof(UnkInst) == AM_SZ_UNKINST, "UnkInst");

__device__ __forceinline__ bool unk_member_type(uint32_t id, bool has_card) { return has_card && (id & 7) != 0; }

// lane 0: the instance table and the decoded values of every source's unknown columns
__device__ static void unk_collect(DocShared& s, const am_doc_desc& dd, const am_chunk_desc* chunks, const ChunkInfo* info,
                                   uint8_t* wsg) {
  const WsLayout& L = s.L;
  UnkInst* inst = reinterpret_cast<UnkInst*>(wsg + L.unk_inst);
  int64_t* cells = reinterpret_cast<int64_t*>(wsg + L.unk_cells);
  const uint64_t cells_cap = (uint64_t)s.b.UV + 2ull * s.b.R + 2;
  const APtr A = AV(s);
  const uint32_t nsrc = (s.has_base ? 1 : 0) + s.napplied;
  uint32_t ni = 0, nc = 0;
  for (uint32_t src = 0; src < nsrc; src++) {
    const SrcInfo si = src_info(s, src);
    const uint32_t ck = si.is_change ? dd.chg_begin + si.chg : (uint32_t)dd.base_chunk;
    if (info[ck].nunk == 0) continue;
    const uint64_t dabs = chunks[ck].off + info[ck].data_off;
    const uint32_t first = ni;
    uint32_t e = visit_unknown_cols(A + dabs, info[ck].data_len, !si.is_change, [&](uint32_t id, uint64_t off, uint32_t len) {
      if (ni >= s.b.UC) return;
      UnkInst& u = inst[ni++];
      u.id = id; u.src = src; u.len = len; u.type = id & 7; u.off = dabs + off;
      u.cells = 0; u.count = 0; u.member = 0; u.card = 0xffffffffu; u.pre = 0; u.uidx = 0;
    });
    if (e) { set_err(s, e); return; }
    // group structure (readOperation: the last GROUP_CARD column before a column sets its group;
    // the known card columns are predNum / succNum, groups 7 / 8, which hold no unknown ids)
    for (uint32_t k = first; k < ni; k++) {
      UnkInst& u = inst[k];
      if (u.type == 0 && (u.id >> 4) < 9) { set_err(s, AM_U_UNKNOWN_COLUMN); return; }  // would regroup known columns
      for (uint32_t j = first; j < k; j++)
        if (inst[j].type == 0 && (inst[j].id >> 4) == (u.id >> 4)) u.card = j;
      u.member = unk_member_type(u.id, u.card != 0xffffffffu);
      if (u.member && (u.type == 6 || u.type == 7)) { set_err(s, AM_U_UNKNOWN_COLUMN); return; }
    }
    // values, in column order (a group's card column and a VALUE_RAW's VALUE_LEN come first)
    for (uint32_t k = first; k < ni; k++) {
      UnkInst& u = inst[k];
      uint32_t n = si.nr;
      if (u.member) n = cells[inst[u.card].pre + si.nr];  // total entries of the group
      u.cells = nc;
      u.count = n;
      if ((uint64_t)nc + n + (u.type == 0 ? si.nr + 1 : 0) > cells_cap) { set_err(s, AM_U_CAPACITY); return; }
      if (u.type == 7) {  // VALUE_RAW: lengths from the VALUE_LEN column id - 1 of this source
        int32_t lv = -1;
        for (uint32_t j = first; j < k; j++) if (inst[j].id == u.id - 1 && inst[j].type == 6) lv = (int32_t)j;
        if (lv < 0) { set_err(s, AM_U_UNKNOWN_COLUMN); return; }
        uint64_t acc = 0;
        for (uint32_t q = 0; q < n; q++) {
          const int64_t t = cells[inst[lv].cells + q];
          const uint64_t nb = t == AM_NULL64 ? 0 : ((uint64_t)t >> 4);
          if (acc + nb > u.len) { set_err(s, AM_E_SUBARRAY); return; }
          cells[nc + q] = (int64_t)(((u.off + acc - s.b.span_lo) << 32) | nb);
          acc += nb;
        }
      } else {
        const uint8_t dt = u.type == 3 ? DT_DELTA : u.type == 4 ? DT_BOOL : u.type == 5 ? DT_UTF8 : DT_UINT;
        ColDec d;
        cd_init(d, dt, A + u.off, u.len);
        const int64_t sbase = (int64_t)(u.off - s.b.span_lo);
        for (uint32_t q = 0; q < n; q++) {
          int64_t v;
          uint32_t er;
          if (dt == DT_BOOL) {
            bool bv;
            er = cd_next_bool(d, bv);
            v = bv;
          } else {
            bool isnull;
            uint32_t l;
            int64_t x;
            er = cd_next(d, x, isnull, l);
            if (isnull) v = AM_NULL64;
            else if (dt == DT_UTF8) v = ((sbase + x) << 32) | (int64_t)l;
            else if (dt == DT_DELTA) v = (d.absolute += x);
            else v = x;
          }
          if (er) { set_err(s, er, 0, 0, 0, 0, si.chg); return; }
          if (u.type == 1 && v != AM_NULL64 && si.is_change) {  // ACTOR_ID through the change's actor table
            if (v < 0 || v >= (int64_t)si.nmap) { set_err(s, AM_U_VALUE); return; }
            v = (int64_t)si.map[v];
          }
          cells[nc + q] = v;
        }
        if (u.type == 0) {  // per-row entry offsets of the group
          u.pre = nc + n;
          int64_t acc = 0;
          for (uint32_t q = 0; q < n; q++) {
            cells[u.pre + q] = acc;
            const int64_t c = cells[nc + q];
            acc += (c == AM_NULL64 || c < 0) ? 0 : c;
          }
          cells[u.pre + n] = acc;
          nc += n + 1;
        }
      }
      nc += n;
    }
  }
  // distinct output columns (ascending id) and the (source, column) -> instance map
  uint32_t* ids = reinterpret_cast<uint32_t*>(wsg + L.unk_ids);
  uint32_t nu = 0;
  for (uint32_t k = 0; k < ni; k++) {
    uint32_t pos = 0;
    while (pos < nu && ids[pos] < inst[k].id) pos++;
    if (pos < nu && ids[pos] == inst[k].id) continue;
    for (uint32_t j = nu; j > pos; j--) ids[j] = ids[j - 1];
    ids[pos] = inst[k].id;
    nu++;
  }
  int32_t* map = reinterpret_cast<int32_t*>(wsg + L.unk_map);
  for (uint32_t x = 0; x < nsrc * nu; x++) map[x] = -1;
  for (uint32_t k = 0; k < ni; k++) {
    uint32_t pos = 0;
    while (ids[pos] != inst[k].id) pos++;
    inst[k].uidx = pos;
    map[inst[k].src * nu + pos] = (int32_t)k;
  }
  s.nunk_inst = ni;
  s.nunk_ids = nu;
}

// whole wave: the distinct unknown columns over the merged rows (sr, document order); column u's
// bytes go to unk_out at ids[nu + u] (length ids[2 nu + u])
__device__ static void unk_encode(DocShared& s, const SortRec* sr, uint32_t NOUT, EncCtx& ex, uint8_t* wsg) {
  const WsLayout& L = s.L;
  const UnkInst* inst = reinterpret_cast<const UnkInst*>(wsg + L.unk_inst);
  const int64_t* cells = reinterpret_cast<const int64_t*>(wsg + L.unk_cells);
  uint32_t* ids = reinterpret_cast<uint32_t*>(wsg + L.unk_ids);
  const int32_t* map = reinterpret_cast<const int32_t*>(wsg + L.unk_map);
  uint32_t* rowoff = reinterpret_cast<uint32_t*>(wsg + L.unk_rowoff);
  const uint32_t nu = s.nunk_ids, t = threadIdx.x;
  uint8_t* out = wsg + L.unk_out;
  uint64_t pos = 0;
  for (uint32_t u = 0; u < nu; u++) {
    const uint32_t id = ids[u], type = id & 7;
    // output group structure: the document's column list holds the card column of the group?
    int32_t cu = -1;
    for (uint32_t j = 0; j < u; j++) if ((ids[j] >> 4) == (id >> 4) && (ids[j] & 7) == 0) cu = (int32_t)j;
    const bool member = unk_member_type(id, cu >= 0);
    uint32_t n = NOUT;
    if (member) {
      for (uint32_t k = t; k < NOUT; k += blockDim.x) {
        const int32_t row = sr[k].row;
        const uint32_t src = src_of(s, (uint32_t)row, false);
        const int32_t ci = map[src * nu + cu];
        int64_t c = 0;
        if (ci >= 0) {
          c = cells[inst[ci].cells + (row - src_info(s, src).row0)];
          if (c == AM_NULL64 || c < 0) c = 0;
        }
        rowoff[k] = (uint32_t)c;
      }
      __syncthreads();
      n = block_excl_scan(rowoff, NOUT, s.tmp);
      __syncthreads();
    }
    if (n > L.enc_n) { if (t == 0) set_err(s, AM_U_CAPACITY); return; }
    for (uint32_t k = t; k < NOUT; k += blockDim.x) {
      const int32_t row = sr[k].row;
      const uint32_t src = src_of(s, (uint32_t)row, false);
      const SrcInfo si = src_info(s, src);
      const uint32_t q = row - si.row0;
      const int32_t ii = map[src * nu + u];
      const int64_t blank = (type == 4 || type == 6 || type == 0) ? 0 : AM_NULL64;
      if (!member) {
        ex.V[k] = ii >= 0 ? cells[inst[ii].cells + q] : (type == 7 ? 0 : blank);
      } else {
        const uint32_t o = rowoff[k], m = (k + 1 < NOUT ? rowoff[k + 1] : n) - o;
        const int32_t ci = map[src * nu + cu];
        const uint32_t base = (ii >= 0 && ci >= 0) ? inst[ii].cells + (uint32_t)cells[inst[ci].pre + q] : 0;
        for (uint32_t j = 0; j < m; j++) ex.V[o + j] = ii >= 0 ? cells[base + j] : blank;
      }
    }
    __syncthreads();
    const uint8_t kind = type == 3 ? EK_D : type == 4 ? EK_B : type == 5 ? EK_S : type == 7 ? EK_W : EK_U;
    if (t < 64) {
      const uint32_t len = encode_column(kind, n, out + pos, ex, nullptr);
      if (t == 0) { ids[nu + u] = (uint32_t)pos; ids[2 * nu + u] = len; }
    }
    __syncthreads();
    pos += ids[2 * nu + u];
  }
}
