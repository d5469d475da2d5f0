// am_doc_impl.h -- the per-document merge kernel (k_doc) and its phases. Included twice by
// am_kernels.hip: namespace lds_mode (kHotLds = true: the hot working set and the document's
// input bytes live in LDS and every access compiles to ds_* instructions) and namespace glb_mode
// (kHotLds = false: documents whose working set exceeds the LDS budget run from the global
// workspace). Keeping the address space a compile-time fact matters on CDNA: generic (flat)
// accesses to LDS go through the vector-memory path and wait on outstanding global stores.

template <typename T>
__device__ __forceinline__ T* hp(DocShared& s, uint64_t off) {
  if constexpr (kHotLds) return reinterpret_cast<T*>(am_lds + off);
  else return reinterpret_cast<T*>(s.hot + off);
}
// View of the arena: AV(s) + arena_offset -> byte of the document's input. In LDS mode the base
// is the staged copy of [span_lo, span_hi); offsets are rebased before forming a pointer, so
// every pointer handed out stays inside the LDS allocation (no wrapped 32-bit arithmetic).
struct APtr {
  const uint8_t* base;
  uint64_t lo;
  __device__ __forceinline__ const uint8_t* operator+(uint64_t off) const { return base + (off - lo); }
  __device__ __forceinline__ uint8_t operator[](uint64_t off) const { return base[off - lo]; }
};
__device__ __forceinline__ APtr AV(DocShared& s) {
  if constexpr (kHotLds) return APtr{am_lds + s.L.input, s.b.span_lo};
  else return APtr{s.A, 0};
}

// A key or message with invalid UTF-8 is replaced by its decoded-and-re-encoded form (U+FFFD for
// every ill-formed subpart; the reference holds strings, encoding.js:15-17) written after the staged
// input bytes, so (off, len) keep addressing the arena view. Documents staged without
// AM_DOC_FIX_UTF8 (no room reserved) report AM_U_UTF8 and the host runs them again with it.
__device__ static bool fix_utf8(DocShared& s, uint64_t& off, uint32_t& len) {
  const APtr A = AV(s);
  if (utf8_valid_dev(A + off, len)) return true;
  if (!(s.b.U & 1) || doc_scattered(s.b)) { set_err(s, AM_U_UTF8); return false; }
  const uint32_t n = utf8_sanitize_dev(A + off, len, nullptr);
  const uint32_t at = atomicAdd(&s.xs_used, n);
  const uint64_t span = s.b.span_hi - s.b.span_lo;
  if ((uint64_t)at + n > 3 * s.b.S + 64) { set_err(s, AM_U_CAPACITY); return false; }
  utf8_sanitize_dev(A + off, len, hp<uint8_t>(s, s.L.input) + span + at);
  off = s.b.span_hi + at;
  len = n;
  return true;
}

__device__ static int64_t base_head_index(DocShared& s, uint32_t h) {
  if (s.dh.has_hidx) {
    Rd r{AV(s) + s.dh.base + s.dh.hidx_off, (uint64_t)1 << 40, 0};
    int64_t v = -1;
    for (uint32_t i = 0; i <= h; i++) rd_u53(r, v);
    return v;
  }
  return s.dh.nheads == 1 ? (int64_t)s.nbc - 1 : -1;
}

// ---- P2a: lane-parallel lookups -- hashes, duplicates, canonical actors, dependency refs ----
// Canonical actor ids: base actors 0..NB-1, the author of change j (first occurrence) NB + j.
// Dependency refs: >= 0 change index (first occurrence of that hash in the list),
// <= -10: base head (-10 - h), -2: host-known hash, -1: missing.
// first 8 bytes of a hash / id, little-endian (byte loads: any alignment)
__device__ __forceinline__ uint64_t pre8(const uint8_t* p) {
  uint64_t v = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) v |= (uint64_t)p[k] << (8 * k);
  return v;
}
// Candidates are found by comparing 8-byte prefixes (one load per candidate, independent of the
// others: the loop keeps several in flight); only a prefix hit compares the whole hash / id.
__device__ static void plan_lookups(DocShared& s, const am_doc_desc& dd, const ChunkInfo* info, const am_known_hash* known) {
  const WsLayout& L = s.L;
  const uint32_t N = dd.chg_count, t = threadIdx.x, T = blockDim.x;
  const ChgHdr* ch = hp<ChgHdr>(s, L.chghdr);
  uint8_t* hashes = hp<uint8_t>(s, L.hashes);
  const uint64_t* hw = reinterpret_cast<const uint64_t*>(hashes);  // 32-byte aligned entries
  const APtr A = AV(s);
  const uint32_t NB = s.has_base ? s.dh.nactors : 0;
  // each change's author id: 8-byte prefix and length, in tables P2b rewrites (queue, applied,
  // order are not read before it)
  uint32_t* apl = hp<uint32_t>(s, L.queue);
  uint32_t* aph = reinterpret_cast<uint32_t*>(hp<int32_t>(s, L.applied));
  uint32_t* alen = hp<uint32_t>(s, L.order);
  for (uint32_t c = t; c < N; c += T) {
    const uint32_t* src = reinterpret_cast<const uint32_t*>(info[dd.chg_begin + c].hash);
    uint32_t* dst = reinterpret_cast<uint32_t*>(hashes + 32 * c);
    for (int k = 0; k < 8; k++) dst[k] = src[k];
    const ChgHdr& h = ch[c];
    uint8_t b8[8];
    for (uint32_t k = 0; k < 8; k++) b8[k] = k < h.actor_len ? A[h.base + h.actor_off + k] : 0;
    uint64_t v = 0;
    for (int k = 0; k < 8; k++) v |= (uint64_t)b8[k] << (8 * k);
    apl[c] = (uint32_t)v;
    aph[c] = (uint32_t)(v >> 32);
    alen[c] = h.actor_len;
  }
  __syncthreads();
  uint32_t* dup_of = hp<uint32_t>(s, L.dup_of);
  int64_t* self_idx = hp<int64_t>(s, L.self_idx);
  int32_t* aut = hp<int32_t>(s, L.aut);
  int32_t* can = hp<int32_t>(s, L.can);
  int32_t* dref = hp<int32_t>(s, L.dref);
  int64_t* dref_idx = hp<int64_t>(s, L.dref_idx);
  const uint32_t* ambase = hp<uint32_t>(s, L.ambase);
  const uint32_t* dbase = hp<uint32_t>(s, L.dbase);
  auto base_actor = [&](uint64_t off, uint32_t len) -> int32_t {
    if (!s.has_base) return -1;
    Rd r{A + s.dh.base + s.dh.actors_off, (uint64_t)1 << 40, 0};
    for (uint32_t i = 0; i < s.dh.nactors; i++) {
      int64_t l;
      rd_u53(r, l);
      if ((uint32_t)l == len && bytes_eq(r.p + r.off, A + off, len)) return (int32_t)i;
      r.off += (uint64_t)l;
    }
    return -1;
  };
  auto author_canon = [&](uint64_t off, uint32_t len, uint32_t upto) -> int32_t {
    int32_t a = base_actor(off, len);
    if (a >= 0) return a;
    uint8_t b8[8];
    for (uint32_t k = 0; k < 8; k++) b8[k] = k < len ? A[off + k] : 0;
    uint64_t v = 0;
    for (int k = 0; k < 8; k++) v |= (uint64_t)b8[k] << (8 * k);
    const uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
    for (uint32_t j0 = 0; j0 < upto; j0 += 8) {
      uint32_t m = 0;  // candidates among j0 .. j0 + 7: their loads issue together
#pragma unroll
      for (uint32_t u = 0; u < 8; u++) {
        const uint32_t j = j0 + u;
        if (j < upto && apl[j] == lo && aph[j] == hi && alen[j] == len) m |= 1u << u;
      }
      for (; m; m &= m - 1) {
        const uint32_t j = j0 + (uint32_t)__builtin_ctz(m);
        const ChgHdr& hj = ch[j];
        if (bytes_eq(A + hj.base + hj.actor_off, A + off, len)) return (int32_t)(NB + j);
      }
    }
    return -1;
  };
  // first change j < n whose hash is h (its 8-byte prefix p): -1 if none
  auto find_hash = [&](const uint8_t* h, uint64_t p, uint32_t n) -> int32_t {
    for (uint32_t j0 = 0; j0 < n; j0 += 8) {
      uint32_t m = 0;
#pragma unroll
      for (uint32_t u = 0; u < 8; u++) {
        const uint32_t j = j0 + u;
        if (j < n && hw[4 * j] == p) m |= 1u << u;
      }
      for (; m; m &= m - 1) {
        const uint32_t j = j0 + (uint32_t)__builtin_ctz(m);
        if (hash_eq(hashes + 32 * j, h)) return (int32_t)j;
      }
    }
    return -1;
  };
  auto match_base = [&](const uint8_t* h, int32_t& ref, int64_t& idx) -> bool {
    if (s.has_base)
      for (uint32_t k = 0; k < s.dh.nheads; k++)
        if (hash_eq(A + s.dh.base + s.dh.heads_off + 32 * k, h)) { ref = -10 - (int32_t)k; idx = base_head_index(s, k); return true; }
    const uint64_t p = pre8(h);
    const am_known_hash* kn = known + dd.known_begin;
    for (uint32_t k0 = 0; k0 < dd.known_count; k0 += 8) {
      uint32_t m = 0;
#pragma unroll
      for (uint32_t u = 0; u < 8; u++)
        if (k0 + u < dd.known_count && *reinterpret_cast<const uint64_t*>(kn[k0 + u].hash) == p) m |= 1u << u;
      for (; m; m &= m - 1) {
        const uint32_t k = k0 + (uint32_t)__builtin_ctz(m);
        if (hash_eq(kn[k].hash, h)) {
          ref = -2;
          idx = kn[k].index;
          return true;
        }
      }
    }
    return false;
  };
  for (uint32_t c = t; c < N; c += T) {
    const ChgHdr& h = ch[c];
    const uint8_t* hc = hashes + 32 * c;
    const uint64_t pc = hw[4 * c];
    const int32_t dj = find_hash(hc, pc, c);
    dup_of[c] = dj >= 0 ? (uint32_t)dj : c;
    int32_t ref;
    int64_t idx;
    self_idx[c] = match_base(hc, ref, idx) ? idx : (int64_t)-2;
    aut[c] = author_canon(h.base + h.actor_off, h.actor_len, c + 1);
    uint32_t am = ambase[c];
    can[am] = aut[c];
    Rd ar{A + h.base + h.actors_off, (uint64_t)1 << 40, 0};
    for (uint32_t k = 1; k < h.nactors; k++) {
      int64_t l;
      rd_u53(ar, l);
      can[am + k] = author_canon(h.base + h.actors_off + ar.off, (uint32_t)l, N);
      ar.off += (uint64_t)l;
    }
    for (uint32_t di = 0; di < h.ndeps; di++) {
      const uint8_t* dep = A + h.base + h.deps_off + 32 * di;
      int32_t r = -1;
      int64_t x = 0;
      if (!match_base(dep, r, x)) r = find_hash(dep, pre8(dep), N);
      dref[dbase[c] + di] = r;
      dref_idx[dbase[c] + di] = x;
    }
  }
}

__device__ static bool plan_heads(DocShared& s, uint32_t nheads, uint32_t nall, uint32_t nq);

// ---- P2b: causal queue, clock, actor table, heads (one lane; integer work only) ----
__device__ static void plan_doc(DocShared& s, const am_doc_desc& dd, const ChunkInfo* info, int32_t* chg_state) {
  const WsLayout& L = s.L;
  const APtr A = AV(s);
  ActorRef* actors = hp<ActorRef>(s, L.actors);
  int64_t* clock = hp<int64_t>(s, L.clock);
  int32_t* docpos = hp<int32_t>(s, L.docpos);
  int32_t* head_ref = hp<int32_t>(s, L.head_ref);
  ChgRow* chg = hp<ChgRow>(s, L.chg);
  int64_t* deps = hp<int64_t>(s, L.deps);
  const ChgHdr* ch = hp<ChgHdr>(s, L.chghdr);
  uint32_t* order = hp<uint32_t>(s, L.order);
  uint32_t* rowbase = hp<uint32_t>(s, L.rowbase);
  uint32_t* entbase = hp<uint32_t>(s, L.entbase);
  uint32_t* ambase_out = hp<uint32_t>(s, L.amb_out);  // per applied change, its amap base
  uint32_t* amap = hp<uint32_t>(s, L.amap);
  uint32_t* queue = hp<uint32_t>(s, L.queue);
  const uint8_t* hashes = hp<uint8_t>(s, L.hashes);
  const uint32_t* dup_of = hp<uint32_t>(s, L.dup_of);
  const int64_t* self_idx = hp<int64_t>(s, L.self_idx);
  const int32_t* aut = hp<int32_t>(s, L.aut);
  const int32_t* can = hp<int32_t>(s, L.can);
  const int32_t* dref = hp<int32_t>(s, L.dref);
  const int64_t* dref_idx = hp<int64_t>(s, L.dref_idx);
  const uint32_t* ambase = hp<uint32_t>(s, L.ambase);
  const uint32_t* dbase = hp<uint32_t>(s, L.dbase);
  int32_t* applied = hp<int32_t>(s, L.applied);  // applied index per change (first occurrence of its hash)
  const uint32_t N = dd.chg_count;
  const uint32_t NB = s.has_base ? s.dh.nactors : 0;

  // base actors + clock (readDocumentChanges, new.js:1645-1675)
  uint32_t na = 0;
  if (s.has_base) {
    Rd r{A + s.dh.base + s.dh.actors_off, (uint64_t)1 << 40, 0};
    for (uint32_t i = 0; i < NB; i++) {
      int64_t l;
      rd_u53(r, l);
      actors[na].off = s.dh.base + s.dh.actors_off + r.off;
      actors[na].len = (uint32_t)l;
      r.off += (uint64_t)l;
      docpos[na] = (int32_t)na;
      na++;
    }
  }
  for (uint32_t i = 0; i < NB + N; i++) clock[i] = 0;
  for (uint32_t j = 0; j < N; j++) { docpos[NB + j] = -1; applied[j] = -1; }
  for (uint32_t i = 0; i < s.nbc; i++) {
    int64_t a = chg[i].actor, seq = chg[i].seq;
    if (a == AM_NULL64 || a < 0 || a >= (int64_t)NB || seq == AM_NULL64) { set_err(s, AM_U_VALUE); return; }
    if (seq != 1 && seq != clock[a] + 1) {
      set_err(s, AM_E_DOC_SEQ, clock[a] == 0 ? AM_NULL64 : clock[a] + 1, seq, actors[a].off, actors[a].len);
      return;
    }
    clock[a] = seq;
  }
  uint32_t nheads = 0;
  if (s.has_base)
    for (uint32_t h = 0; h < s.dh.nheads; h++) head_ref[nheads++] = -10 - (int32_t)h;

  const bool have_graph = (dd.flags & 1) != 0;
  uint32_t nq = N;
  for (uint32_t i = 0; i < nq; i++) { queue[i] = i; chg_state[dd.chg_begin + i] = CHG_UNSEEN; }
  uint32_t nall = 0, nrow = s.nb, nent = s.nbe, nam = 0, ndep = s.nbd;
  int64_t max_op = 0;
  for (;;) {
    // one pass of applyChanges() (new.js:1550-1597)
    uint32_t ne = 0, na_pass = 0;
    for (uint32_t qi = 0; qi < nq; qi++) {
      const uint32_t c = queue[qi];
      const ChunkInfo& ci = info[dd.chg_begin + c];
      const ChgHdr& h = ch[c];
      const uint32_t j0 = dup_of[c];
      if (self_idx[c] != -2 || applied[j0] >= 0) { chg_state[dd.chg_begin + c] = CHG_DUP; continue; }
      bool ready = true;
      for (uint32_t di = 0; di < h.ndeps && ready; di++) {
        int32_t r = dref[dbase[c] + di];
        if (r >= 0) ready = applied[r] >= 0;
        else if (r == -1) ready = false;
        else ready = dref_idx[dbase[c] + di] != -1;
      }
      if (!ready) { queue[ne++] = c; continue; }
      const int32_t a = aut[c];
      const int64_t expected = clock[a] + 1;
      if (h.seq < expected) {
        if (have_graph) { set_err(s, AM_E_REUSE_SEQ, h.seq, 0, h.base + h.actor_off, h.actor_len, c); return; }
        set_err(s, AM_U_HASH_GRAPH);
        return;
      }
      if (h.seq > expected) { set_err(s, AM_E_SKIPPED_SEQ, expected, 0, h.base + h.actor_off, h.actor_len, c); return; }
      clock[a] = h.seq;
      if (docpos[a] < 0) {  // getActorTable appends a new author (new.js:1435-1441)
        docpos[a] = (int32_t)na;
        actors[na].off = h.base + h.actor_off;
        actors[na].len = h.actor_len;
        na++;
      }
      // actor table of the change's columns (getActorTable, new.js:1442-1450)
      ambase_out[nall] = nam;
      Rd ar{A + h.base + h.actors_off, (uint64_t)1 << 40, 0};
      for (uint32_t k = 0; k < h.nactors; k++) {
        int32_t x = can[ambase[c] + k];
        uint64_t aoff = h.base + h.actor_off;
        uint32_t alen = h.actor_len;
        if (k > 0) {
          int64_t l;
          rd_u53(ar, l);
          aoff = h.base + h.actors_off + ar.off;
          alen = (uint32_t)l;
          ar.off += (uint64_t)l;
        }
        if (x < 0 || docpos[x] < 0) { set_err(s, AM_E_UNKNOWN_ACTOR, 0, 0, aoff, alen, c); return; }
        amap[nam++] = (uint32_t)docpos[x];
      }
      // heads: drop the dependencies, add this change (new.js:1581-1583)
      for (uint32_t di = 0; di < h.ndeps; di++) {
        int32_t r = dref[dbase[c] + di];
        for (uint32_t q = 0; q < nheads; q++)
          if (head_ref[q] == r && r != -1 && r != -2) { head_ref[q] = head_ref[--nheads]; break; }
      }
      bool present = false;
      for (uint32_t q = 0; q < nheads; q++) present |= head_ref[q] == (int32_t)j0;
      if (!present) head_ref[nheads++] = (int32_t)j0;
      applied[j0] = (int32_t)nall;
      order[nall] = c;
      rowbase[nall] = nrow;
      entbase[nall] = nent;
      nrow += ci.nops;
      nent += ci.nents;
      // appendChange row (new.js:1680-1692)
      ChgRow& cr = chg[s.nbc + nall];
      cr.actor = docpos[a];
      cr.seq = h.seq;
      cr.max_op = h.start_op + (int64_t)ci.nops - 1;
      cr.time = h.time;
      cr.msg_off = h.base + h.msg_off;
      cr.msg_len = h.msg_len;
      if (!fix_utf8(s, cr.msg_off, cr.msg_len)) return;
      cr.ndeps = h.ndeps;
      cr.deps_off = ndep;
      ndep += h.ndeps;
      cr.extra_len = h.has_extra ? (int64_t)(((uint64_t)h.extra_len << 4) | 7) : 7;
      cr.extra_off = h.base + h.extra_off;
      cr.extra_raw_len = h.has_extra ? h.extra_len : 0;
      if (ci.nops > 0 && cr.max_op > max_op) max_op = cr.max_op;
      chg_state[dd.chg_begin + c] = (int32_t)nall;
      nall++;
      na_pass++;
    }
    // pass boundaries of the applied op stream (the applyChanges patch replays pass by pass)
    if (na_pass > 0 && s.b.P == 2) reinterpret_cast<uint32_t*>(s.ws + L.passend)[s.npass++] = nrow - s.nb;
    nq = ne;
    if (nq == 0) break;
    if (na_pass == 0) {
      if (have_graph) break;
      set_err(s, AM_U_HASH_GRAPH);  // BackendDoc.applyChanges would computeHashGraph() (new.js:1830)
      return;
    }
  }
  for (uint32_t i = 0; i < nq; i++) chg_state[dd.chg_begin + queue[i]] = CHG_QUEUED;
  // deps indexes of the appended change rows: changeIndexByHash[dep]
  for (uint32_t k = 0; k < nall; k++) {
    const uint32_t c = order[k];
    const ChgHdr& h = ch[c];
    ChgRow& cr = chg[s.nbc + k];
    for (uint32_t di = 0; di < h.ndeps; di++) {
      int32_t r = dref[dbase[c] + di];
      deps[cr.deps_off + di] = r >= 0 ? (int64_t)(s.nbc + applied[r]) : dref_idx[dbase[c] + di];
    }
  }
  if (!plan_heads(s, nheads, nall, nq)) return;
  s.napplied = nall;
  s.nqueued = nq;
  s.nactors = na;
  s.nrows = nrow;
  s.nents = nent;
  s.nchg = s.nbc + nall;
  s.ndeps = ndep;
  s.max_op = max_op;
}

// heads (sorted, new.js:1593) with their headsIndexes, from head_ref[0, nheads): false on an error
__device__ static bool plan_heads(DocShared& s, uint32_t nheads, uint32_t nall, uint32_t nq) {
  const WsLayout& L = s.L;
  const APtr A = AV(s);
  uint8_t* heads = hp<uint8_t>(s, L.heads);
  const int32_t* head_ref = hp<int32_t>(s, L.head_ref);
  const uint8_t* hashes = hp<uint8_t>(s, L.hashes);
  const int32_t* applied = hp<int32_t>(s, L.applied);
  int64_t* hidx = hp<int64_t>(s, L.hidx);
  for (uint32_t q = 0; q < nheads; q++) {
    int32_t r = head_ref[q];
    const uint8_t* src = r >= 0 ? hashes + 32 * r : A + s.dh.base + s.dh.heads_off + 32 * (uint32_t)(-10 - r);
    for (int k = 0; k < 32; k++) heads[32 * q + k] = src[k];
    hidx[q] = r >= 0 ? (int64_t)(s.nbc + applied[r]) : base_head_index(s, (uint32_t)(-10 - r));
  }
  for (uint32_t a2 = 1; a2 < nheads; a2++)
    for (uint32_t b2 = a2; b2 > 0 && hash_cmp(heads + 32 * (b2 - 1), heads + 32 * b2) > 0; b2--) {
      for (int k = 0; k < 32; k++) { uint8_t tt = heads[32 * b2 + k]; heads[32 * b2 + k] = heads[32 * (b2 - 1) + k]; heads[32 * (b2 - 1) + k] = tt; }
      int64_t ti = hidx[b2]; hidx[b2] = hidx[b2 - 1]; hidx[b2 - 1] = ti;
    }
  if (nall > 0 || nq > 0)
    for (uint32_t q = 0; q < nheads; q++)
      if (hidx[q] < 0) { set_err(s, AM_U_HASH_GRAPH); return false; }
  s.nheads = nheads;
  return true;
}

// ---- P2b, closed form: when every change of the call applies in the first pass of the queue in
// list order -- no duplicate, every dependency an earlier change of the call or a base head /
// host-known hash with its index, each author's seq the next one, every actor of a change known by
// then, messages valid UTF-8 -- applyChanges' loop (new.js:1550-1597) reduces to prefix sums and
// per-change counts, computed by the whole workgroup (a lane per change) instead of plan_doc's one
// lane over chains of dependent loads. Returns false (nothing the queue reads written) when the
// call is not of that shape: plan_doc then runs the queue and reports the reference's errors. ----
__device__ static bool plan_fast(DocShared& s, const am_doc_desc& dd, const ChunkInfo* info, int32_t* chg_state) {
  const WsLayout& L = s.L;
  const APtr A = AV(s);
  const uint32_t t = threadIdx.x, T = blockDim.x;
  const uint32_t N = dd.chg_count;
  const uint32_t NB = s.has_base ? s.dh.nactors : 0;
  const uint32_t HB = s.has_base ? s.dh.nheads : 0;
  if (N == 0 || HB > T) return false;
  ActorRef* actors = hp<ActorRef>(s, L.actors);
  int64_t* clock = hp<int64_t>(s, L.clock);
  int32_t* docpos = hp<int32_t>(s, L.docpos);
  int32_t* head_ref = hp<int32_t>(s, L.head_ref);
  ChgRow* chg = hp<ChgRow>(s, L.chg);
  int64_t* deps = hp<int64_t>(s, L.deps);
  const ChgHdr* ch = hp<ChgHdr>(s, L.chghdr);
  uint32_t* order = hp<uint32_t>(s, L.order);
  uint32_t* rowbase = hp<uint32_t>(s, L.rowbase);
  uint32_t* entbase = hp<uint32_t>(s, L.entbase);
  uint32_t* ambase_out = hp<uint32_t>(s, L.amb_out);
  uint32_t* amap = hp<uint32_t>(s, L.amap);
  uint32_t* refd = hp<uint32_t>(s, L.queue);  // change j is some change's dependency
  const uint32_t* dup_of = hp<uint32_t>(s, L.dup_of);
  const int64_t* self_idx = hp<int64_t>(s, L.self_idx);
  const int32_t* aut = hp<int32_t>(s, L.aut);
  const int32_t* can = hp<int32_t>(s, L.can);
  const int32_t* dref = hp<int32_t>(s, L.dref);
  const int64_t* dref_idx = hp<int64_t>(s, L.dref_idx);
  const uint32_t* ambase = hp<uint32_t>(s, L.ambase);
  const uint32_t* dbase = hp<uint32_t>(s, L.dbase);
  int32_t* applied = hp<int32_t>(s, L.applied);
  // the base document's actors and clock (readDocumentChanges, new.js:1645-1675), as plan_doc
  if (t == 0) {
    s.pf_ok = 1;
    s.pf_nheads = HB;
    s.pf_maxop = 0;
    if (s.has_base) {
      Rd r{A + s.dh.base + s.dh.actors_off, (uint64_t)1 << 40, 0};
      for (uint32_t i = 0; i < NB; i++) {
        int64_t l;
        rd_u53(r, l);
        actors[i].off = s.dh.base + s.dh.actors_off + r.off;
        actors[i].len = (uint32_t)l;
        r.off += (uint64_t)l;
        docpos[i] = (int32_t)i;
      }
    }
    for (uint32_t i = 0; i < NB + N; i++) clock[i] = 0;
    for (uint32_t i = 0; i < s.nbc && s.pf_ok; i++) {
      const int64_t a = chg[i].actor, seq = chg[i].seq;
      if (a == AM_NULL64 || a < 0 || a >= (int64_t)NB || seq == AM_NULL64 || (seq != 1 && seq != clock[a] + 1)) s.pf_ok = 0;
      else clock[a] = seq;
    }
  }
  __syncthreads();
  if (!s.pf_ok) return false;  // plan_doc reports the base document's error
  // the shape checks, a lane per change
  bool ok = true;
  for (uint32_t c = t; c < N && ok; c += T) {
    const ChgHdr& h = ch[c];
    ok = dup_of[c] == c && self_idx[c] == -2;
    for (uint32_t di = 0; di < h.ndeps && ok; di++) {
      const int32_t r = dref[dbase[c] + di];
      ok = r >= 0 ? (uint32_t)r < c : (r != -1 && dref_idx[dbase[c] + di] != -1);
    }
    const int32_t a = aut[c];
    uint32_t prior = 0;
    for (uint32_t j = 0; j < c; j++) prior += aut[j] == a ? 1u : 0u;
    ok = ok && a >= 0 && h.seq == (a < (int32_t)NB ? clock[a] : 0) + (int64_t)prior + 1;
    for (uint32_t k = 0; k < h.nactors && ok; k++) {
      const int32_t x = can[ambase[c] + k];
      ok = x >= 0 && (x < (int32_t)NB || (uint32_t)(x - (int32_t)NB) <= c);
    }
    ok = ok && utf8_valid_dev(A + h.base + h.msg_off, h.msg_len);
  }
  if (!ok) atomicAnd(&s.pf_ok, 0u);
  __syncthreads();
  if (!s.pf_ok) return false;
  // per-change counts -> prefix sums (rows, entries, new authors)
  for (uint32_t c = t; c < N; c += T) {
    const ChunkInfo& ci = info[dd.chg_begin + c];
    rowbase[c] = ci.nops;
    entbase[c] = ci.nents;
    order[c] = aut[c] == (int32_t)(NB + c) ? 1u : 0u;  // the first change of a new author
    refd[c] = 0;
  }
  __syncthreads();
  const uint32_t nrow = block_excl_scan(rowbase, N, s.tmp);
  const uint32_t nent = block_excl_scan(entbase, N, s.tmp);
  const uint32_t nnew = block_excl_scan(order, N, s.tmp);
  // new authors in application order (getActorTable, new.js:1435-1441)
  for (uint32_t c = t; c < N; c += T) {
    const bool isnew = aut[c] == (int32_t)(NB + c);
    const uint32_t dp = NB + order[c];
    docpos[NB + c] = isnew ? (int32_t)dp : -1;
    if (isnew) {
      actors[dp].off = ch[c].base + ch[c].actor_off;
      actors[dp].len = ch[c].actor_len;
    }
  }
  __syncthreads();
  uint32_t* bref = s.tmp;  // base head h is some change's dependency (HB <= T)
  if (t < HB) bref[t] = 0;
  __syncthreads();
  for (uint32_t c = t; c < N; c += T) {
    const ChgHdr& h = ch[c];
    const ChunkInfo& ci = info[dd.chg_begin + c];
    const int32_t a = aut[c];
    bool last = true;
    for (uint32_t j = c + 1; j < N && last; j++) last = aut[j] != a;
    if (last) clock[a] = h.seq;
    ambase_out[c] = ambase[c];
    for (uint32_t k = 0; k < h.nactors; k++) amap[ambase[c] + k] = (uint32_t)docpos[can[ambase[c] + k]];
    for (uint32_t di = 0; di < h.ndeps; di++) {
      const int32_t r = dref[dbase[c] + di];
      if (r >= 0) refd[r] = 1;
      else if (r <= -10) bref[-10 - r] = 1;
      deps[s.nbd + dbase[c] + di] = r >= 0 ? (int64_t)(s.nbc + (uint32_t)r) : dref_idx[dbase[c] + di];
    }
    applied[c] = (int32_t)c;
    chg_state[dd.chg_begin + c] = (int32_t)c;
    rowbase[c] += s.nb;
    entbase[c] += s.nbe;
    // appendChange row (new.js:1680-1692)
    ChgRow& cr = chg[s.nbc + c];
    cr.actor = docpos[a];
    cr.seq = h.seq;
    cr.max_op = h.start_op + (int64_t)ci.nops - 1;
    cr.time = h.time;
    cr.msg_off = h.base + h.msg_off;
    cr.msg_len = h.msg_len;
    cr.ndeps = h.ndeps;
    cr.deps_off = s.nbd + dbase[c];
    cr.extra_len = h.has_extra ? (int64_t)(((uint64_t)h.extra_len << 4) | 7) : 7;
    cr.extra_off = h.base + h.extra_off;
    cr.extra_raw_len = h.has_extra ? h.extra_len : 0;
    if (ci.nops > 0 && cr.max_op > 0) atomicMax(&s.pf_maxop, (unsigned long long)cr.max_op);
  }
  __syncthreads();
  // heads: the base heads and changes nothing in the call depends on (new.js:1581-1583)
  if (t < HB && !bref[t]) head_ref[atomicAdd(&s.pf_nheads, 1u) - HB] = -10 - (int32_t)t;
  __syncthreads();
  for (uint32_t c = t; c < N; c += T) {
    order[c] = c;
    if (!refd[c]) head_ref[atomicAdd(&s.pf_nheads, 1u) - HB] = (int32_t)c;
  }
  __syncthreads();
  if (t == 0) {
    // pf_nheads counted from HB: the base heads kept and the change heads
    const uint32_t nheads = s.pf_nheads - HB;
    if (s.b.P == 2) reinterpret_cast<uint32_t*>(s.ws + L.passend)[s.npass++] = nrow;
    if (plan_heads(s, nheads, N, 0)) {
      s.napplied = N;
      s.nqueued = 0;
      s.nactors = NB + nnew;
      s.nrows = s.nb + nrow;
      s.nents = s.nbe + nent;
      s.nchg = s.nbc + N;
      s.ndeps = s.nbd + (N ? dbase[N - 1] + ch[N - 1].ndeps : 0);
      s.max_op = (int64_t)s.pf_maxop;
    }
  }
  return true;
}

// ---- P4: column decode. Every lane runs the same stream decoder over one (source, column)
// stream into a dense cell array; a lane-per-row gather then assembles the rows, and two scans
// place the raw values and the pred/succ groups (readOperation new.js:557-611, 700-724). ----
// value type of each op column as decoded: 0 uint RLE, 3 delta, 2 utf8, 4 boolean
__device__ __constant__ static const uint8_t kOpColDec[OC_NCOLS] = {
    DT_UINT, DT_UINT, DT_UINT, DT_DELTA, DT_UTF8, DT_UINT, DT_DELTA, DT_BOOL,
    DT_UINT, DT_UINT, DT_UINT, DT_UINT, DT_DELTA, DT_UINT, DT_UINT, DT_DELTA};
#define DEC_STREAMS 15  // op columns without valRaw
#define DEC_ROWCOLS 13  // per-row cells: streams 0..12; entry cells: 13 (actor), 14 (ctr)

struct SrcInfo {
  uint64_t base;            // arena offset of the chunk data the column offsets are relative to
  const uint32_t* coff;
  const uint32_t* clen;
  const uint32_t* map;      // change: actor index map (amap slice)
  int64_t start_op;
  uint32_t row0, nr, ent0, ne, chg, nmap, self, is_change;
};

__device__ static SrcInfo src_info(DocShared& s, uint32_t src) {
  const WsLayout& L = s.L;
  SrcInfo si;
  if (s.has_base && src == 0) {
    si.base = s.dh.base; si.coff = s.dh.ocol_off; si.clen = s.dh.ocol_len;
    si.row0 = 0; si.nr = s.nb; si.ent0 = 0; si.ne = s.nbe;
    si.chg = 0xffffffffu; si.map = nullptr; si.nmap = 0; si.self = 0; si.start_op = 0; si.is_change = 0;
  } else {
    const uint32_t k = src - (s.has_base ? 1 : 0);
    const uint32_t c = hp<uint32_t>(s, L.order)[k];
    const ChgHdr& h = hp<ChgHdr>(s, L.chghdr)[c];
    si.base = h.base; si.coff = h.col_off; si.clen = h.col_len;
    si.row0 = hp<uint32_t>(s, L.rowbase)[k];
    si.ent0 = hp<uint32_t>(s, L.entbase)[k];
    si.nr = ((k + 1 < s.napplied) ? hp<uint32_t>(s, L.rowbase)[k + 1] : s.nrows) - si.row0;
    si.ne = ((k + 1 < s.napplied) ? hp<uint32_t>(s, L.entbase)[k + 1] : s.nents) - si.ent0;
    si.map = hp<uint32_t>(s, L.amap) + hp<uint32_t>(s, L.amb_out)[k];
    si.nmap = h.nactors; si.self = si.map[0]; si.start_op = h.start_op; si.chg = c; si.is_change = 1;
  }
  return si;
}

// largest source whose first row (entry) is <= i; empty sources share the next source's start
__device__ static uint32_t src_of(DocShared& s, uint32_t i, bool ents) {
  const uint32_t nsrc = (s.has_base ? 1 : 0) + s.napplied;
  const uint32_t* base = hp<uint32_t>(s, ents ? s.L.entbase : s.L.rowbase);
  uint32_t lo = 0, hi = nsrc;  // first source with start > i
  while (lo < hi) {
    const uint32_t m = (lo + hi) >> 1;
    const uint32_t st = (s.has_base && m == 0) ? 0 : base[m - (s.has_base ? 1 : 0)];
    if (st <= i) lo = m + 1; else hi = m;
  }
  return lo - 1;
}

// one stream: decodes n values into cells (utf8: (offset - span_lo) << 32 | length; boolean 0/1).
// With `defer`, a stream of am_dec_long values or more is left alone and reported (returns true).
__device__ static bool decode_stream(DocShared& s, uint32_t item, int64_t* cells, bool defer = false) {
  const uint32_t src = item / DEC_STREAMS, j = item % DEC_STREAMS;
  const uint32_t col = j < OC_VAL_RAW ? j : j + 1;
  const SrcInfo si = src_info(s, src);
  if (si.is_change && (col == OC_ID_ACTOR || col == OC_ID_CTR)) return false;  // ids from the header (new.js:708-709)
  const uint32_t n = j < DEC_ROWCOLS ? si.nr : si.ne;
  if (defer && n >= ::am_dec_long) return true;
  int64_t* dst = cells + (uint64_t)DEC_ROWCOLS * si.row0 + 2ull * si.ent0 +
                 (j < DEC_ROWCOLS ? (uint64_t)j * si.nr : (uint64_t)DEC_ROWCOLS * si.nr + (uint64_t)(j - DEC_ROWCOLS) * si.ne);
  const uint8_t type = kOpColDec[col];
  const uint64_t off = si.base + si.coff[col];
  ColDec d;
  cd_init(d, type, AV(s) + off, si.clen[col]);
  const int64_t sbase = (int64_t)(off - s.b.span_lo);
  // the base document's action column ends the op sequence for readNextDocOp (new.js:658-670): a
  // column that runs out early (the all-null column RLEEncoder writes as no bytes, encoding.js:778-782)
  const bool track_act = !si.is_change && col == OC_ACTION;
  for (uint32_t i = 0; i < n; i++) {
    int64_t v;
    uint32_t e;
    if (track_act && cd_done(d) && s.nb_act == 0xffffffffu) s.nb_act = i;
    if (type == DT_BOOL) {
      bool bv;
      e = cd_next_bool(d, bv);
      v = bv;
    } else {
      bool isnull;
      uint32_t l;
      int64_t x;
      e = cd_next(d, x, isnull, l);
      if (isnull) v = AM_NULL64;
      else if (type == DT_UTF8) v = ((sbase + x) << 32) | (int64_t)l;
      else if (type == DT_DELTA) v = (d.absolute += x);
      else v = x;
    }
    if (e) { set_err(s, e, 0, 0, 0, 0, si.chg); return false; }
    dst[i] = v;
  }
  return false;
}

// position of the q-th (from 0) set bit of m; q < popcount(m)
__device__ __forceinline__ uint32_t nth_bit64(uint64_t m, uint32_t q) {
  uint32_t pos = 0;
#pragma unroll
  for (uint32_t w = 32; w; w >>= 1) {
    const uint32_t c = (uint32_t)__popcll(m & ((1ull << w) - 1));
    if (q >= c) { q -= c; m >>= w; pos += w; }
  }
  return pos;
}
__device__ __forceinline__ int64_t wave_incl_add64(int64_t x) {
  uint64_t v = (uint64_t)x;
  v += ::wave::dpp<::wave::ROW_SHR1>(0ull, v);
  v += ::wave::dpp<::wave::ROW_SHR2>(0ull, v);
  v += ::wave::dpp<::wave::ROW_SHR4>(0ull, v);
  v += ::wave::dpp<::wave::ROW_SHR8>(0ull, v);
  v += ::wave::dpp<::wave::ROW_BCAST15, 0xa>(0ull, v);
  v += ::wave::dpp<::wave::ROW_BCAST31, 0xc>(0ull, v);
  return (int64_t)v;
}

// global-memory accesses of the global modes as global_* instructions: a flat access also counts
// against lgkmcnt, so every later LDS access or cross-lane gather would wait for it to complete
__device__ __forceinline__ void st_cell(int64_t* p, int64_t v) {
  if constexpr (kHotLds) *p = v;
  else *(__attribute__((address_space(1))) int64_t*)p = v;
}
__device__ __forceinline__ uint32_t ld_byte(const uint8_t* p) {
  if constexpr (kHotLds) return *p;
  else return *(const __attribute__((address_space(1))) uint8_t*)p;
}

// One long stream by the 64 lanes of a wave (a saved document's columns hold a value per op: one
// lane walking 100k values is the per-handle call's longest chain). The RLEDecoder / DeltaDecoder /
// BooleanDecoder state is wave-uniform (encoding.js:820-886, 1025-1030, 1171-1183) and the stream
// is read through a 64-byte window held in the wave's registers, a byte per lane, in which every
// lane has decoded the varint starting at its byte: a record header or a run value is a readlane,
// repetition, null and boolean runs are written 64 values a step, and an integer literal run is
// taken a window at a time (varint ends by ballot, the q-th value gathered to lane q, deltas by a
// wave scan); a string value is a length from the window and a wave-wide byte compare against the
// previous one. A varint the window cannot hold (over four bytes, or the stream's truncated end) or any error (a value repeated inside a literal run, a malformed
// record) sends the stream to lane 0's decode_stream, which writes it again and reports the
// reference's first error.
#ifdef AM_PHASE_CLOCK
#define BADR(c) do { bad = true; if (lane == 0 && (blockIdx.x & 63) == 0) { am_phase_cycles[32] = (c); am_phase_cycles[33] = i; am_phase_cycles[34] = d.r.off; am_phase_cycles[35] = j; am_phase_cycles[36] = (uint64_t)d.count; am_phase_cycles[37] = d.state; } } while (0)
#else
#define BADR(c) (bad = true)
#endif
// bytes a[0, len) == b[0, len), 64 a step across the wave (len wave-uniform)
__device__ __forceinline__ bool wave_bytes_eq(const uint8_t* a, const uint8_t* b, uint32_t len) {
  const uint32_t lane = ::wave::lane_id();
  for (uint32_t q = 0; q < len; q += 64) {
    const bool in = q + lane < len;
    const uint32_t x = in ? ld_byte(a + q + lane) : 0u, y = in ? ld_byte(b + q + lane) : 0u;
    if (__ballot(x != y)) return false;
  }
  return true;
}
__device__ __forceinline__ uint32_t rfl(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
__device__ __forceinline__ uint64_t rfl64(uint64_t v) { return (uint64_t)rfl((uint32_t)(v >> 32)) << 32 | rfl((uint32_t)v); }
__device__ __attribute__((noinline)) static void decode_stream_wave(DocShared& s, uint32_t item_, int64_t* cells) {
  // every quantity of the decoder state is wave-uniform: read once through readfirstlane, the state
  // and its control flow stay in scalar registers and scalar branches (values loaded through flat
  // pointers count as per-lane for the compiler, and would drag every step into vector code)
  const uint32_t lane = ::wave::lane_id();
  const uint32_t item = rfl(item_);
  const uint32_t src = item / DEC_STREAMS, j = item % DEC_STREAMS;
  const uint32_t col = j < OC_VAL_RAW ? j : j + 1;
  const SrcInfo si = src_info(s, src);
  const uint32_t n = rfl(j < DEC_ROWCOLS ? si.nr : si.ne);
  int64_t* dst = reinterpret_cast<int64_t*>(rfl64(reinterpret_cast<uint64_t>(
      cells + (uint64_t)DEC_ROWCOLS * si.row0 + 2ull * si.ent0 +
      (j < DEC_ROWCOLS ? (uint64_t)j * si.nr : (uint64_t)DEC_ROWCOLS * si.nr + (uint64_t)(j - DEC_ROWCOLS) * si.ne))));
  const uint8_t type = (uint8_t)rfl(kOpColDec[col]);
  const uint64_t off = rfl64(si.base + si.coff[col]);
  ColDec d;
  cd_init(d, type, reinterpret_cast<const uint8_t*>(rfl64(reinterpret_cast<uint64_t>(AV(s) + off))), rfl(si.clen[col]));
  const int64_t sbase = (int64_t)rfl64(off - s.b.span_lo);
  const bool track_act = rfl(!si.is_change && col == OC_ACTION) != 0;
  const bool sgn = type == DT_DELTA;
#ifdef AM_PHASE_CLOCK
  const uint64_t clk0 = clock64();
#endif
  // the window: bytes [p0, p0 + 64); per lane the varint starting at its byte (wl = its length,
  // 64 when over four bytes or not ended inside the window)
  uint64_t p0 = ~0ull, endm = 0;
  uint32_t wu = 0, wl = 64;
  int32_t ws = 0;
#ifdef AM_PHASE_CLOCK
  uint64_t n_reload = 0, n_iter = 0, n_slow = 0, n_lit = 0;  // (n_slow: none since the hand-back)
#define PCNT(x) (x)++
#else
#define PCNT(x) ((void)0)
#endif
  auto wload = [&](uint64_t at) {
    PCNT(n_reload);
    p0 = at;
    const uint32_t b = at + lane < d.r.n ? ld_byte(d.r.p + at + lane) : 0x80u;  // past the end: never a varint end
    endm = __ballot(!(b & 0x80));
    const uint32_t x1 = ::wave::down1(b, 0x80u), x2 = ::wave::down1(x1, 0x80u), x3 = ::wave::down1(x2, 0x80u);
    const uint64_t rest = endm >> lane;
    wl = rest ? (uint32_t)__builtin_ctzll(rest) + 1 : 64;
    uint32_t u = b & 0x7f, top = b;
    if (wl > 1) { u |= (x1 & 0x7f) << 7; top = x1; }
    if (wl > 2) { u |= (x2 & 0x7f) << 14; top = x2; }
    if (wl > 3) { u |= (x3 & 0x7f) << 21; top = x3; }
    wu = u;
    ws = (wl <= 4 && (top & 0x40)) ? (int32_t)(u | (0xffffffffu << (7 * wl))) : (int32_t)u;
  };
  // the varint at stream offset `at` (wave-uniform) from the window, reloaded at `at` when the
  // varint is not inside it; false: the window cannot hold it
  auto wvar = [&](uint64_t at, uint32_t& u, int32_t& sv, uint32_t& l) -> bool {
    if (at < p0 || at - p0 >= 64 || (at != p0 && ::wave::bcast(wl, (int)(at - p0)) > 4)) wload(at);
    const int q = (int)(at - p0);
    l = ::wave::bcast(wl, q);
    if (l > 4) return false;
    u = ::wave::bcast(wu, q);
    sv = ::wave::bcast(ws, q);
    return true;
  };
  bool bad = false;
  uint32_t i = 0;
  // the staged values [sb, i): lane l holds value sb + l
  uint32_t sb = 0;
  int64_t sv = 0;
  auto flush = [&]() {
    if (lane < i - sb) st_cell(dst + sb + lane, sv);
    sb = i;
  };
  // k values v0 + (q + 1) * step, q = 0..k-1 (step 0: k copies of v0)
  auto put_run = [&](uint32_t k, int64_t v0, int64_t step) {
    uint32_t q0 = 0;
    while (k) {
      const uint32_t off = i - sb, take = min(k, 64u - off);
      if (lane >= off && lane < off + take)
        sv = (int64_t)((uint64_t)v0 + (uint64_t)(lane - off + q0 + 1) * (uint64_t)step);
      i += take; k -= take; q0 += take;
      if (i - sb == 64) flush();
    }
  };
  auto put1 = [&](int64_t v) {
    if (lane == i - sb) sv = v;
    if (++i - sb == 64) flush();
  };
  while (i < n) {
    PCNT(n_iter);
    // the loop-carried state back in scalar registers at every step (see above)
    i = rfl(i); sb = rfl(sb);
    d.count = (int64_t)rfl64((uint64_t)d.count); d.r.off = rfl64(d.r.off); p0 = rfl64(p0);
    d.last = (int64_t)rfl64((uint64_t)d.last); d.absolute = (int64_t)rfl64((uint64_t)d.absolute);
    d.state = (uint8_t)rfl(d.state); d.has_last = (uint8_t)rfl(d.has_last); d.last_null = (uint8_t)rfl(d.last_null);
    d.blast = (uint8_t)rfl(d.blast); d.bfirst = (uint8_t)rfl(d.bfirst);
    if (cd_done(d)) {  // the column ran out: nulls (false) for the rest, as cd_next / cd_next_bool
      if (track_act && lane == 0 && s.nb_act == 0xffffffffu) s.nb_act = i;
      put_run(n - i, type == DT_BOOL ? 0 : AM_NULL64, 0);
      break;
    }
    uint32_t e = AM_OK, hu, hl;
    int32_t hs;
    if (type == DT_BOOL) {
      while (d.count == 0) {
        if (wvar(d.r.off, hu, hs, hl)) { d.count = hu; d.r.off += hl; }
        else { e = AM_E_LEB_INCOMPLETE; break; }  // (or a count over four bytes): the lane decoder's case
        d.blast = !d.blast;
        if (d.count == 0 && !d.bfirst) { e = AM_E_BOOL_ZERO_RUN; break; }
        d.bfirst = 0;
      }
      if (e) { BADR(1); break; }
      const uint32_t k = (uint32_t)min((uint64_t)d.count, (uint64_t)(n - i));
      put_run(k, d.blast, 0);
      d.count -= k;
      continue;
    }
    if (d.count == 0) {  // the next record (cd_record)
      bool done = false;
      if (wvar(d.r.off, hu, hs, hl)) {
        const int64_t c = hs;
        uint32_t vu, vl;
        int32_t vs;
        if (c == 1 || (c < 0 && d.state == 2) || (c == 0 && d.state == 3)) { BADR(2); break; }
        if (c < 0) {
          d.count = -c; d.state = 2; d.r.off += hl;
          done = true;
        } else if (wvar(d.r.off + hl, vu, vs, vl)) {
          if (c > 1 && type == DT_UTF8) {  // the run's string: its length, then its bytes
            const uint64_t at = d.r.off + hl + vl;
            if (at + vu > d.r.n) { BADR(9); break; }  // AM_E_SUBARRAY
            if ((d.state == 1 || d.state == 2) && d.has_last && !d.last_null && vu == d.last_len &&
                wave_bytes_eq(d.r.p + at, d.r.p + d.last, vu)) { BADR(3); break; }
            d.count = c; d.state = 1; d.last = (int64_t)at; d.last_len = vu; d.has_last = 1; d.last_null = 0;
            d.r.off += vu;  // the bytes (the length and the header below)
          } else if (c > 1) {
            const int64_t v = sgn ? (int64_t)vs : (int64_t)vu;
            if ((d.state == 1 || d.state == 2) && d.has_last && !d.last_null && v == d.last) { BADR(3); break; }
            d.count = c; d.state = 1; d.last = v; d.last_len = 0; d.has_last = 1; d.last_null = 0;
          } else {
            if (vu == 0) { BADR(4); break; }
            d.count = vu; d.state = 3; d.has_last = 1; d.last_null = 1;
          }
          d.r.off += hl + vl;
          done = true;
        }
      }
      if (!done) { BADR(5); break; }  // a varint the window cannot hold: the lane decoder's case
    }
    if (d.state != 2) {  // a repetition or a null run
      const uint32_t k = (uint32_t)min((uint64_t)d.count, (uint64_t)(n - i));
      if (d.last_null) {
        put_run(k, AM_NULL64, 0);
      } else if (type == DT_UTF8) {
        put_run(k, ((sbase + d.last) << 32) | (int64_t)d.last_len, 0);
      } else if (sgn) {
        put_run(k, d.absolute, d.last);
        d.absolute = (int64_t)((uint64_t)d.absolute + (uint64_t)k * (uint64_t)d.last);
      } else {
        put_run(k, d.last, 0);
      }
      d.count -= k;
      continue;
    }
    if (!wvar(d.r.off, hu, hs, hl)) { BADR(7); break; }  // a varint the window cannot hold
    if (type == DT_UTF8) {  // a string of a literal run: its length, then its bytes
      const uint64_t at = d.r.off + hl;
      if (at + hu > d.r.n) { BADR(9); break; }  // AM_E_SUBARRAY
      if (d.has_last && !d.last_null && hu == d.last_len && wave_bytes_eq(d.r.p + at, d.r.p + d.last, hu)) {
        BADR(8);  // AM_E_RLE_LIT_REP
        break;
      }
      d.last = (int64_t)at; d.last_len = hu; d.has_last = 1; d.last_null = 0;
      d.r.off = at + hu;
      d.count--;
      put1(((sbase + (int64_t)at) << 32) | (int64_t)hu);
      continue;
    }
    if (d.count <= 4) {  // a short literal: value by value
      const int64_t v = sgn ? (int64_t)hs : (int64_t)hu;
      if (d.has_last && !d.last_null && v == d.last) { BADR(8); break; }  // AM_E_RLE_LIT_REP
      d.last = v; d.last_len = 0; d.has_last = 1; d.last_null = 0;
      d.r.off += hl;
      d.count--;
      put1(sgn ? (d.absolute += v) : v);
      continue;
    }
    {  // an integer literal run: the window's varints
      PCNT(n_lit);
      const uint32_t pos = (uint32_t)(d.r.off - p0);
      const uint64_t startm = (((endm << 1) | 1ull) | (1ull << pos)) & (~0ull << pos);
      const uint64_t badm = __ballot(((startm >> lane) & 1) && wl > 4);
      const uint32_t navail = badm ? (uint32_t)__popcll(startm & ((1ull << __builtin_ctzll(badm)) - 1))
                                   : (uint32_t)__popcll(startm);
      const uint32_t k = (uint32_t)min(min((uint64_t)navail, (uint64_t)d.count), (uint64_t)(n - i));
      const uint32_t S = nth_bit64(startm, lane < k ? lane : 0);
      const int32_t vq = __shfl(sgn ? ws : (int32_t)wu, (int)S);
      const uint32_t endq = S + (uint32_t)__shfl((int)wl, (int)S);  // window byte after the q-th varint
      // (the move runs on every lane: inside a lane-dependent branch, lane 0 would be off and lane 1
      // would read the fill value)
      const int32_t up = ::wave::up1(vq, 0);
      const int64_t vq64 = sgn ? (int64_t)vq : (int64_t)(uint32_t)vq;
      const int64_t prev64 = lane ? (sgn ? (int64_t)up : (int64_t)(uint32_t)up) : d.last;
      const bool rep = lane < k && (lane || (d.has_last && !d.last_null)) && vq64 == prev64;
      if (__ballot(rep)) { BADR(6); break; }  // AM_E_RLE_LIT_REP: lane 0 reports it
      int64_t val = vq64;
      if (sgn) val = d.absolute + wave_incl_add64(lane < k ? vq64 : 0);
      d.last = ::wave::bcast(vq64, (int)k - 1);
      if (sgn) d.absolute = ::wave::bcast(val, (int)k - 1);
      d.r.off = p0 + ::wave::bcast(endq, (int)k - 1);
      d.last_len = 0; d.has_last = 1; d.last_null = 0;
      d.count -= k;
      // value q to lane off + q: one rotation; the values past lane 63 wrap to lanes 0.. after a flush
      const uint32_t off = i - sb, from = (lane - off) & 63;
      const int64_t rot = (int64_t)((uint64_t)(uint32_t)__shfl((int)(uint32_t)((uint64_t)val >> 32), (int)from) << 32 |
                                    (uint32_t)__shfl((int)(uint32_t)val, (int)from));
      if (lane >= off && lane < off + k) sv = rot;
      if (off + k >= 64) {
        i = sb + 64;
        flush();
        const uint32_t rest = off + k - 64;
        if (lane < rest) sv = rot;
        i = sb + rest;
      } else {
        i += k;
      }
      continue;
    }
  }
  if (!bad) flush();
  else if (lane == 0) decode_stream(s, item, cells);
#ifdef AM_PHASE_CLOCK
  // probe builds: the stream's cycles by column (slots 16 + j) and the streams handed back (slot 31)
  if (lane == 0 && (blockIdx.x & 63) == 0) {
    atomicAdd(&am_phase_cycles[16 + j], (unsigned long long)(clock64() - clk0));
    if (bad) atomicAdd(&am_phase_cycles[31], 1ull);
    if (j == 3) { am_phase_cycles[40] = n_reload; am_phase_cycles[41] = n_iter; am_phase_cycles[42] = n_slow; am_phase_cycles[43] = n_lit; am_phase_cycles[44] = n; }
  }
#endif
}

// row i from the cells (lane per row)
__device__ static void gather_row(DocShared& s, uint32_t i, const int64_t* cells, uint32_t* vsum, uint32_t* psum) {
  const uint32_t src = src_of(s, i, false);
  const SrcInfo si = src_info(s, src);
  const uint32_t q = i - si.row0, nr = si.nr;
  const int64_t* c = cells + (uint64_t)DEC_ROWCOLS * si.row0 + 2ull * si.ent0 + q;
  bool bad = false;
  auto mapact = [&](int64_t v) -> int32_t {
    if (v == AM_NULL64) return -1;
    if (si.is_change) {
      if (v < 0 || v >= (int64_t)si.nmap) { set_err(s, AM_E_NO_ACTOR_INDEX, v, 0, 0, 0, si.chg); bad = true; return -1; }
      return (int32_t)si.map[v];
    }
    if (v < 0 || v >= (int64_t)s.nactors) { set_err(s, AM_U_VALUE); bad = true; return -1; }
    return (int32_t)v;
  };
  Row r;
  r.obj_actor = mapact(c[0]);
  r.obj_ctr = c[(uint64_t)1 * nr];
  r.key_actor = mapact(c[(uint64_t)2 * nr]);
  r.key_ctr = c[(uint64_t)3 * nr];
  const int64_t ks = c[(uint64_t)4 * nr];
  if (ks == AM_NULL64) { r.key_len = AM_NOSTR; r.key_off = 0; }
  else {
    r.key_len = (uint32_t)(ks & 0xffffffff);
    r.key_off = s.b.span_lo + (uint64_t)(ks >> 32);
    if (!fix_utf8(s, r.key_off, r.key_len)) bad = true;
  }
  if (si.is_change) { r.id_actor = (int32_t)si.self; r.id_ctr = si.start_op + q; }
  else { r.id_actor = mapact(c[(uint64_t)5 * nr]); r.id_ctr = c[(uint64_t)6 * nr]; }
  r.insert = c[(uint64_t)7 * nr] != 0;
  r.action = c[(uint64_t)8 * nr];
  r.val_len = c[(uint64_t)9 * nr];
  r.chld_actor = mapact(c[(uint64_t)10 * nr]);
  r.chld_ctr = c[(uint64_t)11 * nr];
  const int64_t pc = c[(uint64_t)12 * nr];
  r.ps_cnt = pc == AM_NULL64 ? 0 : (uint32_t)pc;
  r.src_change = (uint8_t)si.is_change;
  r.is_del = si.is_change && r.action == 3 && !r.insert;  // an inserting del stays a row (new.js:1143-1150)
  r.flags = 0;
  r.val_off = 0;
  r.ps_off = 0;
  (void)bad;
  hp<Row>(s, s.L.rows)[i] = r;
  vsum[i] = r.val_len == AM_NULL64 ? 0u : (uint32_t)((uint64_t)r.val_len >> 4);
  psum[i] = r.ps_cnt;
}

__device__ static void gather_ent(DocShared& s, uint32_t j, const int64_t* cells) {
  const uint32_t src = src_of(s, j, true);
  const SrcInfo si = src_info(s, src);
  const uint32_t q = j - si.ent0;
  const int64_t* c = cells + (uint64_t)DEC_ROWCOLS * si.row0 + 2ull * si.ent0 + (uint64_t)DEC_ROWCOLS * si.nr + q;
  const int64_t a = c[0], ctr = c[si.ne];
  Ent e;
  e.row = -1;
  e.ctr = ctr;
  e.actor = -1;
  if (a == AM_NULL64 || ctr == AM_NULL64) { set_err(s, AM_U_VALUE); }
  else if (si.is_change) {
    if (a < 0 || a >= (int64_t)si.nmap) set_err(s, AM_E_NO_ACTOR_INDEX, a, 0, 0, 0, si.chg);
    else e.actor = (int32_t)si.map[a];
  } else {
    if (a < 0 || a >= (int64_t)s.nactors) set_err(s, AM_U_VALUE);
    else e.actor = (int32_t)a;
  }
  hp<Ent>(s, s.L.ents)[j] = e;
}

// after the scans: raw value offsets and group offsets of each row; per-source totals checked
__device__ static void place_row(DocShared& s, uint32_t i, const uint32_t* vsum, const uint32_t* psum) {
  const uint32_t src = src_of(s, i, false);
  const SrcInfo si = src_info(s, src);
  Row& r = hp<Row>(s, s.L.rows)[i];
  r.val_off = si.base + si.coff[OC_VAL_RAW] + (vsum[i] - vsum[si.row0]);
  r.ps_off = psum[i];
  if (i + 1 == si.row0 + si.nr) {  // last row of its source
    const uint64_t vend = (uint64_t)(vsum[i] - vsum[si.row0]) + (r.val_len == AM_NULL64 ? 0 : ((uint64_t)r.val_len >> 4));
    if (vend > si.clen[OC_VAL_RAW]) set_err(s, AM_E_SUBARRAY, 0, 0, 0, 0, si.chg);
    if (psum[i] + r.ps_cnt - psum[si.row0] != si.ne) set_err(s, AM_U_VALUE);
  }
}

// base document change rows (DOCUMENT_COLUMNS), one column per lane
__device__ static void decode_base_chg_col(DocShared& s, uint32_t col) {
  ChgRow* chg = hp<ChgRow>(s, s.L.chg);
  int64_t* deps = hp<int64_t>(s, s.L.deps);
  const APtr A = AV(s);
  const uint64_t off = s.dh.base + s.dh.ccol_off[col];
  const uint32_t len = s.dh.ccol_len[col];
  const uint32_t n = s.nbc;
  ColDec d;
  uint32_t e = AM_OK;
  switch (col) {
    case DC_ACTOR: case DC_SEQ: case DC_MAXOP: case DC_TIME: case DC_EXTRA_LEN: {
      cd_init(d, (col == DC_ACTOR || col == DC_EXTRA_LEN) ? DT_UINT : DT_INT, A + off, len);
      uint64_t acc = 0;
      for (uint32_t i = 0; i < n; i++) {
        int64_t v;
        if ((e = (col == DC_ACTOR || col == DC_EXTRA_LEN) ? cd_next_int(d, v) : cd_next_delta(d, v))) break;
        ChgRow& r = chg[i];
        if (col == DC_ACTOR) r.actor = v;
        else if (col == DC_SEQ) r.seq = v;
        else if (col == DC_MAXOP) r.max_op = v;
        else if (col == DC_TIME) r.time = v;
        else {
          r.extra_len = v;
          uint64_t nb = (v == AM_NULL64) ? 0 : ((uint64_t)v >> 4);
          if (acc + nb > s.dh.ccol_len[DC_EXTRA_RAW]) { e = AM_E_SUBARRAY; break; }
          r.extra_off = s.dh.base + s.dh.ccol_off[DC_EXTRA_RAW] + acc;
          r.extra_raw_len = (uint32_t)nb;
          acc += nb;
        }
      }
      break;
    }
    case DC_MESSAGE: {
      cd_init(d, DT_UTF8, A + off, len);
      for (uint32_t i = 0; i < n; i++) {
        uint64_t so;
        uint32_t sl;
        if ((e = cd_next_str(d, so, sl))) break;
        chg[i].msg_len = sl;
        chg[i].msg_off = sl == AM_NOSTR ? 0 : off + so;
        if (sl != AM_NOSTR && !fix_utf8(s, chg[i].msg_off, chg[i].msg_len)) return;
      }
      break;
    }
    case DC_DEPS_NUM: {
      cd_init(d, DT_UINT, A + off, len);
      uint32_t acc = 0;
      for (uint32_t i = 0; i < n; i++) {
        int64_t v;
        if ((e = cd_next_int(d, v))) break;
        uint32_t c = v == AM_NULL64 ? 0 : (uint32_t)v;
        chg[i].ndeps = c;
        chg[i].deps_off = acc;
        acc += c;
      }
      break;
    }
    case DC_DEPS_INDEX: {
      cd_init(d, DT_INT, A + off, len);
      for (uint32_t j = 0; j < s.nbd; j++) {
        int64_t v;
        if ((e = cd_next_delta(d, v))) break;
        deps[j] = v;
      }
      break;
    }
    default: break;
  }
  if (e) set_err(s, e);
}

// ---- P6: canonical column encoders, one column at a time by the whole wave
// (RLEEncoder / DeltaEncoder / BooleanEncoder, encoding.js:558-1135). A column's values are
// gathered into V; delta columns are differenced into W (nulls keep the running value); then
//   run starts (value != previous) -> maximal runs (scan + scatter of the start positions),
//   runs >= 2 -> repetition records, null runs -> null records, adjacent single values -> one
//   literal record (groups found with a scan over the runs, sized with LDS atomics),
//   record bytes -> exclusive scan -> every run writes its record at its own offset.
// An all-null RLE column encodes to nothing. ----
enum : uint8_t { EK_U = 0, EK_D = 1, EK_S = 2, EK_B = 3, EK_W = 4 };
// output columns: DOC_OPS_COLUMNS (0..15) then DOCUMENT_COLUMNS (16..24)
__device__ __constant__ static const uint8_t kEncKind[OC_NCOLS + DC_NCOLS] = {
    EK_U, EK_U, EK_U, EK_D, EK_S, EK_U, EK_D, EK_B, EK_U, EK_U, EK_W, EK_U, EK_D, EK_U, EK_U, EK_D,
    EK_U, EK_D, EK_D, EK_D, EK_S, EK_U, EK_D, EK_U, EK_W};

struct EncCtx {
  int64_t* V;
  int64_t* W;
  uint32_t *S, *RS, *RB, *RG;
  const uint8_t* As;  // input bytes at span_lo
};

__device__ __forceinline__ bool enc_eq(uint8_t kind, int64_t a, int64_t b, const uint8_t* As) {
  if (kind != EK_S || a == AM_NULL64 || b == AM_NULL64) return a == b;
  const uint32_t la = (uint32_t)(a & 0xffffffff), lb = (uint32_t)(b & 0xffffffff);
  return la == lb && bytes_eq(As + (a >> 32), As + (b >> 32), la);
}
__device__ __forceinline__ uint32_t enc_vsize(uint8_t kind, int64_t v) {
  if (kind == EK_U) return uleb_len((uint64_t)v);
  if (kind == EK_D) return sleb_len(v);
  const uint32_t l = (uint32_t)(v & 0xffffffff);
  return uleb_len(l) + l;
}
__device__ __forceinline__ uint8_t* enc_put(uint8_t kind, uint8_t* o, int64_t v, const uint8_t* As) {
  if (kind == EK_U) return put_uleb(o, (uint64_t)v);
  if (kind == EK_D) return put_sleb(o, v);
  const uint32_t l = (uint32_t)(v & 0xffffffff);
  o = put_uleb(o, l);
  const uint8_t* p = As + (v >> 32);
  for (uint32_t q = 0; q < l; q++) o[q] = p[q];
  return o + l;
}

// wave-level barrier: encode_column runs on one wave (wave 0, or in a large document each wave on
// a column of its own; the other waves wait at the next __syncthreads)
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  __builtin_amdgcn_wave_barrier();
}
// Encodes the n values of column c (V already filled) into out; returns the byte length.
__device__ static uint32_t encode_column(uint8_t kind, uint32_t n, uint8_t* out, EncCtx& x, uint32_t* s_flag) {
  const uint32_t t = threadIdx.x & 63;  // one wave
  if (n == 0) return 0;
  int64_t* X = x.V;
  if (kind == EK_D) {  // differences against the previous non-null value
    int32_t carry = -1;
    for (uint32_t base = 0; base < n; base += 64) {
      const uint32_t i = base + t;
      const int64_t v = i < n ? x.V[i] : AM_NULL64;
      const int32_t inc = wave_incl_max(v != AM_NULL64 ? (int32_t)i : -1);
      int32_t prev = __shfl_up(inc, 1, 64);
      if (t == 0) prev = -1;
      if (carry > prev) prev = carry;
      if (i < n) x.W[i] = v == AM_NULL64 ? AM_NULL64 : v - (prev >= 0 ? x.V[prev] : 0);
      const int32_t top = __shfl(inc, 63, 64);
      if (top > carry) carry = top;
    }
    X = x.W;
    wave_sync();
  }
  // maximal runs: start positions compacted into RS
  uint32_t nr = 0;
  for (uint32_t base = 0; base < n; base += 64) {
    const uint32_t i = base + t;
    const uint32_t f = (i < n && (kind == EK_W || i == 0 || !enc_eq(kind, X[i], X[i - 1], x.As))) ? 1u : 0u;
    const uint32_t inc = wave_incl_add(f);
    if (f) x.RS[nr + inc - 1] = i;
    nr += __shfl(inc, 63, 64);
  }
  const bool rle = kind <= EK_S;
  for (uint32_t r = t; r < nr; r += 64) x.S[r] = 0;
  wave_sync();
  // classify runs; literal groups (consecutive single-value runs) get ids and sizes
  bool any = false;
  if (rle) {
    uint32_t gcarry = 0, prev_single = 0;
    for (uint32_t base = 0; base < nr; base += 64) {
      const uint32_t r = base + t;
      uint32_t single = 0;
      if (r < nr) {
        const uint32_t i0 = x.RS[r], i1 = r + 1 < nr ? x.RS[r + 1] : n;
        const bool isnull = X[i0] == AM_NULL64;
        single = (!isnull && i1 - i0 == 1) ? 1u : 0u;
        any |= !isnull;
      }
      uint32_t ps = __shfl_up(single, 1, 64);
      if (t == 0) ps = prev_single;
      const uint32_t gs = (single && !ps) ? 1u : 0u;
      const uint32_t ginc = wave_incl_add(gs);
      if (r < nr) {
        const uint32_t gid = gcarry + ginc - 1;
        x.RG[r] = single ? (gid | (gs << 31)) : 0xffffffffu;
        if (single) atomicAdd(&x.S[gid], 1u);
      }
      prev_single = __shfl(single, 63, 64);
      gcarry += __shfl(ginc, 63, 64);
    }
    any = __any(any);
    if (!any) return 0;  // all-null column (wave-uniform)
    wave_sync();
  }
  // record bytes -> offsets
  uint32_t total = 0;
  for (uint32_t base = 0; base < nr; base += 64) {
    const uint32_t r = base + t;
    uint32_t bytes = 0;
    if (r < nr) {
      const uint32_t i0 = x.RS[r], i1 = r + 1 < nr ? x.RS[r + 1] : n, len = i1 - i0;
      const int64_t v = X[i0];
      if (kind == EK_B) bytes = uleb_len(len) + ((r == 0 && v) ? 1u : 0u);
      else if (kind == EK_W) bytes = (uint32_t)(v & 0xffffffff);
      else if (v == AM_NULL64) bytes = 1 + uleb_len(len);
      else if (len >= 2) bytes = sleb_len((int64_t)len) + enc_vsize(kind, v);
      else {
        const uint32_t g = x.RG[r];
        bytes = enc_vsize(kind, v) + ((g >> 31) ? sleb_len(-(int64_t)x.S[g & 0x7fffffff]) : 0u);
      }
    }
    const uint32_t inc = wave_incl_add(bytes);
    if (r < nr) x.RB[r] = total + inc - bytes;
    total += __shfl(inc, 63, 64);
  }
  // write records
  for (uint32_t r = t; r < nr; r += 64) {
    const uint32_t i0 = x.RS[r], i1 = r + 1 < nr ? x.RS[r + 1] : n, len = i1 - i0;
    const int64_t v = X[i0];
    uint8_t* o = out + x.RB[r];
    if (kind == EK_B) {
      if (r == 0 && v) *o++ = 0;
      put_uleb(o, len);
    } else if (kind == EK_W) {
      const uint32_t l = (uint32_t)(v & 0xffffffff);
      const uint8_t* p = x.As + (v >> 32);
      for (uint32_t q = 0; q < l; q++) o[q] = p[q];
    } else if (v == AM_NULL64) {
      *o++ = 0;
      put_uleb(o, len);
    } else if (len >= 2) {
      o = put_sleb(o, (int64_t)len);
      enc_put(kind, o, v, x.As);
    } else {
      const uint32_t g = x.RG[r];
      if (g >> 31) o = put_sleb(o, -(int64_t)x.S[g & 0x7fffffff]);
      enc_put(kind, o, v, x.As);
    }
  }
  (void)s_flag;
  wave_sync();
  return total;
}

#include "am_unknown.h"

#define ROW_KEEP_DEL 2  // Row.flags: a change's del without pred that stays a document row
__device__ __forceinline__ bool same_obj(const Row& a, const Row& b) {
  return a.obj_ctr == b.obj_ctr && a.obj_actor == b.obj_actor;
}

// binary search of (ctr, actor) in the id index; returns row or -1
__device__ static int32_t id_lookup(const IdKey* idk, uint32_t n, int64_t ctr, int32_t actor) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    uint32_t mid = (lo + hi) >> 1;
    const IdKey& k = idk[mid];
    if (k.ctr < ctr || (k.ctr == ctr && k.actor < actor)) lo = mid + 1; else hi = mid;
  }
  if (lo < n && idk[lo].ctr == ctr && idk[lo].actor == actor) return idk[lo].row;
  return -1;
}


// first index of (ctr, actor) in the id index (equal ids are adjacent, ordered by row); a document
// may hold the same id under different keys, which the reference accepts
__device__ static uint32_t id_lower(const IdKey* idk, uint32_t n, int64_t ctr, int32_t actor) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    const IdKey& k = idk[mid];
    if (k.ctr < ctr || (k.ctr == ctr && k.actor < actor)) lo = mid + 1; else hi = mid;
  }
  return lo;
}
#define FOR_ID(k, idk, n, c, a) for (uint32_t k = id_lower(idk, n, c, a); k < (n) && idk[k].ctr == (c) && idk[k].actor == (a); k++)

// does row i (stream order) have a row of the same object before it (an op of the object in the
// document when i is applied)?
__device__ static bool obj_has_row_before(const Row* rows, uint32_t i) {
  for (uint32_t j = 0; j < i; j++)
    if (!rows[j].is_del && same_obj(rows[j], rows[i])) return true;
  return false;
}
// the list element (key_ctr, key_actor) of row i: an earlier insert of the same object, or -1
__device__ static int32_t list_elem(const Row* rows, const IdKey* idk, uint32_t R, uint32_t i) {
  const Row& r = rows[i];
  if (r.key_actor < 0 || r.key_ctr == AM_NULL64) return -1;
  FOR_ID(k, idk, R, r.key_ctr, r.key_actor) {
    const int32_t e = idk[k].row;
    if (rows[e].insert && !rows[e].is_del && same_obj(rows[e], r) && rows[e].key_len == AM_NOSTR &&
        (!r.src_change || (uint32_t)e < i))
      return e;
  }
  return -1;
}
__device__ static bool list_elem_ok(const Row* rows, const IdKey* idk, uint32_t R, uint32_t i) {
  return list_elem(rows, idk, R, i) >= 0;
}
// the element is missing: seekWithinBlock scans the object's ops and reports the reference element
// (new.js:177-183, 300); an object without ops is passed over and mergeDocChangeOps reports the
// element (new.js:1163-1167)
__device__ static void elem_missing_err(DocShared& s, const Row* rows, const ActorRef* actors, uint32_t R, uint32_t i) {
  const Row& r = rows[i];
  const uint64_t ao = r.key_actor >= 0 ? actors[r.key_actor].off : 0;
  const uint32_t al = r.key_actor >= 0 ? actors[r.key_actor].len : 0;
  (void)R;
  set_err(s, obj_has_row_before(rows, i) ? AM_E_REF_NOT_FOUND : AM_E_ELEM_NOT_FOUND, r.key_ctr, 0, ao, al);
}

// ---- P7: getPatch log (am_patch.h) over the merged rows in document order ----
struct RowSrc {
  const Row* rows;
  const SortRec* sr;
  const uint32_t* soff;  // exclusive scan of succ counts (document order)
  const Ent* ent;        // succ entries
  uint32_t nout, nsucc_total;
  const ActorRef* actors;
  uint32_t na;
  const ChgRow* chg;
  uint32_t nc;
  APtr A;
  uint32_t nscan;  // ops documentPatch reads: nout, or 0 for a document whose action column is empty
  __device__ const Row& r(uint32_t i) const { return rows[sr[i].row]; }
  __device__ uint32_t n() const { return nscan; }
  __device__ int64_t obj_ctr(uint32_t i) const { const int64_t v = r(i).obj_ctr; return v == AM_NULL64 ? -1 : v; }
  __device__ int32_t obj_actor(uint32_t i) const { return r(i).obj_actor; }
  __device__ bool has_key(uint32_t i) const { return r(i).key_len != AM_NOSTR; }
  __device__ uint32_t key_len(uint32_t i) const { return r(i).key_len; }
  __device__ bool key_eq(uint32_t i, uint32_t j) const {
    const Row& a = r(i);
    const Row& b = r(j);
    return a.key_len == b.key_len && bytes_eq(A + a.key_off, A + b.key_off, a.key_len);
  }
  __device__ void copy_key(uint32_t i, uint8_t* d) const {
    const Row& a = r(i);
    const uint8_t* p = A + a.key_off;
    for (uint32_t q = 0; q < a.key_len; q++) d[q] = p[q];
  }
  __device__ int64_t key_ctr(uint32_t i) const { const int64_t v = r(i).key_ctr; return v == AM_NULL64 ? -1 : v; }
  __device__ int32_t key_actor(uint32_t i) const { return r(i).key_actor; }
  __device__ int64_t id_ctr(uint32_t i) const { return r(i).id_ctr; }
  __device__ int32_t id_actor(uint32_t i) const { return r(i).id_actor; }
  __device__ bool insert(uint32_t i) const { return r(i).insert != 0; }
  __device__ int64_t action(uint32_t i) const { const int64_t v = r(i).action; return v == AM_NULL64 ? -1 : v; }
  __device__ int64_t val_len(uint32_t i) const { const int64_t v = r(i).val_len; return v == AM_NULL64 ? 0 : v; }
  __device__ uint32_t vbytes(uint32_t i) const { return (uint32_t)((uint64_t)val_len(i) >> 4); }
  __device__ void copy_value(uint32_t i, uint8_t* d) const {
    const uint8_t* p = A + r(i).val_off;
    const uint32_t nb = vbytes(i);
    for (uint32_t q = 0; q < nb; q++) d[q] = p[q];
  }
  // new Decoder(bytes).readUint53() / readInt53() (columnar.js:316-325)
  __device__ bool value_int(uint32_t i, bool is_uint, int64_t& out) const {
    Rd rd{A + r(i).val_off, vbytes(i), 0};
    return (is_uint ? rd_u53(rd, out) : rd_i53(rd, out)) == AM_OK;
  }
  __device__ int64_t value_f64_bits(uint32_t i) const {
    const uint8_t* p = A + r(i).val_off;
    uint64_t b = 0;
    for (int q = 7; q >= 0; q--) b = (b << 8) | p[q];
    return (int64_t)b;
  }
  __device__ uint32_t nsucc(uint32_t i) const { return (i + 1 < nout ? soff[i + 1] : nsucc_total) - soff[i]; }
  __device__ int64_t succ_ctr(uint32_t i, uint32_t k) const { return ent[soff[i] + k].ctr; }
  __device__ int32_t succ_actor(uint32_t i, uint32_t k) const { return ent[soff[i] + k].actor; }
  __device__ uint32_t nactors() const { return na; }
  __device__ uint32_t actor_len(uint32_t a) const { return actors[a].len; }
  __device__ void copy_actor(uint32_t a, uint8_t* d) const {
    const uint8_t* p = A + actors[a].off;
    for (uint32_t q = 0; q < actors[a].len; q++) d[q] = p[q];
  }
  __device__ uint32_t nchg() const { return nc; }
  __device__ int64_t chg_actor(uint32_t c) const { return chg[c].actor; }
  __device__ int64_t chg_seq(uint32_t c) const { return chg[c].seq; }
};

// P8 source (am_diff.h): rows in stream order, F = the merged document order
struct DiffSrc {
  const Row* rows;
  const Ent* ents;       // base succ entries / change preds
  const SortRec* sr;
  const uint32_t* soff;  // exclusive scan of succ counts (document order)
  const Ent* fent;       // final succ entries
  const int32_t* etime;  // stream time of each final succ entry's op
  const uint32_t* pend;
  uint32_t np, nbase, nr, nf, nsucc_total;
  uint32_t nmeta;  // base ops documentPatch reads for objectMeta: nbase, 0 for an empty action column
  const ActorRef* actors;
  uint32_t na;
  const ChgRow* chg;
  uint32_t nc;
  APtr A;
  __device__ uint32_t nb() const { return nbase; }
  __device__ uint32_t nmeta_rows() const { return nmeta; }
  __device__ uint32_t nrows() const { return nr; }
  __device__ uint32_t nout() const { return nf; }
  __device__ int32_t frow(int32_t f) const { return sr[f].row; }
  __device__ uint32_t f_nsucc(int32_t f) const { return ((uint32_t)f + 1 < nf ? soff[f + 1] : nsucc_total) - soff[f]; }
  __device__ int64_t f_succ_ctr(int32_t f, uint32_t k) const { return fent[soff[f] + k].ctr; }
  __device__ int32_t f_succ_actor(int32_t f, uint32_t k) const { return fent[soff[f] + k].actor; }
  __device__ int64_t f_succ_time(int32_t f, uint32_t k) const { return etime[soff[f] + k]; }
  __device__ const Row& r(int32_t i) const { return rows[i]; }
  __device__ int64_t obj_ctr(int32_t i) const { const int64_t v = r(i).obj_ctr; return v == AM_NULL64 ? -1 : v; }
  __device__ int32_t obj_actor(int32_t i) const { return r(i).obj_actor; }
  __device__ int64_t key_ctr(int32_t i) const { const int64_t v = r(i).key_ctr; return v == AM_NULL64 ? -1 : v; }
  __device__ int32_t key_actor(int32_t i) const { return r(i).key_actor; }
  __device__ bool has_key(int32_t i) const { return r(i).key_len != AM_NOSTR; }
  __device__ uint32_t key_len(int32_t i) const { return r(i).key_len; }
  __device__ int key_cmp(int32_t i, int32_t j) const {
    return utf16_cmp_dev(A + r(i).key_off, r(i).key_len, A + r(j).key_off, r(j).key_len);
  }
  __device__ bool key_eq(int32_t i, int32_t j) const {
    return r(i).key_len == r(j).key_len && bytes_eq(A + r(i).key_off, A + r(j).key_off, r(i).key_len);
  }
  __device__ void copy_key(int32_t i, uint8_t* d) const {
    const uint8_t* p = A + r(i).key_off;
    for (uint32_t q = 0; q < r(i).key_len; q++) d[q] = p[q];
  }
  __device__ int64_t id_ctr(int32_t i) const { return r(i).id_ctr; }
  __device__ int32_t id_actor(int32_t i) const { return r(i).id_actor; }
  __device__ bool insert(int32_t i) const { return r(i).insert != 0; }
  __device__ int64_t action(int32_t i) const { const int64_t v = r(i).action; return v == AM_NULL64 ? -1 : v; }
  __device__ uint32_t npred(int32_t i) const { return (uint32_t)i >= nbase ? r(i).ps_cnt : 0u; }
  __device__ int64_t pred_ctr(int32_t i, uint32_t k) const { return ents[r(i).ps_off + k].ctr; }
  __device__ int32_t pred_actor(int32_t i, uint32_t k) const { return ents[r(i).ps_off + k].actor; }
  __device__ uint32_t rank(int32_t a) const { return actors[a].rank; }
  // patch_value source (am_patch.h), by row
  __device__ int64_t val_len(uint32_t i) const { const int64_t v = rows[i].val_len; return v == AM_NULL64 ? 0 : v; }
  __device__ uint32_t vbytes(uint32_t i) const { return (uint32_t)((uint64_t)val_len(i) >> 4); }
  __device__ void copy_value(uint32_t i, uint8_t* d) const {
    const uint8_t* p = A + rows[i].val_off;
    const uint32_t nb2 = vbytes(i);
    for (uint32_t q = 0; q < nb2; q++) d[q] = p[q];
  }
  __device__ bool value_int(uint32_t i, bool is_uint, int64_t& out) const {
    Rd rd{A + rows[i].val_off, vbytes(i), 0};
    return (is_uint ? rd_u53(rd, out) : rd_i53(rd, out)) == AM_OK;
  }
  __device__ int64_t value_f64_bits(uint32_t i) const {
    const uint8_t* p = A + rows[i].val_off;
    uint64_t b = 0;
    for (int q = 7; q >= 0; q--) b = (b << 8) | p[q];
    return (int64_t)b;
  }
  __device__ uint32_t nactors() const { return na; }
  __device__ uint32_t actor_len(uint32_t a) const { return actors[a].len; }
  __device__ void copy_actor(uint32_t a, uint8_t* d) const {
    const uint8_t* p = A + actors[a].off;
    for (uint32_t q = 0; q < actors[a].len; q++) d[q] = p[q];
  }
  __device__ uint32_t nchg() const { return nc; }
  __device__ int64_t chg_actor(uint32_t c) const { return chg[c].actor; }
  __device__ int64_t chg_seq(uint32_t c) const { return chg[c].seq; }
  __device__ uint32_t npass() const { return np; }
  __device__ uint32_t pass_end(uint32_t p) const { return pend[p]; }
};

// the log in wire form (am_patch.h patch_pack); a log that does not fit its region reports the
// engine's capacity limit instead (never a truncated patch)
__device__ static void wire_out(PatchOut& po, int64_t max_op, uint8_t* dst, uint64_t cap) {
  if (patch_pack(po, max_op, dst, cap)) return;
  po.status = PATCH_U_CAPACITY;
  patch_pack(po, max_op, dst, cap);
}

// ---- radix sorts of the large-document path (global mode): the id index (P5c) and the document
// order (P5g) as stable LSD radix sorts of packed integer keys (block_radix_sort) instead of
// bitonic sorts; scratch in the tour arrays (dead before P5f, and again once P5g's keys are built:
// 16 R + 16 R bytes). Keys outside the packing (counters >= 2^46, 2^16+ actors) keep the bitonic
// sort. ----
__device__ __forceinline__ uint32_t rs_bits(uint64_t mx) { return mx ? 64u - (uint32_t)__clzll((long long)mx) : 0u; }

// P5c: (ctr, actor index, row) ascending; the rows enter in row order, so a stable sort by
// ctr << 16 | actor keeps equal ids in row order
__device__ static bool radix_idk(DocShared& s, IdKey* idk, uint32_t R) {
  __shared__ unsigned long long s_max;
  __shared__ uint32_t s_bad;
  const uint32_t t = threadIdx.x, T = blockDim.x;
  uint64_t* k0 = hp<uint64_t>(s, s.L.tour_nxt);
  uint64_t* k1 = k0 + R;
  uint32_t* v0 = hp<uint32_t>(s, s.L.tour_w);
  uint32_t* v1 = v0 + R;
  if (t == 0) { s_max = 0; s_bad = 0; }
  __syncthreads();
  for (uint32_t i = t; i < R; i += T) {
    const int64_t c = idk[i].ctr;
    const int32_t a = idk[i].actor;
    if (c < 0 || c >= (1ll << 46) || a < 0 || a >= 65536) { s_bad = 1; continue; }
    const uint64_t key = ((uint64_t)c << 16) | (uint64_t)a;
    k0[i] = key;
    v0[i] = (uint32_t)idk[i].row;
    atomicMax(&s_max, (unsigned long long)key);
  }
  __syncthreads();
  const bool bad = s_bad != 0;
  const uint32_t bits = rs_bits(s_max);
  __syncthreads();
  if (bad) return false;
  block_radix_sort<kDocT / 64>(k0, v0, k1, v1, R, bits);
  for (uint32_t i = t; i < R; i += T) {
    IdKey k;
    k.ctr = (int64_t)(k0[i] >> 16);
    k.actor = (int32_t)(k0[i] & 0xffff);
    k.row = (int32_t)v0[i];
    idk[i] = k;
  }
  __syncthreads();
  return true;
}

// P5f: list elements by (object, parent element, opId descending) -- the children of an element in
// descending opId order (new.js:145-163). Three stable passes; the records are gathered through
// the sortrec region (free until P5g) and copied back.
__device__ static bool radix_elemk(DocShared& s, ElemKey* ek, uint32_t M, uint32_t R) {
  __shared__ unsigned long long s_max;
  __shared__ uint32_t s_bad;
  const uint32_t t = threadIdx.x, T = blockDim.x;
  uint64_t* k0 = hp<uint64_t>(s, s.L.tour_nxt);
  uint64_t* k1 = k0 + M;
  uint32_t* v0 = hp<uint32_t>(s, s.L.tour_w);
  uint32_t* v1 = v0 + M;
  ElemKey* tmp = hp<ElemKey>(s, s.L.sortrec);  // PR * 56 bytes >= M * 32
  if (t == 0) s_bad = 0;
  __syncthreads();
  for (uint32_t i = t; i < M; i += T) {
    const ElemKey& e = ek[i];
    if (e.obj_ctr + 1 < 0 || e.obj_ctr + 1 >= (1ll << 46) || e.obj_rank + 1 < 0 || e.obj_rank + 1 >= 65536 || e.id_ctr < 0 ||
        e.id_ctr >= (1ll << 46) || e.id_rank < 0 || e.id_rank >= 65536 || e.parent < -1 || e.parent >= (int32_t)R)
      s_bad = 1;
  }
  __syncthreads();
  const bool bad = s_bad != 0;
  __syncthreads();
  if (bad || M > R) return false;
  for (int stage = 0; stage < 3; stage++) {
    if (t == 0) s_max = 0;
    __syncthreads();
    for (uint32_t i = t; i < M; i += T) {
      const ElemKey& e = ek[stage == 0 ? i : v0[i]];
      uint64_t key;
      if (stage == 0) key = (((1ull << 46) - 1 - (uint64_t)e.id_ctr) << 16) | (uint64_t)(65535 - e.id_rank);  // descending
      else if (stage == 1) key = (uint64_t)(e.parent + 1);
      else key = ((uint64_t)(e.obj_ctr + 1) << 17) | (uint64_t)(e.obj_rank + 1);
      if (stage == 0) v0[i] = i;
      k0[i] = key;
      atomicMax(&s_max, (unsigned long long)key);
    }
    __syncthreads();
    const uint32_t bits = rs_bits(s_max);
    __syncthreads();
    block_radix_sort<kDocT / 64>(k0, v0, k1, v1, M, bits);
  }
  for (uint32_t i = t; i < M; i += T) tmp[i] = ek[v0[i]];
  __syncthreads();
  for (uint32_t i = t; i < M; i += T) ek[i] = tmp[i];
  __syncthreads();
  return true;
}

// P5h: the new succ entries by (target row, owner opId): two stable passes, records gathered through
// the elemk region (dead after P5f)
__device__ static bool radix_newent(DocShared& s, NewEnt* ne, uint32_t N, uint32_t R) {
  __shared__ unsigned long long s_max;
  __shared__ uint32_t s_bad;
  const uint32_t t = threadIdx.x, T = blockDim.x;
  if (N > R) return false;  // the scratch is sized by rows
  uint64_t* k0 = hp<uint64_t>(s, s.L.tour_nxt);
  uint64_t* k1 = k0 + N;
  uint32_t* v0 = hp<uint32_t>(s, s.L.tour_w);
  uint32_t* v1 = v0 + N;
  NewEnt* tmp = hp<NewEnt>(s, s.L.elemk);  // PR * 32 bytes >= N * 24
  if (t == 0) s_bad = 0;
  __syncthreads();
  for (uint32_t i = t; i < N; i += T) {
    const NewEnt& e = ne[i];
    if (e.ctr < 0 || e.ctr >= (1ll << 46) || e.rank < 0 || e.rank >= 65536 || e.target < 0 || e.target >= (int32_t)R) s_bad = 1;
  }
  __syncthreads();
  const bool bad = s_bad != 0;
  __syncthreads();
  if (bad) return false;
  for (int stage = 0; stage < 2; stage++) {
    if (t == 0) s_max = 0;
    __syncthreads();
    for (uint32_t i = t; i < N; i += T) {
      const NewEnt& e = ne[stage == 0 ? i : v0[i]];
      const uint64_t key = stage == 0 ? (((uint64_t)e.ctr << 16) | (uint64_t)e.rank) : (uint64_t)e.target;
      if (stage == 0) v0[i] = i;
      k0[i] = key;
      atomicMax(&s_max, (unsigned long long)key);
    }
    __syncthreads();
    const uint32_t bits = rs_bits(s_max);
    __syncthreads();
    block_radix_sort<kDocT / 64>(k0, v0, k1, v1, N, bits);
  }
  for (uint32_t i = t; i < N; i += T) tmp[i] = ne[v0[i]];
  __syncthreads();
  for (uint32_t i = t; i < N; i += T) ne[i] = tmp[i];
  __syncthreads();
  return true;
}

// P5g: object, then (map key in UTF-16 order | list position), then opId -- three stable passes,
// least significant first. Map keys get dense ranks from a bitonic sort of the keyed records only
// (few in list-heavy documents). Afterwards only sr[i].row is meaningful (all that later phases read).
__device__ static bool radix_docorder(DocShared& s, SortRec* sr, uint32_t n, uint32_t R, const APtr A) {
  __shared__ unsigned long long s_max;
  __shared__ uint32_t s_bad;
  const uint32_t t = threadIdx.x, T = blockDim.x;
  uint64_t* k0 = hp<uint64_t>(s, s.L.tour_nxt);
  uint64_t* k1 = k0 + n;
  uint32_t* v0 = hp<uint32_t>(s, s.L.tour_w);
  uint32_t* v1 = v0 + n;
  uint32_t* sk = v0 + 2 * (uint64_t)R;  // keyed records (pow2 <= 2 R entries)
  if (t == 0) s_bad = 0;
  __syncthreads();
  for (uint32_t i = t; i < n; i += T) {
    const SortRec& r = sr[i];
    if (r.obj_ctr + 1 < 0 || r.obj_ctr + 1 >= (1ll << 46) || r.obj_rank + 1 < 0 || r.obj_rank + 1 >= 65536 || r.id_ctr < 0 ||
        r.id_ctr >= (1ll << 46) || r.id_rank < 0 || r.id_rank >= 65536 || (r.kind && (r.k1 > 0 || r.k1 < -(1ll << 38))))
      s_bad = 1;
    v1[i] = r.kind == 0 ? 1u : 0u;
  }
  __syncthreads();
  const bool bad = s_bad != 0;
  __syncthreads();
  if (bad) return false;
  // dense UTF-16 ranks of the map keys (into k1 of the keyed records)
  const uint32_t K = block_excl_scan(v1, n, s.tmp);
  __syncthreads();
  if (K) {
    const uint32_t PK = pow2_ceil(K);
    for (uint32_t i = t; i < n; i += T)
      if (sr[i].kind == 0) sk[v1[i]] = i;
    for (uint32_t j = K + t; j < PK; j += T) sk[j] = ~0u;
    __syncthreads();
    auto kcmp = [&](uint32_t a, uint32_t b) {
      return utf16_cmp_dev(A + sr[a].key_off, sr[a].key_len, A + sr[b].key_off, sr[b].key_len);
    };
    block_bitonic_sort(sk, PK, [&](uint32_t a, uint32_t b) {
      if (a == ~0u || b == ~0u) return a != ~0u && b == ~0u;
      const int c = kcmp(a, b);
      return c ? c < 0 : a < b;
    });
    for (uint32_t j = t; j < K; j += T) v1[j] = (j == 0 || kcmp(sk[j - 1], sk[j]) != 0) ? 1u : 0u;
    __syncthreads();
    block_excl_scan(v1, K, s.tmp);
    __syncthreads();
    for (uint32_t j = t; j < K; j += T) {
      const bool fresh = j == 0 || kcmp(sk[j - 1], sk[j]) != 0;
      sr[sk[j]].k1 = (int64_t)(v1[j] + (fresh ? 1u : 0u)) - 1;  // dense rank
    }
    __syncthreads();
  }
  for (int stage = 0; stage < 3; stage++) {
    if (t == 0) s_max = 0;
    __syncthreads();
    for (uint32_t i = t; i < n; i += T) {
      const SortRec& r = sr[stage == 0 ? i : v0[i]];
      uint64_t key;
      if (stage == 0) key = ((uint64_t)r.id_ctr << 16) | (uint64_t)r.id_rank;
      else if (stage == 1) key = r.kind ? ((1ull << 40) | (uint64_t)(r.k1 + (1ll << 39))) : (uint64_t)r.k1;
      else key = ((uint64_t)(r.obj_ctr + 1) << 17) | (uint64_t)(r.obj_rank + 1);
      if (stage == 0) v0[i] = i;
      k0[i] = key;
      atomicMax(&s_max, (unsigned long long)key);
    }
    __syncthreads();
    const uint32_t bits = rs_bits(s_max);
    __syncthreads();
    block_radix_sort<kDocT / 64>(k0, v0, k1, v1, n, bits);
  }
  for (uint32_t i = t; i < n; i += T) v1[i] = (uint32_t)sr[v0[i]].row;
  __syncthreads();
  for (uint32_t i = t; i < n; i += T) sr[i].row = (int32_t)v1[i];
  __syncthreads();
  return true;
}

// One document by the whole workgroup (the body of k_doc below).
// P8 (applyChanges patch, am_diff.h) of one document whose merged rows are described by src: the
// replay into the working-form pools, the wire form at L.pwire and, with AM_DOC_META, the objectMeta
// blob after it. One lane. (The few layout values it needs travel as scalars: a WsLayout passed by
// reference would live in scratch memory.)
struct P8Args {
  uint8_t* patch;                  // working-form pools (L.patch)
  uint64_t nrec, nmval, heap;      // their capacities
  uint8_t* dscr;                   // replay scratch (L.dscr)
  uint8_t* pwire;                  // wire form (L.pwire)
  uint64_t pwire_cap;
  uint32_t R, E, ps;
  const uint8_t* meta;             // the handle's objectMeta blob (AM_DOC_META), or null
  uint32_t meta_len;
  bool meta_mode;
};
__device__ __forceinline__ P8Args p8_args(uint8_t* wsg, const WsLayout& L, const DocBounds& b, const am_doc_desc& dd,
                                          const am_chunk_desc* chunks, const uint8_t* arena) {
  P8Args a;
  a.patch = wsg + L.patch;
  a.nrec = L.patch_nrec; a.nmval = L.patch_nmval; a.heap = L.patch_heap;
  a.dscr = wsg + L.dscr;
  a.pwire = wsg + L.pwire;
  a.pwire_cap = L.pwire_cap;
  a.R = b.R; a.E = b.E; a.ps = (b.U & 2) ? 8 : 1;
  a.meta_mode = (dd.flags & AM_DOC_META) != 0;
  a.meta = nullptr;
  a.meta_len = 0;
  if (a.meta_mode && dd.meta_chunk) {
    const am_chunk_desc mc = chunks[dd.meta_chunk - 1];
    a.meta = arena + mc.off;
    a.meta_len = mc.len;
  }
  return a;
}
// po_ / dw_: where the replay keeps its pool descriptors (k_diff passes LDS; null: locals).
// Wide: every lane of the wave runs it (k_diff); else one lane.
template <bool Wide = false>
__device__ static void p8_run(const DiffSrc& src, const P8Args a, PatchOut* po_ = nullptr, DiffScratch* dw_ = nullptr) {
  PatchOut po_local;
  DiffScratch dw_local;
  PatchOut& po = po_ ? *po_ : po_local;
  DiffScratch& dw = dw_ ? *dw_ : dw_local;
  po.rec = reinterpret_cast<PatchRec*>(a.patch + 64);
  po.mval = reinterpret_cast<PatchVal*>(a.patch + 64 + 64 * a.nrec);
  po.heap = a.patch + 64 + 64 * a.nrec + 32 * a.nmval;
  po.cap_rec = a.nrec; po.cap_mval = a.nmval; po.cap_heap = a.heap;
  diff_scratch_bind(a.dscr, a.R, a.E, dw, a.ps);
  diff_scan<Wide>(src, po, dw, a.meta_mode, a.meta, a.meta_len);
  uint8_t* const pw = a.pwire;
  const uint64_t wl = patch_pack(po, 0, pw, a.pwire_cap);
  if (!wl) {
    wire_out(po, 0, pw, a.pwire_cap);
  } else if (a.meta_mode && (!po.status || po.status == PATCH_U_INC_VALUE)) {
    // the snapshots this call leaves, after the stream (PatchHdr2.meta_bytes)
    const uint64_t mb = diff_meta_pack(src, dw, pw + wl, a.pwire_cap - wl);
    if (!mb) {
      po.status = PATCH_U_CAPACITY;
      patch_pack(po, 0, pw, a.pwire_cap);
    } else {
      for (int q = 0; q < 8; q++) pw[offsetof(PatchHdr2, meta_bytes) + q] = (uint8_t)(mb >> (8 * q));
    }
  }
}

// k_diff: P8 of every document k_doc merged with AM_DOC_WANT_DIFF (either mode), one wave per
// document, from the rows k_doc left in the document's workspace (an LDS-mode document's mirrored
// hot set) and the counts it recorded at L.djob
template <bool Wide>
__device__ static void k_diff_one(uint32_t doc, const uint8_t* __restrict__ arena, const am_chunk_desc* __restrict__ chunks,
                                  const am_doc_desc* __restrict__ docs, const DocBounds* __restrict__ bounds,
                                  const uint64_t* __restrict__ ws_off, uint8_t* __restrict__ ws_base, uint32_t lds_bytes,
                                  const am_doc_result* __restrict__ results, const uint8_t* __restrict__ fast_done) {
  if (!Wide && threadIdx.x) return;
  if (fast_done && fast_done[doc]) return;
  const DocBounds b = bounds[doc];
  if (b.P != 2) return;
  const WsLayout L = ws_layout(b);
  if (results[doc].status) return;
  uint8_t* const wsg = ws_base + ws_off[doc];
  const uint32_t* job = reinterpret_cast<const uint32_t*>(wsg + L.djob);
  // the arena view of the global mode (its staged copy when invalid UTF-8 was replaced)
  const APtr A{((b.U & 1) && !doc_scattered(b)) ? wsg + L.input - b.span_lo : arena, 0};
  // the replay's descriptors in LDS: as locals they sit in scratch memory, one dependent load away
  // on every pool access of the serial chain
  __shared__ DiffSrc src;
  __shared__ PatchOut po;
  __shared__ DiffScratch dw;
  src = DiffSrc{reinterpret_cast<const Row*>(wsg + L.rows), reinterpret_cast<const Ent*>(wsg + L.ents),
              reinterpret_cast<const SortRec*>(wsg + L.sortrec), reinterpret_cast<const uint32_t*>(wsg + L.succ_cnt),
              reinterpret_cast<const Ent*>(wsg + L.outent), reinterpret_cast<const int32_t*>(wsg + L.etime),
              reinterpret_cast<const uint32_t*>(wsg + L.passend), job[0], job[1], job[2], job[3], job[4], job[5],
              reinterpret_cast<const ActorRef*>(wsg + L.actors), job[6], reinterpret_cast<const ChgRow*>(wsg + L.chg), job[7], A};
  p8_run<Wide>(src, p8_args(wsg, L, b, docs[doc], chunks, arena), &po, &dw);
}

__device__ __forceinline__ void k_doc_one(uint32_t doc, const uint8_t* __restrict__ arena, const am_chunk_desc* __restrict__ chunks,
                                          const am_doc_desc* __restrict__ docs, const am_known_hash* __restrict__ known,
                                          const ChunkInfo* __restrict__ info, const DocBounds* __restrict__ bounds,
                                          const uint64_t* __restrict__ ws_off, uint8_t* __restrict__ ws_base,
                                          uint64_t ws_cap, uint32_t lds_bytes, am_doc_result* __restrict__ results,
                                          int32_t* __restrict__ chg_state, const uint8_t* __restrict__ fast_done) {
  __shared__ DocShared s;
  __shared__ uint32_t s_tmp[kDocT + 1];  // block scans' scratch (s.tmp)
  const uint32_t t = threadIdx.x, T = blockDim.x;
  if (fast_done && fast_done[doc]) return;  // merged by k_doc_fast (am_doc_fast.h)
  const am_doc_desc dd = docs[doc];
  uint8_t* const wsg = ws_base + ws_off[doc];  // global (derived from the kernel argument)
  if (t == 0) {
    s.b = bounds[doc];
    s.tmp = s_tmp;
    s.ws = ws_base + ws_off[doc];
    s.L = ws_layout(s.b);
    // hot working set in LDS when it fits (this namespace's mode decides who runs the document)
    s.hot = s.ws;  // global mode only; LDS mode addresses am_lds directly (hp)
    s.A = arena;
    s.status = AM_OK; s.errchg = 0xffffffffu; s.arg0 = s.arg1 = 0; s.arg_actor_off = 0; s.arg_actor_len = 0;
    s.has_base = dd.base_chunk >= 0;
    s.nb = s.nbe = s.nbc = s.nbd = 0;
    s.napplied = s.nqueued = s.nactors = s.nheads = 0;
    s.npass = 0;
    s.nb_act = 0xffffffffu;
    s.nrows = s.nents = s.nchg = s.ndeps = s.nout = s.nnew = 0;
    s.max_op = 0;
    s.out_len = 0;
    s.ph_last = clock64();
    s.xs_used = 0;
#ifdef AM_DIFF_CHECK
    s.dbg_phase = 0xffffu;
    s.dbg_canary = 0xffffu;
#endif
    if (ws_off[doc] + s.L.total > ws_cap) set_err(s, AM_U_CAPACITY);
    // chunk-level errors: the base document first (load), then changes in order (new.js:1798)
    if (s.has_base) {
      const ChunkInfo& ci = info[dd.base_chunk];
      if (ci.status) set_err(s, ci.status, ci.arg0);
      else if (ci.type != 0) set_err(s, AM_E_CHUNK_TYPE, ci.type);
      else { s.nb = ci.nops; s.nbe = ci.nents; s.nbc = ci.nchg; s.nbd = ci.ndeps; }
    }
    for (uint32_t k = 0; k < dd.chg_count && s.status == AM_OK; k++) {
      const ChunkInfo& ci = info[dd.chg_begin + k];
      if (ci.status) set_err(s, ci.status, ci.arg0, 0, 0, 0, k);
      else if (ci.type != 1) set_err(s, AM_E_CHUNK_TYPE, ci.type, 0, 0, 0, k);
    }
    if (s.b.R == 0 && s.b.N == 0 && !s.has_base && dd.chg_count) set_err(s, AM_U_CAPACITY);
  }
  __syncthreads();
  // LDS mode: the hot set fits and the input span is contiguous (chunks of a scattered document
  // are read from the arena by the global mode; k_bounds forces that launch)
  if ((s.L.hot_total <= lds_bytes && !doc_scattered(s.b)) != kHotLds) return;  // the other mode's document
  const WsLayout& L = s.L;
  if (s.status) goto done;
  // P0: stage the document's input bytes (base + changes, adjacent in the arena) into the hot
  // region with 16-byte coalesced loads; every later parse/decode reads them from there.
  // (the global mode stages too when invalid UTF-8 is being replaced: the replacements follow the copy)
  if (kHotLds || ((s.b.U & 1) && !doc_scattered(s.b))) {
    const uint64_t lo = s.b.span_lo, n = s.b.span_hi - s.b.span_lo;
    uint8_t* dst = hp<uint8_t>(s, L.input);
    if (n) {
      const uint64_t head = (16 - (lo & 15)) & 15;  // bytes before the first 16-aligned source address
      for (uint64_t q = t; q < head && q < n; q += T) dst[q] = arena[lo + q];
      if (n > head) {
        const uint64_t nv = (n - head) / 16;
        for (uint64_t v = t; v < nv; v += T) {
          const uint4 x = *reinterpret_cast<const uint4*>(arena + lo + head + 16 * v);
          uint8_t* o = dst + head + 16 * v;
          const uint8_t* xb = reinterpret_cast<const uint8_t*>(&x);
#pragma unroll
          for (int k = 0; k < 16; k++) o[k] = xb[k];
        }
        for (uint64_t q = head + 16 * nv + t; q < n; q += T) dst[q] = arena[lo + q];
      }
    }
    // the global mode now reads its input from the staged copy too (same arena offsets)
    if (!kHotLds && t == 0) s.A = reinterpret_cast<const uint8_t*>(reinterpret_cast<uintptr_t>(dst) - lo);
  }
  __syncthreads();
  PH(0);
  // P1: base document header, change headers (lane per change), base change rows (lane per column)
  if (t == 0 && s.has_base) {
    const ChunkInfo& ci = info[dd.base_chunk];
    const am_chunk_desc cd = chunks[dd.base_chunk];
    parse_doc_hdr(AV(s) + cd.off + ci.data_off, ci.data_len, cd.off + ci.data_off, s.dh);
  }
  if (t == 0 && !s.has_base) { s.dh.nactors = 0; s.dh.nheads = 0; s.dh.has_hidx = 0; s.dh.extra_len = 0; s.dh.base = 0; }
  for (uint32_t k = t; k < dd.chg_count; k += T) {
    const ChunkInfo& ci = info[dd.chg_begin + k];
    const am_chunk_desc cd = chunks[dd.chg_begin + k];
    ChgHdr& h = hp<ChgHdr>(s, L.chghdr)[k];
    parse_change_hdr(AV(s) + cd.off + ci.data_off, ci.data_len, cd.off + ci.data_off, h);
  }
  // prefix offsets of the change actor lists and deps
  for (uint32_t k = t; k < dd.chg_count; k += T) {
    hp<uint32_t>(s, L.ambase)[k] = info[dd.chg_begin + k].nactors;
    hp<uint32_t>(s, L.dbase)[k] = info[dd.chg_begin + k].ndeps;
  }
  __syncthreads();
  block_excl_scan(hp<uint32_t>(s, L.ambase), dd.chg_count, s.tmp);
  block_excl_scan(hp<uint32_t>(s, L.dbase), dd.chg_count, s.tmp);
  __syncthreads();
  if (s.has_base)
    for (uint32_t c = t; c < DC_NCOLS; c += T) decode_base_chg_col(s, c);
#if defined(AM_STOP_PHASE) && AM_STOP_PHASE == 1
  goto done;
#endif
  PH(1);
  // P2: plan -- lane-parallel lookups, then the sequential causal queue on integers
  plan_lookups(s, dd, info, known);
  __syncthreads();
  if (s.status) goto done;
  PH(2);
  if (!plan_fast(s, dd, info, chg_state) && t == 0) plan_doc(s, dd, info, chg_state);
  __syncthreads();
  if (s.status) goto done;
  {
    const APtr A = AV(s);
    Row* rows = hp<Row>(s, L.rows);
    Ent* ents = hp<Ent>(s, L.ents);
    ActorRef* actors = hp<ActorRef>(s, L.actors);
    const uint32_t R = s.nrows;
    PH(3);
    // P4: decode every (source, column) stream into cells, then gather rows and entries
    int64_t* cells = hp<int64_t>(s, L.cells);
    uint32_t* vsum = hp<uint32_t>(s, L.scan);
    uint32_t* psum = hp<uint32_t>(s, L.succ_cnt);
    const uint32_t nsrc = (s.has_base ? 1 : 0) + s.napplied;
#if defined(AM_STOP_PHASE) && AM_STOP_PHASE == 2
    goto done;
#endif
    // a lane per stream; streams of am_dec_long values or more are listed (s.tmp[1..]) and decoded
    // by a wave each afterwards (a list past its kDocT slots decodes the rest on lanes)
    if (t == 0) s.tmp[0] = 0;
    __syncthreads();
    for (uint32_t it = t; it < nsrc * DEC_STREAMS; it += T)
      if (decode_stream(s, it, cells, true)) {
        const uint32_t slot = atomicAdd(&s.tmp[0], 1u);
        if (slot < kDocT) s.tmp[1 + slot] = it;
        else decode_stream(s, it, cells);
      }
    __syncthreads();
    {
      const uint32_t nlong = min(s.tmp[0], kDocT);
      for (uint32_t q = t / 64; q < nlong; q += T / 64) decode_stream_wave(s, s.tmp[1 + q], cells);
    }
    for (uint32_t src = t; src < nsrc; src += T) {
      const SrcInfo si = src_info(s, src);
      if (si.nr == 0 && si.ne != 0) set_err(s, AM_U_VALUE);  // group entries without ops
    }
    __syncthreads();
    // a base document whose action column holds fewer values than it has ops: the reference reads
    // no ops from it when the column is empty (every action null: documentPatch / getPatch see an
    // empty document); merging changes into it, or a column that stops part-way, is not restated
    if (t == 0 && s.has_base && s.nb_act < s.nb && (s.nb_act != 0 || s.napplied > 0)) set_err(s, AM_U_VALUE);
    // actor ranks (lexicographic order of the hex ids)
    for (uint32_t i = t; i < s.nactors; i += T) {
      uint32_t rank = 0;
      for (uint32_t j = 0; j < s.nactors; j++)
        if (actor_cmp_dev(A + actors[j].off, actors[j].len, A + actors[i].off, actors[i].len) < 0) rank++;
      actors[i].rank = rank;
    }
    __syncthreads();
    if (s.status) goto done;
    PH(4);
    for (uint32_t i = t; i < R; i += T) gather_row(s, i, cells, vsum, psum);
    for (uint32_t j = t; j < s.nents; j += T) gather_ent(s, j, cells);
    __syncthreads();
    if (s.status) goto done;
    if (kDocT == 64) {
      wave_excl_scan_arr(vsum, R);
      wave_excl_scan_arr(psum, R);
    } else {
      block_excl_scan(vsum, R, s.tmp);
      block_excl_scan(psum, R, s.tmp);
    }
    __syncthreads();
    for (uint32_t i = t; i < R; i += T) place_row(s, i, vsum, psum);
    // maxOp of the loaded document: the largest counter among its op ids and succs
    // (documentPatch, new.js:1627-1630 -> this.maxOp, new.js:1749); applied changes raise it
    {
      int64_t m = 0;
      const bool read_all = s.nb_act >= s.nb;  // else no op is read (above)
      for (uint32_t i = t; i < s.nb && read_all; i += T) m = rows[i].id_ctr > m ? rows[i].id_ctr : m;
      for (uint32_t j = t; j < s.nbe && read_all; j += T) m = ents[j].ctr > m ? ents[j].ctr : m;
      for (int o = 32; o > 0; o >>= 1) {
        const int64_t x = __shfl_xor(m, o, 64);
        m = x > m ? x : m;
      }
      if ((t & 63) == 0) atomicMax(reinterpret_cast<long long*>(&s.max_op), (long long)m);
    }
    // op columns of a future format version, carried through the merge (am_unknown.h)
    if (s.b.UC && t == 0) unk_collect(s, dd, chunks, info, wsg);
    __syncthreads();
    if (s.status) goto done;
#if defined(AM_STOP_PHASE) && AM_STOP_PHASE == 3
    goto done;
#endif

    PH(5);
    // P5a: per-op checks of change rows (readNextChangeOp new.js:715-723; mergeDocChangeOps shapes)
    for (uint32_t i = t; i < R; i += T) {
      const Row& r = rows[i];
      if (r.id_ctr == AM_NULL64 || r.id_actor < 0) { set_err(s, AM_U_VALUE); continue; }
      if (!r.src_change) continue;
      if ((r.obj_ctr == AM_NULL64) != (r.obj_actor < 0)) { set_err(s, AM_E_MISMATCH_OBJ, r.obj_ctr, r.obj_actor); continue; }
      if ((r.key_ctr == AM_NULL64 && r.key_actor >= 0) || (r.key_ctr == 0 && r.key_actor >= 0) ||
          (r.key_ctr != AM_NULL64 && r.key_ctr > 0 && r.key_actor < 0)) {
        set_err(s, AM_E_MISMATCH_KEY, r.key_ctr, r.key_actor);
        continue;
      }
      if (r.is_del && r.ps_cnt == 0 && r.key_len != AM_NOSTR) {
        // a del without pred disappears once an op of its key with a lower id has been merged
        // (mergeDocChangeOps drops dels whose preds were all seen, new.js:1199-1212); otherwise the
        // change ops are taken first and it stays as a row (new.js:1143-1150)
        bool drop = false;
        for (uint32_t j = 0; j < i && !drop; j++) {
          const Row& x = rows[j];
          drop = !x.is_del && same_obj(x, r) && x.key_len == r.key_len && bytes_eq(A + x.key_off, A + r.key_off, r.key_len) &&
                 (x.id_ctr < r.id_ctr || (x.id_ctr == r.id_ctr && actor_cmp_dev(A + actors[x.id_actor].off, actors[x.id_actor].len,
                                                                                A + actors[r.id_actor].off, actors[r.id_actor].len) < 0));
        }
        if (!drop) rows[i].flags |= ROW_KEEP_DEL;
      }
      if (r.insert && r.ps_cnt > 0) {
        const Ent& p = ents[r.ps_off];
        set_err(s, AM_E_PRED_NOT_FOUND, p.ctr, 0, actors[p.actor].off, actors[p.actor].len);
        continue;
      }
      if (r.key_len == AM_NOSTR && !r.insert && r.key_ctr == AM_NULL64) { set_err(s, AM_U_VALUE); continue; }
    }
    __syncthreads();
    for (uint32_t i = t; i < R; i += T)
      if (rows[i].flags & ROW_KEEP_DEL) rows[i].is_del = 0;
    // P5c: id index sorted by (ctr, actor index)
    const uint32_t PR = pow2_ceil(R > 0 ? R : 1);
    IdKey* idk = hp<IdKey>(s, L.idk);
    for (uint32_t i = t; i < PR; i += T) {
      IdKey k;
      if (i < R) { k.ctr = rows[i].id_ctr; k.actor = rows[i].id_actor; k.row = (int32_t)i; }
      else { k.ctr = INT64_MAX; k.actor = INT32_MAX; k.row = INT32_MAX; }
      idk[i] = k;
    }
    __syncthreads();
    if (s.status) goto done;
    bool idk_sorted = false;
    if constexpr (!kHotLds) idk_sorted = radix_idk(s, idk, R);
    if (!idk_sorted)
      block_bitonic_sort(idk, PR, [](const IdKey& a, const IdKey& b) {
        if (a.ctr != b.ctr) return a.ctr < b.ctr;
        if (a.actor != b.actor) return a.actor < b.actor;
        return a.row < b.row;
      });
    // equal ids: mergeDocChangeOps compares ids only among the ops of one key / list element, so a
    // change op repeating the id of an op in the same key or element fails (new.js:1218-1221) and
    // repeats elsewhere are kept; insertions are placed before that comparison (new.js:1143)
    for (uint32_t i = t + 1; i < R; i += T) {
      if (!(idk[i].ctr == idk[i - 1].ctr && idk[i].actor == idk[i - 1].actor)) continue;
      const Row& y = rows[idk[i].row];
      if (!y.src_change || y.insert) continue;
      for (uint32_t k = i; k-- > 0 && idk[k].ctr == idk[i].ctr && idk[k].actor == idk[i].actor;) {
        const Row& x = rows[idk[k].row];
        if (x.is_del || !same_obj(x, y)) continue;
        bool same;
        if (y.key_len != AM_NOSTR) same = x.key_len == y.key_len && bytes_eq(A + x.key_off, A + y.key_off, y.key_len);
        else same = x.key_len == AM_NOSTR && (x.insert ? x.id_ctr : x.key_ctr) == y.key_ctr &&
                    (x.insert ? x.id_actor : x.key_actor) == y.key_actor;
        if (same) { set_err(s, AM_E_DUP_OPID, idk[i].ctr, 0, actors[idk[i].actor].off, actors[idk[i].actor].len); break; }
      }
    }
    __syncthreads();
    if (s.status) goto done;

    PH(6);
    auto id_less = [&](int64_t c1, int32_t a1, int64_t c2, int32_t a2) {
      if (c1 != c2) return c1 < c2;
      return actors[a1].rank < actors[a2].rank;
    };
    // P5d: resolve preds -> targets (new.js:1173-1188, 1254-1258)
    int32_t* elem_of = hp<int32_t>(s, L.elem_of);
    int32_t* parent = hp<int32_t>(s, L.parent);
    for (uint32_t i = t; i < R; i += T) {
      const Row& r = rows[i];
      elem_of[i] = -1;
      parent[i] = -1;
      if (!r.src_change || r.insert) continue;
      for (uint32_t q = 0; q < r.ps_cnt; q++) {
        Ent& p = ents[r.ps_off + q];
        int32_t tr = -1;
        bool ok = false;
        FOR_ID(k, idk, R, p.ctr, p.actor) {
          tr = idk[k].row;
          ok = (uint32_t)tr < i && !rows[tr].is_del;
          if (ok) {
            const Row& x = rows[tr];
            ok = same_obj(x, r) && id_less(x.id_ctr, x.id_actor, r.id_ctr, r.id_actor);
            if (ok) {
              if (r.key_len != AM_NOSTR) {
                ok = x.key_len == r.key_len && bytes_eq(A + x.key_off, A + r.key_off, r.key_len);
              } else {
                int64_t ec = x.insert ? x.id_ctr : x.key_ctr;
                int32_t ea = x.insert ? x.id_actor : x.key_actor;
                ok = x.key_len == AM_NOSTR && ec == r.key_ctr && ea == r.key_actor;
              }
            }
          }
          if (ok) break;
        }
        if (!ok) {
          // a list update / delete whose element does not exist fails in seekToOp before its preds
          // are checked (new.js:275-300, 1163-1167)
          if (r.key_len == AM_NOSTR && !list_elem_ok(rows, idk, R, i)) elem_missing_err(s, rows, actors, R, i);
          else set_err(s, AM_E_PRED_NOT_FOUND, p.ctr, 0, actors[p.actor].off, actors[p.actor].len);
          break;
        }
        p.row = tr;
      }
    }
    __syncthreads();
    if (s.status) goto done;
    // P5e: list elements: reference elements of inserts, target elements of updates
    for (uint32_t i = t; i < R; i += T) {
      const Row& r = rows[i];
      if (r.key_len != AM_NOSTR) continue;
      if (r.is_del) {  // a del without pred still names an existing element
        if (r.ps_cnt == 0 && !list_elem_ok(rows, idk, R, i)) elem_missing_err(s, rows, actors, R, i);
        continue;
      }
      if (r.insert) {
        elem_of[i] = (int32_t)i;
        if (r.key_ctr == AM_NULL64 || r.key_ctr == 0 || r.key_actor < 0) { parent[i] = -1; continue; }
        const int32_t p = list_elem(rows, idk, R, i);
        if (p < 0) {
          // seekWithinBlock finds nothing to compare against in an object without ops and inserts
          // at the object's start (new.js:62-64); a loaded document keeps such rows as they are
          if (!r.src_change || !obj_has_row_before(rows, i)) { parent[i] = -1; continue; }
          set_err(s, AM_E_REF_NOT_FOUND, r.key_ctr, 0, actors[r.key_actor].off, actors[r.key_actor].len);
          continue;
        }
        if (!(rows[p].id_ctr < r.id_ctr)) { set_err(s, AM_U_NONCAUSAL); continue; }
        parent[i] = p;
      } else {
        const int32_t e = list_elem(rows, idk, R, i);
        if (e < 0) {
          if (r.src_change) elem_missing_err(s, rows, actors, R, i);
          else set_err(s, AM_U_VALUE);
          continue;
        }
        if (!id_less(rows[e].id_ctr, rows[e].id_actor, r.id_ctr, r.id_actor)) { set_err(s, AM_U_NONCAUSAL); continue; }
        elem_of[i] = e;
      }
    }
    __syncthreads();
    if (s.status) goto done;

    PH(7);
    // P5f: RGA order = preorder of the reference-element tree with children in descending opId
    // order (new.js:145-163). Euler tour + Wyllie list ranking (pointer jumping).
    uint32_t* scan = hp<uint32_t>(s, L.scan);
    for (uint32_t i = t; i < R; i += T) scan[i] = (elem_of[i] == (int32_t)i) ? 1u : 0u;
    __syncthreads();
    const uint32_t M = block_excl_scan(scan, R, s.tmp);
    const uint32_t PM = pow2_ceil(M > 0 ? M : 1);
    ElemKey* ek = hp<ElemKey>(s, L.elemk);
    for (uint32_t i = t; i < R; i += T)
      if (elem_of[i] == (int32_t)i) {
        const Row& r = rows[i];
        ElemKey k;
        k.obj_ctr = r.obj_ctr == AM_NULL64 ? -1 : r.obj_ctr;
        k.obj_rank = r.obj_actor < 0 ? -1 : (int32_t)actors[r.obj_actor].rank;
        k.parent = parent[i];
        k.id_ctr = r.id_ctr;
        k.id_rank = (int32_t)actors[r.id_actor].rank;
        k.row = (int32_t)i;
        ek[scan[i]] = k;
      }
    for (uint32_t i = M + t; i < PM; i += T) { ElemKey k; k.obj_ctr = INT64_MAX; k.row = -1; k.obj_rank = 0; k.parent = 0; k.id_ctr = 0; k.id_rank = 0; ek[i] = k; }
    __syncthreads();
    bool ek_sorted = false;
    if constexpr (!kHotLds) ek_sorted = radix_elemk(s, ek, M, R);
    if (!ek_sorted)
    block_bitonic_sort(ek, PM, [](const ElemKey& a, const ElemKey& b) {
      if (a.obj_ctr != b.obj_ctr) return a.obj_ctr < b.obj_ctr;
      if (a.obj_rank != b.obj_rank) return a.obj_rank < b.obj_rank;
      if (a.parent != b.parent) return a.parent < b.parent;
      if (a.id_ctr != b.id_ctr) return a.id_ctr > b.id_ctr;  // children: descending opId
      return a.id_rank > b.id_rank;
    });
    int32_t* first_child = hp<int32_t>(s, L.first_child);
    int32_t* next_sib = hp<int32_t>(s, L.next_sib);
    for (uint32_t i = t; i < R; i += T) { first_child[i] = -1; next_sib[i] = -1; }
    __syncthreads();
    auto same_group = [&](const ElemKey& a, const ElemKey& b) {
      return a.obj_ctr == b.obj_ctr && a.obj_rank == b.obj_rank && a.parent == b.parent;
    };
    for (uint32_t i = t; i < M; i += T) {
      const ElemKey& k = ek[i];
      if (i + 1 < M && same_group(k, ek[i + 1])) next_sib[k.row] = ek[i + 1].row;
      if ((i == 0 || !same_group(ek[i - 1], k)) && k.parent >= 0) first_child[k.parent] = k.row;
    }
    __syncthreads();
    int32_t* nxtA = hp<int32_t>(s, L.tour_nxt);
    int32_t* nxtB = nxtA + 2 * R;
    int32_t* wA = hp<int32_t>(s, L.tour_w);
    int32_t* wB = wA + 2 * R;
    const int32_t END = -1;
    for (uint32_t i = t; i < R; i += T) {
      bool el = elem_of[i] == (int32_t)i;
      nxtA[2 * i] = el ? (first_child[i] >= 0 ? 2 * first_child[i] : (int32_t)(2 * i + 1)) : END;
      wA[2 * i] = el ? 1 : 0;
      nxtA[2 * i + 1] = el ? (next_sib[i] >= 0 ? 2 * next_sib[i] : (parent[i] >= 0 ? 2 * parent[i] + 1 : END)) : END;
      wA[2 * i + 1] = 0;
    }
    __syncthreads();
    for (uint32_t span = 1; span < 2 * R; span <<= 1) {
      // 8 independent jumps in flight per lane (the gathers are latency-bound in global mode)
      constexpr uint32_t kJ = 8;
      for (uint32_t x0 = t; x0 < 2 * R; x0 += kJ * T) {
        int32_t nx[kJ], w0[kJ], w1[kJ], n1[kJ];
#pragma unroll
        for (uint32_t u = 0; u < kJ; u++) {
          const uint32_t x = x0 + u * T;
          nx[u] = x < 2 * R ? nxtA[x] : END;
          w0[u] = x < 2 * R ? wA[x] : 0;
        }
#pragma unroll
        for (uint32_t u = 0; u < kJ; u++) {
          w1[u] = nx[u] != END ? wA[nx[u]] : 0;
          n1[u] = nx[u] != END ? nxtA[nx[u]] : END;
        }
#pragma unroll
        for (uint32_t u = 0; u < kJ; u++) {
          const uint32_t x = x0 + u * T;
          if (x < 2 * R) { wB[x] = w0[u] + w1[u]; nxtB[x] = n1[u]; }
        }
      }
      __syncthreads();
      int32_t* tp = nxtA; nxtA = nxtB; nxtB = tp;
      tp = wA; wA = wB; wB = tp;
    }
    // wA[2v] = number of elements from v to the end of its object's list (suffix count)
#if defined(AM_STOP_PHASE) && AM_STOP_PHASE == 4
    goto done;
#endif

    PH(8);
    // P5g: document order: object, then key (UTF-16) | element position, then opId
    SortRec* sr = hp<SortRec>(s, L.sortrec);
    for (uint32_t i = t; i < R; i += T) scan[i] = rows[i].is_del ? 0u : 1u;
    __syncthreads();
    const uint32_t NOUT = block_excl_scan(scan, R, s.tmp);
    const uint32_t PO = pow2_ceil(NOUT > 0 ? NOUT : 1);
    for (uint32_t i = t; i < R; i += T) {
      const Row& r = rows[i];
      if (r.is_del) continue;
      SortRec k;
      k.obj_ctr = r.obj_ctr == AM_NULL64 ? -1 : r.obj_ctr;
      k.obj_rank = r.obj_actor < 0 ? -1 : (int32_t)actors[r.obj_actor].rank;
      k.kind = r.key_len != AM_NOSTR ? 0 : 1;
      k.k1 = k.kind ? -(int64_t)wA[2 * elem_of[i]] : 0;
      k.key_off = r.key_off;
      k.key_len = r.key_len;
      k.id_ctr = r.id_ctr;
      k.id_rank = (int32_t)actors[r.id_actor].rank;
      k.row = (int32_t)i;
      k.pad = 0;
      sr[scan[i]] = k;
    }
    for (uint32_t i = NOUT + t; i < PO; i += T) { SortRec k; k.row = -1; k.obj_ctr = INT64_MAX; k.obj_rank = 0; k.kind = 0; k.k1 = 0; k.key_off = 0; k.key_len = 0; k.id_ctr = 0; k.id_rank = 0; k.pad = 0; sr[i] = k; }
    __syncthreads();
    bool sr_sorted = false;
    if constexpr (!kHotLds) sr_sorted = radix_docorder(s, sr, NOUT, R, A);
    if (!sr_sorted)
    block_bitonic_sort(sr, PO, [A](const SortRec& a, const SortRec& b) {
      if ((a.row < 0) != (b.row < 0)) return b.row < 0;
      if (a.row < 0) return false;
      if (a.obj_ctr != b.obj_ctr) return a.obj_ctr < b.obj_ctr;
      if (a.obj_rank != b.obj_rank) return a.obj_rank < b.obj_rank;
      if (a.kind != b.kind) return a.kind < b.kind;
      if (a.kind == 0) {
        int c = utf16_cmp_dev(A + a.key_off, a.key_len, A + b.key_off, b.key_len);
        if (c) return c < 0;
      } else if (a.k1 != b.k1) {
        return a.k1 < b.k1;
      }
      if (a.id_ctr != b.id_ctr) return a.id_ctr < b.id_ctr;
      return a.id_rank < b.id_rank;
    });

    PH(9);
    // P5h: succ lists = existing succ (base rows) merged with new succs from preds
    NewEnt* ne = hp<NewEnt>(s, L.newent);
    const uint32_t NNEW = s.nents - s.nbe;
    const uint32_t PN = pow2_ceil(NNEW > 0 ? NNEW : 1);
    for (uint32_t j = t; j < PN; j += T) {
      NewEnt x;
      x.target = j < NNEW ? ents[s.nbe + j].row : INT32_MAX;
      x.ctr = 0; x.actor = 0; x.rank = 0; x.pad = 0;
      ne[j] = x;
    }
    __syncthreads();
    // owning op id of each pred entry
    for (uint32_t i = t; i < R; i += T) {
      const Row& r = rows[i];
      if (!r.src_change) continue;
      for (uint32_t q = 0; q < r.ps_cnt; q++) {
        NewEnt& x = ne[r.ps_off + q - s.nbe];
        x.ctr = r.id_ctr;
        x.actor = r.id_actor;
        x.rank = (int32_t)actors[r.id_actor].rank;
      }
    }
    __syncthreads();
    bool ne_sorted = false;
    if constexpr (!kHotLds) ne_sorted = radix_newent(s, ne, NNEW, R);
    if (!ne_sorted)
    block_bitonic_sort(ne, PN, [](const NewEnt& a, const NewEnt& b) {
      if (a.target != b.target) return a.target < b.target;
      if (a.ctr != b.ctr) return a.ctr < b.ctr;
      return a.rank < b.rank;
    });
    uint32_t* succ_cnt = hp<uint32_t>(s, L.succ_cnt);
    auto new_range = [&](int32_t row, uint32_t& lo_out) -> uint32_t {
      uint32_t lo = 0, hi = NNEW;
      while (lo < hi) { uint32_t m = (lo + hi) >> 1; if (ne[m].target < row) lo = m + 1; else hi = m; }
      uint32_t a = lo;
      hi = NNEW;
      while (lo < hi) { uint32_t m = (lo + hi) >> 1; if (ne[m].target <= row) lo = m + 1; else hi = m; }
      lo_out = a;
      return lo - a;
    };
    for (uint32_t i = t; i < NOUT; i += T) {
      const Row& r = rows[sr[i].row];
      uint32_t lo;
      succ_cnt[i] = (r.src_change ? 0 : r.ps_cnt) + new_range(sr[i].row, lo);
    }
    __syncthreads();
    const uint32_t NSUCC = block_excl_scan(succ_cnt, NOUT, s.tmp);
    Ent* outent = hp<Ent>(s, L.outent);
    for (uint32_t i = t; i < NOUT; i += T) {
      const int32_t ri = sr[i].row;
      const Row& r = rows[ri];
      uint32_t lo;
      uint32_t nn = new_range(ri, lo);
      uint32_t no = r.src_change ? 0 : r.ps_cnt;
      uint32_t a = 0, b2 = 0, w = succ_cnt[i];
      while (a < no || b2 < nn) {
        bool take_old;
        if (a >= no) take_old = false;
        else if (b2 >= nn) take_old = true;
        else {
          const Ent& eo = ents[r.ps_off + a];
          const NewEnt& en = ne[lo + b2];
          // insertion point: first existing succ that is not smaller (new.js:1178-1182)
          take_old = eo.ctr < en.ctr || (eo.ctr == en.ctr && (eo.actor >= 0 && (int32_t)actors[eo.actor].rank < en.rank));
        }
        Ent o;
        if (take_old) { o = ents[r.ps_off + a]; a++; }
        else { o.ctr = ne[lo + b2].ctr; o.actor = ne[lo + b2].actor; b2++; }
        o.row = ri;
        outent[w++] = o;
      }
    }
    if (t == 0) { s.nout = NOUT; s.nnew = NSUCC; }
    __syncthreads();
    // applyChanges patch (P8): stream time of every succ entry's op while the id index is alive
    // (-1: an op of the base document -- rows or deletions it recorded only as succ entries)
    if (s.b.P == 2) {
      int32_t* etime = reinterpret_cast<int32_t*>(wsg + L.etime);
      for (uint32_t i = t; i < NOUT; i += T) {
        const int32_t owner = sr[i].row;
        const uint32_t j1 = i + 1 < NOUT ? succ_cnt[i + 1] : NSUCC;
        for (uint32_t j = succ_cnt[i]; j < j1; j++) {
          // the op of a succ entry: the row with that id (when a document repeats an id under
          // another key, the one whose pred names this row)
          int32_t r = -1;
          FOR_ID(k, idk, R, outent[j].ctr, outent[j].actor) {
            const int32_t c = idk[k].row;
            if (r < 0) r = c;
            const Row& y = rows[c];
            bool hit = false;
            if (y.src_change && !y.insert)
              for (uint32_t q = 0; q < y.ps_cnt; q++) hit |= ents[y.ps_off + q].row == owner;
            if (hit) { r = c; break; }
          }
          etime[j] = (r >= 0 && (uint32_t)r >= s.nb) ? r - (int32_t)s.nb : -1;
        }
      }
    }
    __syncthreads();
#if defined(AM_STOP_PHASE) && AM_STOP_PHASE == 5
    goto done;
#endif

    PH(10);
    // P6: canonical re-encode, one column at a time (DOC_OPS_COLUMNS then DOCUMENT_COLUMNS)
    const ChgRow* chg = hp<ChgRow>(s, L.chg);
    const int64_t* depsv = hp<int64_t>(s, L.deps);
    const uint32_t NC = s.nchg;
    EncCtx ex;
    ex.V = hp<int64_t>(s, L.enc);
    ex.W = ex.V + L.enc_n;
    ex.S = reinterpret_cast<uint32_t*>(ex.W + L.enc_n);
    ex.RS = ex.S + L.enc_n;
    ex.RB = ex.RS + L.enc_n;
    ex.RG = ex.RB + L.enc_n;
    ex.As = A + s.b.span_lo;
    const uint64_t lo = s.b.span_lo;
    auto pk = [lo](uint64_t off, uint32_t len) -> int64_t { return (int64_t)((off - lo) << 32) | (int64_t)len; };
    auto act = [](int32_t a) -> int64_t { return a < 0 ? AM_NULL64 : (int64_t)a; };
    // the value of column c at position i
    auto colval = [&](int c, uint32_t i) -> int64_t {
      int64_t v = 0;
      if (c < OC_GRP_NUM) {
        const Row& r = rows[sr[i].row];
        switch (c) {
          case OC_OBJ_ACTOR: v = act(r.obj_actor); break;
          case OC_OBJ_CTR: v = r.obj_ctr; break;
          case OC_KEY_ACTOR: v = act(r.key_actor); break;
          case OC_KEY_CTR: v = r.key_ctr; break;
          case OC_KEY_STR: v = r.key_len == AM_NOSTR ? AM_NULL64 : pk(r.key_off, r.key_len); break;
          case OC_ID_ACTOR: v = act(r.id_actor); break;
          case OC_ID_CTR: v = r.id_ctr; break;
          case OC_INSERT: v = r.insert; break;
          case OC_ACTION: v = r.action; break;
          case OC_VAL_LEN: v = r.val_len; break;
          case OC_VAL_RAW: v = pk(r.val_off, r.val_len == AM_NULL64 ? 0u : (uint32_t)((uint64_t)r.val_len >> 4)); break;
          case OC_CHLD_ACTOR: v = act(r.chld_actor); break;
          default: v = r.chld_ctr; break;
        }
      } else if (c == OC_GRP_NUM) {
        v = (int64_t)(i + 1 < NOUT ? succ_cnt[i + 1] : NSUCC) - succ_cnt[i];
      } else if (c == OC_GRP_ACTOR) {
        v = act(outent[i].actor);
      } else if (c == OC_GRP_CTR) {
        v = outent[i].ctr;
      } else {
        const ChgRow& g = chg[i < NC ? i : 0];
        switch (c - OC_NCOLS) {
          case DC_ACTOR: v = g.actor; break;
          case DC_SEQ: v = g.seq; break;
          case DC_MAXOP: v = g.max_op; break;
          case DC_TIME: v = g.time; break;
          case DC_MESSAGE: v = g.msg_len == AM_NOSTR ? AM_NULL64 : pk(g.msg_off, g.msg_len); break;
          case DC_DEPS_NUM: v = (int64_t)g.ndeps; break;
          case DC_DEPS_INDEX: v = depsv[i]; break;
          case DC_EXTRA_LEN: v = g.extra_len; break;
          default: v = pk(g.extra_off, g.extra_raw_len); break;
        }
      }
      return v;
    };
    auto coln = [&](int c) -> uint32_t {
      return c < OC_GRP_ACTOR ? NOUT : c < OC_NCOLS ? NSUCC : c == OC_NCOLS + DC_DEPS_INDEX ? s.ndeps : NC;
    };
    // a large document in global mode: each of four waves encodes a column of its own (waves 1..3
    // with the scratch at L.enc_x), four columns at a time; further waves of a 16-wave workgroup wait
    const uint32_t NW = (kDocT > 64 && L.enc_x) ? (kDocT / 64 < 4 ? kDocT / 64 : 4u) : 1u;
    if (NW > 1) {
      const uint32_t wv = t >> 6, ln = t & 63;
      EncCtx exw = ex;
      if (wv > 0) {
        exw.V = reinterpret_cast<int64_t*>(wsg + L.enc_x + (uint64_t)(wv - 1) * 32 * L.enc_n);
        exw.W = exw.V + L.enc_n;
        exw.S = reinterpret_cast<uint32_t*>(exw.W + L.enc_n);
        exw.RS = exw.S + L.enc_n;
        exw.RB = exw.RS + L.enc_n;
        exw.RG = exw.RB + L.enc_n;
      }
      for (int c0 = 0; c0 < OC_NCOLS + DC_NCOLS; c0 += (int)NW) {
        const int c = c0 + (int)wv;
        if (wv < NW && c < OC_NCOLS + DC_NCOLS) {
          const uint32_t n = coln(c);
          for (uint32_t i = ln; i < n; i += 64) exw.V[i] = colval(c, i);
          wave_sync();
          const uint32_t len = encode_column(kEncKind[c], n, wsg + L.colbuf[c], exw, nullptr);
          if (ln == 0) s.col_len[c] = len;
        }
        __syncthreads();
      }
    } else {
      for (int c = 0; c < OC_NCOLS + DC_NCOLS; c++) {
        const uint32_t n = coln(c);
        for (uint32_t i = t; i < n; i += T) ex.V[i] = colval(c, i);
        __syncthreads();
        if (t < 64) {
          const uint32_t len = encode_column(kEncKind[c], n, wsg + L.colbuf[c], ex, nullptr);
          if (t == 0) s.col_len[c] = len;
        }
        __syncthreads();
      }
    }
    __syncthreads();
    if (s.b.UC) unk_encode(s, sr, NOUT, ex, wsg);
    __syncthreads();
    if (s.status) goto done;
    const uint32_t NU = s.b.UC ? s.nunk_ids : 0;
    const uint32_t* uids = reinterpret_cast<const uint32_t*>(wsg + L.unk_ids);
    PH(11);
    // header + body assembly (encodeDocumentHeader, columnar.js:983-1004)
    uint8_t* out = wsg + L.out;
    const uint8_t* heads = hp<uint8_t>(s, L.heads);
    const int64_t* hidx = hp<int64_t>(s, L.hidx);
    if (t == 0) {
      uint64_t body = uleb_len(s.nactors);
      for (uint32_t i = 0; i < s.nactors; i++) body += uleb_len(actors[i].len) + actors[i].len;
      body += uleb_len(s.nheads) + 32ull * s.nheads;
      uint32_t nce = 0, noe = 0;
      for (int c = 0; c < DC_NCOLS; c++) if (s.col_len[16 + c]) { nce++; body += uleb_len(kDocChgColIds[c]) + uleb_len(s.col_len[16 + c]) + s.col_len[16 + c]; }
      for (int c = 0; c < OC_NCOLS; c++) if (s.col_len[c]) { noe++; body += uleb_len(kDocOpColIds[c]) + uleb_len(s.col_len[c]) + s.col_len[c]; }
      for (uint32_t u = 0; u < NU; u++)
        if (uids[2 * NU + u]) { noe++; body += uleb_len(uids[u]) + uleb_len(uids[2 * NU + u]) + uids[2 * NU + u]; }
      body += uleb_len(nce) + uleb_len(noe);
      // headsIndexes only when every head index is known (loaded documents may lack them)
      bool write_hidx = true;
      for (uint32_t i = 0; i < s.nheads; i++) if (hidx[i] < 0) write_hidx = false;
      if (write_hidx)
        for (uint32_t i = 0; i < s.nheads; i++) body += uleb_len((uint64_t)hidx[i]);
      const uint32_t extra_len = s.has_base ? s.dh.extra_len : 0;
      body += extra_len;
      if (9 + 10 + body > L.out_cap) {
        set_err(s, AM_U_CAPACITY);
      } else {
        uint8_t* o = out;
        for (int k = 0; k < 4; k++) *o++ = kMagic[k];
        for (int k = 0; k < 4; k++) *o++ = 0;  // checksum, filled by k_out_hash_ws
        *o++ = 0;  // CHUNK_TYPE_DOCUMENT
        o = put_uleb(o, body);
        o = put_uleb(o, s.nactors);
        for (uint32_t i = 0; i < s.nactors; i++) {
          o = put_uleb(o, actors[i].len);
          for (uint32_t q = 0; q < actors[i].len; q++) *o++ = A[actors[i].off + q];
        }
        o = put_uleb(o, s.nheads);
        for (uint32_t i = 0; i < 32 * s.nheads; i++) *o++ = heads[i];
        o = put_uleb(o, nce);
        for (int c = 0; c < DC_NCOLS; c++) if (s.col_len[16 + c]) { o = put_uleb(o, kDocChgColIds[c]); o = put_uleb(o, s.col_len[16 + c]); }
        o = put_uleb(o, noe);
        // op columns in ascending id: the known ones with the unknown ones interleaved
        {
          uint32_t u = 0;
          for (int c = 0; c <= OC_NCOLS; c++) {
            for (; u < NU && (c == OC_NCOLS || uids[u] < kDocOpColIds[c]); u++)
              if (uids[2 * NU + u]) { o = put_uleb(o, uids[u]); o = put_uleb(o, uids[2 * NU + u]); }
            if (c < OC_NCOLS && s.col_len[c]) { o = put_uleb(o, kDocOpColIds[c]); o = put_uleb(o, s.col_len[c]); }
          }
        }
        uint64_t pos = (uint64_t)(o - out);
        // column data positions, in DOCUMENT_COLUMNS then DOC_OPS_COLUMNS order (unknown op columns
        // keep their output position in uids[NU + u] rewritten as the document offset)
        for (int c = 0; c < DC_NCOLS; c++) { s.col_pos[16 + c] = (uint32_t)pos; pos += s.col_len[16 + c]; }
        {
          uint32_t u = 0;
          uint32_t* uw = reinterpret_cast<uint32_t*>(wsg + L.unk_ids);
          for (int c = 0; c <= OC_NCOLS; c++) {
            for (; u < NU && (c == OC_NCOLS || uids[u] < kDocOpColIds[c]); u++) {
              const uint32_t l = uids[2 * NU + u];
              uw[3 * NU + u] = (uint32_t)pos;  // (unk_ids has room for 4 NU words)
              pos += l;
            }
            if (c < OC_NCOLS) { s.col_pos[c] = (uint32_t)pos; pos += s.col_len[c]; }
          }
        }
        o = out + pos;
        if (write_hidx)
          for (uint32_t i = 0; i < s.nheads; i++) o = put_uleb(o, (uint64_t)hidx[i]);
        for (uint32_t q = 0; q < extra_len; q++) *o++ = A[s.dh.base + s.dh.extra_off + q];
        s.out_len = (uint64_t)(o - out);
      }
    }
    __syncthreads();
    if (s.status) goto done;
    for (int c = 0; c < OC_NCOLS + DC_NCOLS; c++) {
      const uint8_t* src = wsg + L.colbuf[c];
      uint8_t* dst = out + s.col_pos[c];
      for (uint32_t q = t; q < s.col_len[c]; q += T) dst[q] = src[q];
    }
    for (uint32_t u = 0; u < NU; u++) {
      const uint8_t* src = wsg + L.unk_out + uids[NU + u];
      uint8_t* dst = out + uids[3 * NU + u];
      for (uint32_t q = t; q < uids[2 * NU + u]; q += T) dst[q] = src[q];
    }
    // P7: getPatch log (lane 0; the merge arrays of the union region are dead, reuse them). Only for
    // getPatch (P == 1): the applyChanges patch (P == 2) is P8's, which writes the same slot.
    if (s.b.P == 1 && t == 0) {
      const uint64_t R1 = (uint64_t)s.b.R + 1, E1 = (uint64_t)s.b.E + 1;
      uint8_t* ps = hp<uint8_t>(s, L.pscr);
      PatchScratch w;
      w.mk_ctr = reinterpret_cast<int64_t*>(ps);
      w.cs_ctr = w.mk_ctr + R1;
      w.cs_val = w.cs_ctr + R1;
      w.cm_ctr = w.cs_val + R1;
      w.mk_actor = reinterpret_cast<int32_t*>(w.cm_ctr + E1);
      w.cs_actor = w.mk_actor + R1;
      w.cs_left = w.cs_actor + R1;
      w.cm_actor = w.cs_left + R1;
      w.cm_state = w.cm_actor + E1;
      w.mk_vis = reinterpret_cast<uint8_t*>(w.cm_state + E1);
      w.mk_cap = (uint32_t)R1; w.cs_cap = (uint32_t)R1; w.cm_cap = (uint32_t)E1;
      uint8_t* pbase = wsg + L.patch;
      PatchOut po;
      po.rec = reinterpret_cast<PatchRec*>(pbase + 64);
      po.mval = reinterpret_cast<PatchVal*>(pbase + 64 + 64 * L.patch_nrec);
      po.heap = pbase + 64 + 64 * L.patch_nrec + 32 * L.patch_nmval;
      po.cap_rec = L.patch_nrec; po.cap_mval = L.patch_nmval; po.cap_heap = L.patch_heap;
      po.arg0 = po.arg1 = 0;
      RowSrc src{rows, sr, succ_cnt, outent, NOUT, NSUCC, actors, s.nactors, chg, NC, A, s.nb_act < s.nb ? 0u : NOUT};
      int64_t pmax = 0;
      patch_scan(src, po, w, pmax);
      wire_out(po, pmax, wsg + L.pwire, L.pwire_cap);
    }
    // P8: the patch applyChanges returns (am_diff.h), after the merge, in k_diff: a launch of one
    // wave per document after this one (the replay is a chain of dependent loads; at one lane per
    // k_doc workgroup -- LDS mode: two to four per CU -- too few of them are in flight). This
    // workgroup leaves the counts at L.djob; an LDS-mode document first mirrors its hot set (the
    // rows, entries, sort records, actors, change rows and staged input the replay reads) into its
    // global workspace, where a global-mode document keeps it anyway.
    if (s.b.P == 2) {
      if constexpr (kHotLds) {
        const uint4* src = hp<const uint4>(s, 0);
        uint4* dst = reinterpret_cast<uint4*>(wsg);
        for (uint32_t q = t; q < (uint32_t)(L.hot_total / 16); q += T) dst[q] = src[q];
      }
      if (t == 0) {
        uint32_t* job = reinterpret_cast<uint32_t*>(wsg + L.djob);
        job[0] = s.npass; job[1] = s.nb; job[2] = s.nrows; job[3] = NOUT;
        job[4] = NSUCC; job[5] = s.nb_act < s.nb ? 0u : s.nb; job[6] = s.nactors; job[7] = NC;
      }
    }
    // heads for the host (hot region may be LDS): mirror into the global workspace
    if (kHotLds)
      for (uint32_t q = t; q < 32 * s.nheads; q += T) wsg[L.heads + q] = heads[q];
  }
    PH(12);
done:
  __syncthreads();
  if (t == 0) {
    am_doc_result r;
    r.status = s.status;
#ifdef AM_DIFF_CHECK
    if (s.dbg_phase != 0xffffu) r.status = 280 + s.dbg_phase;
    if (s.dbg_canary == 0xffffu && dbg_canary_hit(wsg + s.L.total)) s.dbg_canary = 99;  // after the last marker
    if (s.dbg_canary != 0xffffu) r.status = 300 + s.dbg_canary;
#endif
    r.err_change = s.errchg;
    r.arg0 = s.arg0;
    r.arg1 = s.arg1;
    r.arg_actor_off = s.arg_actor_off;
    r.arg_actor_len = s.arg_actor_len;
    r.napplied = s.napplied;
    r.nqueued = s.nqueued;
    r.nheads = s.nheads;
    r.nops = s.nout;
    r.nchanges = s.nchg;
    r.max_op = s.max_op;
    r.out_off = 0;
    r.out_len = s.status ? 0 : s.out_len;
    r.ws_off = ws_off[doc];
    r.ws_bytes = s.L.total;
    results[doc] = r;
  }
}

// k_doc: workgroup per document (grid = documents), or -- LDS mode after k_doc_fast, with `rest` --
// a grid of a few thousand workgroups looping over the list of the documents k_doc_fast left
// (rest[0] = how many, rest[1..]), so a batch the fast kernel merged whole costs microseconds here.
__global__ void __launch_bounds__(kDocT) K_DOC_WAVES_ATTR k_doc(const uint8_t* __restrict__ arena, const am_chunk_desc* __restrict__ chunks,
                                               const am_doc_desc* __restrict__ docs, const am_known_hash* __restrict__ known,
                                               const ChunkInfo* __restrict__ info, const DocBounds* __restrict__ bounds,
                                               const uint64_t* __restrict__ ws_off, uint8_t* __restrict__ ws_base,
                                               uint64_t ws_cap, uint32_t lds_bytes, am_doc_result* __restrict__ results,
                                               int32_t* __restrict__ chg_state, const uint8_t* __restrict__ fast_done,
                                               const uint32_t* __restrict__ rest) {
  if constexpr (kHotLds) {
    // one call site (the body is large): without `rest` the loop runs once, for blockIdx.x
    const uint32_t n = rest ? rest[0] : blockIdx.x + 1, step = rest ? gridDim.x : 1u;
    for (uint32_t i = blockIdx.x; i < n; i += step) {
      __syncthreads();  // the previous document's shared state is no longer read
      k_doc_one(rest ? rest[1 + i] : i, arena, chunks, docs, known, info, bounds, ws_off, ws_base, ws_cap, lds_bytes, results,
                chg_state, fast_done);
    }
  } else {
    // the global mode keeps one workgroup per document (a loop costs it its register budget)
    (void)rest;
    k_doc_one(blockIdx.x, arena, chunks, docs, known, info, bounds, ws_off, ws_base, ws_cap, lds_bytes, results, chg_state,
              fast_done);
  }
}

