// am_napi.c -- Node N-API addon over the C ABI of libautomerge_amd.so (include/automerge_amd.h).
//
// This is the binding a reference maintainer adds to load the MI355X engine through
// Automerge.setDefaultBackend() (src/automerge.js:147-149): backend.js in this directory wraps
// these functions into the Backend module surface of backend/backend.js:8-197.
// Document handles are N-API externals; errors become JS exceptions of the reference's class
// (RangeError / TypeError) and message.
#include <node_api.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/automerge_amd.h"

typedef struct { am_doc* doc; } DocBox;

static am_engine* g_engine = NULL;

#define NAPI_OK(call)                                                         \
  do {                                                                        \
    if ((call) != napi_ok) {                                                  \
      napi_throw_error(env, NULL, "automerge_amd: N-API call failed: " #call); \
      return NULL;                                                            \
    }                                                                         \
  } while (0)

static napi_value throw_am(napi_env env, const am_error* e) {
  if (e->is_type_error) napi_throw_type_error(env, NULL, e->message);
  else napi_throw_range_error(env, NULL, e->message);
  return NULL;
}

static am_engine* engine(napi_env env) {
  if (!g_engine) {
    am_error e;
    const char* dev = getenv("AM_DEVICE");
    g_engine = am_engine_create(dev ? atoi(dev) : 0, &e);
    if (!g_engine) throw_am(env, &e);
  }
  return g_engine;
}

static void box_finalize(napi_env env, void* data, void* hint) {
  (void)env; (void)hint;
  DocBox* b = (DocBox*)data;
  if (b->doc) am_doc_free(b->doc);
  free(b);
}

static napi_value wrap_doc(napi_env env, am_doc* d) {
  DocBox* b = (DocBox*)malloc(sizeof(DocBox));
  b->doc = d;
  napi_value v;
  NAPI_OK(napi_create_external(env, b, box_finalize, NULL, &v));
  return v;
}

static DocBox* get_box(napi_env env, napi_value v) {
  void* p = NULL;
  if (napi_get_value_external(env, v, &p) != napi_ok || !p) {
    napi_throw_type_error(env, NULL, "automerge_amd: not a document handle");
    return NULL;
  }
  DocBox* b = (DocBox*)p;
  if (!b->doc) {
    napi_throw_error(env, NULL, "automerge_amd: document handle was freed");
    return NULL;
  }
  return b;
}

static int get_bytes(napi_env env, napi_value v, const uint8_t** data, size_t* len) {
  bool is_ta = false;
  napi_is_typedarray(env, v, &is_ta);
  if (is_ta) {
    napi_typedarray_type t;
    void* p;
    napi_value ab;
    size_t off;
    if (napi_get_typedarray_info(env, v, &t, len, &p, &ab, &off) != napi_ok || t != napi_uint8_array) return 0;
    *data = (const uint8_t*)p;
    return 1;
  }
  bool is_buf = false;
  napi_is_buffer(env, v, &is_buf);
  if (is_buf) {
    void* p;
    if (napi_get_buffer_info(env, v, &p, len) != napi_ok) return 0;
    *data = (const uint8_t*)p;
    return 1;
  }
  return 0;
}

static napi_value new_u8(napi_env env, const uint8_t* data, size_t len) {
  napi_value ab, ta;
  void* p;
  NAPI_OK(napi_create_arraybuffer(env, len, &p, &ab));
  if (len) memcpy(p, data, len);
  NAPI_OK(napi_create_typedarray(env, napi_uint8_array, len, ab, 0, &ta));
  return ta;
}

static napi_value hex_list(napi_env env, const uint8_t* h32, size_t n) {
  static const char* hx = "0123456789abcdef";
  napi_value arr;
  NAPI_OK(napi_create_array_with_length(env, n, &arr));
  for (size_t i = 0; i < n; i++) {
    char s[65];
    for (int k = 0; k < 32; k++) { s[2 * k] = hx[h32[32 * i + k] >> 4]; s[2 * k + 1] = hx[h32[32 * i + k] & 15]; }
    s[64] = 0;
    napi_value str;
    NAPI_OK(napi_create_string_utf8(env, s, 64, &str));
    NAPI_OK(napi_set_element(env, arr, (uint32_t)i, str));
  }
  return arr;
}

// ---- exported functions ----
static napi_value js_doc_init(napi_env env, napi_callback_info info) {
  (void)info;
  am_engine* e = engine(env);
  if (!e) return NULL;
  return wrap_doc(env, am_doc_init(e));
}

static napi_value js_doc_load(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  NAPI_OK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  const uint8_t* data;
  size_t len;
  if (argc < 1 || !get_bytes(env, argv[0], &data, &len)) {
    napi_throw_type_error(env, NULL, "Not a byte array");
    return NULL;
  }
  am_engine* e = engine(env);
  if (!e) return NULL;
  am_error err;
  am_doc* d = am_doc_load(e, data, len, &err);
  if (!d) return throw_am(env, &err);
  return wrap_doc(env, d);
}

static napi_value js_doc_clone(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  NAPI_OK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  DocBox* b = get_box(env, argv[0]);
  if (!b) return NULL;
  return wrap_doc(env, am_doc_clone(b->doc));
}

static napi_value js_doc_free(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  NAPI_OK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  void* p = NULL;
  if (napi_get_value_external(env, argv[0], &p) == napi_ok && p) {
    DocBox* b = (DocBox*)p;
    if (b->doc) am_doc_free(b->doc);
    b->doc = NULL;
  }
  return NULL;
}

// applyChanges(handle, [Uint8Array...]) -> undefined (throws on error; the document is unchanged then)
static napi_value js_doc_apply(napi_env env, napi_callback_info info) {
  size_t argc = 3;
  napi_value argv[3];
  NAPI_OK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  DocBox* b = get_box(env, argv[0]);
  if (!b) return NULL;
  bool is_arr = false;
  napi_is_array(env, argv[1], &is_arr);
  if (!is_arr) {
    napi_throw_type_error(env, NULL, "Pass an array of changes");
    return NULL;
  }
  uint32_t n = 0;
  NAPI_OK(napi_get_array_length(env, argv[1], &n));
  const uint8_t** bufs = (const uint8_t**)malloc(sizeof(uint8_t*) * (n ? n : 1));
  size_t* lens = (size_t*)malloc(sizeof(size_t) * (n ? n : 1));
  for (uint32_t i = 0; i < n; i++) {
    napi_value el;
    if (napi_get_element(env, argv[1], i, &el) != napi_ok || !get_bytes(env, el, &bufs[i], &lens[i])) {
      free(bufs); free(lens);
      napi_throw_type_error(env, NULL, "Change is not a byte array");
      return NULL;
    }
  }
  // third argument true: Backend.applyChanges -- return the patch log (am_doc_apply_changes_patch)
  bool want_patch = false;
  if (argc > 2) napi_get_value_bool(env, argv[2], &want_patch);
  am_error err;
  uint8_t* out = NULL;
  size_t len = 0;
  int rc = want_patch ? am_doc_apply_changes_patch(b->doc, bufs, lens, n, &out, &len, &err)
                      : am_doc_apply_changes(b->doc, bufs, lens, n, &err);
  free(bufs); free(lens);
  if (rc) return throw_am(env, &err);
  if (!want_patch) return NULL;
  napi_value v = new_u8(env, out, len);
  am_free(out);
  return v;
}

static napi_value js_doc_save(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  NAPI_OK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  DocBox* b = get_box(env, argv[0]);
  if (!b) return NULL;
  uint8_t* out = NULL;
  size_t len = 0;
  am_error err;
  if (am_doc_save(b->doc, &out, &len, &err)) return throw_am(env, &err);
  napi_value v = new_u8(env, out, len);
  am_free(out);
  return v;
}

static napi_value js_doc_heads(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  NAPI_OK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  DocBox* b = get_box(env, argv[0]);
  if (!b) return NULL;
  size_t n = am_doc_get_heads(b->doc, NULL, 0);
  uint8_t* h = (uint8_t*)malloc(32 * (n ? n : 1));
  am_doc_get_heads(b->doc, h, n);
  napi_value v = hex_list(env, h, n);
  free(h);
  return v;
}

// changes(handle) -> [{hash, bytes}] in application order
static napi_value js_doc_changes(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  NAPI_OK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  DocBox* b = get_box(env, argv[0]);
  if (!b) return NULL;
  am_error e;
  if (am_doc_compute_hash_graph(b->doc, &e)) {  /* computeHashGraph of a loaded document (new.js:1879) */
    napi_throw_range_error(env, NULL, e.message);
    return NULL;
  }
  size_t n = 0;
  {
    const uint8_t* d0;
    size_t l0;
    while (am_doc_change(b->doc, n, &d0, &l0, NULL) == 0) n++;
  }
  napi_value arr;
  NAPI_OK(napi_create_array_with_length(env, n, &arr));
  for (size_t i = 0; i < n; i++) {
    const uint8_t* data;
    size_t len;
    uint8_t h[32];
    if (am_doc_change(b->doc, i, &data, &len, h)) {
      napi_throw_range_error(env, NULL, "automerge_amd: change history unavailable for this document");
      return NULL;
    }
    napi_value o, hv, hs, bv;
    NAPI_OK(napi_create_object(env, &o));
    hv = hex_list(env, h, 1);
    NAPI_OK(napi_get_element(env, hv, 0, &hs));
    bv = new_u8(env, data, len);
    NAPI_OK(napi_set_named_property(env, o, "hash", hs));
    NAPI_OK(napi_set_named_property(env, o, "bytes", bv));
    NAPI_OK(napi_set_element(env, arr, (uint32_t)i, o));
  }
  return arr;
}

static napi_value js_doc_counts(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  NAPI_OK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  DocBox* b = get_box(env, argv[0]);
  if (!b) return NULL;
  napi_value o, a, c, m;
  NAPI_OK(napi_create_object(env, &o));
  NAPI_OK(napi_create_double(env, (double)am_doc_pending(b->doc), &a));
  NAPI_OK(napi_create_double(env, (double)am_doc_num_changes(b->doc), &c));
  NAPI_OK(napi_create_double(env, (double)am_doc_max_op(b->doc), &m));
  NAPI_OK(napi_set_named_property(env, o, "pending", a));
  NAPI_OK(napi_set_named_property(env, o, "changes", c));
  NAPI_OK(napi_set_named_property(env, o, "maxOp", m));
  return o;
}

// patch(handle) -> Uint8Array: the getPatch() log (am_doc_get_patch; materialized in backend.js)
static napi_value js_doc_patch(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  NAPI_OK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  DocBox* b = get_box(env, argv[0]);
  if (!b) return NULL;
  uint8_t* out = NULL;
  size_t len = 0;
  am_error err;
  if (am_doc_get_patch(b->doc, &out, &len, &err)) return throw_am(env, &err);
  napi_value v = new_u8(env, out, len);
  am_free(out);
  return v;
}

// queued(handle) -> [Uint8Array] changes waiting for missing dependencies
static napi_value js_doc_queued(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  NAPI_OK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  DocBox* b = get_box(env, argv[0]);
  if (!b) return NULL;
  const size_t n = am_doc_pending(b->doc);
  napi_value arr;
  NAPI_OK(napi_create_array_with_length(env, n, &arr));
  for (size_t i = 0; i < n; i++) {
    const uint8_t* data;
    size_t len;
    if (am_doc_queued(b->doc, i, &data, &len)) break;
    NAPI_OK(napi_set_element(env, arr, (uint32_t)i, new_u8(env, data, len)));
  }
  return arr;
}

// changeHashes([Uint8Array]) -> [hex]: SHA-256 hashes of change chunks (decodeChangeMeta hash)
static napi_value js_change_hashes(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  NAPI_OK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  uint32_t n = 0;
  NAPI_OK(napi_get_array_length(env, argv[0], &n));
  const uint8_t** bufs = (const uint8_t**)malloc(sizeof(uint8_t*) * (n ? n : 1));
  size_t* lens = (size_t*)malloc(sizeof(size_t) * (n ? n : 1));
  uint8_t* h = (uint8_t*)malloc(32 * (size_t)(n ? n : 1));
  for (uint32_t i = 0; i < n; i++) {
    napi_value el;
    if (napi_get_element(env, argv[0], i, &el) != napi_ok || !get_bytes(env, el, &bufs[i], &lens[i])) {
      free(bufs); free(lens); free(h);
      napi_throw_type_error(env, NULL, "Change is not a byte array");
      return NULL;
    }
  }
  am_engine* e = engine(env);
  am_error err;
  if (!e || am_change_hashes(e, bufs, lens, n, h, &err)) {
    free(bufs); free(lens); free(h);
    return e ? throw_am(env, &err) : NULL;
  }
  napi_value v = hex_list(env, h, n);
  free(bufs); free(lens); free(h);
  return v;
}

// ---- hash-graph queries, local changes and sync (include/automerge_amd.h) ----
#define ARGS(n)                                                  \
  size_t argc = (n);                                             \
  napi_value argv[(n) > 0 ? (n) : 1];                            \
  NAPI_OK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));

// throws the engine error; `applied` marks an error raised after the document changed
static napi_value throw_am2(napi_env env, const am_error* e, int applied) {
  napi_value msg, err, t;
  NAPI_OK(napi_create_string_utf8(env, e->message, NAPI_AUTO_LENGTH, &msg));
  if (e->is_type_error) NAPI_OK(napi_create_type_error(env, NULL, msg, &err));
  else NAPI_OK(napi_create_range_error(env, NULL, msg, &err));
  if (applied) {
    NAPI_OK(napi_get_boolean(env, true, &t));
    NAPI_OK(napi_set_named_property(env, err, "applied", t));
  }
  napi_throw(env, err);
  return NULL;
}

static char* get_string(napi_env env, napi_value v, size_t* len) {
  if (napi_get_value_string_utf8(env, v, NULL, 0, len) != napi_ok) {
    napi_throw_type_error(env, NULL, "automerge_amd: expected a string");
    return NULL;
  }
  char* s = (char*)malloc(*len + 1);
  napi_get_value_string_utf8(env, v, s, *len + 1, len);
  return s;
}

static int arg_bytes(napi_env env, napi_value v, const uint8_t** p, size_t* n) {
  if (!get_bytes(env, v, p, n)) {
    napi_throw_type_error(env, NULL, "automerge_amd: expected a Uint8Array");
    return 0;
  }
  return 1;
}

static napi_value change_list(napi_env env, am_doc* d, const uint64_t* idx, size_t n) {
  napi_value arr;
  NAPI_OK(napi_create_array_with_length(env, n, &arr));
  for (size_t i = 0; i < n; i++) {
    const uint8_t* data;
    size_t len;
    if (am_doc_change(d, (size_t)idx[i], &data, &len, NULL)) {
      napi_throw_range_error(env, NULL, "automerge_amd: change index out of range");
      return NULL;
    }
    NAPI_OK(napi_set_element(env, arr, (uint32_t)i, new_u8(env, data, len)));
  }
  return arr;
}

// getChanges(handle, flatHaveHashes) -> [Uint8Array]
static napi_value js_doc_get_changes(napi_env env, napi_callback_info info) {
  ARGS(2)
  DocBox* b = get_box(env, argv[0]);
  const uint8_t* h;
  size_t hl;
  if (!b || !arg_bytes(env, argv[1], &h, &hl)) return NULL;
  uint64_t* idx = NULL;
  size_t n = 0;
  am_error err;
  if (am_doc_get_changes(b->doc, h, hl / 32, &idx, &n, &err)) return throw_am(env, &err);
  napi_value v = change_list(env, b->doc, idx, n);
  am_free(idx);
  return v;
}

// getChangesAdded(handle1, handle2) -> [Uint8Array]
static napi_value js_doc_get_changes_added(napi_env env, napi_callback_info info) {
  ARGS(2)
  DocBox* b1 = get_box(env, argv[0]);
  DocBox* b2 = b1 ? get_box(env, argv[1]) : NULL;
  if (!b2) return NULL;
  uint64_t* idx = NULL;
  size_t n = 0;
  am_error err;
  if (am_doc_get_changes_added(b1->doc, b2->doc, &idx, &n, &err)) return throw_am(env, &err);
  napi_value v = change_list(env, b2->doc, idx, n);
  am_free(idx);
  return v;
}

// changeByHash(handle, hash32) -> Uint8Array | undefined
static napi_value js_doc_change_by_hash(napi_env env, napi_callback_info info) {
  ARGS(2)
  DocBox* b = get_box(env, argv[0]);
  const uint8_t* h;
  size_t hl;
  if (!b || !arg_bytes(env, argv[1], &h, &hl)) return NULL;
  napi_value undef;
  NAPI_OK(napi_get_undefined(env, &undef));
  if (hl != 32) return undef;
  const int64_t i = am_doc_change_index(b->doc, h);
  if (i == -2) {
    napi_throw_range_error(env, NULL, "automerge_amd: the document history could not be reconstructed");
    return NULL;
  }
  if (i < 0) return undef;
  uint64_t one = (uint64_t)i;
  napi_value arr = change_list(env, b->doc, &one, 1), el;
  if (!arr) return NULL;
  NAPI_OK(napi_get_element(env, arr, 0, &el));
  return el;
}

// missingDeps(handle, flatHeads) -> Uint8Array (sorted 32-byte hashes)
static napi_value js_doc_missing_deps(napi_env env, napi_callback_info info) {
  ARGS(2)
  DocBox* b = get_box(env, argv[0]);
  const uint8_t* h;
  size_t hl;
  if (!b || !arg_bytes(env, argv[1], &h, &hl)) return NULL;
  uint8_t* out = NULL;
  size_t n = 0;
  am_error err;
  if (am_doc_get_missing_deps(b->doc, h, hl / 32, &out, &n, &err)) return throw_am(env, &err);
  napi_value v = new_u8(env, out, 32 * n);
  am_free(out);
  return v;
}

// applyLocal(handle, json) -> {change, patch, newHash, lastHash|null}
static napi_value js_doc_apply_local(napi_env env, napi_callback_info info) {
  ARGS(2)
  DocBox* b = get_box(env, argv[0]);
  if (!b) return NULL;
  size_t jl;
  char* js = get_string(env, argv[1], &jl);
  if (!js) return NULL;
  uint8_t *change = NULL, *patch = NULL, nh[32], lh[32];
  size_t cl = 0, pl = 0;
  int has_last = 0;
  am_error err;
  const int rc = am_doc_apply_local_change(b->doc, js, jl, &change, &cl, &patch, &pl, nh, lh, &has_last, &err);
  free(js);
  if (rc) return throw_am2(env, &err, rc == 2);
  napi_value o, nul;
  NAPI_OK(napi_create_object(env, &o));
  NAPI_OK(napi_get_null(env, &nul));
  NAPI_OK(napi_set_named_property(env, o, "change", new_u8(env, change, cl)));
  NAPI_OK(napi_set_named_property(env, o, "patch", new_u8(env, patch, pl)));
  NAPI_OK(napi_set_named_property(env, o, "newHash", hex_list(env, nh, 1)));
  NAPI_OK(napi_set_named_property(env, o, "lastHash", has_last ? hex_list(env, lh, 1) : nul));
  am_free(change);
  am_free(patch);
  return o;
}

// encodeChange(json) -> Uint8Array
static napi_value js_encode_change(napi_env env, napi_callback_info info) {
  ARGS(1)
  size_t jl;
  char* js = get_string(env, argv[0], &jl);
  if (!js) return NULL;
  uint8_t* out = NULL;
  size_t n = 0;
  am_error err;
  const int rc = am_encode_change(js, jl, &out, &n, NULL, &err);
  free(js);
  if (rc) return throw_am(env, &err);
  napi_value v = new_u8(env, out, n);
  am_free(out);
  return v;
}

// syncGenerate([handle...], [stateBlob...]) -> [[stateBlob, message|null] | Error]
static napi_value js_sync_generate(napi_env env, napi_callback_info info) {
  ARGS(2)
  uint32_t n = 0;
  NAPI_OK(napi_get_array_length(env, argv[0], &n));
  am_doc** docs = (am_doc**)calloc(n ? n : 1, sizeof(am_doc*));
  const uint8_t** st = (const uint8_t**)calloc(n ? n : 1, sizeof(uint8_t*));
  size_t* sl = (size_t*)calloc(n ? n : 1, sizeof(size_t));
  uint8_t** ost = (uint8_t**)calloc(n ? n : 1, sizeof(uint8_t*));
  size_t* osl = (size_t*)calloc(n ? n : 1, sizeof(size_t));
  uint8_t** msg = (uint8_t**)calloc(n ? n : 1, sizeof(uint8_t*));
  size_t* ml = (size_t*)calloc(n ? n : 1, sizeof(size_t));
  uint32_t* codes = (uint32_t*)calloc(n ? n : 1, sizeof(uint32_t));
  char** emsg = (char**)calloc(n ? n : 1, sizeof(char*));
  napi_value res = NULL;
  int ok = 1;
  for (uint32_t i = 0; i < n && ok; i++) {
    napi_value hv, sv;
    DocBox* b;
    ok = napi_get_element(env, argv[0], i, &hv) == napi_ok && (b = get_box(env, hv)) != NULL &&
         napi_get_element(env, argv[1], i, &sv) == napi_ok && arg_bytes(env, sv, &st[i], &sl[i]);
    if (ok) docs[i] = b->doc;
  }
  if (ok) {
    am_sync_generate(n, docs, st, sl, ost, osl, msg, ml, codes, emsg);
    napi_create_array_with_length(env, n, &res);
    for (uint32_t i = 0; i < n; i++) {
      napi_value el;
      if (codes[i]) {
        napi_value m;
        napi_create_string_utf8(env, emsg[i] ? emsg[i] : "", NAPI_AUTO_LENGTH, &m);
        if (codes[i] & 0x80000000u) napi_create_type_error(env, NULL, m, &el);
        else napi_create_range_error(env, NULL, m, &el);
      } else {
        napi_value nul;
        napi_get_null(env, &nul);
        napi_create_array_with_length(env, 2, &el);
        napi_set_element(env, el, 0, new_u8(env, ost[i], osl[i]));
        napi_set_element(env, el, 1, msg[i] ? new_u8(env, msg[i], ml[i]) : nul);
      }
      napi_set_element(env, res, i, el);
      am_free(ost[i]);
      am_free(msg[i]);
    }
  }
  free(docs); free(st); free(sl); free(ost); free(osl); free(msg); free(ml); free(codes);
  for (uint32_t i = 0; i < n; i++) am_free(emsg[i]);
  free(emsg);
  return res;
}

// syncReceive(handle, stateBlob, message) -> [stateBlob, patch|null]
static napi_value js_sync_receive(napi_env env, napi_callback_info info) {
  ARGS(3)
  DocBox* b = get_box(env, argv[0]);
  const uint8_t *st, *m;
  size_t sl, ml;
  if (!b || !arg_bytes(env, argv[1], &st, &sl) || !arg_bytes(env, argv[2], &m, &ml)) return NULL;
  uint8_t *ost = NULL, *patch = NULL;
  size_t osl = 0, pl = 0;
  am_error err;
  const int rc = am_sync_receive(b->doc, st, sl, m, ml, &ost, &osl, &patch, &pl, &err);
  if (rc) return throw_am2(env, &err, rc == 2);
  napi_value o, nul;
  NAPI_OK(napi_get_null(env, &nul));
  NAPI_OK(napi_create_array_with_length(env, 2, &o));
  NAPI_OK(napi_set_element(env, o, 0, new_u8(env, ost, osl)));
  NAPI_OK(napi_set_element(env, o, 1, patch ? new_u8(env, patch, pl) : nul));
  am_free(ost);
  am_free(patch);
  return o;
}

static napi_value js_sync_encode_message(napi_env env, napi_callback_info info) {
  ARGS(1)
  size_t jl;
  char* js = get_string(env, argv[0], &jl);
  if (!js) return NULL;
  uint8_t* out = NULL;
  size_t n = 0;
  am_error err;
  const int rc = am_sync_encode_message(js, jl, &out, &n, &err);
  free(js);
  if (rc) return throw_am(env, &err);
  napi_value v = new_u8(env, out, n);
  am_free(out);
  return v;
}

// syncDecodeMessage(bytes) -> {heads: flat, need: flat, have: [{lastSync: flat, bloom}], changes: [u8]}
static napi_value js_sync_decode_message(napi_env env, napi_callback_info info) {
  ARGS(1)
  const uint8_t* m;
  size_t ml;
  if (!arg_bytes(env, argv[0], &m, &ml)) return NULL;
  am_span* sp = NULL;
  uint64_t off[2];
  uint32_t cnt[4];
  am_error err;
  if (am_sync_decode_messages(1, &m, &ml, &sp, off, cnt, &err)) {
    am_free(sp);
    return throw_am(env, &err);
  }
  napi_value o, have, changes;
  NAPI_OK(napi_create_object(env, &o));
  size_t k = 0;
  NAPI_OK(napi_set_named_property(env, o, "heads", new_u8(env, m + sp[k].off, 32 * sp[k].len))); k++;
  NAPI_OK(napi_set_named_property(env, o, "need", new_u8(env, m + sp[k].off, 32 * sp[k].len))); k++;
  NAPI_OK(napi_create_array_with_length(env, cnt[2], &have));
  for (uint32_t i = 0; i < cnt[2]; i++, k += 2) {
    napi_value h;
    NAPI_OK(napi_create_object(env, &h));
    NAPI_OK(napi_set_named_property(env, h, "lastSync", new_u8(env, m + sp[k].off, 32 * sp[k].len)));
    NAPI_OK(napi_set_named_property(env, h, "bloom", new_u8(env, m + sp[k + 1].off, sp[k + 1].len)));
    NAPI_OK(napi_set_element(env, have, i, h));
  }
  NAPI_OK(napi_create_array_with_length(env, cnt[3], &changes));
  for (uint32_t i = 0; i < cnt[3]; i++, k++) NAPI_OK(napi_set_element(env, changes, i, new_u8(env, m + sp[k].off, sp[k].len)));
  NAPI_OK(napi_set_named_property(env, o, "have", have));
  NAPI_OK(napi_set_named_property(env, o, "changes", changes));
  am_free(sp);
  return o;
}

static napi_value js_sync_state_conv(napi_env env, napi_callback_info info, int encode) {
  ARGS(1)
  const uint8_t* p;
  size_t n;
  if (!arg_bytes(env, argv[0], &p, &n)) return NULL;
  uint8_t* out = NULL;
  size_t on = 0;
  am_error err;
  if (encode ? am_sync_encode_state(p, n, &out, &on, &err) : am_sync_decode_state(p, n, &out, &on, &err))
    return throw_am(env, &err);
  napi_value v = new_u8(env, out, on);
  am_free(out);
  return v;
}
static napi_value js_sync_encode_state(napi_env env, napi_callback_info info) { return js_sync_state_conv(env, info, 1); }
static napi_value js_sync_decode_state(napi_env env, napi_callback_info info) { return js_sync_state_conv(env, info, 0); }

// ---- the batched surface (am_doc_*_batch, am_sync_receive_batch): one GPU batch per call; per
// item the single call's result, or its error object in its place ----
static napi_value err_obj(napi_env env, uint32_t code, const char* msg) {
  napi_value m, e;
  napi_create_string_utf8(env, msg ? msg : "", NAPI_AUTO_LENGTH, &m);
  if (code & 0x80000000u) napi_create_type_error(env, NULL, m, &e);
  else napi_create_range_error(env, NULL, m, &e);
  if (code & 0x40000000u) {
    napi_value t;
    napi_get_boolean(env, true, &t);
    napi_set_named_property(env, e, "applied", t);
  }
  return e;
}
// {log, maxOp, heads, pending}: what a patch log is materialized with, as of its call
static napi_value call_result(napi_env env, uint8_t* log, size_t len, am_call_info* ci) {
  napi_value o, v;
  napi_create_object(env, &o);
  napi_set_named_property(env, o, "log", new_u8(env, log, len));
  napi_create_double(env, (double)ci->max_op, &v);
  napi_set_named_property(env, o, "maxOp", v);
  napi_set_named_property(env, o, "heads", hex_list(env, ci->heads, ci->nheads));
  napi_create_uint32(env, ci->pending, &v);
  napi_set_named_property(env, o, "pending", v);
  am_free(ci->heads);
  ci->heads = NULL;
  return o;
}
static int handles_of(napi_env env, napi_value arr, uint32_t n, am_doc** docs) {
  for (uint32_t i = 0; i < n; i++) {
    napi_value hv;
    DocBox* b;
    if (napi_get_element(env, arr, i, &hv) != napi_ok || (b = get_box(env, hv)) == NULL) return 0;
    docs[i] = b->doc;
  }
  return 1;
}
#define NA(n) ((n) ? (n) : 1)

// docLoadBatch([Uint8Array]) -> [handle | Error]
static napi_value js_doc_load_batch(napi_env env, napi_callback_info info) {
  ARGS(1)
  uint32_t n = 0;
  NAPI_OK(napi_get_array_length(env, argv[0], &n));
  am_engine* e = engine(env);
  if (!e) return NULL;
  const uint8_t** data = (const uint8_t**)calloc(NA(n), sizeof(uint8_t*));
  size_t* lens = (size_t*)calloc(NA(n), sizeof(size_t));
  am_doc** docs = (am_doc**)calloc(NA(n), sizeof(am_doc*));
  uint32_t* codes = (uint32_t*)calloc(NA(n), sizeof(uint32_t));
  char** msgs = (char**)calloc(NA(n), sizeof(char*));
  napi_value res = NULL;
  int ok = 1;
  for (uint32_t i = 0; i < n && ok; i++) {
    napi_value v;
    ok = napi_get_element(env, argv[0], i, &v) == napi_ok && arg_bytes(env, v, &data[i], &lens[i]);
  }
  if (ok) {
    am_doc_load_batch(e, n, data, lens, docs, codes, msgs);
    napi_create_array_with_length(env, n, &res);
    for (uint32_t i = 0; i < n; i++) napi_set_element(env, res, i, codes[i] ? err_obj(env, codes[i], msgs[i]) : wrap_doc(env, docs[i]));
  }
  for (uint32_t i = 0; i < n; i++) am_free(msgs[i]);
  free(data); free(lens); free(docs); free(codes); free(msgs);
  return res;
}

// docApplyBatch([handle], [[Uint8Array]], wantPatch) -> [{log, maxOp, heads, pending} | null | Error]
static napi_value js_doc_apply_batch(napi_env env, napi_callback_info info) {
  ARGS(3)
  uint32_t n = 0;
  NAPI_OK(napi_get_array_length(env, argv[0], &n));
  bool want = false;
  napi_get_value_bool(env, argv[2], &want);
  am_doc** docs = (am_doc**)calloc(NA(n), sizeof(am_doc*));
  size_t* off = (size_t*)calloc(n + 1, sizeof(size_t));
  uint8_t** pats = (uint8_t**)calloc(NA(n), sizeof(uint8_t*));
  size_t* pl = (size_t*)calloc(NA(n), sizeof(size_t));
  am_call_info* ci = (am_call_info*)calloc(NA(n), sizeof(am_call_info));
  uint32_t* codes = (uint32_t*)calloc(NA(n), sizeof(uint32_t));
  char** msgs = (char**)calloc(NA(n), sizeof(char*));
  const uint8_t** bufs = NULL;
  size_t* lens = NULL;
  size_t nb = 0, cap = 0;
  napi_value res = NULL;
  int ok = handles_of(env, argv[0], n, docs);
  for (uint32_t i = 0; i < n && ok; i++) {
    napi_value cl;
    uint32_t k = 0;
    bool is_arr = false;
    ok = napi_get_element(env, argv[1], i, &cl) == napi_ok && napi_is_array(env, cl, &is_arr) == napi_ok && is_arr &&
         napi_get_array_length(env, cl, &k) == napi_ok;
    if (!ok) { napi_throw_type_error(env, NULL, "Pass an array of changes"); break; }
    if (nb + k > cap) {
      cap = 2 * (nb + k) + 16;
      bufs = (const uint8_t**)realloc(bufs, cap * sizeof(uint8_t*));
      lens = (size_t*)realloc(lens, cap * sizeof(size_t));
    }
    for (uint32_t j = 0; j < k && ok; j++) {
      napi_value el;
      ok = napi_get_element(env, cl, j, &el) == napi_ok && get_bytes(env, el, &bufs[nb], &lens[nb]);
      if (!ok) napi_throw_type_error(env, NULL, "Change is not a byte array");
      nb++;
    }
    off[i + 1] = nb;
  }
  if (ok) {
    am_doc_apply_changes_batch(n, docs, off, bufs ? bufs : (const uint8_t**)pats, lens ? lens : pl, want ? pats : NULL,
                               want ? pl : NULL, ci, codes, msgs);
    napi_create_array_with_length(env, n, &res);
    for (uint32_t i = 0; i < n; i++) {
      napi_value el;
      if (codes[i]) {
        el = err_obj(env, codes[i], msgs[i]);
      } else if (want) {
        el = call_result(env, pats[i], pl[i], &ci[i]);
      } else {
        napi_get_null(env, &el);
        am_free(ci[i].heads);
      }
      napi_set_element(env, res, i, el);
      am_free(pats[i]);
    }
  }
  for (uint32_t i = 0; i < n; i++) am_free(msgs[i]);
  free(docs); free(off); free(pats); free(pl); free(ci); free(codes); free(msgs); free(bufs); free(lens);
  return res;
}

// docSaveBatch([handle]) -> [Uint8Array | Error]; docPatchBatch([handle]) -> [{log, ...} | Error]
static napi_value save_or_patch_batch(napi_env env, napi_callback_info info, int patch) {
  ARGS(1)
  uint32_t n = 0;
  NAPI_OK(napi_get_array_length(env, argv[0], &n));
  am_doc** docs = (am_doc**)calloc(NA(n), sizeof(am_doc*));
  uint8_t** out = (uint8_t**)calloc(NA(n), sizeof(uint8_t*));
  size_t* ol = (size_t*)calloc(NA(n), sizeof(size_t));
  am_call_info* ci = (am_call_info*)calloc(NA(n), sizeof(am_call_info));
  uint32_t* codes = (uint32_t*)calloc(NA(n), sizeof(uint32_t));
  char** msgs = (char**)calloc(NA(n), sizeof(char*));
  napi_value res = NULL;
  if (handles_of(env, argv[0], n, docs)) {
    if (patch) am_doc_get_patch_batch(n, docs, out, ol, ci, codes, msgs);
    else am_doc_save_batch(n, docs, out, ol, codes, msgs);
    napi_create_array_with_length(env, n, &res);
    for (uint32_t i = 0; i < n; i++) {
      napi_value el = codes[i] ? err_obj(env, codes[i], msgs[i]) : patch ? call_result(env, out[i], ol[i], &ci[i])
                                                                          : new_u8(env, out[i], ol[i]);
      napi_set_element(env, res, i, el);
      am_free(out[i]);
      am_free(msgs[i]);
    }
  }
  free(docs); free(out); free(ol); free(ci); free(codes); free(msgs);
  return res;
}
static napi_value js_doc_save_batch(napi_env env, napi_callback_info info) { return save_or_patch_batch(env, info, 0); }
static napi_value js_doc_patch_batch(napi_env env, napi_callback_info info) { return save_or_patch_batch(env, info, 1); }

// syncReceiveBatch([handle], [stateBlob], [message]) -> [[stateBlob, {log, ...} | null] | Error]
static napi_value js_sync_receive_batch(napi_env env, napi_callback_info info) {
  ARGS(3)
  uint32_t n = 0;
  NAPI_OK(napi_get_array_length(env, argv[0], &n));
  am_doc** docs = (am_doc**)calloc(NA(n), sizeof(am_doc*));
  const uint8_t** st = (const uint8_t**)calloc(NA(n), sizeof(uint8_t*));
  size_t* sl = (size_t*)calloc(NA(n), sizeof(size_t));
  const uint8_t** m = (const uint8_t**)calloc(NA(n), sizeof(uint8_t*));
  size_t* ml = (size_t*)calloc(NA(n), sizeof(size_t));
  uint8_t** ost = (uint8_t**)calloc(NA(n), sizeof(uint8_t*));
  size_t* osl = (size_t*)calloc(NA(n), sizeof(size_t));
  uint8_t** pa = (uint8_t**)calloc(NA(n), sizeof(uint8_t*));
  size_t* pl = (size_t*)calloc(NA(n), sizeof(size_t));
  am_call_info* ci = (am_call_info*)calloc(NA(n), sizeof(am_call_info));
  uint32_t* codes = (uint32_t*)calloc(NA(n), sizeof(uint32_t));
  char** msgs = (char**)calloc(NA(n), sizeof(char*));
  napi_value res = NULL;
  int ok = handles_of(env, argv[0], n, docs);
  for (uint32_t i = 0; i < n && ok; i++) {
    napi_value a, b;
    ok = napi_get_element(env, argv[1], i, &a) == napi_ok && arg_bytes(env, a, &st[i], &sl[i]) &&
         napi_get_element(env, argv[2], i, &b) == napi_ok && arg_bytes(env, b, &m[i], &ml[i]);
  }
  if (ok) {
    am_sync_receive_batch(n, docs, st, sl, m, ml, ost, osl, pa, pl, ci, codes, msgs);
    napi_create_array_with_length(env, n, &res);
    for (uint32_t i = 0; i < n; i++) {
      napi_value el;
      if (codes[i]) {
        el = err_obj(env, codes[i], msgs[i]);
      } else {
        napi_value nul;
        napi_get_null(env, &nul);
        napi_create_array_with_length(env, 2, &el);
        napi_set_element(env, el, 0, new_u8(env, ost[i], osl[i]));
        napi_set_element(env, el, 1, pa[i] ? call_result(env, pa[i], pl[i], &ci[i]) : nul);
      }
      napi_set_element(env, res, i, el);
      am_free(ost[i]);
      am_free(pa[i]);
      am_free(ci[i].heads);
      am_free(msgs[i]);
    }
  }
  free(docs); free(st); free(sl); free(m); free(ml); free(ost); free(osl); free(pa); free(pl); free(ci); free(codes);
  free(msgs);
  return res;
}

static napi_value js_version(napi_env env, napi_callback_info info) {
  (void)info;
  napi_value v;
  NAPI_OK(napi_create_string_utf8(env, am_version(), NAPI_AUTO_LENGTH, &v));
  return v;
}

static napi_value init_module(napi_env env, napi_value exports) {
  napi_property_descriptor props[] = {
      {"docInit", 0, js_doc_init, 0, 0, 0, (napi_property_attributes)(napi_writable | napi_enumerable | napi_configurable), 0},
      {"docLoad", 0, js_doc_load, 0, 0, 0, (napi_property_attributes)(napi_writable | napi_enumerable | napi_configurable), 0},
      {"docClone", 0, js_doc_clone, 0, 0, 0, (napi_property_attributes)(napi_writable | napi_enumerable | napi_configurable), 0},
      {"docFree", 0, js_doc_free, 0, 0, 0, (napi_property_attributes)(napi_writable | napi_enumerable | napi_configurable), 0},
      {"docApplyChanges", 0, js_doc_apply, 0, 0, 0, (napi_property_attributes)(napi_writable | napi_enumerable | napi_configurable), 0},
      {"docSave", 0, js_doc_save, 0, 0, 0, (napi_property_attributes)(napi_writable | napi_enumerable | napi_configurable), 0},
      {"docHeads", 0, js_doc_heads, 0, 0, 0, (napi_property_attributes)(napi_writable | napi_enumerable | napi_configurable), 0},
      {"docChanges", 0, js_doc_changes, 0, 0, 0, (napi_property_attributes)(napi_writable | napi_enumerable | napi_configurable), 0},
      {"docCounts", 0, js_doc_counts, 0, 0, 0, (napi_property_attributes)(napi_writable | napi_enumerable | napi_configurable), 0},
      {"docPatch", 0, js_doc_patch, 0, 0, 0, (napi_property_attributes)(napi_writable | napi_enumerable | napi_configurable), 0},
      {"docQueued", 0, js_doc_queued, 0, 0, 0, (napi_property_attributes)(napi_writable | napi_enumerable | napi_configurable), 0},
      {"changeHashes", 0, js_change_hashes, 0, 0, 0, (napi_property_attributes)(napi_writable | napi_enumerable | napi_configurable), 0},
      {"docGetChanges", 0, js_doc_get_changes, 0, 0, 0, (napi_property_attributes)(napi_writable | napi_enumerable | napi_configurable), 0},
      {"docGetChangesAdded", 0, js_doc_get_changes_added, 0, 0, 0, (napi_property_attributes)(napi_writable | napi_enumerable | napi_configurable), 0},
      {"docChangeByHash", 0, js_doc_change_by_hash, 0, 0, 0, (napi_property_attributes)(napi_writable | napi_enumerable | napi_configurable), 0},
      {"docMissingDeps", 0, js_doc_missing_deps, 0, 0, 0, (napi_property_attributes)(napi_writable | napi_enumerable | napi_configurable), 0},
      {"docApplyLocal", 0, js_doc_apply_local, 0, 0, 0, (napi_property_attributes)(napi_writable | napi_enumerable | napi_configurable), 0},
      {"encodeChange", 0, js_encode_change, 0, 0, 0, (napi_property_attributes)(napi_writable | napi_enumerable | napi_configurable), 0},
      {"docLoadBatch", 0, js_doc_load_batch, 0, 0, 0, (napi_property_attributes)(napi_writable | napi_enumerable | napi_configurable), 0},
      {"docApplyBatch", 0, js_doc_apply_batch, 0, 0, 0, (napi_property_attributes)(napi_writable | napi_enumerable | napi_configurable), 0},
      {"docSaveBatch", 0, js_doc_save_batch, 0, 0, 0, (napi_property_attributes)(napi_writable | napi_enumerable | napi_configurable), 0},
      {"docPatchBatch", 0, js_doc_patch_batch, 0, 0, 0, (napi_property_attributes)(napi_writable | napi_enumerable | napi_configurable), 0},
      {"syncReceiveBatch", 0, js_sync_receive_batch, 0, 0, 0, (napi_property_attributes)(napi_writable | napi_enumerable | napi_configurable), 0},
      {"syncGenerate", 0, js_sync_generate, 0, 0, 0, (napi_property_attributes)(napi_writable | napi_enumerable | napi_configurable), 0},
      {"syncReceive", 0, js_sync_receive, 0, 0, 0, (napi_property_attributes)(napi_writable | napi_enumerable | napi_configurable), 0},
      {"syncEncodeMessage", 0, js_sync_encode_message, 0, 0, 0, (napi_property_attributes)(napi_writable | napi_enumerable | napi_configurable), 0},
      {"syncDecodeMessage", 0, js_sync_decode_message, 0, 0, 0, (napi_property_attributes)(napi_writable | napi_enumerable | napi_configurable), 0},
      {"syncEncodeState", 0, js_sync_encode_state, 0, 0, 0, (napi_property_attributes)(napi_writable | napi_enumerable | napi_configurable), 0},
      {"syncDecodeState", 0, js_sync_decode_state, 0, 0, 0, (napi_property_attributes)(napi_writable | napi_enumerable | napi_configurable), 0},
      {"version", 0, js_version, 0, 0, 0, (napi_property_attributes)(napi_writable | napi_enumerable | napi_configurable), 0},
  };
  if (napi_define_properties(env, exports, sizeof(props) / sizeof(props[0]), props) != napi_ok) return NULL;
  return exports;
}

NAPI_MODULE(NODE_GYP_MODULE_NAME, init_module)
