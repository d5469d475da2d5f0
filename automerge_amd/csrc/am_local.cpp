// am_local.cpp -- local changes: encodeChange of a frontend change request
// and Backend.applyLocalChange over the engine document. Host code.
//
//   am_encode_change          <- encodeChange(changeObj)            columnar.js:710-739
//                                 parseAllOpIds (:133-174), expandMultiOps (:446-481),
//                                 encodeOps (:370-436), encodeValue (:259-298)
//   am_doc_apply_local_change <- applyLocalChange(backend, change)   backend.js:54-91
//
// The request arrives as JSON (am_json.h conventions). Encoding is host byte work on one small
// change; applying it runs the GPU merge + patch path of am_doc_apply_changes_patch. Every error
// the reference raises on the way is raised here with its class and text, in the reference's order
// (parse of op ids, then the header fields, then the op columns).
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <map>
#include <string>
#include <vector>

#include "../../include/automerge_amd.h"
#include "am_change_enc.h"
#include "am_json.h"

using amjson::JV;
using amjson::js_num;
using amjson::js_str;
using amjson::js_stringify;

namespace {

struct JsErr {
  bool type_error;
  std::string msg;
  uint32_t code = AM_E_LOCAL;
};
[[noreturn]] void range_error(const std::string& m) { throw JsErr{false, m}; }
[[noreturn]] void type_error(const std::string& m) { throw JsErr{true, m}; }

const double kMaxSafe = 9007199254740991.0;

// hexStringToBytes (encoding.js:22-34)
std::string hex_bytes(const JV& v) {
  if (v.k != amjson::STR) type_error("value is not a string");
  const std::string& h = v.s;
  if (h.size() % 2) range_error("value is not hexadecimal");
  std::string out;
  for (size_t i = 0; i < h.size(); i += 2) {
    int b = 0;
    for (int k = 0; k < 2; k++) {
      const char c = h[i + k];
      b <<= 4;
      if (c >= '0' && c <= '9') b |= c - '0';
      else if (c >= 'a' && c <= 'f') b |= c - 'a' + 10;
      else range_error("value is not hexadecimal");
    }
    out += (char)b;
  }
  return out;
}

// appendUint53 / appendInt53 (encoding.js:137-160)
uint64_t uint53(const JV& v) {
  if (!v.is_int()) range_error("value is not an integer");
  if (v.n < 0 || v.n > kMaxSafe) range_error("number out of range");
  return (uint64_t)v.n;
}
// an op id counter as the column encoders take it (appendUint53 at flush)
int64_t ctr53(double c) {
  if (c > kMaxSafe) range_error("number out of range");
  return (int64_t)c;
}
int64_t int53(const JV& v) {
  if (!v.is_int()) range_error("value is not an integer");
  if (v.n < -kMaxSafe || v.n > kMaxSafe) range_error("number out of range");
  return (int64_t)v.n;
}

// parseOpId (src/common.js:22-28) -> {counter, actorId}; actorNum assigned later
struct PId {
  double counter = 0;
  std::string actor;
  int num = -1;  // actorIdToActorNum: -1 when actorId is empty (the object keeps no actorNum)
};
bool line_term(const std::string& s) {
  for (size_t i = 0; i < s.size(); i++) {
    const unsigned char c = s[i];
    if (c == '\n' || c == '\r') return true;
    if (c == 0xe2 && i + 2 < s.size() && (unsigned char)s[i + 1] == 0x80 &&
        ((unsigned char)s[i + 2] == 0xa8 || (unsigned char)s[i + 2] == 0xa9))
      return true;  // U+2028 / U+2029
  }
  return false;
}
PId parse_opid(const JV& v) {
  const std::string s = v.truthy() ? js_str(v) : "";
  size_t i = 0;
  while (i < s.size() && s[i] >= '0' && s[i] <= '9') i++;
  if (i == 0 || i >= s.size() || s[i] != '@' || line_term(s.substr(i + 1))) range_error("Not a valid opId: " + js_str(v));
  PId p;
  p.counter = std::strtod(s.substr(0, i).c_str(), nullptr);
  p.actor = s.substr(i + 1);
  return p;
}
std::string opid_json(const PId& p) {  // JSON.stringify of the parsed form
  std::string r = "{\"counter\":" + js_num(p.counter);
  if (p.num >= 0) r += ",\"actorNum\":" + std::to_string(p.num);
  std::string q;
  amjson::js_quote(p.actor, q);
  return r + ",\"actorId\":" + q + "}";
}

// one op after expandMultiOps + parseAllOpIds
struct LOp {
  JV src;  // the (copied) request op: action, key, insert, value, datatype, ...
  bool obj_root = true;
  PId obj;
  enum { E_NONE, E_HEAD, E_ID, E_OTHER } elem_kind = E_NONE;
  PId elem;
  JV elem_raw;
  bool has_child = false;
  PId child;
  std::vector<PId> pred;
};

// JSON.stringify(op) of a parsed op (the "Unexpected operation key" message)
std::string op_json(const LOp& op, double id_ctr, int id_num, const std::string& id_actor) {
  std::string r = "{";
  bool first = true, saw_id = false;
  auto key = [&](const std::string& k) {
    if (!first) r += ",";
    first = false;
    amjson::js_quote(k, r);
    r += ":";
  };
  for (auto& kv : op.src.o) {
    const std::string& k = kv.first;
    if (k == "obj" && !op.obj_root) { key(k); r += opid_json(op.obj); continue; }
    if (k == "elemId" && op.elem_kind == LOp::E_ID) { key(k); r += opid_json(op.elem); continue; }
    if (k == "child" && op.has_child) { key(k); r += opid_json(op.child); continue; }
    if (k == "pred" && kv.second.k == amjson::ARR) {
      key(k);
      r += "[";
      for (size_t i = 0; i < op.pred.size(); i++) r += (i ? "," : "") + opid_json(op.pred[i]);
      r += "]";
      continue;
    }
    if (k == "id") saw_id = true;
    if (kv.second.k == amjson::UNDEF) continue;
    key(k);
    if (k == "id") {
      PId id;
      id.counter = id_ctr;
      id.actor = id_actor;
      id.num = id_num;
      r += opid_json(id);
    } else {
      r += js_stringify(kv.second);
    }
  }
  if (!saw_id) {
    PId id;
    id.counter = id_ctr;
    id.actor = id_actor;
    id.num = id_num;
    key("id");
    r += opid_json(id);
  }
  return r + "}";
}

JV jstr(const std::string& s) {
  JV v;
  v.k = amjson::STR;
  v.s = s;
  return v;
}

// validDatatype (columnar.js:438-444)
bool valid_datatype(const JV& value, const JV& datatype) {
  if (datatype.k == amjson::UNDEF) return value.k == amjson::STR || value.k == amjson::BOOL || value.k == amjson::NUL;
  return value.k == amjson::NUM;
}

// expandMultiOps (columnar.js:446-481)
std::vector<JV> expand_multi_ops(const JV& ops, const JV& start_op, const JV& actor) {
  if (ops.k != amjson::ARR) type_error("ops is not iterable");
  std::vector<JV> out;
  double op_num = start_op.k == amjson::NUM ? start_op.n : NAN;
  for (const JV& op : ops.a) {
    const JV& action = op["action"];
    const bool is_set = action.k == amjson::STR && action.s == "set";
    const bool is_del = action.k == amjson::STR && action.s == "del";
    if (is_set && op["values"].truthy() && op["insert"].truthy()) {
      const JV& pred = op["pred"];
      if (pred.k != amjson::ARR) type_error("Cannot read property 'length' of " + js_str(pred));
      if (!pred.a.empty()) range_error("multi-insert pred must be empty");
      JV last = op["elemId"];
      const JV& datatype = op["datatype"];
      const JV& values = op["values"];
      if (values.k != amjson::ARR) type_error("op.values is not iterable");
      for (const JV& value : values.a) {
        if (!valid_datatype(value, datatype))
          range_error("Decode failed: bad value/datatype association (" + js_str(value) + "," + js_str(datatype) + ")");
        JV e;
        e.k = amjson::OBJ;
        e.o.emplace_back("action", jstr("set"));
        e.o.emplace_back("obj", op["obj"]);
        e.o.emplace_back("elemId", last);
        e.o.emplace_back("datatype", datatype);
        e.o.emplace_back("value", value);
        JV empty;
        empty.k = amjson::ARR;
        e.o.emplace_back("pred", empty);
        JV t;
        t.k = amjson::BOOL;
        t.b = true;
        e.o.emplace_back("insert", t);
        out.push_back(std::move(e));
        last = jstr(js_num(op_num) + "@" + js_str(actor));
        op_num += 1;
      }
    } else if (is_del && op["multiOp"].k == amjson::NUM && op["multiOp"].n > 1) {
      const JV& pred = op["pred"];
      if (pred.k != amjson::ARR) type_error("Cannot read property 'length' of " + js_str(pred));
      if (pred.a.size() != 1) range_error("multiOp deletion must have exactly one pred");
      const PId se = parse_opid(op["elemId"]), sp = parse_opid(pred.a[0]);
      for (double i = 0; i < op["multiOp"].n; i++) {
        JV e;
        e.k = amjson::OBJ;
        e.o.emplace_back("action", jstr("del"));
        e.o.emplace_back("obj", op["obj"]);
        e.o.emplace_back("elemId", jstr(js_num(se.counter + i) + "@" + se.actor));
        JV pl;
        pl.k = amjson::ARR;
        pl.a.push_back(jstr(js_num(sp.counter + i) + "@" + sp.actor));
        e.o.emplace_back("pred", pl);
        out.push_back(std::move(e));
        op_num += 1;
      }
    } else {
      out.push_back(op);
      op_num += 1;
    }
  }
  return out;
}

// encodeValue (columnar.js:259-298) + getNumberTypeAndValue (:228-253)
void encode_value(const JV& op, int64_t& val_len, std::string& raw) {
  const JV& action = op["action"];
  const JV& value = op["value"];
  const JV& datatype = op["datatype"];
  const bool set_or_inc = action.k == amjson::STR && (action.s == "set" || action.s == "inc");
  raw.clear();
  if (!set_or_inc || value.k == amjson::NUL) { val_len = 0; return; }
  if (value.k == amjson::BOOL) { val_len = value.b ? 2 : 1; return; }
  if (value.k == amjson::STR) { raw = value.s; val_len = (int64_t)raw.size() << 4 | 6; return; }
  if (value.k == amjson::BYTES) { raw = value.s; val_len = (int64_t)raw.size() << 4 | 7; return; }
  if (value.k == amjson::NUM) {
    const std::string dt = datatype.k == amjson::STR ? datatype.s : std::string("\x01");
    Bytes b;
    int tag;
    auto f64 = [&]() {
      uint8_t x[8];
      memcpy(x, &value.n, 8);
      b.assign(x, x + 8);
      return 5;
    };
    if (dt == "counter") { ps(b, int53(value)); tag = 8; }
    else if (dt == "timestamp") { ps(b, int53(value)); tag = 9; }
    else if (dt == "uint") { pu(b, uint53(value)); tag = 3; }
    else if (dt == "int") { ps(b, int53(value)); tag = 4; }
    else if (dt == "float64") tag = f64();
    else if (value.is_int() && std::fabs(value.n) <= kMaxSafe) { ps(b, (int64_t)value.n); tag = 4; }
    else tag = f64();
    raw.assign(b.begin(), b.end());
    val_len = (int64_t)raw.size() << 4 | tag;
    return;
  }
  if (datatype.truthy()) range_error("Unknown datatype " + js_str(datatype) + " for value " + js_str(value));
  range_error("Unsupported value in operation: " + js_str(value));
}

const char* kActions[] = {"makeMap", "set", "makeList", "del", "makeText", "inc", "makeTable", "link"};

struct Encoded {
  Bytes bytes;       // after deflateChange
  uint8_t hash[32];  // of the uncompressed chunk
};

// encodeChange (columnar.js:710-739)
Encoded encode_change(const JV& change) {
  if (change.k != amjson::OBJ) type_error("change request is not an object");
  const JV& actor = change["actor"];
  const JV& start_op = change["startOp"];
  // parseAllOpIds([change], true)
  std::vector<JV> ops = expand_multi_ops(change["ops"], start_op, actor);
  std::map<std::string, bool> actor_set;  // Object.keys(actors).sort()
  actor_set[js_str(actor)] = true;
  std::vector<LOp> lops;
  for (JV& src : ops) {
    LOp op;
    const JV& obj = src["obj"];
    if (!(obj.k == amjson::STR && obj.s == "_root")) { op.obj_root = false; op.obj = parse_opid(obj); }
    const JV& elem = src["elemId"];
    op.elem_raw = elem;
    if (elem.truthy() && !(elem.k == amjson::STR && elem.s == "_head")) { op.elem_kind = LOp::E_ID; op.elem = parse_opid(elem); }
    else if (elem.k == amjson::STR && elem.s == "_head") op.elem_kind = LOp::E_HEAD;
    else if (elem.truthy()) op.elem_kind = LOp::E_OTHER;
    if (src["child"].truthy()) { op.has_child = true; op.child = parse_opid(src["child"]); }
    const JV& pred = src["pred"];
    if (pred.truthy()) {
      if (pred.k != amjson::ARR) type_error("op.pred.map is not a function");
      for (const JV& p : pred.a) op.pred.push_back(parse_opid(p));
    }
    if (!op.obj_root && !op.obj.actor.empty()) actor_set[op.obj.actor] = true;
    if (op.elem_kind == LOp::E_ID && !op.elem.actor.empty()) actor_set[op.elem.actor] = true;
    if (op.has_child && !op.child.actor.empty()) actor_set[op.child.actor] = true;
    if (pred.k != amjson::ARR) type_error("op.pred is not iterable");
    for (const PId& p : op.pred) actor_set[p.actor] = true;
    op.src = std::move(src);
    lops.push_back(std::move(op));
  }
  const std::string author = js_str(actor);
  std::vector<std::string> actor_ids{author};
  for (auto& kv : actor_set)
    if (kv.first != author) actor_ids.push_back(kv.first);
  auto num_of = [&](PId& p) {
    if (p.actor.empty()) return;
    p.num = (int)(std::find(actor_ids.begin(), actor_ids.end(), p.actor) - actor_ids.begin());
  };
  for (LOp& op : lops) {
    if (!op.obj_root) num_of(op.obj);
    if (op.elem_kind == LOp::E_ID) num_of(op.elem);
    if (op.has_child) num_of(op.child);
    for (PId& p : op.pred) num_of(p);
  }

  // header (encodeContainer callback, in the reference's order)
  const JV& deps = change["deps"];
  if (deps.k != amjson::ARR) type_error("deps is not an array");
  std::vector<JV> sorted = deps.a;
  std::stable_sort(sorted.begin(), sorted.end(), [](const JV& a, const JV& b) {  // Array.prototype.sort()
    if (a.k == amjson::UNDEF || b.k == amjson::UNDEF) return a.k != amjson::UNDEF && b.k == amjson::UNDEF;
    return js_str(a) < js_str(b);
  });
  std::vector<std::vector<uint8_t>> dep_bytes;
  for (const JV& h : sorted) {
    const std::string b = hex_bytes(h);
    dep_bytes.emplace_back(b.begin(), b.end());
  }
  hex_bytes(actor);
  HChange c;
  c.actor = 0;
  c.seq = (int64_t)uint53(change["seq"]);
  const int64_t start = (int64_t)uint53(start_op);
  c.time = int53(change["time"]);
  const JV& message = change["message"];
  if (message.truthy() && message.k != amjson::STR) type_error("value is not a string");
  c.message = message.truthy() ? message.s : std::string();
  std::vector<std::string> actor_hex;
  for (size_t i = 0; i < actor_ids.size(); i++) {
    const std::string b = hex_bytes(jstr(actor_ids[i]));
    actor_hex.push_back(actor_ids[i]);
    (void)b;
  }

  // encodeOps (columnar.js:370-436)
  std::vector<HOp> pool;
  for (size_t i = 0; i < lops.size(); i++) {
    const LOp& op = lops[i];
    const JV& src = op.src;
    HOp h{};
    h.id_ctr = start + (int64_t)i;
    h.id_actor = 0;
    if (op.obj_root) { h.obj_actor = -1; }
    else if (op.obj.num >= 0 && op.obj.counter > 0) { h.obj_actor = op.obj.num; h.obj_ctr = ctr53(op.obj.counter); }
    else range_error("Unexpected objectId reference: " + opid_json(op.obj));
    const JV& key = src["key"];
    if (key.truthy()) {
      if (key.k != amjson::STR) type_error("value is not a string");
      h.has_key = true;
      h.key = key.s;
      if (op.elem_kind == LOp::E_ID && op.elem.num >= 0) { h.key_elem_actor = true; h.elem_actor = op.elem.num; }
    } else if (op.elem_kind == LOp::E_HEAD && src["insert"].truthy()) {
      h.elem_actor = -1;
      h.elem_ctr = 0;
    } else if (op.elem_kind == LOp::E_ID && op.elem.num >= 0 && op.elem.counter > 0) {
      h.elem_actor = op.elem.num;
      h.elem_ctr = ctr53(op.elem.counter);
    } else {
      range_error("Unexpected operation key: " + op_json(op, (double)h.id_ctr, 0, author));
    }
    h.insert = src["insert"].truthy();
    const JV& action = src["action"];
    int64_t code = -1;
    if (action.k == amjson::STR)
      for (int a = 0; a < 8; a++)
        if (action.s == kActions[a]) code = a;
    if (code < 0) {
      if (action.k == amjson::NUM) code = (int64_t)uint53(action);
      else range_error("Unexpected operation action: " + js_str(action));
    }
    h.action = code;
    encode_value(src, h.val_len, h.val_raw);
    if (op.has_child && op.child.counter != 0) {
      if (op.child.num < 0) range_error("value is not an integer");
      h.child_actor = op.child.num;
      h.child_ctr = ctr53(op.child.counter);
    }
    for (const PId& p : op.pred) {
      if (p.num < 0) range_error("value is not an integer");
      h.pred.push_back({ctr53(p.counter), p.num});
    }
    pool.push_back(std::move(h));
    c.ops.push_back((int)pool.size() - 1);
  }
  const JV& extra = change["extraBytes"];
  if (extra.truthy()) {
    if (extra.k != amjson::BYTES) type_error("Not a byte array: " + js_str(extra));
    c.extra = extra.s;
  }
  Encoded out;
  Bytes chunk = encode(c, pool, actor_hex, dep_bytes, start, out.hash);
  const JV& given = change["hash"];
  if (given.truthy()) {
    static const char* H = "0123456789abcdef";
    std::string hx;
    for (int i = 0; i < 32; i++) { hx += H[out.hash[i] >> 4]; hx += H[out.hash[i] & 15]; }
    if (given.k != amjson::STR || given.s != hx)
      range_error("Change hash does not match encoding: " + js_str(given) + " != " + hx);
  }
  out.bytes = deflate_change(std::move(chunk));
  return out;
}

void to_err(const JsErr& e, am_error* err) {
  if (!err) return;
  err->code = e.code;
  err->is_type_error = e.type_error ? 1 : 0;
  snprintf(err->message, sizeof(err->message), "%s", e.msg.c_str());
}

bool parse_request(const char* json, size_t len, JV& v, am_error* err) {
  if (!amjson::parse(json, len, v)) {
    to_err(JsErr{true, "automerge_amd: the change request is not valid JSON"}, err);
    return false;
  }
  return true;
}

uint8_t* dup(const void* p, size_t n) {
  uint8_t* q = (uint8_t*)malloc(n ? n : 1);
  if (q && n) memcpy(q, p, n);
  return q;
}

std::string hex32(const uint8_t* h) {
  static const char* H = "0123456789abcdef";
  std::string s;
  for (int i = 0; i < 32; i++) { s += H[h[i] >> 4]; s += H[h[i] & 15]; }
  return s;
}

}  // namespace

extern "C" int am_encode_change(const char* json, size_t len, uint8_t** out, size_t* out_len, uint8_t* hash32,
                                am_error* err) {
  JV req;
  if (!parse_request(json, len, req, err)) return 1;
  try {
    Encoded e = encode_change(req);
    *out = dup(e.bytes.data(), e.bytes.size());
    *out_len = e.bytes.size();
    if (hash32) memcpy(hash32, e.hash, 32);
  } catch (const JsErr& e) {
    to_err(e, err);
    return 1;
  } catch (const std::bad_alloc&) {
    to_err(JsErr{false, "automerge_amd: out of host memory", AM_U_CAPACITY}, err);
    return 1;
  }
  if (err) err->code = 0;
  return 0;
}

// applyLocalChange (backend.js:54-91). Returns 0, 1 (error, document unchanged) or 2 (error raised
// after the change was applied: the caller's backend is updated and its old handle frozen, as in
// the reference where hashByActor throws after applyChanges).
extern "C" int am_doc_apply_local_change(am_doc* d, const char* json, size_t len, uint8_t** change_out,
                                         size_t* change_len, uint8_t** patch_out, size_t* patch_len,
                                         uint8_t* new_hash32, uint8_t* last_hash32, int* has_last, am_error* err) {
  JV req;
  if (!parse_request(json, len, req, err)) return 1;
  *has_last = 0;
  try {
    if (req.k != amjson::OBJ) type_error("Cannot read property 'seq' of " + js_str(req));
    const JV& seq = req["seq"];
    const std::string actor = js_str(req["actor"]);
    // if (change.seq <= state.clock[change.actor] || 0): an actor without changes has no clock entry
    const int64_t clock = am_doc_clock(d, actor.c_str());
    if (clock < 0) range_error("automerge_amd: the document history could not be reconstructed");
    if (clock > 0 && seq.k == amjson::NUM && seq.n <= (double)clock) range_error("Change request has already been applied");
    if (seq.k == amjson::NUM && seq.n > 1) {
      // the local actor's previous change joins deps (hashByActor, backend.js:34-45)
      uint8_t last[32];
      if (!seq.is_int() || am_doc_actor_hash(d, actor.c_str(), (int64_t)seq.n - 1, last))
        range_error("Unknown change: actorId = " + actor + ", seq = " + js_num(seq.n - 1));
      const JV& deps = req["deps"];
      if (deps.k != amjson::ARR) type_error("change.deps is not iterable");
      std::vector<std::string> keys{hex32(last)};
      for (const JV& h : deps.a) {
        const std::string k = js_str(h);
        if (std::find(keys.begin(), keys.end(), k) == keys.end()) keys.push_back(k);
      }
      std::sort(keys.begin(), keys.end());
      JV nd;
      nd.k = amjson::ARR;
      for (auto& k : keys) nd.a.push_back(jstr(k));
      for (auto& kv : req.o)
        if (kv.first == "deps") kv.second = nd;
      memcpy(last_hash32, last, 32);
      *has_last = 1;
    }
    Encoded e = encode_change(req);
    const uint8_t* bufs[1] = {e.bytes.data()};
    const size_t lens[1] = {e.bytes.size()};
    uint8_t* patch = nullptr;
    size_t plen = 0;
    if (am_doc_apply_changes_patch(d, bufs, lens, 1, &patch, &plen, err)) return 1;
    *change_out = dup(e.bytes.data(), e.bytes.size());
    *change_len = e.bytes.size();
    *patch_out = patch;
    *patch_len = plen;
    // the patch omits the hash of the change just made (backend.js:87-89)
    if (am_doc_actor_hash(d, actor.c_str(), (int64_t)seq.n, new_hash32)) {
      free(*change_out);
      free(patch);
      to_err(JsErr{false, "Unknown change: actorId = " + actor + ", seq = " + js_num(seq.n)}, err);
      return 2;
    }
  } catch (const JsErr& e) {
    to_err(e, err);
    return 1;
  } catch (const std::bad_alloc&) {
    to_err(JsErr{false, "automerge_amd: out of host memory", AM_U_CAPACITY}, err);
    return 1;
  }
  if (err) err->code = 0;
  return 0;
}
