// Golden-vector generator. Runs the reference JS backend (read-only at /root/reference, with the
// offline shims in ./node_modules standing in for pako/fast-sha256/uuid) and writes small JSON
// fixtures into tests/golden/. Only this container can run it; the fixtures travel, the reference
// does not. Usage:
//   NODE_PATH=tests/golden/gen/node_modules node tests/golden/gen/make_fixtures.js [refRoot]
// Everything is seeded, so re-running reproduces the committed files byte for byte.
'use strict'
const fs = require('fs')
const path = require('path')
const REF = process.env.AM_REF || (require.main === module && process.argv[2]) || '/root/reference'
const OUT = path.join(__dirname, '..')

const Automerge = require(path.join(REF, 'src/automerge'))
const Backend = require(path.join(REF, 'backend'))
const enc = require(path.join(REF, 'backend/encoding'))
const col = require(path.join(REF, 'backend/columnar'))
const sync = require(path.join(REF, 'backend/sync'))

const hex = u8 => Buffer.from(u8).toString('hex')
const unhex = h => new Uint8Array(Buffer.from(h, 'hex'))

// Seeded LCG, same constants as the workload generators (SURVEY.md §8(d)).
function lcg(seed) {
  let s = seed >>> 0
  const next = () => { s = (Math.imul(s, 1664525) + 1013904223) >>> 0; return s }
  next.int = n => next() % n
  next.pick = arr => arr[next() % arr.length]
  return next
}

function errOf(fn) {
  try { fn(); return null } catch (e) { return {name: e.name, message: e.message} }
}

// ------------------------------------------------------------------------------------------------
// 1. Codec vectors: LEB128, RLE, delta, boolean (encoding.js)
// ------------------------------------------------------------------------------------------------
function codecVectors() {
  const r = lcg(12345)
  const out = {leb: [], leb_decode: [], rle: [], delta: [], bool: [], decode_errors: []}
  const u32 = [0, 1, 0x7f, 0x80, 0x3fff, 0x4000, 0x1fffff, 0x200000, 0xfffffff, 0x10000000, 0xffffffff]
  const i32 = [0, 1, -1, 0x3f, 0x40, -0x40, -0x41, 0x1fff, 0x2000, -0x2000, -0x2001, 0x7fffffff, -0x80000000]
  const u53 = u32.concat([0x100000000, 2 ** 35 - 1, 2 ** 35, 2 ** 42, 2 ** 49 - 1, 2 ** 49, Number.MAX_SAFE_INTEGER])
  const i53 = i32.concat([0x80000000, -0x80000001, 2 ** 34, -(2 ** 34), 2 ** 41 - 1, -(2 ** 41), 2 ** 48, -(2 ** 48),
    Number.MAX_SAFE_INTEGER, Number.MIN_SAFE_INTEGER])
  for (let i = 0; i < 40; i++) {
    u53.push(r() * 0x200000 + r() % 0x200000 * 0) ; i53.push((r() - 0x80000000) * ((r() % 4) + 1))
  }
  const add = (fn, v) => {
    const e = new enc.Encoder()
    e[fn](v)
    out.leb.push({fn, value: v, bytes: hex(e.buffer)})
  }
  for (const v of u32) add('appendUint32', v)
  for (const v of i32) add('appendInt32', v)
  for (const v of u53) if (Number.isSafeInteger(v) && v >= 0) add('appendUint53', v)
  for (const v of i53) if (Number.isSafeInteger(v)) add('appendInt53', v)
  // 64-bit halves
  const halves = [[0, 0], [0, 0xffffffff], [1, 0], [0x7fffffff, 0xffffffff], [0xffffffff, 0xffffffff], [0x12345, 0x6789abcd]]
  for (const [h, l] of halves) {
    let e = new enc.Encoder(); e.appendUint64(h, l); out.leb.push({fn: 'appendUint64', high32: h, low32: l, bytes: hex(e.buffer)})
  }
  const shalves = [[0, 0], [-1, 0xffffffff], [-1, 0], [0x7fffffff, 0xffffffff], [-0x80000000, 0], [-2, 0x12345678]]
  for (const [h, l] of shalves) {
    let e = new enc.Encoder(); e.appendInt64(h, l); out.leb.push({fn: 'appendInt64', high32: h, low32: l, bytes: hex(e.buffer)})
  }
  // Decoding, including malformed/out-of-range inputs (error messages are part of the contract)
  const decBytes = [
    '00', '7f', '8001', 'ff7f', 'ffffffff0f', 'ffffffff1f', 'ffffffff7f', 'ffffffffff00', '80', 'ff', '',
    '808080807f', '8080808078', '8080808008', 'ffffffff07', 'ffffffff08', 'ffffffff77', 'ffffffff78',
    'ffffffffffffff0f', 'ffffffffffffff1f', 'ffffffffffffffff01', 'ffffffffffffffffff01', 'ffffffffffffffffff02',
    'ffffffffffffffffff00', 'ffffffffffffffffff7f', '80808080808080808001', '8080808080808080807f',
    '80808080808080808040', 'ffffffffffffff7f', '808080808080807f', '80808080808080808080', '8080808080808040',
    'feffffffffffff0f', 'ffffffffffffff10', '8180808080808070', '8180808080808070', 'c0bbb8'
  ]
  for (const b of decBytes) {
    for (const fn of ['readUint32', 'readInt32', 'readUint53', 'readInt53', 'readUint64', 'readInt64']) {
      const d = new enc.Decoder(unhex(b))
      let value = null, error = null
      try { value = d[fn](); if (typeof value === 'object') value = [value.high32, value.low32] } catch (e) { error = e.message }
      out.leb_decode.push({fn, bytes: b, value, error, offset: d.offset})
    }
  }

  // RLE sequences
  const strs = ['', 'a', 'b', 'abc', 'é', '😀', '￿', 'x'.repeat(40), 'key', 'k1']
  const genSeq = (type, n) => {
    const vals = []
    const mode = r() % 4
    for (let i = 0; i < n; i++) {
      const k = r() % 10
      let v
      if (k < 2) v = null
      else if (type === 'utf8') v = strs[r() % (mode === 0 ? 3 : strs.length)]
      else if (type === 'uint') v = mode === 0 ? r() % 3 : (mode === 1 ? r() : r() % 200)
      else v = mode === 0 ? (r() % 3) - 1 : (mode === 1 ? (r() - 0x80000000) * 97 : (r() % 200) - 100)
      if (mode === 2 && i > 0 && r() % 3 === 0) v = vals[i - 1]
      vals.push(v)
      if (r() % 5 === 0) { const rep = r() % 6; for (let j = 0; j < rep && vals.length < n; j++) { vals.push(v); i++ } }
    }
    return vals
  }
  const fixed = {
    uint: [[], [null], [null, null, null], [1], [1, 1], [1, 2], [1, 1, 2], [1, 2, 2], [null, 1], [1, null], [1, 2, 3, 3, null, null, 4]],
    int: [[], [-1], [0, 0, 0], [-1, 1, -1], [3, 3, -3, -3]],
    utf8: [[], ['a'], ['a', 'a'], ['a', 'b', null, 'b'], ['😀', '�', '😀']]
  }
  for (const type of ['uint', 'int', 'utf8']) {
    const seqs = fixed[type].slice()
    for (let i = 0; i < 60; i++) seqs.push(genSeq(type, 1 + r() % 40))
    for (const values of seqs) {
      const e = new enc.RLEEncoder(type)
      for (const v of values) e.appendValue(v)
      out.rle.push({type, values, bytes: hex(e.buffer)})
    }
  }
  const dseqs = [[], [null], [1, 2, 3, 4], [5, null, 6, 7, null], [10, 5, 0, -5], [1, 1, 1]]
  for (let i = 0; i < 60; i++) {
    const n = 1 + r() % 40, vals = []
    let cur = r() % 100
    for (let j = 0; j < n; j++) {
      const k = r() % 10
      if (k === 0) vals.push(null); else { cur += (k < 6 ? 1 : (r() % 21) - 10); vals.push(cur) }
    }
    dseqs.push(vals)
  }
  for (const values of dseqs) {
    const e = new enc.DeltaEncoder()
    for (const v of values) e.appendValue(v)
    out.delta.push({values, bytes: hex(e.buffer)})
  }
  const bseqs = [[], [false], [true], [false, false, true], [true, true, false, true]]
  for (let i = 0; i < 40; i++) {
    const n = 1 + r() % 50, vals = []
    let cur = r() % 2 === 0
    for (let j = 0; j < n; j++) { if (r() % 3 === 0) cur = !cur; vals.push(cur) }
    bseqs.push(vals)
  }
  for (const values of bseqs) {
    const e = new enc.BooleanEncoder()
    for (const v of values) e.appendValue(v)
    out.bool.push({values, bytes: hex(e.buffer)})
  }
  // Decoder canonical-form errors (encoding.js:826,867-886,1176-1178)
  const bad = [
    ['uint', '0201'], ['uint', '02010201'], ['uint', '7f017f02'], ['uint', '0001' + '0002'], ['uint', '0000'],
    ['uint', '7e0101'], ['uint', '7f01' + '0201'], ['uint', '0201' + '7f01'], ['int', '03017f02'], ['utf8', '7f0161'],
    ['utf8', '027f'], ['uint', '7e0102'], ['uint', '0102'], ['uint', '02'], ['uint', '7e01'], ['uint', '8080'],
    ['delta', '02017f02'], ['delta', '0201'], ['bool', '0000'], ['bool', '0100'], ['bool', '000100'], ['bool', '01']
  ]
  for (const [type, b] of bad) {
    let d
    if (type === 'delta') d = new enc.DeltaDecoder(unhex(b))
    else if (type === 'bool') d = new enc.BooleanDecoder(unhex(b))
    else d = new enc.RLEDecoder(type, unhex(b))
    const values = []
    let error = null
    try { for (let i = 0; i < 64 && !d.done; i++) values.push(d.readValue()) } catch (e) { error = e.message }
    out.decode_errors.push({type, bytes: b, values, error})
  }
  return out
}

// ------------------------------------------------------------------------------------------------
// 2. Random document histories, built with the reference frontend (fixed actors, time 0)
// ------------------------------------------------------------------------------------------------
const KEYS = ['a', 'b', 'c', 'title', 'k1', 'k2', 'zz', 'é', '😀', '￠', '�', 'A', 'x y', 'k10', '퟿']
function randomActor(r) {
  const len = 1 + r() % 16
  let s = ''
  for (let i = 0; i < len; i++) s += (r() % 256).toString(16).padStart(2, '0')
  return s
}

function randomValue(r) {
  switch (r() % 11) {
    case 0: return null
    case 1: return true
    case 2: return false
    case 3: return r() % 1000
    case 4: return -(r() % 100000)
    case 5: return (r() % 1000) / 8 + 0.5
    case 6: return 'str' + (r() % 50)
    case 7: return new Automerge.Uint(r() % 300)
    case 8: return new Automerge.Int(r() % 300 - 150)
    case 9: return new Automerge.Float64(r() % 7)
    default: return new Date(1600000000000 + r() % 100000)
  }
}

// One random edit session against `doc` (a frontend proxy); keeps ops small.
function randomEdit(r, doc) {
  const nOps = 1 + r() % 4
  for (let i = 0; i < nOps; i++) {
    const kind = r() % 12
    const key = KEYS[r() % KEYS.length]
    if (kind <= 2) {
      doc[key] = randomValue(r)
    } else if (kind === 3) {
      if (doc[key] !== undefined) delete doc[key]
    } else if (kind === 4) {
      if (!doc.list) doc.list = []
      const n = 1 + r() % 3, at = r() % (doc.list.length + 1)
      const vals = []
      for (let j = 0; j < n; j++) vals.push(r() % 2 ? r() % 100 : 'v' + r() % 10)
      doc.list.insertAt(at, ...vals)
    } else if (kind === 5) {
      if (doc.list && doc.list.length > 0) {
        const at = r() % doc.list.length
        doc.list.deleteAt(at, 1 + r() % Math.min(3, doc.list.length - at))
      }
    } else if (kind === 6) {
      if (doc.list && doc.list.length > 0) doc.list[r() % doc.list.length] = randomValue(r)
    } else if (kind === 7) {
      if (!doc.text) doc.text = new Automerge.Text()
      const at = r() % (doc.text.length + 1)
      const n = 1 + r() % 5
      const chars = []
      for (let j = 0; j < n; j++) chars.push(String.fromCharCode(97 + r() % 26))
      doc.text.insertAt(at, ...chars)
    } else if (kind === 8) {
      if (doc.text && doc.text.length > 0) {
        const at = r() % doc.text.length
        doc.text.deleteAt(at, 1 + r() % Math.min(4, doc.text.length - at))
      }
    } else if (kind === 9) {
      if (!(doc.cnt instanceof Automerge.Counter)) doc.cnt = new Automerge.Counter(r() % 10)
      else doc.cnt.increment(r() % 5 - 2)
    } else if (kind === 10) {
      if (!doc.nested || typeof doc.nested !== 'object') doc.nested = {}
      doc.nested[KEYS[r() % 5]] = r() % 3 === 0 ? {deep: randomValue(r)} : randomValue(r)
    } else {
      if (doc.list && doc.list.length > 0 && r() % 2) {
        doc.list.insertAt(r() % (doc.list.length + 1), {m: r() % 9})
      } else {
        doc[key] = [r() % 5, 'q']
      }
    }
  }
}

// The reference frontend rejects a few random edits (e.g. incrementing a counter that the same
// change overwrote); those edits are simply skipped.
function safeChange(doc, opts, fn) {
  try { return Automerge.change(doc, opts, fn) } catch (e) { return doc }
}

function allChanges(doc) { return Automerge.getAllChanges(doc) }
function changeHash(buf) { return col.decodeChangeMeta(buf, true).hash }

function runBackend(steps) {
  // steps: [{op: 'load', bytes} | {op: 'apply', changes: [Uint8Array]}]; records per-step results
  let state = null
  const results = []
  for (const step of steps) {
    const res = {}
    try {
      if (step.op === 'load') {
        state = Backend.load(step.bytes)
        res.getPatch = Backend.getPatch(state)
      } else {
        if (!state) state = Backend.init()
        const [s2, patch] = Backend.applyChanges(state, step.changes)
        state = s2
        res.patch = patch
      }
      res.save = hex(Backend.save(state))
      res.heads = Backend.getHeads(state)
      res.pending = Backend.getPatch(state).pendingChanges
      res.missingDeps = Backend.getMissingDeps(state)
      res.getPatch = Backend.getPatch(Backend.load(Backend.save(state)))
    } catch (e) {
      res.error = {name: e.name, message: e.message}
      results.push(res)
      break
    }
    results.push(res)
  }
  return results
}

function jsonPatch(p) {
  // Make patches JSON-safe: Uint8Array values -> {bytes: hex}
  return JSON.parse(JSON.stringify(p, (k, v) => (v instanceof Uint8Array ? {__bytes: hex(v)} : v)))
}

function scenarioFromDocs(name, r, actorDocs, base) {
  // Collect changes from all actor docs, dedupe, then a (possibly shuffled) delivery order.
  const seen = new Set(), changes = []
  for (const d of actorDocs) for (const c of allChanges(d)) {
    const h = changeHash(c)
    if (!seen.has(h)) { seen.add(h); changes.push(c) }
  }
  const order = changes.slice()
  const mode = r() % 3
  if (mode === 1) order.reverse()
  if (mode === 2) for (let i = order.length - 1; i > 0; i--) { const j = r() % (i + 1); [order[i], order[j]] = [order[j], order[i]] }
  const scenarios = []
  const steps1 = [{op: 'apply', changes: order}]
  scenarios.push({name: name + '/fresh', steps: steps1.map(s => ({op: s.op, changes: s.changes.map(hex)})),
                  results: runBackend(steps1).map(jsonPatch)})
  if (base) {
    const baseBytes = base.bytes
    const baseHashes = new Set(base.changes.map(changeHash))
    const rest = order.filter(c => !baseHashes.has(changeHash(c)))
    const steps2 = [{op: 'load', bytes: baseBytes}, {op: 'apply', changes: rest}]
    scenarios.push({name: name + '/load+apply',
                    steps: [{op: 'load', bytes: hex(baseBytes)}, {op: 'apply', changes: rest.map(hex)}],
                    results: runBackend(steps2).map(jsonPatch)})
  }
  return scenarios
}

function randomScenarios(count, seed, maxEdits) {
  const r = lcg(seed)
  const out = []
  for (let s = 0; s < count; s++) {
    const nActors = 1 + r() % 4
    const actors = []
    while (actors.length < nActors) { const a = randomActor(r); if (!actors.includes(a)) actors.push(a) }
    let base = Automerge.init(actors[0])
    const nBase = 1 + r() % maxEdits
    for (let i = 0; i < nBase; i++) base = safeChange(base, {time: 0}, d => randomEdit(r, d))
    const baseInfo = {bytes: Automerge.save(base), changes: allChanges(base)}
    const docs = actors.map((a, i) => i === 0 ? base : Automerge.load(baseInfo.bytes, a))
    for (let round = 0; round < 1 + r() % 3; round++) {
      for (let i = 0; i < docs.length; i++) {
        const n = r() % maxEdits
        for (let j = 0; j < n; j++) docs[i] = safeChange(docs[i], {time: r() % 3 === 0 ? r() % 1000 : 0}, d => randomEdit(r, d))
      }
      if (r() % 2 && docs.length > 1) { // partial sync between two actors
        const i = r() % docs.length, j = r() % docs.length
        if (i !== j) docs[i] = Automerge.merge(docs[i], docs[j])
      }
    }
    out.push(...scenarioFromDocs(`random${seed}-${s}`, r, docs, baseInfo))
  }
  return out
}

// ------------------------------------------------------------------------------------------------
// 3. Hand-built changes (JSON form -> encodeChange), edge cases of new.js
// ------------------------------------------------------------------------------------------------
function handScenarios() {
  const out = []
  const H = c => changeHash(col.encodeChange(c))
  const add = (name, stepsJson) => {
    const steps = stepsJson.map(s => s.op === 'load' ? s : {op: 'apply', changes: s.changes.map(c => c instanceof Uint8Array ? c : col.encodeChange(c))})
    out.push({name, steps: steps.map(s => s.op === 'load' ? {op: 'load', bytes: hex(s.bytes)} : {op: 'apply', changes: s.changes.map(hex)}),
              results: runBackend(steps).map(jsonPatch)})
  }
  const a1 = '01234567', a2 = '89abcdef', a3 = 'fedcba98'
  const c1 = {actor: a1, seq: 1, startOp: 1, time: 0, deps: [], ops: [
    {action: 'set', obj: '_root', key: 'x', datatype: 'uint', value: 1, pred: []}]}
  const c2 = {actor: a1, seq: 2, startOp: 2, time: 0, deps: [H(c1)], ops: [
    {action: 'set', obj: '_root', key: 'x', datatype: 'uint', value: 2, pred: [`1@${a1}`]}]}
  const c3 = {actor: a2, seq: 1, startOp: 2, time: 0, deps: [H(c1)], ops: [
    {action: 'set', obj: '_root', key: 'x', datatype: 'uint', value: 3, pred: [`1@${a1}`]}]}
  const c4 = {actor: a3, seq: 1, startOp: 2, time: 0, deps: [H(c1)], ops: [
    {action: 'set', obj: '_root', key: 'x', datatype: 'uint', value: 4, pred: [`1@${a1}`]}]}
  add('concurrent-overwrite-order1', [{changes: [c1]}, {changes: [c2, c3, c4]}])
  add('concurrent-overwrite-order2', [{changes: [c1]}, {changes: [c4, c3, c2]}])
  add('concurrent-overwrite-onecall', [{changes: [c1, c3, c2, c4]}])
  add('queue-reordered', [{changes: [c2, c1]}])
  add('queue-missing-dep', [{changes: [c2]}])
  add('duplicate-change', [{changes: [c1]}, {changes: [c1, c2]}])
  // Errors
  const bad1 = {actor: a2, seq: 1, startOp: 1, time: 0, deps: [], ops: [
    {action: 'set', obj: '_root', key: 'x', datatype: 'uint', value: 1, pred: [`9@${a1}`]}]}
  add('err-missing-pred', [{changes: [c1]}, {changes: [bad1]}])
  const skip = {actor: a1, seq: 3, startOp: 3, time: 0, deps: [H(c1)], ops: []}
  add('err-skipped-seq', [{changes: [c1]}, {changes: [skip]}])
  // Text editing (new_backend_test.js:416-911 style)
  const t1 = {actor: a1, seq: 1, startOp: 1, time: 0, deps: [], ops: [
    {action: 'makeText', obj: '_root', key: 'text', pred: []},
    {action: 'set', obj: `1@${a1}`, elemId: '_head', insert: true, value: 'a', pred: []},
    {action: 'set', obj: `1@${a1}`, elemId: `2@${a1}`, insert: true, value: 'b', pred: []},
    {action: 'set', obj: `1@${a1}`, elemId: `3@${a1}`, insert: true, value: 'c', pred: []}]}
  const t2 = {actor: a2, seq: 1, startOp: 5, time: 0, deps: [H(t1)], ops: [
    {action: 'set', obj: `1@${a1}`, elemId: `2@${a1}`, insert: true, value: 'x', pred: []},
    {action: 'del', obj: `1@${a1}`, elemId: `3@${a1}`, pred: [`3@${a1}`]}]}
  const t3 = {actor: a3, seq: 1, startOp: 5, time: 0, deps: [H(t1)], ops: [
    {action: 'set', obj: `1@${a1}`, elemId: `2@${a1}`, insert: true, value: 'y', pred: []},
    {action: 'set', obj: `1@${a1}`, elemId: '_head', insert: true, value: 'z', pred: []},
    {action: 'set', obj: `1@${a1}`, elemId: `4@${a1}`, value: 'C', pred: [`4@${a1}`]}]}
  add('text-concurrent', [{changes: [t1]}, {changes: [t2, t3]}])
  add('text-concurrent-onecall', [{changes: [t1, t3, t2]}])
  const t4 = {actor: a1, seq: 2, startOp: 5, time: 0, deps: [H(t1)], ops: [
    {action: 'set', obj: `1@${a1}`, elemId: `4@${a1}`, insert: true, values: ['d', 'e', 'f'], pred: []},
    {action: 'del', obj: `1@${a1}`, elemId: `2@${a1}`, multiOp: 2, pred: [`2@${a1}`]}]}
  add('text-multiop', [{changes: [t1, t4]}])
  // Counters
  const k1 = {actor: a1, seq: 1, startOp: 1, time: 0, deps: [], ops: [
    {action: 'set', obj: '_root', key: 'c', datatype: 'counter', value: 1, pred: []}]}
  const k2 = {actor: a2, seq: 1, startOp: 2, time: 0, deps: [H(k1)], ops: [
    {action: 'inc', obj: '_root', key: 'c', value: 2, pred: [`1@${a1}`]}]}
  const k3 = {actor: a3, seq: 1, startOp: 2, time: 0, deps: [H(k1)], ops: [
    {action: 'inc', obj: '_root', key: 'c', value: 3, pred: [`1@${a1}`]}]}
  add('counter-concurrent-inc', [{changes: [k1]}, {changes: [k2, k3]}])
  // Key order: UTF-16 vs UTF-8 (U+1F600 sorts before U+FFFD in JS)
  const u1 = {actor: a1, seq: 1, startOp: 1, time: 0, deps: [], ops: [
    {action: 'set', obj: '_root', key: '�', value: 1, datatype: 'int', pred: []},
    {action: 'set', obj: '_root', key: '😀', value: 2, datatype: 'int', pred: []},
    {action: 'set', obj: '_root', key: '', value: 3, datatype: 'int', pred: []},
    {action: 'set', obj: '_root', key: 'z', value: 4, datatype: 'int', pred: []},
    {action: 'set', obj: '_root', key: 'zz', value: 5, datatype: 'int', pred: []},
    {action: 'set', obj: '_root', key: '퟿', value: 6, datatype: 'int', pred: []}]}
  add('key-order-utf16', [{changes: [u1]}])
  // Nested objects and deleting a list element that holds a map
  const n1 = {actor: a1, seq: 1, startOp: 1, time: 0, deps: [], ops: [
    {action: 'makeMap', obj: '_root', key: 'm', pred: []},
    {action: 'makeList', obj: `1@${a1}`, key: 'l', pred: []},
    {action: 'makeMap', obj: `2@${a1}`, elemId: '_head', insert: true, pred: []},
    {action: 'set', obj: `3@${a1}`, key: 'deep', value: 'yes', pred: []}]}
  const n2 = {actor: a2, seq: 1, startOp: 5, time: 0, deps: [H(n1)], ops: [
    {action: 'del', obj: `2@${a1}`, elemId: `3@${a1}`, pred: [`3@${a1}`]},
    {action: 'makeText', obj: '_root', key: 'm', pred: [`1@${a1}`]}]}
  add('nested-objects', [{changes: [n1]}, {changes: [n2]}])
  // Extra (unknown) trailing bytes in a change survive save/load (columnar_test.js:54-84)
  const trailing = Uint8Array.from([0x85, 0x6f, 0x4a, 0x83, 0xb2, 0x98, 0x9e, 0xa9, 1, 61, 0, 2, 0x12, 0x34,
    1, 1, 252, 250, 220, 255, 5, 14, 73, 110, 105, 116, 105, 97, 108, 105, 122, 97, 116, 105, 111, 110,
    0, 6, 0x15, 3, 0x34, 1, 0x42, 2, 0x56, 2, 0x57, 1, 0x70, 2, 0x7f, 1, 0x78, 1, 0x7f, 1, 0x7f, 19, 1,
    0x7f, 0, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9])
  add('trailing-bytes', [{changes: [trailing]}])
  // Rust-generated document (backend_test.js:1043-1057), loaded
  const rust = Uint8Array.from([133, 111, 74, 131, 233, 181, 157, 86, 0, 144, 1, 1, 16, 228, 91, 238, 197, 233, 52, 66, 187, 138, 75, 115, 104, 190, 195, 159, 200, 1, 221, 158, 172, 238, 121, 38, 160, 123, 25, 33, 97, 124, 142, 27, 86, 224, 238, 83, 14, 157, 207, 233, 8, 110, 91, 151, 172, 38, 120, 221, 38, 162, 7, 1, 2, 3, 2, 19, 2, 35, 7, 53, 16, 64, 2, 86, 2, 8, 21, 7, 33, 2, 35, 2, 52, 1, 66, 2, 86, 3, 87, 8, 128, 1, 2, 127, 0, 127, 1, 127, 1, 127, 243, 145, 234, 194, 149, 47, 127, 14, 73, 110, 105, 116, 105, 97, 108, 105, 122, 97, 116, 105, 111, 110, 127, 0, 127, 7, 127, 5, 98, 105, 114, 100, 115, 127, 0, 127, 1, 1, 127, 1, 127, 133, 1, 0, 0, 0, 0, 0, 0, 8, 64, 127, 0])
  add('rust-doc-load', [{op: 'load', bytes: rust}])
  // Long string value -> DEFLATE-compressed column (backend_test.js:1026-1041)
  const longc = {actor: '111111', seq: 1, time: 0, startOp: 1, deps: [], ops: [
    {action: 'set', obj: '_root', key: 'longString', value: 'a'.repeat(1024), pred: []}]}
  add('deflate-long-string', [{changes: [longc]}])
  return out
}

// ------------------------------------------------------------------------------------------------
// 4. Change encoding vectors (columnar.js encodeChange/decodeChange)
// ------------------------------------------------------------------------------------------------
function changeVectors(scen) {
  const out = []
  const change1 = {actor: 'aaaa', seq: 1, startOp: 1, time: 9, message: '', deps: [], ops: [
    {action: 'makeText', obj: '_root', key: 'text', insert: false, pred: []},
    {action: 'set', obj: '1@aaaa', elemId: '_head', insert: true, value: 'h', pred: []},
    {action: 'del', obj: '1@aaaa', elemId: '2@aaaa', insert: false, pred: ['2@aaaa']},
    {action: 'set', obj: '1@aaaa', elemId: '_head', insert: true, value: 'H', pred: []},
    {action: 'set', obj: '1@aaaa', elemId: '4@aaaa', insert: true, value: 'i', pred: []}]}
  const b = col.encodeChange(change1)
  out.push({bytes: hex(b), hash: changeHash(b), decoded: jsonPatch(col.decodeChange(b))})
  const seen = new Set([hex(b)])
  for (const s of scen) for (const st of s.steps) if (st.changes) for (const c of st.changes) {
    if (seen.has(c) || out.length > 400) continue
    seen.add(c)
    const bytes = unhex(c)
    let decoded = null, error = null
    try { decoded = jsonPatch(col.decodeChange(bytes)) } catch (e) { error = e.message }
    out.push({bytes: c, hash: error ? null : changeHash(bytes), decoded, error})
  }
  return out
}

// ------------------------------------------------------------------------------------------------
// 5. Workload generators (SURVEY.md §8(d)) restated with the reference encoder; the C++
//    generator in automerge_amd/csrc/workload.cpp must reproduce these bytes exactly.
// ------------------------------------------------------------------------------------------------
function c4Doc(docIndex) {
  const r = lcg(docIndex)
  const actors = []
  while (actors.length < 4) {
    let a = ''
    for (let i = 0; i < 4; i++) a += r().toString(16).padStart(8, '0')
    if (!actors.includes(a)) actors.push(a)
  }
  const a0 = actors[0]
  const change0 = {actor: a0, seq: 1, startOp: 1, time: 0, message: '', deps: [], ops: [
    {action: 'makeList', obj: '_root', key: 'items', insert: false, pred: []},
    {action: 'set', obj: '_root', key: 'title', insert: false, value: 'untitled', pred: []}]}
  const bin0 = col.encodeChange(change0), h0 = changeHash(bin0)
  const changes = [] // [actor][j]
  for (let i = 0; i < 4; i++) {
    const a = actors[i]
    let lastHash = h0, lastTitle = `2@${a0}`, own = [] // own inserted elemIds
    const seqBase = i === 0 ? 2 : 1
    changes.push([])
    for (let j = 0; j < 3; j++) {
      const startOp = 3 + 5 * j
      const ops = []
      let ref = (own.length === 0 || r() % 4 === 0) ? '_head' : own[r() % own.length]
      for (let k = 0; k < 4; k++) {
        const id = `${startOp + k}@${a}`
        ops.push({action: 'set', obj: `1@${a0}`, elemId: ref, insert: true, value: String.fromCharCode(97 + r() % 26), pred: []})
        own.push(id); ref = id
      }
      const titleId = `${startOp + 4}@${a}`
      ops.push({action: 'set', obj: '_root', key: 'title', insert: false, value: `t${i}.${j}.${r() % 1000}`, pred: [lastTitle]})
      lastTitle = titleId
      const ch = {actor: a, seq: seqBase + j, startOp, time: 0, message: '', deps: [lastHash], ops}
      const bin = col.encodeChange(ch)
      changes[i].push(bin)
      lastHash = changeHash(bin)
    }
  }
  const order = []
  for (let j = 0; j < 3; j++) for (let i = 0; i < 4; i++) order.push(changes[i][j])
  const base = Backend.loadChanges(Backend.init(), [bin0])
  const baseBytes = Backend.save(base)
  return {change0: bin0, baseBytes, order}
}

function c2Doc(docIndex) {
  const r = lcg(docIndex)
  const actors = []
  while (actors.length < 3) {
    let a = ''
    for (let i = 0; i < 4; i++) a += r().toString(16).padStart(8, '0')
    if (!actors.includes(a)) actors.push(a)
  }
  const a0 = actors[0]
  const ops = []
  for (let k = 0; k < 8; k++) ops.push({action: 'set', obj: '_root', key: `k${k}`, insert: false, value: r() % 100000, datatype: 'int', pred: []})
  ops.push({action: 'set', obj: '_root', key: 'count', insert: false, value: r() % 100, datatype: 'counter', pred: []})
  ops.push({action: 'set', obj: '_root', key: 'name', insert: false, value: `doc-${docIndex}`, pred: []})
  const ch1 = {actor: a0, seq: 1, startOp: 1, time: 0, message: '', deps: [], ops}
  const bin1 = col.encodeChange(ch1), h1 = changeHash(bin1)
  const rest = []
  for (let i = 1; i <= 2; i++) {
    const ch = {actor: actors[i], seq: 1, startOp: 11, time: 0, message: '', deps: [h1], ops: [
      {action: 'inc', obj: '_root', key: 'count', insert: false, value: 1 + r() % 9, pred: [`9@${a0}`]},
      {action: 'set', obj: '_root', key: 'k1', insert: false, value: r() % 100000, datatype: 'int', pred: [`2@${a0}`]}]}
    rest.push(col.encodeChange(ch))
  }
  const all = [bin1].concat(rest)
  const docBytes = Backend.save(Backend.loadChanges(Backend.init(), all))
  return {changes: all, docBytes}
}

function workloadVectors() {
  const crypto = require('crypto')
  const sha = u8 => crypto.createHash('sha256').update(Buffer.from(u8)).digest('hex')
  const out = {c4: [], c2: []}
  for (let d = 0; d < 64; d++) {
    const {change0, baseBytes, order} = c4Doc(d)
    const s = Backend.applyChanges(Backend.load(baseBytes), order)[0]
    const rec = {doc: d, change0: sha(change0), base: sha(baseBytes), changes: order.map(sha),
                 merged: sha(Backend.save(s)), heads: Backend.getHeads(s)}
    if (d < 4) { rec.baseBytes = hex(baseBytes); rec.changeBytes = order.map(hex); rec.mergedBytes = hex(Backend.save(s)) }
    out.c4.push(rec)
  }
  for (let d = 0; d < 64; d++) {
    const {changes, docBytes} = c2Doc(d)
    const rec = {doc: d, changes: changes.map(sha), docBytes: d < 4 ? hex(docBytes) : undefined, doc_sha: sha(docBytes),
                 getPatch: d < 4 ? jsonPatch(Backend.getPatch(Backend.load(docBytes))) : undefined}
    out.c2.push(rec)
  }
  return out
}

// ------------------------------------------------------------------------------------------------
// 6. Sync Bloom filter vectors (sync.js:38-125)
// ------------------------------------------------------------------------------------------------
function bloomVectors() {
  const r = lcg(777)
  const out = []
  for (let t = 0; t < 40; t++) {
    const n = t === 0 ? 0 : 1 + r() % 30
    const hashes = []
    for (let i = 0; i < n; i++) { let h = ''; for (let j = 0; j < 8; j++) h += r().toString(16).padStart(8, '0'); hashes.push(h) }
    const bf = new sync.BloomFilter(hashes)
    const probes = []
    for (let i = 0; i < 20; i++) { let h = ''; for (let j = 0; j < 8; j++) h += r().toString(16).padStart(8, '0'); probes.push(h) }
    const all = hashes.concat(probes)
    const decoded = new sync.BloomFilter(bf.bytes)
    out.push({hashes, bytes: hex(bf.bytes), probes: all, contains: all.map(h => decoded.containsHash(h))})
  }
  return out
}

// Hand-made filter headers (numProbes 0/1/2, bits shorter than the header, incomplete numbers):
// containsHash as the reference decodes them (new BloomFilter(bytes), sync.js:47-58, 112-120).
function bloomEdgeVectors() {
  const r = lcg(4242)
  const rh = () => { let h = ''; for (let j = 0; j < 8; j++) h += r().toString(16).padStart(8, '0'); return h }
  const out = []
  const hdr = (ne, bpe, np) => { const e = new enc.Encoder(); e.appendUint32(ne); e.appendUint32(bpe); e.appendUint32(np); return e.buffer }
  for (let t = 0; t < 24; t++) {
    const ne = 1 + r() % 12, bpe = [10, 3, 1, 0][t % 4], np = [0, 1, 2, 7][(t >> 2) % 4]
    const nbytes = Math.ceil(ne * bpe / 8)
    const bits = new Uint8Array(nbytes)
    for (let i = 0; i < nbytes; i++) bits[i] = r() & 0xff
    const h = hdr(ne, bpe, np)
    const bytes = new Uint8Array(h.byteLength + nbytes)
    bytes.set(h, 0); bytes.set(bits, h.byteLength)
    const probes = []
    for (let i = 0; i < 16; i++) probes.push(rh())
    const err = errOf(() => new sync.BloomFilter(bytes))
    const f = err ? null : new sync.BloomFilter(bytes)
    out.push({bytes: hex(bytes), probes, contains: f ? probes.map(x => f.containsHash(x)) : null, error: err})
  }
  // malformed: truncated bits, incomplete header numbers, out-of-range uint32
  const bad = [hex(hdr(4, 10, 7)) + 'ff', '80', '0a80', '0a0a', 'ffffffff7f0a07']
  for (const b of bad) {
    const bytes = unhex(b)
    out.push({bytes: b, probes: [rh()], contains: null, error: errOf(() => new sync.BloomFilter(bytes))})
  }
  return out
}

function main() {
  const write = (name, obj) => {
    fs.writeFileSync(path.join(OUT, name), JSON.stringify(obj) + '\n')
    console.log('wrote', name, fs.statSync(path.join(OUT, name)).size, 'bytes')
  }
  write('codecs.json', codecVectors())
  const hand = handScenarios()
  const rand = randomScenarios(150, 2024, 4).concat(randomScenarios(12, 99, 25))
  write('docs.json', {scenarios: hand.concat(rand)})
  write('changes.json', changeVectors(hand.concat(rand)))
  write('workload.json', workloadVectors())
  write('bloom.json', bloomVectors())
  write('bloom_edge.json', bloomEdgeVectors())
}

if (require.main === module) main()
else module.exports = {c4Doc, c2Doc, lcg, runBackend, jsonPatch, hex, randomActor, randomValue, safeChange, changeHash}
