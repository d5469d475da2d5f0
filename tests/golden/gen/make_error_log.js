// Error-path and edge-input golden vectors at the Backend boundary. Each scenario hand-builds change
// or document chunks (valid containers around one malformed or unusual part: codec records of
// encoding_test.js, container faults of columnar.js, the semantic errors of new.js) and calls the
// reference Backend (init / load / applyChanges / save / getPatch / getHeads) through the recorder
// of make_backend_log.js, so every call is logged with the reference's result or thrown error class
// and message. Output has the schema of tests/golden/backend_log_*.json and is replayed by the same
// replays (tests/backend_log.py, tests/js/backend_log_replay.js).
//   NODE_PATH=tests/golden/gen/node_modules node tests/golden/gen/make_error_log.js
'use strict'
const fs = require('fs')
const path = require('path')
const crypto = require('crypto')
const zlib = require('zlib')
const REF = process.env.AM_REF || '/root/reference'
const OUT = path.join(__dirname, '..', 'backend_log_errors.json')

// ---- canonical values and the recorder (same encoding as make_backend_log.js) ----
function canon(x, handleId) {
  if (x === undefined) return {__undef: 1}
  if (typeof x === 'number') {
    if (!Number.isFinite(x) || Object.is(x, -0)) return {__f64: Object.is(x, -0) ? '-0' : String(x)}
    return x
  }
  if (x instanceof Uint8Array) return {__bytes: Buffer.from(x.buffer, x.byteOffset, x.byteLength).toString('hex')}
  if (Array.isArray(x)) return x.map(v => canon(v, handleId))
  if (x && typeof x === 'object') {
    if (handleId) { const id = handleId(x); if (id !== null) return {$h: id} }
    const o = {}
    for (const k of Object.keys(x).sort()) o[k] = canon(x[k], handleId)
    return o
  }
  return x
}
const Real = require(path.join(REF, 'backend'))
let handles = new Map(), nextHandle = 0, log = null
const isHandle = x => x && typeof x === 'object' && 'state' in x && ('heads' in x)
const handleId = x => {
  if (!isHandle(x)) return null
  if (!handles.has(x)) handles.set(x, nextHandle++)
  return handles.get(x)
}
const B = {}
for (const name of Object.keys(Real)) {
  B[name] = function (...args) {
    const entry = {fn: name, args: canon(args, handleId)}
    log.push(entry)
    try {
      const r = Real[name](...args)
      entry.result = canon(r, handleId)
      return r
    } catch (e) {
      entry.error = {name: e.constructor.name, message: e.message}
      throw e
    }
  }
}

// ---- chunk builders ----
const uleb = n => { const o = []; n = BigInt(n); do { let b = Number(n & 0x7fn); n >>= 7n; if (n) b |= 0x80; o.push(b) } while (n); return o }
const sleb = n => {
  const o = []; n = BigInt(n)
  for (;;) { const b = Number(n & 0x7fn); n >>= 7n; if ((n === 0n && !(b & 0x40)) || (n === -1n && (b & 0x40))) { o.push(b); return o } o.push(b | 0x80) }
}
const str = s => { const b = Buffer.from(s, 'utf8'); return uleb(b.length).concat([...b]) }
const rawstr = bytes => uleb(bytes.length).concat(bytes)
const hexstr = h => rawstr([...Buffer.from(h, 'hex')])
function container(type, body, opts = {}) {
  const hdr = [type].concat(uleb(opts.len !== undefined ? opts.len : body.length))
  const h = crypto.createHash('sha256').update(Buffer.from(hdr.concat(body))).digest()
  const ck = opts.checksum || [...h.subarray(0, 4)]
  return Uint8Array.from([0x85, 0x6f, 0x4a, 0x83].concat(ck, hdr, body, opts.trailing || []))
}
const chash = c => crypto.createHash('sha256').update(Buffer.from(c.subarray(8))).digest('hex')
// change: cols = [[columnId, bytes], ...] in the given order
function change(o) {
  const deps = (o.deps || []).slice().sort()
  let body = uleb(deps.length)
  for (const d of deps) body = body.concat([...Buffer.from(d, 'hex')])
  body = body.concat(hexstr(o.actor), o.seqBytes || uleb(o.seq), uleb(o.startOp), sleb(o.time || 0),
                     o.msgBytes ? rawstr(o.msgBytes) : str(o.message || ''), uleb((o.actors || []).length))
  for (const a of o.actors || []) body = body.concat(hexstr(a))
  body = body.concat(uleb(o.cols.length))
  for (const [id, b] of o.cols) body = body.concat(uleb(id), uleb(b.length))
  for (const [, b] of o.cols) body = body.concat(b)
  if (o.extra) body = body.concat(o.extra)
  if (o.truncate) body = body.slice(0, body.length - o.truncate)
  return container(o.type === undefined ? 1 : o.type, body, o.container || {})
}
const A = '0aaa', Bx = '0bbb', C = '0ccc'
// a one-op change setting root key `key` to uint `v` (no preds), columns in ascending order
function setKey(o) {
  const v = o.v === undefined ? 1 : o.v
  const vb = uleb(v)
  const cols = [[0x15, [0x7f].concat(o.keyBytes ? rawstr(o.keyBytes) : str(o.key || 'x'))], [0x34, [1]], [0x42, [0x7f, 1]],
                [0x56, [0x7f].concat(uleb(vb.length << 4 | 3))], [0x57, vb], [0x70, [0x7f, o.pred ? 1 : 0]]]
  if (o.pred) cols.push([0x71, [0x7f, o.pred[1]]], [0x73, [0x7f].concat(sleb(o.pred[0]))])
  return change(Object.assign({seq: 1, startOp: 1, actor: A, cols}, o, {cols: o.cols || cols}))
}
// ---- scenarios ----
const scenarios = []
function scenario(name, fn) {
  handles = new Map(); nextHandle = 0; log = []
  try { fn() } catch (e) { /* the thrown error is recorded in the log */ }
  scenarios.push({name, log})
  log = null
}
// apply the changes one call at a time; after each success record save, heads and getPatch
function applySeq(doc, batches) {
  for (const cs of batches) {
    const [d2] = B.applyChanges(doc, cs)
    doc = d2
    B.save(doc); B.getHeads(doc); B.getPatch(doc)
  }
  return doc
}
const good1 = setKey({})

// container and header
scenario('bad magic bytes', () => { const c = setKey({}); c[0] = 0x86; applySeq(B.init(), [[c]]) })
scenario('checksum mismatch', () => { const c = setKey({}); c[c.length - 1] ^= 1; applySeq(B.init(), [[c]]) })
scenario('unknown chunk type', () => applySeq(B.init(), [[setKey({type: 5})]]))
scenario('document chunk given to applyChanges', () => {
  const d0 = applySeq(B.init(), [[good1]]); applySeq(B.init(), [[B.save(d0)]])
})
scenario('chunk length beyond buffer', () => applySeq(B.init(), [[setKey({container: {len: 200}})]]))
scenario('change with trailing bytes after the chunk', () => applySeq(B.init(), [[setKey({container: {trailing: [0, 1]}})]]))
scenario('columns not in ascending order', () => applySeq(B.init(), [[setKey({cols: [[0x34, [1]], [0x15, [0x7f, 1, 0x78]], [0x42, [0x7f, 1]], [0x56, [0x7f, 0x13]], [0x57, [1]], [0x70, [0x7f, 0]]]})]]))
scenario('deflated column in a change', () => applySeq(B.init(), [[setKey({cols: [[0x1d, [...zlib.deflateRawSync(Buffer.from([0x7f, 1, 0x78]))]], [0x34, [1]], [0x42, [0x7f, 1]], [0x56, [0x7f, 0x13]], [0x57, [1]], [0x70, [0x7f, 0]]]})]]))
scenario('seq out of range (uint53)', () => applySeq(B.init(), [[setKey({seqBytes: [0x80, 0x80, 0x80, 0x80, 0x80, 0x80, 0x80, 0x10]})]]))
scenario('truncated header', () => applySeq(B.init(), [[setKey({truncate: 40})]]))
scenario('extra bytes after the columns', () => applySeq(B.init(), [[setKey({extra: [1, 2, 3]})]]))

// column codecs (encoding_test.js cases inside the action / key / insert columns of a change)
const withAction = (act, n, o = {}) => change(Object.assign({actor: A, seq: 1, startOp: 1, cols: [
  [0x15, o.keys || sleb(-n).concat(...Array.from({length: n}, (_, i) => str('k' + i)))],
  [0x34, [n]], [0x42, act], [0x56, n > 1 ? [n, 0] : [0x7f, 0]], [0x70, n > 1 ? [n, 0] : [0x7f, 0]]]}, o))
scenario('RLE successive repetitions with the same value', () => applySeq(B.init(), [[withAction([2, 1, 2, 1], 4)]]))
scenario('RLE repetition count of 1', () => applySeq(B.init(), [[withAction([1, 1], 1)]]))
scenario('RLE successive literals', () => applySeq(B.init(), [[withAction([0x7f, 1, 0x7f, 3], 2)]]))
scenario('RLE successive null runs', () => applySeq(B.init(), [[withAction([0, 1, 0, 1], 2)]]))
scenario('RLE zero-length null run', () => applySeq(B.init(), [[withAction([0, 0, 0x7f, 1], 1)]]))
scenario('RLE repetition inside a literal', () => applySeq(B.init(), [[withAction([0x7e, 1, 1], 2)]]))
scenario('RLE number out of range', () => applySeq(B.init(), [[withAction([0x7f, 0x80, 0x80, 0x80, 0x80, 0x80, 0x80, 0x80, 0x80, 0x80, 0x02], 1)]]))
scenario('RLE incomplete number', () => applySeq(B.init(), [[withAction([0x7f, 0x80], 1)]]))
scenario('RLE string column: successive repetitions', () => applySeq(B.init(), [[withAction([4, 1], 4, {keys: [2].concat(str('a'), [2], str('a'))})]]))
scenario('boolean zero-length run', () => applySeq(B.init(), [[change({actor: A, seq: 1, startOp: 1, cols: [
  [0x15, [0x7f].concat(str('x'))], [0x34, [1, 0]], [0x42, [0x7f, 1]], [0x56, [0x7f, 0]], [0x70, [0x7f, 0]]]})]]))
scenario('excess values in a column', () => applySeq(B.init(), [[withAction([0x7f, 1], 1, {keys: [0x7e].concat(str('a'), str('b'))})]]))
scenario('null action', () => applySeq(B.init(), [[withAction([0, 1], 1)]]))

// queue / seq / actor semantics
scenario('skipped sequence number', () => applySeq(B.init(), [[setKey({})], [setKey({seq: 3, startOp: 2, deps: [chash(setKey({}))]})]]))
scenario('reuse of sequence number', () => applySeq(B.init(), [[setKey({})], [setKey({v: 2})]]))
scenario('first change of an actor with seq 2', () => applySeq(B.init(), [[setKey({seq: 2})]]))
scenario('actor in the change actor list not known to the document', () =>
  applySeq(B.init(), [[setKey({key: 'x', actors: [Bx], pred: [1, 1]})]]))
scenario('queued change (missing dependency) then its dependency', () => {
  const c1 = setKey({}), c2 = setKey({seq: 2, startOp: 2, key: 'y', deps: [chash(c1)]})
  applySeq(B.init(), [[c2], [c1]])
})
scenario('duplicate change in one call', () => applySeq(B.init(), [[good1, good1]]))

// op semantics (new.js)
scenario('no matching operation for pred', () => applySeq(B.init(), [[setKey({pred: [5, 0]})]]))
scenario('mismatched object reference', () => applySeq(B.init(), [[change({actor: A, seq: 1, startOp: 1, cols: [
  [0x01, [0x7f, 0]], [0x15, [0x7f].concat(str('x'))], [0x34, [1]], [0x42, [0x7f, 1]], [0x56, [0x7f, 0]], [0x70, [0x7f, 0]]]})]]))
scenario('mismatched operation key', () => applySeq(B.init(), [[change({actor: A, seq: 1, startOp: 1, cols: [
  [0x11, [0x7f, 0]], [0x13, [0x7f, 0]], [0x34, [1]], [0x42, [0x7f, 1]], [0x56, [0x7f, 0]], [0x70, [0x7f, 0]]]})]]))
// makeList at 1@A on key 'l', then ops inside it
const mkList = change({actor: A, seq: 1, startOp: 1, cols: [
  [0x15, [0x7f].concat(str('l'))], [0x34, [1]], [0x42, [0x7f, 2]], [0x70, [0x7f, 0]]]})
const inList = (o, rows) => change(Object.assign({actor: A, seq: 2, startOp: 2, deps: [chash(mkList)], cols: rows}, o))
scenario('reference element not found (empty list)', () => applySeq(B.init(), [[mkList], [inList({}, [
  [0x01, [0x7f, 0]], [0x02, [0x7f, 1]], [0x11, [0x7f, 0]], [0x13, [0x7f, 9]], [0x34, [0, 1]], [0x42, [0x7f, 1]],
  [0x56, [0x7f, 0x16]], [0x57, [0x61]], [0x70, [0x7f, 0]]])]]))
scenario('reference element not found (non-empty list)', () => applySeq(B.init(), [[mkList], [inList({}, [
  [0x01, [2, 0]], [0x02, [2, 1]], [0x11, [0, 1, 0x7f, 0]], [0x13, [0x7e, 0, 9]], [0x34, [0, 2]], [0x42, [2, 1]],
  [0x56, [2, 0x16]], [0x57, [0x61, 0x62]], [0x70, [2, 0]]])]]))
scenario('update of a list element that does not exist', () => applySeq(B.init(), [[mkList], [inList({}, [
  [0x01, [0x7f, 0]], [0x02, [0x7f, 1]], [0x11, [0x7f, 0]], [0x13, [0x7f, 9]], [0x34, [1]], [0x42, [0x7f, 1]],
  [0x56, [0x7f, 0x16]], [0x57, [0x61]], [0x70, [0x7f, 0]]])]]))
scenario('delete of a list element that does not exist', () => applySeq(B.init(), [[mkList], [inList({}, [
  [0x01, [0x7f, 0]], [0x02, [0x7f, 1]], [0x11, [0x7f, 0]], [0x13, [0x7f, 9]], [0x34, [1]], [0x42, [0x7f, 3]],
  [0x70, [0x7f, 1]], [0x71, [0x7f, 0]], [0x73, [0x7f, 9]]])]]))
scenario('duplicate operation ID', () => applySeq(B.init(), [[setKey({})], [setKey({seq: 2, startOp: 1, key: 'y', deps: [chash(good1)]})]]))
scenario('duplicate operation ID (same key)', () => applySeq(B.init(), [[setKey({})], [setKey({seq: 2, startOp: 1, v: 3, deps: [chash(good1)]})]]))
scenario('delete without pred (map key)', () => applySeq(B.init(), [[setKey({})], [change({actor: A, seq: 2, startOp: 2, deps: [chash(good1)], cols: [
  [0x15, [0x7f].concat(str('x'))], [0x34, [1]], [0x42, [0x7f, 3]], [0x70, [0x7f, 0]]]})]]))
scenario('inserting delete', () => applySeq(B.init(), [[mkList], [inList({}, [
  [0x01, [0x7f, 0]], [0x02, [0x7f, 1]], [0x13, [0x7f, 0]], [0x34, [0, 1]], [0x42, [0x7f, 3]], [0x70, [0x7f, 0]]])]]))

// inputs the reference accepts: invalid UTF-8, unknown actions / datatypes / columns, big counters
scenario('invalid UTF-8 in a map key', () => applySeq(B.init(), [[setKey({keyBytes: [0x61, 0xff, 0x62]})], [setKey({seq: 2, startOp: 2, keyBytes: [0xc3], deps: [chash(setKey({keyBytes: [0x61, 0xff, 0x62]}))]})]]))
scenario('invalid UTF-8 in a change message', () => applySeq(B.init(), [[setKey({msgBytes: [0x68, 0xe2, 0x82]})]]))
scenario('overlong UTF-8 and surrogates in keys', () => applySeq(B.init(), [[withAction([3, 1], 3, {keys: [0x7d].concat(rawstr([0xc0, 0xaf]), rawstr([0xed, 0xa0, 0x80]), rawstr([0xf4, 0x90, 0x80, 0x80]))})]]))
scenario('unknown action and datatype', () => applySeq(B.init(), [[change({actor: A, seq: 1, startOp: 1, cols: [
  [0x15, [0x7e].concat(str('x'), str('y'))], [0x34, [2]], [0x42, [0x7e, 17, 1]], [0x56, [0x7e, 0x4e, 0x2c]], [0x57, [1, 2, 3, 4, 5, 6]], [0x70, [2, 0]]]})]]))
scenario('unknown columns in a change', () => applySeq(B.init(), [[change({actor: A, seq: 1, startOp: 1, cols: [
  [0x15, [0x7f].concat(str('x'))], [0x34, [1]], [0x42, [0x7f, 1]], [0x56, [0x7f, 0x13]], [0x57, [7]], [0x70, [0x7f, 0]],
  [0xa2, [0x7f, 5]], [0xb5, [0x7f].concat(str('zz'))]]})],
  [setKey({seq: 2, startOp: 2, key: 'y', deps: [chash(change({actor: A, seq: 1, startOp: 1, cols: [
    [0x15, [0x7f].concat(str('x'))], [0x34, [1]], [0x42, [0x7f, 1]], [0x56, [0x7f, 0x13]], [0x57, [7]], [0x70, [0x7f, 0]],
    [0xa2, [0x7f, 5]], [0xb5, [0x7f].concat(str('zz'))]]}))]})]]))
scenario('uint value of 2^40 and startOp beyond 2^31', () => applySeq(B.init(), [[setKey({v: 2 ** 40, startOp: 2 ** 32 + 5})]]))

// make-like actions without a known type: `op[actionIdx] % 2 === 0` holds for a null action (type
// undefined) and for an even action beyond ACTIONS (type null), new.js:886-897, 972-976
const twoOps = (act, o = {}) => change(Object.assign({actor: A, seq: 1, startOp: 1, cols: [
  [0x15, sleb(-2).concat(str('a'), str('k'))], [0x34, [2]], [0x42, act], [0x56, [0x7e, 0x13, 0]], [0x57, [5]],
  [0x70, [2, 0]]]}, o))
const inObj = (prev, ctr, o = {}) => change(Object.assign({actor: A, seq: 2, startOp: 3, deps: [chash(prev)], cols: [
  [0x01, [0x7f, 0]], [0x02, [0x7f, ctr]], [0x15, [0x7f].concat(str('p'))], [0x34, [1]], [0x42, [0x7f, 1]],
  [0x56, [0x7f, 0x13]], [0x57, [9]], [0x70, [0x7f, 0]]]}, o))
scenario('null action next to a set, then a key inside its object', () => {
  const c1 = twoOps([0x7f, 1, 0, 1])
  const d = applySeq(B.init(), [[c1], [inObj(c1, 2)]])
  B.getPatch(B.load(B.save(d)))
})
scenario('unknown even action, then a key inside its object', () => {
  const c1 = twoOps([0x7e, 1, 8])
  const d = applySeq(B.init(), [[c1], [inObj(c1, 2)]])
  B.getPatch(B.load(B.save(d)))
})
scenario('unknown even action alone', () => { const d = applySeq(B.init(), [[withAction([0x7f, 10], 1)]]); B.getPatch(B.load(B.save(d))) })

// load() of malformed documents
const doc1 = () => { const d = Real.applyChanges(Real.init(), [good1])[0]; return Real.save(d) }
scenario('load: change chunk instead of a document', () => { B.load(good1) })
scenario('load: document with trailing data', () => { const d = doc1(); B.load(Uint8Array.from([...d, 0])) })
scenario('load: checksum mismatch', () => { const d = doc1(); d[d.length - 1] ^= 1; B.load(d) })
scenario('load: bad magic', () => { const d = doc1(); d[1] = 0; B.load(d) })

fs.writeFileSync(OUT, JSON.stringify({file: 'make_error_log.js', passed: scenarios.length, failed: 0, skipped: 0, scenarios}) + '\n')
const nerr = scenarios.reduce((a, s) => a + s.log.filter(e => e.error).length, 0)
for (const s of scenarios) {
  const e = s.log.find(x => x.error)
  console.log((s.name + '                                                  ').slice(0, 58), e ? `${e.error.name}: ${e.error.message}` : 'ok')
}
console.log(`${scenarios.length} scenarios, ${nerr} errors -> ${OUT}`)
