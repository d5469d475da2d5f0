// Change-history golden vectors beyond tests/golden/history.json (SURVEY.md §8(f) row 2):
//  - concurrent histories: several actors editing one document (map overwrites, list inserts and
//    deletions -> succ lists and re-created `del` ops, dependency DAGs with parallel branches), made
//    with the reference's own Automerge API and merged, then saved;
//  - the RangeErrors of groupChangeOps / decodeDocumentChanges (columnar.js:876-981): a valid saved
//    document is decoded with the reference's decodeDocumentHeader / column decoders, one column
//    value is changed, and the document is re-encoded with encodeDocumentHeader.
// Every case records Backend.getAllChanges(Backend.load(doc)) (computeHashGraph, new.js:1879-1904):
// the change chunks, or the error thrown (and whether Backend.load itself threw); and the same loop
// run straight on the document bytes (decodeChanges + encodeChange, new.js:1889-1890) -- the history
// of a document Backend.load rejects.
//   NODE_PATH=tests/golden/gen/node_modules node tests/golden/gen/make_history_cases.js
'use strict'
const fs = require('fs')
const path = require('path')
const REF = process.env.AM_REF || '/root/reference'
const Automerge = require(path.join(REF, 'src', 'automerge'))
const Backend = require(path.join(REF, 'backend'))
const C = require(path.join(REF, 'backend', 'columnar'))
const OUT = path.join(__dirname, '..', 'history_cases.json')
const hex = u8 => Buffer.from(u8).toString('hex')

// deterministic PRNG
let seed = 12345
const rnd = n => { seed = (seed * 1103515245 + 12345) & 0x7fffffff; return seed % n }

function record(name, doc) {
  const c = {name, doc: hex(doc), changes: null, error: null, load_error: null, direct: null, direct_error: null}
  // computeHashGraph's own loop (new.js:1889-1890) on the document bytes, whether or not load accepts them
  try { c.direct = C.decodeChanges([doc]).map(ch => hex(C.encodeChange(ch))) } catch (e) { c.direct_error = e.message }
  let st
  try { st = Backend.load(doc) } catch (e) { c.load_error = e.message; return c }
  try { c.changes = Backend.getAllChanges(st).map(hex) } catch (e) { c.error = e.message }
  return c
}

// ---- concurrent histories ----
function concurrent(nactors, rounds, opsPerChange) {
  const actors = []
  for (let a = 0; a < nactors; a++) actors.push((0x1000 + a * 7919).toString(16).padStart(8, '0') + 'ab'.repeat(a % 3))
  let clock = 1600000000
  let base = Automerge.change(Automerge.init(actors[0]), {time: clock++}, d => { d.list = []; d.text = new Automerge.Text(); d.map = {} })
  let docs = actors.map((a, i) => i === 0 ? base : Automerge.merge(Automerge.init(a), base))
  for (let r = 0; r < rounds; r++) {
    for (let i = 0; i < nactors; i++) {
      docs[i] = Automerge.change(docs[i], {time: clock++, message: rnd(4) ? undefined : 'edit ' + r}, d => {
        for (let k = 0; k < opsPerChange; k++) {
          const x = rnd(6)
          if (x === 0) d.map['k' + rnd(5)] = rnd(1000)
          else if (x === 1) d.list.push(rnd(100))
          else if (x === 2 && d.list.length) d.list.splice(rnd(d.list.length), 1)
          else if (x === 3) d.text.insertAt(rnd(d.text.length + 1), String.fromCharCode(97 + rnd(26)))
          else if (x === 4 && d.text.length) d.text.deleteAt(rnd(d.text.length))
          else d['f' + rnd(3)] = 'v' + rnd(9)
        }
      })
    }
    // some actors sync with a random other actor (DAG with merges and parallel branches)
    for (let i = 0; i < nactors; i++) if (rnd(3) === 0) docs[i] = Automerge.merge(docs[i], docs[rnd(nactors)])
  }
  let all = docs[0]
  for (let i = 1; i < nactors; i++) all = Automerge.merge(all, docs[i])
  return Automerge.save(all)
}

// ---- mutations of a saved document ----
function decodeDoc(buf) {
  const h = C.decodeDocumentHeader(buf)
  const cols = list => list.map(col => {
    if ((col.columnId & 7) === C.COLUMN_TYPE.VALUE_RAW) return {columnId: col.columnId, raw: col.buffer}
    const d = C.decoderByColumnId(col.columnId, col.buffer), values = []
    while (!d.done) values.push(d.readValue())
    return {columnId: col.columnId, values}
  })
  return {actorIds: h.actorIds, heads: h.heads, headsIndexes: h.headsIndexes, extraBytes: h.extraBytes,
          changes: cols(h.changesColumns), ops: cols(h.opsColumns)}
}
function encodeDoc(d) {
  const cols = list => list.map(col => {
    const enc = C.encoderByColumnId(col.columnId)
    if (col.raw) enc.appendRawBytes(col.raw)
    else for (const v of col.values) enc.appendValue(v)
    return {columnId: col.columnId, encoder: enc}
  })
  return C.encodeDocumentHeader({changesColumns: cols(d.changes), opsColumns: cols(d.ops), actorIds: d.actorIds,
                                 heads: d.heads.slice(), headsIndexes: d.headsIndexes, extraBytes: d.extraBytes})
}
const col = (list, id) => list.find(c => c.columnId === id)
const clone = x => JSON.parse(JSON.stringify(x, (k, v) => v instanceof Uint8Array ? {__u8: [...v]} : v),
                              (k, v) => v && v.__u8 ? Uint8Array.from(v.__u8) : v)

const cases = []
// valid concurrent histories
const valid = []
for (const [na, r, k] of [[2, 3, 2], [3, 4, 3], [4, 3, 4], [5, 2, 2], [6, 3, 5], [3, 8, 1], [8, 2, 3]]) {
  const doc = concurrent(na, r, k)
  valid.push(doc)
  cases.push(record(`concurrent ${na}x${r}x${k}`, doc))
}
// a round trip of the decode/encode helpers must reproduce the saved document's history
cases.push(record('re-encoded unchanged', encodeDoc(decodeDoc(valid[2]))))

const CH = {actor: 0x01, seq: 0x03, maxOp: 0x13, time: 0x23, message: 0x35, depsNum: 0x40, depsIndex: 0x43, extraLen: 0x56}
const OP = {idActor: 0x21, idCtr: 0x23, action: 0x42, succNum: 0x80}
function mutate(name, src, fn) {
  const d = clone(decodeDoc(src))
  if (fn(d) === false) return
  const c = record(name, encodeDoc(d))
  cases.push(c)
  // ops moved between changes (a maxOp edit) give a different but consistent history: the same
  // document with the heads the reference computed decodes without error
  const m = /^Mismatched heads hashes: expected .*, got (.*)$/.exec(c.direct_error || '')
  if (m && !name.startsWith('heads')) {
    d.heads = m[1].split(', ')
    cases.push(record(name + ' (heads fixed)', encodeDoc(d)))
  }
}
for (let v = 0; v < valid.length; v += 2) {
  const src = valid[v]
  mutate(`seq bumped #${v}`, src, d => { const s = col(d.changes, CH.seq).values; s[s.length - 1] += 1 })
  mutate(`seq of first change #${v}`, src, d => { col(d.changes, CH.seq).values[0] = 2 })
  mutate(`maxOp decreasing #${v}`, src, d => {
    const a = col(d.changes, CH.actor).values, m = col(d.changes, CH.maxOp).values
    for (let i = 1; i < a.length; i++) for (let j = 0; j < i; j++)
      if (a[i] === a[j]) { m[i] = m[j] - 1; return }
    return false
  })
  mutate(`del row #${v}`, src, d => { const act = col(d.ops, OP.action).values; act[act.length >> 1] = 3 })
  mutate(`maxOp of last change lowered #${v}`, src, d => { const m = col(d.changes, CH.maxOp).values; m[m.length - 1] -= 1 })
  mutate(`maxOp of first change raised #${v}`, src, d => { col(d.changes, CH.maxOp).values[0] += 1 })
  mutate(`depsIndex forward #${v}`, src, d => {
    const di = col(d.changes, CH.depsIndex)
    if (!di || !di.values.length) return false
    di.values[di.values.length - 1] = col(d.changes, CH.actor).values.length + 3
  })
  mutate(`depsIndex self #${v}`, src, d => {
    const dn = col(d.changes, CH.depsNum).values, di = col(d.changes, CH.depsIndex)
    if (!di) return false
    let p = 0
    for (let i = 0; i < dn.length; i++) { if (i > 0 && dn[i] > 0) { di.values[p] = i; return } p += dn[i] }
    return false
  })
  mutate(`heads wrong #${v}`, src, d => { d.heads = ['ab'.repeat(32)] })
  mutate(`heads missing #${v}`, src, d => { d.heads = [] })
  mutate(`extra datatype #${v}`, src, d => {
    const el = col(d.changes, CH.extraLen)
    if (!el) return false
    el.values[0] = 6
  })
  mutate(`actor of a change moved #${v}`, src, d => {
    const a = col(d.changes, CH.actor).values
    if (d.actorIds.length < 2) return false
    a[a.length - 1] = (a[a.length - 1] + 1) % d.actorIds.length
  })
  mutate(`op counter moved #${v}`, src, d => { const c = col(d.ops, OP.idCtr).values; c[c.length - 1] += 1000 })
}
fs.writeFileSync(OUT, JSON.stringify(cases) + '\n')
console.log('wrote', OUT, cases.length, 'cases:', cases.filter(c => c.error).length, 'history errors,',
            cases.filter(c => c.load_error).length, 'load errors')
