// Golden vectors for the objectMeta the reference carries across applyChanges calls on one handle
// (new.js:884-931 updatePatchProperty's children snapshot, 1461-1528 setupPatches, 1812/1857 the
// per-handle objectMeta). Two to four actors create an object under the same root key concurrently,
// most of them touching other root keys in the same change; later changes edit inside the
// objects, create new ones over them, or set the key to a plain value. The merged histories are
// then delivered to one backend handle in several applyChanges calls, so a patch of a later call
// reads the parent key's conflicts from whatever snapshot an earlier call left.
// Output: tests/golden/objmeta.json, the docs.json scenario format (steps + per-step results).
//   NODE_PATH=tests/golden/gen/node_modules node tests/golden/gen/make_objmeta.js
// Seeded; a re-run reproduces the committed file byte for byte.
'use strict'
const fs = require('fs')
const path = require('path')
const REF = process.env.AM_REF || '/root/reference'
const OUT = path.join(__dirname, '..')
const Automerge = require(path.join(REF, 'src/automerge'))
const F = require('./make_fixtures')
const {lcg, runBackend, jsonPatch, hex, randomActor, randomValue, safeChange, changeHash} = F

const CKEYS = ['items', 'm', 'list', 'obj']
const OKEYS = ['a', 'b', 'title', 'z', 'zz', 'items2', 'l']

function makeObj(r, kind) {
  if (kind === 0) return []
  if (kind === 1) return {}
  return new Automerge.Text()
}

// an edit inside whatever the actor currently sees under `key`
function editInside(r, d, key) {
  const o = d[key]
  if (o instanceof Automerge.Text) {
    if (o.length && r() % 3 === 0) o.deleteAt(r() % o.length)
    else o.insertAt(r() % (o.length + 1), String.fromCharCode(97 + r() % 26))
  } else if (Array.isArray(o)) {
    const x = r() % 5
    if (x === 0 && o.length) o.deleteAt(r() % o.length)
    else if (x === 1 && o.length) o[r() % o.length] = r() % 100
    else if (x === 2) o.insertAt(r() % (o.length + 1), {n: r() % 9})
    else o.insertAt(r() % (o.length + 1), r() % 1000)
  } else if (o && typeof o === 'object') {
    const k = 'p' + r() % 4
    if (r() % 4 === 0) o[k] = {q: r() % 7}
    else if (r() % 5 === 0 && o[k] !== undefined) delete o[k]
    else o[k] = r() % 1000
  } else {
    d[key] = makeObj(r, r() % 3)
  }
}

function session(r, d, ck) {
  const n = 1 + r() % 3
  for (let i = 0; i < n; i++) {
    const x = r() % 10
    if (x < 5) editInside(r, d, ck)
    else if (x < 8) d[OKEYS[r() % OKEYS.length]] = randomValue(r)
    else if (x === 8) d[ck] = makeObj(r, r() % 3)           // a new object over the key
    else if (x === 9 && r() % 2) d[ck] = r() % 50           // a plain value over the key
    else d[OKEYS[r() % OKEYS.length]] = makeObj(r, r() % 3)  // another key with a child object
  }
}

function allChanges(docs) {
  const seen = new Set(), out = []
  for (const d of docs) for (const c of Automerge.getAllChanges(d)) {
    const h = changeHash(c)
    if (!seen.has(h)) { seen.add(h); out.push(c) }
  }
  return out
}

// delivery of `changes` in calls of 1..maxPer changes; with `shuffle` a call may hold changes
// whose dependencies come later (the reference queues them)
function chunked(r, changes, maxPer, shuffle) {
  const order = changes.slice()
  if (shuffle) for (let i = order.length - 1; i > 0; i--) { if (r() % 3) continue; const j = Math.max(0, i - 1 - r() % 3); [order[i], order[j]] = [order[j], order[i]] }
  const steps = []
  for (let i = 0; i < order.length;) {
    const n = 1 + r() % maxPer
    steps.push({op: 'apply', changes: order.slice(i, i + n)})
    i += n
  }
  return steps
}

function randomScenarios(count, seed) {
  const r = lcg(seed)
  const out = []
  for (let s = 0; s < count; s++) {
    const nA = 2 + r() % 3
    const actors = []
    while (actors.length < nA) { const a = randomActor(r); if (!actors.includes(a)) actors.push(a) }
    const ck = CKEYS[r() % CKEYS.length]
    // optional shared prefix (plain root keys only)
    let base = Automerge.init(actors[0])
    const shared = r() % 2
    if (shared) base = safeChange(base, {time: 0}, d => { d[OKEYS[r() % OKEYS.length]] = r() % 10 })
    const docs = actors.map((a, i) => i === 0 ? base : Automerge.merge(Automerge.init(a), base))
    // every actor creates the object under the same key, most also set other root keys
    for (let i = 0; i < nA; i++) {
      docs[i] = safeChange(docs[i], {time: 0}, d => {
        const pre = r() % 3
        for (let q = 0; q < pre; q++) d[OKEYS[r() % OKEYS.length]] = r() % 100
        d[ck] = makeObj(r, r() % 3)
        if (r() % 2) editInside(r, d, ck)
        const post = r() % 3
        for (let q = 0; q < post; q++) d[OKEYS[r() % OKEYS.length]] = 'v' + r() % 100
      })
    }
    for (let round = 0; round < 2 + r() % 3; round++) {
      for (let i = 0; i < nA; i++) if (r() % 3) docs[i] = safeChange(docs[i], {time: 0}, d => session(r, d, ck))
      const i = r() % nA, j = r() % nA
      if (i !== j) docs[i] = Automerge.merge(docs[i], docs[j])
    }
    // after a full merge, edits inside the conflicted objects
    const all = docs.reduce((acc, d) => Automerge.merge(acc, d), Automerge.init('ffff'))
    for (let i = 0; i < nA; i++) {
      if (r() % 2) docs[i] = Automerge.merge(docs[i], all)
      docs[i] = safeChange(docs[i], {time: 0}, d => { editInside(r, d, ck); if (r() % 2) editInside(r, d, ck) })
    }
    const changes = allChanges(docs)
    const name = `objmeta${seed}-${s}`
    const steps1 = chunked(r, changes, 3, false)
    out.push({name: name + '/steps', steps: steps1})
    const steps2 = chunked(r, changes, 4, true)
    out.push({name: name + '/shuffled', steps: steps2})
    // load a prefix, then the rest in calls
    const cut = 1 + r() % Math.max(1, changes.length - 1)
    const pre = Automerge.Backend.applyChanges(Automerge.Backend.init(), changes.slice(0, cut))[0]
    const bytes = Automerge.Backend.save(pre)
    out.push({name: name + '/load', steps: [{op: 'load', bytes}].concat(chunked(r, changes.slice(cut), 2, false))})
  }
  return out
}

// The two-actor case of DESIGN.md §1 by hand: peer B creates `items` and sets `z` in one change;
// A (the higher actor) created `items` too; B's change arrives in its own call, then a change
// inside either object.
function handScenarios() {
  const out = []
  const A = 'bbbbbbbb', B = 'aaaaaaaa'
  for (const [ka, kb, name] of [[0, 0, 'list-list'], [1, 0, 'map-list'], [2, 2, 'text-text'], [0, 1, 'list-map']]) {
    let a = Automerge.change(Automerge.init(A), {time: 0}, d => { d.items = makeObj(null, ka) })
    let b = Automerge.change(Automerge.init(B), {time: 0}, d => { d.a = 1; d.items = makeObj(null, kb); d.z = 'x' })
    const ab = Automerge.merge(Automerge.merge(Automerge.init('cccccccc'), a), b)
    let a2 = Automerge.merge(Automerge.clone(a), b)
    a2 = Automerge.change(a2, {time: 0}, d => {
      if (d.items instanceof Automerge.Text) d.items.insertAt(0, 'q')
      else if (Array.isArray(d.items)) d.items.push(7)
      else d.items.k = 7
    })
    let b2 = Automerge.merge(Automerge.clone(b), a)
    b2 = Automerge.change(b2, {time: 0}, d => { d.z = 'y'; d.b = 2 })
    const ca = Automerge.getAllChanges(a), cb = Automerge.getAllChanges(b)
    const extra = Automerge.getChanges(a, a2).concat(Automerge.getChanges(b, b2))
    out.push({name: 'hand/' + name + '/A-then-B', steps: [{op: 'apply', changes: ca}, {op: 'apply', changes: cb},
      {op: 'apply', changes: extra}]})
    out.push({name: 'hand/' + name + '/B-then-A', steps: [{op: 'apply', changes: cb}, {op: 'apply', changes: ca},
      {op: 'apply', changes: extra}]})
    out.push({name: 'hand/' + name + '/one-by-one', steps: ca.concat(cb, extra).map(c => ({op: 'apply', changes: [c]}))})
    out.push({name: 'hand/' + name + '/load', steps: [{op: 'load', bytes: Automerge.save(a)}, {op: 'apply', changes: cb},
      {op: 'apply', changes: extra}]})
    void ab
  }
  return out
}

// One change touching several root keys in ascending order is one mergeDocChangeOps call: a doc op
// of an earlier key with a greater opId than the change's op of that key is taken without
// updatePatchProperty once the call has moved on to the later key (new.js:1125-1128, 1225-1230);
// counter increments of concurrent changes, in both actor orders (new.js:937-965).
function multiKeyScenarios() {
  const col = require(path.join(REF, 'backend/columnar'))
  const H = c => col.decodeChangeMeta(col.encodeChange(c), true).hash
  const out = []
  const set = (key, value, pred, datatype = 'uint') => ({action: 'set', obj: '_root', key, datatype, value, pred})
  const inc = (key, value, pred) => ({action: 'inc', obj: '_root', key, datatype: 'int', value, pred})
  for (const [a, b] of [['aa', 'bb'], ['bb', 'aa']]) {
    const c0 = {actor: '01', seq: 1, startOp: 1, time: 0, deps: [], ops: [set('a', 1, []), set('cnt', 5, [], 'counter'), set('k1', 1, [])]}
    const X = {actor: a, seq: 1, startOp: 4, time: 0, deps: [H(c0)], ops: [set('a', 2, ['1@01']), set('b', 3, [])]}
    const Y = {actor: b, seq: 1, startOp: 4, time: 0, deps: [H(c0)], ops: [set('a', 4, ['1@01'])]}
    const A = {actor: a, seq: 1, startOp: 4, time: 0, deps: [H(c0)], ops: [inc('cnt', 2, ['2@01']), set('k1', 2, ['3@01'])]}
    const B = {actor: b, seq: 1, startOp: 4, time: 0, deps: [H(c0)], ops: [inc('cnt', 3, ['2@01']), set('k1', 3, ['3@01'])]}
    const B2 = {actor: b, seq: 2, startOp: 6, time: 0, deps: [H(B)], ops: [inc('cnt', 7, ['2@01']), set('z', 1, [])]}
    const e = cs => cs.map(c => col.encodeChange(c))
    const saved = cs => Backend.save(Backend.applyChanges(Backend.init(), e(cs))[0])
    const tag = a + b
    out.push({name: `multikey/${tag}/one-call`, steps: [{op: 'apply', changes: e([c0, Y, X])}]})
    out.push({name: `multikey/${tag}/load+apply`, steps: [{op: 'load', bytes: saved([c0, Y])}, {op: 'apply', changes: e([X])}]})
    out.push({name: `counter/${tag}/one-call`, steps: [{op: 'apply', changes: e([c0, A, B])}]})
    out.push({name: `counter/${tag}/load+apply`, steps: [{op: 'load', bytes: saved([c0, A])}, {op: 'apply', changes: e([B])}]})
    out.push({name: `counter/${tag}/load+apply2`, steps: [{op: 'load', bytes: saved([c0, A])}, {op: 'apply', changes: e([B, B2])}]})
    out.push({name: `counter/${tag}/steps`, steps: [{op: 'apply', changes: e([c0])}, {op: 'apply', changes: e([B])},
      {op: 'apply', changes: e([A, B2])}]})
  }
  return out
}
const Backend = require(path.join(REF, 'backend'))

function record(sc) {
  return {name: sc.name,
          steps: sc.steps.map(s => s.op === 'load' ? {op: 'load', bytes: hex(s.bytes)} : {op: 'apply', changes: s.changes.map(hex)}),
          results: runBackend(sc.steps).map(jsonPatch)}
}

function main() {
  const scen = handScenarios().concat(multiKeyScenarios(), randomScenarios(40, 7001)).map(record)
  const file = path.join(OUT, 'objmeta.json')
  fs.writeFileSync(file, JSON.stringify({scenarios: scen}) + '\n')
  const steps = scen.reduce((a, s) => a + s.results.length, 0)
  const errs = scen.filter(s => s.results.some(x => x.error)).length
  console.log('wrote objmeta.json', fs.statSync(file).size, 'bytes,', scen.length, 'scenarios,', steps, 'steps,', errs, 'ending in an error')
}

main()
