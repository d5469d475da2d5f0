// Backend-boundary recorder. Runs test files of the reference (test/sync_test.js, backend_test.js,
// test.js, text_test.js, table_test.js) under a minimal describe/it harness with the reference's
// Backend module replaced by a recorder that forwards every call to the real reference backend and
// logs (function, arguments, result or error). The logs are the golden vectors for the 22
// Backend exports of backend/index.js: tests/js/backend_log_replay.js replays each call against
// automerge_amd/js/backend.js and compares every result.
//   NODE_PATH=tests/golden/gen/node_modules node tests/golden/gen/make_backend_log.js
// AM_LOG_FILES=sync_random AM_LOG_MAX=4000 records the randomized sync sessions instead
// (backend_log_sync_random.json); AM_LOG_FILES=objmeta AM_LOG_MAX=4000 the concurrent-object sessions
// (backend_log_objmeta.json).
// Clock and randomness are pinned (Date without arguments = epoch, seeded randomBytes and
// Math.random), so a re-run reproduces the committed tests/golden/backend_log_*.json byte for byte.
'use strict'
const fs = require('fs')
const path = require('path')
const crypto = require('crypto')
const assert = require('assert')
const REF = process.env.AM_REF || '/root/reference'
const OUT = path.join(__dirname, '..')

// ---- pinned clock and randomness ----
let seed = 0x2545f491
crypto.randomBytes = n => {
  const b = Buffer.alloc(n)
  for (let i = 0; i < n; i++) { seed = (Math.imul(seed, 1664525) + 1013904223) >>> 0; b[i] = seed >>> 24 }
  return b
}
let mseed = 0x9e3779b9
Math.random = () => { mseed = (Math.imul(mseed, 1664525) + 1013904223) >>> 0; return mseed / 4294967296 }
const RealDate = Date
global.Date = class extends RealDate {
  constructor(...a) { if (a.length) super(...a); else super(0) }
  static now() { return 0 }
}

// ---- value encoding shared with the replay (canonical JSON) ----
function canon(x, handleId) {
  if (x === undefined) return {__undef: 1}
  if (typeof x === 'number') {
    if (!Number.isFinite(x) || Object.is(x, -0)) return {__f64: Object.is(x, -0) ? '-0' : String(x)}
    return x
  }
  if (x instanceof Uint8Array) return {__bytes: Buffer.from(x.buffer, x.byteOffset, x.byteLength).toString('hex')}
  if (ArrayBuffer.isView(x)) return {__view: Buffer.from(x.buffer).toString('hex')}
  if (Array.isArray(x)) return x.map(v => canon(v, handleId))
  if (x && typeof x === 'object') {
    if (handleId) { const id = handleId(x); if (id !== null) return {$h: id} }
    const o = {}
    for (const k of Object.keys(x).sort()) o[k] = canon(x[k], handleId)
    return o
  }
  return x
}

// ---- the recorder ----
const realPath = require.resolve(path.join(REF, 'backend'))
const Real = require(realPath)
let handles = new Map(), nextHandle = 0, log = null, calls = 0
const isHandle = x => x && typeof x === 'object' && 'state' in x && ('heads' in x)
const handleId = x => {
  if (!isHandle(x)) return null
  if (!handles.has(x)) handles.set(x, nextHandle++)
  return handles.get(x)
}
const recorder = {}
for (const name of Object.keys(Real)) {
  recorder[name] = function (...args) {
    const entry = {fn: name, args: canon(args, handleId)}
    if (log) log.push(entry)
    calls++
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
require.cache[realPath].exports = recorder

const Automerge = require(path.join(REF, 'src/automerge'))
assert.strictEqual(Automerge.Backend, recorder)

// ---- a minimal describe/it harness ----
function harness(file) {
  const tests = []
  const stack = [{name: '', beforeEach: [], afterEach: []}]
  const g = global
  g.describe = (name, fn) => {
    stack.push({name, beforeEach: [], afterEach: []})
    fn()
    stack.pop()
  }
  g.describe.skip = () => {}
  g.describe.only = g.describe
  g.context = g.describe
  g.it = (name, fn) => tests.push({name: stack.map(s => s.name).filter(Boolean).concat(name).join(' / '),
                                    fn, before: stack.flatMap(s => s.beforeEach), after: stack.flatMap(s => s.afterEach)})
  g.it.skip = () => {}
  g.it.only = g.it
  g.beforeEach = fn => stack[stack.length - 1].beforeEach.push(fn)
  g.afterEach = fn => stack[stack.length - 1].afterEach.push(fn)
  g.before = fn => fn()
  g.after = () => {}
  require(path.join(REF, 'test', file))
  return tests
}

// ---- randomized sync sessions (getChangesToSend, sync.js:246-306, and the protocol around it) ----
// Two peers with a shared prefix and divergent histories (map sets, list inserts/deletes, text),
// synced with the reference's own generateSyncMessage / receiveSyncMessage until both stop sending;
// some sessions edit while syncing, some reconnect midway with a persisted sync state
// (encodeSyncState / decodeSyncState keep lastSync only), large histories make the Bloom filters
// report false positives that the `need` round trip repairs (sync.js:246-306, 327-473).
function randomSyncTests() {
  const tests = []
  let s = 0x5eed
  const rnd = n => { s = (Math.imul(s, 1103515245) + 12345) >>> 0; return (s >>> 8) % n }
  const edit = (doc, k) => Automerge.change(doc, {time: 0}, d => {
    if (!d.list) { d.list = []; d.text = new Automerge.Text(); d.map = {} }
    for (let q = 0; q < 1 + rnd(4); q++) {
      const x = rnd(5)
      if (x === 0) d.map['k' + rnd(6)] = rnd(1000)
      else if (x === 1) d.list.push(k * 100 + q)
      else if (x === 2 && d.list.length) d.list.splice(rnd(d.list.length), 1)
      else if (x === 3) d.text.insertAt(rnd(d.text.length + 1), String.fromCharCode(97 + rnd(26)))
      else if (d.text.length) d.text.deleteAt(rnd(d.text.length))
    }
  })
  for (let k = 0; k < 36; k++) {
    tests.push({name: 'random sync session ' + k, before: [], after: [], fn: () => {
      const big = k % 6 === 5
      // shared = 0: both peers create the list / text / map objects concurrently, so later patches
      // read the root keys' conflicts from the objectMeta.children snapshots earlier calls left
      // (new.js:884-931, 1461-1528)
      const shared = rnd(3) ? rnd(big ? 60 : 15) : 0
      const na = rnd(big ? 150 : 12), nb = rnd(big ? 150 : 12)
      let a = Automerge.init((0xa000 + k).toString(16) + 'aa'), b = Automerge.init((0xb000 + k).toString(16) + 'bb')
      for (let i = 0; i < shared; i++) a = edit(a, i)
      b = Automerge.merge(b, a)
      for (let i = 0; i < na; i++) a = edit(a, 1000 + i)
      for (let i = 0; i < nb; i++) b = edit(b, 2000 + i)
      let sa = Automerge.initSyncState(), sb = Automerge.initSyncState()
      const concurrent = k % 4 === 1, reconnect = k % 4 === 2
      for (let round = 0; round < 40; round++) {
        let msg, sent = false;
        [sa, msg] = Automerge.generateSyncMessage(a, sa)
        if (msg) { sent = true; [b, sb] = Automerge.receiveSyncMessage(b, sb, msg) }
        [sb, msg] = Automerge.generateSyncMessage(b, sb)
        if (msg) { sent = true; [a, sa] = Automerge.receiveSyncMessage(a, sa, msg) }
        if (concurrent && round < 3) { a = edit(a, 3000 + round); b = edit(b, 4000 + round) }
        if (reconnect && round === 1) {
          sa = Automerge.Backend.decodeSyncState(Automerge.Backend.encodeSyncState(sa))
          sb = Automerge.Backend.decodeSyncState(Automerge.Backend.encodeSyncState(sb))
        }
        if (!sent && !(concurrent && round < 3)) break
      }
      const heads = d => Automerge.Backend.getHeads(Automerge.Frontend.getBackendState(d))
      assert.deepStrictEqual(heads(a), heads(b))
    }})
  }
  return tests
}

// ---- concurrent objects under one root key (objectMeta carried across calls, new.js:884-931,
// 1461-1528, 1812/1857) ----
// Two to four peers each create `items` (list, map or text) in their first change, most of them
// also setting other root keys; they exchange changes a few at a time (Automerge.applyChanges of
// getChanges, so every delivery is one Backend.applyChanges call on the receiving handle), edit
// inside whichever object wins for them, and end with a full merge and more edits inside.
function objmetaTests() {
  const tests = []
  let s = 0x0b1e
  const rnd = n => { s = (Math.imul(s, 1103515245) + 12345) >>> 0; return (s >>> 8) % n }
  const mk = k => k === 0 ? [] : k === 1 ? {} : new Automerge.Text()
  const inside = (d) => {
    const o = d.items
    if (o instanceof Automerge.Text) o.insertAt(rnd(o.length + 1), String.fromCharCode(97 + rnd(26)))
    else if (Array.isArray(o)) { if (o.length && rnd(4) === 0) o.deleteAt(rnd(o.length)); else o.insertAt(rnd(o.length + 1), rnd(100)) }
    else if (o && typeof o === 'object') o['p' + rnd(3)] = rnd(100)
    else d.items = mk(rnd(3))
  }
  const keys = ['a', 'b', 'title', 'z']
  for (let k = 0; k < 24; k++) {
    tests.push({name: 'objmeta session ' + k, before: [], after: [], fn: () => {
      const n = 2 + rnd(3)
      let docs = []
      for (let i = 0; i < n; i++) docs.push(Automerge.init((0xc000 + 16 * k + i).toString(16) + 'cc'))
      docs = docs.map(d => Automerge.change(d, {time: 0}, x => {
        for (let q = rnd(3); q > 0; q--) x[keys[rnd(4)]] = rnd(50)
        x.items = mk(rnd(3))
        for (let q = rnd(3); q > 0; q--) x[keys[rnd(4)]] = 'v' + rnd(50)
      }))
      for (let round = 0; round < 4; round++) {
        for (let i = 0; i < n; i++) {
          if (rnd(2)) docs[i] = Automerge.change(docs[i], {time: 0}, x => { inside(x); if (rnd(3) === 0) x[keys[rnd(4)]] = rnd(9) })
          const j = rnd(n)
          if (j !== i) {
            const bs = d => Automerge.Frontend.getBackendState(d)
            const missing = Automerge.Backend.getChangesAdded(bs(docs[i]), bs(docs[j]))
            const cut = 1 + rnd(Math.max(1, missing.length))
            docs[i] = Automerge.applyChanges(docs[i], missing.slice(0, cut))[0]
            if (cut < missing.length) docs[i] = Automerge.applyChanges(docs[i], missing.slice(cut))[0]
          }
        }
      }
      for (let i = 1; i < n; i++) docs[0] = Automerge.merge(docs[0], docs[i])
      for (let i = 1; i < n; i++) docs[i] = Automerge.merge(docs[i], docs[0])
      for (let i = 0; i < n; i++) docs[i] = Automerge.change(docs[i], {time: 0}, inside)
    }})
  }
  return tests
}

const MAX_ENTRIES = +(process.env.AM_LOG_MAX || 400)
function run(file) {
  const scenarios = []
  let passed = 0, failed = 0, skipped = 0
  for (const t of (file === 'sync_random' ? randomSyncTests() : file === 'objmeta' ? objmetaTests() : harness(file))) {
    if (t.fn.length > 0) { skipped++; continue }  // callback-style tests
    handles = new Map()
    nextHandle = 0
    log = []
    let ok = true
    try {
      for (const b of t.before) b()
      const r = t.fn()
      if (r && typeof r.then === 'function') { skipped++; log = null; continue }
      for (const a of t.after) a()
    } catch (e) {
      ok = false
      if (process.env.AM_LOG_DEBUG) console.log(t.name, e.stack)
    }
    if (ok) passed++; else failed++
    if (ok && log.length > 0 && log.length <= MAX_ENTRIES) scenarios.push({name: t.name, log})
    log = null
  }
  return {file, passed, failed, skipped, scenarios}
}

const files = (process.env.AM_LOG_FILES || 'sync_test.js,backend_test.js,test.js,text_test.js,table_test.js').split(',')
for (const f of files) {
  const r = run(f)
  const name = 'backend_log_' + f.replace(/_test\.js$|\.js$/, '') + '.json'
  fs.writeFileSync(path.join(OUT, name), JSON.stringify(r) + '\n')
  const n = r.scenarios.reduce((a, s) => a + s.log.length, 0)
  console.log(`${f}: ${r.passed} passed, ${r.failed} failed, ${r.skipped} skipped; ${r.scenarios.length} scenarios, ${n} calls -> ${name}`)
}
