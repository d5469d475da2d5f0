// Golden vectors of the reference's BackendDoc tests (test/new_backend_test.js): every BackendDoc the
// tests construct is replaced by a recording subclass, which logs each applyChanges / getPatch call
// with its arguments and the reference's patch (or thrown error), and after every successful
// applyChanges the document's save() bytes and heads. checkColumns() in the tests asserts the op
// columns of block 0; save() concatenates and re-encodes those same columns, so the recorded bytes
// pin them (and the multi-block cases too). Replayed by tests/newbackend_log.py through
// automerge_amd.backend (init/load/applyChanges/getPatch/save/getHeads) on the GPU.
//   NODE_PATH=tests/golden/gen/node_modules node tests/golden/gen/make_newbackend_log.js
// uuid() in the tests draws from crypto.randomBytes, which is seeded here so a re-run reproduces
// tests/golden/newbackend_log.json byte for byte.
'use strict'
const fs = require('fs')
const path = require('path')
const crypto = require('crypto')
const REF = process.env.AM_REF || '/root/reference'
const OUT = path.join(__dirname, '..', 'newbackend_log.json')

let seed = 0x1b873593
crypto.randomBytes = n => {
  const b = Buffer.alloc(n)
  for (let i = 0; i < n; i++) { seed = (Math.imul(seed, 1664525) + 1013904223) >>> 0; b[i] = seed >>> 24 }
  return b
}

const hex = u8 => Buffer.from(u8.buffer, u8.byteOffset, u8.byteLength).toString('hex')
function canon(x) {
  if (x instanceof Uint8Array) return {__bytes: hex(x)}
  if (Array.isArray(x)) return x.map(canon)
  if (x && typeof x === 'object') {
    const o = {}
    for (const k of Object.keys(x).sort()) o[k] = canon(x[k])
    return o
  }
  return x
}

const newPath = require.resolve(path.join(REF, 'backend', 'new'))
const New = require(newPath)
const Real = New.BackendDoc
let log = null, nextId = 0
class RecordingDoc extends Real {
  constructor(buffer) {
    super(buffer)
    this.__id = nextId++
    if (log) log.push({fn: 'new', doc: this.__id, args: buffer ? [{__bytes: hex(buffer)}] : []})
  }
  applyChanges(changes, isLocal) {
    const e = {fn: 'applyChanges', doc: this.__id, args: [changes.map(c => ({__bytes: hex(c)}))]}
    if (isLocal) e.local = true
    if (log) log.push(e)
    try {
      const r = super.applyChanges(changes, isLocal)
      e.result = canon(r)
      e.save = hex(super.save())
      e.heads = this.heads.slice()
      return r
    } catch (err) {
      e.error = {name: err.constructor.name, message: err.message}
      throw err
    }
  }
  getPatch() {
    const e = {fn: 'getPatch', doc: this.__id, args: []}
    if (log) log.push(e)
    const r = super.getPatch()
    e.result = canon(r)
    return r
  }
}
require.cache[newPath].exports = Object.assign({}, New, {BackendDoc: RecordingDoc})

const tests = []
const stack = []
global.describe = (name, fn) => { stack.push(name); fn(); stack.pop() }
global.it = (name, fn) => tests.push({name: stack.concat(name).join(' / '), fn})
global.describe.skip = global.it.skip = () => {}
global.beforeEach = global.afterEach = () => {}
require(path.join(REF, 'test', 'new_backend_test.js'))

const scenarios = []
let passed = 0, failed = 0
for (const t of tests) {
  log = []
  nextId = 0
  try { t.fn(); passed++ } catch (e) { failed++; console.log('FAILED', t.name, e.message); log = null; continue }
  scenarios.push({name: t.name, log})
  log = null
}
fs.writeFileSync(OUT, JSON.stringify({file: 'test/new_backend_test.js', passed, failed, scenarios}) + '\n')
const n = scenarios.reduce((a, s) => a + s.log.length, 0)
console.log(`new_backend_test.js: ${passed} passed, ${failed} failed; ${scenarios.length} scenarios, ${n} calls -> ${OUT}`)
