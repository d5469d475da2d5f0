'use strict'
/**
 * backend.js -- the Automerge Backend module on the MI355X engine.
 *
 * Same exports, argument meaning, state handles and error behaviour as the reference's
 * backend/backend.js:8-197 (+ util.js:1-10 frozen-state rule), so it loads through
 *   Automerge.setDefaultBackend(require('<repo>/automerge_amd/js/backend'))
 * (src/automerge.js:147-149). Document state lives in libautomerge_amd.so (the GPU engine) and
 * is reached through the N-API addon am_napi.node (am_napi.c); there is no JS or CPU fallback:
 * if the addon or the HIP device is missing, require() or the first call throws.
 *
 * Hash-graph queries (getChanges, getChangesAdded, getChangeByHash, getMissingDeps) are host
 * traversals over the applied change buffers, as in new.js:1913-2020.
 * getPatch runs documentPatch on the GPU, applyChanges replays the patch of the call on the GPU
 * (k_doc phase P8, am_diff.h); both logs are materialized here.
 * The change history of a loaded document is reconstructed from save() on first use
 * (computeHashGraph, new.js:1879-1904; am_document_changes, 8(f) row 2).
 * Not on the GPU path yet: applyLocalChange (8(f) row 3); it throws.
 */
const path = require('path')
const zlib = require('zlib')
const native = require(process.env.AM_NAPI_PATH || path.join(__dirname, 'am_napi.node'))

const FROZEN_MESSAGE =
  'Attempting to use an outdated Automerge document that has already been updated. ' +
  'Please use the latest document state, or call Automerge.clone() if you really ' +
  'need to use this old document state.'

function backendState(backend) {
  if (backend.frozen) throw new Error(FROZEN_MESSAGE)
  return backend.state
}

function init() {
  return {state: native.docInit(), heads: []}
}

function clone(backend) {
  return {state: native.docClone(backendState(backend)), heads: backend.heads}
}

// Only the latest handle owns the engine document; older (frozen) handles share it.
function free(backend) {
  if (!backend.frozen && backend.state) native.docFree(backend.state)
  backend.state = null
  backend.frozen = true
}

// Backend.applyChanges (backend.js:27-32, new.js:1796-1871): {maxOp, clock, deps, pendingChanges, diffs}
function applyChanges(backend, changes) {
  const state = backendState(backend)
  const log = native.docApplyChanges(state, changes, true)
  backend.frozen = true
  const heads = native.docHeads(state)
  const c = native.docCounts(state)
  return [{state, heads}, materializePatch(log, heads, c.pending, c.maxOp)]
}

function applyLocalChange(backend) {
  backendState(backend)
  throw new RangeError('automerge_amd: applyLocalChange is not implemented by this backend')
}

function save(backend) {
  return native.docSave(backendState(backend))
}

function load(data) {
  const state = native.docLoad(data)
  return {state, heads: native.docHeads(state)}
}

function loadChanges(backend, changes) {
  const state = backendState(backend)
  native.docApplyChanges(state, changes)
  backend.frozen = true
  return {state, heads: native.docHeads(state)}
}

// ---- getPatch: documentPatch runs on the GPU (k_doc phase P7, automerge_amd/csrc/am_patch.h); this
// turns its binary log into the patch object (new.js:2052-2060). Deserialization only: every
// merge decision was taken on the device.
const PR = {ACTOR: 1, CLOCK: 2, OBJ: 3, KEY: 4, PROP: 5, INSERT: 6, MULTI: 7, UPDATE: 8, REMOVE: 9}
const PV = {NULL: 1, FALSE: 2, TRUE: 3, STR: 4, UINT: 5, INT: 6, F64: 7, COUNTER: 8, TIMESTAMP: 9, BYTES: 10, CHILD: 11}
const NAMED_DT = {5: 'uint', 6: 'int', 7: 'float64', 8: 'counter', 9: 'timestamp'}
const OBJ_TYPES = ['map', 'list', 'text', 'table']
const utf8 = new TextDecoder('utf-8')

function materializePatch(log, deps, pendingChanges, maxOp) {
  const dv = new DataView(log.buffer, log.byteOffset, log.byteLength)
  const i64 = o => Number(dv.getBigInt64(o, true))
  const nrec = i64(24), nmval = i64(32), nheap = i64(40)
  const recAt = k => 64 + 64 * k, valAt = k => 64 + 64 * nrec + 32 * k
  const heapOff = 64 + 64 * nrec + 32 * nmval
  const heap = log.subarray(heapOff, heapOff + nheap)
  const actors = [], clock = {}, nodes = new Map()
  const opid = (c, a) => `${c}@${actors[a]}`
  const node = (c, a, t) => {
    const k = `${c}@${a}`
    let n = nodes.get(k)
    if (!n) {
      const type = OBJ_TYPES[t]
      n = (type === 'list' || type === 'text') ? {objectId: opid(c, a), type, edits: []} : {objectId: opid(c, a), type, props: {}}
      nodes.set(k, n)
    }
    return n
  }
  const prim = (vtag, dt, o) => {
    switch (vtag) {
      case PV.NULL: return null
      case PV.FALSE: return false
      case PV.TRUE: return true
      case PV.STR: return utf8.decode(heap.subarray(i64(o), i64(o) + i64(o + 8)))
      case PV.F64: return dv.getFloat64(o, true)
      case PV.BYTES: return heap.slice(i64(o), i64(o) + i64(o + 8))
      default: return i64(o)
    }
  }
  const value = (vtag, dt, o) => {
    if (vtag === PV.CHILD) return node(i64(o), i64(o + 8), dt)
    const v = {type: 'value', value: prim(vtag, dt, o)}
    if (NAMED_DT[vtag]) v.datatype = NAMED_DT[vtag]
    else if (vtag === PV.BYTES) v.datatype = dt
    return v
  }
  const root = {objectId: '_root', type: 'map', props: {}}
  let cur = root, key = null, mv = 0
  for (let k = 0; k < nrec; k++) {
    const r = recAt(k)
    const tag = dv.getUint32(r, true), vtag = dv.getUint32(r + 4, true)
    const index = i64(r + 8), c1 = i64(r + 16), c2 = i64(r + 24)
    const a1 = dv.getInt32(r + 32, true), a2 = dv.getInt32(r + 36, true)
    const dt = dv.getUint32(r + 56, true), n = dv.getUint32(r + 60, true)
    switch (tag) {
      case PR.ACTOR: actors.push(toHex(heap.subarray(i64(r + 40), i64(r + 40) + i64(r + 48)))); break
      case PR.CLOCK: clock[actors[a1]] = index; break
      // getPatch logs announce an object in its parent first; applyChanges logs list object
      // patches in objectMeta order, so a section may create its node
      case PR.OBJ: cur = a1 < 0 ? root : node(c1, a1, dt); break
      case PR.KEY: key = utf8.decode(heap.subarray(i64(r + 40), i64(r + 40) + i64(r + 48))); cur.props[key] = {}; break
      case PR.PROP: cur.props[key][opid(c2, a2)] = value(vtag, dt, r + 40); break
      case PR.INSERT:
        cur.edits.push({action: 'insert', index, elemId: opid(c1, a1), opId: opid(c2, a2), value: value(vtag, dt, r + 40)})
        break
      case PR.MULTI: {
        const e = {action: 'multi-insert', index, elemId: opid(c1, a1)}
        if (dt) e.datatype = dt < 100 ? NAMED_DT[PV.UINT + dt - 1] : dt - 100
        e.values = []
        for (let q = 0; q < n; q++, mv++) {
          const vo = valAt(mv)
          e.values.push(prim(dv.getUint32(vo, true), dv.getUint32(vo + 4, true), vo + 8))
        }
        cur.edits.push(e)
        break
      }
      case PR.UPDATE: cur.edits.push({action: 'update', index, opId: opid(c2, a2), value: value(vtag, dt, r + 40)}); break
      case PR.REMOVE: cur.edits.push({action: 'remove', index, count: n}); break
    }
  }
  return {maxOp, clock, deps, pendingChanges, diffs: root}
}

function getPatch(backend) {
  const state = backendState(backend)
  const log = native.docPatch(state)
  const c = native.docCounts(state)
  return materializePatch(log, native.docHeads(state), c.pending, c.maxOp)
}

function getHeads(backend) {
  return backend.heads
}

// ---- hash graph (host side) ----
function readUleb(buf, pos) {
  let v = 0, mul = 1, b
  do {
    b = buf[pos++]
    v += (b & 0x7f) * mul
    mul *= 128
  } while (b & 0x80)
  return [v, pos]
}

function toHex(bytes) {
  return Buffer.from(bytes.buffer, bytes.byteOffset, bytes.byteLength).toString('hex')
}

// dependency hashes of a change chunk (decodeChangeMeta, columnar.js:768-811)
function changeDeps(bytes) {
  const type = bytes[8]
  let [len, pos] = readUleb(bytes, 9)
  let body = bytes.subarray(pos, pos + len)
  if (type === 2) body = zlib.inflateRawSync(body)
  let [n, q] = readUleb(body, 0)
  const deps = []
  for (let i = 0; i < n; i++, q += 32) deps.push(toHex(body.subarray(q, q + 32)))
  return deps
}

function hashGraph(state) {
  const changes = native.docChanges(state)
  const index = {}, depsOf = {}, dependents = {}
  changes.forEach((c, i) => {
    index[c.hash] = i
    depsOf[c.hash] = changeDeps(c.bytes)
    dependents[c.hash] = []
  })
  for (const c of changes) {
    for (const d of depsOf[c.hash]) {
      if (!dependents[d]) dependents[d] = []
      dependents[d].push(c.hash)
    }
  }
  return {changes, index, depsOf, dependents, heads: native.docHeads(state)}
}

// BackendDoc.getChanges (new.js:1913-1966)
function getChanges(backend, haveDeps) {
  if (!Array.isArray(haveDeps)) {
    throw new TypeError('Pass an array of hashes to Backend.getChanges()')
  }
  const g = hashGraph(backendState(backend))
  if (haveDeps.length === 0) return g.changes.map(c => c.bytes)

  let stack = [], seen = {}, toReturn = []
  for (const hash of haveDeps) {
    seen[hash] = true
    const succ = g.dependents[hash]
    if (!succ) throw new RangeError(`hash not found: ${hash}`)
    stack.push(...succ)
  }
  while (stack.length > 0) {
    const hash = stack.pop()
    seen[hash] = true
    toReturn.push(hash)
    if (!g.depsOf[hash].every(dep => seen[dep])) break
    stack.push(...g.dependents[hash])
  }
  if (stack.length === 0 && g.heads.every(head => seen[head])) {
    return toReturn.map(hash => g.changes[g.index[hash]].bytes)
  }
  stack = haveDeps.slice()
  seen = {}
  while (stack.length > 0) {
    const hash = stack.pop()
    if (!seen[hash]) {
      const deps = g.depsOf[hash]
      if (!deps) throw new RangeError(`hash not found: ${hash}`)
      stack.push(...deps)
      seen[hash] = true
    }
  }
  return g.changes.filter(c => !seen[c.hash]).map(c => c.bytes)
}

function getAllChanges(backend) {
  return getChanges(backend, [])
}

// BackendDoc.getChangesAdded (new.js:1971-1988)
function getChangesAdded(backend1, backend2) {
  const other = hashGraph(backendState(backend1))
  const g = hashGraph(backendState(backend2))
  let stack = g.heads.slice(), seen = {}, toReturn = []
  while (stack.length > 0) {
    const hash = stack.pop()
    if (!seen[hash] && other.index[hash] === undefined) {
      seen[hash] = true
      toReturn.push(hash)
      stack.push(...g.depsOf[hash])
    }
  }
  return toReturn.reverse().map(hash => g.changes[g.index[hash]].bytes)
}

// BackendDoc.getChangeByHash (new.js:1990-1993)
function getChangeByHash(backend, hash) {
  const g = hashGraph(backendState(backend))
  const i = g.index[hash]
  return i === undefined ? undefined : g.changes[i].bytes
}

// BackendDoc.getMissingDeps (new.js:2005-2020)
function getMissingDeps(backend, heads = []) {
  const state = backendState(backend)
  const g = hashGraph(state)
  const queued = native.docQueued(state)
  const qhashes = queued.length ? native.changeHashes(queued) : []
  const allDeps = new Set(heads), inQueue = new Set()
  queued.forEach((bytes, i) => {
    inQueue.add(qhashes[i])
    for (const dep of changeDeps(bytes)) allDeps.add(dep)
  })
  const missing = []
  for (const hash of allDeps) {
    if (g.index[hash] === undefined && !inQueue.has(hash)) missing.push(hash)
  }
  return missing.sort()
}

module.exports = {
  init, clone, free, applyChanges, applyLocalChange, save, load, loadChanges, getPatch,
  getHeads, getAllChanges, getChanges, getChangesAdded, getChangeByHash, getMissingDeps,
  engineVersion: native.version,
  _materializePatch: materializePatch  // host stage of getPatch (exported for tests)
}
