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

// Wire form (am_patch.h): PatchHdr2 (48 B: magic, status, arg0, arg1, maxOp, nbytes, pad) + stream
function materializePatch(log, deps, pendingChanges, maxOp) {
  const dv = new DataView(log.buffer, log.byteOffset, log.byteLength)
  const end = 48 + Number(dv.getBigUint64(32, true))
  let o = 48
  const u = () => {
    let v = 0, mul = 1, b
    do { b = log[o++]; v += (b & 0x7f) * mul; mul *= 128 } while (b & 0x80)
    return v
  }
  const s = () => {
    let v = 0, mul = 1, b
    do { b = log[o++]; v += (b & 0x7f) * mul; mul *= 128 } while (b & 0x80)
    return (b & 0x40) ? v - mul : v
  }
  const raw = n => { const r = log.subarray(o, o + n); o += n; return r }
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
  // [vtag, datatype code, primitive] of the VALUE at the cursor
  const prim = () => {
    const vt = log[o++]
    switch (vt) {
      case PV.NULL: return [vt, 0, null]
      case PV.FALSE: return [vt, 0, false]
      case PV.TRUE: return [vt, 0, true]
      case PV.STR: return [vt, 0, utf8.decode(raw(u()))]
      case PV.UINT: return [vt, 0, u()]
      case PV.INT: case PV.COUNTER: case PV.TIMESTAMP: return [vt, 0, s()]
      case PV.F64: { const x = dv.getFloat64(o, true); o += 8; return [vt, 0, x] }
      case PV.BYTES: { const dt = u(); return [vt, dt, raw(u()).slice()] }
      case PV.CHILD: { const c = u(), a = u(), t = u(); return [vt, t, [c, a]] }
      default: throw new RangeError(`automerge_amd: bad patch value tag ${vt}`)
    }
  }
  const value = () => {
    const [vt, dt, x] = prim()
    if (vt === PV.CHILD) return node(x[0], x[1], dt)
    const v = {type: 'value', value: x}
    if (NAMED_DT[vt]) v.datatype = NAMED_DT[vt]
    else if (vt === PV.BYTES) v.datatype = dt
    return v
  }
  const root = {objectId: '_root', type: 'map', props: {}}
  let cur = root, key = null
  while (o < end) {
    const tag = log[o++]
    switch (tag) {
      case PR.ACTOR: actors.push(toHex(raw(u()))); break
      case PR.CLOCK: { const a = u(); clock[actors[a]] = u(); break }
      // getPatch logs announce an object in its parent first; applyChanges logs list object
      // patches in objectMeta order, so a section may create its node
      case PR.OBJ: { const c = s(), a = s(), t = u(); cur = a < 0 ? root : node(c, a, t); break }
      case PR.KEY: key = utf8.decode(raw(u())); cur.props[key] = {}; break
      case PR.PROP: { const c = u(), a = u(); cur.props[key][opid(c, a)] = value(); break }
      case PR.INSERT: {
        const index = u(), ec = u(), ea = u(), oc = u(), oa = u()
        cur.edits.push({action: 'insert', index, elemId: opid(ec, ea), opId: opid(oc, oa), value: value()})
        break
      }
      case PR.MULTI: {
        const index = u(), ec = u(), ea = u(), dt = u(), n = u()
        const e = {action: 'multi-insert', index, elemId: opid(ec, ea)}
        if (dt) e.datatype = dt < 100 ? NAMED_DT[PV.UINT + dt - 1] : dt - 100
        e.values = []
        for (let q = 0; q < n; q++) e.values.push(prim()[2])
        cur.edits.push(e)
        break
      }
      case PR.UPDATE: { const index = u(), oc = u(), oa = u(); cur.edits.push({action: 'update', index, opId: opid(oc, oa), value: value()}); break }
      case PR.REMOVE: { const index = u(); cur.edits.push({action: 'remove', index, count: u()}); break }
      default: throw new RangeError(`automerge_amd: bad patch record tag ${tag}`)
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
