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
 * Hash-graph queries (getChanges, getChangesAdded, getChangeByHash, getMissingDeps) run in the
 * engine over the document's change graph (am_graph.cpp, new.js:1913-2020); applyLocalChange
 * encodes the request (am_local.cpp, columnar.js:710-739) and applies it on the GPU; the seven sync
 * functions of backend/index.js run the protocol of sync.js in the engine (am_sync_proto.cpp), with
 * Bloom filters and change selection in HIP kernels (am_sync.hip).
 * getPatch runs documentPatch on the GPU, applyChanges replays the patch of the call on the GPU
 * (k_doc phase P8, am_diff.h); both logs are materialized here.
 * The change history of a loaded document is reconstructed from save() on first use
 * (computeHashGraph, new.js:1879-1904; am_document_changes, 8(f) row 2).
 */
const path = require('path')
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
const OBJ_TYPES = ['map', 'list', 'text', 'table', undefined, null]  // 4: null action, 5: unknown even action
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

function toHex(bytes) {
  return Buffer.from(bytes.buffer, bytes.byteOffset, bytes.byteLength).toString('hex')
}

// ---- hashes across the addon: hex strings <-> one flat Uint8Array of 32-byte hashes ----
const HASH_RE = /^[0-9a-f]{64}$/
// A string that is not a hash can never be found; it travels as a sentinel the engine does not
// know (0xff x 28 + its index) and is mapped back where a result or an error names it.
function flatHashes(list) {
  const out = new Uint8Array(32 * list.length), odd = new Map()
  list.forEach((h, i) => {
    if (typeof h === 'string' && HASH_RE.test(h)) out.set(Buffer.from(h, 'hex'), 32 * i)
    else {
      out.fill(0xff, 32 * i, 32 * i + 28)
      new DataView(out.buffer).setUint32(32 * i + 28, i)
      odd.set(toHex(out.subarray(32 * i, 32 * i + 32)), h)
    }
  })
  return [out, odd]
}
const hexList = flat => { const r = []; for (let i = 0; i < flat.length; i += 32) r.push(toHex(flat.subarray(i, i + 32))); return r }
function rethrowNamed(e, odd) {
  for (const [k, v] of odd) if (e.message.includes(k)) e.message = e.message.replace(k, String(v))
  throw e
}

// BackendDoc.getChanges (new.js:1913-1966): the traversal runs in the engine (am_doc_get_changes)
function getChanges(backend, haveDeps) {
  if (!Array.isArray(haveDeps)) {
    throw new TypeError('Pass an array of hashes to Backend.getChanges()')
  }
  const [flat, odd] = flatHashes(haveDeps)
  try { return native.docGetChanges(backendState(backend), flat) } catch (e) { rethrowNamed(e, odd) }
}

function getAllChanges(backend) {
  return getChanges(backend, [])
}

// BackendDoc.getChangesAdded (new.js:1971-1988): changes of backend2 that backend1 lacks
function getChangesAdded(backend1, backend2) {
  return native.docGetChangesAdded(backendState(backend1), backendState(backend2))
}

// BackendDoc.getChangeByHash (new.js:1990-1993)
function getChangeByHash(backend, hash) {
  const state = backendState(backend)
  if (typeof hash !== 'string' || !HASH_RE.test(hash)) return undefined
  return native.docChangeByHash(state, Buffer.from(hash, 'hex'))
}

// BackendDoc.getMissingDeps (new.js:2005-2020)
function getMissingDeps(backend, heads = []) {
  const state = backendState(backend)
  const [flat, odd] = flatHashes(Array.from(heads))
  const missing = hexList(native.docMissingDeps(state, flat)).map(h => odd.has(h) ? odd.get(h) : h)
  return odd.size ? missing.sort() : missing
}

// ---- applyLocalChange (backend.js:54-91): encodeChange + applyChanges(isLocal) in the engine ----
// Uint8Array values and non-finite numbers cross as {__bytes} / {__f64} (include/automerge_amd.h)
function requestJSON(change) {
  return JSON.stringify(change, function (key, value) {
    const raw = this[key]
    // encodeValue takes the whole buffer of a value view (columnar.js:269-271); other bytes are the view
    if (ArrayBuffer.isView(raw)) {
      return {__bytes: toHex(key === 'value' ? new Uint8Array(raw.buffer) : new Uint8Array(raw.buffer, raw.byteOffset, raw.byteLength))}
    }
    if (typeof raw === 'number' && !Number.isFinite(raw)) return {__f64: String(raw)}
    return value
  })
}

function applyLocalChange(backend, change) {
  const state = backendState(backend)
  let r
  try {
    r = native.docApplyLocal(state, requestJSON(change))
  } catch (e) {
    if (e.applied) backend.frozen = true
    throw e
  }
  // the request's deps gain the local actor's previous change, as in the reference (backend.js:80)
  if (r.lastHash) {
    const deps = {[r.lastHash[0]]: true}
    for (const hash of change.deps) deps[hash] = true
    change.deps = Object.keys(deps).sort()
  }
  backend.frozen = true
  const heads = native.docHeads(state)
  const c = native.docCounts(state)
  const patch = materializePatch(r.patch, heads, c.pending, c.maxOp)
  patch.actor = change.actor
  patch.seq = change.seq
  patch.deps = patch.deps.filter(head => head !== r.newHash[0])
  return [{state, heads}, patch, r.change]
}

// ---- sync protocol (backend/sync.js) in the engine (am_sync_*); SyncState objects cross as the
// flat state blob of include/automerge_amd.h ----
function bytesOf(x) {
  if (x instanceof Uint8Array) return x
  throw new TypeError(`Not a byte array: ${x}`)
}
function checkedHash(h) {  // hexStringToBytes + the 256-bit check of encodeHashes (sync.js:130-139)
  if (typeof h !== 'string') throw new TypeError('value is not a string')
  if (!/^([0-9a-f][0-9a-f])*$/.test(h)) throw new RangeError('value is not hexadecimal')
  if (h.length !== 64) throw new TypeError('heads hashes must be 256 bits')
  return Buffer.from(h, 'hex')
}
function packState(s) {
  const out = []
  const uleb = v => { do { let b = v % 128; v = Math.floor(v / 128); out.push(v ? b | 0x80 : b) } while (v) }
  const hashes = list => {
    if (!Array.isArray(list)) throw new TypeError('hashes must be an array')
    uleb(list.length)
    for (const h of list) out.push(...checkedHash(h))
  }
  const sent = s.sentHashes
  const sentKeys = sent && typeof sent === 'object' ? Object.keys(sent).filter(k => HASH_RE.test(k)) : []
  const flags = (s.theirHeads ? 1 : 0) | (s.theirNeed ? 2 : 0) | (s.theirHave ? 4 : 0) | (Array.isArray(sent) ? 8 : 0)
  out.push(0x53, flags)
  hashes(s.sharedHeads)
  hashes(s.lastSentHeads)
  if (s.theirHeads) hashes(s.theirHeads)
  if (s.theirNeed) hashes(s.theirNeed)
  if (s.theirHave) {
    uleb(s.theirHave.length)
    for (const h of s.theirHave) {
      hashes(h.lastSync)
      const b = bytesOf(h.bloom)
      uleb(b.byteLength)
      for (const x of b) out.push(x)
    }
  }
  uleb(sentKeys.length)
  for (const h of sentKeys) out.push(...Buffer.from(h, 'hex'))
  return Uint8Array.from(out)
}
function unpackState(b) {
  let o = 2
  const u = () => { let v = 0, mul = 1, x; do { x = b[o++]; v += (x & 0x7f) * mul; mul *= 128 } while (x & 0x80); return v }
  const hashes = () => { const n = u(), r = []; for (let i = 0; i < n; i++, o += 32) r.push(toHex(b.subarray(o, o + 32))); return r }
  const flags = b[1]
  const s = {sharedHeads: hashes(), lastSentHeads: hashes(), theirHeads: null, theirNeed: null, theirHave: null}
  if (flags & 1) s.theirHeads = hashes()
  if (flags & 2) s.theirNeed = hashes()
  if (flags & 4) {
    s.theirHave = []
    for (let n = u(), i = 0; i < n; i++) {
      const lastSync = hashes(), len = u()
      s.theirHave.push({lastSync, bloom: b.slice(o, o + len)})
      o += len
    }
  }
  const sent = hashes()
  if (flags & 8) s.sentHashes = []
  else { s.sentHashes = {}; for (const h of sent) s.sentHashes[h] = true }
  return s
}

function initSyncState() {
  return {sharedHeads: [], lastSentHeads: [], theirHeads: null, theirNeed: null, theirHave: null, sentHashes: {}}
}

function encodeSyncMessage(message) {
  if (message === undefined || message === null) throw new TypeError(`Cannot read property 'heads' of ${message}`)
  return native.syncEncodeMessage(requestJSON(message))
}

function decodeSyncMessage(bytes) {
  const m = native.syncDecodeMessage(bytesOf(bytes))
  return {heads: hexList(m.heads), need: hexList(m.need),
          have: m.have.map(h => ({lastSync: hexList(h.lastSync), bloom: h.bloom})), changes: m.changes}
}

function encodeSyncState(syncState) {
  return native.syncEncodeState(packState({sharedHeads: syncState.sharedHeads, lastSentHeads: []}))
}

function decodeSyncState(bytes) {
  return unpackState(native.syncDecodeState(bytesOf(bytes)))
}

function generateSyncMessage(backend, syncState) {
  if (!backend) throw new Error('generateSyncMessage called with no Automerge document')
  if (!syncState) throw new Error('generateSyncMessage requires a syncState, which can be created with initSyncState()')
  const packed = packState(syncState)
  const [r] = native.syncGenerate([backendState(backend)], [packed])
  if (r instanceof Error) throw r
  const [blob, message] = r
  if (message === null || Buffer.compare(Buffer.from(blob), Buffer.from(packed)) === 0) return [syncState, message]
  const next = unpackState(blob)
  return [Object.assign({}, syncState, {lastSentHeads: next.lastSentHeads, sentHashes: next.sentHashes}), message]
}

function receiveSyncMessage(backend, oldSyncState, binaryMessage) {
  if (!backend) throw new Error('generateSyncMessage called with no Automerge document')
  if (!oldSyncState) throw new Error('generateSyncMessage requires a syncState, which can be created with initSyncState()')
  const message = decodeSyncMessage(binaryMessage)
  // the reference reaches backendState() through applyChanges / getChangeByHash
  const state = (message.changes.length > 0 || message.heads.length > 0) ? backendState(backend) : backend.state
  let r
  try {
    r = native.syncReceive(state, packState(oldSyncState), binaryMessage)
  } catch (e) {
    if (e.applied) backend.frozen = true
    throw e
  }
  let patch = null
  if (message.changes.length > 0) {
    backend.frozen = true
    backend = {state, heads: native.docHeads(state)}
    const c = native.docCounts(state)
    patch = materializePatch(r[1], backend.heads, c.pending, c.maxOp)
  }
  const s = unpackState(r[0])
  const syncState = {sharedHeads: s.sharedHeads, lastSentHeads: s.lastSentHeads, theirHave: message.have,
                     theirHeads: message.heads, theirNeed: message.need, sentHashes: s.sentHashes}
  // receiveSyncMessage keeps sentHashes unless the peer reset (sync.js:455-458)
  if (!Array.isArray(s.sentHashes)) syncState.sentHashes = oldSyncState.sentHashes
  return [backend, syncState, patch]
}

// ---- the batched surface: the same calls over many documents, ONE GPU batch per call
// (am_doc_*_batch, am_sync_receive_batch). Per item the single call's result, or its error object in
// its place (nothing is thrown for one bad item). Patches are materialized lazily: the [state, patch]
// pairs carry the engine's log and build the patch object on first access of pair[1]. ----
function lazyPatch(pair, at, r) {
  let cached
  Object.defineProperty(pair, at, {
    enumerable: true,
    get() { return cached || (cached = materializePatch(r.log, r.heads, r.pending, r.maxOp)) }
  })
  return pair
}
function partition(items, prep) {
  const idx = [], vals = [], out = new Array(items.length)
  items.forEach((x, i) => {
    try { vals.push(prep(x, i)); idx.push(i) } catch (e) { out[i] = e }
  })
  return [idx, vals, out]
}

// A backend named more than once: as sequential calls. run(items) takes the first occurrence of each
// backend; a later one runs in a following round, where a handle its earlier call froze throws the
// outdated-document error in its own slot (util.js:1-10) and a handle whose earlier call failed
// (unchanged) is applied.
function rounds(backends, run) {
  const out = new Array(backends.length)
  let pending = backends.map((_, i) => i)
  while (pending.length > 0) {
    const seen = new Set(), now = [], later = []
    for (const i of pending) {
      const b = backends[i]
      if (b && typeof b === 'object' && seen.has(b)) later.push(i)
      else { now.push(i); if (b && typeof b === 'object') seen.add(b) }
    }
    run(now).forEach((r, k) => { out[now[k]] = r })
    pending = later
  }
  return out
}

function loadBatch(datas) {
  return native.docLoadBatch(datas).map(r => r instanceof Error ? r : {state: r, heads: native.docHeads(r)})
}

function applyBatch(backends, changeLists, wantPatch) {
  return rounds(backends, items => applyOnce(items.map(i => backends[i]), items.map(i => changeLists[i]), wantPatch))
}
function applyOnce(backends, changeLists, wantPatch) {
  const [idx, states, out] = partition(backends, b => backendState(b))
  const res = native.docApplyBatch(states, idx.map(i => changeLists[i]), wantPatch)
  res.forEach((r, k) => {
    const i = idx[k]
    if (r instanceof Error) { out[i] = r; return }
    backends[i].frozen = true
    if (!wantPatch) { out[i] = {state: states[k], heads: native.docHeads(states[k])}; return }
    out[i] = lazyPatch([{state: states[k], heads: r.heads}, null], 1, r)
  })
  return out
}
const applyChangesBatch = (backends, changeLists) => applyBatch(backends, changeLists, true)
const loadChangesBatch = (backends, changeLists) => applyBatch(backends, changeLists, false)

function saveBatch(backends) {
  const [idx, states, out] = partition(backends, b => backendState(b))
  native.docSaveBatch(states).forEach((r, k) => { out[idx[k]] = r })
  return out
}

// [patch | Error]; each patch object is built when its index is first read
function getPatchBatch(backends) {
  const [idx, states, out] = partition(backends, b => backendState(b))
  native.docPatchBatch(states).forEach((r, k) => {
    if (r instanceof Error) out[idx[k]] = r
    else lazyPatch(out, idx[k], r)
  })
  return out
}

function generateSyncMessages(backends, syncStates) {
  const [idx, vals, out] = partition(backends, (b, i) => {
    if (!b) throw new Error('generateSyncMessage called with no Automerge document')
    if (!syncStates[i]) throw new Error('generateSyncMessage requires a syncState, which can be created with initSyncState()')
    return [backendState(b), packState(syncStates[i])]
  })
  native.syncGenerate(vals.map(v => v[0]), vals.map(v => v[1])).forEach((r, k) => {
    const i = idx[k]
    if (r instanceof Error) { out[i] = r; return }
    const [blob, message] = r
    if (message === null || Buffer.compare(Buffer.from(blob), Buffer.from(vals[k][1])) === 0) { out[i] = [syncStates[i], message]; return }
    const next = unpackState(blob)
    out[i] = [Object.assign({}, syncStates[i], {lastSentHeads: next.lastSentHeads, sentHashes: next.sentHashes}), message]
  })
  return out
}

function receiveSyncMessages(backends, oldSyncStates, binaryMessages) {
  return rounds(backends, items => receiveOnce(items.map(i => backends[i]), items.map(i => oldSyncStates[i]),
                                               items.map(i => binaryMessages[i])))
}
function receiveOnce(backends, oldSyncStates, binaryMessages) {
  const [idx, vals, out] = partition(backends, (b, i) => {
    if (!b) throw new Error('generateSyncMessage called with no Automerge document')
    if (!oldSyncStates[i]) throw new Error('generateSyncMessage requires a syncState, which can be created with initSyncState()')
    const message = decodeSyncMessage(binaryMessages[i])
    const state = (message.changes.length > 0 || message.heads.length > 0) ? backendState(b) : b.state
    return [state, packState(oldSyncStates[i]), binaryMessages[i], message]
  })
  native.syncReceiveBatch(vals.map(v => v[0]), vals.map(v => v[1]), vals.map(v => v[2])).forEach((r, k) => {
    const i = idx[k], [state, , , message] = vals[k]
    let backend = backends[i]
    if (r instanceof Error) {
      if (r.applied) backend.frozen = true
      out[i] = r
      return
    }
    const s = unpackState(r[0])
    const syncState = {sharedHeads: s.sharedHeads, lastSentHeads: s.lastSentHeads, theirHave: message.have,
                       theirHeads: message.heads, theirNeed: message.need, sentHashes: s.sentHashes}
    if (!Array.isArray(s.sentHashes)) syncState.sentHashes = oldSyncStates[i].sentHashes
    if (message.changes.length > 0) {
      backend.frozen = true
      backend = {state, heads: r[1].heads}
      out[i] = lazyPatch([backend, syncState, null], 2, r[1])
    } else {
      out[i] = [backend, syncState, null]
    }
  })
  return out
}

module.exports = {
  init, clone, free, applyChanges, applyLocalChange, save, load, loadChanges, getPatch,
  getHeads, getAllChanges, getChanges, getChangesAdded, getChangeByHash, getMissingDeps,
  receiveSyncMessage, generateSyncMessage, encodeSyncMessage, decodeSyncMessage, encodeSyncState, decodeSyncState,
  initSyncState,
  loadBatch, applyChangesBatch, loadChangesBatch, saveBatch, getPatchBatch, generateSyncMessages, receiveSyncMessages,
  encodeChange: change => native.encodeChange(requestJSON(change)),  // columnar.js encodeChange (tests)
  engineVersion: native.version,
  _materializePatch: materializePatch  // host stage of getPatch (exported for tests)
}
