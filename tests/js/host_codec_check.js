'use strict'
// Host-only parity of the C ABI (no GPU needed): encodeChange (am_encode_change) and the sync
// codecs (am_sync_encode_message / decode_messages / encode_state / decode_state) against the
// calls recorded from the reference's test files (tests/golden/backend_log_*.json).
//  - every applyLocalChange call's binary change is re-encoded from its request (with the deps the
//    reference added: the ones in the recorded change header) by automerge_amd's encodeChange
//  - every recorded encodeSyncMessage / decodeSyncMessage / encodeSyncState / decodeSyncState /
//    initSyncState call is replayed and its result or error compared
// Prints one JSON line.
const fs = require('fs')
const path = require('path')
const zlib = require('zlib')
const B = require(path.join(__dirname, '..', '..', 'automerge_amd', 'js', 'backend.js'))
const GOLDEN = path.join(__dirname, '..', 'golden')

function canon(x) {
  if (x === undefined) return {__undef: 1}
  if (typeof x === 'number') {
    if (!Number.isFinite(x) || Object.is(x, -0)) return {__f64: Object.is(x, -0) ? '-0' : String(x)}
    return x
  }
  if (x instanceof Uint8Array) return {__bytes: Buffer.from(x.buffer, x.byteOffset, x.byteLength).toString('hex')}
  if (Array.isArray(x)) return x.map(canon)
  if (x && typeof x === 'object') { const o = {}; for (const k of Object.keys(x).sort()) o[k] = canon(x[k]); return o }
  return x
}
function decode(r) {
  if (Array.isArray(r)) return r.map(decode)
  if (r && typeof r === 'object') {
    const ks = Object.keys(r)
    if (ks.length === 1 && ks[0] === '__bytes') return new Uint8Array(Buffer.from(r.__bytes, 'hex'))
    if (ks.length === 1 && ks[0] === '__view') return new Uint8Array(Buffer.from(r.__view, 'hex'))
    if (ks.length === 1 && ks[0] === '__undef') return undefined
    if (ks.length === 1 && ks[0] === '__f64') return r.__f64 === '-0' ? -0 : Number(r.__f64)
    const o = {}
    for (const k of ks) o[k] = decode(r[k])
    return o
  }
  return r
}
// deps of a binary change (chunk header, then uleb count + 32-byte hashes)
function changeDeps(b) {
  let o = 9, len = 0, mul = 1, x
  do { x = b[o++]; len += (x & 0x7f) * mul; mul *= 128 } while (x & 0x80)
  let body = b.subarray(o, o + len)
  if (b[8] === 2) body = zlib.inflateRawSync(body)
  let n = 0; mul = 1; o = 0
  do { x = body[o++]; n += (x & 0x7f) * mul; mul *= 128 } while (x & 0x80)
  const deps = []
  for (let i = 0; i < n; i++, o += 32) deps.push(Buffer.from(body.subarray(o, o + 32)).toString('hex'))
  return deps
}

const PURE = new Set(['encodeSyncMessage', 'decodeSyncMessage', 'encodeSyncState', 'decodeSyncState', 'initSyncState'])
const bad = []
let encoded = 0, pure = 0
for (const f of ['sync', 'backend', 'test', 'text', 'table']) {
  const data = JSON.parse(fs.readFileSync(path.join(GOLDEN, `backend_log_${f}.json`)))
  for (const sc of data.scenarios) {
    for (let i = 0; i < sc.log.length; i++) {
      const e = sc.log[i]
      if (e.fn === 'applyLocalChange' && e.result) {
        const want = decode(e.result[2])
        const req = decode(e.args[1])
        req.deps = changeDeps(want)
        let got
        try { got = B.encodeChange(req) } catch (x) { got = x }
        encoded++
        if (!(got instanceof Uint8Array) || Buffer.compare(Buffer.from(got), Buffer.from(want)) !== 0) {
          bad.push({file: f, scenario: sc.name, i, fn: 'encodeChange', got: got instanceof Error ? got.message : canon(got).__bytes,
                    want: canon(want).__bytes})
        }
      } else if (PURE.has(e.fn)) {
        pure++
        let res, err = null
        try { res = B[e.fn](...decode(e.args)) } catch (x) { err = {name: x.constructor.name, message: x.message} }
        if (e.error) {
          if (!err || err.message !== e.error.message || err.name !== e.error.name) bad.push({file: f, scenario: sc.name, i, fn: e.fn, want: e.error, got: err})
        } else if (err || JSON.stringify(canon(res)) !== JSON.stringify(e.result)) {
          bad.push({file: f, scenario: sc.name, i, fn: e.fn, got: err || JSON.stringify(canon(res)).slice(0, 300), want: JSON.stringify(e.result).slice(0, 300)})
        }
      }
    }
  }
}
console.log(JSON.stringify({encoded, pure, nbad: bad.length, bad: bad.slice(0, 30)}))
