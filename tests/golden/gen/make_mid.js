// Mid-size fixtures (round-5 workload, am_workload.cpp gen_mid) from the reference backend. The change bytes
// come from the engine's own generator (workload/am_workload.cpp gen_mid, dumped by
// make_mid.py); this script pins them and the merge results against the reference:
//   * every change decodes (checksum, inflate) and re-encodes to the same bytes
//     (decodeChange -> encodeChange, columnar.js:710-776, incl. deflateChange :798);
//   * full:  save/heads/getPatch of applyChanges(init(), all changes);
//   * split: base = save(applyChanges(init(), first half)), then load(base) + applyChanges(rest):
//            save/heads/getPatch and the applyChanges patch.
// Large outputs are stored as SHA-256 of the bytes / of canonical JSON (sorted keys).
// Usage: NODE_PATH=tests/golden/gen/node_modules node tests/golden/gen/make_mid.js in.json out.json [refRoot]
'use strict'
const fs = require('fs')
const path = require('path')
const crypto = require('crypto')
const REF = process.argv[4] || '/root/reference'
const Backend = require(path.join(REF, 'backend'))
const col = require(path.join(REF, 'backend/columnar'))

const hex = u8 => Buffer.from(u8).toString('hex')
const unhex = h => new Uint8Array(Buffer.from(h, 'hex'))
const sha = u8 => crypto.createHash('sha256').update(Buffer.from(u8)).digest('hex')
function canon(v) {
  if (Array.isArray(v)) return v.map(canon)
  if (v && typeof v === 'object') {
    const o = {}
    for (const k of Object.keys(v).sort()) o[k] = canon(v[k])
    return o
  }
  return v
}
const jsha = obj => crypto.createHash('sha256').update(JSON.stringify(canon(obj))).digest('hex')

const input = JSON.parse(fs.readFileSync(process.argv[2], 'utf8'))
const out = []
for (const cs of input) {
  const rec = Object.assign({}, cs, {docs: []})
  cs.docs.forEach((chunks, d) => {
    const bins = chunks.map(unhex)
    let deflated = 0
    for (const b of bins) {
      if (b[8] === 2) deflated++
      const again = col.encodeChange(col.decodeChange(b))
      if (hex(again) !== hex(b)) throw new Error(`${cs.name} doc ${d}: change does not re-encode to the same bytes`)
    }
    const full = Backend.applyChanges(Backend.init(), bins)[0]
    const fullSave = Backend.save(full)
    const half = Math.floor(bins.length / 2)
    const baseBytes = Backend.save(Backend.applyChanges(Backend.init(), bins.slice(0, half))[0])
    const [st, patch] = Backend.applyChanges(Backend.load(baseBytes), bins.slice(half))
    const save2 = Backend.save(st)
    rec.docs.push({
      changes: sha(Buffer.concat(bins.map(b => Buffer.from(b)))), nchunks: bins.length, deflated,
      full: {save: sha(fullSave), len: fullSave.byteLength, heads: Backend.getHeads(full),
             getPatch: jsha(Backend.getPatch(full))},
      split: {half, base: sha(baseBytes), base_len: baseBytes.byteLength, save: sha(save2), len: save2.byteLength,
              heads: Backend.getHeads(st), getPatch: jsha(Backend.getPatch(st)), applyPatch: jsha(patch)}})
  })
  out.push(rec)
  console.log(cs.name, 'ok', cs.docs.length, 'docs')
}
fs.writeFileSync(process.argv[3], JSON.stringify(out) + '\n')
