'use strict'
// Materializes engine patch logs with backend.js's host stage and compares with the reference's
// getPatch output. Input: a JSON file [{log: hex, deps, pending, expect}]; prints one JSON line.
const fs = require('fs')
const path = require('path')
const B = require(path.join(__dirname, '..', '..', 'automerge_amd', 'js', 'backend.js'))
const toHex = u8 => Buffer.from(u8.buffer, u8.byteOffset, u8.byteLength).toString('hex')
const canon = x => {
  if (x instanceof Uint8Array) return {__bytes: toHex(x)}
  if (Array.isArray(x)) return x.map(canon)
  if (x && typeof x === 'object') { const o = {}; for (const k of Object.keys(x).sort()) o[k] = canon(x[k]); return o }
  return x
}
const cases = JSON.parse(fs.readFileSync(process.argv[2]))
const bad = []
cases.forEach((c, i) => {
  const log = Uint8Array.from(Buffer.from(c.log, 'hex'))
  const maxOp = Number(Buffer.from(c.log, 'hex').readBigInt64LE(24))
  const got = B._materializePatch(log, c.deps, c.pending, maxOp)
  if (JSON.stringify(canon(got)) !== JSON.stringify(canon(c.expect))) bad.push(i)
})
console.log(JSON.stringify({n: cases.length, bad: bad.slice(0, 10), nbad: bad.length}))
