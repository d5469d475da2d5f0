'use strict'
// Host stage of the batched surface: materializePatch (automerge_amd/js/backend.js) over the wire-form
// applyChanges patch logs in a file written by tools/js_materialize.py ([u32 LE length, log bytes]...).
// Prints one JSON line: documents, seconds, microseconds per document.
const fs = require('fs')
const path = require('path')
const B = require(path.join(__dirname, '..', 'automerge_amd', 'js', 'backend.js'))
const buf = fs.readFileSync(process.argv[2])
const logs = []
for (let o = 0; o < buf.length;) {
  const n = buf.readUInt32LE(o)
  logs.push(new Uint8Array(buf.buffer, buf.byteOffset + o + 4, n))
  o += 4 + n
}
let sink = 0
for (let i = 0; i < Math.min(2000, logs.length); i++) sink += Object.keys(B._materializePatch(logs[i], [], 0, 0).diffs.props).length
const t0 = process.hrtime.bigint()
for (const log of logs) sink += Object.keys(B._materializePatch(log, [], 0, 0).diffs.props).length
const s = Number(process.hrtime.bigint() - t0) / 1e9
console.log(JSON.stringify({docs: logs.length, seconds: s, us_per_doc: 1e6 * s / logs.length, docs_per_s: logs.length / s,
                            node: process.version, sink}))
