// Change-history fixtures (SURVEY.md §8(f) row 2): Backend.getAllChanges(Backend.load(saved)) --
// computeHashGraph (new.js:1879-1904) = decodeDocument (columnar.js:1040) + groupChangeOps (:876)
// + decodeDocumentChanges (:945) + encodeChange of every change -- for the saved documents of the
// golden scenarios (tests/golden/docs.json) and of the text histories (tests/golden/text.json inputs).
// Usage: NODE_PATH=tests/golden/gen/node_modules node tests/golden/gen/make_history.js [refRoot]
'use strict'
const fs = require('fs')
const path = require('path')
const REF = process.argv[2] || '/root/reference'
const Backend = require(path.join(REF, 'backend'))
const OUT = path.join(__dirname, '..')
const hex = u8 => Buffer.from(u8).toString('hex')
const unhex = h => new Uint8Array(Buffer.from(h, 'hex'))

const docs = JSON.parse(fs.readFileSync(path.join(OUT, 'docs.json'), 'utf8')).scenarios
const out = []
const seen = new Set()
for (const sc of docs) {
  for (const res of sc.results) {
    if (!res.save || seen.has(res.save)) continue
    seen.add(res.save)
    let changes = null, error = null
    try {
      changes = Backend.getAllChanges(Backend.load(unhex(res.save))).map(hex)
    } catch (e) {
      error = e.message
    }
    out.push({doc: res.save, changes, error})
  }
}
// documents with deflated columns and long histories: save() of the first part of text histories
const extra = process.env.TEXT_IN ? JSON.parse(fs.readFileSync(process.env.TEXT_IN, 'utf8')) : []
for (const cs of extra) {
  for (const chunks of cs.docs) {
    const st = Backend.applyChanges(Backend.init(), chunks.slice(0, 60).map(unhex))[0]
    const saved = Backend.save(st)
    out.push({doc: hex(saved), changes: Backend.getAllChanges(Backend.load(saved)).map(hex), error: null})
  }
}
fs.writeFileSync(path.join(OUT, 'history.json'), JSON.stringify(out) + '\n')
console.log('wrote history.json', out.length, 'documents')
