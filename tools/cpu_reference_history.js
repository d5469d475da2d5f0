'use strict'
// CPU baseline of SURVEY.md §8(f) row 2 (tools/bench_history.py): the reference JS backend under
// Node computing the change history of saved documents -- Backend.getAllChanges(Backend.load(doc)),
// i.e. computeHashGraph (new.js:1879-1904) -- on one process, for the C4 base documents (one change
// each) and for the merged C4 documents (base + its 12 concurrent changes, saved). Runs in the build
// container (the reference cannot travel); writes profiles/cpu_reference_history.json.
//   NODE_PATH=tests/golden/gen/node_modules node tools/cpu_reference_history.js [/root/reference] [seconds]
const path = require('path')
const fs = require('fs')
const REF = process.argv[2] || process.env.AM_REF || '/root/reference'
const SECONDS = Number(process.argv[3] || 10)
const gen = require(path.join(__dirname, '..', 'tests', 'golden', 'gen', 'make_fixtures.js'))
const Backend = require(path.join(REF, 'backend'))

function time(docs) {
  let n = 0, chg = 0
  const t0 = process.hrtime.bigint(), limit = BigInt(Math.round(SECONDS * 1e9))
  while (process.hrtime.bigint() - t0 < limit) {
    chg += Backend.getAllChanges(Backend.load(docs[n % docs.length])).length
    n++
  }
  const s = Number(process.hrtime.bigint() - t0) / 1e9
  return {docs: n, changes: chg, seconds: s, docs_per_sec: n / s, changes_per_sec: chg / s}
}
const base = [], merged = []
for (let d = 0; d < 2000; d++) {
  const {baseBytes, order} = gen.c4Doc(d)
  base.push(baseBytes)
  merged.push(Backend.save(Backend.applyChanges(Backend.load(baseBytes), order)[0]))
}
const out = {what: 'Backend.getAllChanges(Backend.load(doc)) per document, one Node process', cores: 1,
             node: process.version, c4_base: time(base), c4_merged: time(merged)}
fs.writeFileSync(path.join(__dirname, '..', 'profiles', 'cpu_reference_history.json'), JSON.stringify(out, null, 1) + '\n')
console.log(JSON.stringify(out))
