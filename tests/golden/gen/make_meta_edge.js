// Golden vectors for two objectMeta edge cases of the per-handle path, recorded from the reference:
//  * makecounter/*: a root key holding a make op and, concurrently, a counter `set` with its `inc`.
//    documentPatch's children snapshot of the key keeps the visible `set` and make ops only
//    (updatePatchProperty, new.js:919-926): the visible inc row is not a child value. A call after
//    load that only sets another root key (the shape k_doc_fast's patch writer takes) leaves that
//    snapshot to the next call, whose patch edits inside the object and reads it back.
//  * floatinc/*: a counter incremented by a float64 value. The reference adds it as JS does
//    (`counterState.value += ...`, new.js:958); the engine cannot write that patch, but a patchless
//    loadChanges of it must commit as the reference's does and leave objectMeta usable.
// Output: tests/golden/meta_edge.json (the docs.json scenario format: steps + per-step results).
//   NODE_PATH=tests/golden/gen/node_modules node tests/golden/gen/make_meta_edge.js
'use strict'
const fs = require('fs')
const path = require('path')
const REF = process.env.AM_REF || '/root/reference'
const OUT = path.join(__dirname, '..')
const F = require('./make_fixtures')
const {runBackend, jsonPatch, hex} = F
const col = require(path.join(REF, 'backend/columnar'))
const Backend = require(path.join(REF, 'backend'))
const H = c => col.decodeChangeMeta(col.encodeChange(c), true).hash
const e = cs => cs.map(c => col.encodeChange(c))
const saved = cs => Backend.save(Backend.applyChanges(Backend.init(), e(cs))[0])

function makeCounter() {
  const out = []
  const set = (obj, key, value, pred, datatype) => Object.assign({action: 'set', obj, key, value, pred}, datatype ? {datatype} : {})
  for (const [a, b] of [['aa', 'bb'], ['bb', 'aa']]) {
    const c0 = {actor: '01', seq: 1, startOp: 1, time: 0, deps: [], ops: [set('_root', 'a', 1, [], 'uint')]}
    const X = {actor: a, seq: 1, startOp: 2, time: 0, deps: [H(c0)], ops: [{action: 'makeMap', obj: '_root', key: 'x', pred: []}]}
    const Y = {actor: b, seq: 1, startOp: 2, time: 0, deps: [H(c0)], ops: [set('_root', 'x', 5, [], 'counter')]}
    const Z = {actor: b, seq: 2, startOp: 3, time: 0, deps: [H(Y)],
               ops: [{action: 'inc', obj: '_root', key: 'x', datatype: 'int', value: 2, pred: [`2@${b}`]}]}
    const C1 = {actor: 'cc', seq: 1, startOp: 4, time: 0, deps: [H(X), H(Z)].sort(), ops: [set('_root', 'k', 7, [], 'uint')]}
    const C2 = {actor: 'cc', seq: 2, startOp: 5, time: 0, deps: [H(C1)], ops: [set(`2@${a}`, 'p', 1, [], 'uint')]}
    const C3 = {actor: 'cc', seq: 3, startOp: 6, time: 0, deps: [H(C2)],
                ops: [{action: 'inc', obj: '_root', key: 'x', datatype: 'int', value: 3, pred: [`2@${b}`]}]}
    const tag = a + b
    out.push({name: `makecounter/${tag}/load`, steps: [{op: 'load', bytes: saved([c0, X, Y, Z])}, {op: 'apply', changes: e([C1])},
      {op: 'apply', changes: e([C2])}, {op: 'apply', changes: e([C3])}]})
    out.push({name: `makecounter/${tag}/steps`, steps: [{op: 'apply', changes: e([c0, X, Y, Z])}, {op: 'apply', changes: e([C1])},
      {op: 'apply', changes: e([C2])}, {op: 'apply', changes: e([C3])}]})
    out.push({name: `makecounter/${tag}/load2`, steps: [{op: 'load', bytes: saved([c0, X, Y, Z])}, {op: 'apply', changes: e([C1, C2])}]})
  }
  return out
}

function floatInc() {
  const out = []
  const c0 = {actor: '01', seq: 1, startOp: 1, time: 0, deps: [],
              ops: [{action: 'set', obj: '_root', key: 'cnt', datatype: 'counter', value: 5, pred: []},
                    {action: 'makeList', obj: '_root', key: 'l', pred: []}]}
  const A = {actor: 'aa', seq: 1, startOp: 3, time: 0, deps: [H(c0)],
             ops: [{action: 'inc', obj: '_root', key: 'cnt', datatype: 'float64', value: 1.5, pred: ['1@01']}]}
  const B = {actor: 'bb', seq: 1, startOp: 3, time: 0, deps: [H(c0)],
             ops: [{action: 'makeMap', obj: '_root', key: 'l', pred: []}]}
  const C = {actor: 'aa', seq: 2, startOp: 4, time: 0, deps: [H(A), H(B)].sort(),
             ops: [{action: 'set', obj: '2@01', elemId: '_head', insert: true, datatype: 'uint', value: 9, pred: []},
                   {action: 'set', obj: '_root', key: 'z', datatype: 'uint', value: 1, pred: []}]}
  // step 1 (c0 + A + B) carries the float increment: the engine's test runs it as loadChanges
  out.push({name: 'floatinc/steps', steps: [{op: 'apply', changes: e([c0, A, B])}, {op: 'apply', changes: e([C])}]})
  out.push({name: 'floatinc/split', steps: [{op: 'apply', changes: e([c0])}, {op: 'apply', changes: e([A, B])},
    {op: 'apply', changes: e([C])}]})
  return out
}

function record(sc) {
  return {name: sc.name,
          steps: sc.steps.map(s => s.op === 'load' ? {op: 'load', bytes: hex(s.bytes)} : {op: 'apply', changes: s.changes.map(hex)}),
          results: runBackend(sc.steps).map(jsonPatch)}
}

function main() {
  const scen = makeCounter().concat(floatInc()).map(record)
  const file = path.join(OUT, 'meta_edge.json')
  fs.writeFileSync(file, JSON.stringify({scenarios: scen}) + '\n')
  const errs = scen.filter(s => s.results.some(x => x.error))
  console.log('wrote meta_edge.json', fs.statSync(file).size, 'bytes,', scen.length, 'scenarios;', errs.length, 'with an error',
              errs.map(s => s.name + ': ' + JSON.stringify(s.results[s.results.length - 1].error)))
}

main()
