'use strict'
// Replays the golden scenarios (tests/golden/docs.json, produced by the reference backend) through
// automerge_amd/js/backend.js -- the Node host over the N-API addon -- and reports mismatches of
// save() bytes, heads, pending counts, getPatch and applyChanges patches and thrown error
// class/message as one JSON line.
const fs = require('fs')
const path = require('path')
const B = require(path.join(__dirname, '..', '..', 'automerge_amd', 'js', 'backend.js'))

const hex = s => Uint8Array.from(Buffer.from(s, 'hex'))
const toHex = u8 => Buffer.from(u8.buffer, u8.byteOffset, u8.byteLength).toString('hex')
const docs = JSON.parse(fs.readFileSync(path.join(__dirname, '..', 'golden', 'docs.json'))).scenarios
// canonical JSON (sorted keys, Uint8Array -> {__bytes: hex}) for deep comparison
const canon = x => {
  if (x instanceof Uint8Array) return {__bytes: toHex(x)}
  if (Array.isArray(x)) return x.map(canon)
  if (x && typeof x === 'object') { const o = {}; for (const k of Object.keys(x).sort()) o[k] = canon(x[k]); return o }
  return x
}
const bad = []
let steps = 0, patches = 0, applied = 0
for (const sc of docs) {
  let st = null
  for (let i = 0; i < sc.steps.length; i++) {
    const step = sc.steps[i], exp = sc.results[i]
    let res = {}
    try {
      if (step.op === 'load') st = B.load(hex(step.bytes))
      else {
        if (st === null) st = B.init()
        const old = st
        let applyPatch
        ;[st, applyPatch] = B.applyChanges(st, step.changes.map(hex))
        if (exp.patch) {
          applied++
          if (JSON.stringify(canon(applyPatch)) !== JSON.stringify(canon(exp.patch))) bad.push([sc.name, i, 'applyChanges patch'])
        }
        try { B.save(old); bad.push([sc.name, i, 'old handle not frozen']) } catch (e) {
          if (!/outdated Automerge document/.test(e.message)) bad.push([sc.name, i, 'frozen message', e.message])
        }
      }
      res = {save: toHex(B.save(st)), heads: B.getHeads(st), patch: B.getPatch(st)}
    } catch (e) {
      res = {error: e.message, cls: e.constructor.name}
    }
    steps++
    if (exp.error) {
      if (res.error !== exp.error.message) bad.push([sc.name, i, 'error', res.error, exp.error.message])
      break
    }
    if (res.error) { bad.push([sc.name, i, 'unexpected', res.cls, res.error]); break }
    if (res.save !== exp.save) bad.push([sc.name, i, 'save'])
    else if (JSON.stringify(res.heads) !== JSON.stringify(exp.heads)) bad.push([sc.name, i, 'heads'])
    else if (exp.getPatch) {
      patches++
      const want = Object.assign({}, exp.getPatch, {pendingChanges: exp.pending})
      if (JSON.stringify(canon(res.patch)) !== JSON.stringify(canon(want))) bad.push([sc.name, i, 'getPatch'])
    }
  }
}
// hash-graph queries on a fresh document built from the first multi-change scenario
const sc = docs.find(s => s.steps.length >= 2 && s.steps.every(x => x.op === 'apply') && !s.results.some(r => r.error))
let graph = null
if (sc) {
  let st = B.init()
  const all = []
  for (const step of sc.steps) { all.push(...step.changes); [st] = B.applyChanges(st, step.changes.map(hex)) }
  const got = B.getAllChanges(st).map(toHex)
  graph = {changes: got.length, applied_equal_given: JSON.stringify(got.slice().sort()) === JSON.stringify(all.slice().sort()),
           missing: B.getMissingDeps(st), since_heads: B.getChanges(st, B.getHeads(st)).length}
}
// change history of loaded documents (computeHashGraph, new.js:1879-1904) against the reference's
// getAllChanges(load(saved)) (tests/golden/history.json)
const hist = JSON.parse(fs.readFileSync(path.join(__dirname, '..', 'golden', 'history.json')))
let histDocs = 0
for (let i = 0; i < hist.length; i += 3) {
  const h = hist[i]
  let got
  try { got = B.getAllChanges(B.load(hex(h.doc))).map(toHex) } catch (e) { got = {error: e.message} }
  if (JSON.stringify(got) !== JSON.stringify(h.changes)) bad.push(['history', i])
  histDocs++
}
console.log(JSON.stringify({scenarios: docs.length, steps, patches, applied, histDocs, bad: bad.slice(0, 20), nbad: bad.length, graph}))
