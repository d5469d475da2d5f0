'use strict'
// Replays the backend-boundary logs recorded from the reference's own test files
// (tests/golden/backend_log_*.json, made by tests/golden/gen/make_backend_log.js) against
// automerge_amd/js/backend.js: every call of the 22 Backend exports with the recorded arguments,
// every result (patches, binary changes, saved documents, heads, sync messages and sync states,
// handle identity) and every thrown error class and message compared. Prints one JSON line.
const fs = require('fs')
const path = require('path')
const B = require(path.join(__dirname, '..', '..', 'automerge_amd', 'js', 'backend.js'))
const GOLDEN = path.join(__dirname, '..', 'golden')

const isHandle = x => x && typeof x === 'object' && 'state' in x && 'heads' in x
function canon(x) {
  if (x === undefined) return {__undef: 1}
  if (typeof x === 'number') {
    if (!Number.isFinite(x) || Object.is(x, -0)) return {__f64: Object.is(x, -0) ? '-0' : String(x)}
    return x
  }
  if (x instanceof Uint8Array) return {__bytes: Buffer.from(x.buffer, x.byteOffset, x.byteLength).toString('hex')}
  if (ArrayBuffer.isView(x)) return {__view: Buffer.from(x.buffer).toString('hex')}
  if (Array.isArray(x)) return x.map(canon)
  if (x && typeof x === 'object') {
    const o = {}
    for (const k of Object.keys(x).sort()) o[k] = canon(x[k])
    return o
  }
  return x
}
const special = r => r && typeof r === 'object' && !Array.isArray(r) &&
  ['__bytes', '__f64', '__undef', '__view', '$h'].some(k => k in r) && Object.keys(r).length === 1
function decode(r, h) {
  if (Array.isArray(r)) return r.map(v => decode(v, h))
  if (r && typeof r === 'object') {
    if (special(r)) {
      if ('$h' in r) return h.get(r.$h)
      if ('__bytes' in r) return new Uint8Array(Buffer.from(r.__bytes, 'hex'))
      if ('__view' in r) return new Uint8Array(Buffer.from(r.__view, 'hex'))
      if ('__undef' in r) return undefined
      return r.__f64 === '-0' ? -0 : Number(r.__f64)
    }
    const o = {}
    for (const k of Object.keys(r)) o[k] = decode(r[k], h)
    return o
  }
  return r
}
let where = ''
function match(rec, x, h, p = '') {
  where = p
  if (special(rec) && '$h' in rec) {
    if (!isHandle(x)) return false
    if (h.has(rec.$h)) return h.get(rec.$h) === x
    h.set(rec.$h, x)
    return true
  }
  if (Array.isArray(rec)) return Array.isArray(x) && x.length === rec.length && rec.every((v, i) => match(v, x[i], h, p + '/' + i))
  if (rec && typeof rec === 'object' && !special(rec)) {
    if (!x || typeof x !== 'object' || Array.isArray(x) || x instanceof Uint8Array) return false
    const ks = Object.keys(rec)
    // integer-like keys (actor ids such as '76543210') come first in Object.keys: compare sorted
    if (JSON.stringify(ks.slice().sort()) !== JSON.stringify(Object.keys(x).sort())) return false
    return ks.every(k => match(rec[k], x[k], h, p + '/' + k))
  }
  return JSON.stringify(canon(x)) === JSON.stringify(rec)
}

// known divergences (tests/backend_log.py KNOWN_DIVERGENT): they must fail with the engine's
// "unsupported" error
const KNOWN_DIVERGENT = new Set([])  // none since round 4 (the null action is restated)
const files = (process.argv[2] || 'sync,sync_random,objmeta,backend,test,text,table,errors').split(',')
// --lockstep: call k of every scenario at once, the calls of one batched function in one call
// (BATCHED), the rest one by one; results compared the same way
const BATCHED = {applyChanges: 'applyChangesBatch', loadChanges: 'loadChangesBatch', load: 'loadBatch', save: 'saveBatch',
                 getPatch: 'getPatchBatch', generateSyncMessage: 'generateSyncMessages', receiveSyncMessage: 'receiveSyncMessages'}
const ARITY = {save: 1, getPatch: 1, load: 1, receiveSyncMessage: 3}
if (process.argv[3] === '--lockstep') {
  const scens = []
  for (const f of files) for (const sc of JSON.parse(fs.readFileSync(path.join(GOLDEN, `backend_log_${f}.json`))).scenarios) scens.push([f, sc, new Map()])
  const live = scens.map(() => true), bad = []
  let calls = 0, batched = 0
  for (let k = 0; live.some(x => x) && bad.length < 40; k++) {
    const groups = new Map()
    scens.forEach(([f, sc, h], j) => {
      if (!live[j]) return
      if (k >= sc.log.length) { live[j] = false; return }
      const e = sc.log[k], args = decode(e.args, h)
      while (args.length && args[args.length - 1] === undefined) args.pop()
      const key = (e.fn in BATCHED && args.length === (ARITY[e.fn] || 2)) ? e.fn : null
      if (!groups.has(key)) groups.set(key, [])
      groups.get(key).push([j, e, args])
    })
    const results = new Map()
    for (const [key, items] of groups) {
      if (key === null) {
        for (const [j, e, args] of items) {
          try { results.set(j, [B[e.fn](...args), null]) } catch (x) { results.set(j, [undefined, x]) }
        }
        continue
      }
      const cols = items[0][2].map((_, c) => items.map(it => it[2][c]))
      const out = B[BATCHED[key]](...cols)
      batched += items.length
      items.forEach(([j], q) => results.set(j, out[q] instanceof Error ? [undefined, out[q]] : [out[q], null]))
    }
    for (const items of groups.values()) {
      for (const [j, e] of items) {
        const [f, sc, h] = scens[j]
        calls++
        const [res, x] = results.get(j)
        const err = x ? {name: x.constructor.name, message: x.message} : null
        if (e.error) {
          if (!err || err.message !== e.error.message || err.name !== e.error.name) bad.push({file: f, scenario: sc.name, k, fn: e.fn, want: e.error, got: err || 'no error'})
          continue
        }
        if (err) { bad.push({file: f, scenario: sc.name, k, fn: e.fn, unexpected: err}); live[j] = false; continue }
        if (!match(e.result, res, h)) {
          bad.push({file: f, scenario: sc.name, k, fn: e.fn, where, want: JSON.stringify(e.result).slice(0, 400),
                    got: JSON.stringify(canon(res)).slice(0, 400)})
          live[j] = false
        }
      }
    }
  }
  console.log(JSON.stringify({files, lockstep: true, calls, batched, nbad: bad.length, bad: bad.slice(0, 20)}))
  process.exit(0)
}
const bad = [], perFn = {}
let calls = 0, scenarios = 0
for (const f of files) {
  const data = JSON.parse(fs.readFileSync(path.join(GOLDEN, `backend_log_${f}.json`)))
  for (const sc of data.scenarios) {
    scenarios++
    const h = new Map()
    if (KNOWN_DIVERGENT.has(f + '/' + sc.name)) {
      let raised = null
      for (const e of sc.log) {
        try {
          const res = B[e.fn](...decode(e.args, h))
          if ('result' in e) match(e.result, res, h)  // registers the handles the call returned
        } catch (x) { raised = x.message; break }
      }
      if (!raised || !raised.startsWith('automerge_amd: unsupported')) bad.push({file: f, scenario: sc.name, divergent: raised})
      continue
    }
    for (let i = 0; i < sc.log.length; i++) {
      const e = sc.log[i]
      calls++
      perFn[e.fn] = (perFn[e.fn] || 0) + 1
      let res, err = null
      try {
        res = B[e.fn](...decode(e.args, h))
      } catch (x) {
        err = {name: x.constructor.name, message: x.message}
      }
      if (e.error) {
        if (!err || err.message !== e.error.message || err.name !== e.error.name) {
          bad.push({file: f, scenario: sc.name, i, fn: e.fn, want: e.error, got: err || 'no error'})
        }
        continue
      }
      if (err) { bad.push({file: f, scenario: sc.name, i, fn: e.fn, unexpected: err}); break }
      if (!match(e.result, res, h)) {
        bad.push({file: f, scenario: sc.name, i, fn: e.fn, where, want: JSON.stringify(e.result).slice(0, 600),
                  got: JSON.stringify(canon(res)).slice(0, 600)})
        break
      }
    }
  }
}
console.log(JSON.stringify({files, scenarios, calls, perFn, nbad: bad.length, bad: bad.slice(0, 40)}))
