'use strict'
// CPU baseline of SURVEY.md §8(d): the reference JS backend (/root/reference, under Node with the
// offline shims of tests/golden/gen/node_modules) on the C4 workload -- per document
// Backend.load(base) + Backend.applyChanges(12 concurrent changes) (+ save) -- timed on one
// process, then on one process per core in parallel (each over its own documents). The reference
// cannot travel to the GPU box, so this runs in the build container and bench.py quotes the file
// it writes (profiles/cpu_reference_node.json).
//   NODE_PATH=tests/golden/gen/node_modules node tools/cpu_reference.js [/root/reference] [seconds] [procs]
const os = require('os')
const path = require('path')
const fs = require('fs')
const {fork} = require('child_process')
const REF = (process.argv[2] !== '--worker' && process.argv[2]) || process.env.AM_REF || '/root/reference'
const SECONDS = Number(process.argv[3] || 10)
const PROCS = Number(process.argv[4] || os.cpus().length)

function worker(first, ndocs, seconds) {
  const gen = require(path.join(__dirname, '..', 'tests', 'golden', 'gen', 'make_fixtures.js'))
  const Backend = require(path.join(REF, 'backend'))
  const docs = []
  for (let d = first; d < first + ndocs; d++) docs.push(gen.c4Doc(d))
  const run = withSave => {
    let n = 0, ops = 0
    const t0 = process.hrtime.bigint(), limit = BigInt(Math.round(seconds * 5e8))
    while (process.hrtime.bigint() - t0 < limit) {
      const {baseBytes, order} = docs[n % docs.length]
      const [st] = Backend.applyChanges(Backend.load(baseBytes), order)
      if (withSave) Backend.save(st)
      n++
      ops += 60
    }
    return {docs: n, ops, s: Number(process.hrtime.bigint() - t0) / 1e9}
  }
  return {load_apply_save: run(true), load_apply: run(false)}
}

if (process.argv[2] === '--worker') {
  const [first, ndocs, seconds] = process.argv.slice(3).map(Number)
  process.send(worker(first, ndocs, seconds))
  return
}

function spawn(i, ndocs) {
  return new Promise((resolve, reject) => {
    const c = fork(__filename, ['--worker', String(i * ndocs), String(ndocs), String(SECONDS)],
                   {env: Object.assign({}, process.env, {AM_REF: REF}), execArgv: []})
    c.on('message', resolve)
    c.on('error', reject)
  })
}

async function main() {
  const rate = r => r.ops / r.s
  const one = await spawn(0, 400)
  const all = await Promise.all(Array.from({length: PROCS}, (_, i) => spawn(i + 1, 400)))
  const sum = key => all.reduce((a, r) => a + rate(r[key]), 0)
  const out = {
    what: 'reference JS backend (backend/new.js via backend/index.js) under Node, C4 documents: Backend.load(base) + ' +
          'Backend.applyChanges(12 changes) [+ Backend.save], ops merged per second',
    node: process.version, cpu: os.cpus()[0].model, nproc: os.cpus().length, procs: PROCS, seconds_per_run: SECONDS / 2,
    per_core_ops_per_s: rate(one.load_apply_save), per_core_ops_per_s_without_save: rate(one.load_apply),
    all_cores_ops_per_s: sum('load_apply_save'), all_cores_ops_per_s_without_save: sum('load_apply'),
    measured_in: 'build container (the reference does not travel to the GPU box); tools/cpu_reference.js'
  }
  const dst = path.join(__dirname, '..', 'profiles', 'cpu_reference_node.json')
  fs.writeFileSync(dst, JSON.stringify(out, null, 1) + '\n')
  console.log(JSON.stringify(out))
}
main()
