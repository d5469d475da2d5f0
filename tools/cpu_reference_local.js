'use strict'
// Reference side of tools/bench_local.py: Backend.applyLocalChange per call (backend/backend.js:54-91)
// on the same text documents and requests, under Node in the build container (the reference does
// not travel to the GPU box).
//   python tools/bench_local.py --dump /tmp/local && \
//   NODE_PATH=tests/golden/gen/node_modules node tools/cpu_reference_local.js /tmp/local [/root/reference]
const fs = require('fs')
const path = require('path')
const DIR = process.argv[2]
const REF = process.argv[3] || '/root/reference'
const Backend = require(path.join(REF, 'backend'))
const out = []
for (const f of fs.readdirSync(DIR).filter(f => f.startsWith('hist_')).sort()) {
  const n = f.slice(5, -4)
  const buf = fs.readFileSync(path.join(DIR, f))
  const changes = []
  for (let o = 0; o < buf.length;) {
    const len = buf.readUInt32LE(o)
    changes.push(new Uint8Array(buf.slice(o + 4, o + 4 + len)))
    o += 4 + len
  }
  let [st] = Backend.applyChanges(Backend.init(), changes)
  const reqs = JSON.parse(fs.readFileSync(path.join(DIR, 'req_' + n + '.json')))
  const ms = []
  reqs.forEach((rq, k) => {
    const t0 = process.hrtime.bigint()
    const r = Backend.applyLocalChange(st, rq)
    const dt = Number(process.hrtime.bigint() - t0) / 1e6
    st = r[0]
    if (k >= 2) ms.push(dt)
  })
  ms.sort((a, b) => a - b)
  out.push({ops: Number(n), changes: changes.length, calls: ms.length, median_ms: ms[ms.length >> 1], min_ms: ms[0],
            max_ms: ms[ms.length - 1]})
}
console.log(JSON.stringify({what: 'reference Backend.applyLocalChange per call (Node ' + process.version + ', 1 core)',
                            results: out}))
