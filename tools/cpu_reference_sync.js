'use strict'
// Reference side of tools/bench_sync.py --e2e (C5, configs[4]): the same document pairs synced by
// the reference's own sync protocol (backend/sync.js generateSyncMessage / receiveSyncMessage, with
// the Backend applyChanges it calls) under Node in the build container (the reference does not
// travel to the GPU box). Per pair: both sides load the base and apply their own chain (untimed),
// resume from a persisted sync state whose sharedHeads is the base's head (decodeSyncState of
// encodeSyncState, sync.js:217-225), then exchange messages until neither side has one (timed).
//   python tools/bench_sync.py --pairs 2000 --dump /tmp/c5.bin && \
//   NODE_PATH=tests/golden/gen/node_modules node tools/cpu_reference_sync.js /tmp/c5.bin [seconds] [/root/reference]
const fs = require('fs')
const path = require('path')
const FILE = process.argv[2]
const SECONDS = Number(process.argv[3] || 20)
const REF = process.argv[4] || '/root/reference'
const Backend = require(path.join(REF, 'backend'))

const buf = fs.readFileSync(FILE)
const P = buf.readUInt32LE(0), K = buf.readUInt32LE(4)
let o = 8
const next = () => {
  const n = buf.readUInt32LE(o)
  const b = new Uint8Array(buf.slice(o + 4, o + 4 + n))
  o += 4 + n
  return b
}
let pairs = 0, rounds = 0, messages = 0, timed = 0n
const t00 = process.hrtime.bigint()
for (let i = 0; i < P; i++) {
  const base = next()
  const a = [], b = []
  for (let k = 0; k < K; k++) a.push(next())
  for (let k = 0; k < K; k++) b.push(next())
  if (Number(process.hrtime.bigint() - t00) / 1e9 > SECONDS) continue
  let docs = [Backend.loadChanges(Backend.load(base), a), Backend.loadChanges(Backend.load(base), b)]
  const head = Backend.getHeads(Backend.load(base))
  const resumed = () => Backend.decodeSyncState(Backend.encodeSyncState(Object.assign(Backend.initSyncState(), {sharedHeads: head})))
  let states = [resumed(), resumed()]
  const t0 = process.hrtime.bigint()
  // the schedule of bench_sync.py --e2e: every round both sides generate, then every message is
  // delivered
  for (let r = 0; r < 20; r++) {
    const msgs = [null, null]
    for (const s of [0, 1]) {
      const [st, msg] = Backend.generateSyncMessage(docs[s], states[s])
      states[s] = st
      msgs[s] = msg
    }
    if (!msgs[0] && !msgs[1]) break
    for (const s of [0, 1]) {
      if (!msgs[s]) continue
      const [d2, st2] = Backend.receiveSyncMessage(docs[1 - s], states[1 - s], msgs[s])
      docs[1 - s] = d2
      states[1 - s] = st2
      messages++
    }
    rounds++
  }
  timed += process.hrtime.bigint() - t0
  const h0 = Backend.getHeads(docs[0]).join(), h1 = Backend.getHeads(docs[1]).join()
  if (h0 !== h1) throw new Error(`pair ${i} did not converge`)
  pairs++
}
const s = Number(timed) / 1e9
console.log(JSON.stringify({what: 'reference sync.js generateSyncMessage/receiveSyncMessage until converged, C5 pairs (' + K +
                                  ' concurrent changes per side since a resumed sync state), Node ' + process.version + ', 1 core',
                            pairs, seconds: s, pairs_per_s: pairs / s, messages, rounds_total: rounds}))
