'use strict'
// Reference-executed parity oracle: runs the reference service's own index.js
// (tritonmedia/beholder, loaded from --index, never copied) under the stand-ins in stubs/ and
// records, per delivered event, every side effect the business logic (index.js:50-155) has:
//
//   acks       number of rmsg.ack() calls                     (index.js:71,124,151,154)
//   threw      the listener's rejection message, or null      (Q1: index.js:62-90 has no catch)
//   decodeError  proto.decode threw for this body             (index.js:63,129)
//   requests   [method, full URL] of every sink request       (index.js:53,83,99,112)
//   logs       [level, msg] of every pino line                (index.js:51,66,82,88,98,111,121,133,150)
//
// and at the end the counters' label hashes and values (index.js:29-40,57,136-138) and the
// media table's statuses (index.js:68).
//
//   node oracle.js --index /root/reference/index.js --scenario scenario.json
//
// scenario.json: {config, media: [{id,name,creator,creatorId,metadataId,status}],
//   events: [["status"|"progress", hexBody]], faults: [{method, prefix, status|null, message, body}],
//   positionalArgs: "append"|"drop", notFound: "media {id} not found", logLevel: "info",
//   races: {mediaId: status} (the status another writer leaves in the row after each updateStatus)}
//   concurrent: {cap, script} (scenario mode "concurrent", below)
// NO_TRELLO comes from the environment, as in the reference (index.js:70).
// Events are delivered one at a time and each listener's promise is awaited before the next
// (the Python side does the same), so traces are deterministic.
//
// Mode "concurrent" (quirk Q9, index.js:43,62,127: up to prefetch listeners in flight, no
// per-media order): every store call and sink request waits on a gate that only this driver
// opens, so several deliveries are in flight at once and their awaits resume in one scripted
// order. Each step either delivers the next event (while fewer than `cap` are in flight) or opens
// the gate of one in-flight event, chosen by `script[step]` among the events waiting (sorted by
// index; an event waits on one gate at most, its awaits being sequential), then lets everything
// runnable run (setImmediate: the microtask queue is empty). Only that event runs in a step, so
// its log lines and requests are its own. The store applies an UPDATE and reads a row when its
// gate opens, so a status event suspended in getByID sees the UPDATE of another event that
// resolved first (index.js:68,76,94). `order` records each step: [action, event, gate kind,
// log lines, requests, acks, settled]. tests/reference_oracle.py replays the same script.
const fs = require('fs')
const path = require('path')

function arg (name, def) {
  const i = process.argv.indexOf('--' + name)
  return i === -1 ? def : process.argv[i + 1]
}

// request-promise-core's StatusCodeError (simple: true rejects every non-2xx response)
class StatusCodeError extends Error {
  constructor (statusCode, body) {
    super(statusCode + ' - ' + JSON.stringify(body))
    this.name = 'StatusCodeError'
    this.statusCode = statusCode
  }
}

const sc = JSON.parse(fs.readFileSync(arg('scenario'), 'utf8'))
let cur = { acks: 0, threw: null, decodeError: false, requests: [], logs: [] } // init-time sink
const initLogs = cur.logs

const h = global.__beholderHarness = {
  config: sc.config,
  media: new Map(),
  listeners: {},
  counters: [],
  logLevel: sc.logLevel || 'info',
  positionalArgs: sc.positionalArgs || 'append',
  notFound: sc.notFound,
  races: sc.races || {},
  logSink: {
    write (s) {
      for (const line of s.split('\n')) {
        if (!line) continue
        const o = JSON.parse(line)
        cur.logs.push([o.level, o.msg])
      }
    },
    flush () {}
  },
  record (method, url) {
    cur.requests.push([method, url])
  },
  // the first matching fault answers (RecordingHttpClient.fail's order); otherwise 200 {}
  reply (kind, method, url) {
    for (const f of sc.faults || []) {
      if ((f.method === '*' || f.method === method) && url.startsWith(f.prefix)) {
        if (f.status === null || f.status === undefined) return Promise.reject(new Error(f.message || 'ECONNREFUSED'))
        const body = f.body === undefined ? '"error"' : f.body
        if (kind === 'trello') return Promise.resolve(body) // trello@0.9.1 resolves on any status
        if (f.status >= 200 && f.status < 300) return Promise.resolve(body)
        return Promise.reject(new StatusCodeError(f.status, body))
      }
    }
    return Promise.resolve(kind === 'trello' ? {} : '{}')
  },
  onDecodeError () {
    cur.decodeError = true
  },
  current: null, // the event whose code runs in this step (mode "concurrent")
  gate: null
}
// the gate an event's store call / sink request waits on (mode "concurrent")
const waiting = new Map() // event index -> {kind, open}
if (sc.concurrent) {
  h.gate = kind => new Promise(resolve => {
    if (waiting.has(h.current)) throw new Error('event ' + h.current + ' waits on two gates')
    waiting.set(h.current, { kind, open: resolve })
  })
  const answer = h.reply
  h.reply = (kind, method, url) => h.gate('http').then(() => answer(kind, method, url))
}
for (const m of sc.media) h.media.set(m.id, Object.assign({}, m))

const TOPICS = { status: 'v1.telemetry.status', progress: 'v1.telemetry.progress' }
const immediate = () => new Promise(resolve => setImmediate(resolve))

const errText = e => e instanceof Error ? e.message : String(e)

async function sequential () {
  const events = []
  for (const [topic, hex] of sc.events) {
    cur = { acks: 0, threw: null, decodeError: false, requests: [], logs: [] }
    const rmsg = { message: { content: Buffer.from(hex, 'hex') }, ack () { cur.acks++ } }
    try {
      await h.listeners[TOPICS[topic]](rmsg)
    } catch (e) {
      cur.threw = errText(e)
    }
    events.push(cur)
  }
  return { events }
}

async function concurrent () {
  const { cap, script } = sc.concurrent
  const n = sc.events.length
  const events = sc.events.map(() => ({ acks: 0, threw: null, decodeError: false, requests: [], logs: [] }))
  const settled = new Array(n).fill(false)
  const order = []
  let next = 0
  let active = 0
  for (let step = 0; ; step++) {
    const ready = [...waiting.keys()].sort((a, b) => a - b)
    const r = script[step % script.length]
    let i, action, kind
    if (next < n && (ready.length === 0 || (active < cap && r % 2 === 0))) {
      i = next++
      action = 'deliver'
      kind = null
      active++
    } else if (ready.length) {
      i = ready[(r >>> 1) % ready.length]
      action = 'resolve'
      kind = waiting.get(i).kind
    } else {
      if (active) throw new Error(active + ' deliveries in flight, none at a gate')
      break
    }
    h.current = i
    cur = events[i]
    const before = [cur.logs.length, cur.requests.length, cur.acks]
    if (action === 'deliver') {
      const [topic, hex] = sc.events[i]
      const rec = cur
      const rmsg = { message: { content: Buffer.from(hex, 'hex') }, ack () { rec.acks++ } }
      h.listeners[TOPICS[topic]](rmsg).then(() => { settled[i] = true; active-- },
        e => { rec.threw = errText(e); settled[i] = true; active-- })
    } else {
      const g = waiting.get(i)
      waiting.delete(i)
      g.open()
    }
    await immediate()
    order.push([action, i, kind, cur.logs.length - before[0], cur.requests.length - before[1],
      cur.acks - before[2], settled[i]])
  }
  return { events, order }
}

async function main () {
  require(path.resolve(arg('index'))) // the reference service: calls init() at module load
  while (!(h.listeners[TOPICS.status] && h.listeners[TOPICS.progress])) await immediate()
  await immediate() // let init() finish (its last statement logs 'initialized')
  const { events, order } = sc.concurrent ? await concurrent() : await sequential()
  const counters = {}
  for (const c of h.counters) {
    counters[c.name] = Object.keys(c.hashMap).sort().map(k => [k, c.hashMap[k].value])
  }
  const media = {}
  for (const [id, m] of h.media) media[id] = m.status
  process.stdout.write(JSON.stringify({ events, order, counters, media, initLogs, node: process.version }) + '\n',
    () => process.exit(0))
}

main().catch(e => { console.error(e && e.stack ? e.stack : e); process.exit(1) })
