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
// NO_TRELLO comes from the environment, as in the reference (index.js:70).
// Events are delivered one at a time and each listener's promise is awaited before the next
// (the Python side does the same), so traces are deterministic.
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
  }
}
for (const m of sc.media) h.media.set(m.id, Object.assign({}, m))

const TOPICS = { status: 'v1.telemetry.status', progress: 'v1.telemetry.progress' }
const immediate = () => new Promise(resolve => setImmediate(resolve))

async function main () {
  require(path.resolve(arg('index'))) // the reference service: calls init() at module load
  while (!(h.listeners[TOPICS.status] && h.listeners[TOPICS.progress])) await immediate()
  await immediate() // let init() finish (its last statement logs 'initialized')
  const events = []
  for (const [topic, hex] of sc.events) {
    cur = { acks: 0, threw: null, decodeError: false, requests: [], logs: [] }
    const rmsg = { message: { content: Buffer.from(hex, 'hex') }, ack () { cur.acks++ } }
    try {
      await h.listeners[TOPICS[topic]](rmsg)
    } catch (e) {
      cur.threw = e instanceof Error ? e.message : String(e)
    }
    events.push(cur)
  }
  const counters = {}
  for (const c of h.counters) {
    counters[c.name] = Object.keys(c.hashMap).sort().map(k => [k, c.hashMap[k].value])
  }
  const media = {}
  for (const [id, m] of h.media) media[id] = m.status
  process.stdout.write(JSON.stringify({ events, counters, media, initLogs, node: process.version }) + '\n',
    () => process.exit(0))
}

main().catch(e => { console.error(e && e.stack ? e.stack : e); process.exit(1) })
