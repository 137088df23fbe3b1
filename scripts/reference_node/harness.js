'use strict'
// Drives the reference service's own index.js (tritonmedia/beholder) with in-process stand-ins
// for its dependencies (stubs/, resolved through NODE_PATH) over the same synthetic framed
// events the rebuilt service's bench.py consumes. Measures events/s and handle latency
// (handler call -> rmsg.ack()).
//
//   node harness.js --index /root/reference/index.js --config cfg.json --media media.json \
//        --events events.bin --events-per-step E --warmup W --steps K [--wait-go] [--pino-sync]
//
// --pino-sync writes every log line with its own write(2), as pino@5's default destination does;
// without it lines are buffered (cheaper than the real library).
// With --wait-go it prints "ready" after the warm-up steps and waits for a line on stdin before
// the timed steps (the Python driver starts several processes together this way).
const fs = require('fs')
const path = require('path')
const { performance } = require('perf_hooks')

function arg (name, def) {
  const i = process.argv.indexOf('--' + name)
  return i === -1 ? def : process.argv[i + 1]
}

class Sink {
  constructor (fd, sync) {
    this.fd = fd
    this.sync = sync
    this.buf = ''
  }

  write (s) {
    if (this.sync) {
      fs.writeSync(this.fd, s)
      return
    }
    this.buf += s
    if (this.buf.length >= 65536) this.flush()
  }

  flush () {
    if (this.buf) {
      fs.writeSync(this.fd, this.buf)
      this.buf = ''
    }
  }
}

const h = global.__beholderHarness = {
  config: JSON.parse(fs.readFileSync(arg('config'), 'utf8')),
  media: new Map(),
  listeners: {},
  logSink: new Sink(fs.openSync(arg('log', '/dev/null'), 'w'), process.argv.includes('--pino-sync')),
  logLevel: arg('log-level', 'info'),
  calls: 0,
  recent: new Array(16),
  record (method, url) {
    this.recent[this.calls & 15] = url
    this.calls++
  },
  reply (kind, method, url) { // every sink answers 200 {}
    return Promise.resolve(kind === 'trello' ? {} : '{}')
  }
}
for (const m of JSON.parse(fs.readFileSync(arg('media'), 'utf8'))) h.media.set(m.id, m)

const TOPICS = { 1: 'v1.telemetry.status', 2: 'v1.telemetry.progress' }
const data = fs.readFileSync(arg('events'))
const events = []
for (let i = 0; i < data.length;) {
  const L = data.readUInt32LE(i)
  events.push([TOPICS[data[i + 4]], data.subarray(i + 5, i + 4 + L)])
  i += 4 + L
}

const E = Number(arg('events-per-step'))
const W = Number(arg('warmup', '1'))
const K = Number(arg('steps', '5'))
const BATCH = Number(arg('batch', '512'))
if (events.length < E * (W + K)) throw new Error('events file holds ' + events.length + ' events, need ' + E * (W + K))

const lat = new Float64Array(E * K)
let nlat = 0
let timing = false
let settled = 0
let errors = 0
// the status handler has no try/catch (quirk Q1): count its rejections so a step cannot wait forever
process.on('unhandledRejection', () => { errors++; settled++ })

const immediate = () => new Promise(resolve => setImmediate(resolve))

function waitGo () {
  return new Promise(resolve => {
    process.stdin.once('data', () => { process.stdin.pause(); resolve() })
  })
}

async function main () {
  require(path.resolve(arg('index'))) // the reference service: calls init() at module load
  while (!(h.listeners['v1.telemetry.status'] && h.listeners['v1.telemetry.progress'])) await immediate()
  const handlers = h.listeners

  function deliver (topic, content) {
    const t0 = performance.now()
    handlers[topic]({
      message: { content },
      ack () {
        settled++
        if (timing) lat[nlat++] = performance.now() - t0
      }
    })
  }

  async function step (s) {
    const end = (s + 1) * E
    for (let j = s * E; j < end; j += BATCH) {
      const stop = Math.min(end, j + BATCH)
      for (let k = j; k < stop; k++) deliver(events[k][0], events[k][1])
      await immediate()
    }
    while (settled < end) await immediate()
  }

  for (let s = 0; s < W; s++) await step(s)
  h.logSink.flush()
  if (process.argv.includes('--wait-go')) {
    process.stdout.write('ready\n')
    await waitGo()
  }
  timing = true
  const t0 = performance.now()
  for (let s = W; s < W + K; s++) await step(s)
  h.logSink.flush()
  const elapsed = (performance.now() - t0) / 1000
  const sorted = Float64Array.from(lat.subarray(0, nlat)).sort()
  const pct = p => sorted.length ? sorted[Math.min(sorted.length - 1, Math.floor(p / 100 * sorted.length))] * 1000 : null
  process.stdout.write(JSON.stringify({
    events: E * K,
    elapsed_s: elapsed,
    events_per_sec: E * K / elapsed,
    p50_handle_latency_us: pct(50),
    p99_handle_latency_us: pct(99),
    http_requests: h.calls,
    handler_errors: errors,
    node: process.version
  }) + '\n', () => process.exit(0))
}

main().catch(e => { console.error(e); process.exit(1) })
