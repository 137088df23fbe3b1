'use strict'
// In-process stand-in for pino@5 (yarn.lock:1438-1448): the same JSON line envelope the
// reference writes ({"level","time","pid","hostname","name","msg","v":1}) into a sink on
// /dev/null. By default the sink buffers 64 KiB per write(2), which is cheaper than the real
// library. pino@5's default destination (sonic-boom, sync) issues one write(2) per line; the
// harness's --pino-sync mode reproduces that.
const os = require('os')
const h = global.__beholderHarness

const LEVELS = { trace: 10, debug: 20, info: 30, warn: 40, error: 50, fatal: 60 }

function render (a) {
  if (typeof a === 'string') return a
  if (a !== null && typeof a === 'object') return a instanceof Error ? a.message : JSON.stringify(a)
  return String(a)
}

// positional args joined with spaces: the same text volume as the rebuilt service (quirk Q11 fix)
function format (args) {
  let s = render(args[0])
  for (let i = 1; i < args.length; i++) s += ' ' + render(args[i])
  return s
}

module.exports = function pino (opts) {
  const sink = h.logSink
  const head = ',"pid":' + process.pid + ',"hostname":' + JSON.stringify(os.hostname()) +
    ',"name":' + JSON.stringify((opts && opts.name) || 'pino')
  const min = LEVELS[h.logLevel || 'info']
  const logger = {}
  for (const name of Object.keys(LEVELS)) {
    const num = LEVELS[name]
    logger[name] = num < min
      ? function () {}
      : function () {
        sink.write('{"level":' + num + ',"time":' + Date.now() + head + ',"msg":' +
          JSON.stringify(format(arguments)) + ',"v":1}\n')
      }
  }
  return logger
}
