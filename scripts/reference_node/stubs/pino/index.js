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

// positional args joined with spaces: the rebuilt service's default (quirk Q11 fix,
// service.log.positional_args: append)
function format (args) {
  let s = render(args[0])
  for (let i = 1; i < args.length; i++) s += ' ' + render(args[i])
  return s
}

// pino@5 itself (positional_args: drop): the message is quick-format-unescaped(args[0], rest),
// which keeps only what a %-specifier consumes. Every index.js call site that passes extra
// arguments has a constant first argument without '%' (index.js:51,88,121,133,150), so the
// text is args[0]; a '%' there would need the full formatter, which is not modelled here.
function formatDrop (args) {
  const f = args[0]
  if (args.length > 1 && typeof f === 'string' && f.indexOf('%') !== -1) {
    throw new Error('pino stub: %-specifiers with extra arguments are not modelled')
  }
  return render(f)
}

module.exports = function pino (opts) {
  const sink = h.logSink
  const head = ',"pid":' + process.pid + ',"hostname":' + JSON.stringify(os.hostname()) +
    ',"name":' + JSON.stringify((opts && opts.name) || 'pino')
  const min = LEVELS[h.logLevel || 'info']
  const fmt = h.positionalArgs === 'drop' ? formatDrop : format
  const logger = {}
  for (const name of Object.keys(LEVELS)) {
    const num = LEVELS[name]
    logger[name] = num < min
      ? function () {}
      : function () {
        sink.write('{"level":' + num + ',"time":' + Date.now() + head + ',"msg":' +
          JSON.stringify(fmt(arguments)) + ',"v":1}\n')
      }
  }
  return logger
}
