'use strict'
// triton-core/prom stand-in over a prom-client@11-shaped Counter: label validation, label
// hashing ("k:v" joined, keys sorted) and a per-hash value map, as prom-client's inc() does.
function hashObject (labels) {
  let keys = Object.keys(labels)
  if (keys.length === 0) return ''
  if (keys.length > 1) keys = keys.sort()
  let hash = ''
  for (let i = 0; i < keys.length; i++) hash += (i ? ',' : '') + keys[i] + ':' + labels[keys[i]]
  return hash
}

class Counter {
  constructor (cfg) {
    this.name = cfg.name
    this.help = cfg.help
    this.labelNames = cfg.labelNames || []
    this.hashMap = {}
    const h = global.__beholderHarness
    if (h && h.counters) h.counters.push(this) // the oracle reads every counter at the end
  }

  inc (labels, value) {
    if (labels === undefined || labels === null || typeof labels !== 'object') {
      value = labels
      labels = {}
    }
    for (const k of Object.keys(labels)) {
      if (this.labelNames.indexOf(k) === -1) throw new Error('Added label "' + k + '" is not included in initial labelset')
    }
    if (value === undefined) value = 1
    if (value < 0) throw new Error('It is not possible to decrease a counter')
    const hash = hashObject(labels)
    const e = this.hashMap[hash]
    if (e) e.value += value
    else this.hashMap[hash] = { labels: labels, value: value }
  }
}

const registries = {}
module.exports = {
  new (name) {
    const reg = { name, Counter }
    registries[name] = reg
    global.__beholderHarness.prom = reg
    return reg
  },
  expose () {}
}
