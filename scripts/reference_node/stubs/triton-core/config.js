'use strict'
// triton-core/config stand-in: Config('events') resolves to the harness's config object
// (the rebuilt service's bench_config(): same keys, flow ids and enabled sinks).
module.exports = async function Config (name) {
  return global.__beholderHarness.config
}
