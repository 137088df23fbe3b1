'use strict'
// triton-core/dynamics stand-in: dyn(service) -> endpoint string.
module.exports = function dyn (service) {
  return 'harness://' + service
}
