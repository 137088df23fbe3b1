'use strict'
// triton-core/amqp stand-in: connect() resolves; listen(topic, fn) registers the consumer. The
// harness delivers {message: {content}, ack()} envelopes to it, as triton-core's listen does.
class AMQP {
  constructor (host, prefetch, retries, prom) {
    this.host = host
    this.prefetch = prefetch
    this.retries = retries
  }

  async connect () {}

  async listen (topic, fn) {
    global.__beholderHarness.listeners[topic] = fn
  }
}
module.exports = AMQP
