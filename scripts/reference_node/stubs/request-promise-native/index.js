'use strict'
// In-process stand-in for request-promise-native@1.0.7 over request@2.88 (qs 6.5, RFC 3986
// encoding): builds the GET URL from `url` + `qs`, records it and lets the harness answer
// (h.reply): a transport error rejects with that error; a non-2xx status rejects with
// request-promise's StatusCodeError (simple: true), message `${statusCode} - ${JSON.stringify(body)}`.
const h = global.__beholderHarness

function rfc3986 (s) {
  return encodeURIComponent(s).replace(/[!'()*]/g, c => '%' + c.charCodeAt(0).toString(16).toUpperCase())
}

module.exports = function request (opts) {
  let url = opts.url || opts.uri
  if (opts.qs) {
    let q = ''
    for (const k of Object.keys(opts.qs)) {
      const v = opts.qs[k]
      if (v === undefined) continue
      q += (q ? '&' : '') + rfc3986(k) + '=' + rfc3986(String(v))
    }
    if (q) url += (url.indexOf('?') === -1 ? '?' : '&') + q
  }
  const method = opts.method || 'GET'
  h.record(method, url)
  return h.reply('request', method, url)
}
