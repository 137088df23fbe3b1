'use strict'
// In-process stand-in for trello@0.9.1 (yarn.lock:1982-1989): makeRequest validates the method and
// path, merges key/token with the options into the query string (restler + qs 1.2 encoding =
// encodeURIComponent) and resolves without network I/O. The request is recorded, like the
// rebuilt service's bench recorder, and answered by the harness (h.reply): trello@0.9.1's promise
// rejects only on a transport error (restler 'complete' with an Error) and resolves with the
// body on any HTTP status.
const h = global.__beholderHarness
const METHODS = { get: 'GET', post: 'POST', put: 'PUT', delete: 'DELETE' }

function Trello (key, token) {
  this.uri = 'https://api.trello.com'
  this.key = key
  this.token = token
}

Trello.prototype.createQuery = function () {
  return { key: this.key, token: this.token }
}

Trello.prototype.makeRequest = function (requestMethod, path, options) {
  const method = METHODS[requestMethod] || METHODS[String(requestMethod).toLowerCase()]
  if (!method) return Promise.reject(new Error('Unsupported requestMethod. Pass one of these methods: POST, GET, PUT, DELETE.'))
  if (typeof path !== 'string' || path[0] !== '/') return Promise.reject(new Error('Path must start with /'))
  const query = this.createQuery()
  for (const k of Object.keys(options || {})) query[k] = options[k]
  let qs = ''
  for (const k of Object.keys(query)) {
    if (query[k] === undefined) continue
    qs += (qs ? '&' : '') + encodeURIComponent(k) + '=' + encodeURIComponent(query[k])
  }
  const url = this.uri + path + '?' + qs
  h.record(method, url)
  return h.reply('trello', method, url)
}

module.exports = Trello
