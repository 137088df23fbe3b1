'use strict'
// triton-core/db stand-in: the media table as an in-memory Map (the rebuilt service's bench
// uses its in-memory store the same way). Both methods stay async, like the Postgres-backed one.
class Storage {
  constructor () {
    this.media = global.__beholderHarness.media
  }

  async updateStatus (mediaId, status) {
    const m = this.media.get(mediaId)
    if (!m) throw new Error('media ' + mediaId + ' not found')
    m.status = status
  }

  async getByID (mediaId) {
    const m = this.media.get(mediaId)
    if (!m) throw new Error('media ' + mediaId + ' not found')
    return m
  }
}
module.exports = Storage
