'use strict'
// triton-core/db stand-in: the media table as an in-memory Map (the rebuilt service's bench
// uses its in-memory store the same way). Both methods stay async, like the Postgres-backed one.
//
// triton-core/db is not vendored, so two behaviours are [inferred], and match the rebuilt
// service's documented choice (beholder_amd/store/base.py):
//   * updateStatus of an unknown id changes nothing (an SQL UPDATE that matches zero rows);
//   * getByID of an unknown id rejects. The error text is the harness's `notFound` template
//     ("{id}" is replaced by the media id), so the oracle can set one string for both sides.
class Storage {
  constructor () {
    const h = global.__beholderHarness
    this.h = h
    this.media = h.media
    this.notFound = h.notFound || 'media {id} not found'
    this.races = h.races || {}
  }

  // Mode "concurrent" (oracle.js): each call first waits on the harness's gate; the UPDATE
  // lands, and the row is read, when the gate opens. getByID returns a copy of the row, as a
  // query returns a fresh row object: a row read before another event's UPDATE keeps its status.
  async updateStatus (mediaId, status) {
    if (this.h.gate) await this.h.gate('update')
    const m = this.media.get(mediaId)
    if (m) m.status = status
    // scenario mode "reread": another writer's UPDATE of the same row lands between this
    // UPDATE and the listener's getByID (index.js:68,76), so the re-read status is not the
    // message's (quirk Q3: the hooks key off the re-read one, index.js:94)
    if (m && Object.prototype.hasOwnProperty.call(this.races, mediaId)) m.status = this.races[mediaId]
  }

  async getByID (mediaId) {
    if (this.h.gate) await this.h.gate('get')
    const m = this.media.get(mediaId)
    if (!m) throw new Error(this.notFound.split('{id}').join(mediaId))
    return Object.assign({}, m)
  }
}
module.exports = Storage
