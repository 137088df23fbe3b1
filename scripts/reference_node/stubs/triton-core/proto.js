'use strict'
// triton-core/proto stand-in: load / decode / enumToString / stringToEnum over the rebuilt
// service's schema (beholder_amd/models/proto/api.proto, same field numbers).
//
// decode follows protobufjs 6.8.8 (yarn.lock:1506-1518), the library triton-core wraps: on Node a
// Buffer gets a BufferReader, and a message type's generated decoder reads each known field with
// its declared reader method whatever wire type the tag carries, and hands every other tag to
// skipType. The reader below keeps protobufjs's own quirks, because malformed bodies reach the
// handlers' error branches (index.js:62-90 throws, index.js:149-151 logs err.message):
//   * uint32() reads up to five bytes with no per-byte bounds check (buf[pos] past the end is
//     `undefined`: `undefined & 127` is 0 and `undefined < 128` is false, so it reads on), then
//     skips five more bytes unchecked and fails only if that passes the end;
//   * string() clamps to the end of the buffer (BufferReader), bytes()/skip(n) throw;
//   * no UTF-8 validation (Buffer#utf8Slice substitutes U+FFFD);
//   * error texts are protobufjs's: RangeError "index out of range: <pos> + <n> > <len>" and
//     Error "invalid wire type <wt> at offset <pos>".
// This is written from the behaviour of protobufjs's reader.js / reader_buffer.js / decoder.js,
// not from the rebuilt service's C++ reader (beholder_amd/ops/csrc/pbjs.hpp), so the oracle
// (oracle.js) checks one against the other.
const ENUMS = {
  TelemetryStatusEntry: { QUEUED: 0, DOWNLOADING: 1, CONVERTING: 2, UPLOADING: 3, DEPLOYED: 4, ERRORED: 5 },
  CreatorType: { API: 0, TRELLO: 1 }
}
const TYPES = {
  'api.TelemetryStatus': { fields: { 1: ['mediaId', 'string'], 2: ['status', 'int32'] }, defaults: { mediaId: '', status: 0 } },
  'api.TelemetryProgress': {
    fields: { 1: ['mediaId', 'string'], 2: ['status', 'int32'], 3: ['progress', 'int32'], 4: ['host', 'string'] },
    defaults: { mediaId: '', status: 0, progress: 0, host: '' }
  },
  'api.Media': { fields: {}, defaults: {} }
}

function indexOutOfRange (reader, writeLength) {
  return RangeError('index out of range: ' + reader.pos + ' + ' + (writeLength || 1) + ' > ' + reader.len)
}

class Reader {
  constructor (buf) {
    this.buf = buf
    this.pos = 0
    this.len = buf.length
  }

  uint32 () {
    let value = (this.buf[this.pos] & 127) >>> 0; if (this.buf[this.pos++] < 128) return value
    value = (value | (this.buf[this.pos] & 127) << 7) >>> 0; if (this.buf[this.pos++] < 128) return value
    value = (value | (this.buf[this.pos] & 127) << 14) >>> 0; if (this.buf[this.pos++] < 128) return value
    value = (value | (this.buf[this.pos] & 127) << 21) >>> 0; if (this.buf[this.pos++] < 128) return value
    value = (value | (this.buf[this.pos] & 15) << 28) >>> 0; if (this.buf[this.pos++] < 128) return value
    if ((this.pos += 5) > this.len) {
      this.pos = this.len
      throw indexOutOfRange(this, 10)
    }
    return value
  }

  int32 () {
    return this.uint32() | 0
  }

  // BufferReader.prototype.string
  string () {
    const len = this.uint32()
    return this.buf.utf8Slice(this.pos, this.pos = Math.min(this.pos + len, this.len))
  }

  skip (length) {
    if (typeof length === 'number') {
      if (this.pos + length > this.len) throw indexOutOfRange(this, length)
      this.pos += length
    } else {
      do {
        if (this.pos >= this.len) throw indexOutOfRange(this)
      } while (this.buf[this.pos++] & 128)
    }
    return this
  }

  skipType (wireType) {
    switch (wireType) {
      case 0:
        this.skip()
        break
      case 1:
        this.skip(8)
        break
      case 2:
        this.skip(this.uint32())
        break
      case 3:
        while ((wireType = this.uint32() & 7) !== 4) this.skipType(wireType)
        break
      case 5:
        this.skip(4)
        break
      default:
        throw Error('invalid wire type ' + wireType + ' at offset ' + this.pos)
    }
    return this
  }
}

function decode (type, buf) {
  const h = global.__beholderHarness
  const r = new Reader(buf)
  const m = Object.assign({}, type.defaults)
  const fields = type.fields
  try {
    while (r.pos < r.len) {
      const t = r.uint32()
      const f = fields[t >>> 3]
      if (f) m[f[0]] = r[f[1]]()
      else r.skipType(t & 7)
    }
  } catch (e) {
    if (h && h.onDecodeError) h.onDecodeError(e)
    throw e
  }
  return m
}

module.exports = {
  async load (name) {
    const t = TYPES[name]
    if (!t) throw new Error('no such type ' + name)
    return t
  },
  decode,
  Reader,
  enumToString (type, enumName, value) {
    const e = ENUMS[enumName]
    for (const k of Object.keys(e)) if (e[k] === value) return k
    return undefined
  },
  stringToEnum (type, enumName, str) {
    return ENUMS[enumName][str]
  }
}
