'use strict'
// triton-core/proto stand-in: load / decode / enumToString / stringToEnum over the rebuilt
// service's schema (beholder_amd/models/proto/api.proto, same field numbers). decode is a
// straight-line protobuf reader like protobufjs's generated decoders.
const ENUMS = {
  TelemetryStatusEntry: { QUEUED: 0, DOWNLOADING: 1, CONVERTING: 2, UPLOADING: 3, DEPLOYED: 4, ERRORED: 5 },
  CreatorType: { API: 0, TRELLO: 1 }
}
const TYPES = {
  'api.TelemetryStatus': { fields: { 1: ['mediaId', 's'], 2: ['status', 'v'] }, defaults: { mediaId: '', status: 0 } },
  'api.TelemetryProgress': {
    fields: { 1: ['mediaId', 's'], 2: ['status', 'v'], 3: ['progress', 'v'], 4: ['host', 's'] },
    defaults: { mediaId: '', status: 0, progress: 0, host: '' }
  },
  'api.Media': { fields: {}, defaults: {} }
}

function varint (buf, st) {
  let lo = 0
  let shift = 0
  let b
  do {
    if (st.i >= buf.length) throw new RangeError('index out of range')
    b = buf[st.i++]
    if (shift < 32) lo |= (b & 0x7f) << shift
    shift += 7
  } while (b & 0x80)
  return lo
}

function decode (type, buf) {
  const msg = Object.assign({}, type.defaults)
  const st = { i: 0 }
  const fields = type.fields
  while (st.i < buf.length) {
    const tag = varint(buf, st) >>> 0
    const f = fields[tag >>> 3]
    const wt = tag & 7
    if (f && f[1] === 'v' && wt === 0) {
      msg[f[0]] = varint(buf, st)
    } else if (f && f[1] === 's' && wt === 2) {
      const n = varint(buf, st) >>> 0
      if (st.i + n > buf.length) throw new RangeError('index out of range')
      msg[f[0]] = buf.toString('utf8', st.i, st.i + n)
      st.i += n
    } else if (wt === 0) {
      varint(buf, st)
    } else if (wt === 2) {
      st.i += varint(buf, st) >>> 0
    } else if (wt === 1) {
      st.i += 8
    } else if (wt === 5) {
      st.i += 4
    } else {
      throw new Error('invalid wire type ' + wt)
    }
  }
  return msg
}

module.exports = {
  async load (name) {
    const t = TYPES[name]
    if (!t) throw new Error('no such type ' + name)
    return t
  },
  decode,
  enumToString (type, enumName, value) {
    const e = ENUMS[enumName]
    for (const k of Object.keys(e)) if (e[k] === value) return k
    return undefined
  },
  stringToEnum (type, enumName, str) {
    return ENUMS[enumName][str]
  }
}
