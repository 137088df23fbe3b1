// protobufjs 6.8.8 reader semantics (the library under triton-core/proto, yarn.lock:1506-1518).
//
// The reference decodes every delivery with `proto.decode(type, rmsg.message.content)`
// (index.js:63,129). On Node a Buffer gets protobufjs's BufferReader, and the message type's
// generated decoder is
//
//     while (r.pos < r.len) {
//       var t = r.uint32()
//       switch (t >>> 3) {
//         case <n>: m.<field> = r.<type>(); break     // no wire-type check
//         default: r.skipType(t & 7)
//       }
//     }
//
// This differs from upb (wire.hpp) on malformed input, and those are the cases that reach the
// handlers' error branches (Q1, Q7):
//   * a known field is read with its declared type whatever wire type its tag carries;
//   * uint32() reads up to 5 bytes without a bounds check per byte (a byte past the end reads
//     as `undefined`, which counts as a continuation), and when the 5th byte still has its
//     continuation bit it skips 5 more bytes unchecked, failing only if that passes the end;
//   * strings are clamped to the buffer end (BufferReader.string), bytes are bounds-checked;
//   * strings are never validated: invalid UTF-8 becomes U+FFFD (Buffer#utf8Slice);
//   * field number 0 is skipped like any unknown field; a group is skipped up to the next
//     end-group tag of any field number; wire types 4, 6 and 7 are errors;
//   * errors carry protobufjs's messages: "index out of range: <pos> + <n> > <len>" (RangeError)
//     and "invalid wire type <wt> at offset <pos>" (Error).
// Nested groups are counted instead of recursed into; V8 would overflow its stack somewhere past
// ~10^4 nesting levels, this reader does not (the one documented divergence).
#pragma once

#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <cstring>

namespace beholder {
namespace pbjs {

struct Reader {
  const uint8_t* buf;
  uint64_t len;
  uint64_t pos = 0;
  char err[96];
  bool failed = false;

  Reader(const uint8_t* b, size_t n) : buf(b), len(n) { err[0] = 0; }

  bool out_of_range(uint64_t write_length) {  // protobufjs indexOutOfRange(reader, writeLength)
    std::snprintf(err, sizeof err, "index out of range: %llu + %llu > %llu", (unsigned long long)pos,
                  (unsigned long long)(write_length ? write_length : 1), (unsigned long long)len);
    failed = true;
    return false;
  }

  bool invalid_wire_type(uint32_t wt) {
    std::snprintf(err, sizeof err, "invalid wire type %u at offset %llu", wt, (unsigned long long)pos);
    failed = true;
    return false;
  }

  // buf[pos] in JS: a byte past the end is `undefined` (`& 127` -> 0, `< 128` -> false)
  inline int at(uint64_t i) const { return i < len ? int(buf[i]) : -1; }

  // Reader.prototype.uint32
  bool uint32(uint32_t* out) {
    uint32_t v = 0;
    static const int shifts[4] = {0, 7, 14, 21};
    for (int k = 0; k < 4; ++k) {
      int b = at(pos);
      v |= uint32_t(b < 0 ? 0 : (b & 127)) << shifts[k];
      ++pos;
      if (b >= 0 && b < 128) {
        *out = v;
        return true;
      }
    }
    int b = at(pos);
    v |= uint32_t(b < 0 ? 0 : (b & 15)) << 28;
    ++pos;
    if (b >= 0 && b < 128) {
      *out = v;
      return true;
    }
    if ((pos += 5) > len) {
      pos = len;
      return out_of_range(10);
    }
    *out = v;
    return true;
  }

  // Reader.prototype.skip(length)
  bool skip_n(uint64_t n) {
    if (pos + n > len) return out_of_range(n);
    pos += n;
    return true;
  }

  // Reader.prototype.skip() (varint)
  bool skip_varint() {
    do {
      if (pos >= len) return out_of_range(0);
    } while (buf[pos++] & 128);
    return true;
  }

  // Reader.prototype.skipType(wireType)
  bool skip_type(uint32_t wt) {
    uint64_t depth = 0;
    for (;;) {
      switch (wt) {
        case 0:
          if (!skip_varint()) return false;
          break;
        case 1:
          if (!skip_n(8)) return false;
          break;
        case 2: {
          uint32_t n;
          if (!uint32(&n) || !skip_n(n)) return false;
          break;
        }
        case 3:
          ++depth;
          break;
        case 5:
          if (!skip_n(4)) return false;
          break;
        case 4:
          if (depth > 0) {
            --depth;
            break;
          }
          return invalid_wire_type(wt);
        default:
          return invalid_wire_type(wt);
      }
      if (depth == 0) return true;
      // inside a group: `while ((wireType = this.uint32() & 7) !== 4) this.skipType(wireType)`
      uint32_t t;
      if (!uint32(&t)) return false;
      wt = t & 7;
    }
  }

  // BufferReader.prototype.string: clamped slice, no UTF-8 validation (caller decodes)
  bool string(const uint8_t** p, size_t* n) {
    uint32_t L;
    if (!uint32(&L)) return false;
    uint64_t end = pos + L < len ? pos + L : len;
    *p = buf + pos;
    *n = size_t(end - pos);
    pos = end;
    return true;
  }

  // Reader.prototype.bytes
  bool bytes(const uint8_t** p, size_t* n) {
    uint32_t L;
    if (!uint32(&L)) return false;
    if (pos + L > len) return out_of_range(L);
    *p = buf + pos;
    *n = L;
    pos += L;
    return true;
  }

  bool fixed32(uint32_t* out) {
    if (pos + 4 > len) return out_of_range(4);
    std::memcpy(out, buf + pos, 4);
    pos += 4;
    return true;
  }

  bool fixed64(uint64_t* out) {
    if (pos + 8 > len) return out_of_range(8);
    std::memcpy(out, buf + pos, 8);
    pos += 8;
    return true;
  }
};

}  // namespace pbjs
}  // namespace beholder
