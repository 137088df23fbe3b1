// Protobuf wire-format primitives for the native codec (no Python dependency).
//
// Beholder decodes every inbound telemetry message (index.js:63,129 in the
// reference, `proto.decode(...)` via protobufjs). These helpers implement the
// subset of the wire format our flat telemetry messages need, with the same
// acceptance rules as upb (google.protobuf), which the tests use as the oracle:
//   * a known field whose wire type does not match its declared type is
//     treated as an unknown field and skipped;
//   * unknown fields (incl. groups) are skipped;
//   * truncated input, varints longer than 10 bytes, tags longer than 5 bytes
//     or wider than 32 bits, field number 0, stray END_GROUP and wire types 6/7
//     are errors;
//   * a 10-byte value varint keeps bit 63 and drops the overflow bits of its
//     last byte (upb does the same).
#pragma once

#include <cstddef>
#include <cstdint>
#include <cstring>

namespace beholder {
namespace wire {

enum WireType : uint32_t {
  WT_VARINT = 0,
  WT_I64 = 1,
  WT_LEN = 2,
  WT_SGROUP = 3,
  WT_EGROUP = 4,
  WT_I32 = 5,
};

// Field kinds understood by the flat-message codec. Values are part of the
// Python<->C++ contract (mirrored in beholder_amd/ops/__init__.py).
enum Kind : int {
  K_STRING = 1,
  K_BYTES = 2,
  K_INT32 = 3,
  K_INT64 = 4,
  K_UINT32 = 5,
  K_UINT64 = 6,
  K_SINT32 = 7,
  K_SINT64 = 8,
  K_BOOL = 9,
  K_ENUM = 10,
  K_FLOAT = 11,
  K_DOUBLE = 12,
  K_FIXED32 = 13,
  K_FIXED64 = 14,
  K_SFIXED32 = 15,
  K_SFIXED64 = 16,
};

inline uint32_t expected_wire_type(int kind) {
  switch (kind) {
    case K_STRING:
    case K_BYTES:
      return WT_LEN;
    case K_FLOAT:
    case K_FIXED32:
    case K_SFIXED32:
      return WT_I32;
    case K_DOUBLE:
    case K_FIXED64:
    case K_SFIXED64:
      return WT_I64;
    default:
      return WT_VARINT;
  }
}

struct Reader {
  const uint8_t* p;
  const uint8_t* end;
  const char* err = nullptr;

  Reader(const uint8_t* b, size_t n) : p(b), end(b + n) {}

  bool eof() const { return p >= end; }

  // Reads a base-128 varint (max 10 bytes). Returns false + sets err on failure.
  inline bool varint(uint64_t* out) {
    if (p < end && *p < 0x80) {  // 1-byte fast path (tags, small enums, progress %)
      *out = *p++;
      return true;
    }
    uint64_t v = 0;
    for (int shift = 0; shift < 70; shift += 7) {
      if (p >= end) {
        err = "truncated varint";
        return false;
      }
      uint8_t b = *p++;
      // 10th byte: bit 0 is bit 63 of the value; higher bits overflow and are dropped,
      // exactly as upb does (a continuation bit there is still an error, below)
      v |= uint64_t(b & 0x7f) << shift;
      if (b < 0x80) {
        *out = v;
        return true;
      }
    }
    err = "varint too long";
    return false;
  }

  // Reads a field tag: a varint of at most 5 bytes whose value fits 32 bits (upb's rule;
  // a longer encoding of a small tag is still an error).
  inline bool tag(uint64_t* out) {
    if (p < end && *p < 0x80) {
      *out = *p++;
      return true;
    }
    uint64_t v = 0;
    for (int i = 0; i < 5; ++i) {
      if (p >= end) {
        err = "truncated varint";
        return false;
      }
      uint8_t b = *p++;
      v |= uint64_t(b & 0x7f) << (7 * i);
      if (b < 0x80) {
        if (v > 0xffffffffull) {
          err = "tag overflow";
          return false;
        }
        *out = v;
        return true;
      }
    }
    err = "tag too long";
    return false;
  }

  inline bool fixed32(uint32_t* out) {
    if (end - p < 4) {
      err = "truncated fixed32";
      return false;
    }
    std::memcpy(out, p, 4);
    p += 4;
    return true;
  }

  inline bool fixed64(uint64_t* out) {
    if (end - p < 8) {
      err = "truncated fixed64";
      return false;
    }
    std::memcpy(out, p, 8);
    p += 8;
    return true;
  }

  inline bool bytes(const uint8_t** data, size_t* len) {
    uint64_t n;
    if (!varint(&n)) return false;
    if (n > uint64_t(end - p)) {
      err = "truncated length-delimited field";
      return false;
    }
    *data = p;
    *len = size_t(n);
    p += n;
    return true;
  }

  // Skip one field body of wire type `wt` whose tag has been consumed.
  bool skip(uint32_t wt, uint32_t field, int depth = 0) {
    uint64_t tmp;
    const uint8_t* d;
    size_t n;
    switch (wt) {
      case WT_VARINT:
        return varint(&tmp);
      case WT_I64:
        return fixed64(&tmp);
      case WT_LEN:
        return bytes(&d, &n);
      case WT_I32: {
        uint32_t t32;
        return fixed32(&t32);
      }
      case WT_SGROUP: {
        if (depth > 64) {
          err = "group nesting too deep";
          return false;
        }
        for (;;) {
          uint64_t tag;
          if (p >= end) {
            err = "unterminated group";
            return false;
          }
          if (!this->tag(&tag)) return false;
          // field number 0 is tolerated inside a skipped group (upb only rejects it at
          // message level)
          uint32_t f = uint32_t(tag >> 3), w = uint32_t(tag & 7);
          if (w == WT_EGROUP) {
            if (f != field) {
              err = "mismatched end group";
              return false;
            }
            return true;
          }
          if (!skip(w, f, depth + 1)) return false;
        }
      }
      case WT_EGROUP:
        err = "unexpected end group";
        return false;
      default:
        err = "invalid wire type";
        return false;
    }
  }
};

// ---- encoding -----------------------------------------------------------
inline size_t varint_size(uint64_t v) {
  size_t n = 1;
  while (v >= 0x80) {
    v >>= 7;
    ++n;
  }
  return n;
}

inline uint8_t* put_varint(uint8_t* out, uint64_t v) {
  while (v >= 0x80) {
    *out++ = uint8_t(v) | 0x80;
    v >>= 7;
  }
  *out++ = uint8_t(v);
  return out;
}

inline uint64_t zigzag64(int64_t v) { return (uint64_t(v) << 1) ^ uint64_t(v >> 63); }
inline uint32_t zigzag32(int32_t v) { return (uint32_t(v) << 1) ^ uint32_t(v >> 31); }
inline int64_t unzigzag64(uint64_t v) { return int64_t(v >> 1) ^ -int64_t(v & 1); }
inline int32_t unzigzag32(uint32_t v) { return int32_t(v >> 1) ^ -int32_t(v & 1); }

}  // namespace wire
}  // namespace beholder
