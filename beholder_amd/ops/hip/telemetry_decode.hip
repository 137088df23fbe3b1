// Batched telemetry decode on the GPU (gfx950): the offload probe behind docs/DESIGN.md
// "Why there are no HIP kernels".
//
// The service decodes one ~50-byte protobuf per event on the CPU (ops/csrc/py_codec.cpp, the
// `decode` of index.js:63,129). This kernel decodes a whole batch of TelemetryProgress /
// TelemetryStatus messages (models/proto/api.proto: mediaId=1, status=2, progress=3, host=4)
// so scripts/gpu_offload_probe.py can price the alternative design: gather events into a
// pinned batch, copy it to HBM, decode, copy the fields back.
//
// Layout: `buf` holds the concatenated message bodies, `offs[n + 1]` their boundaries (checked
// on the host: offs[0] = 0, non-decreasing, offs[n] = bytes in buf). One lane per message: the
// work is a varint state machine with data-dependent branches, so a 64-wide wavefront decodes 64
// messages side by side and diverges where their layouts differ. Each lane emits 8 int32:
//   [id_off, id_len, status, progress, host_off, host_len, ok, fields_seen]
// (offsets are absolute in buf; ok = 0 where the CPU codec raises DecodeError).
//
// Two dialects, the same two the CPU codec has (ops/__init__.py DIALECTS); valid input decodes
// identically in both:
//
//  * DIALECT_PROTOBUFJS (the service's default, handlers.py `_dialect`): protobufjs 6.8.8's
//    BufferReader and generated decoder, rule for rule as ops/csrc/pbjs.hpp models them:
//      - the tag and every known field are read with Reader.uint32(): up to 5 bytes, a byte past
//        the end reads as `undefined` (0, continuation), a 5th byte with its continuation bit
//        skips 5 more bytes unchecked and fails only if that passes the end;
//      - a known field is read with its declared type whatever wire type its tag carries
//        (mediaId / host: string, status: enum, progress: int32, both `uint32() | 0`);
//      - strings are clamped to the message end (BufferReader.string), never an error;
//      - field number 0 and unknown fields are skipped with skipType(wt & 7): varints unbounded
//        but end-checked, 64/32-bit and length-delimited bounds-checked, groups skipped up to
//        the next end-group tag of any field (counted, not recursed), wire types 4/6/7 fail.
//  * DIALECT_UPB (google.protobuf's rules, the tooling oracle): last value wins, unknown fields
//    of wire types 0/1/2/5 are skipped, a known field with an unexpected wire type is skipped
//    like an unknown one, field 0, truncation or wire types 3/4/6/7 set ok = 0.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

constexpr int DIALECT_UPB = 0;
constexpr int DIALECT_PROTOBUFJS = 1;

// ---- upb ------------------------------------------------------------------------------------

__device__ __forceinline__ bool read_varint(const uint8_t* __restrict__ p, int end, int& i, uint64_t& v) {
  v = 0;
#pragma unroll
  for (int shift = 0; shift < 70; shift += 7) {
    if (i >= end) return false;
    const uint32_t b = p[i++];
    v |= static_cast<uint64_t>(b & 0x7fu) << shift;
    if (!(b & 0x80u)) return true;
  }
  return false;  // more than 10 bytes
}

__device__ __forceinline__ void decode_upb(const uint8_t* __restrict__ buf, int i, const int end, int* r) {
  while (i < end) {
    uint64_t key;
    if (!read_varint(buf, end, i, key)) { r[6] = 0; return; }
    const uint32_t field = static_cast<uint32_t>(key >> 3), wt = static_cast<uint32_t>(key & 7);
    if (field == 0) { r[6] = 0; return; }
    if (wt == 0) {
      uint64_t v;
      if (!read_varint(buf, end, i, v)) { r[6] = 0; return; }
      if (field == 2) { r[2] = static_cast<int32_t>(v); r[7] |= 2; }
      else if (field == 3) { r[3] = static_cast<int32_t>(v); r[7] |= 4; }
    } else if (wt == 2) {
      uint64_t len;
      if (!read_varint(buf, end, i, len) || len > static_cast<uint64_t>(end - i)) { r[6] = 0; return; }
      if (field == 1) { r[0] = i; r[1] = static_cast<int>(len); r[7] |= 1; }
      else if (field == 4) { r[4] = i; r[5] = static_cast<int>(len); r[7] |= 8; }
      i += static_cast<int>(len);
    } else if (wt == 1) {
      if (end - i < 8) { r[6] = 0; return; }
      i += 8;
    } else if (wt == 5) {
      if (end - i < 4) { r[6] = 0; return; }
      i += 4;
    } else {
      r[6] = 0;
      return;
    }
  }
}

// ---- protobufjs 6.8.8 -------------------------------------------------------------------------
// Positions are relative to the message start and may step past its end: Reader.uint32() reads
// `undefined` bytes before it reports the overrun, exactly as pbjs.hpp does. 32-bit arithmetic
// (messages are < 2^31 bytes, checked on the host) and an unchecked fast path while at least 5
// bytes remain keep the per-byte work at the upb kernel's level; only the last bytes of a
// message take the bounds-checked path.

struct PbjsReader {
  const uint8_t* __restrict__ p;  // message start
  int len;
  int pos;

  __device__ __forceinline__ int at(int i) const { return i < len ? int(p[i]) : -1; }

  // Reader.prototype.uint32
  __device__ __forceinline__ bool uint32(uint32_t& out) {
    if (pos + 5 <= len) {  // every byte it may read is inside the message
      uint32_t b = p[pos++];
      uint32_t v = b & 127u;
      if (b < 128u) { out = v; return true; }
      b = p[pos++]; v |= (b & 127u) << 7;
      if (b < 128u) { out = v; return true; }
      b = p[pos++]; v |= (b & 127u) << 14;
      if (b < 128u) { out = v; return true; }
      b = p[pos++]; v |= (b & 127u) << 21;
      if (b < 128u) { out = v; return true; }
      b = p[pos++]; v |= (b & 15u) << 28;
      if (b < 128u) { out = v; return true; }
      pos += 5;  // the 64-bit tail, unchecked byte by byte
      if (pos > len) { pos = len; return false; }
      out = v;
      return true;
    }
    uint32_t v = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int b = at(pos);
      v |= uint32_t(b < 0 ? 0 : (b & 127)) << (7 * k);
      ++pos;
      if (b >= 0 && b < 128) { out = v; return true; }
    }
    const int b = at(pos);
    v |= uint32_t(b < 0 ? 0 : (b & 15)) << 28;
    ++pos;
    if (b >= 0 && b < 128) { out = v; return true; }
    pos += 5;
    if (pos > len) { pos = len; return false; }
    out = v;
    return true;
  }

  __device__ __forceinline__ bool skip_n(uint32_t n) {
    if (n > uint32_t(len - pos)) return false;  // pos <= len here
    pos += int(n);
    return true;
  }

  __device__ __forceinline__ bool skip_varint() {
    for (;;) {
      if (pos >= len) return false;
      if (!(p[pos++] & 128)) return true;
    }
  }

  // Reader.prototype.skipType(wireType), groups counted instead of recursed into
  __device__ __forceinline__ bool skip_type(uint32_t wt) {
    uint32_t depth = 0;
    for (;;) {
      switch (wt) {
        case 0: if (!skip_varint()) return false; break;
        case 1: if (!skip_n(8)) return false; break;
        case 2: {
          uint32_t n;
          if (!uint32(n) || !skip_n(n)) return false;
          break;
        }
        case 3: ++depth; break;
        case 5: if (!skip_n(4)) return false; break;
        case 4:
          if (depth > 0) { --depth; break; }
          return false;
        default: return false;
      }
      if (depth == 0) return true;
      uint32_t t;
      if (!uint32(t)) return false;
      wt = t & 7;
    }
  }

  // BufferReader.prototype.string: the byte range clamped to the end
  __device__ __forceinline__ bool string(int& off, int& n) {
    uint32_t L;
    if (!uint32(L)) return false;
    const int e = L < uint32_t(len - pos) ? pos + int(L) : len;  // pos <= len here
    off = pos;
    n = e - pos;
    pos = e;
    return true;
  }
};

__device__ __forceinline__ void decode_pbjs(const uint8_t* __restrict__ buf, const int start, const int end, int* r) {
  PbjsReader rd{buf + start, end - start, 0};
  while (rd.pos < rd.len) {
    uint32_t t;
    if (!rd.uint32(t)) { r[6] = 0; return; }
    const uint32_t field = t >> 3;
    if (field == 1 || field == 4) {  // string mediaId / host
      int off, n;
      if (!rd.string(off, n)) { r[6] = 0; return; }
      if (field == 1) { r[0] = start + off; r[1] = n; r[7] |= 1; }
      else { r[4] = start + off; r[5] = n; r[7] |= 8; }
    } else if (field == 2 || field == 3) {  // enum status / int32 progress: uint32() | 0
      uint32_t v;
      if (!rd.uint32(v)) { r[6] = 0; return; }
      if (field == 2) { r[2] = static_cast<int32_t>(v); r[7] |= 2; }
      else { r[3] = static_cast<int32_t>(v); r[7] |= 4; }
    } else if (!rd.skip_type(t & 7)) {
      r[6] = 0;
      return;
    }
  }
}

template <int DIALECT>
__global__ __launch_bounds__(256) void decode_telemetry(const uint8_t* __restrict__ buf,
                                                        const int32_t* __restrict__ offs, int n,
                                                        int4* __restrict__ out) {
  const int m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= n) return;
  const int start = offs[m];
  const int end = offs[m + 1];
  int r[8] = {0, 0, 0, 0, 0, 0, 1, 0};
  if (DIALECT == DIALECT_PROTOBUFJS)
    decode_pbjs(buf, start, end, r);
  else
    decode_upb(buf, start, end, r);
  out[2 * m] = make_int4(r[0], r[1], r[2], r[3]);
  out[2 * m + 1] = make_int4(r[4], r[5], r[6], r[7]);
}

}  // namespace

// C ABI for ctypes (ops/gpu_decode.py). All pointers are device pointers from torch tensors on the
// caller's device; `stream` is the torch stream (hipStream_t); `dialect` 0 = upb, 1 = protobufjs.
// Returns a hipError_t (hipErrorInvalidValue for an unknown dialect).
extern "C" __attribute__((visibility("default"))) int bh_decode_telemetry(const void* buf, const void* offs, int n,
                                                                         void* out, void* stream, int dialect) {
  if (n <= 0) return 0;
  if (dialect != DIALECT_UPB && dialect != DIALECT_PROTOBUFJS) return static_cast<int>(hipErrorInvalidValue);
  const int block = 256;
  const int grid = (n + block - 1) / block;
  const auto* b = static_cast<const uint8_t*>(buf);
  const auto* o = static_cast<const int32_t*>(offs);
  auto* t = static_cast<int4*>(out);
  if (dialect == DIALECT_PROTOBUFJS)
    hipLaunchKernelGGL(decode_telemetry<DIALECT_PROTOBUFJS>, dim3(grid), dim3(block), 0,
                       static_cast<hipStream_t>(stream), b, o, n, t);
  else
    hipLaunchKernelGGL(decode_telemetry<DIALECT_UPB>, dim3(grid), dim3(block), 0, static_cast<hipStream_t>(stream),
                       b, o, n, t);
  return static_cast<int>(hipGetLastError());
}
