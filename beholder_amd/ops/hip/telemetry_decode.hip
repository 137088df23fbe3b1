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
// (offsets are absolute in buf). Proto3 rules: last value wins, unknown fields of wire types
// 0/1/2/5 are skipped, a known field with an unexpected wire type is skipped like an unknown
// one, truncation or wire types 3/4/6/7 set ok = 0.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

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

__global__ __launch_bounds__(256) void decode_telemetry(const uint8_t* __restrict__ buf,
                                                        const int32_t* __restrict__ offs, int n,
                                                        int4* __restrict__ out) {
  const int m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= n) return;
  int i = offs[m];
  const int end = offs[m + 1];
  int id_off = 0, id_len = 0, status = 0, progress = 0, host_off = 0, host_len = 0, ok = 1, seen = 0;
  while (i < end) {
    uint64_t key;
    if (!read_varint(buf, end, i, key)) { ok = 0; break; }
    const uint32_t field = static_cast<uint32_t>(key >> 3), wt = static_cast<uint32_t>(key & 7);
    if (field == 0) { ok = 0; break; }
    if (wt == 0) {
      uint64_t v;
      if (!read_varint(buf, end, i, v)) { ok = 0; break; }
      if (field == 2) { status = static_cast<int32_t>(v); seen |= 2; }
      else if (field == 3) { progress = static_cast<int32_t>(v); seen |= 4; }
    } else if (wt == 2) {
      uint64_t len;
      if (!read_varint(buf, end, i, len) || len > static_cast<uint64_t>(end - i)) { ok = 0; break; }
      if (field == 1) { id_off = i; id_len = static_cast<int>(len); seen |= 1; }
      else if (field == 4) { host_off = i; host_len = static_cast<int>(len); seen |= 8; }
      i += static_cast<int>(len);
    } else if (wt == 1) {
      if (end - i < 8) { ok = 0; break; }
      i += 8;
    } else if (wt == 5) {
      if (end - i < 4) { ok = 0; break; }
      i += 4;
    } else {
      ok = 0;
      break;
    }
  }
  out[2 * m] = make_int4(id_off, id_len, status, progress);
  out[2 * m + 1] = make_int4(host_off, host_len, ok, seen);
}

}  // namespace

// C ABI for ctypes (ops/gpu_decode.py). All pointers are device pointers from torch tensors on the
// caller's device; `stream` is the torch stream (hipStream_t). Returns a hipError_t.
extern "C" __attribute__((visibility("default"))) int bh_decode_telemetry(const void* buf, const void* offs, int n,
                                                                         void* out, void* stream) {
  if (n <= 0) return 0;
  const int block = 256;
  const int grid = (n + block - 1) / block;
  hipLaunchKernelGGL(decode_telemetry, dim3(grid), dim3(block), 0, static_cast<hipStream_t>(stream),
                     static_cast<const uint8_t*>(buf), static_cast<const int32_t*>(offs), n,
                     static_cast<int4*>(out));
  return static_cast<int>(hipGetLastError());
}
