// Shared declarations for `_native_bench` (ops/csrc_bench/): the bench and diagnostic
// extension. It is built next to the service's `_native` but never linked into it, and the
// runtime image does not ship it (Dockerfile). It reaches the service's native code through
// `_native._C_API` (csrc/native_api.hpp).
#pragma once

#define PY_SSIZE_T_CLEAN
#include <Python.h>

#include <time.h>

#include <cstdint>

#include "native_api.hpp"

namespace beholder {
namespace bench {

inline int64_t mono_ns() {  // CLOCK_MONOTONIC, the clock of every Delivery timestamp
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return int64_t(ts.tv_sec) * 1000000000LL + ts.tv_nsec;
}

extern const NativeApi* g_api;  // set by PyInit__native_bench

int init_calib(PyObject* m);
int init_paced(PyObject* m);
int init_recorder(PyObject* m);
int init_shared_broker(PyObject* m);
int init_pg_fake(PyObject* m);

}  // namespace bench

int init_bench_prof(PyObject* m);

}  // namespace beholder
