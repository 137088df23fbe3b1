// `beholder_amd.ops._native_bench`: bench, test and diagnostic machinery kept out of the
// service's extension: the in-process sink stub (recorder.cpp), the paced
// producer (paced.cpp), the calibration loops (calib.cpp), the sampling profiler (prof.cpp) and
// the shared-queue broker fake (shared_broker.cpp) and the e2e bench's Postgres fake (pg_fake.cpp).
#include "bench_common.hpp"

namespace beholder {
namespace bench {

const NativeApi* g_api = nullptr;

namespace {

PyModuleDef module_def = {PyModuleDef_HEAD_INIT, "_native_bench",
                          "beholder bench/diagnostic natives (sink stub, paced producer, calibration, profiler)", -1,
                          nullptr};

}  // namespace
}  // namespace bench
}  // namespace beholder

PyMODINIT_FUNC PyInit__native_bench(void) {
  using namespace beholder;
  // the service's extension first: the stub runs its request builder and response code
  void* p = PyCapsule_Import(kNativeApiName, 0);
  if (!p) return nullptr;
  const NativeApi* api = static_cast<const NativeApi*>(p);
  if (api->abi != kNativeApiAbi) {
    PyErr_Format(PyExc_ImportError, "_native_bench: _native C API abi %u, expected %u", api->abi, kNativeApiAbi);
    return nullptr;
  }
  bench::g_api = api;
  PyObject* m = PyModule_Create(&bench::module_def);
  if (!m) return nullptr;
  if (bench::init_calib(m) < 0 || bench::init_paced(m) < 0 || bench::init_recorder(m) < 0 || bench::init_shared_broker(m) < 0 ||
      bench::init_pg_fake(m) < 0 ||
      init_bench_prof(m) < 0) {
    Py_DECREF(m);
    return nullptr;
  }
  return m;
}
