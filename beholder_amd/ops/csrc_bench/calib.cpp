// Fixed-work calibration loops for the bench line (bench.py calib_*): how fast this core and
// its caches are right now, independent of the service's code.
#include <cstdlib>
#include <string>
#include <vector>

#include "bench_common.hpp"
#include "py_common.hpp"  // ScratchStr, BEHOLDER_TRY (header-only: this module keeps its own pool)

namespace beholder {
namespace bench {
namespace {

// calib(iters) -> ns: a fixed amount of integer work (xorshift mixing through a
// 16 KiB, L1-resident table; a dependent chain, so neither vectorised nor
// removable). Its time moves only with the core's clock and with other load on
// the core, never with this service's code, so the bench line can tell a slow
// box from a slow build. Runs without the GIL.
PyObject* mod_calib(PyObject*, PyObject* args) {
  unsigned long long iters;
  if (!PyArg_ParseTuple(args, "K", &iters)) return nullptr;
  int64_t t0, t1;
  uint64_t acc;
  Py_BEGIN_ALLOW_THREADS
  uint32_t table[4096];
  uint64_t x = 0x9E3779B97F4A7C15ull;
  for (uint32_t i = 0; i < 4096; ++i) {
    x ^= x << 13;
    x ^= x >> 7;
    x ^= x << 17;
    table[i] = uint32_t(x);
  }
  t0 = mono_ns();
  acc = 0;
  for (unsigned long long i = 0; i < iters; ++i) {
    x ^= x << 13;
    x ^= x >> 7;
    x ^= x << 17;
    uint32_t v = table[(x ^ acc) & 4095];
    acc = (acc * 31) + v;
    table[acc & 4095] = v ^ uint32_t(i);
  }
  t1 = mono_ns();
  Py_END_ALLOW_THREADS
  return Py_BuildValue("(LK)", (long long)(t1 - t0), (unsigned long long)acc);
}

// calib_mem(bytes, steps) -> (ns, checksum): a dependent random walk over `bytes` of cache lines
// (one random cycle through every line, Sattolo's shuffle). With 16 MiB it lives in the L3 a
// core shares with its CCD neighbours, so its time moves with other tenants' cache and memory
// traffic -- which an L1-resident loop (calib) cannot see and a Python consumer, whose objects
// are scattered over the heap, does. Setup is outside the timed region; runs without the GIL.
PyObject* mod_calib_mem(PyObject*, PyObject* args) {
  unsigned long long bytes, steps;
  if (!PyArg_ParseTuple(args, "KK", &bytes, &steps)) return nullptr;
  const size_t lines = size_t(bytes / 64);
  if (lines < 2 || lines > (size_t(1) << 26)) {
    PyErr_SetString(PyExc_ValueError, "calib_mem: bytes must be in [128, 4 GiB]");
    return nullptr;
  }
  uint64_t* a = static_cast<uint64_t*>(std::aligned_alloc(64, lines * 64));
  if (!a) return PyErr_NoMemory();
  std::vector<uint32_t> perm;
  try {
    perm.resize(lines);
  } catch (const std::bad_alloc&) {
    std::free(a);
    return PyErr_NoMemory();
  }
  int64_t t0, t1;
  uint64_t idx = 0;
  Py_BEGIN_ALLOW_THREADS
  for (size_t i = 0; i < lines; ++i) perm[i] = uint32_t(i);
  uint64_t x = 0x2545F4914F6CDD1Dull;
  for (size_t i = lines - 1; i > 0; --i) {  // Sattolo: a single cycle through every line
    x ^= x << 13;
    x ^= x >> 7;
    x ^= x << 17;
    size_t j = size_t(x % i);
    uint32_t t = perm[i];
    perm[i] = perm[j];
    perm[j] = t;
  }
  for (size_t i = 0; i < lines; ++i) a[size_t(i) * 8] = perm[i];
  for (size_t i = 0; i < lines; ++i) idx = a[idx * 8];  // one warm lap
  t0 = mono_ns();
  for (unsigned long long s = 0; s < steps; ++s) idx = a[idx * 8];
  t1 = mono_ns();
  Py_END_ALLOW_THREADS
  std::free(a);
  return Py_BuildValue("(LK)", (long long)(t1 - t0), (unsigned long long)idx);
}

// scratch_probe(text, fn) -> str: a ScratchStr (py_common.hpp) holding `text`, then fn() (any
// Python code: it may hand the GIL to other threads), then the ScratchStr's content, which nothing
// else may have been lent meanwhile (tests/test_native_tools.py)
PyObject* mod_scratch_probe(PyObject*, PyObject* args) {
  const char* t;
  Py_ssize_t n;
  PyObject* fn;
  if (!PyArg_ParseTuple(args, "s#O", &t, &n, &fn)) return nullptr;
  BEHOLDER_TRY {
    ScratchStr buf_;
    std::string& buf = *buf_;
    buf.assign(t, size_t(n));
    PyObject* r = PyObject_CallNoArgs(fn);
    if (!r) return nullptr;
    Py_DECREF(r);
    return PyUnicode_FromStringAndSize(buf.data(), Py_ssize_t(buf.size()));
  }
  BEHOLDER_CATCH(nullptr)
}

// request_text_probe(method, url, params, key_len) -> (rc, request bytes, full URL, key_len): the
// _C_API's h1_request_text with Host "h", no Authorization and an empty tail (tests)
PyObject* mod_request_text_probe(PyObject*, PyObject* args) {
  PyObject *method, *url, *params;
  Py_ssize_t k;
  if (!PyArg_ParseTuple(args, "OOOn", &method, &url, &params, &k)) return nullptr;
  BEHOLDER_TRY {
    PyObject* host = PyUnicode_FromString("h");
    PyObject* tail = PyBytes_FromString("\r\n");
    if (!host || !tail) {
      Py_XDECREF(host);
      Py_XDECREF(tail);
      return nullptr;
    }
    std::string req;
    PyObject* full = nullptr;
    const int rc = g_api->h1_request_text(method, url, params, host, Py_None, tail, tail, &req, &full, &k);
    Py_DECREF(host);
    Py_DECREF(tail);
    if (rc < 0) return nullptr;
    PyObject* out = Py_BuildValue("(iy#On)", rc, req.data(), Py_ssize_t(req.size()), full ? full : Py_None, k);
    Py_XDECREF(full);
    return out;
  }
  BEHOLDER_CATCH(nullptr)
}

// origin_key_probe(method, url, params) -> (rc, key_len): the _C_API's h1_origin_key (tests)
PyObject* mod_origin_key_probe(PyObject*, PyObject* args) {
  PyObject *method, *url, *params;
  if (!PyArg_ParseTuple(args, "OOO", &method, &url, &params)) return nullptr;
  Py_ssize_t k = 0;
  const int rc = g_api->h1_origin_key(method, url, params, &k);
  if (rc < 0) return nullptr;
  return Py_BuildValue("(in)", rc, k);
}

PyMethodDef calib_methods[] = {
    {"origin_key_probe", mod_origin_key_probe, METH_VARARGS, "origin_key_probe(method, url, params) -> (rc, key_len)"},
    {"request_text_probe", mod_request_text_probe, METH_VARARGS,
     "request_text_probe(method, url, params, key_len) -> (rc, request, full, key_len)"},
    {"scratch_probe", mod_scratch_probe, METH_VARARGS,
     "scratch_probe(text, fn) -> text as a scratch string holds it after fn() ran"},
    {"calib_mem", mod_calib_mem, METH_VARARGS,
     "calib_mem(bytes, steps) -> (ns, checksum): fixed-work dependent random walk over `bytes`"},
    {"calib", mod_calib, METH_VARARGS, "calib(iters) -> (ns, checksum): fixed-work CPU calibration loop"},
    {nullptr, nullptr, 0, nullptr}};

}  // namespace

int init_calib(PyObject* m) { return PyModule_AddFunctions(m, calib_methods); }

}  // namespace bench
}  // namespace beholder
