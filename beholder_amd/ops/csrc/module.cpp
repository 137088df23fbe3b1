// `beholder_amd.ops._native` — native runtime for the beholder service.
//
// Contents: MessageCodec (protobuf decode/encode), Ingest (byte ring + reader
// thread), Delivery / Settler (ack semantics + latency), Counter / Histogram
// (metrics), plus framing helpers. See the per-file headers for the mapping
// to reference behaviour (/root/reference/index.js).
#include <cstdlib>
#include <string>
#include <vector>

#include "py_common.hpp"
#include "ring.hpp"

namespace beholder {

ModuleState g_state = {nullptr, nullptr};

namespace {

// configure(decode_error=None, topics=None)
PyObject* mod_configure(PyObject*, PyObject* args, PyObject* kwds) {
  static const char* kwlist[] = {"decode_error", "topics", nullptr};
  PyObject* de = Py_None;
  PyObject* topics = Py_None;
  if (!PyArg_ParseTupleAndKeywords(args, kwds, "|OO", const_cast<char**>(kwlist), &de, &topics)) return nullptr;
  if (de != Py_None) {
    if (!PyType_Check(de) || !PyType_IsSubtype(reinterpret_cast<PyTypeObject*>(de),
                                                reinterpret_cast<PyTypeObject*>(PyExc_Exception))) {
      PyErr_SetString(PyExc_TypeError, "decode_error must be an Exception subclass");
      return nullptr;
    }
    Py_INCREF(de);
    Py_XSETREF(g_state.decode_error, de);
  }
  if (topics != Py_None) {
    PyObject* t = PySequence_Tuple(topics);
    if (!t) return nullptr;
    Py_XSETREF(g_state.topics, t);
  }
  Py_RETURN_NONE;
}

PyObject* mod_mono_ns(PyObject*, PyObject*) { return PyLong_FromLongLong(mono_ns()); }

void append_frame(std::string& out, int topic, const char* p, size_t n) {
  uint32_t L = uint32_t(n + 1);
  char hdr[5] = {char(L & 0xff), char((L >> 8) & 0xff), char((L >> 16) & 0xff), char((L >> 24) & 0xff),
                 char(topic)};
  out.append(hdr, 5);
  out.append(p, n);
}

// frame(topic, payload) -> bytes  (u32le len | u8 topic | payload)
PyObject* mod_frame_impl(PyObject*, PyObject* args);
PyObject* mod_frame(PyObject*, PyObject* args) {
  BEHOLDER_TRY { return mod_frame_impl(nullptr, args); }
  BEHOLDER_CATCH(nullptr)
}

PyObject* mod_frame_impl(PyObject*, PyObject* args) {
  int topic;
  Py_buffer view;
  if (!PyArg_ParseTuple(args, "iy*", &topic, &view)) return nullptr;
  if (topic < 0 || topic > 255) {
    PyBuffer_Release(&view);
    PyErr_SetString(PyExc_ValueError, "topic must be in [0, 255]");
    return nullptr;
  }
  std::string out;
  out.reserve(size_t(view.len) + 5);
  append_frame(out, topic, static_cast<const char*>(view.buf), size_t(view.len));
  PyBuffer_Release(&view);
  return PyBytes_FromStringAndSize(out.data(), Py_ssize_t(out.size()));
}

// frames(iterable of (topic, payload)) -> bytes
PyObject* mod_frames_impl(PyObject*, PyObject* it_in);
PyObject* mod_frames(PyObject*, PyObject* it_in) {
  BEHOLDER_TRY { return mod_frames_impl(nullptr, it_in); }
  BEHOLDER_CATCH(nullptr)
}

PyObject* mod_frames_impl(PyObject*, PyObject* it_in) {
  PyObject* it = PyObject_GetIter(it_in);
  if (!it) return nullptr;
  std::string out;
  PyObject* item;
  while ((item = PyIter_Next(it))) {
    int topic;
    const char* p;
    Py_ssize_t n;
    if (!PyArg_ParseTuple(item, "iy#", &topic, &p, &n)) {
      Py_DECREF(item);
      Py_DECREF(it);
      return nullptr;
    }
    append_frame(out, topic, p, size_t(n));
    Py_DECREF(item);
  }
  Py_DECREF(it);
  if (PyErr_Occurred()) return nullptr;
  return PyBytes_FromStringAndSize(out.data(), Py_ssize_t(out.size()));
}

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

// untrack_row(row) -> row (store/base.py): a NamedTuple row of atoms leaves the cyclic collector.
PyObject* mod_untrack_row(PyObject*, PyObject* t) {
  if (!PyTuple_Check(t)) {
    PyErr_SetString(PyExc_TypeError, "untrack_row expects a tuple (a Media row)");
    return nullptr;
  }
  untrack_atomic_row(t);
  return Py_NewRef(t);
}

PyMethodDef module_methods[] = {
    {"untrack_row", mod_untrack_row, METH_O,
     "untrack_row(row) -> row: a tuple row holding only atoms leaves the cyclic collector"},
    {"calib_mem", mod_calib_mem, METH_VARARGS,
     "calib_mem(bytes, steps) -> (ns, checksum): fixed-work dependent random walk over `bytes`"},
    {"calib", mod_calib, METH_VARARGS, "calib(iters) -> (ns, checksum): fixed-work CPU calibration loop"},
    {"configure", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(mod_configure)),
     METH_VARARGS | METH_KEYWORDS, "configure(decode_error=None, topics=None)"},
    {"mono_ns", mod_mono_ns, METH_NOARGS, "CLOCK_MONOTONIC in ns (same clock as time.monotonic_ns)"},
    {"frame", mod_frame, METH_VARARGS, "frame(topic, payload) -> framed bytes"},
    {"frames", mod_frames, METH_O, "frames(iterable of (topic, payload)) -> framed bytes"},
    {nullptr, nullptr, 0, nullptr}};

PyModuleDef module_def = {PyModuleDef_HEAD_INIT, "_native",
                          "beholder native runtime (codec, ingest ring, deliveries, metrics)", -1, module_methods};

}  // namespace
}  // namespace beholder

PyMODINIT_FUNC PyInit__native(void) {
  using namespace beholder;
  PyObject* m = PyModule_Create(&module_def);
  if (!m) return nullptr;
  if (init_metric_types(m) < 0 || init_codec_types(m) < 0 || init_ingest_types(m) < 0 ||
      init_text_functions(m) < 0 || init_amqp_types(m) < 0 ||
      init_dispatch_functions(m) < 0 || init_http_types(m) < 0 ||
      init_pg_types(m) < 0 || init_driver_types(m) < 0 ||
      init_ack_types(m) < 0 || init_handler_types(m) < 0 || init_netconn_types(m) < 0 || init_h1call_types(m) < 0 ||
      init_tls_types(m) < 0 || init_netpoll_types(m) < 0 || init_prof_functions(m) < 0 ||
      init_recorder_types(m) < 0) {
    Py_DECREF(m);
    return nullptr;
  }
  g_state.topics = PyTuple_New(0);
  PyModule_AddIntConstant(m, "ABI_VERSION", 1);
  PyModule_AddIntConstant(m, "RECORD_HEADER_BYTES", int(sizeof(RecordHeader)));
  return m;
}
