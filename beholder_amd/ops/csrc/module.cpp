// `beholder_amd.ops._native` — native runtime for the beholder service.
//
// Contents: MessageCodec (protobuf decode/encode), Ingest (byte ring + reader
// thread), Delivery / Settler (ack semantics + latency), Counter / Histogram
// (metrics), plus framing helpers. Bench and diagnostic code (the sink stub, the
// paced producer, calibration loops, the sampling profiler) is not linked here: it
// is `_native_bench` (csrc_bench/), which reaches this module through `_C_API`. See the per-file headers for the mapping
// to reference behaviour (/root/reference/index.js).
#include <cstdlib>
#include <string>
#include <vector>

#include "native_api.hpp"
#include "py_common.hpp"
#include "ring.hpp"

namespace beholder {

ModuleState g_state = {nullptr, nullptr};

PyObject* url_with_query(PyObject* url, PyObject* params);  // py_text.cpp
int api_h1_request_text(PyObject* method, PyObject* url, PyObject* params, PyObject* host, PyObject* auth,
                        PyObject* tail, PyObject* tail_cl0, std::string* req, PyObject** full,
                        Py_ssize_t* key_len);  // py_h1call.cpp
PyObject* api_h1_response(PyObject* parsed, PyObject* full);  // py_h1call.cpp
int api_h1_origin_key(PyObject* method, PyObject* url, PyObject* params, Py_ssize_t* key_len);  // py_h1call.cpp

bool is_h1_parser(PyObject* o);  // py_http.cpp
int h1_parser_start_c(PyObject* o, bool head);
PyObject* h1_parser_feed_c(PyObject* o, const char* data, size_t n);

const NativeApi g_api = {kNativeApiAbi,  api_h1_origin_key, api_h1_request_text, api_h1_response,
                         url_with_query, is_h1_parser,      h1_parser_start_c,   h1_parser_feed_c};

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
      init_tls_types(m) < 0 || init_netpoll_types(m) < 0 || init_clock_functions(m) < 0) {
    Py_DECREF(m);
    return nullptr;
  }
  // the C interface for the package's other extension modules (native_api.hpp)
  PyObject* api = PyCapsule_New(const_cast<NativeApi*>(&g_api), kNativeApiName, nullptr);
  if (!api || PyModule_AddObject(m, "_C_API", api) < 0) {
    Py_XDECREF(api);
    Py_DECREF(m);
    return nullptr;
  }
  g_state.topics = PyTuple_New(0);
  PyModule_AddIntConstant(m, "ABI_VERSION", 1);
  PyModule_AddIntConstant(m, "RECORD_HEADER_BYTES", int(sizeof(RecordHeader)));
  return m;
}
