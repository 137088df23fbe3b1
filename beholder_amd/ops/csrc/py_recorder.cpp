// Native core of the in-process HTTP recorder (sinks/http.py RecordingHttpClient), the sink stub
// of the headline bench and of the tests: "Trello/Telegram/Emby stubbed in-process".
//
// Per request it does what the Python stub did, in C: count it, build the full request URL
// (url + the Trello query, encodeURIComponent-encoded, in key order: index.js:53,83 through
// restler/qs), append (METHOD, url) to the client's bounded call log (a collections.deque), and
// answer 200 "{}". The compiled handlers (py_handlers.cpp http_request) call it directly when the
// client exposes it as `native_record` (no fault rules, no simulated delay), as they call the
// H1 client's native request path in production; everything else goes through the Python
// `request` coroutine, which records through the same core (`record`).
//
// The answer is a shared, already-completed awaitable (`Ready`) whose result is the client's
// shared `200 {}` HttpResponse: awaiting it returns at once, as the Python stub's coroutine did.
#include <string>

#include "py_common.hpp"

namespace beholder {

PyObject* url_with_query(PyObject* url, PyObject* params);  // py_text.cpp

namespace {

// ---- Ready: an awaitable that completes immediately with `value` -------------------------
struct ReadyObject {
  PyObject_HEAD PyObject* value;
};

PyTypeObject ReadyType = {PyVarObject_HEAD_INIT(nullptr, 0)};

void ready_dealloc(ReadyObject* self) {
  Py_XDECREF(self->value);
  Py_TYPE(self)->tp_free(reinterpret_cast<PyObject*>(self));
}

PyObject* ready_await(PyObject* self) { return Py_NewRef(self); }

PySendResult ready_send(PyObject* self, PyObject*, PyObject** result) {
  *result = Py_NewRef(reinterpret_cast<ReadyObject*>(self)->value);
  return PYGEN_RETURN;
}

PyObject* ready_next(PyObject* self) {  // `await` from Python code: StopIteration(value)
  PyObject* v = reinterpret_cast<ReadyObject*>(self)->value;
  PyObject* e = PyObject_CallOneArg(PyExc_StopIteration, v);
  if (!e) return nullptr;
  PyErr_SetObject(PyExc_StopIteration, e);
  Py_DECREF(e);
  return nullptr;
}

PyAsyncMethods ready_async = {ready_await, nullptr, nullptr, ready_send};

// ---- Recorder ------------------------------------------------------------------------------
struct RecorderObject {
  PyObject_HEAD PyObject* append;  // calls.append (bound method of the client's deque)
  PyObject* ready;                 // Ready(ok_response), shared by every answer
  unsigned long long count;
};

PyTypeObject RecorderType = {PyVarObject_HEAD_INIT(nullptr, 0)};

PyObject* recorder_new(PyTypeObject* type, PyObject*, PyObject*) {
  RecorderObject* self = reinterpret_cast<RecorderObject*>(type->tp_alloc(type, 0));
  if (!self) return nullptr;
  self->append = nullptr;
  self->ready = nullptr;
  self->count = 0;
  return reinterpret_cast<PyObject*>(self);
}

// Recorder(calls, ok_response): `calls` has an append method (a deque), `ok_response` is the
// object every fast-path request returns.
int recorder_init(RecorderObject* self, PyObject* args, PyObject*) {
  PyObject *calls, *ok;
  if (!PyArg_ParseTuple(args, "OO", &calls, &ok)) return -1;
  PyObject* app = PyObject_GetAttrString(calls, "append");
  if (!app) return -1;
  ReadyObject* r = PyObject_New(ReadyObject, &ReadyType);
  if (!r) {
    Py_DECREF(app);
    return -1;
  }
  r->value = Py_NewRef(ok);
  Py_XSETREF(self->append, app);
  Py_XSETREF(self->ready, reinterpret_cast<PyObject*>(r));
  return 0;
}

int recorder_traverse(RecorderObject* self, visitproc visit, void* arg) {
  Py_VISIT(self->append);
  return 0;
}

int recorder_clear(RecorderObject* self) {
  Py_CLEAR(self->append);
  Py_CLEAR(self->ready);
  return 0;
}

void recorder_dealloc(RecorderObject* self) {
  PyObject_GC_UnTrack(self);
  recorder_clear(self);
  Py_TYPE(self)->tp_free(reinterpret_cast<PyObject*>(self));
}

// Counts and logs one request; returns the full URL (new reference) or NULL.
PyObject* record_core(RecorderObject* self, PyObject* method, PyObject* url, PyObject* params) {
  if (!self->append) {
    PyErr_SetString(PyExc_RuntimeError, "Recorder not initialised");
    return nullptr;
  }
  PyObject* full = url_with_query(url, params);
  if (!full) return nullptr;
  PyObject* item = PyTuple_Pack(2, method, full);
  if (!item) {
    Py_DECREF(full);
    return nullptr;
  }
  PyObject* r = PyObject_CallOneArg(self->append, item);
  Py_DECREF(item);
  if (!r) {
    Py_DECREF(full);
    return nullptr;
  }
  Py_DECREF(r);
  self->count++;
  return full;
}

// record(method, url, params=None) -> full url (the Python request path)
PyObject* recorder_record(RecorderObject* self, PyObject* const* a, Py_ssize_t n) {
  if (n < 2 || n > 3) {
    PyErr_SetString(PyExc_TypeError, "record(method, url, params=None)");
    return nullptr;
  }
  return record_core(self, a[0], a[1], n == 3 ? a[2] : Py_None);
}

PyObject* recorder_get_count(RecorderObject* self, void*) { return PyLong_FromUnsignedLongLong(self->count); }

PyMethodDef recorder_methods[] = {
    {"record", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(recorder_record)), METH_FASTCALL,
     "record(method, url, params=None) -> full url: count the request and append (method, url) to the log"},
    {nullptr, nullptr, 0, nullptr}};

PyGetSetDef recorder_getset[] = {
    {"count", reinterpret_cast<getter>(recorder_get_count), nullptr, "requests recorded", nullptr},
    {nullptr, nullptr, nullptr, nullptr, nullptr}};

}  // namespace

bool is_recorder(PyObject* o) { return Py_TYPE(o) == &RecorderType; }

// The compiled handlers' fast path: record, then the shared completed awaitable.
PyObject* recorder_request(PyObject* rec, PyObject* method, PyObject* url, PyObject* params) {
  RecorderObject* self = reinterpret_cast<RecorderObject*>(rec);
  PyObject* full = record_core(self, method, url, params);
  if (!full) return nullptr;
  Py_DECREF(full);
  return Py_NewRef(self->ready);
}

int init_recorder_types(PyObject* m) {
  ReadyType.tp_name = "beholder_amd.ops._native.Ready";
  ReadyType.tp_basicsize = sizeof(ReadyObject);
  ReadyType.tp_flags = Py_TPFLAGS_DEFAULT;
  ReadyType.tp_doc = "An awaitable already completed with its value (the recorder's answer)";
  ReadyType.tp_dealloc = reinterpret_cast<destructor>(ready_dealloc);
  ReadyType.tp_as_async = &ready_async;
  ReadyType.tp_iter = PyObject_SelfIter;
  ReadyType.tp_iternext = ready_next;
  if (PyType_Ready(&ReadyType) < 0) return -1;

  RecorderType.tp_name = "beholder_amd.ops._native.Recorder";
  RecorderType.tp_basicsize = sizeof(RecorderObject);
  RecorderType.tp_flags = Py_TPFLAGS_DEFAULT | Py_TPFLAGS_HAVE_GC;
  RecorderType.tp_doc = "Recorder(calls, ok_response): native core of sinks.http.RecordingHttpClient";
  RecorderType.tp_new = recorder_new;
  RecorderType.tp_init = reinterpret_cast<initproc>(recorder_init);
  RecorderType.tp_dealloc = reinterpret_cast<destructor>(recorder_dealloc);
  RecorderType.tp_traverse = reinterpret_cast<traverseproc>(recorder_traverse);
  RecorderType.tp_clear = reinterpret_cast<inquiry>(recorder_clear);
  RecorderType.tp_methods = recorder_methods;
  RecorderType.tp_getset = recorder_getset;
  if (PyType_Ready(&RecorderType) < 0) return -1;
  Py_INCREF(&RecorderType);
  if (PyModule_AddObject(m, "Recorder", reinterpret_cast<PyObject*>(&RecorderType)) < 0) return -1;
  return 0;
}

}  // namespace beholder
