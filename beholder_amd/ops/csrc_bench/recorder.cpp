// The in-process sink stub of the headline bench and of the tests (sinks/http.py
// RecordingHttpClient): "Trello/Telegram/Emby stubbed in-process".
//
// A stub request pays what the production client's native path pays per request, minus the
// socket. Per request (index.js:53,83,99,112):
//
//   * the request bytes are built by the H1 client's own builder (_native._C_API
//     h1_request_text, py_h1call.cpp): request line with the encodeURIComponent query, Host,
//     Authorization, User-Agent (+ Content-Length: 0 for PUT/POST), copied into the stub's
//     send buffer as the NetConn copies them into its output buffer;
//   * the canned answer (`200 {}` as the bench's HTTP fake sends it) goes through an H1Parser,
//     started and fed through the same C entry points the NetConn's reply dispatch uses;
//   * the HttpResponse is built by the H1 client's own code (h1_response) with the request's
//     URL, and the request is counted and logged as (METHOD, url) in the client's bounded deque.
//
// What production does on top: the connection-pool bookkeeping, the reply future and the
// send(2) / epoll / recv(2) round trip; the answer here is an already-completed awaitable
// (Ready), so the handler never suspends on a sink.
//
// The compiled handlers call the stub through its sink hook (`hook`, a capsule: native_api.hpp)
// while the client has no fault rules and no simulated delay; otherwise the Python `request`
// coroutine records through `record`. mode "url" is the round-4 stub (URL + log only, one shared
// `200 {}` response with url ""), kept only as the old arm of the A/B (profiles/box_r5_stub_ab/).
#include <cstring>
#include <new>
#include <string>

#include "bench_common.hpp"

namespace beholder {
namespace bench {
namespace {

// ---- Ready: an awaitable that completes immediately with `value` -------------------------
struct ReadyObject {
  PyObject_HEAD PyObject* value;
};

PyTypeObject ReadyType = {PyVarObject_HEAD_INIT(nullptr, 0)};

PyObject* ready_new_c(PyObject* value) {
  ReadyObject* r = PyObject_New(ReadyObject, &ReadyType);
  if (!r) return nullptr;
  r->value = Py_NewRef(value);
  return reinterpret_cast<PyObject*>(r);
}

void ready_dealloc(ReadyObject* self) {
  Py_XDECREF(self->value);
  PyObject_Free(self);
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
enum : uint8_t { MODE_H1 = 0, MODE_URL = 1 };

struct RecorderObject {
  PyObject_HEAD PyObject* append;  // calls.append (bound method of the client's deque)
  PyObject* ok;                    // MODE_URL: the shared `200 {}` response
  PyObject* ready;                 // MODE_URL: Ready(ok), shared by every answer
  PyObject* parser;                // the H1Parser
  PyObject* start;                 // parser.start
  PyObject* feed;                  // parser.feed
  PyObject* response;              // bytes: the canned answer
  PyObject* origin_fn;             // callable(key) -> (host_header, auth) for a new origin
  PyObject* origins;               // dict: key -> (host_header, auth)
  PyObject* tail;                  // bytes: User-Agent tail (H1Client._tail)
  PyObject* tail_cl0;              // bytes: the same with Content-Length: 0 (H1Client._tail_cl0)
  std::string* out;                // the last request's bytes (the NetConn output buffer's stand-in)
  unsigned long long count, bytes_out, built;
  uint8_t mode;
};

PyTypeObject RecorderType = {PyVarObject_HEAD_INIT(nullptr, 0)};

PyObject *s_head, *s_HEAD, *s_append, *s_start, *s_feed;
PyObject* kw_head;  // ("head",)

PyObject* recorder_new(PyTypeObject* type, PyObject*, PyObject*) {
  RecorderObject* self = reinterpret_cast<RecorderObject*>(type->tp_alloc(type, 0));
  if (!self) return nullptr;
  self->out = new (std::nothrow) std::string();
  if (!self->out) {
    Py_DECREF(self);
    return PyErr_NoMemory();
  }
  return reinterpret_cast<PyObject*>(self);
}

// Recorder(calls, ok, parser, response, origin_fn, tail, tail_cl0, mode="h1")
int recorder_init(RecorderObject* self, PyObject* args, PyObject* kwds) {
  static const char* kwlist[] = {"calls", "ok", "parser", "response", "origin_fn", "tail", "tail_cl0", "mode",
                                 nullptr};
  PyObject *calls, *ok, *parser, *response, *origin_fn, *tail, *tail_cl0;
  const char* mode = "h1";
  if (!PyArg_ParseTupleAndKeywords(args, kwds, "OOOSOSS|s", const_cast<char**>(kwlist), &calls, &ok, &parser,
                                   &response, &origin_fn, &tail, &tail_cl0, &mode))
    return -1;
  uint8_t md;
  if (strcmp(mode, "h1") == 0) {
    md = MODE_H1;
  } else if (strcmp(mode, "url") == 0) {
    md = MODE_URL;
  } else {
    PyErr_SetString(PyExc_ValueError, "mode must be 'h1' or 'url'");
    return -1;
  }
  if (!PyCallable_Check(origin_fn)) {
    PyErr_SetString(PyExc_TypeError, "origin_fn must be callable");
    return -1;
  }
  PyObject* app = PyObject_GetAttr(calls, s_append);
  PyObject* st = app ? PyObject_GetAttr(parser, s_start) : nullptr;
  PyObject* fd = st ? PyObject_GetAttr(parser, s_feed) : nullptr;
  PyObject* ready = fd ? ready_new_c(ok) : nullptr;
  PyObject* origins = ready ? PyDict_New() : nullptr;
  if (!origins) {
    Py_XDECREF(app);
    Py_XDECREF(st);
    Py_XDECREF(fd);
    Py_XDECREF(ready);
    return -1;
  }
  Py_XSETREF(self->append, app);
  Py_XSETREF(self->ok, Py_NewRef(ok));
  Py_XSETREF(self->ready, ready);
  Py_XSETREF(self->parser, Py_NewRef(parser));
  Py_XSETREF(self->start, st);
  Py_XSETREF(self->feed, fd);
  Py_XSETREF(self->response, Py_NewRef(response));
  Py_XSETREF(self->origin_fn, Py_NewRef(origin_fn));
  Py_XSETREF(self->origins, origins);
  Py_XSETREF(self->tail, Py_NewRef(tail));
  Py_XSETREF(self->tail_cl0, Py_NewRef(tail_cl0));
  self->mode = md;
  return 0;
}

int recorder_traverse(RecorderObject* self, visitproc visit, void* arg) {
  Py_VISIT(self->append);
  Py_VISIT(self->ok);
  Py_VISIT(self->ready);
  Py_VISIT(self->parser);
  Py_VISIT(self->start);
  Py_VISIT(self->feed);
  Py_VISIT(self->origin_fn);
  Py_VISIT(self->origins);
  return 0;
}

int recorder_clear(RecorderObject* self) {
  Py_CLEAR(self->append);
  Py_CLEAR(self->ok);
  Py_CLEAR(self->ready);
  Py_CLEAR(self->parser);
  Py_CLEAR(self->start);
  Py_CLEAR(self->feed);
  Py_CLEAR(self->response);
  Py_CLEAR(self->origin_fn);
  Py_CLEAR(self->origins);
  Py_CLEAR(self->tail);
  Py_CLEAR(self->tail_cl0);
  return 0;
}

void recorder_dealloc(RecorderObject* self) {
  PyObject_GC_UnTrack(self);
  recorder_clear(self);
  delete self->out;
  Py_TYPE(self)->tp_free(reinterpret_cast<PyObject*>(self));
}

// (host_header, auth) of the origin `url[:k]`, from the cache or origin_fn. Borrowed into *host
// and *auth (the tuple stays in self->origins). 0, or -1 with an error.
int origin_of(RecorderObject* self, PyObject* url, Py_ssize_t k, PyObject** host, PyObject** auth) {
  PyObject* key = PyUnicode_Substring(url, 0, k);
  if (!key) return -1;
  PyObject* o = PyDict_GetItemWithError(self->origins, key);
  if (!o) {
    if (PyErr_Occurred()) {
      Py_DECREF(key);
      return -1;
    }
    o = PyObject_CallOneArg(self->origin_fn, key);
    if (!o || !PyTuple_CheckExact(o) || PyTuple_GET_SIZE(o) != 2) {
      if (o && !PyErr_Occurred()) PyErr_SetString(PyExc_TypeError, "origin_fn must return (host_header, auth)");
      Py_XDECREF(o);
      Py_DECREF(key);
      return -1;
    }
    int rc = PyDict_SetItem(self->origins, key, o);
    Py_DECREF(o);  // held by the dict
    if (rc < 0) {
      Py_DECREF(key);
      return -1;
    }
  }
  Py_DECREF(key);
  *host = PyTuple_GET_ITEM(o, 0);
  *auth = PyTuple_GET_ITEM(o, 1);
  return 0;
}

// Counts and logs one request; builds its bytes (MODE_H1). Returns the URL it went to (new
// reference) or NULL. The URL: the H1 client's (url + its query) when it sends the request
// natively, else restler's url + "?" + query (the Python client's with_query).
PyObject* record_core(RecorderObject* self, PyObject* method, PyObject* url, PyObject* params) {
  if (!self->append) {
    PyErr_SetString(PyExc_RuntimeError, "Recorder not initialised");
    return nullptr;
  }
  PyObject* full = nullptr;
  if (self->mode == MODE_H1) {
    Py_ssize_t k;
    if (g_api->h1_origin_key(method, url, params, &k) == 1) {
      PyObject *host, *auth;
      if (origin_of(self, url, k, &host, &auth) < 0) return nullptr;
      int rc = g_api->h1_request_text(method, url, params, host, auth, self->tail, self->tail_cl0, self->out, &full,
                                      &k);
      if (rc < 0) return nullptr;
      if (rc == 1) {
        self->built++;
        self->bytes_out += self->out->size();
        // params whose every value is None: restler still appends "?" (the URL the oracle pins)
        if (full == url && params != Py_None && PyDict_GET_SIZE(params)) Py_CLEAR(full);
      }
    }
  }
  if (!full) full = g_api->url_with_query(url, params);
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

// The answer to a request of `method` to `full`: the canned bytes through the parser, then the
// H1 client's HttpResponse. New reference or NULL.
PyObject* answer(RecorderObject* self, PyObject* method, PyObject* full) {
  int head = PyObject_RichCompareBool(method, s_HEAD, Py_EQ);
  if (head < 0) return nullptr;
  PyObject* parsed;
  if (self->parser && g_api->is_h1_parser(self->parser)) {  // as the NetConn drives its parser
    if (g_api->h1_parser_start(self->parser, head != 0) < 0) return nullptr;
    parsed = g_api->h1_parser_feed(self->parser, PyBytes_AS_STRING(self->response),
                                   size_t(PyBytes_GET_SIZE(self->response)));
  } else {
    PyObject* args[1] = {head ? Py_True : Py_False};
    PyObject* r = PyObject_Vectorcall(self->start, args, 0, kw_head);  // parser.start(head=head)
    if (!r) return nullptr;
    Py_DECREF(r);
    parsed = PyObject_CallOneArg(self->feed, self->response);
  }
  if (!parsed) return nullptr;
  if (parsed == Py_None) {
    Py_DECREF(parsed);
    PyErr_SetString(PyExc_RuntimeError, "Recorder: the canned response is incomplete");
    return nullptr;
  }
  PyObject* resp = g_api->h1_response(parsed, full);
  Py_DECREF(parsed);
  return resp;
}

// The sink hook (native_api.hpp): request(method, url, params) -> completed awaitable.
PyObject* hook_request(PyObject* o, PyObject* method, PyObject* url, PyObject* params) {
  RecorderObject* self = reinterpret_cast<RecorderObject*>(o);
  PyObject* full = record_core(self, method, url, params);
  if (!full) return nullptr;
  if (self->mode == MODE_URL) {
    Py_DECREF(full);
    return Py_NewRef(self->ready);
  }
  PyObject* resp = answer(self, method, full);
  Py_DECREF(full);
  if (!resp) return nullptr;
  PyObject* rdy = ready_new_c(resp);
  Py_DECREF(resp);
  return rdy;
}

const SinkHook kHook = {kSinkHookAbi, hook_request};

void hook_capsule_free(PyObject* cap) { Py_XDECREF(static_cast<PyObject*>(PyCapsule_GetContext(cap))); }

// record(method, url, params=None) -> the URL (the Python request path, which answers itself)
PyObject* recorder_record(RecorderObject* self, PyObject* const* a, Py_ssize_t n) {
  if (n < 2 || n > 3) {
    PyErr_SetString(PyExc_TypeError, "record(method, url, params=None)");
    return nullptr;
  }
  return record_core(self, a[0], a[1], n == 3 ? a[2] : Py_None);
}

// request(method, url, params=None) -> awaitable: what the hook does, callable from Python
PyObject* recorder_request(RecorderObject* self, PyObject* const* a, Py_ssize_t n) {
  if (n < 2 || n > 3) {
    PyErr_SetString(PyExc_TypeError, "request(method, url, params=None)");
    return nullptr;
  }
  return hook_request(reinterpret_cast<PyObject*>(self), a[0], a[1], n == 3 ? a[2] : Py_None);
}

// hook -> a new sink-hook capsule bound to this recorder (for the client's `native_record`)
PyObject* recorder_get_hook(RecorderObject* self, void*) {
  PyObject* cap = PyCapsule_New(const_cast<SinkHook*>(&kHook), kSinkHookName, hook_capsule_free);
  if (!cap) return nullptr;
  if (PyCapsule_SetContext(cap, Py_NewRef(reinterpret_cast<PyObject*>(self))) < 0) {
    Py_DECREF(self);
    Py_DECREF(cap);
    return nullptr;
  }
  return cap;
}

PyObject* recorder_get_count(RecorderObject* self, void*) { return PyLong_FromUnsignedLongLong(self->count); }
PyObject* recorder_get_built(RecorderObject* self, void*) { return PyLong_FromUnsignedLongLong(self->built); }
PyObject* recorder_get_bytes_out(RecorderObject* self, void*) { return PyLong_FromUnsignedLongLong(self->bytes_out); }
PyObject* recorder_get_last_request(RecorderObject* self, void*) {
  return PyBytes_FromStringAndSize(self->out->data(), Py_ssize_t(self->out->size()));
}
PyObject* recorder_get_mode(RecorderObject* self, void*) {
  return PyUnicode_FromString(self->mode == MODE_H1 ? "h1" : "url");
}

PyMethodDef recorder_methods[] = {
    {"record", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(recorder_record)), METH_FASTCALL,
     "record(method, url, params=None) -> url: count, build the request bytes, log (method, url)"},
    {"request", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(recorder_request)), METH_FASTCALL,
     "request(method, url, params=None) -> awaitable HttpResponse (the sink hook's work)"},
    {nullptr, nullptr, 0, nullptr}};

PyGetSetDef recorder_getset[] = {
    {"count", reinterpret_cast<getter>(recorder_get_count), nullptr, "requests recorded", nullptr},
    {"built", reinterpret_cast<getter>(recorder_get_built), nullptr,
     "requests whose bytes the H1 builder produced (the native path's shape)", nullptr},
    {"bytes_out", reinterpret_cast<getter>(recorder_get_bytes_out), nullptr, "request bytes built in total", nullptr},
    {"last_request", reinterpret_cast<getter>(recorder_get_last_request), nullptr, "the last request's bytes",
     nullptr},
    {"mode", reinterpret_cast<getter>(recorder_get_mode), nullptr, "'h1' (default) or 'url' (round-4 stub)", nullptr},
    {"hook", reinterpret_cast<getter>(recorder_get_hook), nullptr,
     "a sink-hook capsule for the compiled handlers (native_api.hpp)", nullptr},
    {nullptr, nullptr, nullptr, nullptr, nullptr}};

}  // namespace

int init_recorder(PyObject* m) {
  struct {
    PyObject** slot;
    const char* text;
  } strs[] = {{&s_head, "head"}, {&s_HEAD, "HEAD"}, {&s_append, "append"}, {&s_start, "start"}, {&s_feed, "feed"}};
  for (auto& s : strs)
    if (!(*s.slot = PyUnicode_InternFromString(s.text))) return -1;
  kw_head = PyTuple_Pack(1, s_head);
  if (!kw_head) return -1;

  ReadyType.tp_name = "beholder_amd.ops._native_bench.Ready";
  ReadyType.tp_basicsize = sizeof(ReadyObject);
  ReadyType.tp_flags = Py_TPFLAGS_DEFAULT;
  ReadyType.tp_doc = "An awaitable already completed with its value (the recorder's answer)";
  ReadyType.tp_dealloc = reinterpret_cast<destructor>(ready_dealloc);
  ReadyType.tp_as_async = &ready_async;
  ReadyType.tp_iter = PyObject_SelfIter;
  ReadyType.tp_iternext = ready_next;
  if (PyType_Ready(&ReadyType) < 0) return -1;

  RecorderType.tp_name = "beholder_amd.ops._native_bench.Recorder";
  RecorderType.tp_basicsize = sizeof(RecorderObject);
  RecorderType.tp_flags = Py_TPFLAGS_DEFAULT | Py_TPFLAGS_HAVE_GC;
  RecorderType.tp_doc =
      "Recorder(calls, ok, parser, response, origin_fn, tail, tail_cl0, mode='h1'): native core of "
      "sinks.http.RecordingHttpClient";
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

}  // namespace bench
}  // namespace beholder
