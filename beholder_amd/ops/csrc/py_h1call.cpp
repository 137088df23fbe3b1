// H1 fast path: the common case of sinks/h1.py `H1Client.request` done in C.
//
// The production path issues one sink request per Trello-created progress event and up to
// three per status event (index.js:53,83,99,112). In Python each costs a coroutine, the URL
// split / route lookup, the request text, the idle-connection pop, the reply future, the
// busy-set bookkeeping, the release to the pool and the HttpResponse: about 4 us of CPU on
// the box, the largest Python cost left in `tcp_e2e` after the native NetConn.
//
//   call = h1_fast(client, method, url, params, timeout)   # None: not a stock H1Client
//   resp = await call
//
// Like a coroutine, an H1Call does nothing until it is first awaited. Then it handles exactly
// the shape the sinks produce on a warm pool: a stock H1Client, an
// ASCII URL whose origin is already known, a printable path (no fragment), params None or a
// dict (encodeURIComponent query, the `request` library's qs.stringify), and a live idle
// keep-alive connection on a native NetConn (utils/netconn.py). With no idle connection the
// request joins the origin's queue (H1Client._enqueue: _acquire's accounting, background
// connects and deadline) with an IOFuture waiter and is sent natively on the connection it is
// handed; a freed slot, a closed or non-native connection, the deadline or a failed connect
// continue in H1Client._after_queue. (The first burst after start queues ~250 requests while
// the pools fill, with the loop CPU-bound: the Python request loop cost ~10 us each.)
// Anything else is declined before any state is touched, and the H1Call delegates the whole
// request to H1Client._request (yield from).
//
// The returned H1Call is an awaitable iterator (send/throw/close). It yields the reply
// IOFuture; a handler driven by the native Driver is resumed by the NetConn's reply callback.
// A plain reply (not a redirect of a GET/HEAD) completes in C: the connection goes back to
// the idle pool (or is dropped through H1Client._release), an HttpResponse is built. A failed
// reply (reset, timeout, malformed) or a redirect is handed to H1Client._resume(m, full,
// deadline, conn, fut, reused), which runs the Python request loop from that await on
// (transparent retry on a fresh connection, redirects, error mapping), and the H1Call
// delegates to it (yield from). The pool invariants of sinks/h1.py hold on every path:
// counts, `uses`, `deadline`, `what`, the busy set and the deadline sweeper are updated as
// the Python fast path does.
#include <time.h>

#include <string>

#include "py_common.hpp"
#include "native_api.hpp"
#include "gil_clock.hpp"

#include <structmember.h>

namespace beholder {

PyObject* iofuture_new(PyObject* loop);
int iofuture_peek(PyObject* f, PyObject** result);
PyObject* iofuture_yield(PyObject* f);
bool is_netconn(PyObject* o);
bool netconn_open(PyObject* o);
PyObject* netconn_loop(PyObject* o);
int netconn_h1_request(PyObject* o, const char* data, size_t n, PyObject* waiter, bool head);
bool text_query_pair_append(std::string& out, PyObject* k, PyObject* v, bool* first, bool rfc3986);

namespace {

// Slot offsets of a __slots__ class, from its member descriptors (exact type only).
struct Slots {
  PyTypeObject* type = nullptr;
  Py_ssize_t off[8] = {0};

  bool resolve(PyObject* cls, const char* const* names, int n) {
    if (!PyType_Check(cls)) {
      PyErr_SetString(PyExc_TypeError, "h1_setup: expected a class");
      return false;
    }
    for (int i = 0; i < n; ++i) {
      PyObject* d = PyObject_GetAttrString(cls, names[i]);
      if (!d) return false;
      bool ok = Py_TYPE(d) == &PyMemberDescr_Type &&
                reinterpret_cast<PyMemberDescrObject*>(d)->d_member->type == T_OBJECT_EX;
      if (ok) off[i] = reinterpret_cast<PyMemberDescrObject*>(d)->d_member->offset;
      Py_DECREF(d);
      if (!ok) {
        PyErr_Format(PyExc_TypeError, "h1_setup: %s.%s is not a __slots__ member",
                     reinterpret_cast<PyTypeObject*>(cls)->tp_name, names[i]);
        return false;
      }
    }
    Py_INCREF(cls);
    Py_XSETREF(type, reinterpret_cast<PyTypeObject*>(cls));
    return true;
  }
  // borrowed; NULL when the slot is unset
  PyObject* get(PyObject* o, int i) const { return *reinterpret_cast<PyObject**>(reinterpret_cast<char*>(o) + off[i]); }
  // steals v
  void set(PyObject* o, int i, PyObject* v) const {
    PyObject** p = reinterpret_cast<PyObject**>(reinterpret_cast<char*>(o) + off[i]);
    PyObject* old = *p;
    *p = v;
    Py_XDECREF(old);
  }
};

// sinks/h1.py _Conn / _Origin and sinks/http.py HttpResponse slot indices
enum { C_ORIGIN, C_PARSER, C_CLOSED, C_LAST_USED, C_USES, C_DEADLINE, C_WHAT, C_NET, C_N };
const char* const kConnSlots[C_N] = {"origin", "parser", "closed", "last_used", "uses", "deadline", "what", "net"};
enum { O_HOST_HEADER, O_AUTH, O_IDLE, O_WAITERS, O_N };
const char* const kOriginSlots[O_N] = {"host_header", "auth", "idle", "waiters"};
enum { R_STATUS, R_BODY, R_HEADERS, R_RAW, R_URL, R_N };
const char* const kRespSlots[R_N] = {"status", "body", "_headers", "_raw", "url"};

struct State {
  Slots conn, origin, resp;
  PyTypeObject* client_type = nullptr;
  PyObject* base_time = nullptr;  // asyncio.BaseEventLoop.time (time.monotonic())
  PyObject* get_running_loop = nullptr;  // asyncio.get_running_loop
  bool ready = false;
} g;

PyObject *s_closed_attr, *s_origins, *s_counts, *s_keepalive_s, *s_timeout_s, *s_busy, *s_sweeper, *s_tail,
    *s_tail_cl0, *s_requests, *s_reused, *s_drop, *s_release, *s_arm, *s_resume, *s_time, *s_pop, *s_append,
    *s_buffered, *s_throw, *s_close, *s_request_py, *s_cancel, *s_enqueue, *s_after_queue, *s_exception_name;

double mono_s() { return double(gil_mono_ns()) * 1e-9; }  // time.monotonic()'s clock (gil_clock.hpp)

bool is_body_method(const char* m, Py_ssize_t n) {
  auto eq = [&](const char* s) { return Py_ssize_t(strlen(s)) == n && memcmp(m, s, size_t(n)) == 0; };
  return eq("POST") || eq("PUT") || eq("PATCH") || eq("DELETE");
}

bool is_get_or_head(const char* m, Py_ssize_t n) {
  return (n == 3 && memcmp(m, "GET", 3) == 0) || (n == 4 && memcmp(m, "HEAD", 4) == 0);
}

// owns one reference until destroyed (p = nullptr hands it on)
struct Own {
  PyObject* p;
  ~Own() { Py_XDECREF(p); }
};

// dict[key] += 1 (int counters of H1Client.counts)
int bump(PyObject* d, PyObject* key) {
  PyObject* v = PyDict_GetItemWithError(d, key);
  if (!v) {
    if (!PyErr_Occurred()) PyErr_SetObject(PyExc_KeyError, key);
    return -1;
  }
  PyObject* one = PyLong_FromLong(1);
  PyObject* n = one ? PyNumber_Add(v, one) : nullptr;
  Py_XDECREF(one);
  if (!n) return -1;
  int rc = PyDict_SetItem(d, key, n);
  Py_DECREF(n);
  return rc;
}

// ---- H1Call ---------------------------------------------------------------------------------
// ST_INIT: created, nothing done yet (like a coroutine before its first send: the request is
// prepared and sent when the call is first awaited, so ordering under gather() and an
// H1Call that is never awaited behave as H1Client._request would)
// ST_QUEUED: no idle connection at the first await; the call waits in the origin's queue
// (H1Client._enqueue) for one, then sends natively as from the idle pool
enum : uint8_t { ST_WAIT = 0, ST_DELEGATE = 1, ST_DONE = 2, ST_INIT = 3, ST_QUEUED = 4 };

struct H1CallObject {
  PyObject_HEAD PyObject* client;
  PyObject* conn;
  PyObject* fut;
  PyObject* method;  // str as passed, then upper case once sent
  PyObject* full;    // str: the URL as passed, then with its query (HttpResponse.url, error text)
  PyObject* deadline;
  PyObject* params;   // ST_INIT: the call's params (or NULL)
  PyObject* timeout;  // ST_INIT: the call's timeout (or NULL)
  PyObject* sub;  // the Python continuation (H1Client._resume / _request) once delegated
  PyObject* timer;  // ST_QUEUED: the queue deadline's TimerHandle
  PyObject* req;    // ST_QUEUED: the request bytes, sent once a connection is handed over
  uint8_t state;
  uint8_t reused;  // the connection had served a request before (h1.py `reused`)
  uint8_t path;    // 0 not started, 1 sent natively, 2 delegated to H1Client._request
  uint8_t head;    // ST_QUEUED: a HEAD request
  uint8_t front;   // a continuation of an event's earlier request: waits at the front of the queue
};

PyTypeObject H1CallType = {PyVarObject_HEAD_INIT(nullptr, 0)};

int call_traverse(H1CallObject* s, visitproc visit, void* arg) {
  Py_VISIT(s->client);
  Py_VISIT(s->conn);
  Py_VISIT(s->fut);
  Py_VISIT(s->method);
  Py_VISIT(s->full);
  Py_VISIT(s->deadline);
  Py_VISIT(s->params);
  Py_VISIT(s->timeout);
  Py_VISIT(s->sub);
  Py_VISIT(s->timer);
  Py_VISIT(s->req);
  return 0;
}

int call_clear(H1CallObject* s) {
  Py_CLEAR(s->client);
  Py_CLEAR(s->conn);
  Py_CLEAR(s->fut);
  Py_CLEAR(s->method);
  Py_CLEAR(s->full);
  Py_CLEAR(s->deadline);
  Py_CLEAR(s->params);
  Py_CLEAR(s->timeout);
  Py_CLEAR(s->sub);
  Py_CLEAR(s->timer);
  Py_CLEAR(s->req);
  return 0;
}

// The stock H1Client's attributes the native path reads per request (h1_start, send_on), from its
// instance dict: looked up again only when that dict changed (DictView; `_sweeper` is rebound each
// sweep tick, nothing else after setup).
enum { CV_CLOSED, CV_ORIGINS, CV_COUNTS, CV_KEEPALIVE, CV_TIMEOUT, CV_BUSY, CV_TAIL, CV_TAIL_CL0, CV_SWEEPER, CV_N };
PyObject* const* const kClientKeys[CV_N] = {&s_closed_attr, &s_origins, &s_counts, &s_keepalive_s, &s_timeout_s,
                                            &s_busy,        &s_tail,    &s_tail_cl0, &s_sweeper};
DictView<CV_N> g_client_view;

// The client's instance dict with g_client_view current for it; NULL (no error) without one,
// NULL with an error if a lookup raised.
PyObject* client_view(PyObject* client) {
  PyObject** dp = _PyObject_GetDictPtr(client);
  PyObject* d = dp ? *dp : nullptr;
  if (!d || !PyDict_CheckExact(d)) return nullptr;
  return g_client_view.refresh(d, kClientKeys) ? d : nullptr;
}

PyObject* client_attr(PyObject* client, PyObject* name) {  // borrowed, from the instance dict
  PyObject** dp = _PyObject_GetDictPtr(client);
  PyObject* v = dp && *dp ? PyDict_GetItemWithError(*dp, name) : nullptr;
  if (!v && !PyErr_Occurred()) PyErr_SetObject(PyExc_AttributeError, name);
  return v;
}

// `busy.discard(c); self._release(c, False)`: the request ended without a usable reply
// (cancelled, closed, abandoned). Errors are reported, not raised (cleanup path).
void abandon(H1CallObject* s) {
  PyObject *et, *ev, *tb;
  PyErr_Fetch(&et, &ev, &tb);
  if (s->client && s->conn) {
    PyObject* busy = client_attr(s->client, s_busy);
    if (!busy || PySet_Discard(busy, s->conn) < 0) PyErr_WriteUnraisable(s->client);
    PyObject* r = PyObject_CallMethodObjArgs(s->client, s_release, s->conn, Py_False, nullptr);
    if (!r)
      PyErr_WriteUnraisable(s->client);
    else
      Py_DECREF(r);
  }
  PyErr_Restore(et, ev, tb);
}

// ST_QUEUED, leaving without sending: the deadline timer is cancelled; a connection handed over
// meanwhile goes back to the pool (h1.py _acquire's CancelledError path); a waiter still in the
// queue is cancelled, so _release / _wake pass over it. Errors are reported, not raised.
void leave_queue(H1CallObject* s) {
  PyObject *et, *ev, *tb;
  PyErr_Fetch(&et, &ev, &tb);
  if (s->timer) {
    PyObject* r = PyObject_CallMethodNoArgs(s->timer, s_cancel);
    if (!r)
      PyErr_WriteUnraisable(s->timer);
    else
      Py_DECREF(r);
    Py_CLEAR(s->timer);
  }
  if (s->fut) {
    PyObject* res = nullptr;
    int st = iofuture_peek(s->fut, &res);
    if (st == 0) {
      PyObject* r = PyObject_CallMethodNoArgs(s->fut, s_cancel);
      if (!r)
        PyErr_WriteUnraisable(s->fut);
      else
        Py_DECREF(r);
    } else if (st == 1 && res && Py_TYPE(res) == g.conn.type && s->client) {
      PyObject* r = PyObject_CallMethodObjArgs(s->client, s_release, res, Py_True, nullptr);
      if (!r)
        PyErr_WriteUnraisable(s->client);
      else
        Py_DECREF(r);
    }
  }
  PyErr_Restore(et, ev, tb);
}

void call_finalize(H1CallObject* s) {
  if (s->state == ST_QUEUED) {
    s->state = ST_DONE;
    leave_queue(s);
  } else if (s->state == ST_WAIT) {  // never awaited to the end: like a closed coroutine
    s->state = ST_DONE;
    abandon(s);
  } else if (s->state == ST_DELEGATE && s->sub) {
    s->state = ST_DONE;
    PyObject *et, *ev, *tb;
    PyErr_Fetch(&et, &ev, &tb);
    PyObject* r = PyObject_CallMethodNoArgs(s->sub, s_close);
    if (!r)
      PyErr_WriteUnraisable(s->sub);
    else
      Py_DECREF(r);
    PyErr_Restore(et, ev, tb);
  }
}

void call_dealloc(H1CallObject* s) {
  if (PyObject_CallFinalizerFromDealloc(reinterpret_cast<PyObject*>(s)) < 0) return;  // resurrected
  PyObject_GC_UnTrack(s);
  call_clear(s);
  Py_TYPE(s)->tp_free(reinterpret_cast<PyObject*>(s));
}

// HttpResponse(status, body, None, full, raw) without its __init__ (slots set directly). New
// reference, NULL on error.
PyObject* make_response(PyObject* status, PyObject* body, PyObject* raw, PyObject* full) {
  PyTypeObject* rt = g.resp.type;
  if (!rt) {
    PyErr_SetString(PyExc_RuntimeError, "h1_setup has not run (import beholder_amd.sinks.h1)");
    return nullptr;
  }
  PyObject* resp = rt->tp_alloc(rt, 0);
  if (!resp) return nullptr;
  PyObject* vals[R_N] = {status, body, Py_None, raw, full};
  for (int i = 0; i < R_N; ++i) {
    Py_INCREF(vals[i]);
    g.resp.set(resp, i, vals[i]);
  }
  return resp;
}

// The reply `res` arrived. 1 = finished here (*out = HttpResponse), 0 = the Python loop must
// continue (a redirect to follow), -1 = error.
int finish_fast(H1CallObject* s, PyObject* res, PyObject** out) {
  if (!PyTuple_CheckExact(res) || PyTuple_GET_SIZE(res) != 5) return 0;
  PyObject* status = PyTuple_GET_ITEM(res, 0);
  if (!PyLong_CheckExact(status)) return 0;
  long st = PyLong_AsLong(status);
  if (st == -1 && PyErr_Occurred()) return -1;
  if (st == 301 || st == 302 || st == 303 || st == 307 || st == 308) {
    Py_ssize_t mn;
    const char* m = PyUnicode_AsUTF8AndSize(s->method, &mn);
    if (!m) return -1;
    if (is_get_or_head(m, mn)) return 0;
  }
  PyObject* client = s->client;
  PyObject* conn = s->conn;
  PyObject* busy = client_attr(client, s_busy);
  if (!busy || PySet_Discard(busy, conn) < 0) return -1;
  // from here on the connection is out of `busy`: a failure must still hand it back (closed),
  // or its origin would count it open forever
  auto fail = [s]() {
    abandon(s);
    return -1;
  };
  // keep = keep-alive and c.parser.buffered == 0
  int keep = PyObject_IsTrue(PyTuple_GET_ITEM(res, 4));
  if (keep < 0) return fail();
  if (keep) {
    PyObject* parser = g.conn.get(conn, C_PARSER);
    PyObject* b = parser ? PyObject_GetAttr(parser, s_buffered) : nullptr;
    if (!b) return fail();
    int zero = PyLong_Check(b) && PyLong_AsSsize_t(b) == 0;
    Py_DECREF(b);
    keep = zero;
  }
  PyObject* cclosed = client_attr(client, s_closed_attr);
  if (!cclosed) return fail();
  PyObject* o = g.conn.get(conn, C_ORIGIN);
  PyObject* waiters = o && Py_TYPE(o) == g.origin.type ? g.origin.get(o, O_WAITERS) : nullptr;
  PyObject* idle = waiters ? g.origin.get(o, O_IDLE) : nullptr;
  Py_ssize_t nw = waiters ? PyObject_Size(waiters) : -1;
  if (nw < 0 && PyErr_Occurred()) return fail();
  if (keep && idle && nw == 0 && g.conn.get(conn, C_CLOSED) == Py_False && cclosed == Py_False) {
    // H1Client._release(c, True) with no waiter: back to the idle pool
    PyObject* t = PyFloat_FromDouble(mono_s());
    if (!t) return fail();
    g.conn.set(conn, C_LAST_USED, t);
    PyObject* r = PyObject_CallMethodOneArg(idle, s_append, conn);
    if (!r) return fail();
    Py_DECREF(r);
  } else {
    PyObject* r = PyObject_CallMethodObjArgs(client, s_release, conn, keep ? Py_True : Py_False, nullptr);
    if (!r) return -1;
    Py_DECREF(r);
  }
  PyObject* resp = make_response(status, PyTuple_GET_ITEM(res, 3), PyTuple_GET_ITEM(res, 2), s->full);
  if (!resp) return -1;
  *out = resp;
  return 1;
}

PySendResult delegate_send(H1CallObject* s, PyObject* arg, PyObject** out) {
  PySendResult r = PyIter_Send(s->sub, arg, out);
  if (r != PYGEN_NEXT) {
    s->state = ST_DONE;
    Py_CLEAR(s->sub);
  }
  return r;
}

// The Python request loop takes over at the await: s->sub = client._resume(m, full, deadline,
// conn, fut, reused, thrown), where `thrown` (or None) is an exception thrown in at the await.
int start_delegate(H1CallObject* s, PyObject* thrown) {
  PyObject* args[8] = {s->client,  s->method, s->full, s->deadline, s->conn, s->fut, s->reused ? Py_True : Py_False,
                       thrown ? thrown : Py_None};
  PyObject* sub = PyObject_VectorcallMethod(s_resume, args, 8, nullptr);
  if (!sub) {
    s->state = ST_DONE;
    return -1;
  }
  PyObject* it = sub;
  if (!PyCoro_CheckExact(sub)) {
    unaryfunc getter = Py_TYPE(sub)->tp_as_async ? Py_TYPE(sub)->tp_as_async->am_await : nullptr;
    it = getter ? getter(sub) : nullptr;
    Py_DECREF(sub);
    if (!it) {
      if (!PyErr_Occurred()) PyErr_SetString(PyExc_TypeError, "H1Client._resume must return an awaitable");
      s->state = ST_DONE;
      return -1;
    }
  }
  s->sub = it;
  s->state = ST_DELEGATE;
  return 0;
}

int h1_start(H1CallObject* s);
int queue_resume(H1CallObject* s);

// The fast path declined at the first await: the whole request is H1Client._request's.
int start_python(H1CallObject* s) {
  PyObject* args[5] = {s->client, s->method, s->full, s->params ? s->params : Py_None,
                       s->timeout ? s->timeout : Py_None};
  PyObject* sub = PyObject_VectorcallMethod(s_request_py, args, 5, nullptr);
  if (!sub) {
    s->state = ST_DONE;
    return -1;
  }
  if (!PyCoro_CheckExact(sub)) {
    Py_DECREF(sub);
    PyErr_SetString(PyExc_TypeError, "H1Client._request must be a coroutine function");
    s->state = ST_DONE;
    return -1;
  }
  s->sub = sub;
  s->state = ST_DELEGATE;
  return 0;
}

PySendResult call_am_send(H1CallObject* s, PyObject* arg, PyObject** out) {
  if (s->state == ST_DELEGATE) return delegate_send(s, arg, out);
  if (s->state == ST_DONE) {
    PyErr_SetString(PyExc_RuntimeError, "cannot reuse already awaited H1 request");
    *out = nullptr;
    return PYGEN_ERROR;
  }
  if (s->state == ST_INIT) {
    int k;
    try {
      k = h1_start(s);
    } catch (const std::bad_alloc&) {
      PyErr_NoMemory();
      k = -1;
    }
    if (k < 0) {
      s->state = ST_DONE;
      *out = nullptr;
      return PYGEN_ERROR;
    }
    s->path = uint8_t(k == 0 ? 2 : 1);
    if (k == 0) {
      if (start_python(s) < 0) {
        *out = nullptr;
        return PYGEN_ERROR;
      }
      return delegate_send(s, Py_None, out);
    }
  }
  if (s->state == ST_QUEUED) {
    PyObject* w = nullptr;
    if (iofuture_peek(s->fut, &w) == 0) {
      *out = iofuture_yield(s->fut);
      return *out ? PYGEN_NEXT : PYGEN_ERROR;
    }
    int rc;
    try {
      rc = queue_resume(s);
    } catch (const std::bad_alloc&) {
      PyErr_NoMemory();
      rc = -1;
    }
    if (rc < 0) {
      if (s->state == ST_QUEUED) leave_queue(s);
      s->state = ST_DONE;
      *out = nullptr;
      return PYGEN_ERROR;
    }
    if (s->state == ST_DELEGATE) {
      s->path = 2;
      return delegate_send(s, Py_None, out);
    }
  }
  PyObject* res = nullptr;
  int st = iofuture_peek(s->fut, &res);
  if (st == 0) {
    *out = iofuture_yield(s->fut);
    return *out ? PYGEN_NEXT : PYGEN_ERROR;
  }
  if (st == 1) {
    Py_INCREF(res);
    int k = finish_fast(s, res, out);
    Py_DECREF(res);
    if (k != 0) {
      s->state = ST_DONE;
      if (k < 0) {
        *out = nullptr;
        return PYGEN_ERROR;
      }
      return PYGEN_RETURN;
    }
  }
  // an error, a cancelled future or a redirect: the Python request loop takes over at the await
  if (start_delegate(s, nullptr) < 0) {
    *out = nullptr;
    return PYGEN_ERROR;
  }
  return delegate_send(s, Py_None, out);
}

// iterator protocol on top of am_send: a return value becomes StopIteration(value)
PyObject* call_result(PySendResult r, PyObject* out) {
  if (r == PYGEN_NEXT) return out;
  if (r == PYGEN_ERROR) return nullptr;
  if (out == Py_None) {
    Py_DECREF(out);
    PyErr_SetNone(PyExc_StopIteration);
    return nullptr;
  }
  PyObject* e = PyObject_CallOneArg(PyExc_StopIteration, out);
  Py_DECREF(out);
  if (!e) return nullptr;
  PyErr_SetObject(PyExc_StopIteration, e);
  Py_DECREF(e);
  return nullptr;
}

PyObject* call_iternext(H1CallObject* s) {
  PyObject* out = nullptr;
  PySendResult r = call_am_send(s, Py_None, &out);
  return call_result(r, out);
}

PyObject* call_send(H1CallObject* s, PyObject* v) {
  PyObject* out = nullptr;
  PySendResult r = call_am_send(s, v, &out);
  return call_result(r, out);
}

PyObject* call_throw(H1CallObject* s, PyObject* args) {
  PyObject *typ, *val = nullptr, *tb = nullptr;
  if (!PyArg_UnpackTuple(args, "throw", 1, 3, &typ, &val, &tb)) return nullptr;
  if (s->state == ST_DELEGATE) {
    PyObject* r = PyObject_CallMethodObjArgs(s->sub, s_throw, typ, val, tb, nullptr);
    if (!r) {  // finished (StopIteration) or raised
      s->state = ST_DONE;
      Py_CLEAR(s->sub);
    }
    return r;
  }
  PyObject* exc = nullptr;  // the thrown exception as an instance
  if (PyExceptionInstance_Check(typ)) {
    Py_INCREF(typ);
    exc = typ;
  } else if (PyExceptionClass_Check(typ)) {
    exc = val && PyObject_TypeCheck(val, reinterpret_cast<PyTypeObject*>(typ)) ? (Py_INCREF(val), val)
          : val && val != Py_None ? PyObject_CallOneArg(typ, val)
                                  : PyObject_CallNoArgs(typ);
    if (!exc) return nullptr;
  } else {
    PyErr_SetString(PyExc_TypeError, "exceptions must be classes or instances deriving from BaseException");
    return nullptr;
  }
  if (s->state == ST_INIT) s->state = ST_DONE;  // like throw() into an unstarted coroutine
  if (s->state == ST_QUEUED) {
    // a Task throws the waiter's own exception in (its deadline, a failed connect, the client
    // closing): the request continues as when resumed. Anything else (a cancel, a wrapper's
    // timeout) leaves the queue and propagates, as from _acquire's await.
    bool own = false;
    PyObject* res = nullptr;
    if (iofuture_peek(s->fut, &res) == 2) {
      PyObject* e = PyObject_CallMethodNoArgs(s->fut, s_exception_name);
      if (!e) PyErr_Clear();  // cancelled
      own = e && e == exc;
      Py_XDECREF(e);
    }
    if (own) {
      Py_DECREF(exc);
      int rc = queue_resume(s);
      if (rc < 0) {
        if (s->state == ST_QUEUED) leave_queue(s);
        s->state = ST_DONE;
        return nullptr;
      }
      PyObject* out = nullptr;
      PySendResult r = PyIter_Send(reinterpret_cast<PyObject*>(s), Py_None, &out);  // ST_DELEGATE or ST_WAIT
      return call_result(r, out);
    }
    s->state = ST_DONE;
    leave_queue(s);
  }
  if (s->state == ST_WAIT) {  // the request loop's except clauses see it at the await (h1.py _exchange)
    int rc = start_delegate(s, exc);
    Py_DECREF(exc);
    if (rc < 0) return nullptr;
    PyObject* out = nullptr;
    PySendResult r = delegate_send(s, Py_None, &out);
    return call_result(r, out);
  }
  PyErr_SetObject(reinterpret_cast<PyObject*>(Py_TYPE(exc)), exc);
  Py_DECREF(exc);
  return nullptr;
}

PyObject* call_close(H1CallObject* s, PyObject*) {
  if (s->state == ST_DELEGATE) {
    s->state = ST_DONE;
    PyObject* sub = s->sub;
    s->sub = nullptr;
    PyObject* r = PyObject_CallMethodNoArgs(sub, s_close);
    Py_DECREF(sub);
    return r;
  }
  if (s->state == ST_WAIT) {
    s->state = ST_DONE;
    abandon(s);
  } else if (s->state == ST_QUEUED) {
    s->state = ST_DONE;
    leave_queue(s);
  }
  s->state = ST_DONE;
  Py_RETURN_NONE;
}

PyObject* call_await(H1CallObject* s) {
  Py_INCREF(s);
  return reinterpret_cast<PyObject*>(s);
}

PyObject* call_get_native(H1CallObject* s, void*) {
  if (s->path == 0) Py_RETURN_NONE;
  return PyBool_FromLong(s->path == 1);
}

PyGetSetDef call_getset[] = {
    {"native", reinterpret_cast<getter>(call_get_native), nullptr,
     "None before the first await; True if the request was sent on the native path", nullptr},
    {nullptr, nullptr, nullptr, nullptr, nullptr}};

PyAsyncMethods call_async = {reinterpret_cast<unaryfunc>(call_await), nullptr, nullptr,
                             reinterpret_cast<sendfunc>(call_am_send)};

PyMethodDef call_methods[] = {
    {"send", reinterpret_cast<PyCFunction>(call_send), METH_O, nullptr},
    {"throw", reinterpret_cast<PyCFunction>(call_throw), METH_VARARGS, nullptr},
    {"close", reinterpret_cast<PyCFunction>(call_close), METH_NOARGS, nullptr},
    {"__await__", reinterpret_cast<PyCFunction>(call_await), METH_NOARGS, nullptr},
    {nullptr, nullptr, 0, nullptr}};

// ---- h1_fast ----------------------------------------------------------------------------------
PyObject* make_deadline(PyObject* loop, PyObject* timeout, PyObject* timeout_s);
int send_on(H1CallObject* s, PyObject* conn, const char* req, size_t reqlen, PyObject* method, PyObject* full,
            PyObject* deadline, bool head, bool from_idle);
int queue_start(H1CallObject* s, PyObject* client, PyObject* counts, PyObject* o, PyObject* full,
                const std::string& req, bool head, PyObject* timeout, PyObject* timeout_s);

// The shapes the native path sends (sinks/h1.py _split_url, no quoting needed): a str method
// that is an upper-case ASCII token, an ASCII URL scheme://authority[/path][?query] with a
// printable target and no fragment, params absent or a dict (not combined with a query already
// in the URL). *k = length of "scheme://authority". true = send natively.
bool split_shape(PyObject* method, PyObject* url, PyObject* params, Py_ssize_t* k_out) {
  if (!PyUnicode_CheckExact(method) || !PyUnicode_IS_ASCII(method) || !PyUnicode_CheckExact(url) ||
      !PyUnicode_IS_ASCII(url) || (params && !PyDict_CheckExact(params)))
    return false;
  Py_ssize_t mn = PyUnicode_GET_LENGTH(method);
  const char* m = reinterpret_cast<const char*>(PyUnicode_1BYTE_DATA(method));
  if (mn == 0) return false;
  for (Py_ssize_t i = 0; i < mn; ++i)
    if (m[i] < 'A' || m[i] > 'Z') return false;
  Py_ssize_t un = PyUnicode_GET_LENGTH(url);
  const char* u = reinterpret_cast<const char*>(PyUnicode_1BYTE_DATA(url));
  Py_ssize_t i = 0;
  while (i + 2 < un && !(u[i] == ':' && u[i + 1] == '/' && u[i + 2] == '/')) ++i;
  if (i == 0 || i + 2 >= un) return false;
  Py_ssize_t k = i + 3;
  while (k < un && u[k] != '/' && u[k] != '?' && u[k] != '#') ++k;
  bool has_q = false;
  Py_ssize_t j = k;
  // 8 bytes at a time while none is outside 0x21..0x7E, '#' or '?' (a plain path; the bytes are
  // ASCII, so the per-byte sums below never carry); the byte loop takes over from the first word
  // that has one
  constexpr uint64_t ones = 0x0101010101010101ULL, highs = 0x8080808080808080ULL;
  for (; j + 8 <= un; j += 8) {
    uint64_t w;
    memcpy(&w, u + j, 8);
    const uint64_t ctl = (w - ones * 0x21) & ~w & highs;  // a byte < 0x21
    const uint64_t del = (w + ones) & highs;              // 0x7F
    const uint64_t h = w ^ (ones * '#'), q = w ^ (ones * '?');
    const uint64_t hq = ((h - ones) & ~h & highs) | ((q - ones) & ~q & highs);
    if (ctl | del | hq) break;
  }
  for (; j < un; ++j) {
    unsigned char ch = static_cast<unsigned char>(u[j]);
    if (ch < 0x21 || ch > 0x7E || ch == '#') return false;  // _resolve would quote it
    if (ch == '?') has_q = true;
  }
  if (params && has_q && PyDict_GET_SIZE(params)) return false;  // with_query appends with '&'
  *k_out = k;
  return true;
}

// The request text for a URL that passed split_shape, on an origin whose Host header is `host`
// and Authorization `auth` (str or None): "M target HTTP/1.1\r\nHost: h\r\n[Authorization:
// a\r\n]" + the User-Agent tail (`tail_cl0` for methods with a body). `q` = the encoded query.
// false = not the native shape (a non-ASCII host, a query value the encoder refuses).
bool request_text(PyObject* method, PyObject* url, Py_ssize_t k, PyObject* params, PyObject* host, PyObject* auth,
                  PyObject* tail, PyObject* tail_cl0, std::string& req, std::string& q) {
  if (!PyUnicode_CheckExact(host) || !PyUnicode_IS_ASCII(host) ||
      (auth != Py_None && (!PyUnicode_CheckExact(auth) || !PyUnicode_IS_ASCII(auth))))
    return false;
  Py_ssize_t mn = PyUnicode_GET_LENGTH(method);
  const char* m = reinterpret_cast<const char*>(PyUnicode_1BYTE_DATA(method));
  Py_ssize_t un = PyUnicode_GET_LENGTH(url);
  const char* u = reinterpret_cast<const char*>(PyUnicode_1BYTE_DATA(url));
  req.reserve(size_t(un) + 256);
  req.append(m, size_t(mn));
  req += ' ';
  if (k == un || u[k] != '/') req += '/';
  req.append(u + k, size_t(un - k));
  if (params && PyDict_GET_SIZE(params)) {
    Py_ssize_t pos = 0;
    PyObject *pk, *pv;
    bool first = true;
    while (PyDict_Next(params, &pos, &pk, &pv)) {
      if (!text_query_pair_append(q, pk, pv, &first, false)) {
        PyErr_Clear();  // the Python path raises it at the await
        return false;
      }
    }
    if (!q.empty()) {
      req += '?';
      req += q;
    }
  }
  req += " HTTP/1.1\r\nHost: ";
  req.append(reinterpret_cast<const char*>(PyUnicode_1BYTE_DATA(host)), size_t(PyUnicode_GET_LENGTH(host)));
  req += "\r\n";
  if (auth != Py_None) {
    req += "Authorization: ";
    req.append(reinterpret_cast<const char*>(PyUnicode_1BYTE_DATA(auth)), size_t(PyUnicode_GET_LENGTH(auth)));
    req += "\r\n";
  }
  PyObject* t = is_body_method(m, mn) ? tail_cl0 : tail;
  req.append(PyBytes_AS_STRING(t), size_t(PyBytes_GET_SIZE(t)));
  return true;
}

// `url` with its query `q` appended (new reference).
PyObject* full_url(PyObject* url, const std::string& q) {
  if (q.empty()) return Py_NewRef(url);
  // url (ASCII: split_shape) + "?" + q (percent-encoded: ASCII): one compact ASCII str, filled in
  // place, without a UTF-8 decode of the joined text
  Py_ssize_t un = PyUnicode_GET_LENGTH(url);
  PyObject* f = PyUnicode_New(un + 1 + Py_ssize_t(q.size()), 127);
  if (!f) return nullptr;
  Py_UCS1* d = PyUnicode_1BYTE_DATA(f);
  memcpy(d, PyUnicode_1BYTE_DATA(url), size_t(un));
  d[un] = '?';
  memcpy(d + un + 1, q.data(), q.size());
  return f;
}

// At the first await: send the request on an idle pooled connection. 1 = sent (s->conn, fut,
// method, full, deadline, reused set), 0 = declined before any pool state changed (the Python
// path runs instead and reproduces any error at its await), -1 = error.
int h1_start(H1CallObject* s) {
  PyObject* client = s->client;
  PyObject* method = s->method;
  PyObject* url = s->full;
  PyObject* params = s->params;
  PyObject* timeout = s->timeout;
  // the shapes the sinks produce (split_shape): anything else takes the Python path, which
  // raises or handles it (a Mapping that is not a dict, a non-ASCII host, a bytes method, ...)
  if (!client_view(client)) return PyErr_Occurred() ? -1 : 0;
  PyObject* const* v = g_client_view.v;
  PyObject *cclosed = v[CV_CLOSED], *origins = v[CV_ORIGINS], *counts = v[CV_COUNTS],
           *keepalive = v[CV_KEEPALIVE], *timeout_s = v[CV_TIMEOUT], *busy = v[CV_BUSY], *tail = v[CV_TAIL],
           *tail_cl0 = v[CV_TAIL_CL0];
  if (!cclosed || !origins || !counts || !keepalive || !timeout_s || !busy || !tail || !tail_cl0) return 0;
  if (cclosed != Py_False || !PyDict_CheckExact(origins) || !PyDict_CheckExact(counts) || !PySet_CheckExact(busy) ||
      !PyBytes_CheckExact(tail) || !PyBytes_CheckExact(tail_cl0) || !PyFloat_CheckExact(keepalive))
    return 0;

  Py_ssize_t k;
  if (!split_shape(method, url, params, &k)) return 0;
  PyObject* key = PyUnicode_FromStringAndSize(reinterpret_cast<const char*>(PyUnicode_1BYTE_DATA(url)), k);
  if (!key) return -1;
  PyObject* o = PyDict_GetItemWithError(origins, key);
  Py_DECREF(key);
  if (!o) {
    if (PyErr_Occurred()) return -1;
    return 0;  // first request to this origin: the Python path creates it
  }
  if (Py_TYPE(o) != g.origin.type) return 0;
  PyObject* host = g.origin.get(o, O_HOST_HEADER);
  PyObject* auth = g.origin.get(o, O_AUTH);
  PyObject* idle = g.origin.get(o, O_IDLE);
  if (!host || !auth || !idle) return 0;
  ScratchStr req_buf, q_buf;  // the request goes to the connection's buffer (or a bytes) below
  std::string &req = *req_buf, &q = *q_buf;
  if (!request_text(method, url, k, params, host, auth, tail, tail_cl0, req, q)) return 0;
  const char* m = reinterpret_cast<const char*>(PyUnicode_1BYTE_DATA(method));
  bool head = PyUnicode_GET_LENGTH(method) == 4 && memcmp(m, "HEAD", 4) == 0;
  PyObject* full = full_url(url, q);  // the URL with its query (HttpResponse.url, error text)
  if (!full) return -1;
  Own own_full{full};

  // a live idle keep-alive connection on a NetConn (the Python fast path's idle pop)
  double ka = PyFloat_AS_DOUBLE(keepalive);
  PyObject* conn = nullptr;
  for (;;) {
    Py_ssize_t n = PyObject_Size(idle);
    if (n < 0) return -1;
    if (n == 0) return queue_start(s, client, counts, o, full, req, head, timeout, timeout_s);
    PyObject* cand = PyObject_CallMethodNoArgs(idle, s_pop);
    if (!cand) return -1;
    if (Py_TYPE(cand) != g.conn.type) {
      PyObject* r = PyObject_CallMethodOneArg(idle, s_append, cand);  // put it back
      Py_DECREF(cand);
      if (!r) return -1;
      Py_DECREF(r);
      return 0;
    }
    PyObject* closed = g.conn.get(cand, C_CLOSED);
    PyObject* last = g.conn.get(cand, C_LAST_USED);
    double lu = last ? PyFloat_AsDouble(last) : -1e300;
    if (lu == -1.0 && PyErr_Occurred()) {
      Py_DECREF(cand);
      return -1;
    }
    if (closed == Py_False && mono_s() - lu < ka) {
      PyObject* net = g.conn.get(cand, C_NET);
      if (!net || !is_netconn(net) || !netconn_open(net)) {  // asyncio transport: Python path
        PyObject* r = PyObject_CallMethodOneArg(idle, s_append, cand);
        Py_DECREF(cand);
        if (!r) return -1;
        Py_DECREF(r);
        return 0;
      }
      conn = cand;
      break;
    }
    PyObject* r = PyObject_CallMethodOneArg(client, s_drop, cand);  // stale: self._drop(cand)
    Py_DECREF(cand);
    if (!r) return -1;
    Py_DECREF(r);
  }

  // committed: the request goes out on `conn` (send_on owns it from here, and hands it back on
  // a failure); the connection's loop, as asyncio.get_running_loop() would cost a getpid(2)
  PyObject* deadline = bump(counts, s_requests) < 0 ? nullptr
                       : make_deadline(netconn_loop(g.conn.get(conn, C_NET)), timeout, timeout_s);
  if (!deadline) {
    PyObject *et, *ev, *tb;
    PyErr_Fetch(&et, &ev, &tb);
    PyObject* r = PyObject_CallMethodObjArgs(client, s_release, conn, Py_False, nullptr);
    Py_DECREF(conn);
    if (!r)
      PyErr_WriteUnraisable(client);
    else
      Py_DECREF(r);
    PyErr_Restore(et, ev, tb);
    return -1;
  }
  Own own_deadline{deadline};
  return send_on(s, conn, req.data(), req.size(), method, full, deadline, head, true);
}

// The queue deadline and request deadlines: loop.time() + (timeout or client.timeout_s). New
// reference, NULL on error.
PyObject* make_deadline(PyObject* loop, PyObject* timeout, PyObject* timeout_s) {
  double dl;
  if (g.base_time && _PyType_Lookup(Py_TYPE(loop), s_time) == g.base_time) {
    dl = mono_s();  // BaseEventLoop.time() is time.monotonic()
  } else {
    PyObject* now = PyObject_CallMethodNoArgs(loop, s_time);
    if (!now) return nullptr;
    dl = PyFloat_AsDouble(now);
    Py_DECREF(now);
    if (dl == -1.0 && PyErr_Occurred()) return nullptr;
  }
  PyObject* tmo = timeout;  // `timeout or self.timeout_s`
  if (tmo) {
    int truth = PyObject_IsTrue(tmo);
    if (truth < 0) return nullptr;
    if (!truth) tmo = nullptr;
  }
  double add = PyFloat_AsDouble(tmo ? tmo : timeout_s);
  if (add == -1.0 && PyErr_Occurred()) return nullptr;
  return PyFloat_FromDouble(dl + add);
}

// Sends `req` on the live NetConn connection `conn` (a new reference, consumed) and moves the
// call to ST_WAIT: the pool bookkeeping of h1.py _exchange (uses, reused, deadline, what, the
// busy set, the sweeper). `from_idle`: popped from the idle pool (counted reused, as the Python
// idle pop does); else handed to a queued request (reused when it served one before, as
// _acquire counts). 1, or -1 with the connection handed back to the pool accounting.
int send_on(H1CallObject* s, PyObject* conn, const char* req, size_t reqlen, PyObject* method, PyObject* full,
            PyObject* deadline, bool head, bool from_idle) {
  Own own_conn{conn};
  PyObject* client = s->client;
  // a failure hands the connection back to the pool accounting (dropped, h1.py _release(c,
  // False)), or its origin would count it open forever
  auto fail = [client, conn]() {
    PyObject *et, *ev, *tb;
    PyErr_Fetch(&et, &ev, &tb);
    PyObject* r = PyObject_CallMethodObjArgs(client, s_release, conn, Py_False, nullptr);
    if (!r)
      PyErr_WriteUnraisable(client);
    else
      Py_DECREF(r);
    PyErr_Restore(et, ev, tb);
    return -1;
  };
  PyObject* d = client_view(client);
  PyObject* counts = d ? g_client_view.v[CV_COUNTS] : nullptr;
  PyObject* busy = d ? g_client_view.v[CV_BUSY] : nullptr;
  if (!counts || !busy || !PyDict_CheckExact(counts) || !PySet_CheckExact(busy)) {
    if (!PyErr_Occurred()) PyErr_SetString(PyExc_RuntimeError, "H1Client state changed under a request");
    return fail();
  }
  PyObject* uses = g.conn.get(conn, C_USES);
  bool reused = true;
  if (uses) {
    int pos = PyObject_IsTrue(uses);  // reused = c.uses > 0
    if (pos < 0) return fail();
    reused = pos != 0;
    PyObject* one = PyLong_FromLong(1);
    PyObject* nu = one ? PyNumber_Add(uses, one) : nullptr;
    Py_XDECREF(one);
    if (!nu) return fail();
    g.conn.set(conn, C_USES, nu);
  }
  if ((from_idle || reused) && bump(counts, s_reused) < 0) return fail();
  PyObject* loop = netconn_loop(g.conn.get(conn, C_NET));
  Py_INCREF(loop);
  Own own_loop{loop};
  Py_INCREF(method);
  PyObject* what = PyTuple_Pack(2, method, full);
  Py_DECREF(method);
  if (!what) return fail();
  Py_INCREF(deadline);
  g.conn.set(conn, C_DEADLINE, deadline);
  g.conn.set(conn, C_WHAT, what);
  PyObject* fut = iofuture_new(loop);
  if (!fut) return fail();
  Own own_fut{fut};
  if (netconn_h1_request(g.conn.get(conn, C_NET), req, reqlen, fut, head) < 0) return fail();
  if (PySet_Add(busy, conn) < 0) return fail();
  PyObject* sweeper = PyDict_GetItemWithError(d, s_sweeper);
  if (!sweeper && PyErr_Occurred()) {
    PySet_Discard(busy, conn);
    return fail();
  }
  if (!sweeper || sweeper == Py_None) {
    PyObject* r = PyObject_CallMethodOneArg(client, s_arm, loop);
    if (!r) {
      PySet_Discard(busy, conn);
      return fail();
    }
    Py_DECREF(r);
  }
  own_conn.p = nullptr;
  Py_XSETREF(s->conn, conn);
  own_fut.p = nullptr;
  Py_XSETREF(s->fut, fut);
  Py_INCREF(method);
  Py_SETREF(s->method, method);
  Py_INCREF(full);
  Py_SETREF(s->full, full);
  Py_INCREF(deadline);
  Py_XSETREF(s->deadline, deadline);
  s->reused = reused;
  Py_CLEAR(s->params);
  Py_CLEAR(s->timeout);
  Py_CLEAR(s->req);
  s->state = ST_WAIT;
  return 1;
}

// No idle connection: the request joins the origin's queue (H1Client._enqueue: the same
// accounting, background connects and deadline as _acquire) with an IOFuture waiter, and the
// call waits for a connection in ST_QUEUED. 2 = queued, -1 = error.
int queue_start(H1CallObject* s, PyObject* client, PyObject* counts, PyObject* o, PyObject* full,
                const std::string& req, bool head, PyObject* timeout, PyObject* timeout_s) {
  if (!g.get_running_loop) return 0;
  PyObject* loop = PyObject_CallNoArgs(g.get_running_loop);
  if (!loop) return -1;
  Own own_loop{loop};
  PyObject* deadline = make_deadline(loop, timeout, timeout_s);
  if (!deadline) return -1;
  Own own_deadline{deadline};
  PyObject* reqb = PyBytes_FromStringAndSize(req.data(), Py_ssize_t(req.size()));
  if (!reqb) return -1;
  Own own_req{reqb};
  PyObject* w = iofuture_new(loop);
  if (!w) return -1;
  Own own_w{w};
  if (bump(counts, s_requests) < 0) return -1;
  PyObject* args[5] = {client, o, deadline, w, s->front ? Py_True : Py_False};
  PyObject* timer = PyObject_VectorcallMethod(s_enqueue, args, 5, nullptr);
  if (!timer) return -1;
  s->timer = timer;
  own_w.p = nullptr;
  Py_XSETREF(s->fut, w);
  Py_INCREF(full);
  Py_SETREF(s->full, full);
  own_deadline.p = nullptr;
  Py_XSETREF(s->deadline, deadline);
  own_req.p = nullptr;
  Py_XSETREF(s->req, reqb);
  s->head = head;
  s->state = ST_QUEUED;
  return 2;
}

// ST_QUEUED, resumed: the waiter finished. A live native connection: the request is sent on it
// (ST_WAIT). Anything else (a freed slot, a connection closed meanwhile or not native, the
// client closing, the deadline, a failed connect): H1Client._after_queue continues the request
// in Python (ST_DELEGATE). 0, or -1 with an error set.
int queue_resume(H1CallObject* s) {
  PyObject* r = PyObject_CallMethodNoArgs(s->timer, s_cancel);
  if (!r) return -1;
  Py_DECREF(r);
  Py_CLEAR(s->timer);
  PyObject* w = s->fut;
  PyObject* res = nullptr;
  int st = iofuture_peek(w, &res);
  PyObject* got = nullptr;  // new reference: the result, or the exception
  if (st == 1) {
    got = res;
    Py_INCREF(got);
  } else {
    got = PyObject_CallMethodNoArgs(w, s_exception_name);  // raises CancelledError when cancelled
    if (!got) return -1;
  }
  Own own_got{got};
  if (st == 1 && Py_TYPE(got) == g.conn.type) {
    PyObject* cclosed = client_attr(s->client, s_closed_attr);
    if (!cclosed) return -1;
    PyObject* net = g.conn.get(got, C_NET);
    if (cclosed == Py_False && g.conn.get(got, C_CLOSED) == Py_False && net && is_netconn(net) &&
        netconn_open(net)) {
      own_got.p = nullptr;
      PyObject* req = s->req;
      Py_INCREF(req);  // send_on clears s->req
      Own own_req{req};
      Py_CLEAR(s->fut);
      return send_on(s, got, PyBytes_AS_STRING(req), size_t(PyBytes_GET_SIZE(req)), s->method, s->full,
                     s->deadline, s->head != 0, false) < 0 ? -1 : 0;
    }
  }
  Py_CLEAR(s->fut);
  Py_CLEAR(s->req);
  PyObject* args[5] = {s->client, s->method, s->full, s->deadline, got};
  PyObject* sub = PyObject_VectorcallMethod(s_after_queue, args, 5, nullptr);
  if (!sub) {
    if (Py_TYPE(got) == g.conn.type) {  // handed over but not taken: back to the pool accounting
      PyObject *et, *ev, *tb;
      PyErr_Fetch(&et, &ev, &tb);
      PyObject* r = PyObject_CallMethodObjArgs(s->client, s_release, got, Py_False, nullptr);
      if (!r)
        PyErr_WriteUnraisable(s->client);
      else
        Py_DECREF(r);
      PyErr_Restore(et, ev, tb);
    }
    return -1;
  }
  if (!PyCoro_CheckExact(sub)) {
    Py_DECREF(sub);
    PyErr_SetString(PyExc_TypeError, "H1Client._after_queue must be a coroutine function");
    return -1;
  }
  s->sub = sub;
  s->state = ST_DELEGATE;
  return 0;
}

// h1_fast(client, method, url, params=None, timeout=None, front=False) -> H1Call or None
PyObject* mod_h1_fast(PyObject*, PyObject* const* a, Py_ssize_t n) {
  if (n < 3 || n > 6) {
    PyErr_SetString(PyExc_TypeError, "h1_fast(client, method, url, params=None, timeout=None, front=False)");
    return nullptr;
  }
  if (!g.ready || Py_TYPE(a[0]) != g.client_type) Py_RETURN_NONE;
  int front = n > 5 ? PyObject_IsTrue(a[5]) : 0;
  if (front < 0) return nullptr;
  H1CallObject* call = PyObject_GC_New(H1CallObject, &H1CallType);
  if (!call) return nullptr;
  PyObject* params = n > 3 && a[3] != Py_None ? a[3] : nullptr;
  PyObject* timeout = n > 4 && a[4] != Py_None ? a[4] : nullptr;
  Py_INCREF(a[0]);
  call->client = a[0];
  Py_INCREF(a[1]);
  call->method = a[1];
  Py_INCREF(a[2]);
  call->full = a[2];
  Py_XINCREF(params);
  call->params = params;
  Py_XINCREF(timeout);
  call->timeout = timeout;
  call->conn = call->fut = call->deadline = call->sub = call->timer = call->req = nullptr;
  call->head = 0;
  call->front = uint8_t(front);
  call->state = ST_INIT;
  call->reused = 0;
  call->path = 0;
  PyObject_GC_Track(call);
  return reinterpret_cast<PyObject*>(call);
}

}  // namespace

// h1_fast for a caller in C (the compiled handlers): an H1Call, or None when `client` is not a
// stock H1Client (new reference either way), NULL on error.
PyObject* h1_call_new(PyObject* client, PyObject* method, PyObject* url, PyObject* params, PyObject* timeout,
                      bool front) {
  PyObject* a[6] = {client, method, url, params, timeout, front ? Py_True : Py_False};
  return mod_h1_fast(nullptr, a, 6);
}

// ---- NativeApi entries (native_api.hpp) -------------------------------------------------------
// The arguments of the last h1_origin_key call that passed the shape check (GIL-held, like every
// API entry). h1_request_text trusts a caller's key_len only for those very objects (the caller
// that asked h1_origin_key and builds the request next, the stub's order); any other key_len, or
// the same URL after another check, gets the full check (a key_len taken for another
// URL must not build a malformed request line). One use: the next request_text takes it. The
// entry holds references, so a freed URL's address cannot come back as another URL that matches.
struct LastKey {
  PyObject* method = nullptr;  // strong references, compared by identity
  PyObject* url = nullptr;
  PyObject* params = nullptr;
  Py_ssize_t len = 0;
  Py_ssize_t k = 0;
  void drop() {
    Py_CLEAR(method);
    Py_CLEAR(url);
    Py_CLEAR(params);
  }
} g_last_key;

int api_h1_request_text(PyObject* method, PyObject* url, PyObject* params, PyObject* host, PyObject* auth,
                        PyObject* tail, PyObject* tail_cl0, std::string* req, PyObject** full, Py_ssize_t* key_len) {
  BEHOLDER_TRY {
    if (params == Py_None) params = nullptr;
    if (!PyBytes_Check(tail) || !PyBytes_Check(tail_cl0)) {
      PyErr_SetString(PyExc_TypeError, "h1_request_text: tail and tail_cl0 must be bytes");
      return -1;
    }
    Py_ssize_t k = *key_len;
    LastKey& last = g_last_key;
    const bool known = k > 0 && last.url == url && last.method == method && last.params == params &&
                       last.k == k && PyUnicode_CheckExact(url) && PyUnicode_GET_LENGTH(url) == last.len;
    last.drop();
    if (!known && !split_shape(method, url, params, &k)) return 0;
    ScratchStr q_buf;
    std::string& q = *q_buf;
    req->clear();
    if (!request_text(method, url, k, params, host, auth, tail, tail_cl0, *req, q)) return 0;
    *full = full_url(url, q);
    if (!*full) return -1;
    *key_len = k;
    return 1;
  }
  BEHOLDER_CATCH(-1)
}

PyTypeObject* h1_response_type() { return g.resp.type; }

PyObject* h1_response_status(PyObject* resp) { return g.resp.get(resp, R_STATUS); }

int api_h1_origin_key(PyObject* method, PyObject* url, PyObject* params, Py_ssize_t* key_len) {
  if (params == Py_None) params = nullptr;
  LastKey& last = g_last_key;
  last.drop();
  if (!split_shape(method, url, params, key_len)) return 0;
  Py_INCREF(method);
  last.method = method;
  Py_INCREF(url);
  last.url = url;
  Py_XINCREF(params);
  last.params = params;
  last.len = PyUnicode_GET_LENGTH(url);
  last.k = *key_len;
  return 1;
}

PyObject* api_h1_response(PyObject* parsed, PyObject* full) {
  if (!PyTuple_CheckExact(parsed) || PyTuple_GET_SIZE(parsed) != 5) {
    PyErr_SetString(PyExc_TypeError, "h1_response: expected an H1Parser result tuple");
    return nullptr;
  }
  return make_response(PyTuple_GET_ITEM(parsed, 0), PyTuple_GET_ITEM(parsed, 3), PyTuple_GET_ITEM(parsed, 2), full);
}

namespace {

// h1_setup(client_cls, conn_cls, origin_cls, response_cls)
PyObject* mod_h1_setup(PyObject*, PyObject* args) {
  PyObject *client_cls, *conn_cls, *origin_cls, *resp_cls;
  if (!PyArg_ParseTuple(args, "OOOO", &client_cls, &conn_cls, &origin_cls, &resp_cls)) return nullptr;
  g.ready = false;
  if (!PyType_Check(client_cls)) {
    PyErr_SetString(PyExc_TypeError, "h1_setup: client_cls must be a class");
    return nullptr;
  }
  if (!g.conn.resolve(conn_cls, kConnSlots, C_N) || !g.origin.resolve(origin_cls, kOriginSlots, O_N) ||
      !g.resp.resolve(resp_cls, kRespSlots, R_N))
    return nullptr;
  if (reinterpret_cast<PyTypeObject*>(resp_cls)->tp_dictoffset != 0) {
    PyErr_SetString(PyExc_TypeError, "h1_setup: the response class must have __slots__ only");
    return nullptr;
  }
  Py_INCREF(client_cls);
  Py_XSETREF(g.client_type, reinterpret_cast<PyTypeObject*>(client_cls));
  PyObject* be = PyImport_ImportModule("asyncio.base_events");
  PyObject* cls = be ? PyObject_GetAttrString(be, "BaseEventLoop") : nullptr;
  Py_XDECREF(be);
  if (!cls) return nullptr;
  PyObject* bt = _PyType_Lookup(reinterpret_cast<PyTypeObject*>(cls), s_time);
  Py_XINCREF(bt);
  Py_XSETREF(g.base_time, bt);
  Py_DECREF(cls);
  PyObject* aio = PyImport_ImportModule("asyncio");
  PyObject* grl = aio ? PyObject_GetAttrString(aio, "get_running_loop") : nullptr;
  Py_XDECREF(aio);
  if (!grl) return nullptr;
  Py_XSETREF(g.get_running_loop, grl);
  g.ready = true;
  Py_RETURN_NONE;
}

PyObject* mod_h1_disable(PyObject*, PyObject*) {
  g.ready = false;
  Py_RETURN_NONE;
}

PyMethodDef h1_functions[] = {
    {"h1_fast", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(mod_h1_fast)), METH_FASTCALL,
     "h1_fast(client, method, url, params=None, timeout=None, front=False) -> awaitable H1Call, or None for the Python path "
     "(sinks/h1.py)"},
    {"h1_setup", mod_h1_setup, METH_VARARGS,
     "h1_setup(H1Client, _Conn, _Origin, HttpResponse): enable h1_fast for these classes"},
    {"h1_disable", mod_h1_disable, METH_NOARGS, "h1_disable(): h1_fast always returns None"},
    {nullptr, nullptr, 0, nullptr}};

}  // namespace

int init_h1call_types(PyObject* m) {
  struct {
    PyObject** slot;
    const char* text;
  } strs[] = {{&s_closed_attr, "_closed"},   {&s_origins, "_origins"},   {&s_counts, "counts"},
              {&s_keepalive_s, "keepalive_s"}, {&s_timeout_s, "timeout_s"}, {&s_busy, "_busy"},
              {&s_sweeper, "_sweeper"},       {&s_tail, "_tail"},         {&s_tail_cl0, "_tail_cl0"},
              {&s_requests, "requests"},      {&s_reused, "reused"},      {&s_drop, "_drop"},
              {&s_release, "_release"},       {&s_arm, "_arm"},           {&s_resume, "_resume"},
              {&s_time, "time"},              {&s_pop, "pop"},            {&s_append, "append"},
              {&s_buffered, "buffered"},      {&s_throw, "throw"},        {&s_close, "close"},
              {&s_request_py, "_request"},    {&s_cancel, "cancel"},      {&s_enqueue, "_enqueue"},
              {&s_after_queue, "_after_queue"}, {&s_exception_name, "exception"}};
  for (auto& s : strs)
    if (!(*s.slot = PyUnicode_InternFromString(s.text))) return -1;
  H1CallType.tp_name = "beholder_amd.ops._native.H1Call";
  H1CallType.tp_basicsize = sizeof(H1CallObject);
  H1CallType.tp_flags = Py_TPFLAGS_DEFAULT | Py_TPFLAGS_HAVE_GC;
  H1CallType.tp_doc = "An HTTP/1.1 request in flight on the native fast path (awaitable; see h1_fast)";
  H1CallType.tp_dealloc = reinterpret_cast<destructor>(call_dealloc);
  H1CallType.tp_finalize = reinterpret_cast<destructor>(call_finalize);
  H1CallType.tp_traverse = reinterpret_cast<traverseproc>(call_traverse);
  H1CallType.tp_clear = reinterpret_cast<inquiry>(call_clear);
  H1CallType.tp_as_async = &call_async;
  H1CallType.tp_iter = PyObject_SelfIter;
  H1CallType.tp_iternext = reinterpret_cast<iternextfunc>(call_iternext);
  H1CallType.tp_methods = call_methods;
  H1CallType.tp_getset = call_getset;
  if (PyType_Ready(&H1CallType) < 0) return -1;
  Py_INCREF(&H1CallType);
  if (PyModule_AddObject(m, "H1Call", reinterpret_cast<PyObject*>(&H1CallType)) < 0) return -1;
  return PyModule_AddFunctions(m, h1_functions);
}

}  // namespace beholder
