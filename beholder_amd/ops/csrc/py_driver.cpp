// Driver: resumes a suspended handler coroutine without an asyncio.Task.
//
// A handler (index.js:62,127) that awaits real I/O (a Postgres lookup, a Trello
// POST) leaves dispatch_batch with a started coroutine and the future it is
// waiting on. asyncio would wrap it in a Task: Task creation, a call_soon per
// step, context switching and done-callback scheduling cost ~10 us per
// suspension in CPython 3.10. A Driver is the future's done-callback. When the
// future completes, it sends the result (or throws the exception) into the
// coroutine with PyIter_Send, and re-arms on the next future the coroutine
// yields. When the coroutine returns or raises, it calls
// on_done(driver, exc_or_None) once.
//
//   drv = Driver(coro, on_done, payload=None)
//   drv.start(first_yield)     # the future dispatch_batch got from the first send
//   drv.cancel()               # like Task.cancel(): CancelledError at the await
//
// Task semantics that are kept:
//   * `_asyncio_future_blocking` handshake: a bare `yield` (asyncio.sleep(0))
//     reschedules through loop.call_soon;
//   * a yield of anything else is thrown back as RuntimeError;
//   * cancellation cancels the awaited future;
//   * KeyboardInterrupt / SystemExit propagate to the loop after on_done.
// Context variables are not switched. Handlers run in the dispatch loop's context.
// asyncio.current_task() is not set while a Driver steps a coroutine (and during the
// eager first step it is the dispatch loop's task). Library code that needs its own
// task must run in one. sinks/http.py AiohttpClient does this, because aiohttp's
// timeouts cancel current_task().
#include "py_common.hpp"

namespace beholder {

namespace {

struct DriverObject {
  PyObject_HEAD PyObject* coro;  // NULL once finished
  PyObject* on_done;
  PyObject* payload;
  PyObject* waiting;  // future currently awaited (holds us as its callback)
  PyObject* loop;     // running loop, for bare-yield rescheduling
  uint8_t must_cancel;
  uint8_t done;
  uint8_t cancelled;
  uint64_t steps;
};

PyTypeObject DriverType = {PyVarObject_HEAD_INIT(nullptr, 0)};

PyObject* g_cancelled_error = nullptr;   // asyncio.CancelledError
PyObject* g_get_running_loop = nullptr;  // asyncio.get_running_loop
PyObject* s_blocking = nullptr;          // "_asyncio_future_blocking"
PyObject* s_add_done_callback = nullptr;
PyObject* s_result = nullptr;
PyObject* s_throw = nullptr;
PyObject* s_call_soon = nullptr;
PyObject* s_cancel = nullptr;

int driver_traverse(DriverObject* s, visitproc visit, void* arg) {
  Py_VISIT(s->coro);
  Py_VISIT(s->on_done);
  Py_VISIT(s->payload);
  Py_VISIT(s->waiting);
  Py_VISIT(s->loop);
  return 0;
}

int driver_clear(DriverObject* s) {
  Py_CLEAR(s->coro);
  Py_CLEAR(s->on_done);
  Py_CLEAR(s->payload);
  Py_CLEAR(s->waiting);
  Py_CLEAR(s->loop);
  return 0;
}

void driver_dealloc(DriverObject* s) {
  PyObject_GC_UnTrack(s);
  driver_clear(s);
  Py_TYPE(s)->tp_free(reinterpret_cast<PyObject*>(s));
}

PyObject* driver_new(PyTypeObject* type, PyObject*, PyObject*) {
  DriverObject* s = reinterpret_cast<DriverObject*>(type->tp_alloc(type, 0));
  if (!s) return nullptr;
  s->coro = s->on_done = s->payload = s->waiting = s->loop = nullptr;
  s->must_cancel = s->done = s->cancelled = 0;
  s->steps = 0;
  return reinterpret_cast<PyObject*>(s);
}

int driver_init(DriverObject* s, PyObject* args, PyObject* kwds) {
  static const char* kwlist[] = {"coro", "on_done", "payload", nullptr};
  PyObject *coro, *on_done, *payload = Py_None;
  if (!PyArg_ParseTupleAndKeywords(args, kwds, "OO|O", const_cast<char**>(kwlist), &coro, &on_done, &payload))
    return -1;
  if (!PyCallable_Check(on_done)) {
    PyErr_SetString(PyExc_TypeError, "on_done must be callable");
    return -1;
  }
  Py_INCREF(coro);
  Py_XSETREF(s->coro, coro);
  Py_INCREF(on_done);
  Py_XSETREF(s->on_done, on_done);
  Py_INCREF(payload);
  Py_XSETREF(s->payload, payload);
  return 0;
}

// Fetches the current exception as a normalized instance (new reference).
PyObject* fetch_exc() {
  PyObject *t, *v, *tb;
  PyErr_Fetch(&t, &v, &tb);
  PyErr_NormalizeException(&t, &v, &tb);
  if (tb && v) PyException_SetTraceback(v, tb);
  Py_XDECREF(t);
  Py_XDECREF(tb);
  return v;
}

// ---- Window: the set of handlers suspended on I/O (at most `limit`: the prefetch window,
// index.js:43). A Driver whose on_done is a Window reports to it in C.
struct WindowObject {
  PyObject_HEAD PyObject* drivers;  // set of live Drivers
  PyObject* on_error;               // callable(payload, exc): a handler raised
  PyObject* on_wake;                // callable(): a slot freed after the window was full, or it emptied
  Py_ssize_t limit;
  uint64_t suspended;
  uint64_t wakes;
};

PyTypeObject WindowType = {PyVarObject_HEAD_INIT(nullptr, 0)};

// A driver finished (`exc` borrowed, may be NULL): forget it, report errors, wake waiters on the
// transitions that matter. 0, or -1 with an exception set.
int window_done(WindowObject* w, DriverObject* drv, PyObject* exc) {
  Py_ssize_t before = PySet_GET_SIZE(w->drivers);
  if (PySet_Discard(w->drivers, reinterpret_cast<PyObject*>(drv)) < 0) return -1;
  if (exc && exc != Py_None && !drv->cancelled && w->on_error != Py_None) {
    PyObject* r = PyObject_CallFunctionObjArgs(w->on_error, drv->payload ? drv->payload : Py_None, exc, nullptr);
    if (!r) return -1;
    Py_DECREF(r);
  }
  Py_ssize_t n = PySet_GET_SIZE(w->drivers);
  if (((before >= w->limit && n < w->limit) || n == 0) && w->on_wake != Py_None) {
    ++w->wakes;
    PyObject* r = PyObject_CallNoArgs(w->on_wake);
    if (!r) return -1;
    Py_DECREF(r);
  }
  return 0;
}

// The coroutine is finished: report once. Returns 0, or -1 with an exception set
// (on_done raised, or a KeyboardInterrupt/SystemExit that must reach the loop).
int finish(DriverObject* s, PyObject* exc) {
  s->done = 1;
  Py_CLEAR(s->coro);
  Py_CLEAR(s->waiting);
  Py_CLEAR(s->loop);
  if (exc && PyErr_GivenExceptionMatches(exc, g_cancelled_error)) s->cancelled = 1;
  PyObject* cb = s->on_done;
  s->on_done = nullptr;
  PyObject* r;
  if (Py_TYPE(cb) == &WindowType) {
    r = window_done(reinterpret_cast<WindowObject*>(cb), s, exc) < 0 ? nullptr : Py_NewRef(Py_None);
  } else {
    r = PyObject_CallFunctionObjArgs(cb, reinterpret_cast<PyObject*>(s), exc ? exc : Py_None, nullptr);
  }
  Py_DECREF(cb);
  Py_CLEAR(s->payload);  // release the delivery promptly (an un-acked one is then counted as abandoned)
  if (!r) return -1;
  Py_DECREF(r);
  if (exc && !PyErr_GivenExceptionMatches(exc, PyExc_Exception) &&
      !PyErr_GivenExceptionMatches(exc, g_cancelled_error)) {
    Py_INCREF(exc);
    PyErr_SetObject(reinterpret_cast<PyObject*>(Py_TYPE(exc)), exc);
    Py_DECREF(exc);
    return -1;
  }
  return 0;
}

int step(DriverObject* s, PyObject* value, PyObject* exc);

// The coroutine yielded `y`: wait on it (a Future) or reschedule (bare yield).
int on_yield(DriverObject* s, PyObject* y) {
  if (y == Py_None) {
    if (!s->loop) {
      s->loop = PyObject_CallNoArgs(g_get_running_loop);
      if (!s->loop) return -1;
    }
    PyObject* h = PyObject_CallMethodObjArgs(s->loop, s_call_soon, reinterpret_cast<PyObject*>(s), Py_None,
                                             nullptr);
    if (!h) return -1;
    Py_DECREF(h);
    return 0;
  }
  PyObject* blocking = PyObject_GetAttr(y, s_blocking);
  if (!blocking) {
    PyErr_Clear();
  } else {
    int b = PyObject_IsTrue(blocking);
    Py_DECREF(blocking);
    if (b < 0) return -1;
    if (b) {
      if (PyObject_SetAttr(y, s_blocking, Py_False) < 0) return -1;
      PyObject* r = PyObject_CallMethodObjArgs(y, s_add_done_callback, reinterpret_cast<PyObject*>(s), nullptr);
      if (!r) return -1;
      Py_DECREF(r);
      Py_INCREF(y);
      Py_XSETREF(s->waiting, y);
      if (s->must_cancel) {
        s->must_cancel = 0;
        PyObject* c = PyObject_CallMethodNoArgs(y, s_cancel);
        if (!c) return -1;
        Py_DECREF(c);
      }
      return 0;
    }
  }
  // not an awaitable asyncio future: throw into the coroutine, as Task does
  PyObject* err = PyObject_CallFunction(PyExc_RuntimeError, "s",
                                        "handler coroutine yielded a non-Future (use `await`, not `yield`)");
  if (!err) return -1;
  int rc = step(s, nullptr, err);
  Py_DECREF(err);
  return rc;
}

// Resumes the coroutine with `value` or by throwing `exc` (borrowed references).
int step(DriverObject* s, PyObject* value, PyObject* exc) {
  if (!s->coro) return 0;
  ++s->steps;
  PyObject* y = nullptr;
  if (exc) {
    y = PyObject_CallMethodOneArg(s->coro, s_throw, exc);
    if (!y) {
      if (PyErr_ExceptionMatches(PyExc_StopIteration)) {
        PyErr_Clear();
        return finish(s, nullptr);
      }
      PyObject* e = fetch_exc();
      int rc = finish(s, e);
      Py_XDECREF(e);
      return rc;
    }
  } else {
    PySendResult r = PyIter_Send(s->coro, value, &y);
    if (r == PYGEN_RETURN) {
      Py_XDECREF(y);
      return finish(s, nullptr);
    }
    if (r == PYGEN_ERROR) {
      PyObject* e = fetch_exc();
      int rc = finish(s, e);
      Py_XDECREF(e);
      return rc;
    }
  }
  int rc = on_yield(s, y);
  Py_DECREF(y);
  return rc;
}

PyObject* driver_start(DriverObject* s, PyObject* first) {
  if (s->done || !s->coro || s->steps || s->waiting) {
    PyErr_SetString(PyExc_RuntimeError, "Driver.start() called twice or after completion");
    return nullptr;
  }
  ++s->steps;
  if (on_yield(s, first) < 0) return nullptr;
  Py_RETURN_NONE;
}

// tp_call: the awaited future's done-callback (or call_soon(self, None) for a bare yield).
PyObject* driver_call(DriverObject* s, PyObject* args, PyObject* kwds) {
  if (kwds && PyDict_GET_SIZE(kwds)) {
    PyErr_SetString(PyExc_TypeError, "Driver() takes no keyword arguments");
    return nullptr;
  }
  if (PyTuple_GET_SIZE(args) != 1) {
    PyErr_SetString(PyExc_TypeError, "Driver(fut) takes one argument");
    return nullptr;
  }
  if (s->done) Py_RETURN_NONE;
  PyObject* fut = PyTuple_GET_ITEM(args, 0);
  Py_INCREF(reinterpret_cast<PyObject*>(s));  // on_done may drop the last outside reference
  int rc;
  Py_CLEAR(s->waiting);
  if (fut == Py_None) {
    if (s->must_cancel) {
      s->must_cancel = 0;
      PyObject* e = PyObject_CallNoArgs(g_cancelled_error);
      if (!e) {
        Py_DECREF(reinterpret_cast<PyObject*>(s));
        return nullptr;
      }
      rc = step(s, nullptr, e);
      Py_DECREF(e);
    } else {
      rc = step(s, Py_None, nullptr);
    }
  } else {
    PyObject* r = PyObject_CallMethodNoArgs(fut, s_result);
    if (r) {
      rc = step(s, r, nullptr);
      Py_DECREF(r);
    } else {
      PyObject* e = fetch_exc();
      rc = step(s, nullptr, e);
      Py_XDECREF(e);
    }
  }
  Py_DECREF(reinterpret_cast<PyObject*>(s));
  if (rc < 0) return nullptr;
  Py_RETURN_NONE;
}

PyObject* driver_cancel(DriverObject* s, PyObject*) {
  if (s->done) Py_RETURN_FALSE;
  if (s->waiting) {
    PyObject* r = PyObject_CallMethodNoArgs(s->waiting, s_cancel);
    if (!r) return nullptr;
    int ok = PyObject_IsTrue(r);
    Py_DECREF(r);
    if (ok) Py_RETURN_TRUE;
  }
  s->must_cancel = 1;
  Py_RETURN_TRUE;
}

PyObject* driver_is_done(DriverObject* s, PyObject*) { return PyBool_FromLong(s->done); }

PyObject* driver_get_payload(DriverObject* s, void*) {
  PyObject* p = s->payload ? s->payload : Py_None;
  Py_INCREF(p);
  return p;
}
PyObject* driver_get_cancelled(DriverObject* s, void*) { return PyBool_FromLong(s->cancelled); }
PyObject* driver_get_steps(DriverObject* s, void*) { return PyLong_FromUnsignedLongLong(s->steps); }

PyMethodDef driver_methods[] = {
    {"start", reinterpret_cast<PyCFunction>(driver_start), METH_O,
     "start(first_yield): wait on the future the coroutine yielded first"},
    {"cancel", reinterpret_cast<PyCFunction>(driver_cancel), METH_NOARGS,
     "cancel() -> bool: CancelledError at the coroutine's current await"},
    {"done", reinterpret_cast<PyCFunction>(driver_is_done), METH_NOARGS, "done() -> bool"},
    {nullptr, nullptr, 0, nullptr}};

PyGetSetDef driver_getset[] = {
    {"payload", reinterpret_cast<getter>(driver_get_payload), nullptr, "user payload (the delivery)", nullptr},
    {"cancelled", reinterpret_cast<getter>(driver_get_cancelled), nullptr, "finished by CancelledError", nullptr},
    {"steps", reinterpret_cast<getter>(driver_get_steps), nullptr, "resumptions so far", nullptr},
    {nullptr, nullptr, nullptr, nullptr, nullptr}};

// ---- IOFuture ------------------------------------------------------------------
// A minimal asyncio-compatible future for the I/O clients' replies (store/pgwire.py,
// sinks/h1.py). It implements the subset of the asyncio.Future API that Task, gather and
// wait_for use: _asyncio_future_blocking, get_loop, done/cancelled/result/exception,
// add/remove_done_callback(context=), cancel, _make_cancelled_error, and __await__.
// The point is resolve()/reject(). When a protocol callback (data_received) completes a
// reply, a Driver waiting on it is resumed right there. asyncio would instead pay a
// call_soon, a Handle and a trip through the event loop per reply. Every other
// callback (a Task, gather, wait_for) is still scheduled with loop.call_soon, as
// asyncio does. set_result/set_exception/cancel always schedule.
struct IOFutureObject {
  PyObject_HEAD PyObject* loop;
  PyObject* result;
  PyObject* exc;
  PyObject* cancel_msg;
  PyObject* cb0;    // first callback (common case: exactly one)
  PyObject* ctx0;   // its context or NULL
  PyObject* more;   // list of (fn, ctx) for further callbacks, or NULL
  uint8_t state;    // 0 pending, 1 finished, 2 cancelled
  uint8_t blocking;
};

PyTypeObject IOFutureType = {PyVarObject_HEAD_INIT(nullptr, 0)};
PyObject* g_invalid_state = nullptr;  // asyncio.InvalidStateError
PyObject* s_call_exception_handler = nullptr;

int iof_traverse(IOFutureObject* f, visitproc visit, void* arg) {
  Py_VISIT(f->loop);
  Py_VISIT(f->result);
  Py_VISIT(f->exc);
  Py_VISIT(f->cancel_msg);
  Py_VISIT(f->cb0);
  Py_VISIT(f->ctx0);
  Py_VISIT(f->more);
  return 0;
}

int iof_clear(IOFutureObject* f) {
  Py_CLEAR(f->loop);
  Py_CLEAR(f->result);
  Py_CLEAR(f->exc);
  Py_CLEAR(f->cancel_msg);
  Py_CLEAR(f->cb0);
  Py_CLEAR(f->ctx0);
  Py_CLEAR(f->more);
  return 0;
}

void iof_dealloc(IOFutureObject* f) {
  PyObject_GC_UnTrack(f);
  iof_clear(f);
  Py_TYPE(f)->tp_free(reinterpret_cast<PyObject*>(f));
}

PyObject* iof_new(PyTypeObject* type, PyObject* args, PyObject* kwds) {
  static const char* kwlist[] = {"loop", nullptr};
  PyObject* loop = nullptr;
  if (!PyArg_ParseTupleAndKeywords(args, kwds, "|O", const_cast<char**>(kwlist), &loop)) return nullptr;
  IOFutureObject* f = reinterpret_cast<IOFutureObject*>(type->tp_alloc(type, 0));
  if (!f) return nullptr;
  f->result = f->exc = f->cancel_msg = f->cb0 = f->ctx0 = f->more = nullptr;
  f->state = 0;
  f->blocking = 0;
  if (!loop || loop == Py_None) {
    f->loop = PyObject_CallNoArgs(g_get_running_loop);
    if (!f->loop) {
      Py_DECREF(f);
      return nullptr;
    }
  } else {
    Py_INCREF(loop);
    f->loop = loop;
  }
  return reinterpret_cast<PyObject*>(f);
}

PyObject* make_cancelled(IOFutureObject* f) {
  if (f->cancel_msg) return PyObject_CallOneArg(g_cancelled_error, f->cancel_msg);
  return PyObject_CallNoArgs(g_cancelled_error);
}

// Schedules fn(self) with loop.call_soon(fn, self, context=ctx).
int schedule_cb(IOFutureObject* f, PyObject* fn, PyObject* ctx) {
  PyObject* call_soon = PyObject_GetAttr(f->loop, s_call_soon);
  if (!call_soon) return -1;
  PyObject* args = PyTuple_Pack(2, fn, reinterpret_cast<PyObject*>(f));
  if (!args) {
    Py_DECREF(call_soon);
    return -1;
  }
  PyObject* kw = nullptr;
  if (ctx) {
    kw = PyDict_New();
    if (!kw || PyDict_SetItemString(kw, "context", ctx) < 0) {
      Py_XDECREF(kw);
      Py_DECREF(args);
      Py_DECREF(call_soon);
      return -1;
    }
  }
  PyObject* h = PyObject_Call(call_soon, args, kw);
  Py_XDECREF(kw);
  Py_DECREF(args);
  Py_DECREF(call_soon);
  if (!h) return -1;
  Py_DECREF(h);
  return 0;
}

// Runs fn(self) now (Driver callbacks on the synchronous path). Exception subclasses go to
// the loop's exception handler, as asyncio does for callbacks; anything else propagates.
int call_now(IOFutureObject* f, PyObject* fn) {
  PyObject* r = PyObject_CallOneArg(fn, reinterpret_cast<PyObject*>(f));
  if (r) {
    Py_DECREF(r);
    return 0;
  }
  if (!PyErr_ExceptionMatches(PyExc_Exception)) return -1;
  PyObject* e = fetch_exc();
  PyObject* ctx = Py_BuildValue("{s:s,s:O,s:O}", "message", "Exception in IOFuture done callback", "exception",
                                e ? e : Py_None, "future", reinterpret_cast<PyObject*>(f));
  Py_XDECREF(e);
  if (!ctx) return -1;
  PyObject* h = PyObject_CallMethodOneArg(f->loop, s_call_exception_handler, ctx);
  Py_DECREF(ctx);
  if (!h) return -1;
  Py_DECREF(h);
  return 0;
}

// Fires the callbacks after a state change. sync: Driver callbacks run immediately.
int fire(IOFutureObject* f, bool sync) {
  PyObject* fn = f->cb0;
  PyObject* ctx = f->ctx0;
  PyObject* more = f->more;
  f->cb0 = f->ctx0 = f->more = nullptr;
  int rc = 0;
  if (fn) {
    if (sync && Py_TYPE(fn) == &DriverType)
      rc = call_now(f, fn);
    else
      rc = schedule_cb(f, fn, ctx);
    Py_DECREF(fn);
    Py_XDECREF(ctx);
  }
  if (more) {
    Py_ssize_t n = PyList_GET_SIZE(more);
    for (Py_ssize_t i = 0; i < n && rc == 0; ++i) {
      PyObject* pair = PyList_GET_ITEM(more, i);
      PyObject* fn2 = PyTuple_GET_ITEM(pair, 0);
      PyObject* ctx2 = PyTuple_GET_ITEM(pair, 1);
      if (sync && Py_TYPE(fn2) == &DriverType)
        rc = call_now(f, fn2);
      else
        rc = schedule_cb(f, fn2, ctx2 == Py_None ? nullptr : ctx2);
    }
    Py_DECREF(more);
  }
  return rc;
}

PyObject* invalid_state(const char* msg) {
  PyErr_SetString(g_invalid_state, msg);
  return nullptr;
}

PyObject* iof_finish_result(IOFutureObject* f, PyObject* v, bool sync) {
  if (f->state) return invalid_state("invalid state");
  Py_INCREF(v);
  f->result = v;
  f->state = 1;
  if (fire(f, sync) < 0) return nullptr;
  Py_RETURN_NONE;
}

PyObject* iof_finish_exc(IOFutureObject* f, PyObject* e, bool sync) {
  if (f->state) return invalid_state("invalid state");
  PyObject* inst = e;
  if (PyType_Check(e)) {
    inst = PyObject_CallNoArgs(e);
    if (!inst) return nullptr;
  } else {
    Py_INCREF(inst);
  }
  if (!PyExceptionInstance_Check(inst)) {
    Py_DECREF(inst);
    PyErr_SetString(PyExc_TypeError, "invalid exception object");
    return nullptr;
  }
  if (PyErr_GivenExceptionMatches(inst, PyExc_StopIteration)) {
    Py_DECREF(inst);
    PyErr_SetString(PyExc_TypeError, "StopIteration interacts badly with generators and cannot be raised into a Future");
    return nullptr;
  }
  f->exc = inst;
  f->state = 1;
  if (fire(f, sync) < 0) return nullptr;
  Py_RETURN_NONE;
}

PyObject* iof_set_result(IOFutureObject* f, PyObject* v) { return iof_finish_result(f, v, false); }
PyObject* iof_resolve(IOFutureObject* f, PyObject* v) { return iof_finish_result(f, v, true); }
PyObject* iof_set_exception(IOFutureObject* f, PyObject* e) { return iof_finish_exc(f, e, false); }
PyObject* iof_reject(IOFutureObject* f, PyObject* e) { return iof_finish_exc(f, e, true); }

PyObject* iof_cancel(IOFutureObject* f, PyObject* args, PyObject* kwds) {
  static const char* kwlist[] = {"msg", nullptr};
  PyObject* msg = Py_None;
  if (!PyArg_ParseTupleAndKeywords(args, kwds, "|O", const_cast<char**>(kwlist), &msg)) return nullptr;
  if (f->state) Py_RETURN_FALSE;
  f->state = 2;
  if (msg != Py_None) {
    Py_INCREF(msg);
    f->cancel_msg = msg;
  }
  if (fire(f, false) < 0) return nullptr;
  Py_RETURN_TRUE;
}

PyObject* iof_result(IOFutureObject* f, PyObject*) {
  if (f->state == 2) {
    PyObject* e = make_cancelled(f);
    if (!e) return nullptr;
    PyErr_SetObject(g_cancelled_error, e);
    Py_DECREF(e);
    return nullptr;
  }
  if (!f->state) return invalid_state("Result is not ready.");
  if (f->exc) {
    PyErr_SetObject(reinterpret_cast<PyObject*>(Py_TYPE(f->exc)), f->exc);
    return nullptr;
  }
  Py_INCREF(f->result);
  return f->result;
}

PyObject* iof_exception(IOFutureObject* f, PyObject*) {
  if (f->state == 2) {
    PyObject* e = make_cancelled(f);
    if (!e) return nullptr;
    PyErr_SetObject(g_cancelled_error, e);
    Py_DECREF(e);
    return nullptr;
  }
  if (!f->state) return invalid_state("Exception is not set.");
  PyObject* e = f->exc ? f->exc : Py_None;
  Py_INCREF(e);
  return e;
}

PyObject* iof_add_done_callback(IOFutureObject* f, PyObject* args, PyObject* kwds) {
  static const char* kwlist[] = {"fn", "context", nullptr};
  PyObject *fn, *ctx = Py_None;
  if (!PyArg_ParseTupleAndKeywords(args, kwds, "O|$O", const_cast<char**>(kwlist), &fn, &ctx)) return nullptr;
  PyObject* c = ctx == Py_None ? nullptr : ctx;
  if (f->state) {
    if (schedule_cb(f, fn, c) < 0) return nullptr;
    Py_RETURN_NONE;
  }
  if (!f->cb0) {
    Py_INCREF(fn);
    f->cb0 = fn;
    Py_XINCREF(c);
    f->ctx0 = c;
    Py_RETURN_NONE;
  }
  if (!f->more && !(f->more = PyList_New(0))) return nullptr;
  PyObject* pair = PyTuple_Pack(2, fn, c ? c : Py_None);
  if (!pair) return nullptr;
  int rc = PyList_Append(f->more, pair);
  Py_DECREF(pair);
  if (rc < 0) return nullptr;
  Py_RETURN_NONE;
}

PyObject* iof_remove_done_callback(IOFutureObject* f, PyObject* fn) {
  Py_ssize_t removed = 0;
  if (f->cb0) {
    int eq = PyObject_RichCompareBool(f->cb0, fn, Py_EQ);
    if (eq < 0) return nullptr;
    if (eq) {
      Py_CLEAR(f->cb0);
      Py_CLEAR(f->ctx0);
      ++removed;
    }
  }
  if (f->more) {
    PyObject* keep = PyList_New(0);
    if (!keep) return nullptr;
    for (Py_ssize_t i = 0; i < PyList_GET_SIZE(f->more); ++i) {
      PyObject* pair = PyList_GET_ITEM(f->more, i);
      int eq = PyObject_RichCompareBool(PyTuple_GET_ITEM(pair, 0), fn, Py_EQ);
      if (eq < 0) {
        Py_DECREF(keep);
        return nullptr;
      }
      if (eq) {
        ++removed;
      } else if (PyList_Append(keep, pair) < 0) {
        Py_DECREF(keep);
        return nullptr;
      }
    }
    Py_SETREF(f->more, keep);
  }
  return PyLong_FromSsize_t(removed);
}

PyObject* iof_done(IOFutureObject* f, PyObject*) { return PyBool_FromLong(f->state != 0); }
PyObject* iof_cancelled(IOFutureObject* f, PyObject*) { return PyBool_FromLong(f->state == 2); }
PyObject* iof_get_loop(IOFutureObject* f, PyObject*) {
  Py_INCREF(f->loop);
  return f->loop;
}
PyObject* iof_make_cancelled_error(IOFutureObject* f, PyObject*) { return make_cancelled(f); }

PyObject* iof_get_blocking(IOFutureObject* f, void*) { return PyBool_FromLong(f->blocking); }
int iof_set_blocking(IOFutureObject* f, PyObject* v, void*) {
  if (!v) {
    PyErr_SetString(PyExc_AttributeError, "cannot delete _asyncio_future_blocking");
    return -1;
  }
  int b = PyObject_IsTrue(v);
  if (b < 0) return -1;
  f->blocking = uint8_t(b);
  return 0;
}
PyObject* iof_get_log_tb(IOFutureObject*, void*) { Py_RETURN_FALSE; }
int iof_set_log_tb(IOFutureObject*, PyObject*, void*) { return 0; }

// await protocol: the future is its own iterator (one awaiter at a time, as in our clients)
PyObject* iof_await(IOFutureObject* f) {
  Py_INCREF(f);
  return reinterpret_cast<PyObject*>(f);
}

PySendResult iof_am_send(IOFutureObject* f, PyObject*, PyObject** out) {
  if (!f->state) {
    f->blocking = 1;
    Py_INCREF(f);
    *out = reinterpret_cast<PyObject*>(f);
    return PYGEN_NEXT;
  }
  PyObject* r = iof_result(f, nullptr);
  if (!r) {
    *out = nullptr;
    return PYGEN_ERROR;
  }
  *out = r;
  return PYGEN_RETURN;
}

PyObject* iof_iternext(IOFutureObject* f) {
  PyObject* out;
  PySendResult r = iof_am_send(f, Py_None, &out);
  if (r == PYGEN_NEXT) return out;
  if (r == PYGEN_ERROR) return nullptr;
  // return value -> StopIteration(value)
  if (out == Py_None) {
    Py_DECREF(out);
    PyErr_SetNone(PyExc_StopIteration);
  } else {
    PyObject* e = PyObject_CallOneArg(PyExc_StopIteration, out);
    Py_DECREF(out);
    if (!e) return nullptr;
    PyErr_SetObject(PyExc_StopIteration, e);
    Py_DECREF(e);
  }
  return nullptr;
}

PyObject* iof_send(IOFutureObject* f, PyObject*) { return iof_iternext(f); }

PyObject* iof_throw(IOFutureObject*, PyObject* args) {
  PyObject *t, *v = nullptr, *tb = nullptr;
  if (!PyArg_ParseTuple(args, "O|OO", &t, &v, &tb)) return nullptr;
  if (PyExceptionInstance_Check(t))
    PyErr_SetObject(reinterpret_cast<PyObject*>(Py_TYPE(t)), t);
  else
    PyErr_SetObject(t, v ? v : Py_None);
  return nullptr;
}

PyAsyncMethods iof_async = {reinterpret_cast<unaryfunc>(iof_await), nullptr, nullptr,
                            reinterpret_cast<sendfunc>(iof_am_send)};

PyMethodDef iof_methods[] = {
    {"get_loop", reinterpret_cast<PyCFunction>(iof_get_loop), METH_NOARGS, nullptr},
    {"done", reinterpret_cast<PyCFunction>(iof_done), METH_NOARGS, nullptr},
    {"cancelled", reinterpret_cast<PyCFunction>(iof_cancelled), METH_NOARGS, nullptr},
    {"result", reinterpret_cast<PyCFunction>(iof_result), METH_NOARGS, nullptr},
    {"exception", reinterpret_cast<PyCFunction>(iof_exception), METH_NOARGS, nullptr},
    {"add_done_callback", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(iof_add_done_callback)),
     METH_VARARGS | METH_KEYWORDS, nullptr},
    {"remove_done_callback", reinterpret_cast<PyCFunction>(iof_remove_done_callback), METH_O, nullptr},
    {"cancel", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(iof_cancel)),
     METH_VARARGS | METH_KEYWORDS, nullptr},
    {"set_result", reinterpret_cast<PyCFunction>(iof_set_result), METH_O, "set_result(v): callbacks via call_soon"},
    {"set_exception", reinterpret_cast<PyCFunction>(iof_set_exception), METH_O, nullptr},
    {"resolve", reinterpret_cast<PyCFunction>(iof_resolve), METH_O,
     "resolve(v): like set_result, but a waiting Driver resumes immediately (protocol callbacks only)"},
    {"reject", reinterpret_cast<PyCFunction>(iof_reject), METH_O,
     "reject(exc): like set_exception, but a waiting Driver resumes immediately"},
    {"_make_cancelled_error", reinterpret_cast<PyCFunction>(iof_make_cancelled_error), METH_NOARGS, nullptr},
    {"send", reinterpret_cast<PyCFunction>(iof_send), METH_O, nullptr},
    {"throw", reinterpret_cast<PyCFunction>(iof_throw), METH_VARARGS, nullptr},
    {nullptr, nullptr, 0, nullptr}};

PyGetSetDef iof_getset[] = {
    {"_asyncio_future_blocking", reinterpret_cast<getter>(iof_get_blocking),
     reinterpret_cast<setter>(iof_set_blocking), nullptr, nullptr},
    {"_log_traceback", reinterpret_cast<getter>(iof_get_log_tb), reinterpret_cast<setter>(iof_set_log_tb), nullptr,
     nullptr},
    {nullptr, nullptr, nullptr, nullptr, nullptr}};

// ---- Window methods ------------------------------------------------------------
PyObject* window_new(PyTypeObject* type, PyObject* args, PyObject* kwds) {
  static const char* kwlist[] = {"limit", "on_error", "on_wake", nullptr};
  Py_ssize_t limit;
  PyObject* on_error = Py_None;
  PyObject* on_wake = Py_None;
  if (!PyArg_ParseTupleAndKeywords(args, kwds, "n|OO", const_cast<char**>(kwlist), &limit, &on_error, &on_wake))
    return nullptr;
  if (limit < 1) {
    PyErr_SetString(PyExc_ValueError, "limit must be >= 1");
    return nullptr;
  }
  WindowObject* w = reinterpret_cast<WindowObject*>(type->tp_alloc(type, 0));
  if (!w) return nullptr;
  w->drivers = PySet_New(nullptr);
  if (!w->drivers) {
    Py_DECREF(w);
    return nullptr;
  }
  Py_INCREF(on_error);
  w->on_error = on_error;
  Py_INCREF(on_wake);
  w->on_wake = on_wake;
  w->limit = limit;
  return reinterpret_cast<PyObject*>(w);
}

int window_traverse(WindowObject* w, visitproc visit, void* arg) {
  Py_VISIT(w->drivers);
  Py_VISIT(w->on_error);
  Py_VISIT(w->on_wake);
  return 0;
}

int window_clear(WindowObject* w) {
  Py_CLEAR(w->drivers);
  Py_CLEAR(w->on_error);
  Py_CLEAR(w->on_wake);
  return 0;
}

void window_dealloc(WindowObject* w) {
  PyObject_GC_UnTrack(w);
  window_clear(w);
  Py_TYPE(w)->tp_free(reinterpret_cast<PyObject*>(w));
}

Py_ssize_t window_len(WindowObject* w) { return w->drivers ? PySet_GET_SIZE(w->drivers) : 0; }

PyObject* window_iter(WindowObject* w) {
  PyObject* lst = PySequence_List(w->drivers);  // a snapshot: drivers may finish while iterating
  if (!lst) return nullptr;
  PyObject* it = PyObject_GetIter(lst);
  Py_DECREF(lst);
  return it;
}

// suspend(payload, coro, first_yield) -> bool: a Driver resumes `coro` (reporting here);
// True when the window is now full.
PyObject* window_suspend_impl(WindowObject* w, PyObject* payload, PyObject* coro, PyObject* first) {
  DriverObject* drv = reinterpret_cast<DriverObject*>(driver_new(&DriverType, nullptr, nullptr));
  if (!drv) return nullptr;
  Py_INCREF(coro);
  drv->coro = coro;
  Py_INCREF(reinterpret_cast<PyObject*>(w));
  drv->on_done = reinterpret_cast<PyObject*>(w);
  Py_INCREF(payload);
  drv->payload = payload;
  if (PySet_Add(w->drivers, reinterpret_cast<PyObject*>(drv)) < 0) {
    Py_DECREF(drv);
    return nullptr;
  }
  ++w->suspended;
  PyObject* r = driver_start(drv, first);
  if (!r) {
    PyObject *et, *ev, *tb;
    PyErr_Fetch(&et, &ev, &tb);
    PySet_Discard(w->drivers, reinterpret_cast<PyObject*>(drv));
    PyErr_Restore(et, ev, tb);
    Py_DECREF(drv);
    return nullptr;
  }
  Py_DECREF(r);
  Py_DECREF(drv);  // the set (and the awaited future's callback) keep it alive
  return PyBool_FromLong(PySet_GET_SIZE(w->drivers) >= w->limit);
}

PyObject* window_suspend(WindowObject* w, PyObject* const* a, Py_ssize_t n) {
  if (n != 3) {
    PyErr_SetString(PyExc_TypeError, "suspend(payload, coro, first_yield)");
    return nullptr;
  }
  return window_suspend_impl(w, a[0], a[1], a[2]);
}

// track(driver): a Driver created elsewhere (with its own on_done) counts against the window
PyObject* window_track(WindowObject* w, PyObject* drv) {
  if (Py_TYPE(drv) != &DriverType) {
    PyErr_SetString(PyExc_TypeError, "track() takes a Driver");
    return nullptr;
  }
  if (PySet_Add(w->drivers, drv) < 0) return nullptr;
  ++w->suspended;
  Py_RETURN_NONE;
}

// release(driver, exc=None): the tracked driver finished (its own on_done calls this)
PyObject* window_release(WindowObject* w, PyObject* const* a, Py_ssize_t n) {
  if (n < 1 || n > 2 || Py_TYPE(a[0]) != &DriverType) {
    PyErr_SetString(PyExc_TypeError, "release(driver, exc=None)");
    return nullptr;
  }
  if (window_done(w, reinterpret_cast<DriverObject*>(a[0]), n == 2 ? a[1] : nullptr) < 0) return nullptr;
  Py_RETURN_NONE;
}

PyObject* window_stats(WindowObject* w, PyObject*) {
  return Py_BuildValue("{s:n,s:n,s:K,s:K}", "inflight", window_len(w), "limit", w->limit, "suspended",
                       static_cast<unsigned long long>(w->suspended), "wakes",
                       static_cast<unsigned long long>(w->wakes));
}

PyObject* window_get_limit(WindowObject* w, void*) { return PyLong_FromSsize_t(w->limit); }

PyMethodDef window_methods[] = {
    {"suspend", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(window_suspend)), METH_FASTCALL,
     "suspend(payload, coro, first_yield) -> bool: resume coro with a Driver; True = window full"},
    {"track", reinterpret_cast<PyCFunction>(window_track), METH_O, "track(driver)"},
    {"release", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(window_release)), METH_FASTCALL,
     "release(driver, exc=None)"},
    {"stats", reinterpret_cast<PyCFunction>(window_stats), METH_NOARGS, "counters"},
    {nullptr, nullptr, 0, nullptr}};

PyGetSetDef window_getset[] = {{"limit", reinterpret_cast<getter>(window_get_limit), nullptr, "capacity", nullptr},
                               {nullptr, nullptr, nullptr, nullptr, nullptr}};

PySequenceMethods window_seq = {};

}  // namespace

bool is_window(PyObject* o) { return Py_TYPE(o) == &WindowType; }

PyObject* window_suspend_c(PyObject* w, PyObject* payload, PyObject* coro, PyObject* first) {
  return window_suspend_impl(reinterpret_cast<WindowObject*>(w), payload, coro, first);
}

int init_driver_types(PyObject* m) {
  PyObject* aio = PyImport_ImportModule("asyncio");
  if (!aio) return -1;
  g_cancelled_error = PyObject_GetAttrString(aio, "CancelledError");
  g_get_running_loop = PyObject_GetAttrString(aio, "get_running_loop");
  Py_DECREF(aio);
  if (!g_cancelled_error || !g_get_running_loop) return -1;
  s_blocking = PyUnicode_InternFromString("_asyncio_future_blocking");
  s_add_done_callback = PyUnicode_InternFromString("add_done_callback");
  s_result = PyUnicode_InternFromString("result");
  s_throw = PyUnicode_InternFromString("throw");
  s_call_soon = PyUnicode_InternFromString("call_soon");
  s_cancel = PyUnicode_InternFromString("cancel");
  if (!s_blocking || !s_add_done_callback || !s_result || !s_throw || !s_call_soon || !s_cancel) return -1;

  DriverType.tp_name = "beholder_amd.ops._native.Driver";
  DriverType.tp_basicsize = sizeof(DriverObject);
  DriverType.tp_flags = Py_TPFLAGS_DEFAULT | Py_TPFLAGS_HAVE_GC;
  DriverType.tp_doc = "Driver(coro, on_done, payload=None): Task-free resumption of a suspended coroutine";
  DriverType.tp_new = driver_new;
  DriverType.tp_init = reinterpret_cast<initproc>(driver_init);
  DriverType.tp_dealloc = reinterpret_cast<destructor>(driver_dealloc);
  DriverType.tp_traverse = reinterpret_cast<traverseproc>(driver_traverse);
  DriverType.tp_clear = reinterpret_cast<inquiry>(driver_clear);
  DriverType.tp_call = reinterpret_cast<ternaryfunc>(driver_call);
  DriverType.tp_methods = driver_methods;
  DriverType.tp_getset = driver_getset;
  if (PyType_Ready(&DriverType) < 0) return -1;
  Py_INCREF(&DriverType);
  if (PyModule_AddObject(m, "Driver", reinterpret_cast<PyObject*>(&DriverType)) < 0) return -1;

  window_seq.sq_length = reinterpret_cast<lenfunc>(window_len);
  WindowType.tp_name = "beholder_amd.ops._native.Window";
  WindowType.tp_basicsize = sizeof(WindowObject);
  WindowType.tp_flags = Py_TPFLAGS_DEFAULT | Py_TPFLAGS_HAVE_GC;
  WindowType.tp_doc =
      "Window(limit, on_error=None, on_wake=None): handlers suspended on I/O (the prefetch window); "
      "Drivers started by suspend() report back in C";
  WindowType.tp_new = window_new;
  WindowType.tp_dealloc = reinterpret_cast<destructor>(window_dealloc);
  WindowType.tp_traverse = reinterpret_cast<traverseproc>(window_traverse);
  WindowType.tp_clear = reinterpret_cast<inquiry>(window_clear);
  WindowType.tp_as_sequence = &window_seq;
  WindowType.tp_iter = reinterpret_cast<getiterfunc>(window_iter);
  WindowType.tp_methods = window_methods;
  WindowType.tp_getset = window_getset;
  if (PyType_Ready(&WindowType) < 0) return -1;
  Py_INCREF(&WindowType);
  if (PyModule_AddObject(m, "Window", reinterpret_cast<PyObject*>(&WindowType)) < 0) return -1;

  PyObject* aio2 = PyImport_ImportModule("asyncio");
  if (!aio2) return -1;
  g_invalid_state = PyObject_GetAttrString(aio2, "InvalidStateError");
  Py_DECREF(aio2);
  if (!g_invalid_state) return -1;
  s_call_exception_handler = PyUnicode_InternFromString("call_exception_handler");
  if (!s_call_exception_handler) return -1;
  IOFutureType.tp_name = "beholder_amd.ops._native.IOFuture";
  IOFutureType.tp_basicsize = sizeof(IOFutureObject);
  IOFutureType.tp_flags = Py_TPFLAGS_DEFAULT | Py_TPFLAGS_HAVE_GC;
  IOFutureType.tp_doc = "IOFuture(loop=None): asyncio-compatible reply future with synchronous Driver wake-up";
  IOFutureType.tp_new = iof_new;
  IOFutureType.tp_dealloc = reinterpret_cast<destructor>(iof_dealloc);
  IOFutureType.tp_traverse = reinterpret_cast<traverseproc>(iof_traverse);
  IOFutureType.tp_clear = reinterpret_cast<inquiry>(iof_clear);
  IOFutureType.tp_as_async = &iof_async;
  IOFutureType.tp_iter = reinterpret_cast<getiterfunc>(iof_await);
  IOFutureType.tp_iternext = reinterpret_cast<iternextfunc>(iof_iternext);
  IOFutureType.tp_methods = iof_methods;
  IOFutureType.tp_getset = iof_getset;
  if (PyType_Ready(&IOFutureType) < 0) return -1;
  Py_INCREF(&IOFutureType);
  return PyModule_AddObject(m, "IOFuture", reinterpret_cast<PyObject*>(&IOFutureType));
}

// C-level IOFuture access for other translation units (py_netconn.cpp): reply futures created
// and completed without a Python-level call.
PyObject* iofuture_new(PyObject* loop) {
  PyObject* args = PyTuple_Pack(1, loop);
  if (!args) return nullptr;
  PyObject* f = iof_new(&IOFutureType, args, nullptr);
  Py_DECREF(args);
  return f;
}

PyObject* interned(PyObject** slot, const char* text) {
  if (!*slot) *slot = PyUnicode_InternFromString(text);
  return *slot;
}
PyObject *g_done_name, *g_set_result_name, *g_set_exception_name;
#define s_done_name interned(&g_done_name, "done")
#define s_set_result_name interned(&g_set_result_name, "set_result")
#define s_set_exception_name interned(&g_set_exception_name, "set_exception")

// The helpers below also accept a foreign future (an asyncio.Future, e.g. a caller's own reply
// waiter); it goes through its Python methods.
bool iofuture_done(PyObject* f) {
  if (Py_TYPE(f) == &IOFutureType) return reinterpret_cast<IOFutureObject*>(f)->state != 0;
  PyObject* r = PyObject_CallMethodNoArgs(f, s_done_name);
  int d = r ? PyObject_IsTrue(r) : -1;
  Py_XDECREF(r);
  if (d < 0) {
    PyErr_WriteUnraisable(f);
    return true;  // unusable: treat as finished (nothing is delivered to it)
  }
  return d != 0;
}

// 0 pending; 1 finished with a result (*result borrowed); 2 finished with an exception or cancelled
int iofuture_peek(PyObject* f, PyObject** result) {
  if (Py_TYPE(f) != &IOFutureType) return iofuture_done(f) ? 2 : 0;  // foreign: its owner reads it
  IOFutureObject* x = reinterpret_cast<IOFutureObject*>(f);
  if (!x->state) return 0;
  if (x->state == 2 || x->exc) return 2;
  *result = x->result;
  return 1;
}

// What an awaiter yields for a pending future: the future, with the asyncio blocking handshake set
PyObject* iofuture_yield(PyObject* f) {
  if (Py_TYPE(f) == &IOFutureType) {
    reinterpret_cast<IOFutureObject*>(f)->blocking = 1;
  } else if (PyObject_SetAttrString(f, "_asyncio_future_blocking", Py_True) < 0) {
    return nullptr;
  }
  Py_INCREF(f);
  return f;
}

// resolve / reject unless already finished: 0 ok (or already done), -1 error
int iofuture_resolve(PyObject* f, PyObject* v) {
  if (iofuture_done(f)) return 0;
  PyObject* r = Py_TYPE(f) == &IOFutureType ? iof_finish_result(reinterpret_cast<IOFutureObject*>(f), v, true)
                                            : PyObject_CallMethodOneArg(f, s_set_result_name, v);
  if (!r) return -1;
  Py_DECREF(r);
  return 0;
}

int iofuture_reject(PyObject* f, PyObject* exc) {
  if (iofuture_done(f)) return 0;
  PyObject* r = Py_TYPE(f) == &IOFutureType ? iof_finish_exc(reinterpret_cast<IOFutureObject*>(f), exc, true)
                                            : PyObject_CallMethodOneArg(f, s_set_exception_name, exc);
  if (!r) return -1;
  Py_DECREF(r);
  return 0;
}


}  // namespace beholder
