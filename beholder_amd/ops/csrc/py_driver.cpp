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
  PyObject* r = PyObject_CallFunctionObjArgs(cb, reinterpret_cast<PyObject*>(s), exc ? exc : Py_None, nullptr);
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

}  // namespace

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
  return PyModule_AddObject(m, "Driver", reinterpret_cast<PyObject*>(&DriverType));
}

}  // namespace beholder
