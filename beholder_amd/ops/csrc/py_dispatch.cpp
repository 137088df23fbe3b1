// dispatch_batch: the service's per-delivery dispatch loop in C.
//
// For each Delivery of a batch (the `rmsg` of index.js:62,127): count it,
// stamp its handler start time, call the topic's async handler and drive the
// returned coroutine eagerly with PyIter_Send. A handler that completes
// without suspending (in-memory store, buffered sinks) costs no Task, no
// event-loop round trip and no StopIteration object. Only the rare paths call
// back into Python:
//   on_error(delivery, exc)            handler raised (quirk Q1 policy lives in Python)
//   on_suspend(delivery, coro, fut) -> bool
//                                      handler awaited real I/O: a Driver resumes the
//                                      started coroutine; returning True means
//                                      "prefetch window full, stop here". A native
//                                      Window (py_driver.cpp) does this in C.
//   on_unroutable(delivery)            no handler for the topic id
// Returns the index of the first delivery not dispatched (len(batch) when done).
#include "py_common.hpp"
#include "gil_clock.hpp"
#include "ring.hpp"

namespace beholder {

namespace {

// dispatch_batch(batch, start, routes, counts, on_error, on_suspend, on_unroutable) -> int
PyObject* mod_dispatch_batch(PyObject*, PyObject* const* a, Py_ssize_t n) {
  if (n != 7 || !PyList_Check(a[0]) || !PyTuple_Check(a[2])) {
    PyErr_SetString(PyExc_TypeError,
                    "dispatch_batch(batch: list, start: int, routes: tuple, counts, on_error, on_suspend, "
                    "on_unroutable)");
    return nullptr;
  }
  PyObject* batch = a[0];
  Py_ssize_t i = PyLong_AsSsize_t(a[1]);
  if (i == -1 && PyErr_Occurred()) return nullptr;
  PyObject* routes = a[2];
  const Py_ssize_t nroutes = PyTuple_GET_SIZE(routes);
  PyObject *on_error = a[4], *on_suspend = a[5], *on_unroutable = a[6];

  Py_buffer counts;
  if (PyObject_GetBuffer(a[3], &counts, PyBUF_WRITABLE | PyBUF_FORMAT) < 0) return nullptr;
  if (counts.itemsize != 8 || counts.len / 8 < nroutes) {
    PyBuffer_Release(&counts);
    PyErr_SetString(PyExc_TypeError, "counts must be a writable array('Q') with one slot per route");
    return nullptr;
  }
  uint64_t* cnt = static_cast<uint64_t*>(counts.buf);

  const Py_ssize_t len = PyList_GET_SIZE(batch);
  PyObject* ret = nullptr;
  for (; i < len; ++i) {
    PyObject* item = PyList_GET_ITEM(batch, i);
    if (Py_TYPE(item) != &DeliveryType) {
      PyErr_SetString(PyExc_TypeError, "batch items must be Delivery objects");
      goto done;
    }
    DeliveryObject* d = reinterpret_cast<DeliveryObject*>(item);
    Py_ssize_t tid = d->topic;
    PyObject* handler = tid < nroutes ? PyTuple_GET_ITEM(routes, tid) : Py_None;
    if (handler == Py_None) {
      PyObject* r = PyObject_CallOneArg(on_unroutable, item);
      if (!r) goto done;
      Py_DECREF(r);
      continue;
    }
    cnt[tid]++;
    d->start_ns = gil_mono_ns();
    PyObject* coro = PyObject_CallOneArg(handler, item);
    if (!coro) {  // the handler itself failed before producing a coroutine
      PyObject *et, *ev, *tb;
      PyErr_Fetch(&et, &ev, &tb);
      PyErr_NormalizeException(&et, &ev, &tb);
      if (tb) PyException_SetTraceback(ev, tb);
      PyObject* r = PyObject_CallFunctionObjArgs(on_error, item, ev, nullptr);
      Py_XDECREF(et);
      Py_XDECREF(ev);
      Py_XDECREF(tb);
      if (!r) goto done;
      Py_DECREF(r);
      continue;
    }
    PyObject* result = nullptr;
    PySendResult sr = PyIter_Send(coro, Py_None, &result);
    if (sr == PYGEN_RETURN) {
      Py_XDECREF(result);
      Py_DECREF(coro);
      continue;
    }
    if (sr == PYGEN_ERROR) {
      Py_DECREF(coro);
      PyObject *et, *ev, *tb;
      PyErr_Fetch(&et, &ev, &tb);
      PyErr_NormalizeException(&et, &ev, &tb);
      if (tb) PyException_SetTraceback(ev, tb);
      if (et && PyErr_GivenExceptionMatches(et, PyExc_KeyboardInterrupt)) {
        PyErr_Restore(et, ev, tb);  // never swallow Ctrl-C / SystemExit
        goto done;
      }
      PyObject* r = PyObject_CallFunctionObjArgs(on_error, item, ev ? ev : Py_None, nullptr);
      Py_XDECREF(et);
      Py_XDECREF(ev);
      Py_XDECREF(tb);
      if (!r) goto done;
      Py_DECREF(r);
      continue;
    }
    // PYGEN_NEXT: suspended on real I/O (a native Window takes it without a Python call)
    PyObject* r = is_window(on_suspend) ? window_suspend_c(on_suspend, item, coro, result)
                                        : PyObject_CallFunctionObjArgs(on_suspend, item, coro, result, nullptr);
    Py_DECREF(coro);
    Py_XDECREF(result);
    if (!r) goto done;
    int stop = PyObject_IsTrue(r);
    Py_DECREF(r);
    if (stop < 0) goto done;
    if (stop) {
      ++i;
      break;
    }
  }
  ret = PyLong_FromSsize_t(i);
done:
  PyBuffer_Release(&counts);
  return ret;
}

PyMethodDef dispatch_methods[] = {
    {"dispatch_batch", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(mod_dispatch_batch)),
     METH_FASTCALL,
     "dispatch_batch(batch, start, routes, counts, on_error, on_suspend, on_unroutable) -> next index"},
    {nullptr, nullptr, 0, nullptr}};

}  // namespace

int init_dispatch_functions(PyObject* m) { return PyModule_AddFunctions(m, dispatch_methods); }

}  // namespace beholder
