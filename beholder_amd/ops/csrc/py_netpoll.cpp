// NetPoller: one epoll set for all NetConns of an event loop.
//
// A NetConn registered with `loop.add_reader(fd, cb)` costs, per readiness, a selector event
// processed in Python (selectors.select, _process_events, a Handle on the ready queue) and a
// Handle._run -> Context.run trip before its C callback runs. On the production path
// (`tcp_e2e`: AMQP, Postgres and up to 100 sink connections) that is about one such trip per
// event. A NetPoller keeps the NetConn sockets in its own epoll set and registers only that
// epoll fd with the loop: when any of them is ready the loop makes ONE callback, `_run`, which
// takes every ready socket from epoll_wait(timeout=0) and dispatches it in C.
//
// The poller lives as `loop._beholder_netpoller` while it has sockets and is closed (epoll fd
// closed, reader removed, attribute dropped) when the last one leaves. Level-triggered: a
// socket with data left unread is reported again on the next loop iteration. (NetConns exist only
// with native I/O on: BEHOLDER_NATIVE_IO=0 keeps every socket on an asyncio transport.)
#include <sys/epoll.h>
#include <unistd.h>

#include <cstdlib>
#include <cstring>
#include <deque>
#include <memory>
#include <unordered_map>
#include <vector>

#include "hs_wake.hpp"
#include "py_common.hpp"

namespace beholder {

PyObject* netconn_dispatch(PyObject* conn, uint32_t events);
void netconn_flush(PyObject* conn);
void netconn_tls_done(void* job);

uint64_t g_netpoll_runs, g_netpoll_ready;  // _run callbacks and the ready sockets they took (io_counts)

namespace {

struct PollerObject {
  PyObject_HEAD int epfd;
  int running;    // nested _run depth: closing waits until it is 0
  PyObject* loop;
  PyObject* run_cb;                              // bound _run handed to loop.add_reader
  PyObject* flush_cb;                            // bound _flush (call_soon)
  std::unordered_map<int, PyObject*>* conns;     // fd -> NetConn (strong)
  std::vector<PyObject*>* to_flush;              // connections with queued queries (strong)
  std::vector<PyObject*>* deferred;              // callables run once at the end of this batch (strong)
  std::shared_ptr<HsWake>* wake;                 // TLS handshake completions (created on first use)
  bool flush_scheduled;
};

PyTypeObject PollerType = {PyVarObject_HEAD_INIT(nullptr, 0)};
PyObject *s_attr, *s_add_reader_p, *s_remove_reader_p, *s_call_soon_p;
bool g_enabled = true;

// Closes the epoll fd and leaves the loop (reader removed, attribute dropped). Errors are
// swallowed: this runs when the last socket leaves, possibly while the loop shuts down.
void drain_wake(PollerObject* p) {
  if (!p->wake || !*p->wake) return;
  std::deque<void*> jobs;
  (*p->wake)->take(jobs);
  for (void* j : jobs) netconn_tls_done(j);
}

void poller_close(PollerObject* p) {
  if (p->epfd < 0) return;
  PyObject *et, *ev, *tb;
  PyErr_Fetch(&et, &ev, &tb);
  if (p->wake && *p->wake) {  // finished handshakes of connections that have left: dropped
    std::deque<void*> jobs;
    (*p->wake)->close(jobs);
    for (void* j : jobs) netconn_tls_done(j);
  }
  if (p->loop) {
    PyObject* fdo = PyLong_FromLong(p->epfd);
    PyObject* r = fdo ? PyObject_CallMethodOneArg(p->loop, s_remove_reader_p, fdo) : nullptr;
    Py_XDECREF(r);
    Py_XDECREF(fdo);
    PyErr_Clear();
    PyObject* cur = PyObject_GetAttr(p->loop, s_attr);
    if (cur == reinterpret_cast<PyObject*>(p) && PyObject_DelAttr(p->loop, s_attr) < 0) PyErr_Clear();
    Py_XDECREF(cur);
    PyErr_Clear();
  }
  ::close(p->epfd);
  p->epfd = -1;
  // the channel's eventfd goes with the epoll set, not when the GC gets to this object (it sits
  // in a cycle with its bound _run / _flush); a handshake thread still holding it finds it
  // closed and frees its job itself
  if (p->wake) p->wake->reset();
  PyErr_Restore(et, ev, tb);
}

void flush_all(PollerObject* p) {
  if (!p->to_flush || p->to_flush->empty()) return;
  std::vector<PyObject*> tmp;
  tmp.swap(*p->to_flush);
  for (PyObject* c : tmp) {
    netconn_flush(c);
    Py_DECREF(c);
  }
}

// The callables deferred to the end of the batch (defer()): the AMQP ack flush, so the acks of the
// handlers a batch finished share one write with no extra trip through the loop.
void run_deferred(PollerObject* p) {
  while (p->deferred && !p->deferred->empty()) {
    std::vector<PyObject*> tmp;
    tmp.swap(*p->deferred);
    for (PyObject* cb : tmp) {
      PyObject* r = PyObject_CallNoArgs(cb);
      if (!r)
        PyErr_WriteUnraisable(cb);
      else
        Py_DECREF(r);
      Py_DECREF(cb);
    }
  }
}

// End of a batch (the outermost _run or _enter/_exit scope): queued queries go out, deferred
// callables run, and an empty poller leaves the loop.
void end_batch(PollerObject* p) {
  flush_all(p);
  run_deferred(p);
  if (!p->running && p->conns && p->conns->empty()) poller_close(p);
}

void drop_all(PollerObject* p) {
  if (p->deferred) {
    std::vector<PyObject*> tmp;
    tmp.swap(*p->deferred);
    for (PyObject* c : tmp) Py_DECREF(c);
  }
  if (p->to_flush) {
    std::vector<PyObject*> tmp;
    tmp.swap(*p->to_flush);
    for (PyObject* c : tmp) Py_DECREF(c);
  }
  if (!p->conns) return;
  std::unordered_map<int, PyObject*> tmp;
  tmp.swap(*p->conns);  // decrefs below may re-enter netpoll_del
  for (auto& kv : tmp) Py_DECREF(kv.second);
}

int poller_traverse(PollerObject* p, visitproc visit, void* arg) {
  Py_VISIT(p->loop);
  Py_VISIT(p->run_cb);
  Py_VISIT(p->flush_cb);
  if (p->to_flush)
    for (PyObject* c : *p->to_flush) Py_VISIT(c);
  if (p->deferred)
    for (PyObject* c : *p->deferred) Py_VISIT(c);
  if (p->conns)
    for (auto& kv : *p->conns) Py_VISIT(kv.second);
  return 0;
}

int poller_clear(PollerObject* p) {
  drop_all(p);
  Py_CLEAR(p->run_cb);
  Py_CLEAR(p->flush_cb);
  Py_CLEAR(p->loop);
  return 0;
}

void poller_dealloc(PollerObject* p) {
  PyObject_GC_UnTrack(p);
  drop_all(p);
  if (p->wake && *p->wake) {  // never closed (collected with its loop): same as poller_close
    std::deque<void*> jobs;
    (*p->wake)->close(jobs);
    for (void* j : jobs) netconn_tls_done(j);
  }
  if (p->epfd >= 0) {
    ::close(p->epfd);
    p->epfd = -1;
  }
  Py_CLEAR(p->run_cb);
  Py_CLEAR(p->flush_cb);
  Py_CLEAR(p->loop);
  delete p->conns;
  delete p->to_flush;
  delete p->deferred;
  delete p->wake;
  Py_TYPE(p)->tp_free(reinterpret_cast<PyObject*>(p));
}

// _run(): the loop's reader callback for the epoll fd
PyObject* poller_run(PollerObject* p, PyObject*) {
  if (p->epfd < 0) Py_RETURN_NONE;
  epoll_event evs[256];
  int n;
  do {
    n = epoll_wait(p->epfd, evs, 256, 0);
  } while (n < 0 && errno == EINTR);
  if (n < 0) return PyErr_SetFromErrno(PyExc_OSError);
  ++g_netpoll_runs;
  g_netpoll_ready += uint64_t(n);
  Py_INCREF(p);
  ++p->running;
  const int wfd = p->wake && *p->wake ? (*p->wake)->efd : -1;
  for (int i = 0; i < n && p->conns; ++i) {
    if (evs[i].data.fd == wfd) {  // handshake threads finished some handshakes
      drain_wake(p);
      continue;
    }
    auto it = p->conns->find(evs[i].data.fd);
    if (it == p->conns->end()) continue;  // left during this batch
    PyObject* c = it->second;
    Py_INCREF(c);
    PyObject* r = netconn_dispatch(c, evs[i].events);
    if (!r)
      PyErr_WriteUnraisable(c);  // a NetConn reports its own failures; this is a bug guard
    else
      Py_DECREF(r);
    Py_DECREF(c);
  }
  --p->running;
  if (!p->running) end_batch(p);  // queries the resumed handlers issued go out now, batched
  Py_DECREF(p);
  Py_RETURN_NONE;
}

// _enter() / _exit(): a batch scope for work that starts outside a _run, e.g. deliveries dispatched
// from the AMQP transport's read callback. Queries issued inside go out at _exit, together, and
// deferred callables run there, instead of one call_soon trip each.
PyObject* poller_enter(PollerObject* p, PyObject*) {
  ++p->running;
  Py_RETURN_NONE;
}

PyObject* poller_exit(PollerObject* p, PyObject*) {
  if (p->running <= 0) {
    PyErr_SetString(PyExc_RuntimeError, "NetPoller._exit without _enter");
    return nullptr;
  }
  Py_INCREF(p);
  if (--p->running == 0) end_batch(p);
  Py_DECREF(p);
  Py_RETURN_NONE;
}

// defer(cb) -> bool: inside a batch, run cb() once at its end and return True; outside one,
// return False (the caller schedules it itself).
PyObject* poller_defer(PollerObject* p, PyObject* cb) {
  if (!p->running || !p->deferred) Py_RETURN_FALSE;
  Py_INCREF(cb);
  p->deferred->push_back(cb);
  Py_RETURN_TRUE;
}

// _flush(): call_soon callback for queries queued outside a dispatch
PyObject* poller_flush(PollerObject* p, PyObject*) {
  p->flush_scheduled = false;
  Py_INCREF(p);
  flush_all(p);
  Py_DECREF(p);
  Py_RETURN_NONE;
}

PyMethodDef poller_methods[] = {
    {"_run", reinterpret_cast<PyCFunction>(poller_run), METH_NOARGS, "loop reader callback: dispatch ready sockets"},
    {"_flush", reinterpret_cast<PyCFunction>(poller_flush), METH_NOARGS, "send the queued Postgres queries"},
    {"_enter", reinterpret_cast<PyCFunction>(poller_enter), METH_NOARGS, "open a batch scope (see _exit)"},
    {"_exit", reinterpret_cast<PyCFunction>(poller_exit), METH_NOARGS,
     "close a batch scope: queued queries go out, deferred callables run"},
    {"defer", reinterpret_cast<PyCFunction>(poller_defer), METH_O,
     "defer(cb) -> bool: run cb() at the end of the batch in progress (False: no batch)"},
    {nullptr, nullptr, 0, nullptr}};

PyObject* poller_get_size(PollerObject* p, void*) { return PyLong_FromSize_t(p->conns ? p->conns->size() : 0); }
PyObject* poller_get_fd(PollerObject* p, void*) { return PyLong_FromLong(p->epfd); }

PyGetSetDef poller_getset[] = {
    {"size", reinterpret_cast<getter>(poller_get_size), nullptr, "registered sockets", nullptr},
    {"fd", reinterpret_cast<getter>(poller_get_fd), nullptr, "the epoll fd (-1 once closed)", nullptr},
    {nullptr, nullptr, nullptr, nullptr, nullptr}};

PyObject* mod_netpoll_enabled(PyObject*, PyObject*) { return PyBool_FromLong(g_enabled); }

PyMethodDef poll_functions[] = {
    {"netpoll_enabled", mod_netpoll_enabled, METH_NOARGS, "NetConns share one epoll set per loop (always true)"},
    {nullptr, nullptr, 0, nullptr}};

}  // namespace

// The loop's poller (new reference), created on first use; Py_None (new reference) when pollers
// are off or the loop cannot hold one; NULL with an exception on failure.
PyObject* netpoll_for(PyObject* loop) {
  if (!g_enabled) Py_RETURN_NONE;
  PyObject* cur = PyObject_GetAttr(loop, s_attr);
  if (cur) {
    if (Py_TYPE(cur) == &PollerType && reinterpret_cast<PollerObject*>(cur)->epfd >= 0) return cur;
    Py_DECREF(cur);
  } else {
    if (!PyErr_ExceptionMatches(PyExc_AttributeError)) return nullptr;
    PyErr_Clear();
  }
  PollerObject* p = PyObject_GC_New(PollerObject, &PollerType);
  if (!p) return nullptr;
  p->epfd = -1;
  p->running = 0;
  p->loop = nullptr;
  p->run_cb = nullptr;
  p->flush_cb = nullptr;
  p->flush_scheduled = false;
  p->wake = nullptr;
  p->conns = new (std::nothrow) std::unordered_map<int, PyObject*>();
  p->to_flush = new (std::nothrow) std::vector<PyObject*>();
  p->deferred = new (std::nothrow) std::vector<PyObject*>();
  PyObject_GC_Track(p);
  PyObject* po = reinterpret_cast<PyObject*>(p);
  if (!p->conns || !p->to_flush || !p->deferred) {
    Py_DECREF(po);
    return PyErr_NoMemory();
  }
  p->epfd = epoll_create1(EPOLL_CLOEXEC);
  if (p->epfd < 0) {
    Py_DECREF(po);
    return PyErr_SetFromErrno(PyExc_OSError);
  }
  Py_INCREF(loop);
  p->loop = loop;
  p->run_cb = PyObject_GetAttrString(po, "_run");
  p->flush_cb = p->run_cb ? PyObject_GetAttrString(po, "_flush") : nullptr;
  if (!p->flush_cb) {
    Py_DECREF(po);
    return nullptr;
  }
  if (PyObject_SetAttr(loop, s_attr, po) < 0) {  // a loop without a __dict__: per-socket readers
    PyErr_Clear();
    Py_DECREF(po);
    Py_RETURN_NONE;
  }
  PyObject* fdo = PyLong_FromLong(p->epfd);
  PyObject* r = fdo ? PyObject_CallMethodObjArgs(loop, s_add_reader_p, fdo, p->run_cb, nullptr) : nullptr;
  Py_XDECREF(fdo);
  if (!r) {
    PyObject *et, *ev, *tb;
    PyErr_Fetch(&et, &ev, &tb);
    if (PyObject_DelAttr(loop, s_attr) < 0) PyErr_Clear();
    PyErr_Restore(et, ev, tb);
    Py_DECREF(po);
    return nullptr;
  }
  Py_DECREF(r);
  return po;
}

// Watch `fd` for reading (and for writing when `write`), dispatching to `conn`. 0 or -1.
int netpoll_add(PyObject* po, int fd, PyObject* conn) {
  PollerObject* p = reinterpret_cast<PollerObject*>(po);
  if (p->epfd < 0 || !p->conns) {
    PyErr_SetString(PyExc_RuntimeError, "NetPoller is closed");
    return -1;
  }
  epoll_event ev;
  memset(&ev, 0, sizeof ev);
  ev.events = EPOLLIN | EPOLLRDHUP;
  ev.data.fd = fd;
  if (epoll_ctl(p->epfd, EPOLL_CTL_ADD, fd, &ev) < 0) {
    PyErr_SetFromErrno(PyExc_OSError);
    return -1;
  }
  Py_INCREF(conn);
  auto res = p->conns->emplace(fd, conn);
  if (!res.second) {  // a stale entry for a reused fd
    Py_DECREF(res.first->second);
    res.first->second = conn;
  }
  return 0;
}

int netpoll_set_write(PyObject* po, int fd, bool write) {
  PollerObject* p = reinterpret_cast<PollerObject*>(po);
  if (p->epfd < 0) return 0;
  epoll_event ev;
  memset(&ev, 0, sizeof ev);
  ev.events = EPOLLIN | EPOLLRDHUP | (write ? EPOLLOUT : 0u);
  ev.data.fd = fd;
  if (epoll_ctl(p->epfd, EPOLL_CTL_MOD, fd, &ev) < 0) {
    PyErr_SetFromErrno(PyExc_OSError);
    return -1;
  }
  return 0;
}

// The completion channel of this poller's loop (created and added to the epoll set on first
// use); empty when the poller is closed or the eventfd cannot be made.
std::shared_ptr<HsWake> netpoll_wake(PyObject* po) {
  PollerObject* p = reinterpret_cast<PollerObject*>(po);
  if (p->epfd < 0) return nullptr;
  if (p->wake && *p->wake) return *p->wake;
  try {
    auto w = std::make_shared<HsWake>();
    if (w->efd < 0) return nullptr;
    epoll_event ev;
    memset(&ev, 0, sizeof ev);
    ev.events = EPOLLIN;
    ev.data.fd = w->efd;
    if (epoll_ctl(p->epfd, EPOLL_CTL_ADD, w->efd, &ev) < 0) return nullptr;
    if (!p->wake) p->wake = new std::shared_ptr<HsWake>();
    *p->wake = w;
    return w;
  } catch (const std::exception&) {
    return nullptr;
  }
}

// Stop reporting readiness of `fd` while a handshake thread owns the socket; netpoll_set_write
// restores it. The fd stays in the set (its entry in `conns` too), but epoll reports EPOLLERR and
// EPOLLHUP whatever the mask says, and the set is level-triggered: a peer reset during the
// offload would wake this loop on every iteration until the handshake thread posts the job.
// EPOLLONESHOT disarms the fd after the first such report. 0 or -1.
int netpoll_pause(PyObject* po, int fd) {
  PollerObject* p = reinterpret_cast<PollerObject*>(po);
  if (p->epfd < 0) return 0;
  epoll_event ev;
  memset(&ev, 0, sizeof ev);
  ev.events = EPOLLONESHOT;
  ev.data.fd = fd;
  if (epoll_ctl(p->epfd, EPOLL_CTL_MOD, fd, &ev) < 0) {
    PyErr_SetFromErrno(PyExc_OSError);
    return -1;
  }
  return 0;
}

// `conn` queued queries (its flush_scheduled flag is set by the caller): flushed at the end of the
// dispatch in progress, else by one call_soon(_flush) shared by all connections. 0 or -1.
int netpoll_request_flush(PyObject* po, PyObject* conn) {
  PollerObject* p = reinterpret_cast<PollerObject*>(po);
  if (!p->to_flush) {
    PyErr_SetString(PyExc_RuntimeError, "NetPoller is closed");
    return -1;
  }
  if (!p->running && !p->flush_scheduled) {
    if (!p->loop) {
      PyErr_SetString(PyExc_RuntimeError, "NetPoller has no loop");
      return -1;
    }
    PyObject* h = PyObject_CallMethodOneArg(p->loop, s_call_soon_p, p->flush_cb);
    if (!h) return -1;
    Py_DECREF(h);
    p->flush_scheduled = true;
  }
  Py_INCREF(conn);
  p->to_flush->push_back(conn);
  return 0;
}

// Stop watching `fd` (before it is closed). Never fails; the poller closes once empty.
void netpoll_del(PyObject* po, int fd) {
  PollerObject* p = reinterpret_cast<PollerObject*>(po);
  if (p->epfd >= 0) epoll_ctl(p->epfd, EPOLL_CTL_DEL, fd, nullptr);
  if (!p->conns) return;
  auto it = p->conns->find(fd);
  if (it == p->conns->end()) return;
  PyObject* c = it->second;
  p->conns->erase(it);
  if (!p->running && p->conns->empty()) poller_close(p);
  Py_DECREF(c);
}

int init_netpoll_types(PyObject* m) {
  if (!(s_attr = PyUnicode_InternFromString("_beholder_netpoller")) ||
      !(s_add_reader_p = PyUnicode_InternFromString("add_reader")) ||
      !(s_remove_reader_p = PyUnicode_InternFromString("remove_reader")) ||
      !(s_call_soon_p = PyUnicode_InternFromString("call_soon")))
    return -1;
  PollerType.tp_name = "beholder_amd.ops._native.NetPoller";
  PollerType.tp_basicsize = sizeof(PollerObject);
  PollerType.tp_flags = Py_TPFLAGS_DEFAULT | Py_TPFLAGS_HAVE_GC;
  PollerType.tp_doc = "One epoll set for the NetConns of an event loop (see py_netpoll.cpp)";
  PollerType.tp_dealloc = reinterpret_cast<destructor>(poller_dealloc);
  PollerType.tp_traverse = reinterpret_cast<traverseproc>(poller_traverse);
  PollerType.tp_clear = reinterpret_cast<inquiry>(poller_clear);
  PollerType.tp_methods = poller_methods;
  PollerType.tp_getset = poller_getset;
  if (PyType_Ready(&PollerType) < 0) return -1;
  Py_INCREF(&PollerType);
  if (PyModule_AddObject(m, "NetPoller", reinterpret_cast<PyObject*>(&PollerType)) < 0) return -1;
  return PyModule_AddFunctions(m, poll_functions);
}

}  // namespace beholder
