// Native ingest runtime: Settler (ack accounting + latency histograms),
// Delivery (the `rmsg` handed to a handler, index.js:62,127) and Ingest (byte
// ring + GIL-free reader thread for framed stdin/pipe/file streams).
//
// Ack semantics reproduced from the reference:
//   * a delivery is settled at most once: ack() (index.js:71,124,151,154),
//     nack(requeue) or reject(); settling twice raises (amqplib would close
//     the channel with PRECONDITION_FAILED "unknown delivery tag");
//   * a delivery that is garbage-collected while still pending was never
//     acked — quirk Q1 (status handler threw). It is counted as `abandoned`
//     and reported to `on_abandon` so a source can dead-letter / redeliver it.
#include <poll.h>
#include <sys/eventfd.h>
#include <unistd.h>

#include <atomic>
#include <cerrno>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "py_common.hpp"
#include "gil_clock.hpp"
#include "ring.hpp"

namespace beholder {

// ================================ Settler ===================================
namespace {

PyObject* settler_new(PyTypeObject* type, PyObject*, PyObject*) {
  SettlerObject* self = reinterpret_cast<SettlerObject*>(type->tp_alloc(type, 0));
  if (!self) return nullptr;
  self->handle_hist = reinterpret_cast<HistogramObject*>(PyObject_CallNoArgs(reinterpret_cast<PyObject*>(&HistogramType)));
  self->ingest_hist = reinterpret_cast<HistogramObject*>(PyObject_CallNoArgs(reinterpret_cast<PyObject*>(&HistogramType)));
  self->queue_hist = reinterpret_cast<HistogramObject*>(PyObject_CallNoArgs(reinterpret_cast<PyObject*>(&HistogramType)));
  if (!self->handle_hist || !self->ingest_hist || !self->queue_hist) {
    Py_DECREF(self);
    return nullptr;
  }
  self->created = self->acked = self->nacked = self->rejected = self->abandoned = 0;
  self->on_settle = nullptr;
  self->batcher = nullptr;
  self->on_abandon = nullptr;
  self->slow_threshold_ns = 0;
  self->slow_cap = self->slow_dropped = 0;
  self->slow = nullptr;
  return reinterpret_cast<PyObject*>(self);
}

int settler_init(SettlerObject* self, PyObject* args, PyObject* kwds) {
  static const char* kwlist[] = {"on_settle", "on_abandon", nullptr};
  PyObject *on_settle = Py_None, *on_abandon = Py_None;
  if (!PyArg_ParseTupleAndKeywords(args, kwds, "|OO", const_cast<char**>(kwlist), &on_settle, &on_abandon))
    return -1;
  Py_CLEAR(self->on_settle);
  Py_CLEAR(self->on_abandon);
  if (on_settle != Py_None) {
    Py_INCREF(on_settle);
    self->on_settle = on_settle;
  }
  if (on_abandon != Py_None) {
    Py_INCREF(on_abandon);
    self->on_abandon = on_abandon;
  }
  return 0;
}

int settler_traverse(SettlerObject* self, visitproc visit, void* arg) {
  Py_VISIT(self->on_settle);
  Py_VISIT(self->on_abandon);
  Py_VISIT(self->batcher);
  return 0;
}

int settler_clear(SettlerObject* self) {
  Py_CLEAR(self->on_settle);
  Py_CLEAR(self->on_abandon);
  Py_CLEAR(self->batcher);
  return 0;
}

PyObject* settler_get_batcher(SettlerObject* self, void*) {
  PyObject* b = self->batcher ? self->batcher : Py_None;
  Py_INCREF(b);
  return b;
}

int settler_set_batcher(SettlerObject* self, PyObject* v, void*) {
  if (v == nullptr || v == Py_None) {
    Py_CLEAR(self->batcher);
    return 0;
  }
  if (!is_ack_batcher(v)) {
    PyErr_SetString(PyExc_TypeError, "ack_batcher must be an AckBatcher or None");
    return -1;
  }
  Py_INCREF(v);
  Py_XSETREF(self->batcher, v);
  return 0;
}

void settler_dealloc(SettlerObject* self) {
  PyObject_GC_UnTrack(self);
  settler_clear(self);
  Py_XDECREF(self->handle_hist);
  Py_XDECREF(self->ingest_hist);
  Py_XDECREF(self->queue_hist);
  delete static_cast<std::vector<int64_t>*>(self->slow);
  Py_TYPE(self)->tp_free(reinterpret_cast<PyObject*>(self));
}

PyObject* settler_stats(SettlerObject* self, PyObject*) {
  uint64_t settled = self->acked + self->nacked + self->rejected;
  uint64_t pending = self->created - settled - self->abandoned;
  return Py_BuildValue("{s:K,s:K,s:K,s:K,s:K,s:K}", "created", (unsigned long long)self->created, "acked",
                       (unsigned long long)self->acked, "nacked", (unsigned long long)self->nacked, "rejected",
                       (unsigned long long)self->rejected, "abandoned", (unsigned long long)self->abandoned,
                       "pending", (unsigned long long)pending);
}

PyObject* settler_reset_latency(SettlerObject* self, PyObject*) {
  self->handle_hist->h->reset();
  self->ingest_hist->h->reset();
  self->queue_hist->h->reset();
  Py_RETURN_NONE;
}

// trace_slow(threshold_ns, capacity=65536): start recording (recv, start, settle) of deliveries
// whose start->settle time is >= threshold_ns (0 stops and clears). slow_deliveries() returns
// them as a list of tuples and the count that did not fit.
PyObject* settler_trace_slow(SettlerObject* self, PyObject* args) {
  long long thr;
  unsigned long long cap = 65536;
  if (!PyArg_ParseTuple(args, "L|K", &thr, &cap)) return nullptr;
  if (cap > (1ULL << 28)) {  // 3 x 8 bytes each: at most 6 GiB, and cap * 3 cannot wrap
    PyErr_SetString(PyExc_ValueError, "trace_slow: capacity must be <= 2**28");
    return nullptr;
  }
  auto* v = static_cast<std::vector<int64_t>*>(self->slow);
  if (!v) {
    v = new (std::nothrow) std::vector<int64_t>();
    if (!v) return PyErr_NoMemory();
    self->slow = v;
  }
  self->slow_threshold_ns = 0;  // off while the buffer changes
  if (thr <= 0) cap = 0;         // stop: give the buffer back
  std::vector<int64_t>().swap(*v);
  try {
    v->reserve(size_t(cap) * 3);  // settle() appends without allocating (it must not throw)
  } catch (const std::exception&) {
    return PyErr_NoMemory();
  }
  self->slow_dropped = 0;
  self->slow_threshold_ns = thr > 0 ? thr : 0;
  self->slow_cap = cap;
  Py_RETURN_NONE;
}

PyObject* settler_slow_deliveries(SettlerObject* self, PyObject*) {
  auto* v = static_cast<std::vector<int64_t>*>(self->slow);
  size_t n = v ? v->size() / 3 : 0;
  PyObject* list = PyList_New(Py_ssize_t(n));
  if (!list) return nullptr;
  for (size_t i = 0; i < n; ++i) {
    PyObject* t = Py_BuildValue("(LLL)", (long long)(*v)[3 * i], (long long)(*v)[3 * i + 1], (long long)(*v)[3 * i + 2]);
    if (!t) {
      Py_DECREF(list);
      return nullptr;
    }
    PyList_SET_ITEM(list, Py_ssize_t(i), t);
  }
  return Py_BuildValue("(NK)", list, (unsigned long long)self->slow_dropped);
}

PyObject* settler_get_handle(SettlerObject* self, void*) {
  Py_INCREF(self->handle_hist);
  return reinterpret_cast<PyObject*>(self->handle_hist);
}
PyObject* settler_get_ingest(SettlerObject* self, void*) {
  Py_INCREF(self->ingest_hist);
  return reinterpret_cast<PyObject*>(self->ingest_hist);
}
PyObject* settler_get_queue(SettlerObject* self, void*) {
  Py_INCREF(self->queue_hist);
  return reinterpret_cast<PyObject*>(self->queue_hist);
}
#define SETTLER_U64(fld)                                                     \
  PyObject* settler_get_##fld(SettlerObject* self, void*) {                  \
    return PyLong_FromUnsignedLongLong((unsigned long long)self->fld);       \
  }
SETTLER_U64(created)
SETTLER_U64(acked)
SETTLER_U64(nacked)
SETTLER_U64(rejected)
SETTLER_U64(abandoned)
PyObject* settler_get_pending(SettlerObject* self, void*) {
  return PyLong_FromUnsignedLongLong(self->created - self->acked - self->nacked - self->rejected - self->abandoned);
}

PyMethodDef settler_methods[] = {
    {"stats", reinterpret_cast<PyCFunction>(settler_stats), METH_NOARGS, "settlement counters"},
    {"reset_latency", reinterpret_cast<PyCFunction>(settler_reset_latency), METH_NOARGS, "clear histograms"},
    {"trace_slow", reinterpret_cast<PyCFunction>(settler_trace_slow), METH_VARARGS,
     "trace_slow(threshold_ns, capacity=65536): record (recv, start, settle) of slow deliveries (0 = off)"},
    {"slow_deliveries", reinterpret_cast<PyCFunction>(settler_slow_deliveries), METH_NOARGS,
     "-> ([(recv_ns, start_ns, settle_ns), ...], dropped)"},
    {nullptr, nullptr, 0, nullptr}};

PyGetSetDef settler_getset[] = {
    {"handle_latency", reinterpret_cast<getter>(settler_get_handle), nullptr, "start()->settle ns", nullptr},
    {"ingest_latency", reinterpret_cast<getter>(settler_get_ingest), nullptr, "receive->settle ns", nullptr},
    {"queue_latency", reinterpret_cast<getter>(settler_get_queue), nullptr,
     "receive->start() ns (ring + event-loop wait; ingest = queue + handle)", nullptr},
    {"created", reinterpret_cast<getter>(settler_get_created), nullptr, nullptr, nullptr},
    {"acked", reinterpret_cast<getter>(settler_get_acked), nullptr, nullptr, nullptr},
    {"nacked", reinterpret_cast<getter>(settler_get_nacked), nullptr, nullptr, nullptr},
    {"rejected", reinterpret_cast<getter>(settler_get_rejected), nullptr, nullptr, nullptr},
    {"abandoned", reinterpret_cast<getter>(settler_get_abandoned), nullptr, nullptr, nullptr},
    {"pending", reinterpret_cast<getter>(settler_get_pending), nullptr, nullptr, nullptr},
    {"ack_batcher", reinterpret_cast<getter>(settler_get_batcher), reinterpret_cast<setter>(settler_set_batcher),
     "AckBatcher receiving acks of its channel's deliveries natively (None: every settle calls on_settle)",
     nullptr},
    {nullptr, nullptr, nullptr, nullptr, nullptr}};

}  // namespace

PyTypeObject SettlerType = {PyVarObject_HEAD_INIT(nullptr, 0)};

// ================================ Delivery ==================================
PyObject* delivery_new(PyObject* content, uint8_t topic, uint64_t tag, int64_t recv_ns, SettlerObject* settler,
                       bool redelivered) {
  DeliveryObject* d = PyObject_New(DeliveryObject, &DeliveryType);
  if (!d) return nullptr;
  Py_INCREF(content);
  d->content = content;
  d->settler = settler;
  Py_XINCREF(settler);
  d->extra = nullptr;
  d->headers = nullptr;
  d->tag = tag;
  d->recv_ns = recv_ns;
  d->start_ns = 0;
  d->topic = topic;
  d->state = D_PENDING;
  d->redelivered = redelivered ? 1 : 0;
  if (settler) settler->created++;
  return reinterpret_cast<PyObject*>(d);
}

namespace {

const char* state_name(uint8_t s) {
  switch (s) {
    case D_PENDING:
      return "pending";
    case D_ACKED:
      return "acked";
    case D_NACKED:
      return "nacked";
    case D_REJECTED:
      return "rejected";
  }
  return "?";
}

PyObject* delivery_py_new(PyTypeObject*, PyObject* args, PyObject* kwds) {
  static const char* kwlist[] = {"content", "topic_id", "tag", "settler", "recv_ns", "redelivered", "extra", nullptr};
  PyObject* content;
  int topic = 0;
  unsigned long long tag = 0;
  PyObject* settler = Py_None;
  PyObject* recv = Py_None;
  int redelivered = 0;
  PyObject* extra = Py_None;
  if (!PyArg_ParseTupleAndKeywords(args, kwds, "O|iKOOpO", const_cast<char**>(kwlist), &content, &topic, &tag,
                                   &settler, &recv, &redelivered, &extra))
    return nullptr;
  if (!PyBytes_Check(content)) {
    PyErr_SetString(PyExc_TypeError, "content must be bytes");
    return nullptr;
  }
  if (topic < 0 || topic > 255) {
    PyErr_SetString(PyExc_ValueError, "topic_id must be in [0, 255]");
    return nullptr;
  }
  if (settler != Py_None && !PyObject_TypeCheck(settler, &SettlerType)) {
    PyErr_SetString(PyExc_TypeError, "settler must be a Settler or None");
    return nullptr;
  }
  int64_t recv_ns;
  if (recv == Py_None) {
    recv_ns = gil_mono_ns();
  } else {
    recv_ns = PyLong_AsLongLong(recv);
    if (recv_ns == -1 && PyErr_Occurred()) return nullptr;
  }
  PyObject* d = delivery_new(content, uint8_t(topic), tag, recv_ns,
                             settler == Py_None ? nullptr : reinterpret_cast<SettlerObject*>(settler), redelivered);
  if (d && extra != Py_None) {
    Py_INCREF(extra);
    reinterpret_cast<DeliveryObject*>(d)->extra = extra;
  }
  return d;
}

void delivery_dealloc(DeliveryObject* self) {
  SettlerObject* s = self->settler;
  if (s && self->state == D_PENDING) {
    s->abandoned++;
    if (s->batcher && self->extra) ack_batcher_abandon(s->batcher, self->extra, self->tag);
    if (s->on_abandon) {
      PyObject *et, *ev, *tb;
      PyErr_Fetch(&et, &ev, &tb);
      PyObject* r = PyObject_CallFunction(s->on_abandon, "KiO", (unsigned long long)self->tag, int(self->topic),
                                          self->content);
      if (!r) {
        PyErr_WriteUnraisable(s->on_abandon);
      } else {
        Py_DECREF(r);
      }
      PyErr_Restore(et, ev, tb);
    }
  }
  Py_XDECREF(self->content);
  Py_XDECREF(self->extra);
  Py_XDECREF(self->headers);
  Py_XDECREF(s);
  PyObject_Del(self);
}

// Settle: record latency + counters, then the transport callback.
PyObject* settle(DeliveryObject* self, uint8_t to, const char* kind, bool requeue) {
  if (self->state != D_PENDING) {
    PyErr_Format(PyExc_RuntimeError, "delivery %llu already settled (%s)", (unsigned long long)self->tag,
                 state_name(self->state));
    return nullptr;
  }
  self->state = to;
  SettlerObject* s = self->settler;
  if (s) {
    int64_t now = gil_mono_ns();
    if (self->start_ns > 0) s->handle_hist->h->record(uint64_t(now > self->start_ns ? now - self->start_ns : 0));
    if (self->recv_ns > 0) s->ingest_hist->h->record(uint64_t(now > self->recv_ns ? now - self->recv_ns : 0));
    if (self->recv_ns > 0 && self->start_ns > 0)
      s->queue_hist->h->record(uint64_t(self->start_ns > self->recv_ns ? self->start_ns - self->recv_ns : 0));
    if (s->slow_threshold_ns > 0 && self->start_ns > 0 && now - self->start_ns >= s->slow_threshold_ns) {
      auto* v = static_cast<std::vector<int64_t>*>(s->slow);
      if (v->size() / 3 < s->slow_cap) {
        v->push_back(self->recv_ns);
        v->push_back(self->start_ns);
        v->push_back(now);
      } else {
        s->slow_dropped++;
      }
    }
    if (to == D_ACKED)
      s->acked++;
    else if (to == D_NACKED)
      s->nacked++;
    else
      s->rejected++;
    if (to == D_ACKED && s->batcher && self->extra) {
      int h = ack_batcher_ack(s->batcher, self->extra, self->tag);
      if (h < 0) return nullptr;
      if (h == 1) Py_RETURN_NONE;  // queued natively; the source flushes once per loop iteration
    }
    if (s->on_settle) {
      PyObject* r = PyObject_CallFunction(s->on_settle, "OsO", reinterpret_cast<PyObject*>(self), kind,
                                          requeue ? Py_True : Py_False);
      if (!r) return nullptr;
      Py_DECREF(r);
    }
  }
  Py_RETURN_NONE;
}

PyObject* delivery_ack(DeliveryObject* self, PyObject*) { return settle(self, D_ACKED, "ack", false); }

PyObject* delivery_nack(DeliveryObject* self, PyObject* args, PyObject* kwds) {
  static const char* kwlist[] = {"requeue", nullptr};
  int requeue = 1;
  if (!PyArg_ParseTupleAndKeywords(args, kwds, "|p", const_cast<char**>(kwlist), &requeue)) return nullptr;
  return settle(self, D_NACKED, "nack", requeue != 0);
}

PyObject* delivery_reject(DeliveryObject* self, PyObject* args, PyObject* kwds) {
  static const char* kwlist[] = {"requeue", nullptr};
  int requeue = 0;
  if (!PyArg_ParseTupleAndKeywords(args, kwds, "|p", const_cast<char**>(kwlist), &requeue)) return nullptr;
  return settle(self, D_REJECTED, "reject", requeue != 0);
}

PyObject* delivery_start(DeliveryObject* self, PyObject*) {
  self->start_ns = gil_mono_ns();
  Py_RETURN_NONE;
}

PyObject* delivery_get_content(DeliveryObject* self, void*) {
  Py_INCREF(self->content);
  return self->content;
}
PyObject* delivery_get_message(DeliveryObject* self, void*) {
  // `rmsg.message.content` (index.js:63,129): the message is the delivery itself.
  Py_INCREF(self);
  return reinterpret_cast<PyObject*>(self);
}
PyObject* delivery_get_topic(DeliveryObject* self, void*) {
  PyObject* t = g_state.topics;
  if (t && PyTuple_Check(t) && self->topic < PyTuple_GET_SIZE(t)) {
    PyObject* v = PyTuple_GET_ITEM(t, self->topic);
    Py_INCREF(v);
    return v;
  }
  Py_RETURN_NONE;
}
PyObject* delivery_get_topic_id(DeliveryObject* self, void*) { return PyLong_FromLong(self->topic); }
PyObject* delivery_get_tag(DeliveryObject* self, void*) { return PyLong_FromUnsignedLongLong(self->tag); }
PyObject* delivery_get_recv_ns(DeliveryObject* self, void*) { return PyLong_FromLongLong(self->recv_ns); }
PyObject* delivery_get_start_ns(DeliveryObject* self, void*) { return PyLong_FromLongLong(self->start_ns); }
PyObject* delivery_get_state(DeliveryObject* self, void*) { return PyUnicode_FromString(state_name(self->state)); }
PyObject* delivery_get_settled(DeliveryObject* self, void*) { return PyBool_FromLong(self->state != D_PENDING); }
PyObject* delivery_get_acked(DeliveryObject* self, void*) { return PyBool_FromLong(self->state == D_ACKED); }
PyObject* delivery_get_redelivered(DeliveryObject* self, void*) { return PyBool_FromLong(self->redelivered); }
PyObject* delivery_get_extra(DeliveryObject* self, void*) {
  PyObject* e = self->extra ? self->extra : Py_None;
  Py_INCREF(e);
  return e;
}
int delivery_set_extra(DeliveryObject* self, PyObject* v, void*) {
  PyObject* old = self->extra;
  if (v == nullptr || v == Py_None) {
    self->extra = nullptr;
  } else {
    Py_INCREF(v);
    self->extra = v;
  }
  Py_XDECREF(old);
  return 0;
}

PyObject* delivery_get_headers(DeliveryObject* self, void*) {
  PyObject* h = self->headers ? self->headers : Py_None;
  Py_INCREF(h);
  return h;
}
int delivery_set_headers(DeliveryObject* self, PyObject* v, void*) {
  PyObject* old = self->headers;
  if (v == nullptr || v == Py_None) {
    self->headers = nullptr;
  } else {
    Py_INCREF(v);
    self->headers = v;
  }
  Py_XDECREF(old);
  return 0;
}

PyObject* delivery_repr(DeliveryObject* self) {
  return PyUnicode_FromFormat("<Delivery tag=%llu topic=%d state=%s bytes=%zd>", (unsigned long long)self->tag,
                              int(self->topic), state_name(self->state), PyBytes_GET_SIZE(self->content));
}

PyMethodDef delivery_methods[] = {
    {"ack", reinterpret_cast<PyCFunction>(delivery_ack), METH_NOARGS, "acknowledge (settle once)"},
    {"nack", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(delivery_nack)),
     METH_VARARGS | METH_KEYWORDS, "negative-acknowledge; requeue=True"},
    {"reject", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(delivery_reject)),
     METH_VARARGS | METH_KEYWORDS, "reject; requeue=False"},
    {"start", reinterpret_cast<PyCFunction>(delivery_start), METH_NOARGS, "stamp handler start time"},
    {nullptr, nullptr, 0, nullptr}};

PyGetSetDef delivery_getset[] = {
    {"content", reinterpret_cast<getter>(delivery_get_content), nullptr, "message body (bytes)", nullptr},
    {"message", reinterpret_cast<getter>(delivery_get_message), nullptr, "self (rmsg.message.content parity)",
     nullptr},
    {"topic", reinterpret_cast<getter>(delivery_get_topic), nullptr, "topic name", nullptr},
    {"topic_id", reinterpret_cast<getter>(delivery_get_topic_id), nullptr, "topic id", nullptr},
    {"tag", reinterpret_cast<getter>(delivery_get_tag), nullptr, "delivery tag", nullptr},
    {"recv_ns", reinterpret_cast<getter>(delivery_get_recv_ns), nullptr, "receive time (CLOCK_MONOTONIC ns)",
     nullptr},
    {"start_ns", reinterpret_cast<getter>(delivery_get_start_ns), nullptr, "handler start time", nullptr},
    {"state", reinterpret_cast<getter>(delivery_get_state), nullptr, "pending|acked|nacked|rejected", nullptr},
    {"settled", reinterpret_cast<getter>(delivery_get_settled), nullptr, nullptr, nullptr},
    {"acked", reinterpret_cast<getter>(delivery_get_acked), nullptr, nullptr, nullptr},
    {"redelivered", reinterpret_cast<getter>(delivery_get_redelivered), nullptr, nullptr, nullptr},
    {"extra", reinterpret_cast<getter>(delivery_get_extra), reinterpret_cast<setter>(delivery_set_extra),
     "transport-specific data (must not reference the delivery)", nullptr},
    {"headers", reinterpret_cast<getter>(delivery_get_headers), reinterpret_cast<setter>(delivery_set_headers),
     "message headers: dict, raw AMQP field-table bytes (native demux), or None", nullptr},
    {nullptr, nullptr, nullptr, nullptr, nullptr}};

}  // namespace

PyTypeObject DeliveryType = {PyVarObject_HEAD_INIT(nullptr, 0)};

// rmsg.ack() for a native Delivery without the method lookup (the compiled handlers' last step).
PyObject* delivery_ack_c(PyObject* d) { return settle(reinterpret_cast<DeliveryObject*>(d), D_ACKED, "ack", false); }

// ================================= Ingest ===================================
namespace {

struct IngestObject {
  PyObject_HEAD ByteRing* ring;
  SettlerObject* settler;
  std::thread* reader;
  std::atomic<bool>* stop;
  std::atomic<uint64_t>* bytes_read;
  std::atomic<uint64_t>* frames_read;
  std::mutex* err_mu;
  std::string* error;
  Framer* py_framer;  // for feed() from Python
  uint32_t max_frame;
  int fd;
  int own_fd;
  int efd;  // eventfd the ring signals when the armed event loop may pop (-1 until notify_fd is read)
};

void set_error(IngestObject* self, const std::string& e) {
  std::lock_guard<std::mutex> g(*self->err_mu);
  if (self->error->empty()) *self->error = e;
}

void reader_loop(IngestObject* self, int fd, size_t chunk_bytes);

// Thread entry: an exception escaping a std::thread would terminate the process.
void reader_main(IngestObject* self, int fd, size_t chunk_bytes) {
  try {
    reader_loop(self, fd, chunk_bytes);
  } catch (const std::exception& e) {
    set_error(self, std::string("reader thread: ") + e.what());
    self->ring->set_eof();
  }
}

void reader_loop(IngestObject* self, int fd, size_t chunk_bytes) {
  std::vector<uint8_t> chunk(chunk_bytes);
  Framer framer(self->max_frame);
  struct pollfd pfd;
  pfd.fd = fd;
  pfd.events = POLLIN;
  bool ring_closed = false;
  while (!self->stop->load(std::memory_order_relaxed) && !ring_closed) {
    pfd.revents = 0;
    int pr = poll(&pfd, 1, 50);
    if (pr < 0) {
      if (errno == EINTR) continue;
      set_error(self, std::string("poll: ") + strerror(errno));
      break;
    }
    if (pr == 0) continue;
    ssize_t n = read(fd, chunk.data(), chunk.size());
    if (n < 0) {
      if (errno == EINTR || errno == EAGAIN) continue;
      set_error(self, std::string("read: ") + strerror(errno));
      break;
    }
    if (n == 0) {
      if (framer.partial()) set_error(self, "stream ended inside a frame (truncated input)");
      break;
    }
    int64_t ts = mono_ns();
    self->bytes_read->fetch_add(uint64_t(n), std::memory_order_relaxed);
    uint64_t frames = 0;
    bool ok = framer.feed(chunk.data(), size_t(n), [&](uint8_t topic, const uint8_t* p, uint32_t len) {
      if (ring_closed) return;
      if (self->ring->push(topic, 0, p, len, ts) < 0) ring_closed = true;
      ++frames;
    });
    self->frames_read->fetch_add(frames, std::memory_order_relaxed);
    if (!ok) {
      set_error(self, std::string("corrupt frame stream: ") + framer.error());
      break;
    }
  }
  self->ring->set_eof();
}

void ingest_stop_reader(IngestObject* self) {
  if (self->reader) {
    self->stop->store(true);
    self->ring->close();
    Py_BEGIN_ALLOW_THREADS self->reader->join();
    Py_END_ALLOW_THREADS delete self->reader;
    self->reader = nullptr;
  }
  if (self->own_fd && self->fd >= 0) {
    close(self->fd);
    self->fd = -1;
  }
}

PyObject* ingest_new(PyTypeObject* type, PyObject*, PyObject*) {
  IngestObject* self = reinterpret_cast<IngestObject*>(type->tp_alloc(type, 0));
  if (!self) return nullptr;
  self->ring = nullptr;
  self->settler = nullptr;
  self->reader = nullptr;
  self->stop = new std::atomic<bool>(false);
  self->bytes_read = new std::atomic<uint64_t>(0);
  self->frames_read = new std::atomic<uint64_t>(0);
  self->err_mu = new std::mutex();
  self->error = new std::string();
  self->py_framer = nullptr;
  self->max_frame = 16u << 20;
  self->fd = -1;
  self->own_fd = 0;
  self->efd = -1;
  return reinterpret_cast<PyObject*>(self);
}

int ingest_init_impl(IngestObject* self, PyObject* args, PyObject* kwds);
int ingest_init(IngestObject* self, PyObject* args, PyObject* kwds) {
  BEHOLDER_TRY { return ingest_init_impl(self, args, kwds); }
  BEHOLDER_CATCH(-1)
}

int ingest_init_impl(IngestObject* self, PyObject* args, PyObject* kwds) {
  static const char* kwlist[] = {"capacity_bytes", "capacity_events", "policy", "max_frame", "settler", nullptr};
  unsigned long long cap_bytes = 64ull << 20, cap_events = 0;
  const char* policy = "block";
  unsigned long max_frame = 0;  // 0 = min(16 MiB, capacity_bytes / 4)
  PyObject* settler = Py_None;
  if (!PyArg_ParseTupleAndKeywords(args, kwds, "|KKskO", const_cast<char**>(kwlist), &cap_bytes, &cap_events,
                                   &policy, &max_frame, &settler))
    return -1;
  int pol;
  if (!strcmp(policy, "block"))
    pol = POLICY_BLOCK;
  else if (!strcmp(policy, "drop_newest"))
    pol = POLICY_DROP_NEWEST;
  else {
    PyErr_SetString(PyExc_ValueError, "policy must be 'block' or 'drop_newest'");
    return -1;
  }
  if (cap_bytes < 4096) {
    PyErr_SetString(PyExc_ValueError, "capacity_bytes must be >= 4096");
    return -1;
  }
  if (max_frame == 0) max_frame = (unsigned long)((cap_bytes / 4) < (16ull << 20) ? (cap_bytes / 4) : (16ull << 20));
  if (max_frame < 2 || max_frame > cap_bytes / 4) {
    PyErr_SetString(PyExc_ValueError, "max_frame must be in [2, capacity_bytes/4]");
    return -1;
  }
  if (settler != Py_None && !PyObject_TypeCheck(settler, &SettlerType)) {
    PyErr_SetString(PyExc_TypeError, "settler must be a Settler or None");
    return -1;
  }
  if (self->ring) {
    PyErr_SetString(PyExc_RuntimeError, "Ingest already initialised");
    return -1;
  }
  self->ring = new ByteRing(size_t(cap_bytes), size_t(cap_events), pol);
  self->max_frame = uint32_t(max_frame);
  self->py_framer = new Framer(self->max_frame);
  if (settler == Py_None) {
    settler = PyObject_CallNoArgs(reinterpret_cast<PyObject*>(&SettlerType));
    if (!settler) return -1;
  } else {
    Py_INCREF(settler);
  }
  self->settler = reinterpret_cast<SettlerObject*>(settler);
  return 0;
}

void ingest_dealloc(IngestObject* self) {
  if (self->ring) ingest_stop_reader(self);
  delete self->ring;  // nothing signals the eventfd any more
  if (self->efd >= 0) close(self->efd);
  delete self->stop;
  delete self->bytes_read;
  delete self->frames_read;
  delete self->err_mu;
  delete self->error;
  delete self->py_framer;
  Py_XDECREF(self->settler);
  Py_TYPE(self)->tp_free(reinterpret_cast<PyObject*>(self));
}

bool check_ready(IngestObject* self) {
  if (!self->ring) {
    PyErr_SetString(PyExc_RuntimeError, "Ingest not initialised");
    return false;
  }
  return true;
}

// start_reader(fd, chunk_bytes=1MiB, own_fd=False)
PyObject* ingest_start_reader_impl(IngestObject* self, PyObject* args, PyObject* kwds);
PyObject* ingest_start_reader(IngestObject* self, PyObject* args, PyObject* kwds) {
  BEHOLDER_TRY { return ingest_start_reader_impl(self, args, kwds); }
  BEHOLDER_CATCH(nullptr)
}

PyObject* ingest_start_reader_impl(IngestObject* self, PyObject* args, PyObject* kwds) {
  static const char* kwlist[] = {"fd", "chunk_bytes", "own_fd", nullptr};
  int fd;
  unsigned long chunk = 1ul << 20;
  int own = 0;
  if (!PyArg_ParseTupleAndKeywords(args, kwds, "i|kp", const_cast<char**>(kwlist), &fd, &chunk, &own))
    return nullptr;
  if (!check_ready(self)) return nullptr;
  if (self->reader) {
    PyErr_SetString(PyExc_RuntimeError, "reader already started");
    return nullptr;
  }
  if (chunk < 4096) chunk = 4096;
  self->fd = fd;
  self->own_fd = own;
  self->stop->store(false);
  try {
    self->reader = new std::thread(reader_main, self, fd, size_t(chunk));
  } catch (const std::exception& e) {
    PyErr_Format(PyExc_RuntimeError, "cannot start reader thread: %s", e.what());
    return nullptr;
  }
  Py_RETURN_NONE;
}

PyObject* ingest_push(IngestObject* self, PyObject* args) {
  int topic;
  Py_buffer view;
  if (!PyArg_ParseTuple(args, "iy*", &topic, &view)) return nullptr;
  if (!check_ready(self)) {
    PyBuffer_Release(&view);
    return nullptr;
  }
  if (topic < 0 || topic > 255) {
    PyBuffer_Release(&view);
    PyErr_SetString(PyExc_ValueError, "topic must be in [0, 255]");
    return nullptr;
  }
  int r;
  int64_t ts = mono_ns();
  Py_BEGIN_ALLOW_THREADS r = self->ring->push(uint8_t(topic), 0, static_cast<const uint8_t*>(view.buf),
                                              uint32_t(view.len), ts);
  Py_END_ALLOW_THREADS PyBuffer_Release(&view);
  if (r < 0) {
    PyErr_SetString(PyExc_RuntimeError, "ingest is closed");
    return nullptr;
  }
  return PyBool_FromLong(r);
}

// feed(data): frame a byte stream fed from Python; returns frames accepted.
PyObject* ingest_feed_impl(IngestObject* self, PyObject* arg);
PyObject* ingest_feed(IngestObject* self, PyObject* arg) {
  BEHOLDER_TRY { return ingest_feed_impl(self, arg); }
  BEHOLDER_CATCH(nullptr)
}

PyObject* ingest_feed_impl(IngestObject* self, PyObject* arg) {
  if (!check_ready(self)) return nullptr;
  Py_buffer view;
  if (PyObject_GetBuffer(arg, &view, PyBUF_SIMPLE) < 0) return nullptr;
  int64_t ts = mono_ns();
  long accepted = 0;
  bool closed = false;
  bool ok;
  Py_BEGIN_ALLOW_THREADS ok = self->py_framer->feed(
      static_cast<const uint8_t*>(view.buf), size_t(view.len), [&](uint8_t topic, const uint8_t* p, uint32_t len) {
        if (closed) return;
        int r = self->ring->push(topic, 0, p, len, ts);
        if (r < 0) closed = true;
        accepted += r > 0;
      });
  Py_END_ALLOW_THREADS PyBuffer_Release(&view);
  if (!ok) {
    PyErr_Format(PyExc_ValueError, "corrupt frame stream: %s", self->py_framer->error());
    return nullptr;
  }
  if (closed) {
    PyErr_SetString(PyExc_RuntimeError, "ingest is closed");
    return nullptr;
  }
  return PyLong_FromLong(accepted);
}

PyObject* ingest_set_eof(IngestObject* self, PyObject*) {
  if (!check_ready(self)) return nullptr;
  self->ring->set_eof();
  Py_RETURN_NONE;
}

// pop(max_n=256, timeout=-1.0) -> list[Delivery] ([] on timeout) | None when drained
PyObject* ingest_pop_impl(IngestObject* self, PyObject* args, PyObject* kwds);
PyObject* ingest_pop(IngestObject* self, PyObject* args, PyObject* kwds) {
  BEHOLDER_TRY { return ingest_pop_impl(self, args, kwds); }
  BEHOLDER_CATCH(nullptr)
}

PyObject* ingest_pop_impl(IngestObject* self, PyObject* args, PyObject* kwds) {
  static const char* kwlist[] = {"max_n", "timeout", nullptr};
  Py_ssize_t max_n = 256;
  double timeout = -1.0;
  if (!PyArg_ParseTupleAndKeywords(args, kwds, "|nd", const_cast<char**>(kwlist), &max_n, &timeout)) return nullptr;
  if (!check_ready(self)) return nullptr;
  if (max_n < 1) max_n = 1;
  int64_t tns = timeout < 0 ? -1 : int64_t(timeout * 1e9);
  size_t avail;
  ByteRing* ring = self->ring;
  if (tns == 0) {
    avail = ring->wait_readable(0);
  } else {
    Py_BEGIN_ALLOW_THREADS avail = ring->wait_readable(tns);
    Py_END_ALLOW_THREADS
  }
  if (avail == 0) {
    if (ring->drained()) Py_RETURN_NONE;
    return PyList_New(0);
  }
  uint64_t pos = ring->read_begin(), end = ring->read_end();
  std::vector<PyObject*> items;
  items.reserve(size_t(max_n) < 4096 ? size_t(max_n) : 4096);
  SettlerObject* settler = self->settler;
  while (Py_ssize_t(items.size()) < max_n) {
    const RecordHeader* h = ring->next_record(pos, end);
    if (!h) break;
    PyObject* body = PyBytes_FromStringAndSize(reinterpret_cast<const char*>(ByteRing::payload_of(h)),
                                               Py_ssize_t(h->payload_len));
    if (!body) goto fail;
    PyObject* d = delivery_new(body, h->topic, h->seq + 1, h->recv_ns, settler, false);
    Py_DECREF(body);
    if (!d) goto fail;
    items.push_back(d);
  }
  ring->consume(pos, items.size());
  {
    PyObject* list = PyList_New(Py_ssize_t(items.size()));
    if (!list) {
      for (PyObject* o : items) Py_DECREF(o);
      return nullptr;
    }
    for (size_t i = 0; i < items.size(); ++i) PyList_SET_ITEM(list, Py_ssize_t(i), items[i]);
    return list;
  }
fail:
  // Records already turned into deliveries are consumed (they will be
  // abandoned -> on_abandon); the rest stay in the ring.
  {
    uint64_t p2 = ring->read_begin();
    for (size_t i = 0; i < items.size(); ++i) ring->next_record(p2, end);
    ring->consume(p2, items.size());
  }
  for (PyObject* o : items) Py_DECREF(o);
  return nullptr;
}

PyObject* ingest_close(IngestObject* self, PyObject*) {
  if (!self->ring) Py_RETURN_NONE;
  ingest_stop_reader(self);
  self->ring->close();
  Py_RETURN_NONE;
}

PyObject* ingest_stats(IngestObject* self, PyObject*) {
  if (!check_ready(self)) return nullptr;
  RingStats st = self->ring->stats();
  PyObject* dropped = PyDict_New();
  if (!dropped) return nullptr;
  for (int t = 0; t < MAX_TOPICS; ++t) {
    if (!st.dropped[t]) continue;
    PyObject* k = PyLong_FromLong(t);
    PyObject* v = PyLong_FromUnsignedLongLong(st.dropped[t]);
    PyDict_SetItem(dropped, k, v);
    Py_DECREF(k);
    Py_DECREF(v);
  }
  std::string err;
  {
    std::lock_guard<std::mutex> g(*self->err_mu);
    err = *self->error;
  }
  PyObject* errobj = err.empty() ? (Py_INCREF(Py_None), Py_None) : PyUnicode_FromString(err.c_str());
  PyObject* out = Py_BuildValue(
      "{s:K,s:K,s:K,s:N,s:K,s:K,s:K,s:K,s:K,s:n,s:O,s:N}", "pushed", (unsigned long long)st.pushed, "popped",
      (unsigned long long)st.popped, "dropped_total", (unsigned long long)st.dropped_total, "dropped_by_topic", dropped,
      "bytes_pushed", (unsigned long long)st.bytes_pushed, "blocked_ns", (unsigned long long)st.blocked_ns,
      "high_water_events", (unsigned long long)st.high_water_events, "bytes_read",
      (unsigned long long)self->bytes_read->load(), "frames_read", (unsigned long long)self->frames_read->load(),
      "depth", Py_ssize_t(self->ring->depth_events()), "eof", self->ring->eof() ? Py_True : Py_False, "error",
      errobj);
  return out;
}

PyObject* ingest_get_settler(IngestObject* self, void*) {
  if (!self->settler) Py_RETURN_NONE;
  Py_INCREF(self->settler);
  return reinterpret_cast<PyObject*>(self->settler);
}
// notify_fd: eventfd for loop.add_reader; created on first use and owned by the Ingest.
PyObject* ingest_get_notify_fd(IngestObject* self, void*) {
  if (!check_ready(self)) return nullptr;
  if (self->efd < 0) {
    int fd = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
    if (fd < 0) return PyErr_SetFromErrno(PyExc_OSError);
    self->efd = fd;
    self->ring->set_notify_fd(fd);
  }
  return PyLong_FromLong(self->efd);
}

// arm() -> bool: True = parked (the next push / EOF / close signals notify_fd);
// False = something is already poppable, pop again instead of waiting.
PyObject* ingest_arm(IngestObject* self, PyObject*) {
  if (!check_ready(self)) return nullptr;
  if (self->efd < 0) {
    PyErr_SetString(PyExc_RuntimeError, "arm() before notify_fd was created");
    return nullptr;
  }
  return PyBool_FromLong(self->ring->arm());
}

// clear_notify(): drains the eventfd counter (readiness callback; never blocks).
PyObject* ingest_clear_notify(IngestObject* self, PyObject*) {
  if (self->efd >= 0) {
    uint64_t v;
    ssize_t r;
    do {
      r = read(self->efd, &v, sizeof v);
    } while (r < 0 && errno == EINTR);
  }
  Py_RETURN_NONE;
}

PyObject* ingest_get_depth(IngestObject* self, void*) {
  if (!check_ready(self)) return nullptr;
  return PyLong_FromSize_t(self->ring->depth_events());
}
PyObject* ingest_get_drained(IngestObject* self, void*) {
  if (!check_ready(self)) return nullptr;
  return PyBool_FromLong(self->ring->drained());
}

PyMethodDef ingest_methods[] = {
    {"start_reader", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(ingest_start_reader)),
     METH_VARARGS | METH_KEYWORDS, "start_reader(fd, chunk_bytes=1MiB, own_fd=False)"},
    {"push", reinterpret_cast<PyCFunction>(ingest_push), METH_VARARGS, "push(topic, payload) -> accepted"},
    {"feed", reinterpret_cast<PyCFunction>(ingest_feed), METH_O, "feed(framed_bytes) -> frames accepted"},
    {"set_eof", reinterpret_cast<PyCFunction>(ingest_set_eof), METH_NOARGS, "no more input"},
    {"pop", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(ingest_pop)), METH_VARARGS | METH_KEYWORDS,
     "pop(max_n=256, timeout=-1.0) -> list[Delivery] | None when drained"},
    {"close", reinterpret_cast<PyCFunction>(ingest_close), METH_NOARGS, "stop the reader and close"},
    {"arm", reinterpret_cast<PyCFunction>(ingest_arm), METH_NOARGS,
     "arm() -> True if parked until notify_fd is signalled, False if a pop would succeed now"},
    {"clear_notify", reinterpret_cast<PyCFunction>(ingest_clear_notify), METH_NOARGS, "drain notify_fd"},
    {"stats", reinterpret_cast<PyCFunction>(ingest_stats), METH_NOARGS, "ring / reader statistics"},
    {nullptr, nullptr, 0, nullptr}};

PyGetSetDef ingest_getset[] = {
    {"settler", reinterpret_cast<getter>(ingest_get_settler), nullptr, "Settler of popped deliveries", nullptr},
    {"depth", reinterpret_cast<getter>(ingest_get_depth), nullptr, "records queued", nullptr},
    {"notify_fd", reinterpret_cast<getter>(ingest_get_notify_fd), nullptr,
     "eventfd signalled once per arm() by the next push / EOF / close (for loop.add_reader)", nullptr},
    {"drained", reinterpret_cast<getter>(ingest_get_drained), nullptr, "EOF/closed and empty", nullptr},
    {nullptr, nullptr, nullptr, nullptr, nullptr}};

}  // namespace

PyTypeObject IngestType = {PyVarObject_HEAD_INIT(nullptr, 0)};

int init_ingest_types(PyObject* m) {
  SettlerType.tp_name = "beholder_amd.ops._native.Settler";
  SettlerType.tp_basicsize = sizeof(SettlerObject);
  SettlerType.tp_flags = Py_TPFLAGS_DEFAULT | Py_TPFLAGS_HAVE_GC;
  SettlerType.tp_doc = "Settler(on_settle=None, on_abandon=None): ack accounting and latency histograms";
  SettlerType.tp_new = settler_new;
  SettlerType.tp_init = reinterpret_cast<initproc>(settler_init);
  SettlerType.tp_dealloc = reinterpret_cast<destructor>(settler_dealloc);
  SettlerType.tp_traverse = reinterpret_cast<traverseproc>(settler_traverse);
  SettlerType.tp_clear = reinterpret_cast<inquiry>(settler_clear);
  SettlerType.tp_methods = settler_methods;
  SettlerType.tp_getset = settler_getset;
  if (PyType_Ready(&SettlerType) < 0) return -1;

  DeliveryType.tp_name = "beholder_amd.ops._native.Delivery";
  DeliveryType.tp_basicsize = sizeof(DeliveryObject);
  DeliveryType.tp_flags = Py_TPFLAGS_DEFAULT;
  DeliveryType.tp_doc = "Delivery(content, topic_id=0, tag=0, settler=None, recv_ns=None, redelivered=False, extra=None)";
  DeliveryType.tp_new = delivery_py_new;
  DeliveryType.tp_dealloc = reinterpret_cast<destructor>(delivery_dealloc);
  DeliveryType.tp_methods = delivery_methods;
  DeliveryType.tp_getset = delivery_getset;
  DeliveryType.tp_repr = reinterpret_cast<reprfunc>(delivery_repr);
  if (PyType_Ready(&DeliveryType) < 0) return -1;

  IngestType.tp_name = "beholder_amd.ops._native.Ingest";
  IngestType.tp_basicsize = sizeof(IngestObject);
  IngestType.tp_flags = Py_TPFLAGS_DEFAULT;
  IngestType.tp_doc =
      "Ingest(capacity_bytes=64MiB, capacity_events=0, policy='block', max_frame=16MiB, settler=None)";
  IngestType.tp_new = ingest_new;
  IngestType.tp_init = reinterpret_cast<initproc>(ingest_init);
  IngestType.tp_dealloc = reinterpret_cast<destructor>(ingest_dealloc);
  IngestType.tp_methods = ingest_methods;
  IngestType.tp_getset = ingest_getset;
  if (PyType_Ready(&IngestType) < 0) return -1;

  PyObject* types[] = {reinterpret_cast<PyObject*>(&SettlerType), reinterpret_cast<PyObject*>(&DeliveryType),
                       reinterpret_cast<PyObject*>(&IngestType)};
  const char* names[] = {"Settler", "Delivery", "Ingest"};
  for (int i = 0; i < 3; ++i) {
    Py_INCREF(types[i]);
    if (PyModule_AddObject(m, names[i], types[i]) < 0) return -1;
  }
  return 0;
}

}  // namespace beholder
