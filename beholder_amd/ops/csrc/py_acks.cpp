// AckBatcher: native AMQP ack coalescing for the consumer channel.
//
// The handlers settle with rmsg.ack() (index.js:71,124,151,154). Each ack used to
// call into Python (Settler.on_settle -> the source's coalescer), about 1.7 us per
// message. With a batcher attached to the Settler, Delivery.ack() of a delivery
// from the batcher's current channel is recorded here in C. The batcher calls
// `schedule()` once per burst, and the source then calls flush() once per event-loop
// iteration and writes the returned frames:
//
//   * the longest run of settled tags starting at the lowest unsettled one
//     -> one basic.ack(multiple=true);
//   * acks above a gap -> one basic.ack each, in the same write.
//
// Delivery tags are a per-channel counter (1, 2, 3, ...), so the run needs no
// record of which tags were seen. A tag that will never be acked (a Q1 status
// message left un-acked, reported by the Settler when its Delivery is freed)
// blocks `multiple` for the rest of the channel's life: multiple=true would
// cover it. From then on every ack goes out individually and nothing is
// buffered, so memory stays bounded. `max_settled` bounds the settled set in
// the case where a gap is never reported (a delivery dropped before it reached
// a handler).
#include <string>
#include <unordered_set>
#include <vector>

#include "py_common.hpp"

namespace beholder {

namespace {

struct AckBatcherObject {
  PyObject_HEAD PyObject* channel;  // current channel token (identity compare with Delivery.extra)
  PyObject* schedule;               // callable(): arrange one flush() this loop iteration
  uint16_t channel_id;
  bool scheduled;
  uint64_t low;    // lowest tag not known to be settled
  uint64_t stuck;  // lowest tag that will never be settled here (0 = none)
  std::unordered_set<uint64_t>* settled;  // settled tags > low (only while stuck == 0)
  std::vector<uint64_t>* pending;         // acks to send at the next flush
  uint64_t frames, acks, multiples, max_settled;
};

PyTypeObject AckBatcherType = {PyVarObject_HEAD_INIT(nullptr, 0)};

void reset(AckBatcherObject* b) {
  b->low = 1;
  b->stuck = 0;
  b->settled->clear();
  b->pending->clear();
}

int schedule_flush(AckBatcherObject* b) {
  if (b->scheduled || !b->schedule) return 0;
  b->scheduled = true;
  PyObject* r = PyObject_CallNoArgs(b->schedule);
  if (!r) {
    b->scheduled = false;
    return -1;
  }
  Py_DECREF(r);
  return 0;
}

void mark_settled(AckBatcherObject* b, uint64_t tag) {
  if (tag < b->low) return;
  if (b->stuck) return;  // no multiple acks any more: nothing to track
  if (tag == b->low) {
    ++b->low;
    while (!b->settled->empty()) {
      auto it = b->settled->find(b->low);
      if (it == b->settled->end()) break;
      b->settled->erase(it);
      ++b->low;
    }
    return;
  }
  b->settled->insert(tag);
  if (b->settled->size() > b->max_settled) {
    // an unreported permanent gap at `low`: stop multiple acks for this channel
    b->stuck = b->low;
    b->settled->clear();
  }
}

int add_ack(AckBatcherObject* b, uint64_t tag) {
  b->pending->push_back(tag);
  ++b->acks;
  mark_settled(b, tag);
  return schedule_flush(b);
}

void abandon(AckBatcherObject* b, uint64_t tag) {
  if (tag < b->low) return;
  if (!b->stuck || tag < b->stuck) b->stuck = tag;
  b->settled->clear();
}

void put_ack(std::string& out, uint16_t ch, uint64_t tag, bool multiple) {
  char f[21];
  f[0] = 1;  // method frame
  f[1] = char(ch >> 8);
  f[2] = char(ch);
  f[3] = 0;
  f[4] = 0;
  f[5] = 0;
  f[6] = 13;
  f[7] = 0;
  f[8] = 60;  // basic
  f[9] = 0;
  f[10] = 80;  // ack
  for (int i = 0; i < 8; ++i) f[11 + i] = char(tag >> (56 - 8 * i));
  f[19] = multiple ? 1 : 0;
  f[20] = char(0xCE);
  out.append(f, sizeof(f));
}

PyObject* ab_new(PyTypeObject* type, PyObject*, PyObject*) {
  AckBatcherObject* b = reinterpret_cast<AckBatcherObject*>(type->tp_alloc(type, 0));
  if (!b) return nullptr;
  try {
    b->settled = new std::unordered_set<uint64_t>();
    b->pending = new std::vector<uint64_t>();
  } catch (const std::bad_alloc&) {
    Py_DECREF(b);
    return PyErr_NoMemory();
  }
  b->channel = b->schedule = nullptr;
  b->channel_id = 0;
  b->scheduled = false;
  b->frames = b->acks = b->multiples = 0;
  b->max_settled = 65536;
  reset(b);
  return reinterpret_cast<PyObject*>(b);
}

int ab_init(AckBatcherObject* b, PyObject* args, PyObject* kwds) {
  static const char* kwlist[] = {"schedule", "max_settled", nullptr};
  PyObject* schedule;
  unsigned long long ms = 65536;
  if (!PyArg_ParseTupleAndKeywords(args, kwds, "O|K", const_cast<char**>(kwlist), &schedule, &ms)) return -1;
  if (!PyCallable_Check(schedule)) {
    PyErr_SetString(PyExc_TypeError, "schedule must be callable");
    return -1;
  }
  Py_INCREF(schedule);
  Py_XSETREF(b->schedule, schedule);
  b->max_settled = ms ? ms : 1;
  return 0;
}

int ab_traverse(AckBatcherObject* b, visitproc visit, void* arg) {
  Py_VISIT(b->channel);
  Py_VISIT(b->schedule);
  return 0;
}

int ab_clear(AckBatcherObject* b) {
  Py_CLEAR(b->channel);
  Py_CLEAR(b->schedule);
  return 0;
}

void ab_dealloc(AckBatcherObject* b) {
  PyObject_GC_UnTrack(b);
  ab_clear(b);
  delete b->settled;
  delete b->pending;
  Py_TYPE(b)->tp_free(reinterpret_cast<PyObject*>(b));
}

// bind(channel, channel_id): deliveries of `channel` are batched from now on (fresh tag space)
PyObject* ab_bind(AckBatcherObject* b, PyObject* args) {
  PyObject* ch;
  int cid;
  if (!PyArg_ParseTuple(args, "Oi", &ch, &cid)) return nullptr;
  if (cid < 0 || cid > 65535) {
    PyErr_SetString(PyExc_ValueError, "channel id must be in [0, 65535]");
    return nullptr;
  }
  Py_INCREF(ch);
  Py_XSETREF(b->channel, ch);
  b->channel_id = uint16_t(cid);
  reset(b);
  Py_RETURN_NONE;
}

PyObject* ab_unbind(AckBatcherObject* b, PyObject*) {
  Py_CLEAR(b->channel);
  reset(b);
  Py_RETURN_NONE;
}

uint64_t tag_arg(PyObject* arg, bool* ok) {
  unsigned long long t = PyLong_AsUnsignedLongLong(arg);
  *ok = !(t == (unsigned long long)-1 && PyErr_Occurred());
  return t;
}

PyObject* ab_ack(AckBatcherObject* b, PyObject* arg) {
  BEHOLDER_TRY {
    bool ok;
    uint64_t t = tag_arg(arg, &ok);
    if (!ok) return nullptr;
    if (add_ack(b, t) < 0) return nullptr;
    Py_RETURN_NONE;
  }
  BEHOLDER_CATCH(nullptr)
}

PyObject* ab_settled_elsewhere(AckBatcherObject* b, PyObject* arg) {
  BEHOLDER_TRY {
    bool ok;
    uint64_t t = tag_arg(arg, &ok);
    if (!ok) return nullptr;
    mark_settled(b, t);
    Py_RETURN_NONE;
  }
  BEHOLDER_CATCH(nullptr)
}

PyObject* ab_abandon(AckBatcherObject* b, PyObject* arg) {
  bool ok;
  uint64_t t = tag_arg(arg, &ok);
  if (!ok) return nullptr;
  abandon(b, t);
  Py_RETURN_NONE;
}

// flush() -> bytes: the ack frames for everything acked since the last flush
PyObject* ab_flush(AckBatcherObject* b, PyObject*) {
  BEHOLDER_TRY {
    b->scheduled = false;
    std::vector<uint64_t>& p = *b->pending;
    if (p.empty()) return PyBytes_FromStringAndSize(nullptr, 0);
    uint64_t prefix = b->low - 1;  // every tag <= prefix is settled
    if (b->stuck && prefix >= b->stuck) prefix = b->stuck - 1;
    uint64_t top = 0;
    std::string out;
    out.reserve(21 * (p.size() + 1));
    size_t n_single = 0;
    for (uint64_t t : p)
      if (t <= prefix) {
        if (t > top) top = t;
      } else {
        ++n_single;
      }
    if (top) {
      put_ack(out, b->channel_id, top, true);
      ++b->multiples;
    }
    for (uint64_t t : p)
      if (t > prefix) put_ack(out, b->channel_id, t, false);
    b->frames += n_single + (top ? 1 : 0);
    p.clear();
    return PyBytes_FromStringAndSize(out.data(), Py_ssize_t(out.size()));
  }
  BEHOLDER_CATCH(nullptr)
}

PyObject* ab_get_channel(AckBatcherObject* b, void*) {
  PyObject* c = b->channel ? b->channel : Py_None;
  Py_INCREF(c);
  return c;
}
#define AB_U64(name, expr) \
  PyObject* ab_get_##name(AckBatcherObject* b, void*) { return PyLong_FromUnsignedLongLong((unsigned long long)(expr)); }
AB_U64(low, b->low)
AB_U64(stuck, b->stuck)
AB_U64(pending, b->pending->size())
AB_U64(tracked, b->settled->size())
AB_U64(frames, b->frames)
AB_U64(acks, b->acks)
AB_U64(multiples, b->multiples)

PyMethodDef ab_methods[] = {
    {"bind", reinterpret_cast<PyCFunction>(ab_bind), METH_VARARGS,
     "bind(channel, channel_id): batch acks of this channel's deliveries (tags restart at 1)"},
    {"unbind", reinterpret_cast<PyCFunction>(ab_unbind), METH_NOARGS, "stop batching (channel gone)"},
    {"ack", reinterpret_cast<PyCFunction>(ab_ack), METH_O, "ack(tag): queue an ack (Delivery.ack does this in C)"},
    {"settled_elsewhere", reinterpret_cast<PyCFunction>(ab_settled_elsewhere), METH_O,
     "settled_elsewhere(tag): nack/reject already sent for tag"},
    {"abandon", reinterpret_cast<PyCFunction>(ab_abandon), METH_O,
     "abandon(tag): tag will never be settled (no more multiple acks on this channel)"},
    {"flush", reinterpret_cast<PyCFunction>(ab_flush), METH_NOARGS, "flush() -> bytes of basic.ack frames"},
    {nullptr, nullptr, 0, nullptr}};

PyGetSetDef ab_getset[] = {
    {"channel", reinterpret_cast<getter>(ab_get_channel), nullptr, "bound channel token", nullptr},
    {"low", reinterpret_cast<getter>(ab_get_low), nullptr, "lowest tag not known settled", nullptr},
    {"stuck", reinterpret_cast<getter>(ab_get_stuck), nullptr, "lowest never-settled tag (0 = none)", nullptr},
    {"pending", reinterpret_cast<getter>(ab_get_pending), nullptr, "acks waiting for flush()", nullptr},
    {"tracked", reinterpret_cast<getter>(ab_get_tracked), nullptr, "settled tags above the gap", nullptr},
    {"frames", reinterpret_cast<getter>(ab_get_frames), nullptr, "ack frames produced", nullptr},
    {"acks", reinterpret_cast<getter>(ab_get_acks), nullptr, "acks queued", nullptr},
    {"multiples", reinterpret_cast<getter>(ab_get_multiples), nullptr, "multiple=true frames", nullptr},
    {nullptr, nullptr, nullptr, nullptr, nullptr}};

}  // namespace

// Hooks for the Settler (py_ingest.cpp). Return 1 = handled, 0 = not this batcher's channel,
// -1 = Python error.
int ack_batcher_ack(PyObject* batcher, PyObject* channel, uint64_t tag) {
  AckBatcherObject* b = reinterpret_cast<AckBatcherObject*>(batcher);
  if (!b->channel || channel != b->channel) return 0;
  try {
    return add_ack(b, tag) < 0 ? -1 : 1;
  } catch (const std::bad_alloc&) {
    PyErr_NoMemory();
    return -1;
  }
}

void ack_batcher_abandon(PyObject* batcher, PyObject* channel, uint64_t tag) {
  AckBatcherObject* b = reinterpret_cast<AckBatcherObject*>(batcher);
  if (b->channel && channel == b->channel) abandon(b, tag);
}

bool is_ack_batcher(PyObject* o) { return PyObject_TypeCheck(o, &AckBatcherType); }

int init_ack_types(PyObject* m) {
  AckBatcherType.tp_name = "beholder_amd.ops._native.AckBatcher";
  AckBatcherType.tp_basicsize = sizeof(AckBatcherObject);
  AckBatcherType.tp_flags = Py_TPFLAGS_DEFAULT | Py_TPFLAGS_HAVE_GC;
  AckBatcherType.tp_doc = "AckBatcher(schedule, max_settled=65536): native AMQP ack coalescing";
  AckBatcherType.tp_new = ab_new;
  AckBatcherType.tp_init = reinterpret_cast<initproc>(ab_init);
  AckBatcherType.tp_dealloc = reinterpret_cast<destructor>(ab_dealloc);
  AckBatcherType.tp_traverse = reinterpret_cast<traverseproc>(ab_traverse);
  AckBatcherType.tp_clear = reinterpret_cast<inquiry>(ab_clear);
  AckBatcherType.tp_methods = ab_methods;
  AckBatcherType.tp_getset = ab_getset;
  if (PyType_Ready(&AckBatcherType) < 0) return -1;
  Py_INCREF(&AckBatcherType);
  return PyModule_AddObject(m, "AckBatcher", reinterpret_cast<PyObject*>(&AckBatcherType));
}

}  // namespace beholder
