// AmqpDemux: native AMQP 0-9-1 frame demultiplexer for the consumer hot path.
//
// The reference's ingest path is amqplib's socket reader handing each
// basic.deliver (method + content header + body frames) to a handler
// (index.js:62,127). Here the asyncio reader feeds raw socket bytes to
// AmqpDemux.feed(): frames are split in C, and a basic.deliver for a
// registered (channel, consumer-tag) is assembled straight into a native
// Delivery (the `rmsg`) without creating per-frame Python objects. Every other
// frame — connection/channel methods, content for unknown consumers,
// basic.return — is passed through as (type, channel, payload) in stream order
// for the Python protocol code (transport/amqp/connection.py).
#include <map>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

#include "py_common.hpp"
#include "gil_clock.hpp"
#include "ring.hpp"

namespace beholder {

namespace {

struct ConsumerInfo {
  int topic;
  PyObject* extra;  // strong ref
};

struct Pending {
  enum Mode : uint8_t { NONE = 0, NATIVE = 1, PASS = 2 } mode = NONE;
  bool have_header = false;
  uint64_t size = 0;
  std::string body;
  uint64_t tag = 0;
  bool redelivered = false;
  int topic = 0;
  PyObject* extra = nullptr;  // borrowed from ConsumerInfo (kept alive by the map)
  std::string headers;        // raw `headers` field table (u32 length + body) when captured
};

// RabbitMQ's hard upper bound for a message body (max_message_size <= 512 MiB).
constexpr uint64_t kMaxBody = 512ull << 20;

struct AmqpDemuxObject {
  PyObject_HEAD SettlerObject* settler;
  std::string* carry;
  std::unordered_map<uint16_t, Pending>* pending;
  std::map<std::pair<uint16_t, std::string>, ConsumerInfo>* consumers;
  uint32_t frame_max;
  uint64_t deliveries, frames, passthrough, heartbeats;
  uint8_t capture_headers;  // keep the `headers` property of deliveries (trace context)
};

inline uint16_t be16(const uint8_t* p) { return uint16_t((p[0] << 8) | p[1]); }
inline uint32_t be32(const uint8_t* p) {
  return (uint32_t(p[0]) << 24) | (uint32_t(p[1]) << 16) | (uint32_t(p[2]) << 8) | uint32_t(p[3]);
}
inline uint64_t be64(const uint8_t* p) { return (uint64_t(be32(p)) << 32) | be32(p + 4); }

PyObject* demux_new(PyTypeObject* type, PyObject*, PyObject*) {
  AmqpDemuxObject* self = reinterpret_cast<AmqpDemuxObject*>(type->tp_alloc(type, 0));
  if (!self) return nullptr;
  self->settler = nullptr;
  self->carry = new std::string();
  self->pending = new std::unordered_map<uint16_t, Pending>();
  self->consumers = new std::map<std::pair<uint16_t, std::string>, ConsumerInfo>();
  self->frame_max = 0;
  self->deliveries = self->frames = self->passthrough = self->heartbeats = 0;
  return reinterpret_cast<PyObject*>(self);
}

int demux_init(AmqpDemuxObject* self, PyObject* args, PyObject* kwds) {
  static const char* kwlist[] = {"settler", "frame_max", nullptr};
  PyObject* settler = Py_None;
  unsigned long fm = 0;
  if (!PyArg_ParseTupleAndKeywords(args, kwds, "|Ok", const_cast<char**>(kwlist), &settler, &fm)) return -1;
  if (settler != Py_None) {
    if (!PyObject_TypeCheck(settler, &SettlerType)) {
      PyErr_SetString(PyExc_TypeError, "settler must be a Settler");
      return -1;
    }
    Py_INCREF(settler);
    Py_XSETREF(self->settler, reinterpret_cast<SettlerObject*>(settler));
  }
  self->frame_max = uint32_t(fm);
  return 0;
}

int demux_traverse(AmqpDemuxObject* self, visitproc visit, void* arg) {
  Py_VISIT(self->settler);
  for (auto& kv : *self->consumers) Py_VISIT(kv.second.extra);
  return 0;
}

int demux_clear(AmqpDemuxObject* self) {
  Py_CLEAR(self->settler);
  for (auto& kv : *self->consumers) Py_CLEAR(kv.second.extra);
  self->consumers->clear();
  self->pending->clear();
  return 0;
}

void demux_dealloc(AmqpDemuxObject* self) {
  PyObject_GC_UnTrack(self);
  demux_clear(self);
  delete self->carry;
  delete self->pending;
  delete self->consumers;
  Py_TYPE(self)->tp_free(reinterpret_cast<PyObject*>(self));
}

PyObject* demux_add_consumer(AmqpDemuxObject* self, PyObject* args) {
  int ch, topic;
  const char* tag;
  Py_ssize_t tlen;
  PyObject* extra;
  if (!PyArg_ParseTuple(args, "is#iO", &ch, &tag, &tlen, &topic, &extra)) return nullptr;
  if (ch < 0 || ch > 65535 || topic < 0 || topic > 255) {
    PyErr_SetString(PyExc_ValueError, "channel/topic out of range");
    return nullptr;
  }
  auto key = std::make_pair(uint16_t(ch), std::string(tag, size_t(tlen)));
  auto it = self->consumers->find(key);
  Py_INCREF(extra);
  if (it != self->consumers->end()) {
    Py_DECREF(it->second.extra);
    it->second = ConsumerInfo{topic, extra};
  } else {
    (*self->consumers)[key] = ConsumerInfo{topic, extra};
  }
  Py_RETURN_NONE;
}

PyObject* demux_remove_consumer(AmqpDemuxObject* self, PyObject* args) {
  int ch;
  const char* tag;
  Py_ssize_t tlen;
  if (!PyArg_ParseTuple(args, "is#", &ch, &tag, &tlen)) return nullptr;
  auto it = self->consumers->find(std::make_pair(uint16_t(ch), std::string(tag, size_t(tlen))));
  if (it != self->consumers->end()) {
    Py_DECREF(it->second.extra);
    self->consumers->erase(it);
  }
  Py_RETURN_NONE;
}

// reset_channel(ch): forget consumers + partial content of a closed channel
PyObject* demux_reset_channel(AmqpDemuxObject* self, PyObject* arg) {
  long ch = PyLong_AsLong(arg);
  if (ch == -1 && PyErr_Occurred()) return nullptr;
  self->pending->erase(uint16_t(ch));
  for (auto it = self->consumers->begin(); it != self->consumers->end();) {
    if (it->first.first == uint16_t(ch)) {
      Py_DECREF(it->second.extra);
      it = self->consumers->erase(it);
    } else {
      ++it;
    }
  }
  Py_RETURN_NONE;
}

PyObject* demux_set_frame_max(AmqpDemuxObject* self, PyObject* arg) {
  unsigned long v = PyLong_AsUnsignedLong(arg);
  if (PyErr_Occurred()) return nullptr;
  self->frame_max = uint32_t(v);
  Py_RETURN_NONE;
}

bool emit_pass(PyObject* out, uint8_t type, uint16_t ch, const uint8_t* p, uint32_t n) {
  PyObject* t = Py_BuildValue("(iiy#)", int(type), int(ch), reinterpret_cast<const char*>(p), Py_ssize_t(n));
  if (!t) return false;
  int r = PyList_Append(out, t);
  Py_DECREF(t);
  return r == 0;
}

bool emit_delivery(AmqpDemuxObject* self, PyObject* out, Pending& pd, int64_t now) {
  PyObject* body = PyBytes_FromStringAndSize(pd.body.data(), Py_ssize_t(pd.body.size()));
  if (!body) return false;
  PyObject* d = delivery_new(body, uint8_t(pd.topic), pd.tag, now, self->settler, pd.redelivered);
  Py_DECREF(body);
  if (!d) return false;
  if (pd.extra) {
    Py_INCREF(pd.extra);
    reinterpret_cast<DeliveryObject*>(d)->extra = pd.extra;
  }
  if (!pd.headers.empty()) {
    PyObject* h = PyBytes_FromStringAndSize(pd.headers.data(), Py_ssize_t(pd.headers.size()));
    if (!h) {
      Py_DECREF(d);
      return false;
    }
    reinterpret_cast<DeliveryObject*>(d)->headers = h;
    pd.headers.clear();
  }
  int r = PyList_Append(out, d);
  Py_DECREF(d);
  pd.mode = Pending::NONE;
  pd.have_header = false;
  pd.body.clear();
  pd.extra = nullptr;
  self->deliveries++;
  return r == 0;
}

// Parse basic.deliver arguments: consumer_tag, delivery_tag, redelivered, exchange, routing_key.
bool parse_deliver(const uint8_t* a, uint32_t n, std::string* ctag, uint64_t* tag, bool* redelivered) {
  uint32_t i = 0;
  if (n < 1) return false;
  uint32_t cl = a[i++];
  if (i + cl + 8 + 1 > n) return false;
  ctag->assign(reinterpret_cast<const char*>(a + i), cl);
  i += cl;
  *tag = be64(a + i);
  i += 8;
  *redelivered = (a[i] & 1) != 0;
  return true;
}

bool handle_frame(AmqpDemuxObject* self, PyObject* out, uint8_t type, uint16_t ch, const uint8_t* p, uint32_t n,
                  int64_t now) {
  self->frames++;
  if (type == 8) {  // heartbeat
    self->heartbeats++;
    return true;
  }
  if (type == 1) {
    if (n >= 4 && be16(p) == 60 && be16(p + 2) == 60) {  // basic.deliver
      std::string ctag;
      uint64_t tag;
      bool redel;
      if (parse_deliver(p + 4, n - 4, &ctag, &tag, &redel)) {
        auto it = self->consumers->find(std::make_pair(ch, ctag));
        if (it != self->consumers->end()) {
          Pending& pd = (*self->pending)[ch];
          pd.mode = Pending::NATIVE;
          pd.have_header = false;
          pd.size = 0;
          pd.body.clear();
          pd.tag = tag;
          pd.redelivered = redel;
          pd.topic = it->second.topic;
          pd.extra = it->second.extra;
          return true;
        }
      }
      (*self->pending)[ch].mode = Pending::PASS;
      self->passthrough++;
      return emit_pass(out, type, ch, p, n);
    }
    if (n >= 4 && be16(p) == 60 && (be16(p + 2) == 50 || be16(p + 2) == 71)) {  // return / get_ok carry content
      (*self->pending)[ch].mode = Pending::PASS;
    }
    self->passthrough++;
    return emit_pass(out, type, ch, p, n);
  }
  auto pit = self->pending->find(ch);
  if (pit == self->pending->end() || pit->second.mode != Pending::NATIVE) {
    // content of a passthrough method (Python tracks completion) or a stray frame
    self->passthrough++;
    return emit_pass(out, type, ch, p, n);
  }
  Pending& pd = pit->second;
  if (type == 2) {
    if (n < 14 || pd.have_header) {
      PyErr_SetString(PyExc_ValueError, "malformed or unexpected content header");
      return false;
    }
    pd.have_header = true;
    pd.size = be64(p + 4);
    pd.headers.clear();
    if (self->capture_headers) {
      // property flags (bit 15 content-type, 14 content-encoding, 13 headers), then the values
      uint16_t flags = be16(p + 12);
      uint32_t off = 14;
      bool ok = true;
      for (uint16_t bit : {uint16_t(0x8000), uint16_t(0x4000)}) {
        if (!(flags & bit)) continue;
        if (off + 1 > n || off + 1 + p[off] > n) {
          ok = false;
          break;
        }
        off += 1 + p[off];
      }
      if (ok && (flags & 0x2000) && off + 4 <= n) {
        uint32_t tl = be32(p + off);
        if (uint64_t(off) + 4 + tl <= n) pd.headers.assign(reinterpret_cast<const char*>(p + off), 4 + size_t(tl));
      }
    }
    if (pd.size > kMaxBody) {
      PyErr_Format(PyExc_ValueError, "content body size %llu exceeds the %llu byte limit",
                   (unsigned long long)pd.size, (unsigned long long)kMaxBody);
      return false;
    }
    if (pd.size == 0) return emit_delivery(self, out, pd, now);
    pd.body.reserve(size_t(pd.size < (1u << 20) ? pd.size : (1u << 20)));
    return true;
  }
  if (type == 3) {
    if (!pd.have_header) {
      PyErr_SetString(PyExc_ValueError, "body frame before content header");
      return false;
    }
    pd.body.append(reinterpret_cast<const char*>(p), n);
    if (pd.body.size() > pd.size) {
      PyErr_SetString(PyExc_ValueError, "content body larger than announced");
      return false;
    }
    if (pd.body.size() == pd.size) return emit_delivery(self, out, pd, now);
    return true;
  }
  PyErr_Format(PyExc_ValueError, "unexpected frame type %d", int(type));
  return false;
}

// feed(data) -> list of Delivery | (type, channel, payload)
PyObject* demux_feed_impl(AmqpDemuxObject* self, PyObject* arg);
PyObject* demux_feed(AmqpDemuxObject* self, PyObject* arg) {
  BEHOLDER_TRY { return demux_feed_impl(self, arg); }
  BEHOLDER_CATCH(nullptr)
}

PyObject* demux_feed_impl(AmqpDemuxObject* self, PyObject* arg) {
  Py_buffer view;
  if (PyObject_GetBuffer(arg, &view, PyBUF_SIMPLE) < 0) return nullptr;
  PyObject* out = PyList_New(0);
  if (!out) {
    PyBuffer_Release(&view);
    return nullptr;
  }
  const uint8_t* base;
  size_t len;
  std::string& carry = *self->carry;
  if (carry.empty()) {
    base = static_cast<const uint8_t*>(view.buf);
    len = size_t(view.len);
  } else {
    carry.append(static_cast<const char*>(view.buf), size_t(view.len));
    base = reinterpret_cast<const uint8_t*>(carry.data());
    len = carry.size();
  }
  int64_t now = gil_mono_ns();
  size_t i = 0;
  bool ok = true;
  while (len - i >= 7) {
    uint8_t type = base[i];
    uint16_t ch = be16(base + i + 1);
    uint32_t size = be32(base + i + 3);
    if (self->frame_max && size > self->frame_max) {
      PyErr_Format(PyExc_ValueError, "frame of %u bytes exceeds frame_max %u", size, self->frame_max);
      ok = false;
      break;
    }
    if (len - i < size_t(size) + 8) break;
    if (base[i + 7 + size] != 0xCE) {
      PyErr_SetString(PyExc_ValueError, "missing frame-end octet");
      ok = false;
      break;
    }
    if (!handle_frame(self, out, type, ch, base + i + 7, size, now)) {
      ok = false;
      break;
    }
    i += size_t(size) + 8;
  }
  if (ok) {
    if (carry.empty()) {
      if (i < len) carry.assign(reinterpret_cast<const char*>(base + i), len - i);
    } else {
      carry.erase(0, i);
    }
  }
  PyBuffer_Release(&view);
  if (!ok) {
    Py_DECREF(out);
    return nullptr;
  }
  return out;
}

PyObject* demux_stats(AmqpDemuxObject* self, PyObject*) {
  return Py_BuildValue("{s:K,s:K,s:K,s:K,s:n,s:n}", "deliveries", (unsigned long long)self->deliveries, "frames",
                       (unsigned long long)self->frames, "passthrough", (unsigned long long)self->passthrough,
                       "heartbeats", (unsigned long long)self->heartbeats, "consumers",
                       Py_ssize_t(self->consumers->size()), "buffered", Py_ssize_t(self->carry->size()));
}

PyObject* demux_get_passthrough(AmqpDemuxObject* self, void*) {
  return PyLong_FromUnsignedLongLong(self->passthrough);
}

PyObject* demux_get_capture(AmqpDemuxObject* self, void*) { return PyBool_FromLong(self->capture_headers); }
int demux_set_capture(AmqpDemuxObject* self, PyObject* v, void*) {
  int t = v ? PyObject_IsTrue(v) : 0;
  if (t < 0) return -1;
  self->capture_headers = uint8_t(t);
  return 0;
}

PyGetSetDef demux_getset[] = {
    {"capture_headers", reinterpret_cast<getter>(demux_get_capture), reinterpret_cast<setter>(demux_set_capture),
     "attach each delivery's raw `headers` field table (Delivery.headers)", nullptr},
    {"passthrough", reinterpret_cast<getter>(demux_get_passthrough), nullptr,
     "frames handed to Python so far (unchanged across a feed() = the result holds only deliveries)", nullptr},
    {nullptr, nullptr, nullptr, nullptr, nullptr}};

PyMethodDef demux_methods[] = {
    {"feed", reinterpret_cast<PyCFunction>(demux_feed), METH_O,
     "feed(bytes) -> list of Delivery | (frame_type, channel, payload)"},
    {"add_consumer", reinterpret_cast<PyCFunction>(demux_add_consumer), METH_VARARGS,
     "add_consumer(channel, consumer_tag, topic_id, extra)"},
    {"remove_consumer", reinterpret_cast<PyCFunction>(demux_remove_consumer), METH_VARARGS,
     "remove_consumer(channel, consumer_tag)"},
    {"reset_channel", reinterpret_cast<PyCFunction>(demux_reset_channel), METH_O, "reset_channel(channel)"},
    {"set_frame_max", reinterpret_cast<PyCFunction>(demux_set_frame_max), METH_O, "set_frame_max(n)"},
    {"stats", reinterpret_cast<PyCFunction>(demux_stats), METH_NOARGS, "counters"},
    {nullptr, nullptr, 0, nullptr}};

}  // namespace

PyTypeObject AmqpDemuxType = {PyVarObject_HEAD_INIT(nullptr, 0)};

int init_amqp_types(PyObject* m) {
  AmqpDemuxType.tp_name = "beholder_amd.ops._native.AmqpDemux";
  AmqpDemuxType.tp_basicsize = sizeof(AmqpDemuxObject);
  AmqpDemuxType.tp_flags = Py_TPFLAGS_DEFAULT | Py_TPFLAGS_HAVE_GC;
  AmqpDemuxType.tp_doc = "AmqpDemux(settler=None, frame_max=0): native basic.deliver assembly";
  AmqpDemuxType.tp_new = demux_new;
  AmqpDemuxType.tp_init = reinterpret_cast<initproc>(demux_init);
  AmqpDemuxType.tp_dealloc = reinterpret_cast<destructor>(demux_dealloc);
  AmqpDemuxType.tp_traverse = reinterpret_cast<traverseproc>(demux_traverse);
  AmqpDemuxType.tp_clear = reinterpret_cast<inquiry>(demux_clear);
  AmqpDemuxType.tp_methods = demux_methods;
  AmqpDemuxType.tp_getset = demux_getset;
  if (PyType_Ready(&AmqpDemuxType) < 0) return -1;
  Py_INCREF(&AmqpDemuxType);
  return PyModule_AddObject(m, "AmqpDemux", reinterpret_cast<PyObject*>(&AmqpDemuxType));
}

}  // namespace beholder
