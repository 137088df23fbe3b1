// SharedBroker: the competing-consumer AMQP broker fake of the shared-queue bench
// (bench/shared_queue.py, bench/replay_broker.py --shared --native), in C++.
//
// The Python SharedQueueBroker (replay_broker.py) is one asyncio process; at about 0.45 us of
// its CPU per event it saturated at 2.1-2.2M events/s, below what 8 workers consume, so the top
// of the shared-queue curve measured the fake. This one serves the same protocol subset from an
// epoll loop on its own thread (no GIL held), so the curve measures the consumers:
//
//   * AMQP 0-9-1 server side of what transport/amqp (AmqpSource) sends: the connection
//     handshake, channel.open, basic.qos, queue.declare, basic.consume, basic.ack (single and
//     `multiple`), basic.cancel, channel.close, connection.close; heartbeats and anything else
//     are ignored;
//   * one shared queue head over every connection that consumes all the queues (competing
//     consumers, index.js:43,62,127): delivery starts once `consumers` connections have
//     subscribed; each connection gets the next events while its window (prefetch x its
//     consumers) has room; delivery tags per channel; a connection that closes with deliveries
//     unacked has them requeued (redelivered), as RabbitMQ does;
//   * exactly-once accounting: every ack is mapped to the event it settles and counted per event
//     (`acked` = events acked at least once, `dup_acks`, `unknown_acks`, `lost` at the end);
//     the clock runs from the first delivery to the ack that settles the last event, and the
//     thread's CPU over that span is reported.
//
// Content (header + body frames for channel 1) comes pre-encoded from Python, as the Python
// broker pre-encodes it. Bench code: part of `_native_bench`, never of the service.
#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/epoll.h>
#include <sys/resource.h>
#include <sys/socket.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <cstring>
#include <deque>
#include <memory>
#include <new>
#include <string>
#include <unordered_map>
#include <vector>

#include "bench_common.hpp"

namespace beholder {
namespace bench {
namespace {

double thread_cpu_s() {
  timespec ts;
  clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts);
  return double(ts.tv_sec) + double(ts.tv_nsec) * 1e-9;
}

// ---- AMQP encoding helpers -------------------------------------------------------------------
void put8(std::string& o, uint8_t v) { o.push_back(char(v)); }
void put16(std::string& o, uint16_t v) {
  o.push_back(char(v >> 8));
  o.push_back(char(v));
}
void put32(std::string& o, uint32_t v) {
  for (int s = 24; s >= 0; s -= 8) o.push_back(char(v >> s));
}
void put64(std::string& o, uint64_t v) {
  for (int s = 56; s >= 0; s -= 8) o.push_back(char(v >> s));
}
void putshort(std::string& o, const std::string& s) {
  put8(o, uint8_t(s.size()));
  o += s;
}
uint16_t rd16(const uint8_t* p) { return uint16_t((p[0] << 8) | p[1]); }
uint32_t rd32(const uint8_t* p) { return (uint32_t(p[0]) << 24) | (uint32_t(p[1]) << 16) | (uint32_t(p[2]) << 8) | p[3]; }
uint64_t rd64(const uint8_t* p) { return (uint64_t(rd32(p)) << 32) | rd32(p + 4); }

// a method frame: type 1, channel, size, class, method, args, frame end
void method(std::string& o, uint16_t ch, uint16_t cls, uint16_t mth, const std::string& args) {
  put8(o, 1);
  put16(o, ch);
  put32(o, uint32_t(4 + args.size()));
  put16(o, cls);
  put16(o, mth);
  o += args;
  put8(o, 0xCE);
}

struct Conn {
  int fd = -1;
  std::string in;
  std::string out;
  size_t out_off = 0;
  bool got_header = false;
  uint16_t channel = 0;
  uint32_t prefetch = 0;
  std::unordered_map<int, std::string> consumers;  // queue index -> consumer tag
  bool subscribed = false;
  bool writable = true;  // false: waiting for EPOLLOUT
  std::vector<uint32_t> tags;      // tag - 1 -> event index
  std::vector<uint8_t> settled;    // tag - 1 -> settled on this channel
  size_t low = 0;                  // lowest unsettled tag - 1
  size_t open = 0;                 // deliveries not yet settled
  uint64_t delivered = 0;
  std::vector<std::string> pre;    // per queue: frame header + basic.deliver up to the tag
  std::vector<std::string> post[2];  // per queue, redelivered 0/1: the rest of the method frame
};

struct SharedBrokerObject {
  PyObject_HEAD std::string* content;  // concatenated content frames (channel 1)
  std::vector<uint64_t>* coff;         // event i: [coff[i], coff[i+1])
  std::vector<uint8_t>* qidx;          // event -> queue index
  std::vector<std::string>* qnames;
  int expected;
  int lfd;
  int efd;
  uint16_t port;
  // state (the loop thread's; counters read by stats() while it runs are atomic)
  std::vector<uint8_t>* ack_counts;
  std::deque<uint32_t>* requeue;
  uint64_t cursor;
  std::atomic<uint64_t> acked, sent, dup_acks, unknown_acks, redelivered, connections;
  std::atomic<bool> done, running, stop;
  int64_t t_first, t_done;
  double cpu_first, cpu_s;
  std::vector<uint64_t>* per_conn;  // deliveries per connection (in connection order)
  // the same, readable while the loop runs (stats() of a broker serving until stop()); the first
  // kLiveSlots connections only
  std::atomic<uint64_t>* per_conn_live;
};

constexpr size_t kLiveSlots = 4096;

PyTypeObject SharedBrokerType = {PyVarObject_HEAD_INIT(nullptr, 0)};

// ---- the loop ----------------------------------------------------------------------------------
struct Loop {
  SharedBrokerObject* b;
  std::unordered_map<int, std::unique_ptr<Conn>> conns;
  std::unordered_map<int, size_t> slot_of;  // fd -> per_conn slot (order of arrival)
  bool go = false;
  int subscribed = 0;

  void add_acked(uint64_t k) {
    uint64_t a = b->acked.fetch_add(k) + k;
    if (a == b->coff->size() - 1 && !b->done.load()) {
      b->t_done = mono_ns();
      b->cpu_s = thread_cpu_s() - b->cpu_first;
      b->done.store(true);
    }
  }

  void settle(Conn& c, size_t t) {  // t = tag - 1
    if (t >= c.tags.size() || c.settled[t]) {
      b->unknown_acks.fetch_add(1);
      return;
    }
    c.settled[t] = 1;
    --c.open;
    uint32_t idx = c.tags[t];
    uint8_t n = (*b->ack_counts)[idx];
    if (n) {
      b->dup_acks.fetch_add(1);
    } else {
      add_acked(1);
    }
    if (n < 255) (*b->ack_counts)[idx] = uint8_t(n + 1);
  }

  void on_ack(Conn& c, uint64_t tag, bool multiple) {
    if (multiple) {
      size_t upto = size_t(tag);
      if (upto > c.tags.size()) {
        b->unknown_acks.fetch_add(1);
        upto = c.tags.size();
      }
      uint64_t fresh = 0;
      std::vector<uint8_t>& counts = *b->ack_counts;
      for (size_t t = c.low; t < upto; ++t) {
        if (c.settled[t]) continue;
        c.settled[t] = 1;
        --c.open;
        uint32_t idx = c.tags[t];
        uint8_t n = counts[idx];
        if (n) {
          b->dup_acks.fetch_add(1);
        } else {
          ++fresh;
        }
        if (n < 255) counts[idx] = uint8_t(n + 1);
      }
      if (fresh) add_acked(fresh);
    } else {
      settle(c, size_t(tag) - 1);
    }
    while (c.low < c.settled.size() && c.settled[c.low]) ++c.low;
  }

  void build_prefixes(Conn& c) {
    const auto& names = *b->qnames;
    c.pre.assign(names.size(), std::string());
    c.post[0].assign(names.size(), std::string());
    c.post[1].assign(names.size(), std::string());
    for (size_t q = 0; q < names.size(); ++q) {
      auto it = c.consumers.find(int(q));
      const std::string& ctag = it->second;
      const std::string& rk = names[q];
      uint32_t size = uint32_t(4 + 1 + ctag.size() + 8 + 1 + 1 + 1 + rk.size());
      std::string& p = c.pre[q];
      put8(p, 1);
      put16(p, c.channel);
      put32(p, size);
      put16(p, 60);
      put16(p, 60);  // basic.deliver
      putshort(p, ctag);
      for (int rd = 0; rd < 2; ++rd) {
        std::string& s = c.post[rd][q];
        put8(s, uint8_t(rd));  // redelivered
        putshort(s, "");       // exchange: the default one
        putshort(s, rk);       // routing key = queue name
        put8(s, 0xCE);
      }
    }
  }

  // Methods from the client. false: close the connection.
  bool on_method(Conn& c, uint16_t ch, const uint8_t* p, size_t n) {
    if (n < 4) return false;
    uint16_t cls = rd16(p), mth = rd16(p + 2);
    const uint8_t* a = p + 4;
    size_t an = n - 4;
    std::string args;
    if (cls == 60 && mth == 80) {  // basic.ack
      if (an < 9) return false;
      on_ack(c, rd64(a), (a[8] & 1) != 0);
      return true;
    }
    if (cls == 10 && mth == 11) {  // connection.start_ok -> tune
      put16(args, 2047);
      put32(args, 131072);
      put16(args, 0);
      method(c.out, 0, 10, 30, args);
    } else if (cls == 10 && mth == 40) {  // connection.open -> open_ok
      putshort(args, "");
      method(c.out, 0, 10, 41, args);
    } else if (cls == 20 && mth == 10) {  // channel.open -> open_ok
      c.channel = ch;
      put32(args, 0);
      method(c.out, ch, 20, 11, args);
    } else if (cls == 60 && mth == 10) {  // basic.qos
      if (an < 6) return false;
      c.prefetch = rd16(a + 4);
      method(c.out, ch, 60, 11, args);
    } else if (cls == 50 && mth == 10) {  // queue.declare -> declare_ok(queue, 0, 0)
      if (an < 3 || size_t(a[2]) + 3 > an) return false;
      std::string q(reinterpret_cast<const char*>(a + 3), a[2]);
      putshort(args, q);
      put32(args, 0);
      put32(args, 0);
      method(c.out, ch, 50, 11, args);
    } else if (cls == 60 && mth == 20) {  // basic.consume -> consume_ok
      if (an < 3) return false;
      size_t ql = a[2];
      if (3 + ql + 1 > an) return false;
      std::string q(reinterpret_cast<const char*>(a + 3), ql);
      size_t tl = a[3 + ql];
      if (4 + ql + tl > an) return false;
      std::string tag(reinterpret_cast<const char*>(a + 4 + ql), tl);
      putshort(args, tag);
      method(c.out, ch, 60, 21, args);
      const auto& names = *b->qnames;
      for (size_t i = 0; i < names.size(); ++i)
        if (names[i] == q) c.consumers[int(i)] = tag;
      if (!c.subscribed && c.consumers.size() == names.size()) {
        if (c.channel != 1) return false;  // content frames are pre-encoded for channel 1
        c.subscribed = true;
        build_prefixes(c);
        if (++subscribed >= b->expected) go = true;
      }
    } else if (cls == 60 && mth == 30) {  // basic.cancel -> cancel_ok
      if (an < 1 || size_t(a[0]) + 1 > an) return false;
      std::string tag(reinterpret_cast<const char*>(a + 1), a[0]);
      putshort(args, tag);
      method(c.out, ch, 60, 31, args);
    } else if (cls == 20 && mth == 40) {  // channel.close -> close_ok
      method(c.out, ch, 20, 41, args);
    } else if (cls == 10 && mth == 50) {  // connection.close -> close_ok, then close
      method(c.out, 0, 10, 51, args);
      flush(c);
      return false;
    }
    return true;
  }

  // Parses every complete frame in c.in. false: close the connection.
  bool on_input(Conn& c) {
    size_t i = 0;
    const uint8_t* d = reinterpret_cast<const uint8_t*>(c.in.data());
    size_t n = c.in.size();
    if (!c.got_header) {
      if (n < 8) return true;
      if (memcmp(d, "AMQP", 4) != 0) return false;
      c.got_header = true;
      i = 8;
      std::string args;  // connection.start(0, 9, {}, "PLAIN", "en_US")
      put8(args, 0);
      put8(args, 9);
      put32(args, 0);
      put32(args, 5);
      args += "PLAIN";
      put32(args, 5);
      args += "en_US";
      method(c.out, 0, 10, 10, args);
    }
    while (n - i >= 8) {
      uint8_t type = d[i];
      uint16_t ch = rd16(d + i + 1);
      uint32_t size = rd32(d + i + 3);
      if (size > (64u << 20)) return false;
      if (n - i < size_t(size) + 8) break;
      if (d[i + 7 + size] != 0xCE) return false;
      if (type == 1 && !on_method(c, ch, d + i + 7, size)) {
        c.in.erase(0, i + 8 + size);
        return false;
      }
      i += size_t(size) + 8;
    }
    c.in.erase(0, i);
    return true;
  }

  // Deliveries into c.out while the window has room.
  void pump(Conn& c) {
    if (!go || !c.subscribed || b->done.load()) return;
    const std::string& content = *b->content;
    const auto& coff = *b->coff;
    const auto& qidx = *b->qidx;
    const size_t total = coff.size() - 1;
    size_t window = c.prefetch ? size_t(c.prefetch) * c.consumers.size() : 512;
    while (c.open < window && c.out.size() - c.out_off < (1u << 20)) {
      uint32_t idx;
      bool rd = false;
      if (!b->requeue->empty()) {
        idx = b->requeue->front();
        b->requeue->pop_front();
        rd = true;
      } else if (b->cursor < total) {
        idx = uint32_t(b->cursor++);
      } else {
        break;
      }
      if (!b->t_first) {
        b->t_first = mono_ns();
        b->cpu_first = thread_cpu_s();
      }
      int q = qidx[idx];
      c.tags.push_back(idx);
      c.settled.push_back(0);
      c.out += c.pre[q];
      put64(c.out, c.tags.size());
      c.out += c.post[rd][q];
      c.out.append(content, coff[idx], coff[idx + 1] - coff[idx]);
      ++c.open;
      ++c.delivered;
      b->sent.fetch_add(1);
      if (rd) b->redelivered.fetch_add(1);
    }
  }

  // Sends what is buffered. false: the connection failed.
  bool flush(Conn& c) {
    while (c.out_off < c.out.size()) {
      ssize_t w = ::send(c.fd, c.out.data() + c.out_off, c.out.size() - c.out_off, MSG_NOSIGNAL);
      if (w < 0) {
        if (errno == EINTR) continue;
        if (errno == EAGAIN || errno == EWOULDBLOCK) {
          if (c.writable) {
            c.writable = false;
            epoll_event ev{};
            ev.events = EPOLLIN | EPOLLOUT;
            ev.data.fd = c.fd;
            epoll_ctl(b->efd, EPOLL_CTL_MOD, c.fd, &ev);
          }
          return true;
        }
        return false;
      }
      c.out_off += size_t(w);
    }
    c.out.clear();
    c.out_off = 0;
    if (!c.writable) {
      c.writable = true;
      epoll_event ev{};
      ev.events = EPOLLIN;
      ev.data.fd = c.fd;
      epoll_ctl(b->efd, EPOLL_CTL_MOD, c.fd, &ev);
    }
    return true;
  }

  void drop(int fd) {
    auto it = conns.find(fd);
    if (it == conns.end()) return;
    Conn& c = *it->second;
    // un-acked deliveries back to the head, redelivered (RabbitMQ's requeue on close)
    for (size_t t = c.low; t < c.tags.size(); ++t)
      if (!c.settled[t] && !(*b->ack_counts)[c.tags[t]]) b->requeue->push_back(c.tags[t]);
    (*b->per_conn)[slot_of[fd]] = c.delivered;
    if (slot_of[fd] < kLiveSlots) b->per_conn_live[slot_of[fd]].store(c.delivered, std::memory_order_relaxed);
    epoll_ctl(b->efd, EPOLL_CTL_DEL, fd, nullptr);
    ::close(fd);
    conns.erase(it);
  }

  void accept_all() {
    for (;;) {
      int fd = ::accept4(b->lfd, nullptr, nullptr, SOCK_NONBLOCK | SOCK_CLOEXEC);
      if (fd < 0) return;
      int one = 1;
      setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
      epoll_event ev{};
      ev.events = EPOLLIN;
      ev.data.fd = fd;
      epoll_ctl(b->efd, EPOLL_CTL_ADD, fd, &ev);
      auto c = std::make_unique<Conn>();
      c->fd = fd;
      slot_of[fd] = b->per_conn->size();
      b->per_conn->push_back(0);
      b->connections.fetch_add(1);
      conns[fd] = std::move(c);
    }
  }

  void run(double linger_s) {  // linger_s < 0: serve until stop() (done or not)
    std::vector<epoll_event> evs(256);
    std::vector<char> buf(1 << 17);
    int64_t linger_until = 0;
    while (!b->stop.load()) {
      if (b->done.load() && linger_s >= 0) {
        if (!linger_until) linger_until = mono_ns() + int64_t(linger_s * 1e9);
        if (mono_ns() >= linger_until) break;
      }
      int timeout = b->done.load() ? 10 : 100;  // stop() is seen within one timeout
      int k = epoll_wait(b->efd, evs.data(), int(evs.size()), timeout);
      if (k < 0) {
        if (errno == EINTR) continue;
        break;
      }
      for (int e = 0; e < k; ++e) {
        int fd = evs[size_t(e)].data.fd;
        if (fd == b->lfd) {
          accept_all();
          continue;
        }
        auto it = conns.find(fd);
        if (it == conns.end()) continue;
        Conn& c = *it->second;
        bool ok = true;
        if (evs[size_t(e)].events & (EPOLLERR | EPOLLHUP)) ok = false;
        if (ok && (evs[size_t(e)].events & EPOLLIN)) {
          for (;;) {
            ssize_t r = ::recv(fd, buf.data(), buf.size(), 0);
            if (r > 0) {
              c.in.append(buf.data(), size_t(r));
              if (size_t(r) < buf.size()) break;
              continue;
            }
            if (r == 0) ok = false;
            else if (errno != EAGAIN && errno != EWOULDBLOCK && errno != EINTR) ok = false;
            break;
          }
          if (ok) ok = on_input(c);
        }
        if (ok && (evs[size_t(e)].events & EPOLLOUT)) ok = flush(c);
        if (!ok) drop(fd);
      }
      // deliveries for every connection with room, then one send each
      std::vector<int> dead;
      for (auto& kv : conns) {
        Conn& c = *kv.second;
        pump(c);
        size_t slot = slot_of[kv.first];
        if (slot < kLiveSlots) b->per_conn_live[slot].store(c.delivered, std::memory_order_relaxed);
        if (c.writable && c.out.size() > c.out_off && !flush(c)) dead.push_back(kv.first);
      }
      for (int fd : dead) drop(fd);
    }
    for (auto& kv : conns) (*b->per_conn)[slot_of[kv.first]] = kv.second->delivered;
  }
};

// ---- Python type -----------------------------------------------------------------------------
PyObject* sb_new(PyTypeObject* type, PyObject*, PyObject*) {
  SharedBrokerObject* s = reinterpret_cast<SharedBrokerObject*>(type->tp_alloc(type, 0));
  if (!s) return nullptr;
  s->lfd = s->efd = -1;
  new (&s->acked) std::atomic<uint64_t>(0);
  new (&s->sent) std::atomic<uint64_t>(0);
  new (&s->dup_acks) std::atomic<uint64_t>(0);
  new (&s->unknown_acks) std::atomic<uint64_t>(0);
  new (&s->redelivered) std::atomic<uint64_t>(0);
  new (&s->connections) std::atomic<uint64_t>(0);
  new (&s->done) std::atomic<bool>(false);
  new (&s->running) std::atomic<bool>(false);
  new (&s->stop) std::atomic<bool>(false);
  s->content = new (std::nothrow) std::string();
  s->coff = new (std::nothrow) std::vector<uint64_t>();
  s->qidx = new (std::nothrow) std::vector<uint8_t>();
  s->qnames = new (std::nothrow) std::vector<std::string>();
  s->ack_counts = new (std::nothrow) std::vector<uint8_t>();
  s->requeue = new (std::nothrow) std::deque<uint32_t>();
  s->per_conn = new (std::nothrow) std::vector<uint64_t>();
  s->per_conn_live = new (std::nothrow) std::atomic<uint64_t>[kLiveSlots]();
  if (!s->content || !s->coff || !s->qidx || !s->qnames || !s->ack_counts || !s->requeue || !s->per_conn ||
      !s->per_conn_live) {
    Py_DECREF(s);
    return PyErr_NoMemory();
  }
  return reinterpret_cast<PyObject*>(s);
}

void sb_dealloc(SharedBrokerObject* s) {
  for (int fd : {s->lfd, s->efd})
    if (fd >= 0) ::close(fd);
  delete s->content;
  delete s->coff;
  delete s->qidx;
  delete s->qnames;
  delete s->ack_counts;
  delete s->requeue;
  delete s->per_conn;
  delete[] s->per_conn_live;
  Py_TYPE(s)->tp_free(reinterpret_cast<PyObject*>(s));
}

// SharedBroker(content: bytes, offsets: bytes (u64, n+1), queues: bytes (u8, n), queue_names, consumers)
int sb_init(SharedBrokerObject* s, PyObject* args, PyObject*) {
  Py_buffer content, offs, qs;
  PyObject* names;
  int consumers;
  if (!PyArg_ParseTuple(args, "y*y*y*Oi", &content, &offs, &qs, &names, &consumers)) return -1;
  int rc = -1;
  try {
    size_t n = size_t(qs.len);
    if (offs.len % 8 != 0 || size_t(offs.len) / 8 != n + 1 || consumers < 1) {
      PyErr_SetString(PyExc_ValueError, "SharedBroker: offsets must be n+1 u64, queues n u8, consumers >= 1");
    } else {
      const uint64_t* o = static_cast<const uint64_t*>(offs.buf);
      bool ok = o[0] == 0 && o[n] == uint64_t(content.len);
      for (size_t i = 0; ok && i < n; ++i) ok = o[i] <= o[i + 1];
      PyObject* seq = ok ? PySequence_Tuple(names) : nullptr;
      if (!ok) {
        PyErr_SetString(PyExc_ValueError, "SharedBroker: offsets must rise from 0 to len(content)");
      } else if (seq) {
        s->qnames->clear();
        for (Py_ssize_t i = 0; i < PyTuple_GET_SIZE(seq); ++i) {
          Py_ssize_t ln;
          const char* t = PyUnicode_AsUTF8AndSize(PyTuple_GET_ITEM(seq, i), &ln);
          if (!t || ln > 255) {
            if (t) PyErr_SetString(PyExc_ValueError, "SharedBroker: queue name too long");
            ok = false;
            break;
          }
          s->qnames->emplace_back(t, size_t(ln));
        }
        Py_DECREF(seq);
        const uint8_t* q = static_cast<const uint8_t*>(qs.buf);
        for (size_t i = 0; ok && i < n; ++i)
          if (q[i] >= s->qnames->size()) {
            PyErr_SetString(PyExc_ValueError, "SharedBroker: queue index out of range");
            ok = false;
          }
        if (ok) {
          s->content->assign(static_cast<const char*>(content.buf), size_t(content.len));
          s->coff->assign(o, o + n + 1);
          s->qidx->assign(q, q + n);
          s->ack_counts->assign(n, 0);
          s->expected = consumers;
          rc = 0;
        }
      }
    }
  } catch (const std::bad_alloc&) {
    PyErr_NoMemory();
  }
  PyBuffer_Release(&content);
  PyBuffer_Release(&offs);
  PyBuffer_Release(&qs);
  return rc;
}

// listen() -> port (127.0.0.1, ephemeral)
PyObject* sb_listen(SharedBrokerObject* s, PyObject*) {
  if (s->lfd >= 0) return PyLong_FromLong(s->port);
  int fd = ::socket(AF_INET, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
  if (fd < 0) return PyErr_SetFromErrno(PyExc_OSError);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  socklen_t al = sizeof(a);
  if (::bind(fd, reinterpret_cast<sockaddr*>(&a), sizeof(a)) < 0 || ::listen(fd, 256) < 0 ||
      getsockname(fd, reinterpret_cast<sockaddr*>(&a), &al) < 0) {
    int e = errno;
    ::close(fd);
    errno = e;
    return PyErr_SetFromErrno(PyExc_OSError);
  }
  int efd = epoll_create1(EPOLL_CLOEXEC);
  if (efd < 0) {
    ::close(fd);
    return PyErr_SetFromErrno(PyExc_OSError);
  }
  epoll_event ev{};
  ev.events = EPOLLIN;
  ev.data.fd = fd;
  epoll_ctl(efd, EPOLL_CTL_ADD, fd, &ev);
  s->lfd = fd;
  s->efd = efd;
  s->port = ntohs(a.sin_port);
  return PyLong_FromLong(s->port);
}

// run(linger_s=0.2): serves until every event is acked (then `linger_s` more, so late duplicate
// acks are counted) or stop(); linger_s < 0: until stop() only (a consumer that connects after the
// last ack still gets its session). Blocks without the GIL.
PyObject* sb_run(SharedBrokerObject* s, PyObject* args) {
  double linger = 0.2;
  if (!PyArg_ParseTuple(args, "|d", &linger)) return nullptr;
  if (s->lfd < 0) {
    PyErr_SetString(PyExc_RuntimeError, "SharedBroker.run() before listen()");
    return nullptr;
  }
  if (s->running.exchange(true)) {
    PyErr_SetString(PyExc_RuntimeError, "SharedBroker.run() is already running");
    return nullptr;
  }
  bool oom = false;
  Py_INCREF(s);
  Py_BEGIN_ALLOW_THREADS
  try {
    Loop loop{s};
    loop.run(linger);
  } catch (const std::bad_alloc&) {
    oom = true;
  }
  Py_END_ALLOW_THREADS
  s->running.store(false);
  Py_DECREF(s);
  if (oom) return PyErr_NoMemory();
  Py_RETURN_NONE;
}

PyObject* sb_stop(SharedBrokerObject* s, PyObject*) {
  s->stop.store(true);
  Py_RETURN_NONE;
}

// stats() -> dict; safe while run() is going (per-connection counts then from the live slots,
// `lost` = events not acked yet)
PyObject* sb_stats(SharedBrokerObject* s, PyObject*) {
  uint64_t lost = 0;
  bool finished = !s->running.load();
  const uint64_t published = s->coff->size() - 1, acked_now = s->acked.load();  // a snapshot
  if (finished)
    for (uint8_t c : *s->ack_counts) lost += c == 0;
  else
    lost = published - acked_now;  // events not acked yet (acked counts each event once)
  PyObject* per = PyList_New(0);
  if (!per) return nullptr;
  const size_t nconn = size_t(s->connections.load());
  const size_t nper = finished ? s->per_conn->size() : (nconn < kLiveSlots ? nconn : kLiveSlots);
  for (size_t i = 0; i < nper; ++i) {
    uint64_t v = finished ? (*s->per_conn)[i] : s->per_conn_live[i].load(std::memory_order_relaxed);
    PyObject* x = PyLong_FromUnsignedLongLong(v);
    if (!x || PyList_Append(per, x) < 0) {
      Py_XDECREF(x);
      Py_DECREF(per);
      return nullptr;
    }
    Py_DECREF(x);
  }
  // t_first / t_done / cpu_s are written by the loop thread before it sets `done`
  const bool done = s->done.load();
  double span = done && s->t_first ? double(s->t_done - s->t_first) * 1e-9 : 0.0;
  double cpu = done ? s->cpu_s : 0.0;
  return Py_BuildValue("{s:K,s:K,s:K,s:K,s:K,s:K,s:K,s:K,s:N,s:d,s:d,s:O,s:O}", "published",
                       (unsigned long long)(s->coff->size() - 1), "sent", (unsigned long long)s->sent.load(), "acked",
                       (unsigned long long)s->acked.load(), "dup_acks", (unsigned long long)s->dup_acks.load(),
                       "unknown_acks", (unsigned long long)s->unknown_acks.load(), "redelivered",
                       (unsigned long long)s->redelivered.load(), "connections",
                       (unsigned long long)s->connections.load(), "lost", (unsigned long long)lost,
                       "per_conn", per, "broker_s", span, "cpu_s", cpu, "done", done ? Py_True : Py_False,
                       "finished", finished ? Py_True : Py_False);
}

PyMethodDef sb_methods[] = {
    {"listen", reinterpret_cast<PyCFunction>(sb_listen), METH_NOARGS, "listen() -> port (127.0.0.1)"},
    {"run", reinterpret_cast<PyCFunction>(sb_run), METH_VARARGS,
     "run(linger_s=0.2): serve until every event is acked (+ linger; < 0: until stop()) or stop(); releases the GIL"},
    {"stop", reinterpret_cast<PyCFunction>(sb_stop), METH_NOARGS, "stop(): make run() return"},
    {"stats", reinterpret_cast<PyCFunction>(sb_stats), METH_NOARGS, "stats() -> dict"},
    {nullptr, nullptr, 0, nullptr}};

}  // namespace

int init_shared_broker(PyObject* m) {
  SharedBrokerType.tp_name = "beholder_amd.ops._native_bench.SharedBroker";
  SharedBrokerType.tp_basicsize = sizeof(SharedBrokerObject);
  SharedBrokerType.tp_flags = Py_TPFLAGS_DEFAULT;
  SharedBrokerType.tp_doc =
      "SharedBroker(content, offsets, queues, queue_names, consumers): competing-consumer AMQP broker fake "
      "(bench/shared_queue.py)";
  SharedBrokerType.tp_new = sb_new;
  SharedBrokerType.tp_init = reinterpret_cast<initproc>(sb_init);
  SharedBrokerType.tp_dealloc = reinterpret_cast<destructor>(sb_dealloc);
  SharedBrokerType.tp_methods = sb_methods;
  if (PyType_Ready(&SharedBrokerType) < 0) return -1;
  Py_INCREF(&SharedBrokerType);
  if (PyModule_AddObject(m, "SharedBroker", reinterpret_cast<PyObject*>(&SharedBrokerType)) < 0) return -1;
  return 0;
}

}  // namespace bench
}  // namespace beholder
