// PgFake: the Postgres stand-in of the production-shaped bench (`tcp_e2e` / `tls_e2e`,
// bench/pg_sink_server.py), in C++.
//
// The asyncio fake costs about 5 us of its CPU per query. Two copies share the port with
// SO_REUSEPORT, and the kernel spreads the consumer's 4 pool connections over them by a hash of
// the 4-tuple: a 2/2 split left each copy ~70% busy, a 3/1 split one copy ~90%, and a 4/0 split
// one copy at 98%, which then capped the run (225k events/s and half the events per loop turn
// in the consumer, against 265k; profiles/box_r5_util/). So the e2e numbers partly measured the
// fake. This one serves the same protocol subset from one epoll loop on its own thread (no GIL
// held) at a fraction of that cost, so the run measures the consumer:
//
//   * startup: an SSLRequest is refused ('N', as the asyncio fake), any other startup message
//     gets trust auth (AuthenticationOk, server_version, BackendKeyData, ReadyForQuery);
//   * the extended protocol with pipelined Sync groups: Parse (the statement is classified as
//     the media SELECT by id, the status UPDATE, or other), Bind (text parameters), Describe
//     (RowDescription of the ten media columns / NoData), Execute (a DataRow + CommandComplete;
//     other statements fail with an ErrorResponse that skips to the next Sync), Sync, Terminate;
//   * the table is the synthetic media population the stream was generated from (rows given as
//     text columns), with the UPDATE applied to the status column.
//
// Busy spells of the loop longer than a threshold are kept as stall intervals (CLOCK_MONOTONIC,
// the clock of the deliveries' timestamps), so the bench's slow-delivery attribution can still
// blame this process. Bench code: part of `_native_bench`, never of the service.
#include <arpa/inet.h>
#include <errno.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/epoll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cctype>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <new>
#include <string>
#include <unordered_map>
#include <vector>

#include "bench_common.hpp"

namespace beholder {
namespace bench {
namespace {

constexpr int kCols = 10;
constexpr int kStatusCol = 9;
const char* const kColNames[kCols] = {"id",     "name",       "creator", "creator_id",  "type",
                                      "source", "source_uri", "metadata", "metadata_id", "status"};
const bool kIntCol[kCols] = {false, false, true, false, true, true, false, true, false, true};

void put16(std::string& o, uint16_t v) {
  o.push_back(char(v >> 8));
  o.push_back(char(v));
}
void put32(std::string& o, uint32_t v) {
  for (int s = 24; s >= 0; s -= 8) o.push_back(char(v >> s));
}
uint16_t rd16(const uint8_t* p) { return uint16_t((p[0] << 8) | p[1]); }
uint32_t rd32(const uint8_t* p) { return (uint32_t(p[0]) << 24) | (uint32_t(p[1]) << 16) | (uint32_t(p[2]) << 8) | p[3]; }

// One backend message: type, length (itself included), body.
void msg(std::string& o, char type, const std::string& body) {
  o.push_back(type);
  put32(o, uint32_t(body.size() + 4));
  o += body;
}

struct Row {
  std::string cols[kCols];
  std::string data_row;  // the encoded DataRow, rebuilt when the status changes
  void encode() {
    std::string b;
    put16(b, kCols);
    for (const std::string& c : cols) {
      put32(b, uint32_t(c.size()));
      b += c;
    }
    data_row.clear();
    msg(data_row, 'D', b);
  }
};

enum Kind : uint8_t { K_OTHER = 0, K_SELECT = 1, K_UPDATE = 2 };

struct Conn {
  int fd = -1;
  bool started = false;
  bool failed = false;  // an error: skip to the next Sync
  bool writable = true;
  Kind kind = K_OTHER;
  std::unordered_map<std::string, Kind> stmts;
  std::vector<std::string> params;
  std::string in, out;
  size_t out_off = 0;
};

struct PgFakeObject {
  PyObject_HEAD int lfd;
  int efd;
  int port;
  int64_t stall_ns;  // a busy spell at least this long is a stall
  std::unordered_map<std::string, Row>* table;
  std::string* rowdesc;
  std::string* auth_ok;
  std::vector<std::pair<int64_t, int64_t>>* stalls;  // written by the loop; read after run()
  std::atomic<uint64_t> queries, connections, batches;
  std::atomic<int64_t> max_busy_ns;
  std::atomic<bool> running, stop;
};

PyTypeObject PgFakeType = {PyVarObject_HEAD_INIT(nullptr, 0)};

// The statement's kind, as the asyncio fake classifies it: upper-cased, quotes dropped.
Kind classify(const char* q, size_t n) {
  std::string s;
  s.reserve(n);
  for (size_t i = 0; i < n; ++i)
    if (q[i] != '"') s.push_back(char(std::toupper(static_cast<unsigned char>(q[i]))));
  size_t a = s.find_first_not_of(" \t\r\n");
  if (a == std::string::npos) return K_OTHER;
  if (s.compare(a, 6, "SELECT") == 0 && s.find("WHERE ID = $1") != std::string::npos) return K_SELECT;
  if (s.compare(a, 6, "UPDATE") == 0 && s.find("SET STATUS = $1") != std::string::npos) return K_UPDATE;
  return K_OTHER;
}

struct Loop {
  PgFakeObject* f;
  std::unordered_map<int, std::unique_ptr<Conn>> conns;

  // Parses what `c` sent; appends the replies to c.out. false: close the connection.
  bool on_input(Conn& c) {
    const uint8_t* b = reinterpret_cast<const uint8_t*>(c.in.data());
    size_t n = c.in.size(), i = 0;
    while (!c.started) {
      if (n - i < 8) break;
      uint32_t ln = rd32(b + i);
      if (ln < 8 || ln > (1u << 20)) return false;
      if (n - i < ln) break;
      uint32_t code = rd32(b + i + 4);
      i += ln;
      if (code == 80877103) {  // SSLRequest: refused, a plain startup follows
        c.out.push_back('N');
        continue;
      }
      c.started = true;
      c.out += *f->auth_ok;
    }
    while (c.started && n - i >= 5) {
      char t = char(b[i]);
      uint32_t ln = rd32(b + i + 1);
      if (ln < 4 || ln > (64u << 20)) return false;
      if (n - i - 1 < ln) break;
      const uint8_t* body = b + i + 5;
      size_t bn = ln - 4;
      i += 1 + ln;
      if (t == 'S') {
        c.failed = false;
        msg(c.out, 'Z', "I");
        continue;
      }
      if (t == 'X') return false;
      if (c.failed) continue;
      if (t == 'P') {
        const char* nm = reinterpret_cast<const char*>(body);
        size_t l1 = strnlen(nm, bn);
        if (l1 >= bn) return false;
        const char* q = nm + l1 + 1;
        size_t l2 = strnlen(q, bn - l1 - 1);
        c.stmts[std::string(nm, l1)] = classify(q, l2);
        msg(c.out, '1', "");
      } else if (t == 'B') {
        const char* portal = reinterpret_cast<const char*>(body);
        size_t l1 = strnlen(portal, bn);
        if (l1 >= bn) return false;
        const char* st = portal + l1 + 1;
        size_t rest = bn - l1 - 1, l2 = strnlen(st, rest);
        if (l2 >= rest) return false;
        auto it = c.stmts.find(std::string(st, l2));
        c.kind = it == c.stmts.end() ? K_OTHER : it->second;
        size_t j = l1 + 1 + l2 + 1;
        if (j + 2 > bn) return false;
        size_t nf = rd16(body + j);
        j += 2 + 2 * nf;
        if (j + 2 > bn) return false;
        size_t np = rd16(body + j);
        j += 2;
        c.params.clear();
        for (size_t k = 0; k < np; ++k) {
          if (j + 4 > bn) return false;
          int32_t pl = int32_t(rd32(body + j));
          j += 4;
          if (pl < 0) {
            c.params.emplace_back();
            continue;
          }
          if (j + size_t(pl) > bn) return false;
          c.params.emplace_back(reinterpret_cast<const char*>(body + j), size_t(pl));
          j += size_t(pl);
        }
        msg(c.out, '2', "");
      } else if (t == 'D') {
        if (c.kind == K_SELECT)
          c.out += *f->rowdesc;
        else
          msg(c.out, 'n', "");
      } else if (t == 'E') {
        f->queries.fetch_add(1, std::memory_order_relaxed);
        if (c.kind == K_SELECT && !c.params.empty()) {
          auto it = f->table->find(c.params[0]);
          if (it != f->table->end()) c.out += it->second.data_row;
          msg(c.out, 'C', it != f->table->end() ? std::string("SELECT 1", 9) : std::string("SELECT 0", 9));
        } else if (c.kind == K_UPDATE && c.params.size() >= 2) {
          auto it = f->table->find(c.params[1]);
          if (it != f->table->end()) {
            it->second.cols[kStatusCol] = std::to_string(std::strtoll(c.params[0].c_str(), nullptr, 10));
            it->second.encode();
          }
          msg(c.out, 'C', it != f->table->end() ? std::string("UPDATE 1", 9) : std::string("UPDATE 0", 9));
        } else {
          msg(c.out, 'E', std::string("SERROR\0C0A000\0Mbench endpoint: unsupported statement\0", 54));
          c.failed = true;
        }
      }
      // anything else (Flush, Close, ...) needs no reply here
    }
    c.in.erase(0, i);
    return true;
  }

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
            epoll_ctl(f->efd, EPOLL_CTL_MOD, c.fd, &ev);
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
      epoll_ctl(f->efd, EPOLL_CTL_MOD, c.fd, &ev);
    }
    return true;
  }

  void drop(int fd) {
    epoll_ctl(f->efd, EPOLL_CTL_DEL, fd, nullptr);
    ::close(fd);
    conns.erase(fd);
  }

  void accept_all() {
    for (;;) {
      int fd = ::accept4(f->lfd, nullptr, nullptr, SOCK_NONBLOCK | SOCK_CLOEXEC);
      if (fd < 0) return;
      int one = 1;
      setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
      epoll_event ev{};
      ev.events = EPOLLIN;
      ev.data.fd = fd;
      epoll_ctl(f->efd, EPOLL_CTL_ADD, fd, &ev);
      auto c = std::make_unique<Conn>();
      c->fd = fd;
      conns[fd] = std::move(c);
      f->connections.fetch_add(1, std::memory_order_relaxed);
    }
  }

  void run() {
    std::vector<epoll_event> evs(256);
    std::vector<char> buf(1 << 17);
    while (!f->stop.load()) {
      int k = epoll_wait(f->efd, evs.data(), int(evs.size()), 50);  // stop() is seen within 50 ms
      if (k < 0) {
        if (errno == EINTR) continue;
        break;
      }
      if (k == 0) continue;
      const int64_t t0 = mono_ns();
      for (int e = 0; e < k; ++e) {
        int fd = evs[size_t(e)].data.fd;
        if (fd == f->lfd) {
          accept_all();
          continue;
        }
        auto it = conns.find(fd);
        if (it == conns.end()) continue;
        Conn& c = *it->second;
        bool ok = !(evs[size_t(e)].events & (EPOLLERR | EPOLLHUP)) || (evs[size_t(e)].events & EPOLLIN);
        if (ok && (evs[size_t(e)].events & EPOLLIN)) {
          for (;;) {
            ssize_t r = ::recv(fd, buf.data(), buf.size(), 0);
            if (r > 0) {
              c.in.append(buf.data(), size_t(r));
              if (size_t(r) < buf.size()) break;
              continue;
            }
            if (r == 0)
              ok = false;
            else if (errno != EAGAIN && errno != EWOULDBLOCK && errno != EINTR)
              ok = false;
            break;
          }
          // replies to what arrived, even from a peer that has hung up after sending it
          bool parsed = on_input(c);
          if (c.out.size() > c.out_off && !flush(c)) ok = false;
          if (!parsed) ok = false;
        } else if (ok && (evs[size_t(e)].events & EPOLLOUT)) {
          ok = flush(c);
        }
        if (!ok) drop(fd);
      }
      const int64_t t1 = mono_ns(), busy = t1 - t0;
      f->batches.fetch_add(1, std::memory_order_relaxed);
      if (busy > f->max_busy_ns.load(std::memory_order_relaxed)) f->max_busy_ns.store(busy, std::memory_order_relaxed);
      if (busy >= f->stall_ns && f->stalls->size() < 100000) f->stalls->emplace_back(t0, t1);
    }
    for (auto& kv : conns) ::close(kv.first);
    conns.clear();
  }
};

// ---- Python type -----------------------------------------------------------------------------
PyObject* pf_new(PyTypeObject* type, PyObject*, PyObject*) {
  PgFakeObject* f = reinterpret_cast<PgFakeObject*>(type->tp_alloc(type, 0));
  if (!f) return nullptr;
  f->lfd = f->efd = -1;
  f->stall_ns = 1000000;
  new (&f->queries) std::atomic<uint64_t>(0);
  new (&f->connections) std::atomic<uint64_t>(0);
  new (&f->batches) std::atomic<uint64_t>(0);
  new (&f->max_busy_ns) std::atomic<int64_t>(0);
  new (&f->running) std::atomic<bool>(false);
  new (&f->stop) std::atomic<bool>(false);
  f->table = new (std::nothrow) std::unordered_map<std::string, Row>();
  f->rowdesc = new (std::nothrow) std::string();
  f->auth_ok = new (std::nothrow) std::string();
  f->stalls = new (std::nothrow) std::vector<std::pair<int64_t, int64_t>>();
  if (!f->table || !f->rowdesc || !f->auth_ok || !f->stalls) {
    Py_DECREF(f);
    return PyErr_NoMemory();
  }
  return reinterpret_cast<PyObject*>(f);
}

void pf_dealloc(PgFakeObject* f) {
  for (int fd : {f->lfd, f->efd})
    if (fd >= 0) ::close(fd);
  delete f->table;
  delete f->rowdesc;
  delete f->auth_ok;
  delete f->stalls;
  Py_TYPE(f)->tp_free(reinterpret_cast<PyObject*>(f));
}

// PgFake(rows, stall_us=1000): rows = sequences of the ten media columns, served as str(value)
// (as the asyncio fake does), keyed by column 0.
int pf_init(PgFakeObject* f, PyObject* args, PyObject* kwds) {
  static const char* kwlist[] = {"rows", "stall_us", nullptr};
  PyObject* rows;
  double stall_us = 1000.0;
  if (!PyArg_ParseTupleAndKeywords(args, kwds, "O|d", const_cast<char**>(kwlist), &rows, &stall_us)) return -1;
  PyObject* seq = PySequence_Fast(rows, "PgFake: rows must be a sequence");
  if (!seq) return -1;
  int rc = -1;
  try {
    f->table->clear();
    f->stall_ns = int64_t(stall_us * 1e3);
    bool ok = true;
    for (Py_ssize_t r = 0; ok && r < PySequence_Fast_GET_SIZE(seq); ++r) {
      PyObject* row = PySequence_Fast(PySequence_Fast_GET_ITEM(seq, r), "PgFake: a row must be a sequence");
      if (!row) {
        ok = false;
        break;
      }
      if (PySequence_Fast_GET_SIZE(row) != kCols) {
        PyErr_SetString(PyExc_ValueError, "PgFake: a row has the ten media columns");
        ok = false;
      }
      Row out;
      for (int i = 0; ok && i < kCols; ++i) {
        PyObject* s = PyObject_Str(PySequence_Fast_GET_ITEM(row, i));
        Py_ssize_t n;
        const char* t = s ? PyUnicode_AsUTF8AndSize(s, &n) : nullptr;
        if (t) out.cols[i].assign(t, size_t(n));
        Py_XDECREF(s);
        if (!t) ok = false;
      }
      Py_DECREF(row);
      if (ok) {
        out.encode();
        std::string key = out.cols[0];
        (*f->table)[key] = std::move(out);
      }
    }
    if (ok) {
      std::string b;
      put16(b, kCols);
      for (int i = 0; i < kCols; ++i) {
        b += kColNames[i];
        b.push_back('\0');
        put32(b, 0);                     // table oid
        put16(b, 0);                     // column number
        put32(b, kIntCol[i] ? 23 : 25);  // int4 / text
        put16(b, 0xFFFF);                // type size -1
        put32(b, 0xFFFFFFFF);            // type modifier -1
        put16(b, 0);                     // text format
      }
      f->rowdesc->clear();
      msg(*f->rowdesc, 'T', b);
      f->auth_ok->clear();
      std::string z;
      put32(z, 0);
      msg(*f->auth_ok, 'R', z);
      msg(*f->auth_ok, 'S', std::string("server_version\0" "16.0-bench\0", 26));
      std::string k;
      put32(k, 1);
      put32(k, 1);
      msg(*f->auth_ok, 'K', k);
      msg(*f->auth_ok, 'Z', "I");
      rc = 0;
    }
  } catch (const std::bad_alloc&) {
    PyErr_NoMemory();
  }
  Py_DECREF(seq);
  return rc;
}

// listen(port=0) -> port: 127.0.0.1, SO_REUSEPORT (copies may share the port, as the asyncio
// fake's do)
PyObject* pf_listen(PgFakeObject* f, PyObject* args) {
  int want = 0;
  if (!PyArg_ParseTuple(args, "|i", &want)) return nullptr;
  if (f->lfd >= 0) return PyLong_FromLong(f->port);
  if (want < 0 || want > 65535) {
    PyErr_SetString(PyExc_ValueError, "PgFake.listen: port out of range");
    return nullptr;
  }
  int fd = ::socket(AF_INET, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, IPPROTO_TCP);
  if (fd < 0) return PyErr_SetFromErrno(PyExc_OSError);
  int one = 1;
  setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  setsockopt(fd, SOL_SOCKET, SO_REUSEPORT, &one, sizeof(one));
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  a.sin_port = htons(uint16_t(want));
  socklen_t al = sizeof(a);
  if (::bind(fd, reinterpret_cast<sockaddr*>(&a), sizeof(a)) < 0 || ::listen(fd, 1024) < 0 ||
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
  f->lfd = fd;
  f->efd = efd;
  f->port = ntohs(a.sin_port);
  return PyLong_FromLong(f->port);
}

// run(): serves until stop(). Blocks without the GIL.
PyObject* pf_run(PgFakeObject* f, PyObject*) {
  if (f->lfd < 0) {
    PyErr_SetString(PyExc_RuntimeError, "PgFake.run() before listen()");
    return nullptr;
  }
  if (f->running.exchange(true)) {
    PyErr_SetString(PyExc_RuntimeError, "PgFake.run() is already running");
    return nullptr;
  }
  bool oom = false;
  Py_INCREF(f);
  Py_BEGIN_ALLOW_THREADS
  try {
    Loop loop{f, {}};
    loop.run();
  } catch (const std::bad_alloc&) {
    oom = true;
  }
  Py_END_ALLOW_THREADS
  f->running.store(false);
  Py_DECREF(f);
  if (oom) return PyErr_NoMemory();
  Py_RETURN_NONE;
}

PyObject* pf_stop(PgFakeObject* f, PyObject*) {
  f->stop.store(true);
  Py_RETURN_NONE;
}

// stats() -> {queries, connections, batches, max_busy_us, stall_intervals (once run() returned)}
PyObject* pf_stats(PgFakeObject* f, PyObject*) {
  PyObject* iv = PyList_New(0);
  if (!iv) return nullptr;
  if (!f->running.load())
    for (const auto& s : *f->stalls) {
      PyObject* p = Py_BuildValue("[LL]", (long long)s.first, (long long)s.second);
      if (!p || PyList_Append(iv, p) < 0) {
        Py_XDECREF(p);
        Py_DECREF(iv);
        return nullptr;
      }
      Py_DECREF(p);
    }
  return Py_BuildValue("{s:K,s:K,s:K,s:d,s:N}", "queries", (unsigned long long)f->queries.load(), "connections",
                       (unsigned long long)f->connections.load(), "batches", (unsigned long long)f->batches.load(),
                       "max_busy_us", double(f->max_busy_ns.load()) / 1e3, "stall_intervals", iv);
}

PyObject* pf_status_of(PgFakeObject* f, PyObject* key) {  // tests: the status column of a row
  if (f->running.load()) {
    PyErr_SetString(PyExc_RuntimeError, "PgFake.status_of() while running");
    return nullptr;
  }
  Py_ssize_t n;
  const char* k = PyUnicode_AsUTF8AndSize(key, &n);
  if (!k) return nullptr;
  auto it = f->table->find(std::string(k, size_t(n)));
  if (it == f->table->end()) Py_RETURN_NONE;
  const std::string& s = it->second.cols[kStatusCol];
  return PyUnicode_FromStringAndSize(s.data(), Py_ssize_t(s.size()));
}

PyMethodDef pf_methods[] = {
    {"listen", reinterpret_cast<PyCFunction>(pf_listen), METH_VARARGS, "listen(port=0) -> port (127.0.0.1)"},
    {"run", reinterpret_cast<PyCFunction>(pf_run), METH_NOARGS, "run(): serve until stop(); releases the GIL"},
    {"stop", reinterpret_cast<PyCFunction>(pf_stop), METH_NOARGS, "stop(): make run() return (within 50 ms)"},
    {"stats", reinterpret_cast<PyCFunction>(pf_stats), METH_NOARGS, "stats() -> dict"},
    {"status_of", reinterpret_cast<PyCFunction>(pf_status_of), METH_O, "status_of(id) -> str or None"},
    {nullptr, nullptr, 0, nullptr}};

}  // namespace

int init_pg_fake(PyObject* m) {
  PgFakeType.tp_name = "beholder_amd.ops._native_bench.PgFake";
  PgFakeType.tp_basicsize = sizeof(PgFakeObject);
  PgFakeType.tp_flags = Py_TPFLAGS_DEFAULT;
  PgFakeType.tp_doc = "PgFake(rows, stall_us=1000): the e2e bench's Postgres stand-in (bench/pg_sink_server.py)";
  PgFakeType.tp_new = pf_new;
  PgFakeType.tp_init = reinterpret_cast<initproc>(pf_init);
  PgFakeType.tp_dealloc = reinterpret_cast<destructor>(pf_dealloc);
  PgFakeType.tp_methods = pf_methods;
  if (PyType_Ready(&PgFakeType) < 0) return -1;
  Py_INCREF(&PgFakeType);
  if (PyModule_AddObject(m, "PgFake", reinterpret_cast<PyObject*>(&PgFakeType)) < 0) return -1;
  return 0;
}

}  // namespace bench
}  // namespace beholder
