// NetConn: a plain-TCP client socket driven straight from the asyncio loop, with the wire
// protocol handled here.
//
// The production path (every status event does up to 2 Postgres round trips
// and 3 HTTP requests, index.js:68,76,83,99,112; every progress event 1 + 1, index.js:53,140)
// spends most of its CPU in asyncio's Python-level transport machinery: per reply a
// `_read_ready` -> `_read_ready__data_received` -> `Protocol.data_received` chain, per request
// a `transport.write`. A NetConn replaces that for plain TCP connections once they are
// established (handshakes, TLS and authentication stay on asyncio transports):
//
//   c = NetConn(fd, loop, kind, owner, parser, ...)
//       the loop's selector calls c's bound on_readable for the fd (loop.add_reader): one
//       recv(2), the bytes fed to the native parser (H1Parser / PgReader), completed replies
//       resolve their IOFuture here (ops.IOFuture.resolve: a handler waiting through the
//       native Driver resumes in the same call).
//   c.write(data)          send(2) now; what the kernel does not take is kept and sent from
//                          on_writable (loop.add_writer), in order.
//
// kind "h1": one request in flight (HTTP/1.1 keep-alive, no pipelining):
//   c.request(data, waiter, head)   starts the parser, sets the waiter, writes the request.
// kind "pg": pipelined extended-protocol queries (store/pgwire.py semantics):
//   c.execute(sql, params) -> IOFuture   Parse (first use of sql on this connection) + Bind +
//                          Describe + Execute + Sync appended to the output, flushed once per
//                          loop iteration (loop.call_soon), replies matched FIFO.
//
// netconn_connect(ip, port, loop, kind, owner, parser, **kw) makes the TCP connection itself
// (non-blocking connect; `handshake` resolves once it is usable, after TLS when `tls=` is given),
// so an HTTP sink connection never has an asyncio transport at all.
//
// Rare paths call back into Python on `owner`: _net_lost(exc or None) when the peer closes or
// the socket fails (the fd is already closed and unregistered), _net_error(exc) for a protocol
// error or an unsolicited reply, _net_message(type, body) for out-of-band Postgres messages.
#include <errno.h>
#include <pthread.h>
#include <time.h>
#include <openssl/err.h>
#include <openssl/ssl.h>
#include <arpa/inet.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/epoll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <cstdlib>
#include <atomic>
#include <memory>
#include <deque>
#include <mutex>
#include <string>
#include <thread>

#include "hs_reactor.hpp"
#include "hs_wake.hpp"
#include "py_common.hpp"

namespace beholder {

PyObject* iofuture_new(PyObject* loop);
bool iofuture_done(PyObject* f);
int iofuture_resolve(PyObject* f, PyObject* v);
int iofuture_reject(PyObject* f, PyObject* exc);
int pg_bind_append(std::string& o, const char* name, size_t nlen, PyObject* params);
bool is_tls_context(PyObject* o);
PyObject* netpoll_for(PyObject* loop);
int netpoll_add(PyObject* po, int fd, PyObject* conn);
int netpoll_set_write(PyObject* po, int fd, bool write);
int netpoll_request_flush(PyObject* po, PyObject* conn);
void netpoll_del(PyObject* po, int fd);
SSL* tls_new_ssl(PyObject* ctx_obj, int fd, const char* host, int port);
void tls_count_handshake(SSL* ssl, bool offloaded);
int netpoll_pause(PyObject* po, int fd);
std::shared_ptr<HsWake> netpoll_wake(PyObject* po);
void tls_describe_failure(SSL* ssl, std::string& reason, std::string& message, bool& verify);
bool tls_warm_handshake();

bool is_h1_parser(PyObject* o);  // py_http.cpp
int h1_parser_start_c(PyObject* o, bool head);
PyObject* h1_parser_feed_c(PyObject* o, const char* data, size_t n);
bool is_pg_reader(PyObject* o);  // py_pg.cpp
PyObject* pg_reader_feed_c(PyObject* o, const char* data, size_t n);
extern uint64_t g_netpoll_runs, g_netpoll_ready;  // py_netpoll.cpp

// Process-wide socket call counts by connection kind ([kind][0] sends, [kind][1] receives), read
// by io_counts(): the bench's syscalls-per-event keys (one loop thread: plain increments).
uint64_t g_io_calls[2][2];

namespace {

PyObject *s_add_reader, *s_remove_reader, *s_add_writer, *s_remove_writer, *s_call_soon, *s_feed, *s_start,
    *s_head, *s_net_lost, *s_net_error, *s_net_message;

enum : uint8_t { K_H1 = 0, K_PG = 1 };
constexpr size_t kReadSize = 256 * 1024;

struct PgPending {
  PyObject* fut;
  PyObject* new_sql;  // the statement text if this query carried its Parse, else NULL
  PyObject* name;     // bytes
};

struct NetConnObject {
  PyObject_HEAD int fd;
  uint8_t kind;
  uint8_t closed;
  uint8_t writing;          // add_writer registered
  uint8_t flush_scheduled;  // pg: a call_soon(flush) is pending
  uint8_t connecting;       // created by netconn_connect: the TCP connect is in progress
  PyObject* loop;
  PyObject* owner;
  PyObject* on_readable;  // bound builtins handed to the loop
  PyObject* on_writable;
  PyObject* flush_cb;
  PyObject* parser;  // H1Parser / PgReader
  PyObject* feed;    // parser.feed
  PyObject* start;   // h1: parser.start
  PyObject* waiter;  // h1: the reply future of the request in flight
  PyObject* stmts;   // pg: dict sql -> statement name (shared with store/pgwire.py)
  PyObject* pg_error;
  PyObject* closed_exc;  // raised by write/request/execute once closed
  std::string* out;
  std::deque<PgPending>* pending;
  uint64_t n_stmts, bytes_in, bytes_out, recvs, sends;
  // TLS (py_tls.cpp): NULL ssl = plain TCP
  SSL* ssl;
  uint8_t tls_state;         // 0 plain, 1 handshaking, 2 established
  uint8_t write_wants_read;  // an SSL_write needs the peer's next record first (renegotiation)
  PyObject* tls_ctx;         // TlsContext (owns the SSL_CTX and the session cache)
  PyObject* hs_fut;          // handshake IOFuture: None when established, rejected on failure
  PyObject* tls_error;       // callable(reason, message, verify) -> exception for a failed handshake
  PyObject* poller;          // the loop's NetPoller (py_netpoll.cpp), or NULL: own loop.add_reader
  void* hs_job;              // HsJob*: the handshake is running on a handshake thread (tls_state 3)
};

PyTypeObject NetConnType = {PyVarObject_HEAD_INIT(nullptr, 0)};

char* read_buf() {
  static char* buf = static_cast<char*>(PyMem_RawMalloc(kReadSize));  // one event-loop thread
  return buf;
}

// ---- TLS handshakes off the event loop --------------------------------------------------------
// A TLS handshake costs the client a few hundred microseconds of CPU (key exchange, certificate
// and signature checks). On the loop thread that time is taken from every delivery in flight: a
// burst of new sink connections (the first deliveries after start, a pool growing, reconnects
// after an outage) shows up as the handle-latency tail. With a NetPoller, a NetConn hands its
// handshake to the handshake threads instead (hs_reactor.hpp: they share one epoll set and run
// only the CPU steps, so any number of handshakes wait for their peers at once): the fd leaves
// the NetPoller's interest set, the threads step SSL_do_handshake until it completes or fails,
// and the result is queued on the poller's completion channel (hs_wake.hpp: an eventfd in the
// same epoll set, so no thread ever needs the GIL); the poller's `_run` then resumes the
// connection on the loop thread exactly as after an on-loop handshake (same stats, same
// errors). While the threads own the handshake the loop never touches the SSL: closing the
// connection marks the job orphaned and shuts the socket down, and the thread that takes it next
// frees the SSL, closes the fd and drops the job.
enum HsResult : int { HR_OK = 0, HR_SSL = 1, HR_TIMEOUT = 2 };
constexpr double kHandshakeCapS = 120.0;  // safety net; callers abort on their own deadlines

struct HsJob : ReactorJob {
  NetConnObject* conn;  // no reference: read only on the loop thread, cleared when the conn closes
  std::shared_ptr<HsWake> wake;  // the loop's completion channel
  SSL* ssl;
  int result = HR_OK;
  std::string reason, message;
  bool verify = false;
};

// A handshake running on a thread for `c` is given up: true when the thread still runs it (it
// then frees the SSL, the fd and the job itself); a finished one is marked connection-less so
// that the drain of the completion channel just frees it. Must run before `c` leaves its
// poller: leaving can close the poller, which drains the channel, and the drain must not treat
// a connection that is closing as one whose handshake just succeeded.
bool detach_job(NetConnObject* c) {
  if (!c->hs_job) return false;
  auto* j = static_cast<HsJob*>(c->hs_job);
  c->hs_job = nullptr;
  // Wake the job first, while the fd is surely still open: a thread closes it only once it has
  // seen ORPHANED, and a shutdown(2) after the exchange could hit a closed (or reused) number.
  // Woken before the exchange, the job just fails and lands on the DONE path below.
  ::shutdown(c->fd, SHUT_RDWR);
  if (j->state.exchange(HS_ORPHANED) == HS_RUNNING) return true;
  j->conn = nullptr;  // finished and queued for this loop: the drain drops it
  return false;
}

// Stops watching the fd and closes it (idempotent). Errors from the loop are swallowed: this
// runs on teardown paths.
void shut(NetConnObject* c) {
  if (c->fd < 0) return;
  bool thread_owns = detach_job(c);
  PyObject *et, *ev, *tb;
  PyErr_Fetch(&et, &ev, &tb);
  if (c->poller) {
    netpoll_del(c->poller, c->fd);
    Py_CLEAR(c->poller);
  } else {
    PyObject* fdo = PyLong_FromLong(c->fd);
    if (fdo && c->loop) {
      PyObject* r = PyObject_CallMethodOneArg(c->loop, s_remove_reader, fdo);
      if (!r) PyErr_Clear();
      Py_XDECREF(r);
      if (c->writing) {
        r = PyObject_CallMethodOneArg(c->loop, s_remove_writer, fdo);
        if (!r) PyErr_Clear();
        Py_XDECREF(r);
      }
    }
    Py_XDECREF(fdo);
  }
  PyErr_Clear();
  PyErr_Restore(et, ev, tb);
  if (thread_owns) {
    // the handshake thread still uses the SSL and the fd (woken by detach_job): it frees both
    // (and the job) when done
    c->ssl = nullptr;
    c->fd = -1;
    c->writing = 0;
    c->closed = 1;
    c->out->clear();
    return;
  }
  if (c->ssl) {
    // an established session stays resumable when its connection is dropped without close_notify
    // (idle keep-alive expiry, peer reset): OpenSSL would otherwise mark the cached session
    // not resumable in SSL_free
    if (c->tls_state == 2) SSL_set_shutdown(c->ssl, SSL_SENT_SHUTDOWN | SSL_RECEIVED_SHUTDOWN);
    SSL_free(c->ssl);
    c->ssl = nullptr;
  }
  ::close(c->fd);
  c->fd = -1;
  c->writing = 0;
  c->closed = 1;
  c->out->clear();
}

// Rejects a pending handshake future with `exc` (borrowed; NULL = ConnectionResetError).
void hs_fail(NetConnObject* c, PyObject* exc) {
  PyObject* f = c->hs_fut;
  if (!f || iofuture_done(f)) return;
  PyObject *et, *ev, *tb;
  PyErr_Fetch(&et, &ev, &tb);
  PyObject* own = nullptr;
  if (!exc) exc = own = PyObject_CallFunction(PyExc_ConnectionResetError, "s", "connection closed during TLS handshake");
  if (!exc || iofuture_reject(f, exc) < 0) PyErr_WriteUnraisable(f);
  Py_XDECREF(own);
  PyErr_Restore(et, ev, tb);
}

// owner.<name>(arg) for a rare path; the error (if any) is reported, never propagated into the loop
void notify(NetConnObject* c, PyObject* name, PyObject* arg) {
  if (!c->owner || c->owner == Py_None) return;  // owner None: nobody to tell
  PyObject* r = PyObject_CallMethodOneArg(c->owner, name, arg ? arg : Py_None);
  if (!r) {
    PyErr_WriteUnraisable(c->owner);
  } else {
    Py_DECREF(r);
  }
}

// Peer closed (exc NULL) or the socket failed: close, then tell the owner.
void lost(NetConnObject* c, int err) {
  shut(c);
  if (err) {
    PyObject *et0, *ev0, *tb0;  // keep a pending exception of the caller intact
    PyErr_Fetch(&et0, &ev0, &tb0);
    errno = err;
    PyErr_SetFromErrno(PyExc_OSError);
    PyObject *et, *ev, *tb;
    PyErr_Fetch(&et, &ev, &tb);
    PyErr_NormalizeException(&et, &ev, &tb);
    Py_XDECREF(et);
    Py_XDECREF(tb);
    PyErr_Restore(et0, ev0, tb0);
    hs_fail(c, ev);  // a TLS handshake in progress fails with the socket error itself
    notify(c, s_net_lost, ev);
    Py_XDECREF(ev);
  } else {
    hs_fail(c, nullptr);
    notify(c, s_net_lost, nullptr);
  }
}

int watch_writes(NetConnObject* c) {
  if (c->writing) return 0;
  if (c->poller) {
    if (netpoll_set_write(c->poller, c->fd, true) < 0) return -1;
    c->writing = 1;
    return 0;
  }
  PyObject* fdo = PyLong_FromLong(c->fd);
  if (!fdo) return -1;
  PyObject* r = PyObject_CallMethodObjArgs(c->loop, s_add_writer, fdo, c->on_writable, nullptr);
  Py_DECREF(fdo);
  if (!r) return -1;
  Py_DECREF(r);
  c->writing = 1;
  return 0;
}

// Sends c->out (after anything already queued). 0 ok, -1 Python error. A socket error closes
// the connection and is reported to the owner (_net_lost) before this returns.
int send_out_tls(NetConnObject* c);
int unwatch_writes(NetConnObject* c);

int send_out(NetConnObject* c) {
  if (c->connecting) return 0;  // queued until the connect completes
  if (c->ssl) return send_out_tls(c);
  std::string& o = *c->out;
  size_t off = 0;
  while (off < o.size()) {
    ssize_t n = ::send(c->fd, o.data() + off, o.size() - off, MSG_NOSIGNAL);
    if (n > 0) {
      off += size_t(n);
      c->bytes_out += uint64_t(n);
      ++c->sends;
      ++g_io_calls[c->kind][0];
      continue;
    }
    if (n < 0 && errno == EINTR) continue;
    if (n < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) break;
    int err = n < 0 ? errno : EPIPE;
    o.clear();
    lost(c, err);
    return 0;
  }
  o.erase(0, off);
  if (!o.empty()) return watch_writes(c);
  return unwatch_writes(c);
}

int unwatch_writes(NetConnObject* c) {
  if (!c->writing) return 0;
  if (c->poller) {
    if (netpoll_set_write(c->poller, c->fd, false) < 0) return -1;
    c->writing = 0;
    return 0;
  }
  PyObject* fdo = PyLong_FromLong(c->fd);
  if (!fdo) return -1;
  PyObject* r = PyObject_CallMethodOneArg(c->loop, s_remove_writer, fdo);
  Py_DECREF(fdo);
  if (!r) return -1;
  Py_DECREF(r);
  c->writing = 0;
  return 0;
}

// send_out over TLS: SSL_write what is queued (nothing before the handshake completes).
int send_out_tls(NetConnObject* c) {
  if (c->tls_state != 2) return 0;
  std::string& o = *c->out;
  size_t off = 0;
  while (off < o.size()) {
    ERR_clear_error();
    size_t len = o.size() - off;
    int n = SSL_write(c->ssl, o.data() + off, len > (1u << 30) ? int(1u << 30) : int(len));
    if (n > 0) {
      off += size_t(n);
      c->bytes_out += uint64_t(n);
      ++c->sends;
      ++g_io_calls[c->kind][0];
      continue;
    }
    int e = SSL_get_error(c->ssl, n);
    if (e == SSL_ERROR_WANT_WRITE) break;
    if (e == SSL_ERROR_WANT_READ) {
      c->write_wants_read = 1;
      break;
    }
    int err = e == SSL_ERROR_SYSCALL && errno ? errno : EPIPE;
    o.clear();
    lost(c, err);
    return 0;
  }
  o.erase(0, off);
  if (!o.empty() && !c->write_wants_read) return watch_writes(c);
  return unwatch_writes(c);
}

// Drives the handshake. On success: counted, the future resolved, queued output sent.
// On failure: the future rejected with tls_error(reason, message, verify), the socket closed.
int tls_handshake(NetConnObject* c) {
  ERR_clear_error();
  int r = SSL_do_handshake(c->ssl);
  if (r == 1) {
    c->tls_state = 2;
    tls_count_handshake(c->ssl, false);
    if (unwatch_writes(c) < 0) return -1;
    PyObject* f = c->hs_fut;
    if (f && !iofuture_done(f) && iofuture_resolve(f, Py_None) < 0) return -1;
    if (c->fd >= 0 && !c->out->empty()) return send_out(c);
    return 0;
  }
  int e = SSL_get_error(c->ssl, r);
  if (e == SSL_ERROR_WANT_READ) return unwatch_writes(c);
  if (e == SSL_ERROR_WANT_WRITE) return watch_writes(c);
  std::string reason, message;
  bool verify = false;
  tls_describe_failure(c->ssl, reason, message, verify);
  ERR_clear_error();
  PyObject* exc = c->tls_error ? PyObject_CallFunction(c->tls_error, "ssO", reason.c_str(), message.c_str(),
                                                       verify ? Py_True : Py_False)
                               : PyObject_CallFunction(PyExc_ConnectionError, "s", message.c_str());
  if (!exc) return -1;
  shut(c);
  hs_fail(c, exc);
  Py_DECREF(exc);
  return 0;
}

double mono_now() { return reactor_now(); }

// One non-blocking step of an offloaded handshake, on a handshake thread: 0 when finished (the
// outcome is in the job), else the readiness to wait for.
int hs_step(ReactorJob* rj) {
  auto* j = static_cast<HsJob*>(rj);
  if (j->state.load() == HS_ORPHANED) return 0;  // closed: hs_finish frees it
  if (j->expired.load()) {
    j->result = HR_TIMEOUT;
    return 0;
  }
  ERR_clear_error();  // the error queue is per thread; a job's steps may run on different ones
  int r = SSL_do_handshake(j->ssl);
  if (r == 1) {
    j->result = j->expired.load() ? HR_TIMEOUT : HR_OK;  // the scan may have shut it down meanwhile
    return 0;
  }
  int e = SSL_get_error(j->ssl, r);
  if (e == SSL_ERROR_WANT_READ) return EPOLLIN;
  if (e == SSL_ERROR_WANT_WRITE) return EPOLLOUT;
  if (j->expired.load()) {
    j->result = HR_TIMEOUT;
  } else {
    tls_describe_failure(j->ssl, j->reason, j->message, j->verify);
    j->result = HR_SSL;
  }
  ERR_clear_error();
  return 0;
}

// The job has left the reactor: hand it to its loop, or free it if its connection is gone.
void hs_finish(ReactorJob* rj) {
  auto* j = static_cast<HsJob*>(rj);
  // The deadline scan walks the registry until the unlink that precedes this call, so it can shut
  // the socket of a job whose last step had already succeeded: that connection is unusable, and
  // the honest outcome is the timeout the scan enforced, not a success whose first request fails
  // as a connection error. Past the unlink the flag can no longer change.
  if (j->result == HR_OK && j->expired.load()) j->result = HR_TIMEOUT;
  if (j->sys_errno && j->result == HR_OK) {
    j->reason = "SYSCALL";
    j->message = std::string("[SSL: SYSCALL] epoll_ctl: ") + strerror(j->sys_errno);
    j->result = HR_SSL;
  }
  std::shared_ptr<HsWake> wake = j->wake;
  if (j->state.exchange(HS_DONE) == HS_ORPHANED) {  // closed meanwhile: the SSL, fd and job are ours
    SSL_free(j->ssl);
    ::close(j->fd);
    delete j;
    return;
  }
  if (!wake->post(j)) delete j;  // posted: the loop thread owns the job from here
}

void hs_thread(HsReactor* r) {
  // OpenSSL 3 keeps per-thread state (random generators, provider caches) that a thread's first
  // handshake would build inside the first burst of connects: one in-memory handshake first
  tls_warm_handshake();
  r->run();
}

HsReactor* g_hs = nullptr;  // process-lifetime (its threads never exit); replaced in a forked child
unsigned g_hs_threads = 0;

void hs_after_fork_child() {
  if (g_hs) g_hs->abandon_after_fork();  // the object itself is leaked: a parent thread may hold its lock
  g_hs = nullptr;
  g_hs_threads = 0;
}

// The process's handshake reactor with its threads started (on the calling thread, which holds
// the GIL; the threads never take it). Throws std::bad_alloc / std::system_error.
HsReactor* hs_pool() {
  static bool atfork = (pthread_atfork(nullptr, nullptr, hs_after_fork_child), true);
  (void)atfork;
  if (!g_hs) g_hs = new HsReactor(hs_step, hs_finish);
  // 4: the threads only run CPU steps now, and on the box's 16-CPU share more of them compete
  // with the loop and the peers for the same CPUs (profiles/box_r3_warmup/threads/)
  unsigned want = std::max(1u, std::min(4u, std::thread::hardware_concurrency() / 4));
  while (g_hs_threads < want) {
    std::thread(hs_thread, g_hs).detach();
    ++g_hs_threads;
  }
  return g_hs;
}

bool hs_submit(HsJob* j) {
  try {
    return hs_pool()->submit(j);
  } catch (const std::exception&) {
    return false;
  }
}

// Starts the handshake of `c` (connected, SSL set up) on a handshake thread when it can (a
// NetPoller to take the fd out of), else on the loop. 0 or -1 with a Python error.
int tls_start(NetConnObject* c) {
  c->tls_state = 1;
  if (!c->poller) return tls_handshake(c);
  std::shared_ptr<HsWake> wake = netpoll_wake(c->poller);
  if (!wake) return tls_handshake(c);
  auto* j = new (std::nothrow) HsJob();
  if (!j) return tls_handshake(c);
  if (netpoll_pause(c->poller, c->fd) < 0) {
    delete j;
    return -1;
  }
  j->conn = c;
  j->wake = std::move(wake);
  j->ssl = c->ssl;
  j->fd = c->fd;
  j->deadline = mono_now() + kHandshakeCapS;
  c->hs_job = j;
  c->tls_state = 3;
  if (!hs_submit(j)) {  // no thread: run it here after all
    c->hs_job = nullptr;
    c->tls_state = 1;
    delete j;
    if (netpoll_set_write(c->poller, c->fd, c->writing) < 0) return -1;
    return tls_handshake(c);
  }
  return 0;
}

// The loop-thread half of an offloaded handshake (the poller drains its completion channel).
// 0, or -1 with a Python error.
int tls_done(HsJob* j) {
  NetConnObject* c = j->conn;
  if (!c) {  // the connection closed after the thread finished
    delete j;
    return 0;
  }
  c->hs_job = nullptr;
  int result = j->result;
  std::string reason = std::move(j->reason), message = std::move(j->message);
  bool verify = j->verify;
  delete j;
  if (c->fd < 0 || !c->ssl) return 0;
  Py_INCREF(c);  // a resumed handler may drop the last other reference
  int rc = 0;
  c->tls_state = 1;
  if (c->poller && netpoll_set_write(c->poller, c->fd, c->writing) < 0) {
    rc = -1;
  } else if (result == HR_OK) {
    c->tls_state = 2;
    tls_count_handshake(c->ssl, true);
    PyObject* f = c->hs_fut;
    if (f && !iofuture_done(f) && iofuture_resolve(f, Py_None) < 0) rc = -1;
    if (rc == 0 && c->fd >= 0 && !c->out->empty()) rc = send_out(c);
  } else if (result == HR_TIMEOUT) {
    lost(c, ETIMEDOUT);
  } else {
    PyObject* exc = c->tls_error ? PyObject_CallFunction(c->tls_error, "ssO", reason.c_str(), message.c_str(),
                                                         verify ? Py_True : Py_False)
                                 : PyObject_CallFunction(PyExc_ConnectionError, "s", message.c_str());
    if (!exc) {
      rc = -1;
    } else {
      shut(c);
      hs_fail(c, exc);
      Py_DECREF(exc);
    }
  }
  Py_DECREF(c);
  return rc;
}

int append_bytes(NetConnObject* c, PyObject* data) {
  Py_buffer v;
  if (PyObject_GetBuffer(data, &v, PyBUF_SIMPLE) < 0) return -1;
  c->out->append(static_cast<const char*>(v.buf), size_t(v.len));
  PyBuffer_Release(&v);
  return 0;
}

PyObject* closed_error(NetConnObject* c) {
  PyErr_SetString(c->closed_exc ? c->closed_exc : PyExc_ConnectionError, "connection is closed");
  return nullptr;
}

// ---- reply dispatch -----------------------------------------------------------------------
// parser.feed(bytes received): the stock parsers directly in C, any other through its method
PyObject* feed_parser(NetConnObject* c, const char* data, size_t n) {
  if (c->kind == K_H1 ? is_h1_parser(c->parser) : is_pg_reader(c->parser))
    return c->kind == K_H1 ? h1_parser_feed_c(c->parser, data, n) : pg_reader_feed_c(c->parser, data, n);
  PyObject* mv = PyMemoryView_FromMemory(const_cast<char*>(data), Py_ssize_t(n), PyBUF_READ);
  if (!mv) return nullptr;
  PyObject* r = PyObject_CallOneArg(c->feed, mv);
  Py_DECREF(mv);
  return r;
}

// parser.start(head=head) before a request: the stock H1Parser directly in C
int start_parser(NetConnObject* c, bool head) {
  if (is_h1_parser(c->parser)) return h1_parser_start_c(c->parser, head);
  PyObject* kw = PyTuple_Pack(1, s_head);
  if (!kw) return -1;
  PyObject* args[1] = {head ? Py_True : Py_False};
  PyObject* r = PyObject_Vectorcall(c->start, args, 0, kw);
  Py_DECREF(kw);
  if (!r) return -1;
  Py_DECREF(r);
  return 0;
}

void on_h1_data(NetConnObject* c, const char* data, size_t n) {
  PyObject* r = feed_parser(c, data, n);
  if (!r) {  // malformed response: the owner fails the request and drops the connection
    PyObject *et, *ev, *tb;
    PyErr_Fetch(&et, &ev, &tb);
    PyErr_NormalizeException(&et, &ev, &tb);
    Py_XDECREF(et);
    Py_XDECREF(tb);
    notify(c, s_net_error, ev);
    Py_XDECREF(ev);
    return;
  }
  if (r == Py_None) {
    Py_DECREF(r);
    return;
  }
  PyObject* w = c->waiter;
  c->waiter = nullptr;
  if (!w || iofuture_done(w)) {
    Py_XDECREF(w);
    Py_DECREF(r);
    notify(c, s_net_error, nullptr);  // unsolicited response
    return;
  }
  if (iofuture_resolve(w, r) < 0) PyErr_WriteUnraisable(w);  // the waiting handler resumes here
  Py_DECREF(w);
  Py_DECREF(r);
}

void on_pg_data(NetConnObject* c, const char* data, size_t len) {
  PyObject* items = feed_parser(c, data, len);
  if (!items) {
    PyObject *et, *ev, *tb;
    PyErr_Fetch(&et, &ev, &tb);
    PyErr_NormalizeException(&et, &ev, &tb);
    Py_XDECREF(et);
    Py_XDECREF(tb);
    notify(c, s_net_error, ev);
    Py_XDECREF(ev);
    return;
  }
  Py_ssize_t n = PyList_GET_SIZE(items);
  for (Py_ssize_t i = 0; i < n; ++i) {
    PyObject* it = PyList_GET_ITEM(items, i);
    if (PyTuple_GET_SIZE(it) != 4) {  // NoticeResponse / ParameterStatus / ...
      if (!c->owner || c->owner == Py_None) continue;  // nobody to tell
      PyObject* r = PyObject_CallMethodObjArgs(c->owner, s_net_message, PyTuple_GET_ITEM(it, 0),
                                               PyTuple_GET_ITEM(it, 1), nullptr);
      if (!r) PyErr_WriteUnraisable(c->owner);
      Py_XDECREF(r);
      continue;
    }
    if (c->pending->empty()) {  // ReadyForQuery with nothing outstanding
      notify(c, s_net_error, nullptr);
      break;
    }
    PgPending p = c->pending->front();
    c->pending->pop_front();
    PyObject* rows = PyTuple_GET_ITEM(it, 0);
    PyObject* tag = PyTuple_GET_ITEM(it, 1);
    PyObject* err = PyTuple_GET_ITEM(it, 2);
    int rc = 0;
    if (err != Py_None) {
      if (p.new_sql && PyTuple_GET_ITEM(it, 3) != Py_True) {  // failed Parse: forget the statement
        PyObject* cur = PyDict_GetItemWithError(c->stmts, p.new_sql);
        if (cur && PyObject_RichCompareBool(cur, p.name, Py_EQ) == 1) {
          if (PyDict_DelItem(c->stmts, p.new_sql) < 0) PyErr_Clear();
        }
        PyErr_Clear();
      }
      PyObject* exc = PyObject_CallOneArg(c->pg_error, err);
      rc = exc ? iofuture_reject(p.fut, exc) : -1;
      Py_XDECREF(exc);
    } else {
      PyObject* res = PyTuple_Pack(2, rows, tag);
      rc = res ? iofuture_resolve(p.fut, res) : -1;  // a handler waiting on it resumes here
      Py_XDECREF(res);
    }
    if (rc < 0) PyErr_WriteUnraisable(p.fut);
    Py_DECREF(p.fut);
    Py_XDECREF(p.new_sql);
    Py_DECREF(p.name);
  }
  Py_DECREF(items);
}

// ---- type ---------------------------------------------------------------------------------
PyObject* nc_new(PyTypeObject* type, PyObject*, PyObject*) {
  NetConnObject* c = reinterpret_cast<NetConnObject*>(type->tp_alloc(type, 0));
  if (!c) return nullptr;
  c->fd = -1;
  c->closed = 1;
  c->out = new (std::nothrow) std::string();
  c->pending = new (std::nothrow) std::deque<PgPending>();
  if (!c->out || !c->pending) {
    Py_DECREF(c);
    return PyErr_NoMemory();
  }
  return reinterpret_cast<PyObject*>(c);
}

void drop_pending(NetConnObject* c) {
  while (!c->pending->empty()) {
    PgPending p = c->pending->front();
    c->pending->pop_front();
    Py_DECREF(p.fut);
    Py_XDECREF(p.new_sql);
    Py_DECREF(p.name);
  }
}

int nc_traverse(NetConnObject* c, visitproc visit, void* arg) {
  Py_VISIT(c->loop);
  Py_VISIT(c->owner);
  Py_VISIT(c->on_readable);
  Py_VISIT(c->on_writable);
  Py_VISIT(c->flush_cb);
  Py_VISIT(c->parser);
  Py_VISIT(c->feed);
  Py_VISIT(c->start);
  Py_VISIT(c->waiter);
  Py_VISIT(c->stmts);
  Py_VISIT(c->pg_error);
  Py_VISIT(c->closed_exc);
  Py_VISIT(c->tls_ctx);
  Py_VISIT(c->hs_fut);
  Py_VISIT(c->tls_error);
  Py_VISIT(c->poller);
  if (c->pending) {
    for (const PgPending& p : *c->pending) {
      Py_VISIT(p.fut);
      Py_VISIT(p.new_sql);
      Py_VISIT(p.name);
    }
  }
  return 0;
}

int nc_clear(NetConnObject* c) {
  Py_CLEAR(c->owner);
  Py_CLEAR(c->on_readable);
  Py_CLEAR(c->on_writable);
  Py_CLEAR(c->flush_cb);
  Py_CLEAR(c->parser);
  Py_CLEAR(c->feed);
  Py_CLEAR(c->start);
  Py_CLEAR(c->waiter);
  Py_CLEAR(c->stmts);
  Py_CLEAR(c->pg_error);
  Py_CLEAR(c->closed_exc);
  Py_CLEAR(c->hs_fut);
  Py_CLEAR(c->tls_error);
  if (c->poller) {  // registered: leave the epoll set first (the poller's reference cycle)
    if (c->fd >= 0 && detach_job(c)) {  // the handshake thread frees the SSL and the fd
      netpoll_del(c->poller, c->fd);
      c->ssl = nullptr;
      c->fd = -1;
    } else if (c->fd >= 0) {
      netpoll_del(c->poller, c->fd);
    }
    Py_CLEAR(c->poller);
  }
  if (c->pending) drop_pending(c);
  return 0;
}

void nc_dealloc(NetConnObject* c) {
  PyObject_GC_UnTrack(c);
  if (c->fd >= 0) shut(c);  // normally closed by the owner first
  if (c->ssl) {  // set up but never owned the fd (init failed)
    SSL_free(c->ssl);
    c->ssl = nullptr;
  }
  nc_clear(c);
  Py_CLEAR(c->loop);
  Py_CLEAR(c->tls_ctx);  // after shut(): the SSL refers to it
  delete c->out;
  delete c->pending;
  Py_TYPE(c)->tp_free(reinterpret_cast<PyObject*>(c));
}

PyObject* nc_on_readable(NetConnObject* c, PyObject*);
PyObject* nc_on_writable(NetConnObject* c, PyObject*);
PyObject* nc_flush(NetConnObject* c, PyObject*);

// NetConn(fd, loop, kind, owner, parser, stmts=None, pg_error=None, closed_exc=ConnectionError):
// takes ownership of fd (a connected TCP socket) and starts watching it. `owner` gets the
// _net_lost / _net_error / _net_message calls (None: nobody is told; a reply future still ends).
int nc_init(NetConnObject* c, PyObject* args, PyObject* kwds) {
  static const char* kwlist[] = {"fd",        "loop", "kind",       "owner",     "parser", "stmts", "pg_error",
                                 "closed_exc", "tls",  "server_hostname", "port", "tls_error", nullptr};
  int fd;
  PyObject *loop, *owner, *parser, *stmts = Py_None, *pg_error = Py_None, *closed_exc = PyExc_ConnectionError;
  PyObject *tls = Py_None, *tls_error = Py_None;
  const char* kind;
  const char* host = nullptr;
  int port = 0;
  if (!PyArg_ParseTupleAndKeywords(args, kwds, "iOsOO|OOOOziO", const_cast<char**>(kwlist), &fd, &loop, &kind, &owner,
                                   &parser, &stmts, &pg_error, &closed_exc, &tls, &host, &port, &tls_error))
    return -1;
  if (tls != Py_None && (!is_tls_context(tls) || !host)) {
    PyErr_SetString(PyExc_TypeError, "tls needs a TlsContext and server_hostname");
    return -1;
  }
  if (!PyExceptionClass_Check(closed_exc)) {
    PyErr_SetString(PyExc_TypeError, "closed_exc must be an exception class");
    return -1;
  }
  if (c->fd >= 0 || c->loop) {
    PyErr_SetString(PyExc_RuntimeError, "NetConn already initialised");
    return -1;
  }
  if (strcmp(kind, "h1") == 0) {
    c->kind = K_H1;
  } else if (strcmp(kind, "pg") == 0) {
    c->kind = K_PG;
    if (!PyDict_Check(stmts) || pg_error == Py_None) {
      PyErr_SetString(PyExc_TypeError, "kind 'pg' needs stmts (dict) and pg_error");
      return -1;
    }
  } else {
    PyErr_SetString(PyExc_ValueError, "kind must be 'h1' or 'pg'");
    return -1;
  }
  if (fd < 0) {
    PyErr_SetString(PyExc_ValueError, "invalid fd");
    return -1;
  }
  Py_INCREF(loop);
  c->loop = loop;
  Py_INCREF(closed_exc);
  c->closed_exc = closed_exc;
  Py_INCREF(owner);
  c->owner = owner;
  Py_INCREF(parser);
  c->parser = parser;
  c->feed = PyObject_GetAttr(parser, s_feed);
  if (!c->feed) return -1;
  if (c->kind == K_H1) {
    c->start = PyObject_GetAttr(parser, s_start);
    if (!c->start) return -1;
  } else {
    Py_INCREF(stmts);
    c->stmts = stmts;
    Py_INCREF(pg_error);
    c->pg_error = pg_error;
  }
  c->on_readable = PyObject_GetAttrString(reinterpret_cast<PyObject*>(c), "_on_readable");
  c->on_writable = c->on_readable ? PyObject_GetAttrString(reinterpret_cast<PyObject*>(c), "_on_writable") : nullptr;
  c->flush_cb = c->on_writable ? PyObject_GetAttrString(reinterpret_cast<PyObject*>(c), "flush") : nullptr;
  if (!c->flush_cb) return -1;
  if (tls != Py_None) {  // set up before the fd is owned: a failure here leaves it to the caller
    c->hs_fut = iofuture_new(loop);
    if (!c->hs_fut) return -1;
    c->ssl = tls_new_ssl(tls, fd, host, port);
    if (!c->ssl) return -1;
    Py_INCREF(tls);
    c->tls_ctx = tls;
    if (tls_error != Py_None) {
      Py_INCREF(tls_error);
      c->tls_error = tls_error;
    }
  }
  PyObject* poller = netpoll_for(loop);  // the loop's shared epoll set, or None
  if (!poller) return -1;
  if (poller != Py_None) {
    if (netpoll_add(poller, fd, reinterpret_cast<PyObject*>(c)) < 0) {
      Py_DECREF(poller);
      return -1;
    }
    c->poller = poller;
  } else {
    Py_DECREF(poller);
    PyObject* fdo = PyLong_FromLong(fd);
    if (!fdo) return -1;
    PyObject* r = PyObject_CallMethodObjArgs(loop, s_add_reader, fdo, c->on_readable, nullptr);
    Py_DECREF(fdo);
    if (!r) return -1;
    Py_DECREF(r);
  }
  c->fd = fd;  // owned from here on
  c->closed = 0;
  if (c->ssl && !c->connecting) {
    if (tls_start(c) < 0) {  // ClientHello goes out now (here or on a handshake thread)
      shut(c);  // unregistered and closed: the caller only gets the exception
      return -1;
    }
  }
  return 0;
}

PyObject* on_readable_tls(NetConnObject* c, char* buf);

// The socket of a connecting NetConn became writable (or reported an error): finish the
// connect. Failure: the ready future is rejected with the OSError and the socket closed.
// Success: TLS starts its handshake; plain TCP resolves the ready future.
int connect_done(NetConnObject* c) {
  int err = 0;
  socklen_t len = sizeof err;
  if (getsockopt(c->fd, SOL_SOCKET, SO_ERROR, &err, &len) < 0) err = errno;
  if (err == EINPROGRESS || err == EALREADY) return 0;  // spurious wake-up
  if (!err) {  // writable and no error: connected, unless the event was stale (fd reuse)
    sockaddr_storage peer;
    socklen_t plen = sizeof peer;
    if (getpeername(c->fd, reinterpret_cast<sockaddr*>(&peer), &plen) < 0 && errno == ENOTCONN) return 0;
  }
  c->connecting = 0;
  if (err) {
    errno = err;
    PyErr_SetFromErrno(PyExc_OSError);
    PyObject *et, *ev, *tb;
    PyErr_Fetch(&et, &ev, &tb);
    PyErr_NormalizeException(&et, &ev, &tb);
    Py_XDECREF(et);
    Py_XDECREF(tb);
    shut(c);
    hs_fail(c, ev);
    Py_XDECREF(ev);
    return 0;
  }
  if (unwatch_writes(c) < 0) return -1;
  if (c->ssl) return tls_start(c);
  PyObject* f = c->hs_fut;
  if (f && !iofuture_done(f) && iofuture_resolve(f, Py_None) < 0) return -1;
  if (c->fd >= 0 && !c->out->empty()) return send_out(c);
  return 0;
}

PyObject* nc_on_readable(NetConnObject* c, PyObject*) {
  if (c->fd < 0) Py_RETURN_NONE;
  if (c->connecting) {
    if (connect_done(c) < 0) return nullptr;
    Py_RETURN_NONE;
  }
  char* buf = read_buf();
  if (!buf) return PyErr_NoMemory();
  if (c->ssl) return on_readable_tls(c, buf);
  ssize_t n;
  do {
    n = ::recv(c->fd, buf, kReadSize, 0);
  } while (n < 0 && errno == EINTR);
  if (n < 0) {
    if (errno == EAGAIN || errno == EWOULDBLOCK) Py_RETURN_NONE;
    lost(c, errno);
    Py_RETURN_NONE;
  }
  if (n == 0) {
    lost(c, 0);
    Py_RETURN_NONE;
  }
  c->bytes_in += uint64_t(n);
  ++c->recvs;
  ++g_io_calls[c->kind][1];
  Py_INCREF(c);  // a resumed handler may drop the last other reference
  if (c->kind == K_H1) {
    on_h1_data(c, buf, size_t(n));
  } else {
    on_pg_data(c, buf, size_t(n));
  }
  Py_DECREF(c);
  Py_RETURN_NONE;
}

// TLS: records are decrypted until OpenSSL wants more bytes; each plaintext chunk goes to the
// parser as on the plain path (a completed reply resumes its handler right here).
PyObject* on_readable_tls(NetConnObject* c, char* buf) {
  if (c->tls_state == 3) Py_RETURN_NONE;  // a handshake thread owns the SSL (an error / hang-up event)
  if (c->tls_state == 1) {
    if (tls_handshake(c) < 0) return nullptr;
    Py_RETURN_NONE;
  }
  Py_INCREF(c);  // a resumed handler may drop the last other reference
  if (c->write_wants_read) {
    c->write_wants_read = 0;
    if (send_out(c) < 0) {
      Py_DECREF(c);
      return nullptr;
    }
  }
  while (c->ssl && c->fd >= 0) {
    ERR_clear_error();
    int n = SSL_read(c->ssl, buf, int(kReadSize));
    if (n > 0) {
      c->bytes_in += uint64_t(n);
      ++c->recvs;
      ++g_io_calls[c->kind][1];
      if (c->kind == K_H1) {
        on_h1_data(c, buf, size_t(n));
      } else {
        on_pg_data(c, buf, size_t(n));
      }
      // nothing buffered in OpenSSL: stop without the recv(2) that would only say EAGAIN (the
      // loop's level-triggered poll comes back if the kernel holds more)
      if (c->ssl && !SSL_has_pending(c->ssl)) break;
      continue;
    }
    int e = SSL_get_error(c->ssl, n);
    if (e == SSL_ERROR_WANT_READ) break;
    if (e == SSL_ERROR_WANT_WRITE) {
      if (watch_writes(c) < 0) {
        Py_DECREF(c);
        return nullptr;
      }
      break;
    }
    int err = 0;  // close_notify, or EOF without it: the peer closed
    if (e == SSL_ERROR_SYSCALL) {
      err = errno;
    } else if (e == SSL_ERROR_SSL) {
      unsigned long le = ERR_peek_last_error();
      if (ERR_GET_REASON(le) != SSL_R_UNEXPECTED_EOF_WHILE_READING) err = EPROTO;
    }
    ERR_clear_error();
    lost(c, err);
    break;
  }
  Py_DECREF(c);
  Py_RETURN_NONE;
}

PyObject* nc_on_writable(NetConnObject* c, PyObject*) {
  if (c->fd < 0) Py_RETURN_NONE;
  if (c->connecting) {
    if (connect_done(c) < 0) return nullptr;
    Py_RETURN_NONE;
  }
  if (c->ssl && c->tls_state == 3) Py_RETURN_NONE;  // on a handshake thread
  if (c->ssl && c->tls_state == 1) {
    if (tls_handshake(c) < 0) return nullptr;
    Py_RETURN_NONE;
  }
  if (send_out(c) < 0) return nullptr;
  Py_RETURN_NONE;
}

// write(data): send now, keep the rest for on_writable
PyObject* nc_write(NetConnObject* c, PyObject* data) {
  BEHOLDER_TRY {
    if (c->fd < 0) return closed_error(c);
    if (append_bytes(c, data) < 0) return nullptr;
    if (c->writing) Py_RETURN_NONE;  // queued behind earlier bytes
    if (send_out(c) < 0) return nullptr;
    Py_RETURN_NONE;
  }
  BEHOLDER_CATCH(nullptr)
}

// h1: request(data, waiter, head) — parser.start(head=head), waiter set, request written
PyObject* nc_request(NetConnObject* c, PyObject* const* a, Py_ssize_t n) {
  BEHOLDER_TRY {
    if (n != 3 || c->kind != K_H1) {
      PyErr_SetString(PyExc_TypeError, "request(data, waiter, head) on an h1 NetConn");
      return nullptr;
    }
    if (c->fd < 0) return closed_error(c);
    int head = PyObject_IsTrue(a[2]);
    if (head < 0 || start_parser(c, head != 0) < 0) return nullptr;  // parser.start(head=head)
    Py_INCREF(a[1]);
    Py_XSETREF(c->waiter, a[1]);
    if (append_bytes(c, a[0]) < 0) return nullptr;
    if (c->writing) Py_RETURN_NONE;
    if (send_out(c) < 0) return nullptr;
    Py_RETURN_NONE;
  }
  BEHOLDER_CATCH(nullptr)
}

// pg: execute(sql, params) -> IOFuture resolving to (rows, tag) or rejected with pg_error(fields)
PyObject* nc_execute(NetConnObject* c, PyObject* const* a, Py_ssize_t n) {
  BEHOLDER_TRY {
    if (n < 1 || n > 2 || c->kind != K_PG) {
      PyErr_SetString(PyExc_TypeError, "execute(sql, params=()) on a pg NetConn");
      return nullptr;
    }
    if (c->fd < 0) return closed_error(c);
    PyObject* sql = a[0];
    PyObject* params = n > 1 ? a[1] : nullptr;
    PyObject* name = PyDict_GetItemWithError(c->stmts, sql);
    PyObject* new_sql = nullptr;
    std::string& o = *c->out;
    size_t mark = o.size();
    if (name) {
      Py_INCREF(name);
    } else {
      if (PyErr_Occurred()) return nullptr;
      Py_ssize_t sl;
      const char* st = PyUnicode_AsUTF8AndSize(sql, &sl);
      if (!st) return nullptr;
      name = PyBytes_FromFormat("b%zu", static_cast<size_t>(++c->n_stmts));
      if (!name || PyDict_SetItem(c->stmts, sql, name) < 0) {
        Py_XDECREF(name);
        return nullptr;
      }
      new_sql = sql;
      Py_INCREF(new_sql);
      size_t nl = size_t(PyBytes_GET_SIZE(name));
      uint32_t len = uint32_t(4 + nl + 1 + size_t(sl) + 1 + 2);
      char hdr[5] = {'P', char(len >> 24), char(len >> 16), char(len >> 8), char(len)};
      o.append(hdr, 5);
      o.append(PyBytes_AS_STRING(name), nl);
      o.push_back('\0');
      o.append(st, size_t(sl));
      o.append("\0\0\0", 3);  // terminator + no parameter types
    }
    PyObject* empty = nullptr;
    if (!params) {
      empty = PyTuple_New(0);
      params = empty;
    }
    int rc = params ? pg_bind_append(o, PyBytes_AS_STRING(name), size_t(PyBytes_GET_SIZE(name)), params) : -1;
    Py_XDECREF(empty);
    PyObject* fut = rc < 0 ? nullptr : iofuture_new(c->loop);
    if (!fut) {
      o.resize(mark);  // the Parse of a new statement goes too: forget its name
      if (new_sql) {
        PyObject *et, *ev, *tb;
        PyErr_Fetch(&et, &ev, &tb);
        if (PyDict_DelItem(c->stmts, new_sql) < 0) PyErr_Clear();
        PyErr_Restore(et, ev, tb);
      }
      Py_DECREF(name);
      Py_XDECREF(new_sql);
      return nullptr;
    }
    Py_INCREF(fut);
    c->pending->push_back({fut, new_sql, name});
    if (!c->flush_scheduled) {
      // with a NetPoller: one flush for all its connections (at the end of its dispatch, or one
      // call_soon), else a call_soon of this connection's flush
      PyObject* h = c->poller ? (netpoll_request_flush(c->poller, reinterpret_cast<PyObject*>(c)) < 0
                                     ? nullptr
                                     : (Py_INCREF(Py_None), Py_None))
                              : PyObject_CallMethodOneArg(c->loop, s_call_soon, c->flush_cb);
      if (!h) {
        c->pending->pop_back();
        o.resize(mark);  // the Parse of a new statement goes too: forget its name (as above)
        if (new_sql) {
          PyObject *et, *ev, *tb;
          PyErr_Fetch(&et, &ev, &tb);
          if (PyDict_DelItem(c->stmts, new_sql) < 0) PyErr_Clear();
          PyErr_Restore(et, ev, tb);
        }
        Py_DECREF(fut);
        Py_DECREF(fut);
        Py_DECREF(name);
        Py_XDECREF(new_sql);
        return nullptr;
      }
      Py_DECREF(h);
      c->flush_scheduled = 1;
    }
    return fut;
  }
  BEHOLDER_CATCH(nullptr)
}

// flush(): write out what execute() queued (scheduled once per loop iteration)
PyObject* nc_flush(NetConnObject* c, PyObject*) {
  c->flush_scheduled = 0;
  if (c->fd < 0 || c->out->empty() || c->writing) Py_RETURN_NONE;
  if (send_out(c) < 0) return nullptr;
  Py_RETURN_NONE;
}

// fail_all(exc): pg: every outstanding query fails with exc (connection gone)
PyObject* nc_fail_all(NetConnObject* c, PyObject* exc) {
  c->closed = 1;
  while (!c->pending->empty()) {
    PgPending p = c->pending->front();
    c->pending->pop_front();
    int rc = iofuture_reject(p.fut, exc);
    Py_DECREF(p.fut);
    Py_XDECREF(p.new_sql);
    Py_DECREF(p.name);
    if (rc < 0) return nullptr;
  }
  Py_RETURN_NONE;
}

// take_waiter(): h1: the pending reply future (or None), cleared
PyObject* nc_take_waiter(NetConnObject* c, PyObject*) {
  PyObject* w = c->waiter;
  c->waiter = nullptr;
  if (!w) Py_RETURN_NONE;
  return w;
}

PyObject* nc_close(NetConnObject* c, PyObject*) {
  c->flush_scheduled = 0;
  if (c->ssl) {  // best effort: queued records, then close_notify
    if (c->tls_state == 2) {
      if (!c->out->empty() && !c->writing) SSL_write(c->ssl, c->out->data(), int(c->out->size()));
      SSL_shutdown(c->ssl);
    }
    ERR_clear_error();
  } else if (c->fd >= 0 && !c->out->empty() && !c->writing) {  // best effort: what is queued goes out
    ::send(c->fd, c->out->data(), c->out->size(), MSG_NOSIGNAL | MSG_DONTWAIT);
  }
  shut(c);
  hs_fail(c, nullptr);
  Py_RETURN_NONE;
}

PyObject* nc_abort(NetConnObject* c, PyObject*) {
  shut(c);
  hs_fail(c, nullptr);
  Py_RETURN_NONE;
}

PyObject* nc_get_closed(NetConnObject* c, void*) { return PyBool_FromLong(c->closed || c->fd < 0); }
PyObject* nc_get_fd(NetConnObject* c, void*) { return PyLong_FromLong(c->fd); }
PyObject* nc_get_pending(NetConnObject* c, void*) { return PyLong_FromSize_t(c->pending->size()); }
PyObject* nc_get_buffered(NetConnObject* c, void*) { return PyLong_FromSize_t(c->out->size()); }
PyObject* nc_get_waiting(NetConnObject* c, void*) { return PyBool_FromLong(c->waiter != nullptr); }
PyObject* nc_get_handshake(NetConnObject* c, void*) {
  if (!c->hs_fut) Py_RETURN_NONE;
  Py_INCREF(c->hs_fut);
  return c->hs_fut;
}
PyObject* nc_get_tls(NetConnObject* c, void*) {
  if (c->tls_state == 0) Py_RETURN_NONE;
  if (c->tls_state != 2 || !c->ssl) Py_RETURN_FALSE;
  return PyUnicode_FromString(SSL_get_version(c->ssl));
}
PyObject* nc_get_stats(NetConnObject* c, void*) {
  return Py_BuildValue("{s:K,s:K,s:K,s:K}", "bytes_in", c->bytes_in, "bytes_out", c->bytes_out, "recvs", c->recvs,
                       "sends", c->sends);
}

PyMethodDef nc_methods[] = {
    {"_on_readable", reinterpret_cast<PyCFunction>(nc_on_readable), METH_NOARGS, "loop reader callback"},
    {"_on_writable", reinterpret_cast<PyCFunction>(nc_on_writable), METH_NOARGS, "loop writer callback"},
    {"write", reinterpret_cast<PyCFunction>(nc_write), METH_O, "write(data): send, queue what the kernel refuses"},
    {"request", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(nc_request)), METH_FASTCALL,
     "h1: request(data, waiter, head): start the parser, set the reply future, send"},
    {"execute", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(nc_execute)), METH_FASTCALL,
     "pg: execute(sql, params=()) -> IOFuture of (rows, tag)"},
    {"flush", reinterpret_cast<PyCFunction>(nc_flush), METH_NOARGS, "pg: send the queued queries"},
    {"fail_all", reinterpret_cast<PyCFunction>(nc_fail_all), METH_O, "pg: reject every outstanding query"},
    {"take_waiter", reinterpret_cast<PyCFunction>(nc_take_waiter), METH_NOARGS, "h1: pop the reply future"},
    {"close", reinterpret_cast<PyCFunction>(nc_close), METH_NOARGS, "send what is queued (best effort), close"},
    {"abort", reinterpret_cast<PyCFunction>(nc_abort), METH_NOARGS, "close now"},
    {nullptr, nullptr, 0, nullptr}};

PyGetSetDef nc_getset[] = {
    {"closed", reinterpret_cast<getter>(nc_get_closed), nullptr, "fd closed (or failed)", nullptr},
    {"fd", reinterpret_cast<getter>(nc_get_fd), nullptr, "the socket fd, -1 once closed", nullptr},
    {"pending", reinterpret_cast<getter>(nc_get_pending), nullptr, "pg: queries awaiting their reply", nullptr},
    {"buffered", reinterpret_cast<getter>(nc_get_buffered), nullptr, "bytes not yet taken by the kernel", nullptr},
    {"waiting", reinterpret_cast<getter>(nc_get_waiting), nullptr, "h1: a reply is awaited", nullptr},
    {"stats", reinterpret_cast<getter>(nc_get_stats), nullptr, "bytes / syscall counters", nullptr},
    {"handshake", reinterpret_cast<getter>(nc_get_handshake), nullptr, "TLS: the handshake future (None: plain TCP)",
     nullptr},
    {"tls", reinterpret_cast<getter>(nc_get_tls), nullptr,
     "None (plain TCP), False (handshaking) or the negotiated protocol ('TLSv1.3')", nullptr},
    {nullptr, nullptr, nullptr, nullptr, nullptr}};

}  // namespace

// Called when a TlsContext is made (service startup): the threads start and warm up before the
// first connect needs them. Failure is not an error here; hs_submit tries again.
void hs_prestart() {
  try {
    hs_pool();
  } catch (const std::exception&) {
  }
}

bool is_netconn(PyObject* o) { return Py_TYPE(o) == &NetConnType; }


// The NetPoller's dispatch (py_netpoll.cpp): epoll `events` for this connection.
PyObject* netconn_dispatch(PyObject* o, uint32_t events) {
  NetConnObject* c = reinterpret_cast<NetConnObject*>(o);
  if (events & (EPOLLIN | EPOLLERR | EPOLLHUP | EPOLLRDHUP)) {
    PyObject* r = nc_on_readable(c, nullptr);
    if (!r) return nullptr;
    Py_DECREF(r);
  }
  if ((events & EPOLLOUT) && c->fd >= 0 && (c->writing || c->connecting)) {
    PyObject* r = nc_on_writable(c, nullptr);
    if (!r) return nullptr;
    Py_DECREF(r);
  }
  Py_RETURN_NONE;
}

PyObject* netconn_loop(PyObject* o) { return reinterpret_cast<NetConnObject*>(o)->loop; }

bool netconn_open(PyObject* o) {
  NetConnObject* c = reinterpret_cast<NetConnObject*>(o);
  return c->fd >= 0 && !c->closed;
}

// The h1 request of nc_request for a caller in C (sinks/h1.py fast path, py_h1call.cpp): parser
// started, `waiter` set, the request bytes written. 0, or -1 with an exception set.
int netconn_h1_request(PyObject* o, const char* data, size_t n, PyObject* waiter, bool head) {
  NetConnObject* c = reinterpret_cast<NetConnObject*>(o);
  if (c->kind != K_H1) {
    PyErr_SetString(PyExc_TypeError, "not an h1 NetConn");
    return -1;
  }
  if (c->fd < 0) {
    closed_error(c);
    return -1;
  }
  if (start_parser(c, head) < 0) return -1;  // parser.start(head=head)
  Py_INCREF(waiter);
  Py_XSETREF(c->waiter, waiter);
  c->out->append(data, n);
  if (c->writing) return 0;
  return send_out(c);
}

namespace {

PyObject *s_closed_name, *s_net_name;

// netconn_connect(ip, port, loop, kind, owner, parser, **NetConn keywords) -> NetConn
// A non-blocking TCP connect to the IP literal `ip` (IPv4 or IPv6) made here, without an asyncio
// transport: socket(2) + TCP_NODELAY + connect(2), then the NetConn watches for completion. Its
// `handshake` future resolves once the connection is usable (after the TLS handshake for `tls=`),
// or is rejected with the connect OSError (ECONNREFUSED, ...) or the TLS failure.
PyObject* mod_netconn_connect(PyObject*, PyObject* args, PyObject* kwds) {
  const char* ip;
  int port;
  PyObject *loop, *kind, *owner, *parser;
  if (!PyArg_ParseTuple(args, "siOOOO", &ip, &port, &loop, &kind, &owner, &parser)) return nullptr;
  sockaddr_storage ss;
  socklen_t slen;
  int family;
  memset(&ss, 0, sizeof ss);
  auto* s4 = reinterpret_cast<sockaddr_in*>(&ss);
  auto* s6 = reinterpret_cast<sockaddr_in6*>(&ss);
  if (inet_pton(AF_INET, ip, &s4->sin_addr) == 1) {
    family = AF_INET;
    s4->sin_family = AF_INET;
    s4->sin_port = htons(uint16_t(port));
    slen = sizeof *s4;
  } else if (inet_pton(AF_INET6, ip, &s6->sin6_addr) == 1) {
    family = AF_INET6;
    s6->sin6_family = AF_INET6;
    s6->sin6_port = htons(uint16_t(port));
    slen = sizeof *s6;
  } else {
    PyErr_Format(PyExc_ValueError, "netconn_connect: not an IP address: %s", ip);
    return nullptr;
  }
  if (port <= 0 || port > 65535) {
    PyErr_SetString(PyExc_ValueError, "netconn_connect: bad port");
    return nullptr;
  }
  int fd = ::socket(family, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
  if (fd < 0) return PyErr_SetFromErrno(PyExc_OSError);
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);  // small requests go out at once (as asyncio)
  int rc;
  do {
    rc = ::connect(fd, reinterpret_cast<sockaddr*>(&ss), slen);
  } while (rc < 0 && errno == EINTR);
  int cerr = rc < 0 ? errno : 0;
  if (cerr && cerr != EINPROGRESS) {
    ::close(fd);
    errno = cerr;
    return PyErr_SetFromErrno(PyExc_OSError);
  }
  // NetConn(fd, loop, kind, owner, parser, **kwds) with the connect pending: the TLS handshake
  // waits for connect_done()
  PyObject* fdo = PyLong_FromLong(fd);
  PyObject* a5 = fdo ? PyTuple_Pack(5, fdo, loop, kind, owner, parser) : nullptr;
  Py_XDECREF(fdo);
  if (!a5) {
    ::close(fd);
    return nullptr;
  }
  NetConnObject* c = reinterpret_cast<NetConnObject*>(NetConnType.tp_new(&NetConnType, a5, kwds));
  if (!c) {
    Py_DECREF(a5);
    ::close(fd);
    return nullptr;
  }
  c->connecting = 1;  // nc_init: no handshake yet
  int ok = NetConnType.tp_init(reinterpret_cast<PyObject*>(c), a5, kwds);
  Py_DECREF(a5);
  if (ok < 0) {
    if (c->fd < 0) ::close(fd);  // not owned yet
    Py_DECREF(c);
    return nullptr;
  }
  int rc2 = 0;
  if (!c->hs_fut && !(c->hs_fut = iofuture_new(loop))) rc2 = -1;
  if (rc2 == 0) rc2 = cerr == 0 ? connect_done(c) : watch_writes(c);  // connected at once: finish now
  if (rc2 < 0) {
    shut(c);  // registered with the loop: leave it before the reference goes
    Py_DECREF(c);
    return nullptr;
  }
  return reinterpret_cast<PyObject*>(c);
}

// pg_pool_execute(nets, sql, params, spread_at, size) -> IOFuture, or None for the Python path.
// store/pgwire.py Pool.execute for a pool whose connections are all native: `nets` is the pool's
// list of their NetConns (Pool._nets, None while any connection is on the asyncio path). The open
// one with the fewest queries in flight (the first on ties) gets the query, unless every one has
// `spread_at` or more in flight and the pool may still grow (fewer than `size` open). A NetConn's
// own closed flag is its connection's: PgConnection.closed is set in the same call that closes it.
PyObject* mod_pg_pool_execute(PyObject*, PyObject* const* a, Py_ssize_t n) {
  if (n != 5) {
    PyErr_SetString(PyExc_TypeError, "pg_pool_execute(nets: list | None, sql, params, spread_at, size)");
    return nullptr;
  }
  if (a[0] == Py_None) Py_RETURN_NONE;
  if (!PyList_CheckExact(a[0])) {
    PyErr_SetString(PyExc_TypeError, "pg_pool_execute: nets must be a list of NetConn or None");
    return nullptr;
  }
  Py_ssize_t spread = PyLong_AsSsize_t(a[3]);
  Py_ssize_t size = spread == -1 && PyErr_Occurred() ? -1 : PyLong_AsSsize_t(a[4]);
  if (size == -1 && PyErr_Occurred()) return nullptr;
  PyObject* nets = a[0];
  Py_ssize_t nc = PyList_GET_SIZE(nets);
  NetConnObject* best = nullptr;
  size_t bp = 0;
  Py_ssize_t live = 0;  // open connections: a closed one left in the list does not fill the pool
  for (Py_ssize_t i = 0; i < nc; ++i) {
    PyObject* net = PyList_GET_ITEM(nets, i);
    if (Py_TYPE(net) != &NetConnType) Py_RETURN_NONE;
    NetConnObject* nc_ = reinterpret_cast<NetConnObject*>(net);
    if (nc_->closed) continue;
    if (nc_->kind != K_PG) Py_RETURN_NONE;
    ++live;
    size_t p = nc_->pending->size();
    if (!best || p < bp) {
      best = nc_;
      bp = p;
    }
  }
  if (!best || !(bp < size_t(spread < 0 ? 0 : spread) || live >= size)) Py_RETURN_NONE;
  PyObject* args[2] = {a[1], a[2]};
  return nc_execute(best, args, 2);
}

// io_counts() -> {"h1_sends", "h1_recvs", "pg_sends", "pg_recvs", "poll_runs", "poll_ready"}:
// socket calls made by every NetConn of the process (a TLS record write / read counts as one),
// NetPoller callbacks and the sockets they found ready. Monotonic; callers take differences.
PyObject* mod_io_counts(PyObject*, PyObject*) {
  return Py_BuildValue("{s:K,s:K,s:K,s:K,s:K,s:K}", "h1_sends", g_io_calls[K_H1][0], "h1_recvs", g_io_calls[K_H1][1],
                       "pg_sends", g_io_calls[K_PG][0], "pg_recvs", g_io_calls[K_PG][1], "poll_runs", g_netpoll_runs,
                       "poll_ready", g_netpoll_ready);
}

PyMethodDef pool_functions[] = {
    {"io_counts", mod_io_counts, METH_NOARGS, "io_counts() -> dict of process-wide NetConn / NetPoller call counts"},
    {"netconn_connect", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(mod_netconn_connect)),
     METH_VARARGS | METH_KEYWORDS,
     "netconn_connect(ip, port, loop, kind, owner, parser, **NetConn keywords) -> NetConn; `handshake` resolves once "
     "connected (and TLS established)"},
    {"pg_pool_execute", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(mod_pg_pool_execute)),
     METH_FASTCALL, "pg_pool_execute(nets, sql, params, spread_at, size) -> IOFuture or None (store/pgwire.py Pool)"},
    {nullptr, nullptr, 0, nullptr}};

}  // namespace

// The NetPoller's drain of its completion channel: one finished handshake job.
void netconn_tls_done(void* job) {
  if (tls_done(static_cast<HsJob*>(job)) < 0) PyErr_WriteUnraisable(Py_None);
}

// The NetPoller's flush of a connection whose queries it collected.
void netconn_flush(PyObject* o) {
  PyObject* r = nc_flush(reinterpret_cast<NetConnObject*>(o), nullptr);
  if (!r)
    PyErr_WriteUnraisable(o);
  else
    Py_DECREF(r);
}

// pg_pool_execute for a caller in C (the compiled handlers' Postgres queries): the same pick,
// IOFuture or None (Python path), NULL on error.
PyObject* pg_pool_execute_c(PyObject* nets, PyObject* sql, PyObject* params, PyObject* spread_at, PyObject* size) {
  PyObject* a[5] = {nets, sql, params, spread_at, size};
  return mod_pg_pool_execute(nullptr, a, 5);
}

int init_netconn_types(PyObject* m) {
  struct {
    PyObject** slot;
    const char* text;
  } strs[] = {{&s_add_reader, "add_reader"},   {&s_remove_reader, "remove_reader"}, {&s_add_writer, "add_writer"},
              {&s_remove_writer, "remove_writer"}, {&s_call_soon, "call_soon"},   {&s_feed, "feed"},
              {&s_start, "start"},             {&s_head, "head"},                 {&s_net_lost, "_net_lost"},
              {&s_net_error, "_net_error"},    {&s_net_message, "_net_message"}};
  for (auto& s : strs)
    if (!(*s.slot = PyUnicode_InternFromString(s.text))) return -1;
  NetConnType.tp_name = "beholder_amd.ops._native.NetConn";
  NetConnType.tp_basicsize = sizeof(NetConnObject);
  NetConnType.tp_flags = Py_TPFLAGS_DEFAULT | Py_TPFLAGS_HAVE_GC;
  NetConnType.tp_doc =
      "NetConn(fd, loop, kind, owner, parser, stmts=None, pg_error=None, closed_exc=ConnectionError): plain-TCP "
      "client socket on the "
      "asyncio loop with native reply dispatch (kind 'h1' or 'pg')";
  NetConnType.tp_new = nc_new;
  NetConnType.tp_init = reinterpret_cast<initproc>(nc_init);
  NetConnType.tp_dealloc = reinterpret_cast<destructor>(nc_dealloc);
  NetConnType.tp_traverse = reinterpret_cast<traverseproc>(nc_traverse);
  NetConnType.tp_clear = reinterpret_cast<inquiry>(nc_clear);
  NetConnType.tp_methods = nc_methods;
  NetConnType.tp_getset = nc_getset;
  if (PyType_Ready(&NetConnType) < 0) return -1;
  Py_INCREF(&NetConnType);
  if (PyModule_AddObject(m, "NetConn", reinterpret_cast<PyObject*>(&NetConnType)) < 0) return -1;
  if (!(s_closed_name = PyUnicode_InternFromString("closed")) || !(s_net_name = PyUnicode_InternFromString("_net")))
    return -1;
  return PyModule_AddFunctions(m, pool_functions);
}

}  // namespace beholder
