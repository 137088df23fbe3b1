// Shared declarations for the `_native` CPython extension.
#pragma once

#define PY_SSIZE_T_CLEAN
#include <Python.h>

#include <pthread.h>

#include <cstdint>

#include "histogram.hpp"

#include <new>
#include <stdexcept>
#include <string>

namespace beholder {

// Per-event text (a log line, a URL path, a query, a request) is built in a std::string and turned
// into a str or handed to a socket buffer before the code that built it returns. A ScratchStr lends
// one of a few strings kept across events (cleared, capacity kept), so that text costs no heap
// allocation per event; a nested lender (a js_str() that runs Python code that logs) takes the next
// one, last in first out, and past kDepth a fresh local.
//
// The pool belongs to one thread: the first that makes a ScratchStr (the event loop's, in the
// service). Python code runs while a lent string is alive (a logger, a token callable, a __str__),
// and it may hand the GIL to another thread; a ScratchStr made on any other thread is a fresh local,
// so it never takes, or returns, a slot of the owner's stack.
class ScratchStr {
 public:
  ScratchStr() : s_(&own_) {
    const uintptr_t me = self_id();
    if (!owner_) owner_ = me;
    if (depth_ < kDepth && owner_ == me) s_ = &pool_[depth_++];
    s_->clear();
  }
  ~ScratchStr() {
    if (s_ == &own_) return;
    if (s_->capacity() > kKeepBytes) std::string().swap(*s_);  // an outsized one is not kept
    --depth_;
  }
  ScratchStr(const ScratchStr&) = delete;
  ScratchStr& operator=(const ScratchStr&) = delete;
  std::string& operator*() { return *s_; }

 private:
  static constexpr int kDepth = 8;
  static constexpr size_t kKeepBytes = 65536;
  // the calling thread's identity: its thread pointer (the TCB address, what pthread_self()
  // returns on glibc), read inline on x86-64 / aarch64 instead of a libc call per string
  static uintptr_t self_id() {
#if defined(__x86_64__) || defined(__aarch64__)
    return reinterpret_cast<uintptr_t>(__builtin_thread_pointer());
#else
    return static_cast<uintptr_t>(pthread_self());
#endif
  }
  static inline std::string pool_[kDepth];
  static inline int depth_ = 0;
  static inline uintptr_t owner_ = 0;
  std::string own_;
  std::string* s_;
};

// C++ exceptions must never cross into CPython (std::terminate). Entry points
// that allocate wrap their body: BEHOLDER_TRY { ... } BEHOLDER_CATCH(nullptr)
#define BEHOLDER_TRY try
#define BEHOLDER_CATCH(errval)                                 \
  catch (const std::bad_alloc&) {                              \
    PyErr_NoMemory();                                          \
    return errval;                                             \
  }                                                            \
  catch (const std::exception& e) {                            \
    PyErr_Format(PyExc_RuntimeError, "native error: %s", e.what()); \
    return errval;                                             \
  }

// Values of a fixed set of keys in one dict, looked up again only after that dict changed. Every
// modification of a dict gives it a new process-wide version (CPython 3.10/3.11 `ma_version_tag`, a
// global counter), so the same dict object at the same version still holds the same values: the
// hot paths read a client's or a store's configuration attributes from its instance dict per
// request, and those never change after setup. Zero-initialised (tp_alloc / static) is empty.
// Values are borrowed, exactly as PyDict_GetItemWithError's are (valid until the dict changes).
template <int N>
struct DictView {
  PyObject* dict;
  uint64_t version;
  PyObject* v[N];
  // `keys`: addresses of the interned key objects. false = a lookup raised (v not valid).
  bool refresh(PyObject* d, PyObject* const* const* keys) {
#if PY_VERSION_HEX < 0x030C0000
    const uint64_t ver = reinterpret_cast<PyDictObject*>(d)->ma_version_tag;
    if (d == dict && ver == version) return true;
#else  // the version tag is deprecated from 3.12 (PEP 699): look the keys up every time
    const uint64_t ver = 0;
#endif
    dict = nullptr;
    for (int i = 0; i < N; ++i) {
      v[i] = PyDict_GetItemWithError(d, *keys[i]);
      if (!v[i] && PyErr_Occurred()) return false;
    }
    dict = d;
    version = ver;
    return true;
  }
};

// Module-level state (single-phase init; one interpreter).
struct ModuleState {
  PyObject* decode_error;  // exception raised by MessageCodec.decode
  PyObject* topics;        // tuple: topic id -> topic name (str) or None
};
extern ModuleState g_state;

// ---- Histogram ------------------------------------------------------------
struct HistogramObject {
  PyObject_HEAD LogHistogram* h;
};
extern PyTypeObject HistogramType;

// ---- Counter --------------------------------------------------------------
struct CounterObject {
  PyObject_HEAD double value;
};
extern PyTypeObject CounterType;

// ---- Settler: ack accounting shared by all deliveries of one source --------
struct SettlerObject {
  PyObject_HEAD HistogramObject* handle_hist;  // start() -> settle, ns
  HistogramObject* ingest_hist;                // recv -> settle, ns
  HistogramObject* queue_hist;                 // recv -> start(), ns (ring + loop wait)
  uint64_t created, acked, nacked, rejected, abandoned;
  PyObject* on_settle;   // optional callable(delivery, kind:str, requeue:bool)
  PyObject* on_abandon;  // optional callable(tag, topic_id, content)
  PyObject* batcher;     // optional AckBatcher: acks of its channel's deliveries stay in C
  // slow-delivery trace (bench attribution): (recv, start, settle) ns of every delivery whose
  // start->settle took >= slow_threshold_ns, up to slow_cap entries; 0 = off
  int64_t slow_threshold_ns;
  uint64_t slow_cap, slow_dropped;
  void* slow;  // std::vector<int64_t>*, owned (3 values per entry)
};

// AckBatcher hooks (py_acks.cpp): 1 = handled, 0 = other channel, -1 = error
int ack_batcher_ack(PyObject* batcher, PyObject* channel, uint64_t tag);
void ack_batcher_abandon(PyObject* batcher, PyObject* channel, uint64_t tag);
bool is_ack_batcher(PyObject* o);
extern PyTypeObject SettlerType;

// ---- Delivery: one inbound message (rmsg of index.js:62,127) ---------------
enum DeliveryState : uint8_t { D_PENDING = 0, D_ACKED = 1, D_NACKED = 2, D_REJECTED = 3 };

struct DeliveryObject {
  PyObject_HEAD PyObject* content;  // bytes
  SettlerObject* settler;           // may be NULL
  PyObject* extra;                  // transport-specific payload, may be NULL
  PyObject* headers;                // message headers (dict, or raw AMQP field-table bytes), may be NULL
  uint64_t tag;
  int64_t recv_ns;
  int64_t start_ns;
  uint8_t topic;
  uint8_t state;
  uint8_t redelivered;
};
extern PyTypeObject DeliveryType;

// A tuple row holding only atoms leaves the cyclic collector (py_handlers.cpp).
void untrack_atomic_row(PyObject* t);

// rmsg.ack() of a native Delivery, called directly (py_handlers.cpp). New reference or NULL.
PyObject* delivery_ack_c(PyObject* d);

// Creates a pending delivery; steals nothing (increfs content/settler).
PyObject* delivery_new(PyObject* content, uint8_t topic, uint64_t tag, int64_t recv_ns,
                       SettlerObject* settler, bool redelivered);

// ---- Ingest ring + reader thread --------------------------------------------
extern PyTypeObject IngestType;

// ---- MessageCodec -----------------------------------------------------------
extern PyTypeObject CodecType;

int init_codec_types(PyObject* m);
int init_metric_types(PyObject* m);
int init_ingest_types(PyObject* m);
int init_text_functions(PyObject* m);
int init_amqp_types(PyObject* m);
int init_dispatch_functions(PyObject* m);
int init_http_types(PyObject* m);
int init_pg_types(PyObject* m);
int init_driver_types(PyObject* m);
int init_ack_types(PyObject* m);
int init_handler_types(PyObject* m);
int init_netconn_types(PyObject* m);
int init_h1call_types(PyObject* m);
int init_tls_types(PyObject* m);
int init_netpoll_types(PyObject* m);
int init_clock_functions(PyObject* m);  // gil_clock.cpp

// ---- Window (py_driver.cpp): the in-flight set dispatch_batch hands suspended handlers to ----
bool is_window(PyObject* o);
PyObject* window_suspend_c(PyObject* w, PyObject* payload, PyObject* coro, PyObject* first);

}  // namespace beholder
