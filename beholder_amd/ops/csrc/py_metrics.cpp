// Native metric primitives: Counter (prom-client Counter semantics, used for
// `beholder_progress_updates_total` / `beholder_trello_comments`,
// index.js:29-40) and Histogram (log-linear latency histogram, ns).
#include <cmath>
#include <cstring>
#include <string>

#include "py_common.hpp"

namespace beholder {

// ============================== Histogram ===================================
namespace {

PyObject* hist_new(PyTypeObject* type, PyObject*, PyObject*) {
  HistogramObject* self = reinterpret_cast<HistogramObject*>(type->tp_alloc(type, 0));
  if (!self) return nullptr;
  self->h = new (std::nothrow) LogHistogram();
  if (!self->h) {
    Py_DECREF(self);
    return PyErr_NoMemory();
  }
  return reinterpret_cast<PyObject*>(self);
}

void hist_dealloc(HistogramObject* self) {
  delete self->h;
  Py_TYPE(self)->tp_free(reinterpret_cast<PyObject*>(self));
}

bool as_u64(PyObject* v, uint64_t* out) {
  if (PyFloat_Check(v)) {
    double d = PyFloat_AS_DOUBLE(v);
    *out = d <= 0 ? 0 : uint64_t(d);
    return true;
  }
  long long x = PyLong_AsLongLong(v);
  if (x == -1 && PyErr_Occurred()) return false;
  *out = x < 0 ? 0 : uint64_t(x);
  return true;
}

PyObject* hist_record(HistogramObject* self, PyObject* const* args, Py_ssize_t nargs) {
  if (nargs < 1 || nargs > 2) {
    PyErr_SetString(PyExc_TypeError, "record(value, count=1)");
    return nullptr;
  }
  uint64_t v, n = 1;
  if (!as_u64(args[0], &v)) return nullptr;
  if (nargs == 2 && !as_u64(args[1], &n)) return nullptr;
  self->h->record(v, n);
  Py_RETURN_NONE;
}

PyObject* hist_record_many(HistogramObject* self, PyObject* seq_in) {
  PyObject* seq = PySequence_Fast(seq_in, "record_many expects a sequence");
  if (!seq) return nullptr;
  Py_ssize_t n = PySequence_Fast_GET_SIZE(seq);
  for (Py_ssize_t i = 0; i < n; ++i) {
    uint64_t v;
    if (!as_u64(PySequence_Fast_GET_ITEM(seq, i), &v)) {
      Py_DECREF(seq);
      return nullptr;
    }
    self->h->record(v);
  }
  Py_DECREF(seq);
  Py_RETURN_NONE;
}

PyObject* hist_percentile(HistogramObject* self, PyObject* arg) {
  double p = PyFloat_AsDouble(arg);
  if (p == -1.0 && PyErr_Occurred()) return nullptr;
  return PyFloat_FromDouble(self->h->percentile(p));
}

PyObject* hist_count_le(HistogramObject* self, PyObject* arg) {
  uint64_t v;
  if (!as_u64(arg, &v)) return nullptr;
  return PyLong_FromUnsignedLongLong(self->h->count_le(v));
}

PyObject* hist_reset(HistogramObject* self, PyObject*) {
  self->h->reset();
  Py_RETURN_NONE;
}

PyObject* hist_merge(HistogramObject* self, PyObject* other) {
  if (!PyObject_TypeCheck(other, &HistogramType)) {
    PyErr_SetString(PyExc_TypeError, "merge() expects a Histogram");
    return nullptr;
  }
  self->h->merge(*reinterpret_cast<HistogramObject*>(other)->h);
  Py_RETURN_NONE;
}

// Serialization for cross-rank aggregation: header (total, sum, min, max) +
// sparse (index, count) pairs.
PyObject* hist_to_bytes_impl(HistogramObject* self, PyObject*);
PyObject* hist_to_bytes(HistogramObject* self, PyObject*) {
  BEHOLDER_TRY { return hist_to_bytes_impl(self, nullptr); }
  BEHOLDER_CATCH(nullptr)
}

PyObject* hist_to_bytes_impl(HistogramObject* self, PyObject*) {
  const auto& c = self->h->counts();
  std::string out;
  uint64_t hdr[4] = {self->h->total(), 0, self->h->min(), self->h->max()};
  double s = self->h->sum();
  memcpy(&hdr[1], &s, 8);
  out.append(reinterpret_cast<const char*>(hdr), sizeof hdr);
  for (size_t i = 0; i < c.size(); ++i) {
    if (!c[i]) continue;
    uint64_t pair[2] = {uint64_t(i), c[i]};
    out.append(reinterpret_cast<const char*>(pair), sizeof pair);
  }
  return PyBytes_FromStringAndSize(out.data(), Py_ssize_t(out.size()));
}

PyObject* hist_merge_bytes_impl(HistogramObject* self, PyObject* arg);
PyObject* hist_merge_bytes(HistogramObject* self, PyObject* arg) {
  BEHOLDER_TRY { return hist_merge_bytes_impl(self, arg); }
  BEHOLDER_CATCH(nullptr)
}

PyObject* hist_merge_bytes_impl(HistogramObject* self, PyObject* arg) {
  char* p;
  Py_ssize_t n;
  if (PyBytes_AsStringAndSize(arg, &p, &n) < 0) return nullptr;
  if (n < 32 || (n - 32) % 16 != 0) {
    PyErr_SetString(PyExc_ValueError, "corrupt histogram bytes");
    return nullptr;
  }
  uint64_t hdr[4];
  memcpy(hdr, p, 32);
  LogHistogram tmp;
  auto& c = tmp.mutable_counts();
  for (Py_ssize_t off = 32; off < n; off += 16) {
    uint64_t pair[2];
    memcpy(pair, p + off, 16);
    if (pair[0] >= c.size()) {
      PyErr_SetString(PyExc_ValueError, "corrupt histogram bytes (bucket index)");
      return nullptr;
    }
    c[pair[0]] += pair[1];
  }
  double s;
  memcpy(&s, &hdr[1], 8);
  tmp.set_stats(hdr[0], s, hdr[0] ? hdr[2] : UINT64_MAX, hdr[3]);
  self->h->merge(tmp);
  Py_RETURN_NONE;
}

PyObject* hist_summary(HistogramObject* self, PyObject*) {
  LogHistogram* h = self->h;
  return Py_BuildValue("{s:K,s:d,s:K,s:K,s:d,s:d,s:d,s:d,s:d}", "count", (unsigned long long)h->total(), "sum",
                       h->sum(), "min", (unsigned long long)h->min(), "max", (unsigned long long)h->max(), "mean",
                       h->total() ? h->sum() / double(h->total()) : 0.0, "p50", h->percentile(50), "p90",
                       h->percentile(90), "p99", h->percentile(99), "p999", h->percentile(99.9));
}

PyObject* hist_get_count(HistogramObject* self, void*) { return PyLong_FromUnsignedLongLong(self->h->total()); }
PyObject* hist_get_sum(HistogramObject* self, void*) { return PyFloat_FromDouble(self->h->sum()); }
PyObject* hist_get_min(HistogramObject* self, void*) { return PyLong_FromUnsignedLongLong(self->h->min()); }
PyObject* hist_get_max(HistogramObject* self, void*) { return PyLong_FromUnsignedLongLong(self->h->max()); }

PyMethodDef hist_methods[] = {
    {"record", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(hist_record)), METH_FASTCALL,
     "record(value, count=1)"},
    {"record_many", reinterpret_cast<PyCFunction>(hist_record_many), METH_O, "record each value of a sequence"},
    {"percentile", reinterpret_cast<PyCFunction>(hist_percentile), METH_O, "percentile(p in [0,100])"},
    {"count_le", reinterpret_cast<PyCFunction>(hist_count_le), METH_O, "number of samples <= value"},
    {"reset", reinterpret_cast<PyCFunction>(hist_reset), METH_NOARGS, "clear all samples"},
    {"merge", reinterpret_cast<PyCFunction>(hist_merge), METH_O, "add another Histogram's samples"},
    {"to_bytes", reinterpret_cast<PyCFunction>(hist_to_bytes), METH_NOARGS, "serialize (sparse)"},
    {"merge_bytes", reinterpret_cast<PyCFunction>(hist_merge_bytes), METH_O, "merge a to_bytes() payload"},
    {"summary", reinterpret_cast<PyCFunction>(hist_summary), METH_NOARGS, "dict of count/sum/min/max/percentiles"},
    {nullptr, nullptr, 0, nullptr}};

PyGetSetDef hist_getset[] = {
    {"count", reinterpret_cast<getter>(hist_get_count), nullptr, "number of samples", nullptr},
    {"sum", reinterpret_cast<getter>(hist_get_sum), nullptr, "sum of samples", nullptr},
    {"min", reinterpret_cast<getter>(hist_get_min), nullptr, "smallest sample", nullptr},
    {"max", reinterpret_cast<getter>(hist_get_max), nullptr, "largest sample", nullptr},
    {nullptr, nullptr, nullptr, nullptr, nullptr}};

// ================================ Counter ===================================
PyObject* counter_new(PyTypeObject* type, PyObject*, PyObject*) {
  CounterObject* self = reinterpret_cast<CounterObject*>(type->tp_alloc(type, 0));
  if (self) self->value = 0.0;
  return reinterpret_cast<PyObject*>(self);
}

void counter_dealloc(CounterObject* self) { Py_TYPE(self)->tp_free(reinterpret_cast<PyObject*>(self)); }

PyObject* counter_inc(CounterObject* self, PyObject* const* args, Py_ssize_t nargs) {
  if (nargs == 0) {
    self->value += 1.0;
    Py_RETURN_NONE;
  }
  if (nargs > 1) {
    PyErr_SetString(PyExc_TypeError, "inc(amount=1)");
    return nullptr;
  }
  double d = PyFloat_AsDouble(args[0]);
  if (d == -1.0 && PyErr_Occurred()) return nullptr;
  if (!(d >= 0.0) || std::isinf(d)) {
    // prom-client: "It is not possible to decrease a counter"
    PyErr_SetString(PyExc_ValueError, "counters can only be incremented by a non-negative finite amount");
    return nullptr;
  }
  self->value += d;
  Py_RETURN_NONE;
}

PyObject* counter_reset(CounterObject* self, PyObject*) {
  self->value = 0.0;
  Py_RETURN_NONE;
}

PyObject* counter_get(CounterObject* self, void*) { return PyFloat_FromDouble(self->value); }

PyMethodDef counter_methods[] = {
    {"inc", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(counter_inc)), METH_FASTCALL,
     "inc(amount=1)"},
    {"reset", reinterpret_cast<PyCFunction>(counter_reset), METH_NOARGS, "reset to 0"},
    {nullptr, nullptr, 0, nullptr}};

PyGetSetDef counter_getset[] = {{"value", reinterpret_cast<getter>(counter_get), nullptr, "current value", nullptr},
                                {nullptr, nullptr, nullptr, nullptr, nullptr}};

}  // namespace

PyTypeObject HistogramType = {PyVarObject_HEAD_INIT(nullptr, 0)};
PyTypeObject CounterType = {PyVarObject_HEAD_INIT(nullptr, 0)};

// ---- Buckets: prom-client fixed-bucket histogram cell (one label set) ----------
// observe(v) counts v in the first bucket whose upper bound is >= v (`le`), plus sum/count.
struct BucketsObject {
  PyObject_HEAD double* bounds;
  uint64_t* counts;  // per bucket, non-cumulative
  Py_ssize_t n;
  double sum;
  uint64_t count;
};

PyTypeObject BucketsType = {PyVarObject_HEAD_INIT(nullptr, 0)};

PyObject* buckets_new(PyTypeObject* type, PyObject* args, PyObject* kwds) {
  static const char* kwlist[] = {"bounds", nullptr};
  PyObject* seq;
  if (!PyArg_ParseTupleAndKeywords(args, kwds, "O", const_cast<char**>(kwlist), &seq)) return nullptr;
  PyObject* fast = PySequence_Fast(seq, "bounds must be a sequence of numbers");
  if (!fast) return nullptr;
  Py_ssize_t n = PySequence_Fast_GET_SIZE(fast);
  if (n < 1 || n > 4096) {
    Py_DECREF(fast);
    PyErr_SetString(PyExc_ValueError, "1..4096 bucket bounds required");
    return nullptr;
  }
  BucketsObject* self = reinterpret_cast<BucketsObject*>(type->tp_alloc(type, 0));
  if (!self) {
    Py_DECREF(fast);
    return nullptr;
  }
  self->bounds = static_cast<double*>(PyMem_Calloc(size_t(n), sizeof(double)));
  self->counts = static_cast<uint64_t*>(PyMem_Calloc(size_t(n), sizeof(uint64_t)));
  self->n = n;
  self->sum = 0.0;
  self->count = 0;
  if (!self->bounds || !self->counts) {
    Py_DECREF(fast);
    Py_DECREF(self);
    return PyErr_NoMemory();
  }
  for (Py_ssize_t i = 0; i < n; ++i) {
    double b = PyFloat_AsDouble(PySequence_Fast_GET_ITEM(fast, i));
    if (b == -1.0 && PyErr_Occurred()) {
      Py_DECREF(fast);
      Py_DECREF(self);
      return nullptr;
    }
    if (i && !(b > self->bounds[i - 1])) {
      Py_DECREF(fast);
      Py_DECREF(self);
      PyErr_SetString(PyExc_ValueError, "bucket bounds must be strictly increasing");
      return nullptr;
    }
    self->bounds[i] = b;
  }
  Py_DECREF(fast);
  return reinterpret_cast<PyObject*>(self);
}

void buckets_dealloc(BucketsObject* self) {
  PyMem_Free(self->bounds);
  PyMem_Free(self->counts);
  Py_TYPE(self)->tp_free(reinterpret_cast<PyObject*>(self));
}

PyObject* buckets_observe(BucketsObject* self, PyObject* arg) {
  double v = PyFloat_AsDouble(arg);
  if (v == -1.0 && PyErr_Occurred()) return nullptr;
  // lower_bound: first bound >= v (bisect_left); NaN lands past the last bucket (+Inf only)
  Py_ssize_t lo = 0, hi = self->n;
  while (lo < hi) {
    Py_ssize_t mid = (lo + hi) >> 1;
    if (self->bounds[mid] < v) lo = mid + 1; else hi = mid;
  }
  if (lo < self->n && !(v != v)) self->counts[lo]++;
  self->sum += v;
  self->count++;
  Py_RETURN_NONE;
}

PyObject* buckets_snapshot(BucketsObject* self, PyObject*) {
  PyObject* counts = PyList_New(self->n);
  if (!counts) return nullptr;
  for (Py_ssize_t i = 0; i < self->n; ++i) {
    PyObject* c = PyLong_FromUnsignedLongLong(self->counts[i]);
    if (!c) {
      Py_DECREF(counts);
      return nullptr;
    }
    PyList_SET_ITEM(counts, i, c);
  }
  return Py_BuildValue("(NdK)", counts, self->sum, (unsigned long long)self->count);
}

PyObject* buckets_reset(BucketsObject* self, PyObject*) {
  for (Py_ssize_t i = 0; i < self->n; ++i) self->counts[i] = 0;
  self->sum = 0.0;
  self->count = 0;
  Py_RETURN_NONE;
}

PyMethodDef buckets_methods[] = {
    {"observe", reinterpret_cast<PyCFunction>(buckets_observe), METH_O, "observe(value)"},
    {"snapshot", reinterpret_cast<PyCFunction>(buckets_snapshot), METH_NOARGS,
     "snapshot() -> ([per-bucket counts], sum, count)"},
    {"reset", reinterpret_cast<PyCFunction>(buckets_reset), METH_NOARGS, "zero everything"},
    {nullptr, nullptr, 0, nullptr}};

// ---- SinkStats: per-sink request accounting (sinks/http.py SinkObserver.child) --------
// record(status, seconds): beholder_sink_requests_total{sink,code} += 1 (code = HTTP status,
// or "error" for a transport failure) and beholder_sink_request_seconds{sink}.observe(seconds).
struct SinkStatsObject {
  PyObject_HEAD PyObject* requests;  // the labelled Counter metric (Python, labels(sink, code))
  PyObject* hist;                    // histogram child for this sink (Buckets or any .observe)
  PyObject* sink;                    // sink name (str)
  PyObject* codes;                   // dict: status (int / None) -> counter child
};

PyTypeObject SinkStatsType = {PyVarObject_HEAD_INIT(nullptr, 0)};

bool observe_value(PyObject* hist, double v) {
  if (Py_TYPE(hist) == &BucketsType) {
    BucketsObject* b = reinterpret_cast<BucketsObject*>(hist);
    Py_ssize_t lo = 0, hi = b->n;
    while (lo < hi) {
      Py_ssize_t mid = (lo + hi) >> 1;
      if (b->bounds[mid] < v) lo = mid + 1; else hi = mid;
    }
    if (lo < b->n && !(v != v)) b->counts[lo]++;
    b->sum += v;
    b->count++;
    return true;
  }
  PyObject* f = PyFloat_FromDouble(v);
  if (!f) return false;
  PyObject* r = PyObject_CallMethod(hist, "observe", "O", f);
  Py_DECREF(f);
  if (!r) return false;
  Py_DECREF(r);
  return true;
}

bool sink_stats_record(PyObject* obj, PyObject* status, double seconds) {
  SinkStatsObject* s = reinterpret_cast<SinkStatsObject*>(obj);
  PyObject* c = PyDict_GetItemWithError(s->codes, status);
  if (!c) {
    if (PyErr_Occurred()) return false;
    PyObject* code = status == Py_None ? PyUnicode_FromString("error") : PyObject_Str(status);
    if (!code) return false;
    c = PyObject_CallMethod(s->requests, "labels", "OO", s->sink, code);
    Py_DECREF(code);
    if (!c) return false;
    int rc = PyDict_SetItem(s->codes, status, c);
    Py_DECREF(c);  // the dict holds it
    if (rc < 0) return false;
  }
  if (Py_TYPE(c) == &CounterType) {
    reinterpret_cast<CounterObject*>(c)->value += 1.0;
  } else {
    PyObject* r = PyObject_CallMethod(c, "inc", nullptr);
    if (!r) return false;
    Py_DECREF(r);
  }
  return observe_value(s->hist, seconds);
}

bool is_sink_stats(PyObject* o) { return Py_TYPE(o) == &SinkStatsType; }

namespace {

PyObject* sinkstats_new(PyTypeObject* type, PyObject* args, PyObject* kwds) {
  static const char* kwlist[] = {"requests", "hist", "sink", nullptr};
  PyObject *req, *hist, *sink;
  if (!PyArg_ParseTupleAndKeywords(args, kwds, "OOU", const_cast<char**>(kwlist), &req, &hist, &sink))
    return nullptr;
  SinkStatsObject* s = reinterpret_cast<SinkStatsObject*>(type->tp_alloc(type, 0));
  if (!s) return nullptr;
  Py_INCREF(req);
  s->requests = req;
  Py_INCREF(hist);
  s->hist = hist;
  Py_INCREF(sink);
  s->sink = sink;
  s->codes = PyDict_New();
  if (!s->codes) {
    Py_DECREF(s);
    return nullptr;
  }
  return reinterpret_cast<PyObject*>(s);
}

int sinkstats_traverse(SinkStatsObject* s, visitproc visit, void* arg) {
  Py_VISIT(s->requests);
  Py_VISIT(s->hist);
  Py_VISIT(s->codes);
  return 0;
}

int sinkstats_clear(SinkStatsObject* s) {
  Py_CLEAR(s->requests);
  Py_CLEAR(s->hist);
  Py_CLEAR(s->sink);
  Py_CLEAR(s->codes);
  return 0;
}

void sinkstats_dealloc(SinkStatsObject* s) {
  PyObject_GC_UnTrack(s);
  sinkstats_clear(s);
  Py_TYPE(s)->tp_free(reinterpret_cast<PyObject*>(s));
}

PyObject* sinkstats_record(SinkStatsObject* s, PyObject* const* a, Py_ssize_t n) {
  if (n != 2) {
    PyErr_SetString(PyExc_TypeError, "record(status, seconds)");
    return nullptr;
  }
  double sec = PyFloat_AsDouble(a[1]);
  if (sec == -1.0 && PyErr_Occurred()) return nullptr;
  if (!sink_stats_record(reinterpret_cast<PyObject*>(s), a[0], sec)) return nullptr;
  Py_RETURN_NONE;
}

PyObject* sinkstats_get_sink(SinkStatsObject* s, void*) {
  Py_INCREF(s->sink);
  return s->sink;
}

PyMethodDef sinkstats_methods[] = {
    {"record", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(sinkstats_record)), METH_FASTCALL,
     "record(status or None, seconds)"},
    {nullptr, nullptr, 0, nullptr}};

PyGetSetDef sinkstats_getset[] = {{"sink", reinterpret_cast<getter>(sinkstats_get_sink), nullptr, "sink name", nullptr},
                                  {nullptr, nullptr, nullptr, nullptr, nullptr}};

}  // namespace

int init_metric_types(PyObject* m) {
  SinkStatsType.tp_name = "beholder_amd.ops._native.SinkStats";
  SinkStatsType.tp_basicsize = sizeof(SinkStatsObject);
  SinkStatsType.tp_flags = Py_TPFLAGS_DEFAULT | Py_TPFLAGS_HAVE_GC;
  SinkStatsType.tp_doc = "SinkStats(requests, hist, sink): per-sink request counter + latency histogram";
  SinkStatsType.tp_new = sinkstats_new;
  SinkStatsType.tp_dealloc = reinterpret_cast<destructor>(sinkstats_dealloc);
  SinkStatsType.tp_traverse = reinterpret_cast<traverseproc>(sinkstats_traverse);
  SinkStatsType.tp_clear = reinterpret_cast<inquiry>(sinkstats_clear);
  SinkStatsType.tp_methods = sinkstats_methods;
  SinkStatsType.tp_getset = sinkstats_getset;
  if (PyType_Ready(&SinkStatsType) < 0) return -1;
  Py_INCREF(&SinkStatsType);
  if (PyModule_AddObject(m, "SinkStats", reinterpret_cast<PyObject*>(&SinkStatsType)) < 0) return -1;

  BucketsType.tp_name = "beholder_amd.ops._native.Buckets";
  BucketsType.tp_basicsize = sizeof(BucketsObject);
  BucketsType.tp_flags = Py_TPFLAGS_DEFAULT;
  BucketsType.tp_doc = "Buckets(bounds): prom fixed-bucket histogram cell (le semantics)";
  BucketsType.tp_new = buckets_new;
  BucketsType.tp_dealloc = reinterpret_cast<destructor>(buckets_dealloc);
  BucketsType.tp_methods = buckets_methods;
  if (PyType_Ready(&BucketsType) < 0) return -1;
  Py_INCREF(&BucketsType);
  if (PyModule_AddObject(m, "Buckets", reinterpret_cast<PyObject*>(&BucketsType)) < 0) return -1;

  HistogramType.tp_name = "beholder_amd.ops._native.Histogram";
  HistogramType.tp_basicsize = sizeof(HistogramObject);
  HistogramType.tp_flags = Py_TPFLAGS_DEFAULT;
  HistogramType.tp_doc = "Log-linear histogram of non-negative integers (ns), <0.8% relative error";
  HistogramType.tp_new = hist_new;
  HistogramType.tp_dealloc = reinterpret_cast<destructor>(hist_dealloc);
  HistogramType.tp_methods = hist_methods;
  HistogramType.tp_getset = hist_getset;
  if (PyType_Ready(&HistogramType) < 0) return -1;

  CounterType.tp_name = "beholder_amd.ops._native.Counter";
  CounterType.tp_basicsize = sizeof(CounterObject);
  CounterType.tp_flags = Py_TPFLAGS_DEFAULT;
  CounterType.tp_doc = "Monotonic float64 counter (prom-client Counter semantics)";
  CounterType.tp_new = counter_new;
  CounterType.tp_dealloc = reinterpret_cast<destructor>(counter_dealloc);
  CounterType.tp_methods = counter_methods;
  CounterType.tp_getset = counter_getset;
  if (PyType_Ready(&CounterType) < 0) return -1;

  Py_INCREF(&HistogramType);
  if (PyModule_AddObject(m, "Histogram", reinterpret_cast<PyObject*>(&HistogramType)) < 0) return -1;
  Py_INCREF(&CounterType);
  if (PyModule_AddObject(m, "Counter", reinterpret_cast<PyObject*>(&CounterType)) < 0) return -1;
  return 0;
}

}  // namespace beholder
