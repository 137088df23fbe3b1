// Native text helpers for the per-message hot path:
//   * js_number / js_str — JavaScript String() rendering (ECMAScript
//     Number::toString), used for log text and template literals;
//   * format_line — a complete pino v5 JSON log line (index.js:11-13), with
//     quick-format-unescaped %s/%d/%i/%f/%j/%o/%O handling (+ the Q11 fix:
//     extra positional args are appended, not dropped);
//   * quote_component / encode_query — encodeURIComponent + Node querystring
//     (Trello / Telegram / Emby URLs, index.js:53,83,99,112).
// Semantics are pinned by tests/test_text.py against the Python reference
// implementations in beholder_amd/utils/log.py and sinks/http.py.
#include <time.h>

#include <cmath>
#include <cstddef>
#include <cstdio>
#include <cstring>
#include <string>

#include "py_common.hpp"
#include "gil_clock.hpp"

namespace beholder {

namespace {

PyObject* g_fallback_str = nullptr;   // python js_str for unsupported types
PyObject* g_fallback_json = nullptr;  // python json.dumps-like for %j/%o/%O

// ---- JS number formatting ----------------------------------------------------
void js_number_append(std::string& out, double x) {
  if (std::isnan(x)) {
    out += "NaN";
    return;
  }
  if (std::isinf(x)) {
    out += x > 0 ? "Infinity" : "-Infinity";
    return;
  }
  if (x == 0) {
    out += "0";
    return;
  }
  if (x < 0) {
    out += '-';
    x = -x;
  }
  // shortest round-trip digits, e.g. "1e-07", "45.5", "1.2345678901234569e+23"
  char* r = PyOS_double_to_string(x, 'r', 0, 0, nullptr);
  if (!r) {
    PyErr_Clear();
    char buf[64];
    snprintf(buf, sizeof buf, "%.17g", x);
    out += buf;
    return;
  }
  std::string s(r);
  PyMem_Free(r);
  int exp = 0;
  size_t epos = s.find_first_of("eE");
  std::string mant = s;
  if (epos != std::string::npos) {
    exp = atoi(s.c_str() + epos + 1);
    mant = s.substr(0, epos);
  }
  std::string ip, fp;
  size_t dot = mant.find('.');
  if (dot == std::string::npos) {
    ip = mant;
  } else {
    ip = mant.substr(0, dot);
    fp = mant.substr(dot + 1);
  }
  std::string all = ip + fp;
  size_t lead = 0;
  while (lead < all.size() && all[lead] == '0') ++lead;
  std::string digits = all.substr(lead);
  int n = int(ip.size()) - int(lead) + exp;
  while (!digits.empty() && digits.back() == '0') digits.pop_back();
  if (digits.empty()) digits = "0";
  int k = int(digits.size());
  if (k <= n && n <= 21) {
    out += digits;
    out.append(size_t(n - k), '0');
  } else if (0 < n && n <= 21) {
    out.append(digits, 0, size_t(n));
    out += '.';
    out.append(digits, size_t(n), std::string::npos);
  } else if (-6 < n && n <= 0) {
    out += "0.";
    out.append(size_t(-n), '0');
    out += digits;
  } else {
    int e = n - 1;
    out += digits[0];
    if (k > 1) {
      out += '.';
      out.append(digits, 1, std::string::npos);
    }
    out += 'e';
    out += e >= 0 ? '+' : '-';
    out += std::to_string(e >= 0 ? e : -e);
  }
}

// Decimal text of a 64-bit integer (the hot log / query path: no snprintf).
void append_i64(std::string& out, long long x) {
  char buf[24];
  char* e = buf + sizeof buf;
  char* p = e;
  unsigned long long u = x < 0 ? 0ULL - static_cast<unsigned long long>(x) : static_cast<unsigned long long>(x);
  do {
    *--p = char('0' + u % 10);
    u /= 10;
  } while (u);
  if (x < 0) *--p = '-';
  out.append(p, size_t(e - p));
}

// Appends String(v). Returns false with a Python error set on failure.
bool js_str_append(std::string& out, PyObject* v) {
  if (PyUnicode_CheckExact(v)) {
    Py_ssize_t n;
    const char* s = PyUnicode_AsUTF8AndSize(v, &n);
    if (!s) return false;
    out.append(s, size_t(n));
    return true;
  }
  if (v == Py_None) {
    out += "undefined";
    return true;
  }
  if (v == Py_True) {
    out += "true";
    return true;
  }
  if (v == Py_False) {
    out += "false";
    return true;
  }
  if (PyLong_CheckExact(v)) {
    int overflow = 0;
    long long x = PyLong_AsLongLongAndOverflow(v, &overflow);
    if (!overflow) {
      append_i64(out, x);
      return true;
    }
  }
  if (PyFloat_CheckExact(v)) {
    js_number_append(out, PyFloat_AS_DOUBLE(v));
    return true;
  }
  PyObject* s = g_fallback_str ? PyObject_CallOneArg(g_fallback_str, v) : PyObject_Str(v);
  if (!s) return false;
  Py_ssize_t n;
  const char* c = PyUnicode_Check(s) ? PyUnicode_AsUTF8AndSize(s, &n) : nullptr;
  if (!c) {
    Py_DECREF(s);
    if (!PyErr_Occurred()) PyErr_SetString(PyExc_TypeError, "js_str fallback must return str");
    return false;
  }
  out.append(c, size_t(n));
  Py_DECREF(s);
  return true;
}

// JSON string body escaping, json.dumps(ensure_ascii=False) compatible.
// true when one of the 8 bytes of `w` is < 0x20, '"' or '\\' (SWAR; bytes >= 0x80 never match)
inline bool word_needs_escape(uint64_t w) {
  constexpr uint64_t ones = 0x0101010101010101ULL, highs = 0x8080808080808080ULL;
  uint64_t ctl = (w - ones * 0x20) & ~w & highs;
  uint64_t q = w ^ (ones * '"'), b = w ^ (ones * '\\');
  uint64_t quote = (q - ones) & ~q & highs, bslash = (b - ones) & ~b & highs;
  return (ctl | quote | bslash) != 0;
}

bool needs_escape(const char* s, size_t n) {
  size_t i = 0;
  for (; i + 8 <= n; i += 8) {
    uint64_t w;
    memcpy(&w, s + i, 8);
    if (word_needs_escape(w)) return true;
  }
  for (; i < n; ++i) {
    unsigned char c = static_cast<unsigned char>(s[i]);
    if (c < 0x20 || c == '"' || c == '\\') return true;
  }
  return false;
}

void json_escape_append(std::string& out, const char* s, size_t n) {
  static const char* hex = "0123456789abcdef";
  size_t i = 0;
  while (i + 8 <= n) {  // clean prefix, 8 bytes at a time (the common case: nothing to escape)
    uint64_t w;
    memcpy(&w, s + i, 8);
    if (word_needs_escape(w)) break;
    i += 8;
  }
  if (i == n) {
    out.append(s, n);
    return;
  }
  size_t run = 0;
  for (; i < n; ++i) {
    unsigned char c = static_cast<unsigned char>(s[i]);
    if (c >= 0x20 && c != '"' && c != '\\') continue;
    out.append(s + run, i - run);
    run = i + 1;
    switch (c) {
      case '"':
        out += "\\\"";
        break;
      case '\\':
        out += "\\\\";
        break;
      case '\n':
        out += "\\n";
        break;
      case '\r':
        out += "\\r";
        break;
      case '\t':
        out += "\\t";
        break;
      case '\b':
        out += "\\b";
        break;
      case '\f':
        out += "\\f";
        break;
      default: {
        char u[7] = {'\\', 'u', '0', '0', hex[c >> 4], hex[c & 15], 0};
        out.append(u, 6);
      }
    }
  }
  out.append(s + run, n - run);
}

bool json_fallback_append(std::string& out, PyObject* v) {
  if (!g_fallback_json) {
    PyErr_SetString(PyExc_RuntimeError, "json fallback not configured");
    return false;
  }
  PyObject* s = PyObject_CallOneArg(g_fallback_json, v);
  if (!s) return false;
  Py_ssize_t n;
  const char* c = PyUnicode_AsUTF8AndSize(s, &n);
  if (!c) {
    Py_DECREF(s);
    return false;
  }
  out.append(c, size_t(n));
  Py_DECREF(s);
  return true;
}

bool number_like(PyObject* v, double* d) {
  if (PyLong_Check(v)) {
    *d = PyLong_AsDouble(v);
    if (*d == -1.0 && PyErr_Occurred()) {
      PyErr_Clear();
      *d = NAN;
    }
    return true;
  }
  if (PyFloat_Check(v)) {
    *d = PyFloat_AS_DOUBLE(v);
    return true;
  }
  if (PyUnicode_Check(v)) {
    PyObject* f = PyFloat_FromString(v);
    if (!f) {
      PyErr_Clear();
      *d = NAN;
      return true;
    }
    *d = PyFloat_AS_DOUBLE(f);
    Py_DECREF(f);
    return true;
  }
  *d = NAN;
  return true;
}

// quick-format-unescaped (pino v5) + appended extra args. args = all positional args.
// drop_extra: pino@5 exactly (args with no specifier are dropped, quirk Q11 kept).
bool quick_format_append(std::string& out, PyObject* const* args, Py_ssize_t nargs, bool drop_extra) {
  if (nargs == 0) return true;
  PyObject* f = args[0];
  if (!PyUnicode_CheckExact(f)) {
    for (Py_ssize_t i = 0; i < (drop_extra ? 1 : nargs); ++i) {
      if (i) out += ' ';
      if (!js_str_append(out, args[i])) return false;
    }
    return true;
  }
  Py_ssize_t flen;
  const char* fs = PyUnicode_AsUTF8AndSize(f, &flen);
  if (!fs) return false;
  Py_ssize_t ai = 1;
  if (nargs == 1) {
    out.append(fs, size_t(flen));
    return true;
  }
  size_t last = 0;
  for (Py_ssize_t i = 0; i + 1 < flen;) {
    if (fs[i] != '%') {  // jump to the next '%' (most messages have none)
      const void* p = memchr(fs + i, '%', size_t(flen - i));
      if (!p) break;
      i = static_cast<const char*>(p) - fs;
      continue;
    }
    char c = fs[i + 1];
    if (c == '%') {
      out.append(fs + last, size_t(i) - last);
      out += '%';
      i += 2;
      last = size_t(i);
      continue;
    }
    if (ai < nargs && strchr("sdifjoO", c) && c) {
      out.append(fs + last, size_t(i) - last);
      PyObject* a = args[ai++];
      if (c == 's') {
        if (!js_str_append(out, a)) return false;
      } else if (c == 'd' || c == 'i' || c == 'f') {
        double d;
        number_like(a, &d);
        if (c == 'i' && std::isfinite(d)) d = std::floor(d);
        if (PyLong_CheckExact(a) && c != 'f') {
          if (!js_str_append(out, a)) return false;
        } else {
          js_number_append(out, d);
        }
      } else {
        if (!json_fallback_append(out, a)) return false;
      }
      i += 2;
      last = size_t(i);
      continue;
    }
    ++i;
  }
  out.append(fs + last, size_t(flen) - last);
  if (drop_extra) return true;
  for (; ai < nargs; ++ai) {
    out += ' ';
    if (!js_str_append(out, args[ai])) return false;
  }
  return true;
}

// Appends one pino line for `args` to `out`. Returns false with a Python error set.
bool append_line(std::string& out, long lvl, long long t, const char* prefix, Py_ssize_t plen, PyObject* extra,
                 PyObject* const* argv, Py_ssize_t nargs, bool drop_extra) {
  // `{"level":L,"time":T,` is the same for every line of one level within one millisecond
  // (~1,800 lines at the headline rate): format it once per (level, ms) and copy it
  struct Head {
    long lvl = -1;
    long long t = -1;
    std::string s;
  };
  static Head head;  // the GIL guards it (a thread_local costs a __tls_get_addr call in a module)
  if (head.lvl != lvl || head.t != t) {
    head.s.assign("{\"level\":");
    append_i64(head.s, lvl);
    head.s += ",\"time\":";
    append_i64(head.s, t);
    head.s += ',';
    head.lvl = lvl;
    head.t = t;
  }
  out.reserve(out.size() + head.s.size() + size_t(plen) + 160);
  out.append(head.s);
  out.append(prefix, size_t(plen));
  if (extra && extra != Py_None) {
    Py_ssize_t el;
    const char* ex = PyUnicode_AsUTF8AndSize(extra, &el);
    if (!ex) return false;
    out.append(ex, size_t(el));
  }
  if (nargs) {
    out += ",\"msg\":\"";
    // format straight into the line; escape afterwards only if the text needs it (rare: the
    // handlers' messages are plain text), which saves a copy of every message
    const size_t at = out.size();
    if (!quick_format_append(out, argv, nargs, drop_extra)) return false;
    if (needs_escape(out.data() + at, out.size() - at)) {
      static std::string msg;  // scratch, GIL-guarded: no allocation per line
      msg.assign(out, at, std::string::npos);
      out.resize(at);
      json_escape_append(out, msg.data(), msg.size());
    }
    out += '"';
  }
  out += ",\"v\":1}\n";
  return true;
}

// format_line(level:int, time_ms:int, prefix:str, extra:str|None, args:tuple) -> str
PyObject* mod_format_line_impl(PyObject*, PyObject* const* a, Py_ssize_t n);
PyObject* mod_format_line(PyObject*, PyObject* const* a, Py_ssize_t n) {
  BEHOLDER_TRY { return mod_format_line_impl(nullptr, a, n); }
  BEHOLDER_CATCH(nullptr)
}

PyObject* mod_format_line_impl(PyObject*, PyObject* const* a, Py_ssize_t n) {
  if (n != 5 || !PyUnicode_Check(a[2]) || !PyTuple_Check(a[4])) {
    PyErr_SetString(PyExc_TypeError, "format_line(level, time_ms, prefix, extra, args)");
    return nullptr;
  }
  long lvl = PyLong_AsLong(a[0]);
  long long t = PyLong_AsLongLong(a[1]);
  if (PyErr_Occurred()) return nullptr;
  Py_ssize_t plen;
  const char* prefix = PyUnicode_AsUTF8AndSize(a[2], &plen);
  if (!prefix) return nullptr;
  std::string out;
  out.reserve(192);
  if (!append_line(out, lvl, t, prefix, plen, a[3], &PyTuple_GET_ITEM(a[4], 0), PyTuple_GET_SIZE(a[4]), false))
    return nullptr;
  return PyUnicode_DecodeUTF8(out.data(), Py_ssize_t(out.size()), "strict");
}

// ---- LogSink: buffered pino writer ------------------------------------------
// LogSink(write, buffer_bytes=65536): emit() formats into a C++ buffer; the
// buffer is handed to `write` (e.g. sys.stdout.write) as one str when it
// passes `buffer_bytes`, on flush(), and immediately for level >= 50.
struct LogSinkObject {
  PyObject_HEAD PyObject* write;
  PyObject* flush_cb;
  std::string* buf;
  size_t limit;
  bool binary;  // write() takes bytes (UTF-8): no decode here and no encode in a text layer
  bool drop_extra;  // service.log.positional_args == "drop": pino@5's message text exactly
  unsigned long long counts[7];  // trace..fatal by level/10 - 1, [6] other
  unsigned long long bytes;
};

int sink_drain(LogSinkObject* self) {
  if (self->buf->empty()) return 0;
  PyObject* s = self->binary ? PyBytes_FromStringAndSize(self->buf->data(), Py_ssize_t(self->buf->size()))
                             : PyUnicode_DecodeUTF8(self->buf->data(), Py_ssize_t(self->buf->size()), "replace");
  self->bytes += self->buf->size();
  self->buf->clear();
  if (!s) return -1;
  PyObject* r = PyObject_CallOneArg(self->write, s);
  Py_DECREF(s);
  if (!r) return -1;
  Py_DECREF(r);
  return 0;
}

PyObject* sink_new(PyTypeObject* type, PyObject*, PyObject*) {
  LogSinkObject* self = reinterpret_cast<LogSinkObject*>(type->tp_alloc(type, 0));
  if (!self) return nullptr;
  self->write = nullptr;
  self->flush_cb = nullptr;
  self->buf = new std::string();
  self->limit = 65536;
  self->binary = false;
  self->drop_extra = false;
  memset(self->counts, 0, sizeof self->counts);
  self->bytes = 0;
  return reinterpret_cast<PyObject*>(self);
}

int sink_init(LogSinkObject* self, PyObject* args, PyObject* kwds) {
  static const char* kwlist[] = {"write", "flush", "buffer_bytes", "binary", "drop_extra", nullptr};
  PyObject* w;
  PyObject* f = Py_None;
  Py_ssize_t lim = 65536;
  int binary = 0;
  int drop = 0;
  if (!PyArg_ParseTupleAndKeywords(args, kwds, "O|Onpp", const_cast<char**>(kwlist), &w, &f, &lim, &binary, &drop))
    return -1;
  self->binary = binary != 0;
  self->drop_extra = drop != 0;
  if (!PyCallable_Check(w)) {
    PyErr_SetString(PyExc_TypeError, "write must be callable");
    return -1;
  }
  Py_INCREF(w);
  Py_XSETREF(self->write, w);
  if (f != Py_None) {
    Py_INCREF(f);
    Py_XSETREF(self->flush_cb, f);
  }
  self->limit = lim < 0 ? 0 : size_t(lim);
  self->buf->reserve(self->limit + 512);
  return 0;
}

int sink_traverse(LogSinkObject* self, visitproc visit, void* arg) {
  Py_VISIT(self->write);
  Py_VISIT(self->flush_cb);
  return 0;
}

int sink_clear(LogSinkObject* self) {
  Py_CLEAR(self->write);
  Py_CLEAR(self->flush_cb);
  return 0;
}

void sink_dealloc(LogSinkObject* self) {
  PyObject_GC_UnTrack(self);
  if (self->write && !self->buf->empty()) {
    PyObject *et, *ev, *tb;
    PyErr_Fetch(&et, &ev, &tb);
    if (sink_drain(self) < 0) PyErr_Clear();
    PyErr_Restore(et, ev, tb);
  }
  sink_clear(self);
  delete self->buf;
  Py_TYPE(self)->tp_free(reinterpret_cast<PyObject*>(self));
}

// Formats one line into the sink buffer; drains on size / error level.
bool sink_emit_core(LogSinkObject* self, long lvl, const char* prefix, Py_ssize_t plen, PyObject* extra,
                    PyObject* const* argv, Py_ssize_t nargs) {
  size_t before = self->buf->size();
  if (!append_line(*self->buf, lvl, gil_wall_ms(), prefix, plen, extra, argv, nargs, self->drop_extra)) {
    self->buf->resize(before);
    return false;
  }
  int slot = (lvl >= 10 && lvl <= 60 && lvl % 10 == 0) ? int(lvl / 10 - 1) : 6;
  self->counts[slot]++;
  if (lvl >= 50 || self->buf->size() >= self->limit) {
    if (sink_drain(self) < 0) return false;
    if (lvl >= 50 && self->flush_cb) {
      PyObject* r = PyObject_CallNoArgs(self->flush_cb);
      if (!r) return false;
      Py_DECREF(r);
    }
  }
  return true;
}

// emit(level, prefix, extra, args)
PyObject* sink_emit_impl(LogSinkObject* self, PyObject* const* a, Py_ssize_t n);
PyObject* sink_emit(LogSinkObject* self, PyObject* const* a, Py_ssize_t n) {
  BEHOLDER_TRY { return sink_emit_impl(self, a, n); }
  BEHOLDER_CATCH(nullptr)
}

PyObject* sink_emit_impl(LogSinkObject* self, PyObject* const* a, Py_ssize_t n) {
  if (n != 4 || !PyUnicode_Check(a[1]) || !PyTuple_Check(a[3])) {
    PyErr_SetString(PyExc_TypeError, "emit(level, prefix, extra, args)");
    return nullptr;
  }
  long lvl = PyLong_AsLong(a[0]);
  if (lvl == -1 && PyErr_Occurred()) return nullptr;
  Py_ssize_t plen;
  const char* prefix = PyUnicode_AsUTF8AndSize(a[1], &plen);
  if (!prefix) return nullptr;
  if (!sink_emit_core(self, lvl, prefix, plen, a[2], &PyTuple_GET_ITEM(a[3], 0), PyTuple_GET_SIZE(a[3])))
    return nullptr;
  Py_RETURN_NONE;
}

// retarget(write, flush=None, binary=False): flush, then send future lines elsewhere
PyObject* sink_retarget(LogSinkObject* self, PyObject* args) {
  PyObject* w;
  PyObject* f = Py_None;
  int binary = 0;
  if (!PyArg_ParseTuple(args, "O|Op", &w, &f, &binary)) return nullptr;
  if (!PyCallable_Check(w)) {
    PyErr_SetString(PyExc_TypeError, "write must be callable");
    return nullptr;
  }
  if (sink_drain(self) < 0) return nullptr;
  Py_INCREF(w);
  Py_XSETREF(self->write, w);
  self->binary = binary != 0;
  if (f == Py_None) {
    Py_CLEAR(self->flush_cb);
  } else {
    Py_INCREF(f);
    Py_XSETREF(self->flush_cb, f);
  }
  Py_RETURN_NONE;
}

PyObject* sink_flush(LogSinkObject* self, PyObject*) {
  if (sink_drain(self) < 0) return nullptr;
  if (self->flush_cb) {
    PyObject* r = PyObject_CallNoArgs(self->flush_cb);
    if (!r) return nullptr;
    Py_DECREF(r);
  }
  Py_RETURN_NONE;
}

PyObject* sink_get_counts(LogSinkObject* self, void*) {
  return Py_BuildValue("{s:K,s:K,s:K,s:K,s:K,s:K}", "trace", self->counts[0], "debug", self->counts[1], "info",
                       self->counts[2], "warn", self->counts[3], "error", self->counts[4], "fatal", self->counts[5]);
}
PyObject* sink_get_pending(LogSinkObject* self, void*) { return PyLong_FromSize_t(self->buf->size()); }
PyObject* sink_get_bytes(LogSinkObject* self, void*) { return PyLong_FromUnsignedLongLong(self->bytes); }
PyObject* sink_get_drop(LogSinkObject* self, void*) { return PyBool_FromLong(self->drop_extra); }
int sink_set_drop(LogSinkObject* self, PyObject* v, void*) {
  int t = v ? PyObject_IsTrue(v) : 0;
  if (t < 0) return -1;
  self->drop_extra = t != 0;
  return 0;
}

PyMethodDef sink_methods[] = {
    {"emit", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(sink_emit)), METH_FASTCALL,
     "emit(level, prefix, extra, args): format one pino line into the buffer"},
    {"flush", reinterpret_cast<PyCFunction>(sink_flush), METH_NOARGS, "write out buffered lines"},
    {"retarget", reinterpret_cast<PyCFunction>(sink_retarget), METH_VARARGS,
     "retarget(write, flush=None, binary=False)"},
    {nullptr, nullptr, 0, nullptr}};

PyGetSetDef sink_getset[] = {
    {"counts", reinterpret_cast<getter>(sink_get_counts), nullptr, "lines emitted per level", nullptr},
    {"pending_bytes", reinterpret_cast<getter>(sink_get_pending), nullptr, "buffered bytes", nullptr},
    {"bytes_written", reinterpret_cast<getter>(sink_get_bytes), nullptr, "bytes handed to write()", nullptr},
    {"drop_extra", reinterpret_cast<getter>(sink_get_drop), reinterpret_cast<setter>(sink_set_drop),
     "drop positional args that no format specifier consumes (pino@5 exactly)", nullptr},
    {nullptr, nullptr, nullptr, nullptr, nullptr}};

PyTypeObject LogSinkType = {PyVarObject_HEAD_INIT(nullptr, 0)};

PyObject* mod_quick_format_impl(PyObject*, PyObject* args);
PyObject* mod_quick_format(PyObject*, PyObject* args) {
  BEHOLDER_TRY { return mod_quick_format_impl(nullptr, args); }
  BEHOLDER_CATCH(nullptr)
}

PyObject* mod_quick_format_impl(PyObject*, PyObject* args) {
  std::string msg;
  if (!quick_format_append(msg, &PyTuple_GET_ITEM(args, 0), PyTuple_GET_SIZE(args), false)) return nullptr;
  return PyUnicode_DecodeUTF8(msg.data(), Py_ssize_t(msg.size()), "strict");
}

PyObject* mod_quick_format_drop(PyObject*, PyObject* args) {
  BEHOLDER_TRY {
    std::string msg;
    if (!quick_format_append(msg, &PyTuple_GET_ITEM(args, 0), PyTuple_GET_SIZE(args), true)) return nullptr;
    return PyUnicode_DecodeUTF8(msg.data(), Py_ssize_t(msg.size()), "strict");
  }
  BEHOLDER_CATCH(nullptr)
}

PyObject* mod_js_str_impl(PyObject*, PyObject* v);
PyObject* mod_js_str(PyObject*, PyObject* v) {
  BEHOLDER_TRY { return mod_js_str_impl(nullptr, v); }
  BEHOLDER_CATCH(nullptr)
}

PyObject* mod_js_str_impl(PyObject*, PyObject* v) {
  std::string out;
  if (!js_str_append(out, v)) return nullptr;
  return PyUnicode_DecodeUTF8(out.data(), Py_ssize_t(out.size()), "strict");
}

PyObject* mod_js_number(PyObject*, PyObject* v) {
  std::string out;
  if (PyLong_CheckExact(v)) {
    if (!js_str_append(out, v)) return nullptr;
  } else {
    double d = PyFloat_AsDouble(v);
    if (d == -1.0 && PyErr_Occurred()) return nullptr;
    js_number_append(out, d);
  }
  return PyUnicode_FromStringAndSize(out.data(), Py_ssize_t(out.size()));
}

// ---- URL encoding -----------------------------------------------------------
// encodeURIComponent leaves A-Z a-z 0-9 - _ . ! ~ * ' ( ) unescaped; RFC 3986 strict (the
// `qs` 6.x encoder behind request's `qs` option) escapes ! * ' ( ) too.
bool unreserved(unsigned char c, bool rfc3986) {
  if ((c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z') || (c >= '0' && c <= '9') || c == '-' || c == '_' ||
      c == '.' || c == '~')
    return true;
  return !rfc3986 && (c == '!' || c == '*' || c == '\'' || c == '(' || c == ')');
}

// unreserved(c, rfc3986) as two 256-entry tables
struct UnreservedTables {
  bool t[2][256];
  UnreservedTables() {
    for (int m = 0; m < 2; ++m)
      for (int c = 0; c < 256; ++c) t[m][c] = unreserved(static_cast<unsigned char>(c), m == 1);
  }
};
const UnreservedTables kUnreserved;

// Percent-encodes the UTF-8 bytes s[0..n) (every byte that is not unreserved), writing into
// the output's buffer directly (one resize, no per-byte capacity checks).
void quote_append(std::string& out, const char* s, size_t n, bool rfc3986 = false) {
  static const char* hex = "0123456789ABCDEF";
  const bool* t = kUnreserved.t[rfc3986 ? 1 : 0];
  size_t old = out.size();
  out.resize(old + 3 * n);
  char* p = &out[old];
  for (size_t i = 0; i < n; ++i) {
    unsigned char c = static_cast<unsigned char>(s[i]);
    if (t[c]) {
      *p++ = char(c);
    } else {
      p[0] = '%';
      p[1] = hex[c >> 4];
      p[2] = hex[c & 15];
      p += 3;
    }
  }
  out.resize(size_t(p - out.data()));
}

// quote_append of String(v): a str is encoded from its UTF-8 form in place (a lone surrogate
// raises, as encodeURIComponent throws URIError); other values through a scratch buffer.
bool quote_js_str_append(std::string& out, PyObject* v, bool rfc3986) {
  if (PyUnicode_CheckExact(v)) {
    Py_ssize_t n;
    const char* s = PyUnicode_AsUTF8AndSize(v, &n);
    if (!s) return false;
    quote_append(out, s, size_t(n), rfc3986);
    return true;
  }
  std::string tmp;  // short (numbers, booleans): stays in the small-string buffer
  if (!js_str_append(tmp, v)) return false;
  quote_append(out, tmp.data(), tmp.size(), rfc3986);
  return true;
}

// querystring value rendering: None -> "", bool -> true/false, numbers JS-style
bool qs_value_append(std::string& out, PyObject* v, bool rfc3986 = false) {
  if (v == Py_None) return true;
  return quote_js_str_append(out, v, rfc3986);
}

PyObject* mod_quote_component(PyObject*, PyObject* v) {
  std::string out;
  if (!qs_value_append(out, v)) return nullptr;
  return PyUnicode_FromStringAndSize(out.data(), Py_ssize_t(out.size()));
}

// encode_query(mapping, rfc3986=False) -> "k=v&k2=v2" (insertion order). The `qs` library the
// reference's HTTP clients use (1.2 under restler/trello, 6.5 under request) drops keys whose
// value is undefined (None here); values are String(v), JS-style.
PyObject* mod_encode_query_impl(PyObject* m, bool rfc3986);
PyObject* mod_encode_query(PyObject*, PyObject* const* args, Py_ssize_t nargs, PyObject* kwnames) {
  bool rfc3986 = false;
  Py_ssize_t nkw = kwnames ? PyTuple_GET_SIZE(kwnames) : 0;
  if (nargs < 1 || nargs + nkw > 2 || nargs > 2) {
    PyErr_SetString(PyExc_TypeError, "encode_query(mapping, rfc3986=False)");
    return nullptr;
  }
  PyObject* flag = nargs == 2 ? args[1] : nullptr;
  for (Py_ssize_t i = 0; i < nkw; ++i) {
    if (PyUnicode_CompareWithASCIIString(PyTuple_GET_ITEM(kwnames, i), "rfc3986") != 0) {
      PyErr_SetString(PyExc_TypeError, "encode_query: unexpected keyword");
      return nullptr;
    }
    flag = args[nargs + i];
  }
  if (flag) {
    int t = PyObject_IsTrue(flag);
    if (t < 0) return nullptr;
    rfc3986 = t != 0;
  }
  BEHOLDER_TRY { return mod_encode_query_impl(args[0], rfc3986); }
  BEHOLDER_CATCH(nullptr)
}

PyObject* mod_encode_query_impl(PyObject* m, bool rfc3986) {
  if (!PyDict_Check(m)) {
    PyErr_SetString(PyExc_TypeError, "encode_query expects a dict");
    return nullptr;
  }
  std::string out;
  Py_ssize_t pos = 0;
  PyObject *k, *v;
  bool first = true;
  while (PyDict_Next(m, &pos, &k, &v)) {
    if (v == Py_None) continue;  // undefined: qs omits the key
    if (!first) out += '&';
    first = false;
    if (!quote_js_str_append(out, k, rfc3986)) return nullptr;
    out += '=';
    if (!qs_value_append(out, v, rfc3986)) return nullptr;
  }
  return PyUnicode_FromStringAndSize(out.data(), Py_ssize_t(out.size()));
}

PyObject* mod_configure_text(PyObject*, PyObject* args) {
  PyObject *fs, *fj;
  if (!PyArg_ParseTuple(args, "OO", &fs, &fj)) return nullptr;
  Py_XINCREF(fs);
  Py_XSETREF(g_fallback_str, fs);
  Py_XINCREF(fj);
  Py_XSETREF(g_fallback_json, fj);
  Py_RETURN_NONE;
}


// ---- LogCore: native base class of utils.log.Logger -------------------------
// logger.info(...) etc. resolve to these C methods directly. A dict or
// exception first argument (pino merge-object / error forms) is delegated to
// the Python subclass's `_emit(level, name, args)`.
struct LogCoreObject {
  PyObject_HEAD PyObject* dict;
  LogSinkObject* sink;
  PyObject* prefix;
  long min_level;
};

const char* level_name(long lvl) {
  switch (lvl) {
    case 10:
      return "trace";
    case 20:
      return "debug";
    case 30:
      return "info";
    case 40:
      return "warn";
    case 50:
      return "error";
    default:
      return "fatal";
  }
}

PyObject* core_new(PyTypeObject* type, PyObject*, PyObject*) {
  LogCoreObject* self = reinterpret_cast<LogCoreObject*>(type->tp_alloc(type, 0));
  if (!self) return nullptr;
  self->sink = nullptr;
  self->prefix = nullptr;
  self->min_level = 30;
  return reinterpret_cast<PyObject*>(self);
}

int core_traverse(LogCoreObject* self, visitproc visit, void* arg) {
  Py_VISIT(self->dict);
  Py_VISIT(self->sink);
  return 0;
}

int core_clear(LogCoreObject* self) {
  Py_CLEAR(self->dict);
  Py_CLEAR(self->sink);
  Py_CLEAR(self->prefix);
  return 0;
}

void core_dealloc(LogCoreObject* self) {
  PyObject_GC_UnTrack(self);
  core_clear(self);
  Py_TYPE(self)->tp_free(reinterpret_cast<PyObject*>(self));
}

// _set_core(sink, prefix, min_level)
PyObject* core_set(LogCoreObject* self, PyObject* args) {
  PyObject *sink, *prefix;
  double minl;
  if (!PyArg_ParseTuple(args, "OUd", &sink, &prefix, &minl)) return nullptr;
  if (!PyObject_TypeCheck(sink, &LogSinkType)) {
    PyErr_SetString(PyExc_TypeError, "sink must be a LogSink");
    return nullptr;
  }
  Py_INCREF(sink);
  Py_XSETREF(self->sink, reinterpret_cast<LogSinkObject*>(sink));
  Py_INCREF(prefix);
  Py_XSETREF(self->prefix, prefix);
  self->min_level = minl > 1e9 ? 1000000000L : long(minl);
  Py_RETURN_NONE;
}

PyObject* core_log_impl(LogCoreObject* self, long lvl, PyObject* const* args, Py_ssize_t nargs);
PyObject* core_log(LogCoreObject* self, long lvl, PyObject* const* args, Py_ssize_t nargs) {
  BEHOLDER_TRY { return core_log_impl(self, lvl, args, nargs); }
  BEHOLDER_CATCH(nullptr)
}

PyObject* core_log_impl(LogCoreObject* self, long lvl, PyObject* const* args, Py_ssize_t nargs) {
  if (lvl < self->min_level) Py_RETURN_NONE;
  if (!self->sink || !self->prefix) {
    PyErr_SetString(PyExc_RuntimeError, "logger core not configured");
    return nullptr;
  }
  if (nargs && (PyDict_Check(args[0]) || PyExceptionInstance_Check(args[0]))) {
    PyObject* tup = PyTuple_New(nargs);
    if (!tup) return nullptr;
    for (Py_ssize_t i = 0; i < nargs; ++i) {
      Py_INCREF(args[i]);
      PyTuple_SET_ITEM(tup, i, args[i]);
    }
    PyObject* r = PyObject_CallMethod(reinterpret_cast<PyObject*>(self), "_emit", "lsN", lvl, level_name(lvl), tup);
    return r;
  }
  Py_ssize_t plen;
  const char* prefix = PyUnicode_AsUTF8AndSize(self->prefix, &plen);
  if (!prefix) return nullptr;
  if (!sink_emit_core(self->sink, lvl, prefix, plen, nullptr, args, nargs)) return nullptr;
  Py_RETURN_NONE;
}

#define CORE_LEVEL(name, lvl)                                                          \
  PyObject* core_##name(LogCoreObject* self, PyObject* const* args, Py_ssize_t nargs) { \
    return core_log(self, lvl, args, nargs);                                           \
  }
CORE_LEVEL(trace, 10)
CORE_LEVEL(debug, 20)
CORE_LEVEL(info, 30)
CORE_LEVEL(warn, 40)
CORE_LEVEL(error, 50)
CORE_LEVEL(fatal, 60)

#define CORE_METHOD(name, doc) \
  {#name, reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(core_##name)), METH_FASTCALL, doc}

PyMethodDef core_methods[] = {CORE_METHOD(trace, "log at level 10"),
                              CORE_METHOD(debug, "log at level 20"),
                              CORE_METHOD(info, "log at level 30"),
                              CORE_METHOD(warn, "log at level 40"),
                              {"warning", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(core_warn)),
                               METH_FASTCALL, "alias of warn"},
                              CORE_METHOD(error, "log at level 50"),
                              CORE_METHOD(fatal, "log at level 60"),
                              {"_set_core", reinterpret_cast<PyCFunction>(core_set), METH_VARARGS,
                               "_set_core(sink, prefix, min_level)"},
                              {nullptr, nullptr, 0, nullptr}};

PyTypeObject LogCoreType = {PyVarObject_HEAD_INIT(nullptr, 0)};

PyMethodDef text_methods[] = {
    {"format_line", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(mod_format_line)), METH_FASTCALL,
     "format_line(level, time_ms, prefix, extra, args) -> pino JSON line"},
    {"quick_format", mod_quick_format, METH_VARARGS, "quick_format(*args) -> message text"},
    {"quick_format_drop", mod_quick_format_drop, METH_VARARGS,
     "quick_format_drop(*args) -> pino@5's message text (unconsumed positional args dropped)"},
    {"js_str", mod_js_str, METH_O, "JavaScript String(v)"},
    {"js_number", mod_js_number, METH_O, "JavaScript Number::toString"},
    {"quote_component", mod_quote_component, METH_O, "encodeURIComponent(String(v))"},
    {"encode_query", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(mod_encode_query)),
     METH_FASTCALL | METH_KEYWORDS,
     "encode_query(dict, rfc3986=False): qs.stringify (undefined/None keys omitted; rfc3986 also escapes !'()*)"},
    {"configure_text", mod_configure_text, METH_VARARGS, "configure_text(js_str_fallback, json_fallback)"},
    {nullptr, nullptr, 0, nullptr}};

}  // namespace

// The recorded request URL: `url` + "?" + encode_query(params) for a non-empty dict (what
// restler builds for the trello client, index.js:53,83: "?" even when the path already has one,
// and even when every value is None), `url` alone for None or {}. For the native bench
// recorder (py_recorder.cpp). NULL with a Python error.
PyObject* url_with_query(PyObject* url, PyObject* params) {
  if (params == nullptr || params == Py_None) return Py_NewRef(url);
  if (!PyDict_Check(params)) {
    PyErr_SetString(PyExc_TypeError, "params must be a dict or None");
    return nullptr;
  }
  if (PyDict_GET_SIZE(params) == 0) return Py_NewRef(url);
  try {
    std::string q;
    Py_ssize_t pos = 0;
    PyObject *k, *v;
    bool first = true;
    while (PyDict_Next(params, &pos, &k, &v)) {
      if (v == Py_None) continue;
      if (!first) q += '&';
      first = false;
      if (!quote_js_str_append(q, k, false)) return nullptr;
      q += '=';
      if (!qs_value_append(q, v, false)) return nullptr;
    }
    Py_ssize_t ulen;
    const char* u = PyUnicode_AsUTF8AndSize(url, &ulen);
    if (!u) return nullptr;
    std::string out;
    out.reserve(size_t(ulen) + 1 + q.size());
    out.append(u, size_t(ulen));
    out += '?';
    out += q;
    return PyUnicode_DecodeUTF8(out.data(), Py_ssize_t(out.size()), "strict");
  } catch (const std::bad_alloc&) {
    return PyErr_NoMemory();
  }
}

// ---- used by the native handlers (py_handlers.cpp) ---------------------------
bool text_js_str_append(std::string& out, PyObject* v) { return js_str_append(out, v); }

// one `key=value` pair of encode_query() (None values omitted; `first` tracks the '&')
bool text_query_pair_append(std::string& out, PyObject* k, PyObject* v, bool* first, bool rfc3986) {
  if (v == Py_None) return true;
  if (!*first) out += '&';
  *first = false;
  if (!quote_js_str_append(out, k, rfc3986)) return false;
  out += '=';
  return qs_value_append(out, v, rfc3986);
}

bool is_native_logger(PyObject* logger) {
  // the level methods must be LogCore's own (a subclass overriding them keeps its override)
  if (!PyObject_TypeCheck(logger, &LogCoreType)) return false;
  static PyObject* names[3] = {nullptr, nullptr, nullptr};
  static const char* raw[3] = {"info", "warn", "error"};
  for (int i = 0; i < 3; ++i) {
    if (!names[i] && !(names[i] = PyUnicode_InternFromString(raw[i]))) {
      PyErr_Clear();
      return false;
    }
    PyObject* mine = _PyType_Lookup(Py_TYPE(logger), names[i]);
    PyObject* base = _PyType_Lookup(&LogCoreType, names[i]);
    if (!mine || mine != base) return false;
  }
  return true;
}

bool logcore_emit(PyObject* logger, bool native, long lvl, PyObject* const* args, Py_ssize_t nargs) {
  PyObject* r;
  if (native) {
    r = core_log(reinterpret_cast<LogCoreObject*>(logger), lvl, args, nargs);
  } else {
    PyObject* meth = PyObject_GetAttrString(logger, level_name(lvl));
    if (!meth) return false;
    r = PyObject_Vectorcall(meth, args, size_t(nargs), nullptr);
    Py_DECREF(meth);
  }
  if (!r) return false;
  Py_DECREF(r);
  return true;
}

int init_text_functions(PyObject* m) {
  LogSinkType.tp_name = "beholder_amd.ops._native.LogSink";
  LogSinkType.tp_basicsize = sizeof(LogSinkObject);
  LogSinkType.tp_flags = Py_TPFLAGS_DEFAULT | Py_TPFLAGS_HAVE_GC;
  LogSinkType.tp_doc =
      "LogSink(write, flush=None, buffer_bytes=65536, binary=False): buffered pino JSON-lines writer "
      "(binary: write() gets UTF-8 bytes)";
  LogSinkType.tp_new = sink_new;
  LogSinkType.tp_init = reinterpret_cast<initproc>(sink_init);
  LogSinkType.tp_dealloc = reinterpret_cast<destructor>(sink_dealloc);
  LogSinkType.tp_traverse = reinterpret_cast<traverseproc>(sink_traverse);
  LogSinkType.tp_clear = reinterpret_cast<inquiry>(sink_clear);
  LogSinkType.tp_methods = sink_methods;
  LogSinkType.tp_getset = sink_getset;
  if (PyType_Ready(&LogSinkType) < 0) return -1;
  LogCoreType.tp_name = "beholder_amd.ops._native.LogCore";
  LogCoreType.tp_basicsize = sizeof(LogCoreObject);
  LogCoreType.tp_dictoffset = offsetof(LogCoreObject, dict);
  LogCoreType.tp_flags = Py_TPFLAGS_DEFAULT | Py_TPFLAGS_BASETYPE | Py_TPFLAGS_HAVE_GC;
  LogCoreType.tp_doc = "native base of the pino-compatible Logger (level methods in C)";
  LogCoreType.tp_new = core_new;
  LogCoreType.tp_dealloc = reinterpret_cast<destructor>(core_dealloc);
  LogCoreType.tp_traverse = reinterpret_cast<traverseproc>(core_traverse);
  LogCoreType.tp_clear = reinterpret_cast<inquiry>(core_clear);
  LogCoreType.tp_methods = core_methods;
  if (PyType_Ready(&LogCoreType) < 0) return -1;
  Py_INCREF(&LogCoreType);
  if (PyModule_AddObject(m, "LogCore", reinterpret_cast<PyObject*>(&LogCoreType)) < 0) return -1;
  Py_INCREF(&LogSinkType);
  if (PyModule_AddObject(m, "LogSink", reinterpret_cast<PyObject*>(&LogSinkType)) < 0) return -1;
  return PyModule_AddFunctions(m, text_methods);
}

}  // namespace beholder
