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
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>

#include "py_common.hpp"

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
      char buf[32];
      int len = snprintf(buf, sizeof buf, "%lld", x);
      out.append(buf, size_t(len));
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
void json_escape_append(std::string& out, const char* s, size_t n) {
  static const char* hex = "0123456789abcdef";
  size_t run = 0;
  for (size_t i = 0; i < n; ++i) {
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
bool quick_format_append(std::string& out, PyObject* const* args, Py_ssize_t nargs) {
  if (nargs == 0) return true;
  PyObject* f = args[0];
  if (!PyUnicode_CheckExact(f)) {
    for (Py_ssize_t i = 0; i < nargs; ++i) {
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
    if (fs[i] != '%') {
      ++i;
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
  for (; ai < nargs; ++ai) {
    out += ' ';
    if (!js_str_append(out, args[ai])) return false;
  }
  return true;
}

// format_line(level:int, time_ms:int, prefix:str, extra:str|None, args:tuple) -> str
PyObject* mod_format_line(PyObject*, PyObject* const* a, Py_ssize_t n) {
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
  char head[64];
  int hl = snprintf(head, sizeof head, "{\"level\":%ld,\"time\":%lld,", lvl, t);
  out.append(head, size_t(hl));
  out.append(prefix, size_t(plen));
  if (a[3] != Py_None) {
    Py_ssize_t el;
    const char* ex = PyUnicode_AsUTF8AndSize(a[3], &el);
    if (!ex) return nullptr;
    out.append(ex, size_t(el));
  }
  Py_ssize_t nargs = PyTuple_GET_SIZE(a[4]);
  if (nargs) {
    std::string msg;
    msg.reserve(128);
    if (!quick_format_append(msg, &PyTuple_GET_ITEM(a[4], 0), nargs)) return nullptr;
    out += ",\"msg\":\"";
    json_escape_append(out, msg.data(), msg.size());
    out += '"';
  }
  out += ",\"v\":1}\n";
  return PyUnicode_DecodeUTF8(out.data(), Py_ssize_t(out.size()), "strict");
}

PyObject* mod_quick_format(PyObject*, PyObject* args) {
  std::string msg;
  if (!quick_format_append(msg, &PyTuple_GET_ITEM(args, 0), PyTuple_GET_SIZE(args))) return nullptr;
  return PyUnicode_DecodeUTF8(msg.data(), Py_ssize_t(msg.size()), "strict");
}

PyObject* mod_js_str(PyObject*, PyObject* v) {
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
bool unreserved(unsigned char c) {
  return (c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z') || (c >= '0' && c <= '9') || c == '-' || c == '_' ||
         c == '.' || c == '!' || c == '~' || c == '*' || c == '\'' || c == '(' || c == ')';
}

void quote_append(std::string& out, const char* s, size_t n) {
  static const char* hex = "0123456789ABCDEF";
  for (size_t i = 0; i < n; ++i) {
    unsigned char c = static_cast<unsigned char>(s[i]);
    if (unreserved(c)) {
      out += char(c);
    } else {
      out += '%';
      out += hex[c >> 4];
      out += hex[c & 15];
    }
  }
}

// querystring value rendering: None -> "", bool -> true/false, numbers JS-style
bool qs_value_append(std::string& out, PyObject* v) {
  std::string tmp;
  if (v == Py_None) return true;
  if (!js_str_append(tmp, v)) return false;
  quote_append(out, tmp.data(), tmp.size());
  return true;
}

PyObject* mod_quote_component(PyObject*, PyObject* v) {
  std::string out;
  if (!qs_value_append(out, v)) return nullptr;
  return PyUnicode_FromStringAndSize(out.data(), Py_ssize_t(out.size()));
}

// encode_query(mapping) -> "k=v&k2=v2" (insertion order)
PyObject* mod_encode_query(PyObject*, PyObject* m) {
  if (!PyDict_Check(m)) {
    PyErr_SetString(PyExc_TypeError, "encode_query expects a dict");
    return nullptr;
  }
  std::string out;
  Py_ssize_t pos = 0;
  PyObject *k, *v;
  bool first = true;
  while (PyDict_Next(m, &pos, &k, &v)) {
    if (!first) out += '&';
    first = false;
    std::string ks;
    if (!js_str_append(ks, k)) return nullptr;
    quote_append(out, ks.data(), ks.size());
    out += '=';
    if (!qs_value_append(out, v)) return nullptr;
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

PyMethodDef text_methods[] = {
    {"format_line", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(mod_format_line)), METH_FASTCALL,
     "format_line(level, time_ms, prefix, extra, args) -> pino JSON line"},
    {"quick_format", mod_quick_format, METH_VARARGS, "quick_format(*args) -> message text"},
    {"js_str", mod_js_str, METH_O, "JavaScript String(v)"},
    {"js_number", mod_js_number, METH_O, "JavaScript Number::toString"},
    {"quote_component", mod_quote_component, METH_O, "encodeURIComponent(String(v))"},
    {"encode_query", mod_encode_query, METH_O, "querystring.stringify(dict)"},
    {"configure_text", mod_configure_text, METH_VARARGS, "configure_text(js_str_fallback, json_fallback)"},
    {nullptr, nullptr, 0, nullptr}};

}  // namespace

int init_text_functions(PyObject* m) { return PyModule_AddFunctions(m, text_methods); }

}  // namespace beholder
