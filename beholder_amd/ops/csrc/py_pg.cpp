// PgReader: PostgreSQL v3 backend-message reader for the pipelined store client.
//
// The reference reads the media row on every progress event and updates it on
// every status event (index.js:68,76,140 via triton-core/db -> pg). With the
// extended protocol, store/pgwire.py pipelines many Bind/Describe/Execute/Sync
// groups on one connection. This reader turns the server's byte stream back into
// one result per Sync:
//
//   r = PgReader()
//   r.query_mode = True          # after startup / authentication
//   r.feed(data) -> [item, ...]  # in stream order
//
// An item is either
//   (rows, tag, error, parse_ok)  one query completed (ReadyForQuery seen):
//                                 rows = [tuple, ...] decoded from text format by
//                                 column type OID, tag = CommandComplete text,
//                                 error = {field-code: str} or None
//   (type, body)                  any other message: everything while not in
//                                 query_mode (startup / auth), and out-of-band
//                                 NoticeResponse / ParameterStatus /
//                                 NotificationResponse in query mode.
//
// Value decoding (text format): bool 16; int2/4/8, oid 21/23/20/26 -> int;
// float4/8 700/701 -> float; numeric 1700 -> int, or float if it has a
// fraction or exponent; bytea 17 -> bytes (hex format); everything else -> str.
// Malformed messages raise ValueError (the connection must be dropped).
#include <cstring>
#include <string>
#include <vector>

#include "py_common.hpp"

namespace beholder {

namespace {

struct PgReaderObject {
  PyObject_HEAD std::string* carry;
  std::vector<uint32_t>* oids;
  PyObject* rows;    // list or NULL
  PyObject* tag;     // str or NULL
  PyObject* error;   // dict or NULL
  bool parse_ok;
  bool query_mode;
  uint32_t max_message;
  uint64_t messages, results;
};

PyTypeObject PgReaderType = {PyVarObject_HEAD_INIT(nullptr, 0)};

inline uint32_t rd32(const uint8_t* p) {
  return (uint32_t(p[0]) << 24) | (uint32_t(p[1]) << 16) | (uint32_t(p[2]) << 8) | uint32_t(p[3]);
}
inline uint16_t rd16(const uint8_t* p) { return uint16_t((p[0] << 8) | p[1]); }

[[noreturn]] void bad(const char* what) { throw std::invalid_argument(what); }

PyObject* decode_text(uint32_t oid, const char* s, size_t n) {
  switch (oid) {
    case 16:
      return PyBool_FromLong(n == 1 && s[0] == 't');
    case 20: case 21: case 23: case 26: {
      // the common case (a status, a creator, an id that fits in 18 digits): no string copy and
      // no PyLong_FromString parse; anything else (a sign, spaces, longer) takes the general path
      if (n && n <= 18) {
        size_t i = s[0] == '-' ? 1 : 0;
        long long v = 0;
        bool ok = i < n;
        for (; ok && i < n; ++i) {
          unsigned d = unsigned(s[i]) - '0';
          if (d > 9) ok = false;
          else v = v * 10 + d;
        }
        if (ok) return PyLong_FromLongLong(s[0] == '-' ? -v : v);
      }
      std::string tmp(s, n);
      return PyLong_FromString(tmp.c_str(), nullptr, 10);
    }
    case 700: case 701: {
      std::string tmp(s, n);
      PyObject* str = PyUnicode_FromStringAndSize(tmp.data(), Py_ssize_t(n));
      if (!str) return nullptr;
      PyObject* f = PyFloat_FromString(str);
      Py_DECREF(str);
      return f;
    }
    case 1700: {
      bool frac = false;
      for (size_t i = 0; i < n; ++i)
        if (s[i] == '.' || s[i] == 'e' || s[i] == 'E' || s[i] == 'N' || s[i] == 'I') frac = true;  // NaN/Infinity too
      std::string tmp(s, n);
      if (!frac) return PyLong_FromString(tmp.c_str(), nullptr, 10);
      PyObject* str = PyUnicode_FromStringAndSize(tmp.data(), Py_ssize_t(n));
      if (!str) return nullptr;
      PyObject* f = PyFloat_FromString(str);
      Py_DECREF(str);
      return f;
    }
    case 17: {
      if (n >= 2 && s[0] == '\\' && s[1] == 'x') {
        PyObject* hex = PyUnicode_FromStringAndSize(s + 2, Py_ssize_t(n - 2));
        if (!hex) return nullptr;
        PyObject* b = PyObject_CallMethod(reinterpret_cast<PyObject*>(&PyBytes_Type), "fromhex", "O", hex);
        Py_DECREF(hex);
        return b;
      }
      return PyBytes_FromStringAndSize(s, Py_ssize_t(n));
    }
    default:
      return PyUnicode_DecodeUTF8(s, Py_ssize_t(n), "replace");
  }
}

void clear_query(PgReaderObject* r) {
  Py_CLEAR(r->rows);
  Py_CLEAR(r->tag);
  Py_CLEAR(r->error);
  r->parse_ok = false;
}

// RowDescription: int16 n, then per field: name\0, int32 table, int16 attnum, int32 oid,
// int16 typlen, int32 typmod, int16 format.
void on_row_description(PgReaderObject* r, const uint8_t* b, size_t n) {
  if (n < 2) bad("short RowDescription");
  uint16_t k = rd16(b);
  size_t i = 2;
  r->oids->clear();
  for (uint16_t f = 0; f < k; ++f) {
    const void* z = std::memchr(b + i, 0, n - i);
    if (!z) bad("malformed RowDescription");
    i = size_t(static_cast<const uint8_t*>(z) - b) + 1;
    if (i + 18 > n) bad("short RowDescription");
    r->oids->push_back(rd32(b + i + 6));
    i += 18;
  }
}

PyObject* on_data_row(PgReaderObject* r, const uint8_t* b, size_t n) {
  if (n < 2) bad("short DataRow");
  uint16_t k = rd16(b);
  PyObject* row = PyTuple_New(k);
  if (!row) return nullptr;
  size_t i = 2;
  for (uint16_t c = 0; c < k; ++c) {
    if (i + 4 > n) {
      Py_DECREF(row);
      bad("short DataRow");
    }
    int32_t len = int32_t(rd32(b + i));
    i += 4;
    PyObject* v;
    if (len < 0) {
      v = Py_None;
      Py_INCREF(v);
    } else {
      if (i + size_t(len) > n) {
        Py_DECREF(row);
        bad("short DataRow");
      }
      uint32_t oid = c < r->oids->size() ? (*r->oids)[c] : 25;
      v = decode_text(oid, reinterpret_cast<const char*>(b + i), size_t(len));
      if (!v) {
        Py_DECREF(row);
        return nullptr;
      }
      i += size_t(len);
    }
    PyTuple_SET_ITEM(row, c, v);
  }
  return row;
}

PyObject* error_fields(const uint8_t* b, size_t n) {
  PyObject* d = PyDict_New();
  if (!d) return nullptr;
  size_t i = 0;
  while (i < n && b[i] != 0) {
    char code = char(b[i]);
    const void* z = std::memchr(b + i + 1, 0, n - i - 1);
    size_t e = z ? size_t(static_cast<const uint8_t*>(z) - b) : n;
    PyObject* v = PyUnicode_DecodeUTF8(reinterpret_cast<const char*>(b + i + 1), Py_ssize_t(e - i - 1), "replace");
    if (!v) {
      Py_DECREF(d);
      return nullptr;
    }
    char key[2] = {code, 0};
    int rc = PyDict_SetItemString(d, key, v);
    Py_DECREF(v);
    if (rc < 0) {
      Py_DECREF(d);
      return nullptr;
    }
    i = e + 1;
  }
  return d;
}

// Appends (type, body) to out.
int emit_raw(PyObject* out, uint8_t typ, const uint8_t* b, size_t n) {
  char t[1] = {char(typ)};
  PyObject* item = Py_BuildValue("(y#y#)", t, Py_ssize_t(1), reinterpret_cast<const char*>(b), Py_ssize_t(n));
  if (!item) return -1;
  int rc = PyList_Append(out, item);
  Py_DECREF(item);
  return rc;
}

// One backend message in query mode. Returns -1 on a Python error.
int on_message(PgReaderObject* r, PyObject* out, uint8_t typ, const uint8_t* b, size_t n) {
  switch (typ) {
    case '1':  // ParseComplete
      r->parse_ok = true;
      return 0;
    case '2': case '3': case 'n': case 's': case 'I': case 't':  // Bind/CloseComplete, NoData, Suspended, Empty, ParamDesc
      return 0;
    case 'T':
      on_row_description(r, b, n);
      return 0;
    case 'D': {
      if (!r->rows && !(r->rows = PyList_New(0))) return -1;
      PyObject* row = on_data_row(r, b, n);
      if (!row) return -1;
      int rc = PyList_Append(r->rows, row);
      Py_DECREF(row);
      return rc;
    }
    case 'C': {
      size_t e = n && b[n - 1] == 0 ? n - 1 : n;
      Py_XSETREF(r->tag, PyUnicode_DecodeUTF8(reinterpret_cast<const char*>(b), Py_ssize_t(e), "replace"));
      return r->tag ? 0 : -1;
    }
    case 'E':
      if (!r->error) {  // the first error of a Sync group is the one that matters
        r->error = error_fields(b, n);
        if (!r->error) return -1;
      }
      return 0;
    case 'Z': {
      PyObject* rows = r->rows ? r->rows : PyList_New(0);
      if (!rows) return -1;
      r->rows = nullptr;
      PyObject* tag = r->tag ? r->tag : PyUnicode_FromString("");
      r->tag = nullptr;
      if (!tag) {
        Py_DECREF(rows);
        return -1;
      }
      PyObject* err = r->error ? r->error : (Py_INCREF(Py_None), Py_None);
      r->error = nullptr;
      PyObject* item = PyTuple_New(4);
      if (!item) {
        Py_DECREF(rows);
        Py_DECREF(tag);
        Py_DECREF(err);
        return -1;
      }
      PyTuple_SET_ITEM(item, 0, rows);
      PyTuple_SET_ITEM(item, 1, tag);
      PyTuple_SET_ITEM(item, 2, err);
      PyObject* ok = r->parse_ok ? Py_True : Py_False;
      Py_INCREF(ok);
      PyTuple_SET_ITEM(item, 3, ok);
      r->parse_ok = false;
      r->oids->clear();
      ++r->results;
      int rc = PyList_Append(out, item);
      Py_DECREF(item);
      return rc;
    }
    default:  // N notice, S parameter status, A notification, anything unexpected: to Python
      return emit_raw(out, typ, b, n);
  }
}

PyObject* pg_new(PyTypeObject* type, PyObject*, PyObject*) {
  PgReaderObject* r = reinterpret_cast<PgReaderObject*>(type->tp_alloc(type, 0));
  if (!r) return nullptr;
  try {
    r->carry = new std::string();
    r->oids = new std::vector<uint32_t>();
  } catch (const std::bad_alloc&) {
    Py_DECREF(r);
    return PyErr_NoMemory();
  }
  r->rows = r->tag = r->error = nullptr;
  r->parse_ok = false;
  r->query_mode = false;
  r->max_message = 1u << 30;  // Postgres' own limit for a single message
  r->messages = r->results = 0;
  return reinterpret_cast<PyObject*>(r);
}

int pg_init(PgReaderObject* r, PyObject* args, PyObject* kwds) {
  static const char* kwlist[] = {"max_message", nullptr};
  unsigned long mm = 1ul << 30;
  if (!PyArg_ParseTupleAndKeywords(args, kwds, "|k", const_cast<char**>(kwlist), &mm)) return -1;
  if (mm < 16) {
    PyErr_SetString(PyExc_ValueError, "max_message must be >= 16");
    return -1;
  }
  r->max_message = uint32_t(mm);
  return 0;
}

void pg_dealloc(PgReaderObject* r) {
  clear_query(r);
  delete r->carry;
  delete r->oids;
  Py_TYPE(r)->tp_free(reinterpret_cast<PyObject*>(r));
}

PyObject* pg_feed_bytes(PgReaderObject* r, const char* in, size_t in_len) {
  const uint8_t* data;
  size_t len;
  std::string& carry = *r->carry;
  if (carry.empty()) {
    data = reinterpret_cast<const uint8_t*>(in);
    len = in_len;
  } else {
    carry.append(in, in_len);
    data = reinterpret_cast<const uint8_t*>(carry.data());
    len = carry.size();
  }
  PyObject* out = PyList_New(0);
  if (!out) return nullptr;
  size_t i = 0;
  try {
    while (len - i >= 5) {
      uint8_t typ = data[i];
      uint32_t ml = rd32(data + i + 1);
      if (ml < 4 || ml > r->max_message) bad("invalid backend message length");
      if (len - i - 1 < ml) break;
      const uint8_t* body = data + i + 5;
      size_t bn = ml - 4;
      ++r->messages;
      int rc = r->query_mode ? on_message(r, out, typ, body, bn) : emit_raw(out, typ, body, bn);
      if (rc < 0) {
        Py_DECREF(out);
        carry.clear();
        clear_query(r);
        return nullptr;
      }
      i += 1 + ml;
    }
  } catch (const std::invalid_argument& e) {
    Py_DECREF(out);
    carry.clear();
    clear_query(r);
    PyErr_SetString(PyExc_ValueError, e.what());
    return nullptr;
  }
  if (carry.empty()) {
    if (i < len) carry.assign(reinterpret_cast<const char*>(data + i), len - i);
  } else {
    carry.erase(0, i);
  }
  return out;
}

PyObject* pg_feed_impl(PgReaderObject* r, PyObject* arg) {
  Py_buffer view;
  if (PyObject_GetBuffer(arg, &view, PyBUF_SIMPLE) < 0) return nullptr;
  PyObject* out;
  try {
    out = pg_feed_bytes(r, static_cast<const char*>(view.buf), size_t(view.len));
  } catch (...) {
    PyBuffer_Release(&view);
    throw;
  }
  PyBuffer_Release(&view);
  return out;
}

PyObject* pg_feed(PgReaderObject* r, PyObject* arg) {
  BEHOLDER_TRY { return pg_feed_impl(r, arg); }
  BEHOLDER_CATCH(nullptr)
}

PyObject* pg_get_query_mode(PgReaderObject* r, void*) { return PyBool_FromLong(r->query_mode); }
int pg_set_query_mode(PgReaderObject* r, PyObject* v, void*) {
  if (!v) {
    PyErr_SetString(PyExc_TypeError, "cannot delete query_mode");
    return -1;
  }
  int b = PyObject_IsTrue(v);
  if (b < 0) return -1;
  r->query_mode = b != 0;
  return 0;
}
PyObject* pg_get_buffered(PgReaderObject* r, void*) { return PyLong_FromSize_t(r->carry->size()); }
PyObject* pg_get_messages(PgReaderObject* r, void*) { return PyLong_FromUnsignedLongLong(r->messages); }
PyObject* pg_get_results(PgReaderObject* r, void*) { return PyLong_FromUnsignedLongLong(r->results); }

PyObject* pg_decode(PyObject*, PyObject* args) {
  // decode_text(oid, text: bytes) -> value (exposed for tests)
  unsigned long oid;
  const char* s;
  Py_ssize_t n;
  if (!PyArg_ParseTuple(args, "ky#", &oid, &s, &n)) return nullptr;
  return decode_text(uint32_t(oid), s, size_t(n));
}

PyMethodDef pg_methods[] = {
    {"feed", reinterpret_cast<PyCFunction>(pg_feed), METH_O, "feed(data) -> [result | (type, body), ...]"},
    {nullptr, nullptr, 0, nullptr}};

PyGetSetDef pg_getset[] = {
    {"query_mode", reinterpret_cast<getter>(pg_get_query_mode), reinterpret_cast<setter>(pg_set_query_mode),
     "assemble query results (after startup)", nullptr},
    {"buffered", reinterpret_cast<getter>(pg_get_buffered), nullptr, "bytes of an incomplete message", nullptr},
    {"messages", reinterpret_cast<getter>(pg_get_messages), nullptr, "backend messages read", nullptr},
    {"results", reinterpret_cast<getter>(pg_get_results), nullptr, "query results completed", nullptr},
    {nullptr, nullptr, nullptr, nullptr, nullptr}};

void put32(std::string& o, uint32_t v) {
  char b[4] = {char(v >> 24), char(v >> 16), char(v >> 8), char(v)};
  o.append(b, 4);
}

// Appends one parameter in text format (store/pgwire.py encode_param semantics).
int put_param(std::string& o, PyObject* v) {
  if (v == Py_None) {
    put32(o, 0xffffffffu);
    return 0;
  }
  if (PyBool_Check(v)) {
    put32(o, 1);
    o.push_back(v == Py_True ? 't' : 'f');
    return 0;
  }
  if (PyBytes_Check(v) || PyByteArray_Check(v)) {
    const char* p = PyBytes_Check(v) ? PyBytes_AS_STRING(v) : PyByteArray_AS_STRING(v);
    size_t n = size_t(PyBytes_Check(v) ? PyBytes_GET_SIZE(v) : PyByteArray_GET_SIZE(v));
    static const char hx[] = "0123456789abcdef";
    put32(o, uint32_t(2 + 2 * n));
    o.append("\\x", 2);
    for (size_t i = 0; i < n; ++i) {
      unsigned char c = static_cast<unsigned char>(p[i]);
      o.push_back(hx[c >> 4]);
      o.push_back(hx[c & 15]);
    }
    return 0;
  }
  PyObject* s = PyUnicode_Check(v) ? (Py_INCREF(v), v) : PyObject_Str(v);
  if (!s) return -1;
  Py_ssize_t n;
  const char* u = PyUnicode_AsUTF8AndSize(s, &n);
  if (!u) {
    Py_DECREF(s);
    return -1;
  }
  put32(o, uint32_t(n));
  o.append(u, size_t(n));
  Py_DECREF(s);
  return 0;
}

}  // namespace

// PgReader.feed for a caller in C (py_netconn.cpp): the received bytes without a memoryview and
// a method call. The same result as feed(); exact PgReader only (is_pg_reader).
bool is_pg_reader(PyObject* o) { return Py_TYPE(o) == &PgReaderType; }

PyObject* pg_reader_feed_c(PyObject* o, const char* data, size_t n) {
  BEHOLDER_TRY { return pg_feed_bytes(reinterpret_cast<PgReaderObject*>(o), data, n); }
  BEHOLDER_CATCH(nullptr)
}

// Appends Bind + Describe(portal) + Execute + Sync for statement `name` to `o`. -1 on error.
int pg_bind_append(std::string& o, const char* name, size_t nlen, PyObject* params) {
  PyObject* seq = PySequence_Fast(params, "params must be a sequence");
  if (!seq) return -1;
  Py_ssize_t np = PySequence_Fast_GET_SIZE(seq);
  if (np > 65535) {
    Py_DECREF(seq);
    PyErr_SetString(PyExc_ValueError, "too many parameters");
    return -1;
  }
  size_t start = o.size();
  o.reserve(start + size_t(64 + nlen + np * 48));
  o.push_back('B');
  put32(o, 0);  // length, patched below
  o.push_back('\0');  // unnamed portal
  o.append(name, size_t(nlen));
  o.push_back('\0');
  o.append("\0\0", 2);  // no parameter format codes: all text
  o.push_back(char(np >> 8));
  o.push_back(char(np & 0xff));
  PyObject** items = PySequence_Fast_ITEMS(seq);
  for (Py_ssize_t i = 0; i < np; ++i) {
    if (put_param(o, items[i]) < 0) {
      Py_DECREF(seq);
      o.resize(start);
      return -1;
    }
  }
  Py_DECREF(seq);
  o.append("\0\0", 2);  // no result format codes: all text
  uint32_t blen = uint32_t(o.size() - start - 1);
  o[start + 1] = char(blen >> 24);
  o[start + 2] = char(blen >> 16);
  o[start + 3] = char(blen >> 8);
  o[start + 4] = char(blen);
  static const char tail[] = {'D', 0, 0, 0, 6, 'P', 0,           // Describe portal ""
                              'E', 0, 0, 0, 9, 0, 0, 0, 0, 0,    // Execute "", no row limit
                              'S', 0, 0, 0, 4};                   // Sync
  o.append(tail, sizeof(tail));
  return 0;
}

namespace {

// pg_bind(statement: bytes, params: sequence) -> Bind + Describe(portal) + Execute + Sync
PyObject* pg_bind_impl(PyObject*, PyObject* args) {
  const char* name;
  Py_ssize_t nlen;
  PyObject* params;
  if (!PyArg_ParseTuple(args, "y#O", &name, &nlen, &params)) return nullptr;
  std::string o;
  if (pg_bind_append(o, name, size_t(nlen), params) < 0) return nullptr;
  return PyBytes_FromStringAndSize(o.data(), Py_ssize_t(o.size()));
}

PyObject* pg_bind(PyObject* self, PyObject* args) {
  BEHOLDER_TRY { return pg_bind_impl(self, args); }
  BEHOLDER_CATCH(nullptr)
}

PyMethodDef pg_functions[] = {
    {"pg_bind", pg_bind, METH_VARARGS,
     "pg_bind(statement, params) -> Bind+Describe+Execute+Sync messages (text-format parameters)"},
    {"pg_decode_text", pg_decode, METH_VARARGS, "pg_decode_text(oid, text) -> value (PgReader's decoding)"},
    {nullptr, nullptr, 0, nullptr}};

}  // namespace

int init_pg_types(PyObject* m) {
  PgReaderType.tp_name = "beholder_amd.ops._native.PgReader";
  PgReaderType.tp_basicsize = sizeof(PgReaderObject);
  PgReaderType.tp_flags = Py_TPFLAGS_DEFAULT;
  PgReaderType.tp_doc = "PgReader(max_message=1GiB): PostgreSQL v3 backend message reader";
  PgReaderType.tp_new = pg_new;
  PgReaderType.tp_init = reinterpret_cast<initproc>(pg_init);
  PgReaderType.tp_dealloc = reinterpret_cast<destructor>(pg_dealloc);
  PgReaderType.tp_methods = pg_methods;
  PgReaderType.tp_getset = pg_getset;
  if (PyType_Ready(&PgReaderType) < 0) return -1;
  Py_INCREF(&PgReaderType);
  if (PyModule_AddObject(m, "PgReader", reinterpret_cast<PyObject*>(&PgReaderType)) < 0) return -1;
  return PyModule_AddFunctions(m, pg_functions);
}

}  // namespace beholder
