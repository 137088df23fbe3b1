// H1Parser: incremental HTTP/1.1 response parser for the outbound sink client.
//
// The reference reaches Trello / Telegram / Emby through `request` (index.js:53,
// 83,99,112 via the trello npm client and request-promise-native). Each progress
// event for a Trello-created media costs one HTTPS round trip, so the client's
// per-request CPU is the production ceiling of the service. The asyncio protocol
// in sinks/h1.py hands socket bytes to feed(); framing (status line, headers,
// Content-Length / chunked / close-delimited bodies, 1xx interim responses) is
// done here in one pass without per-line Python objects.
//
//   p = H1Parser(max_header=65536, max_body=64 MiB)
//   p.start(head=False)          # before each request's response
//   p.feed(data) -> None | (status, reason, raw_headers, body, keep_alive)
//   p.eof()      -> None | (...)  # peer closed: completes a close-delimited body
//
// Malformed input raises ValueError; the connection must then be discarded.
// Bytes after a complete response stay buffered (`buffered`), which a
// non-pipelining client treats as a protocol error.
#include <cstring>
#include <string>

#include "py_common.hpp"

namespace beholder {

namespace {

enum class St : uint8_t { IDLE, HEAD, BODY_LEN, CHUNK_SIZE, CHUNK_DATA, CHUNK_CRLF, TRAILERS, BODY_EOF, DONE };

struct H1ParserObject {
  PyObject_HEAD std::string* buf;  // unconsumed input
  std::string* body;
  size_t pos;        // read offset into buf
  size_t scan;       // HEAD: offset already scanned for the end of the header block
  uint64_t remain;   // BODY_LEN / CHUNK_DATA bytes left
  uint64_t max_header, max_body;
  int status;
  std::string* reason;
  std::string* headers;  // raw header lines (CRLF separated), without the status line
  St st;
  bool head_req;
  bool keep_alive;
  bool http11;
  uint64_t responses;
  PyObject* last_reason;   // the last reply's reason / raw headers / body objects (reuse_or_make)
  PyObject* last_headers;
  PyObject* last_body;
};

PyTypeObject H1ParserType = {PyVarObject_HEAD_INIT(nullptr, 0)};

inline bool is_tchar(unsigned char c) {
  return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9') ||
         std::strchr("!#$%&'*+-.^_`|~", c) != nullptr;
}

inline unsigned char lower(unsigned char c) { return (c >= 'A' && c <= 'Z') ? c + 32 : c; }

bool ieq(const char* a, size_t n, const char* lit) {
  size_t m = std::strlen(lit);
  if (n != m) return false;
  for (size_t i = 0; i < n; ++i)
    if (lower(static_cast<unsigned char>(a[i])) != static_cast<unsigned char>(lit[i])) return false;
  return true;
}

void trim(const char*& p, size_t& n) {
  while (n && (*p == ' ' || *p == '\t')) ++p, --n;
  while (n && (p[n - 1] == ' ' || p[n - 1] == '\t')) --n;
}

// Does the comma-separated header value contain `token` (case-insensitive)?
bool has_token(const char* p, size_t n, const char* token) {
  size_t i = 0;
  while (i <= n) {
    size_t j = i;
    while (j < n && p[j] != ',') ++j;
    const char* t = p + i;
    size_t tn = j - i;
    trim(t, tn);
    if (ieq(t, tn, token)) return true;
    i = j + 1;
  }
  return false;
}

// Is the last transfer-coding "chunked"?
bool last_is_chunked(const char* p, size_t n) {
  size_t j = n;
  while (j && p[j - 1] != ',') --j;
  const char* t = p + j;
  size_t tn = n - j;
  trim(t, tn);
  return ieq(t, tn, "chunked");
}

void reset_response(H1ParserObject* s) {
  s->status = 0;
  s->reason->clear();
  s->headers->clear();
  s->body->clear();
  s->remain = 0;
  s->keep_alive = false;
  s->http11 = false;
}

[[noreturn]] void fail(const char* what) { throw std::invalid_argument(what); }

// Next line from buf at *at (terminated by LF, optional CR stripped); false if incomplete.
bool next_line(const std::string& b, size_t* at, const char** p, size_t* n) {
  size_t e = b.find('\n', *at);
  if (e == std::string::npos) return false;
  *p = b.data() + *at;
  *n = e - *at;
  if (*n && (*p)[*n - 1] == '\r') --*n;
  *at = e + 1;
  return true;
}

// Parses the header block buf[pos, end) (end = just past the blank line). Returns true when
// a final (non-1xx) response head was parsed; false for an interim 1xx that was skipped.
bool parse_head(H1ParserObject* s, size_t end) {
  const std::string& b = *s->buf;
  size_t at = s->pos;
  const char* p = nullptr;
  size_t n = 0;
  if (!next_line(b, &at, &p, &n)) fail("malformed HTTP status line");
  // status line: HTTP/d.d SP ddd [SP reason]
  if (n < 12 || std::memcmp(p, "HTTP/", 5) != 0 || p[5] < '0' || p[5] > '9' || p[6] != '.' || p[7] < '0' ||
      p[7] > '9' || p[8] != ' ')
    fail("malformed HTTP status line");
  int major = p[5] - '0', minor = p[7] - '0';
  if (major != 1) fail("unsupported HTTP version");
  for (int i = 9; i < 12; ++i)
    if (p[i] < '0' || p[i] > '9') fail("malformed HTTP status code");
  int status = (p[9] - '0') * 100 + (p[10] - '0') * 10 + (p[11] - '0');
  if (status < 100) fail("malformed HTTP status code");
  if (n > 12 && p[12] != ' ') fail("malformed HTTP status line");
  if (status < 200) {
    if (status == 101) fail("unexpected 101 Switching Protocols");
    s->pos = end;  // interim response: skip it entirely
    return false;
  }
  s->status = status;
  s->http11 = minor >= 1;
  if (n > 13) s->reason->assign(p + 13, n - 13);

  bool conn_close = false, conn_keep = false, chunked = false, has_te = false, has_cl = false;
  uint64_t cl = 0;
  while (at < end) {
    if (!next_line(b, &at, &p, &n) || n == 0) break;
    if (*p == ' ' || *p == '\t') fail("obsolete header line folding");
    const char* colon = static_cast<const char*>(std::memchr(p, ':', n));
    if (!colon || colon == p) fail("malformed HTTP header");
    size_t nn = size_t(colon - p);
    for (size_t i = 0; i < nn; ++i)
      if (!is_tchar(static_cast<unsigned char>(p[i]))) fail("invalid character in header name");
    const char* v = colon + 1;
    size_t vn = n - nn - 1;
    trim(v, vn);
    s->headers->append(p, n);
    s->headers->append("\r\n", 2);
    if (ieq(p, nn, "content-length")) {
      if (vn == 0 || vn > 18) fail("invalid Content-Length");
      uint64_t x = 0;
      for (size_t i = 0; i < vn; ++i) {
        if (v[i] < '0' || v[i] > '9') fail("invalid Content-Length");
        x = x * 10 + uint64_t(v[i] - '0');
      }
      if (has_cl && x != cl) fail("conflicting Content-Length headers");
      has_cl = true;
      cl = x;
    } else if (ieq(p, nn, "transfer-encoding")) {
      has_te = true;
      chunked = last_is_chunked(v, vn);
    } else if (ieq(p, nn, "connection")) {
      if (has_token(v, vn, "close")) conn_close = true;
      if (has_token(v, vn, "keep-alive")) conn_keep = true;
    }
  }
  s->pos = end;
  s->keep_alive = s->http11 ? !conn_close : (conn_keep && !conn_close);
  if (s->head_req || status == 204 || status == 304) {
    s->st = St::DONE;
  } else if (has_te) {
    if (chunked) {
      s->st = St::CHUNK_SIZE;
    } else {
      s->st = St::BODY_EOF;  // non-chunked transfer coding: body runs to connection close
      s->keep_alive = false;
    }
  } else if (has_cl) {
    if (cl > s->max_body) fail("response body exceeds max_body");
    s->remain = cl;
    s->st = cl ? St::BODY_LEN : St::DONE;
  } else {
    s->st = St::BODY_EOF;
    s->keep_alive = false;
  }
  return true;
}

void take_body(H1ParserObject* s, uint64_t want) {
  size_t avail = s->buf->size() - s->pos;
  size_t k = size_t(want < avail ? want : avail);
  s->body->append(s->buf->data() + s->pos, k);
  s->pos += k;
  s->remain -= k;
}

// Advances the state machine over the buffered input. Returns true when a response is complete.
bool run(H1ParserObject* s) {
  std::string& b = *s->buf;
  for (;;) {
    switch (s->st) {
      case St::IDLE:
        if (s->pos < b.size()) fail("unexpected data before request");
        return false;
      case St::HEAD: {
        // find the blank line ending the header block (LF LF or CRLF CRLF, mixed allowed)
        size_t i = s->scan > s->pos ? s->scan : s->pos;
        size_t end = std::string::npos;
        while (true) {
          size_t e = b.find('\n', i);
          if (e == std::string::npos) break;
          size_t nx = e + 1;
          if (nx < b.size() && b[nx] == '\n') {
            end = nx + 1;
            break;
          }
          if (nx + 1 < b.size() && b[nx] == '\r' && b[nx + 1] == '\n') {
            end = nx + 2;
            break;
          }
          if (nx >= b.size() || (b[nx] == '\r' && nx + 1 >= b.size())) {
            i = e;  // blank-line candidate not fully buffered yet; rescan from this LF
            break;
          }
          i = nx;
        }
        if (end == std::string::npos) {
          if (b.size() - s->pos > s->max_header) fail("response header block too large");
          s->scan = i;
          return false;
        }
        if (end - s->pos > s->max_header + 4) fail("response header block too large");
        s->scan = 0;
        if (!parse_head(s, end)) continue;  // 1xx skipped, parse the next head
        break;
      }
      case St::BODY_LEN:
        take_body(s, s->remain);
        if (s->remain) return false;
        s->st = St::DONE;
        break;
      case St::CHUNK_SIZE: {
        size_t at = s->pos;
        const char* p;
        size_t n;
        if (!next_line(b, &at, &p, &n)) {
          if (b.size() - s->pos > 4096) fail("chunk size line too long");
          return false;
        }
        size_t k = 0;
        uint64_t x = 0;
        while (k < n) {
          char c = p[k];
          int d = (c >= '0' && c <= '9') ? c - '0' : (c >= 'a' && c <= 'f') ? c - 'a' + 10
                                                   : (c >= 'A' && c <= 'F') ? c - 'A' + 10 : -1;
          if (d < 0) break;
          if (k >= 15) fail("chunk size too large");
          x = x * 16 + uint64_t(d);
          ++k;
        }
        if (k == 0) fail("malformed chunk size");
        while (k < n && (p[k] == ' ' || p[k] == '\t')) ++k;
        if (k < n && p[k] != ';') fail("malformed chunk size");
        s->pos = at;
        if (x == 0) {
          s->st = St::TRAILERS;
        } else {
          if (s->body->size() + x > s->max_body) fail("response body exceeds max_body");
          s->remain = x;
          s->st = St::CHUNK_DATA;
        }
        break;
      }
      case St::CHUNK_DATA:
        take_body(s, s->remain);
        if (s->remain) return false;
        s->st = St::CHUNK_CRLF;
        break;
      case St::CHUNK_CRLF: {
        size_t at = s->pos;
        const char* p;
        size_t n;
        if (!next_line(b, &at, &p, &n)) {
          if (b.size() - s->pos >= 2) fail("missing CRLF after chunk data");
          return false;
        }
        if (n != 0) fail("missing CRLF after chunk data");
        s->pos = at;
        s->st = St::CHUNK_SIZE;
        break;
      }
      case St::TRAILERS: {
        size_t at = s->pos;
        const char* p;
        size_t n;
        for (;;) {
          if (!next_line(b, &at, &p, &n)) {
            if (b.size() - s->pos > s->max_header) fail("trailer block too large");
            return false;
          }
          s->pos = at;
          if (n == 0) break;
        }
        s->st = St::DONE;
        break;
      }
      case St::BODY_EOF: {
        size_t avail = b.size() - s->pos;
        if (s->body->size() + avail > s->max_body) fail("response body exceeds max_body");
        s->body->append(b.data() + s->pos, avail);
        s->pos += avail;
        return false;
      }
      case St::DONE:
        return true;
    }
  }
}

// An immutable object equal to the last one made from the same field, or a new one (then kept).
// A keep-alive connection's replies mostly repeat the reason phrase and often the headers and
// body, so most replies reuse the objects (they are immutable: sharing is invisible).
PyObject* reuse_or_make(PyObject** cache, const std::string& v, bool text) {
  PyObject* c = *cache;
  if (c) {
    const char* d;
    Py_ssize_t n;
    if (text) {
      d = reinterpret_cast<const char*>(PyUnicode_1BYTE_DATA(c));
      n = PyUnicode_GET_LENGTH(c);
    } else {
      d = PyBytes_AS_STRING(c);
      n = PyBytes_GET_SIZE(c);
    }
    if (size_t(n) == v.size() && memcmp(d, v.data(), v.size()) == 0) return Py_NewRef(c);
  }
  PyObject* o;
  if (text) {
    // reason phrases are opaque octets: UTF-8 when they are, else latin-1
    o = PyUnicode_DecodeUTF8(v.data(), Py_ssize_t(v.size()), nullptr);
    if (!o) {
      PyErr_Clear();
      o = PyUnicode_DecodeLatin1(v.data(), Py_ssize_t(v.size()), nullptr);
    }
    if (o && !PyUnicode_IS_ASCII(o)) return o;  // only ASCII ones are cached (compared bytewise above)
  } else {
    o = PyBytes_FromStringAndSize(v.data(), Py_ssize_t(v.size()));
  }
  if (!o) return nullptr;
  if (v.size() <= 4096) Py_XSETREF(*cache, Py_NewRef(o));
  return o;
}

PyObject* make_result(H1ParserObject* s) {
  PyObject* st = PyLong_FromLong(s->status);
  PyObject* reason = st ? reuse_or_make(&s->last_reason, *s->reason, true) : nullptr;
  PyObject* hdr = reason ? reuse_or_make(&s->last_headers, *s->headers, false) : nullptr;
  PyObject* body = hdr ? reuse_or_make(&s->last_body, *s->body, false) : nullptr;
  PyObject* r = body ? PyTuple_New(5) : nullptr;
  if (!r) {
    Py_XDECREF(st);
    Py_XDECREF(reason);
    Py_XDECREF(hdr);
    Py_XDECREF(body);
    return nullptr;
  }
  PyTuple_SET_ITEM(r, 0, st);
  PyTuple_SET_ITEM(r, 1, reason);
  PyTuple_SET_ITEM(r, 2, hdr);
  PyTuple_SET_ITEM(r, 3, body);
  PyTuple_SET_ITEM(r, 4, Py_NewRef(s->keep_alive ? Py_True : Py_False));
  ++s->responses;
  s->st = St::IDLE;
  s->body->clear();
  if (s->pos == s->buf->size()) {
    s->buf->clear();
    s->pos = 0;
  }
  return r;
}

void compact(H1ParserObject* s) {
  if (s->pos && (s->pos == s->buf->size() || s->pos > (s->buf->size() >> 1))) {
    s->buf->erase(0, s->pos);
    if (s->scan >= s->pos) s->scan -= s->pos; else s->scan = 0;
    s->pos = 0;
  }
}

PyObject* h1_new(PyTypeObject* type, PyObject*, PyObject*) {
  H1ParserObject* s = reinterpret_cast<H1ParserObject*>(type->tp_alloc(type, 0));
  if (!s) return nullptr;
  try {
    s->buf = new std::string();
    s->body = new std::string();
    s->reason = new std::string();
    s->headers = new std::string();
  } catch (const std::bad_alloc&) {
    Py_DECREF(s);
    return PyErr_NoMemory();
  }
  s->pos = s->scan = 0;
  s->remain = 0;
  s->max_header = 65536;
  s->max_body = 64ull << 20;
  s->st = St::IDLE;
  s->head_req = false;
  s->responses = 0;
  reset_response(s);
  return reinterpret_cast<PyObject*>(s);
}

int h1_init(H1ParserObject* s, PyObject* args, PyObject* kwds) {
  static const char* kwlist[] = {"max_header", "max_body", nullptr};
  unsigned long long mh = 65536, mb = 64ull << 20;
  if (!PyArg_ParseTupleAndKeywords(args, kwds, "|KK", const_cast<char**>(kwlist), &mh, &mb)) return -1;
  if (mh < 64) {
    PyErr_SetString(PyExc_ValueError, "max_header must be >= 64");
    return -1;
  }
  s->max_header = mh;
  s->max_body = mb;
  return 0;
}

void h1_dealloc(H1ParserObject* s) {
  Py_XDECREF(s->last_reason);
  Py_XDECREF(s->last_headers);
  Py_XDECREF(s->last_body);
  delete s->buf;
  delete s->body;
  delete s->reason;
  delete s->headers;
  Py_TYPE(s)->tp_free(reinterpret_cast<PyObject*>(s));
}

int start_core(H1ParserObject* s, bool head) {
  if (s->st != St::IDLE) {
    PyErr_SetString(PyExc_RuntimeError, "H1Parser.start() while a response is in progress");
    return -1;
  }
  reset_response(s);
  s->head_req = head;
  s->scan = 0;
  s->st = St::HEAD;
  return 0;
}

// start(head=False): vectorcall, one optional argument (positional or `head=`)
PyObject* h1_start(H1ParserObject* s, PyObject* const* args, Py_ssize_t nargs, PyObject* kwnames) {
  Py_ssize_t nkw = kwnames ? PyTuple_GET_SIZE(kwnames) : 0;
  PyObject* v = nullptr;
  if (nargs > 1 || nargs + nkw > 1) {
    PyErr_SetString(PyExc_TypeError, "start(head=False) takes one optional argument");
    return nullptr;
  }
  if (nargs == 1) {
    v = args[0];
  } else if (nkw == 1) {
    if (PyUnicode_CompareWithASCIIString(PyTuple_GET_ITEM(kwnames, 0), "head") != 0) {
      PyErr_Format(PyExc_TypeError, "start() got an unexpected keyword argument '%U'", PyTuple_GET_ITEM(kwnames, 0));
      return nullptr;
    }
    v = args[0];
  }
  int head = v ? PyObject_IsTrue(v) : 0;
  if (head < 0 || start_core(s, head != 0) < 0) return nullptr;
  Py_RETURN_NONE;
}

PyObject* feed_core(H1ParserObject* s, const char* data, size_t n) {
  BEHOLDER_TRY {
    s->buf->append(data, n);
    bool done;
    try {
      done = run(s);
    } catch (const std::invalid_argument& e) {
      s->st = St::IDLE;
      s->buf->clear();
      s->pos = 0;
      PyErr_SetString(PyExc_ValueError, e.what());
      return nullptr;
    }
    if (done) return make_result(s);
    compact(s);
    Py_RETURN_NONE;
  }
  BEHOLDER_CATCH(nullptr)
}

PyObject* h1_feed(H1ParserObject* s, PyObject* arg) {
  Py_buffer view;
  if (PyObject_GetBuffer(arg, &view, PyBUF_SIMPLE) < 0) return nullptr;
  PyObject* r = feed_core(s, static_cast<const char*>(view.buf), size_t(view.len));
  PyBuffer_Release(&view);
  return r;
}

PyObject* h1_eof(H1ParserObject* s, PyObject*) {
  BEHOLDER_TRY {
    if (s->st == St::IDLE) Py_RETURN_NONE;
    if (s->st == St::BODY_EOF) {
      s->st = St::DONE;
      return make_result(s);
    }
    if (s->st == St::DONE) return make_result(s);
    bool fresh = s->st == St::HEAD && s->pos == s->buf->size();
    s->st = St::IDLE;
    s->buf->clear();
    s->pos = 0;
    if (fresh) Py_RETURN_NONE;  // closed before any byte of the response
    PyErr_SetString(PyExc_ValueError, "connection closed mid-response");
    return nullptr;
  }
  BEHOLDER_CATCH(nullptr)
}

PyObject* h1_get_buffered(H1ParserObject* s, void*) { return PyLong_FromSize_t(s->buf->size() - s->pos); }
PyObject* h1_get_responses(H1ParserObject* s, void*) { return PyLong_FromUnsignedLongLong(s->responses); }
PyObject* h1_get_idle(H1ParserObject* s, void*) { return PyBool_FromLong(s->st == St::IDLE); }
PyObject* h1_get_started(H1ParserObject* s, void*) {
  // any byte of the current response received yet (a reused connection that fails
  // before this point never saw the request processed... as far as the client can tell)
  return PyBool_FromLong(s->st != St::IDLE && !(s->st == St::HEAD && s->pos == s->buf->size()));
}

PyMethodDef h1_methods[] = {
    {"start", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(h1_start)), METH_FASTCALL | METH_KEYWORDS,
     "start(head=False): expect the response to a new request"},
    {"feed", reinterpret_cast<PyCFunction>(h1_feed), METH_O,
     "feed(data) -> None | (status, reason, raw_headers, body, keep_alive)"},
    {"eof", reinterpret_cast<PyCFunction>(h1_eof), METH_NOARGS,
     "eof() -> None | result: the peer closed the connection"},
    {nullptr, nullptr, 0, nullptr}};

PyGetSetDef h1_getset[] = {
    {"buffered", reinterpret_cast<getter>(h1_get_buffered), nullptr, "unconsumed input bytes", nullptr},
    {"responses", reinterpret_cast<getter>(h1_get_responses), nullptr, "complete responses parsed", nullptr},
    {"idle", reinterpret_cast<getter>(h1_get_idle), nullptr, "no response expected", nullptr},
    {"started", reinterpret_cast<getter>(h1_get_started), nullptr, "bytes of the current response seen", nullptr},
    {nullptr, nullptr, nullptr, nullptr, nullptr}};

}  // namespace

// H1Parser.start / feed for a caller in C (py_netconn.cpp): no argument parsing, no memoryview.
// Exact H1Parser only (is_h1_parser); the same semantics as the methods.
bool is_h1_parser(PyObject* o) { return Py_TYPE(o) == &H1ParserType; }

int h1_parser_start_c(PyObject* o, bool head) { return start_core(reinterpret_cast<H1ParserObject*>(o), head); }

PyObject* h1_parser_feed_c(PyObject* o, const char* data, size_t n) {
  return feed_core(reinterpret_cast<H1ParserObject*>(o), data, n);
}

int init_http_types(PyObject* m) {
  H1ParserType.tp_name = "beholder_amd.ops._native.H1Parser";
  H1ParserType.tp_basicsize = sizeof(H1ParserObject);
  H1ParserType.tp_flags = Py_TPFLAGS_DEFAULT;
  H1ParserType.tp_doc = "H1Parser(max_header=65536, max_body=64MiB): incremental HTTP/1.1 response parser";
  H1ParserType.tp_new = h1_new;
  H1ParserType.tp_init = reinterpret_cast<initproc>(h1_init);
  H1ParserType.tp_dealloc = reinterpret_cast<destructor>(h1_dealloc);
  H1ParserType.tp_methods = h1_methods;
  H1ParserType.tp_getset = h1_getset;
  if (PyType_Ready(&H1ParserType) < 0) return -1;
  Py_INCREF(&H1ParserType);
  return PyModule_AddObject(m, "H1Parser", reinterpret_cast<PyObject*>(&H1ParserType));
}

}  // namespace beholder
