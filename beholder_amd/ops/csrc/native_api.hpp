// The C interface `_native` offers to other extension modules of the package (today only the
// bench/test module `_native_bench`, ops/csrc_bench/), so that bench and diagnostic code lives
// outside the service's extension and still runs the service's own native code paths.
//
// * `_native._C_API`: a capsule named kNativeApiName holding a NativeApi table.
// * A sink hook: an HTTP client may expose, as its `native_record` attribute, a capsule named
//   kSinkHookName whose pointer is a SinkHook and whose context is the object the hook is called
//   on. The compiled handlers (py_handlers.cpp http_request) then make the client's sink
//   requests through the hook, without entering its Python `request` coroutine.
#pragma once

#define PY_SSIZE_T_CLEAN
#include <Python.h>

#include <cstdint>
#include <string>

namespace beholder {

constexpr const char* kNativeApiName = "beholder_amd.ops._native._C_API";
constexpr uint32_t kNativeApiAbi = 3;

struct NativeApi {
  uint32_t abi;  // kNativeApiAbi
  // Whether the H1 client's native path sends http.request(method, url, params=params) (the
  // shape check of py_h1call.cpp): 1 with *key_len = length of "scheme://authority" in `url`
  // (the origin's key), or 0 (the Python client would take it). Never raises.
  int (*h1_origin_key)(PyObject* method, PyObject* url, PyObject* params, Py_ssize_t* key_len);
  // The H1 client's request text (py_h1call.cpp, what its native path writes to the socket) for
  // http.request(method, url, params=params) on an origin with Host `host` and Authorization
  // `auth` (str, or None): "M target?query HTTP/1.1\r\nHost: ...\r\n[Authorization: ...\r\n]" then
  // `tail` (bytes; `tail_cl0` for methods with a body). *full = the URL with its query (new
  // reference). *key_len = length of "scheme://authority" in `url`; a caller that has it from
  // h1_origin_key for the same (method, url, params) objects, as its very next API call, passes
  // it in (> 0) and the byte scan of the shape check is not repeated, as the H1 client's own path
  // checks once. Any other key_len (another URL's, or one passed later) is not trusted: the full
  // check runs. 1 = built, 0 = not the shape the native path sends (the Python client would take
  // it), -1 = error.
  int (*h1_request_text)(PyObject* method, PyObject* url, PyObject* params, PyObject* host, PyObject* auth,
                         PyObject* tail, PyObject* tail_cl0, std::string* req, PyObject** full,
                         Py_ssize_t* key_len);
  // The HttpResponse the native path completes a request with, from an H1Parser result tuple
  // (status, reason, raw_headers, body, keep_alive) and the request's full URL. New reference.
  PyObject* (*h1_response)(PyObject* parsed, PyObject* full);
  // url + "?" + encode_query(params) for a non-empty dict (restler's URL), else url. New reference.
  PyObject* (*url_with_query)(PyObject* url, PyObject* params);
  // H1Parser.start(head=...) / .feed(data) as the NetConn calls them (py_http.cpp): exact
  // H1Parser only (is_h1_parser). start: 0 or -1; feed: the parse result (None: incomplete).
  bool (*is_h1_parser)(PyObject* o);
  int (*h1_parser_start)(PyObject* parser, bool head);
  PyObject* (*h1_parser_feed)(PyObject* parser, const char* data, size_t n);
};

constexpr const char* kSinkHookName = "beholder_amd.sink_hook";
constexpr uint32_t kSinkHookAbi = 1;

struct SinkHook {
  uint32_t abi;  // kSinkHookAbi
  // http.request(method, url, params=params): an awaitable (new reference), or NULL with an
  // exception set. `self` is the capsule's context.
  PyObject* (*request)(PyObject* self, PyObject* method, PyObject* url, PyObject* params);
};

}  // namespace beholder
