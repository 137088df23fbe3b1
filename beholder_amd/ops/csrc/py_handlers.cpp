// NativeHandlers: the reference's two queue handlers (index.js:62-125 status,
// index.js:127-155 progress) as native state machines.
//
// `NativeHandlers(handlers)` binds to a beholder_amd.handlers.TelemetryHandlers
// and uses the same dependencies: its logger, decoders, enum tables, counters,
// config lists, store and sink clients. `on_status(rmsg)` / `on_progress(rmsg)`
// return a HandlerCall. It is an awaitable iterator (am_send, send, throw, close)
// that dispatch_batch, the Driver and `await` all drive like the coroutine of
// the Python method. Every step runs in C, up to the first await that really
// suspends. An await on the store or a sink delegates to the Python awaitable
// (`yield from` semantics). A store or sink that completes synchronously (the
// in-memory store, buffered sinks) never leaves C.
//
// Branch and quirk mapping is the Python method's, line for line:
//   status:   decode (errors escape: Q1) -> log -> updateStatus -> NO_TRELLO ack (Q2)
//             -> enumToString -> getByID -> Trello move / missing-list warn (Q5, Q6)
//             -> try { DEPLOYED hooks (Q3, Q4; TelemetryHandlers._deployed_hooks) } -> ack
//   progress: try { decode -> log -> enumToString + counter (Q6) -> getByID ->
//             comment (Q8) } catch -> warn -> ack (Q7)
// The rare branches (missing-list warning, DEPLOYED hooks) call the Python helpers that the
// Python method calls too, so their text and ordering come from one place.
#include <cstdlib>
#include <string>
#include <vector>

#include "native_api.hpp"
#include "py_common.hpp"

namespace beholder {
PyTypeObject* h1_response_type();       // py_h1call.cpp: sinks/http.py HttpResponse, once registered
PyObject* h1_response_status(PyObject* resp);  // its `status` slot (borrowed; NULL when unset)
}  // namespace beholder
#include "gil_clock.hpp"
#include "ring.hpp"

namespace beholder {

bool text_js_str_append(std::string& out, PyObject* v);
bool text_query_pair_append(std::string& out, PyObject* k, PyObject* v, bool* first, bool rfc3986);
PyObject* pg_pool_execute_c(PyObject* nets, PyObject* sql, PyObject* params, PyObject* spread_at, PyObject* size);
PyObject* h1_call_new(PyObject* client, PyObject* method, PyObject* url, PyObject* params, PyObject* timeout,
                      bool front);
bool is_native_logger(PyObject* logger);
bool logcore_emit(PyObject* logger, bool native, long lvl, PyObject* const* args, Py_ssize_t nargs);
bool sink_stats_record(PyObject* stats, PyObject* status, double seconds);
bool is_sink_stats(PyObject* o);

namespace {

// interned attribute / literal strings
PyObject *s_ack, *s_message, *s_content, *s_mediaId, *s_status, *s_progress, *s_host, *s_creator, *s_creatorId,
    *s_get_nowait, *s_update_nowait, *s_store, *s_get_by_id, *s_update_status, *s_trello, *s_make_request, *s_post,
    *s_put, *s_deployed_hooks, *s_warn_missing_list, *s_child_for, *s_inc, *s_lower,
    *s_throw, *s_close, *s_lists, *s_no_trello, *s_deployed, *s_trello_creator, *s_log, *s_decode_status,
    *s_decode_progress, *s_status_names_s, *s_status_names_p, *s_progress_counter, *s_comment_inc, *s_key,
    *s_token, *s_native_record, *s_base_url, *s_http, *s_timeout, *s_strict, *s_stats, *s_request, *s_params, *s_POST, *s_PUT,
    *s_record, *s_raise_for_status, *s_rows, *s_get_calls, *s_update_calls, *s_limiter, *s_retry,
    *s_hooks_plan, *s_telegram, *s_emby, *s_name, *s_metadataId, *s_GET,
    *s_api_key, *s_send_message, *s_refresh_library, *s_pool, *s_select, *s_update,
    *s_execute, *s_conns, *s_spread_at, *s_size, *s_native_call, *s_native_pick, *kw_params_timeout, *kw_timeout;

// Reference-visible text: read from beholder_amd/texts.py TEXTS when a NativeHandlers is built
// (the same table handlers.py and the sink clients read; no such string is spelled here).
enum TextObj : int {
  X_LOG_COMMENT_0, X_LOG_COMMENT_1,                        // index.js:51
  X_LOG_PROGRESS_0, X_LOG_PROGRESS_1, X_LOG_PROGRESS_2,    // index.js:133
  X_WARN_HOOKS, X_WARN_PROGRESS,                           // index.js:121,150
  X_COMMENT_FALLBACK, X_PARSE_MODE, X_MOVE_POS,            // index.js:54,105,85
  X_Q_KEY, X_Q_TOKEN, X_Q_TEXT, X_Q_LIST, X_Q_POS, X_Q_CHAT, X_Q_PARSE_MODE, X_Q_API_KEY,
  X_ERR_TO_LOWER,                                          // index.js:80,134 (Q6)
  X_N
};
struct TextSpec {
  int slot;
  const char* key;
  int item;  // index into a tuple value, -1 = the value itself
  bool is_int;
};
const TextSpec kTextSpecs[] = {
    {X_LOG_COMMENT_0, "log_comment", 0, false},   {X_LOG_COMMENT_1, "log_comment", 1, false},
    {X_LOG_PROGRESS_0, "log_progress", 0, false}, {X_LOG_PROGRESS_1, "log_progress", 1, false},
    {X_LOG_PROGRESS_2, "log_progress", 2, false}, {X_WARN_HOOKS, "warn_hooks", -1, false},
    {X_WARN_PROGRESS, "warn_progress", -1, false}, {X_COMMENT_FALLBACK, "comment_fallback", -1, false},
    {X_PARSE_MODE, "telegram_parse_mode", -1, false}, {X_MOVE_POS, "trello_move_pos", -1, true},
    {X_Q_KEY, "q_trello_key", -1, false},          {X_Q_TOKEN, "q_trello_token", -1, false},
    {X_Q_TEXT, "q_text", -1, false},               {X_Q_LIST, "q_list", -1, false},
    {X_Q_POS, "q_pos", -1, false},                 {X_Q_CHAT, "q_chat", -1, false},
    {X_Q_PARSE_MODE, "q_parse_mode", -1, false},   {X_Q_API_KEY, "q_api_key", -1, false},
    {X_ERR_TO_LOWER, "err_to_lower", -1, false}};

// templates: pieces between the `{}` holes
enum Tpl : int {
  T_LOG_STATUS, T_LOG_MOVE, T_LOG_TELEGRAM, T_LOG_EMBY,  // index.js:66,82,98,111
  T_COMMENT, T_COMMENT_HOST,                             // index.js:143-146 (Q8)
  T_TELEGRAM_TEXT,                                       // index.js:104
  T_PATH_COMMENT, T_PATH_CARD, T_PATH_TELEGRAM, T_PATH_EMBY,
  T_N
};
struct TplSpec {
  int slot;
  const char* key;
  int holes;
};
const TplSpec kTplSpecs[] = {{T_LOG_STATUS, "log_status", 2},       {T_LOG_MOVE, "log_move", 2},
                             {T_LOG_TELEGRAM, "log_telegram", 1},   {T_LOG_EMBY, "log_emby", 1},
                             {T_COMMENT, "comment", 2},             {T_COMMENT_HOST, "comment_host", 1},
                             {T_TELEGRAM_TEXT, "telegram_text", 2}, {T_PATH_COMMENT, "path_comment", 1},
                             {T_PATH_CARD, "path_card", 1},         {T_PATH_TELEGRAM, "path_telegram", 1},
                             {T_PATH_EMBY, "path_emby", 1}};
struct Templates {
  std::vector<std::string> t[T_N];
};

struct HandlersObject {
  PyObject_HEAD PyObject* h;  // the TelemetryHandlers
  PyObject* hdict;            // h.__dict__ (store / sinks are read per call: swappable)
  PyObject* log;
  PyObject* decode_s;
  PyObject* decode_p;
  PyObject* names_s;        // dict: status number -> enum name (index.js:74)
  PyObject* names_p;        // (index.js:134)
  PyObject* progress_plan;  // dict: status -> (statusText, counter child inc)
  PyObject* progress_counter;
  PyObject* comment_inc;
  PyObject* deployed;
  PyObject* trello_creator;
  PyObject* lists;
  PyObject* get_fn;         // handlers._get (JS property read on config nodes)
  PyObject* err_message;    // handlers.err_message
  PyObject* js_type_error;  // handlers.JsTypeError
  PyObject* x[X_N];         // TEXTS strings / constants (see TextObj)
  Templates* tpl;           // TEXTS templates, split at their holes
  PyObject* res_s;          // decoded-message types when the decoders are native codecs (else NULL)
  PyObject* res_p;
  Py_ssize_t ix_s[2];       // TelemetryStatus slots: mediaId, status
  Py_ssize_t ix_p[4];       // TelemetryProgress slots: mediaId, status, progress, host
  PyObject* media_cls;      // store.base.Media (a NamedTuple)
  Py_ssize_t ix_m[3];       // Media slots: creator, creatorId, status
  PyObject* trello_cls;     // sinks.trello.TrelloClient (exact type: request built here)
  PyObject* telegram_cls;   // sinks.telegram.TelegramClient (exact type: request built here)
  PyObject* emby_cls;       // sinks.emby.EmbyClient (exact type: request built here)
  PyObject* memory_cls;     // store.memory.MemoryStore (exact type: row read here)
  PyObject* pg_cls;         // store.postgres.PostgresStore (exact type: queries issued here)
  PyObject* pool_cls;       // store.pgwire.Pool: its `native_pick` capability is used here when set
  PyObject* h1_fast_fn;     // ops._native.h1_fast: an H1Client's `native_call` capability, called directly
  PyObject* pick_fn;        // ops._native.pg_pool_execute: a Pool's `native_pick` capability
  PyObject* row_to_media;   // store.postgres.row_to_media (rows that are not all-int / NULL-free)
  PyObject* not_found;      // store.base.MediaNotFound
  PyObject* one;            // TRELLO_CREATOR (index.js:79)
  uint64_t completed_sync;
  uint64_t suspended;
  uint8_t no_trello;
  uint8_t native_log;
  // per-request attribute reads of the stock clients / store, cached per dict version (DictView)
  DictView<9> trello_view;  // the Trello client's instance dict (TV_*)
  DictView<2> http_view;    // the sink HTTP client's native_record / native_call
  DictView<3> store_view;   // PostgresStore: _pool, _select, _update
  DictView<4> pool_view;    // Pool: native_pick, _nets, spread_at, size
};

// out += template `t` with its holes filled by String(vals[i]) (as the reference's template literals)
bool tpl_append(std::string& out, const HandlersObject* hs, int t, PyObject* v0, PyObject* v1 = nullptr) {
  const std::vector<std::string>& p = hs->tpl->t[t];
  out += p[0];
  if (!text_js_str_append(out, v0)) return false;
  out += p[1];
  if (p.size() > 2) {
    if (!text_js_str_append(out, v1)) return false;
    out += p[2];
  }
  return true;
}

enum : uint8_t { K_STATUS = 0, K_PROGRESS = 1 };

struct CallObject {
  PyObject_HEAD HandlersObject* hs;
  PyObject* rmsg;
  PyObject* sub;  // awaitable iterator currently delegated to
  PyObject* media_id;
  PyObject* status;
  PyObject* status_text;  // NULL = undefined
  PyObject* progress;
  PyObject* host;
  PyObject* media;
  PyObject* plan;       // DEPLOYED-hooks plan (handlers._hooks_plan()) while the hooks run natively
  PyObject* req_stats;  // sink stats of the request in flight (native path), may be NULL
  int64_t req_t0;
  uint8_t req_native;   // a sink request built here is in flight: request_finish() applies
  uint8_t pg_get;       // a Postgres getByID issued here is in flight: pg_media() applies
  uint8_t req_strict;
  uint8_t kind;
  uint8_t state;
  uint8_t started;
  uint8_t done;
  uint8_t did_suspend;
  uint8_t nreq;  // sink requests this event has issued (a later one is a continuation: front of the queue)
};

PyTypeObject HandlersType = {PyVarObject_HEAD_INIT(nullptr, 0)};
PyTypeObject CallType = {PyVarObject_HEAD_INIT(nullptr, 0)};

// ---------------------------------------------------------------- helpers ---
bool js_truthy(PyObject* v, int* out) {
  if (v == Py_None || v == Py_False) {
    *out = 0;
  } else if (v == Py_True) {
    *out = 1;
  } else if (PyUnicode_Check(v)) {
    *out = PyUnicode_GET_LENGTH(v) != 0;
  } else if (PyLong_Check(v)) {
    *out = Py_SIZE(v) != 0;
  } else if (PyFloat_Check(v)) {
    double d = PyFloat_AS_DOUBLE(v);
    *out = d == d && d != 0.0;
  } else {
    *out = 1;  // objects / arrays, even empty ones
  }
  return true;
}

PyObject* unicode_from(const std::string& s) { return PyUnicode_DecodeUTF8(s.data(), Py_ssize_t(s.size()), "strict"); }

bool log_line(HandlersObject* hs, long lvl, PyObject* const* args, Py_ssize_t n) {
  return logcore_emit(hs->log, hs->native_log != 0, lvl, args, n);
}

// msg.<name>: tuple slot for the known decoded / row types, attribute lookup otherwise
inline PyObject* field(PyObject* obj, PyObject* type, Py_ssize_t ix, PyObject* name) {
  if (type && reinterpret_cast<PyObject*>(Py_TYPE(obj)) == type) {
    PyObject* v = PyTuple_GET_ITEM(obj, ix);
    Py_INCREF(v);
    return v;
  }
  return PyObject_GetAttr(obj, name);
}

// counter.inc(): native Counter bumped in place, anything else called
bool call_inc(PyObject* inc) {
  if (PyCFunction_Check(inc)) {
    PyObject* self = PyCFunction_GET_SELF(inc);
    if (self && Py_TYPE(self) == &CounterType) {
      reinterpret_cast<CounterObject*>(self)->value += 1.0;
      return true;
    }
  }
  PyObject* r = PyObject_CallNoArgs(inc);
  if (!r) return false;
  Py_DECREF(r);
  return true;
}

// rmsg.message.content
PyObject* content_of(PyObject* rmsg) {
  if (Py_TYPE(rmsg) == &DeliveryType) {
    PyObject* c = reinterpret_cast<DeliveryObject*>(rmsg)->content;
    Py_INCREF(c);
    return c;
  }
  PyObject* m = PyObject_GetAttr(rmsg, s_message);
  if (!m) return nullptr;
  PyObject* c = PyObject_GetAttr(m, s_content);
  Py_DECREF(m);
  return c;
}

// instance attribute of the handlers object (store / sinks / sync accessors), borrowed
PyObject* hattr(HandlersObject* hs, PyObject* name) {
  PyObject* v = PyDict_GetItemWithError(hs->hdict, name);
  if (!v && !PyErr_Occurred()) PyErr_Format(PyExc_AttributeError, "handlers have no attribute %U", name);
  return v;
}

// Starts awaiting `aw` (reference stolen). 1 = finished synchronously (*out = result),
// 0 = suspended (*out = the yielded future, c->sub set), -1 = raised.
int await_start(CallObject* c, PyObject* aw, PyObject** out) {
  PyObject* it;
  if (PyCoro_CheckExact(aw)) {
    it = aw;
  } else {
    unaryfunc getter = Py_TYPE(aw)->tp_as_async ? Py_TYPE(aw)->tp_as_async->am_await : nullptr;
    if (!getter) {
      PyErr_Format(PyExc_TypeError, "object %.100s can't be used in 'await' expression", Py_TYPE(aw)->tp_name);
      Py_DECREF(aw);
      return -1;
    }
    it = getter(aw);
    Py_DECREF(aw);
    if (!it) return -1;
  }
  PyObject* y = nullptr;
  PySendResult r = PyIter_Send(it, Py_None, &y);
  if (r == PYGEN_RETURN) {
    Py_DECREF(it);
    *out = y;
    return 1;
  }
  if (r == PYGEN_ERROR) {
    Py_DECREF(it);
    return -1;
  }
  c->sub = it;
  c->did_suspend = 1;
  *out = y;
  return 0;
}

// `except Exception as err: log.warn(text, err_message(err))`. Returns false when the
// pending exception is not an Exception (CancelledError, KeyboardInterrupt) or logging failed.
bool catch_and_warn(HandlersObject* hs, PyObject* text) {
  if (!PyErr_ExceptionMatches(PyExc_Exception)) return false;
  PyObject *et, *ev, *tb;
  PyErr_Fetch(&et, &ev, &tb);
  PyErr_NormalizeException(&et, &ev, &tb);
  Py_XDECREF(tb);
  Py_XDECREF(et);
  if (ev) PyException_SetTraceback(ev, Py_None);  // drop frames (and the delivery they hold)
  PyObject* msg = PyObject_CallOneArg(hs->err_message, ev ? ev : Py_None);
  Py_XDECREF(ev);
  if (!msg) return false;
  PyObject* args[2] = {text, msg};
  bool ok = log_line(hs, 40, args, 2);
  Py_DECREF(msg);
  return ok;
}

PySendResult finish_ack(CallObject* c, PyObject** result) {
  c->done = 1;
  PyObject* r = Py_TYPE(c->rmsg) == &DeliveryType ? delivery_ack_c(c->rmsg)  // rmsg.ack(), index.js:124,151,154
                                                   : PyObject_CallMethodNoArgs(c->rmsg, s_ack);
  if (!r) return PYGEN_ERROR;
  *result = r;
  return PYGEN_RETURN;
}

PySendResult fail(CallObject* c) {
  c->done = 1;
  return PYGEN_ERROR;
}

bool raise_to_lower_case(HandlersObject* hs) {
  PyErr_SetObject(hs->js_type_error, hs->x[X_ERR_TO_LOWER]);
  return false;
}

// The stock Postgres store with an open pool: `pool.execute(sql, params)` issued here (the
// store's own coroutine is skipped). 2 = not applicable (use the store's API), else as await_start.
PyObject* const* const kStoreKeys[3] = {&s_pool, &s_select, &s_update};
PyObject* const* const kPoolKeys[4] = {&s_native_pick, &s_conns, &s_spread_at, &s_size};

int pg_execute(CallObject* c, PyObject* store, PyObject* sql_name, PyObject* params, PyObject** out) {
  HandlersObject* hs = c->hs;
  if (reinterpret_cast<PyObject*>(Py_TYPE(store)) != hs->pg_cls) return 2;
  PyObject** dp = _PyObject_GetDictPtr(store);
  PyObject* sd = dp ? *dp : nullptr;
  if (!sd || !PyDict_CheckExact(sd)) return 2;
  if (!hs->store_view.refresh(sd, kStoreKeys)) return -1;
  PyObject* pool = hs->store_view.v[0];
  PyObject* sql = sql_name == s_select ? hs->store_view.v[1] : sql_name == s_update ? hs->store_view.v[2] : nullptr;
  if (!sql && pool && sql_name != s_select && sql_name != s_update) {
    sql = PyDict_GetItemWithError(sd, sql_name);
    if (!sql && PyErr_Occurred()) return -1;
  }
  if (!pool || pool == Py_None || !sql) return 2;  // not connected yet: the store connects first
  PyObject** pdp = reinterpret_cast<PyObject*>(Py_TYPE(pool)) == hs->pool_cls ? _PyObject_GetDictPtr(pool) : nullptr;
  PyObject* pd = pdp ? *pdp : nullptr;
  if (pd && PyDict_CheckExact(pd) && !hs->pool_view.refresh(pd, kPoolKeys)) return -1;
  PyObject* pick = pd && PyDict_CheckExact(pd) ? hs->pool_view.v[0] : nullptr;
  if (pick && pick == hs->pick_fn) {
    // the pool's native_pick capability (Pool.execute's fast path) in C: the least-loaded native
    // connection takes the query (Pool._nets: None while a connection is on the asyncio path)
    PyObject* conns = hs->pool_view.v[1];
    PyObject* spread = hs->pool_view.v[2];
    PyObject* size = hs->pool_view.v[3];
    if (conns && spread && size && PyList_CheckExact(conns)) {
      Py_INCREF(conns);
      PyObject* f = pg_pool_execute_c(conns, sql, params, spread, size);
      Py_DECREF(conns);
      if (!f) return -1;
      if (f != Py_None) return await_start(c, f, out);
      Py_DECREF(f);  // not all native / must grow: Pool.execute below
    }
  }
  PyObject* args[3] = {pool, sql, params};
  Py_INCREF(pool);  // the call may drop the store's reference (a reconnect)
  PyObject* aw = PyObject_VectorcallMethod(s_execute, args, 3, nullptr);
  Py_DECREF(pool);
  if (!aw) return -1;
  return await_start(c, aw, out);
}

// A Media row (a NamedTuple: a tuple subclass without __dict__) whose fields are all atoms (str,
// int, None: nothing the collector tracks) can never be part of a reference cycle, so it leaves
// the collector's lists at birth. CPython does this lazily for exact tuples only, so a row type
// is otherwise tracked for life: every fresh row from Postgres (one per event) and every row the
// in-memory store replaces filled the young generation, and each full collection walked them.
void untrack_row(PyObject* t) {
  if (!PyObject_GC_IsTracked(t) || Py_TYPE(t)->tp_dictoffset != 0) return;
  for (Py_ssize_t i = 0, n = PyTuple_GET_SIZE(t); i < n; ++i) {
    PyObject* v = PyTuple_GET_ITEM(t, i);
    if (PyObject_IS_GC(v) && PyObject_GC_IsTracked(v)) return;
  }
  PyObject_GC_UnTrack(t);
}

// (rows, tag) of the media SELECT -> Media (store/postgres.py get_by_id + row_to_media).
// Takes and returns a reference; NULL = raised.
PyObject* pg_media(CallObject* c, PyObject* res) {
  HandlersObject* hs = c->hs;
  PyObject* rows = PyTuple_Check(res) && PyTuple_GET_SIZE(res) == 2 ? PyTuple_GET_ITEM(res, 0) : nullptr;
  if (!rows || !PyList_Check(rows)) {
    Py_DECREF(res);
    PyErr_SetString(PyExc_TypeError, "unexpected Postgres result");
    return nullptr;
  }
  if (PyList_GET_SIZE(rows) == 0) {
    Py_DECREF(res);
    PyErr_SetObject(hs->not_found, c->media_id);
    return nullptr;
  }
  PyObject* r = PyList_GET_ITEM(rows, 0);
  Py_INCREF(r);
  Py_DECREF(res);
  bool fast = hs->media_cls && PyTuple_CheckExact(r) && PyTuple_GET_SIZE(r) == 10;
  for (Py_ssize_t i = 0; fast && i < 10; ++i) {
    PyObject* v = PyTuple_GET_ITEM(r, i);
    bool is_int_col = i == 2 || i == 4 || i == 5 || i == 7 || i == 9;
    if (v == Py_None || (is_int_col && !PyLong_CheckExact(v))) fast = false;
  }
  PyObject* m;
  if (fast) {  // Media._make(r)
    PyObject* args = PyTuple_Pack(1, r);
    m = args ? PyTuple_Type.tp_new(reinterpret_cast<PyTypeObject*>(hs->media_cls), args, nullptr) : nullptr;
    Py_XDECREF(args);
    if (m) untrack_row(m);
  } else {
    m = PyObject_CallOneArg(hs->row_to_media, r);
  }
  Py_DECREF(r);
  return m;
}

}  // namespace

void untrack_atomic_row(PyObject* t) { untrack_row(t); }

namespace {

// media = await db.getByID(mediaId). The in-memory store's row read (store/memory.py
// get_by_id_nowait) runs inline; other stores go through their nowait accessor or the coroutine.
int get_media(CallObject* c, PyObject** out) {
  HandlersObject* hs = c->hs;
  PyObject* store = hattr(hs, s_store);
  if (!store) return -1;
  if (reinterpret_cast<PyObject*>(Py_TYPE(store)) == hs->memory_cls) {
    PyObject** dp = _PyObject_GetDictPtr(store);
    PyObject* sd = dp ? *dp : nullptr;
    PyObject* rows = sd ? PyDict_GetItemWithError(sd, s_rows) : nullptr;
    PyObject* calls = rows ? PyDict_GetItemWithError(sd, s_get_calls) : nullptr;
    if (calls && PyDict_CheckExact(rows)) {
      PyObject* n = PyNumber_Add(calls, hs->one);  // self.get_calls += 1
      if (!n) return -1;
      int rc = PyDict_SetItem(sd, s_get_calls, n);
      Py_DECREF(n);
      if (rc < 0) return -1;
      PyObject* m = PyDict_GetItemWithError(rows, c->media_id);
      if (!m) {
        if (!PyErr_Occurred()) PyErr_SetObject(hs->not_found, c->media_id);
        return -1;
      }
      Py_INCREF(m);
      *out = m;
      return 1;
    }
    if (PyErr_Occurred()) return -1;
  }
  PyObject* params = PyTuple_Pack(1, c->media_id);
  if (!params) return -1;
  int k = pg_execute(c, store, s_select, params, out);
  Py_DECREF(params);
  if (k != 2) {
    if (k == 0) c->pg_get = 1;
    if (k == 1 && !(*out = pg_media(c, *out))) return -1;
    return k;
  }
  PyObject* get = hattr(hs, s_get_nowait);
  if (!get) return -1;
  if (get != Py_None) {
    PyObject* m = PyObject_CallOneArg(get, c->media_id);
    if (!m) return -1;
    *out = m;
    return 1;
  }
  PyObject* aw = PyObject_CallMethodOneArg(store, s_get_by_id, c->media_id);
  if (!aw) return -1;
  return await_start(c, aw, out);
}

// db.updateStatus(mediaId, status) on the stock in-memory store, inline (store/memory.py
// update_status_nowait: count the call, replace the row with status = int(status)).
// 1 = done, 0 = not the stock store (caller uses the store's API), -1 = raised.
int update_inline(CallObject* c) {
  HandlersObject* hs = c->hs;
  PyObject* store = hattr(hs, s_store);
  if (!store) return -1;
  if (reinterpret_cast<PyObject*>(Py_TYPE(store)) != hs->memory_cls || !hs->media_cls ||
      !PyLong_CheckExact(c->status))
    return 0;
  PyObject** dp = _PyObject_GetDictPtr(store);
  PyObject* sd = dp ? *dp : nullptr;
  PyObject* rows = sd ? PyDict_GetItemWithError(sd, s_rows) : nullptr;
  PyObject* calls = rows ? PyDict_GetItemWithError(sd, s_update_calls) : nullptr;
  if (!calls || !PyDict_CheckExact(rows)) return PyErr_Occurred() ? -1 : 0;
  PyObject* n = PyNumber_Add(calls, hs->one);  // self.update_calls += 1
  if (!n) return -1;
  int rc = PyDict_SetItem(sd, s_update_calls, n);
  Py_DECREF(n);
  if (rc < 0) return -1;
  PyObject* m = PyDict_GetItemWithError(rows, c->media_id);
  if (!m) return PyErr_Occurred() ? -1 : 1;  // unknown media: nothing to update
  if (reinterpret_cast<PyObject*>(Py_TYPE(m)) != hs->media_cls) {  // foreign row type: m._replace(status=...)
    PyObject* kw = Py_BuildValue("{s:O}", "status", c->status);
    PyObject* meth = kw ? PyObject_GetAttrString(m, "_replace") : nullptr;
    PyObject* nm = meth ? PyObject_Call(meth, PyTuple_New(0), kw) : nullptr;
    Py_XDECREF(meth);
    Py_XDECREF(kw);
    if (!nm) return -1;
    rc = PyDict_SetItem(rows, c->media_id, nm);
    Py_DECREF(nm);
    return rc < 0 ? -1 : 1;
  }
  // Media is a NamedTuple: a copy with the status slot replaced, same type
  Py_ssize_t len = PyTuple_GET_SIZE(m);
  PyObject* items = PyTuple_New(len);
  if (!items) return -1;
  for (Py_ssize_t i = 0; i < len; ++i) {
    PyObject* v = i == hs->ix_m[2] ? c->status : PyTuple_GET_ITEM(m, i);
    Py_INCREF(v);
    PyTuple_SET_ITEM(items, i, v);
  }
  PyObject* args = PyTuple_Pack(1, items);
  Py_DECREF(items);
  if (!args) return -1;
  PyObject* nm = PyTuple_Type.tp_new(reinterpret_cast<PyTypeObject*>(hs->media_cls), args, nullptr);
  Py_DECREF(args);
  if (!nm) return -1;
  untrack_row(nm);
  rc = PyDict_SetItem(rows, c->media_id, nm);
  Py_DECREF(nm);
  return rc < 0 ? -1 : 1;
}

bool record_stats(PyObject* stats, PyObject* status, double seconds) {
  if (is_sink_stats(stats)) return sink_stats_record(stats, status, seconds);
  PyObject* sec = PyFloat_FromDouble(seconds);
  if (!sec) return false;
  PyObject* r = PyObject_CallMethodObjArgs(stats, s_record, status, sec, nullptr);
  Py_DECREF(sec);
  if (!r) return false;
  Py_DECREF(r);
  return true;
}

void count_request(CallObject* c) {
  if (c->nreq < 255) ++c->nreq;
}

// http.request(method, url, params=params, timeout=timeout): for a stock H1Client whose
// `native_call` capability is the native request path, the H1Call is made here without the
// Python method frame. The event's second and later sink requests (a status event's move, then
// its hooks: index.js:83,99,112) are continuations: if they have to wait for a connection they
// wait at the front of the origin's queue, not behind the first requests of newer deliveries.
PyObject* const* const kHttpKeys[2] = {&s_native_record, &s_native_call};

PyObject* http_request(CallObject* c, PyObject* http, PyObject* method, PyObject* url, PyObject* params,
                       PyObject* timeout) {
  HandlersObject* hs = c->hs;
  const bool front = c->nreq > 0;
  count_request(c);
  PyObject** dp = _PyObject_GetDictPtr(http);
  PyObject* hd = dp && *dp && PyDict_CheckExact(*dp) ? *dp : nullptr;
  if (hd && !hs->http_view.refresh(hd, kHttpKeys)) return nullptr;
  PyObject* rec = hd ? hs->http_view.v[0] : nullptr;
  if (rec && PyCapsule_CheckExact(rec) && PyCapsule_IsValid(rec, kSinkHookName)) {
    // a client with a native sink hook (native_api.hpp; the in-process stub of the benches and
    // tests, sinks/http.py RecordingHttpClient): its request, without its coroutine
    const SinkHook* hook = static_cast<const SinkHook*>(PyCapsule_GetPointer(rec, kSinkHookName));
    PyObject* self = static_cast<PyObject*>(PyCapsule_GetContext(rec));
    if (!hook || !self || hook->abi != kSinkHookAbi) {
      if (!PyErr_Occurred()) PyErr_SetString(PyExc_RuntimeError, "native_record: incompatible sink hook");
      return nullptr;
    }
    Py_INCREF(rec);  // borrowed from the client's dict; held (with its context) while it runs
    PyObject* r = hook->request(self, method, url, params ? params : Py_None);
    Py_DECREF(rec);
    return r;
  }
  PyObject* cur = hd ? hs->http_view.v[1] : nullptr;
  if (cur && cur == hs->h1_fast_fn) {
    PyObject* call = h1_call_new(http, method, url, params ? params : Py_None, timeout, front);
    if (call != Py_None) return call;  // an H1Call, or NULL with an exception
    Py_DECREF(call);  // not a stock H1Client
  } else if (PyErr_Occurred()) {
    return nullptr;
  }
  if (params) {
    PyObject* args[5] = {http, method, url, params, timeout};
    return PyObject_VectorcallMethod(s_request, args, 3, kw_params_timeout);
  }
  PyObject* args[4] = {http, method, url, timeout};
  return PyObject_VectorcallMethod(s_request, args, 3, kw_timeout);
}

// Completes a sink request issued on the native path (after its await): per-sink stats, then
// strict mode (Trello's `strict`; Telegram / Emby always raise_for_status, like request-promise).
// Takes and returns the result reference; NULL = raised.
PyObject* request_finish(CallObject* c, PyObject* value) {
  if (!c->req_native) return value;
  c->req_native = 0;
  PyObject* stats = c->req_stats;
  c->req_stats = nullptr;
  double dt = double(gil_mono_ns() - c->req_t0) * 1e-9;
  if (!value) {
    if (stats) {  // stats.record(None, dt); raise
      PyObject *et, *ev, *tb;
      PyErr_Fetch(&et, &ev, &tb);
      if (record_stats(stats, Py_None, dt)) {
        PyErr_Restore(et, ev, tb);
      } else {
        Py_XDECREF(et);
        Py_XDECREF(ev);
        Py_XDECREF(tb);
      }
      Py_DECREF(stats);
    }
    return nullptr;
  }
  // the stock HttpResponse (sinks/http.py): its status read from the slot, and a 2xx needs no
  // raise_for_status() call (it only raises for a non-2xx status)
  PyObject* rt = reinterpret_cast<PyObject*>(h1_response_type());
  long code = -1;
  if (rt && reinterpret_cast<PyObject*>(Py_TYPE(value)) == rt) {
    PyObject* st = h1_response_status(value);
    if (st && PyLong_CheckExact(st)) {
      code = PyLong_AsLong(st);
      if (code == -1 && PyErr_Occurred()) PyErr_Clear();
    }
  }
  if (stats) {
    PyObject* st = PyObject_GetAttr(value, s_status);
    bool ok = st && record_stats(stats, st, dt);
    Py_XDECREF(st);
    Py_DECREF(stats);
    if (!ok) {
      Py_DECREF(value);
      return nullptr;
    }
  }
  if (c->req_strict && !(code >= 200 && code < 300)) {
    PyObject* r = PyObject_CallMethodNoArgs(value, s_raise_for_status);
    if (!r) {
      Py_DECREF(value);
      return nullptr;
    }
    Py_DECREF(r);
  }
  return value;
}

// await trello.makeRequest(method, path, {keys[i]: vals[i]}). For the stock TrelloClient the
// request is built here: query {key, token, ...options} handed to http.request, as
// sinks/trello.py does, with stats recorded by request_finish().
enum { TV_LIMITER, TV_RETRY, TV_KEY, TV_TOKEN, TV_BASE_URL, TV_HTTP, TV_TIMEOUT, TV_STRICT, TV_STATS, TV_N };
PyObject* const* const kTrelloKeys[TV_N] = {&s_limiter, &s_retry,   &s_key,    &s_token, &s_base_url,
                                            &s_http,    &s_timeout, &s_strict, &s_stats};

int trello_request(CallObject* c, PyObject* method, PyObject* method_upper, PyObject* path, PyObject* const* keys,
                   PyObject* const* vals, int nopt, PyObject** out) {
  HandlersObject* hs = c->hs;
  PyObject* trello = hattr(hs, s_trello);
  if (!trello) return -1;
  bool fast = reinterpret_cast<PyObject*>(Py_TYPE(trello)) == hs->trello_cls;
  PyObject** dp = fast ? _PyObject_GetDictPtr(trello) : nullptr;
  PyObject* td = dp && *dp && PyDict_CheckExact(*dp) ? *dp : nullptr;
  PyObject* const* tv = hs->trello_view.v;
  if (td) {  // a rate limit or 429 retries (sinks/ratelimit.py): the client's own make_request
    if (!hs->trello_view.refresh(td, kTrelloKeys)) return -1;
    PyObject* lim = tv[TV_LIMITER];
    PyObject* rty = tv[TV_RETRY];
    if ((lim && lim != Py_None) || (rty && rty != Py_None)) td = nullptr;
  }
  PyObject* query = PyDict_New();
  if (!query) return -1;
  if (td) {  // {"key": self.key, "token": self.token, **options}
    PyObject* key = tv[TV_KEY];
    PyObject* token = key ? tv[TV_TOKEN] : nullptr;
    if (!token || PyDict_SetItem(query, hs->x[X_Q_KEY], key) < 0 || PyDict_SetItem(query, hs->x[X_Q_TOKEN], token) < 0) {
      Py_DECREF(query);
      if (PyErr_Occurred()) return -1;
      td = nullptr;  // unexpected layout: generic path
      query = PyDict_New();
      if (!query) return -1;
    }
  }
  for (int i = 0; i < nopt; ++i) {
    if (PyDict_SetItem(query, keys[i], vals[i]) < 0) {
      Py_DECREF(query);
      return -1;
    }
  }
  PyObject* aw;
  if (!td) {
    PyObject* args[4] = {trello, method, path, query};
    count_request(c);  // a sink request through the client's own method
    aw = PyObject_VectorcallMethod(s_make_request, args, 4, nullptr);
    Py_DECREF(query);
    if (!aw) return -1;
    return await_start(c, aw, out);
  }
  // the view is current for td: nothing ran since its refresh but dict stores on `query`
  PyObject* base = tv[TV_BASE_URL];
  PyObject* http = base ? tv[TV_HTTP] : nullptr;
  PyObject* timeout = http ? tv[TV_TIMEOUT] : nullptr;
  PyObject* strict = timeout ? tv[TV_STRICT] : nullptr;
  PyObject* stats = strict ? tv[TV_STATS] : nullptr;
  if (!stats) {
    Py_DECREF(query);
    if (!PyErr_Occurred()) PyErr_SetString(PyExc_AttributeError, "TrelloClient attributes missing");
    return -1;
  }
  // own them: the calls below may run Python code that rebinds the client's attributes
  PyObject* held[5] = {base, http, timeout, strict, stats};
  for (PyObject* o : held) Py_INCREF(o);
  struct Release {
    PyObject** objs;
    ~Release() {
      for (int i = 0; i < 5; ++i) Py_DECREF(objs[i]);
    }
  } release{held};
  int is_strict = PyObject_IsTrue(strict);
  if (is_strict < 0) {
    Py_DECREF(query);
    return -1;
  }
  PyObject* url = PyUnicode_Concat(base, path);  // self.base_url + path
  if (!url) {
    Py_DECREF(query);
    return -1;
  }
  c->req_t0 = gil_mono_ns();
  aw = http_request(c, http, method_upper, url, query, timeout);  // http.request(M, url, params=, timeout=)
  Py_DECREF(url);
  Py_DECREF(query);
  c->req_native = 1;
  c->req_strict = uint8_t(is_strict);
  if (stats != Py_None) {
    Py_INCREF(stats);
    c->req_stats = stats;
  }
  int k = aw ? await_start(c, aw, out) : -1;
  if (k != 0) {  // finished (or failed) without suspending
    PyObject* v = request_finish(c, k == 1 ? *out : nullptr);
    if (!v) return -1;
    *out = v;
  }
  return k;
}

// Stock Telegram / Emby client without a rate limit or retry policy: its instance dict, else NULL.
PyObject* plain_client_dict(PyObject* client, PyObject* cls) {
  if (reinterpret_cast<PyObject*>(Py_TYPE(client)) != cls) return nullptr;
  PyObject** dp = _PyObject_GetDictPtr(client);
  PyObject* d = dp ? *dp : nullptr;
  if (!d) return nullptr;
  PyObject* lim = PyDict_GetItemWithError(d, s_limiter);
  PyObject* rty = PyDict_GetItemWithError(d, s_retry);
  if (PyErr_Occurred()) {
    PyErr_Clear();
    return nullptr;
  }
  if ((lim && lim != Py_None) || (rty && rty != Py_None)) return nullptr;
  return d;
}

// `await observed(stats, http.request("GET", with_query(url, pairs, rfc3986=True), timeout=...))`
// then raise_for_status() in request_finish: sinks/telegram.py send_message, sinks/emby.py
// refresh_library. `url` is the base URL text; `cd` the client's instance dict.
int sink_get(CallObject* c, PyObject* cd, std::string& url, PyObject* const* keys, PyObject* const* vals, int n,
             PyObject** out) {
  ScratchStr q_buf;
  std::string& q = *q_buf;
  bool first = true;
  for (int i = 0; i < n; ++i)
    if (!text_query_pair_append(q, keys[i], vals[i], &first, true)) return -1;
  if (!q.empty()) {
    url += url.find('?') == std::string::npos ? '?' : '&';
    url += q;
  }
  PyObject* http = PyDict_GetItemWithError(cd, s_http);
  PyObject* timeout = http ? PyDict_GetItemWithError(cd, s_timeout) : nullptr;
  PyObject* stats = timeout ? PyDict_GetItemWithError(cd, s_stats) : nullptr;
  if (!stats) {
    if (!PyErr_Occurred()) PyErr_SetString(PyExc_AttributeError, "sink client attributes missing");
    return -1;
  }
  PyObject* held[3] = {http, timeout, stats};
  for (PyObject* o : held) Py_INCREF(o);
  struct Release {
    PyObject** objs;
    ~Release() {
      for (int i = 0; i < 3; ++i) Py_DECREF(objs[i]);
    }
  } release{held};
  PyObject* full = unicode_from(url);
  if (!full) return -1;
  PyObject* aw = http_request(c, http, s_GET, full, nullptr, timeout);  // http.request("GET", full, timeout=)
  Py_DECREF(full);
  c->req_t0 = gil_mono_ns();
  c->req_native = 1;
  c->req_strict = 1;
  if (stats != Py_None) {
    Py_INCREF(stats);
    c->req_stats = stats;
  }
  int k = aw ? await_start(c, aw, out) : -1;
  if (k != 0) {
    PyObject* v = request_finish(c, k == 1 ? *out : nullptr);
    if (!v) return -1;
    *out = v;
  }
  return k;
}

// Telegram step of the DEPLOYED hooks (index.js:97-107). 2 = nothing to send, else as await_start.
int hook_telegram(CallObject* c, PyObject** out) {
  HandlersObject* hs = c->hs;
  PyObject* plan = c->plan;
  int on = PyObject_IsTrue(PyTuple_GET_ITEM(plan, 0));
  if (on <= 0) return on < 0 ? -1 : 2;
  ScratchStr line_buf;
  std::string& line = *line_buf;
  if (!tpl_append(line, hs, T_LOG_TELEGRAM, c->media_id)) return -1;
  PyObject* lo = unicode_from(line);
  bool ok = lo && log_line(hs, 30, &lo, 1);
  Py_XDECREF(lo);
  if (!ok) return -1;
  // arguments in the order Python evaluates them: chat_id, deployed_text(name, metadataId), token
  PyObject* name = PyObject_GetAttr(c->media, s_name);
  PyObject* meta = name ? PyObject_GetAttr(c->media, s_metadataId) : nullptr;
  ScratchStr text_buf;
  std::string& text = *text_buf;
  ok = meta && tpl_append(text, hs, T_TELEGRAM_TEXT, name, meta);
  Py_XDECREF(name);
  Py_XDECREF(meta);
  if (!ok) return -1;
  PyObject* textobj = unicode_from(text);
  if (!textobj) return -1;
  PyObject* tok = PyObject_CallNoArgs(PyTuple_GET_ITEM(plan, 2));  // config.keys.telegram.token (may throw)
  if (!tok) {
    Py_DECREF(textobj);
    return -1;
  }
  PyObject* tg = hattr(hs, s_telegram);
  PyObject* cd = tg ? plain_client_dict(tg, hs->telegram_cls) : nullptr;
  int k;
  if (!cd) {  // another client, or a rate limit / retries: its own send_message
    if (!tg) {
      Py_DECREF(textobj);
      Py_DECREF(tok);
      return -1;
    }
    PyObject* args[5] = {tg, PyTuple_GET_ITEM(plan, 1), textobj, hs->x[X_PARSE_MODE], tok};
    PyObject* kw = PyTuple_Pack(1, s_token);
    count_request(c);  // a sink request through the client's own method
    PyObject* aw = kw ? PyObject_VectorcallMethod(s_send_message, args, 4, kw) : nullptr;
    Py_XDECREF(kw);
    Py_DECREF(textobj);
    Py_DECREF(tok);
    if (!aw) return -1;
    return await_start(c, aw, out);
  }
  PyObject* base = PyDict_GetItemWithError(cd, s_base_url);
  ScratchStr url_buf;
  std::string& url = *url_buf;
  ok = base && text_js_str_append(url, base);
  ok = ok && tpl_append(url, hs, T_PATH_TELEGRAM, tok);
  Py_DECREF(tok);
  if (!ok) {
    Py_DECREF(textobj);
    if (!PyErr_Occurred()) PyErr_SetString(PyExc_AttributeError, "TelegramClient.base_url missing");
    return -1;
  }
  PyObject* keys[3] = {hs->x[X_Q_CHAT], hs->x[X_Q_TEXT], hs->x[X_Q_PARSE_MODE]};
  PyObject* vals[3] = {PyTuple_GET_ITEM(plan, 1), textobj, hs->x[X_PARSE_MODE]};
  k = sink_get(c, cd, url, keys, vals, 3, out);
  Py_DECREF(textobj);
  return k;
}

// Emby step of the DEPLOYED hooks (index.js:110-118). 2 = nothing to send, else as await_start.
int hook_emby(CallObject* c, PyObject** out) {
  HandlersObject* hs = c->hs;
  PyObject* plan = c->plan;
  int on = PyObject_IsTrue(PyTuple_GET_ITEM(plan, 3));
  if (on <= 0) return on < 0 ? -1 : 2;
  PyObject* host = PyTuple_GET_ITEM(plan, 4);
  PyObject* key = PyTuple_GET_ITEM(plan, 5);
  ScratchStr line_buf;
  std::string& line = *line_buf;
  if (!tpl_append(line, hs, T_LOG_EMBY, host)) return -1;
  PyObject* lo = unicode_from(line);
  bool ok = lo && log_line(hs, 30, &lo, 1);
  Py_XDECREF(lo);
  if (!ok) return -1;
  PyObject* em = hattr(hs, s_emby);
  PyObject* cd = em ? plain_client_dict(em, hs->emby_cls) : nullptr;
  if (!cd) {
    if (!em) return -1;
    PyObject* args[3] = {em, host, key};
    PyObject* kw = PyTuple_Pack(2, s_host, s_api_key);
    count_request(c);  // a sink request through the client's own method
    PyObject* aw = kw ? PyObject_VectorcallMethod(s_refresh_library, args, 1, kw) : nullptr;
    Py_XDECREF(kw);
    if (!aw) return -1;
    return await_start(c, aw, out);
  }
  ScratchStr url_buf;
  std::string& url = *url_buf;
  if (!tpl_append(url, hs, T_PATH_EMBY, host)) return -1;
  PyObject* keys[1] = {hs->x[X_Q_API_KEY]};
  PyObject* vals[1] = {key};
  return sink_get(c, cd, url, keys, vals, 1, out);
}

// ------------------------------------------------------ progress handler ---
// index.js:127-155. state: 0 start, 1 after getByID, 2 after the Trello comment.
PySendResult step_progress(CallObject* c, PyObject* value, PyObject** result) {
  HandlersObject* hs = c->hs;
  int k;
  PyObject* v = nullptr;
  switch (c->state) {
    case 0: {
      PyObject* content = content_of(c->rmsg);
      if (!content) goto catch_;
      PyObject* msg = PyObject_CallOneArg(hs->decode_p, content);  // index.js:129
      Py_DECREF(content);
      if (!msg) goto catch_;
      c->media_id = field(msg, hs->res_p, hs->ix_p[0], s_mediaId);
      c->status = c->media_id ? field(msg, hs->res_p, hs->ix_p[1], s_status) : nullptr;
      c->progress = c->status ? field(msg, hs->res_p, hs->ix_p[2], s_progress) : nullptr;
      c->host = c->progress ? field(msg, hs->res_p, hs->ix_p[3], s_host) : nullptr;
      Py_DECREF(msg);
      if (!c->host) goto catch_;
      {  // index.js:133
        PyObject* args[6] = {hs->x[X_LOG_PROGRESS_0], c->media_id, hs->x[X_LOG_PROGRESS_1], c->status,
                             hs->x[X_LOG_PROGRESS_2], c->progress};
        if (!log_line(hs, 30, args, 6)) goto catch_;
      }
      PyObject* plan = PyDict_GetItemWithError(hs->progress_plan, c->status);
      if (!plan) {
        if (PyErr_Occurred()) goto catch_;
        PyObject* text = PyDict_GetItemWithError(hs->names_p, c->status);  // index.js:134
        if (!text) {
          if (!PyErr_Occurred()) raise_to_lower_case(hs);  // Q6
          goto catch_;
        }
        PyObject* lower = PyObject_CallMethodNoArgs(text, s_lower);
        if (!lower) goto catch_;
        PyObject* child = PyObject_CallMethodOneArg(hs->progress_counter, s_child_for, lower);
        Py_DECREF(lower);
        if (!child) goto catch_;
        PyObject* inc = PyObject_GetAttr(child, s_inc);
        Py_DECREF(child);
        if (!inc) goto catch_;
        plan = PyTuple_Pack(2, text, inc);
        Py_DECREF(inc);
        if (!plan) goto catch_;
        int rc = PyDict_SetItem(hs->progress_plan, c->status, plan);
        Py_DECREF(plan);  // the dict holds it
        if (rc < 0) goto catch_;
      }
      c->status_text = PyTuple_GET_ITEM(plan, 0);
      Py_INCREF(c->status_text);
      if (!call_inc(PyTuple_GET_ITEM(plan, 1))) goto catch_;  // index.js:136-138
      k = get_media(c, &v);  // index.js:140
      if (k < 0) goto catch_;
      if (k == 0) {
        c->state = 1;
        *result = v;
        return PYGEN_NEXT;
      }
      c->media = v;
      goto have_media;
    }
    case 1:
      if (c->pg_get) {
        c->pg_get = 0;
        if (value) value = pg_media(c, value);
      }
      if (!value) goto catch_;
      c->media = value;
    have_media: {
      PyObject* creator = field(c->media, hs->media_cls, hs->ix_m[0], s_creator);
      if (!creator) goto catch_;
      int is_trello = PyObject_RichCompareBool(creator, hs->trello_creator, Py_EQ);  // index.js:142
      Py_DECREF(creator);
      if (is_trello < 0) goto catch_;
      if (!is_trello) goto finish;
      ScratchStr s_buf;  // index.js:143-146 (Q8)
      std::string& s = *s_buf;
      if (!tpl_append(s, hs, T_COMMENT, c->status_text, c->progress)) goto catch_;
      int has_host;
      js_truthy(c->host, &has_host);
      if (has_host && !tpl_append(s, hs, T_COMMENT_HOST, c->host)) goto catch_;
      PyObject* text = unicode_from(s);
      if (!text) goto catch_;
      PyObject* card = field(c->media, hs->media_cls, hs->ix_m[1], s_creatorId);
      if (!card) {
        Py_DECREF(text);
        goto catch_;
      }
      // comment(cardId, text), index.js:50-58
      PyObject* largs[4] = {hs->x[X_LOG_COMMENT_0], card, hs->x[X_LOG_COMMENT_1], text};
      bool ok = log_line(hs, 30, largs, 4);
      ScratchStr path_buf;
      std::string& path = *path_buf;
      ok = ok && tpl_append(path, hs, T_PATH_COMMENT, card);
      Py_DECREF(card);
      if (!ok) {
        Py_DECREF(text);
        goto catch_;
      }
      PyObject* pathobj = unicode_from(path);
      if (!pathobj) {
        Py_DECREF(text);
        goto catch_;
      }
      int truthy;
      js_truthy(text, &truthy);
      PyObject* okeys[1] = {hs->x[X_Q_TEXT]};
      PyObject* ovals[1] = {truthy ? text : hs->x[X_COMMENT_FALLBACK]};
      k = trello_request(c, s_post, s_POST, pathobj, okeys, ovals, 1, &v);  // index.js:53-55
      Py_DECREF(pathobj);
      Py_DECREF(text);
      if (k < 0) goto catch_;
      if (k == 0) {
        c->state = 2;
        *result = v;
        return PYGEN_NEXT;
      }
      Py_DECREF(v);
      goto commented;
    }
    case 2:
      value = request_finish(c, value);
      if (!value) goto catch_;
      Py_DECREF(value);
    commented: {
      if (!call_inc(hs->comment_inc)) goto catch_;  // index.js:57
      goto finish;
    }
    default:
      PyErr_SetString(PyExc_RuntimeError, "HandlerCall: bad state");
      return fail(c);
  }
catch_:  // index.js:149-151 (Q7)
  if (!catch_and_warn(hs, hs->x[X_WARN_PROGRESS])) return fail(c);
finish:
  return finish_ack(c, result);  // index.js:151 / 154
}

// -------------------------------------------------------- status handler ---
// index.js:62-125. Errors outside the hooks try escape (Q1).
// state: 0 start, 1 after updateStatus, 2 after getByID, 3 after the card move,
// 5 after the Telegram message, 6 after the Emby refresh.
PySendResult step_status(CallObject* c, PyObject* value, PyObject** result) {
  HandlersObject* hs = c->hs;
  int k;
  PyObject* v = nullptr;
  switch (c->state) {
    case 0: {
      PyObject* content = content_of(c->rmsg);
      if (!content) return fail(c);
      PyObject* msg = PyObject_CallOneArg(hs->decode_s, content);  // index.js:63
      Py_DECREF(content);
      if (!msg) return fail(c);
      c->media_id = field(msg, hs->res_s, hs->ix_s[0], s_mediaId);
      c->status = c->media_id ? field(msg, hs->res_s, hs->ix_s[1], s_status) : nullptr;
      Py_DECREF(msg);
      if (!c->status) return fail(c);
      ScratchStr s_buf;  // index.js:66
      std::string& s = *s_buf;
      if (!tpl_append(s, hs, T_LOG_STATUS, c->media_id, c->status)) return fail(c);
      PyObject* line = unicode_from(s);
      if (!line) return fail(c);
      bool ok = log_line(hs, 30, &line, 1);
      Py_DECREF(line);
      if (!ok) return fail(c);
      int inl = update_inline(c);  // index.js:68
      if (inl < 0) return fail(c);
      if (inl) goto updated;
      if (PyLong_CheckExact(c->status)) {  // Postgres: UPDATE ... SET status = int(status)
        PyObject* store = hattr(hs, s_store);
        if (!store) return fail(c);
        PyObject* params = PyTuple_Pack(2, c->status, c->media_id);
        if (!params) return fail(c);
        k = pg_execute(c, store, s_update, params, &v);
        Py_DECREF(params);
        if (k < 0) return fail(c);
        if (k == 0) {
          c->state = 1;
          *result = v;
          return PYGEN_NEXT;
        }
        if (k == 1) {
          Py_DECREF(v);
          goto updated;
        }
      }
      PyObject* upd = hattr(hs, s_update_nowait);
      if (!upd) return fail(c);
      if (upd != Py_None) {
        PyObject* args[2] = {c->media_id, c->status};
        PyObject* r = PyObject_Vectorcall(upd, args, 2, nullptr);
        if (!r) return fail(c);
        Py_DECREF(r);
        goto updated;
      }
      PyObject* store = hattr(hs, s_store);
      if (!store) return fail(c);
      PyObject* args[3] = {store, c->media_id, c->status};
      PyObject* aw = PyObject_VectorcallMethod(s_update_status, args, 3, nullptr);
      if (!aw) return fail(c);
      k = await_start(c, aw, &v);
      if (k < 0) return fail(c);
      if (k == 0) {
        c->state = 1;
        *result = v;
        return PYGEN_NEXT;
      }
      Py_DECREF(v);
      goto updated;
    }
    case 1:
      if (!value) return fail(c);
      Py_DECREF(value);
    updated: {
      if (hs->no_trello) return finish_ack(c, result);  // index.js:70-72 (Q2)
      PyObject* text = PyDict_GetItemWithError(hs->names_s, c->status);  // index.js:74
      if (!text && PyErr_Occurred()) return fail(c);
      Py_XINCREF(text);
      c->status_text = text;
      k = get_media(c, &v);  // index.js:76
      if (k < 0) return fail(c);
      if (k == 0) {
        c->state = 2;
        *result = v;
        return PYGEN_NEXT;
      }
      c->media = v;
      goto have_media;
    }
    case 2:
      if (c->pg_get) {
        c->pg_get = 0;
        if (value) value = pg_media(c, value);
      }
      if (!value) return fail(c);
      c->media = value;
    have_media: {  // TRELLO Movement, index.js:78-90
      PyObject* creator = field(c->media, hs->media_cls, hs->ix_m[0], s_creator);
      if (!creator) return fail(c);
      int is_trello = PyObject_RichCompareBool(creator, hs->one, Py_EQ);  // index.js:79
      Py_DECREF(creator);
      if (is_trello < 0) return fail(c);
      if (!is_trello) goto hooks;
      if (!c->status_text) {  // `statusText.toLowerCase()` on undefined (Q6)
        raise_to_lower_case(hs);
        return fail(c);
      }
      PyObject* lower = PyObject_CallMethodNoArgs(c->status_text, s_lower);
      if (!lower) return fail(c);
      PyObject* lp;  // index.js:80
      if (PyDict_CheckExact(hs->lists)) {
        lp = PyDict_GetItemWithError(hs->lists, lower);
        if (!lp && PyErr_Occurred()) {
          Py_DECREF(lower);
          return fail(c);
        }
        lp = lp ? lp : Py_None;
        Py_INCREF(lp);
      } else {
        lp = PyObject_CallFunctionObjArgs(hs->get_fn, hs->lists, lower, nullptr);
      }
      Py_DECREF(lower);
      if (!lp) return fail(c);
      int truthy;
      js_truthy(lp, &truthy);
      if (!truthy) {  // Q5
        Py_DECREF(lp);
        PyObject* text = c->status_text;
        PyObject* r = PyObject_CallMethodObjArgs(hs->h, s_warn_missing_list, c->status, text, nullptr);
        if (!r) return fail(c);
        Py_DECREF(r);
        goto hooks;
      }
      PyObject* card = field(c->media, hs->media_cls, hs->ix_m[1], s_creatorId);
      if (!card) {
        Py_DECREF(lp);
        return fail(c);
      }
      ScratchStr s_buf, path_buf;  // index.js:82
      std::string &s = *s_buf, &path = *path_buf;
      bool ok = tpl_append(s, hs, T_LOG_MOVE, c->media_id, card);
      ok = ok && tpl_append(path, hs, T_PATH_CARD, card);
      Py_DECREF(card);
      PyObject* line = ok ? unicode_from(s) : nullptr;
      ok = line && log_line(hs, 30, &line, 1);
      Py_XDECREF(line);
      PyObject* pathobj = ok ? unicode_from(path) : nullptr;
      if (!pathobj) {
        Py_DECREF(lp);
        return fail(c);
      }
      PyObject* okeys[2] = {hs->x[X_Q_LIST], hs->x[X_Q_POS]};
      PyObject* ovals[2] = {lp, hs->x[X_MOVE_POS]};
      k = trello_request(c, s_put, s_PUT, pathobj, okeys, ovals, 2, &v);  // index.js:83-86
      Py_DECREF(pathobj);
      Py_DECREF(lp);
      if (k < 0) return fail(c);
      if (k == 0) {
        c->state = 3;
        *result = v;
        return PYGEN_NEXT;
      }
      Py_DECREF(v);
      goto hooks;
    }
    case 3:
      value = request_finish(c, value);
      if (!value) return fail(c);
      Py_DECREF(value);
    hooks: {  // try { ... } catch, index.js:92-122
      PyObject* ms = field(c->media, hs->media_cls, hs->ix_m[2], s_status);
      if (!ms) goto hooks_catch;
      int deployed = PyObject_RichCompareBool(ms, hs->deployed, Py_EQ);  // index.js:94 (Q3)
      Py_DECREF(ms);
      if (deployed < 0) goto hooks_catch;
      if (!deployed) return finish_ack(c, result);
      // the DEPLOYED branch: handlers._deployed_hooks, step by step (config plan from the same helper)
      PyObject* plan = PyObject_CallMethodNoArgs(hs->h, s_hooks_plan);
      if (!plan) goto hooks_catch;
      if (!PyTuple_Check(plan) || PyTuple_GET_SIZE(plan) != 6) {
        Py_DECREF(plan);
        PyErr_SetString(PyExc_TypeError, "_hooks_plan() must return a 6-tuple");
        goto hooks_catch;
      }
      c->plan = plan;
      k = hook_telegram(c, &v);
      if (k < 0) goto hooks_catch;
      if (k == 0) {
        c->state = 5;
        *result = v;
        return PYGEN_NEXT;
      }
      if (k == 1) Py_DECREF(v);
      goto emby;
    }
    case 5:
      value = request_finish(c, value);
      if (!value) goto hooks_catch;
      Py_DECREF(value);
    emby: {
      k = hook_emby(c, &v);
      if (k < 0) goto hooks_catch;
      if (k == 0) {
        c->state = 6;
        *result = v;
        return PYGEN_NEXT;
      }
      if (k == 1) Py_DECREF(v);
      return finish_ack(c, result);  // index.js:124
    }
    case 6:
      value = request_finish(c, value);
      if (!value) goto hooks_catch;
      Py_DECREF(value);
      return finish_ack(c, result);  // index.js:124
    default:
      PyErr_SetString(PyExc_RuntimeError, "HandlerCall: bad state");
      return fail(c);
  }
hooks_catch:  // index.js:120-122 (Q4)
  if (!catch_and_warn(hs, hs->x[X_WARN_HOOKS])) return fail(c);
  return finish_ack(c, result);
}

PySendResult step(CallObject* c, PyObject* value, PyObject** result) {
  PySendResult r = c->kind == K_STATUS ? step_status(c, value, result) : step_progress(c, value, result);
  if (r != PYGEN_NEXT) {
    c->done = 1;
    if (c->did_suspend)
      c->hs->suspended++;
    else
      c->hs->completed_sync++;
  }
  return r;
}

// ------------------------------------------------------ HandlerCall type ---
PySendResult call_am_send(CallObject* c, PyObject* arg, PyObject** result) {
  if (c->done) {
    PyErr_SetString(PyExc_RuntimeError, "cannot reuse already awaited handler call");
    return PYGEN_ERROR;
  }
  if (!c->started) {
    if (arg != Py_None) {
      PyErr_SetString(PyExc_TypeError, "can't send non-None value to a just-started handler call");
      return PYGEN_ERROR;
    }
    c->started = 1;
    return step(c, nullptr, result);
  }
  if (!c->sub) {
    PyErr_SetString(PyExc_RuntimeError, "handler call is not suspended");
    return PYGEN_ERROR;
  }
  PyObject* y = nullptr;
  PySendResult r = PyIter_Send(c->sub, arg, &y);
  if (r == PYGEN_NEXT) {
    *result = y;
    return PYGEN_NEXT;
  }
  Py_CLEAR(c->sub);
  return step(c, r == PYGEN_RETURN ? y : nullptr, result);
}

// Converts an am_send outcome to the iterator-protocol return (value or NULL + StopIteration).
PyObject* as_iter_result(PySendResult r, PyObject* res) {
  if (r == PYGEN_NEXT) return res;
  if (r == PYGEN_RETURN) {
    if (res != Py_None) _PyGen_SetStopIterationValue(res);
    else PyErr_SetNone(PyExc_StopIteration);
    Py_DECREF(res);
  }
  return nullptr;
}

PyObject* call_iternext(CallObject* c) {
  PyObject* res = nullptr;
  PySendResult r = call_am_send(c, Py_None, &res);
  if (r == PYGEN_RETURN) {  // tp_iternext: plain NULL (no exception) means StopIteration(None)
    if (res == Py_None) {
      Py_DECREF(res);
      return nullptr;
    }
  }
  return as_iter_result(r, res);
}

PyObject* call_send(CallObject* c, PyObject* arg) {
  PyObject* res = nullptr;
  PySendResult r = call_am_send(c, arg, &res);
  return as_iter_result(r, res);
}

// throw(exc) / throw(type, value=None, tb=None): raise at the current await
PyObject* call_throw(CallObject* c, PyObject* const* a, Py_ssize_t n) {
  if (n < 1 || n > 3) {
    PyErr_SetString(PyExc_TypeError, "throw expected 1 to 3 arguments");
    return nullptr;
  }
  PyObject* exc = a[0];
  if (c->sub) {
    PyObject* meth = PyObject_GetAttr(c->sub, s_throw);
    PyObject* y = nullptr;
    if (meth) {
      y = PyObject_Vectorcall(meth, a, size_t(n), nullptr);
      Py_DECREF(meth);
      if (y) return y;  // the delegate handled it and is still suspended
    } else {
      PyErr_Clear();
      if (PyExceptionInstance_Check(exc))
        PyErr_SetObject(reinterpret_cast<PyObject*>(Py_TYPE(exc)), exc);
      else
        PyErr_SetObject(exc, n > 1 ? a[1] : nullptr);
    }
    Py_CLEAR(c->sub);
    PyObject* value = nullptr;
    if (PyErr_ExceptionMatches(PyExc_StopIteration)) {
      if (_PyGen_FetchStopIterationValue(&value) < 0) value = nullptr;
    }
    PyObject* res = nullptr;
    PySendResult r = step(c, value, &res);
    return as_iter_result(r, res);
  }
  c->done = 1;  // not suspended in a delegate: the exception ends the call, like a fresh coroutine
  if (PyExceptionInstance_Check(exc))
    PyErr_SetObject(reinterpret_cast<PyObject*>(Py_TYPE(exc)), exc);
  else
    PyErr_SetObject(exc, n > 1 ? a[1] : nullptr);
  return nullptr;
}

PyObject* call_close(CallObject* c, PyObject*) {
  c->done = 1;
  if (c->sub) {
    PyObject* sub = c->sub;
    c->sub = nullptr;
    PyObject* r = PyObject_CallMethodNoArgs(sub, s_close);
    Py_DECREF(sub);
    if (!r) {
      if (!PyErr_ExceptionMatches(PyExc_AttributeError)) return nullptr;
      PyErr_Clear();
    } else {
      Py_DECREF(r);
    }
  }
  Py_RETURN_NONE;
}

PyObject* call_await(CallObject* c) {
  Py_INCREF(c);
  return reinterpret_cast<PyObject*>(c);
}

int call_traverse(CallObject* c, visitproc visit, void* arg) {
  Py_VISIT(c->hs);
  Py_VISIT(c->rmsg);
  Py_VISIT(c->sub);
  Py_VISIT(c->media_id);
  Py_VISIT(c->status);
  Py_VISIT(c->status_text);
  Py_VISIT(c->progress);
  Py_VISIT(c->host);
  Py_VISIT(c->media);
  Py_VISIT(c->req_stats);
  Py_VISIT(c->plan);
  return 0;
}

int call_clear(CallObject* c) {
  Py_CLEAR(c->hs);
  Py_CLEAR(c->rmsg);
  Py_CLEAR(c->sub);
  Py_CLEAR(c->media_id);
  Py_CLEAR(c->status);
  Py_CLEAR(c->status_text);
  Py_CLEAR(c->progress);
  Py_CLEAR(c->host);
  Py_CLEAR(c->media);
  Py_CLEAR(c->req_stats);
  Py_CLEAR(c->plan);
  return 0;
}

void call_dealloc(CallObject* c) {
  PyObject_GC_UnTrack(c);
  call_clear(c);
  Py_TYPE(c)->tp_free(reinterpret_cast<PyObject*>(c));
}

PyObject* call_get_state(CallObject* c, void*) { return PyLong_FromLong(c->state); }
PyObject* call_get_done(CallObject* c, void*) { return PyBool_FromLong(c->done); }

PyMethodDef call_methods[] = {
    {"send", reinterpret_cast<PyCFunction>(call_send), METH_O, "send(value): resume at the current await"},
    {"throw", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(call_throw)), METH_FASTCALL,
     "throw(exc): raise at the current await"},
    {"close", reinterpret_cast<PyCFunction>(call_close), METH_NOARGS, "close(): abandon the call"},
    {nullptr, nullptr, 0, nullptr}};

PyGetSetDef call_getset[] = {
    {"state", reinterpret_cast<getter>(call_get_state), nullptr, "resume point (per-handler numbering)", nullptr},
    {"done", reinterpret_cast<getter>(call_get_done), nullptr, "finished (returned or raised)", nullptr},
    {nullptr, nullptr, nullptr, nullptr, nullptr}};

PyAsyncMethods call_async = {reinterpret_cast<unaryfunc>(call_await), nullptr, nullptr,
                             reinterpret_cast<sendfunc>(call_am_send)};

PyObject* make_call(HandlersObject* hs, PyObject* rmsg, uint8_t kind) {
  CallObject* c = PyObject_GC_New(CallObject, &CallType);
  if (!c) return nullptr;
  Py_INCREF(hs);
  c->hs = hs;
  Py_INCREF(rmsg);
  c->rmsg = rmsg;
  c->sub = c->media_id = c->status = c->status_text = c->progress = c->host = c->media = c->req_stats = nullptr;
  c->plan = nullptr;
  c->req_t0 = 0;
  c->req_native = c->req_strict = 0;
  c->pg_get = 0;
  c->kind = kind;
  c->state = 0;
  c->started = c->done = c->did_suspend = 0;
  c->nreq = 0;
  PyObject_GC_Track(c);
  return reinterpret_cast<PyObject*>(c);
}

// ---------------------------------------------------- NativeHandlers type ---
PyObject* hs_on_status(HandlersObject* hs, PyObject* rmsg) { return make_call(hs, rmsg, K_STATUS); }
PyObject* hs_on_progress(HandlersObject* hs, PyObject* rmsg) { return make_call(hs, rmsg, K_PROGRESS); }

PyObject* hs_stats(HandlersObject* hs, PyObject*) {
  return Py_BuildValue("{s:K,s:K,s:O}", "completed_sync", static_cast<unsigned long long>(hs->completed_sync),
                       "suspended", static_cast<unsigned long long>(hs->suspended), "native_log",
                       hs->native_log ? Py_True : Py_False);
}

int hs_traverse(HandlersObject* hs, visitproc visit, void* arg) {
  Py_VISIT(hs->h);
  Py_VISIT(hs->hdict);
  Py_VISIT(hs->log);
  Py_VISIT(hs->decode_s);
  Py_VISIT(hs->decode_p);
  Py_VISIT(hs->names_s);
  Py_VISIT(hs->names_p);
  Py_VISIT(hs->progress_plan);
  Py_VISIT(hs->progress_counter);
  Py_VISIT(hs->comment_inc);
  Py_VISIT(hs->deployed);
  Py_VISIT(hs->trello_creator);
  Py_VISIT(hs->lists);
  Py_VISIT(hs->get_fn);
  Py_VISIT(hs->err_message);
  Py_VISIT(hs->js_type_error);
  for (PyObject* o : hs->x) Py_VISIT(o);
  Py_VISIT(hs->res_s);
  Py_VISIT(hs->res_p);
  Py_VISIT(hs->media_cls);
  Py_VISIT(hs->trello_cls);
  Py_VISIT(hs->telegram_cls);
  Py_VISIT(hs->emby_cls);
  Py_VISIT(hs->memory_cls);
  Py_VISIT(hs->pg_cls);
  Py_VISIT(hs->pool_cls);
  Py_VISIT(hs->pick_fn);
  Py_VISIT(hs->h1_fast_fn);
  Py_VISIT(hs->row_to_media);
  Py_VISIT(hs->not_found);
  return 0;
}

int hs_clear(HandlersObject* hs) {
  Py_CLEAR(hs->h);
  Py_CLEAR(hs->hdict);
  Py_CLEAR(hs->log);
  Py_CLEAR(hs->decode_s);
  Py_CLEAR(hs->decode_p);
  Py_CLEAR(hs->names_s);
  Py_CLEAR(hs->names_p);
  Py_CLEAR(hs->progress_plan);
  Py_CLEAR(hs->progress_counter);
  Py_CLEAR(hs->comment_inc);
  Py_CLEAR(hs->deployed);
  Py_CLEAR(hs->trello_creator);
  Py_CLEAR(hs->lists);
  Py_CLEAR(hs->get_fn);
  Py_CLEAR(hs->err_message);
  Py_CLEAR(hs->js_type_error);
  for (PyObject*& o : hs->x) Py_CLEAR(o);
  Py_CLEAR(hs->res_s);
  Py_CLEAR(hs->res_p);
  Py_CLEAR(hs->media_cls);
  Py_CLEAR(hs->trello_cls);
  Py_CLEAR(hs->telegram_cls);
  Py_CLEAR(hs->emby_cls);
  Py_CLEAR(hs->memory_cls);
  Py_CLEAR(hs->pg_cls);
  Py_CLEAR(hs->pool_cls);
  Py_CLEAR(hs->pick_fn);
  Py_CLEAR(hs->h1_fast_fn);
  Py_CLEAR(hs->row_to_media);
  Py_CLEAR(hs->not_found);
  return 0;
}

void hs_dealloc(HandlersObject* hs) {
  PyObject_GC_UnTrack(hs);
  hs_clear(hs);
  Py_XDECREF(hs->one);
  delete hs->tpl;
  Py_TYPE(hs)->tp_free(reinterpret_cast<PyObject*>(hs));
}

PyObject* hs_new(PyTypeObject* type, PyObject*, PyObject*) {
  HandlersObject* hs = reinterpret_cast<HandlersObject*>(type->tp_alloc(type, 0));
  if (!hs) return nullptr;
  hs->one = PyLong_FromLong(1);
  hs->tpl = new Templates();
  return reinterpret_cast<PyObject*>(hs);
}

// fetch `name` from the module of the handlers' class (beholder_amd.handlers)
PyObject* module_attr(PyObject* h, const char* name) {
  PyObject* modname = PyObject_GetAttrString(reinterpret_cast<PyObject*>(Py_TYPE(h)), "__module__");
  if (!modname) return nullptr;
  PyObject* mod = PyImport_Import(modname);
  Py_DECREF(modname);
  if (!mod) return nullptr;
  PyObject* v = PyObject_GetAttrString(mod, name);
  Py_DECREF(mod);
  return v;
}

// index of each of `names` in the tuple of str `fields`; false if one is missing
bool slots_of(PyObject* fields, const char* const* names, int n, Py_ssize_t* ix) {
  if (!PyTuple_Check(fields)) return false;
  for (int k = 0; k < n; ++k) {
    ix[k] = -1;
    for (Py_ssize_t i = 0; i < PyTuple_GET_SIZE(fields); ++i) {
      PyObject* f = PyTuple_GET_ITEM(fields, i);
      if (PyUnicode_Check(f) && PyUnicode_CompareWithASCIIString(f, names[k]) == 0) {
        ix[k] = i;
        break;
      }
    }
    if (ix[k] < 0) return false;
  }
  return true;
}

// When `decoder` is a native MessageCodec's bound decode, *type = its result type (a struct
// sequence) and ix = the slots of `names`; otherwise *type stays NULL (attribute reads).
bool codec_slots(PyObject* decoder, const char* const* names, int n, PyObject** type, Py_ssize_t* ix) {
  *type = nullptr;
  if (!PyCFunction_Check(decoder)) return true;
  PyObject* self = PyCFunction_GET_SELF(decoder);
  if (!self || Py_TYPE(self) != &CodecType) return true;
  PyObject* fields = PyObject_GetAttrString(self, "field_names");
  PyObject* rt = fields ? PyObject_GetAttrString(self, "result_type") : nullptr;
  if (!rt) {
    Py_XDECREF(fields);
    return false;
  }
  if (slots_of(fields, names, n, ix) && PyType_Check(rt) &&
      PyType_IsSubtype(reinterpret_cast<PyTypeObject*>(rt), &PyTuple_Type)) {
    *type = rt;
  } else {
    Py_DECREF(rt);
  }
  Py_DECREF(fields);
  return true;
}

PyObject* import_attr(const char* module, const char* name) {
  PyObject* mod = PyImport_ImportModule(module);
  if (!mod) return nullptr;
  PyObject* v = PyObject_GetAttrString(mod, name);
  Py_DECREF(mod);
  return v;
}

// TEXTS (beholder_amd/texts.py) -> hs->x / hs->tpl. Shapes are checked: a template with the
// wrong number of holes fails construction instead of rendering wrong text.
int load_texts(HandlersObject* hs) {
  PyObject* table = import_attr("beholder_amd.texts", "TEXTS");
  if (!table) return -1;
  if (!PyDict_Check(table)) {
    Py_DECREF(table);
    PyErr_SetString(PyExc_TypeError, "texts.TEXTS must be a dict");
    return -1;
  }
  for (const TextSpec& sp : kTextSpecs) {
    PyObject* v = PyDict_GetItemString(table, sp.key);
    if (v && sp.item >= 0) v = PyTuple_Check(v) && PyTuple_GET_SIZE(v) > sp.item ? PyTuple_GET_ITEM(v, sp.item) : nullptr;
    if (!v || (sp.is_int ? !PyLong_CheckExact(v) : !PyUnicode_CheckExact(v))) {
      Py_DECREF(table);
      PyErr_Format(PyExc_TypeError, "texts.TEXTS[%s]: missing or of the wrong type", sp.key);
      return -1;
    }
    Py_INCREF(v);
    Py_XSETREF(hs->x[sp.slot], v);
  }
  for (const TplSpec& sp : kTplSpecs) {
    PyObject* v = PyDict_GetItemString(table, sp.key);
    Py_ssize_t n = 0;
    const char* u = v && PyUnicode_CheckExact(v) ? PyUnicode_AsUTF8AndSize(v, &n) : nullptr;
    std::vector<std::string>& out = hs->tpl->t[sp.slot];
    out.clear();
    if (u) {
      std::string str(u, size_t(n));
      size_t at = 0;
      for (size_t h; (h = str.find("{}", at)) != std::string::npos; at = h + 2) out.push_back(str.substr(at, h - at));
      out.push_back(str.substr(at));
    }
    if (!u || int(out.size()) != sp.holes + 1) {
      Py_DECREF(table);
      if (!PyErr_Occurred())
        PyErr_Format(PyExc_ValueError, "texts.TEXTS[%s]: expected a str with %d holes", sp.key, sp.holes);
      return -1;
    }
  }
  Py_DECREF(table);
  return 0;
}

// NativeHandlers(handlers)
int hs_init(HandlersObject* hs, PyObject* args, PyObject* kwds) {
  PyObject* h;
  static const char* kwlist[] = {"handlers", nullptr};
  if (!PyArg_ParseTupleAndKeywords(args, kwds, "O", const_cast<char**>(kwlist), &h)) return -1;
  hs_clear(hs);
  Py_INCREF(h);
  hs->h = h;
  hs->hdict = PyObject_GenericGetDict(h, nullptr);
  if (!hs->hdict) return -1;
  struct {
    PyObject** slot;
    PyObject* name;
  } attrs[] = {{&hs->log, s_log},
               {&hs->decode_s, s_decode_status},
               {&hs->decode_p, s_decode_progress},
               {&hs->names_s, s_status_names_s},
               {&hs->names_p, s_status_names_p},
               {&hs->progress_counter, s_progress_counter},
               {&hs->comment_inc, s_comment_inc},
               {&hs->deployed, s_deployed},
               {&hs->trello_creator, s_trello_creator},
               {&hs->lists, s_lists}};
  for (auto& a : attrs) {
    *a.slot = PyObject_GetAttr(h, a.name);
    if (!*a.slot) return -1;
  }
  if (!PyDict_CheckExact(hs->names_s) || !PyDict_CheckExact(hs->names_p)) {
    PyErr_SetString(PyExc_TypeError, "enum name tables must be dicts");
    return -1;
  }
  PyObject* nt = PyObject_GetAttr(h, s_no_trello);
  if (!nt) return -1;
  int t = PyObject_IsTrue(nt);
  Py_DECREF(nt);
  if (t < 0) return -1;
  hs->no_trello = uint8_t(t);
  hs->native_log = is_native_logger(hs->log) ? 1 : 0;
  hs->progress_plan = PyDict_New();
  hs->get_fn = module_attr(h, "_get");
  hs->err_message = hs->get_fn ? module_attr(h, "err_message") : nullptr;
  hs->js_type_error = hs->err_message ? module_attr(h, "JsTypeError") : nullptr;
  if (!hs->progress_plan || !hs->js_type_error || !hs->one || load_texts(hs) < 0) return -1;
  hs->trello_cls = import_attr("beholder_amd.sinks.trello", "TrelloClient");
  hs->telegram_cls = hs->trello_cls ? import_attr("beholder_amd.sinks.telegram", "TelegramClient") : nullptr;
  hs->emby_cls = hs->telegram_cls ? import_attr("beholder_amd.sinks.emby", "EmbyClient") : nullptr;
  hs->memory_cls = hs->emby_cls ? import_attr("beholder_amd.store.memory", "MemoryStore") : nullptr;
  hs->not_found = hs->memory_cls ? import_attr("beholder_amd.store.base", "MediaNotFound") : nullptr;
  hs->pg_cls = hs->not_found ? import_attr("beholder_amd.store.postgres", "PostgresStore") : nullptr;
  hs->row_to_media = hs->pg_cls ? import_attr("beholder_amd.store.postgres", "row_to_media") : nullptr;
  if (!hs->row_to_media) return -1;
  // the capabilities a Pool (`native_pick`) and an H1Client (`native_call`) hand out are compared
  // with these when a request is issued: the native paths are called directly
  hs->pool_cls = import_attr("beholder_amd.store.pgwire", "Pool");
  hs->pick_fn = hs->pool_cls ? import_attr("beholder_amd.ops._native", "pg_pool_execute") : nullptr;
  hs->h1_fast_fn = hs->pick_fn ? import_attr("beholder_amd.ops._native", "h1_fast") : nullptr;
  if (!hs->h1_fast_fn) return -1;
  if (!hs->not_found) return -1;
  static const char* pnames[4] = {"mediaId", "status", "progress", "host"};
  if (!codec_slots(hs->decode_s, pnames, 2, &hs->res_s, hs->ix_s) ||
      !codec_slots(hs->decode_p, pnames, 4, &hs->res_p, hs->ix_p))
    return -1;
  hs->media_cls = import_attr("beholder_amd.store.base", "Media");
  if (!hs->media_cls) return -1;
  static const char* mnames[3] = {"creator", "creatorId", "status"};
  PyObject* mfields = PyObject_GetAttrString(hs->media_cls, "_fields");
  if (!mfields) return -1;
  bool ok = PyType_Check(hs->media_cls) &&
            PyType_IsSubtype(reinterpret_cast<PyTypeObject*>(hs->media_cls), &PyTuple_Type) &&
            slots_of(mfields, mnames, 3, hs->ix_m);
  Py_DECREF(mfields);
  if (PyErr_Occurred()) return -1;
  if (!ok) Py_CLEAR(hs->media_cls);  // unexpected layout: attribute reads
  return 0;
}

PyMethodDef hs_methods[] = {
    {"on_status", reinterpret_cast<PyCFunction>(hs_on_status), METH_O,
     "on_status(rmsg) -> awaitable: the v1.telemetry.status handler (index.js:62-125)"},
    {"on_progress", reinterpret_cast<PyCFunction>(hs_on_progress), METH_O,
     "on_progress(rmsg) -> awaitable: the v1.telemetry.progress handler (index.js:127-155)"},
    {"stats", reinterpret_cast<PyCFunction>(hs_stats), METH_NOARGS, "calls finished without / after suspending"},
    {nullptr, nullptr, 0, nullptr}};

PyObject* intern(const char* s) { return PyUnicode_InternFromString(s); }

}  // namespace

int init_handler_types(PyObject* m) {
  struct {
    PyObject** slot;
    const char* text;
  } strs[] = {{&s_ack, "ack"},
              {&s_message, "message"},
              {&s_content, "content"},
              {&s_mediaId, "mediaId"},
              {&s_status, "status"},
              {&s_progress, "progress"},
              {&s_host, "host"},
              {&s_creator, "creator"},
              {&s_creatorId, "creatorId"},
              {&s_get_nowait, "_get_nowait"},
              {&s_update_nowait, "_update_nowait"},
              {&s_store, "_store"},
              {&s_get_by_id, "get_by_id"},
              {&s_update_status, "update_status"},
              {&s_trello, "trello"},
              {&s_make_request, "make_request"},
              {&s_post, "post"},
              {&s_put, "put"},
              {&s_deployed_hooks, "_deployed_hooks"},
              {&s_warn_missing_list, "_warn_missing_list"},
              {&s_child_for, "child_for"},
              {&s_inc, "inc"},
              {&s_lower, "lower"},
              {&s_throw, "throw"},
              {&s_close, "close"},
              {&s_lists, "lists"},
              {&s_no_trello, "no_trello"},
              {&s_deployed, "deployed"},
              {&s_trello_creator, "trello_creator"},
              {&s_log, "log"},
              {&s_decode_status, "decode_status"},
              {&s_decode_progress, "decode_progress"},
              {&s_status_names_s, "_status_names_s"},
              {&s_status_names_p, "_status_names_p"},
              {&s_progress_counter, "progress_counter"},
              {&s_comment_inc, "_comment_inc"},
              {&s_key, "key"},
              {&s_token, "token"},
              {&s_base_url, "base_url"},
              {&s_http, "http"},
              {&s_timeout, "timeout"},
              {&s_strict, "strict"},
              {&s_stats, "stats"},
              {&s_request, "request"},
              {&s_native_record, "native_record"},
              {&s_params, "params"},
              {&s_POST, "POST"},
              {&s_PUT, "PUT"},
              {&s_record, "record"},
              {&s_raise_for_status, "raise_for_status"},
              {&s_rows, "_rows"},
              {&s_get_calls, "get_calls"},
              {&s_update_calls, "update_calls"},
              {&s_limiter, "limiter"},
              {&s_hooks_plan, "_hooks_plan"},
              {&s_telegram, "telegram"},
              {&s_emby, "emby"},
              {&s_name, "name"},
              {&s_metadataId, "metadataId"},
              {&s_GET, "GET"},
              {&s_api_key, "api_key"},
              {&s_send_message, "send_message"},
              {&s_refresh_library, "refresh_library"},
              {&s_pool, "_pool"},
              {&s_select, "_select"},
              {&s_update, "_update"},
              {&s_execute, "execute"},
              {&s_conns, "_nets"},
              {&s_spread_at, "spread_at"},
              {&s_size, "size"},
              {&s_native_call, "native_call"}, {&s_native_pick, "native_pick"},
              {&s_retry, "retry"}};

  for (auto& s : strs)
    if (!(*s.slot = intern(s.text))) return -1;
  kw_params_timeout = PyTuple_Pack(2, s_params, s_timeout);
  kw_timeout = PyTuple_Pack(1, s_timeout);
  if (!kw_params_timeout || !kw_timeout) return -1;

  CallType.tp_name = "beholder_amd.ops._native.HandlerCall";
  CallType.tp_basicsize = sizeof(CallObject);
  CallType.tp_flags = Py_TPFLAGS_DEFAULT | Py_TPFLAGS_HAVE_GC;
  CallType.tp_doc = "one native handler invocation: an awaitable iterator (send / throw / close)";
  CallType.tp_dealloc = reinterpret_cast<destructor>(call_dealloc);
  CallType.tp_traverse = reinterpret_cast<traverseproc>(call_traverse);
  CallType.tp_clear = reinterpret_cast<inquiry>(call_clear);
  CallType.tp_as_async = &call_async;
  CallType.tp_iter = PyObject_SelfIter;
  CallType.tp_iternext = reinterpret_cast<iternextfunc>(call_iternext);
  CallType.tp_methods = call_methods;
  CallType.tp_getset = call_getset;
  if (PyType_Ready(&CallType) < 0) return -1;

  HandlersType.tp_name = "beholder_amd.ops._native.NativeHandlers";
  HandlersType.tp_basicsize = sizeof(HandlersObject);
  HandlersType.tp_flags = Py_TPFLAGS_DEFAULT | Py_TPFLAGS_HAVE_GC;
  HandlersType.tp_doc = "NativeHandlers(handlers): the status / progress handlers compiled to native state machines";
  HandlersType.tp_new = hs_new;
  HandlersType.tp_init = reinterpret_cast<initproc>(hs_init);
  HandlersType.tp_dealloc = reinterpret_cast<destructor>(hs_dealloc);
  HandlersType.tp_traverse = reinterpret_cast<traverseproc>(hs_traverse);
  HandlersType.tp_clear = reinterpret_cast<inquiry>(hs_clear);
  HandlersType.tp_methods = hs_methods;
  if (PyType_Ready(&HandlersType) < 0) return -1;
  Py_INCREF(&HandlersType);
  if (PyModule_AddObject(m, "NativeHandlers", reinterpret_cast<PyObject*>(&HandlersType)) < 0) return -1;
  Py_INCREF(&CallType);
  if (PyModule_AddObject(m, "HandlerCall", reinterpret_cast<PyObject*>(&CallType)) < 0) return -1;
  return 0;
}

}  // namespace beholder
