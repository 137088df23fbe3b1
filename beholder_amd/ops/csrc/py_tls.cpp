// TlsContext: the client-side OpenSSL context of the native HTTPS path.
//
// The production sinks are HTTPS (api.trello.com, api.telegram.org; index.js:53,83,99). With
// asyncio's SSL transport every request and reply also crosses asyncio's pure-Python
// SSLProtocol (memory BIOs, several Python frames per record), which costs more CPU than the
// whole plain-TCP request path. A TLS NetConn (py_netconn.cpp) runs the handshake and the
// record layer on the socket with OpenSSL directly.
//
// The context mirrors what `ssl.create_default_context(cafile=...)` sets up for a client:
// TLS 1.2 minimum, peer verification against `cafile` / `capath` or OpenSSL's default
// verify paths (which honour SSL_CERT_FILE / SSL_CERT_DIR like Python's), the same cipher
// string, no compression, hostname (or IP address) checked against the certificate, SNI sent
// for names (not for IP literals). Only H1Client's own contexts (default or built from its
// `ssl_cafile`) are mirrored: a caller-supplied ssl.SSLContext keeps the asyncio TLS path.
//
// Client sessions are cached per "host:port" (the last ticket each origin gave us), so a
// reconnect after the server closed an idle keep-alive connection resumes instead of running
// a full handshake. A TLS 1.3 ticket is used once (RFC 8446 C.4); the resumed connection's
// own tickets take its place.
#include <arpa/inet.h>
#include <openssl/err.h>
#include <openssl/evp.h>
#include <openssl/ssl.h>
#include <openssl/x509v3.h>

#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>

#include "py_common.hpp"

namespace beholder {

namespace {

// Python 3.10's default cipher string for ssl.create_default_context (Lib/ssl.py / _ssl.c)
constexpr const char* kCiphers = "@SECLEVEL=2:ECDH+AESGCM:ECDH+CHACHA20:ECDH+AES:DHE+AES:!aNULL:!eNULL:!aDSS:!SHA1:!AESCCM";

// The per-origin session cache. Shared with the handshake threads (py_netconn.cpp): a TLS 1.2
// session is stored by the new-session callback inside SSL_do_handshake, which may run on one
// of them. Every SSL holds a reference (SslTag), so the cache outlives the TlsContext while a
// handshake thread still works on an SSL of a connection closed meanwhile.
struct SessionStore {
  std::mutex mu;
  std::map<std::string, std::deque<SSL_SESSION*>> sessions;  // "host:port" -> newest sessions (one ref each)

  void clear() {
    for (auto& kv : sessions)
      for (SSL_SESSION* x : kv.second) SSL_SESSION_free(x);
    sessions.clear();
  }
  ~SessionStore() { clear(); }
};

// SSL ex_data (g_key_index): the session-cache key of the SSL's origin and the cache itself
struct SslTag {
  std::string key;
  std::shared_ptr<SessionStore> store;
};

struct TlsContextObject {
  PyObject_HEAD SSL_CTX* ctx;
  std::shared_ptr<SessionStore>* store;
  uint64_t handshakes, resumed, offloaded;
  bool check_hostname;  // the certificate must name the host (verify-full / HTTPS)
};

PyTypeObject TlsContextType = {PyVarObject_HEAD_INIT(nullptr, 0)};
int g_ex_index = -1;  // SSL ex_data: the TlsContextObject* of an SSL (loop thread only: counts)
int g_key_index = -1;  // SSL ex_data: SslTag*

std::string last_error_text() {
  unsigned long e = ERR_peek_last_error();
  char buf[256];
  ERR_error_string_n(e, buf, sizeof buf);
  return buf;
}

constexpr size_t kTicketsPerOrigin = 16;  // enough for a burst of reconnects to resume

// new-session callback: keep the newest sessions of each origin (TLS 1.3 tickets arrive after
// the handshake, in the first reads; servers usually send two)
int on_new_session(SSL* ssl, SSL_SESSION* sess) {
  auto* tag = static_cast<SslTag*>(SSL_get_ex_data(ssl, g_key_index));
  if (!tag || !tag->store) return 0;
  SessionStore& st = *tag->store;
  std::lock_guard<std::mutex> lock(st.mu);
  auto it = st.sessions.find(tag->key);
  if (it == st.sessions.end()) {
    if (st.sessions.size() >= 1024) st.clear();  // bounded: rebuilt on demand
    it = st.sessions.emplace(tag->key, std::deque<SSL_SESSION*>()).first;
  }
  it->second.push_back(sess);
  if (it->second.size() > kTicketsPerOrigin) {
    SSL_SESSION_free(it->second.front());
    it->second.pop_front();
  }
  return 1;  // we hold the reference
}

// ex_data free callback: SSL_free (on whichever thread) drops the tag and its cache reference
void free_tag(void*, void* ptr, CRYPTO_EX_DATA*, int, long, void*) { delete static_cast<SslTag*>(ptr); }

}  // namespace

void hs_prestart();

// One TLS 1.3 handshake between two in-memory endpoints. OpenSSL 3 looks up and caches each
// algorithm implementation (key exchange, ECDSA, HKDF, AES-GCM, certificate decoding) the first
// time a handshake needs it, and builds per-thread state (random generators) on a thread's
// first use. Run once on the loop thread when the first TlsContext is made (service startup)
// and once on each handshake thread as it starts (py_netconn.cpp hs_worker); without it the
// first burst of sink connects paid 0.6-1.35 ms of client CPU per handshake against 0.15-0.4
// ms later (box). The certificate is a throwaway P-256 one made here. RSA, which the real
// sinks' chains may use, gets its lookups warmed without a key (making a 2048-bit key would
// cost more than it saves). Best effort: false only means a colder first handshake.
bool tls_warm_handshake() {
  bool finished = false;
  {
    EVP_PKEY* key = EVP_EC_gen("P-256");
    X509* cert = key ? X509_new() : nullptr;
    SSL_CTX* sctx = cert ? SSL_CTX_new(TLS_server_method()) : nullptr;
    SSL_CTX* cctx = sctx ? SSL_CTX_new(TLS_client_method()) : nullptr;
    SSL *cli = nullptr, *srv = nullptr;
    BIO *bc = nullptr, *bs = nullptr;
    bool ok = cctx != nullptr;
    if (ok) {
      X509_set_version(cert, 2);
      ASN1_INTEGER_set(X509_get_serialNumber(cert), 1);
      X509_gmtime_adj(X509_getm_notBefore(cert), -60);
      X509_gmtime_adj(X509_getm_notAfter(cert), 3600);
      X509_set_pubkey(cert, key);
      X509_NAME* name = X509_get_subject_name(cert);
      X509_NAME_add_entry_by_txt(name, "CN", MBSTRING_ASC, reinterpret_cast<const unsigned char*>("warm-up.invalid"),
                                 -1, -1, 0);
      X509_set_issuer_name(cert, name);
      ok = X509_sign(cert, key, EVP_sha256()) > 0 && SSL_CTX_use_certificate(sctx, cert) == 1 &&
           SSL_CTX_use_PrivateKey(sctx, key) == 1 && X509_STORE_add_cert(SSL_CTX_get_cert_store(cctx), cert) == 1 &&
           SSL_CTX_set_cipher_list(cctx, kCiphers) == 1 && BIO_new_bio_pair(&bc, 0, &bs, 0) == 1;
    }
    if (ok) {
      SSL_CTX_set_verify(cctx, SSL_VERIFY_PEER, nullptr);
      cli = SSL_new(cctx);
      srv = SSL_new(sctx);
      ok = cli && srv && SSL_set1_host(cli, "warm-up.invalid") == 1;
    }
    if (ok) {
      SSL_set_bio(cli, bc, bc);  // each SSL owns its end of the pair
      SSL_set_bio(srv, bs, bs);
      bc = bs = nullptr;
      SSL_set_connect_state(cli);
      SSL_set_accept_state(srv);
      bool cdone = false, sdone = false;
      for (int i = 0; i < 16 && !(cdone && sdone); ++i) {
        if (!cdone) cdone = SSL_do_handshake(cli) == 1;
        if (!sdone) sdone = SSL_do_handshake(srv) == 1;
      }
      char b = 'x';
      finished = cdone && sdone && SSL_write(cli, &b, 1) == 1 && SSL_read(srv, &b, 1) == 1;  // one AEAD record
    }
    SSL_free(cli);
    SSL_free(srv);
    BIO_free(bc);
    BIO_free(bs);
    SSL_CTX_free(cctx);
    SSL_CTX_free(sctx);
    X509_free(cert);
    EVP_PKEY_free(key);
  }
  ERR_clear_error();
  return finished;
}

namespace {

void warm_up_once() {
  static std::once_flag once;
  std::call_once(once, [] {
    for (const char* alg : {"RSA", "RSA-PSS", "EC", "X25519"}) EVP_KEYMGMT_free(EVP_KEYMGMT_fetch(nullptr, alg, nullptr));
    for (const char* alg : {"RSA", "ECDSA"}) EVP_SIGNATURE_free(EVP_SIGNATURE_fetch(nullptr, alg, nullptr));
    tls_warm_handshake();
  });
}

PyObject* tc_new(PyTypeObject* type, PyObject* args, PyObject* kwds) {
  static const char* kwlist[] = {"cafile", "capath", "verify", "check_hostname", nullptr};
  const char* cafile = nullptr;
  const char* capath = nullptr;
  int verify = 1, check_hostname = 1;
  if (!PyArg_ParseTupleAndKeywords(args, kwds, "|zzpp", const_cast<char**>(kwlist), &cafile, &capath, &verify,
                                   &check_hostname))
    return nullptr;
  TlsContextObject* s = reinterpret_cast<TlsContextObject*>(type->tp_alloc(type, 0));
  if (!s) return nullptr;
  s->ctx = nullptr;
  s->check_hostname = verify && check_hostname;
  try {
    s->store = new std::shared_ptr<SessionStore>(std::make_shared<SessionStore>());
  } catch (const std::bad_alloc&) {
    s->store = nullptr;
  }
  if (!s->store) {
    Py_DECREF(s);
    return PyErr_NoMemory();
  }
  warm_up_once();
  ERR_clear_error();
  SSL_CTX* ctx = SSL_CTX_new(TLS_client_method());
  if (!ctx) {
    Py_DECREF(s);
    PyErr_Format(PyExc_RuntimeError, "SSL_CTX_new: %s", last_error_text().c_str());
    return nullptr;
  }
  s->ctx = ctx;
  SSL_CTX_set_min_proto_version(ctx, TLS1_2_VERSION);
  SSL_CTX_set_options(ctx, SSL_OP_NO_COMPRESSION);
  SSL_CTX_set_mode(ctx, SSL_MODE_ENABLE_PARTIAL_WRITE | SSL_MODE_ACCEPT_MOVING_WRITE_BUFFER);
  SSL_CTX_set_read_ahead(ctx, 1);  // one recv(2) takes every record the kernel holds, not header + body
  if (SSL_CTX_set_cipher_list(ctx, kCiphers) != 1) {
    Py_DECREF(s);
    PyErr_Format(PyExc_RuntimeError, "SSL_CTX_set_cipher_list: %s", last_error_text().c_str());
    return nullptr;
  }
  if (verify) {
    SSL_CTX_set_verify(ctx, SSL_VERIFY_PEER, nullptr);
    int ok = (cafile || capath) ? SSL_CTX_load_verify_locations(ctx, cafile, capath)
                                : SSL_CTX_set_default_verify_paths(ctx);
    if (ok != 1) {
      Py_DECREF(s);
      PyErr_Format(PyExc_FileNotFoundError, "cannot load verify locations (%s): %s", cafile ? cafile : "default",
                   last_error_text().c_str());
      return nullptr;
    }
  } else {
    SSL_CTX_set_verify(ctx, SSL_VERIFY_NONE, nullptr);
  }
  SSL_CTX_set_session_cache_mode(ctx, SSL_SESS_CACHE_CLIENT | SSL_SESS_CACHE_NO_INTERNAL_STORE);
  SSL_CTX_sess_set_new_cb(ctx, on_new_session);
  hs_prestart();  // the handshake threads start (and warm up) now, not in the first burst
  return reinterpret_cast<PyObject*>(s);
}

void tc_dealloc(TlsContextObject* s) {
  delete s->store;  // the cache itself goes with the last SSL that still refers to it
  if (s->ctx) SSL_CTX_free(s->ctx);
  Py_TYPE(s)->tp_free(reinterpret_cast<PyObject*>(s));
}

PyObject* tc_get_stats(TlsContextObject* s, void*) {
  Py_ssize_t n = 0;
  {
    SessionStore& st = **s->store;
    std::lock_guard<std::mutex> lock(st.mu);
    for (auto& kv : st.sessions) n += Py_ssize_t(kv.second.size());
  }
  return Py_BuildValue("{s:K,s:K,s:n,s:K}", "handshakes", static_cast<unsigned long long>(s->handshakes), "resumed",
                       static_cast<unsigned long long>(s->resumed), "cached_sessions", n, "offloaded",
                       static_cast<unsigned long long>(s->offloaded));
}

PyGetSetDef tc_getset[] = {
    {"stats", reinterpret_cast<getter>(tc_get_stats), nullptr,
     "handshakes, resumed, cached_sessions, offloaded (handshakes run on a handshake thread)", nullptr},
    {nullptr, nullptr, nullptr, nullptr, nullptr}};

}  // namespace

bool is_tls_context(PyObject* o) { return Py_TYPE(o) == &TlsContextType; }

// A client SSL on connected socket `fd` for `host` (a name or an IP literal) and `port`:
// verification target, SNI, a cached session of that origin. NULL with a Python error set.
SSL* tls_new_ssl(PyObject* ctx_obj, int fd, const char* host, int port) {
  TlsContextObject* tc = reinterpret_cast<TlsContextObject*>(ctx_obj);
  ERR_clear_error();
  SSL* ssl = SSL_new(tc->ctx);
  if (!ssl) {
    PyErr_Format(PyExc_RuntimeError, "SSL_new: %s", last_error_text().c_str());
    return nullptr;
  }
  unsigned char addr[16];
  bool is_ip = inet_pton(AF_INET, host, addr) == 1 || inet_pton(AF_INET6, host, addr) == 1;
  bool ok = SSL_set_fd(ssl, fd) == 1;
  if (ok && !is_ip) ok = SSL_set_tlsext_host_name(ssl, host) == 1;  // SNI for names only
  if (ok && tc->check_hostname)
    ok = is_ip ? X509_VERIFY_PARAM_set1_ip_asc(SSL_get0_param(ssl), host) == 1 : SSL_set1_host(ssl, host) == 1;
  SslTag* tag = ok ? new (std::nothrow) SslTag{std::string(host) + ":" + std::to_string(port), *tc->store} : nullptr;
  if (!tag || SSL_set_ex_data(ssl, g_ex_index, tc) != 1 || SSL_set_ex_data(ssl, g_key_index, tag) != 1) {
    if (tag && SSL_get_ex_data(ssl, g_key_index) != tag) delete tag;
    SSL_free(ssl);
    PyErr_Format(PyExc_RuntimeError, "TLS setup for %s: %s", host, last_error_text().c_str());
    return nullptr;
  }
  {
    SessionStore& st = **tc->store;
    std::lock_guard<std::mutex> lock(st.mu);
    auto it = st.sessions.find(tag->key);
    if (it != st.sessions.end() && !it->second.empty()) {
      SSL_SESSION* sess = it->second.back();
      SSL_set_session(ssl, sess);  // the SSL holds its own reference
      if (SSL_SESSION_get_protocol_version(sess) == TLS1_3_VERSION) {
        // TLS 1.3 tickets are single use (RFC 8446 C.4): the resumed connection brings new ones
        SSL_SESSION_free(sess);
        it->second.pop_back();
      }
    }
  }
  SSL_set_connect_state(ssl);
  return ssl;
}

// Handshake finished on `ssl`: count it (resumed or full; run on a handshake thread). Called on
// the loop thread.
void tls_count_handshake(SSL* ssl, bool offloaded) {
  auto* tc = static_cast<TlsContextObject*>(SSL_get_ex_data(ssl, g_ex_index));
  if (!tc) return;
  ++tc->handshakes;
  if (SSL_session_reused(ssl)) ++tc->resumed;
  if (offloaded) ++tc->offloaded;
}

// Description of a failed handshake, Python-ssl style: reason ("CERTIFICATE_VERIFY_FAILED",
// "WRONG_VERSION_NUMBER", ...), message ("[SSL: REASON] text"), verify = certificate problem.
void tls_describe_failure(SSL* ssl, std::string& reason, std::string& message, bool& verify) {
  long vr = SSL_get_verify_result(ssl);
  verify = vr != X509_V_OK;
  if (verify) {
    reason = "CERTIFICATE_VERIFY_FAILED";
    message = std::string("[SSL: CERTIFICATE_VERIFY_FAILED] certificate verify failed: ") +
              X509_verify_cert_error_string(vr);
    return;
  }
  unsigned long e = ERR_peek_last_error();
  const char* r = e ? ERR_reason_error_string(e) : nullptr;
  std::string text = r ? r : "unexpected eof while reading";
  reason.clear();
  for (char ch : text) reason += ch == ' ' ? '_' : char(ch >= 'a' && ch <= 'z' ? ch - 32 : ch);
  message = "[SSL: " + reason + "] " + text;
}

int init_tls_types(PyObject* m) {
  g_ex_index = SSL_get_ex_new_index(0, nullptr, nullptr, nullptr, nullptr);
  g_key_index = SSL_get_ex_new_index(0, nullptr, nullptr, nullptr, free_tag);
  if (g_ex_index < 0 || g_key_index < 0) {
    PyErr_SetString(PyExc_RuntimeError, "SSL_get_ex_new_index failed");
    return -1;
  }
  TlsContextType.tp_name = "beholder_amd.ops._native.TlsContext";
  TlsContextType.tp_basicsize = sizeof(TlsContextObject);
  TlsContextType.tp_flags = Py_TPFLAGS_DEFAULT;
  TlsContextType.tp_doc =
      "TlsContext(cafile=None, capath=None, verify=True, check_hostname=True): OpenSSL client context for TLS "
      "NetConns (ssl.create_default_context semantics; verify=False = libpq sslmode require/prefer, "
      "check_hostname=False = verify-ca)";
  TlsContextType.tp_new = tc_new;
  TlsContextType.tp_dealloc = reinterpret_cast<destructor>(tc_dealloc);
  TlsContextType.tp_getset = tc_getset;
  if (PyType_Ready(&TlsContextType) < 0) return -1;
  Py_INCREF(&TlsContextType);
  return PyModule_AddObject(m, "TlsContext", reinterpret_cast<PyObject*>(&TlsContextType));
}

}  // namespace beholder
