// In-process sampling CPU profiler (native-level), for the per-event cost work on hosts without
// `perf` (neither this build container nor the MI355X boxes have it). Part of `_native_bench`:
// diagnostic code, not linked into the service's extension.
//
// prof_start(hz): ITIMER_PROF fires every 1/hz s of process CPU time; the kernel delivers SIGPROF
// to a thread that is running, whose handler stores the interrupted instruction pointer (and the
// thread id) into a preallocated buffer. prof_stop() disarms the timer and returns the samples as
// (ip, tid) pairs; scripts/cprof.py resolves them against /proc/self/maps and the objects' symbol
// tables (our extension's own symbols, the interpreter's exported ones) into a flat profile.
//
// The handler is async-signal-safe: one atomic increment and two stores into memory allocated
// before the timer is armed. No allocation, no locks, no Python.
//
// prof_start(hz, depth): with depth > 0 each sample also keeps up to `depth` return addresses of
// the interrupted thread (glibc backtrace(), unwinding through the signal frame with the
// objects' .eh_frame tables), so cprof.py can charge a sample to every function on the stack
// (inclusive cost) and name a leaf's callers. backtrace() is called once before the timer is
// armed (it loads the unwinder on first use); it is not formally async-signal-safe, which is
// acceptable for this diagnostic: the samples of one profiling run, never the service.
#include <execinfo.h>
#include <signal.h>
#include <sys/syscall.h>
#include <sys/time.h>
#include <ucontext.h>
#include <unistd.h>

#include <atomic>
#include <cstdint>
#include <cstdlib>

#include "bench_common.hpp"

namespace beholder {
namespace {

constexpr size_t kMaxSamples = 1 << 20;
constexpr int kMaxDepth = 32;
uint64_t* g_ip = nullptr;
uint32_t* g_tid = nullptr;
void** g_stk = nullptr;     // kMaxSamples x g_depth return addresses (depth > 0)
uint8_t* g_stk_n = nullptr;  // frames kept per sample
int g_depth = 0;
std::atomic<size_t> g_n{0};
std::atomic<uint64_t> g_lost{0};
std::atomic<bool> g_active{false};
bool g_armed = false;
bool g_installed = false;

// Installed once and never removed: a SIGPROF generated just before the timer is disarmed can
// still be pending for another thread, and under the default disposition it would end the
// process. While no profile is being taken the handler returns at once.
void on_sigprof(int, siginfo_t*, void* uc_v) {
  if (!g_active.load(std::memory_order_relaxed)) return;
  size_t i = g_n.fetch_add(1, std::memory_order_relaxed);
  if (i >= kMaxSamples) {
    g_lost.fetch_add(1, std::memory_order_relaxed);
    return;
  }
  const ucontext_t* uc = static_cast<const ucontext_t*>(uc_v);
  g_ip[i] = uint64_t(uc->uc_mcontext.gregs[REG_RIP]);
  g_tid[i] = uint32_t(syscall(SYS_gettid));
  if (g_depth) {
    // frames 0-1: this handler and the signal trampoline; then the interrupted function and its callers
    void* buf[kMaxDepth + 2];
    int n = backtrace(buf, g_depth + 2);
    int k = n > 2 ? n - 2 : 0;
    void** dst = g_stk + i * size_t(g_depth);
    for (int j = 0; j < k; ++j) dst[j] = buf[j + 2];
    g_stk_n[i] = uint8_t(k);
  }
}

PyObject* prof_start(PyObject*, PyObject* args) {
  int hz = 997, depth = 0;
  if (!PyArg_ParseTuple(args, "|ii", &hz, &depth)) return nullptr;
  if (depth < 0 || depth > kMaxDepth) {
    PyErr_Format(PyExc_ValueError, "depth must be in [0, %d]", kMaxDepth);
    return nullptr;
  }
  if (g_armed) {
    PyErr_SetString(PyExc_RuntimeError, "profiler already running");
    return nullptr;
  }
  if (hz < 1 || hz > 20000) {
    PyErr_SetString(PyExc_ValueError, "hz must be in [1, 20000]");
    return nullptr;
  }
  if (!g_ip) {
    g_ip = static_cast<uint64_t*>(std::calloc(kMaxSamples, sizeof(uint64_t)));
    g_tid = static_cast<uint32_t*>(std::calloc(kMaxSamples, sizeof(uint32_t)));
    if (!g_ip || !g_tid) {
      std::free(g_ip);
      std::free(g_tid);
      g_ip = nullptr;
      g_tid = nullptr;
      return PyErr_NoMemory();
    }
  }
  if (depth != g_depth || (depth && !g_stk)) {
    std::free(g_stk);
    std::free(g_stk_n);
    g_stk = nullptr;
    g_stk_n = nullptr;
    g_depth = 0;
    if (depth) {
      g_stk = static_cast<void**>(std::calloc(kMaxSamples * size_t(depth), sizeof(void*)));
      g_stk_n = static_cast<uint8_t*>(std::calloc(kMaxSamples, 1));
      if (!g_stk || !g_stk_n) {
        std::free(g_stk);
        std::free(g_stk_n);
        g_stk = nullptr;
        g_stk_n = nullptr;
        return PyErr_NoMemory();
      }
      void* warm[4];
      backtrace(warm, 4);  // loads the unwinder outside the signal handler
    }
    g_depth = depth;
  }
  g_n.store(0);
  g_lost.store(0);
  if (!g_installed) {
    struct sigaction sa = {};
    sa.sa_sigaction = on_sigprof;
    sa.sa_flags = SA_SIGINFO | SA_RESTART;
    sigemptyset(&sa.sa_mask);
    if (sigaction(SIGPROF, &sa, nullptr) < 0) return PyErr_SetFromErrno(PyExc_OSError);
    g_installed = true;
  }
  g_active.store(true);
  struct itimerval it = {};
  it.it_interval.tv_sec = 0;
  it.it_interval.tv_usec = 1000000 / hz;
  it.it_value = it.it_interval;
  if (setitimer(ITIMER_PROF, &it, nullptr) < 0) {
    g_active.store(false);
    return PyErr_SetFromErrno(PyExc_OSError);
  }
  g_armed = true;
  Py_RETURN_NONE;
}

PyObject* prof_stop(PyObject*, PyObject*) {
  if (!g_armed) {
    PyErr_SetString(PyExc_RuntimeError, "profiler not running");
    return nullptr;
  }
  g_active.store(false);
  struct itimerval off = {};
  setitimer(ITIMER_PROF, &off, nullptr);
  g_armed = false;
  size_t n = g_n.load();
  if (n > kMaxSamples) n = kMaxSamples;
  PyObject* ips = PyList_New(Py_ssize_t(n));
  if (!ips) return nullptr;
  for (size_t i = 0; i < n; ++i) {
    PyObject* t;
    if (g_depth) {
      PyObject* fr = PyTuple_New(g_stk_n[i]);
      if (!fr) {
        Py_DECREF(ips);
        return nullptr;
      }
      void** src = g_stk + i * size_t(g_depth);
      for (int j = 0; j < g_stk_n[i]; ++j) {
        PyObject* a = PyLong_FromUnsignedLongLong((unsigned long long)(uintptr_t)src[j]);
        if (!a) {
          Py_DECREF(fr);
          Py_DECREF(ips);
          return nullptr;
        }
        PyTuple_SET_ITEM(fr, j, a);
      }
      t = Py_BuildValue("(KIN)", (unsigned long long)g_ip[i], (unsigned int)g_tid[i], fr);
    } else {
      t = Py_BuildValue("(KI)", (unsigned long long)g_ip[i], (unsigned int)g_tid[i]);
    }
    if (!t) {
      Py_DECREF(ips);
      return nullptr;
    }
    PyList_SET_ITEM(ips, Py_ssize_t(i), t);
  }
  return Py_BuildValue("(NK)", ips, (unsigned long long)g_lost.load());
}

PyMethodDef prof_methods[] = {
    {"prof_start", prof_start, METH_VARARGS,
     "prof_start(hz=997, depth=0): sample instruction pointers (and `depth` return addresses) on SIGPROF"},
    {"prof_stop", prof_stop, METH_NOARGS, "prof_stop() -> ([(ip, tid[, frames]), ...], lost)"},
    {nullptr, nullptr, 0, nullptr}};

}  // namespace

int init_bench_prof(PyObject* m) { return PyModule_AddFunctions(m, prof_methods); }

}  // namespace beholder
