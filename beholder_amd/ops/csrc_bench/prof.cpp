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
uint64_t* g_ip = nullptr;
uint32_t* g_tid = nullptr;
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
}

PyObject* prof_start(PyObject*, PyObject* args) {
  int hz = 997;
  if (!PyArg_ParseTuple(args, "|i", &hz)) return nullptr;
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
    PyObject* t = Py_BuildValue("(KI)", (unsigned long long)g_ip[i], (unsigned int)g_tid[i]);
    if (!t) {
      Py_DECREF(ips);
      return nullptr;
    }
    PyList_SET_ITEM(ips, Py_ssize_t(i), t);
  }
  return Py_BuildValue("(NK)", ips, (unsigned long long)g_lost.load());
}

PyMethodDef prof_methods[] = {
    {"prof_start", prof_start, METH_VARARGS, "prof_start(hz=997): sample instruction pointers on SIGPROF"},
    {"prof_stop", prof_stop, METH_NOARGS, "prof_stop() -> ([(ip, tid), ...], lost)"},
    {nullptr, nullptr, 0, nullptr}};

}  // namespace

int init_bench_prof(PyObject* m) { return PyModule_AddFunctions(m, prof_methods); }

}  // namespace beholder
