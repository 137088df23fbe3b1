// The GIL-held clock's mode selection and anchoring (gil_clock.hpp), and its test hooks.
#include "py_common.hpp"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "gil_clock.hpp"

namespace beholder {

GilClock g_gil_clock;

namespace {

constexpr double kBracketNs = 100;  // a clean rdtsc / clock_gettime / rdtsc bracket is ~30-60 ns

bool kernel_uses_tsc() {
  FILE* f = fopen("/sys/devices/system/clocksource/clocksource0/current_clocksource", "r");
  if (!f) return false;
  char buf[32] = {0};
  const bool got = fgets(buf, sizeof buf, f) != nullptr;
  fclose(f);
  return got && strncmp(buf, "tsc", 3) == 0 && (buf[3] == '\n' || buf[3] == 0);
}

}  // namespace

void gil_clock_init() {
  GilClock& c = g_gil_clock;
  c = GilClock();
  const char* env = getenv("BEHOLDER_TSC_CLOCK");
  if (env && env[0] == '0') return;
  c.mode = BEHOLDER_HAVE_TSC && kernel_uses_tsc() ? 1 : 0;
}

int64_t gil_clock_anchor(uint64_t) {
  GilClock& c = g_gil_clock;
  // the TSC read on both sides of the CLOCK_MONOTONIC read, their midpoint paired with it; a pair
  // taken across an interrupt or a preemption (a wide bracket) is read again, up to 4 times
  timespec m = {0, 0}, r;
  uint64_t t = 0, width = ~uint64_t(0);
  for (int i = 0; i < 4; ++i) {
    timespec mi;
    const uint64_t a = gil_tsc();
    clock_gettime(CLOCK_MONOTONIC, &mi);
    const uint64_t b = gil_tsc();
    if (b - a < width) {
      width = b - a;
      t = a + (b - a) / 2;
      m = mi;
    }
    if (c.ns_per_tick > 0 ? double(width) * c.ns_per_tick < kBracketNs : i > 0) break;
  }
  clock_gettime(CLOCK_REALTIME, &r);
  int64_t mono = int64_t(m.tv_sec) * 1000000000LL + m.tv_nsec;
  const int64_t real = int64_t(r.tv_sec) * 1000000000LL + r.tv_nsec;
  ++c.anchors;
  if (!c.base_tsc || t <= c.base_tsc || mono <= c.base_mono) {
    c.base_tsc = t;
    c.base_mono = mono;
    c.ns_per_tick = 0;
  } else if (mono - c.base_mono >= kCalibNs) {
    const double rate = double(mono - c.base_mono) / double(t - c.base_tsc);
    if (c.ns_per_tick != 0 && std::fabs(rate / c.ns_per_tick - 1.0) > 1e-3) {
      // the TSC jumped against CLOCK_MONOTONIC (a migrated VM, a suspend): start a new baseline
      c.base_tsc = t;
      c.base_mono = mono;
      c.ns_per_tick = 0;
    } else {
      c.ns_per_tick = rate;
    }
  }
  // uncalibrated: span 0, so every read comes back here and reads the clock
  c.span = c.ns_per_tick > 0 ? uint64_t(double(kAnchorNs) / c.ns_per_tick) : 0;
  c.tsc0 = t;
  c.mono0 = mono;
  c.real_off = real - mono;
  if (mono < c.last) mono = c.last;
  c.last = mono;
  return mono;
}

namespace {

// gil_clock() -> (CLOCK_MONOTONIC ns, CLOCK_REALTIME ms) as the event path reads them
PyObject* mod_gil_clock(PyObject*, PyObject*) {
  const long long mono = gil_mono_ns();
  const long long wall = gil_wall_ms();
  return Py_BuildValue("(LL)", mono, wall);
}

// gil_clock_info() -> {"mode": "tsc" | "clock_gettime", "ns_per_tick", "anchors"}
PyObject* mod_gil_clock_info(PyObject*, PyObject*) {
  const GilClock& c = g_gil_clock;
  return Py_BuildValue("{s:s,s:d,s:K}", "mode", c.mode == 1 ? "tsc" : "clock_gettime", "ns_per_tick",
                       c.ns_per_tick, "anchors", static_cast<unsigned long long>(c.anchors));
}

// gil_clock_reset(): re-reads BEHOLDER_TSC_CLOCK and the clocksource (tests)
PyObject* mod_gil_clock_reset(PyObject*, PyObject*) {
  gil_clock_init();
  Py_RETURN_NONE;
}

PyMethodDef clock_methods[] = {
    {"gil_clock", mod_gil_clock, METH_NOARGS,
     "gil_clock() -> (monotonic ns, realtime ms) as the event path reads them (TSC-extrapolated)"},
    {"gil_clock_info", mod_gil_clock_info, METH_NOARGS, "gil_clock_info() -> {mode, ns_per_tick, anchors}"},
    {"gil_clock_reset", mod_gil_clock_reset, METH_NOARGS, "re-read BEHOLDER_TSC_CLOCK and the kernel clocksource"},
    {nullptr, nullptr, 0, nullptr}};

}  // namespace

int init_clock_functions(PyObject* m) {
  gil_clock_init();
  return PyModule_AddFunctions(m, clock_methods);
}

}  // namespace beholder
