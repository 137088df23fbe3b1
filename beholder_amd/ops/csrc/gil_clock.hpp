// Per-event timestamps for code that holds the GIL: CLOCK_MONOTONIC (and CLOCK_REALTIME for log
// lines) extrapolated from the TSC between anchors.
//
// The event path reads the clock about five times per event (dispatch start, sink request start
// and end, a log line's `time`, the settle). A vDSO clock_gettime costs 17.7 ns on the MI355X
// box's EPYC 9575F against 7.6 ns for rdtsc (`profiles/box_r5_clock/`), and those reads were
// 9.6% of the headline consumer's CPU (`profiles/box_r5_prof4/headline.txt`).
//
// How: an anchor (tsc, CLOCK_MONOTONIC, CLOCK_REALTIME - CLOCK_MONOTONIC) is re-read every
// kAnchorNs of TSC time. In between, now = anchor + ticks * ns_per_tick, with ns_per_tick measured
// over the first anchor to the latest (so its error shrinks as the process runs, and NTP slewing
// of CLOCK_MONOTONIC, at most 500 ppm, moves a value by at most 500 ppm of kAnchorNs = 125 ns;
// typical slews are 10-50 ppm). Values never go backwards: a re-anchor that reads an earlier
// instant than the last extrapolated value returns that value again. The TSC going backwards or
// jumping (migration, suspend) reads as a huge tick count and re-anchors.
//
// Used only on x86 where the kernel itself uses the TSC (`current_clocksource` is `tsc`: invariant
// and synchronised across CPUs); elsewhere (other architectures included), or with
// BEHOLDER_TSC_CLOCK=0, every read is a clock_gettime. The state is one global guarded by the GIL: threads that run without the GIL (the
// ingest reader, the handshake reactor) keep calling mono_ns() (ring.hpp).
#pragma once

#include <time.h>

#include <cstdint>

#if (defined(__x86_64__) || defined(__i386__)) && !defined(BEHOLDER_NO_TSC)
#include <x86intrin.h>
#define BEHOLDER_HAVE_TSC 1
#else  // no TSC: mode 0 (clock_gettime on every read) is the only mode
#define BEHOLDER_HAVE_TSC 0
#endif

namespace beholder {

inline uint64_t gil_tsc() {
#if BEHOLDER_HAVE_TSC
  return __rdtsc();
#else
  return 0;
#endif
}

struct GilClock {
  int mode = 0;            // 1 = TSC extrapolation, 0 = clock_gettime on every read
  uint64_t tsc0 = 0;       // current anchor
  int64_t mono0 = 0;
  int64_t real_off = 0;    // CLOCK_REALTIME - CLOCK_MONOTONIC at the anchor
  uint64_t base_tsc = 0;   // first anchor: the ns_per_tick baseline
  int64_t base_mono = 0;
  double ns_per_tick = 0;  // 0 until the baseline spans kCalibNs
  uint64_t span = 0;       // ticks between anchors
  int64_t last = 0;        // last value handed out
  uint64_t anchors = 0;    // re-anchors so far (tests, diagnostics)
};

extern GilClock g_gil_clock;

constexpr int64_t kAnchorNs = 250000;  // 250 us between anchors
constexpr int64_t kCalibNs = 1000000;  // the first ns_per_tick needs 1 ms of baseline

void gil_clock_init();                  // module init: picks the mode (gil_clock.cpp)
int64_t gil_clock_anchor(uint64_t tsc);  // the slow path: re-anchor, return CLOCK_MONOTONIC

// CLOCK_MONOTONIC in ns; the caller holds the GIL.
inline int64_t gil_mono_ns() {
  GilClock& c = g_gil_clock;
  if (c.mode == 1) {
    const uint64_t t = gil_tsc();
    const uint64_t d = t - c.tsc0;
    if (d < c.span) {
      int64_t v = c.mono0 + int64_t(double(d) * c.ns_per_tick);
      if (v < c.last) v = c.last;
      c.last = v;
      return v;
    }
    return gil_clock_anchor(t);
  }
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return int64_t(ts.tv_sec) * 1000000000LL + ts.tv_nsec;
}

// CLOCK_REALTIME in ms (a log line's `time`, Date.now()); the caller holds the GIL.
inline long long gil_wall_ms() {
  GilClock& c = g_gil_clock;
  if (c.mode == 1) {
    const int64_t m = gil_mono_ns();
    return (m + c.real_off) / 1000000;
  }
  timespec ts;
  clock_gettime(CLOCK_REALTIME, &ts);
  return (long long)ts.tv_sec * 1000 + ts.tv_nsec / 1000000;
}

}  // namespace beholder
