// The paced producer of BASELINE configs 2-4 (bench/harness.py _Producer).
#include <errno.h>
#include <poll.h>
#include <sys/prctl.h>
#include <time.h>
#include <unistd.h>

#include "bench_common.hpp"

namespace beholder {
namespace bench {
namespace {

// paced_write(fd, data, ends, rate) -> (elapsed_s, writes, t0_ns)
//
// Writes the frames of `data` (frame i ends at byte ends[i], native-endian
// u64 array) to `fd` at `rate` frames/s: frame i is written no earlier than
// t0 + i/rate, every frame already due goes out in one write(2). The whole
// call runs without the GIL and sleeps with clock_nanosleep(TIMER_ABSTIME) and
// 1 ns timer slack, so a bench producer neither competes with the consumer's
// event loop for the GIL nor wakes late by the default 50 us slack
// (BASELINE configs 2-4: 1k / 10k / 100k events/s). Used by bench/harness.py.
// t0_ns (CLOCK_MONOTONIC, the clock of every Delivery timestamp) is when frame 0
// was due, so the caller can measure each event from its due time to its ack.

bool write_all(int fd, const uint8_t* p, size_t n) {
  while (n) {
    ssize_t w = write(fd, p, n);
    if (w < 0) {
      if (errno == EINTR) continue;
      if (errno == EAGAIN) {
        struct pollfd pfd = {fd, POLLOUT, 0};
        poll(&pfd, 1, 100);
        continue;
      }
      return false;
    }
    p += w;
    n -= size_t(w);
  }
  return true;
}

PyObject* mod_paced_write(PyObject*, PyObject* args) {
  int fd;
  Py_buffer data, ends;
  double rate;
  if (!PyArg_ParseTuple(args, "iy*y*d", &fd, &data, &ends, &rate)) return nullptr;
  size_t n = size_t(ends.len) / sizeof(uint64_t);
  const uint64_t* endv = static_cast<const uint64_t*>(ends.buf);
  const uint8_t* base = static_cast<const uint8_t*>(data.buf);
  bool bad = rate <= 0 || ends.len % sizeof(uint64_t) != 0;
  for (size_t i = 0; !bad && i < n; ++i)
    bad = endv[i] > uint64_t(data.len) || (i && endv[i] < endv[i - 1]);
  if (bad) {
    PyBuffer_Release(&data);
    PyBuffer_Release(&ends);
    PyErr_SetString(PyExc_ValueError, "paced_write: rate must be > 0 and ends a non-decreasing u64 array within data");
    return nullptr;
  }
  int64_t t0 = 0, t1 = 0;
  uint64_t writes = 0;
  bool ok = true;
  int err = 0;
  Py_BEGIN_ALLOW_THREADS
  int old_slack = prctl(PR_GET_TIMERSLACK, 0, 0, 0, 0);
  prctl(PR_SET_TIMERSLACK, 1, 0, 0, 0);
  const double ns_per = 1e9 / rate;
  t0 = mono_ns();
  size_t sent = 0;
  while (sent < n) {
    int64_t now = mono_ns();
    size_t due = size_t(double(now - t0) / ns_per) + 1;
    if (due > n) due = n;
    if (due > sent) {
      uint64_t from = sent ? endv[sent - 1] : 0;
      if (!write_all(fd, base + from, size_t(endv[due - 1] - from))) {
        ok = false;
        err = errno;
        break;
      }
      ++writes;
      sent = due;
    } else {
      int64_t at = t0 + int64_t(double(sent) * ns_per);
      struct timespec ts = {time_t(at / 1000000000LL), long(at % 1000000000LL)};
      while (clock_nanosleep(CLOCK_MONOTONIC, TIMER_ABSTIME, &ts, nullptr) == EINTR) {
      }
    }
  }
  t1 = mono_ns();
  if (old_slack > 0) prctl(PR_SET_TIMERSLACK, old_slack, 0, 0, 0);
  Py_END_ALLOW_THREADS
  PyBuffer_Release(&data);
  PyBuffer_Release(&ends);
  if (!ok) {
    errno = err;
    return PyErr_SetFromErrno(PyExc_OSError);
  }
  return Py_BuildValue("(dKL)", double(t1 - t0) / 1e9, (unsigned long long)writes, (long long)t0);
}

PyMethodDef pace_methods[] = {
    {"paced_write", mod_paced_write, METH_VARARGS,
     "paced_write(fd, data, ends_u64, rate) -> (elapsed_s, writes, t0_ns): GIL-free paced frame writer; "
     "frame i is due at t0_ns + i * 1e9 / rate"},
    {nullptr, nullptr, 0, nullptr}};


}  // namespace

int init_paced(PyObject* m) { return PyModule_AddFunctions(m, pace_methods); }

}  // namespace bench
}  // namespace beholder
