// Event-driven handshake threads (py_netconn.cpp; tests/native/hs_reactor_stress.cpp).
//
// A TLS handshake is a few short bursts of CPU (key share, certificate and signature checks)
// separated by round trips to the peer. The first design ran each handshake start to finish on
// one thread, blocked in poll(2) between its bursts: a thread was held for the whole handshake,
// round trips included, so at most `threads` handshakes made progress at once and the others
// queued behind the slowest peer. Measured on the box, 8 handshakes at start-up on 4 threads:
// the second four waited 1.2-1.6 ms for a thread while the first four mostly waited for their
// peer (profiles/box_r3_warmup/). Against real remote sinks a round trip is tens of ms, so the
// cap mattered more in production than on loopback.
//
// Here the threads share one epoll set and only do the CPU part. Each job's socket sits in the
// set with EPOLLONESHOT: a thread takes a ready job, runs one non-blocking step, and re-arms the
// socket for what the step wants (EPOLLIN / EPOLLOUT) or takes the job out when it is finished.
// ONESHOT hands every readiness to exactly one thread, so one job is never stepped by two threads
// at once, and its `turns` counter orders one step's memory before the next (also for TSan).
//
// Ownership is the same as before (hs_wake.hpp): RUNNING while the reactor has the job; the
// owner of the connection gives it up with exchange(ORPHANED) and shutdown(2) on the socket
// (readiness wakes the job, the step sees ORPHANED, and `finish` frees what the connection no
// longer owns). A job past its deadline is marked expired and its socket shut down the same way;
// the scan runs about once a second (scan_every_s) on whichever thread comes by.
#pragma once

#include <errno.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <mutex>

namespace beholder {

enum HsState : int { HS_RUNNING = 0, HS_DONE = 1, HS_ORPHANED = 2 };

inline double reactor_now() {
  timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return double(t.tv_sec) + double(t.tv_nsec) * 1e-9;
}

struct ReactorJob {
  int fd = -1;
  double deadline = 0;                // CLOCK_MONOTONIC seconds
  std::atomic<int> state{HS_RUNNING};  // RUNNING / DONE / ORPHANED, as above
  std::atomic<bool> expired{false};    // set by the deadline scan, which also shut the socket down
  std::atomic<unsigned> turns{0};      // one acq_rel increment at every hand-over between threads
  int sys_errno = 0;                   // re-arming the socket failed: the job ends with this error
  ReactorJob* prev = nullptr;          // registry of jobs in the reactor (for the deadline scan)
  ReactorJob* next = nullptr;
};

class HsReactor {
 public:
  // step(job): one non-blocking attempt. 0 = finished (the outcome is recorded in the job), or
  // EPOLLIN / EPOLLOUT = step again once the socket is ready for that.
  // finish(job): the job has left the reactor (disarmed, out of the registry); called once.
  using Step = int (*)(ReactorJob*);
  using Finish = void (*)(ReactorJob*);

  HsReactor(Step step, Finish finish, double scan_every_s = 1.0)
      : step_(step), finish_(finish), scan_every_s_(scan_every_s) {
    epfd_ = ::epoll_create1(EPOLL_CLOEXEC);
    stopfd_ = ::eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
    if (epfd_ >= 0 && stopfd_ >= 0) {
      epoll_event ev{};
      ev.events = EPOLLIN;  // level-triggered: once written, every thread sees it
      ev.data.ptr = nullptr;
      if (::epoll_ctl(epfd_, EPOLL_CTL_ADD, stopfd_, &ev) == 0) ok_ = true;
    }
  }
  // Only after stop() has been called and every thread has returned from run().
  ~HsReactor() { close_fds(); }
  HsReactor(const HsReactor&) = delete;
  HsReactor& operator=(const HsReactor&) = delete;

  bool ok() const { return ok_; }

  // Any thread. false: not taken (the caller runs the handshake itself).
  bool submit(ReactorJob* j) {
    if (!ok_) return false;
    {
      std::lock_guard<std::mutex> lock(mu_);
      j->prev = nullptr;
      j->next = head_;
      if (head_) head_->prev = j;
      head_ = j;
    }
    j->turns.fetch_add(1, std::memory_order_acq_rel);
    epoll_event ev{};
    ev.events = EPOLLOUT | EPOLLONESHOT;  // a connected socket is writable: the first step runs at once
    ev.data.ptr = j;
    if (::epoll_ctl(epfd_, EPOLL_CTL_ADD, j->fd, &ev) == 0) return true;
    unlink(j);
    return false;
  }

  // Thread body: returns after stop().
  void run() {
    for (;;) {
      epoll_event ev;
      int n = ::epoll_wait(epfd_, &ev, 1, int(scan_every_s_ * 1000) + 1);
      if (stop_.load(std::memory_order_acquire)) return;
      if (n == 1 && ev.data.ptr) {
        auto* j = static_cast<ReactorJob*>(ev.data.ptr);
        j->turns.fetch_add(1, std::memory_order_acq_rel);
        int want = step_(j);
        if (want && !rearm(j, want)) want = 0;
        if (!want) {
          if (!j->sys_errno) ::epoll_ctl(epfd_, EPOLL_CTL_DEL, j->fd, nullptr);  // (a failed re-arm left it out)
          unlink(j);
          finish_(j);
        }
      } else if (n < 0 && errno != EINTR) {
        timespec pause{0, 1000000};  // not expected (EBADF after a fork): do not spin
        ::nanosleep(&pause, nullptr);
      }
      scan_if_due();
    }
  }

  // Wakes every thread in run() and makes them return. Jobs still in the reactor stay there.
  void stop() {
    stop_.store(true, std::memory_order_release);
    uint64_t one = 1;
    ssize_t w = ::write(stopfd_, &one, sizeof one);
    (void)w;
  }

  // A forked child: the parent's threads do not exist here. Drops the descriptors (the parent's
  // epoll set is shared with the child's copy of the fd) without touching the mutex, which a
  // parent thread may have held at the fork.
  void abandon_after_fork() {
    ok_ = false;
    close_fds();
  }

 private:
  // DEL + ADD rather than MOD: the kernel orders either with the epoll_wait that hands the job
  // to the next thread, but ThreadSanitizer models that only for ADD (its MOD interceptor
  // touches the fd without a release), and would report every later close of the fd as a race.
  // The extra syscall is about a microsecond per step against a few hundred of handshake CPU.
  bool rearm(ReactorJob* j, int want) {
    j->turns.fetch_add(1, std::memory_order_acq_rel);
    epoll_event ev{};
    ev.events = uint32_t(want) | EPOLLONESHOT;
    ev.data.ptr = j;
    ::epoll_ctl(epfd_, EPOLL_CTL_DEL, j->fd, nullptr);
    if (::epoll_ctl(epfd_, EPOLL_CTL_ADD, j->fd, &ev) == 0) return true;
    j->sys_errno = errno;
    return false;
  }

  void unlink(ReactorJob* j) {
    std::lock_guard<std::mutex> lock(mu_);
    if (j->prev) j->prev->next = j->next;
    else head_ = j->next;
    if (j->next) j->next->prev = j->prev;
    j->prev = j->next = nullptr;
  }

  // Marks the jobs past their deadline expired and shuts their sockets down, which wakes them.
  // A job's fd stays open while the job is in the registry (its connection no longer closes it
  // once it is ours, and `finish` runs only after the unlink), so the shutdown never hits a
  // reused descriptor.
  void scan_if_due() {
    double now = reactor_now();
    double due = next_scan_.load(std::memory_order_relaxed);
    if (now < due || !next_scan_.compare_exchange_strong(due, now + scan_every_s_)) return;
    std::lock_guard<std::mutex> lock(mu_);
    for (ReactorJob* j = head_; j; j = j->next) {
      if (j->deadline <= now && !j->expired.exchange(true)) ::shutdown(j->fd, SHUT_RDWR);
    }
  }

  void close_fds() {
    if (epfd_ >= 0) ::close(epfd_);
    if (stopfd_ >= 0) ::close(stopfd_);
    epfd_ = stopfd_ = -1;
  }

  Step step_;
  Finish finish_;
  double scan_every_s_;
  int epfd_ = -1, stopfd_ = -1;
  bool ok_ = false;
  std::atomic<bool> stop_{false};
  std::atomic<double> next_scan_{0.0};
  std::mutex mu_;
  ReactorJob* head_ = nullptr;
};

}  // namespace beholder
