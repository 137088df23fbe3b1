// Completion channel between the TLS handshake threads and one event loop (py_netconn.cpp,
// py_netpoll.cpp).
//
// A handshake thread never takes the GIL: it queues the finished job here and writes the
// eventfd, which sits in the loop's NetPoller epoll set. The poller's `_run` (loop thread, GIL
// held) drains the queue. Taking the GIL from a thread instead would wait for the loop to
// drop it (up to the 5 ms switch interval each time while the loop is busy), and a burst of
// handshakes finishing together would queue their completions behind one another.
#pragma once

#include <sys/eventfd.h>
#include <unistd.h>

#include <cstdint>
#include <deque>
#include <mutex>

namespace beholder {

struct HsWake {
  std::mutex mu;
  std::deque<void*> done;  // finished HsJob* of this loop
  bool closed = false;     // the poller has closed: nothing drains this channel any more
  int efd = -1;

  HsWake() { efd = ::eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC); }
  ~HsWake() {
    if (efd >= 0) ::close(efd);
  }

  // handshake thread. false: the poller has closed, which it does only once every connection
  // has left, so the job's connection is gone (the loop freed its SSL and socket) and the caller
  // frees the job itself. Without this a job posted just after the close would never be drained,
  // and its reference would keep this channel and its eventfd alive for good.
  bool post(void* job) {
    {
      std::lock_guard<std::mutex> lock(mu);
      if (closed) return false;
      done.push_back(job);
    }
    uint64_t one = 1;
    ssize_t n = ::write(efd, &one, sizeof one);
    (void)n;  // EAGAIN only when the counter would overflow: the loop is woken already
    return true;
  }

  // loop thread, the poller closing: refuse later posts, take what is queued
  void close(std::deque<void*>& out) {
    std::lock_guard<std::mutex> lock(mu);
    closed = true;
    out.swap(done);
  }

  // loop thread: take everything finished so far
  void take(std::deque<void*>& out) {
    uint64_t v;
    ssize_t n = ::read(efd, &v, sizeof v);
    (void)n;
    std::lock_guard<std::mutex> lock(mu);
    out.swap(done);
  }
};

}  // namespace beholder
