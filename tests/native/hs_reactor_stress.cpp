// Stress test of the handshake reactor (beholder_amd/ops/csrc/hs_reactor.hpp) under
// ThreadSanitizer / ASan, with the job ownership protocol of py_netconn.cpp around it and real
// sockets (socketpairs) in place of TLS connections.
//
//   a job's "handshake": write a hello to its socket, then read `need` bytes that the loop
//     thread sends one at a time (each byte is one readiness, often stepped by another thread);
//   loop thread: sends bytes, drains finished jobs from the completion channel (hs_wake.hpp),
//     "closes connections" at random (shutdown(2), then exchange ORPHANED: a RUNNING job is
//     then the reactor's to free; a DONE one is marked connection-less, the drain frees it),
//     leaves some jobs starved so that the deadline scan expires them, and at the end of each
//     round closes everything and the channel.
//
// Every job must be freed exactly once, every orphaned or expired job must be woken (else the
// final wait times out), and the sanitizers must see no race or leak.
#include <fcntl.h>
#include <sys/socket.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <deque>
#include <memory>
#include <random>
#include <thread>
#include <vector>

#include "hs_reactor.hpp"
#include "hs_wake.hpp"

using beholder::HS_DONE;
using beholder::HS_ORPHANED;
using beholder::HS_RUNNING;
using beholder::HsReactor;
using beholder::HsWake;
using beholder::ReactorJob;

enum Result { RES_OK, RES_EOF, RES_TIMEOUT, RES_NONE };

std::atomic<long> created{0}, freed{0}, oks{0}, timeouts{0}, eofs{0}, freed_by_reactor{0};

struct Job : ReactorJob {
  std::shared_ptr<HsWake> wake;
  int need = 1, got = 0;
  bool hello = false;
  int result = RES_NONE;
  std::atomic<bool> conn{true};  // the loop still has the connection (and closes the fd itself)
  Job() { created.fetch_add(1); }
  ~Job() { freed.fetch_add(1); }
};

int step(ReactorJob* rj) {
  Job* j = static_cast<Job*>(rj);
  if (j->state.load() == HS_ORPHANED) return 0;
  if (j->expired.load()) {
    j->result = RES_TIMEOUT;
    return 0;
  }
  if (!j->hello) {
    char h = 'h';
    if (::send(j->fd, &h, 1, MSG_NOSIGNAL) != 1) return errno == EAGAIN ? EPOLLOUT : (j->result = RES_EOF, 0);
    j->hello = true;
    return EPOLLIN;
  }
  char b;
  ssize_t n = ::recv(j->fd, &b, 1, 0);
  if (n == 1) {
    if (++j->got == j->need) {
      j->result = j->expired.load() ? RES_TIMEOUT : RES_OK;
      return 0;
    }
    return EPOLLIN;
  }
  if (n < 0 && errno == EAGAIN) return EPOLLIN;
  j->result = j->expired.load() ? RES_TIMEOUT : RES_EOF;
  return 0;
}

void finish(ReactorJob* rj) {
  Job* j = static_cast<Job*>(rj);
  if (j->sys_errno) j->result = RES_EOF;
  std::shared_ptr<HsWake> wake = j->wake;
  if (j->state.exchange(HS_DONE) == HS_ORPHANED) {
    ::close(j->fd);
    freed_by_reactor.fetch_add(1);
    delete j;
    return;
  }
  if (!wake->post(j)) delete j;  // the channel closed: the connection is gone, so is its fd
}

struct Conn {  // the loop's side of one job
  Job* job;
  int peer;
  int sent;
};

int main() {
  const int kRounds = 60, kJobs = 120, kThreads = 4;
  HsReactor reactor(step, finish, 0.01);
  if (!reactor.ok()) {
    std::perror("reactor");
    return 1;
  }
  std::vector<std::thread> ts;
  for (int i = 0; i < kThreads; ++i) ts.emplace_back([&reactor] { reactor.run(); });
  std::mt19937 rng(4242);
  auto drain = [](std::deque<void*>& done, std::vector<Conn>& live) {
    for (void* p : done) {
      Job* d = static_cast<Job*>(p);
      if (d->result == RES_OK) oks.fetch_add(1);
      else if (d->result == RES_TIMEOUT) timeouts.fetch_add(1);
      else eofs.fetch_add(1);
      if (d->conn.load()) {  // still the loop's: it closes the socket (and forgets the job)
        ::close(d->fd);
        for (auto& c : live)
          if (c.job == d) {
            ::close(c.peer);
            c.job = nullptr;
          }
      }
      delete d;
    }
    done.clear();
  };
  for (int round = 0; round < kRounds; ++round) {
    auto wake = std::make_shared<HsWake>();
    std::vector<Conn> live;
    for (int i = 0; i < kJobs; ++i) {
      int sv[2];
      if (::socketpair(AF_UNIX, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0, sv) < 0) {
        std::perror("socketpair");
        return 1;
      }
      Job* j = new Job();
      j->fd = sv[0];
      j->wake = wake;
      j->need = 1 + int(rng() % 3);
      bool starve = rng() % 10 == 0;  // never fed: the deadline scan must end it
      j->deadline = beholder::reactor_now() + (starve ? 0.02 : 60.0);
      live.push_back({j, sv[1], starve ? 1 << 20 : 0});
      if (!reactor.submit(j)) {
        std::fprintf(stderr, "submit failed\n");
        return 1;
      }
    }
    // feed, drain and orphan until every job of the round has ended one way or the other
    auto until = std::chrono::steady_clock::now() + std::chrono::seconds(20);
    for (;;) {
      std::deque<void*> done;
      wake->take(done);
      drain(done, live);
      bool any = false;
      for (auto& c : live) {
        if (!c.job) continue;
        any = true;
        if (c.sent < c.job->need && rng() % 2 == 0) {
          char b = 'x';
          if (::send(c.peer, &b, 1, MSG_NOSIGNAL) == 1) ++c.sent;
        }
        if (rng() % 400 == 0) {  // the connection closes while its handshake runs (or just ended)
          Job* x = c.job;
          int fd = x->fd;
          c.job = nullptr;
          ::shutdown(fd, SHUT_RDWR);  // wake it before giving it up: after that, x may be gone
          if (x->state.exchange(HS_ORPHANED) != HS_RUNNING) {
            x->conn = false;  // DONE: queued for the drain, which just frees it
            ::close(fd);
          }  // else the reactor frees the job and closes its fd
          ::close(c.peer);
        }
      }
      if (!any) break;
      if (std::chrono::steady_clock::now() > until) {
        std::fprintf(stderr, "hs_reactor_stress: round %d did not finish (a job was never woken)\n", round);
        return 1;
      }
      std::this_thread::yield();
    }
    std::deque<void*> rest;
    wake->close(rest);
    drain(rest, live);
  }
  // orphaned jobs are freed by the reactor threads once their shutdown wakes them
  auto until = std::chrono::steady_clock::now() + std::chrono::seconds(20);
  while (created.load() != freed.load() && std::chrono::steady_clock::now() < until)
    std::this_thread::sleep_for(std::chrono::milliseconds(5));
  reactor.stop();
  for (auto& t : ts) t.join();
  if (created.load() != freed.load()) {
    std::fprintf(stderr, "hs_reactor_stress: %ld jobs created, %ld freed\n", created.load(), freed.load());
    return 1;
  }
  if (oks.load() == 0 || timeouts.load() == 0 || freed_by_reactor.load() == 0) {
    std::fprintf(stderr, "hs_reactor_stress: a path was not exercised (ok %ld, timeout %ld, orphaned %ld)\n",
                 oks.load(), timeouts.load(), freed_by_reactor.load());
    return 1;
  }
  std::printf("hs_reactor_stress: %ld jobs (%ld ok, %ld expired, %ld eof, %ld orphaned while running), each freed once\n",
              created.load(), oks.load(), timeouts.load(), eofs.load(), freed_by_reactor.load());
  return 0;
}
