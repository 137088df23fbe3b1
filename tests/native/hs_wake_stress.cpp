// Stress test of the TLS handshake completion channel (beholder_amd/ops/csrc/hs_wake.hpp) under
// ThreadSanitizer / ASan, with the job ownership protocol of py_netconn.cpp around it:
//
//   handshake thread: run the job, then state RUNNING -> DONE; if the loop had ORPHANED it
//     meanwhile, the thread frees the job; else it posts the job, and if the channel is closed
//     (the poller closed) it frees the job itself.
//   loop thread: drains finished jobs (tls_done frees them); "closes a connection" by
//     state -> ORPHANED (a RUNNING job is then the thread's to free) or, for a DONE job, marks it
//     connection-less (the drain frees it); finally closes the channel (poller_close) and frees
//     what was queued.
//
// Every job must be freed exactly once: created == freed at the end, and the sanitizers see no
// race or leak.
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <deque>
#include <memory>
#include <mutex>
#include <random>
#include <thread>
#include <vector>

#include "hs_wake.hpp"

using beholder::HsWake;

enum { RUNNING, DONE, ORPHANED };

std::atomic<long> created{0}, freed{0};

struct Job {
  std::atomic<int> state{RUNNING};
  std::atomic<bool> conn{true};  // the loop still has the connection
  std::shared_ptr<HsWake> wake;
  Job() { created.fetch_add(1); }
  ~Job() { freed.fetch_add(1); }
};

struct Queue {  // the handshake pool's job queue
  std::mutex mu;
  std::condition_variable cv;
  std::deque<Job*> q;
  bool stop = false;
};

void worker(Queue* pool) {
  std::mt19937 rng(std::random_device{}());
  for (;;) {
    Job* j;
    {
      std::unique_lock<std::mutex> lock(pool->mu);
      pool->cv.wait(lock, [pool] { return pool->stop || !pool->q.empty(); });
      if (pool->q.empty()) return;
      j = pool->q.front();
      pool->q.pop_front();
    }
    if (rng() % 4 == 0) std::this_thread::yield();  // "the handshake"
    std::shared_ptr<HsWake> wake = j->wake;
    if (j->state.exchange(DONE) == ORPHANED) {
      delete j;
      continue;
    }
    if (!wake->post(j)) delete j;
  }
}

int main() {
  const int kRounds = 200, kJobs = 200, kThreads = 4;
  Queue pool;
  std::vector<std::thread> ts;
  for (int i = 0; i < kThreads; ++i) ts.emplace_back(worker, &pool);
  std::mt19937 rng(12345);
  for (int round = 0; round < kRounds; ++round) {
    auto wake = std::make_shared<HsWake>();
    if (wake->efd < 0) {
      std::perror("eventfd");
      return 1;
    }
    std::vector<Job*> live;
    for (int i = 0; i < kJobs; ++i) {
      Job* j = new Job();
      j->wake = wake;
      live.push_back(j);
      {
        std::lock_guard<std::mutex> lock(pool.mu);
        pool.q.push_back(j);
      }
      pool.cv.notify_one();
      // the loop meanwhile: drain finished ones, close some connections
      std::deque<void*> done;
      wake->take(done);
      for (void* p : done) {
        Job* d = static_cast<Job*>(p);
        for (auto& x : live)
          if (x == d) x = nullptr;
        delete d;  // tls_done (connection-less or not, the loop frees a drained job)
      }
      if (!live.empty() && rng() % 3 == 0) {
        size_t k = rng() % live.size();
        Job* x = live[k];
        if (x) {
          live[k] = nullptr;
          if (x->state.exchange(ORPHANED) != RUNNING) x->conn = false;  // DONE: queued, the drain frees it
        }
      }
    }
    // every connection leaves, then the poller closes: later posts are refused
    for (Job*& x : live) {
      if (!x) continue;
      if (x->state.exchange(ORPHANED) != RUNNING) x->conn = false;
      x = nullptr;
    }
    std::deque<void*> rest;
    wake->close(rest);
    for (void* p : rest) delete static_cast<Job*>(p);
  }
  {
    std::lock_guard<std::mutex> lock(pool.mu);
    pool.stop = true;
  }
  pool.cv.notify_all();
  for (auto& t : ts) t.join();
  // a job that finished after its round's close was freed by its thread; none may be left
  if (created.load() != freed.load()) {
    std::fprintf(stderr, "hs_wake_stress: %ld jobs created, %ld freed\n", created.load(), freed.load());
    return 1;
  }
  std::printf("hs_wake_stress: %ld jobs, each freed once\n", created.load());
  return 0;
}
