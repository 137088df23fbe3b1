// Stress test for the native ingest ring + framer (beholder_amd/ops/csrc/ring.hpp).
// Built twice by tests/test_native_sanitizers.py: -fsanitize=thread and
// -fsanitize=address,undefined. Checks, under concurrency:
//   * N producers x M records each arrive exactly once, per-producer in order,
//     with intact payloads (wrap-around exercised by a tiny ring);
//   * DROP_NEWEST accounting: accepted + dropped == offered;
//   * the Framer reassembles a stream split at random chunk boundaries;
//   * close() wakes a blocked producer and a waiting consumer;
//   * the event-loop consumer (pop without waiting, arm(), sleep on the eventfd) never misses a
//     wake-up: every record is consumed while producers push at random intervals.
#include <poll.h>
#include <sys/eventfd.h>
#include <unistd.h>

#include <atomic>
#include <cassert>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

#include "ring.hpp"

using namespace beholder;

#define CHECK(c)                                                           \
  do {                                                                     \
    if (!(c)) {                                                            \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      std::exit(1);                                                        \
    }                                                                      \
  } while (0)

static void fill(uint8_t* p, uint32_t n, uint32_t producer, uint32_t i) {
  for (uint32_t k = 0; k < n; ++k) p[k] = uint8_t(producer * 31 + i * 7 + k);
}

static void mpsc_block(int producers, int per, size_t cap) {
  ByteRing ring(cap, 0, POLICY_BLOCK);
  std::vector<std::thread> ts;
  for (int p = 0; p < producers; ++p) {
    ts.emplace_back([&, p] {
      std::vector<uint8_t> buf(300);
      for (int i = 0; i < per; ++i) {
        uint32_t n = 8 + (uint32_t(i * 13 + p) % 250);
        std::memcpy(buf.data(), &i, 4);
        fill(buf.data() + 4, n - 4, uint32_t(p), uint32_t(i));
        CHECK(ring.push(uint8_t(p + 1), 0, buf.data(), n, mono_ns()) == 1);
      }
    });
  }
  std::vector<int> next(producers, 0);
  long total = 0, want = long(producers) * per;
  while (total < want) {
    if (!ring.wait_readable(50000000)) continue;
    uint64_t pos = ring.read_begin(), end = ring.read_end();
    uint64_t n = 0;
    while (const RecordHeader* h = ring.next_record(pos, end)) {
      int p = h->topic - 1;
      CHECK(p >= 0 && p < producers);
      const uint8_t* pl = ByteRing::payload_of(h);
      int i;
      std::memcpy(&i, pl, 4);
      CHECK(i == next[p]);
      uint32_t expect_n = 8 + (uint32_t(i * 13 + p) % 250);
      CHECK(h->payload_len == expect_n);
      std::vector<uint8_t> ref(expect_n - 4);
      fill(ref.data(), expect_n - 4, uint32_t(p), uint32_t(i));
      CHECK(std::memcmp(ref.data(), pl + 4, expect_n - 4) == 0);
      next[p]++;
      ++n;
    }
    ring.consume(pos, n);
    total += long(n);
  }
  for (auto& t : ts) t.join();
  RingStats st = ring.stats();
  CHECK(long(st.pushed) == want && long(st.popped) == want && st.dropped_total == 0);
  std::printf("mpsc_block ok: %d producers x %d, blocked %.1f ms\n", producers, per, st.blocked_ns / 1e6);
}

static void drop_newest(int per) {
  ByteRing ring(1 << 14, 64, POLICY_DROP_NEWEST);
  std::atomic<bool> done{false};
  long accepted = 0;
  std::thread prod([&] {
    uint8_t buf[40] = {0};
    for (int i = 0; i < per; ++i) accepted += ring.push(2, 0, buf, sizeof buf, 0);
    done = true;
    ring.set_eof();
  });
  long got = 0;
  for (;;) {
    ring.wait_readable(10000000);
    uint64_t pos = ring.read_begin(), end = ring.read_end();
    uint64_t n = 0;
    while (ring.next_record(pos, end)) ++n;
    ring.consume(pos, n);
    got += long(n);
    if (done && ring.drained()) break;
  }
  prod.join();
  RingStats st = ring.stats();
  CHECK(got == accepted);
  CHECK(long(st.dropped_total) + accepted == per && st.dropped[2] == st.dropped_total);
  std::printf("drop_newest ok: offered %d accepted %ld dropped %llu\n", per, accepted,
              (unsigned long long)st.dropped_total);
}

static void framer_random_chunks() {
  std::mt19937 rng(1234);
  std::vector<uint8_t> stream;
  std::vector<std::vector<uint8_t>> frames;
  for (int i = 0; i < 5000; ++i) {
    uint32_t n = rng() % 400;
    std::vector<uint8_t> pl(n);
    for (auto& b : pl) b = uint8_t(rng());
    uint32_t L = n + 1;
    uint8_t hdr[5] = {uint8_t(L), uint8_t(L >> 8), uint8_t(L >> 16), uint8_t(L >> 24), uint8_t(1 + i % 2)};
    stream.insert(stream.end(), hdr, hdr + 5);
    stream.insert(stream.end(), pl.begin(), pl.end());
    frames.push_back(pl);
  }
  Framer fr(1 << 20);
  size_t idx = 0, off = 0;
  while (off < stream.size()) {
    size_t take = std::min<size_t>(stream.size() - off, 1 + rng() % 700);
    CHECK(fr.feed(stream.data() + off, take, [&](uint8_t topic, const uint8_t* p, uint32_t len) {
      CHECK(idx < frames.size());
      CHECK(topic == uint8_t(1 + idx % 2));
      CHECK(len == frames[idx].size() && (len == 0 || std::memcmp(p, frames[idx].data(), len) == 0));
      ++idx;
    }));
    off += take;
  }
  CHECK(idx == frames.size() && !fr.partial());
  std::printf("framer ok: %zu frames\n", idx);
}

static void close_wakes_everyone() {
  ByteRing ring(4096, 1, POLICY_BLOCK);
  uint8_t b[8] = {0};
  CHECK(ring.push(1, 0, b, 8, 0) == 1);
  std::atomic<int> r{2};
  std::thread blocked([&] { r = ring.push(1, 0, b, 8, 0); });
  std::this_thread::sleep_for(std::chrono::milliseconds(50));
  ring.close();
  blocked.join();
  CHECK(r == -1);
  ByteRing empty(4096, 0, POLICY_BLOCK);
  std::thread waiter([&] { empty.wait_readable(-1); });
  std::this_thread::sleep_for(std::chrono::milliseconds(20));
  empty.close();
  waiter.join();
  std::printf("close ok\n");
}

// The FdSource pattern (transport/ingest.py): non-blocking pop; when empty, arm() and poll the
// eventfd (with a long timeout that must never be what wakes us up).
static void eventfd_consumer(int producers, int per) {
  ByteRing ring(1 << 16, 0, POLICY_BLOCK);
  int efd = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
  CHECK(efd >= 0);
  ring.set_notify_fd(efd);
  std::atomic<int> live{producers};
  std::vector<std::thread> ts;
  for (int p = 0; p < producers; ++p) {
    ts.emplace_back([&, p] {
      std::mt19937 rng(uint32_t(p) + 7);
      uint8_t buf[24] = {0};
      for (int i = 0; i < per; ++i) {
        if (rng() % 8 == 0) std::this_thread::sleep_for(std::chrono::microseconds(rng() % 200));
        CHECK(ring.push(1, 0, buf, sizeof buf, 0) == 1);
      }
      if (--live == 0) ring.set_eof();
    });
  }
  long got = 0, parks = 0, timeouts = 0;
  const long want = long(producers) * per;
  for (;;) {
    size_t avail = ring.wait_readable(0);
    if (avail) {
      uint64_t pos = ring.read_begin(), end = ring.read_end();
      uint64_t n = 0;
      while (ring.next_record(pos, end)) ++n;
      ring.consume(pos, n);
      got += long(n);
      continue;
    }
    if (ring.drained()) break;
    if (!ring.arm()) continue;  // something arrived between the pop and arm()
    ++parks;
    pollfd pfd = {efd, POLLIN, 0};
    int r = poll(&pfd, 1, 5000);
    if (r == 0) ++timeouts;  // a lost wake-up: only the timeout got us out
    uint64_t v;
    ssize_t rd = read(efd, &v, sizeof v);
    (void)rd;
  }
  for (auto& t : ts) t.join();
  close(efd);
  CHECK(got == want && timeouts == 0);
  std::printf("eventfd_consumer ok: %ld records, %ld parks, no lost wake-up\n", got, parks);
}

int main() {
  mpsc_block(4, 20000, 8192);
  mpsc_block(1, 50000, 4096);
  drop_newest(200000);
  framer_random_chunks();
  close_wakes_everyone();
  eventfd_consumer(3, 20000);
  std::printf("ALL OK\n");
  return 0;
}
