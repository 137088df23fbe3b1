// Bounded multi-producer / single-consumer byte ring of framed records, plus
// the stream framer used by the native ingest thread. No Python dependency, so
// the same code is stress-tested under ThreadSanitizer / ASan in
// tests/native/ (SURVEY.md §5 "race detection").
//
// Role in the service: the reference receives each message from amqplib's
// socket reader and hands it to an async handler (index.js:62,127) with at
// most `prefetch` = 100 in flight (index.js:43). Our stdin/file/pipe sources
// get the same decoupling from a dedicated reader thread that reads large
// chunks, splits frames and copies them into this ring *without the GIL*; the
// Python event loop pops whole batches. Backpressure (BASELINE config 4) is a
// ring policy: BLOCK stalls the reader (and, through the pipe, the producer),
// DROP_NEWEST discards and counts.
//
// Record layout (8-byte aligned):
//   u32 rec_bytes | u8 topic | u8 flags | u16 reserved | u32 payload_len |
//   u32 reserved  | u64 seq  | u64 recv_ns | payload[payload_len] | pad
// rec_bytes == 0 is a wrap marker: the consumer jumps to offset 0.
#pragma once

#include <pthread.h>
#include <time.h>
#include <unistd.h>

#include <cerrno>
#include <cstdint>
#include <cstring>
#include <vector>

namespace beholder {

// Thin pthread wrappers. The condition variable waits on CLOCK_MONOTONIC via
// pthread_cond_timedwait: std::condition_variable::wait_for in libstdc++ 11
// uses pthread_cond_clockwait, which ThreadSanitizer (GCC 11) does not
// intercept, producing false race reports in tests/native/.
class Mutex {
 public:
  Mutex() { pthread_mutex_init(&m_, nullptr); }
  ~Mutex() { pthread_mutex_destroy(&m_); }
  Mutex(const Mutex&) = delete;
  Mutex& operator=(const Mutex&) = delete;
  void lock() { pthread_mutex_lock(&m_); }
  void unlock() { pthread_mutex_unlock(&m_); }
  pthread_mutex_t* native() { return &m_; }

 private:
  pthread_mutex_t m_;
};

class Lock {
 public:
  explicit Lock(Mutex& m) : m_(m) { m_.lock(); }
  ~Lock() { m_.unlock(); }
  Lock(const Lock&) = delete;
  Lock& operator=(const Lock&) = delete;
  Mutex& mutex() { return m_; }

 private:
  Mutex& m_;
};

class CondVar {
 public:
  CondVar() {
    pthread_condattr_t a;
    pthread_condattr_init(&a);
    pthread_condattr_setclock(&a, CLOCK_MONOTONIC);
    pthread_cond_init(&c_, &a);
    pthread_condattr_destroy(&a);
  }
  ~CondVar() { pthread_cond_destroy(&c_); }
  CondVar(const CondVar&) = delete;
  CondVar& operator=(const CondVar&) = delete;
  void wait(Lock& l) { pthread_cond_wait(&c_, l.mutex().native()); }
  // Waits until the absolute CLOCK_MONOTONIC deadline; returns false on timeout.
  bool wait_until(Lock& l, int64_t deadline_ns) {
    struct timespec ts;
    ts.tv_sec = time_t(deadline_ns / 1000000000LL);
    ts.tv_nsec = long(deadline_ns % 1000000000LL);
    return pthread_cond_timedwait(&c_, l.mutex().native(), &ts) == 0;
  }
  void notify_one() { pthread_cond_signal(&c_); }
  void notify_all() { pthread_cond_broadcast(&c_); }

 private:
  pthread_cond_t c_;
};

inline int64_t mono_ns() {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return int64_t(ts.tv_sec) * 1000000000LL + ts.tv_nsec;
}

struct RecordHeader {
  uint32_t rec_bytes;
  uint8_t topic;
  uint8_t flags;
  uint16_t reserved0;
  uint32_t payload_len;
  uint32_t reserved1;
  uint64_t seq;
  int64_t recv_ns;
};
static_assert(sizeof(RecordHeader) == 32, "record header must be 32 bytes");

enum Policy : int { POLICY_BLOCK = 0, POLICY_DROP_NEWEST = 1 };

static constexpr int MAX_TOPICS = 16;

struct RingStats {
  uint64_t pushed = 0;
  uint64_t popped = 0;
  uint64_t dropped[MAX_TOPICS] = {0};
  uint64_t dropped_total = 0;
  uint64_t bytes_pushed = 0;
  uint64_t blocked_ns = 0;  // time the producer spent waiting for space
  uint64_t high_water_events = 0;
};

class ByteRing {
 public:
  ByteRing(size_t capacity_bytes, size_t capacity_events, int policy)
      : cap_((capacity_bytes + 7) & ~size_t(7)),
        max_events_(capacity_events ? capacity_events : SIZE_MAX),
        policy_(policy),
        buf_(cap_) {}

  size_t capacity() const { return cap_; }
  size_t max_record_payload() const { return cap_ / 4; }

  static inline size_t record_size(size_t payload) {
    return (sizeof(RecordHeader) + payload + 7) & ~size_t(7);
  }

  // ---- producer side ----------------------------------------------------
  // Push one record. Returns 1 on success, 0 if dropped (policy / too big),
  // -1 if the ring was closed while waiting.
  int push(uint8_t topic, uint8_t flags, const uint8_t* payload, uint32_t len, int64_t recv_ns) {
    size_t need = record_size(len);
    Lock lk(mu_);
    if (need > cap_ / 2) {
      count_drop_locked(topic);
      return 0;
    }
    size_t off;
    for (;;) {
      if (closed_) return -1;
      off = size_t(wpos_ % cap_);
      size_t pad = (off + need > cap_) ? (cap_ - off) : 0;
      bool fits = (wpos_ - rpos_) + pad + need <= cap_ && (wcount_ - rcount_) < max_events_;
      if (fits) {
        if (pad) {
          // Offsets are 8-aligned, so pad >= 8: room for the 4-byte wrap marker.
          uint32_t zero = 0;
          std::memcpy(&buf_[off], &zero, 4);
          wpos_ += pad;
          off = 0;
        }
        break;
      }
      if (policy_ == POLICY_DROP_NEWEST) {
        count_drop_locked(topic);
        return 0;
      }
      int64_t t0 = mono_ns();
      ++producers_waiting_;
      cv_space_.wait(lk);
      --producers_waiting_;
      stats_.blocked_ns += uint64_t(mono_ns() - t0);
    }
    // [off, off+need) lies outside the consumer's readable window [rpos, wpos),
    // so writing it while holding the lock is race-free for any number of
    // producers; the consumer copies out of its window without the lock.
    RecordHeader h;
    h.rec_bytes = uint32_t(need);
    h.topic = topic;
    h.flags = flags;
    h.reserved0 = 0;
    h.payload_len = len;
    h.reserved1 = 0;
    h.seq = seq_++;
    h.recv_ns = recv_ns;
    std::memcpy(&buf_[off], &h, sizeof h);
    if (len) std::memcpy(&buf_[off + sizeof h], payload, len);
    wpos_ += need;
    ++wcount_;
    stats_.pushed++;
    stats_.bytes_pushed += len;
    uint64_t depth = wcount_ - rcount_;
    if (depth > stats_.high_water_events) stats_.high_water_events = depth;
    if (consumer_waiting_) cv_data_.notify_one();
    if (armed_) {  // the event loop found the ring empty and is parked on the notify fd
      armed_ = false;
      signal_locked();
    }
    return 1;
  }

  // ---- consumer side ----------------------------------------------------
  // Wait until at least one record is available, the ring is closed or the
  // timeout passes. Returns the number of bytes readable [rpos, wpos).
  // timeout_ns < 0 waits forever.
  size_t wait_readable(int64_t timeout_ns) {
    Lock lk(mu_);
    if (wpos_ == rpos_ && !closed_ && !eof_ && timeout_ns != 0) {
      consumer_waiting_ = true;
      auto ready = [&] { return wpos_ != rpos_ || closed_ || eof_; };
      if (timeout_ns < 0) {
        while (!ready()) cv_data_.wait(lk);
      } else {
        const int64_t deadline = mono_ns() + timeout_ns;
        while (!ready()) {
          if (!cv_data_.wait_until(lk, deadline) && mono_ns() >= deadline) break;
        }
      }
      consumer_waiting_ = false;
    }
    return size_t(wpos_ - rpos_);
  }

  // Event-loop wake-up (one hop, no worker thread): the loop watches `fd`
  // (an eventfd, loop.add_reader) and calls arm() when a non-blocking pop came
  // back empty. arm() returns false if a record, EOF or close arrived in the
  // meantime (pop again); otherwise the next push, set_eof() or close() writes
  // the fd once. Under load the consumer never arms, so pushes never touch it.
  void set_notify_fd(int fd) {
    Lock g(mu_);
    notify_fd_ = fd;
  }
  bool arm() {
    Lock g(mu_);
    if (wpos_ != rpos_ || closed_ || eof_) return false;
    armed_ = true;
    return true;
  }

  // Snapshot of the readable region (call after wait_readable). The consumer
  // walks records with next_record() and then releases with consume().
  uint64_t read_begin() {
    Lock g(mu_);
    return rpos_;
  }
  uint64_t read_end() {
    Lock g(mu_);
    return wpos_;
  }

  // Returns pointer to the header of the record at logical position `pos`
  // (skipping a wrap marker / tail padding), and advances `pos` past it.
  const RecordHeader* next_record(uint64_t& pos, uint64_t end) const {
    while (pos < end) {
      size_t off = size_t(pos % cap_);
      size_t tail = cap_ - off;
      if (tail < sizeof(RecordHeader)) {
        pos += tail;
        continue;
      }
      uint32_t rb;
      std::memcpy(&rb, &buf_[off], 4);
      if (rb == 0) {
        pos += tail;
        continue;
      }
      const RecordHeader* h = reinterpret_cast<const RecordHeader*>(&buf_[off]);
      pos += rb;
      return h;
    }
    return nullptr;
  }

  static const uint8_t* payload_of(const RecordHeader* h) {
    return reinterpret_cast<const uint8_t*>(h) + sizeof(RecordHeader);
  }

  void consume(uint64_t new_rpos, uint64_t nrecords) {
    Lock g(mu_);
    rpos_ = new_rpos;
    rcount_ += nrecords;
    stats_.popped += nrecords;
    if (producers_waiting_) cv_space_.notify_all();
  }

  // ---- lifecycle ----------------------------------------------------------
  void set_eof() {
    Lock g(mu_);
    eof_ = true;
    cv_data_.notify_all();
    armed_ = false;
    signal_locked();
  }
  void close() {
    Lock g(mu_);
    closed_ = true;
    cv_data_.notify_all();
    cv_space_.notify_all();
    armed_ = false;
    signal_locked();
  }
  bool eof() {
    Lock g(mu_);
    return eof_;
  }
  bool closed() {
    Lock g(mu_);
    return closed_;
  }
  bool drained() {
    Lock g(mu_);
    return (eof_ || closed_) && wpos_ == rpos_;
  }
  size_t depth_events() {
    Lock g(mu_);
    return size_t(wcount_ - rcount_);
  }
  RingStats stats() {
    Lock g(mu_);
    return stats_;
  }
  void count_external_drop(uint8_t topic) {
    Lock g(mu_);
    count_drop_locked(topic);
  }

 private:
  void signal_locked() {
    if (notify_fd_ < 0) return;
    uint64_t one = 1;
    ssize_t r;
    do {
      r = ::write(notify_fd_, &one, sizeof one);  // eventfd: never blocks (EFD_NONBLOCK), counts up
    } while (r < 0 && errno == EINTR);
  }

  void count_drop_locked(uint8_t topic) {
    stats_.dropped[topic < MAX_TOPICS ? topic : 0]++;
    stats_.dropped_total++;
  }

  const size_t cap_;
  const size_t max_events_;
  const int policy_;
  std::vector<uint8_t> buf_;

  Mutex mu_;
  CondVar cv_data_, cv_space_;
  uint64_t wpos_ = 0, rpos_ = 0;      // logical byte positions (monotonic)
  uint64_t wcount_ = 0, rcount_ = 0;  // records pushed / consumed
  uint64_t seq_ = 0;
  int producers_waiting_ = 0;
  bool consumer_waiting_ = false;
  bool armed_ = false;  // the loop is parked on notify_fd_
  int notify_fd_ = -1;
  bool closed_ = false, eof_ = false;
  RingStats stats_;
};

// Incremental splitter for the stdin/pipe frame format:
//   u32 little-endian length L (= 1 + payload bytes) | u8 topic | payload[L-1]
// Feed arbitrary chunks; complete frames are emitted through `emit`.
class Framer {
 public:
  explicit Framer(uint32_t max_frame) : max_frame_(max_frame) {}

  // Returns false (and sets error()) on a corrupt stream.
  template <class Emit>
  bool feed(const uint8_t* data, size_t n, Emit&& emit) {
    size_t i = 0;
    // finish a partially buffered frame first
    if (!carry_.empty()) {
      while (i < n) {
        if (carry_.size() < 4) {
          carry_.push_back(data[i++]);
          if (carry_.size() == 4 && !check_len(carry_.data())) return false;
          continue;
        }
        uint32_t L = load_len(carry_.data());
        size_t want = 4 + size_t(L) - carry_.size();
        size_t take = want < (n - i) ? want : (n - i);
        carry_.insert(carry_.end(), data + i, data + i + take);
        i += take;
        if (carry_.size() == 4 + size_t(L)) {
          emit(carry_[4], carry_.data() + 5, L - 1);
          carry_.clear();
          break;
        }
      }
      if (!carry_.empty()) return true;
    }
    // fast path: frames fully inside `data`
    while (n - i >= 4) {
      if (!check_len(data + i)) return false;
      uint32_t L = load_len(data + i);
      if (n - i - 4 < L) break;
      emit(data[i + 4], data + i + 5, L - 1);
      i += 4 + size_t(L);
    }
    if (i < n) carry_.assign(data + i, data + n);
    return true;
  }

  bool partial() const { return !carry_.empty(); }
  const char* error() const { return err_; }

 private:
  static uint32_t load_len(const uint8_t* p) {
    return uint32_t(p[0]) | (uint32_t(p[1]) << 8) | (uint32_t(p[2]) << 16) | (uint32_t(p[3]) << 24);
  }
  bool check_len(const uint8_t* p) {
    uint32_t L = load_len(p);
    if (L == 0) {
      err_ = "zero-length frame (missing topic byte)";
      return false;
    }
    if (L > max_frame_) {
      err_ = "frame exceeds max_frame";
      return false;
    }
    return true;
  }

  uint32_t max_frame_;
  std::vector<uint8_t> carry_;
  const char* err_ = nullptr;
};

}  // namespace beholder
