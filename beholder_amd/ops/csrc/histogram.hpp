// Log-linear latency histogram (HDR-style), no Python dependency.
//
// Used for the §6 measurement plan (p50/p99 handle/ingest latency)
// and for Prometheus latency histograms. Values are unsigned integers
// (nanoseconds). Values < 2^S are exact; above that each power-of-two octave
// is split into 2^(S-1) linear sub-buckets, i.e. <= 2^-(S-1) relative error
// (0.78% with S = 8). Recording is O(1) (one clz); single-writer (the caller
// holds the GIL), merges are element-wise adds so per-rank histograms combine
// exactly.
#pragma once

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

namespace beholder {

class LogHistogram {
 public:
  static constexpr int S = 8;                      // sub-bucket bits
  static constexpr uint64_t M = uint64_t(1) << S;  // exact range [0, M)
  static constexpr uint64_t HALF = M >> 1;
  static constexpr int MAX_EXP = 56;  // values up to 2^57 ns (~4.5 years)
  static constexpr size_t NBUCKETS = M + size_t(MAX_EXP - S + 1) * HALF;

  LogHistogram() : counts_(NBUCKETS, 0) {}

  static inline size_t index_of(uint64_t v) {
    if (v < M) return size_t(v);
    int e = 63 - __builtin_clzll(v);  // e >= S
    if (e > MAX_EXP) return NBUCKETS - 1;
    int s = e - (S - 1);               // >= 1
    uint64_t mant = v >> s;            // in [HALF, M)
    return size_t(M + uint64_t(s - 1) * HALF + (mant - HALF));
  }

  // Inclusive lower bound of bucket i.
  static inline uint64_t lower_of(size_t i) {
    if (i < M) return i;
    size_t j = i - M;
    int s = int(j / HALF) + 1;
    uint64_t mant = HALF + (j % HALF);
    return mant << s;
  }

  // Inclusive upper bound of bucket i.
  static inline uint64_t upper_of(size_t i) {
    if (i < M) return i;
    if (i + 1 >= NBUCKETS) return UINT64_MAX;
    return lower_of(i + 1) - 1;
  }

  inline void record(uint64_t v, uint64_t n = 1) {
    counts_[index_of(v)] += n;
    total_ += n;
    sum_ += double(v) * double(n);
    if (v < min_) min_ = v;
    if (v > max_) max_ = v;
  }

  void reset() {
    std::fill(counts_.begin(), counts_.end(), 0);
    total_ = 0;
    sum_ = 0;
    min_ = UINT64_MAX;
    max_ = 0;
  }

  void merge(const LogHistogram& o) {
    for (size_t i = 0; i < NBUCKETS; ++i) counts_[i] += o.counts_[i];
    total_ += o.total_;
    sum_ += o.sum_;
    min_ = std::min(min_, o.min_);
    max_ = std::max(max_, o.max_);
  }

  // Value at percentile p in [0, 100]: the midpoint of the bucket holding the
  // ceil(p/100 * N)-th smallest sample, clamped to [min, max].
  double percentile(double p) const {
    if (total_ == 0) return 0.0;
    if (p <= 0) return double(min_);
    if (p >= 100) return double(max_);
    uint64_t rank = uint64_t(std::ceil(p / 100.0 * double(total_)));
    if (rank < 1) rank = 1;
    uint64_t cum = 0;
    for (size_t i = 0; i < NBUCKETS; ++i) {
      cum += counts_[i];
      if (cum >= rank) {
        double lo = double(lower_of(i)), hi = double(upper_of(i));
        double mid = (i < M) ? lo : 0.5 * (lo + hi);
        return std::min(std::max(mid, double(min_)), double(max_));
      }
    }
    return double(max_);
  }

  // Number of samples <= le (exact at bucket boundaries, otherwise counts the
  // whole bucket containing `le` only if its upper bound is <= le).
  uint64_t count_le(uint64_t le) const {
    uint64_t cum = 0;
    for (size_t i = 0; i < NBUCKETS; ++i) {
      if (upper_of(i) > le) break;
      cum += counts_[i];
    }
    return cum;
  }

  uint64_t total() const { return total_; }
  double sum() const { return sum_; }
  uint64_t min() const { return total_ ? min_ : 0; }
  uint64_t max() const { return max_; }
  const std::vector<uint64_t>& counts() const { return counts_; }
  std::vector<uint64_t>& mutable_counts() { return counts_; }
  void set_stats(uint64_t total, double sum, uint64_t mn, uint64_t mx) {
    total_ = total;
    sum_ = sum;
    min_ = mn;
    max_ = mx;
  }

 private:
  std::vector<uint64_t> counts_;
  uint64_t total_ = 0;
  double sum_ = 0;
  uint64_t min_ = UINT64_MAX;
  uint64_t max_ = 0;
};

}  // namespace beholder
