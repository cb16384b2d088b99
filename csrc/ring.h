// Lock-free single-producer ring of fixed-width metric rows in (optionally pinned) host memory.
//
// Reference counterpart: none. The reference keeps exactly one instant sample per
// series per refresh (app.py:167-188, `value[1]` of an instant query) and paces
// itself with `time.sleep(5)` (app.py:486). Here every sample of every series is
// kept in a time-major ring so the HIP window-stats kernel can reduce the last W
// samples, and the refresh never blocks the sampler.
//
// Layout: rows[cap][width] float32 (row = one sample of all series of one source),
// ts[cap] uint64 CLOCK_REALTIME ns. Time-major rows make the rows produced since
// the last refresh ONE contiguous range (two on wrap), so the device mirror is
// updated with at most two hipMemcpyAsync calls per refresh (device_window.cpp).
//
// Concurrency contract (SPSC + snapshot readers):
//   * exactly one producer calls push() (a Sampler thread, or sample_once());
//   * readers load head() with acquire and may read rows [head-n, head) for
//     n <= cap - slack; the producer only overwrites row (head % cap) after it has
//     written every byte of the rows before it, and publishes with a release store.
//   * a reader that copies rows while the producer keeps writing must re-check
//     head() after the copy: rows older than head_after - cap were overwritten
//     (torn) and must be discarded (see read_window()).
#pragma once

#include <atomic>
#include <cstddef>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>

namespace rocmdash {

// Allocator hooks so the HIP side can hand out pinned memory (hipHostMalloc) without
// this header depending on HIP. Defaults to 4 KiB-aligned pageable memory.
struct HostAlloc {
  void* (*alloc)(size_t bytes, bool* pinned) = nullptr;
  void (*release)(void* p, bool pinned) = nullptr;
};
HostAlloc& host_allocator();

class SeriesRing {
 public:
  SeriesRing(uint32_t width, uint64_t capacity) : width_(width), cap_(capacity) {
    if (width == 0) throw std::invalid_argument("ring width must be > 0");
    if (capacity < 2 || (capacity & (capacity - 1)))
      throw std::invalid_argument("ring capacity must be a power of two >= 2");
    mask_ = cap_ - 1;
    const size_t row_bytes = size_t(width_) * sizeof(float);
    bytes_ = cap_ * row_bytes;
    auto& ha = host_allocator();
    if (ha.alloc) {
      rows_ = static_cast<float*>(ha.alloc(bytes_, &pinned_));
      ts_ = static_cast<uint64_t*>(ha.alloc(cap_ * sizeof(uint64_t), &ts_pinned_));
    } else {
      rows_ = static_cast<float*>(std::aligned_alloc(4096, round_up(bytes_, 4096)));
      ts_ = static_cast<uint64_t*>(std::aligned_alloc(4096, round_up(cap_ * 8, 4096)));
    }
    if (!rows_ || !ts_) throw std::bad_alloc();
    std::memset(rows_, 0, bytes_);
    std::memset(ts_, 0, cap_ * sizeof(uint64_t));
  }
  ~SeriesRing() {
    auto& ha = host_allocator();
    if (ha.release) {
      ha.release(rows_, pinned_);
      ha.release(ts_, ts_pinned_);
    } else {
      std::free(rows_);
      std::free(ts_);
    }
  }
  SeriesRing(const SeriesRing&) = delete;
  SeriesRing& operator=(const SeriesRing&) = delete;

  // Producer side. `row` holds `width` floats.
  void push(const float* row, uint64_t t_ns) {
    const uint64_t h = head_.load(std::memory_order_relaxed);
    const uint64_t idx = h & mask_;
    wpos_.store(h + 1, std::memory_order_relaxed);  // row h (slot of row h - cap) in progress
    std::atomic_thread_fence(std::memory_order_release);
    store_words(rows_ + idx * width_, row, width_);
    __atomic_store_n(ts_ + idx, t_ns, __ATOMIC_RELAXED);
    head_.store(h + 1, std::memory_order_release);
  }

  // Rows ever written (monotonic).
  uint64_t head() const { return head_.load(std::memory_order_acquire); }
  uint32_t width() const { return width_; }
  uint64_t capacity() const { return cap_; }
  bool pinned() const { return pinned_; }
  float* rows() const { return rows_; }
  uint64_t* timestamps() const { return ts_; }
  size_t bytes() const { return bytes_; }

  // Copy the newest <= n rows into out[n][width] (oldest first) and their timestamps.
  // Returns the number of rows copied; rows overwritten during the copy are dropped.
  uint64_t read_window(uint64_t n, float* out, uint64_t* out_ts) const {
    const uint64_t h = head();
    const uint64_t avail = h < cap_ ? h : cap_;
    if (n > avail) n = avail;
    uint64_t lo = h - n;
    for (uint64_t i = lo; i < h; ++i) {
      const uint64_t idx = i & mask_;
      load_words(out + (i - lo) * width_, rows_ + idx * width_, width_);
      if (out_ts) out_ts[i - lo] = __atomic_load_n(ts_ + idx, __ATOMIC_RELAXED);
    }
    // Torn-read check (seqlock style): the producer announces a row in wpos_ (then a
    // release fence) BEFORE writing it; after our data loads and an acquire fence,
    // wpos_ bounds every row whose bytes we may have seen being rewritten: writing row
    // w - 1 overwrites row w - 1 - cap, so rows <= w - 1 - cap are dropped.
    std::atomic_thread_fence(std::memory_order_acquire);
    const uint64_t w2 = wpos_.load(std::memory_order_relaxed);
    if (w2 > cap_ && w2 - 1 - cap_ >= lo) {
      const uint64_t drop = (w2 - 1 - cap_) - lo + 1;
      if (drop >= n) return 0;
      std::memmove(out, out + drop * width_, size_t(n - drop) * width_ * sizeof(float));
      if (out_ts) std::memmove(out_ts, out_ts + drop, size_t(n - drop) * sizeof(uint64_t));
      return n - drop;
    }
    return n;
  }

  uint64_t last_timestamp() const {
    const uint64_t h = head();
    return h ? __atomic_load_n(ts_ + ((h - 1) & mask_), __ATOMIC_RELAXED) : 0;
  }

 private:
  // Row payloads move as relaxed atomic 32-bit words: a reader may copy a row the
  // producer is overwriting (it then drops it, see read_window), and word-wise atomics
  // keep that overlap well-defined (no data race for the C++ model / ThreadSanitizer).
  static void store_words(float* dst, const float* src, uint32_t n) {
    auto* d = reinterpret_cast<uint32_t*>(dst);
    const auto* s = reinterpret_cast<const uint32_t*>(src);
    for (uint32_t i = 0; i < n; ++i) __atomic_store_n(d + i, s[i], __ATOMIC_RELAXED);
  }
  static void load_words(float* dst, const float* src, uint32_t n) {
    auto* d = reinterpret_cast<uint32_t*>(dst);
    const auto* s = reinterpret_cast<const uint32_t*>(src);
    for (uint32_t i = 0; i < n; ++i) d[i] = __atomic_load_n(s + i, __ATOMIC_RELAXED);
  }

  static size_t round_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

  alignas(64) std::atomic<uint64_t> head_{0};  // rows completely written
  std::atomic<uint64_t> wpos_{0};              // rows whose writing has started
  alignas(64) uint32_t width_;
  uint64_t cap_, mask_;
  size_t bytes_ = 0;
  float* rows_ = nullptr;
  uint64_t* ts_ = nullptr;
  bool pinned_ = false, ts_pinned_ = false;
};

}  // namespace rocmdash
