// Host side of the tagged-word hand-off (window_stats.h `tagged_out`, publish.hip).
//
// A GPU writes each value as ONE aligned 8-byte word {float bits, seq << 32} into mapped
// host memory; the host knows every value's publication from the word itself, so no
// completion flag has to be ordered behind the values. The reader accepts a word only
// when its tag is EXACTLY `seq`: an older tag means the word is not written yet, a newer
// one (modulo 2^32) means a later publication overwrote the buffer before this one was
// read out - the copy would mix two publications, so the wait reports "superseded" and
// the caller gets no values. Words are copied out in order; a word once seen is not read
// again.
#pragma once

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <thread>
#include <cstdint>
#include <cstring>

namespace rocmdash {

enum class TagScan : int { kPending = 0, kDone = 1, kSuperseded = -1 };

// Copy words [i, n) tagged `seq` into dst, advancing i. kDone once all n are; kPending
// at the first word not yet written; kSuperseded at the first word of a newer publication.
inline TagScan scan_tagged(const uint64_t* words, uint32_t n, uint32_t seq, float* dst, uint32_t& i) {
  for (; i < n; ++i) {
    const uint64_t w = __atomic_load_n(words + i, __ATOMIC_ACQUIRE);
    const int32_t d = int32_t(uint32_t(w >> 32) - seq);
    if (d < 0) return TagScan::kPending;
    if (d > 0) return TagScan::kSuperseded;
    const uint32_t bits = uint32_t(w);
    std::memcpy(dst + i, &bits, sizeof bits);
  }
  return TagScan::kDone;
}

// Spin (pause loop) until every word carries `seq`, at most timeout_us. kDone when the
// whole publication was copied; kPending on timeout; kSuperseded when a newer
// publication overwrote part of it (dst then holds no complete publication).
// The host's waits for the device (a refresh's outputs, a gather's publication, the
// bracket report): spin for wait_spin_us() - the common case, a result a few to a few
// hundred microseconds away, returns at once - then sleep-poll with a backoff from 20 us
// to 1 ms, so a rank waiting for a slower peer gives its core back (8 oversubscribed ranks
// at 1 Hz spun ~0.3 CPU-s/s each, profiles/r05/nodecpu/). ROCMDASH_WAIT_SPIN_US sets the
// spin budget (default 200).
inline double wait_spin_us() {
  static const double v = [] {
    const char* e = std::getenv("ROCMDASH_WAIT_SPIN_US");
    return e ? std::max(0.0, std::atof(e)) : 200.0;
  }();
  return v;
}
struct SpinBackoff {
  std::chrono::steady_clock::time_point spin_end;
  uint32_t it = 0, sleep_us = 20;
  bool spinning = true;
  SpinBackoff()
      : spin_end(std::chrono::steady_clock::now() +
                 std::chrono::microseconds(static_cast<long long>(wait_spin_us()))) {}
  // between two polls; true when the caller should look at its deadline
  bool pause() {
    ++it;
    if (spinning) {
      if ((it & 63) != 0 || std::chrono::steady_clock::now() < spin_end) {
#if defined(__x86_64__) || defined(__i386__)
        __builtin_ia32_pause();
#elif defined(__aarch64__)
        __asm__ __volatile__("yield");
#endif
        return (it & 255) == 0;
      }
      spinning = false;  // the spin budget is spent: sleep-poll from here on
    }
    std::this_thread::sleep_for(std::chrono::microseconds(sleep_us));
    sleep_us = std::min<uint32_t>(sleep_us * 2, 1000);
    return true;
  }
};

inline TagScan wait_tagged(const uint64_t* words, uint32_t n, uint32_t seq, float* dst, double timeout_us) {
  if (seq == 0) return TagScan::kPending;  // 0 is never published
  uint32_t i = 0;
  TagScan s = scan_tagged(words, n, seq, dst, i);
  if (s != TagScan::kPending) return s;
  const auto end = std::chrono::steady_clock::now() + std::chrono::duration<double, std::micro>(timeout_us);
  SpinBackoff wait;
  for (;;) {
    s = scan_tagged(words, n, seq, dst, i);
    if (s != TagScan::kPending) return s;
    if (wait.pause() && std::chrono::steady_clock::now() >= end) return scan_tagged(words, n, seq, dst, i);
  }
}

// RAII marker of a wait in progress: a publication enqueued while another thread is
// still copying the previous one out would overwrite the words under the reader, so
// publish()/refresh() refuse while one is held (std::logic_error).
struct WaitGuard {
  int* flag;
  explicit WaitGuard(int* f) : flag(f) { __atomic_add_fetch(flag, 1, __ATOMIC_ACQ_REL); }
  ~WaitGuard() { __atomic_sub_fetch(flag, 1, __ATOMIC_ACQ_REL); }
  WaitGuard(const WaitGuard&) = delete;
  WaitGuard& operator=(const WaitGuard&) = delete;
};

inline bool wait_in_progress(const int* flag) { return __atomic_load_n(flag, __ATOMIC_ACQUIRE) != 0; }

}  // namespace rocmdash
