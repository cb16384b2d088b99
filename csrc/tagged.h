// Host side of the tagged-word hand-off (window_stats.h `tagged_out`, publish.hip).
//
// A GPU writes each value as ONE aligned 8-byte word {float bits, seq << 32} into mapped
// host memory; the host knows every value's publication from the word itself, so no
// completion flag has to be ordered behind the values. The reader spins until every word
// of publication `seq` carries `seq` (or a later number, modulo 2^32) and copies the
// values out in order; a word once seen is not read again.
#pragma once

#include <chrono>
#include <cstdint>
#include <cstring>

namespace rocmdash {

// Copy words [i, n) whose tag has reached `seq` into dst, advancing i; true once all n are.
inline bool scan_tagged(const uint64_t* words, uint32_t n, uint32_t seq, float* dst, uint32_t& i) {
  for (; i < n; ++i) {
    const uint64_t w = __atomic_load_n(words + i, __ATOMIC_ACQUIRE);
    if (int32_t(uint32_t(w >> 32) - seq) < 0) return false;
    const uint32_t bits = uint32_t(w);
    std::memcpy(dst + i, &bits, sizeof bits);
  }
  return true;
}

// Spin (pause loop) until every word carries `seq`, at most timeout_us; true when seen.
inline bool wait_tagged(const uint64_t* words, uint32_t n, uint32_t seq, float* dst, double timeout_us) {
  if (seq == 0) return false;  // 0 is never published
  uint32_t i = 0;
  if (scan_tagged(words, n, seq, dst, i)) return true;
  const auto end = std::chrono::steady_clock::now() + std::chrono::duration<double, std::micro>(timeout_us);
  for (uint32_t it = 1;; ++it) {
    if (scan_tagged(words, n, seq, dst, i)) return true;
#if defined(__x86_64__)
    __builtin_ia32_pause();
#endif
    if ((it & 255) == 0 && std::chrono::steady_clock::now() >= end) return scan_tagged(words, n, seq, dst, i);
  }
}

}  // namespace rocmdash
