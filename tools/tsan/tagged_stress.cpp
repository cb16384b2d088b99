// Race check of the tagged-word hand-off (csrc/tagged.h) on the CPU, built with
// -fsanitize=thread: a writer thread plays the GPU - it publishes refresh after refresh,
// each word {value, seq} stored on its own in a shuffled order with random pauses (the
// device's stores land in no particular order) - and the reader waits for each
// refresh with wait_tagged(). The writer runs up to two publications ahead of the
// reader's acknowledgement, so the reader often finds words of seq + 1 / seq + 2 in the
// buffer. Rule under test: a wait returns kDone only with EVERY value of its own
// publication (never a mix), else kSuperseded (nothing usable), never an older value.
//
// A deterministic case first: half the words of seq, half of seq + 1. The round-2 rule
// (accept a tag >= seq, `legacy_scan` below) returns that mix as complete; the current
// rule must report kSuperseded.
//
//   g++ -std=c++17 -O1 -g -fsanitize=thread -Icsrc tools/tsan/tagged_stress.cpp -lpthread
//   ./a.out [publications] [words]   -> prints "... mixed=0 bad=0" on success
#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

#include "tagged.h"

using rocmdash::TagScan;
using rocmdash::wait_tagged;

static float value_of(uint32_t seq, uint32_t i) { return float(seq) * 4096.0f + float(i); }

static uint64_t word_of(uint32_t seq, uint32_t i) {
  float v = value_of(seq, i);
  uint32_t bits;
  std::memcpy(&bits, &v, sizeof bits);
  return (uint64_t(seq) << 32) | bits;
}

// The round-2 scan (tag at or after seq accepted): kept to show what the test catches.
static bool legacy_scan(const uint64_t* words, uint32_t n, uint32_t seq, float* dst) {
  for (uint32_t i = 0; i < n; ++i) {
    const uint64_t w = __atomic_load_n(words + i, __ATOMIC_ACQUIRE);
    if (int32_t(uint32_t(w >> 32) - seq) < 0) return false;
    const uint32_t bits = uint32_t(w);
    std::memcpy(dst + i, &bits, sizeof bits);
  }
  return true;
}

static bool is_mix(const std::vector<float>& dst, uint32_t seq) {
  for (uint32_t i = 0; i < dst.size(); ++i)
    if (dst[i] != value_of(seq, i)) return true;
  return false;
}

int main(int argc, char** argv) {
  const uint32_t pubs = argc > 1 ? uint32_t(std::atoi(argv[1])) : 3000;
  const uint32_t n = argc > 2 ? uint32_t(std::atoi(argv[2])) : 128;
  uint64_t bad = 0;

  {  // deterministic: a publication half overwritten by the next one
    std::vector<uint64_t> w(n);
    for (uint32_t i = 0; i < n; ++i) w[i] = word_of(i < n / 2 ? 5 : 6, i);
    std::vector<float> dst(n);
    const bool legacy_done = legacy_scan(w.data(), n, 5, dst.data());
    const bool legacy_mixed = legacy_done && is_mix(dst, 5);
    const TagScan s = wait_tagged(w.data(), n, 5, dst.data(), 1000.0);
    std::printf("deterministic: legacy_returns_mix=%d current=%s\n", int(legacy_mixed),
                s == TagScan::kSuperseded ? "superseded" : (s == TagScan::kDone ? "done" : "pending"));
    if (!legacy_mixed || s != TagScan::kSuperseded) ++bad;
    // and the newer publication itself is not complete either (words of 5 are older)
    if (wait_tagged(w.data(), n, 6, dst.data(), 1000.0) != TagScan::kPending) ++bad;
  }

  std::vector<uint64_t> words(n, 0);  // tag 0: never published
  std::atomic<uint32_t> acked{0};     // last publication the reader has consumed
  std::atomic<bool> stop{false};

  std::thread writer([&] {
    std::mt19937 rng(7);
    std::vector<uint32_t> order(n);
    for (uint32_t i = 0; i < n; ++i) order[i] = i;
    for (uint32_t seq = 1; seq <= pubs && !stop.load(); ++seq) {
      while (acked.load(std::memory_order_acquire) + 3 <= seq && !stop.load()) std::this_thread::yield();
      std::shuffle(order.begin(), order.end(), rng);
      for (uint32_t k = 0; k < n; ++k) {
        const uint32_t i = order[k];
        __atomic_store_n(&words[i], word_of(seq, i), __ATOMIC_RELAXED);
        if ((rng() & 31) == 0) std::this_thread::yield();
      }
    }
  });

  std::vector<float> dst(n);
  uint64_t done = 0, superseded = 0, mixed = 0;
  for (uint32_t seq = 1; seq <= pubs; ++seq) {
    const TagScan s = wait_tagged(words.data(), n, seq, dst.data(), 5e6);
    if (s == TagScan::kPending) {
      std::printf("timeout at seq %u\n", seq);
      ++bad;
      break;
    }
    if (s == TagScan::kDone) {
      ++done;
      if (is_mix(dst, seq)) ++mixed;  // a complete publication is exactly its own values
    } else {
      ++superseded;
    }
    acked.store(seq, std::memory_order_release);
  }
  // a publication that never comes is never seen
  if (wait_tagged(words.data(), n, pubs + 1, dst.data(), 1000.0) != TagScan::kPending) ++bad;
  stop.store(true);
  writer.join();
  bad += mixed;
  std::printf("pubs=%u words=%u done=%llu superseded=%llu mixed=%llu bad=%llu\n", pubs, n, (unsigned long long)done,
              (unsigned long long)superseded, (unsigned long long)mixed, (unsigned long long)bad);
  return bad ? 1 : 0;
}
