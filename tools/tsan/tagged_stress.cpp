// Race check of the tagged-word hand-off (csrc/tagged.h) on the CPU, built with
// -fsanitize=thread: a writer thread plays the GPU - it publishes refresh after refresh,
// each word {value, seq} stored on its own in a shuffled order with random pauses (the
// device's stores land in no particular order) - and the reader waits for each
// refresh with wait_tagged() and checks every copied value belongs to it. The writer
// may run one publication ahead of the reader's acknowledgement, so the reader also
// sees words of seq + 1 mixed in (allowed: never older than seq).
//
//   g++ -std=c++17 -O1 -g -fsanitize=thread -Icsrc tools/tsan/tagged_stress.cpp -lpthread
//   ./a.out [publications] [words]   -> prints "bad=0" on success
#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

#include "tagged.h"

using rocmdash::wait_tagged;

static float value_of(uint32_t seq, uint32_t i) { return float(seq) * 4096.0f + float(i); }

int main(int argc, char** argv) {
  const uint32_t pubs = argc > 1 ? uint32_t(std::atoi(argv[1])) : 3000;
  const uint32_t n = argc > 2 ? uint32_t(std::atoi(argv[2])) : 128;
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
        float v = value_of(seq, i);
        uint32_t bits;
        std::memcpy(&bits, &v, sizeof bits);
        __atomic_store_n(&words[i], (uint64_t(seq) << 32) | bits, __ATOMIC_RELAXED);
        if ((rng() & 31) == 0) std::this_thread::yield();
      }
    }
  });

  std::vector<float> dst(n);
  uint64_t bad = 0, ahead = 0;
  for (uint32_t seq = 1; seq <= pubs; ++seq) {
    if (!wait_tagged(words.data(), n, seq, dst.data(), 5e6)) {
      std::printf("timeout at seq %u\n", seq);
      ++bad;
      break;
    }
    for (uint32_t i = 0; i < n; ++i) {
      if (dst[i] == value_of(seq, i)) continue;
      if (dst[i] == value_of(seq + 1, i)) {
        ++ahead;  // the writer's next publication (never an older one)
        continue;
      }
      ++bad;
    }
    acked.store(seq, std::memory_order_release);
  }
  // a publication that never comes is never seen
  if (wait_tagged(words.data(), n, pubs + 1, dst.data(), 1000.0)) ++bad;
  stop.store(true);
  writer.join();
  std::printf("pubs=%u words=%u ahead=%llu bad=%llu\n", pubs, n, (unsigned long long)ahead, (unsigned long long)bad);
  return bad ? 1 : 0;
}
