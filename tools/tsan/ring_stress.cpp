// Host-only ThreadSanitizer stress of the SPSC ring + sampler (no HIP): one native
// sampler thread producing as fast as it can, two readers copying windows and
// checking every row they keep is internally consistent, a stats poller, and a second
// sampler driven through request()/wait() from the main thread.
//   g++ -std=c++17 -O1 -g -fsanitize=thread -Icsrc -I/opt/rocm/include tools/tsan/ring_stress.cpp \
//       csrc/sampler.cpp csrc/sources.cpp -L/opt/rocm/lib -lamd_smi -lpthread -Wl,-rpath,/opt/rocm/lib
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#include "ring.h"
#include "sampler.h"
#include "sources.h"

namespace rocmdash {
HostAlloc& host_allocator() {  // pageable memory (the HIP build hands out pinned memory)
  static HostAlloc a{};
  return a;
}
}  // namespace rocmdash

using namespace rocmdash;

int main(int argc, char** argv) {
  const double seconds = argc > 1 ? std::atof(argv[1]) : 1.0;
  auto ring = std::make_shared<SeriesRing>(SMI_NUM_FIELDS, 64);
  Sampler producer(make_synthetic_source("smi", 1), ring, 1e6);
  producer.start();
  std::atomic<bool> stop{false};
  std::atomic<long> bad{0}, kept{0};
  auto reader = [&] {
    std::vector<float> rows(64 * SMI_NUM_FIELDS);
    std::vector<uint64_t> ts(64);
    while (!stop.load()) {
      const uint64_t n = ring->read_window(64, rows.data(), ts.data());
      for (uint64_t i = 0; i < n; ++i) {
        const float* r = rows.data() + i * SMI_NUM_FIELDS;
        if (r[SMI_EDGE_TEMP] != r[SMI_HOTSPOT_TEMP] || r[SMI_USED_VRAM] > r[SMI_TOTAL_VRAM]) ++bad;
        if (i && ts[i] < ts[i - 1]) ++bad;
      }
      kept += long(n);
    }
  };
  std::thread r1(reader), r2(reader);
  std::thread poller([&] {
    while (!stop.load()) (void)producer.stats();
  });
  auto ring2 = std::make_shared<SeriesRing>(CTR_NUM_FIELDS, 64);
  Sampler async_sampler(make_synthetic_source("counter", 2), ring2, 100.0);
  async_sampler.set_spin_us(argc > 2 ? std::atof(argv[2]) : 50.0);  // spin hand-off path
  std::thread r3([&] {
    std::vector<float> rows(64 * CTR_NUM_FIELDS);
    while (!stop.load()) ring2->read_window(64, rows.data(), nullptr);
  });
  const auto t_end = std::chrono::steady_clock::now() + std::chrono::duration<double>(seconds);
  long requests = 0;
  while (std::chrono::steady_clock::now() < t_end) {
    async_sampler.request();
    if (!async_sampler.wait()) ++bad;
    ++requests;
  }
  stop = true;
  r1.join();
  r2.join();
  r3.join();
  poller.join();
  producer.stop();
  const auto st = producer.stats();
  std::printf("produced=%llu kept=%ld requests=%ld bad=%ld\n", (unsigned long long)st.samples, kept.load(), requests,
              bad.load());
  return bad.load() == 0 && st.samples > 1000 && requests > 100 ? 0 : 1;
}
