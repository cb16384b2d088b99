// Host-only ThreadSanitizer stress of the node counter process's per-GPU lanes
// (csrc/node_counters.cpp ShmPublisher): three synthetic counter
// sources at 5 kHz, lane 1's reads hang after 0.2 s; one ShmSource reader per ring copies
// rows while the main thread polls stats() and replaces lane 1 twice (the hung lane is
// abandoned, a fresh one publishes into a new ring file), then stops with a lane still
// blocked (it is left behind, not joined). Rows must stay finite and in time order.
//   g++ -std=c++17 -O1 -g -fsanitize=thread -Icsrc -I/opt/rocm/include tools/tsan/lanes_stress.cpp \
//       csrc/node_counters.cpp csrc/sources.cpp -L/opt/rocm/lib -lamd_smi -lpthread -Wl,-rpath,/opt/rocm/lib
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

#include "node_counters.h"
#include "sources.h"

using namespace rocmdash;

int main(int argc, char** argv) {
  const double seconds = argc > 1 ? std::atof(argv[1]) : 1.0;
  const std::string dir = argc > 2 ? argv[2] : "/tmp";
  std::vector<std::string> paths;
  std::vector<std::shared_ptr<Source>> srcs;
  for (int d = 0; d < 3; ++d) {
    paths.push_back(dir + "/lane" + std::to_string(d) + "." + std::to_string(getpid()) + ".ring");
    auto s = make_synthetic_source("counter", 7 + d);
    srcs.push_back(d == 1 ? make_hanging_source(s, 0.2) : s);
  }
  auto pub = std::make_shared<ShmPublisher>(paths, srcs, 5000.0, 256);
  pub->start();
  std::atomic<bool> stop{false};
  std::atomic<long> bad{0}, rows{0};
  std::vector<std::thread> readers;
  for (int d = 0; d < 3; ++d) {
    readers.emplace_back([&, d] {
      ShmSource src(paths[d], 5000.0);
      std::vector<float> row(src.width());
      uint64_t last = 0;
      while (!stop.load()) {
        if (!src.sample(row.data())) continue;
        rows.fetch_add(1);
        for (float v : row)
          if (!(std::isnan(v) || std::isfinite(v))) bad.fetch_add(1);
        const uint64_t t = src.row_time_ns();
        if (t && last && t + 1000000000ull < last) bad.fetch_add(1);  // a fresh lane starts a new ring; never far back
        last = t;
      }
    });
  }
  const auto t0 = std::chrono::steady_clock::now();
  int replaced = 0;
  while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < seconds) {
    const auto st = pub->stats();
    if (st.size() != 3) bad.fetch_add(1);
    const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if ((replaced == 0 && el > 0.4) || (replaced == 1 && el > 0.7)) {
      // the second replacement hangs again (make_hanging_source with 0 s): left behind at stop
      auto s = make_synthetic_source("counter", 100 + replaced);
      pub->replace(1, replaced == 1 ? make_hanging_source(s, 0.0) : s);
      ++replaced;
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(2));
  }
  stop.store(true);
  for (auto& t : readers) t.join();
  const auto ts = std::chrono::steady_clock::now();
  pub->stop(0.2);
  const double stop_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - ts).count();
  const auto st = pub->stats();
  for (const auto& p : paths) std::remove(p.c_str());
  std::printf("rows=%ld bad=%ld replaced=%d lane1_gen=%g stop_s=%.3f lane0_samples=%g\n", rows.load(), bad.load(),
              replaced, st[1][5], stop_s, st[0][0]);
  std::fflush(stdout);
  std::_Exit(bad.load() == 0 && replaced == 2 && stop_s < 1.0 ? 0 : 1);  // a lane is still blocked: no static teardown
}
