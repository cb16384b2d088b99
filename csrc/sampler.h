// Fixed-rate sampler thread: Source -> SeriesRing.
//
// Reference counterpart: the `while True: ... time.sleep(REFRESH_INTERVAL)` loop of
// app.py:326-486, which couples sampling to rendering at 0.2 Hz. Here sampling runs
// on its own native thread at the source's rate (10 Hz amd-smi, 100 Hz counters),
// paced by absolute deadlines so it does not drift, and never waits for a refresh.
#pragma once

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "ring.h"
#include "sources.h"

namespace rocmdash {

struct SamplerStats {
  uint64_t samples = 0;   // rows pushed
  uint64_t failures = 0;  // sample() returned false
  uint64_t overruns = 0;  // deadlines missed by more than one period
  double last_us = 0.0;   // duration of the last sample() call
  double max_us = 0.0;
  double mean_us = 0.0;
  double p50_us = 0.0;  // over the last kRecent sample() calls
  double p99_us = 0.0;
};

class Sampler {
 public:
  Sampler(std::shared_ptr<Source> src, std::shared_ptr<SeriesRing> ring, double hz);
  ~Sampler();
  Sampler(const Sampler&) = delete;
  Sampler& operator=(const Sampler&) = delete;

  void start();
  // Free-running: the background thread reads back to back (the bench at N > 1: each
  // rank reads at its own pace, so no rank's refresh waits for another rank's read).
  // Reads start at most max_hz apart (a cap hardware reads never reach - 20 us against
  // their 50-80 us - that keeps instant synthetic sources from flooding the ring).
  void start_free(double max_hz);
  void stop();
  // Completed sample() calls (rows + failures), and the steady-clock time (ns, the
  // clock of Python's time.perf_counter_ns) at which the newest completed call started.
  uint64_t calls() const { return calls_.load(std::memory_order_acquire); }
  int64_t last_start_ns() const { return last_start_ns_.load(std::memory_order_acquire); }
  // Spin until calls() >= target or timeout_s elapses; returns calls().
  uint64_t wait_calls(uint64_t target, double timeout_s) const;
  bool running() const { return running_.load(); }
  // Synchronous sample on the caller's thread (closed-loop mode). The ring is SPSC:
  // this throws while the background thread is running.
  bool sample_once();
  // Asynchronous closed-loop sample on this sampler's worker thread: request()
  // returns at once, wait() blocks until the row is in the ring and returns whether
  // the read succeeded. One caller can so read several sources concurrently (an
  // amd-smi read and a device-counter read take ~130-200 us each on MI355X).
  void request();
  bool wait();
  SamplerStats stats() const;
  // samples / failures / overruns only: no percentile sort (read every refresh by
  // the per-rank health rows, rocmdash/runtime/pipeline.py)
  SamplerStats counts() const;
  // Durations (us) of the last min(calls, kRecent) sample() calls, oldest first.
  std::vector<float> recent_us() const;
  // Pin this sampler's threads (worker and background) to these CPUs, e.g. the GPU's
  // NUMA-local cores (rocmdash/runtime/agent.py). Empty = no pinning.
  void set_affinity(const std::vector<int>& cpus);
  // Hand-off between request()/wait() and the worker spins this long on an atomic
  // before sleeping on the condition variable: a futex wake-up from a deep C-state
  // costs tens of microseconds, as much as the sample itself.
  void set_spin_us(double us) { spin_ns_ = int64_t(us * 1000.0); }
  double hz() const { return hz_; }
  const std::shared_ptr<SeriesRing>& ring() const { return ring_; }
  const std::shared_ptr<Source>& source() const { return src_; }

 private:
  bool do_sample();
  void loop();

  std::shared_ptr<Source> src_;
  std::shared_ptr<SeriesRing> ring_;
  double hz_;
  std::vector<float> row_;
  std::atomic<bool> running_{false};
  std::atomic<bool> free_{false};
  int64_t free_min_ns_ = 0;
  std::atomic<uint64_t> calls_{0};
  std::atomic<int64_t> last_start_ns_{0};
  std::thread th_;
  void worker_loop();
  std::thread worker_;
  void apply_affinity(std::thread& t);
  std::mutex wmu_;
  std::condition_variable wcv_;
  std::atomic<int> wstate_{0};  // 0 idle, 1 requested, 2 done
  std::atomic<bool> wresult_{false};
  std::atomic<bool> wstop_{false};
  std::atomic<int64_t> spin_ns_{0};
  std::vector<int> cpus_;
  // the ring is single-producer: do_sample() holds this, so the background thread,
  // the request() worker and sample_once() can never push concurrently even if the
  // state checks below are raced by two controlling threads
  std::mutex produce_mu_;
  mutable std::mutex stats_mu_;
  SamplerStats st_;
  double total_us_ = 0.0;
  static constexpr int kRecent = 1024;
  std::vector<float> recent_us_ = std::vector<float>(kRecent, 0.0f);
};

}  // namespace rocmdash
