#include "sampler.h"

#include <pthread.h>

#include <string>
#include <sched.h>

#include <algorithm>
#include <chrono>
#include <ctime>
#include <stdexcept>

namespace rocmdash {

namespace {
uint64_t realtime_ns() {
  timespec ts;
  clock_gettime(CLOCK_REALTIME, &ts);
  return uint64_t(ts.tv_sec) * 1000000000ull + uint64_t(ts.tv_nsec);
}

inline void cpu_relax() { __builtin_ia32_pause(); }

// spin until pred() or `ns` elapse; true if pred() became true
template <class Pred>
bool spin_for(int64_t ns, Pred pred) {
  if (ns <= 0) return pred();
  const auto end = std::chrono::steady_clock::now() + std::chrono::nanoseconds(ns);
  for (int i = 0;; ++i) {
    if (pred()) return true;
    cpu_relax();
    if ((i & 63) == 63 && std::chrono::steady_clock::now() >= end) return pred();
  }
}
}  // namespace

Sampler::Sampler(std::shared_ptr<Source> src, std::shared_ptr<SeriesRing> ring, double hz)
    : src_(std::move(src)), ring_(std::move(ring)), hz_(hz) {
  if (!src_ || !ring_) throw std::invalid_argument("sampler needs a source and a ring");
  if (src_->width() != ring_->width()) throw std::invalid_argument("source width != ring width");
  if (!(hz > 0)) throw std::invalid_argument("sampling rate must be > 0");
  row_.resize(src_->width());
}

Sampler::~Sampler() {
  stop();
  {
    std::lock_guard<std::mutex> lk(wmu_);
    wstop_ = true;
  }
  wcv_.notify_all();
  if (worker_.joinable()) worker_.join();
}

// Thread names ("rd-smi", "rd-counter-w", ...) so per-thread CPU accounting
// (/proc/<pid>/task/*/comm, tools/footprint_probe.py) tells rocmdash's threads apart
// from the runtime's.
static void name_thread(std::thread& t, const std::string& kind, const char* suffix) {
  const std::string name = ("rd-" + kind + suffix).substr(0, 15);
  pthread_setname_np(t.native_handle(), name.c_str());
}

// Hand-off protocol: wstate_ 0 -> 1 (request, caller) -> 2 (done, worker) -> 0 (wait,
// caller). Every transition is an atomic store made under wmu_, so a side that went
// to sleep on wcv_ after re-checking the state under the lock cannot miss it; a side
// that is still spinning sees it without the futex round trip.
void Sampler::worker_loop() {
  for (;;) {
    const int64_t spin = spin_ns_.load(std::memory_order_relaxed);
    if (!spin_for(spin, [this] { return wstate_.load(std::memory_order_acquire) == 1 || wstop_.load(); })) {
      std::unique_lock<std::mutex> lk(wmu_);
      wcv_.wait(lk, [this] { return wstop_.load() || wstate_.load() == 1; });
    }
    if (wstop_.load()) return;
    const bool ok = do_sample();
    {
      std::lock_guard<std::mutex> lk(wmu_);
      wresult_.store(ok, std::memory_order_relaxed);
      wstate_.store(2, std::memory_order_release);
    }
    wcv_.notify_all();
  }
}

void Sampler::request() {
  if (running_.load()) throw std::runtime_error("request() while the sampler thread is running (SPSC ring)");
  {
    std::lock_guard<std::mutex> lk(wmu_);
    if (wstate_.load() == 1) throw std::runtime_error("request() while a request is pending");
    if (!worker_.joinable()) {
      worker_ = std::thread([this] { worker_loop(); });
      name_thread(worker_, src_->kind(), "-w");
      apply_affinity(worker_);
    }
    wstate_.store(1, std::memory_order_release);
  }
  wcv_.notify_all();
}

bool Sampler::wait() {
  if (wstate_.load(std::memory_order_acquire) == 0) return false;
  if (!spin_for(spin_ns_.load(std::memory_order_relaxed), [this] { return wstate_.load(std::memory_order_acquire) == 2; })) {
    std::unique_lock<std::mutex> lk(wmu_);
    wcv_.wait(lk, [this] { return wstate_.load() == 2; });
  }
  const bool ok = wresult_.load(std::memory_order_relaxed);
  std::lock_guard<std::mutex> lk(wmu_);
  wstate_.store(0, std::memory_order_release);
  return ok;
}

void Sampler::apply_affinity(std::thread& t) {
  if (cpus_.empty() || !t.joinable()) return;
  cpu_set_t set;
  CPU_ZERO(&set);
  for (int c : cpus_)
    if (c >= 0 && c < CPU_SETSIZE) CPU_SET(c, &set);
  pthread_setaffinity_np(t.native_handle(), sizeof set, &set);  // best effort
}

void Sampler::set_affinity(const std::vector<int>& cpus) {
  cpus_ = cpus;
  apply_affinity(worker_);
  apply_affinity(th_);
}

bool Sampler::do_sample() {
  std::lock_guard<std::mutex> produce(produce_mu_);
  const auto t0 = std::chrono::steady_clock::now();
  const uint64_t ts = realtime_ns();
  const bool ok = src_->sample(row_.data());
  if (ok) {
    const uint64_t rt = src_->row_time_ns();
    ring_->push(row_.data(), rt ? rt : ts);
  }
  const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
  last_start_ns_.store(std::chrono::duration_cast<std::chrono::nanoseconds>(t0.time_since_epoch()).count(),
                       std::memory_order_relaxed);
  calls_.fetch_add(1, std::memory_order_release);
  std::lock_guard<std::mutex> lk(stats_mu_);
  if (ok) ++st_.samples;
  else ++st_.failures;
  st_.last_us = us;
  if (us > st_.max_us) st_.max_us = us;
  total_us_ += us;
  const uint64_t calls = st_.samples + st_.failures;
  st_.mean_us = total_us_ / double(calls);
  recent_us_[size_t((calls - 1) % kRecent)] = float(us);
  return ok;
}

bool Sampler::sample_once() {
  if (running_.load()) throw std::runtime_error("sample_once() while the sampler thread is running (SPSC ring)");
  if (wstate_.load(std::memory_order_acquire) != 0)
    throw std::runtime_error("sample_once() while a request() is pending or unwaited (SPSC ring)");
  return do_sample();
}

void Sampler::loop() {
  using clock = std::chrono::steady_clock;
  const auto period = std::chrono::duration_cast<clock::duration>(std::chrono::duration<double>(1.0 / hz_));
  auto next = clock::now();
  const bool free_running = free_.load();
  while (running_.load(std::memory_order_relaxed)) {
    if (free_running) {  // back to back, starts at least free_min_ns_ apart
      const auto due = next;
      // a long gap (a low cap on an instant source) sleeps, the last 100 us spin
      if (due - clock::now() > std::chrono::microseconds(300)) std::this_thread::sleep_until(due - std::chrono::microseconds(100));
      spin_for(std::chrono::duration_cast<std::chrono::nanoseconds>(due - clock::now()).count(),
               [&] { return clock::now() >= due || !running_.load(std::memory_order_relaxed); });
      next = clock::now() + std::chrono::nanoseconds(free_min_ns_);
      do_sample();
      continue;
    }
    do_sample();
    next += period;
    const auto now = clock::now();
    if (now > next + period) {  // fell more than a period behind: re-anchor, count it
      {
        std::lock_guard<std::mutex> lk(stats_mu_);
        ++st_.overruns;
      }
      next = now;
      continue;
    }
    std::this_thread::sleep_until(next);
  }
}

void Sampler::start() {
  if (wstate_.load(std::memory_order_acquire) != 0)
    throw std::runtime_error("start() while a request() is pending or unwaited (SPSC ring)");
  bool expected = false;
  if (!running_.compare_exchange_strong(expected, true)) return;
  th_ = std::thread([this] { loop(); });
  name_thread(th_, src_->kind(), "");
  apply_affinity(th_);
}

void Sampler::start_free(double max_hz) {
  if (!(max_hz > 0)) throw std::invalid_argument("start_free: max_hz must be > 0");
  if (running_.load()) throw std::runtime_error("start_free() while the sampler thread is running");
  if (wstate_.load(std::memory_order_acquire) != 0)
    throw std::runtime_error("start_free() while a request() is pending or unwaited (SPSC ring)");
  free_min_ns_ = int64_t(1e9 / max_hz);
  free_.store(true);
  start();
}

uint64_t Sampler::wait_calls(uint64_t target, double timeout_s) const {
  const auto end = std::chrono::steady_clock::now() + std::chrono::duration_cast<std::chrono::steady_clock::duration>(
                                                          std::chrono::duration<double>(timeout_s));
  for (int i = 0;; ++i) {
    const uint64_t c = calls_.load(std::memory_order_acquire);
    if (c >= target) return c;
    cpu_relax();
    if ((i & 63) == 63 && std::chrono::steady_clock::now() >= end) return calls_.load(std::memory_order_acquire);
  }
}

void Sampler::stop() {
  bool expected = true;
  if (!running_.compare_exchange_strong(expected, false)) return;
  if (th_.joinable()) th_.join();
  free_.store(false);
}

SamplerStats Sampler::counts() const {
  SamplerStats s;
  std::lock_guard<std::mutex> lk(stats_mu_);
  s.samples = st_.samples;
  s.failures = st_.failures;
  s.overruns = st_.overruns;
  return s;
}

std::vector<float> Sampler::recent_us() const {
  std::lock_guard<std::mutex> lk(stats_mu_);
  const uint64_t calls = st_.samples + st_.failures;
  const size_t n = size_t(std::min<uint64_t>(calls, kRecent));
  std::vector<float> v(n);
  for (size_t i = 0; i < n; ++i) v[i] = recent_us_[size_t((calls - n + i) % kRecent)];
  return v;
}

SamplerStats Sampler::stats() const {
  SamplerStats s;
  std::vector<float> v;
  {
    std::lock_guard<std::mutex> lk(stats_mu_);  // copy only; sort outside the sampler's lock
    s = st_;
    v.assign(recent_us_.begin(), recent_us_.begin() + long(std::min<uint64_t>(st_.samples + st_.failures, kRecent)));
  }
  const size_t n = v.size();
  if (n) {
    std::sort(v.begin(), v.end());
    s.p50_us = v[n / 2];
    s.p99_us = v[std::min(n - 1, size_t(0.99 * double(n)))];
  }
  return s;
}

}  // namespace rocmdash
