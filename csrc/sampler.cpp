#include "sampler.h"

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

void Sampler::worker_loop() {
  std::unique_lock<std::mutex> lk(wmu_);
  for (;;) {
    wcv_.wait(lk, [this] { return wstop_ || wstate_ == 1; });
    if (wstop_) return;
    lk.unlock();
    const bool ok = do_sample();
    lk.lock();
    wresult_ = ok;
    wstate_ = 2;
    wcv_.notify_all();
  }
}

void Sampler::request() {
  if (running_.load()) throw std::runtime_error("request() while the sampler thread is running (SPSC ring)");
  std::lock_guard<std::mutex> lk(wmu_);
  if (wstate_ == 1) throw std::runtime_error("request() while a request is pending");
  if (!worker_.joinable()) worker_ = std::thread([this] { worker_loop(); });
  wstate_ = 1;
  wcv_.notify_all();
}

bool Sampler::wait() {
  std::unique_lock<std::mutex> lk(wmu_);
  if (wstate_ == 0) return false;
  wcv_.wait(lk, [this] { return wstate_ == 2; });
  wstate_ = 0;
  return wresult_;
}

bool Sampler::do_sample() {
  const auto t0 = std::chrono::steady_clock::now();
  const uint64_t ts = realtime_ns();
  const bool ok = src_->sample(row_.data());
  if (ok) ring_->push(row_.data(), ts);
  const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
  std::lock_guard<std::mutex> lk(stats_mu_);
  if (ok) ++st_.samples;
  else ++st_.failures;
  st_.last_us = us;
  if (us > st_.max_us) st_.max_us = us;
  total_us_ += us;
  const uint64_t calls = st_.samples + st_.failures;
  st_.mean_us = total_us_ / double(calls);
  return ok;
}

bool Sampler::sample_once() {
  if (running_.load()) throw std::runtime_error("sample_once() while the sampler thread is running (SPSC ring)");
  return do_sample();
}

void Sampler::loop() {
  using clock = std::chrono::steady_clock;
  const auto period = std::chrono::duration_cast<clock::duration>(std::chrono::duration<double>(1.0 / hz_));
  auto next = clock::now();
  while (running_.load(std::memory_order_relaxed)) {
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
  bool expected = false;
  if (!running_.compare_exchange_strong(expected, true)) return;
  th_ = std::thread([this] { loop(); });
}

void Sampler::stop() {
  bool expected = true;
  if (!running_.compare_exchange_strong(expected, false)) return;
  if (th_.joinable()) th_.join();
}

SamplerStats Sampler::stats() const {
  std::lock_guard<std::mutex> lk(stats_mu_);
  return st_;
}

}  // namespace rocmdash
