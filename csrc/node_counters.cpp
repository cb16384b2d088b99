// One device-counter process per node: ShmPublisher (producer) / ShmSource (rank side).
// See node_counters.h and shm_ring.h.
#include "node_counters.h"

#include <pthread.h>
#include <sys/stat.h>
#include <unistd.h>

#include <chrono>
#include <cmath>
#include <ctime>
#include <random>
#include <stdexcept>

namespace rocmdash {

namespace {
uint64_t realtime_ns() {
  timespec ts;
  clock_gettime(CLOCK_REALTIME, &ts);
  return uint64_t(ts.tv_sec) * 1000000000ull + uint64_t(ts.tv_nsec);
}

void sleep_ns(int64_t ns) {
  if (ns <= 0) return;
  timespec ts{time_t(ns / 1000000000), long(ns % 1000000000)};
  nanosleep(&ts, nullptr);
}
}  // namespace

// ------------------------------------------------------------------ producer
ShmPublisher::ShmPublisher(const std::vector<std::string>& paths, std::vector<std::shared_ptr<Source>> sources,
                           double hz, uint64_t cap)
    : src_(std::move(sources)), hz_(hz) {
  if (paths.size() != src_.size() || src_.empty()) throw std::invalid_argument("one ring path per source");
  if (!(hz > 0)) throw std::invalid_argument("rate must be > 0");
  std::random_device rd;
  const uint64_t gen = (uint64_t(rd()) << 32) ^ rd() ^ uint64_t(getpid());
  for (size_t i = 0; i < src_.size(); ++i) {
    if (!src_[i]) throw std::invalid_argument("null source");
    rings_.push_back(ShmRing::create(paths[i], src_[i]->width(), cap, hz, src_[i]->kind(), src_[i]->backend(),
                                     gen | 1));
    rows_.emplace_back(src_[i]->width());
  }
  samples_.assign(src_.size(), 0);
  failures_.assign(src_.size(), 0);
  total_us_.assign(src_.size(), 0.0);
  last_us_.assign(src_.size(), 0.0);
}

ShmPublisher::~ShmPublisher() { stop(); }

void ShmPublisher::start() {
  if (running_.exchange(true)) return;
  th_ = std::thread([this] { loop(); });
  pthread_setname_np(th_.native_handle(), "rd-counterd");
}

void ShmPublisher::stop() {
  if (!running_.exchange(false)) return;
  if (th_.joinable()) th_.join();
}

// Absolute deadlines (no drift); a tick that overran skips to the next due deadline.
void ShmPublisher::loop() {
  const int64_t period = int64_t(1e9 / hz_);
  auto next = std::chrono::steady_clock::now();
  while (running_.load(std::memory_order_relaxed)) {
    for (size_t i = 0; i < src_.size(); ++i) {
      const auto t0 = std::chrono::steady_clock::now();
      const uint64_t ts = realtime_ns();
      const bool ok = src_[i]->sample(rows_[i].data());
      const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
      ShmRingHeader* h = rings_[i].header();
      if (ok) rings_[i].push(rows_[i].data(), ts);
      else h->failures.fetch_add(1, std::memory_order_relaxed);
      h->read_ns_total.fetch_add(uint64_t(us * 1e3), std::memory_order_relaxed);
      h->beat_ns.store(realtime_ns(), std::memory_order_release);
      std::lock_guard<std::mutex> lk(mu_);
      (ok ? samples_ : failures_)[i] += 1;
      total_us_[i] += us;
      last_us_[i] = us;
    }
    next += std::chrono::nanoseconds(period);
    auto now = std::chrono::steady_clock::now();
    if (now > next + std::chrono::nanoseconds(period)) next = now;  // overrun: no burst to catch up
    while (running_.load(std::memory_order_relaxed) && std::chrono::steady_clock::now() < next) {
      const int64_t left = std::chrono::duration_cast<std::chrono::nanoseconds>(next - std::chrono::steady_clock::now()).count();
      sleep_ns(std::min<int64_t>(left, 50000000));  // wake at least every 50 ms to see stop()
    }
  }
}

std::vector<std::vector<double>> ShmPublisher::stats() const {
  std::lock_guard<std::mutex> lk(mu_);
  std::vector<std::vector<double>> out;
  for (size_t i = 0; i < src_.size(); ++i) {
    const double n = double(samples_[i] + failures_[i]);
    out.push_back({double(samples_[i]), double(failures_[i]), n > 0 ? total_us_[i] / n : 0.0, last_us_[i]});
  }
  return out;
}

// ------------------------------------------------------------------ rank side
ShmSource::ShmSource(std::string path, double hz, std::string kind)
    : path_(std::move(path)), hz_(hz), kind_(std::move(kind)), backend_("node-counterd") {
  if (!(hz > 0)) throw std::invalid_argument("rate must be > 0");
  width_ = kind_ == "counter" ? uint32_t(CTR_NUM_FIELDS) : uint32_t(SMI_NUM_FIELDS);
  ensure_open();  // best effort: the node's counter process may start after this rank
}

bool ShmSource::ensure_open() {
  struct stat st;
  if (ring_.valid()) {
    // the producer started again: a new file replaced the old one
    if (::stat(path_.c_str(), &st) != 0 || st.st_ino == inode_) return true;
  }
  try {
    ino_t ino = 0;
    ShmRing r = ShmRing::open(path_, &ino);
    if (r.width() != width_) return false;  // another layout: never mixed into this ring
    ring_ = std::move(r);
    inode_ = ino;
    generation_ = ring_.header()->generation;
    next_ = ring_.head();  // new rows only: counter rows are rates of their own interval
    reopens_.fetch_add(1, std::memory_order_relaxed);
    return true;
  } catch (const std::exception&) {
    return ring_.valid();
  }
}

// One row per call, in order: the oldest row not handed out yet, or - when none is
// there - sleep until the next one is due (its predecessor's time + one period), then
// poll briefly. No row within 1.5 periods (the counter process is slow, restarting or
// gone) is a failed read: the rank's health rows count it and its window goes stale.
bool ShmSource::sample(float* row) {
  const int64_t period = int64_t(1e9 / hz_);
  const auto t_end = std::chrono::steady_clock::now() + std::chrono::nanoseconds(period + period / 2);
  bool checked_file = false;
  for (;;) {
    if (!ring_.valid() && !ensure_open()) {
      sleep_ns(period);
      return false;
    }
    const uint64_t h = ring_.head();
    if (h > next_) {
      const uint64_t cap = ring_.cap();
      if (h - next_ > cap / 2) {  // fell far behind: jump to the newest rows
        skipped_.fetch_add(h - 1 - next_, std::memory_order_relaxed);
        next_ = h - 1;
      }
      uint64_t ts = 0;
      if (!ring_.read(next_, row, &ts)) {  // overwritten while copied: take the newest
        torn_.fetch_add(1, std::memory_order_relaxed);
        next_ = ring_.head() - 1;
        continue;
      }
      ++next_;
      row_ts_ = ts;
      last_ts_ = ts;
      return true;
    }
    const auto now = std::chrono::steady_clock::now();
    if (now >= t_end) {
      if (!checked_file) {  // a restarted producer writes a new file: follow it once
        checked_file = true;
        ensure_open();
        if (ring_.valid() && ring_.head() > next_) continue;
      }
      return false;
    }
    // sleep until the next row is due (or 200 us, polling near the due time)
    int64_t wait = 200000;
    if (last_ts_) {
      const int64_t due = int64_t(last_ts_ + uint64_t(period)) - int64_t(realtime_ns()) - 300000;
      if (due > wait) wait = due;
    }
    const int64_t left = std::chrono::duration_cast<std::chrono::nanoseconds>(t_end - now).count();
    sleep_ns(std::min(wait, left));
  }
}

std::vector<std::pair<std::string, double>> ShmSource::counts() const {
  std::vector<std::pair<std::string, double>> out = {
      {"shm_reopens", double(reopens_.load())},
      {"shm_rows_skipped", double(skipped_.load())},
      {"shm_torn_reads", double(torn_.load())},
  };
  if (ring_.valid()) {
    const ShmRingHeader* h = ring_.header();
    out.push_back({"shm_producer_pid", double(h->producer_pid)});
    out.push_back({"shm_producer_failures", double(h->failures.load())});
    out.push_back({"shm_producer_beat_age_s",
                   h->beat_ns.load() ? (double(realtime_ns()) - double(h->beat_ns.load())) * 1e-9 : NAN});
  }
  return out;
}

}  // namespace rocmdash
