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
namespace {
// Blocks every read once `after_s` passed since the first one (fault injection).
class HangingSource final : public Source {
 public:
  HangingSource(std::shared_ptr<Source> inner, double after_s) : inner_(std::move(inner)), after_s_(after_s) {}
  uint32_t width() const override { return inner_->width(); }
  std::string kind() const override { return inner_->kind(); }
  std::string backend() const override { return inner_->backend(); }
  GpuInfo info() const override { return inner_->info(); }
  bool sample(float* row) override {
    const auto now = std::chrono::steady_clock::now();
    if (!started_) {
      started_ = true;
      t0_ = now;
    }
    if (std::chrono::duration<double>(now - t0_).count() >= after_s_)
      for (;;) sleep_ns(1000000000);  // a read that never returns
    return inner_->sample(row);
  }

 private:
  std::shared_ptr<Source> inner_;
  double after_s_;
  bool started_ = false;
  std::chrono::steady_clock::time_point t0_;
};
}  // namespace

std::shared_ptr<Source> make_hanging_source(std::shared_ptr<Source> inner, double after_s) {
  if (!inner) throw std::invalid_argument("null source");
  return std::make_shared<HangingSource>(std::move(inner), after_s);
}

// One GPU's lane: its source, ring and counters. The lane's thread holds it (shared), so
// an abandoned lane - or one whose read never returns - outlives the publisher safely.
struct ShmPublisher::Lane {
  std::shared_ptr<Source> src;
  ShmRing ring;
  std::vector<float> row;
  int gen = 0;
  size_t index = 0;
  int64_t period_ns = 0;
  std::chrono::steady_clock::time_point grid;
  std::shared_ptr<std::atomic<bool>> running;
  std::atomic<bool> abandoned{false};
  std::atomic<bool> exited{false};
  std::atomic<uint64_t> samples{0}, failures{0}, total_ns{0}, last_ns{0};
  std::atomic<int64_t> read_start_ns{0};  // steady-clock ns of the read in progress, 0 if none
};

namespace {
int64_t steady_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

// Absolute deadlines on the publisher's grid (every lane reads at the same instants, so a
// node's GPUs are sampled together); a tick that overran skips to the next due deadline.
void lane_loop(std::shared_ptr<ShmPublisher::Lane> L) {
  const auto period = std::chrono::nanoseconds(L->period_ns);
  auto next = L->grid;
  const auto now0 = std::chrono::steady_clock::now();
  if (next < now0) next += period * ((now0 - next) / period + 1);
  auto live = [&] { return L->running->load(std::memory_order_relaxed) && !L->abandoned.load(std::memory_order_relaxed); };
  while (live()) {
    while (live() && std::chrono::steady_clock::now() < next) {
      const int64_t left = std::chrono::duration_cast<std::chrono::nanoseconds>(next - std::chrono::steady_clock::now()).count();
      sleep_ns(std::min<int64_t>(left, 50000000));  // wake at least every 50 ms to see stop()
    }
    if (!live()) break;
    const int64_t t0 = steady_ns();
    L->read_start_ns.store(t0, std::memory_order_relaxed);
    const uint64_t ts = realtime_ns();
    const bool ok = L->src->sample(L->row.data());
    const int64_t dt = steady_ns() - t0;
    L->read_start_ns.store(0, std::memory_order_relaxed);
    if (L->abandoned.load(std::memory_order_acquire)) break;  // replaced while it read: push nothing
    ShmRingHeader* h = L->ring.header();
    if (ok) L->ring.push(L->row.data(), ts);
    else h->failures.fetch_add(1, std::memory_order_relaxed);
    h->read_ns_total.fetch_add(uint64_t(dt), std::memory_order_relaxed);
    h->beat_ns.store(realtime_ns(), std::memory_order_release);
    (ok ? L->samples : L->failures).fetch_add(1, std::memory_order_relaxed);
    L->total_ns.fetch_add(uint64_t(dt), std::memory_order_relaxed);
    L->last_ns.store(uint64_t(dt), std::memory_order_relaxed);
    next += period;
    const auto now = std::chrono::steady_clock::now();
    if (now > next) next += period * ((now - next) / period + 1);  // overrun: no burst to catch up
  }
  L->exited.store(true, std::memory_order_release);
}
}  // namespace

ShmPublisher::ShmPublisher(const std::vector<std::string>& paths, std::vector<std::shared_ptr<Source>> sources,
                           double hz, uint64_t cap)
    : paths_(paths), cap_(cap), hz_(hz), running_(std::make_shared<std::atomic<bool>>(false)),
      epoch_(std::chrono::steady_clock::now()) {
  if (paths.size() != sources.size() || sources.empty()) throw std::invalid_argument("one ring path per source");
  if (!(hz > 0)) throw std::invalid_argument("rate must be > 0");
  std::random_device rd;
  gen_ = ((uint64_t(rd()) << 32) ^ rd() ^ uint64_t(getpid())) | 1;
  for (size_t i = 0; i < sources.size(); ++i) lanes_.push_back(make_lane(i, std::move(sources[i]), 0));
}

std::shared_ptr<ShmPublisher::Lane> ShmPublisher::make_lane(size_t i, std::shared_ptr<Source> src, int gen) {
  if (!src) throw std::invalid_argument("null source");
  auto L = std::make_shared<Lane>();
  L->ring = ShmRing::create(paths_[i], src->width(), cap_, hz_, src->kind(), src->backend(), gen_, gen);
  L->row.assign(src->width(), 0.f);
  L->src = std::move(src);
  L->gen = gen;
  L->index = i;
  L->period_ns = int64_t(1e9 / hz_);
  L->grid = epoch_;
  L->running = running_;
  return L;
}

void ShmPublisher::launch(const std::shared_ptr<Lane>& L) {
  std::thread th(lane_loop, L);
  pthread_setname_np(th.native_handle(), ("rd-counterd" + std::to_string(L->index)).substr(0, 15).c_str());
  th.detach();  // the lane owns its state; stop() waits on `exited`
}

ShmPublisher::~ShmPublisher() { stop(); }

void ShmPublisher::start() {
  if (running_->exchange(true)) return;
  std::lock_guard<std::mutex> lk(mu_);
  for (auto& L : lanes_) launch(L);
}

void ShmPublisher::stop(double grace_s) {
  if (!running_->exchange(false)) return;
  std::vector<std::shared_ptr<Lane>> all;
  {
    std::lock_guard<std::mutex> lk(mu_);
    all = lanes_;
    all.insert(all.end(), left_.begin(), left_.end());
  }
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::duration<double>(grace_s);
  for (auto& L : all)
    while (!L->exited.load(std::memory_order_acquire) && std::chrono::steady_clock::now() < deadline)
      sleep_ns(1000000);
  // a lane still inside a read stays behind: it holds its own state and ends with its read
}

int ShmPublisher::replace(size_t i, std::shared_ptr<Source> src) {
  std::lock_guard<std::mutex> lk(mu_);
  if (i >= lanes_.size()) throw std::out_of_range("no such lane");
  auto old = lanes_[i];
  auto L = make_lane(i, std::move(src), old->gen + 1);  // may throw: then the old lane stays
  old->abandoned.store(true, std::memory_order_release);
  left_.push_back(old);
  lanes_[i] = L;
  if (running_->load()) launch(L);
  return L->gen;
}

std::vector<std::vector<double>> ShmPublisher::stats() const {
  std::lock_guard<std::mutex> lk(mu_);
  std::vector<std::vector<double>> out;
  const uint64_t now_rt = realtime_ns();
  const int64_t now = steady_ns();
  for (const auto& L : lanes_) {
    const double n = double(L->samples.load() + L->failures.load());
    const uint64_t beat = L->ring.header()->beat_ns.load(std::memory_order_acquire);
    const int64_t rs = L->read_start_ns.load(std::memory_order_relaxed);
    out.push_back({double(L->samples.load()), double(L->failures.load()), n > 0 ? double(L->total_ns.load()) * 1e-3 / n : 0.0,
                   double(L->last_ns.load()) * 1e-3, beat ? double(now_rt - std::min(now_rt, beat)) * 1e-9 : NAN,
                   double(L->gen), rs ? double(now - rs) * 1e-9 : 0.0});
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
