#include "device_window.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <cstdio>
#include <stdexcept>
#include <string>

#include "tagged.h"
#include "window_stats.h"

namespace rocmdash {

namespace {
bool g_pinned = false;

void* pinned_alloc(size_t bytes, bool* pinned) {
  if (g_pinned) {
    void* p = nullptr;
    // Mapped + coherent (fine-grained): the stats kernel reads new rows straight from
    // this memory (pull mode, window_stats.h) and must always see the CPU's latest
    // stores, never a stale GPU-cached line.
    if (hipHostMalloc(&p, bytes, hipHostMallocMapped | hipHostMallocCoherent) == hipSuccess ||
        hipHostMalloc(&p, bytes, hipHostMallocDefault) == hipSuccess) {
      *pinned = true;
      return p;
    }
    (void)hipGetLastError();
  }
  *pinned = false;
  return std::aligned_alloc(4096, (bytes + 4095) / 4096 * 4096);
}

void pinned_release(void* p, bool pinned) {
  if (!p) return;
  if (pinned) (void)hipHostFree(p);
  else std::free(p);
}

void check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

// The device ring, resident sorted windows and series states. (Uncached device memory
// for them - loads and stores bypassing L2 - measured no different in the kernel trace:
// profiles/r02/onerow/trace_ab_k1_k10.txt.)
void* window_alloc(size_t bytes) {
  void* p = nullptr;
  check(hipMalloc(&p, bytes), "hipMalloc");
  return p;
}

// Switch the calling thread to `dev` and restore its previous device on scope exit, so
// a refresh never changes the device PyTorch (or any caller) believes is current.
struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    check(hipGetDevice(&prev), "hipGetDevice");
    if (prev != dev) check(hipSetDevice(dev), "hipSetDevice");
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};
}  // namespace

HostAlloc& host_allocator() {
  static HostAlloc a{&pinned_alloc, &pinned_release};
  return a;
}

void set_pinned_host_rings(bool on) { g_pinned = on; }

namespace {
bool g_pull = true;
}
void set_pull_mode(bool on) { g_pull = on; }
bool pull_enabled() { return g_pull; }

int hip_device_count() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return n;
}

uint64_t hip_device_bdf(int device) {
  hipDeviceProp_t p{};
  check(hipGetDeviceProperties(&p, device), "hipGetDeviceProperties");
  return (uint64_t(p.pciDomainID) << 32) | (uint64_t(p.pciBusID) << 8) | (uint64_t(p.pciDeviceID) << 3);
}

DeviceWindowSet::DeviceWindowSet(uint32_t window, int device) : window_(window), device_(device) {
  if (window < 2 || (window & (window - 1)) || window > 32768)
    throw std::invalid_argument("window must be a power of two in [2, 32768]");
  if (!g_pinned) return;  // completion flag only with pinned, mapped host memory
  DeviceGuard guard(device_);
  void* h = nullptr;
  if (hipHostMalloc(&h, 64, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) {
    (void)hipGetLastError();
    return;
  }
  void* d = nullptr;
  if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess || hipMalloc(reinterpret_cast<void**>(&wg_counter_), 64) != hipSuccess) {
    (void)hipGetLastError();
    (void)hipHostFree(h);
    wg_counter_ = nullptr;
    return;
  }
  check(hipMemset(wg_counter_, 0, 64), "hipMemset");
  done_host_ = static_cast<uint32_t*>(h);
  done_dev_ = static_cast<uint32_t*>(d);
  __atomic_store_n(done_host_, 0u, __ATOMIC_RELEASE);
}

bool spin_for_flag(const uint32_t* flag, uint32_t seq, double timeout_us) {
  if (flag == nullptr || seq == 0) return false;
  auto reached = [&] { return int32_t(__atomic_load_n(flag, __ATOMIC_ACQUIRE) - seq) >= 0; };
  if (reached()) return true;
  const auto end = std::chrono::steady_clock::now() + std::chrono::duration<double, std::micro>(timeout_us);
  SpinBackoff wait;  // tagged.h: spin, then sleep-poll
  for (;;) {
    if (reached()) return true;
    if (wait.pause() && std::chrono::steady_clock::now() >= end) return reached();
  }
}

bool DeviceWindowSet::wait_done(uint32_t seq, double timeout_us) const {
  if (seq == 0) return false;
  WaitGuard busy(&waiting_);
  if (seq != tag_seq_ || tag_dst_ == nullptr) {
    // only a flag refresh at or after `seq` moves the flag: an older tagged refresh with
    // none after it is never signalled there - say so now instead of burning the timeout
    if (flag_seq_ == 0 || int32_t(flag_seq_ - seq) < 0) return false;
    return spin_for_flag(done_host_, seq, timeout_us);
  }
  const TagScan s = wait_tagged(tag_host_, tag_n_ * uint32_t(STAT_NUM), seq, tag_dst_, timeout_us);  // tagged.h
  if (s == TagScan::kSuperseded) ++superseded_;
  return s == TagScan::kDone;
}

DeviceWindowSet::~DeviceWindowSet() {
  int cur = 0;
  (void)hipGetDevice(&cur);
  (void)hipSetDevice(device_);
  for (auto& r : rings_) {
    if (r.dev) (void)hipFree(r.dev);
    if (r.sorted) (void)hipFree(r.sorted);
    if (r.state) (void)hipFree(r.state);
  }
  if (wg_counter_) (void)hipFree(wg_counter_);
  if (done_host_) (void)hipHostFree(done_host_);
  if (tag_host_) (void)hipHostFree(tag_host_);
  (void)hipSetDevice(cur);
}

uint32_t DeviceWindowSet::add_ring(std::shared_ptr<SeriesRing> ring) {
  if (!ring) throw std::invalid_argument("null ring");
  const uint64_t D = dev_rows();
  if (ring->capacity() % D)
    throw std::invalid_argument("ring capacity must be a multiple of 2 x window (the device ring depth)");
  RingState rs;
  rs.ring = std::move(ring);
  rs.first_series = nseries_;
  if (rs.ring->pinned() && pull_enabled()) {
    void* dptr = nullptr;
    if (hipHostGetDevicePointer(&dptr, rs.ring->rows(), 0) == hipSuccess && dptr) rs.host_dev = static_cast<const float*>(dptr);
    else (void)hipGetLastError();
  }
  const uint32_t width = rs.ring->width();
  DeviceGuard guard(device_);
  const size_t ring_bytes = size_t(D) * width * sizeof(float);
  // + one sort width of slack: the one-row kernel path loads whole float4 groups up to
  // the sort width from any series' half, past `window_` (values it masks out)
  const size_t sorted_bytes = (size_t(2) * window_ * width + sort_width_for(window_)) * sizeof(float);
  const size_t state_bytes = size_t(width) * sizeof(SeriesState);
  rs.dev = static_cast<float*>(window_alloc(ring_bytes));
  rs.sorted = static_cast<float*>(window_alloc(sorted_bytes));
  rs.state = static_cast<SeriesState*>(window_alloc(state_bytes));
  check(hipMemset(rs.dev, 0, ring_bytes), "hipMemset");
  check(hipMemset(rs.state, 0, state_bytes), "hipMemset");  // valid = 0: first refresh sorts
  nseries_ += width;
  rings_.push_back(std::move(rs));
  return rings_.back().first_series;
}

void DeviceWindowSet::invalidate() {
  DeviceGuard guard(device_);
  for (auto& r : rings_) {
    r.copied = 0;
    r.state_valid = false;
    check(hipMemset(r.state, 0, size_t(r.ring->width()) * sizeof(SeriesState)), "hipMemset");
  }
}

bool DeviceWindowSet::ensure_tags(void* stream) {
  if (tag_host_ != nullptr && tag_cap_ >= nseries_) return true;
  if (done_host_ == nullptr) return false;  // no pinned, mapped host memory
  if (tag_host_) {  // grown (a ring added after a refresh): no kernel may still write the old
    // one - the tagged refreshes that wrote it ran on tag_stream_ (then `stream`, in order)
    (void)hipStreamSynchronize(static_cast<hipStream_t>(tag_stream_));
    if (stream != tag_stream_) (void)hipStreamSynchronize(static_cast<hipStream_t>(stream));
    (void)hipHostFree(tag_host_);
  }
  tag_host_ = tag_dev_ = nullptr;
  tag_cap_ = 0;
  const size_t bytes = size_t(nseries_) * STAT_NUM * sizeof(uint64_t);
  void* h = nullptr;
  void* d = nullptr;
  if (hipHostMalloc(&h, bytes, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) {
    (void)hipGetLastError();
    (void)hipHostFree(h);
    return false;
  }
  std::memset(h, 0, bytes);  // tag 0: never a refresh's sequence number
  tag_host_ = static_cast<uint64_t*>(h);
  tag_dev_ = static_cast<uint64_t*>(d);
  tag_cap_ = nseries_;
  return true;
}

uint32_t DeviceWindowSet::refresh(float* out, void* stream_ptr, float p0, float p1, float p2, int signal) {
  auto stream = static_cast<hipStream_t>(stream_ptr);
  if (wait_in_progress(&waiting_)) throw std::logic_error("refresh: a wait on the previous refresh is in progress");
  DeviceGuard guard(device_);
  if (signal == kSignalTagged && !ensure_tags(stream_ptr)) signal = kSignalFlag;
  if (signal != kSignalNone && done_host_ == nullptr) signal = kSignalNone;
  const uint64_t W = window_;
  const uint64_t D = dev_rows();
  const uint32_t pad = sort_width_for(window_);
  StatsArgs args{};
  args.pct[0] = p0;
  args.pct[1] = p1;
  args.pct[2] = p2;
  uint32_t first_in_launch = 0;
  bool all_inc = true;  // host-side prediction of the device path for this launch
  uint64_t max_new = 0;  // most rows entering any series of this launch (launch width choice)
  uint32_t seq = 0;  // 0 = no completion signal
  if (signal != kSignalNone) {
    if (++seq_ == 0) ++seq_;  // skip 0 on wrap
    seq = seq_;
  }
  // tagged: the kernel never writes `out` (host memory); wait_done() fills it
  float* const kout = signal == kSignalTagged ? nullptr : out;
  auto flush = [&](bool last) {
    if (!args.num_series) return;
    if (signal == kSignalFlag) {
      // ONLY the refresh's last launch publishes: an earlier launch's last workgroup
      // would flag `seq` while later launches have not written their rows. Stream order
      // puts every earlier launch's outputs before the last launch starts.
      args.wg_counter = last ? wg_counter_ : nullptr;
      args.done_flag = last ? done_dev_ : nullptr;
      args.wg_expect = wg_total_ + args.num_series;  // the device counter's value once this grid is done
      args.done_seq = seq;
    } else if (signal == kSignalTagged) {
      args.tagged_out = tag_dev_ + size_t(first_in_launch) * STAT_NUM;
      args.done_seq = seq;
    }
    check(hipError_t(launch_window_stats(args, pad, kout ? kout + size_t(first_in_launch) * STAT_NUM : nullptr, stream,
                                         all_inc, uint32_t(std::min<uint64_t>(max_new, 0xFFFFFFFFu)))),
          "window_stats launch");
    if (signal == kSignalFlag && last) wg_total_ += args.num_series;  // only a grid that counted counts
    ++st_.launches;
    if (all_inc) ++st_.incremental_launches;
    first_in_launch += args.num_series;
    args.num_series = 0;
    args.num_rings = 0;
    all_inc = true;
    max_new = 0;
  };
  for (auto& r : rings_) {
    const auto& ring = *r.ring;
    const uint32_t width = ring.width();
    const uint64_t h = ring.head();
    const uint64_t cap_mask = ring.capacity() - 1;
    const uint32_t n = uint32_t(std::min<uint64_t>(h, W));
    // Mirror of the kernel's path choice (window_stats.hip): the state left by the
    // previous launch covers [last_head - last_n, last_head).
    const bool inc = r.state_valid && h >= r.last_head && h - r.last_head <= uint64_t(kMaxIncremental) &&
                     (h - n) >= (r.last_head - r.last_n) &&
                     (h - n) - (r.last_head - r.last_n) <= uint64_t(kMaxIncremental) &&
                     (r.last_head - r.last_n) + D >= h;
    const uint64_t prev_head = r.last_head;
    const uint32_t prev_n = r.last_n;
    const uint32_t prev_cur = r.cur;
    // the half this launch leaves current (kernel rule): the incremental path updates
    // it in place, a full sort writes the other one
    r.cur = r.state_valid ? (inc ? r.cur : (r.cur ^ 1u)) : 0u;
    r.state_valid = true;
    r.last_head = h;
    r.last_n = n;
    // Entering rows of an incremental launch: the newest <= kInlineRows travel by value
    // in the kernel argument, older ones (pinned ring) are pulled by the kernel from
    // the mapped host ring. Before a full sort (which needs the whole window; reading W
    // column-strided values over the host link per series is slow) the new rows are
    // staged with hipMemcpyAsync instead: at most the device ring's depth, in segments
    // split at device-ring wraps (the host ring's capacity is a multiple of D, so a
    // segment never crosses a host wrap either). All keep the device ring complete.
    const uint64_t k_new = inc ? h - prev_head : 0;
    const uint32_t n_inline =
        (inc && width <= uint32_t(kMaxInlineWidth)) ? uint32_t(std::min<uint64_t>(k_new, kInlineRows)) : 0;
    const bool pull = inc && k_new > n_inline && r.host_dev != nullptr;
    const bool staged = !inc || (k_new > n_inline && !pull);
    uint64_t lo = staged ? std::max<uint64_t>(r.copied, h > D ? h - D : 0) : h;
    while (lo < h) {
      const uint64_t seg_end = std::min<uint64_t>(h, (lo / D + 1) * D);
      const uint64_t rows = seg_end - lo;
      const size_t bytes = size_t(rows) * width * sizeof(float);
      check(hipMemcpyAsync(r.dev + (lo & (D - 1)) * width, ring.rows() + (lo & cap_mask) * width, bytes,
                           hipMemcpyHostToDevice, stream),
            "hipMemcpyAsync");
      st_.rows_copied += rows;
      st_.bytes_copied += bytes;
      ++st_.memcpy_calls;
      lo = seg_end;
    }
    r.copied = h;
    if (args.num_rings == uint32_t(kMaxRingsPerLaunch) || args.num_series + width > uint32_t(kMaxSeriesPerLaunch))
      flush(false);
    const uint32_t ri = args.num_rings++;
    RingDesc& d = args.rings[ri];
    d.base = r.dev;
    d.host_rows = pull ? r.host_dev : nullptr;
    d.sorted = r.sorted;
    d.state = r.state;
    d.head = h;
    d.pred_head0 = inc ? prev_head : ~0ull;
    d.stride = width;
    d.cols = width;
    d.mask = uint32_t(D - 1);
    d.n = n;
    d.sorted_cap = window_;
    d.host_mask = uint32_t(cap_mask);
    d.pred_n0 = prev_n;
    d.pred_cur = prev_cur;
    d.n_inline = n_inline;
    for (uint32_t j = 0; j < n_inline; ++j) {  // rows h - n_inline .. h - 1 (complete: < head)
      const uint64_t row = h - n_inline + j;
      std::memcpy(d.inl[j], ring.rows() + (row & cap_mask) * width, size_t(width) * sizeof(float));
    }
    st_.pulled_series += pull ? width : 0;
    st_.inline_rows += n_inline;
    all_inc = all_inc && inc;
    max_new = std::max<uint64_t>(max_new, inc ? k_new : ~0ull);
    args.num_series += width;  // the ring's columns, in ring order (window_stats.h)
  }
  flush(true);
  ++st_.refreshes;
  if (signal == kSignalTagged) {
    tag_dst_ = out;
    tag_n_ = nseries_;
    tag_seq_ = seq;
    tag_stream_ = stream_ptr;
  } else if (signal == kSignalFlag) {
    flag_seq_ = seq;
  }
  return seq;
}

}  // namespace rocmdash
