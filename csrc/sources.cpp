// Synthetic and amd-smi metric sources (see sources.h).
#include "sources.h"

#include <amd_smi/amdsmi.h>

#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <chrono>
#include <cstring>
#include <limits>
#include <mutex>
#include <stdexcept>

namespace rocmdash {

namespace {
const char* const kSmiNames[SMI_NUM_FIELDS + 1] = {
    "amd_gpu_edge_temperature", "amd_gpu_gfx_activity",     "amd_gpu_average_package_power",
    "amd_gpu_used_vram",        "amd_gpu_total_vram",       "amd_gpu_junction_temperature",
    "amd_gpu_memory_temperature", "amd_gpu_umc_activity",   "amd_gpu_xgmi_read_bandwidth",
    "amd_gpu_xgmi_write_bandwidth", "amd_gpu_pcie_bandwidth", nullptr};
const char* const kCtrNames[CTR_NUM_FIELDS + 1] = {
    "amd_gpu_mfma_utilization", "amd_gpu_hbm_read_bandwidth", "amd_gpu_hbm_write_bandwidth",
    "amd_gpu_gfx_busy", "amd_gpu_cu_active", nullptr};
constexpr float kNaN = std::numeric_limits<float>::quiet_NaN();
}  // namespace

const char* const* smi_field_names() { return kSmiNames; }
const char* const* ctr_field_names() { return kCtrNames; }

// =============================== synthetic ========================================
namespace {

class Rng {
 public:
  explicit Rng(uint64_t seed) : s_(seed ? seed : 0x9E3779B97F4A7C15ull) {}
  uint64_t next() {  // splitmix64
    uint64_t z = (s_ += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
  double uniform() { return double(next() >> 11) * (1.0 / 9007199254740992.0); }
  double normal() {  // Irwin-Hall(12) - 6: cheap, bounded, good enough for telemetry noise
    double s = 0;
    for (int i = 0; i < 12; ++i) s += uniform();
    return s - 6.0;
  }

 private:
  uint64_t s_;
};

// Shared workload model: phase 0 idle, 1 compute-bound (MFMA), 2 memory-bound.
struct Workload {
  explicit Workload(uint64_t seed) : rng(seed) {}
  void step() {
    if (rng.uniform() < 0.01) phase = int(rng.uniform() * 3.0) % 3;
    const double target = phase == 0 ? 3.0 : (phase == 1 ? 92.0 : 70.0);
    util += 0.15 * (target - util) + 2.0 * rng.normal();
    util = std::clamp(util, 0.0, 100.0);
  }
  Rng rng;
  int phase = 1;
  double util = 50.0;
};

class SyntheticSmi final : public Source {
 public:
  SyntheticSmi(uint64_t seed, double total) : w_(seed), xrng_(seed ^ 0x5A5A5A5Aull), total_(total), used_(0.35 * total) {}
  uint32_t width() const override { return SMI_NUM_FIELDS; }
  std::string kind() const override { return "smi"; }
  std::string backend() const override { return "synthetic"; }
  GpuInfo info() const override {
    GpuInfo g;
    g.model_number = "102-G36236-0C";
    g.product_name = "AMD Instinct MI355 OAM (synthetic)";
    g.market_name = g.product_name;
    g.power_limit_w = 1400.0;
    g.vram_total_mb = total_;
    g.edge_is_hotspot = true;
    return g;
  }
  bool sample(float* row) override {
    w_.step();
    const double power = 160.0 + 11.5 * w_.util + 8.0 * w_.rng.normal();
    hot_ += 0.05 * (32.0 + 0.045 * power - hot_) + 0.2 * w_.rng.normal();
    mem_ += 0.03 * (30.0 + 0.030 * power - mem_) + 0.1 * w_.rng.normal();
    if (w_.rng.uniform() < 0.02) used_target_ = (0.05 + 0.9 * w_.rng.uniform()) * total_;
    used_ += 0.1 * (used_target_ - used_);
    const double umc = w_.phase == 2 ? 0.8 * w_.util : 0.25 * w_.util;
    row[SMI_EDGE_TEMP] = float(hot_);
    row[SMI_GFX_ACTIVITY] = float(std::round(w_.util));
    row[SMI_SOCKET_POWER] = float(std::max(0.0, std::round(power)));
    row[SMI_USED_VRAM] = float(std::round(used_));
    row[SMI_TOTAL_VRAM] = float(total_);
    row[SMI_HOTSPOT_TEMP] = float(hot_);
    row[SMI_MEM_TEMP] = float(mem_);
    row[SMI_UMC_ACTIVITY] = float(std::clamp(umc, 0.0, 100.0));
    // collectives between the phases of a data-parallel step: xGMI traffic follows
    // the communication phase, host traffic stays small
    const double xgmi = w_.phase == 1 ? 2.2 * w_.util : 0.15 * w_.util;
    row[SMI_XGMI_READ_GBPS] = float(std::max(0.0, xgmi + 2.0 * w_.rng.normal()));
    row[SMI_XGMI_WRITE_GBPS] = float(std::max(0.0, xgmi + 2.0 * w_.rng.normal()));
    row[SMI_PCIE_GBPS] = float(std::max(0.0, std::round(1.0 + 0.05 * w_.util + w_.rng.normal())));
    // per XCD: the device's busy with a little imbalance, clocks that dip with power
    // (own generator: the row streams above stay what they were)
    std::array<float, 2 * kMaxXcds> x;
    for (int i = 0; i < kMaxXcds; ++i) {
      x[i] = float(std::clamp(std::round(w_.util + 1.5 * xrng_.normal()), 0.0, 100.0));
      x[kMaxXcds + i] = float(std::round(std::min(2400.0, 2900.0 - 0.45 * power) + 4.0 * xrng_.normal()));
    }
    std::lock_guard<std::mutex> lk(xcd_mu_);
    xcd_ = x;
    return true;
  }
  std::vector<float> xcd_detail() const override {
    std::lock_guard<std::mutex> lk(xcd_mu_);
    if (std::isnan(xcd_[0]) && std::isnan(xcd_[kMaxXcds])) return {};
    return std::vector<float>(xcd_.begin(), xcd_.end());
  }

 private:
  Workload w_;
  Rng xrng_;
  mutable std::mutex xcd_mu_;
  std::array<float, 2 * kMaxXcds> xcd_ = [] {
    std::array<float, 2 * kMaxXcds> a;
    a.fill(kNaN);
    return a;
  }();
  double total_, used_, used_target_ = 0.35 * 294896.0;
  double hot_ = 40.0, mem_ = 35.0;
};

class SyntheticCtr final : public Source {
 public:
  explicit SyntheticCtr(uint64_t seed) : w_(seed ^ 0xC0FFEEull) {}
  uint32_t width() const override { return CTR_NUM_FIELDS; }
  std::string kind() const override { return "counter"; }
  std::string backend() const override { return "synthetic"; }
  bool sample(float* row) override {
    w_.step();
    const double u = w_.util / 100.0;
    const double mfma = w_.phase == 1 ? 78.0 * u : (w_.phase == 2 ? 12.0 * u : 0.0);
    const double rd = w_.phase == 2 ? 5200.0 * u : 900.0 * u;
    row[CTR_MFMA_UTIL] = float(std::clamp(mfma + 1.5 * w_.rng.normal() * u, 0.0, 100.0));
    row[CTR_HBM_READ_GBPS] = float(std::max(0.0, rd + 60.0 * w_.rng.normal() * u));
    row[CTR_HBM_WRITE_GBPS] = float(std::max(0.0, 0.45 * rd + 30.0 * w_.rng.normal() * u));
    row[CTR_GFX_BUSY] = float(std::clamp(w_.util + 0.5 * w_.rng.normal(), 0.0, 100.0));
    row[CTR_CU_ACTIVE] = float(std::clamp(0.9 * w_.util + 0.5 * w_.rng.normal(), 0.0, 100.0));
    return true;
  }

 private:
  Workload w_;
};

}  // namespace

namespace {
class NullSource final : public Source {
 public:
  explicit NullSource(std::string kind) : kind_(std::move(kind)) {}
  uint32_t width() const override { return kind_ == "smi" ? SMI_NUM_FIELDS : CTR_NUM_FIELDS; }
  std::string kind() const override { return kind_; }
  std::string backend() const override { return "unavailable"; }
  bool sample(float* row) override {
    for (uint32_t i = 0; i < width(); ++i) row[i] = kNaN;
    return true;
  }

 private:
  std::string kind_;
};
}  // namespace

namespace {
// Replays recorded rows (e.g. a capture of a live MI355X) in order, wrapping around:
// deterministic, hardware-shaped input for CPU tests and benchmarks.
class ReplaySource final : public Source {
 public:
  ReplaySource(std::string kind, std::vector<float> rows, uint32_t width, GpuInfo info)
      : kind_(std::move(kind)), rows_(std::move(rows)), width_(width), info_(std::move(info)) {}
  uint32_t width() const override { return width_; }
  std::string kind() const override { return kind_; }
  std::string backend() const override { return "replay"; }
  GpuInfo info() const override { return info_; }
  bool sample(float* row) override {
    const size_t n = rows_.size() / width_;
    std::memcpy(row, rows_.data() + (next_ % n) * width_, size_t(width_) * sizeof(float));
    ++next_;
    return true;
  }

 private:
  std::string kind_;
  std::vector<float> rows_;
  uint32_t width_;
  GpuInfo info_;
  uint64_t next_ = 0;
};
}  // namespace

std::shared_ptr<Source> make_replay_source(const std::string& kind, const std::vector<float>& rows, uint32_t width,
                                           const GpuInfo& info) {
  const uint32_t want = kind == "smi" ? uint32_t(SMI_NUM_FIELDS) : kind == "counter" ? uint32_t(CTR_NUM_FIELDS) : 0;
  if (!want) throw std::invalid_argument("replay source kind must be 'smi' or 'counter'");
  if (width != want) throw std::invalid_argument("replay rows have the wrong width for this kind");
  if (rows.empty() || rows.size() % width) throw std::invalid_argument("replay needs at least one complete row");
  return std::make_shared<ReplaySource>(kind, rows, width, info);
}

std::shared_ptr<Source> make_null_source(const std::string& kind) {
  if (kind != "smi" && kind != "counter") throw std::invalid_argument("null source kind must be 'smi' or 'counter'");
  return std::make_shared<NullSource>(kind);
}

std::shared_ptr<Source> make_synthetic_source(const std::string& kind, uint64_t seed, double total_vram_mb) {
  if (kind == "smi") return std::make_shared<SyntheticSmi>(seed, total_vram_mb);
  if (kind == "counter") return std::make_shared<SyntheticCtr>(seed);
  throw std::invalid_argument("synthetic source kind must be 'smi' or 'counter', got '" + kind + "'");
}

// ================================ amd-smi ==========================================
namespace {

std::once_flag g_smi_once;
amdsmi_status_t g_smi_status = AMDSMI_STATUS_INIT_ERROR;
std::vector<amdsmi_processor_handle> g_smi_handles;

void smi_init() {
  std::call_once(g_smi_once, [] {
    g_smi_status = amdsmi_init(AMDSMI_INIT_AMD_GPUS);
    if (g_smi_status != AMDSMI_STATUS_SUCCESS) return;
    uint32_t nsock = 0;
    if (amdsmi_get_socket_handles(&nsock, nullptr) != AMDSMI_STATUS_SUCCESS) return;
    std::vector<amdsmi_socket_handle> socks(nsock);
    amdsmi_get_socket_handles(&nsock, socks.data());
    for (auto s : socks) {
      uint32_t np = 0;
      if (amdsmi_get_processor_handles(s, &np, nullptr) != AMDSMI_STATUS_SUCCESS) continue;
      std::vector<amdsmi_processor_handle> ph(np);
      amdsmi_get_processor_handles(s, &np, ph.data());
      for (auto h : ph) {
        processor_type_t type{};
        if (amdsmi_get_processor_type(h, &type) == AMDSMI_STATUS_SUCCESS && type == AMDSMI_PROCESSOR_TYPE_AMD_GPU)
          g_smi_handles.push_back(h);
      }
    }
  });
}

inline bool valid16(uint16_t v) { return v != 0xFFFF; }

GpuInfo smi_info(amdsmi_processor_handle h, int index) {
  GpuInfo g;
  g.index = index;
  amdsmi_get_gpu_bdf_id(h, &g.bdf);
  amdsmi_board_info_t b{};
  if (amdsmi_get_gpu_board_info(h, &b) == AMDSMI_STATUS_SUCCESS) {
    g.model_number = b.model_number;
    g.product_name = b.product_name;
  }
  amdsmi_asic_info_t a{};
  if (amdsmi_get_gpu_asic_info(h, &a) == AMDSMI_STATUS_SUCCESS) g.market_name = a.market_name;
  amdsmi_power_info_t p{};
  if (amdsmi_get_power_info(h, &p) == AMDSMI_STATUS_SUCCESS && p.power_limit != 0xFFFFFFFFu && p.power_limit) {
    double w = double(p.power_limit);
    g.power_limit_w = w > 1e5 ? w / 1e6 : w;  // uW on MI355X (1400000000), W elsewhere
  }
  amdsmi_vram_usage_t v{};
  if (amdsmi_get_gpu_vram_usage(h, &v) == AMDSMI_STATUS_SUCCESS) g.vram_total_mb = v.vram_total;
  amdsmi_gpu_metrics_t m{};
  if (amdsmi_get_gpu_metrics_info(h, &m) == AMDSMI_STATUS_SUCCESS) g.edge_is_hotspot = !valid16(m.temperature_edge);
  return g;
}

// VRAM used straight from the amdgpu sysfs attribute amd-smi itself reads: one pread
// on a descriptor kept open (~4 us) instead of amdsmi_get_gpu_vram_usage (~67 us on
// MI355X, profiles/r01/probe_smi_latency.txt). -1 when the attribute is absent.
int open_vram_used(uint64_t bdf) {
  char path[128];
  std::snprintf(path, sizeof path, "/sys/bus/pci/devices/%04x:%02x:%02x.%x/mem_info_vram_used",
                unsigned(bdf >> 32), unsigned((bdf >> 8) & 0xFF), unsigned((bdf >> 3) & 0x1F), unsigned(bdf & 0x7));
  return ::open(path, O_RDONLY | O_CLOEXEC);
}

bool read_u64_attr(int fd, uint64_t* v) {
  char buf[64];
  const ssize_t n = ::pread(fd, buf, sizeof buf - 1, 0);
  if (n <= 0) return false;
  buf[n] = 0;
  char* end = nullptr;
  const unsigned long long x = std::strtoull(buf, &end, 10);
  if (end == buf) return false;
  *v = x;
  return true;
}

// ---- raw SMU metrics table ---------------------------------------------------------
// amdsmi_get_gpu_metrics_info reads the amdgpu `gpu_metrics` sysfs blob and converts
// whichever table version it finds into one wide struct: ~130 us per call on MI355X,
// of which the pread of the blob is ~49 us (profiles/r01/probe_smi_latency.txt). The
// sample needs six 16-bit fields, so the fast path preads the blob itself into a
// buffer kept across samples and picks them out. The blob layout is versioned by its
// 4-byte header and is not published in the ROCm headers; the offsets below are the
// layout of the format-1 (MI300-class) tables, and they are used only after they
// reproduce amd-smi's own decoding exactly on repeated paired reads at start-up
// (calibrate_raw). Any other table version, or any mismatch, keeps amd-smi.
struct RawLayout {
  int hotspot, mem, power, gfx, umc;
};
constexpr RawLayout kFormat1Layout{4, 6, 10, 12, 14};
// The interconnect fields of the v1.8 table (MI355X; profiles/r01/metrics_layout.txt
// places every one of them against amd-smi's decoding): the instantaneous PCIe
// bandwidth (u64 GB/s), the per-link xGMI read / write data accumulators (8 x u64 KB)
// and the firmware timestamp of the publication (u64, 10 ns). Used only when they too
// reproduce amd-smi at start-up (calibrate_raw); otherwise they come from amd-smi.
struct RawIcLayout {
  int pcie_inst, xgmi_rd, xgmi_wr, fw_ts, min_size;
};
constexpr RawIcLayout kV18Interconnect{96, 136, 200, 288, 296};
// Per-XCD words of the v1.8 table (profiles/r01/probe_xcd.txt): the current gfx clock
// of each XCD (u16[8], MHz) and partition 0's instantaneous busy per XCD (u32[8], %;
// in SPX mode partition 0 spans all eight XCDs). Verified against amd-smi's
// current_gfxclks / xcp_stats[0].gfx_busy_inst at start-up like the other fields.
struct RawXcdLayout {
  int gfxclk, busy, min_size;
};
constexpr RawXcdLayout kV18Xcd{296, 344, 376};
constexpr int kXgmiLinks = 8;
// The table's "instantaneous PCIe bandwidth" is not in GB/s: a 52.2 GB/s pinned
// host-to-device stream reads 5.6e5 (profiles/r01/probe_pcie_units.txt), i.e. units of
// 0.1 MB/s of link traffic (payload + ~7 % TLP overhead). The xGMI accumulators are in
// KB as amd-smi documents them (not calibrated: a 1-GPU box moves nothing over xGMI).
constexpr double kPcieUnitGBps = 1e-4;

inline uint16_t rd16(const uint8_t* p, int off) { return uint16_t(p[off] | (p[off + 1] << 8)); }
inline uint32_t rd32(const uint8_t* p, int off) {
  uint32_t v;
  std::memcpy(&v, p + off, 4);
  return v;
}
inline uint64_t rd64(const uint8_t* p, int off) {
  uint64_t v;
  std::memcpy(&v, p + off, 8);
  return v;
}

// xGMI rates from the accumulating counters of the SMU table. The firmware publishes
// a new table every ~20 ms while the table is read far more often: a rate is formed
// only when the firmware timestamp moved (over that publication interval) and is
// repeated until the next publication. Links without a counter (all-ones) add nothing.
class XgmiRates {
 public:
  void update(uint64_t fw_ts, const uint64_t* rd_kb, const uint64_t* wr_kb, int links) {
    uint64_t rd = 0, wr = 0;
    for (int i = 0; i < links; ++i) {
      if (rd_kb[i] != ~0ull) rd += rd_kb[i];
      if (wr_kb[i] != ~0ull) wr += wr_kb[i];
    }
    if (fw_ts == ts_ || fw_ts == 0 || fw_ts == ~0ull) return;
    if (ts_ && fw_ts > ts_ && rd >= rd_ && wr >= wr_) {
      const double dt = double(fw_ts - ts_) * 1e-8;  // 10 ns units
      rd_gbps_ = float(double(rd - rd_) * 1024.0 / dt / 1e9);
      wr_gbps_ = float(double(wr - wr_) * 1024.0 / dt / 1e9);
    }
    ts_ = fw_ts;
    rd_ = rd;
    wr_ = wr;
  }
  float read_gbps() const { return rd_gbps_; }
  float write_gbps() const { return wr_gbps_; }

 private:
  uint64_t ts_ = 0, rd_ = 0, wr_ = 0;
  float rd_gbps_ = std::numeric_limits<float>::quiet_NaN(), wr_gbps_ = std::numeric_limits<float>::quiet_NaN();
};

int open_gpu_metrics(uint64_t bdf) {
  char path[128];
  std::snprintf(path, sizeof path, "/sys/bus/pci/devices/%04x:%02x:%02x.%x/gpu_metrics",
                unsigned(bdf >> 32), unsigned((bdf >> 8) & 0xFF), unsigned((bdf >> 3) & 0x1F), unsigned(bdf & 0x7));
  return ::open(path, O_RDONLY | O_CLOEXEC);
}

bool env_disabled(const char* name) {
  const char* v = std::getenv(name);
  return v && (v[0] == '0' || v[0] == 'n' || v[0] == 'N' || v[0] == 'f' || v[0] == 'F');
}

class SmiSource final : public Source {
 public:
  SmiSource(amdsmi_processor_handle h, int index)
      : h_(h), info_(smi_info(h, index)), policy_(env_seconds("ROCMDASH_SMI_RECALIBRATE_S", 60.0)) {
    vram_fd_ = open_vram_used(info_.bdf);
    if (!env_disabled("ROCMDASH_SMI_RAW")) calibrate_raw();
    else record_calibration(0, true, "disabled by ROCMDASH_SMI_RAW=0");
    info_.metrics_path = raw_ ? "sysfs" : "amdsmi";
    // The firmware publishes a new metrics table every ~20 ms (~50 / s); a table read
    // (an SMU round trip, ~50 us) more often than this returns the previous table. With
    // ROCMDASH_SMU_TABLE_MIN_US > 0 the table is read at most that often and rows in
    // between repeat its values (as back-to-back reads do anyway); used VRAM - the live
    // column - is still read on every sample.
    if (const char* v = std::getenv("ROCMDASH_SMU_TABLE_MIN_US")) table_min_ns_ = int64_t(std::atof(v) * 1000.0);
  }
  ~SmiSource() override {
    if (vram_fd_ >= 0) ::close(vram_fd_);
    if (metrics_fd_ >= 0) ::close(metrics_fd_);
  }
  uint32_t width() const override { return SMI_NUM_FIELDS; }
  std::string kind() const override { return "smi"; }
  std::string backend() const override { return "amdsmi"; }
  GpuInfo info() const override {
    std::lock_guard<std::mutex> lk(info_mu_);
    return info_;
  }
  bool sample(float* row) override {
    // a start-up calibration refused by mismatch is retried here, on the sampling thread
    // (the only one that touches the table fd and buffers), every ROCMDASH_SMI_RECALIBRATE_S
    if (!raw_ && policy_.due(now_ns())) {
      ++recalibrations_;
      calibrate_raw();
      std::lock_guard<std::mutex> lk(info_mu_);
      info_.metrics_path = raw_ ? "sysfs" : "amdsmi";
    }
    bool any = false;
    const int64_t now = table_min_ns_ > 0 ? std::chrono::duration_cast<std::chrono::nanoseconds>(
                                                std::chrono::steady_clock::now().time_since_epoch()).count()
                                          : 0;
    if (table_min_ns_ > 0 && have_last_ && now - last_table_ns_ < table_min_ns_) {
      std::memcpy(row, last_row_, sizeof last_row_);  // the table as last read
      ++table_skips_;
      any = true;
    } else {
      for (int i = 0; i < SMI_NUM_FIELDS; ++i) row[i] = kNaN;
      any = raw_ && sample_raw(row);
      if (!any) any = sample_smi(row);
      if (any && table_min_ns_ > 0) {
        std::memcpy(last_row_, row, sizeof last_row_);
        last_table_ns_ = now;
        have_last_ = true;
      }
    }
    uint64_t used_bytes = 0;
    if (vram_fd_ >= 0 && info_.vram_total_mb > 0 && read_u64_attr(vram_fd_, &used_bytes)) {
      any = true;
      row[SMI_USED_VRAM] = float(double(used_bytes) / (1024.0 * 1024.0));  // MB, as amd-smi reports
      row[SMI_TOTAL_VRAM] = float(info_.vram_total_mb);
    } else {
      amdsmi_vram_usage_t v{};
      if (amdsmi_get_gpu_vram_usage(h_, &v) == AMDSMI_STATUS_SUCCESS) {
        any = true;
        row[SMI_USED_VRAM] = float(v.vram_used);
        row[SMI_TOTAL_VRAM] = float(v.vram_total);
      }
    }
    return any;
  }
  bool fast_vram() const { return vram_fd_ >= 0; }
  std::vector<std::pair<std::string, double>> counts() const override {
    return {{"raw_reads", double(raw_reads_.load(std::memory_order_relaxed))},
            {"raw_table_changes", double(raw_changes_.load(std::memory_order_relaxed))},
            {"raw_misses", double(raw_misses_.load(std::memory_order_relaxed))},
            {"table_skips", double(table_skips_.load(std::memory_order_relaxed))},
            {"table_min_us", double(table_min_ns_) / 1000.0},
            {"raw_volatile_words", double(volatile_words_.size())},
            {"raw_interconnect", raw_ic_ ? 1.0 : 0.0},
            {"raw_xcd", raw_xcd_ ? 1.0 : 0.0},
            // the fast path's state: 1 = raw SMU table, 0 = amd-smi; calibration attempts
            // (start-up + retries), the last attempt's matched triples (of 8; -1: none),
            // promotions to the raw path by a retry, 1 = refused for good (layout)
            {"raw_path", raw_ ? 1.0 : 0.0},
            {"calibration_attempts", double(cal_attempts_.load(std::memory_order_relaxed))},
            {"calibration_matched", double(cal_matched_.load(std::memory_order_relaxed))},
            {"calibration_promotions", double(cal_promotions_.load(std::memory_order_relaxed))},
            {"calibration_final", cal_final_.load(std::memory_order_relaxed) ? 1.0 : 0.0}};
  }
  std::vector<float> xcd_detail() const override {
    std::lock_guard<std::mutex> lk(xcd_mu_);
    if (!xcd_valid_) return {};
    return std::vector<float>(xcd_.begin(), xcd_.end());
  }

 private:
  // blob -> row through the calibrated layout; false (=> amd-smi) if the table read
  // fails or its header is no longer the calibrated one
  bool sample_raw(float* row) {
    const ssize_t n = ::pread(metrics_fd_, buf_.data(), buf_.size(), 0);
    if (n < raw_size_ || rd16(buf_.data(), 0) != raw_size_ || buf_[2] != raw_fmt_ || buf_[3] != raw_content_) {
      ++raw_misses_;
      return false;
    }
    const uint8_t* b = buf_.data();
    ++raw_reads_;
    const RawLayout& L = kFormat1Layout;
    const uint16_t hot = rd16(b, L.hotspot), mem = rd16(b, L.mem), pw = rd16(b, L.power);
    const uint16_t gfx = rd16(b, L.gfx), umc = rd16(b, L.umc);
    if (valid16(hot)) row[SMI_EDGE_TEMP] = row[SMI_HOTSPOT_TEMP] = float(hot);
    if (valid16(gfx)) row[SMI_GFX_ACTIVITY] = float(gfx);
    if (valid16(pw)) row[SMI_SOCKET_POWER] = float(pw);
    if (valid16(mem)) row[SMI_MEM_TEMP] = float(mem);
    if (valid16(umc)) row[SMI_UMC_ACTIVITY] = float(umc);
    if (raw_ic_) {
      const RawIcLayout& I = kV18Interconnect;
      uint64_t rdk[kXgmiLinks], wrk[kXgmiLinks];
      for (int i = 0; i < kXgmiLinks; ++i) {
        rdk[i] = rd64(b, I.xgmi_rd + 8 * i);
        wrk[i] = rd64(b, I.xgmi_wr + 8 * i);
      }
      interconnect(rd64(b, I.fw_ts), rdk, wrk, rd64(b, I.pcie_inst), row);
    }
    if (raw_xcd_) {
      uint32_t busy[kMaxXcds];
      uint16_t clk[kMaxXcds];
      for (int i = 0; i < kMaxXcds; ++i) {
        busy[i] = rd32(b, kV18Xcd.busy + 4 * i);
        clk[i] = rd16(b, kV18Xcd.gfxclk + 2 * i);
      }
      set_xcd(busy, clk);
    }
    // Count the reads that saw a table the firmware had published since the previous
    // read (the rate of fresh telemetry): compare with the previous blob, ignoring the
    // bytes the driver rewrites on every read (its read timestamp, found at start-up).
    for (uint32_t w : volatile_words_) std::memset(buf_.data() + 8 * size_t(w), 0, 8);
    if (std::memcmp(buf_.data(), prev_.data(), raw_size_) != 0) {
      ++raw_changes_;
      std::memcpy(prev_.data(), buf_.data(), raw_size_);
    }
    return true;
  }

  bool sample_smi(float* row) {
    amdsmi_gpu_metrics_t m;
    if (amdsmi_get_gpu_metrics_info(h_, &m) == AMDSMI_STATUS_SUCCESS) {
      const uint16_t edge = valid16(m.temperature_edge) ? m.temperature_edge : m.temperature_hotspot;
      if (valid16(edge)) row[SMI_EDGE_TEMP] = float(edge);
      if (valid16(m.average_gfx_activity)) row[SMI_GFX_ACTIVITY] = float(m.average_gfx_activity);
      const uint16_t pw = valid16(m.current_socket_power) ? m.current_socket_power : m.average_socket_power;
      if (valid16(pw)) row[SMI_SOCKET_POWER] = float(pw);
      if (valid16(m.temperature_hotspot)) row[SMI_HOTSPOT_TEMP] = float(m.temperature_hotspot);
      if (valid16(m.temperature_mem)) row[SMI_MEM_TEMP] = float(m.temperature_mem);
      if (valid16(m.average_umc_activity)) row[SMI_UMC_ACTIVITY] = float(m.average_umc_activity);
      interconnect(m.firmware_timestamp, m.xgmi_read_data_acc, m.xgmi_write_data_acc, m.pcie_bandwidth_inst, row);
      static_assert(AMDSMI_MAX_NUM_XCC >= kMaxXcds && AMDSMI_MAX_NUM_GFX_CLKS >= kMaxXcds, "amd-smi XCD arrays");
      set_xcd(m.xcp_stats[0].gfx_busy_inst, m.current_gfxclks);
      return true;
    }
    return false;
  }

  void interconnect(uint64_t fw_ts, const uint64_t* rd_kb, const uint64_t* wr_kb, uint64_t pcie_inst, float* row) {
    xgmi_.update(fw_ts, rd_kb, wr_kb, kXgmiLinks);
    row[SMI_XGMI_READ_GBPS] = xgmi_.read_gbps();
    row[SMI_XGMI_WRITE_GBPS] = xgmi_.write_gbps();
    if (pcie_inst != ~0ull) row[SMI_PCIE_GBPS] = float(double(pcie_inst) * kPcieUnitGBps);
  }

  void set_xcd(const uint32_t* busy, const uint16_t* clk) {
    std::array<float, 2 * kMaxXcds> v;
    bool any = false;
    for (int i = 0; i < kMaxXcds; ++i) {
      v[i] = busy[i] <= 100u ? float(busy[i]) : kNaN;  // all-ones: no such XCD / N/A
      v[kMaxXcds + i] = valid16(clk[i]) ? float(clk[i]) : kNaN;
      any = any || busy[i] <= 100u || valid16(clk[i]);
    }
    std::lock_guard<std::mutex> lk(xcd_mu_);
    xcd_ = v;
    xcd_valid_ = any;
  }

  // Enable the raw path only if the format-1 offsets reproduce amd-smi's decoding
  // of the same table: raw read, amd-smi read, raw read, 8 times; a trial matches when
  // every field amd-smi reports equals the field at its offset in one of the two
  // surrounding raw reads (the table can refresh in between). 6 of 8 must match.
  static int64_t now_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
  }
  static double env_seconds(const char* name, double dflt) {
    const char* v = std::getenv(name);
    return v && *v ? std::atof(v) : dflt;
  }
  void set_calibration(const std::string& why) {
    std::lock_guard<std::mutex> lk(info_mu_);
    info_.metrics_calibration = why + (policy_.attempts() > 1 ? " [attempt " + std::to_string(policy_.attempts()) + "]"
                                                                : std::string());
  }
  // one calibration attempt's outcome -> the policy (and the exported counts)
  void record_calibration(int matched, bool final, const std::string& why) {
    policy_.record(matched, now_ns(), final);
    cal_attempts_.store(policy_.attempts(), std::memory_order_relaxed);
    cal_matched_.store(matched, std::memory_order_relaxed);
    cal_promotions_.store(policy_.promotions(), std::memory_order_relaxed);
    cal_final_.store(policy_.final_refusal(), std::memory_order_relaxed);
    set_calibration(why);
  }

  // One calibration attempt (start-up, then retries while the policy says so).
  void calibrate_raw() {
    if (metrics_fd_ < 0) metrics_fd_ = open_gpu_metrics(info_.bdf);
    if (metrics_fd_ < 0) return record_calibration(0, true, "no gpu_metrics file");
    buf_.assign(4096, 0);
    const ssize_t n = ::pread(metrics_fd_, buf_.data(), buf_.size(), 0);
    if (n < 16) return record_calibration(0, false, "gpu_metrics read failed");
    raw_size_ = rd16(buf_.data(), 0);
    raw_fmt_ = buf_[2];
    raw_content_ = buf_[3];
    char tag[48];
    std::snprintf(tag, sizeof tag, "v%u.%u %u B", unsigned(raw_fmt_), unsigned(raw_content_), unsigned(raw_size_));
    {
      std::lock_guard<std::mutex> lk(info_mu_);
      info_.metrics_table = tag;
    }
    // format 1 tables have no edge sensor (amd-smi reports it invalid): the row's
    // edge column then carries the hotspot, as on the amd-smi path
    if (raw_fmt_ != 1 || raw_size_ < 16 || raw_size_ > n || !info_.edge_is_hotspot)
      return record_calibration(0, true, "not a calibrated layout (format 1 with an invalid edge sensor)");
    std::vector<uint8_t> a(raw_size_), b(raw_size_);
    const RawLayout& L = kFormat1Layout;
    int matched = 0, matched_ic = 0, matched_xcd = 0;
    for (int t = 0; t < 8; ++t) {
      amdsmi_gpu_metrics_t m;
      if (::pread(metrics_fd_, a.data(), raw_size_, 0) != raw_size_ ||
          amdsmi_get_gpu_metrics_info(h_, &m) != AMDSMI_STATUS_SUCCESS ||
          ::pread(metrics_fd_, b.data(), raw_size_, 0) != raw_size_)
        return record_calibration(matched, false, "a calibration read failed after " + std::to_string(t) + " trials");
      if (!valid16(m.current_socket_power) || !valid16(m.temperature_hotspot))
        return record_calibration(0, true, "amd-smi reports no socket power / hotspot");
      auto same = [&](uint16_t v, int off) { return v == rd16(a.data(), off) || v == rd16(b.data(), off); };
      matched += same(m.temperature_hotspot, L.hotspot) && same(m.temperature_mem, L.mem) &&
                 same(m.current_socket_power, L.power) && same(m.average_gfx_activity, L.gfx) &&
                 same(m.average_umc_activity, L.umc);
      // interconnect fields: every one equals amd-smi's in one of the two reads
      if (raw_content_ == 8 && raw_size_ >= kV18Interconnect.min_size) {
        const RawIcLayout& I = kV18Interconnect;
        auto same64 = [&](uint64_t v, int off) { return v == rd64(a.data(), off) || v == rd64(b.data(), off); };
        bool ok = same64(m.pcie_bandwidth_inst, I.pcie_inst) && same64(m.firmware_timestamp, I.fw_ts);
        for (int i = 0; i < kXgmiLinks; ++i)
          ok = ok && same64(m.xgmi_read_data_acc[i], I.xgmi_rd + 8 * i) && same64(m.xgmi_write_data_acc[i], I.xgmi_wr + 8 * i);
        matched_ic += ok;
      }
      if (raw_content_ == 8 && raw_size_ >= kV18Xcd.min_size) {
        auto same32 = [&](uint32_t v, int off) { return v == rd32(a.data(), off) || v == rd32(b.data(), off); };
        bool ok = true;
        for (int i = 0; i < kMaxXcds; ++i)
          ok = ok && same(m.current_gfxclks[i], kV18Xcd.gfxclk + 2 * i) &&
               same32(m.xcp_stats[0].gfx_busy_inst[i], kV18Xcd.busy + 4 * i);
        matched_xcd += ok;
      }
    }
    const bool ok = matched >= policy_.need();
    // the volatile words are found before the raw path turns on (sample_raw reads them)
    prev_.assign(raw_size_, 0);
    volatile_words_.clear();
    if (ok) find_volatile_words(a, b);
    raw_ic_ = ok && matched_ic >= policy_.need();
    raw_xcd_ = ok && matched_xcd >= policy_.need();
    record_calibration(matched, false,
                       "amd-smi matched " + std::to_string(matched) + "/8 (interconnect " + std::to_string(matched_ic) +
                           ", xcd " + std::to_string(matched_xcd) + "; >= 6 needed)" +
                           (ok ? "" : "; retried every " + std::to_string(int(env_seconds("ROCMDASH_SMI_RECALIBRATE_S",
                                                                                           60.0))) + " s"));
    raw_ = policy_.raw();
  }

  void find_volatile_words(std::vector<uint8_t>& a, std::vector<uint8_t>& b) {
    // 8-byte words that differ between EVERY pair of back-to-back reads are rewritten
    // by the driver per read, not by the firmware per update (a firmware update lands
    // between some pairs only): the intersection over 6 pairs
    const size_t nw = raw_size_ / 8;
    std::vector<uint8_t> always(nw, 1);
    for (int t = 0; t < 6; ++t) {
      if (::pread(metrics_fd_, a.data(), raw_size_, 0) != raw_size_ || ::pread(metrics_fd_, b.data(), raw_size_, 0) != raw_size_)
        break;
      for (size_t w = 0; w < nw; ++w)
        if (std::memcmp(a.data() + 8 * w, b.data() + 8 * w, 8) == 0) always[w] = 0;
    }
    for (size_t w = 0; w < nw; ++w)
      if (always[w]) volatile_words_.push_back(uint32_t(w));
  }

  amdsmi_processor_handle h_;
  GpuInfo info_;
  mutable std::mutex info_mu_;  // info_ strings change on a recalibration (sampler thread)
  RawCalibrationPolicy policy_;  // sampler thread only
  int vram_fd_ = -1;
  int metrics_fd_ = -1;
  // written by the sampling thread, read by counts() from others
  std::atomic<bool> raw_{false};
  std::atomic<bool> raw_ic_{false};  // interconnect fields read raw too (else: from amd-smi, or NaN)
  std::atomic<bool> raw_xcd_{false};  // per-XCD busy / clocks read raw too (else: from amd-smi)
  std::atomic<int> cal_attempts_{0}, cal_matched_{-1}, cal_promotions_{0};
  std::atomic<bool> cal_final_{false};
  uint64_t recalibrations_ = 0;
  mutable std::mutex xcd_mu_;
  std::array<float, 2 * kMaxXcds> xcd_{};
  bool xcd_valid_ = false;
  XgmiRates xgmi_;
  uint16_t raw_size_ = 0;
  uint8_t raw_fmt_ = 0, raw_content_ = 0;
  std::atomic<uint64_t> raw_misses_{0}, raw_reads_{0}, raw_changes_{0}, table_skips_{0};
  int64_t table_min_ns_ = 0;  // ROCMDASH_SMU_TABLE_MIN_US
  int64_t last_table_ns_ = 0;
  bool have_last_ = false;
  float last_row_[SMI_NUM_FIELDS];
  std::vector<uint8_t> buf_, prev_;
  std::vector<uint32_t> volatile_words_;  // per-read driver fields, excluded from change detection
};

}  // namespace

int amdsmi_gpu_count() {
  smi_init();
  if (g_smi_status != AMDSMI_STATUS_SUCCESS) return -1;
  return int(g_smi_handles.size());
}

std::vector<GpuInfo> amdsmi_enumerate() {
  std::vector<GpuInfo> out;
  if (amdsmi_gpu_count() <= 0) return out;
  for (size_t i = 0; i < g_smi_handles.size(); ++i) out.push_back(smi_info(g_smi_handles[i], int(i)));
  return out;
}

std::shared_ptr<Source> make_smi_source(uint64_t bdf, int index) {
  if (amdsmi_gpu_count() <= 0) throw std::runtime_error("amd-smi: no AMD GPU available (amdsmi_init failed or no devices)");
  for (size_t i = 0; i < g_smi_handles.size(); ++i) {
    uint64_t b = 0;
    amdsmi_get_gpu_bdf_id(g_smi_handles[i], &b);
    if ((bdf != 0 && b == bdf) || (bdf == 0 && int(i) == index)) return std::make_shared<SmiSource>(g_smi_handles[i], int(i));
  }
  throw std::runtime_error("amd-smi: no GPU with the requested bdf/index");
}

}  // namespace rocmdash
