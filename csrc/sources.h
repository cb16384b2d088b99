// Metric sources: one call to sample() produces one time-major row for a SeriesRing.
//
// Reference counterpart: the five `amd_gpu_*` series the reference queries from an
// external exporter (app.py:168-171) plus the `card_model` label (app.py:192). Here
// the node's own GPUs are read directly:
//   SmiSource      libamd_smi  (gpu_metrics table, VRAM usage, board info) ~10 Hz
//   CounterSource  rocprofiler-sdk device counting (MFMA busy, HBM requests) ~100 Hz
//   SyntheticSource deterministic streams with the same layouts (CPU tests, bench
//                   rehearsal without hardware; BASELINE.json "synthetic streams")
#pragma once

#include <cstdint>
#include <memory>
#include <string>
#include <utility>
#include <vector>

namespace rocmdash {

// Row layout of the amd-smi group (order is the device/ring column order).
enum SmiField : int {
  SMI_EDGE_TEMP = 0,    // degC; MI355 has no edge sensor -> hotspot (GpuInfo::edge_is_hotspot)
  SMI_GFX_ACTIVITY,     // %
  SMI_SOCKET_POWER,     // W (current_socket_power on MI300+, average on older parts)
  SMI_USED_VRAM,        // MB
  SMI_TOTAL_VRAM,       // MB
  SMI_HOTSPOT_TEMP,     // degC (junction)
  SMI_MEM_TEMP,         // degC (HBM)
  SMI_UMC_ACTIVITY,     // % memory-controller activity
  // interconnect, from the same SMU table: the xGMI rates are the change of the
  // table's per-link data accumulators (KB, summed over links) between two
  // publications of the table, over the change of its firmware timestamp (10 ns)
  SMI_XGMI_READ_GBPS,   // GB/s received over xGMI (all links)
  SMI_XGMI_WRITE_GBPS,  // GB/s sent over xGMI (all links)
  SMI_PCIE_GBPS,        // GB/s over the PCIe link (the table's instantaneous figure, calibrated)
  SMI_NUM_FIELDS
};

// Row layout of the hardware-counter group (rates over the last sampling interval).
enum CtrField : int {
  CTR_MFMA_UTIL = 0,  // % of SIMD-cycles with the matrix pipe busy
  CTR_HBM_READ_GBPS,  // GB/s L2 misses read from the memory side (TCC->EA, 32 B units; incl. MALL hits)
  CTR_HBM_WRITE_GBPS, // GB/s L2 write-backs to the memory side (64 B / 32 B requests; incl. MALL)
  CTR_GFX_BUSY,       // % of cycles the graphics/compute engine was active
  CTR_CU_ACTIVE,      // % of CU-cycles with a wave resident (SQ_BUSY_CU_CYCLES, calibrated)
  CTR_NUM_FIELDS
};

const char* const* smi_field_names();
const char* const* ctr_field_names();

struct GpuInfo {
  int index = -1;               // amd-smi enumeration index
  uint64_t bdf = 0;             // amdsmi bdf id: domain<<32 | bus<<8 | dev<<3 | fn
  std::string model_number;     // board part number ("102-G36236-0C"), the exporter's card_model
  std::string product_name;     // "AMD Instinct MI355 OAM"
  std::string market_name;
  double power_limit_w = 0.0;   // 0 = unknown
  double vram_total_mb = 0.0;
  bool edge_is_hotspot = false;  // edge sensor missing, SMI_EDGE_TEMP carries hotspot
  // how the SMU metrics table is read each sample: "sysfs" (pread of the amdgpu
  // gpu_metrics blob, layout calibrated against amd-smi at start-up) or "amdsmi"
  std::string metrics_path = "amdsmi";
  std::string metrics_table;  // "v<format>.<content> <size> B" of the gpu_metrics blob
  std::string metrics_calibration;  // why the raw table is (not) used: matches per 8 trials, or the refusal
};

class Source {
 public:
  virtual ~Source() = default;
  virtual uint32_t width() const = 0;
  virtual std::string kind() const = 0;   // "smi" | "counter"
  virtual std::string backend() const = 0; // "amdsmi" | "rocprofiler" | "synthetic"
  // Fill `row` (width() floats). Returns false when no valid row was produced (e.g.
  // the first counter read, which only sets the baseline for rates).
  virtual bool sample(float* row) = 0;
  // When non-zero after a successful sample(): the time (CLOCK_REALTIME ns) the row was
  // actually read, if another process read it (ShmSource); the sampler then stamps the
  // row with it instead of the time of the call.
  virtual uint64_t row_time_ns() const { return 0; }
  virtual GpuInfo info() const { return {}; }
  // Source-specific running counts (e.g. how many SMU table reads returned a table the
  // firmware had refreshed since the previous read). Read from the sampling thread's
  // owner only between samples, or approximately while sampling.
  virtual std::vector<std::pair<std::string, double>> counts() const { return {}; }
  // Per-XCD detail of the last sample: n busy percentages then n gfx clocks (MHz),
  // one per accelerator complex die (8 on an MI355X in SPX mode); NaN where the
  // firmware reports none. Empty for sources without it. Safe to call while sampling.
  virtual std::vector<float> xcd_detail() const { return {}; }
};

constexpr int kMaxXcds = 8;

// ---- synthetic ----------------------------------------------------------------
// Deterministic in (seed, call count): an AR(1) utilisation process with workload
// phases drives power, temperatures, HBM traffic and MFMA busy the way a training
// job would. `total_vram_mb` defaults to the MI355X's 294896 MB (amd-smi, test box).
std::shared_ptr<Source> make_synthetic_source(const std::string& kind, uint64_t seed,
                                              double total_vram_mb = 294896.0);

// A source of the given kind whose reads all fail soft: rows of NaN (backend
// "unavailable"). Keeps the series layout identical on every rank when one GPU's
// counters cannot be configured; its statistics come out NaN with count 0.
std::shared_ptr<Source> make_null_source(const std::string& kind);

// Replays `rows` ([n][width] row-major) in order, wrapping; `info` is what info()
// reports (the recorded GPU's identity).
std::shared_ptr<Source> make_replay_source(const std::string& kind, const std::vector<float>& rows, uint32_t width,
                                           const GpuInfo& info);

// ---- amd-smi ------------------------------------------------------------------
// When the fast SMU-table path may be used (SmiSource): the raw table is trusted only
// after `need` of `trials` raw / amd-smi / raw triples decoded the same values. A
// refusal by MISMATCH (a busy box: the table refreshed between reads too often, or a
// contended driver) is retried every `retry_s` seconds on the sampler thread and the
// source is promoted to the raw path as soon as one attempt matches; a refusal of the
// layout itself (another table format, no sensor) is final. Header-only and clock-free
// (the caller passes the time), so its decisions are unit-tested on the CPU.
class RawCalibrationPolicy {
 public:
  explicit RawCalibrationPolicy(double retry_s = 60.0, int need = 6, int trials = 8)
      : retry_ns_(int64_t(retry_s * 1e9)), need_(need), trials_(trials) {}
  // a retry should run now: refused by mismatch, not final, the period elapsed
  bool due(int64_t now_ns) const { return !raw_ && !final_ && attempts_ > 0 && now_ns - last_ns_ >= retry_ns_; }
  // one attempt's outcome: `matched` of trials() triples (final: the layout can never
  // calibrate); returns whether the raw path is on now
  bool record(int matched, int64_t now_ns, bool final = false) {
    ++attempts_;
    last_ns_ = now_ns;
    last_matched_ = matched;
    final_ = final_ || final;
    if (!final && matched >= need_) {
      if (!raw_ && attempts_ > 1) ++promotions_;
      raw_ = true;
    }
    return raw_;
  }
  bool raw() const { return raw_; }
  bool final_refusal() const { return final_; }
  int attempts() const { return attempts_; }
  int promotions() const { return promotions_; }  // raw path gained by a retry
  int last_matched() const { return last_matched_; }
  int trials() const { return trials_; }
  int need() const { return need_; }
  int64_t last_ns() const { return last_ns_; }

 private:
  int64_t retry_ns_;
  int need_, trials_;
  bool raw_ = false, final_ = false;
  int attempts_ = 0, promotions_ = 0, last_matched_ = -1;
  int64_t last_ns_ = 0;
};

int amdsmi_gpu_count();                  // -1 if amd-smi cannot initialise
std::vector<GpuInfo> amdsmi_enumerate();
// Open the GPU with this bdf id (or the `index`-th GPU when bdf == 0).
std::shared_ptr<Source> make_smi_source(uint64_t bdf, int index);

// ---- rocprofiler-sdk device counting --------------------------------------------
// Must run before the HIP/HSA runtime initialises in this process. Returns 0 on
// success, otherwise a rocprofiler status (or -1 if the SDK library is missing).
// only_ordinal >= 0 configures just that GPU agent (HSA/HIP enumeration order).
// only_bdf (domain<<32 | bus<<8 | dev<<3 | fn) wins over only_ordinal when non-zero
int counters_preinit(const std::vector<std::string>& counter_names, int only_ordinal = -1, uint64_t only_bdf = 0);
bool counters_ready();
std::string counters_status();
// Device-counting source for the GPU agent at this PCI location (bdf id as above;
// bdf == 0 selects the `index`-th GPU agent).
std::shared_ptr<Source> make_counter_source(uint64_t bdf, int index);
// The whole physical GPU at this PCI address: in a compute-partition mode every
// partition agent's counters combined into the GPU's row (csrc/counters.cpp
// GroupCounterSource); the one agent otherwise (= make_counter_source).
std::shared_ptr<Source> make_counter_source_all(uint64_t bdf, int index);

}  // namespace rocmdash
