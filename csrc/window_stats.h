// Host/device interface of the CDNA4 windowed-statistics kernel (window_stats.hip).
#pragma once

#include <cstdint>

namespace rocmdash {

// Statistics computed per series, in output order.
enum StatSlot : int {
  STAT_MIN = 0,
  STAT_MAX = 1,
  STAT_MEAN = 2,
  STAT_P0 = 3,  // first percentile (default p50)
  STAT_P1 = 4,  // second percentile (default p90)
  STAT_P2 = 5,  // third percentile (default p99)
  STAT_LAST = 6,
  STAT_COUNT = 7,
  STAT_NUM = 8,
};

// One time series inside a device-resident, time-major ring [cap][stride] float32.
// The window is rows (head - n) .. (head - 1), taken modulo cap (cap = mask + 1).
struct SeriesDesc {
  const float* base;  // device pointer to row 0 of the ring
  uint64_t head;      // rows ever written to the host ring at copy time
  uint32_t stride;    // floats per row
  uint32_t col;       // column of this series inside a row
  uint32_t mask;      // ring capacity - 1 (power of two)
  uint32_t n;         // window length (<= mask + 1, <= head)
};

constexpr int kMaxSeriesPerLaunch = 96;  // keeps the by-value kernel argument < 4 KiB

struct StatsArgs {
  uint32_t num_series;
  float pct[3];
  SeriesDesc d[kMaxSeriesPerLaunch];
};

// Launch the stats kernel for args.num_series series on `stream`; out is a device
// pointer to [num_series][STAT_NUM] float32. `pad_pow2` is the sort width: the next
// power of two >= max(d[i].n), at least 64, at most 32768. Returns a hipError_t.
int launch_window_stats(const StatsArgs& args, uint32_t pad_pow2, float* out, void* stream);

// Smallest supported sort width for a window of n samples.
uint32_t sort_width_for(uint32_t n);

}  // namespace rocmdash
