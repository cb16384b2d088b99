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

// Persistent per-series state of the incremental path (device memory, written only
// by the kernel). `sorted` holds two halves of `sorted_cap` floats; half `cur` has the
// `nvalid` non-NaN samples of window [head - n, head) in ascending order.
struct SeriesState {
  uint64_t head;
  uint32_t n;
  uint32_t nvalid;
  uint32_t cur;
  uint32_t valid;  // 0 = no state yet (first refresh, or invalidated): full sort
};

// One ring of series: a device-resident, time-major ring [cap][stride] float32 whose
// columns are the series. A series' window is rows (head - n) .. (head - 1), taken
// modulo cap (cap = mask + 1).
//
// Where the rows that enter the window since the previous launch come from:
//   * inline (steady state): the newest `n_inline` (<= kInlineRows) rows travel by
//     value in the kernel argument itself;
//   * pull: older entering rows are read straight from the pinned, coherent host
//     ring (`host_rows`, device-mapped, capacity host_mask + 1);
//   * copy: the host staged them into the device ring with hipMemcpyAsync.
// Inline and pulled rows are written into the device ring by the kernel, where a
// later launch finds them again when they leave the window - no staging copies.
constexpr int kInlineRows = 4;
constexpr int kMaxInlineWidth = 16;
constexpr int kMaxRingsPerLaunch = 4;

struct RingDesc {
  float* base;              // device pointer to row 0 of the device ring
  const float* host_rows;   // pull mode: device-mapped pinned host ring; nullptr = none
  float* sorted;            // nullptr: stateless (always a full sort); else [stride][2][sorted_cap]
  SeriesState* state;       // [stride]; nullptr when stateless
  uint64_t head;            // rows ever written to the host ring (snapshot at enqueue time)
  // Host prediction of the state the previous launch left (~0 = none): lets the
  // incremental path issue every load before the state arrives (validated on device).
  uint64_t pred_head0;
  uint32_t stride;          // floats per row
  uint32_t cols;            // series taken from this ring: columns 0 .. cols - 1 (<= stride)
  uint32_t first;           // series index of column 0 in the launch (filled in by launch_window_stats)
  uint32_t mask;            // device ring capacity - 1 (power of two)
  uint32_t n;               // window length (<= mask + 1, <= head)
  uint32_t sorted_cap;      // >= n; floats per half of a series' `sorted`
  uint32_t host_mask;       // host ring capacity - 1 (pull mode)
  uint32_t pred_n0;
  uint32_t pred_cur;
  uint32_t n_inline;        // rows head - n_inline .. head - 1 are in `inl`
  float inl[kInlineRows][kMaxInlineWidth];
};

// Samples that may enter (and leave) a window between two refreshes for the
// incremental path; more than this falls back to a full sort.
constexpr int kMaxIncremental = 256;
constexpr int kMaxSeriesPerLaunch = 256;

// Passed by value (~1.2 KiB kernel argument). The series of a launch are the columns
// of its rings in ring order: series i is column i - (cols of the rings before r) of
// ring r, so num_series must equal the sum of the rings' cols.
struct StatsArgs {
  uint32_t num_series;
  uint32_t num_rings;
  float pct[3];
  double qfrac[3];  // pct / 100, filled in by launch_window_stats (no fp64 division on device)
  // Completion flag (optional, nullptr = none): every workgroup adds 1 to *wg_counter
  // after its outputs are visible system-wide; the one that brings it to wg_expect
  // (modulo 2^32) stores done_seq to *done_flag - mapped host memory the host spins
  // on instead of waiting for the stream's completion signal.
  uint32_t* wg_counter;
  uint32_t* done_flag;
  uint32_t wg_expect;
  uint32_t done_seq;
  // Tagged outputs (optional, nullptr = none; replaces `out`): every statistic is written
  // as ONE 8-byte word {float bits, done_seq << 32} into mapped host memory
  // [num_series][STAT_NUM], so the host knows each value's refresh from the word itself:
  // no arrival count, acknowledgement wait or flag store behind the outputs.
  uint64_t* tagged_out;
  RingDesc rings[kMaxRingsPerLaunch];
};

// Launch the stats kernel for args.num_series series on `stream`; out is a device
// pointer to [num_series][STAT_NUM] float32. `pad_pow2` is the sort width: the next
// power of two >= every ring's n (and sorted_cap), at least 64, at most 32768.
// Returns a hipError_t.
// `incremental` = the caller expects every series to take the incremental path (it
// tracks the state the previous launch left), `max_new_rows` = the most rows entering
// any series (~0 = unknown): together they select the launch width (W <= 8192: 512
// threads when at most one row enters, 1024 for more - the one-row path and the
// general merge prefer different widths, profiles/r02/onerow/).
int launch_window_stats(const StatsArgs& args, uint32_t pad_pow2, float* out, void* stream, bool incremental = false,
                        uint32_t max_new_rows = ~0u);

// Smallest supported sort width for a window of n samples.
uint32_t sort_width_for(uint32_t n);

}  // namespace rocmdash
