// Native dashboard-frame renderer: one refresh's JSON payload (every Plotly figure,
// the statistics table, the optional window table) from a precompiled plan and the
// node snapshot's numbers, without Python objects and without holding the GIL.
//
// Reference counterpart: the per-refresh figure construction + serialisation of
// app.py:331-484 (4 + 4N go.Figure objects, BASELINE.md's "full refresh"). The
// Python implementation (rocmdash/viz/panels.py Frame.to_json) defines the format;
// this renderer reproduces it byte for byte (tests/test_frame_render.py).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace rocmdash {

struct PanelPlan {
  std::string key_prefix;  // plot key without the refresh timestamp
  std::string head, mid, tail;  // cached figure JSON around colour and value
  double max_val = 100.0;  // colour band denominator
  int src = 0;             // 0: values[row][col], 1: selected-GPU average of col, 2: literal int 0
  int row = 0;
  int col = 0;
};

struct FramePlan {
  std::vector<PanelPlan> panels;  // display order
  std::vector<int> sel_rows;      // rows averaged by src == 1 panels
  int power_col = -1;             // average over non-zero readings when any (app.py:341-345)
  std::string headers_json;       // JSON list of the per-GPU headers
  std::string stats_columns_json; // JSON list of the statistics-table columns
  int num_columns = 0;            // C: values are [G][C]
  bool window = false;            // emit the window table
  std::string window_gpus_json, window_series_json, window_stats_json;
  std::vector<int> window_stat_idx;  // which of the 8 kernel statistics, in order
  int window_series = 0;             // S: window is [G][S][8] float32
  mutable int ascii = -1;            // every plan string is 7-bit (-1: not checked yet)
  bool all_ascii() const;
};

// Python's repr() of a float (shortest round-trip digits, fixed notation for
// 1e-4 <= |x| < 1e16 else scientific), as json.dumps writes it.
void append_py_float(std::string& out, double x);
// json.dumps(float(np.round(x, 2))) ("null" for NaN / inf)
void append_round2(std::string& out, double x);

// values: [G][C] float64 row-major; window: [G][S][8] float32 or nullptr.
std::string render_frame(const FramePlan& plan, const double* values, int G, const float* window,
                         const std::string& ts_key, const std::string& updated_json);
// Same, into `out` (cleared first; its capacity is reused across refreshes).
void render_frame_into(std::string& out, const FramePlan& plan, const double* values, int G, const float* window,
                       const std::string& ts_key, const std::string& updated_json);

bool is_ascii(const std::string& s);

}  // namespace rocmdash
