// Native dashboard-frame renderer (see frame_render.h).
#include "frame_render.h"

#include <charconv>
#include <cmath>
#include <cstdlib>
#include <cstring>

namespace rocmdash {

void append_py_float(std::string& out, double x) {
  char buf[64];
  auto res = std::to_chars(buf, buf + sizeof buf, x, std::chars_format::scientific);
  *res.ptr = 0;
  // buf = [-]d[.ddd]e(+|-)XX  (shortest round-trip digits)
  const char* p = buf;
  if (*p == '-') {
    out.push_back('-');
    ++p;
  }
  char digits[32];
  int nd = 0;
  for (; *p && *p != 'e'; ++p)
    if (*p != '.') digits[nd++] = *p;
  const int exp = std::atoi(p + 1);
  if (exp >= -4 && exp < 16) {  // fixed notation, like repr()
    const int decpt = exp + 1;
    if (decpt <= 0) {
      out.append("0.");
      out.append(size_t(-decpt), '0');
      out.append(digits, size_t(nd));
    } else if (decpt >= nd) {
      out.append(digits, size_t(nd));
      out.append(size_t(decpt - nd), '0');
      out.append(".0");
    } else {
      out.append(digits, size_t(decpt));
      out.push_back('.');
      out.append(digits + decpt, size_t(nd - decpt));
    }
  } else {  // scientific: d[.ddd]e(+|-)XX
    out.push_back(digits[0]);
    if (nd > 1) {
      out.push_back('.');
      out.append(digits + 1, size_t(nd - 1));
    }
    char e[16];
    std::snprintf(e, sizeof e, "e%c%02d", exp < 0 ? '-' : '+', exp < 0 ? -exp : exp);
    out.append(e);
  }
}

namespace {

// get_color_for_value (app.py:56-68): NaN compares false everywhere -> red.
const char* band_color(double value, double max_val) {
  const double pct = (value / max_val) * 100.0;
  if (pct <= 20) return "#2ecc71";
  if (pct <= 40) return "#27ae60";
  if (pct <= 60) return "#f1c40f";
  if (pct <= 80) return "#e67e22";
  return "#e74c3c";
}

void append_value(std::string& out, double v) {
  if (std::isfinite(v)) append_py_float(out, v);
  else out.append("null");
}

}  // namespace

// np.round(x, 2) then json.dumps(...).replace("NaN", "null"). np.round computes
// r = rint(x * 100) / 100; for |r| < 1e13 two different 2-decimal values are more
// than an ulp apart, so repr(r) - the shortest round-trip string - is that decimal
// itself with trailing zeros trimmed ("12.5", "12.0"): print it from the integer
// k = rint(x * 100) directly instead of running the shortest-digits search.
void append_round2(std::string& out, double v) {
  const double t = std::nearbyint(v * 100.0);
  const double r = t / 100.0;
  if (!std::isfinite(r)) {
    out.append("null");
    return;
  }
  if (std::fabs(t) >= 1e15) {
    append_py_float(out, r);
    return;
  }
  if (std::signbit(r)) out.push_back('-');  // includes -0.0
  const long long k = std::llabs(static_cast<long long>(t));
  char buf[24];
  auto res = std::to_chars(buf, buf + sizeof buf, k / 100);
  out.append(buf, size_t(res.ptr - buf));
  const int f = int(k % 100);
  out.push_back('.');
  out.push_back(char('0' + f / 10));
  if (f % 10) out.push_back(char('0' + f % 10));
}

namespace {

void append_rounded(std::string& out, double v) { append_round2(out, v); }

// numpy's pairwise_sum for n <= 128 (the 1-D mean of the power column)
double numpy_pairwise_sum(const double* a, int n) {
  if (n < 8) {
    double res = 0.0;
    for (int i = 0; i < n; ++i) res += a[i];
    return res;
  }
  double r[8];
  for (int j = 0; j < 8; ++j) r[j] = a[j];
  int i = 8;
  for (; i + 8 <= n; i += 8)
    for (int j = 0; j < 8; ++j) r[j] += a[i + j];
  double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < n; ++i) res += a[i];
  return res;
}

// Column-wise NaN-skipping mean / max / min over `rows` (in order), as
// rocmdash/viz/panels.py _nan_mean_max_min computes them with numpy.
void nan_mean_max_min(const double* values, int C, const int* rows, int nrows, double* mean, double* mx, double* mn) {
  for (int c = 0; c < C; ++c) {
    double s = 0.0, hi = NAN, lo = NAN;
    int cnt = 0;
    for (int k = 0; k < nrows; ++k) {
      const double v = values[size_t(rows[k]) * C + c];
      const double w = std::isnan(v) ? 0.0 : v;
      s = k == 0 ? w : s + w;
      if (!std::isnan(v)) {
        ++cnt;
        hi = std::isnan(hi) ? v : std::fmax(hi, v);
        lo = std::isnan(lo) ? v : std::fmin(lo, v);
      }
    }
    mean[c] = nrows ? s / double(cnt) : NAN;  // cnt == 0 -> 0/0 = NaN
    mx[c] = hi;
    mn[c] = lo;
  }
}

}  // namespace

bool is_ascii(const std::string& s) {
  unsigned char acc = 0;
  for (unsigned char c : s) acc |= c;
  return acc < 0x80;
}

bool FramePlan::all_ascii() const {
  if (ascii < 0) {
    bool ok = is_ascii(headers_json) && is_ascii(stats_columns_json) && is_ascii(window_gpus_json) &&
              is_ascii(window_series_json) && is_ascii(window_stats_json);
    for (const auto& p : panels)
      ok = ok && is_ascii(p.key_prefix) && is_ascii(p.head) && is_ascii(p.mid) && is_ascii(p.tail);
    ascii = ok ? 1 : 0;
  }
  return ascii == 1;
}

std::string render_frame(const FramePlan& plan, const double* values, int G, const float* window,
                         const std::string& ts_key, const std::string& updated_json) {
  std::string out;
  render_frame_into(out, plan, values, G, window, ts_key, updated_json);
  return out;
}

void render_frame_into(std::string& out, const FramePlan& plan, const double* values, int G, const float* window,
                       const std::string& ts_key, const std::string& updated_json) {
  const int C = plan.num_columns;
  // selected-GPU averages (app.py:338-345)
  const size_t Cn = static_cast<size_t>(C);
  std::vector<double> avg(Cn, NAN), tmp1(Cn), tmp2(Cn);
  if (!plan.sel_rows.empty()) {
    nan_mean_max_min(values, C, plan.sel_rows.data(), int(plan.sel_rows.size()), avg.data(), tmp1.data(), tmp2.data());
    if (plan.power_col >= 0) {
      double nz[128];
      int n = 0;
      for (int r : plan.sel_rows) {
        const double p = values[size_t(r) * C + plan.power_col];
        if (p > 0 && n < 128) nz[n++] = p;
      }
      // ndarray.mean() of a contiguous 1-D array: numpy pairwise summation of all n
      if (n) avg[size_t(plan.power_col)] = numpy_pairwise_sum(nz, n) / double(n);
    }
  }
  out.clear();
  size_t reserve = 256 + plan.headers_json.size();
  for (const auto& p : plan.panels) reserve += p.head.size() + p.mid.size() + p.tail.size() + p.key_prefix.size() + 64;
  out.reserve(reserve + size_t(G) * 1024);
  out.append("{\"updated\":");
  out.append(updated_json);
  out.append(",\"figures\":{");
  bool first = true;
  for (const auto& p : plan.panels) {
    if (!first) out.push_back(',');
    first = false;
    out.push_back('"');
    out.append(p.key_prefix);
    out.append(ts_key);
    out.append("\":");
    out.append(p.head);
    if (p.src == 2) {
      out.append(band_color(0.0, p.max_val));
      out.append(p.mid);
      out.push_back('0');
    } else {
      const double v = p.src == 1 ? avg[size_t(p.col)] : values[size_t(p.row) * C + p.col];
      out.append(band_color(v, p.max_val));
      out.append(p.mid);
      append_value(out, v);
    }
    out.append(p.tail);
  }
  out.append("},\"headers\":");
  out.append(plan.headers_json);
  // statistics over ALL GPUs (app.py:216-221)
  std::vector<int> all(static_cast<size_t>(G));
  for (int g = 0; g < G; ++g) all[size_t(g)] = g;
  std::vector<double> mean(Cn), mx(Cn), mn(Cn);
  if (G) nan_mean_max_min(values, C, all.data(), G, mean.data(), mx.data(), mn.data());
  else for (int c = 0; c < C; ++c) mean[size_t(c)] = mx[size_t(c)] = mn[size_t(c)] = NAN;
  out.append(",\"stats\":{\"rows\":[\"mean\",\"max\",\"min\"],\"columns\":");
  out.append(plan.stats_columns_json);
  out.append(",\"values\":[");
  const std::vector<double>* rows3[3] = {&mean, &mx, &mn};
  for (int k = 0; k < 3; ++k) {
    if (k) out.append(", ");
    out.push_back('[');
    for (int c = 0; c < C; ++c) {
      if (c) out.append(", ");
      append_rounded(out, (*rows3[k])[size_t(c)]);
    }
    out.push_back(']');
  }
  out.append("]}");
  if (plan.window && window != nullptr) {
    out.append(",\"window\":{\"gpus\":");
    out.append(plan.window_gpus_json);
    out.append(",\"series\":");
    out.append(plan.window_series_json);
    out.append(",\"stats\":");
    out.append(plan.window_stats_json);
    out.append(",\"values\":[");
    const int S = plan.window_series;
    for (int g = 0; g < G; ++g) {
      if (g) out.append(", ");
      out.push_back('[');
      for (int s = 0; s < S; ++s) {
        if (s) out.append(", ");
        out.push_back('[');
        for (size_t k = 0; k < plan.window_stat_idx.size(); ++k) {
          if (k) out.append(", ");
          append_rounded(out, double(window[(size_t(g) * S + s) * 8 + size_t(plan.window_stat_idx[k])]));
        }
        out.push_back(']');
      }
      out.push_back(']');
    }
    out.append("]}");
  }
  out.push_back('}');
}

}  // namespace rocmdash
