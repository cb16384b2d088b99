// Node-wide window statistics (see node_window.h): export of the resident sorted
// windows, and the rank-selection kernel over the all-gathered union.
#include "node_window.h"

#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <stdexcept>
#include <string>

#include "device_window.h"
#include "window_stats.h"

namespace rocmdash {
namespace {

constexpr int NT = 256;
constexpr int kMaxLists = 64;              // ranks in one node tensor
constexpr uint32_t kLdsFloats = 32768;     // union staged in LDS up to this many samples
constexpr int kExportPerLaunch = 128;

struct ExportRef {
  const float* sorted;       // the series' two halves of `cap` floats
  const SeriesState* state;  // written by the window-stats kernel on the same stream
  uint32_t cap;
};

struct ExportArgs {
  ExportRef s[kExportPerLaunch];
};

// One workgroup per series: [nvalid, sorted[0 .. nvalid), +inf ...] into dst row s.
__global__ __launch_bounds__(NT) void export_sorted_kernel(const ExportArgs a, float* __restrict__ dst, uint32_t W) {
  const ExportRef r = a.s[blockIdx.x];
  const SeriesState st = *r.state;
  const uint32_t nv = st.valid ? min(st.nvalid, min(W, r.cap)) : 0u;
  const float* src = r.sorted + size_t(st.cur & 1u) * r.cap;
  float* row = dst + size_t(blockIdx.x) * (W + 1);
  if (threadIdx.x == 0) row[0] = float(nv);
  for (uint32_t i = threadIdx.x; i < W; i += NT) row[1 + i] = i < nv ? src[i] : INFINITY;
}

__device__ inline uint32_t lower_bound(const float* a, uint32_t n, float x) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (a[mid] < x) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

__device__ inline uint32_t upper_bound(const float* a, uint32_t n, float x) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (a[mid] <= x) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// One workgroup per series. LDS = stage the N sorted lists compactly in LDS (dynamic
// shared memory, total <= kLdsFloats); else binary-search them in place (L2).
template <bool LDS>
__global__ __launch_bounds__(NT) void node_select_kernel(const float* __restrict__ node, uint32_t N, uint32_t S,
                                                        uint32_t W, float p0, float p1, float p2,
                                                        float* __restrict__ out) {
  extern __shared__ float vals[];
  __shared__ uint32_t cnt[kMaxLists], offs[kMaxLists + 1];
  __shared__ const float* base[kMaxLists];
  __shared__ float picked[6];
  __shared__ double red[NT / 64];
  const uint32_t s = blockIdx.x;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;

  if (t == 0) {
    uint32_t o = 0;
    for (uint32_t i = 0; i < N; ++i) {
      const float* row = node + (size_t(i) * S + s) * (W + 1);
      const float c = row[0];
      cnt[i] = (c > 0.f) ? min(uint32_t(c), W) : 0u;
      offs[i] = o;
      base[i] = row + 1;
      o += cnt[i];
    }
    offs[N] = o;
  }
  if (t < 6) picked[t] = __builtin_nanf("");
  __syncthreads();
  const uint32_t total = offs[N];
  if constexpr (LDS) {
    for (uint32_t i = 0; i < N; ++i)
      for (uint32_t j = t; j < cnt[i]; j += NT) vals[offs[i] + j] = base[i][j];
    __syncthreads();
  }
  auto list = [&](uint32_t i) -> const float* { return LDS ? vals + offs[i] : base[i]; };

  // percentile positions over the union (numpy 'linear', as window_stats.hip)
  const float pct[3] = {p0, p1, p2};
  uint32_t pos[6];
  float frac[3];
  const uint32_t last = total ? total - 1 : 0;
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const double p = double(pct[q]) / 100.0 * double(last);
    uint32_t lo = uint32_t(floor(p));
    if (lo > last) lo = last;
    pos[2 * q] = lo;
    pos[2 * q + 1] = lo + 1 < total ? lo + 1 : last;
    frac[q] = float(p - double(lo));
  }

  // every element's rank in the merged order: its index in its own list + the elements
  // of the other lists before it (ties: lists with a smaller index first)
  double sum = 0.0;
  for (uint32_t i = 0; i < N; ++i) {
    const float* Li = list(i);
    for (uint32_t j = t; j < cnt[i]; j += NT) {
      const float x = Li[j];
      sum += double(x);
      uint32_t r = j;
      for (uint32_t k = 0; k < N; ++k) {
        if (k == i) continue;
        r += k < i ? upper_bound(list(k), cnt[k], x) : lower_bound(list(k), cnt[k], x);
      }
#pragma unroll
      for (int q = 0; q < 6; ++q)
        if (r == pos[q]) picked[q] = x;
    }
  }
  // sum in a fixed order: wave butterflies, then the waves in index order
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) sum += __shfl_xor(sum, off);
  if (lane == 0) red[wave] = sum;
  __syncthreads();

  if (t < STAT_NUM) {
    float o = __builtin_nanf("");
    if (t == STAT_COUNT) {
      o = float(total);
    } else if (total && t != STAT_LAST) {
      if (t == STAT_MIN || t == STAT_MAX) {
        float m = t == STAT_MIN ? INFINITY : -INFINITY;
        for (uint32_t i = 0; i < N; ++i)
          if (cnt[i]) m = t == STAT_MIN ? fminf(m, list(i)[0]) : fmaxf(m, list(i)[cnt[i] - 1]);
        o = m;
      } else if (t == STAT_MEAN) {
        double tot = 0.0;
        for (int w = 0; w < NT / 64; ++w) tot += red[w];
        o = float(tot / double(total));
      } else {
        const int q = t - STAT_P0;
        const double x0 = picked[2 * q], x1 = picked[2 * q + 1];
        const double f = frac[q];
        o = float(f >= 0.5 ? x1 - (x1 - x0) * (1.0 - f) : x0 + (x1 - x0) * f);
      }
    }
    out[size_t(s) * STAT_NUM + t] = o;
  }
}

}  // namespace

int launch_node_select(const float* node, uint32_t N, uint32_t S, uint32_t W, float p0, float p1, float p2, float* out,
                       void* stream_ptr) {
  if (N == 0 || S == 0) return hipSuccess;
  if (N > uint32_t(kMaxLists) || W == 0) return hipErrorInvalidValue;
  auto stream = static_cast<hipStream_t>(stream_ptr);
  if (uint64_t(N) * W <= kLdsFloats) {
    static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&node_select_kernel<true>),
                                                       hipFuncAttributeMaxDynamicSharedMemorySize,
                                                       int(kLdsFloats * sizeof(float)));
    if (attr != hipSuccess) return attr;
    hipLaunchKernelGGL(node_select_kernel<true>, dim3(S), dim3(NT), size_t(N) * W * sizeof(float), stream, node, N, S,
                       W, p0, p1, p2, out);
  } else {
    hipLaunchKernelGGL(node_select_kernel<false>, dim3(S), dim3(NT), 0, stream, node, N, S, W, p0, p1, p2, out);
  }
  return hipGetLastError();
}

// DeviceWindowSet::export_sorted lives here with its kernel (device_window.h declares it)
void DeviceWindowSet::export_sorted(float* dst, void* stream_ptr) const {
  auto stream = static_cast<hipStream_t>(stream_ptr);
  int prev = -1;
  (void)hipGetDevice(&prev);
  if (prev != device_) (void)hipSetDevice(device_);
  ExportArgs a{};
  uint32_t n = 0, first = 0;
  auto flush = [&]() {
    if (!n) return;
    hipLaunchKernelGGL(export_sorted_kernel, dim3(n), dim3(NT), 0, stream, a, dst + size_t(first) * (window_ + 1),
                       window_);
    first += n;
    n = 0;
  };
  for (const auto& r : rings_) {
    for (uint32_t c = 0; c < r.ring->width(); ++c) {
      a.s[n++] = ExportRef{r.sorted + size_t(c) * 2 * window_, r.state + c, window_};
      if (n == uint32_t(kExportPerLaunch)) flush();
    }
  }
  flush();
  const hipError_t e = hipGetLastError();
  if (prev >= 0 && prev != device_) (void)hipSetDevice(prev);
  if (e != hipSuccess) throw std::runtime_error(std::string("export_sorted launch: ") + hipGetErrorString(e));
}

}  // namespace rocmdash
