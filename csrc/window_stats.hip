// CDNA4 (gfx950) windowed statistics over time-major metric rings.
//
// Reference counterpart: the pandas min/mean/max over GPUs at app.py:216-221 and the
// selected-GPU mean at app.py:338-345 - one instant sample per series. Here every
// series gets min / max / mean / three percentiles / last / count over its last
// W samples, for all series of all rings of this rank in ONE launch.
//
// Mapping to the hardware (cdna_hip_programming.md, MI355X_MICROARCH.md):
//   * one workgroup per series (grid = #series), NT = min(P, 1024) threads = up to
//     16 wave64s, E = P / NT samples per thread in registers, P = pow2 >= W;
//   * bitonic sort with the three classes of compare-exchange stages placed where
//     the partner lives:
//       j <  E        partner in the same thread   -> register min/max, unrolled
//       E <= j < 64E  partner in the same wave64   -> __shfl_xor (ds_bpermute, no LDS
//                                                     bank traffic, no barrier)
//       j >= 64E      partner in another wave      -> LDS round trip (blocked
//                                                     E-float rows: ds_write_b128 /
//                                                     ds_read_b128, conflict-free)
//     at W = 4096 that is 10 LDS stages out of 78;
//   * samples are loaded lane-consecutive (thread t takes rows t, t+NT, ...) so a
//     wave instruction touches 64 consecutive rows of the ring (the order of the
//     input is irrelevant to a sort); NaN and padding become +inf and sort last;
//   * sum / count reduce wave-level with __shfl_xor (64 lanes), then across waves
//     through LDS; the sorted window is staged in LDS once and lanes 0..7 each emit
//     one statistic (one 32-byte store per series).
// Percentiles use numpy's default 'linear' definition (tests/test_window_stats.py).

#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "window_stats.h"

namespace rocmdash {
namespace {

template <int NT, int E>
__global__ __launch_bounds__(NT) void window_stats_kernel(const StatsArgs args, float* __restrict__ out) {
  constexpr int P = NT * E;
  constexpr int NW = NT / 64;
  __shared__ __attribute__((aligned(16))) float lds[P];
  __shared__ double red_sum[NW];
  __shared__ unsigned red_cnt[NW];

  const int t = threadIdx.x;
  const SeriesDesc d = args.d[blockIdx.x];
  const uint64_t start = d.head - d.n;

  float a[E];
  float sum = 0.f;
  unsigned cnt = 0;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const uint32_t i = uint32_t(t) + uint32_t(NT) * e;
    float v = INFINITY;
    if (i < d.n) {
      const uint64_t row = (start + i) & d.mask;
      const float x = d.base[row * d.stride + d.col];
      if (!isnan(x)) {
        v = x;
        sum += x;
        ++cnt;
      }
    }
    a[e] = v;
  }

  // ---- bitonic sort, ascending, blocked layout: sort index = t * E + e ----------
  for (uint32_t k = 2; k <= uint32_t(P); k <<= 1) {
    uint32_t j = k >> 1;
    // (1) partner in another wave: LDS round trip.
    for (; j >= 64u * E; j >>= 1) {
      __syncthreads();  // previous stage's partner reads are done
#pragma unroll
      for (int e = 0; e < E; ++e) lds[t * E + e] = a[e];
      __syncthreads();
      const int m = int(j / E);
      const int pt = t ^ m;
      const bool keep_min = ((t & m) == 0) == (((uint32_t(t) * E) & k) == 0);
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const float w = lds[pt * E + e];
        a[e] = keep_min ? fminf(a[e], w) : fmaxf(a[e], w);
      }
    }
    // (2) partner in the same wave: lane xor m, m in [1, 32].
    for (; j >= uint32_t(E); j >>= 1) {
      const int m = int(j / E);
      const bool keep_min = ((t & m) == 0) == (((uint32_t(t) * E) & k) == 0);
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const float w = __shfl_xor(a[e], m);
        a[e] = keep_min ? fminf(a[e], w) : fmaxf(a[e], w);
      }
    }
    // (3) partner in the same thread: compile-time register pairs.
#pragma unroll
    for (int jj = E / 2; jj >= 1; jj >>= 1) {
      if (uint32_t(jj) < k) {
#pragma unroll
        for (int e = 0; e < E; ++e) {
          if ((e & jj) == 0) {
            const int f = e | jj;
            const bool asc = ((uint32_t(t) * E + e) & k) == 0;
            const float lo = fminf(a[e], a[f]);
            const float hi = fmaxf(a[e], a[f]);
            a[e] = asc ? lo : hi;
            a[f] = asc ? hi : lo;
          }
        }
      }
    }
  }

  // ---- reductions + stage the sorted window in LDS -------------------------------
  double ds = sum;
  unsigned c = cnt;
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    ds += __shfl_xor(ds, off);
    c += __shfl_xor(c, off);
  }
  __syncthreads();  // last LDS-stage reads are done before the buffer is rewritten
  if ((t & 63) == 0) {
    red_sum[t >> 6] = ds;
    red_cnt[t >> 6] = c;
  }
#pragma unroll
  for (int e = 0; e < E; ++e) lds[t * E + e] = a[e];
  __syncthreads();

  if (t < STAT_NUM) {
    double total = 0.0;
    unsigned nv = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      total += red_sum[w];
      nv += red_cnt[w];
    }
    const float qnan = __builtin_nanf("");
    float r = qnan;
    if (t == STAT_COUNT) {
      r = float(nv);
    } else if (t == STAT_LAST) {
      if (d.head) r = d.base[((d.head - 1) & d.mask) * d.stride + d.col];
    } else if (nv) {
      if (t == STAT_MIN) {
        r = lds[0];
      } else if (t == STAT_MAX) {
        r = lds[nv - 1];
      } else if (t == STAT_MEAN) {
        r = float(total / double(nv));
      } else {
        const double pos = double(args.pct[t - STAT_P0]) / 100.0 * double(nv - 1);
        uint32_t lo = uint32_t(floor(pos));
        if (lo > nv - 1) lo = nv - 1;
        const uint32_t hi = lo + 1 < nv ? lo + 1 : nv - 1;
        const double frac = pos - double(lo);
        const double x0 = lds[lo], x1 = lds[hi];
        r = float(frac >= 0.5 ? x1 - (x1 - x0) * (1.0 - frac) : x0 + (x1 - x0) * frac);
      }
    }
    out[size_t(blockIdx.x) * STAT_NUM + t] = r;
  }
}

template <int NT, int E>
hipError_t launch(const StatsArgs& args, float* out, hipStream_t stream) {
  hipLaunchKernelGGL((window_stats_kernel<NT, E>), dim3(args.num_series), dim3(NT), 0, stream, args, out);
  return hipGetLastError();
}

}  // namespace

uint32_t sort_width_for(uint32_t n) {
  uint32_t p = 64;
  while (p < n) p <<= 1;
  return p;
}

int launch_window_stats(const StatsArgs& args, uint32_t pad_pow2, float* out, void* stream_ptr) {
  if (args.num_series == 0) return hipSuccess;
  if (args.num_series > uint32_t(kMaxSeriesPerLaunch)) return hipErrorInvalidValue;
  auto stream = static_cast<hipStream_t>(stream_ptr);
  switch (pad_pow2) {
    case 64: return launch<64, 1>(args, out, stream);
    case 128: return launch<128, 1>(args, out, stream);
    case 256: return launch<256, 1>(args, out, stream);
    case 512: return launch<512, 1>(args, out, stream);
    case 1024: return launch<1024, 1>(args, out, stream);
    case 2048: return launch<1024, 2>(args, out, stream);
    case 4096: return launch<1024, 4>(args, out, stream);
    case 8192: return launch<1024, 8>(args, out, stream);
    case 16384: return launch<1024, 16>(args, out, stream);
    case 32768: return launch<1024, 32>(args, out, stream);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace rocmdash
