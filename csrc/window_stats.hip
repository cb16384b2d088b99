// CDNA4 (gfx950) windowed statistics over time-major metric rings.
//
// Reference counterpart: the pandas min/mean/max over GPUs at app.py:216-221 and the
// selected-GPU mean at app.py:338-345 - one instant sample per series. Here every
// series gets min / max / mean / three percentiles / last / count over its last
// W samples, for all series of all rings of this rank in ONE launch.
//
// Two paths, chosen per series (uniformly per workgroup) from the series' resident
// state (SeriesState, written by the previous launch on the same stream):
//
// INCREMENTAL (the steady state: a refresh sees k <= 256 new samples per series)
//   The sorted window of the previous refresh stays resident in HBM; this launch
//   merges it with the k samples that entered and removes the k' that left, IN PLACE:
//     (0) old sorted window -> registers (blocked chunk of E per thread, float4 loads)
//         and LDS (padded: conflict-free ds_write_b128); the leaving / entering samples
//         (read from the device ring, which holds 2W rows so the leaving rows are still
//         there) are sorted by one wave64 each in registers + __shfl_xor (no barrier);
//     (1) k searches over the LDS window give the old positions of the leaving samples
//         (taken from the END of their run of equal values) and the insertion points
//         of the entering ones (after their run);
//     (2) only the span [first change point, last change point] of the window moves;
//         it is rewritten in the resident buffer itself with coalesced stores:
//           k <= 1 (one new row per refresh): each position of the span is gathered
//             from its source in LDS (a shift by one around the entering sample);
//           more: each thread walks its chunk in registers (new rank = i - #leaving
//             before i + #entering before i, both changing only at the <= 2k change
//             points), scatters it into a second LDS buffer (conflict-free padding) and
//             the span is copied out in float4s;
//     (3) the order statistics are read at their positions; the sum is the old
//         window's minus the leaving plus the entering samples (fp64).
//   Work is O(W / NT + k log W) per thread instead of the O(W log^2 W) full sort, and
//   a steady series (one repeated value) rewrites one position per refresh.
//   ONE ROW IN / ONE OUT (the bench's steady state, 256-thread launches): no LDS copy
//   and no searches - each thread counts its register chunk against the two samples,
//   ballots of the count bits + one barrier give both positions, and each thread
//   shifts and stores its own chunk (0 LDS bank conflicts, profiles/r02/onerow/).
//
// FULL (first refresh, after invalidation, or > 256 new samples)
//   one workgroup per series, NT = min(P, 1024) threads = up to 16 wave64s, E = P / NT
//   samples per thread in registers, P = pow2 >= W; bitonic sort with the three
//   classes of compare-exchange stages placed where the partner lives:
//       j <  E        partner in the same thread   -> register min/max, unrolled
//       E <= j < 64E  partner in the same wave64   -> __shfl_xor (ds_bpermute, no LDS
//                                                     bank traffic, no barrier)
//       j >= 64E      partner in another wave      -> LDS round trip (blocked E-float
//                                                     rows: ds_write_b128 / ds_read_b128)
//   at W = 4096 that is 10 LDS stages out of 78. The result seeds the resident state.
//
// NaN samples (failed reads) are excluded from every statistic but `last`; padding
// and NaNs become +inf inside the sorts and are counted out. sum / count reduce
// wave-level with __shfl_xor (64 lanes), then across waves through LDS. Percentiles
// use numpy's default 'linear' definition (tests/test_gpu.py compares against an fp64
// PyTorch reference).

#include <hip/hip_runtime.h>

#include <cmath>
#include <cstddef>
#include <cstdint>
#include <cstdlib>

#include "window_stats.h"

// Diagnostic build only (-DWS_STAMPS, tools/stamps/): s_memtime stamps by thread 0
// of each workgroup at phase boundaries. In the real kernel no stamp executes.
#ifdef WS_STAMPS
__device__ unsigned long long g_ws_stamps[64][8];
#define WS_STAMP(k)                                                                   \
  do {                                                                                \
    __builtin_amdgcn_sched_barrier(0);                                                \
    unsigned long long t_;                                                            \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");      \
    __builtin_amdgcn_sched_barrier(0);                                                \
    if (threadIdx.x == 0 && series < 64) g_ws_stamps[series][k] = t_;                \
  } while (0)
#else
#define WS_STAMP(k) \
  do {            \
  } while (0)
#endif

namespace rocmdash {
namespace {

constexpr int KE = kMaxIncremental / 64;  // removed/added samples per lane in the wave sorts

__device__ inline uint32_t upper_bound(const float* a, uint32_t lo, uint32_t n, float x) {
  uint32_t hi = n;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (a[mid] <= x) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// Ascending bitonic sort of 64*E values held E per lane, blocked layout
// (sort index = lane * E + e); registers and cross-lane shuffles only.
template <int E>
__device__ inline void wave_sort(float (&a)[E], int lane) {
#pragma unroll
  for (uint32_t k = 2; k <= 64u * E; k <<= 1) {
    for (uint32_t j = k >> 1; j >= uint32_t(E); j >>= 1) {
      const int m = int(j / E);
      const bool keep_min = ((lane & m) == 0) == (((uint32_t(lane) * E) & k) == 0);
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const float w = __shfl_xor(a[e], m);
        a[e] = keep_min ? fminf(a[e], w) : fmaxf(a[e], w);
      }
    }
#pragma unroll
    for (int jj = E / 2; jj >= 1; jj >>= 1) {
      if (uint32_t(jj) < k) {
#pragma unroll
        for (int e = 0; e < E; ++e) {
          if ((e & jj) == 0) {
            const int f = e | jj;
            const bool asc = ((uint32_t(lane) * E + e) & k) == 0;
            const float lo = fminf(a[e], a[f]);
            const float hi = fmaxf(a[e], a[f]);
            a[e] = asc ? lo : hi;
            a[f] = asc ? hi : lo;
          }
        }
      }
    }
  }
}

// Padded LDS layout of the old window in the incremental path: 4 spare floats after
// every 2^PS. With PS = log2(E) a thread's blocked E-float chunk sits E + 4 floats from
// its neighbour's, an odd multiple of 16 B for E >= 8: the 8 lanes of each group of a
// ds_write_b128 cover all 32 banks (no conflict), and float4 runs stay 16-byte aligned.
template <int PS>
__device__ __forceinline__ uint32_t pad(uint32_t i) { return i + ((i >> PS) << 2); }
__host__ __device__ constexpr uint32_t padded_size(uint32_t n, int ps) { return n + ((n >> ps) << 2) + 4; }
__host__ __device__ constexpr int pad_shift(int E) { return E >= 32 ? 5 : E >= 16 ? 4 : E >= 8 ? 3 : 6; }

// Layout of the merged window in the walk path: 1 spare float after every 16, so the
// blocked scatter (lanes ~16 floats apart) hits 32 distinct banks with ds_write_b32.
__device__ __forceinline__ uint32_t pad2(uint32_t i) { return i + (i >> 4); }
__host__ __device__ constexpr uint32_t padded2_size(uint32_t n) { return n + (n >> 4) + 1; }

template <int PS>
__device__ inline uint32_t upper_bound_p(const float* a, uint32_t n, float x) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (a[pad<PS>(mid)] <= x) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// 64-ary upper_bound by a whole wave over an ascending (padded) LDS array: each round
// every lane tests one pivot and a ballot narrows the range 64-fold; the result is uniform.
template <int PS>
__device__ inline uint32_t wave_upper_bound(const float* a, uint32_t n, float x, int lane) {
  uint32_t lo = 0, len = n;
  while (len > 64) {
    uint32_t step = (len + 63) / 64;
    step += (step & 7u) == 0 ? 1u : 0u;  // pivots a multiple of 8 apart would share 2 LDS banks
    const uint32_t i = lo + uint32_t(lane) * step;
    const bool before = i < lo + len && a[pad<PS>(i)] <= x;
    const uint32_t c = __popcll(__ballot(before));  // chunks whose first element is <= x
    if (c == 0) return lo;
    const uint32_t end = lo + len;
    lo += (c - 1) * step;
    len = (lo + step < end ? lo + step : end) - lo;
  }
  const bool before = uint32_t(lane) < len && a[pad<PS>(lo + lane)] <= x;
  return lo + __popcll(__ballot(before));
}

__device__ inline uint32_t lower_bound_u(const uint32_t* a, uint32_t n, uint32_t x) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (a[mid] < x) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

__device__ inline uint32_t upper_bound_u(const uint32_t* a, uint32_t n, uint32_t x) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (a[mid] <= x) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// Value at position p of the merged window, found by binary searches (incremental path,
// windows too long for a second LDS buffer): entering sample a if it lands on p, else
// kept element m = p - a of the old window.
template <int PS>
__device__ inline float merged_at(const float* lds, const float* abuf, const uint32_t* pnew, const uint32_t* padj,
                                  uint32_t ka, uint32_t kr, uint32_t p) {
  const uint32_t a = lower_bound_u(pnew, ka, p);
  if (a < ka && pnew[a] == p) return abuf[a];
  const uint32_t m = p - a;
  return lds[pad<PS>(m + upper_bound_u(padj, kr, m))];
}

// The series state through the vector memory path (a buffer load into VGPRs). A plain
// load of this uniform address becomes a scalar load whose SGPRs the compiler spills
// to VGPR lanes at once - waiting for the load right there, before the incremental
// path's own loads could go out; in VGPRs it is first waited for where it is used.
__device__ inline SeriesState load_state_vmem(const SeriesState* p) {
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<SeriesState*>(p), 0, int(sizeof(SeriesState)), 0x00020000);
  const auto a = __builtin_amdgcn_raw_buffer_load_b128(r, 0, 0, 0);  // head (lo, hi), n, nvalid
  const auto b = __builtin_amdgcn_raw_buffer_load_b64(r, 16, 0, 0);   // cur, valid
  SeriesState s;
  s.head = uint64_t(a[0]) | (uint64_t(a[1]) << 32);
  s.n = a[2];
  s.nvalid = a[3];
  s.cur = b[0];
  s.valid = b[1];
  return s;
}

// One series as the kernel sees it: its ring's descriptor fields + its column.
struct SeriesView {
  float* base;
  const float* host_rows;
  float* sorted;
  SeriesState* state;
  const float* inl;  // &ring.inl[0][col]; row r at inl[r * kMaxInlineWidth]
  uint64_t head, pred_head0;
  uint32_t stride, col, mask, n, sorted_cap, host_mask, pred_n0, pred_cur, n_inline, ri, first, cols;
};

// The workgroup of column `col` of ring `ri` (blockIdx.x, blockIdx.y): its ring's
// fields come from ONE round of scalar loads at an offset known at launch - no kernarg
// load waits for another (a series -> ring search over the rings' column counts did:
// two dependent kernel-argument round trips before the first global load).
// RingDesc's fields before the inline rows, in the same order: copied in one go, so the
// compiler issues every scalar load of the ring before the first use waits for any.
struct RingHead {
  float* base;
  const float* host_rows;
  float* sorted;
  SeriesState* state;
  uint64_t head, pred_head0;
  uint32_t stride, cols, first, mask, n, sorted_cap, host_mask, pred_n0, pred_cur, n_inline;
};
static_assert(sizeof(RingHead) == offsetof(RingDesc, inl), "RingHead must mirror RingDesc's leading fields");

__device__ inline SeriesView make_view(const StatsArgs& args, uint32_t ri, uint32_t col) {
  RingHead R;
  __builtin_memcpy(&R, &args.rings[ri], sizeof R);
  SeriesView v;
  v.base = R.base;
  v.host_rows = R.host_rows;
  v.sorted = R.sorted;
  v.state = R.state;
  v.head = R.head;
  v.pred_head0 = R.pred_head0;
  v.stride = R.stride;
  v.mask = R.mask;
  v.n = R.n;
  v.sorted_cap = R.sorted_cap;
  v.host_mask = R.host_mask;
  v.pred_n0 = R.pred_n0;
  v.pred_cur = R.pred_cur;
  v.n_inline = R.n_inline;
  v.col = col;
  v.ri = ri;
  v.first = R.first;
  v.cols = R.cols;
  v.inl = &args.rings[ri].inl[0][0];  // indexed, not selected: keeps the kernarg a kernarg
  if (v.sorted) v.sorted += size_t(col) * 2 * v.sorted_cap;
  if (v.state) v.state += col;
  v.inl += col < uint32_t(kMaxInlineWidth) ? col : 0u;
  if (col >= uint32_t(kMaxInlineWidth)) v.n_inline = 0;
  return v;
}

// Sample `row` of a series: the newest rows by value from the kernel argument,
// older entering rows from the pinned host ring in pull mode - both then also stored
// into the device ring for the launch that later removes them - else from the device
// ring the host filled with hipMemcpyAsync.
__device__ inline float take_sample(const SeriesView& d, uint64_t row) {
  float x;
  if (row + d.n_inline >= d.head) {
    x = d.inl[(row + d.n_inline - d.head) * kMaxInlineWidth];  // by value, in the kernarg
  } else if (d.host_rows != nullptr) {
    x = d.host_rows[(row & d.host_mask) * d.stride + d.col];
  } else {
    return d.base[(row & d.mask) * d.stride + d.col];
  }
  d.base[(row & d.mask) * d.stride + d.col] = x;
  return x;
}

// The entering sample `row` without storing it (every thread of the one-row path reads
// it; thread 0 stores it): `store` tells whether it still has to go into the device ring.
__device__ inline float peek_sample(const SeriesView& d, uint64_t row, bool& store) {
  store = true;
  if (row + d.n_inline >= d.head) return d.inl[(row + d.n_inline - d.head) * kMaxInlineWidth];
  if (d.host_rows != nullptr) return d.host_rows[(row & d.host_mask) * d.stride + d.col];
  store = false;
  return d.base[(row & d.mask) * d.stride + d.col];
}

// Bits that hold a count in [0, E].
__host__ __device__ constexpr int count_bits(int e) { return e <= 1 ? 1 : 1 + count_bits(e >> 1); }

// One wave: read k (<= 64*E) consecutive ring rows of a series starting at `first`,
// sort them ascending (NaN and padding -> +inf, counted out) and store 64*E floats to
// LDS `dst`; `valid` / `sum` come back wave-reduced (same value in every lane).
template <int E>
__device__ inline void load_sort_store(const SeriesView& d, uint64_t first, uint32_t k, int lane, float* dst,
                                       unsigned& valid, double& sum, bool entering, float* lastv) {
  valid = 0;
  sum = 0.0;
  if (E == 1 && k <= 16) {
    // few rows (the steady state): rank sort - every lane counts, through k uniform
    // readlanes, the values that precede its own; no 21-stage shuffle network
    float v = INFINITY;
    if (uint32_t(lane) < k) {
      const float x = entering ? take_sample(d, first + lane) : d.base[((first + lane) & d.mask) * d.stride + d.col];
      if (entering && uint32_t(lane) == k - 1) *lastv = x;
      if (!isnan(x)) {
        v = x;
        valid = 1;
        sum = x;
      }
    }
    uint32_t rank = 0;
    for (uint32_t j = 0; j < k; ++j) {
      const float w = __shfl(v, int(j));
      rank += (w < v || (w == v && j < uint32_t(lane))) ? 1u : 0u;
    }
    dst[uint32_t(lane) < k ? rank : uint32_t(lane)] = v;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
      valid += __shfl_xor(valid, off);
      sum += __shfl_xor(sum, off);
    }
    return;
  }
  float a[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const uint32_t i = uint32_t(lane) * E + e;
    float v = INFINITY;
    if (i < k) {
      // leaving rows are always in the device ring; entering rows come from the source
      const float x = entering ? take_sample(d, first + i) : d.base[((first + i) & d.mask) * d.stride + d.col];
      if (entering && i == k - 1) *lastv = x;  // newest raw sample (may be NaN)
      if (!isnan(x)) {
        v = x;
        ++valid;
        sum += x;
      }
    }
    a[e] = v;
  }
  wave_sort<E>(a, lane);
#pragma unroll
  for (int e = 0; e < E; ++e) dst[lane * E + e] = a[e];
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    valid += __shfl_xor(valid, off);
    sum += __shfl_xor(sum, off);
  }
}

// Wave64 sums through DPP (VALU lane moves, no LDS pipeline): xor 1 and xor 2 inside
// each quad, the half-row and row mirrors, so every lane of a 16-lane row holds the row
// sum; the four row sums are then read from lanes 0 / 16 / 32 / 48. (The shuffles they
// replace were ds_bpermute round trips, 12 dependent ones for one double.)
template <int Ctrl>
__device__ __forceinline__ double dpp_f64(double v) {
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const int lo = __builtin_amdgcn_update_dpp(0, int(uint32_t(u)), Ctrl, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, int(uint32_t(u >> 32)), Ctrl, 0xF, 0xF, false);
  return __builtin_bit_cast(double, uint64_t(uint32_t(lo)) | (uint64_t(uint32_t(hi)) << 32));
}

__device__ inline double wave_sum(double v) {
  v += dpp_f64<0xB1>(v);   // quad_perm [1, 0, 3, 2]
  v += dpp_f64<0x4E>(v);   // quad_perm [2, 3, 0, 1]
  v += dpp_f64<0x141>(v);  // row_half_mirror
  v += dpp_f64<0x140>(v);  // row_mirror
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  double r = 0.0;
#pragma unroll
  for (int row = 0; row < 4; ++row) {
    const uint32_t lo = uint32_t(__builtin_amdgcn_readlane(int(uint32_t(u)), 16 * row));
    const uint32_t hi = uint32_t(__builtin_amdgcn_readlane(int(uint32_t(u >> 32)), 16 * row));
    r += __builtin_bit_cast(double, uint64_t(lo) | (uint64_t(hi) << 32));
  }
  return r;
}

__device__ inline uint32_t wave_sum(uint32_t v) {
  v += uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0xB1, 0xF, 0xF, false));
  v += uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x4E, 0xF, 0xF, false));
  v += uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x141, 0xF, 0xF, false));
  v += uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x140, 0xF, 0xF, false));
  return uint32_t(__builtin_amdgcn_readlane(int(v), 0)) + uint32_t(__builtin_amdgcn_readlane(int(v), 16)) +
         uint32_t(__builtin_amdgcn_readlane(int(v), 32)) + uint32_t(__builtin_amdgcn_readlane(int(v), 48));
}

// Sorted positions the outputs need: [min, max, lo0, hi0, lo1, hi1, lo2, hi2].
__device__ inline void wanted_positions(uint32_t nv, const double qfrac[3], uint32_t (&idx)[8], float (&frac)[3]) {
  const uint32_t last = nv ? nv - 1 : 0;
  idx[0] = 0;
  idx[1] = last;
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const double pos = qfrac[q] * double(last);  // qfrac = double(pct) / 100, host-computed
    uint32_t lo = uint32_t(floor(pos));
    if (lo > last) lo = last;
    idx[2 + 2 * q] = lo;
    idx[3 + 2 * q] = lo + 1 < nv ? lo + 1 : last;
    frac[q] = float(pos - double(lo));
  }
}

template <int NT, int E>
__global__ __launch_bounds__(NT) void window_stats_kernel(const StatsArgs args, float* __restrict__ out) {
  constexpr int P = NT * E;
  constexpr int NW = NT / 64;
  constexpr int PS = pad_shift(E);
  __shared__ __attribute__((aligned(16))) float lds[padded_size(P, PS)];
  __shared__ float rbuf[kMaxIncremental];
  __shared__ float abuf[kMaxIncremental];
  __shared__ double red_sum[NW];
  __shared__ unsigned red_cnt[NW];
  __shared__ float wv[8];
  __shared__ unsigned kcount[2];
  __shared__ double asum, rsum;
  __shared__ uint32_t prem[kMaxIncremental];  // old-window positions of leaving samples
  __shared__ uint32_t qins[kMaxIncremental];  // old-window insertion points of entering ones
  __shared__ uint32_t pnew[kMaxIncremental];  // new-window positions of entering samples
  __shared__ uint32_t padj[kMaxIncremental];  // prem[r] - r
  __shared__ int bad;
  __shared__ float lastv;
  __shared__ uint32_t fcnt[NW][3];  // one-row path: per-wave counts
  __shared__ float edge_lo[NW][E / 4 > 0 ? E / 4 : 1], edge_hi[NW][E / 4 > 0 ? E / 4 : 1];  // and wave edges
  // the walk path assembles the merged window in a second LDS buffer when both fit
  constexpr bool kLdsOut = P <= 16384;
  // the one-row path in the 256-thread steady-state configuration (W <= 8192); with
  // 1024 threads it measured ~1 us slower than the general path (profiles/r02)
  constexpr bool kOneRowPath = NT <= 1024 && E % 4 == 0 && P <= 8192;
  __shared__ float lds2[kLdsOut ? padded2_size(P) : 1];

  const int t = threadIdx.x;
  const int lane = t & 63;
  const int wave = t >> 6;
  const uint32_t ring = blockIdx.y, col = blockIdx.x;
  const SeriesView d = make_view(args, ring, col);  // issued before the exit test below waits
  const uint32_t series = d.first + col;  // output row
  if (col >= d.cols) return;  // the grid is max(cols) x rings: whole workgroup, before any barrier
  WS_STAMP(0);
  const uint64_t h1 = d.head;
  const uint32_t n1 = d.n;
  const uint64_t s1 = h1 - n1;

  // ---- path selection (uniform: every input is a kernel argument or one state load)
  // With a host prediction of the state the previous launch left (head, n, half), the
  // incremental path issues all of its loads - state, old window, leaving and
  // entering rows - at once and validates the prediction when the state arrives; a
  // mismatch falls back to the full sort. Without one, it first waits for the state.
  const bool predicted = d.state != nullptr && d.pred_head0 != ~0ull;
  SeriesState st{0, 0, 0, 0, 0};
  uint64_t h0 = 0;
  uint32_t n0 = 0, cur = 0;
  bool have_state = false;
  if (predicted) {
    h0 = d.pred_head0;
    n0 = d.pred_n0;
    cur = d.pred_cur;
    have_state = true;
  } else if (d.state != nullptr) {  // no prediction: the selection waits for the state
    st = *d.state;
    h0 = st.head;
    n0 = st.n;
    cur = st.cur;
    have_state = st.valid != 0;
  }
  // with a prediction the state load is only issued here: nothing before the paths'
  // own loads (old window, leaving / entering rows) waits for it - it is first used
  // by their validation
  if (predicted) st = load_state_vmem(d.state);
  bool inc = false;
  uint32_t kadd = 0, krem = 0;
  if (have_state && h1 >= h0 && n0 <= h0 && cur <= 1) {
    const uint64_t s0 = h0 - n0;
    if (s1 >= s0 && h1 - h0 <= uint64_t(kMaxIncremental) && s1 - s0 <= uint64_t(kMaxIncremental) &&
        s0 + uint64_t(d.mask) + 1 >= h1 && n0 <= d.sorted_cap && n1 <= d.sorted_cap) {
      inc = true;
      kadd = uint32_t(h1 - h0);
      krem = uint32_t(s1 - s0);
    }
  }
  const bool inc_selected = inc;  // a fall-back below clears `inc`, not this

  double sum = 0.0;
  unsigned cnt = 0;
  uint32_t nv = 0;
  uint32_t idx[8];
  float frac[3];

  bool onerow = false;  // the one-row path ran: its order statistics are in `lds`
  if (kOneRowPath && inc && kadd <= 1u && krem <= 1u && (d.sorted_cap & 3u) == 0) {
    // ==================== INCREMENTAL, at most one row in and one out ====================
    // The steady state (one new row per refresh) without an LDS copy of the window or
    // searches over it. Each thread holds G = E / 4 float4 groups of the old window in
    // registers, STRIPED: group g covers positions 4 (t + NT g) .. + 3, so every float4
    // load and store instruction of a wave touches 1 KiB of consecutive memory. It
    // counts its elements < / <= the leaving sample and <= the entering one; the block's
    // totals (ballots of the count bits, one barrier) are the leaving sample's position
    // at the end of its run and the entering one's insertion point after its run: what
    // the searches of the general path return. Each thread then shifts its groups in
    // registers (neighbours from the adjacent lanes, across waves through LDS) and
    // stores the groups that meet the changed span; the new groups also go to LDS in
    // natural order, where the outputs read their order statistics.
    constexpr int G = E / 4 > 0 ? E / 4 : 1;  // (E >= 4 whenever this path runs)
    const uint64_t s0 = h0 - n0;
    const uint32_t cap = d.sorted_cap;
    float* Sres = d.sorted + size_t(cur) * cap;
    // straight-line float4 loads, all in flight at once: the buffer has a sort width of
    // slack past every half (device_window.cpp) and cap % 4 == 0, so no group needs a
    // bounds branch (positions past the valid entries are masked below)
    float xs[G][4];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const float4 v = *reinterpret_cast<const float4*>(Sres + 4u * (uint32_t(t) + uint32_t(NT) * g));
      xs[g][0] = v.x;
      xs[g][1] = v.y;
      xs[g][2] = v.z;
      xs[g][3] = v.w;
    }
    // the leaving row is in the device ring; the entering one by value in the kernel
    // argument (or the pinned host ring): uniform addresses, loaded by every thread
    bool ring_store = false;
    const float rs = krem ? d.base[(s0 & d.mask) * d.stride + d.col] : __builtin_nanf("");
    float as = __builtin_nanf("");
    if (kadd) {
      if (h0 + d.n_inline >= d.head) {  // by value in the kernel argument: a scalar load
        as = args.rings[d.ri].inl[h0 + d.n_inline - d.head][d.col];
        ring_store = true;
      } else {
        as = peek_sample(d, h0, ring_store);
      }
    }
    const bool state_ok = st.valid && st.head == h0 && st.n == n0 && st.cur == cur && st.nvalid <= cap;
    const uint32_t n0v = state_ok ? st.nvalid : 0;
    double old_sum = 0.0;
    uint32_t c_lt = 0, c_le = 0, c_la = 0;  // elements < rs, <= rs, <= as (NaN: none)
#pragma unroll
    for (int g = 0; g < G; ++g) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {  // branch-free: selects only
        const bool valid = 4u * (uint32_t(t) + uint32_t(NT) * g) + e < n0v;
        const float x = xs[g][e];
        xs[g][e] = valid ? x : INFINITY;
        old_sum += valid ? double(x) : 0.0;
        c_lt += valid && x < rs ? 1u : 0u;
        c_le += valid && x <= rs ? 1u : 0u;
        c_la += valid && x <= as ? 1u : 0u;
      }
    }
    uint32_t w_lt = 0, w_le = 0, w_la = 0;
#pragma unroll
    for (int bit = 0; bit < count_bits(E); ++bit) {
      w_lt += uint32_t(__popcll(__ballot((c_lt >> bit) & 1u))) << bit;
      w_le += uint32_t(__popcll(__ballot((c_le >> bit) & 1u))) << bit;
      w_la += uint32_t(__popcll(__ballot((c_la >> bit) & 1u))) << bit;
    }
    if (lane == 0) {
      fcnt[wave][0] = w_lt;
      fcnt[wave][1] = w_le;
      fcnt[wave][2] = w_la;
    }
    // the wave's edge elements, for the neighbours across waves
#pragma unroll
    for (int g = 0; g < G; ++g) {
      if (lane == 0) edge_lo[wave][g] = xs[g][0];
      if (lane == 63) edge_hi[wave][g] = xs[g][3];
    }
    // neighbours inside the wave: the adjacent lanes' edge elements (DPP wave shifts,
    // VALU lane moves; lanes 0 / 63 are filled from LDS after the barrier)
    float left[G], right[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      left[g] = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, xs[g][3]), 0x138,
                                                                        0xF, 0xF, false));  // wave_shr:1
      right[g] = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, xs[g][0]), 0x130,
                                                                         0xF, 0xF, false));  // wave_shl:1
    }
    WS_STAMP(1);
    __syncthreads();
    WS_STAMP(2);
    if (t == 0 && kadd) {  // after the barrier: no load of the phase above waits for it
      if (ring_store) d.base[(h0 & d.mask) * d.stride + d.col] = as;  // for the launch it leaves in
      lastv = as;  // newest raw sample (may be NaN)
    }
    uint32_t lt = 0, le = 0, la = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      lt += fcnt[w][0];
      le += fcnt[w][1];
      la += fcnt[w][2];
    }
    // position 4 (t + NT g) - 1 of lane 0 is the previous wave's last lane (for wave
    // 0, the last thread's previous group); + 4 of lane 63 likewise the next wave's
#pragma unroll
    for (int g = 0; g < G; ++g) {
      if (lane == 0) left[g] = wave > 0 ? edge_hi[wave - 1][g] : (g > 0 ? edge_hi[NW - 1][g - 1] : -INFINITY);
      if (lane == 63) right[g] = wave < NW - 1 ? edge_lo[wave + 1][g] : (g < G - 1 ? edge_lo[0][g + 1] : INFINITY);
    }
    WS_STAMP(3);
    const uint32_t kr = krem && !isnan(rs) ? 1u : 0u;
    const uint32_t ka = kadd && !isnan(as) ? 1u : 0u;
    if (!state_ok || (kr && le == lt)) {
      inc = false;  // stale prediction, or the state does not hold the leaving sample
      __syncthreads();
    } else {
      onerow = true;
      nv = n0v - kr + ka;
      wanted_positions(nv, args.qfrac, idx, frac);
      const uint32_t x = kr ? le - 1u : 0xFFFFFFFFu;  // old position of the leaving sample
      const uint32_t pn = ka ? la - (x < la ? 1u : 0u) : 0xFFFFFFFFu;  // new position of the entering one
      uint32_t lo = x;
      if (ka && la < lo) lo = la;
      uint32_t hi = nv;
      if (kr == ka) {
        hi = kr ? x + 1u : 0u;
        if (ka && la > hi) hi = la;
        if (hi > nv) hi = nv;
      }
      // new groups: position p takes the entering sample or the kept old element
      // m + (x <= m), m = p - (pn < p): one of the old elements p - 1, p, p + 1
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const uint32_t q = 4u * (uint32_t(t) + uint32_t(NT) * g);
        float4 v4 = make_float4(xs[g][0], xs[g][1], xs[g][2], xs[g][3]);
        // only groups that meet [lo, hi) change (outside the span the values stay, past
        // nv the buffer is don't-care); whole waves outside it skip the shift
        if (q < hi && q + 4u > lo) {
          float nw[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const uint32_t p = q + uint32_t(e);
            const uint32_t m = p - (pn < p ? 1u : 0u);
            const uint32_t src = m + (x <= m ? 1u : 0u);
            const float prev = e == 0 ? left[g] : xs[g][e - 1];
            const float next = e == 3 ? right[g] : xs[g][e + 1];
            const float v = src < p ? prev : (src == p ? xs[g][e] : next);
            nw[e] = p == pn ? as : v;
          }
          v4 = make_float4(nw[0], nw[1], nw[2], nw[3]);
          *reinterpret_cast<float4*>(Sres + q) = v4;  // cap % 4 == 0: never past the half
        }
        *reinterpret_cast<float4*>(lds + q) = v4;  // natural order: lanes 16 B apart
      }
      WS_STAMP(4);
      sum = old_sum;
      if (t == 0) sum += (ka ? double(as) : 0.0) - (kr ? double(rs) : 0.0);
      cnt = t == 0 ? nv : 0;
      WS_STAMP(5);
    }
  } else if (inc) {
    // ================================ INCREMENTAL =================================
    const uint64_t s0 = h0 - n0;
    const float* S = d.sorted + size_t(cur) * d.sorted_cap;
    double old_sum = 0.0;
    // (0) the old sorted window: blocked chunk [b, b + E) per thread, loaded before the
    //     number of valid entries is known (the buffer holds sorted_cap floats), kept in
    //     registers and staged in LDS for the searches of step (1)
    const uint32_t b = uint32_t(t) * E;
    float xs[E];
    if (E % 4 == 0 && b + E <= d.sorted_cap) {
#pragma unroll
      for (int v = 0; v < E / 4; ++v) {
        const float4 q = reinterpret_cast<const float4*>(S + b)[v];
        xs[4 * v] = q.x;
        xs[4 * v + 1] = q.y;
        xs[4 * v + 2] = q.z;
        xs[4 * v + 3] = q.w;
      }
    } else {
#pragma unroll
      for (int e = 0; e < E; ++e) xs[e] = b + e < d.sorted_cap ? S[b + e] : INFINITY;
    }
    //     ... meanwhile one wave each sorts the leaving (R) and entering (A) samples
#pragma unroll
    for (int list = 0; list < 2; ++list) {
      if (wave == (list % NW)) {
        const uint64_t first = list == 0 ? s0 : h0;  // = st.head when the prediction holds (validated below)
        const uint32_t k = list == 0 ? krem : kadd;
        float* dst = list == 0 ? rbuf : abuf;
        // sort width = smallest of 64 / 128 / 256 that holds k (wave-uniform branch)
        unsigned valid;
        double ls;
        const bool entering = list == 1;
        if (k <= 64) load_sort_store<1>(d, first, k, lane, dst, valid, ls, entering, &lastv);
        else if (k <= 128) load_sort_store<2>(d, first, k, lane, dst, valid, ls, entering, &lastv);
        else load_sort_store<KE>(d, first, k, lane, dst, valid, ls, entering, &lastv);
        if (lane == 0) {
          kcount[list] = valid;
          if (list == 1) asum = ls;
          else rsum = ls;
        }
      }
    }
    // the state has arrived by now: validate the prediction (uniform), mask the chunk
    const bool state_ok = st.valid && st.head == h0 && st.n == n0 && st.cur == cur && st.nvalid <= d.sorted_cap;
    const uint32_t n0v = state_ok ? st.nvalid : 0;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      if (b + e >= n0v) xs[e] = INFINITY;
      else old_sum += xs[e];
    }
    if constexpr (E % 4 == 0) {
#pragma unroll
      for (int v = 0; v < E / 4; ++v)
        *reinterpret_cast<float4*>(lds + pad<PS>(b + 4 * v)) = make_float4(xs[4 * v], xs[4 * v + 1], xs[4 * v + 2], xs[4 * v + 3]);
    } else {
#pragma unroll
      for (int e = 0; e < E; ++e) lds[pad<PS>(b + e)] = xs[e];
    }
    if (t == 0) bad = state_ok ? 0 : 1;
    WS_STAMP(1);
    __syncthreads();
    WS_STAMP(2);
    const uint32_t kr = kcount[0], ka = kcount[1];
    // (1) where the leaving samples sit in the old window and where the entering ones
    //     go. Equal values are interchangeable, so a leaving value is taken from the
    //     END of its run of equal old elements (the j-th of c equal leaving samples at
    //     upper_bound - c + j) and an entering one goes after its run (upper_bound):
    //     a steady series (one repeated value) then changes one position per refresh,
    //     not its whole run. k searches over the LDS window.
    if (kr + ka <= uint32_t(2 * NW)) {
      // few items (the steady state: one new row per refresh): one wave per item,
      // 64-ary searches = 2 dependent LDS reads for a 4096-sample window instead of 12
      for (uint32_t item = wave; item < kr + ka; item += NW) {
        if (item < kr) {
          const uint32_t j = item;
          const float r = rbuf[j];
          const uint32_t ub = wave_upper_bound<PS>(lds, n0v, r, lane);
          const uint32_t c = upper_bound(rbuf, j, kr, r);  // equal leaving samples before + incl. j's run end
          if (lane == 0) {
            const bool ok = ub + j >= c && ub + j - c < n0v && lds[pad<PS>(ub + j - c)] == r;
            if (!ok) bad = 1;  // state does not hold this sample
            prem[j] = ok ? ub + j - c : 0u;
          }
        } else {
          const uint32_t j = item - kr;
          const uint32_t q = wave_upper_bound<PS>(lds, n0v, abuf[j], lane);
          if (lane == 0) qins[j] = q;
        }
      }
    } else {  // one thread per item, leaving and entering ones side by side
      for (uint32_t item = t; item < kr + ka; item += NT) {
        if (item < kr) {
          const uint32_t j = item;
          const float r = rbuf[j];
          const uint32_t ub = upper_bound_p<PS>(lds, n0v, r);
          const uint32_t c = upper_bound(rbuf, j, kr, r);
          const bool ok = ub + j >= c && ub + j - c < n0v && lds[pad<PS>(ub + j - c)] == r;
          if (!ok) bad = 1;
          prem[j] = ok ? ub + j - c : 0u;
        } else {
          qins[item - kr] = upper_bound_p<PS>(lds, n0v, abuf[item - kr]);
        }
      }
    }
    __syncthreads();
    WS_STAMP(3);
    if (bad || kr > n0v) {
      inc = false;  // inconsistent state: rebuild with the full sort (uniform branch)
      __syncthreads();
    } else {
      nv = n0v - kr + ka;
      wanted_positions(nv, args.qfrac, idx, frac);
      // (2) only positions [lo, hi) of the new window can differ from the old one:
      //     below the first change point nothing moved, and with as many samples in as
      //     out nothing moved past the last one either. That span is rewritten in
      //     place in the resident buffer; consecutive lanes take consecutive positions
      //     (coalesced stores).
      uint32_t lo = kr ? prem[0] : 0xFFFFFFFFu;
      if (ka && qins[0] < lo) lo = qins[0];
      uint32_t hi = nv;
      if (kr == ka) {
        hi = kr ? prem[kr - 1] + 1 : 0u;
        if (ka && qins[ka - 1] > hi) hi = qins[ka - 1];
        if (hi > nv) hi = nv;
      }
      float* Sres = d.sorted + size_t(cur) * d.sorted_cap;
      // Entering sample j lands on pnew[j] = qins[j] - #(prem < qins[j]) + j; the m-th
      // kept old element sits at old index m + #(padj <= m), padj[r] = prem[r] - r.
      if (kr <= 1u && ka <= 1u) {
        // (3a) at most one sample out and one in (the steady state: one new row per
        //      refresh): the span is a shift by one around the entering sample, each
        //      position gathered from its source - no merge buffer, no barrier
        const uint32_t x = kr ? prem[0] : 0xFFFFFFFFu;  // old position of the leaving sample
        const uint32_t pn = ka ? qins[0] - (x < qins[0] ? 1u : 0u) : 0xFFFFFFFFu;  // new position of the entering one
        const float av = ka ? abuf[0] : 0.f;
        auto at = [&](uint32_t p) -> float {
          if (p == pn) return av;
          const uint32_t m = p - (pn < p ? 1u : 0u);  // kept-element index
          return lds[pad<PS>(m + (x <= m ? 1u : 0u))];
        };
        for (uint32_t p = lo + uint32_t(t); p < hi; p += NT) Sres[p] = at(p);
        if (t < 8) wv[t] = at(idx[t]);
      } else if constexpr (kLdsOut) {
        // (3b) more samples: each thread walks its blocked chunk in registers - new
        //      rank = i - #leaving before i + #entering before i, both counts changing
        //      only at the <= 2k change points - and scatters it into the merge buffer
        //      (conflict-free padding); then the span is copied out
        uint32_t r = lower_bound_u(prem, kr, b);  // leaving positions < b
        uint32_t q = upper_bound_u(qins, ka, b);  // insertion points <= b
        uint32_t next_r = r < kr ? prem[r] : 0xFFFFFFFFu;
        uint32_t next_q = q < ka ? qins[q] : 0xFFFFFFFFu;
#pragma unroll
        for (int e = 0; e < E; ++e) {
          const uint32_t i = b + e;
          if (i < n0v) {
            if (i == next_r) {  // this element leaves the window
              ++r;
              next_r = r < kr ? prem[r] : 0xFFFFFFFFu;
            } else {
              while (next_q <= i) {
                ++q;
                next_q = q < ka ? qins[q] : 0xFFFFFFFFu;
              }
              lds2[pad2(i - r + q)] = xs[e];
            }
          }
        }
        for (uint32_t j = t; j < ka; j += NT) {
          const uint32_t qj = qins[j];
          lds2[pad2(qj - lower_bound_u(prem, kr, qj) + j)] = abuf[j];
        }
        __syncthreads();
        // span copy-out in aligned float4s (positions of [lo & ~3, hi) outside the span
        // are rewritten with their unchanged values; past nv the buffer is don't-care)
        if (d.sorted_cap % 4 == 0) {
          const uint32_t lo4 = lo & ~3u;
#pragma unroll 2
          for (uint32_t p = lo4 + 4u * uint32_t(t); p < hi; p += 4u * NT) {
            const uint32_t q0 = pad2(p);  // the 4 floats never straddle a pad slot (p % 4 == 0)
            *reinterpret_cast<float4*>(Sres + p) = make_float4(lds2[q0], lds2[q0 + 1], lds2[q0 + 2], lds2[q0 + 3]);
          }
        } else {
          for (uint32_t p = lo + uint32_t(t); p < hi; p += NT) Sres[p] = lds2[pad2(p)];
        }
        if (t < 8) wv[t] = lds2[pad2(idx[t])];
      } else {
        // (3c) more samples, window too long for a merge buffer: binary searches
        for (uint32_t j = t; j < ka; j += NT) pnew[j] = qins[j] - lower_bound_u(prem, kr, qins[j]) + j;
        for (uint32_t j = t; j < kr; j += NT) padj[j] = prem[j] - j;
        __syncthreads();
        for (uint32_t p = lo + uint32_t(t); p < hi; p += NT) Sres[p] = merged_at<PS>(lds, abuf, pnew, padj, ka, kr, p);
        if (t < 8) wv[t] = merged_at<PS>(lds, abuf, pnew, padj, ka, kr, idx[t]);
      }
      WS_STAMP(4);
      // sum of the new window = old window - leaving + entering (fp64)
      sum = old_sum;
      if (t == 0) sum += asum - rsum;
      cnt = t == 0 ? nv : 0;
      WS_STAMP(5);
    }
  }

  if (!inc) {
    // =================================== FULL =====================================
    const uint64_t start = s1;
    float a[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const uint32_t i = uint32_t(t) + uint32_t(NT) * e;
      float v = INFINITY;
      if (i < n1) {
        const float x = take_sample(d, start + i);
        if (i == n1 - 1) lastv = x;
        if (!isnan(x)) {
          v = x;
          sum += x;
          ++cnt;
        }
      }
      a[e] = v;
    }
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
    __syncthreads();  // last LDS-stage reads are done before the buffer is rewritten
#pragma unroll
    for (int e = 0; e < E; ++e) lds[t * E + e] = a[e];
  }

  // the incremental path updates half `cur` in place; a full sort (first refresh or
  // rebuild) writes the other half (or half 0 without state). A fall-back from the
  // incremental path keeps `cur`: its sort does not read the resident window.
  auto next_half = [&]() -> uint32_t { return inc_selected ? cur : (st.valid ? (st.cur ^ 1u) : 0u); };

  // ---- reductions (both paths): sum and count per wave, then across waves --------
  const double ds = wave_sum(sum);
  const unsigned c = wave_sum(uint32_t(cnt));
  if (lane == 0) {
    red_sum[wave] = ds;
    red_cnt[wave] = c;
  }
  __syncthreads();
  WS_STAMP(6);
  double total = 0.0;
  unsigned nvt = 0;
#pragma unroll
  for (int w = 0; w < NW; ++w) {
    total += red_sum[w];
    nvt += red_cnt[w];
  }
  nv = nvt;
  if (!inc) {
    wanted_positions(nv, args.qfrac, idx, frac);
    if (t < 8) wv[t] = lds[idx[t]];
    if (d.sorted != nullptr) {  // seed the resident state with the sorted window
      float* Sout = d.sorted + size_t(next_half()) * d.sorted_cap;
      for (uint32_t i = t; i < nv; i += NT) Sout[i] = lds[i];
    }
    __syncthreads();
  }
  if (t == 0 && d.state != nullptr) {
    SeriesState ns;
    ns.head = h1;
    ns.n = n1;
    ns.nvalid = nv;
    ns.cur = next_half();
    ns.valid = 1;
    *d.state = ns;
  }

  WS_STAMP(7);
  // order statistic j of the new window: the one-row path left the whole window in
  // LDS (written before the reduction barrier above), the other paths picked wv[]
  auto order_stat = [&](int j) -> float { return onerow ? lds[idx[j]] : wv[j]; };
  if (t < STAT_NUM) {
    float r = __builtin_nanf("");
    if (t == STAT_COUNT) {
      r = float(nv);
    } else if (t == STAT_LAST) {
      // newest raw sample: captured by this launch unless no row entered the window
      if (h1) r = (inc && kadd == 0) ? d.base[((h1 - 1) & d.mask) * d.stride + d.col] : lastv;
    } else if (nv) {
      if (t == STAT_MIN) {
        r = order_stat(0);
      } else if (t == STAT_MAX) {
        r = order_stat(1);
      } else if (t == STAT_MEAN) {
        r = float(total / double(nv));
      } else {
        const int q = t - STAT_P0;
        const double x0 = order_stat(2 + 2 * q), x1 = order_stat(3 + 2 * q);
        const double f = frac[q];
        r = float(f >= 0.5 ? x1 - (x1 - x0) * (1.0 - f) : x0 + (x1 - x0) * f);
      }
    }
    // system-scope stores: written through to memory whatever the mapping of the
    // target (pinned host memory with the completion flag / tags), never left dirty in L2
    if (args.tagged_out != nullptr) {
      // value and refresh tag in one aligned 8-byte store (lanes 0..7: one 64 B line)
      const uint64_t w = uint64_t(__builtin_bit_cast(uint32_t, r)) | (uint64_t(args.done_seq) << 32);
      __hip_atomic_store(args.tagged_out + size_t(series) * STAT_NUM + t, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    } else {
      __hip_atomic_store(out + size_t(series) * STAT_NUM + t, r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
  // Completion flag: the outputs come from lanes 0..7 of wave 0 and are written
  // through to (host) memory by system-scope stores, so lane 0 waiting for the wave's
  // store acknowledgements orders them before its arrival count - no L2 writeback is needed, unlike a full
  // system-scope fence (which also wrote back the resident windows and cost ~1.4 us
  // of kernel tail). The last workgroup to arrive publishes the launch's sequence
  // number with a posted store behind everyone's acknowledged outputs.
  if (args.done_flag != nullptr && t == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t before = __hip_atomic_fetch_add(args.wg_counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (before == args.wg_expect - 1u) {
      asm volatile("" ::: "memory");
      __hip_atomic_store(args.done_flag, args.done_seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

template <int NT, int E>
hipError_t launch(const StatsArgs& args, float* out, hipStream_t stream) {
  uint32_t max_cols = 0;
  for (uint32_t r = 0; r < args.num_rings; ++r) max_cols = args.rings[r].cols > max_cols ? args.rings[r].cols : max_cols;
  hipLaunchKernelGGL((window_stats_kernel<NT, E>), dim3(max_cols, args.num_rings), dim3(NT), 0, stream, args, out);
  return hipGetLastError();
}

}  // namespace

uint32_t sort_width_for(uint32_t n) {
  uint32_t p = 64;
  while (p < n) p <<= 1;
  return p;
}

static int launch_sized(const StatsArgs& args, uint32_t pad_pow2, float* out, hipStream_t stream, bool incremental,
                        uint32_t max_new_rows);

int launch_window_stats(const StatsArgs& args, uint32_t pad_pow2, float* out, void* stream_ptr, bool incremental,
                        uint32_t max_new_rows) {
  if (args.num_series == 0) return hipSuccess;
  if (args.num_series > uint32_t(kMaxSeriesPerLaunch)) return hipErrorInvalidValue;
  if (args.num_rings == 0 || args.num_rings > uint32_t(kMaxRingsPerLaunch)) return hipErrorInvalidValue;
  for (uint32_t i = 0; i < args.num_rings; ++i) {  // host-side shape checks before any launch
    const RingDesc& r = args.rings[i];
    if (r.n > pad_pow2 || r.n > r.mask + 1 || r.n > r.head || ((r.mask + 1) & r.mask) || r.stride == 0) return hipErrorInvalidValue;
    if (r.sorted != nullptr && (r.state == nullptr || r.sorted_cap < r.n || r.sorted_cap > pad_pow2)) return hipErrorInvalidValue;
    if (r.n_inline > uint32_t(kInlineRows) || r.n_inline > r.head) return hipErrorInvalidValue;
    if (r.n_inline && r.stride > uint32_t(kMaxInlineWidth)) return hipErrorInvalidValue;
    if (r.host_rows != nullptr && ((r.host_mask + 1) & r.host_mask)) return hipErrorInvalidValue;
  }
  uint32_t cols = 0;
  for (uint32_t i = 0; i < args.num_rings; ++i) {
    if (args.rings[i].cols > args.rings[i].stride) return hipErrorInvalidValue;
    cols += args.rings[i].cols;
  }
  if (cols != args.num_series) return hipErrorInvalidValue;  // series = the rings' columns, in ring order
  auto stream = static_cast<hipStream_t>(stream_ptr);
  StatsArgs a = args;
  for (int q = 0; q < 3; ++q) a.qfrac[q] = double(a.pct[q]) / 100.0;
  for (uint32_t i = 0, first = 0; i < a.num_rings; first += a.rings[i].cols, ++i) a.rings[i].first = first;
  return launch_sized(a, pad_pow2, out, stream, incremental, max_new_rows);
}

static int launch_sized(const StatsArgs& args, uint32_t pad_pow2, float* out, hipStream_t stream, bool incremental,
                        uint32_t max_new_rows) {
  if (incremental && pad_pow2 > 256 && pad_pow2 <= 8192) {
    // Steady state: every series is expected to take the incremental path. With at
    // most one row in (the one-row path) 512 threads - two waves per SIMD overlap
    // each other's dependent instructions - measured fastest; the general merge of
    // k > 1 rows gains from 1024 (HIP events, W = 4096 x 15: k = 1 8.5 vs 9.1 us at
    // 512 vs 1024 threads, k = 10 15.4 vs 14.0 us; profiles/r02/onerow/). (A series
    // whose state turns out invalid still sorts correctly, with E = P / NT.)
    // (free-running sampling brings 2 rows of the faster source into many refreshes:
    // the series with one row keep the one-row path, those with two take the general
    // path at 512 threads - ROCMDASH_SMALL_K_ROWS moves the threshold for A/B runs)
    static const uint32_t small_k = [] {
      const char* e = std::getenv("ROCMDASH_SMALL_K_ROWS");
      return e ? uint32_t(std::strtoul(e, nullptr, 10)) : 2u;
    }();
    const bool one_row = max_new_rows <= small_k;
    switch (pad_pow2) {
      case 512: return launch<256, 2>(args, out, stream);
      case 1024: return launch<256, 4>(args, out, stream);
      case 2048: return launch<512, 4>(args, out, stream);
      case 4096: return one_row ? launch<512, 8>(args, out, stream) : launch<1024, 4>(args, out, stream);
      case 8192: return one_row ? launch<512, 16>(args, out, stream) : launch<1024, 8>(args, out, stream);
      default: break;
    }
  }
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
