// Long-window statistics (see long_window.h): multi-workgroup radix select over
// HBM-resident windows of up to 2^26 samples per series, captured in a hipGraph.
#include "long_window.h"
#include "tagged.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>

#include "rccl_comm.h"
#include "window_stats.h"

namespace rocmdash {
namespace {

void check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

struct Guard {
  int prev = -1;
  explicit Guard(int dev) {
    (void)hipGetDevice(&prev);
    if (prev != dev) check(hipSetDevice(dev), "hipSetDevice");
  }
  ~Guard() {
    int cur = -1;
    (void)hipGetDevice(&cur);
    if (prev >= 0 && cur != prev) (void)hipSetDevice(prev);
  }
};

}  // namespace

// The passes' argument block and what it points at (outside the anonymous namespace: the
// class builds it, long_window.h forward-declares it).
constexpr int NT = 256;
constexpr int kSlots = 16;  // pinned parameter staging slots
constexpr int kD0 = 10;                 // pass 0 digit: at most 10 key bits, 1024 bins
constexpr uint32_t kB0 = 1u << kD0;
constexpr uint32_t kPredMaxNew = NT;    // new rows pass 0 reads for its prediction (one per thread)

struct LwParams {
  uint64_t head[kLongMaxRings];
  uint64_t prev_head[kLongMaxRings];  // the head at this set's previous refresh (0: none)
  uint32_t n[kLongMaxRings];
  float pct[3];
  uint32_t seq;  // this refresh's number: the host-mapped report word carries it
};

struct LwPartial {  // one (series, chunk): identity = {0, 0, ~0u, 0, 0, 0}
  double sum;
  uint32_t cnt, minkey, maxkey, orx;  // orx: OR of (key ^ ref) - the bits that vary
  // the key orx is relative to: a window member while cnt > 0 (the newest sample when the
  // chunk was streamed: a chunk is streamed again before W rows entered). Partials of
  // different refreshes combine exactly in the lowest varying bit: orx_a | orx_b | (ref_a
  // ^ ref_b) (lw_combine) - the only bit of orx anything reads
  uint32_t ref, pad;
};

// a += b (partials of disjoint sample sets), sums added in the caller's fixed order
__device__ __forceinline__ void lw_combine(double& sm, uint32_t& cn, uint32_t& lo, uint32_t& hi, uint32_t& ox,
                                           uint32_t& rf, double bs, uint32_t bc, uint32_t bl, uint32_t bh, uint32_t bo,
                                           uint32_t br) {
  sm += bs;
  if (bc) {
    if (cn) {
      ox |= bo | (br ^ rf);
    } else {
      ox = bo;
      rf = br;
    }
    cn += bc;
    lo = min(lo, bl);
    hi = max(hi, bh);
  }
}

// Node mode (refresh_node): one series' predicted key range on one rank, all-gathered so
// that every rank histograms the SAME digit in pass 0.
struct LwPred {
  uint32_t pmin, pmax;  // predicted key range (0 / ~0: no prediction)
  uint32_t lo;          // lowest key bit predicted to vary
  uint32_t ref;         // key of the ring's newest sample (a window member when has)
  uint32_t has;         // the ring holds samples
  uint32_t pad[3];
};

struct LwSel {  // one series, carried from scan to scan (min / max also to the next refresh)
  uint32_t nv, minkey, maxkey;
  uint32_t done;   // bracket mode: scan B resolved the series this refresh (the radix chain skips it)
  double sum;
  uint32_t shift;  // prefix bits >= shift are found
  uint32_t width;  // the next digit: key bits [shift - width, shift); 0 = resolved
  uint32_t lo;     // lowest bit that varies over the window (32: none)
  uint32_t pad2;
  uint32_t resid[kLongRanks];   // rank inside the bucket the prefix names
  uint32_t prefix[kLongRanks];  // key bits found so far (high bits first)
};

// Bracket mode (lw_pass_brk, lw_scan_brk). A window changes by the few rows that
// entered and left since the previous refresh, so each percentile moves by at most a few
// ranks: the previous refresh's percentile keys, widened by an adaptive half-width, bracket
// the new ones. One streaming pass counts, per percentile q, the samples below the
// bracket (lt), ON its bounds (counted, never kept) and strictly inside it (kept); if both
// sorted positions of every percentile fall inside their brackets (lt <= pos < lt + in),
// the percentiles are the lower bound, the upper bound or order statistics of the kept
// keys - a select over ~kBrkTarget keys in LDS instead of 2-3 more streams of the window.
// Otherwise (the first refresh, a jump in the data, a bracket that overflowed) the series
// takes the exact radix chain in the same refresh. The half-width adapts so that a bracket
// holds ~kBrkTarget samples; a bracket on tied values (integer telemetry, a percentile
// between two readings) is exactly those keys and stores nothing - its ties are counts.
// Known limit: each (chunk, bracket) keeps at most qcap keys, so a series whose bracket
// samples are consecutive rows (a monotone ramp) overflows one chunk's slab and takes the
// radix chain every refresh (exact, at the chain's cost); the service's series are gauges
// and rates, not ramps.
constexpr int kPassBrk = 4;
constexpr int kBrkQ = 3;                  // one bracket per percentile (its lo and hi position)
constexpr uint32_t kBrkTarget = 2048;     // samples a bracket aims to hold
constexpr uint32_t kBrkCap = 8192;        // kept keys scan B selects among (LDS)
constexpr uint32_t kSelBits = 8;          // scan B's LDS radix digit (one bin per thread: no bank conflicts, one-word scans)
struct LwBrk {  // one series (persists across refreshes)
  uint32_t lo[kBrkQ], hi[kBrkQ];  // key bounds, inclusive (lo <= hi)
  uint32_t delta[kBrkQ];          // half-width in VALUE units (float bits; 0: an exact-key bracket)
  uint32_t cin[kBrkQ];            // samples inside at the last refresh that used it
  uint32_t valid;                 // the bounds apply to the next refresh
  uint32_t hit;                   // the last refresh was resolved by the brackets
  uint32_t refreshes, hits;       // counters (diagnostics)
  uint32_t nounion[kBrkQ];        // the last miss overflowed: the next exact bracket is only the new keys
  uint32_t dsave[kBrkQ];          // the value half-width an overflow put aside (float bits; 0: none)
};
struct LwBrkPart {  // one (series, chunk) of pass B
  uint32_t lt[kBrkQ];   // samples below the bracket
  uint32_t mid[kBrkQ];  // samples strictly inside (lo < k < hi): the kept keys of the slab
  uint32_t eq[kBrkQ];   // samples ON the bounds: count(k == lo) | count(k == hi, hi != lo) << 16
};                      // (a chunk holds < 2^16 rows); they are counted, never kept
__device__ inline uint32_t eq_lo(uint32_t e) { return e & 0xFFFFu; }
__device__ inline uint32_t eq_hi(uint32_t e) { return e >> 16; }

// Node bracket mode (refresh_node): the node's brackets aim at fewer samples (the union of
// the ranks' kept keys crosses the node), and every rank contributes at most `cap` keys per
// bracket (<= kNodeCap); more (or a chunk slab that overflowed) is a miss and the node
// radix chain resolves the series. kNodeBrkRanks: the most ranks whose union fits scan B's
// LDS.
constexpr uint32_t kNodeBrkTarget = 256;  // 2x it (a sized bracket's most) fits one rank's kNodeCap twice over
constexpr uint32_t kNodeCap = 1024;
constexpr uint32_t kNodeBrkRanks = 8;
struct LwNodeHdr {  // one rank, one series (all-gathered over the node)
  LwPartial p;                      // the rank's partials over its chunks
  uint32_t lt[kBrkQ], mid[kBrkQ];   // below / strictly inside each node bracket
  uint32_t elo[kBrkQ], ehi[kBrkQ];  // on its lower / upper bound (counted, not kept)
  uint32_t ovf;                     // bracket bits whose kept keys did not all fit
  uint32_t ent;                     // rows that entered the rank's window since its last refresh (~0: unknown)
  uint32_t pad[2];
};
static_assert(sizeof(LwNodeHdr) % sizeof(LwPartial) == 0, "records stride in partials");
// One rank's all-gathered block: the S headers, then the kept keys [S][kBrkQ][cap] (chunk
// order). `cap` is the refresh's record cap, the same on every rank (LongWindowSet::
// node_cap_: sized from the previous refresh's node-wide most kept keys), so the one
// collective carries ~2x the keys the node's brackets keep, not kNodeCap per bracket: at
// 8 ranks 12 series move 20 KB per rank instead of 150 KB.
__host__ __device__ constexpr size_t lw_node_block(uint32_t S, uint32_t cap) {
  return size_t(S) * (sizeof(LwNodeHdr) + kBrkQ * sizeof(uint32_t) * size_t(cap));
}
// the next refresh's record cap from this one's most kept keys of any (rank, series,
// bracket) that a cap could hold (<= kNodeCap; a bracket over it re-sizes): 2x headroom, a floor of 4x a rank's share of the node target, 64-key steps
// (keeps every block a multiple of the partials' 32 B), at most kNodeCap
inline uint32_t lw_node_cap_next(uint32_t maxmid, uint32_t nranks) {
  uint32_t c = 2 * maxmid;
  const uint32_t floor = 4 * kNodeBrkTarget / (nranks ? nranks : 1);
  if (c < floor) c = floor;
  c = (c + 63) / 64 * 64;
  return c < kNodeCap ? c : kNodeCap;
}

// pass B keeps at most this many keys per (chunk, bracket): a bracket holds ~kBrkTarget of
// the window's samples, so a chunk is rarely near it; a fuller chunk makes scan B miss
// (the radix chain resolves the series, exact) and the bracket narrows. 3 / 64 of the
// window per series of HBM (the slabs were 3 / 4 of it, plus compaction's)
__host__ __device__ constexpr uint32_t lw_qcap(uint32_t chunk_rows) {
  return chunk_rows / 64 > 64 ? chunk_rows / 64 : 64;
}

struct LwRing {
  const float* dev;
  uint32_t width, first_series;
  uint32_t chunk_rows;  // rows one pass workgroup streams (per ring: balanced by row bytes)
  uint32_t nchunks;     // workgroups per segment of the ring
  uint32_t qcap;        // pass B: kept keys per (chunk, bracket) slab (lw_qcap)
  uint32_t pad;
  uint64_t boff;        // pass B slabs: the ring's first series' keys in LwArgs::bcand
  uint64_t bstride;     // keys per series: nchunks x kBrkQ x qcap
};

// A pass workgroup streams the rows of one ring segment: <= 8 of its series (a 16-wide
// ring is two segments), so no code path holds more than 8 series' state in registers.
// The pass grid is flat: segment g owns workgroups [wg0, wg0 + its ring's nchunks).
constexpr uint32_t kSegCols = 8;
struct LwSeg {
  uint32_t ring, col0, ncols, wg0;
};

struct LwArgs {
  LwRing rings[kLongMaxRings];
  LwSeg segs[2 * kLongMaxRings];
  uint32_t num_rings, num_segs, num_series, mask, max_chunks;  // max_chunks: over the rings
  const LwParams* params;
  LwPartial* part;  // [S][max_chunks]; slots past a ring's nchunks hold the identity
  uint32_t* hist0;  // [S][kB0]
  uint32_t* histk;  // [S][6][256]
  LwSel* sel;       // [S]
  uint32_t* dig0;   // [S][3]: pass 0's digit shift, the reference key of its orx, digit width
  float* out;       // [S][8]
  // node mode (0 = this rank's window only): ranks whose windows form the node window
  uint32_t node_n;
  LwPred* pred_local;       // [S] this rank's prediction
  const LwPred* pred_all;   // [node_n][S] every rank's (all-gathered)
  LwPartial* agg_local;     // [S] this rank's partials reduced over its chunks
  const LwPartial* agg_all; // [node_n][S] every rank's (all-gathered)
  uint32_t wave_priv;       // pass 0: per-wave LDS histogram copies for 8-bit digits
  // bracket mode (0: off - node refreshes, or disabled): pass B + scan B run first, and
  // the radix chain skips the series scan B resolved (LwSel::done)
  uint32_t brk_on;
  LwBrk* brk;               // [S] the next refresh's brackets
  LwBrk* brk_used;          // [S] the brackets this refresh's pass B used (its copy)
  uint32_t* hflags;         // [S] host-mapped: a series wants brackets (a launch hint; may be null)
  LwBrkPart* bpart;         // [S][max_chunks]
  uint32_t* bcand;          // pass B's kept keys (LwRing::boff / bstride / qcap)
  // incremental bracket mode (incr): a bracket stays put while the percentiles sit well
  // inside it, so the chunks' counts stay valid and pass B streams only the chunks new
  // rows landed in (its grid: the work list, seg << 20 | chunk; nwork = 0: every chunk).
  // colsplit: the list is seg << 23 | column << 20 | chunk - one workgroup per (chunk,
  // series): a short list's few chunks then spread over 8x the CUs (a lone workgroup
  // streaming a whole chunk of 8 series is latency-bound), with the same sums
  uint32_t incr;
  const uint32_t* work;
  uint32_t nwork;
  uint32_t colsplit;
  uint32_t* bchg;           // [S] host-mapped: the series' brackets changed (its chunks' counts are stale)
  const uint32_t* fwork;    // lw_scan_brk_fused: the chunks scan B streams itself (seg << 20 | chunk)
  uint32_t nfused;
  unsigned long long* report;  // host-mapped: seq (24 bits) | series the chain must resolve (24) | node select's most
                               // kept keys of one rank's bracket (16) - lw_brk_finish: one 8-byte system-scope store
  uint32_t node_brk;        // the brackets are the node's (refresh_node): their target is kNodeBrkTarget
  unsigned char* nbl;       // this rank's node-bracket block (lw_node_block(S, node_cap) bytes)
  unsigned long long* dbg;  // diagnostics (null: off): scan B's phase clocks [S][kBrkQ][8]
  uint32_t* brk_cnt;        // device [2]: scan B's finished workgroups (the last one writes the report);
                            // node select's most kept keys of one rank's bracket (the report's top 16 bits)
  uint32_t brk_target;      // samples a local bracket aims to hold (LongWindowSet::brk_target, <= kBrkTarget)
  const unsigned char* nball;  // [node_n] every rank's block (all-gathered)
  uint32_t node_cap;        // the records' key cap (a multiple of 64, <= kNodeCap)

  // candidate compaction (compact = 0: off): pass 2 keeps the keys of the samples it counts
  // (those whose found bits match a rank's prefix) and pass 3 histograms those instead of
  // streaming the window again. Workgroup c of pass 2 owns the slab
  // cand[s][c * chunk_rows ..) of each of its series (its chunk has that many rows, so the
  // slab never overflows) and counts into it with LDS atomics: no device atomics.
  uint32_t compact;
  uint32_t* cand;           // [S][cand_cap]: compaction's and pass B's slabs
  uint32_t* cand_n;         // [S][max_chunks] keys in each slab
  uint32_t cand_cap;        // >= nchunks x chunk_rows of every ring (>= W)
};

namespace {

// order-preserving float <-> uint32 key (NaN never keyed: callers skip it)
__device__ __forceinline__ uint32_t fkey(float x) {
  const uint32_t u = __float_as_uint(x);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float kfloat(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k);
}

// sorted positions [lo0, hi0, lo1, hi1, lo2, hi2] and interpolation weights of the
// three percentiles over nv valid samples (numpy 'linear', as window_stats.hip)
__device__ inline void lw_positions(uint32_t nv, const float pct[3], uint32_t (&pos)[kLongRanks], double (&frac)[3]) {
  const uint32_t last = nv ? nv - 1 : 0;
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const double p = double(pct[q]) / 100.0 * double(last);
    uint32_t lo = uint32_t(floor(p));
    if (lo > last) lo = last;
    pos[2 * q] = lo;
    pos[2 * q + 1] = lo + 1 < nv ? lo + 1 : last;
    frac[q] = double(float(p - double(lo)));  // float weight, as the LDS kernel
  }
}

__device__ inline void series_ring(const LwArgs& a, uint32_t s, uint32_t& r, uint32_t& col) {
  r = 0;
  for (uint32_t i = 0; i < a.num_rings; ++i)
    if (s >= a.rings[i].first_series) r = i;
  col = s - a.rings[r].first_series;
}

// width of the digit below `shift` when bits below `lo` never vary: <= 8 bits, 0 = done
__device__ __forceinline__ uint32_t next_width(uint32_t shift, uint32_t lo) {
  return shift > lo ? min(8u, shift - lo) : 0u;
}

// ---- pass k: stream one chunk of one ring, histogram one digit ------------------------
// Adaptive digits. Only the key bits that vary over the window need resolving: bits
// above the highest differing bit of (min, max) and below the lowest bit any key
// differs in from a window member are shared by every sample. Pass 0 cannot know the
// exact range before it has read the window, so it predicts it from the previous
// refresh's exact min / max and the <= 256 rows that entered since (the window is a
// subset of the previous window and those rows, so the prediction is a superset of the
// varying bits: never wrong, at worst wider) and histograms the 10 (or 8, when 10 would
// not save a pass) bits just below the predicted top varying bit; without a prediction
// (first refresh, or more new rows than one workgroup reads) it takes the top key byte,
// as a fixed-digit radix select would. Passes 1..3 take 8-bit digits
// below it, down to the exact lowest varying bit; a series whose bits are all found
// skips the remaining passes, and a ring whose series all did exits at once. Integer
// telemetry in a band (temperatures, W, %) varies in <= 10 bits: one streaming pass
// instead of four; continuous data spans ~25 bits: three.
//
// LDS histograms hold two 16-bit bins per word (a chunk has <= 4096 rows, so a bin
// never overflows into its neighbour), sized at launch for the widest ring: pass 0
// [width][kB0 / 2] words (32 KB for 16 series), passes k [width][6 ranks][128] words.
//
// The stream is latency-bound, not bandwidth-bound, at the few waves per CU a window's
// chunks give: each thread therefore issues the loads of U rows (U x WM floats in
// registers, WM = the ring width rounded up to 4 / 8 / 16, chosen per ring by a uniform
// branch) before it histograms any of them. Ranks whose prefixes agree (the lo / hi
// positions of one percentile usually do) share one histogram: only the first rank
// of each prefix counts (cmask), the scan reads that rank's histogram for the others.
//
// Pass 0 adds a wave's count with one atomic for the lanes that share the first lane's
// bin, one atomic per sample for the others. Measured and rejected: the general form
// (a ballot per distinct bin, up to 3 rounds, in every pass) cost more VALU than the
// conflicts it removed - 2.6x slower overall at W = 2^20
// (profiles/r01/long_window_profile.json).
struct LwShared {
  const uint32_t* pre;    // [width][kLongRanks] prefixes of the ranks (passes > 0)
  const uint32_t* shift;  // [width] pass 0: digit shift; passes > 0: found-bits shift
  const uint32_t* width;  // [width] passes > 0: digit width (0 = resolved)
  const uint32_t* ref;    // [width] pass 0: the reference key of orx
  double (*rsum)[kSegCols];
  uint32_t (*rcnt)[kSegCols];
  uint32_t (*rmin)[kSegCols];
  uint32_t (*rmax)[kSegCols];
  uint32_t (*ror)[kSegCols];
  uint32_t* ccount;  // pass 2 compaction: candidates of each series in this chunk (LDS)
  uint32_t colmask;  // pass 0 / B: the segment's series this pass works on (bit per column)
  uint32_t* bcnt;    // pass B: samples strictly inside each (column, bracket) in this chunk (LDS)
  uint32_t* beq;     // pass B: samples on each (column, bracket)'s bounds, packed as LwBrkPart::eq (LDS)
  uint32_t (*rlt)[kSegCols * kBrkQ];  // pass B: per-wave below-bracket counts
};

struct LwView {  // one segment of one ring
  const float* dev;  // the ring's window + the segment's first column
  uint32_t stride;   // floats per row (the ring's width)
  uint32_t chunk_rows;  // the ring's rows per workgroup
  uint32_t nc;       // series in the segment (<= kSegCols)
  bool vec;          // 16-byte aligned float4 loads
  uint32_t sb;       // the segment's first series
  uint32_t* bkeys;   // pass B: the segment's first series' kept-key slabs
  uint64_t bstride;  // keys per series
  uint32_t qcap;     // keys per (chunk, bracket)
  const LwBrk* brk;  // pass B: the brackets it counts against (brk; the fused pass: brk_used)
  uint32_t qkeys;    // pass B: brackets whose kept keys it stores (bit per bracket)
  // the fused pass B (one column): orx's reference read here, after the rows' loads are in
  // flight (one memory latency for both), instead of from LDS (sh_.ref); its key -> *ref_out
  const float* newest;  // the column's newest sample (nullptr: none / not fused)
  bool fused_ref;
  uint32_t* ref_out;    // LDS
};

// PF: the thread's next U rows are loaded before this iteration's samples are counted
// (two register buffers), so the loads are in flight while the wave computes. A compile-
// time choice: a runtime switch would make every pass kernel carry the registers of both.
template <int PASS, int WM, int U, bool PF, int UG = (WM <= 4 ? 8 : 4)>
__device__ __forceinline__ void pass_chunk(const LwArgs& a, const LwView& V, uint32_t r, uint32_t c, uint32_t* h,
                                           uint32_t hw, const LwShared& sh_) {
  const uint32_t w = V.nc;  // <= WM
  // Chunks are PHYSICAL: chunk c is the device ring's slots [c x chunk_rows, ..) - rows that
  // entered the window overwrite the slots of rows that left, so a refresh changes only
  // the chunks its new rows landed in and every other chunk's partials / bracket counts
  // stay valid (incremental pass B). The window is the set of its slots: slots a filling
  // window has not reached yet hold NaN (never counted), like failed reads.
  const uint32_t wslots = a.mask + 1u;
  const uint32_t row0 = c * V.chunk_rows;
  const int t = threadIdx.x;
  const int lane = t & 63, wave = t >> 6;
  const uint32_t rows = row0 < wslots ? min(wslots - row0, V.chunk_rows) : 0u;
  (void)r;

  double sum[WM];
  uint32_t cnt[WM], mn[WM], mx[WM], orx[WM];
  uint32_t dsh[WM], dwd[WM], fsh[WM], ref[WM];  // workgroup-uniform: scalar registers
  uint32_t pre[WM][kLongRanks];  // passes > 0: the rank's found bits (prefix >> fsh)
  uint32_t cmask[WM];  // ranks that own a histogram (first of each distinct prefix)
  // pass B: per lane, the samples below each bracket; narrow variants (<= 4 columns) also
  // count the samples on its bounds here (lo | hi << 16), wide ones with LDS atomics
  constexpr bool EQREG = WM <= 4;
  uint32_t lt[WM][kBrkQ];
  uint32_t eqr[EQREG ? WM : 1][kBrkQ];
  const uint32_t colmask = sh_.colmask;
  const uint32_t qcap = V.qcap;  // pass B: kept keys per (chunk, bracket) slab
#pragma unroll
  for (int col = 0; col < WM; ++col) {
    sum[col] = 0.0;
    cnt[col] = 0;
    mn[col] = 0xFFFFFFFFu;
    mx[col] = 0;
    orx[col] = 0;
    cmask[col] = 0;
    dsh[col] = fsh[col] = ref[col] = dwd[col] = 0;
#pragma unroll
    for (int q = 0; q < kBrkQ; ++q) {
      lt[col][q] = 0;
      if constexpr (EQREG) eqr[col][q] = 0;
    }
    if (uint32_t(col) < w) {
      if constexpr (PASS == kPassBrk) {
        if (!V.fused_ref) ref[col] = __builtin_amdgcn_readfirstlane(sh_.ref[col]);  // bounds: per column in the loop
      } else if constexpr (PASS == 0) {
        dsh[col] = __builtin_amdgcn_readfirstlane(sh_.shift[col]);
        ref[col] = __builtin_amdgcn_readfirstlane(sh_.ref[col]);
        dwd[col] = __builtin_amdgcn_readfirstlane(sh_.width[col]);
      } else {
        const uint32_t wd = __builtin_amdgcn_readfirstlane(sh_.width[col]);
        fsh[col] = __builtin_amdgcn_readfirstlane(sh_.shift[col]);
        dsh[col] = fsh[col] - wd;
        dwd[col] = wd;
        if (wd) {
#pragma unroll
          for (int q = 0; q < kLongRanks; ++q) {
            pre[col][q] = sh_.pre[col * kLongRanks + q] >> fsh[col];
            bool first = true;
#pragma unroll
            for (int q2 = 0; q2 < q; ++q2) first = first && pre[col][q2] != pre[col][q];
            if (first) cmask[col] |= 1u << q;
          }
        }
      }
    }
  }
  const bool vec = V.vec;
  // the U rows of a thread's next iteration are loaded before this iteration's samples
  // are counted (a.prefetch): the loads are in flight while the wave computes, instead of
  // the wave's memory pipe idling through every counting phase
  const auto load_rows = [&](float (&dst)[U][WM], uint32_t i0) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t i = i0 + uint32_t(u) * NT;
      const float* p = V.dev + size_t(row0 + i) * V.stride;
      if (i < rows && vec) {
#pragma unroll
        for (int q4 = 0; q4 < WM / 4; ++q4) {
          if (uint32_t(4 * q4) < w) {
            const float4 f = reinterpret_cast<const float4*>(p)[q4];
            dst[u][4 * q4] = f.x;
            dst[u][4 * q4 + 1] = f.y;
            dst[u][4 * q4 + 2] = f.z;
            dst[u][4 * q4 + 3] = f.w;
          }
        }
      } else {
#pragma unroll
        for (int col = 0; col < WM; ++col) dst[u][col] = (i < rows && uint32_t(col) < w) ? p[col] : __builtin_nanf("");
      }
    }
  };
  constexpr bool pf = PF;
  float v[U][WM], vn[U][WM];
  // pass 0 / B: a thread's values of a series are summed in fp32 over groups of UG rows
  // (its rows i0 + u x NT in order), then added to the fp64 total once per group (a
  // quarter of the fp64 adds; <= UG terms per fp32 partial). UG is fixed by the segment
  // width, not by U, so every pass variant sums the same groups: the same mean bits
  // (a column-split pass B - WM 1 - takes its segment's UG: the same groups, the same sums).
  // U > UG (the column-split pass B: many rows in flight per thread) flushes every UG rows
  // inside the iteration - the same groups
  static_assert(UG % U == 0 || (U % UG == 0 && WM == 1 && PASS == kPassBrk), "rows per sum group");
  constexpr bool INNER_FLUSH = U > UG;
  float psum[WM];
#pragma unroll
  for (int col = 0; col < WM; ++col) psum[col] = 0.f;
  int git = 0;  // iterations into the current group
  const auto flush = [&]() {
#pragma unroll
    for (int col = 0; col < WM; ++col) {
      sum[col] += double(psum[col]);
      psum[col] = 0.f;
    }
  };
  if (uint32_t(t) < rows) load_rows(v, uint32_t(t));
  if constexpr (PASS == kPassBrk) {
    if (V.fused_ref) {  // one column (WM 1): its newest sample's key, loaded behind the rows
      const float xn = V.newest ? *V.newest : __builtin_nanf("");
      ref[0] = isnan(xn) ? 0u : fkey(xn);
      if (t == 0) *V.ref_out = ref[0];
    }
  }
  for (uint32_t i0 = uint32_t(t); i0 < rows; i0 += NT * U) {
    const uint32_t inext = i0 + NT * U;
    if constexpr (pf) {
      if (inext < rows) load_rows(vn, inext);
    }
    if constexpr (PASS == kPassBrk) {
      // pass B, column by column: the column's bounds once per iteration, then its U
      // samples
#pragma unroll
      for (int col = 0; col < WM; ++col) {
        if (uint32_t(col) < w && ((colmask >> col) & 1u)) {  // uniform
          // this refresh's brackets of the column: read through the constant address space
          // (scalar loads - nothing writes brk while pass B runs), here in the loop, not
          // hoisted: 8 columns' bounds held across the loop spill
          asm volatile("" ::: "memory");
          typedef const __attribute__((address_space(4))) uint32_t* cptr;
          const cptr cb = (cptr)(V.brk + V.sb + col);  // LwBrk: lo[3], hi[3], ...
          const uint32_t l0 = cb[0], l1 = cb[1], l2 = cb[2], h0 = cb[3], h1 = cb[4], h2 = cb[5];
#pragma unroll
          for (int u = 0; u < U; ++u) {
            if constexpr (INNER_FLUSH) {
              if (u && u % UG == 0) {  // a group of UG rows done (uniform: u is unrolled)
                sum[col] += double(psum[col]);
                psum[col] = 0.f;
              }
            }
            const float x = v[u][col];
            if (isnan(x)) continue;  // failed reads, rows past the chunk
            const uint32_t k = fkey(x);
            psum[col] += x;
            ++cnt[col];
            mn[col] = min(mn[col], k);
            mx[col] = max(mx[col], k);
            orx[col] |= k ^ ref[col];
            const bool b0 = k < l0, b1 = k < l1, b2 = k < l2;
            lt[col][0] += b0 ? 1u : 0u;
            lt[col][1] += b1 ? 1u : 0u;
            lt[col][2] += b2 ? 1u : 0u;
            // inside a bracket: rare for continuous data (a bracket holds ~kBrkTarget of
            // the window's samples). On a bound - counted, not kept: a bracket whose bounds
            // are tied values (a percentile of telemetry readings) then holds the rank with
            // no keys at all, however many samples tie. Strictly inside: per bracket, the
            // wave's count goes to the chunk's LDS counter and its keys to the slab
            const bool i0 = !b0 && k <= h0, i1 = !b1 && k <= h1, i2 = !b2 && k <= h2;
            const bool e0 = i0 && (k == l0 || k == h0), e1 = i1 && (k == l1 || k == h1),
                       e2 = i2 && (k == l2 || k == h2);
            if constexpr (EQREG) {  // per-lane counters: no ballots for ties
              eqr[col][0] += e0 ? (k == l0 ? 1u : 0x10000u) : 0u;
              eqr[col][1] += e1 ? (k == l1 ? 1u : 0x10000u) : 0u;
              eqr[col][2] += e2 ? (k == l2 ? 1u : 0x10000u) : 0u;
            } else if (__ballot(e0 || e1 || e2)) {
#pragma unroll
              for (int q = 0; q < kBrkQ; ++q) {
                const uint32_t lo = q == 0 ? l0 : (q == 1 ? l1 : l2);
                const bool onb = q == 0 ? e0 : (q == 1 ? e1 : e2);
                const uint64_t me = __ballot(onb);
                if (me) {
                  const uint32_t nlo = uint32_t(__popcll(__ballot(onb && k == lo)));
                  if (lane == __builtin_ctzll(me))
                    atomicAdd(&sh_.beq[col * kBrkQ + q], nlo | ((uint32_t(__popcll(me)) - nlo) << 16));  // LDS
                }
              }
            }
            const bool m0 = i0 && !e0, m1 = i1 && !e1, m2 = i2 && !e2;
            if (__ballot(m0 || m1 || m2)) {
#pragma unroll
              for (int q = 0; q < kBrkQ; ++q) {
                const bool mid = q == 0 ? m0 : (q == 1 ? m1 : m2);
                const uint64_t mb = __ballot(mid);
                if (mb) {
                  const int leader = __builtin_ctzll(mb);
                  uint32_t base = 0;
                  if (lane == leader) base = atomicAdd(&sh_.bcnt[col * kBrkQ + q], uint32_t(__popcll(mb)));  // LDS
                  base = uint32_t(__builtin_amdgcn_readlane(int(base), leader));
                  if (mid) {
                    const uint32_t slot =
                        base + __builtin_amdgcn_mbcnt_hi(uint32_t(mb >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(mb), 0u));
                    if (slot < qcap && ((V.qkeys >> q) & 1u))  // a fuller slab: scan B sees mid > qcap, the chain
                      V.bkeys[size_t(col) * V.bstride + (size_t(c) * kBrkQ + q) * qcap + slot] = k;
                  }
                }
              }
            }
          }
        }
      }
    } else {
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int col = 0; col < WM; ++col) {
        if (uint32_t(col) < w && ((colmask >> col) & 1u)) {  // uniform: w is the segment's
          const float x = v[u][col];
          if (isnan(x)) continue;  // failed reads, rows past the chunk
          const uint32_t k = fkey(x);
          const uint32_t bin = __builtin_amdgcn_ubfe(k, dsh[col], dwd[col]);  // one v_bfe_u32
          if constexpr (PASS == 0) {
            psum[col] += x;
            ++cnt[col];
            mn[col] = min(mn[col], k);
            mx[col] = max(mx[col], k);
            orx[col] |= k ^ ref[col];
            // the first lane's bin is added as one count for every lane that shares it,
            // only lanes with another bin add one each
            const uint64_t act = __ballot(1);  // the lanes here: valid samples
            const int first = __builtin_ctzll(act);
            const uint32_t lb = uint32_t(__builtin_amdgcn_readlane(int(bin), first));
            const uint64_t grp = __ballot(bin == lb);
            if (lane == first) atomicAdd(&h[col * hw + (lb >> 1)], uint32_t(__popcll(grp)) << ((lb & 1u) * 16u));
            if (grp != act && bin != lb) atomicAdd(&h[col * hw + (bin >> 1)], 1u << ((bin & 1u) * 16u));
          } else {
            // a sample counts for a rank when its found bits (>= fsh, < 32) are the rank's
            const uint32_t hk = k >> fsh[col];
            bool hit = false;
#pragma unroll
            for (int q = 0; q < kLongRanks; ++q)
              if ((cmask[col] >> q) & 1u)
                if (hk == pre[col][q]) {
                  atomicAdd(&h[(col * kLongRanks + q) * 128 + (bin >> 1)], 1u << ((bin & 1u) * 16u));
                  hit = true;
                }
            if constexpr (PASS == 2) {
              // compaction: the wave's hits of this series go to its candidate list with
              // one device atomic (the wave's count), each lane at its rank among them
              if (a.compact) {
                const uint64_t mb = __ballot(hit);
                if (mb) {
                  const int leader = __builtin_ctzll(mb);
                  uint32_t base = 0;
                  if (lane == leader) base = atomicAdd(&sh_.ccount[col], uint32_t(__popcll(mb)));  // LDS
                  base = uint32_t(__builtin_amdgcn_readlane(int(base), leader));
                  if (hit) {
                    const uint32_t off =
                        __builtin_amdgcn_mbcnt_hi(uint32_t(mb >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(mb), 0u));
                    a.cand[size_t(V.sb + col) * a.cand_cap + size_t(c) * V.chunk_rows + base + off] = k;
                  }
                }
              }
            }
          }
        }
      }
    }
    }  // passes 0-3
    if constexpr (PASS == 0 || PASS == kPassBrk) {
      if constexpr (INNER_FLUSH) {
        flush();  // the iteration's last group
      } else if (++git == UG / U) {
        git = 0;
        flush();
      }
    }
    if (inext < rows) {
      if constexpr (pf) {
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
          for (int col = 0; col < WM; ++col) v[u][col] = vn[u][col];
      } else {
        load_rows(v, inext);
      }
    }
  }

  if constexpr (PASS == 0 || PASS == kPassBrk) {
    if (git) flush();  // a group the chunk's end cut short (its missing rows were NaN)
    // per-chunk partials: wave butterflies, then the 4 waves in a fixed order
#pragma unroll
    for (int col = 0; col < WM; ++col) {
      if (uint32_t(col) < w && ((colmask >> col) & 1u)) {
        double s = sum[col];
        uint32_t cn = cnt[col], lo = mn[col], hi = mx[col], ox = orx[col];
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
          s += __shfl_xor(s, off);
          cn += __shfl_xor(cn, off);
          lo = min(lo, uint32_t(__shfl_xor(int(lo), off)));
          hi = max(hi, uint32_t(__shfl_xor(int(hi), off)));
          ox |= uint32_t(__shfl_xor(int(ox), off));
        }
        if (lane == 0) {
          sh_.rsum[wave][col] = s;
          sh_.rcnt[wave][col] = cn;
          sh_.rmin[wave][col] = lo;
          sh_.rmax[wave][col] = hi;
          sh_.ror[wave][col] = ox;
        }
        if constexpr (PASS == kPassBrk) {
#pragma unroll
          for (int q = 0; q < kBrkQ; ++q) {
            uint32_t l = lt[col][q];
#pragma unroll
            for (int off = 32; off >= 1; off >>= 1) l += uint32_t(__shfl_xor(int(l), off));
            if (lane == 0) sh_.rlt[wave][col * kBrkQ + q] = l;
            if constexpr (EQREG) {
              // lo | hi << 16 halves: a chunk holds < 2^16 rows, so neither half carries
              uint32_t e = eqr[col][q];
#pragma unroll
              for (int off = 32; off >= 1; off >>= 1) e += uint32_t(__shfl_xor(int(e), off));
              if (lane == 0) atomicAdd(&sh_.beq[col * kBrkQ + q], e);  // LDS: the 4 waves
            }
          }
        }
      }
    }
  }
}

// Pass 0's prediction of the key bits that vary over ring r's segment (threads t < w
// of the workgroup, one series each; LDS arrays of kSegCols): the previous refresh's
// exact min / max / lowest varying bit and the <= kPredMaxNew rows that entered since
// (0 / ~0 / 0 - no prediction - otherwise), and the newest sample's key as the reference
// of orx. Ends with a barrier.
__device__ inline void lw_predict(const LwArgs& a, uint32_t r, const float* seg, uint32_t stride, uint32_t w,
                                  uint32_t sb, uint32_t* pmin, uint32_t* pmax, uint32_t* plo, uint32_t* plx,
                                  uint32_t* dref) {
  const int t = threadIdx.x;
  const uint64_t head = a.params->head[r], prev = a.params->prev_head[r];
  const uint32_t n = a.params->n[r];
  const bool pred = prev != 0 && head >= prev && head - prev <= kPredMaxNew;
  if (uint32_t(t) < w) {
    const LwSel& sl = a.sel[sb + t];
    pmin[t] = pred ? sl.minkey : 0u;
    pmax[t] = pred ? sl.maxkey : 0xFFFFFFFFu;
    plo[t] = pred ? sl.lo : 0u;  // the previous window's lowest varying bit
    plx[t] = 0;
    // orx's reference: the newest sample (a window member: orx is then exact)
    const float x = n ? seg[((head - 1) & uint64_t(a.mask)) * stride + t] : __builtin_nanf("");
    dref[t] = isnan(x) ? 0u : fkey(x);
  }
  __syncthreads();
  if (pred && uint32_t(t) < uint32_t(head - prev)) {
    const float* p = seg + ((prev + uint32_t(t)) & uint64_t(a.mask)) * stride;
    for (uint32_t col = 0; col < w; ++col) {
      const float x = p[col];
      if (!isnan(x)) {
        const uint32_t k = fkey(x);
        atomicMin(&pmin[col], k);
        atomicMax(&pmax[col], k);
        atomicOr(&plx[col], k ^ a.sel[sb + col].minkey);  // vs a previous member
      }
    }
  }
  __syncthreads();
}

// node mode, before pass 0: this rank's prediction of every series (one workgroup per
// ring segment) -> pred_local, all-gathered by the host between the launches
__global__ __launch_bounds__(NT) void lw_node_predict(const LwArgs a) {
  __shared__ uint32_t pmin[kSegCols], pmax[kSegCols], plo[kSegCols], plx[kSegCols], dref[kSegCols];
  if (blockIdx.x >= a.num_segs) return;  // uniform
  const LwSeg G = a.segs[blockIdx.x];
  const LwRing R = a.rings[G.ring];
  const uint32_t w = G.ncols, sb = R.first_series + G.col0;
  lw_predict(a, G.ring, R.dev + G.col0, R.width, w, sb, pmin, pmax, plo, plx, dref);
  const int t = threadIdx.x;
  if (uint32_t(t) < w) {
    LwPred p{};
    p.pmin = pmin[t];
    p.pmax = pmax[t];
    p.lo = min(plo[t], plx[t] ? uint32_t(__builtin_ctz(plx[t])) : 32u);
    p.ref = dref[t];
    p.has = a.params->n[G.ring] ? 1u : 0u;
    a.pred_local[sb + t] = p;
  }
}

// one series' partials over `count` entries (stride apart) in a fixed order: per thread
// in index order, a wave butterfly (both partners add the same pair: every lane holds the
// same bits), then the 4 waves in order -> every thread (deterministic sum)
// The block's reduction of per-thread combined partials (thread order fixed: butterflies,
// then the waves in order) - every caller's partials reduce to the same bits.
__device__ inline LwPartial block_reduce_partial(double sm, uint32_t cn, uint32_t lo, uint32_t hi, uint32_t ox,
                                                 uint32_t rf, double* dsum, uint32_t* dcnt, uint32_t* dmin,
                                                 uint32_t* dmax, uint32_t* dor, uint32_t* dref);

__device__ inline LwPartial reduce_partials(const LwPartial* P, uint32_t count, uint32_t stride, double* dsum,
                                            uint32_t* dcnt, uint32_t* dmin, uint32_t* dmax, uint32_t* dor,
                                            uint32_t* dref) {
  const int t = threadIdx.x;
  double sm = 0.0;
  uint32_t cn = 0, lo = 0xFFFFFFFFu, hi = 0, ox = 0, rf = 0;
  for (uint32_t i = t; i < count; i += NT) {
    const LwPartial pp = P[size_t(i) * stride];
    lw_combine(sm, cn, lo, hi, ox, rf, pp.sum, pp.cnt, pp.minkey, pp.maxkey, pp.orx, pp.ref);
  }
  return block_reduce_partial(sm, cn, lo, hi, ox, rf, dsum, dcnt, dmin, dmax, dor, dref);
}

__device__ inline LwPartial block_reduce_partial(double sm, uint32_t cn, uint32_t lo, uint32_t hi, uint32_t ox,
                                                 uint32_t rf, double* dsum, uint32_t* dcnt, uint32_t* dmin,
                                                 uint32_t* dmax, uint32_t* dor, uint32_t* dref) {
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  (void)t;
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const double os = __shfl_xor(sm, off);
    const uint32_t oc = uint32_t(__shfl_xor(int(cn), off)), ol = uint32_t(__shfl_xor(int(lo), off)),
                   oh = uint32_t(__shfl_xor(int(hi), off)), oo = uint32_t(__shfl_xor(int(ox), off)),
                   orf = uint32_t(__shfl_xor(int(rf), off));
    lw_combine(sm, cn, lo, hi, ox, rf, os, oc, ol, oh, oo, orf);
  }
  if (lane == 0) {
    dsum[wave] = sm;
    dcnt[wave] = cn;
    dmin[wave] = lo;
    dmax[wave] = hi;
    dor[wave] = ox;
    dref[wave] = rf;
  }
  __syncthreads();
  LwPartial r{0.0, 0, 0xFFFFFFFFu, 0, 0, 0, 0};
  for (int wv = 0; wv < NT / 64; ++wv)
    lw_combine(r.sum, r.cnt, r.minkey, r.maxkey, r.orx, r.ref, dsum[wv], dcnt[wv], dmin[wv], dmax[wv], dor[wv],
               dref[wv]);
  __syncthreads();  // the arrays are reusable
  return r;
}

// node mode, after pass 0: this rank's chunk partials of each series -> agg_local (one
// workgroup per series), all-gathered by the host; scan 0 then reduces the ranks' in rank
// order, so every rank holds the same node-wide count, sum, min, max and varying bits
__global__ __launch_bounds__(NT) void lw_node_partials(const LwArgs a) {
  __shared__ double dsum[NT];
  __shared__ uint32_t dcnt[NT], dmin[NT], dmax[NT], dor[NT], drf[NT];
  const uint32_t s = blockIdx.x;
  const LwPartial p =
      reduce_partials(a.part + size_t(s) * a.max_chunks, a.max_chunks, 1, dsum, dcnt, dmin, dmax, dor, drf);
  if (threadIdx.x == 0) a.agg_local[s] = p;
}

// PF: 0 = no prefetch (U = 4 rows per thread for 8-series segments, 8 for <= 4), 1 =
// prefetch with the same U (two register buffers: fewer waves fit), 2 = prefetch with
// half the rows per buffer (the registers of PF 0)
template <int PASS, int PF>
__device__ __forceinline__ void lw_pass_body(const LwArgs& a) {
  // LDS histogram words per series (pass B keeps no histogram)
  constexpr uint32_t HW = PASS == 0 ? kB0 / 2 : (PASS == kPassBrk ? 0u : kLongRanks * 128);
  static_assert(kLongChunkRowsMax < 65536, "16-bit LDS bins");
  extern __shared__ uint32_t h[];
  __shared__ uint32_t pre[kSegCols * kLongRanks];
  __shared__ uint32_t dshift[kSegCols], dwidth[kSegCols], dref[kSegCols];
  __shared__ uint32_t pmin[kSegCols], pmax[kSegCols], plx[kSegCols], plo[kSegCols];
  __shared__ uint32_t live, maxdw;
  __shared__ uint32_t ccount[kSegCols];
  __shared__ double rsum[NT / 64][kSegCols];
  __shared__ uint32_t rcnt[NT / 64][kSegCols], rmin[NT / 64][kSegCols], rmax[NT / 64][kSegCols], ror[NT / 64][kSegCols];
  __shared__ uint32_t bcnt[kSegCols * kBrkQ], beq[kSegCols * kBrkQ], rlt[NT / 64][kSegCols * kBrkQ];

  uint32_t gi = 0, c = 0, cs1 = 0;
  bool split = false;  // column-split pass B: this workgroup streams column cs1 of the segment only
  if (PASS == kPassBrk && a.nwork) {  // incremental pass B: the host's list of (segment, chunk)
    const uint32_t e = a.work[blockIdx.x];
    c = e & 0xFFFFFu;
    if (a.colsplit) {
      gi = e >> 23;
      cs1 = (e >> 20) & 7u;
      split = true;
    } else {
      gi = e >> 20;
    }
  } else {
    for (uint32_t i = 1; i < a.num_segs; ++i)  // the segment whose workgroup range holds this one
      if (blockIdx.x >= a.segs[i].wg0) gi = i;
    c = blockIdx.x - a.segs[gi].wg0;
  }
  const LwSeg G = a.segs[gi];
  const uint32_t r = G.ring;
  const LwRing R = a.rings[r];
  const uint32_t col0 = G.col0 + cs1;                 // the first column this workgroup streams
  const uint32_t w = split ? 1u : G.ncols;            // series it streams
  const uint32_t sb = R.first_series + col0;          // its first series
  const float* seg = R.dev + col0;                    // row i: seg + i * R.width
  const int t = threadIdx.x;

  if constexpr (PASS == 0) {
    if (t == 0) {
      maxdw = 1;
      live = 0;  // columns to stream: those scan B did not resolve
    }
    __syncthreads();
    if (uint32_t(t) < w && !(a.brk_on && a.sel[sb + t].done)) atomicOr(&live, 1u << t);
    __syncthreads();
    if (!live) return;  // scan B resolved every series of the segment (uniform): no prediction either
    if (a.node_n == 0) {
      lw_predict(a, r, seg, R.width, w, sb, pmin, pmax, plo, plx, dref);
    } else {
      // node mode: every rank combines the all-gathered predictions in rank order, so
      // every rank picks the same digit. The node window lies inside the union of the
      // ranks' predicted sets: min / max over them; the varying bits are each rank's
      // plus those where the ranks' reference keys differ, and the common reference
      // key is the first rank's that holds samples (a node-window member)
      if (uint32_t(t) < w) {
        uint32_t mn = 0xFFFFFFFFu, mx = 0u, lo = 32u, ref = 0u;
        bool any = false;
        for (uint32_t q = 0; q < a.node_n; ++q) {
          const LwPred p = a.pred_all[size_t(q) * a.num_series + sb + t];
          mn = min(mn, p.pmin);
          mx = max(mx, p.pmax);
          lo = min(lo, p.lo);
          if (p.has) {
            if (!any) {
              ref = p.ref;
              any = true;
            } else if (p.ref != ref) {
              lo = min(lo, uint32_t(__builtin_ctz(p.ref ^ ref)));
            }
          }
        }
        pmin[t] = mn;
        pmax[t] = mx;
        plo[t] = lo;
        plx[t] = 0;
        dref[t] = ref;
      }
      __syncthreads();
    }
    if (uint32_t(t) < w) {
      const uint32_t d = pmin[t] ^ pmax[t];
      const uint32_t top = d ? 31u - uint32_t(__builtin_clz(d)) : 0u;
      // the digit width: 10 bits when that saves a pass over 8 (the predicted span, down
      // to the predicted lowest varying bit), else 8 - the top byte of mixed-sign data
      // falls into few bins (one atomic per wave), 10 bits would not
      const uint32_t lo = min(plo[t], plx[t] ? uint32_t(__builtin_ctz(plx[t])) : 32u);
      const uint32_t span = top >= lo ? top - lo + 1 : 1u;
      const auto passes = [span](uint32_t dw) { return span > dw ? (span - dw + 7) / 8 : 0u; };
      const uint32_t dw = passes(kD0) < passes(8) ? uint32_t(kD0) : 8u;
      dwidth[t] = dw;
      atomicMax(&maxdw, dw);
      dshift[t] = top >= dw - 1 ? top - (dw - 1) : 0u;
      if (c == 0) {  // every workgroup of the ring computes the same: chunk 0 tells scan 0
        a.dig0[3 * (sb + t)] = dshift[t];
        a.dig0[3 * (sb + t) + 1] = dref[t];
        a.dig0[3 * (sb + t) + 2] = dw;
      }
    }
  } else if constexpr (PASS == kPassBrk) {
    if (t == 0) live = 0;
    // scan B decides with a copy of every series' brackets (it writes the next ones into
    // brk while its other workgroups still read): the grid's first workgroup makes it, in
    // the flat grid and in the incremental work list alike
    if (blockIdx.x == 0)
      for (uint32_t i = t; i < a.num_series; i += NT) a.brk_used[i] = a.brk[i];
    __syncthreads();
    if (uint32_t(t) < w && a.brk[sb + t].valid) atomicOr(&live, 1u << t);
    if (uint32_t(t) < kSegCols * kBrkQ) bcnt[t] = beq[t] = 0;
    __syncthreads();
    if (!live) return;  // no series of the segment has brackets this refresh (uniform)
    if (uint32_t(t) < w) {
      // orx's reference: the newest sample (a window member), as pass 0's
      const uint32_t n = a.params->n[r];
      const float x = n ? seg[((a.params->head[r] - 1) & uint64_t(a.mask)) * R.width + t] : __builtin_nanf("");
      dref[t] = isnan(x) ? 0u : fkey(x);
    }
    __syncthreads();
  } else {
    if (t == 0) live = 0;
    __syncthreads();
    if (uint32_t(t) < w) {
      const LwSel& sl = a.sel[sb + t];
      dshift[t] = sl.shift;
      dwidth[t] = sl.width;
      if (sl.width) atomicOr(&live, 1u);
    }
    for (uint32_t i = t; i < w * kLongRanks; i += NT) pre[i] = a.sel[sb + i / kLongRanks].prefix[i % kLongRanks];
    __syncthreads();
    if (!live) return;  // every series of the ring is resolved: nothing to stream
  }
  if constexpr (PASS == 0) __syncthreads();  // maxdw
  // LDS words per series: pass 0 sized by the ring's widest digit (the launch reserves 10 bits)
  const uint32_t hw = PASS == 0 ? (1u << maxdw) / 2 : HW;
  // pass 0 with 8-bit digits (the top byte: mixed signs, or no prediction) puts most
  // samples of a series into one or two bins, and the 4 waves' atomics then queue on the
  // same LDS words: with wave_priv each wave counts into its own copy (4 x 8-bit copies
  // fit the 10-bit reservation), summed word-wise in the merge (a bin's halves stay
  // below 2^16 over all copies: <= kLongChunkRows samples per workgroup)
  // wave_priv 2: a copy per half wave (32 lanes), the copies 16 banks apart - half the
  // lanes that share a bin per atomic (launch reserves 8 x (w x 128 + 16) words)
  const uint32_t lvl = (PASS == 0 && maxdw == 8) ? a.wave_priv : 0u;
  const uint32_t copies = lvl == 2 ? 2 * (NT / 64) : (lvl == 1 ? NT / 64 : 1u);
  const uint32_t cs = w * hw + (lvl == 2 ? 16u : 0u);  // words per copy
  for (uint32_t i = t; i < copies * cs; i += NT) h[i] = 0;
  if (uint32_t(t) < kSegCols) ccount[t] = 0;
  __syncthreads();

  const uint32_t colmask = (PASS == 0 || PASS == kPassBrk) ? live : 0xFFFFFFFFu;
  const LwShared sh_{pre, dshift, dwidth, dref, rsum, rcnt, rmin, rmax, ror, ccount, colmask, bcnt, beq, rlt};
  const LwView V{seg,
                 R.width,
                 R.chunk_rows,
                 w,
                 !split && ((R.width | col0) & 3u) == 0,
                 sb,
                 a.bcand ? a.bcand + R.boff + size_t(col0) * R.bstride : nullptr,
                 R.bstride,
                 R.qcap,
                 a.brk,
                 (1u << kBrkQ) - 1u,
                 nullptr,
                 false,
                 nullptr};
  uint32_t* hmine = h + (lvl == 2 ? uint32_t(t >> 5) : (lvl == 1 ? uint32_t(t >> 6) : 0u)) * cs;
  // rows per thread per buffer, 8-series segments (pass B: 2 - its bracket counters take
  // the registers of the other rows)
  constexpr int UN = (PF == 2 || PASS == kPassBrk) ? 2 : 4;
  if constexpr (PASS == kPassBrk) {
    if (split) {  // one column, in its segment's sum groups
      // (with the next rows' loads in flight: a lone workgroup per chunk is latency-bound)
      // 32 rows per thread per iteration, the next 32 in flight: a chunk of 24576 rows is 3
      // iterations, ~3 memory latencies instead of 24
      if (G.ncols <= 4) pass_chunk<PASS, 1, 32, true, 8>(a, V, r, c, hmine, hw, sh_);
      else pass_chunk<PASS, 1, 32, true, 4>(a, V, r, c, hmine, hw, sh_);
    } else if (w <= 4) {
      pass_chunk<PASS, 4, 2 * UN, PF != 0>(a, V, r, c, hmine, hw, sh_);
    } else {
      pass_chunk<PASS, kSegCols, UN, PF != 0>(a, V, r, c, hmine, hw, sh_);
    }
  } else {
    if (w <= 4) pass_chunk<PASS, 4, 2 * UN, PF != 0>(a, V, r, c, hmine, hw, sh_);
    else pass_chunk<PASS, kSegCols, UN, PF != 0>(a, V, r, c, hmine, hw, sh_);
  }
  __syncthreads();
  if (copies > 1) {  // fold the wave copies into copy 0
    for (uint32_t i = t; i < w * hw; i += NT) {
      uint32_t x = h[i];
      for (uint32_t k = 1; k < copies; ++k) x += h[k * cs + i];
      h[i] = x;
    }
    __syncthreads();
  }
  if constexpr (PASS == 2) {  // the chunk's candidate count per series (pass 3 reads its slab)
    if (a.compact && uint32_t(t) < w) a.cand_n[size_t(sb + t) * a.max_chunks + c] = ccount[t];
  }
  if constexpr (PASS == 0 || PASS == kPassBrk) {
    if (uint32_t(t) < w && ((colmask >> t) & 1u)) {
      LwPartial pp{0.0, 0, 0xFFFFFFFFu, 0, 0, dref[t], 0};  // every sample's orx is relative to dref
      for (int wv = 0; wv < NT / 64; ++wv) {
        pp.sum += rsum[wv][t];
        pp.cnt += rcnt[wv][t];
        pp.minkey = min(pp.minkey, rmin[wv][t]);
        pp.maxkey = max(pp.maxkey, rmax[wv][t]);
        pp.orx |= ror[wv][t];
      }
      a.part[size_t(sb + t) * a.max_chunks + c] = pp;
      if constexpr (PASS == kPassBrk) {
        LwBrkPart bp{};
        for (int q = 0; q < kBrkQ; ++q) {
          bp.mid[q] = bcnt[t * kBrkQ + q];
          bp.eq[q] = beq[t * kBrkQ + q];
          for (int wv = 0; wv < NT / 64; ++wv) bp.lt[q] += rlt[wv][t * kBrkQ + q];
        }
        a.bpart[size_t(sb + t) * a.max_chunks + c] = bp;
      }
    }
  }
  if constexpr (PASS != kPassBrk) {  // pass B keeps no histogram
    // merge the non-zero bins: one device-scope atomic each (kernel boundary publishes)
    constexpr uint32_t GB = PASS == 0 ? kB0 : kLongRanks * 256;  // global bins per series
    uint32_t* g = (PASS == 0 ? a.hist0 : a.histk) + size_t(sb) * GB;
    for (uint32_t i = t; i < w * hw; i += NT) {
      const uint32_t x = h[i];
      const uint32_t b = PASS == 0 ? (i / hw) * GB + 2 * (i % hw) : 2 * i;  // pass 0: series, bin
      if (x & 0xFFFFu) atomicAdd(&g[b], x & 0xFFFFu);
      if (x >> 16) atomicAdd(&g[b + 1], x >> 16);
    }
  }
}

template <int PASS, int PF>
__global__ __launch_bounds__(NT) void lw_pass(const LwArgs a) {
  lw_pass_body<PASS, PF>(a);
}

// pass B (bracket counts): 4 waves per SIMD, as pass 0 - its per-lane bracket counters
// would otherwise take it to 3
__global__ __launch_bounds__(NT, 4) void lw_pass_brk(const LwArgs a) {
  lw_pass_body<kPassBrk, 0>(a);
}

// pass 3 over the candidates pass 2 kept (compaction on): one workgroup per (block of
// chunk_rows candidates, series); the same prefix test and LDS histogram as lw_pass<3>,
// merged into the same global histogram, so scan 3 does not know the difference
__global__ __launch_bounds__(NT) void lw_pass_cand(const LwArgs a) {
  __shared__ uint32_t h[kLongRanks * 128];
  __shared__ uint32_t pre_s[kLongRanks];
  const uint32_t s = blockIdx.y;
  const int t = threadIdx.x;
  const uint32_t wd = __builtin_amdgcn_readfirstlane(a.sel[s].width);
  if (!wd) return;  // resolved: nothing to count (uniform)
  // workgroup (c, s) reads the slab pass 2's workgroup c filled for series s
  const uint32_t rows = __builtin_amdgcn_readfirstlane(a.cand_n[size_t(s) * a.max_chunks + blockIdx.x]);
  if (!rows) return;
  uint32_t r, col;
  series_ring(a, s, r, col);
  const uint32_t row0 = blockIdx.x * a.rings[r].chunk_rows;
  const uint32_t fsh = __builtin_amdgcn_readfirstlane(a.sel[s].shift), dsh = fsh - wd;
  if (t < kLongRanks) pre_s[t] = a.sel[s].prefix[t] >> fsh;
  for (uint32_t i = t; i < kLongRanks * 128; i += NT) h[i] = 0;
  __syncthreads();
  uint32_t pre[kLongRanks], cmask = 0;
#pragma unroll
  for (int q = 0; q < kLongRanks; ++q) {
    pre[q] = pre_s[q];
    bool first = true;
#pragma unroll
    for (int q2 = 0; q2 < q; ++q2) first = first && pre[q2] != pre[q];
    if (first) cmask |= 1u << q;
  }
  const uint32_t* c = a.cand + size_t(s) * a.cand_cap + row0;
  for (uint32_t i = t; i < rows; i += NT) {
    const uint32_t k = c[i];
    const uint32_t bin = __builtin_amdgcn_ubfe(k, dsh, wd);
    const uint32_t hk = k >> fsh;
#pragma unroll
    for (int q = 0; q < kLongRanks; ++q)
      if (((cmask >> q) & 1u) && hk == pre[q]) atomicAdd(&h[q * 128 + (bin >> 1)], 1u << ((bin & 1u) * 16u));
  }
  __syncthreads();
  uint32_t* g = a.histk + size_t(s) * kLongRanks * 256;
  for (uint32_t i = t; i < kLongRanks * 128; i += NT) {
    const uint32_t x = h[i];
    if (x & 0xFFFFu) atomicAdd(&g[2 * i], x & 0xFFFFu);
    if (x >> 16) atomicAdd(&g[2 * i + 1], x >> 16);
  }
}

// exclusive / inclusive prefix of one value per thread over the 256-thread block
__device__ inline void block_scan(uint32_t v, uint32_t* tmp, uint32_t& excl, uint32_t& incl) {
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  uint32_t x = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t y = __shfl_up(x, off);
    if (lane >= off) x += y;
  }
  if (lane == 63) tmp[wave] = x;
  __syncthreads();
  uint32_t base = 0;
  for (int wv = 0; wv < wave; ++wv) base += tmp[wv];
  incl = base + x;
  excl = incl - v;
  __syncthreads();  // tmp reusable
}

// The next refresh's bracket q: around this refresh's percentile keys (its lo / hi
// position), half-width adapted so the bracket holds ~kBrkTarget samples. `had`: the
// bracket was used this refresh and b.cin[q] holds what it held (else a first estimate
// `est` from the key range: uniform density over [min, max]).
// samples a bracket aims to hold: kBrkTarget, or 1/16 of a small window (a chunk's slab
// keeps at most a quarter of its rows per bracket)
__device__ inline uint32_t lw_brk_target(const LwArgs& a, uint32_t nv) {
  return max(64u, min(a.node_brk ? kNodeBrkTarget : a.brk_target, nv / 16));
}
// The half-width is kept in value units: the number of samples inside grows linearly with
// it there, while in key units it does not (near 0 a key step is a tiny value step, far
// from it a large one: mixed-sign data centred on 0 made a key-unit half-width oscillate
// between a few hundred and tens of thousands of samples)
// The first estimate assumes a quarter of the uniform density's width: near a normal
// distribution's median the density is ~3x the uniform one over [min, max], and a first
// bracket that overflows its kept-key cap is read as ties (below)
__device__ inline float lw_brk_est(uint32_t minkey, uint32_t maxkey, uint32_t nv, uint32_t target) {
  if (!nv) return 0.f;
  const double est = (double(kfloat(maxkey)) - double(kfloat(minkey))) * double(target) / (8.0 * nv);
  return est > 0.0 && est < 3.0e38 ? float(est) : (est > 0.0 ? 3.0e38f : 0.f);
}
// delta (float bits) / cin: the bracket's half-width and what it held this refresh -> its
// next half-width and bounds (delta, lo, hi updated in place); a half-width of 0 makes the
// bracket exactly [klo, khi] (ties: a one-key bracket stores no keys)
__device__ inline void lw_next_bracket(uint32_t& delta, uint32_t cin, uint32_t& lo, uint32_t& hi, uint32_t klo,
                                       uint32_t khi, float est, bool had, uint32_t target, bool join = true,
                                       uint32_t* dsave = nullptr) {
  const float dv = __uint_as_float(delta);
  double d;
  if (!had) {
    d = est;
  } else if (dv == 0.f) {  // an exact-key bracket: keep it while ties hold the rank
    if (cin >= target / 8) {
      // the percentile moved to a neighbouring tied value (a median between two readings
      // flips between them): the next exact bracket spans the old keys and the new, and
      // holds both with their ties counted on its bounds. Not after an overflow (a value
      // between them had too many ties to keep): then only the new keys
      if (join) {
        lo = min(lo, klo);
        hi = max(hi, khi);
      } else {
        lo = klo;
        hi = khi;
      }
      return;
    }
    // not ties after all (an overflow read as ties on continuous data with heavy tails):
    // back to the value half-width the overflow put aside, else the estimate
    const float ds = dsave ? __uint_as_float(*dsave) : 0.f;
    d = ds > 0.f ? double(ds) : double(est);
  } else {
    // to the target in one step when it held too many (the local density), at most 8x
    // wider when too few
    d = double(dv) * fmin(8.0, double(target) / double(max(cin, 1u)));
  }
  if (dsave) *dsave = 0u;
  if (!(d < 3.0e38)) d = 3.0e38;
  const float df = float(d);
  delta = __float_as_uint(df);
  if (df == 0.f) {
    lo = klo;
    hi = khi;
    return;
  }
  lo = min(klo, fkey(kfloat(klo) - df));  // rounding never leaves the keys outside
  hi = max(khi, fkey(kfloat(khi) + df));
  if (klo - lo <= 1u && hi - khi <= 1u) {
    // narrower than the keys' spacing: ties (a bracket around tied values keeps every tie
    // and overflows, shrinking it further cannot help) - exactly the keys, whose ties are
    // then counted on the bounds instead of kept
    delta = 0u;
    lo = klo;
    hi = khi;
  }
}
// Brackets pay when the radix chain needs more than one streaming pass: a window whose
// varying key bits [lo, top] span <= 10 bits (integer telemetry in a band) is resolved
// by pass 0's digit alone, which costs less than pass B
__device__ inline uint32_t lw_brk_wanted(uint32_t nv, uint32_t minkey, uint32_t maxkey, uint32_t lo) {
  const uint32_t d = minkey ^ maxkey;
  const uint32_t top = d ? 31u - uint32_t(__builtin_clz(d)) : 0u;
  const uint32_t span = top >= lo ? top - lo + 1 : 1u;
  return nv && span > uint32_t(kD0) ? 1u : 0u;
}

// exclusive / inclusive prefix of one value per thread over the 256-thread block; total:
// the block's sum (every thread)
__device__ inline void block_scan_total(uint32_t v, uint32_t* tmp, uint32_t& excl, uint32_t& incl, uint32_t& total) {
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  uint32_t x = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t y = __shfl_up(x, off);
    if (lane >= off) x += y;
  }
  if (lane == 63) tmp[wave] = x;
  __syncthreads();
  uint32_t base = 0, tot = 0;
  for (int wv = 0; wv < NT / 64; ++wv) {
    if (wv < wave) base += tmp[wv];
    tot += tmp[wv];
  }
  incl = base + x;
  excl = incl - v;
  total = tot;
  __syncthreads();  // tmp reusable
}

// The keys at sorted positions ra <= rb among the n keys of a bracket [lo, lo + 2^bits)
// in LDS: an LDS radix select on key - lo, kSelBits per pass from the top (two prefixes
// while the ranks' digits agree, one histogram each once they differ).
__device__ inline void lds_select2(const uint32_t* keys, uint32_t n, uint32_t lo, uint32_t bits, uint32_t ra,
                                   uint32_t rb, uint32_t* hist, uint32_t* tmp, uint32_t* found, uint32_t& ka,
                                   uint32_t& kb) {
  constexpr uint32_t NB = 1u << kSelBits, BPT = NB / NT;
  const int t = threadIdx.x;
  uint32_t pa = 0, pb = 0;  // found bits of key - lo (above `shift`)
  uint32_t shift = bits;
  while (shift > 0) {
    const uint32_t wd = min(kSelBits, shift), ns = shift - wd;
    for (uint32_t i = t; i < 2 * NB; i += NT) hist[i] = 0;
    __syncthreads();
    for (uint32_t i = t; i < n; i += NT) {
      const uint32_t d = keys[i] - lo;
      const uint32_t hi = shift >= 32 ? 0u : d >> shift;
      const uint32_t dig = (d >> ns) & ((1u << wd) - 1u);
      if (hi == pa) atomicAdd(&hist[dig], 1u);
      if (pb != pa && hi == pb) atomicAdd(&hist[NB + dig], 1u);
    }
    __syncthreads();
    for (int k = 0; k < 2; ++k) {
      const uint32_t* H = hist + (k == 1 && pb != pa ? NB : 0u);
      const uint32_t rq = k == 0 ? ra : rb;
      uint32_t v[BPT], tot = 0;
#pragma unroll
      for (uint32_t j = 0; j < BPT; ++j) {
        v[j] = H[t * BPT + j];
        tot += v[j];
      }
      uint32_t excl, incl, all;
      block_scan_total(tot, tmp, excl, incl, all);
      if (tot && excl <= rq && rq < incl) {
        for (uint32_t j = 0; j < BPT; ++j) {
          if (v[j] && excl <= rq && rq < excl + v[j]) {
            found[2 * k] = t * BPT + j;
            found[2 * k + 1] = rq - excl;
          }
          excl += v[j];
        }
      }
      __syncthreads();
    }
    pa = (pa << wd) | found[0];
    ra = found[1];
    pb = (pb << wd) | found[2];
    rb = found[3];
    __syncthreads();  // found reusable
    shift = ns;
  }
  ka = lo + pa;
  kb = lo + pb;
}

// scan B: one workgroup per (series, bracket q). Each reduces pass B's partials and the
// bracket counts of all three brackets (the same decision in the three workgroups): if
// every percentile's lo and hi positions fall inside their brackets (and no slab
// overflowed), workgroup q selects its two keys among bracket q's kept keys and writes
// percentile q; workgroup 0 writes min / max / mean / count / last and marks the series
// done - the radix chain then skips it; else it is left to the radix chain (done = 0).
// The brackets pass B used come from brk_used (pass B's copy); the next refresh's go to
// brk.
// scan B's phase clocks (LongWindowSet::set_phase_clocks): workgroup (s, q) thread 0
// writes the shader clock at phase k - a vector store to device memory
__device__ inline void lw_clock(const LwArgs& a, uint32_t s, int q, int k) {
  if (a.dbg && threadIdx.x == 0) a.dbg[(size_t(s) * kBrkQ + q) * 8 + k] = __builtin_readcyclecounter();
}

// The rest of scan B, shared by its local (lw_scan_brk) and node (lw_node_brk_select)
// forms once the bracket counts are known: the hit decision, this workgroup's select (the
// ranks on a bound are the bound; the others among the kept keys, `gather` fills LDS with
// bracket q's), the next brackets and the outputs.
struct LwBrkCounts {
  uint32_t lt[kBrkQ];   // below
  uint32_t mid[kBrkQ];  // strictly inside (kept)
  uint32_t elo[kBrkQ];  // on lo
  uint32_t ehi[kBrkQ];  // on hi (hi != lo)
  uint32_t ovf;         // bracket bits whose kept keys did not all fit
};
template <class Gather>
__device__ inline void lw_brk_resolve(const LwArgs& a, uint32_t s, int q, const LwBrk& b, const LwPartial& tot,
                                      const LwBrkCounts& C, uint64_t entered, uint32_t r, uint32_t col,
                                      uint32_t* keys, uint32_t* hist, uint32_t* tmp, uint32_t* found,
                                      uint32_t (*red)[NT / 64], Gather gather) {
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const LwRing R = a.rings[r];
  const uint32_t nv = tot.cnt;
  uint32_t pos[kLongRanks];
  double frac[3];
  lw_positions(nv, a.params->pct, pos, frac);
  bool hit = nv > 0;
  // this workgroup's bracket (selected by unrolled compares: no dynamic register indexing)
  uint32_t lq = 0, hq = 0, dq = 0, ltq = 0, inq = 0, midq = 0, eloq = 0, p0 = 0, p1 = 0;
  bool ovq = false;
  double fq = 0.0;
#pragma unroll
  for (int k = 0; k < kBrkQ; ++k) {
    const uint32_t in = C.mid[k] + C.elo[k] + C.ehi[k];
    const bool ov = ((C.ovf >> k) & 1u) || C.mid[k] > kBrkCap;
    hit = hit && !ov && C.lt[k] <= pos[2 * k] && pos[2 * k + 1] < C.lt[k] + in;
    if (k == q) {
      lq = b.lo[k];
      hq = b.hi[k];
      dq = b.delta[k];
      ltq = C.lt[k];
      inq = in;
      midq = C.mid[k];
      eloq = C.elo[k];
      ovq = ov;
      p0 = pos[2 * k];
      p1 = pos[2 * k + 1];
      fq = frac[k];
    }
  }
  LwBrk* nb = a.brk + s;  // the next refresh's brackets (this workgroup writes field q)
  if (!hit) {  // the radix chain resolves the series; its scan 3 sets the next brackets
    if (t == 0) {
      nb->cin[q] = inq;
      // more kept keys than fit: read as ties between the percentile's keys (telemetry
      // readings) - the next bracket is exactly the keys the chain finds, their ties then
      // counted on its bounds, not kept. Continuous data that overflowed (rare: the first
      // estimate aims low) gets a value half-width back a refresh later (few inside)
      if (ovq) {
        // put the value half-width the normal rule would take aside: if the exact bracket
        // then holds few samples (not ties), the bracket resumes from it
        const float dv = __uint_as_float(dq);
        if (dv > 0.f)
          nb->dsave[q] = __float_as_uint(float(double(dv) * fmin(8.0, double(lw_brk_target(a, nv)) /
                                                                        double(max(inq, 1u)))));
        nb->delta[q] = 0u;
        nb->nounion[q] = 1u;
      }
      if (q == 0) {
        a.sel[s].done = 0;
        nb->refreshes = b.refreshes + 1;
      }
    }
    return;
  }
  const uint32_t target = lw_brk_target(a, nv);
  // every percentile inside its bracket: ranks on the lower bound are lo, past the kept
  // keys hi, between them a select among the kept keys
  const uint32_t r0 = p0 - ltq, r1 = p1 - ltq;
  const bool m0 = r0 >= eloq && r0 < eloq + midq, m1 = r1 >= eloq && r1 < eloq + midq;
  uint32_t k0 = r0 < eloq ? lq : hq, k1 = r1 < eloq ? lq : hq;
  lw_clock(a, s, q, 2);
  if (m0 || m1) {  // uniform
    gather(keys);  // bracket q's kept keys into LDS (midq of them)
    __syncthreads();
    lw_clock(a, s, q, 3);
    const uint32_t span = hq - lq;
    const uint32_t bits = 32u - uint32_t(__builtin_clz(span));
    uint32_t s0 = 0, s1 = 0;
    lds_select2(keys, midq, lq, bits, m0 ? r0 - eloq : r1 - eloq, m1 ? r1 - eloq : r0 - eloq, hist, tmp, found, s0,
                s1);
    if (m0) k0 = s0;
    if (m1) k1 = s1;
    lw_clock(a, s, q, 4);
  }
  // ties: every kept key is the percentile's own (integer telemetry) - an exact-key
  // bracket then holds the rank with no keys to keep (red[0] / red[1]: key min / max)
  bool ties = false;
  if (midq && k0 == k1 && m0 && m1) {  // uniform
    uint32_t kmn = 0xFFFFFFFFu, kmx = 0;
    for (uint32_t i = t; i < midq; i += NT) {
      kmn = min(kmn, keys[i]);
      kmx = max(kmx, keys[i]);
    }
    for (int off = 32; off >= 1; off >>= 1) {
      kmn = min(kmn, uint32_t(__shfl_xor(int(kmn), off)));
      kmx = max(kmx, uint32_t(__shfl_xor(int(kmx), off)));
    }
    if (lane == 0) {
      red[0][wave] = kmn;
      red[1][wave] = kmx;
    }
    __syncthreads();
    if (t == 0) {
      for (int wv = 1; wv < NT / 64; ++wv) {
        red[0][0] = min(red[0][0], red[0][wv]);
        red[1][0] = max(red[1][0], red[1][wv]);
      }
    }
    __syncthreads();
    ties = red[0][0] == k0 && red[1][0] == k0;
  }
  if (t == 0) {
    uint32_t nlo = lq, nhi = hq, nd = dq;
    // incremental mode: the bracket stays put while both positions sit well inside it and
    // it holds a sane number of samples (an exact-key bracket: any number - its ties are
    // counted, not kept) - its chunks' counts then stay valid and the next pass B streams
    // only the chunks new rows landed in; otherwise (and always without incr) it is
    // re-centred on the keys just found
    bool keep = false;
    if (a.incr) {
      // the margin: twice the rows that entered (how far a position can move by the next
      // refresh at this rate), at most an eighth of the bracket. Node brackets: the rows
      // that entered the whole node (the same on every rank - the brackets must stay so)
      const uint64_t ent = entered == ~uint64_t(0) ? uint64_t(inq) : entered;
      const uint32_t m = max(8u, uint32_t(min<uint64_t>(inq / 8, 2 * ent)));
      const bool exact = dq == 0u;
      const bool inside = p0 >= ltq + m && p1 + m < ltq + inq;
      const bool sized = exact || (inq <= 2 * target && 4 * inq >= target);  // the select costs what it keeps
      keep = inside && sized && !ties;
    }
    if (ties) {  // -> an exact-key bracket on the tied value
      nlo = nhi = k0;
      nd = 0u;
      if (a.bchg) a.bchg[s] = 1u;
    } else if (!keep) {
      lw_next_bracket(nd, inq, nlo, nhi, k0, k1, lw_brk_est(tot.minkey, tot.maxkey, nv, target), true, target, true,
                      &nb->dsave[q]);
      if (a.bchg && (nlo != lq || nhi != hq)) a.bchg[s] = 1u;  // its chunks' counts are stale now
    }
    nb->lo[q] = nlo;
    nb->hi[q] = nhi;
    nb->delta[q] = nd;
    nb->cin[q] = inq;
    const double x0 = kfloat(k0), x1 = kfloat(k1);
    a.out[size_t(s) * STAT_NUM + STAT_P0 + q] = float(fq >= 0.5 ? x1 - (x1 - x0) * (1.0 - fq) : x0 + (x1 - x0) * fq);
  }
  lw_clock(a, s, q, 5);
  if (q != 0) return;
  const uint32_t lov = tot.orx ? uint32_t(__builtin_ctz(tot.orx)) : 32u;
  if (t == 0) {
    LwSel S = a.sel[s];
    S.nv = nv;
    S.minkey = tot.minkey;
    S.maxkey = tot.maxkey;
    S.sum = tot.sum;
    S.lo = lov;
    S.width = 0;
    S.done = 1;
    a.sel[s] = S;
    const uint32_t want = a.incr ? (nv ? 1u : 0u) : lw_brk_wanted(nv, tot.minkey, tot.maxkey, lov);
    if (a.bchg && want != b.valid) a.bchg[s] = 1u;
    nb->valid = want;
    nb->hit = 1;
    nb->hits = b.hits + 1;
    nb->refreshes = b.refreshes + 1;
    if (a.hflags) a.hflags[s] = want;
  }
  if (t < STAT_NUM && (t < STAT_P0 || t >= STAT_P0 + kBrkQ)) {
    const uint64_t head = a.params->head[r];
    const uint32_t n = a.params->n[r];
    float o = __builtin_nanf("");
    if (t == STAT_COUNT) {
      o = float(nv);
    } else if (t == STAT_LAST) {  // node brackets: no node-wide newest sample (NaN)
      if (n && !a.node_brk) o = R.dev[((head - 1) & uint64_t(a.mask)) * R.width + col];
    } else if (t == STAT_MIN) {
      o = kfloat(tot.minkey);
    } else if (t == STAT_MAX) {
      o = kfloat(tot.maxkey);
    } else if (t == STAT_MEAN) {
      o = float(tot.sum / double(nv));
    }
    a.out[size_t(s) * STAT_NUM + t] = o;
  }
}

// Pass B's per-chunk bracket counts of series s, summed over the ring's chunks (every
// thread gets the totals). ovf: a chunk kept fewer keys than were strictly inside.
// tot != nullptr (scan B): the chunks' partials combined in the same loop (one memory round
// trip for both; the partial's reduction order is reduce_partials')
__device__ inline LwBrkCounts lw_brk_counts(const LwArgs& a, uint32_t s, const LwRing& R, const LwBrk& b,
                                            uint32_t (*red)[NT / 64], LwPartial* tot = nullptr,
                                            double* dsum = nullptr, uint32_t* dcnt = nullptr, uint32_t* dmin = nullptr,
                                            uint32_t* dmax = nullptr, uint32_t* dor = nullptr, uint32_t* drf = nullptr) {
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  uint32_t v[4 * kBrkQ + 1];
#pragma unroll
  for (int i = 0; i < 4 * kBrkQ + 1; ++i) v[i] = 0;
  double sm = 0.0;
  uint32_t cn = 0, lo = 0xFFFFFFFFu, hi = 0, ox = 0, rf = 0;
  if (b.valid) {
    // unrolled: a thread's chunks' loads in flight together (scan B's first phase was one
    // memory round trip per 256 chunks)
#pragma unroll 8
    for (uint32_t i = t; i < R.nchunks; i += NT) {
      if (tot) {
        const LwPartial pp = a.part[size_t(s) * a.max_chunks + i];
        lw_combine(sm, cn, lo, hi, ox, rf, pp.sum, pp.cnt, pp.minkey, pp.maxkey, pp.orx, pp.ref);
      }
      const LwBrkPart bp = a.bpart[size_t(s) * a.max_chunks + i];
#pragma unroll
      for (int k = 0; k < kBrkQ; ++k) {
        v[k] += bp.lt[k];
        v[kBrkQ + k] += bp.mid[k];
        v[2 * kBrkQ + k] += eq_lo(bp.eq[k]);
        v[3 * kBrkQ + k] += eq_hi(bp.eq[k]);
        if (bp.mid[k] > R.qcap) v[4 * kBrkQ] |= 1u << k;
      }
    }
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
#pragma unroll
    for (int i = 0; i < 4 * kBrkQ; ++i) v[i] += uint32_t(__shfl_xor(int(v[i]), off));
    v[4 * kBrkQ] |= uint32_t(__shfl_xor(int(v[4 * kBrkQ]), off));
  }
  __syncthreads();  // red may still be read by the caller's previous phase
  if (lane == 0)
    for (int i = 0; i < 4 * kBrkQ + 1; ++i) red[i][wave] = v[i];
  __syncthreads();
  LwBrkCounts C{};
  for (int wv = 0; wv < NT / 64; ++wv) {
    for (int k = 0; k < kBrkQ; ++k) {
      C.lt[k] += red[k][wv];
      C.mid[k] += red[kBrkQ + k][wv];
      C.elo[k] += red[2 * kBrkQ + k][wv];
      C.ehi[k] += red[3 * kBrkQ + k][wv];
    }
    C.ovf |= red[4 * kBrkQ][wv];
  }
  __syncthreads();  // red reusable
  if (tot) *tot = block_reduce_partial(sm, cn, lo, hi, ox, rf, dsum, dcnt, dmin, dmax, dor, drf);
  return C;
}

// Bracket q's kept keys of series s (every chunk's slab, chunk order) into dst. Thread t
// owns a contiguous run of chunks (<= kGatherRun of them): their counts are loaded at once,
// one block scan places the runs, then the first kGatherKeys keys of each of its chunks are
// loaded into registers with independent (predicated) loads - one memory round trip for
// the whole run - and stored; a chunk with more keys (rare: a bracket holds ~2048 samples
// over thousands of chunks) copies the rest in order.
constexpr uint32_t kGatherRun = 16, kGatherKeys = 4;
template <bool BATCH, class Dst>
__device__ inline void lw_gather_slabs(const LwArgs& a, uint32_t s, const LwRing& R, uint32_t col, int q, Dst dst,
                                       uint32_t* tmp) {
  const int t = threadIdx.x;
  const LwBrkPart* bp = a.bpart + size_t(s) * a.max_chunks;
  const uint32_t* slab = a.bcand + R.boff + size_t(col) * R.bstride;
  const uint32_t n = R.nchunks;
  const uint32_t per = (n + NT - 1) / NT;
  const uint32_t c_lo = min(uint32_t(t) * per, n), c_hi = min(c_lo + per, n);
  if (BATCH && per <= kGatherRun) {
    uint32_t m[kGatherRun];
#pragma unroll
    for (uint32_t k = 0; k < kGatherRun; ++k) m[k] = c_lo + k < c_hi ? bp[c_lo + k].mid[q] : 0u;
    uint32_t mine = 0;
#pragma unroll
    for (uint32_t k = 0; k < kGatherRun; ++k) mine += m[k];
    uint32_t excl, incl, total;
    block_scan_total(mine, tmp, excl, incl, total);
    uint32_t v[kGatherRun][kGatherKeys];
#pragma unroll
    for (uint32_t k = 0; k < kGatherRun; ++k) {
      const uint32_t* src = slab + (size_t(c_lo + k) * kBrkQ + q) * R.qcap;
#pragma unroll
      for (uint32_t j = 0; j < kGatherKeys; ++j) v[k][j] = j < m[k] ? src[j] : 0u;
    }
#pragma unroll
    for (uint32_t k = 0; k < kGatherRun; ++k) {
#pragma unroll
      for (uint32_t j = 0; j < kGatherKeys; ++j)
        if (j < m[k]) dst(excl + j, v[k][j]);
      if (m[k] > kGatherKeys) {
        const uint32_t* src = slab + (size_t(c_lo + k) * kBrkQ + q) * R.qcap;
        for (uint32_t j = kGatherKeys; j < m[k]; ++j) dst(excl + j, src[j]);
      }
      excl += m[k];
    }
    return;
  }
  uint32_t mine = 0;
  for (uint32_t c = c_lo; c < c_hi; ++c) mine += bp[c].mid[q];
  uint32_t excl, incl, total;
  block_scan_total(mine, tmp, excl, incl, total);
  for (uint32_t c = c_lo; c < c_hi; ++c) {
    const uint32_t m = bp[c].mid[q];
    const uint32_t* src = slab + (size_t(c) * kBrkQ + q) * R.qcap;
    for (uint32_t j = 0; j < m; ++j) dst(excl + j, src[j]);
    excl += m;
  }
}

__device__ inline void lw_brk_finish(const LwArgs& a);

// Fused pass B (a short work list - the steady state: the 1-2 chunks new rows landed in):
// workgroup (s, q) of scan B streams series s's changed chunks itself, one after another,
// exactly as a column-split pass B workgroup would (the same rows per thread, the same
// segment sum groups: the same partial bits), against the brackets pass B would use
// (brk_used: lw_ingest copied them) - one kernel fewer, and no pass B workgroups to drain.
// The three workgroups of a series write the same partials and bracket counts (identical
// bits: counts do not depend on order), but only bracket q's kept keys (their slab order
// is the workgroup's own), so each reads back exactly what it needs.
__device__ inline void lw_fused_passb(const LwArgs& a, uint32_t s, uint32_t qkeys, uint32_t r, uint32_t col) {
  __shared__ double rsum[NT / 64][kSegCols];
  __shared__ uint32_t rcnt[NT / 64][kSegCols], rmin[NT / 64][kSegCols], rmax[NT / 64][kSegCols],
      ror[NT / 64][kSegCols];
  __shared__ uint32_t bcnt[kSegCols * kBrkQ], beq[kSegCols * kBrkQ], rlt[NT / 64][kSegCols * kBrkQ];
  __shared__ uint32_t dref[kSegCols];
  const int t = threadIdx.x;
  const LwRing R = a.rings[r];
  uint32_t gi = 0;  // the segment holding the series (the work list names segments)
  for (uint32_t i = 0; i < a.num_segs; ++i)
    if (a.segs[i].ring == r && col >= a.segs[i].col0) gi = i;
  const LwSeg G = a.segs[gi];
  const float* seg = R.dev + col;
  // orx's reference, the newest sample (a window member), as pass B's: pass_chunk loads it
  // behind the rows (fused_ref) and leaves its key in dref[0]
  const uint32_t n = a.params->n[r];
  const float* newest = n ? seg + ((a.params->head[r] - 1) & uint64_t(a.mask)) * R.width : nullptr;
  const LwShared sh_{nullptr, nullptr, nullptr, dref, rsum, rcnt, rmin, rmax, ror, nullptr, 1u, bcnt, beq, rlt};
  const LwView V{seg,      R.width, R.chunk_rows, 1u,     false, s,   a.bcand + R.boff + size_t(col) * R.bstride,
                 R.bstride, R.qcap, a.brk_used,  qkeys,   newest, true, dref};
  if (uint32_t(t) < kSegCols * kBrkQ) bcnt[t] = beq[t] = 0;
  __syncthreads();
  for (uint32_t i = 0; i < a.nfused; ++i) {
    const uint32_t e = a.fwork[i];
    if ((e >> 20) != gi) continue;  // uniform
    const uint32_t c = e & 0xFFFFFu;
    if (G.ncols <= 4) pass_chunk<kPassBrk, 1, 32, true, 8>(a, V, r, c, nullptr, 0, sh_);
    else pass_chunk<kPassBrk, 1, 32, true, 4>(a, V, r, c, nullptr, 0, sh_);
    __syncthreads();
    if (t == 0) {  // as lw_pass_body's epilogue: the 4 waves in a fixed order
      LwPartial pp{0.0, 0, 0xFFFFFFFFu, 0, 0, dref[0], 0};
      LwBrkPart bp{};
      for (int wv = 0; wv < NT / 64; ++wv) {
        pp.sum += rsum[wv][0];
        pp.cnt += rcnt[wv][0];
        pp.minkey = min(pp.minkey, rmin[wv][0]);
        pp.maxkey = max(pp.maxkey, rmax[wv][0]);
        pp.orx |= ror[wv][0];
      }
      for (int k = 0; k < kBrkQ; ++k) {
        bp.mid[k] = bcnt[k];
        bp.eq[k] = beq[k];
        bcnt[k] = beq[k] = 0;  // the next chunk's
        for (int wv = 0; wv < NT / 64; ++wv) bp.lt[k] += rlt[wv][k];
      }
      a.part[size_t(s) * a.max_chunks + c] = pp;
      a.bpart[size_t(s) * a.max_chunks + c] = bp;
    }
    __syncthreads();  // the LDS counters and sums are the next chunk's
  }
  // the slab keys and counts written above are this workgroup's own: the barrier (workgroup
  // scope) orders them before its reads - no device-scope fence (an L2 write-back)
  __syncthreads();
}

template <bool FUSED>
__device__ __forceinline__ void lw_scan_brk_body(const LwArgs& a) {
  __shared__ double dsum[NT];
  __shared__ uint32_t dcnt[NT], dmin[NT], dmax[NT], dor[NT], drf[NT];
  __shared__ uint32_t tmp[NT / 64], found[4];
  __shared__ uint32_t red[4 * kBrkQ + 1][NT / 64];
  __shared__ uint32_t keys[kBrkCap];
  __shared__ uint32_t hist[2 << kSelBits];
  const uint32_t s = blockIdx.x;
  const int q = int(blockIdx.y);
  const int t = threadIdx.x;
  const LwBrk b = a.brk_used[s];
  if (!b.valid) {  // no brackets this refresh: the radix chain (its scan 3 sets them)
    if (t == 0 && q == 0) a.sel[s].done = 0;
    return;
  }
  uint32_t r, col;
  series_ring(a, s, r, col);
  const LwRing R = a.rings[r];
  const uint32_t qcap = R.qcap;
  lw_clock(a, s, q, 0);
  if constexpr (FUSED) {
    lw_fused_passb(a, s, 1u << q, r, col);
    lw_clock(a, s, q, 6);
  }
  LwPartial tot;
  const LwBrkCounts C = lw_brk_counts(a, s, R, b, red, &tot, dsum, dcnt, dmin, dmax, dor, drf);
  lw_clock(a, s, q, 1);
  const uint64_t ent = a.params->prev_head[r] ? a.params->head[r] - a.params->prev_head[r] : ~uint64_t(0);
  (void)qcap;
  lw_brk_resolve(a, s, q, b, tot, C, ent, r, col, keys, hist, tmp, found, red, [&](uint32_t* dst) {
    lw_gather_slabs<true>(a, s, R, col, q, [dst](uint32_t i, uint32_t k) { dst[i] = k; }, tmp);
  });
}

// ---- node bracket mode (refresh_node) ------------------------------------------------
// After pass B with the node's brackets: this rank's record of every series - its partials
// over its chunks (in the same order as lw_node_partials: the node mean keeps its bits),
// the bracket counts, and the kept keys of each bracket compacted from the chunk slabs (at
// most kNodeCap; more, or a chunk slab that overflowed, sets the bracket's ovf bit). The
// records are all-gathered: ONE collective carries everything the node's select needs.
__device__ __forceinline__ void lw_node_brk_local_body(const LwArgs& a) {
  __shared__ double dsum[NT];
  __shared__ uint32_t dcnt[NT], dmin[NT], dmax[NT], dor[NT], drf[NT];
  __shared__ uint32_t tmp[NT / 64];
  __shared__ uint32_t red[4 * kBrkQ + 1][NT / 64];
  const uint32_t s = blockIdx.x;
  const int t = threadIdx.x;
  LwNodeHdr* rec = reinterpret_cast<LwNodeHdr*>(a.nbl) + s;
  uint32_t* kept = reinterpret_cast<uint32_t*>(a.nbl + size_t(a.num_series) * sizeof(LwNodeHdr)) +
                   size_t(s) * kBrkQ * a.node_cap;
  const LwBrk b = a.brk_used[s];
  uint32_t r, col;
  series_ring(a, s, r, col);
  const LwRing R = a.rings[r];
  const LwPartial p =
      reduce_partials(a.part + size_t(s) * a.max_chunks, a.max_chunks, 1, dsum, dcnt, dmin, dmax, dor, drf);
  const LwBrkCounts C = lw_brk_counts(a, s, R, b, red);
  uint32_t ovf = C.ovf;
  for (int k = 0; k < kBrkQ; ++k)
    if (C.mid[k] > a.node_cap) ovf |= 1u << k;
  if (!b.valid) ovf = (1u << kBrkQ) - 1u;
  if (t == 0) {
    rec->p = p;
    for (int k = 0; k < kBrkQ; ++k) {
      rec->lt[k] = C.lt[k];
      rec->mid[k] = C.mid[k];
      rec->elo[k] = C.elo[k];
      rec->ehi[k] = C.ehi[k];
    }
    rec->ovf = ovf;
    const uint64_t ph = a.params->prev_head[r];
    rec->ent = ph ? uint32_t(min<uint64_t>(a.params->head[r] - ph, 0xFFFFFFFEull)) : 0xFFFFFFFFu;
  }
  // the kept keys, chunk order; a bracket that overflowed keeps none (it is a miss)
  for (int k = 0; k < kBrkQ; ++k) {
    if (!b.valid || ((ovf >> k) & 1u) || C.mid[k] == 0) continue;  // uniform
    uint32_t* dk = kept + size_t(k) * a.node_cap;
    lw_gather_slabs<false>(a, s, R, col, k, [dk](uint32_t i, uint32_t key) { dk[i] = key; }, tmp);
  }
}

// (A variant streaming short work lists itself, as the local scan B does, was measured in
// rounds 5-6 - 0 to 10 % on a 0.12 ms node refresh, within box noise, profiles/r06/nodewin/ -
// and removed: pass B's own launch stays.)
__global__ __launch_bounds__(NT) void lw_node_brk_local(const LwArgs a) { lw_node_brk_local_body(a); }

// The node's scan B: one workgroup per (series, bracket q). Every rank reduces the
// all-gathered records in rank order - the same node totals, the same decision, the same
// keys selected from the union of the ranks' kept keys - so every rank holds the same
// exact statistics of the node window and the same next brackets.
__device__ __forceinline__ void lw_node_brk_select_body(const LwArgs& a) {
  __shared__ double dsum[NT];
  __shared__ uint32_t dcnt[NT], dmin[NT], dmax[NT], dor[NT], drf[NT];
  __shared__ uint32_t tmp[NT / 64], found[4];
  __shared__ uint32_t red[4 * kBrkQ + 1][NT / 64];
  __shared__ uint32_t keys[kBrkCap];
  __shared__ uint32_t hist[2 << kSelBits];
  const uint32_t s = blockIdx.x;
  const int q = int(blockIdx.y);
  const int t = threadIdx.x;
  const LwBrk b = a.brk_used[s];
  if (!b.valid) {
    if (t == 0 && q == 0) a.sel[s].done = 0;
    return;
  }
  uint32_t r, col;
  series_ring(a, s, r, col);
  // node totals: the partials reduced exactly as the node radix chain's scan 0 reduces them
  // (the same mean bits either way), the counts in rank order
  const size_t block = lw_node_block(a.num_series, a.node_cap);
  auto hdr = [&](uint32_t k) -> const LwNodeHdr& {
    return reinterpret_cast<const LwNodeHdr*>(a.nball + k * block)[s];
  };
  const LwPartial tot =
      reduce_partials(&hdr(0).p, a.node_n, uint32_t(block / sizeof(LwPartial)), dsum, dcnt, dmin, dmax, dor, drf);
  LwBrkCounts C{};
  uint64_t ent = 0;  // rows that entered the node (unknown if any rank's is)
  uint32_t maxmid = 0;
  for (uint32_t k = 0; k < a.node_n; ++k) {
    const LwNodeHdr& rc = hdr(k);
    if (rc.mid[q] <= kNodeCap) maxmid = max(maxmid, rc.mid[q]);  // more misses at any cap
    for (int j = 0; j < kBrkQ; ++j) {
      C.lt[j] += rc.lt[j];
      C.mid[j] += rc.mid[j];
      C.elo[j] += rc.elo[j];
      C.ehi[j] += rc.ehi[j];
    }
    C.ovf |= rc.ovf;
    ent = (ent == ~uint64_t(0) || rc.ent == 0xFFFFFFFFu) ? ~uint64_t(0) : ent + rc.ent;
  }
  // the next refresh's record cap (lw_brk_finish hands the node's most to the host)
  if (t == 0) atomicMax(a.brk_cnt + 1, maxmid);
  lw_brk_resolve(a, s, q, b, tot, C, ent, r, col, keys, hist, tmp, found, red, [&](uint32_t* dst) {
    // the union of the ranks' kept keys of bracket q, rank order
    uint32_t base = 0;
    for (uint32_t k = 0; k < a.node_n; ++k) {
      const uint32_t m = hdr(k).mid[q];
      const uint32_t* src = reinterpret_cast<const uint32_t*>(a.nball + k * block +
                                                              size_t(a.num_series) * sizeof(LwNodeHdr)) +
                            (size_t(s) * kBrkQ + q) * a.node_cap;
      for (uint32_t j = t; j < m; j += NT) dst[base + j] = src[j];
      base += m;
    }
  });
}

// The end of scan B (local and node): every workgroup counts itself done; the last one
// (its device atomic returns the grid size - 1) counts the series the radix chain still has
// to resolve and writes the report word - the host's wait ends one kernel earlier than with
// a separate report launch. Every writer fences before the barrier, the counter's
// increment is a vector atomic on device memory, and the last workgroup resets it.
__device__ inline void lw_brk_finish(const LwArgs& a) {
  __shared__ uint32_t last, left;
  const int t = threadIdx.x;
  __threadfence();
  __syncthreads();
  if (t == 0) {
    left = 0;
    last = atomicAdd(a.brk_cnt, 1u) == gridDim.x * gridDim.y - 1 ? 1u : 0u;
  }
  __syncthreads();
  if (!last) return;
  __threadfence();
  for (uint32_t s = t; s < a.num_series; s += NT)
    if (!a.sel[s].done) atomicAdd(&left, 1u);
  __syncthreads();
  if (t == 0) {
    a.brk_cnt[0] = 0u;
    const uint32_t maxmid = atomicExch(a.brk_cnt + 1, 0u);
    if (a.report)  // one word: no system fence between two stores the host must see in order
      __hip_atomic_store(a.report,
                         (static_cast<unsigned long long>(min(maxmid, 0xFFFFu)) << 48) |
                             (static_cast<unsigned long long>(left) << 24) | (a.params->seq & 0xFFFFFFu),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

__global__ __launch_bounds__(NT) void lw_scan_brk(const LwArgs a) {
  lw_scan_brk_body<false>(a);
  lw_brk_finish(a);
}

// scan B with pass B fused in (LongWindowSet::refresh_incremental: a short work list)
__global__ __launch_bounds__(NT) void lw_scan_brk_fused(const LwArgs a) {
  lw_scan_brk_body<true>(a);
  lw_brk_finish(a);
}

__global__ __launch_bounds__(NT) void lw_node_brk_select(const LwArgs a) {
  lw_node_brk_select_body(a);
  lw_brk_finish(a);
}

// A small refresh's staging in one launch: block 0 copies the parameter block and the work
// list from the pinned host slot, blocks 1.. the new rows of one ring segment each from the
// pinned host ring into the device window (rows that cross neither ring's wrap). Replaces
// 2-4 DMA copies whose fixed cost dominated a refresh that changes a few chunks.
struct LwIngestSeg {
  const float* src;  // host ring rows (device view)
  float* dst;        // device window rows
  uint32_t floats;
  uint32_t pad;
};
constexpr int kIngestSegs = 2 * kLongMaxRings;
struct LwIngest {
  const LwParams* hp;  // the slot (device view)
  LwParams* dp;
  const uint32_t* hwork;
  uint32_t* dwork;
  uint32_t nwork;
  uint32_t nseg;
  LwIngestSeg seg[kIngestSegs];
  const uint32_t* bsrc;  // the fused pass B's brackets: brk -> brk_used (bwords = 0: none), its own workgroup
  uint32_t* bdst;
  uint32_t bwords;
};
// Host reads cross the fabric (microseconds each): a thread issues kIngestBatch of them
// before it stores any, so a copy of a few KB is one round trip, not one per 256 words.
constexpr uint32_t kIngestBatch = 8;
__device__ inline void lw_copy_batched(uint32_t* dst, const uint32_t* src, uint32_t n) {
  for (uint32_t base = threadIdx.x; base < n; base += NT * kIngestBatch) {
    uint32_t v[kIngestBatch];
#pragma unroll
    for (uint32_t k = 0; k < kIngestBatch; ++k) v[k] = base + k * NT < n ? src[base + k * NT] : 0u;
#pragma unroll
    for (uint32_t k = 0; k < kIngestBatch; ++k)
      if (base + k * NT < n) dst[base + k * NT] = v[k];
  }
}
__global__ __launch_bounds__(NT) void lw_ingest(const LwIngest in) {
  if (blockIdx.x == 0) {
    lw_copy_batched(reinterpret_cast<uint32_t*>(in.dp), reinterpret_cast<const uint32_t*>(in.hp),
                    uint32_t(sizeof(LwParams) / 4));
    lw_copy_batched(in.dwork, in.hwork, in.nwork);
    return;
  }
  if (blockIdx.x == 1 + in.nseg) {
    lw_copy_batched(in.bdst, in.bsrc, in.bwords);
    return;
  }
  const LwIngestSeg g = in.seg[blockIdx.x - 1];
  lw_copy_batched(reinterpret_cast<uint32_t*>(g.dst), reinterpret_cast<const uint32_t*>(g.src), g.floats);
}

// ---- scan k: per series, find each rank's digit; the last scan writes the statistics ---
template <int PASS>
__global__ __launch_bounds__(NT) void lw_scan(const LwArgs a) {
  constexpr uint32_t BPT = PASS == 0 ? kB0 / NT : 1;  // bins per thread
  __shared__ uint32_t tmp[NT / 64];
  __shared__ double dsum[NT];
  __shared__ uint32_t dcnt[NT], dmin[NT], dmax[NT], dor[NT], drf[NT];
  __shared__ LwSel S;
  __shared__ uint32_t found_digit[kLongRanks], found_resid[kLongRanks];
  __shared__ uint32_t low_bits;  // the last scan: the key bits below the last digit (min's)
  const uint32_t s = blockIdx.x;
  const int t = threadIdx.x;
  if (a.brk_on && a.sel[s].done) return;  // scan B resolved the series (uniform)

  if constexpr (PASS == 0) {
    // partials in a fixed order -> deterministic mean (node mode: the ranks' all-gathered
    // partials in rank order - the same bits on every rank)
    const bool node = a.node_n != 0;
    const LwPartial tot = node ? reduce_partials(a.agg_all + s, a.node_n, a.num_series, dsum, dcnt, dmin, dmax, dor, drf)
                               : reduce_partials(a.part + size_t(s) * a.max_chunks, a.max_chunks, 1, dsum, dcnt, dmin,
                                                 dmax, dor, drf);
    if (t == 0) {
      S.nv = tot.cnt;
      S.done = 0;
      S.minkey = tot.minkey;
      S.maxkey = tot.maxkey;
      S.sum = tot.sum;
      S.shift = a.dig0[3 * s];
      S.width = a.dig0[3 * s + 2];  // this scan's digit: [shift, shift + width)
      // every key agrees with the reference key outside orx; bits above the predicted
      // range agree with min (the prediction is a superset of the varying bits)
      S.lo = tot.orx ? uint32_t(__builtin_ctz(tot.orx)) : 32u;
      uint32_t pos[kLongRanks];
      double frac[3];
      lw_positions(S.nv, a.params->pct, pos, frac);
      const uint32_t hb = S.shift + S.width;
      const uint32_t high = hb >= 32 ? 0u : (S.minkey >> hb) << hb;
      for (int q = 0; q < kLongRanks; ++q) {
        S.resid[q] = pos[q];
        S.prefix[q] = high;
      }
    }
  } else {
    if (t == 0) S = a.sel[s];
  }
  if (t < kLongRanks) {
    found_digit[t] = 0;
    found_resid[t] = 0;
  }
  __syncthreads();

  const uint32_t nv = S.nv;
  const bool search = nv && S.width;
  if (search) {
    for (int q = 0; q < kLongRanks; ++q) {
      // pass 0: every rank searches the one histogram of the series
      // passes > 0: ranks with one prefix share the histogram of the first of them
      int qc = q;
      if constexpr (PASS > 0) {
        for (int q2 = q - 1; q2 >= 0; --q2)
          if (S.prefix[q2] == S.prefix[q]) qc = q2;
      }
      const uint32_t* H = PASS == 0 ? a.hist0 + size_t(s) * kB0 : a.histk + (size_t(s) * kLongRanks + qc) * 256;
      uint32_t v[BPT], tot = 0;
#pragma unroll
      for (uint32_t j = 0; j < BPT; ++j) {
        v[j] = H[t * BPT + j];
        tot += v[j];
      }
      uint32_t excl, incl;
      block_scan(tot, tmp, excl, incl);
      const uint32_t rq = S.resid[q];
      if (tot && excl <= rq && rq < incl) {
#pragma unroll
        for (uint32_t j = 0; j < BPT; ++j) {
          if (v[j] && excl <= rq && rq < excl + v[j]) {
            found_digit[q] = t * BPT + j;
            found_resid[q] = rq - excl;
          }
          excl += v[j];
        }
      }
      __syncthreads();
    }
  }
  // re-zero what this scan consumed (the next pass / refresh accumulates into it)
  if constexpr (PASS == 0) {
#pragma unroll
    for (uint32_t j = 0; j < BPT; ++j) a.hist0[size_t(s) * kB0 + t * BPT + j] = 0;
  } else {
    for (int q = 0; q < kLongRanks; ++q) a.histk[(size_t(s) * kLongRanks + q) * 256 + t] = 0;
  }
  if (t == 0) {
    if (search) {
      for (int q = 0; q < kLongRanks; ++q) {
        S.prefix[q] |= found_digit[q] << (PASS == 0 ? S.shift : S.shift - S.width);
        S.resid[q] = found_resid[q];
      }
    }
    if constexpr (PASS > 0) S.shift -= S.width;
    S.width = nv ? next_width(S.shift, S.lo) : 0u;
    // bits below the last digit never vary: min's (shift <= 22 here)
    low_bits = S.minkey & ~(0xFFFFFFFFu << S.shift);
  }
  __syncthreads();
  if constexpr (PASS < 3) {
    if (t == 0) a.sel[s] = S;
  } else {
    if (t == 0) {
      a.sel[s] = S;  // min / max: the next refresh's prediction
      // the next refresh's brackets around the percentile keys just found
      uint32_t klo[kBrkQ], khi[kBrkQ];
      for (int q = 0; q < kBrkQ; ++q) {
        klo[q] = S.prefix[2 * q] | low_bits;
        khi[q] = S.prefix[2 * q + 1] | low_bits;
      }
      LwBrk b = a.brk[s];
      const bool had = a.brk_on && b.valid;
      const float est = lw_brk_est(S.minkey, S.maxkey, nv, lw_brk_target(a, nv));
      for (int q = 0; q < kBrkQ; ++q) {
        lw_next_bracket(b.delta[q], b.cin[q], b.lo[q], b.hi[q], klo[q], khi[q], est, had, lw_brk_target(a, nv),
                        !b.nounion[q], &b.dsave[q]);
        b.nounion[q] = 0u;
      }
      // incremental mode: brackets pay for every series (pass B then streams only the
      // chunks that changed); else only where the radix chain needs > 1 streaming pass
      b.valid = a.incr ? (nv ? 1u : 0u) : lw_brk_wanted(nv, S.minkey, S.maxkey, S.lo);
      b.hit = 0;
      a.brk[s] = b;
      if (a.hflags) a.hflags[s] = b.valid;  // the host's hint: launch pass B next refresh
      if (a.bchg) a.bchg[s] = 1u;  // new brackets: every chunk's counts must be taken again
    }
    if (t < STAT_NUM) {
      uint32_t r, col;
      series_ring(a, s, r, col);
      const LwRing R = a.rings[r];
      const uint64_t head = a.params->head[r];
      const uint32_t n = a.params->n[r];
      float o = __builtin_nanf("");
      if (t == STAT_COUNT) {
        o = float(nv);
      } else if (t == STAT_LAST) {  // node mode: no node-wide newest sample (NaN)
        if (n && !a.node_n) o = R.dev[((head - 1) & uint64_t(a.mask)) * R.width + col];
      } else if (nv) {
        if (t == STAT_MIN) {
          o = kfloat(S.minkey);
        } else if (t == STAT_MAX) {
          o = kfloat(S.maxkey);
        } else if (t == STAT_MEAN) {
          o = float(S.sum / double(nv));
        } else {
          const int q = t - STAT_P0;
          uint32_t pos[kLongRanks];
          double frac[3];
          lw_positions(nv, a.params->pct, pos, frac);
          const double x0 = kfloat(S.prefix[2 * q] | low_bits), x1 = kfloat(S.prefix[2 * q + 1] | low_bits);
          const double f = frac[q];
          o = float(f >= 0.5 ? x1 - (x1 - x0) * (1.0 - f) : x0 + (x1 - x0) * f);
        }
      }
      a.out[size_t(s) * STAT_NUM + t] = o;
    }
  }
}

}  // namespace

LongWindowSet::LongWindowSet(uint32_t window, int device, bool use_graph, uint32_t chunk_rows)
    : window_(window), device_(device), use_graph_(use_graph), chunk_rows_(chunk_rows) {
  if (const char* e = std::getenv("ROCMDASH_LW_PLAN_ROUNDS")) plan_rounds_ = uint32_t(std::clamp(std::atoi(e), 1, 16));
  if (const char* e = std::getenv("ROCMDASH_LW_BRK_TARGET"))
    brk_target_ = uint32_t(std::clamp(std::atoi(e), 256, int(kBrkTarget)));
  if (chunk_rows && (chunk_rows < 256 || chunk_rows > kLongChunkRows || (chunk_rows & (chunk_rows - 1))))
    throw std::invalid_argument("chunk_rows must be 0 (auto) or a power of two in [256, 32768]");
  if (window < kLongMinWindow || window > kLongMaxWindow || (window & (window - 1)))
    throw std::invalid_argument("long window must be a power of two in [2^10, 2^26]");
  const auto off = [](const char* v) { return v[0] == '0' || v[0] == 'n' || v[0] == 'f'; };
  if (const char* v = std::getenv("ROCMDASH_LW_WAVE_PRIVATE")) wave_priv_ = off(v) ? 0 : (v[0] == '2' ? 2 : 1);
  if (const char* v = std::getenv("ROCMDASH_LW_COMPACT")) compact_ = !off(v);
  if (const char* v = std::getenv("ROCMDASH_LW_PREFETCH")) prefetch_ = std::max(0, std::min(2, std::atoi(v)));
  if (const char* v = std::getenv("ROCMDASH_LW_BRACKETS")) brackets_ = !off(v);
  if (const char* v = std::getenv("ROCMDASH_LW_INCREMENTAL")) incremental_ = !off(v);
}

LongWindowSet::~LongWindowSet() {
  int cur = 0;
  (void)hipGetDevice(&cur);
  (void)hipSetDevice(device_);
  // refreshes still in flight write the work buffers and the host-mapped flags: wait for
  // this set's own last refresh only - never hipDeviceSynchronize, which
  // would also wait for an RCCL kernel stuck on a dead peer and hang the exit
  if (last_done_) (void)hipEventSynchronize(last_done_);
  if (exec_) (void)hipGraphExecDestroy(exec_);
  if (graph_) (void)hipGraphDestroy(graph_);
  if (cap_stream_) (void)hipStreamDestroy(cap_stream_);
  if (dbg_) (void)hipFree(dbg_);
  for (auto e : slot_done_) (void)hipEventDestroy(e);
  for (auto& r : rings_)
    if (r.dev) (void)hipFree(r.dev);
  for (void* p : {params_, part_, static_cast<void*>(hist0_), static_cast<void*>(histk_), sel_, static_cast<void*>(dig0_),
                  pred_local_, pred_all_, agg_local_, agg_all_, nbl_, nball_, static_cast<void*>(cand_),
                  static_cast<void*>(cand_n_), static_cast<void*>(work_dev_)})
    if (p) (void)hipFree(p);
  for (auto& m : bm_) {
    for (void* p : {m.brk, m.brk_used, m.bpart, static_cast<void*>(m.bcand), static_cast<void*>(m.brk_cnt)})
      if (p) (void)hipFree(p);
    for (void* p : {static_cast<void*>(m.hflags), static_cast<void*>(m.bchg), static_cast<void*>(m.report)})
      if (p) (void)hipHostFree(p);
    if (m.done) (void)hipEventDestroy(m.done);
  }
  for (auto e : node_events_) (void)hipEventDestroy(e);
  if (host_params_) (void)hipHostFree(host_params_);
  if (work_host_) (void)hipHostFree(work_host_);
  if (last_done_) (void)hipEventDestroy(last_done_);
  (void)hipSetDevice(cur);
}

uint32_t LongWindowSet::add_ring(std::shared_ptr<SeriesRing> ring) {
  if (!ring) throw std::invalid_argument("null ring");
  if (part_) throw std::logic_error("add_ring after the first refresh");
  if (rings_.size() == size_t(kLongMaxRings)) throw std::invalid_argument("at most 4 rings per long window set");
  const uint32_t width = ring->width();
  if (width == 0 || width > uint32_t(kLongMaxWidth)) throw std::invalid_argument("ring width must be in [1, 16]");
  Guard g(device_);
  RingState rs;
  rs.ring = std::move(ring);
  rs.first_series = nseries_;
  const size_t bytes = size_t(window_) * width * sizeof(float);
  check(hipMalloc(reinterpret_cast<void**>(&rs.dev), bytes), "hipMalloc long window");
  check(hipMemset(rs.dev, 0xFF, bytes), "hipMemset");  // NaN until written
  if (rs.ring->pinned()) {  // lw_ingest reads the new rows straight from the pinned host ring
    void* d = nullptr;
    if (hipHostGetDevicePointer(&d, const_cast<float*>(rs.ring->rows()), 0) == hipSuccess && d)
      rs.host_dev = static_cast<const float*>(d);
    else
      (void)hipGetLastError();
  }
  nseries_ += width;
  rings_.push_back(std::move(rs));
  return rings_.back().first_series;
}

void LongWindowSet::allocate_work() {
  if (rings_.empty()) throw std::logic_error("no rings");
  plan_chunks();
  const uint32_t max_chunks = max_chunks_;
  const size_t S = nseries_;
  check(hipMalloc(&params_, sizeof(LwParams)), "hipMalloc");
  check(hipMalloc(&part_, S * max_chunks * sizeof(LwPartial)), "hipMalloc");
  {  // a ring with fewer chunks never writes the slots past them: identity partials
    const std::vector<LwPartial> ident(S * max_chunks, LwPartial{0.0, 0, 0xFFFFFFFFu, 0, 0, 0, 0});
    check(hipMemcpy(part_, ident.data(), ident.size() * sizeof(LwPartial), hipMemcpyHostToDevice), "hipMemcpy");
  }
  check(hipMalloc(reinterpret_cast<void**>(&hist0_), S * kB0 * sizeof(uint32_t)), "hipMalloc");
  check(hipMalloc(reinterpret_cast<void**>(&histk_), S * kLongRanks * 256 * sizeof(uint32_t)), "hipMalloc");
  check(hipMalloc(&sel_, S * sizeof(LwSel)), "hipMalloc");
  check(hipMalloc(reinterpret_cast<void**>(&dig0_), S * 3 * sizeof(uint32_t)), "hipMalloc");
  check(hipMemset(sel_, 0, S * sizeof(LwSel)), "hipMemset");
  check(hipMemset(hist0_, 0, S * kB0 * sizeof(uint32_t)), "hipMemset");
  check(hipMemset(histk_, 0, S * kLongRanks * 256 * sizeof(uint32_t)), "hipMemset");
  check(hipHostMalloc(&host_params_, kSlots * sizeof(LwParams), hipHostMallocMapped | hipHostMallocCoherent),
        "hipHostMalloc");
  if (hipHostGetDevicePointer(&host_params_dev_, host_params_, 0) != hipSuccess) host_params_dev_ = nullptr;
  slot_done_.resize(kSlots);
  for (auto& e : slot_done_) check(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
  check(hipStreamCreateWithFlags(&cap_stream_, hipStreamNonBlocking), "hipStreamCreate");
  check(hipEventCreateWithFlags(&last_done_, hipEventDisableTiming), "hipEventCreate");
  // the incremental pass B's work lists: one pinned staging list per parameter slot
  check(hipMalloc(reinterpret_cast<void**>(&work_dev_), size_t(pass_wgs_) * sizeof(uint32_t)), "hipMalloc");
  check(hipHostMalloc(reinterpret_cast<void**>(&work_host_), size_t(kSlots) * pass_wgs_ * sizeof(uint32_t),
                      hipHostMallocMapped | hipHostMallocCoherent),
        "hipHostMalloc");
  {
    void* d = nullptr;
    work_host_dev_ = hipHostGetDevicePointer(&d, work_host_, 0) == hipSuccess ? static_cast<uint32_t*>(d) : nullptr;
  }
  allocate_mode(0);  // the local refresh's brackets (the node's at its first refresh_node)
}

// One bracket state (0: local refreshes, 1: node refreshes - around different percentiles,
// so neither invalidates the other's chunk counts): the brackets, pass B's per-chunk
// counts and kept-key slabs (3 / 64 of the window per series, lw_qcap), and the host-mapped
// flags the kernels leave for the host (wants brackets, brackets changed, the report word).
void LongWindowSet::allocate_mode(int mode) {
  BrkMode& m = bm_[mode];
  if (m.brk) return;
  const size_t S = nseries_;
  check(hipMalloc(&m.brk, S * sizeof(LwBrk)), "hipMalloc");
  check(hipMemset(m.brk, 0, S * sizeof(LwBrk)), "hipMemset");  // no brackets: the first refresh takes the radix chain
  check(hipMalloc(&m.brk_used, S * sizeof(LwBrk)), "hipMalloc");
  check(hipMemset(m.brk_used, 0, S * sizeof(LwBrk)), "hipMemset");
  check(hipMalloc(&m.bpart, S * max_chunks_ * sizeof(LwBrkPart)), "hipMalloc");
  check(hipMemset(m.bpart, 0, S * max_chunks_ * sizeof(LwBrkPart)), "hipMemset");
  check(hipMalloc(reinterpret_cast<void**>(&m.bcand), std::max<size_t>(1, bcand_keys_) * sizeof(uint32_t)), "hipMalloc slabs");
  const auto host_mapped = [](auto** h, auto** d, size_t bytes) {
    check(hipHostMalloc(reinterpret_cast<void**>(h), bytes, hipHostMallocMapped), "hipHostMalloc");
    std::memset(*h, 0, bytes);
    check(hipHostGetDevicePointer(reinterpret_cast<void**>(d), *h, 0), "hipHostGetDevicePointer");
  };
  host_mapped(&m.hflags, &m.hflags_dev, S * sizeof(uint32_t));
  host_mapped(&m.bchg, &m.bchg_dev, S * sizeof(uint32_t));
  host_mapped(&m.report, &m.report_dev, sizeof(unsigned long long));
  check(hipMalloc(reinterpret_cast<void**>(&m.brk_cnt), 2 * sizeof(uint32_t)), "hipMalloc");
  check(hipMemset(m.brk_cnt, 0, 2 * sizeof(uint32_t)), "hipMemset");
  check(hipEventCreateWithFlags(&m.done, hipEventDisableTiming), "hipEventCreate");
  m.seg_head.assign(2 * kLongMaxRings, kNever);
}

std::vector<std::pair<uint32_t, uint32_t>> long_window_chunk_plan(uint32_t window, const std::vector<uint32_t>& widths,
                                                                  int cus, uint32_t chunk_rows, uint32_t rounds) {
  // inputs of the exposed free function are checked here: the search below
  // ends for every valid window, and is bounded anyway
  if (window < kLongMinWindow || window > kLongMaxWindow || (window & (window - 1)))
    throw std::invalid_argument("long_window_chunk_plan: window must be a power of two in [2^10, 2^26]");
  if (widths.empty() || widths.size() > size_t(kLongMaxRings))
    throw std::invalid_argument("long_window_chunk_plan: 1 to 4 ring widths");
  for (uint32_t w : widths)
    if (w == 0 || w > uint32_t(kLongMaxWidth)) throw std::invalid_argument("long_window_chunk_plan: widths in [1, 16]");
  if (chunk_rows && (chunk_rows < 256 || chunk_rows > kLongChunkRows || (chunk_rows & (chunk_rows - 1))))
    throw std::invalid_argument("long_window_chunk_plan: chunk_rows must be 0 or a power of two in [256, 32768]");
  if (rounds < 1 || rounds > 16) throw std::invalid_argument("long_window_chunk_plan: rounds in [1, 16]");
  std::vector<std::pair<uint32_t, uint32_t>> plan(widths.size());
  if (chunk_rows) {  // uniform chunks (the caller's; tests and A/B)
    for (auto& p : plan) p = {chunk_rows, std::max<uint32_t>(1, window / chunk_rows)};
    return plan;
  }
  // Balanced by bytes: the passes are latency-bound per wave, so a pass lasts as long as
  // its slowest workgroup. Equal rows per workgroup over an 8-series and a 4-series ring
  // leave the 4-series workgroups done at half time and the chip at half occupancy for
  // the rest (profiles/r04/lw_ab/). Instead every workgroup streams about the same
  // bytes, and the grid is one round of the chip's workgroup slots (4 per CU at the
  // passes' registers) - or whole rounds, when a ring would need more rows per workgroup
  // than its 16-bit LDS bins allow. Rows per workgroup: a multiple of 256, >= 256.
  uint32_t total = 0;
  for (uint32_t w : widths) total += w;
  const uint64_t slots = uint64_t(std::max(cus, 1)) * 4;
  // every ring fits once a segment's workgroups reach window / kLongChunkRowsMax: at most
  // that many rounds of the slots
  const uint64_t max_rounds = uint64_t(kLongMaxWindow) / 256 + 1;
  for (uint64_t G = slots * rounds, round = 0; round < max_rounds; G += slots, ++round) {
    bool fits = true;
    for (size_t i = 0; i < widths.size() && fits; ++i) {
      const uint32_t nseg = (widths[i] + kSegCols - 1) / kSegCols;
      const double share = double(G) * widths[i] / double(std::max(total, 1u)) / nseg;  // workgroups per segment
      const uint64_t wg = std::max<uint64_t>(1, uint64_t(share + 0.5));
      uint64_t rows = (uint64_t(window) + wg - 1) / wg;
      rows = std::max<uint64_t>(256, (rows + 255) / 256 * 256);
      if (rows > kLongChunkRowsMax) fits = false;
      else plan[i] = {uint32_t(rows), uint32_t((uint64_t(window) + rows - 1) / rows)};
    }
    if (fits) {
      if (rounds > 1) {
        // an incremental plan: every ring takes the smallest ring chunk - pass B's
        // column-split workgroups stream chunk_rows rows whatever the ring's width, so the
        // steady refresh waits for the longest chunk, not the widest ring
        uint32_t rmin = plan[0].first;
        for (const auto& p : plan) rmin = std::min(rmin, p.first);
        for (auto& p : plan) p = {rmin, uint32_t((uint64_t(window) + rmin - 1) / rmin)};
      }
      return plan;
    }
  }
  throw std::logic_error("long_window_chunk_plan: no plan found");
}

void LongWindowSet::plan_chunks() {
  int cus = 256;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device_);
  std::vector<uint32_t> widths;
  for (const auto& r : rings_) widths.push_back(r.ring->width());
  const auto plan = long_window_chunk_plan(window_, widths, cus, chunk_rows_, plan_rounds_);
  max_chunks_ = 1;
  cand_cap_ = 1;
  pass_wgs_ = 0;
  bcand_keys_ = 0;
  for (size_t i = 0; i < rings_.size(); ++i) {
    auto& r = rings_[i];
    r.chunk_rows = plan[i].first;
    r.nchunks = plan[i].second;
    r.qcap = lw_qcap(r.chunk_rows);
    r.bstride = uint64_t(r.nchunks) * kBrkQ * r.qcap;
    r.boff = bcand_keys_;
    bcand_keys_ += r.bstride * widths[i];
    max_chunks_ = std::max(max_chunks_, r.nchunks);
    cand_cap_ = std::max(cand_cap_, r.nchunks * r.chunk_rows);
    pass_wgs_ += r.nchunks * ((widths[i] + kSegCols - 1) / kSegCols);
  }
}

template <int PASS>
void launch_pass(int prefetch, dim3 grid, size_t lds, hipStream_t stream, const LwArgs& a) {
  if (prefetch == 1) hipLaunchKernelGGL((lw_pass<PASS, 1>), grid, dim3(NT), lds, stream, a);
  else if (prefetch == 2) hipLaunchKernelGGL((lw_pass<PASS, 2>), grid, dim3(NT), lds, stream, a);
  else hipLaunchKernelGGL((lw_pass<PASS, 0>), grid, dim3(NT), lds, stream, a);
}

LwArgs LongWindowSet::make_args(float* out, int mode) const {
  LwArgs a{};
  for (size_t i = 0; i < rings_.size(); ++i) {
    const auto& r = rings_[i];
    a.rings[i] = LwRing{r.dev, r.ring->width(), r.first_series, r.chunk_rows, r.nchunks, r.qcap, 0u, r.boff, r.bstride};
  }
  a.num_rings = uint32_t(rings_.size());
  a.num_segs = 0;
  uint32_t wg0 = 0;
  for (uint32_t i = 0; i < a.num_rings; ++i)
    for (uint32_t c0 = 0; c0 < rings_[i].ring->width(); c0 += kSegCols) {
      a.segs[a.num_segs++] = LwSeg{i, c0, std::min(kSegCols, rings_[i].ring->width() - c0), wg0};
      wg0 += rings_[i].nchunks;
    }
  a.num_series = nseries_;
  a.mask = window_ - 1;
  a.max_chunks = max_chunks_;
  a.params = static_cast<const LwParams*>(params_);
  a.part = static_cast<LwPartial*>(part_);
  a.hist0 = hist0_;
  a.histk = histk_;
  a.sel = static_cast<LwSel*>(sel_);
  a.dig0 = dig0_;
  a.out = out;
  a.wave_priv = uint32_t(wave_priv_);
  const BrkMode& m = bm_[mode];
  a.brk_on = brk_now_ ? 1u : 0u;
  a.brk = static_cast<LwBrk*>(m.brk);
  a.brk_used = static_cast<LwBrk*>(m.brk_used);
  a.hflags = m.hflags_dev;
  a.bpart = static_cast<LwBrkPart*>(m.bpart);
  a.bcand = m.bcand;
  a.incr = incr_now_ ? 1u : 0u;
  a.work = work_dev_;
  a.nwork = 0;
  a.bchg = m.bchg_dev;
  a.report = m.report_dev;
  a.brk_cnt = m.brk_cnt;
  a.brk_target = brk_target_;
  a.dbg = dbg_;
  // candidate compaction (pass 2 -> pass 3), its own slabs
  a.compact = compact_ ? 1u : 0u;
  a.cand = compact_ ? cand_ : nullptr;
  a.cand_n = compact_ ? cand_n_ : nullptr;
  a.cand_cap = cand_cap_;
  return a;
}

size_t LongWindowSet::lds_bytes(int pass) const {
  uint32_t maxw = 0;  // series per segment
  for (const auto& r : rings_) maxw = std::max(maxw, std::min(kSegCols, r.ring->width()));
  if (pass == 0)  // one 10-bit copy, 4 per-wave 8-bit copies, or 8 per-half-wave ones (+16 words each)
    return std::max<size_t>(size_t(maxw) * (kB0 / 2), wave_priv_ == 2 ? 8 * (size_t(maxw) * 128 + 16) : 0) *
           sizeof(uint32_t);
  return size_t(maxw) * kLongRanks * 128 * sizeof(uint32_t);
}

void LongWindowSet::check_args(const LwArgs& a) const {
  // the slabs pass B and pass 2 write must exist before any kernel indexes them
  if (a.compact && (a.cand == nullptr || a.cand_n == nullptr || cand_cap_ < window_))
    throw std::logic_error("long window: compaction buffers missing");
  if (a.brk_on && (a.bcand == nullptr || a.bpart == nullptr || a.brk == nullptr || a.brk_used == nullptr))
    throw std::logic_error("long window: bracket buffers missing");
}

// The radix chain (passes 0-3 with their scans); series scan B resolved are skipped.
void LongWindowSet::enqueue_chain(hipStream_t stream, const LwArgs& a) {
  const size_t lds0 = lds_bytes(0), ldsk = lds_bytes(1);
  const dim3 pass_grid(pass_wgs_), scan_grid(nseries_);
  launch_pass<0>(prefetch_, pass_grid, lds0, stream, a);
  hipLaunchKernelGGL(lw_scan<0>, scan_grid, dim3(NT), 0, stream, a);
  launch_pass<1>(prefetch_, pass_grid, ldsk, stream, a);
  hipLaunchKernelGGL(lw_scan<1>, scan_grid, dim3(NT), 0, stream, a);
  launch_pass<2>(prefetch_, pass_grid, ldsk, stream, a);
  hipLaunchKernelGGL(lw_scan<2>, scan_grid, dim3(NT), 0, stream, a);
  if (a.compact) hipLaunchKernelGGL(lw_pass_cand, dim3(a.max_chunks, nseries_), dim3(NT), 0, stream, a);
  else launch_pass<3>(prefetch_, pass_grid, ldsk, stream, a);
  hipLaunchKernelGGL(lw_scan<3>, scan_grid, dim3(NT), 0, stream, a);
  st_.kernel_launches += 8;
}

void LongWindowSet::enqueue_passes(hipStream_t stream, float* out) {
  const LwArgs a = make_args(out, 0);
  check_args(a);
  if (a.brk_on) {  // bracket mode: pass B + scan B, then the radix chain for what they left
    hipLaunchKernelGGL(lw_pass_brk, dim3(pass_wgs_), dim3(NT), 0, stream, a);
    hipLaunchKernelGGL(lw_scan_brk, dim3(nseries_, kBrkQ), dim3(NT), 0, stream, a);
    st_.kernel_launches += 2;
  }
  enqueue_chain(stream, a);
  check(hipGetLastError(), "long-window launch");
}

void LongWindowSet::stage(hipStream_t stream, float p0, float p1, float p2) {
  if (!part_) allocate_work();
  if (compact_ && !cand_) {  // pass 2's candidate slabs: one key per window sample at most
    const size_t chunks = max_chunks_;
    check(hipMalloc(reinterpret_cast<void**>(&cand_), size_t(nseries_) * cand_cap_ * sizeof(uint32_t)), "hipMalloc cand");
    check(hipMalloc(reinterpret_cast<void**>(&cand_n_), size_t(nseries_) * chunks * sizeof(uint32_t)), "hipMalloc cand_n");
    check(hipMemsetAsync(cand_n_, 0, size_t(nseries_) * chunks * sizeof(uint32_t), stream), "hipMemsetAsync");
  }
  const uint64_t W = window_;
  LwParams P{};
  // a small refresh - every ring pinned (device-visible), no lost rows, few rows in all -
  // stages through lw_ingest (flush_stage) instead of DMA copies
  ingest_segs_.clear();
  ingest_pending_ = host_params_dev_ != nullptr && work_host_dev_ != nullptr;
  {
    uint64_t floats = 0;
    for (const auto& r : rings_) {
      const uint64_t h = r.ring->head();
      const uint64_t lo = std::max<uint64_t>(r.copied, h > W ? h - W : 0);
      if (!r.host_dev || h - lo > r.ring->capacity()) ingest_pending_ = false;
      floats += (h - lo) * r.ring->width();
    }
    if (floats * sizeof(float) > kIngestMaxBytes) ingest_pending_ = false;
  }
  for (size_t i = 0; i < rings_.size(); ++i) {
    auto& r = rings_[i];
    const SeriesRing& ring = *r.ring;
    const uint32_t width = ring.width();
    const uint64_t cap = ring.capacity();
    const uint64_t h = ring.head();
    uint64_t lo = std::max<uint64_t>(r.copied, h > W ? h - W : 0);  // older rows leave the window anyway
    if (h - lo > cap) {
      // the host ring overwrote rows [lo, h - cap) before this refresh: NaN in the window
      const uint64_t lost_end = h - cap;
      st_.rows_lost += lost_end - lo;
      while (lo < lost_end) {
        const uint64_t seg_end = std::min<uint64_t>(lost_end, (lo / W + 1) * W);
        check(hipMemsetAsync(r.dev + (lo & (W - 1)) * width, 0xFF, size_t(seg_end - lo) * width * sizeof(float), stream),
              "hipMemsetAsync");
        lo = seg_end;
      }
    }
    // copy [lo, h) in segments that cross neither the device wrap (multiple of W) nor
    // the host wrap (multiple of cap): both powers of two, so split at the smaller
    const uint64_t m = std::min<uint64_t>(W, cap);
    while (lo < h) {
      const uint64_t seg_end = std::min<uint64_t>(h, (lo / m + 1) * m);
      const size_t bytes = size_t(seg_end - lo) * width * sizeof(float);
      if (ingest_pending_) {
        ingest_segs_.push_back({uint64_t(i), lo, seg_end - lo});
      } else {
        check(hipMemcpyAsync(r.dev + (lo & (W - 1)) * width, ring.rows() + (lo & (cap - 1)) * width, bytes,
                             hipMemcpyHostToDevice, stream),
              "hipMemcpyAsync");
        ++st_.memcpy_calls;
      }
      st_.rows_copied += seg_end - lo;
      st_.bytes_copied += bytes;
      lo = seg_end;
    }
    r.copied = h;
    P.head[i] = h;
    P.prev_head[i] = r.last_head;  // pass 0 predicts the varying key bits from what entered since
    r.last_head = h;
    P.n[i] = uint32_t(std::min<uint64_t>(h, W));
  }
  P.pct[0] = p0;
  P.pct[1] = p1;
  P.pct[2] = p2;
  P.seq = ++seq_;
  // parameter block: pinned staging slot (reused only once its copy has executed)
  const uint32_t slot = slot_++ % kSlots;
  cur_slot_ = slot;
  check(hipEventSynchronize(slot_done_[slot]), "hipEventSynchronize");
  LwParams* hp = static_cast<LwParams*>(host_params_) + slot;
  std::memcpy(hp, &P, sizeof P);
  if (ingest_pending_) return;  // lw_ingest copies the block (flush_stage)
  check(hipMemcpyAsync(params_, hp, sizeof P, hipMemcpyHostToDevice, stream), "hipMemcpyAsync params");
  // (the slot's event is recorded by the caller, after the work list that shares it)
}

void LongWindowSet::flush_stage(hipStream_t stream, uint32_t nwork, int copy_brk_mode) {
  if (!ingest_pending_) return;
  ingest_pending_ = false;
  LwIngest in{};
  in.hp = static_cast<const LwParams*>(host_params_dev_) + cur_slot_;
  in.dp = static_cast<LwParams*>(params_);
  in.hwork = work_host_dev_ + size_t(cur_slot_) * pass_wgs_;
  in.dwork = work_dev_;
  in.nwork = nwork;
  for (const auto& sg : ingest_segs_) {
    const auto& r = rings_[sg[0]];
    const uint32_t width = r.ring->width();
    const uint64_t cap = r.ring->capacity();
    LwIngestSeg& g = in.seg[in.nseg++];
    g.src = r.host_dev + (sg[1] & (cap - 1)) * width;
    g.dst = r.dev + (sg[1] & (uint64_t(window_) - 1)) * width;
    g.floats = uint32_t(sg[2] * width);
  }
  if (copy_brk_mode >= 0) {  // the fused pass B's brackets (its first workgroup cannot copy them)
    in.bsrc = static_cast<const uint32_t*>(bm_[copy_brk_mode].brk);
    in.bdst = static_cast<uint32_t*>(bm_[copy_brk_mode].brk_used);
    in.bwords = uint32_t(nseries_ * sizeof(LwBrk) / sizeof(uint32_t));
  }
  hipLaunchKernelGGL(lw_ingest, dim3(1 + in.nseg + (in.bwords ? 1 : 0)), dim3(NT), 0, stream, in);
  check(hipGetLastError(), "long-window ingest launch");
  ++st_.ingest_launches;
}

// Incremental pass B's work list for bracket state `mode`: per segment, every chunk when
// one of its series' brackets changed since the segment's last pass B (or it never had
// one), else only the chunks the rows that entered since then landed in (physical chunks,
// long_window.hip pass_chunk). Segments with no series that wants brackets: none. Needs
// the mode's previous refresh complete (its flags final): the caller synchronised on it.
std::vector<uint32_t> LongWindowSet::work_list(int mode) {
  BrkMode& m = bm_[mode];
  std::vector<uint32_t> work;
  const uint64_t W = window_;
  uint32_t g = 0;
  for (size_t i = 0; i < rings_.size(); ++i) {
    const auto& r = rings_[i];
    const uint32_t width = r.ring->width();
    const uint64_t h = r.copied;
    for (uint32_t c0 = 0; c0 < width; c0 += kSegCols, ++g) {
      const uint32_t ncols = std::min(kSegCols, width - c0);
      bool want = false, full = m.seg_head[g] == kNever || h < m.seg_head[g] || h - m.seg_head[g] >= W;
      for (uint32_t col = 0; col < ncols; ++col) {
        const uint32_t s = r.first_series + c0 + col;
        want = want || m.hflags[s] != 0;
        full = full || m.bchg[s] != 0;
      }
      if (!want) {  // pass B does not look at this segment: its counts go stale
        m.seg_head[g] = kNever;
        continue;
      }
      if (full) {
        for (uint32_t c = 0; c < r.nchunks; ++c) work.push_back((g << 20) | c);
      } else if (h > m.seg_head[g]) {
        // slots [lo, hi) of the device ring, possibly wrapping
        const uint64_t lo = m.seg_head[g] & (W - 1), n = h - m.seg_head[g];
        const uint32_t c_lo = uint32_t(lo / r.chunk_rows), c_hi = uint32_t(((lo + n - 1) & (W - 1)) / r.chunk_rows);
        if (lo + n <= W) {
          for (uint32_t c = c_lo; c <= c_hi; ++c) work.push_back((g << 20) | c);
        } else {
          for (uint32_t c = c_lo; c < r.nchunks; ++c) work.push_back((g << 20) | c);
          for (uint32_t c = 0; c <= c_hi && c < c_lo; ++c) work.push_back((g << 20) | c);
        }
      }
      m.seg_head[g] = h;
    }
  }
  for (uint32_t s = 0; s < nseries_; ++s) m.bchg[s] = 0;  // consumed (the kernels set them again)
  return work;
}

// Incremental pass B's grid: the chunks rows landed in (work_list) uploaded through the
// parameter slot's pinned staging; a short list is split by column (one workgroup per
// (chunk, series): the same counts and sums, spread over more CUs). Nothing changed at all:
// one workgroup still runs - the grid's first copies the brackets scan B decides with
// (lw_pass_body) - on a chunk whose counts it rewrites unchanged. The whole grid (no list)
// when every chunk changed.
uint32_t LongWindowSet::upload_work(hipStream_t stream, LwArgs& a, int mode, uint32_t slot, bool fuse) {
  std::vector<uint32_t> work = work_list(mode);
  st_.passb_chunks += work.size();
  a.colsplit = 0;
  a.nfused = 0;
  if (!work.empty() && work.size() >= pass_wgs_) {  // every chunk: the flat grid
    flush_stage(stream, 0);
    return pass_wgs_;
  }
  // fused pass B (staged by lw_ingest): the segments with at most kFuseChunks changed chunks
  // are streamed by scan B's own workgroups (lw_scan_brk_fused); a segment with more (its
  // brackets moved: every chunk) keeps pass B. The list: pass B's entries, then the fused
  const bool fused = fuse && ingest_pending_;
  std::vector<uint32_t> fl;
  if (fused) {
    std::vector<uint32_t> per(a.num_segs, 0);
    for (uint32_t e : work) ++per[e >> 20];
    std::vector<uint32_t> rest;
    for (uint32_t e : work) (per[e >> 20] <= kFuseChunks ? fl : rest).push_back(e);
    work.swap(rest);
  }
  if (work.empty() && !fused) work.push_back(0u);  // pass B's first workgroup copies brk -> brk_used
  if (!work.empty()) {
    // columns per segment, in segment order (as make_args lays the segments out)
    std::vector<uint32_t> ncols;
    for (const auto& r : rings_)
      for (uint32_t c0 = 0; c0 < r.ring->width(); c0 += kSegCols)
        ncols.push_back(std::min(kSegCols, r.ring->width() - c0));
    size_t split_n = 0;
    for (uint32_t e : work) split_n += ncols[e >> 20];
    if (split_n + fl.size() <= pass_wgs_ && split_n <= kSplitMax) {
      std::vector<uint32_t> sw;
      sw.reserve(split_n);
      for (uint32_t e : work)
        for (uint32_t col = 0; col < ncols[e >> 20]; ++col)
          sw.push_back(((e >> 20) << 23) | (col << 20) | (e & 0xFFFFFu));
      work.swap(sw);
      a.colsplit = 1;
    }
  }
  const size_t nall = work.size() + fl.size();  // <= pass_wgs_ (the slot's and the device list's size)
  uint32_t* wh = work_host_ + size_t(slot) * pass_wgs_;
  if (!work.empty()) std::memcpy(wh, work.data(), work.size() * sizeof(uint32_t));
  if (!fl.empty()) std::memcpy(wh + work.size(), fl.data(), fl.size() * sizeof(uint32_t));
  a.nwork = uint32_t(work.size());
  a.fwork = work_dev_ + work.size();
  a.nfused = uint32_t(fl.size());
  if (fused) {
    flush_stage(stream, uint32_t(nall), mode);  // rows, parameters, both lists and brk -> brk_used
    ++st_.fused_refreshes;
    std::vector<bool> seen(a.num_segs, false);
    for (uint32_t e : fl)
      if (!seen[e >> 20]) {
        seen[e >> 20] = true;
        ++st_.fused_segments;
      }
  } else if (ingest_pending_) {
    flush_stage(stream, a.nwork);  // rows, parameters and this list in one kernel
  } else {
    check(hipMemcpyAsync(work_dev_, wh, work.size() * sizeof(uint32_t), hipMemcpyHostToDevice, stream),
          "hipMemcpyAsync work");
  }
  return a.nwork;
}

// Wait for the report word of refresh `seq` (lw_brk_finish); returns the series the radix
// chain still has to resolve. Bounded: a device that never gets there is an error.
uint32_t LongWindowSet::wait_report(int mode, uint32_t seq, double timeout_s, uint32_t* maxmid,
                                   const std::function<bool()>* abandon) {
  volatile unsigned long long* w = bm_[mode].report;
  const auto t0 = std::chrono::steady_clock::now();
  const auto t_end = t0 + std::chrono::duration<double>(timeout_s);
  auto t_poll = t0 + std::chrono::milliseconds(20);
  SpinBackoff wait;  // tagged.h: spin, then sleep-poll (node mode waits for its peers here)
  for (;;) {
    const unsigned long long v = *w;
    if (uint32_t(v & 0xFFFFFFu) == (seq & 0xFFFFFFu)) {  // seq mod 2^24: the previous refresh's differs
      if (maxmid) *maxmid = uint32_t(v >> 48);
      return uint32_t(v >> 24) & 0xFFFFFFu;
    }
    if (wait.pause()) {
      const auto now = std::chrono::steady_clock::now();
      if (now > t_end)
        throw std::runtime_error("long window: the bracket report of refresh " + std::to_string(seq) +
                                 " never arrived (device hung or a collective waits for a lost rank)");
      if (abandon && *abandon && now >= t_poll) {
        t_poll = now + std::chrono::milliseconds(20);
        if ((*abandon)())
          throw std::runtime_error("long window: node refresh " + std::to_string(seq) +
                                   " abandoned (the node moved on to a newer epoch)");
      }
    }
  }
}

// Incremental bracket refresh (local): pass B over the work list, scan B, the report; the
// host waits for it and launches the radix chain only when some series needs it.
void LongWindowSet::refresh_incremental(hipStream_t stream, float* out) {
  BrkMode& m = bm_[0];
  check(hipEventSynchronize(m.done), "hipEventSynchronize");  // the previous refresh's flags are final
  bool any = false;
  for (uint32_t i = 0; i < nseries_ && !any; ++i) any = m.hflags[i] != 0;
  brk_now_ = any;
  incr_now_ = true;
  LwArgs a = make_args(out, 0);
  check_args(a);
  uint32_t left = nseries_;
  if (brk_now_) {
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    ++st_.bracket_refreshes;
    const uint32_t slot = cur_slot_;
    const uint64_t fused0 = st_.fused_refreshes;
    const uint32_t grid = upload_work(stream, a, 0, slot, fuse_);
    if (grid) {  // pass B for the segments it streams (all of them unless fused)
      hipLaunchKernelGGL(lw_pass_brk, dim3(grid), dim3(NT), 0, stream, a);
      ++st_.kernel_launches;
    }
    if (st_.fused_refreshes != fused0) {  // scan B streams the short segments' chunks itself
      hipLaunchKernelGGL(lw_scan_brk_fused, dim3(nseries_, kBrkQ), dim3(NT), 0, stream, a);  // + the report
      if (!grid) ++st_.single_kernel_refreshes;
    } else {
      hipLaunchKernelGGL(lw_scan_brk, dim3(nseries_, kBrkQ), dim3(NT), 0, stream, a);  // + the report
    }
    ++st_.kernel_launches;
    check(hipEventRecord(slot_done_[slot], stream), "hipEventRecord");
    check(hipGetLastError(), "long-window launch");
    const auto t1 = clk::now();
    left = wait_report(0, seq_, 60.0);
    st_.host_enqueue_ns += uint64_t(std::chrono::duration_cast<std::chrono::nanoseconds>(t1 - t0).count());
    st_.host_wait_ns += uint64_t(std::chrono::duration_cast<std::chrono::nanoseconds>(clk::now() - t1).count());
  } else {
    flush_stage(stream, 0);
    check(hipEventRecord(slot_done_[cur_slot_], stream), "hipEventRecord");
  }
  if (left) {
    ++st_.chain_refreshes;
    enqueue_chain(stream, a);
    check(hipGetLastError(), "long-window launch");
  }
  check(hipEventRecord(m.done, stream), "hipEventRecord");
}

void LongWindowSet::refresh(float* out, void* stream_ptr, float p0, float p1, float p2) {
  auto stream = static_cast<hipStream_t>(stream_ptr);
  Guard g(device_);
  const auto t0 = std::chrono::steady_clock::now();
  stage(stream, p0, p1, p2);
  st_.host_stage_ns += uint64_t(std::chrono::duration_cast<std::chrono::nanoseconds>(
                                    std::chrono::steady_clock::now() - t0).count());
  if (brackets_ && incremental_ && !use_graph_) {
    refresh_incremental(stream, out);
  } else {
    flush_stage(stream, 0);
    check(hipEventRecord(slot_done_[cur_slot_], stream), "hipEventRecord");
    incr_now_ = false;
    // bracket mode this refresh: pass B + scan B only when some series wants brackets (the
    // kernels' hint in host memory, from an earlier refresh: a stale hint costs time,
    // never exactness - the radix chain resolves whatever scan B does not). A graph keeps
    // the launches it captured.
    bool any = false;
    for (uint32_t i = 0; i < nseries_ && !any; ++i) any = static_cast<volatile uint32_t*>(bm_[0].hflags)[i] != 0;
    brk_now_ = brackets_ && (use_graph_ || any);
    if (brk_now_) ++st_.bracket_refreshes;
    if (use_graph_) {
      if (!exec_ || graph_out_ != out || exec_stale_) {
        exec_stale_ = false;
        if (exec_) {
          check(hipGraphExecDestroy(exec_), "hipGraphExecDestroy");
          check(hipGraphDestroy(graph_), "hipGraphDestroy");
          exec_ = nullptr;
          graph_ = nullptr;
        }
        check(hipStreamBeginCapture(cap_stream_, hipStreamCaptureModeThreadLocal), "hipStreamBeginCapture");
        const uint64_t launches = st_.kernel_launches;
        enqueue_passes(cap_stream_, out);
        st_.kernel_launches = launches;  // replayed as one graph launch
        check(hipStreamEndCapture(cap_stream_, &graph_), "hipStreamEndCapture");
        check(hipGraphInstantiate(&exec_, graph_, nullptr, nullptr, 0), "hipGraphInstantiate");
        graph_out_ = out;
      }
      check(hipGraphLaunch(exec_, stream), "hipGraphLaunch");
      ++st_.graph_launches;
    } else {
      enqueue_passes(stream, out);
    }
    // every series' chunk counts are stale for the incremental mode after this
    for (auto& h : bm_[0].seg_head) h = kNever;
  }
  check(hipEventRecord(last_done_, stream), "hipEventRecord");
  ++st_.refreshes;
}

uint32_t long_window_node_cap(uint32_t maxmid, uint32_t nranks) { return lw_node_cap_next(maxmid, nranks); }

void LongWindowSet::allocate_node(int nranks) {
  const size_t S = nseries_;
  if (node_ranks_ == nranks) return;
  for (void* p : {pred_local_, pred_all_, agg_local_, agg_all_, nbl_, nball_})
    if (p) (void)hipFree(p);
  check(hipMalloc(&pred_local_, S * sizeof(LwPred)), "hipMalloc");
  check(hipMalloc(&pred_all_, size_t(nranks) * S * sizeof(LwPred)), "hipMalloc");
  check(hipMalloc(&agg_local_, S * sizeof(LwPartial)), "hipMalloc");
  check(hipMalloc(&agg_all_, size_t(nranks) * S * sizeof(LwPartial)), "hipMalloc");
  check(hipMalloc(&nbl_, lw_node_block(uint32_t(S), kNodeCap)), "hipMalloc");
  check(hipMalloc(&nball_, size_t(nranks) * lw_node_block(uint32_t(S), kNodeCap)), "hipMalloc");
  node_cap_ = kNodeCap;  // until a bracket refresh has measured the node's kept keys
  if (node_events_.empty()) {
    node_events_.resize(2 * kNodeCollectives);
    for (auto& e : node_events_) check(hipEventCreate(&e), "hipEventCreate");
  }
  node_ranks_ = nranks;
}

void LongWindowSet::reset_node() {
  Guard g(device_);
  if (last_done_) check(hipEventSynchronize(last_done_), "hipEventSynchronize");
  BrkMode& m = bm_[1];
  if (m.brk) {
    check(hipEventSynchronize(m.done), "hipEventSynchronize");
    const size_t S = nseries_;
    check(hipMemset(m.brk, 0, S * sizeof(LwBrk)), "hipMemset");  // no brackets: the radix chain first
    check(hipMemset(m.brk_used, 0, S * sizeof(LwBrk)), "hipMemset");
    check(hipMemset(m.bpart, 0, S * max_chunks_ * sizeof(LwBrkPart)), "hipMemset");
    check(hipMemset(m.brk_cnt, 0, 2 * sizeof(uint32_t)), "hipMemset");
    check(hipDeviceSynchronize(), "hipDeviceSynchronize");  // done before any stream reads them
    std::memset(m.hflags, 0, S * sizeof(uint32_t));
    std::memset(m.bchg, 0, S * sizeof(uint32_t));
    m.seg_head.assign(m.seg_head.size(), kNever);
  }
  node_cap_ = kNodeCap;
  node_maxmid_ = 0;
  ++st_.node_resets;
}

void LongWindowSet::set_node_brackets(uint32_t s, const std::vector<uint32_t>& lo, const std::vector<uint32_t>& hi) {
  if (s >= nseries_ || lo.size() != size_t(kBrkQ) || hi.size() != size_t(kBrkQ))
    throw std::invalid_argument("set_node_brackets: a series index and 3 lo / 3 hi keys");
  for (int q = 0; q < kBrkQ; ++q)
    if (lo[q] > hi[q]) throw std::invalid_argument("set_node_brackets: lo > hi");
  Guard g(device_);
  allocate_mode(1);
  if (last_done_) check(hipEventSynchronize(last_done_), "hipEventSynchronize");
  BrkMode& m = bm_[1];
  check(hipEventSynchronize(m.done), "hipEventSynchronize");
  LwBrk b{};
  auto* dev = static_cast<LwBrk*>(m.brk) + s;
  check(hipMemcpy(&b, dev, sizeof(LwBrk), hipMemcpyDeviceToHost), "hipMemcpy bracket");
  for (int q = 0; q < kBrkQ; ++q) {
    b.lo[q] = lo[q];
    b.hi[q] = hi[q];
    b.nounion[q] = 0u;
    b.dsave[q] = 0u;
  }
  b.valid = 1u;
  check(hipMemcpy(dev, &b, sizeof(LwBrk), hipMemcpyHostToDevice), "hipMemcpy bracket");
  m.hflags[s] = 1u;
  m.bchg[s] = 1u;  // every chunk of the series is counted again
}

void LongWindowSet::refresh_node(float* out, void* stream_ptr, float p0, float p1, float p2, RcclComm* comm,
                                 bool timing, double timeout_s, const std::function<bool()>& abandon) {
  auto stream = static_cast<hipStream_t>(stream_ptr);
  Guard g(device_);
  const int nranks = comm ? comm->nranks() : 1;
  stage(stream, p0, p1, p2);
  allocate_node(nranks);
  allocate_mode(1);  // the node's own brackets: never the local ones
  BrkMode& m = bm_[1];
  // Node bracket mode: the node's brackets are the same on every rank (every kernel that
  // writes them reads only all-gathered data), and so are the flags they leave: once the
  // previous node refresh completed, every rank takes the same branch below - the same
  // collectives in the same order
  const bool use_brk = brackets_ && incremental_ && !use_graph_ && nranks <= int(kNodeBrkRanks);
  bool any = false;
  if (use_brk) {
    check(hipEventSynchronize(m.done), "hipEventSynchronize");
    for (uint32_t i = 0; i < nseries_ && !any; ++i) any = m.hflags[i] != 0;
  }
  brk_now_ = use_brk && any;
  incr_now_ = use_brk;
  LwArgs a = make_args(out, 1);
  a.node_n = uint32_t(nranks);
  a.pred_local = static_cast<LwPred*>(pred_local_);
  a.pred_all = static_cast<const LwPred*>(comm ? pred_all_ : pred_local_);
  a.agg_local = static_cast<LwPartial*>(agg_local_);
  a.agg_all = static_cast<const LwPartial*>(comm ? agg_all_ : agg_local_);
  a.node_brk = 1;
  a.nbl = static_cast<unsigned char*>(nbl_);
  a.nball = static_cast<const unsigned char*>(comm ? nball_ : nbl_);
  a.node_cap = node_cap_;
  check_args(a);
  const size_t S = nseries_;
  const size_t lds0 = lds_bytes(0), ldsk = lds_bytes(1);
  const dim3 pass_grid(pass_wgs_), scan_grid(nseries_);
  timed_ = timing && comm;
  for (auto& f : node_timed_) f = false;
  // the node's collectives on this stream, between the kernels that consume them
  auto collective = [&](int k, auto&& fn) {
    if (!comm) return;
    if (timed_) check(hipEventRecord(node_events_[2 * k], stream), "hipEventRecord");
    fn();
    if (timed_) {
      check(hipEventRecord(node_events_[2 * k + 1], stream), "hipEventRecord");
      node_timed_[k] = true;
    }
  };
  uint32_t left = nseries_;
  if (brk_now_) {
    ++st_.bracket_refreshes;
    const uint32_t slot = cur_slot_;
    const uint32_t grid = upload_work(stream, a, 1, slot, false);
    if (grid) {
      hipLaunchKernelGGL(lw_pass_brk, dim3(grid), dim3(NT), 0, stream, a);
      ++st_.kernel_launches;
    }
    hipLaunchKernelGGL(lw_node_brk_local, scan_grid, dim3(NT), 0, stream, a);
    // ONE collective per hit: every rank's counts, partials and kept keys
    const size_t block = lw_node_block(uint32_t(S), node_cap_);
    st_.node_record_bytes += block;
    collective(0, [&] { comm->all_gather_bytes(nbl_, nball_, block, stream); });
    hipLaunchKernelGGL(lw_node_brk_select, dim3(nseries_, kBrkQ), dim3(NT), 0, stream, a);  // + the report
    check(hipEventRecord(slot_done_[slot], stream), "hipEventRecord");
    st_.kernel_launches += 2;
    check(hipGetLastError(), "long-window node launch");
    uint32_t maxmid = 0;
    left = wait_report(1, seq_, timeout_s, &maxmid, &abandon);
    node_maxmid_ = maxmid;
    // every rank read the same records: the same next cap, the same collective size
    node_cap_ = lw_node_cap_next(maxmid, uint32_t(nranks));
  } else {
    flush_stage(stream, 0);
    check(hipEventRecord(slot_done_[cur_slot_], stream), "hipEventRecord");
    if (!use_brk)
      for (auto& h : m.seg_head) h = kNever;
  }
  if (left) {  // the node radix chain for the series the brackets left (all of them without)
    ++st_.chain_refreshes;
    hipLaunchKernelGGL(lw_node_predict, dim3(a.num_segs), dim3(NT), 0, stream, a);
    collective(1, [&] { comm->all_gather_bytes(pred_local_, pred_all_, S * sizeof(LwPred), stream); });
    launch_pass<0>(prefetch_, pass_grid, lds0, stream, a);
    hipLaunchKernelGGL(lw_node_partials, scan_grid, dim3(NT), 0, stream, a);
    collective(2, [&] {
      comm->all_gather_bytes(agg_local_, agg_all_, S * sizeof(LwPartial), stream);
      comm->all_reduce_sum_u32(hist0_, hist0_, S * kB0, stream);
    });
    hipLaunchKernelGGL(lw_scan<0>, scan_grid, dim3(NT), 0, stream, a);
    launch_pass<1>(prefetch_, pass_grid, ldsk, stream, a);
    collective(3, [&] { comm->all_reduce_sum_u32(histk_, histk_, S * kLongRanks * 256, stream); });
    hipLaunchKernelGGL(lw_scan<1>, scan_grid, dim3(NT), 0, stream, a);
    launch_pass<2>(prefetch_, pass_grid, ldsk, stream, a);
    collective(4, [&] { comm->all_reduce_sum_u32(histk_, histk_, S * kLongRanks * 256, stream); });
    hipLaunchKernelGGL(lw_scan<2>, scan_grid, dim3(NT), 0, stream, a);
    if (a.compact) hipLaunchKernelGGL(lw_pass_cand, dim3(a.max_chunks, nseries_), dim3(NT), 0, stream, a);
    else launch_pass<3>(prefetch_, pass_grid, ldsk, stream, a);
    collective(5, [&] { comm->all_reduce_sum_u32(histk_, histk_, S * kLongRanks * 256, stream); });
    hipLaunchKernelGGL(lw_scan<3>, scan_grid, dim3(NT), 0, stream, a);
    check(hipGetLastError(), "long-window node launch");
    st_.kernel_launches += 10;
  }
  check(hipEventRecord(m.done, stream), "hipEventRecord");
  check(hipEventRecord(last_done_, stream), "hipEventRecord");
  ++st_.node_refreshes;
  ++st_.refreshes;
}

void LongWindowSet::set_phase_clocks(bool on) {
  Guard g(device_);
  if (on && !dbg_) {
    check(hipMalloc(reinterpret_cast<void**>(&dbg_), std::max<size_t>(1, nseries_) * kBrkQ * 8 * sizeof(unsigned long long)),
          "hipMalloc");
    check(hipMemset(dbg_, 0, std::max<size_t>(1, nseries_) * kBrkQ * 8 * sizeof(unsigned long long)), "hipMemset");
  } else if (!on && dbg_) {
    if (last_done_) check(hipEventSynchronize(last_done_), "hipEventSynchronize");
    (void)hipFree(dbg_);
    dbg_ = nullptr;
  }
}

std::vector<unsigned long long> LongWindowSet::phase_clocks() const {
  std::vector<unsigned long long> v;
  if (!dbg_) return v;
  Guard g(device_);
  v.resize(size_t(nseries_) * kBrkQ * 8);
  if (last_done_) check(hipEventSynchronize(last_done_), "hipEventSynchronize");
  check(hipMemcpy(v.data(), dbg_, v.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost), "hipMemcpy clocks");
  return v;
}

std::vector<std::array<uint32_t, 3>> LongWindowSet::bracket_stats(int mode) const {
  std::vector<std::array<uint32_t, 3>> v;
  for (const auto& x : bracket_state(mode)) v.push_back({x[16], x[17], x[15]});
  return v;
}

// Every series' bracket record of a mode (0 local, 1 node) as its 22 words: lo[3], hi[3],
// delta[3] (float bits), cin[3], valid, hit, refreshes, hits, nounion[3] - reordered
// below to [lo 0-2, hi 3-5, delta 6-8, cin 9-11, valid 12, nounion 13, -, hit 15,
// refreshes 16, hits 17]
std::vector<std::array<uint32_t, 18>> LongWindowSet::bracket_state(int mode) const {
  std::vector<std::array<uint32_t, 18>> v;
  if (mode < 0 || mode > 1 || !bm_[mode].brk) return v;
  Guard g(device_);
  std::vector<LwBrk> b(nseries_);
  if (last_done_) check(hipEventSynchronize(last_done_), "hipEventSynchronize");
  check(hipMemcpy(b.data(), bm_[mode].brk, nseries_ * sizeof(LwBrk), hipMemcpyDeviceToHost), "hipMemcpy brackets");
  for (const auto& x : b) {
    std::array<uint32_t, 18> r{};
    for (int q = 0; q < kBrkQ; ++q) {
      r[q] = x.lo[q];
      r[3 + q] = x.hi[q];
      r[6 + q] = x.delta[q];
      r[9 + q] = x.cin[q];
      r[13] |= x.nounion[q] << q;
    }
    r[12] = x.valid;
    r[15] = x.hit;
    r[16] = x.refreshes;
    r[17] = x.hits;
    v.push_back(r);
  }
  return v;
}

std::vector<double> LongWindowSet::node_collective_us() const {
  std::vector<double> us;
  if (!timed_) return us;
  for (int k = 0; k < kNodeCollectives; ++k) {
    if (!node_timed_[k]) {  // not run this refresh (bracket hit: no chain; no brackets: no record gather)
      us.push_back(std::nan(""));
      continue;
    }
    float ms = 0.f;
    check(hipEventSynchronize(node_events_[2 * k + 1]), "hipEventSynchronize");
    check(hipEventElapsedTime(&ms, node_events_[2 * k], node_events_[2 * k + 1]), "hipEventElapsedTime");
    us.push_back(double(ms) * 1e3);
  }
  return us;
}

}  // namespace rocmdash
