// Long-window statistics: windows far beyond what one workgroup's LDS holds.
//
// DeviceWindowSet (device_window.h) keeps a window of <= 32768 samples per series
// sorted in LDS / HBM and updates it incrementally. A window of hours of 100 Hz
// telemetry (2^20 .. 2^26 samples per series) lives only in HBM here - the host ring
// is just the staging queue in front of it - and every refresh recomputes the exact
// statistics over the whole window with a multi-workgroup radix select:
//
//   pass 0  every workgroup streams a chunk of rows of one ring segment (<= 8 of its
//           series at once, coalesced 16-B loads), reduces min / max / sum / count / varying bits
//           into a per-chunk partial and histograms a 10-bit digit of each sample's
//           order-preserving key in LDS - the top 10 of the bits predicted to vary
//           (previous window's min / max + the rows that entered) - then merges the
//           non-zero bins into a global per-series histogram with one atomic each;
//   scan 0  one workgroup per series reduces the partials in a fixed order
//           (deterministic mean), turns the percentile positions into 6 ranks
//           (lo / hi of each percentile, numpy's linear interpolation) and finds, per
//           rank, the digit and the residual rank inside it;
//   pass k, scan k (k = 1..3): the same for the next <= 8 bits, counting only samples
//           whose higher bits match the rank's prefix, down to the lowest bit that
//           varies; a series with no bits left skips the pass (a ring with none left
//           skips the whole stream). The prefix (+ the bits no sample varies in) IS
//           the key of the sample at that rank. The last scan writes [S, 8].
//
// Bracket mode (default; long_window.hip "Bracket mode"): in front of the chain, pass B
// streams the window once, counting per percentile the samples below and inside a
// bracket around the previous refresh's percentile key and keeping the keys inside; scan
// B selects the percentiles among those keys when every one fell inside its bracket, and
// the radix chain then skips the series. A series whose bracket missed takes the chain in
// the same refresh, so every refresh is exact either way.
//
// 8 kernels per refresh (10 with pass B + scan B) with fixed arguments (the per-refresh ring heads travel through a
// small device parameter block), so a refresh is <= 3 hipMemcpyAsync of new rows + 1
// parameter copy + 8 launches - or, optionally, 1 launch of a hipGraph that captured them.
// All buffers a pass writes are consumed and re-zeroed by the next scan: no memsets
// per refresh.
//
// Reference counterpart: none (SURVEY.md §5 "Long-context": scale W beyond LDS with a
// multi-pass histogram / radix select).
#pragma once

#include <hip/hip_runtime.h>

#include <array>
#include <cstdint>
#include <functional>
#include <memory>
#include <stdexcept>
#include <utility>
#include <vector>

#include "ring.h"

namespace rocmdash {

constexpr uint32_t kLongMinWindow = 1u << 10;
constexpr uint32_t kLongMaxWindow = 1u << 26;
constexpr int kLongMaxRings = 4;
constexpr int kLongMaxWidth = 16;  // series per ring
constexpr int kLongRanks = 6;      // lo / hi sorted positions of the 3 percentiles
// rows one pass workgroup streams: its LDS histograms hold 16-bit bins, so <= 65535
// samples of one series per workgroup. Large chunks: each workgroup merges its histograms
// into the global ones ONCE - the merge's device atomics, not the stream, bounded the
// passes at 4096-row chunks. kLongChunkRows: the largest uniform (power-of-two) chunk a
// caller may ask for; kLongChunkRowsMax: the largest balanced chunk (plan_chunks)
constexpr uint32_t kLongChunkRows = 32768;
constexpr uint32_t kLongChunkRowsMax = 65280;

struct LongWindowStats {
  uint64_t refreshes = 0;
  uint64_t rows_copied = 0;
  uint64_t bytes_copied = 0;
  uint64_t memcpy_calls = 0;
  uint64_t rows_lost = 0;      // rows the host ring overwrote before a refresh copied them
  uint64_t graph_launches = 0;
  uint64_t kernel_launches = 0;  // without the graph: 8 per refresh, 10 in bracket mode (10 per node refresh)
  uint64_t ingest_launches = 0;  // lw_ingest: a small refresh's staging as one kernel
  uint64_t node_refreshes = 0;
  uint64_t bracket_refreshes = 0;  // refreshes that launched pass B + scan B
  uint64_t passb_chunks = 0;       // incremental mode: (segment, chunk) workgroups pass B streamed
  uint64_t chain_refreshes = 0;    // incremental mode: refreshes that also needed the radix chain
  uint64_t fused_refreshes = 0;    // bracket refreshes whose scan B streamed chunks itself (lw_scan_brk_fused)
  uint64_t single_kernel_refreshes = 0;  // ... of them with no pass B kernel at all
  uint64_t fused_segments = 0;     // segments streamed by scan B's workgroups, summed
  uint64_t node_record_bytes = 0;  // node bracket mode: bytes of this rank's all-gathered records, summed
  uint64_t node_resets = 0;        // reset_node() calls (one per membership epoch)
  // host time of refresh(), summed: staging (rows, parameters), a bracket refresh's
  // work list + launches (incl. lw_ingest), and its wait for scan B's report
  uint64_t host_stage_ns = 0;
  uint64_t host_enqueue_ns = 0;
  uint64_t host_wait_ns = 0;
};

class RcclComm;
struct LwArgs;

// The passes' chunking of rings of `widths` series over `window` rows on a device with
// `cus` compute units: per ring (rows per workgroup, workgroups per 8-series segment).
// chunk_rows != 0: that many rows for every ring; 0: balanced by bytes (long_window.hip),
// the grid `rounds` rounds of the chip's workgroup slots (smaller chunks: an incremental
// pass B streams fewer rows per changed chunk).
std::vector<std::pair<uint32_t, uint32_t>> long_window_chunk_plan(uint32_t window, const std::vector<uint32_t>& widths,
                                                                  int cus, uint32_t chunk_rows, uint32_t rounds = 1);

// node bracket mode: the next refresh's record cap (kept keys per rank and bracket) from
// this refresh's node-wide most kept keys - lw_node_cap_next (rocmdash.runtime.lw_brackets
// node_cap_next mirrors it)
uint32_t long_window_node_cap(uint32_t maxmid, uint32_t nranks);

class LongWindowSet {
 public:
  // chunk_rows: rows one workgroup streams per pass, the same for every ring (power of two
  // in [256, 32768]); 0 = planned per ring at the first refresh so that every workgroup
  // streams about the same bytes (plan_chunks; tools/bench_long_window.py A/Bs it)
  // use_graph: capture the 8 kernels once and replay them with one call; measured 2-7 %
  // slower on the GPU than direct launches (bench_long_window_v3.json), so off by default
  LongWindowSet(uint32_t window, int device, bool use_graph = false, uint32_t chunk_rows = 0);
  ~LongWindowSet();
  LongWindowSet(const LongWindowSet&) = delete;
  LongWindowSet& operator=(const LongWindowSet&) = delete;

  // Register a ring (width <= 16); returns the index of its first series.
  uint32_t add_ring(std::shared_ptr<SeriesRing> ring);
  uint32_t num_series() const { return nseries_; }
  uint32_t window() const { return window_; }
  // the first ring's rows per workgroup (0 until the first refresh when planned)
  uint32_t chunk_rows() const { return rings_.empty() ? chunk_rows_ : rings_[0].chunk_rows; }
  // per ring: (rows per workgroup, workgroups per segment); empty until the first refresh
  std::vector<std::pair<uint32_t, uint32_t>> chunk_plan() const {
    std::vector<std::pair<uint32_t, uint32_t>> v;
    if (part_)
      for (const auto& r : rings_) v.emplace_back(r.chunk_rows, r.nchunks);
    return v;
  }
  // pass 0: per-wave LDS histogram copies when the digit is 8 bits (A/B switch; default
  // from ROCMDASH_LW_WAVE_PRIVATE). Takes effect at the next refresh (graphs re-capture).
  void set_wave_private(bool on) { set_wave_private_level(on ? 1 : 0); }
  bool wave_private() const { return wave_priv_ != 0; }
  // 0: one shared copy, 1: a copy per wave, 2: a copy per half wave (A/B)
  void set_wave_private_level(int level) {
    if (level < 0 || level > 2) throw std::invalid_argument("wave-private level 0, 1 or 2");
    if (level != wave_priv_) exec_stale_ = true;
    wave_priv_ = level;
  }
  int wave_private_level() const { return wave_priv_; }
  // candidate compaction: pass 2 keeps the keys it counts, pass 3 reads only those (the
  // 4th stream of the window becomes a read of the ~few % of samples in the ranks'
  // 16-bit buckets). Costs S x W x 4 B of HBM, allocated at the next refresh. Default
  // from ROCMDASH_LW_COMPACT.
  void set_compact(bool on) {
    if (on != compact_) exec_stale_ = true;
    compact_ = on;
  }
  bool compact() const { return compact_; }
  // rounds of the chip's workgroup slots a planned full pass takes (chunk_rows 0): more
  // rounds, smaller chunks - the steady incremental refresh re-streams fewer rows, a full
  // pass (a miss, a bracket move) pays a little more per-workgroup overhead. Before the
  // first refresh only. Default from ROCMDASH_LW_PLAN_ROUNDS.
  void set_plan_rounds(uint32_t n) {
    if (n < 1 || n > 16) throw std::invalid_argument("plan rounds in [1, 16]");
    if (part_) throw std::logic_error("plan rounds: set before the first refresh");
    plan_rounds_ = n;
  }
  uint32_t plan_rounds() const { return plan_rounds_; }
  // samples a local bracket aims to hold (256..2048): fewer kept keys make scan B's gather
  // and select cheaper, a narrower bracket re-centres more often. Default from
  // ROCMDASH_LW_BRK_TARGET.
  void set_brk_target(uint32_t n) {
    if (n < 256 || n > 2048) throw std::invalid_argument("bracket target in [256, 2048]");
    brk_target_ = n;
  }
  uint32_t brk_target() const { return brk_target_; }
  // diagnostics: scan B's workgroups record shader-clock timestamps at their phases
  // (counts + partials, gather, select, outputs); phase_clocks() returns the last local
  // refresh's [S][3][8] raw clocks (0: not reached)
  void set_phase_clocks(bool on);
  std::vector<unsigned long long> phase_clocks() const;
  // 0: the passes load a thread's rows, then count them; 1: the next iteration's rows are
  // loaded while this one's are counted (two register buffers); 2: the same with half the
  // rows per buffer (A/B; default from ROCMDASH_LW_PREFETCH)
  void set_prefetch(int mode) {
    if (mode < 0 || mode > 2) throw std::invalid_argument("prefetch mode 0, 1 or 2");
    if (mode != prefetch_) exec_stale_ = true;
    prefetch_ = mode;
  }
  int prefetch() const { return prefetch_; }
  // bracket mode (default from ROCMDASH_LW_BRACKETS, on): one streaming pass counts the
  // samples below / inside brackets around the previous refresh's percentiles and keeps
  // the keys inside; when every percentile falls inside its bracket, a select over those
  // keys replaces the radix passes 0-3 (which still run, exact, for any series it misses)
  void set_brackets(bool on) {
    if (on != brackets_) exec_stale_ = true;
    brackets_ = on;
  }
  bool brackets() const { return brackets_; }
  // incremental bracket mode (default from ROCMDASH_LW_INCREMENTAL, on; with brackets and
  // without the graph): chunks are the device ring's slots, a bracket stays put while the
  // percentiles sit well inside it, so pass B streams only the chunks the new rows landed in
  // and reuses every other chunk's counts, partials and kept keys; the host waits for scan
  // B's report and launches the radix chain only for a refresh some series needs it for
  void set_incremental(bool on) { incremental_ = on; }
  bool incremental() const { return incremental_; }
  // a short incremental work list: scan B streams the changed chunks itself (one kernel)
  void set_fused_passb(bool on) { fuse_ = on; }
  bool fused_passb() const { return fuse_; }
  // per series: (refreshes scan B saw brackets, of them resolved by brackets, the last
  // refresh's outcome); synchronises the device
  std::vector<std::array<uint32_t, 3>> bracket_stats(int mode = 0) const;
  std::vector<std::array<uint32_t, 18>> bracket_state(int mode = 0) const;
  // Enqueue new-row copies + the statistics passes on `stream`; out = device [S][8].
  void refresh(float* out, void* stream, float p0, float p1, float p2);
  // Node-wide statistics over the union of every rank's window (collective: every rank
  // of `comm` calls it with the same series layout): the same passes as refresh(), with
  // the ranks' pass-0 predictions and partials all-gathered and every digit histogram
  // all-reduced (ncclAllReduce sum, exact) on `stream` between the kernels, so every
  // rank selects the same digits and holds the same node statistics (out [S][8], last =
  // NaN). comm == nullptr: a one-rank node (no collectives). timing: HIP events around
  // the 5 collective steps (node_collective_us()).
  //
  // Node bracket mode (with brackets + incremental, <= 8 ranks): pass B with the node's
  // brackets (the same on every rank), then ONE all-gather of every rank's bracket counts,
  // partials and kept keys; every rank selects the node percentiles among the union of
  // the kept keys. The host waits for the outcome (bounded by timeout_s) and runs the node
  // radix chain only for the series the brackets missed.
  //
  // abandon (optional): polled (~every 20 ms) while the host waits for the node brackets'
  // outcome; true = the node moved on to a newer membership epoch, the wait ends at once
  // with an error instead of after timeout_s (a peer lost mid-refresh must
  // cost its peers no collective timeout once the supervisor re-formed the node).
  void refresh_node(float* out, void* stream, float p0, float p1, float p2, RcclComm* comm, bool timing = false,
                    double timeout_s = 60.0, const std::function<bool()>& abandon = nullptr);
  // Forget the node's bracket state: brackets, flags, chunk heads and the records' key
  // cap. Every rank of a NEW membership epoch calls it before its first node refresh, so
  // that every member takes the same branch (a restarted rank starts with no brackets;
  // the survivors kept theirs - different collectives on one communicator otherwise) and
  // sizes its records alike. Waits for this set's last refresh.
  void reset_node();
  // Test hook (tools/node_long_window_check.py --full-cap): series s's NODE brackets become
  // [lo[q], hi[q]] (order-preserving keys), valid, and its chunks' counts stale - the next
  // refresh_node takes bracket mode with them. Lets a check put exactly kNodeCap keys per
  // rank into a bracket (the union at scan B's LDS bound). Waits for the last refresh.
  void set_node_brackets(uint32_t s, const std::vector<uint32_t>& lo, const std::vector<uint32_t>& hi);
  uint32_t node_cap() const { return node_cap_; }            // the next node refresh's record key cap
  uint32_t node_last_maxmid() const { return node_maxmid_; }  // the last bracket node refresh's most kept keys
  // µs of the last timed node refresh's collective steps (synchronises their events; NaN
  // for a step that did not run): [bracket records all-gather, pred all-gather, partials
  // all-gather + pass-0 all-reduce, pass 1, pass 2, pass 3]
  std::vector<double> node_collective_us() const;
  LongWindowStats stats() const { return st_; }
  static constexpr int kNodeCollectives = 6;

 private:
  struct RingState {
    std::shared_ptr<SeriesRing> ring;
    float* dev = nullptr;  // [W][width]: row r at slot r & (W - 1)
    uint64_t copied = 0;   // rows [0, copied) are on the device (or were lost)
    uint64_t last_head = 0;  // the ring head at the previous refresh
    uint32_t first_series = 0;
    uint32_t chunk_rows = 0;  // plan_chunks
    uint32_t nchunks = 0;
    uint32_t qcap = 0;      // pass B's kept keys per (chunk, bracket)
    uint64_t boff = 0;      // the ring's first series' kept-key slots
    uint64_t bstride = 0;   // kept-key slots per series
    const float* host_dev = nullptr;  // the pinned host ring's rows as the device sees them (ingest)
  };
  void allocate_work();
  void plan_chunks();  // per-ring chunk rows and the flat pass grid
  void allocate_node(int nranks);
  void stage(hipStream_t stream, float p0, float p1, float p2);  // new-row copies + parameter block
  // a small refresh's staging as ONE kernel (lw_ingest: new rows from the pinned host rings,
  // the parameter block, the work list) instead of 2-4 DMA copies; a no-op when stage()
  // used the copies. Called before the first kernel that reads them.
  void flush_stage(hipStream_t stream, uint32_t nwork, int copy_brk_mode = -1);
  bool ingest_pending_ = false;
  static constexpr size_t kIngestMaxBytes = 256 << 10;  // larger stagings (a fill) take the DMA copies
  std::vector<std::array<uint64_t, 3>> ingest_segs_;  // (ring, first row, rows) to ingest
  void* host_params_dev_ = nullptr;  // host_params_ as the device sees it
  uint32_t* work_host_dev_ = nullptr;  // work_host_ as the device sees it
  LwArgs make_args(float* out, int mode) const;
  size_t lds_bytes(int pass) const;
  void check_args(const LwArgs& a) const;
  void enqueue_chain(hipStream_t stream, const LwArgs& a);
  void enqueue_passes(hipStream_t stream, float* out);
  void allocate_mode(int mode);
  std::vector<uint32_t> work_list(int mode);
  uint32_t upload_work(hipStream_t stream, LwArgs& a, int mode, uint32_t slot, bool fuse = false);
  static constexpr uint32_t kFuseChunks = 4;  // fused pass B: at most this many changed chunks per segment
  static constexpr size_t kSplitMax = 2048;  // column-split pass B: at most this many workgroups
  uint32_t wait_report(int mode, uint32_t seq, double timeout_s, uint32_t* maxmid = nullptr,
                       const std::function<bool()>* abandon = nullptr);
  void refresh_incremental(hipStream_t stream, float* out);

  uint32_t window_;
  int device_;
  bool use_graph_;
  uint32_t chunk_rows_;  // the caller's uniform chunk (0: planned per ring)
  // 3: 8192-row chunks for every ring at 2^24 - the steady refresh (100 new rows)
  // re-streams 1-2 of them in ~61 / 49 us (continuous / telemetry) instead of 106 / 87 us
  // with one round's byte-balanced chunks; a full radix chain (a miss) costs more
  // (profiles/r05/lw_rounds/, lw_incr_v4/)
  uint32_t plan_rounds_ = 3;
  uint32_t brk_target_ = 2048;
  unsigned long long* dbg_ = nullptr;
  uint32_t nseries_ = 0;
  uint32_t max_chunks_ = 0;  // the most chunks of any ring (partials / slab-count stride)
  uint32_t cand_cap_ = 0;    // candidate slots per series (>= every ring's chunks x rows)
  uint32_t pass_wgs_ = 0;    // the flat pass grid: every segment's chunks
  std::vector<RingState> rings_;
  // work buffers (allocated at the first refresh, when every ring is known)
  void* params_ = nullptr;      // device LwParams
  void* part_ = nullptr;        // per (series, chunk) partials
  uint32_t* hist0_ = nullptr;   // [S][1024]
  uint32_t* dig0_ = nullptr;    // [S][3]: pass 0's digit shift, reference key, width
  uint32_t* histk_ = nullptr;   // [S][6][256]
  void* sel_ = nullptr;         // per series: ranks, residuals, prefixes
  void* host_params_ = nullptr;  // pinned staging slots for the parameter copy
  std::vector<hipEvent_t> slot_done_;
  uint32_t slot_ = 0;
  hipStream_t cap_stream_ = nullptr;
  hipGraph_t graph_ = nullptr;
  hipGraphExec_t exec_ = nullptr;
  float* graph_out_ = nullptr;
  // node mode (refresh_node): predictions and partials, this rank's and all-gathered
  void* pred_local_ = nullptr;
  void* pred_all_ = nullptr;
  void* agg_local_ = nullptr;
  void* agg_all_ = nullptr;
  void* nbl_ = nullptr;    // node bracket mode: this rank's records [S]
  void* nball_ = nullptr;  // ... every rank's [nranks][S]
  uint32_t node_maxmid_ = 0;
  uint32_t node_cap_ = 1024;  // the records' key cap this refresh (lw_node_cap_next; kNodeCap until measured)
  bool node_timed_[6] = {false, false, false, false, false, false};
  int node_ranks_ = 0;
  int wave_priv_ = 1;
  // compaction's slabs cost S x W x 4 B; with brackets the radix chain runs only on a miss,
  // so it is off by default
  bool compact_ = false;
  int prefetch_ = 0;  // modes 1 and 2 measured 2-7 % slower (profiles/r04/lw_ab/)
  bool brackets_ = true;
  bool incremental_ = true;
  bool fuse_ = true;
  static constexpr uint64_t kNever = ~0ull;
  // one bracket state per kind of refresh: 0 = local (refresh), 1 = node (refresh_node)
  struct BrkMode {
    void* brk = nullptr;       // [S] brackets (persist across refreshes)
    void* brk_used = nullptr;  // [S] the brackets the current refresh's pass B used
    void* bpart = nullptr;     // [S][chunks] pass B's per-chunk bracket counts
    uint32_t* bcand = nullptr;  // pass B's kept keys (LwRing::boff / bstride)
    uint32_t* hflags = nullptr;  // [S] pinned host: series that want brackets (kernels write)
    uint32_t* hflags_dev = nullptr;
    uint32_t* bchg = nullptr;  // [S] pinned host: the series' brackets moved (kernels write, host clears)
    uint32_t* bchg_dev = nullptr;
    unsigned long long* report = nullptr;  // pinned host: {seq, series left to the chain, node's most kept keys}
    unsigned long long* report_dev = nullptr;
    uint32_t* brk_cnt = nullptr;  // device: scan B's finished workgroups (lw_brk_finish)
    std::vector<uint64_t> seg_head;  // per segment: the ring head at its last pass B (kNever: none)
    hipEvent_t done = nullptr;       // the mode's last refresh
  };
  BrkMode bm_[2];
  bool brk_now_ = false;   // this refresh launches pass B + scan B
  bool incr_now_ = false;  // ... incrementally
  uint64_t bcand_keys_ = 0;  // kept-key slots of one mode (every series)
  uint32_t* work_dev_ = nullptr;   // incremental pass B's work list
  uint32_t* work_host_ = nullptr;  // pinned staging, one list per parameter slot
  uint32_t seq_ = 0;               // refreshes staged (the report word's number)
  uint32_t cur_slot_ = 0;          // the parameter slot of the refresh being enqueued
  hipEvent_t last_done_ = nullptr;  // after this set's last enqueued kernel (destructor waits on it)
  uint32_t* cand_ = nullptr;    // [S][W] candidate keys (compaction)
  uint32_t* cand_n_ = nullptr;  // [S][chunks] keys per pass-2 workgroup slab
  bool exec_stale_ = false;  // the captured graph predates a setting change
  std::vector<hipEvent_t> node_events_;
  bool timed_ = false;
  LongWindowStats st_;
};

}  // namespace rocmdash
