// Device mirrors of host rings + the per-refresh stats launch.
//
// Each host SeriesRing gets a device ring of 2W rows (W = window): the window plus
// the rows that leave it, which the incremental stats path removes from the resident
// sorted window (window_stats.hip). A refresh
// enqueues, on ONE stream and with no host synchronisation:
//   1. hipMemcpyAsync of the rows produced since the previous refresh (at most two
//      segments per ring: the device ring wraps at multiples of 2W, and the host ring
//      capacity is a multiple of 2W so a segment never crosses a host wrap);
//   2. one window_stats launch covering every series of every ring.
// The head/length of each ring travel as by-value kernel arguments (a snapshot taken
// when the copies are enqueued), so nothing on the host is re-read by the GPU later.
#pragma once

#include <cstdint>
#include <memory>
#include <vector>

#include "ring.h"
#include "window_stats.h"

namespace rocmdash {

void set_pinned_host_rings(bool on);  // hipHostMalloc for rings created afterwards
// Pull mode (default on): pinned rings added afterwards are read by the stats kernel
// directly (no per-refresh hipMemcpyAsync); off = stage new rows with copies.
void set_pull_mode(bool on);
bool pull_enabled();
int hip_device_count();
// Spin (pause loop) until *flag - a mapped host word a kernel publishes sequence numbers
// to - has reached `seq` (modulo 2^32), at most timeout_us. True when seen.
bool spin_for_flag(const uint32_t* flag, uint32_t seq, double timeout_us);
uint64_t hip_device_bdf(int device);  // amd-smi style bdf id of a HIP device

struct WindowSetStats {
  uint64_t refreshes = 0;
  uint64_t rows_copied = 0;
  uint64_t bytes_copied = 0;
  uint64_t memcpy_calls = 0;
  uint64_t launches = 0;
  uint64_t incremental_launches = 0;  // launches predicted to take the incremental path
  uint64_t pulled_series = 0;         // series whose entering rows the kernel read from host
  uint64_t inline_rows = 0;           // entering rows passed by value in the kernel argument
};

class DeviceWindowSet {
 public:
  DeviceWindowSet(uint32_t window, int device);
  ~DeviceWindowSet();
  DeviceWindowSet(const DeviceWindowSet&) = delete;
  DeviceWindowSet& operator=(const DeviceWindowSet&) = delete;

  // Register a ring; returns the index of its first series (columns are consecutive).
  uint32_t add_ring(std::shared_ptr<SeriesRing> ring);
  uint32_t num_series() const { return nseries_; }
  uint32_t window() const { return window_; }
  int device() const { return device_; }

  // How the host learns that a refresh's outputs are in (needs pinned host memory):
  //   kSignalNone   - no signal: synchronise the stream (device outputs the stream goes on
  //                   to use, e.g. the N > 1 gather: no epilogue in the kernel);
  //   kSignalFlag   - the last workgroup publishes the refresh's sequence number to a
  //                   mapped host word after every workgroup's outputs are acknowledged;
  //   kSignalTagged - `out` is HOST memory: the kernel writes {value, seq} words into a
  //                   mapped buffer of this set's own and wait_done() copies the values
  //                   to `out` once every word carries the refresh's tag.
  enum Signal : int { kSignalNone = 0, kSignalFlag = 1, kSignalTagged = 2 };
  // Enqueue delta copies + stats kernel; out points to [num_series][8] (device-accessible,
  // or host memory with kSignalTagged). Returns the refresh's completion sequence number
  // (see wait_done; 0 = no signal).
  uint32_t refresh(float* out, void* stream, float p0, float p1, float p2, int signal = kSignalFlag);
  // Spin until the kernels of refresh `seq` have written their outputs, at most
  // timeout_us (tagged: and copy them to the refresh's `out`). True when seen; false on
  // timeout, without a signal (then synchronise the stream), for an older tagged refresh
  // (never signalled again: returns at once), or when a newer refresh overwrote a tagged
  // one before it was read out (superseded(): no mixed copy is ever returned). Faster
  // than a stream synchronisation: no wait for the end-of-kernel signal. refresh()
  // throws std::logic_error while another thread is inside this wait.
  bool wait_done(uint32_t seq, double timeout_us) const;
  // Forget what was mirrored (next refresh re-copies the whole window).
  void invalidate();
  // Enqueue, after the refresh that produced them, every series' resident sorted window
  // as [num_series][1 + W] floats (count, then ascending samples, +inf padding): the
  // per-rank block of the node-wide window statistics (node_window.h).
  void export_sorted(float* dst, void* stream) const;
  WindowSetStats stats() const { return st_; }
  // Tagged waits that found part of their refresh overwritten by a newer one (they
  // returned false and copied nothing usable: never a mix of two refreshes).
  uint64_t superseded() const { return superseded_; }

 private:
  uint64_t dev_rows() const { return uint64_t(window_) * 2; }  // device ring depth D = 2W
  bool ensure_tags(void* stream);  // the tag buffer holds every series (false: no mapped host memory)

  struct RingState {
    std::shared_ptr<SeriesRing> ring;
    float* dev = nullptr;        // device ring [2W][width]: the window plus the rows leaving it
    const float* host_dev = nullptr;  // device-mapped pinned host ring (pull mode) or nullptr
    float* sorted = nullptr;     // per series: two halves of W floats (resident sorted window)
    SeriesState* state = nullptr;  // per series
    bool state_valid = false;      // host mirror of what the last launch left on device
    uint64_t last_head = 0;
    uint32_t last_n = 0;
    uint32_t cur = 0;              // resident-buffer half the last launch wrote
    uint64_t copied = 0;
    uint32_t first_series = 0;
  };
  uint32_t window_;
  int device_;
  uint32_t nseries_ = 0;
  uint32_t* wg_counter_ = nullptr;      // device: workgroups finished, cumulative mod 2^32
  uint32_t* done_host_ = nullptr;       // mapped pinned host: last completed sequence
  uint32_t* done_dev_ = nullptr;        // its device address
  uint32_t wg_total_ = 0;               // workgroups launched so far (mod 2^32)
  uint32_t seq_ = 0;
  uint64_t* tag_host_ = nullptr;        // tagged outputs: mapped pinned host [tag_cap_][8] words
  uint64_t* tag_dev_ = nullptr;         // their device address
  uint32_t tag_cap_ = 0;                // series the tag buffer holds
  float* tag_dst_ = nullptr;            // host [tag_n_][8] the last tagged refresh's values go to
  uint32_t tag_n_ = 0;
  uint32_t tag_seq_ = 0;                // sequence number of the last tagged refresh
  void* tag_stream_ = nullptr;          // its stream
  uint32_t flag_seq_ = 0;               // sequence number of the last flag refresh
  mutable int waiting_ = 0;             // wait_done() calls in progress (tagged.h WaitGuard)
  mutable uint64_t superseded_ = 0;     // tagged waits that found a newer refresh's words
  std::vector<RingState> rings_;
  WindowSetStats st_;
};

}  // namespace rocmdash
