// One device-counter process per node.
//
//   ShmPublisher  (the node's counter process, rocmdash/runtime/counterd.py): one LANE per
//                 GPU - a thread of its own reading that GPU's counter source at the
//                 counter rate and pushing its rows into the GPU's shared-memory ring
//                 (shm_ring.h), stamping the ring's heartbeat after every read. A read
//                 that blocks (a GPU in reset, a hung firmware call) stops only its own
//                 lane: the node supervisor sees that ring's heartbeat stall while the
//                 others advance (rocmdash/runtime/lanes.py), reports the GPU's counter
//                 source down and later asks for a fresh lane (replace()), which gets a
//                 new source and a new ring file. Lane threads hold only their lane
//                 (shared ownership), so a lane that never returns is left behind on
//                 stop() instead of blocking it. The rocprofiler-sdk counting contexts
//                 - and the runtime's completion-polling thread that comes with them
//                 (rocmdash/runtime/threads.py) - exist in this process only, once per
//                 node instead of once per rank.
//   ShmSource     (a rank's counter source): hands the rank's Sampler each row of its
//                 GPU's ring in order, with the row's own read time, without touching
//                 the counter hardware. The rank's sampler runs free (one call per
//                 published row); a call sleeps until the next row is due.
#pragma once

#include <sys/types.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "shm_ring.h"
#include "sources.h"

namespace rocmdash {

// A source whose reads block forever once `after_s` seconds passed since its first read
// (ROCMDASH_FAULT=ctrhang:<dev>, rocmdash/runtime/counterd.py): the fault a GPU reset
// or a hung firmware call puts on one lane. Unblocks only at process exit.
std::shared_ptr<Source> make_hanging_source(std::shared_ptr<Source> inner, double after_s);

class ShmPublisher {
 public:
  // paths[i] receives sources[i]'s rows; rings of `cap` rows.
  ShmPublisher(const std::vector<std::string>& paths, std::vector<std::shared_ptr<Source>> sources, double hz,
               uint64_t cap = 4096);
  ~ShmPublisher();
  void start();
  // Ask every lane to end, wait up to `grace_s` for them; a lane still blocked in a read
  // is left behind (it owns its state and exits when its read returns).
  void stop(double grace_s = 2.0);
  // Lane i gets a fresh source: the old lane is abandoned (it pushes nothing more, even
  // if its read returns) and a new lane starts with a NEW ring file renamed over the
  // path (readers re-open it on the new inode). Returns the new lane generation.
  int replace(size_t i, std::shared_ptr<Source> src);
  // per ring: {samples, failures, mean_read_us, last_read_us, beat_age_s, lane generation,
  //            in_read_s (how long the lane's current read has been running, 0 if none)}
  std::vector<std::vector<double>> stats() const;
  double hz() const { return hz_; }
  size_t lanes() const { return paths_.size(); }

  struct Lane;

 private:
  std::shared_ptr<Lane> make_lane(size_t i, std::shared_ptr<Source> src, int gen);
  void launch(const std::shared_ptr<Lane>& lane);
  std::vector<std::string> paths_;
  uint64_t cap_;
  double hz_;
  uint64_t gen_;
  std::shared_ptr<std::atomic<bool>> running_;
  std::chrono::steady_clock::time_point epoch_;  // every lane's deadlines are on one grid
  mutable std::mutex mu_;
  std::vector<std::shared_ptr<Lane>> lanes_;
  std::vector<std::shared_ptr<Lane>> left_;  // abandoned lanes (their threads may still run)
};

class ShmSource : public Source {
 public:
  ShmSource(std::string path, double hz, std::string kind = "counter");
  uint32_t width() const override { return width_; }
  std::string kind() const override { return kind_; }
  std::string backend() const override { return backend_; }
  bool sample(float* row) override;
  uint64_t row_time_ns() const override { return row_ts_; }
  std::vector<std::pair<std::string, double>> counts() const override;

 private:
  bool ensure_open();
  std::string path_;
  double hz_;
  std::string kind_, backend_;
  uint32_t width_;
  ShmRing ring_;
  ino_t inode_ = 0;
  uint64_t generation_ = 0;
  uint64_t next_ = 0;  // next row to hand out
  uint64_t row_ts_ = 0;
  uint64_t last_ts_ = 0;
  std::atomic<uint64_t> reopens_{0}, skipped_{0}, torn_{0};
};

}  // namespace rocmdash
