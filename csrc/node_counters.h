// One device-counter process per node.
//
//   ShmPublisher  (the node's counter process, rocmdash/runtime/counterd.py): ONE thread
//                 reads every GPU's counter source at the counter rate and pushes each
//                 GPU's rows into its shared-memory ring (shm_ring.h). The rocprofiler-
//                 sdk counting contexts - and the runtime's completion-polling thread
//                 that comes with them (rocmdash/runtime/threads.py) - exist in this
//                 process only, once per node instead of once per rank.
//   ShmSource     (a rank's counter source): hands the rank's Sampler each row of its
//                 GPU's ring in order, with the row's own read time, without touching
//                 the counter hardware. The rank's sampler runs free (one call per
//                 published row); a call sleeps until the next row is due.
#pragma once

#include <sys/types.h>

#include <atomic>
#include <cstdint>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "shm_ring.h"
#include "sources.h"

namespace rocmdash {

class ShmPublisher {
 public:
  // paths[i] receives sources[i]'s rows; rings of `cap` rows.
  ShmPublisher(const std::vector<std::string>& paths, std::vector<std::shared_ptr<Source>> sources, double hz,
               uint64_t cap = 4096);
  ~ShmPublisher();
  void start();
  void stop();
  // per ring: {samples, failures, mean_read_us, last_read_us}
  std::vector<std::vector<double>> stats() const;
  double hz() const { return hz_; }

 private:
  void loop();
  std::vector<std::shared_ptr<Source>> src_;
  std::vector<ShmRing> rings_;
  std::vector<std::vector<float>> rows_;
  double hz_;
  std::atomic<bool> running_{false};
  std::thread th_;
  mutable std::mutex mu_;
  std::vector<uint64_t> samples_, failures_;
  std::vector<double> total_us_, last_us_;
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
