// Host publication of a device tensor + completion flag (publish.hip).
#pragma once

#include <cstdint>

namespace rocmdash {

class HostPublisher {
 public:
  explicit HostPublisher(int device);
  ~HostPublisher();
  HostPublisher(const HostPublisher&) = delete;
  HostPublisher& operator=(const HostPublisher&) = delete;

  // Enqueue on `stream`: copy n floats from `src` (device) to `dst` (pinned host memory,
  // device-accessible; n = 0 copies nothing), then publish the returned sequence number.
  uint32_t publish(const float* src, float* dst, uint32_t n, void* stream);
  // Spin until `seq` is published (at most timeout_us); false on timeout.
  bool wait(uint32_t seq, double timeout_us) const;

 private:
  int device_;
  uint32_t* host_ = nullptr;  // mapped pinned host flag
  uint32_t* dev_ = nullptr;   // its device address
  uint32_t seq_ = 0;
};

}  // namespace rocmdash
