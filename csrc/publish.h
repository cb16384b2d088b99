// Host publication of a device tensor + completion flag (publish.hip).
#pragma once

#include <cstdint>

namespace rocmdash {

class HostPublisher {
 public:
  // tagged: n > 0 publications go out as {value, seq} words into a mapped buffer of the
  // publisher's own and wait() copies them to `dst` (no acknowledgement wait + flag in
  // the kernel); false: copy to `dst` + completion flag.
  explicit HostPublisher(int device, bool tagged = true);
  ~HostPublisher();
  HostPublisher(const HostPublisher&) = delete;
  HostPublisher& operator=(const HostPublisher&) = delete;

  // Enqueue on `stream`: copy n floats from `src` (device) to `dst` (pinned host memory,
  // device-accessible; n = 0 copies nothing), then publish the returned sequence number.
  // Throws std::logic_error while another thread is inside wait().
  uint32_t publish(const float* src, float* dst, uint32_t n, void* stream);
  // Spin until `seq` is published (at most timeout_us; tagged: and copy the values to
  // that publication's `dst` - host memory); false on timeout, for a publication nothing
  // will ever signal (an older tagged one), or when a newer publication overwrote a
  // tagged one before it was read out (counted in superseded(); no mixed copy).
  bool wait(uint32_t seq, double timeout_us) const;
  uint64_t superseded() const { return superseded_; }

 private:
  bool ensure_words(uint32_t n, void* stream);
  int device_;
  bool tagged_;
  uint64_t* words_host_ = nullptr;  // tagged words: mapped pinned host
  uint64_t* words_dev_ = nullptr;
  uint32_t words_cap_ = 0;
  void* words_stream_ = nullptr;    // stream of the last tagged publication
  uint32_t tag_seq_ = 0;            // the last publication, if tagged
  float* tag_dst_ = nullptr;
  uint32_t tag_n_ = 0;
  uint32_t flag_seq_ = 0;           // the last flag publication
  uint32_t* host_ = nullptr;  // mapped pinned host flag
  uint32_t* dev_ = nullptr;   // its device address
  uint32_t seq_ = 0;
  mutable int waiting_ = 0;   // waits in progress (tagged.h WaitGuard)
  mutable uint64_t superseded_ = 0;
};

}  // namespace rocmdash
