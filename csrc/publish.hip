// Publishing a gathered node tensor to the host without a stream synchronisation.
//
// After the refresh's RCCL all-gather (N > 1), rank 0 needs the [N, rows, 8] node
// tensor on the host, and every rank needs to know the refresh is done. A D2H copy +
// hipStreamSynchronize waits for the copy engine and then the stream's completion
// signal. Instead ONE small kernel, enqueued behind the all-gather, copies the tensor
// into pinned host memory (rank 0; the other ranks copy nothing) and then publishes a
// sequence number to mapped host memory, which the host spins on - the N > 1 form of
// the stats kernel's own completion flag (device_window.cpp). Rank 0's copy goes out as
// tagged {value, seq} words by default (publish_tagged_kernel): the host knows each
// value's publication from the word itself and copies the values out.
#include "publish.h"

#include <hip/hip_runtime.h>

#include <cstring>
#include <stdexcept>
#include <string>

#include "device_window.h"
#include "tagged.h"

namespace rocmdash {
namespace {

constexpr int kThreads = 256;

__global__ __launch_bounds__(kThreads) void publish_kernel(const float* __restrict__ src, float* __restrict__ dst,
                                                           uint32_t n, uint32_t* flag, uint32_t seq) {
  // system-scope stores: written through to host memory whatever its mapping
  for (uint32_t i = threadIdx.x; i < n; i += kThreads)
    __hip_atomic_store(dst + i, src[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  // every wave waits for its stores' acknowledgements (nothing is left dirty in L2 to
  // write back), the block agrees, then one lane publishes with a posted store
  // behind them: the host that sees `seq` sees the whole tensor (window_stats.hip's
  // completion flag, same argument)
  if (n) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  if (threadIdx.x == 0) __hip_atomic_store(flag, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Tagged form: every value leaves as ONE aligned 8-byte write-through store {float bits,
// seq << 32} into the publisher's mapped buffer; the host copies the values out once
// every word carries `seq` (HostPublisher::wait) - no acknowledgement wait, barrier or
// flag store behind the copy (the stats kernel's tagged outputs, window_stats.h).
__global__ __launch_bounds__(kThreads) void publish_tagged_kernel(const float* __restrict__ src, uint64_t* words,
                                                                  uint32_t n, uint32_t seq) {
  const uint64_t tag = uint64_t(seq) << 32;
  for (uint32_t i = threadIdx.x; i < n; i += kThreads)
    __hip_atomic_store(words + i, tag | __builtin_bit_cast(uint32_t, src[i]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

void check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

}  // namespace

HostPublisher::HostPublisher(int device, bool tagged) : device_(device), tagged_(tagged) {
  int prev = 0;
  check(hipGetDevice(&prev), "hipGetDevice");
  check(hipSetDevice(device_), "hipSetDevice");
  void* h = nullptr;
  hipError_t e = hipHostMalloc(&h, 64, hipHostMallocMapped | hipHostMallocCoherent);
  void* d = nullptr;
  if (e == hipSuccess) e = hipHostGetDevicePointer(&d, h, 0);
  (void)hipSetDevice(prev);
  if (e != hipSuccess) {
    if (h) (void)hipHostFree(h);
    throw std::runtime_error(std::string("HostPublisher: mapped host flag: ") + hipGetErrorString(e));
  }
  host_ = static_cast<uint32_t*>(h);
  dev_ = static_cast<uint32_t*>(d);
  __atomic_store_n(host_, 0u, __ATOMIC_RELEASE);
}

HostPublisher::~HostPublisher() {
  if (host_) (void)hipHostFree(host_);
  if (words_host_) (void)hipHostFree(words_host_);
}

bool HostPublisher::ensure_words(uint32_t n, void* stream) {
  if (words_host_ != nullptr && words_cap_ >= n) return true;
  if (words_host_) {  // grown: no kernel may still write the old buffer - the publications
    // that wrote it ran on words_stream_ (and the one before on `stream`, in its order)
    (void)hipStreamSynchronize(static_cast<hipStream_t>(words_stream_));
    if (stream != words_stream_) (void)hipStreamSynchronize(static_cast<hipStream_t>(stream));
    (void)hipHostFree(words_host_);
  }
  words_host_ = words_dev_ = nullptr;
  words_cap_ = 0;
  void* h = nullptr;
  void* d = nullptr;
  if (hipHostMalloc(&h, size_t(n) * sizeof(uint64_t), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) {
    (void)hipGetLastError();
    (void)hipHostFree(h);
    return false;
  }
  std::memset(h, 0, size_t(n) * sizeof(uint64_t));  // tag 0: never published
  words_host_ = static_cast<uint64_t*>(h);
  words_dev_ = static_cast<uint64_t*>(d);
  words_cap_ = n;
  return true;
}

uint32_t HostPublisher::publish(const float* src, float* dst, uint32_t n, void* stream) {
  if (n && (src == nullptr || dst == nullptr)) throw std::invalid_argument("publish: null buffer");
  if (wait_in_progress(&waiting_)) throw std::logic_error("publish: a wait on the previous publication is in progress");
  if (++seq_ == 0) ++seq_;  // 0 never published
  int prev = 0;
  check(hipGetDevice(&prev), "hipGetDevice");
  if (prev != device_) check(hipSetDevice(device_), "hipSetDevice");
  const bool tagged = tagged_ && n > 0 && ensure_words(n, stream);
  if (tagged) {
    hipLaunchKernelGGL(publish_tagged_kernel, dim3(1), dim3(kThreads), 0, static_cast<hipStream_t>(stream), src,
                       words_dev_, n, seq_);
  } else {
    hipLaunchKernelGGL(publish_kernel, dim3(1), dim3(kThreads), 0, static_cast<hipStream_t>(stream), src, dst, n, dev_,
                       seq_);
  }
  const hipError_t e = hipGetLastError();
  if (prev != device_) (void)hipSetDevice(prev);
  check(e, "publish launch");
  if (tagged) {
    tag_seq_ = seq_;
    tag_dst_ = dst;
    tag_n_ = n;
    words_stream_ = stream;
  } else {
    flag_seq_ = seq_;
  }
  return seq_;
}

bool HostPublisher::wait(uint32_t seq, double timeout_us) const {
  if (seq == 0) return false;
  WaitGuard busy(&waiting_);
  if (seq != tag_seq_) {
    // a flag publication at or after `seq` is what the flag will show; an older tagged
    // publication with none after it is never signalled: do not burn the timeout
    if (flag_seq_ == 0 || int32_t(flag_seq_ - seq) < 0) return false;
    return spin_for_flag(host_, seq, timeout_us);
  }
  const TagScan s = wait_tagged(words_host_, tag_n_, seq, tag_dst_, timeout_us);  // tagged.h
  if (s == TagScan::kSuperseded) ++superseded_;
  return s == TagScan::kDone;
}

}  // namespace rocmdash
