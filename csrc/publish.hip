// Publishing a gathered node tensor to the host without a stream synchronisation.
//
// After the refresh's RCCL all-gather (N > 1), rank 0 needs the [N, rows, 8] node
// tensor on the host, and every rank needs to know the refresh is done. A D2H copy +
// hipStreamSynchronize waits for the copy engine and then the stream's completion
// signal. Instead ONE small kernel, enqueued behind the all-gather, copies the tensor
// into pinned host memory (rank 0; the other ranks copy nothing) and then publishes a
// sequence number to mapped host memory, which the host spins on - the N > 1 form of
// the stats kernel's own completion flag (device_window.cpp).
#include "publish.h"

#include <hip/hip_runtime.h>

#include <stdexcept>
#include <string>

#include "device_window.h"

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
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(flag, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

void check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

}  // namespace

HostPublisher::HostPublisher(int device) : device_(device) {
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
}

uint32_t HostPublisher::publish(const float* src, float* dst, uint32_t n, void* stream) {
  if (n && (src == nullptr || dst == nullptr)) throw std::invalid_argument("publish: null buffer");
  if (++seq_ == 0) ++seq_;  // 0 never published
  int prev = 0;
  check(hipGetDevice(&prev), "hipGetDevice");
  if (prev != device_) check(hipSetDevice(device_), "hipSetDevice");
  hipLaunchKernelGGL(publish_kernel, dim3(1), dim3(kThreads), 0, static_cast<hipStream_t>(stream), src, dst, n, dev_,
                     seq_);
  const hipError_t e = hipGetLastError();
  if (prev != device_) (void)hipSetDevice(prev);
  check(e, "publish launch");
  return seq_;
}

bool HostPublisher::wait(uint32_t seq, double timeout_us) const { return spin_for_flag(host_, seq, timeout_us); }

}  // namespace rocmdash
