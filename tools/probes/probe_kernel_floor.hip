// Floor of a small latency-bound dispatch on MI355X: what does rocprofv3's kernel
// trace report for kernels shaped like the steady-state window-stats launch (15
// workgroups x 256 threads, one launch per ~80 us refresh) that do (almost) nothing?
//   empty      : no memory access
//   load       : every thread loads 64 B of a 256 KiB buffer the previous launch wrote
//   load_store : + stores the 64 B back (dirty lines at kernel end)
//   load_host  : + 8 floats per workgroup to mapped host memory, store acknowledged
//   *_unc      : the same buffer allocated uncached (hipDeviceMallocUncached)
// Build: hipcc -O3 --offload-arch=gfx950 tools/probes/probe_kernel_floor.hip -o /tmp/floor
// Run:   rocprofv3 --kernel-trace --stats -d DIR -o floor --output-format csv -- /tmp/floor
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <thread>

#define CK(x)                                                                            \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                       \
      return 1;                                                                          \
    }                                                                                    \
  } while (0)

__global__ __launch_bounds__(256) void k_empty(float* out) {
  if (out == nullptr && threadIdx.x == 1023) out[0] = 0.f;  // never taken
}

__global__ __launch_bounds__(256) void k_load(const float* __restrict__ buf, float* out) {
  const float4* p = reinterpret_cast<const float4*>(buf) + (size_t(blockIdx.x) * 256 + threadIdx.x) * 4;
  float s = 0.f;
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    const float4 q = p[v];
    s += q.x + q.y + q.z + q.w;
  }
  if (s == -1.f) out[blockIdx.x] = s;  // keeps the loads
}

template <int Uncached>
__global__ __launch_bounds__(256) void k_load_store(float* __restrict__ buf, float* out) {
  float4* p = reinterpret_cast<float4*>(buf) + (size_t(blockIdx.x) * 256 + threadIdx.x) * 4;
  float4 q[4];
#pragma unroll
  for (int v = 0; v < 4; ++v) q[v] = p[v];
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    q[v].x += 1.f;
    p[v] = q[v];
  }
  if (q[0].y == -1.f) out[blockIdx.x] = 0.f;
}

__global__ __launch_bounds__(256) void k_load_host(const float* __restrict__ buf, float* host) {
  const float4* p = reinterpret_cast<const float4*>(buf) + (size_t(blockIdx.x) * 256 + threadIdx.x) * 4;
  float s = 0.f;
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    const float4 q = p[v];
    s += q.x + q.y + q.z + q.w;
  }
  if (threadIdx.x < 8) {
    host[blockIdx.x * 8 + threadIdx.x] = s;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
}

int main() {
  const int G = 15, iters = 300;
  const size_t bytes = size_t(G) * 256 * 64;
  float *buf = nullptr, *unc = nullptr, *host = nullptr, *hdev = nullptr, *out = nullptr;
  CK(hipMalloc(&buf, bytes));
  CK(hipExtMallocWithFlags(reinterpret_cast<void**>(&unc), bytes, hipDeviceMallocUncached));
  CK(hipMalloc(&out, 4096));
  CK(hipHostMalloc(reinterpret_cast<void**>(&host), 4096, hipHostMallocMapped | hipHostMallocCoherent));
  CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&hdev), host, 0));
  CK(hipMemset(buf, 0, bytes));
  CK(hipMemset(unc, 0, bytes));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  auto pace = [] { std::this_thread::sleep_for(std::chrono::microseconds(60)); };
  for (int it = 0; it < iters; ++it) {
    hipLaunchKernelGGL(k_empty, dim3(G), dim3(256), 0, s, out);
    CK(hipStreamSynchronize(s));
    pace();
    hipLaunchKernelGGL(k_load, dim3(G), dim3(256), 0, s, buf, out);
    CK(hipStreamSynchronize(s));
    pace();
    hipLaunchKernelGGL(k_load_store<0>, dim3(G), dim3(256), 0, s, buf, out);
    CK(hipStreamSynchronize(s));
    pace();
    hipLaunchKernelGGL(k_load_host, dim3(G), dim3(256), 0, s, buf, hdev);
    CK(hipStreamSynchronize(s));
    pace();
  }
  // the uncached buffer: same code, its own kernel name in the trace
  for (int it = 0; it < iters; ++it) {
    hipLaunchKernelGGL(k_load_store<1>, dim3(G), dim3(256), 0, s, unc, out + 512);
    CK(hipStreamSynchronize(s));
    pace();
  }
  std::printf("done: %d iterations per kernel (k_load_store<1>: uncached buffer)\n", iters);
  return 0;
}
