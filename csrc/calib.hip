// Calibration loads for the device-counter series (tests/test_gpu.py, tools/probes):
//   spin      `workgroups` one-wave workgroups that each keep their CU busy for `us`
//             microseconds of wall time and exit. With at most one workgroup per CU the
//             share of busy CUs is known exactly (the CU-active series must report it).
//   gather32  one 32 B read per thread at a hashed 32 B slot of a buffer (random lines:
//             the memory side fills one 128 B L2 line per read), one float per workgroup
//             written back;
//   store64   one 64 B store per thread at a 256 B stride (no two in one line): 64 B
//             write requests of known count.
// The HBM byte series (csrc/counters.cpp) are checked against these in tests/test_gpu.py.
#include <hip/hip_runtime.h>

#include <cstdint>

namespace rocmdash {
namespace {

__global__ __launch_bounds__(64) void spin_kernel(uint64_t ticks, float* sink) {
  // wall_clock64() runs at a constant 100 MHz; every wave leaves after `ticks`
  const uint64_t t0 = wall_clock64();
  float x = float(threadIdx.x);
  while (wall_clock64() - t0 < ticks) {
#pragma unroll 8
    for (int i = 0; i < 64; ++i) x = __builtin_fmaf(x, 0.999f, 1e-3f);
  }
  if (x == -1.f) sink[threadIdx.x] = x;  // never taken; keeps the loop
}

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}

__global__ __launch_bounds__(256) void gather32_kernel(const float4* __restrict__ src, uint64_t slots,
                                                       float* __restrict__ out, uint32_t seed) {
  const uint32_t t = blockIdx.x * 256u + threadIdx.x;
  const uint64_t slot = ((uint64_t(mix32(t ^ seed)) << 32) | mix32(t + seed * 0x9e3779b9U)) % slots;
  const float4 a = src[2 * slot];
  const float4 b = src[2 * slot + 1];
  float v = a.x + a.y + a.z + a.w + b.x + b.y + b.z + b.w;
  for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
  __shared__ float ws[4];
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = ws[0] + ws[1] + ws[2] + ws[3];
}

__global__ __launch_bounds__(256) void store64_kernel(float4* __restrict__ dst, float v) {
  const uint64_t t = blockIdx.x * 256ull + threadIdx.x;
  const float4 x = make_float4(v, v + 1.f, v + 2.f, v + 3.f);
  float4* p = dst + t * 16;  // 256 B apart
  p[0] = x;
  p[1] = x;
  p[2] = x;
  p[3] = x;
}

// 32 B per thread, 256 B apart: the dirty half-sector leaves L2 as one 32 B write request
__global__ __launch_bounds__(256) void store32_kernel(float4* __restrict__ dst, float v) {
  const uint64_t t = blockIdx.x * 256ull + threadIdx.x;
  const float4 x = make_float4(v, v + 1.f, v + 2.f, v + 3.f);
  float4* p = dst + t * 16;
  p[0] = x;
  p[1] = x;
}

}  // namespace

// Shapes are checked here, on the host, before any launch: `src_bytes` / `out_bytes` /
// `dst_bytes` are the sizes of the buffers behind the pointers.
int launch_gather32(const void* src, uint64_t src_bytes, void* out, uint64_t out_bytes, uint32_t threads,
                    uint32_t seed, void* stream) {
  if (!src || !out || threads == 0 || threads % 256 || src_bytes < 64) return int(hipErrorInvalidValue);
  if (out_bytes < uint64_t(threads / 256) * sizeof(float)) return int(hipErrorInvalidValue);
  const uint64_t slots = src_bytes / 32;  // every read stays inside [src, src + 32 slots)
  hipLaunchKernelGGL(gather32_kernel, dim3(threads / 256), dim3(256), 0, static_cast<hipStream_t>(stream),
                     static_cast<const float4*>(src), slots, static_cast<float*>(out), seed);
  return int(hipGetLastError());
}

int launch_store64(void* dst, uint64_t dst_bytes, uint32_t threads, void* stream) {
  if (!dst || threads == 0 || threads % 256 || dst_bytes < uint64_t(threads) * 256) return int(hipErrorInvalidValue);
  hipLaunchKernelGGL(store64_kernel, dim3(threads / 256), dim3(256), 0, static_cast<hipStream_t>(stream),
                     static_cast<float4*>(dst), 1.0f);
  return int(hipGetLastError());
}

int launch_store32(void* dst, uint64_t dst_bytes, uint32_t threads, void* stream) {
  if (!dst || threads == 0 || threads % 256 || dst_bytes < uint64_t(threads) * 256) return int(hipErrorInvalidValue);
  hipLaunchKernelGGL(store32_kernel, dim3(threads / 256), dim3(256), 0, static_cast<hipStream_t>(stream),
                     static_cast<float4*>(dst), 1.0f);
  return int(hipGetLastError());
}

int launch_spin(uint32_t workgroups, double us, void* stream) {
  if (workgroups == 0 || workgroups > 65536 || us <= 0 || us > 2e6) return int(hipErrorInvalidValue);
  const uint64_t ticks = uint64_t(us * 100.0);  // 100 MHz
  hipLaunchKernelGGL(spin_kernel, dim3(workgroups), dim3(64), 0, static_cast<hipStream_t>(stream), ticks, nullptr);
  return int(hipGetLastError());
}

}  // namespace rocmdash
