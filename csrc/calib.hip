// Calibration load for the device-counter series (tests/test_gpu.py, tools/probes):
// `workgroups` one-wave workgroups that each keep their CU busy for `us` microseconds
// of wall time and exit. With at most one workgroup per CU the share of busy CUs is
// known exactly, which is what the CU-active series (csrc/counters.cpp) must report.
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

}  // namespace

int launch_spin(uint32_t workgroups, double us, void* stream) {
  if (workgroups == 0 || workgroups > 65536 || us <= 0 || us > 2e6) return int(hipErrorInvalidValue);
  const uint64_t ticks = uint64_t(us * 100.0);  // 100 MHz
  hipLaunchKernelGGL(spin_kernel, dim3(workgroups), dim3(64), 0, static_cast<hipStream_t>(stream), ticks, nullptr);
  return int(hipGetLastError());
}

}  // namespace rocmdash
