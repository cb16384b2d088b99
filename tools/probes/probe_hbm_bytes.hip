// Known-traffic kernels for the HBM byte accounting. Run under
// rocprofv3 --pmc: every dispatch moves a known number of bytes, so per-dispatch TCC
// request counters can be checked against it by request size.
//   copy_wide   : float4 copy, N bytes read + N bytes written (128 B lines, full)
//   gather32    : one 32 B read per thread at a random 32 B-aligned offset of a 4 GiB
//                 buffer (beyond the 256 MB MALL); one float written per workgroup
//   store64     : one 64 B store per thread at a 256 B stride (no two in one line)
//   copy_mall   : float4 copy of 64 MiB (fits in the MALL), repeated
// Prints one JSON line per kernel with its dispatches, bytes per dispatch and time.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
      std::exit(1);                                                             \
    }                                                                           \
  } while (0)

__global__ void copy_wide(const float4* __restrict__ a, float4* __restrict__ b, size_t n4) {
  size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x;
  size_t stride = size_t(gridDim.x) * blockDim.x;
  for (; i < n4; i += stride) b[i] = a[i];
}

__device__ __forceinline__ unsigned hash32(unsigned x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return x;
}

// each thread: one 32 B read (two float4) at a random 32 B slot of n32 slots
__global__ void gather32(const float4* __restrict__ a, size_t n32, float* __restrict__ out, unsigned seed) {
  unsigned t = blockIdx.x * blockDim.x + threadIdx.x;
  size_t slot = (size_t(hash32(t ^ seed)) * 2654435761ULL + hash32(t + seed)) % n32;
  float4 x = a[2 * slot];
  float4 y = a[2 * slot + 1];
  float s = x.x + x.y + x.z + x.w + y.x + y.y + y.z + y.w;
  for (int o = 32; o > 0; o >>= 1) s += __shfl_down(s, o);
  __shared__ float ws[16];
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float tot = 0.f;
    for (int w = 0; w < int(blockDim.x >> 6); ++w) tot += ws[w];
    out[blockIdx.x] = tot;
  }
}

// each thread: one 64 B store (four float4) at byte offset 256 * t
__global__ void store64(float4* __restrict__ b, float v) {
  size_t t = blockIdx.x * size_t(blockDim.x) + threadIdx.x;
  float4 x = make_float4(v, v + 1.f, v + 2.f, v + 3.f);
  float4* p = b + t * 16;  // 16 float4 = 256 B
  p[0] = x; p[1] = x; p[2] = x; p[3] = x;
}

int main(int argc, char** argv) {
  int reps = argc > 1 ? std::atoi(argv[1]) : 5;
  const size_t big = size_t(4) << 30;
  float4 *a = nullptr, *b = nullptr;
  float* out = nullptr;
  CK(hipMalloc(&a, big));
  CK(hipMalloc(&b, big));
  CK(hipMalloc(&out, 1 << 24));
  CK(hipMemset(a, 0, big));
  CK(hipMemset(b, 0, big));
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto run = [&](const char* name, double rd, double wr, int n, auto launch) {
    launch();  // warm
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int i = 0; i < n; ++i) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::printf("{\"kernel\": \"%s\", \"dispatches\": %d, \"read_bytes\": %.0f, \"write_bytes\": %.0f, "
                "\"ms_per_dispatch\": %.4f, \"read_GBps\": %.1f, \"write_GBps\": %.1f}\n",
                name, n + 1, rd, wr, ms / n, rd / (ms / n) * 1e-6, wr / (ms / n) * 1e-6);
    std::fflush(stdout);
  };
  // 1 GiB wide copy
  const size_t cw = size_t(1) << 30;
  run("copy_wide", double(cw), double(cw), reps, [&] {
    copy_wide<<<4096, 256>>>(a, b, cw / 16);
  });
  // 32 B random gathers over 4 GiB: 16M threads -> 512 MiB of requests
  const unsigned gthreads = 1u << 24;
  unsigned seed = 1;
  run("gather32", double(gthreads) * 32, double(gthreads / 256) * 4, reps, [&] {
    gather32<<<gthreads / 256, 256>>>(a, big / 32, out, seed++);
  });
  // 64 B stores at 256 B stride: 8M threads -> 512 MiB stored, 2 GiB spanned
  const unsigned sthreads = 1u << 23;
  run("store64", 0.0, double(sthreads) * 64, reps, [&] {
    store64<<<sthreads / 256, 256>>>(b, 1.0f);
  });
  // 64 MiB copy loop: fits in the 256 MB MALL
  const size_t cm = size_t(64) << 20;
  run("copy_mall", double(cm), double(cm), reps * 4, [&] {
    copy_wide<<<2048, 256>>>(a, b, cm / 16);
  });
  CK(hipFree(a));
  CK(hipFree(b));
  CK(hipFree(out));
  return 0;
}
