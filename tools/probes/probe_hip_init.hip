// Device memory taken by the HIP runtime alone: what a process
// that only starts HIP holds, against torch's 487 MiB. Prints one JSON line with the
// device's used VRAM (amdgpu sysfs, whole device: run it alone on the box) after each
// stage. argv[1] = sysfs path of mem_info_vram_used.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <string>

static long long used(const char* path) {
  std::ifstream f(path);
  long long v = -1;
  f >> v;
  return v;
}

__global__ void touch(float* p) { p[threadIdx.x] = 1.0f; }

// a kernel with a private array indexed at run time: the compiler puts it in scratch
__global__ void scratchy(float* p, int k) {
  float a[256];
  for (int i = 0; i < 256; ++i) a[i] = p[i & 63] + float(i);
  p[threadIdx.x] = a[(k + threadIdx.x) & 255];
}

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  const char* p = argv[1];
  long long s0 = used(p);
  if (hipInit(0) != hipSuccess) return 3;
  long long s1 = used(p);
  if (hipSetDevice(0) != hipSuccess) return 4;
  hipFree(nullptr);  // context creation
  long long s2 = used(p);
  float* d = nullptr;
  if (hipMalloc(&d, 64 * sizeof(float)) != hipSuccess) return 5;
  touch<<<1, 64>>>(d);
  if (hipDeviceSynchronize() != hipSuccess) return 6;
  long long s3 = used(p);
  hipStream_t st;
  hipStreamCreate(&st);
  touch<<<1, 64, 0, st>>>(d);
  hipStreamSynchronize(st);
  long long s4 = used(p);
  hipStream_t st2;
  hipStreamCreate(&st2);
  touch<<<1, 64, 0, st2>>>(d);
  hipStreamSynchronize(st2);
  long long s5 = used(p);
  scratchy<<<1, 64, 0, st>>>(d, 3);
  hipStreamSynchronize(st);
  long long s6 = used(p);
  std::printf("{\"start\": %lld, \"hipInit\": %lld, \"context\": %lld, \"first_kernel\": %lld, \"stream\": %lld, "
              "\"stream2\": %lld, \"scratch_kernel\": %lld}\n",
              s0, s1, s2, s3, s4, s5, s6);
  hipFree(d);
  return 0;
}
