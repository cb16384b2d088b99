// Diagnostic build of the window-stats kernel with s_memtime phase stamps
// (cdna_hip_programming.md §7 "In-kernel stamps"): where does an incremental
// refresh spend its cycles? Shares only - the stamps' own waits distort lengths.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -DWS_STAMPS -Icsrc tools/stamps/ws_stamps.hip csrc/device_window.cpp -o ws_stamps
#include "../../csrc/window_stats.hip"

#include <cstdio>
#include <memory>
#include <vector>

#include "device_window.h"
#include "ring.h"

using namespace rocmdash;

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

int main(int argc, char** argv) {
  const uint32_t W = argc > 1 ? uint32_t(std::atoi(argv[1])) : 4096;
  const uint32_t S = argc > 2 ? uint32_t(std::atoi(argv[2])) : 15;
  set_pinned_host_rings(true);
  auto ring = std::make_shared<SeriesRing>(S, 8 * W);
  DeviceWindowSet dws(W, 0);
  dws.add_ring(ring);
  float* out = nullptr;
  CK(hipMalloc(&out, S * STAT_NUM * sizeof(float)));
  hipStream_t stream;
  CK(hipStreamCreate(&stream));
  std::vector<float> row(S);
  uint64_t t = 0, seed = 1;
  auto push = [&](int k) {
    for (int i = 0; i < k; ++i) {
      for (uint32_t c = 0; c < S; ++c) {
        seed = seed * 6364136223846793005ull + 1442695040888963407ull;
        row[c] = float((seed >> 33) % 400);
      }
      ring->push(row.data(), ++t);
    }
  };
  push(W);
  dws.refresh(out, stream, 50, 90, 99);
  CK(hipStreamSynchronize(stream));
  // phase = interval between consecutive WS_STAMP(k) in csrc/window_stats.hip
  const char* names[7] = {"load+sort lists", "barrier 1", "searches+barrier", "merge", "merge tail", "reduce+barrier",
                          "state+epilogue"};
  for (int k : {1, 10, 100}) {
    double acc[7] = {0};
    int n = 0;
    for (int it = 0; it < 300; ++it) {
      push(k);
      dws.refresh(out, stream, 50, 90, 99);
      CK(hipStreamSynchronize(stream));
      if (it < 50) continue;
      unsigned long long st[64][8];
      CK(hipMemcpyFromSymbol(st, HIP_SYMBOL(g_ws_stamps), sizeof st));
      for (uint32_t b = 0; b < S; ++b) {
        for (int p = 0; p < 7; ++p) acc[p] += double(st[b][p + 1] - st[b][p]);
      }
      n += S;
    }
    double total = 0;
    for (double a : acc) total += a;
    std::printf("W=%u k=%d  total %.0f cycles/series (stamped build):", W, k, total / n);
    for (int p = 0; p < 7; ++p) std::printf("  %s %.0f (%.0f%%)", names[p], acc[p] / n, 100.0 * acc[p] / total);
    std::printf("\n");
  }
  return 0;
}
