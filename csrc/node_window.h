// Node-wide window statistics: exact order statistics over the union of every GPU's
// window (all N ranks x W samples of one series), the windowed counterpart of the
// reference's statistics over ALL GPUs (app.py:216-221: mean / max / min of one
// instant sample per GPU).
//
// Every rank already keeps each series' window sorted in HBM (the resident state of
// the incremental window-stats path, window_stats.hip). A node refresh therefore
//   1. exports, per rank, every series' sorted window into one [S][1 + W] float32 row
//      block (element 0 = the number of valid samples, then the sorted samples, +inf
//      after them) - one small kernel, no host round trip (export_sorted);
//   2. all-gathers the blocks over RCCL / xGMI into [N][S][1 + W] (8 ranks x 16 series
//      x 4097 floats = 2.1 MB at W = 4096: the one bandwidth-sized collective of the
//      dashboard, 262 KB per rank);
//   3. selects the order statistics of the union on rank 0 WITHOUT re-sorting: one
//      workgroup per series stages the N sorted lists in LDS (N x W <= 32768 floats,
//      128 KB of the CU's 160 KB; larger unions are read from L2), and every element
//      finds its rank in the merged order with N - 1 binary searches (ties broken by
//      rank index, so ranks are unique); the elements whose ranks are the percentile
//      positions (numpy 'linear', the window-stats definition) write themselves out.
//      Work is N*W*(N-1)*log2(W) LDS reads per series, ~4x fewer than a bitonic sort of
//      the union, and it needs no second buffer.
//   Output per series: [min, max, mean, p0, p1, p2, NaN, count] like the per-GPU kernel
//   (there is no single "last" sample across GPUs).
#pragma once

#include <cstdint>

namespace rocmdash {

// node: device [N][S][1 + W] (the all-gathered export blocks); out: device [S][8].
// Returns a hipError_t.
int launch_node_select(const float* node, uint32_t N, uint32_t S, uint32_t W, float p0, float p1, float p2, float* out,
                       void* stream);

}  // namespace rocmdash
