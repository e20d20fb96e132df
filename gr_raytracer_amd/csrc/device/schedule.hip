// schedule.hip — tile queue order for the persistent integrate kernel.
//
// Pixels cost very different amounts: in Kerr-Schild (C4) the rays that fall into the
// horizon take ~5e5 accepted steps and the trapped ones the full max_steps (1e6),
// while an escaping ray takes ~1.6e4.  The integrate kernel hands out 8x8 tiles from
// one counter, so a long tile queued late ends the frame on a single busy lane.  The
// probe kernel (geodesic.hip) traces one ray per tile for a capped number of steps;
// here each tile's key is the largest probe count in its 3x3 tile neighbourhood (a
// shadow edge can cut a tile whose probe pixel escapes), and the tiles are sorted by
// key, descending and stable (row-major among equals), with hipCUB's radix sort.  The
// order changes which lane traces a pixel, never its result.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "kernels.h"

namespace grt {

__global__ void __launch_bounds__(256) dilate_kernel(const uint32_t* __restrict__ probe, uint32_t tiles_x,
                                                     uint32_t tiles_y, uint32_t* __restrict__ keys,
                                                     uint32_t* __restrict__ idx) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= tiles_x * tiles_y) return;
  const int tr = (int)(t / tiles_x), tc = (int)(t % tiles_x);
  uint32_t k = 0;
  for (int dr = -1; dr <= 1; ++dr)
    for (int dc = -1; dc <= 1; ++dc) {
      const int r = tr + dr, c = tc + dc;
      if (r >= 0 && r < (int)tiles_y && c >= 0 && c < (int)tiles_x) k = max(k, probe[(uint32_t)r * tiles_x + c]);
    }
  keys[t] = k;
  idx[t] = t;
}

hipError_t launch_tile_order(const uint32_t* d_probe, uint32_t tiles_x, uint32_t tiles_y, uint32_t* d_keys,
                             uint32_t* d_keys_sorted, uint32_t* d_idx, uint32_t* d_order, void* temp,
                             size_t* temp_bytes, hipStream_t stream) {
  const uint32_t n = tiles_x * tiles_y;
  if (temp == nullptr)
    return hipcub::DeviceRadixSort::SortPairsDescending(nullptr, *temp_bytes, d_keys, d_keys_sorted, d_idx, d_order,
                                                        (int)n, 0, 32, stream);
  hipLaunchKernelGGL(dilate_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, d_probe, tiles_x, tiles_y, d_keys,
                     d_idx);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  return hipcub::DeviceRadixSort::SortPairsDescending(temp, *temp_bytes, d_keys, d_keys_sorted, d_idx, d_order, (int)n,
                                                      0, 32, stream);
}

}  // namespace grt
