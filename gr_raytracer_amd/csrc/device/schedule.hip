// schedule.hip — tile queue order for the persistent integrate kernel.
//
// Pixels cost very different amounts: in Kerr-Schild (C4) the rays that fall into the
// horizon take ~5e5 accepted steps and the trapped ones the full max_steps (1e6),
// while an escaping ray takes ~1.6e4.  The integrate kernel hands out 8x8 tiles from
// one counter, so a long tile queued late ends the frame on a single busy lane.  The
// probe kernel (geodesic.hip) traces one ray per tile for a capped number of steps (a
// probe still going at the cap gets a key above the cap from its state there); here each
// tile's key is the largest probe key in its 3x3 tile neighbourhood (a shadow edge can
// cut a tile whose probe pixel escapes; edge tiles get more, below), and the tiles are sorted by
// key, descending and stable (row-major among equals), with hipCUB's radix sort.  The
// order changes which lane traces a pixel, never its result.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "kernels.h"

namespace grt {

// Edge tiles (own probe finished, a neighbour's capped: the tile straddles the border of
// a long-ray region) get twice the neighbour's excess over the cap.  The rays that graze
// that border run longer than the ones inside it: in a C4 shard the edge tiles' longest
// rays reach 0.9-1.9x the neighbour's prediction at the 90th-99th percentile, and a tile
// of 6e5-step rays queued by its neighbour's key ended the shard 2 s after the rest
// (profiles/r04d); most edge tiles are short, so queueing them early costs little.
__global__ void __launch_bounds__(256) dilate_kernel(const uint32_t* __restrict__ probe, uint32_t tiles_x,
                                                     uint32_t tiles_y, uint32_t cap, uint32_t* __restrict__ keys,
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
  if (probe[t] < cap && k > cap) {
    const uint64_t boosted = (uint64_t)cap + 2ull * (uint64_t)(k - cap);
    k = boosted > 0xffffffffull ? 0xffffffffu : (uint32_t)boosted;
  }
  keys[t] = k;
  idx[t] = t;
}

hipError_t launch_tile_order(const uint32_t* d_probe, uint32_t tiles_x, uint32_t tiles_y, uint32_t cap, uint32_t* d_keys,
                             uint32_t* d_keys_sorted, uint32_t* d_idx, uint32_t* d_order, void* temp,
                             size_t* temp_bytes, hipStream_t stream) {
  const uint32_t n = tiles_x * tiles_y;
  if (temp == nullptr)
    return hipcub::DeviceRadixSort::SortPairsDescending(nullptr, *temp_bytes, d_keys, d_keys_sorted, d_idx, d_order,
                                                        (int)n, 0, 32, stream);
  hipLaunchKernelGGL(dilate_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, d_probe, tiles_x, tiles_y, cap,
                     d_keys, d_idx);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  return hipcub::DeviceRadixSort::SortPairsDescending(temp, *temp_bytes, d_keys, d_keys_sorted, d_idx, d_order, (int)n,
                                                      0, 32, stream);
}

}  // namespace grt
