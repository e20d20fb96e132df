// adaptive.hip — device side of the reference's adaptive supersampling
// (render_section_to_cie_buffer_supersampled, raytracer.rs:257-458).
//
//  * select_kernel: the 8-neighbour stencil of collect_pixels_to_supersample
//    (:386-458), one lane per pixel, neighbours in the reference order, first
//    trigger wins (should_supersample_pair :91-108).  The reference loop is serial
//    but every pixel's decision depends only on the 1-spp buffer, so it is a pure
//    data-parallel stencil.
//  * offsets_kernel: stratified jitter (stratified_sample_offset :145-159, splitmix64
//    mix64 :132-143), samples_per_axis^2 samples per selected pixel, stratum order.
//  * average_kernel: the ordered sum of the valid sub-samples and the 1/valid scale
//    (supersample :334-380).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdint.h>

#include <climits>
#include <cstring>

#include "grt_api.h"
#include "kernels.h"

namespace grt {

// should_supersample_pair (:91-108) on the luminance Y and opacity alpha of two pixels
__device__ __forceinline__ bool pair_triggers(double py, double pa, int pc, double qy, double qa, int qc,
                                              const AdaptiveParams& a) {
  if (pc != qc) return true;
  if (a.exclude_background_contrast && pc == GRT_CLASS_ESCAPED) return false;
  bool visible = fmax(py, qy) > a.min_lum;
  double lc = fabs(py - qy) / (py + qy + 1e-4);
  double oc = fabs(pa - qa);
  return visible && (lc > a.luminance_contrast_threshold || oc > a.opacity_contrast_threshold);
}

__global__ void select_kernel(const double* __restrict__ xyza, const uint8_t* __restrict__ cls,
                              AdaptiveParams a, const double* __restrict__ d_min_lum, uint8_t* __restrict__ flags) {
  if (d_min_lum) a.min_lum = *d_min_lum;  // the floor selected on the device
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t n = (uint64_t)a.w * a.h;
  if (i >= n) return;
  int row = (int)(i / a.w), col = (int)(i % a.w);
  const int sh[8][2] = {{-1, -1}, {-1, 0}, {-1, 1}, {0, -1}, {0, 1}, {1, -1}, {1, 0}, {1, 1}};
  const double* p = xyza + 4 * i;
  int pc = cls[i];
  uint8_t f = 0;
  for (int s = 0; s < 8; ++s) {
    int nr = row + sh[s][0], nc = col + sh[s][1];
    if (nr < 0 || nr >= (int)a.h || nc < 0 || nc >= (int)a.w) continue;
    uint64_t j = (uint64_t)nr * a.w + nc;
    if (pair_triggers(p[1], p[3], pc, xyza[4 * j + 1], xyza[4 * j + 3], cls[j], a)) {
      f = 1;
      break;
    }
  }
  flags[i] = f;
}

// The same stencil for the local pixels of one row-band shard (grt_row_shard) of a
// frame whose 1-spp luminance / opacity and class are known frame-wide: ya holds
// (Y, alpha) per frame pixel, cls the class, both in frame order (the allgather of the
// multi-GPU adaptive pass).  a.w x a.h is the frame; neighbours outside
// it are skipped exactly as outside a single-process section.  flags: local order.
__global__ void select_shard_kernel(const double* __restrict__ ya, const uint8_t* __restrict__ cls,
                                    AdaptiveParams a, const double* __restrict__ d_min_lum, uint32_t band_rows,
                                    uint32_t shard, uint32_t n_shards, uint32_t local_rows,
                                    uint8_t* __restrict__ flags) {
  if (d_min_lum) a.min_lum = *d_min_lum;
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (uint64_t)local_rows * a.w) return;
  int row = (int)shard_frame_row(band_rows, shard, n_shards, (uint32_t)(i / a.w)), col = (int)(i % a.w);
  const int sh[8][2] = {{-1, -1}, {-1, 0}, {-1, 1}, {0, -1}, {0, 1}, {1, -1}, {1, 0}, {1, 1}};
  uint64_t c = (uint64_t)row * a.w + col;
  double py = ya[2 * c], pa = ya[2 * c + 1];
  int pc = cls[c];
  uint8_t f = 0;
  for (int s = 0; s < 8; ++s) {
    int nr = row + sh[s][0], nc = col + sh[s][1];
    if (nr < 0 || nr >= (int)a.h || nc < 0 || nc >= (int)a.w) continue;
    uint64_t j = (uint64_t)nr * a.w + nc;
    if (pair_triggers(py, pa, pc, ya[2 * j], ya[2 * j + 1], cls[j], a)) {
      f = 1;
      break;
    }
  }
  flags[i] = f;
}

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ double hash_pixel_samples(int64_t row, int64_t col, uint64_t k) {
  uint64_t z = mix64((uint64_t)row + mix64((uint64_t)col + mix64(k)));
  return (double)(z >> 11) * (1.0 / (double)(1ull << 53));
}

// sel: this chunk's selected pixels (chunk base `base` of the whole list, which holds
// *d_count entries when d_count is set); one lane per sub-sample
__global__ void offsets_kernel(const uint32_t* __restrict__ sel, uint64_t n_sel, const unsigned long long* d_count,
                               uint64_t base, uint32_t spa, uint32_t row0, uint32_t col0, uint32_t w,
                               uint32_t* __restrict__ pix, double* __restrict__ dx, double* __restrict__ dy) {
  uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t per = (uint64_t)spa * spa;
  if (k >= n_sel * per) return;
  uint64_t j = k / per, s = k % per;
  if (d_count && base + j >= *d_count) return;
  uint32_t p = sel[j];
  int64_t row = row0 + p / w, col = col0 + p % w;
  uint64_t sr = s / spa, sc = s % spa;
  uint64_t idx = sr * spa + sc;
  pix[k] = p;
  dx[k] = ((double)sc + hash_pixel_samples(row, col, 2 * idx)) / (double)spa;
  dy[k] = ((double)sr + hash_pixel_samples(row, col, 2 * idx + 1)) / (double)spa;
}

// sel_out: output index per selected pixel; sel_px: its pixel index in the traced rect
// (for the failure records).  A failed sub-sample (supersample's Err arm, :357-362) is
// appended to f.key (pixel * spa^2 + stratum) / f.status when f.cap allows; f.count
// counts them all (and the NaN / no-terminal-event sub-rays when f.stop is set).
__global__ void average_kernel(const uint32_t* __restrict__ sel_out, const uint32_t* __restrict__ sel_px,
                               uint64_t n_sel, const unsigned long long* d_count, uint64_t base, uint32_t spa,
                               const double* __restrict__ samples, const uint8_t* __restrict__ status,
                               double* __restrict__ out, SubsampleFailures f) {
  uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n_sel || (d_count && base + j >= *d_count)) return;
  uint64_t per = (uint64_t)spa * spa;
  double x = 0.0, y = 0.0, z = 0.0, a = 0.0;
  uint32_t valid = 0;
  for (uint64_t s = 0; s < per; ++s) {
    uint64_t k = j * per + s;
    const int st = status[k] & 0x7f;
    // scene.rs:178-183, :196-202: an error-free ray that hit NaN coordinates or no
    // terminal event is logged by color_of_ray (the caller asked for those: f.stop)
    const int stop = f.ray_stop ? f.ray_stop[k] : GRT_STOP_CELESTIAL;
    const bool event = f.stop && st == GRT_OK && (stop == GRT_STOP_NAN || stop == GRT_STOP_NONE);
    if ((st != GRT_OK || event) && f.count) {
      const unsigned long long slot = atomicAdd(f.count, 1ull);
      if (slot < f.cap) {
        f.key[slot] = (uint64_t)sel_px[j] * per + s;
        f.status[slot] = (uint8_t)st;
        if (f.stop) {
          f.stop[slot] = (uint8_t)stop;
          f.steps[slot] = f.ray_steps ? f.ray_steps[k] : 0u;
        }
      }
    }
    if (st != GRT_OK) continue;
    const double* c = samples + 4 * k;
    x = x + c[0];
    y = y + c[1];
    z = z + c[2];
    a = a + c[3];
    valid++;
  }
  if (valid > 0) {
    double inv = 1.0 / (double)valid;
    double* o = out + 4 * (uint64_t)sel_out[j];
    o[0] = x * inv;
    o[1] = y * inv;
    o[2] = z * inv;
    o[3] = a * inv;
  }
}

__global__ void paint_kernel(const uint32_t* __restrict__ sel, uint64_t n_sel, const unsigned long long* d_count,
                             double m0, double m1, double m2, double m3, double* __restrict__ out) {
  uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n_sel || (d_count && j >= *d_count)) return;
  double* o = out + 4 * (uint64_t)sel[j];
  o[0] = m0;
  o[1] = m1;
  o[2] = m2;
  o[3] = m3;
}

// Sub-rays present in each chunk of the supersample pass: chunk c holds selected pixels
// [c P, (c + 1) P) of *d_count, spa^2 sub-rays each (the integrate / shade kernels' n_live).
__global__ void chunk_live_kernel(const unsigned long long* __restrict__ d_count, uint32_t n_chunks, uint64_t P,
                                  uint32_t per, unsigned long long* __restrict__ live) {
  const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n_chunks) return;
  const uint64_t n = *d_count, lo = (uint64_t)c * P;
  live[c] = n > lo ? (unsigned long long)(min(n - lo, P) * per) : 0ull;
}

// Local pixel index of a shard -> frame pixel index (jitter hash and camera ray).
__global__ void frame_index_kernel(const uint32_t* __restrict__ sel_local, const unsigned long long* __restrict__ d_count,
                                   uint64_t n_max, uint32_t w, uint32_t band_rows, uint32_t shard, uint32_t n_shards,
                                   uint32_t* __restrict__ sel_frame) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n_max || j >= *d_count) return;
  const uint32_t i = sel_local[j];
  sel_frame[j] = shard_frame_row(band_rows, shard, n_shards, i / w) * w + i % w;
}

static inline unsigned nblocks(uint64_t n, unsigned t) { return (unsigned)((n + t - 1) / t); }

// Work order of the supersample pass, longest sub-rays first.  A pixel's sort key is the
// most 1-spp steps in its 3 x 3 neighbourhood (its sub-rays sample the pixel's square,
// between its own centre ray and its neighbours'), + 1 so that the unused entries (key 0)
// sort last.  C5: the pass's lane occupancy 0.69 -> 0.78 and its end after the queue
// drains 0.17 -> 0.10 s (tools/ray_timeline.py c5); C5 1,639-1,665 -> 1,604-1,621 ms, the
// frame bit-identical (profiles/r06i).  The pixel's own steps as the key: no gain.
__global__ void sub_order_keys_kernel(const uint32_t* __restrict__ sel, const unsigned long long* __restrict__ d_count,
                                      uint64_t n_max, const uint32_t* __restrict__ steps, uint32_t w, uint32_t h,
                                      uint32_t* __restrict__ keys, uint32_t* __restrict__ vals) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n_max) return;
  uint32_t key = 0, p = 0;
  if (j < *d_count) {
    p = sel[j];
    const int row = (int)(p / w), col = (int)(p % w);
    uint32_t m = steps[p];
    for (int dr = -1; dr <= 1; ++dr)
      for (int dc = -1; dc <= 1; ++dc) {
        const int r = row + dr, c = col + dc;
        if (r >= 0 && r < (int)h && c >= 0 && c < (int)w) m = max(m, steps[(uint64_t)r * w + c]);
      }
    key = m == 0xffffffffu ? m : m + 1;
  }
  keys[j] = key;
  vals[j] = p;
}

hipError_t order_selection(const uint32_t* d_sel, const unsigned long long* d_count, uint64_t n_max,
                           const uint32_t* d_steps, uint32_t w, uint32_t h, uint32_t* d_out, void* d_temp,
                           size_t* temp_bytes, hipStream_t stream) {
  if (n_max == 0 || n_max > (uint64_t)INT_MAX) return n_max ? hipErrorInvalidValue : hipSuccess;
  const size_t arr = (n_max * 4 + 255) & ~(size_t)255;
  size_t sort_bytes = 0;
  hipError_t e = hipcub::DeviceRadixSort::SortPairsDescending(nullptr, sort_bytes, (const uint32_t*)nullptr,
                                                              (uint32_t*)nullptr, (const uint32_t*)nullptr,
                                                              (uint32_t*)nullptr, (int)n_max, 0, 32, stream);
  if (e != hipSuccess) return e;
  if (d_temp == nullptr) {
    *temp_bytes = 3 * arr + sort_bytes;
    return hipSuccess;
  }
  uint32_t* keys = (uint32_t*)d_temp;
  uint32_t* keys_sorted = (uint32_t*)((char*)d_temp + arr);
  uint32_t* vals = (uint32_t*)((char*)d_temp + 2 * arr);
  void* tmp = (char*)d_temp + 3 * arr;
  hipLaunchKernelGGL(sub_order_keys_kernel, dim3(nblocks(n_max, 256)), dim3(256), 0, stream, d_sel, d_count, n_max,
                     d_steps, w, h, keys, vals);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  // a stable sort: equal keys keep the selection order
  return hipcub::DeviceRadixSort::SortPairsDescending(tmp, sort_bytes, keys, keys_sorted, vals, d_out, (int)n_max, 0,
                                                      32, stream);
}

// resolve_minimum_luminance's order (raytracer.rs:118-129): f64::total_cmp of the
// luminance Y, as an unsigned radix key (total_cmp's signed key with the sign bit
// flipped).  The map is its own inverse on the low 63 bits, so the selected key gives
// back the exact f64.
__device__ __forceinline__ uint64_t total_cmp_ukey(double v) {
  const int64_t b = __double_as_longlong(v);
  return (uint64_t)(b ^ (int64_t)((uint64_t)(b >> 63) >> 1)) ^ 0x8000000000000000ull;
}

__global__ void lum_keys_kernel(const double* __restrict__ y, uint32_t stride, uint64_t n,
                                uint64_t* __restrict__ keys) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) keys[i] = total_cmp_ukey(y[(uint64_t)stride * i]);
}

// 1e-3 x the index-th key (resolve_minimum_luminance, raytracer.rs:125-128), on the device
__global__ void floor_kernel(const uint64_t* __restrict__ sorted, uint64_t index, double* __restrict__ d_min_lum) {
  const int64_t sk = (int64_t)(sorted[index] ^ 0x8000000000000000ull);
  const int64_t b = sk ^ (int64_t)((uint64_t)(sk >> 63) >> 1);
  *d_min_lum = 1e-3 * __longlong_as_double(b);
}
__global__ void key_to_value_kernel(const uint64_t* __restrict__ sorted, uint64_t index, double* __restrict__ out) {
  const int64_t sk = (int64_t)(sorted[index] ^ 0x8000000000000000ull);
  *out = __longlong_as_double(sk ^ (int64_t)((uint64_t)(sk >> 63) >> 1));
}

// The index-th luminance in total_cmp order -> d_out (times `scale` == 1e-3: the floor).
// hipCUB counts items in int: n beyond INT_MAX is refused.
static hipError_t order_stat_device(const double* d_y, uint32_t stride, uint64_t n, uint64_t index, void* d_mem,
                                    size_t* mem_bytes, bool floor, double* d_out, hipStream_t stream) {
  if (n == 0 || n > (uint64_t)INT_MAX || index >= n) return hipErrorInvalidValue;
  const size_t keys_bytes = ((n * 8 + 255) & ~(size_t)255);
  size_t temp = 0;
  hipcub::DoubleBuffer<uint64_t> db((uint64_t*)nullptr, (uint64_t*)nullptr);
  hipError_t e = hipcub::DeviceRadixSort::SortKeys(nullptr, temp, db, (int)n, 0, 64, stream);
  if (e != hipSuccess) return e;
  if (d_mem == nullptr) {
    *mem_bytes = 2 * keys_bytes + temp;
    return hipSuccess;
  }
  uint64_t* keys = (uint64_t*)d_mem;
  hipcub::DoubleBuffer<uint64_t> buf(keys, (uint64_t*)((char*)d_mem + keys_bytes));
  void* tmp = (char*)d_mem + 2 * keys_bytes;
  hipLaunchKernelGGL(lum_keys_kernel, dim3(nblocks(n, 256)), dim3(256), 0, stream, d_y, stride, n, keys);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  if ((e = hipcub::DeviceRadixSort::SortKeys(tmp, temp, buf, (int)n, 0, 64, stream)) != hipSuccess) return e;
  if (floor) hipLaunchKernelGGL(floor_kernel, dim3(1), dim3(1), 0, stream, buf.Current(), index, d_out);
  else hipLaunchKernelGGL(key_to_value_kernel, dim3(1), dim3(1), 0, stream, buf.Current(), index, d_out);
  return hipGetLastError();
}

hipError_t luminance_floor_device(const double* d_y, uint32_t stride, uint64_t n, uint64_t index, void* d_mem,
                                  size_t* mem_bytes, double* d_min_lum, hipStream_t stream) {
  return order_stat_device(d_y, stride, n, index, d_mem, mem_bytes, true, d_min_lum, stream);
}

hipError_t luminance_order_stat(const double* d_y, uint32_t stride, uint64_t n, uint64_t index, void* d_mem,
                                size_t* mem_bytes, double* value, hipStream_t stream) {
  // d_mem: scratch of *mem_bytes (query with d_mem == NULL) followed by 8 bytes for the value
  if (d_mem == nullptr) {
    hipError_t e = order_stat_device(d_y, stride, n, index, nullptr, mem_bytes, false, nullptr, stream);
    *mem_bytes = ((*mem_bytes + 255) & ~(size_t)255) + 256;
    return e;
  }
  size_t bytes = 0;
  hipError_t e = order_stat_device(d_y, stride, n, index, nullptr, &bytes, false, nullptr, stream);
  if (e != hipSuccess) return e;
  double* d_val = (double*)((char*)d_mem + ((bytes + 255) & ~(size_t)255));
  if ((e = order_stat_device(d_y, stride, n, index, d_mem, &bytes, false, d_val, stream)) != hipSuccess) return e;
  if ((e = hipMemcpyAsync(value, d_val, 8, hipMemcpyDeviceToHost, stream)) != hipSuccess) return e;
  return hipStreamSynchronize(stream);
}

// DeviceSelect::Flagged over 0..n-1: the selected indices in order and their count
// (collect_pixels_to_supersample's serial order, raytracer.rs:386-458).
hipError_t compact_flags(const uint8_t* d_flags, uint64_t n, uint32_t* d_out, unsigned long long* d_count, void* d_temp,
                         size_t* temp_bytes, hipStream_t stream) {
  if (n > (uint64_t)INT_MAX) return hipErrorInvalidValue;
  hipcub::CountingInputIterator<uint32_t> it(0u);
  return hipcub::DeviceSelect::Flagged(d_temp, *temp_bytes, it, d_flags, d_out, d_count, (int)n, stream);
}

hipError_t launch_select(const double* d_xyza64, const uint8_t* d_cls, const AdaptiveParams& p,
                         const double* d_min_lum, uint8_t* d_flags, hipStream_t stream) {
  uint64_t n = (uint64_t)p.w * p.h;
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(select_kernel, dim3(nblocks(n, 256)), dim3(256), 0, stream, d_xyza64, d_cls, p, d_min_lum,
                     d_flags);
  return hipGetLastError();
}
hipError_t launch_select_shard(const double* d_ya, const uint8_t* d_cls, const AdaptiveParams& p,
                               const double* d_min_lum, uint32_t band_rows, uint32_t shard, uint32_t n_shards,
                               uint32_t local_rows, uint8_t* d_flags, hipStream_t stream) {
  uint64_t n = (uint64_t)local_rows * p.w;
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(select_shard_kernel, dim3(nblocks(n, 256)), dim3(256), 0, stream, d_ya, d_cls, p, d_min_lum,
                     band_rows, shard, n_shards, local_rows, d_flags);
  return hipGetLastError();
}
hipError_t launch_make_offsets(const uint32_t* d_sel, uint64_t n_sel, const unsigned long long* d_count, uint64_t base,
                               uint32_t spa, uint32_t row0, uint32_t col0, uint32_t w, uint32_t* d_pix, double* d_dx,
                               double* d_dy, hipStream_t stream) {
  uint64_t n = n_sel * spa * spa;
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(offsets_kernel, dim3(nblocks(n, 256)), dim3(256), 0, stream, d_sel, n_sel, d_count, base, spa,
                     row0, col0, w, d_pix, d_dx, d_dy);
  return hipGetLastError();
}
hipError_t launch_average(const uint32_t* d_sel_out, const uint32_t* d_sel_px, uint64_t n_sel,
                          const unsigned long long* d_count, uint64_t base, uint32_t spa, const double* d_samples,
                          const uint8_t* d_status, double* d_out, const SubsampleFailures& f, hipStream_t stream) {
  if (n_sel == 0) return hipSuccess;
  hipLaunchKernelGGL(average_kernel, dim3(nblocks(n_sel, 256)), dim3(256), 0, stream, d_sel_out, d_sel_px, n_sel,
                     d_count, base, spa, d_samples, d_status, d_out, f);
  return hipGetLastError();
}
hipError_t launch_paint(const uint32_t* d_sel, uint64_t n_sel, const unsigned long long* d_count, const double* mask,
                        double* d_out, hipStream_t stream) {
  if (n_sel == 0) return hipSuccess;
  hipLaunchKernelGGL(paint_kernel, dim3(nblocks(n_sel, 256)), dim3(256), 0, stream, d_sel, n_sel, d_count, mask[0],
                     mask[1], mask[2], mask[3], d_out);
  return hipGetLastError();
}
hipError_t launch_chunk_live(const unsigned long long* d_count, uint32_t n_chunks, uint64_t P, uint32_t per,
                             unsigned long long* d_live, hipStream_t stream) {
  hipLaunchKernelGGL(chunk_live_kernel, dim3(nblocks(n_chunks, 64)), dim3(64), 0, stream, d_count, n_chunks, P, per,
                     d_live);
  return hipGetLastError();
}
hipError_t launch_frame_index(const uint32_t* d_sel_local, const unsigned long long* d_count, uint64_t n_max, uint32_t w,
                              uint32_t band_rows, uint32_t shard, uint32_t n_shards, uint32_t* d_sel_frame,
                              hipStream_t stream) {
  if (n_max == 0) return hipSuccess;
  hipLaunchKernelGGL(frame_index_kernel, dim3(nblocks(n_max, 256)), dim3(256), 0, stream, d_sel_local, d_count, n_max,
                     w, band_rows, shard, n_shards, d_sel_frame);
  return hipGetLastError();
}

}  // namespace grt
