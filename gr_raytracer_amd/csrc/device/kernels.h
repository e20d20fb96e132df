// kernels.h — launch entry points of the gfx950 kernels (geodesic.hip, adaptive.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "dev_scene.h"

namespace grt {

// integrate_kernel (persistent, lane refill) then shade_kernel, all on `stream`.  With
// `vol` (the scene has VolumetricDiscs): integrate, job gathering, march_kernel and the
// composite; the workspace then needs its volumetric arrays, ws.march zeroed.
// `tl.cap` != 0 (every Kerr-Schild trace, volumetric or not): long rays are handed to
// tail_kernel (launched between integrate and shade on `stream`, `tail_blocks` blocks of
// 256 threads); tl.ctl must be zeroed.
hipError_t launch_trace(int geometry, const DevScene* d_scene, const WorkList& wl, const Workspace& ws,
                        const Outputs& out, unsigned long long* d_counter, unsigned long long* d_stats,
                        int blocks, int threads, bool vol, const TailList& tl, int tail_blocks,
                        hipStream_t stream);
// Diagnostic builds (-DGRT_RAY_TIMES=1): the per-ray schedule record ([6][n] words, see
// geodesic.hip), or NULL.
hipError_t set_ray_times(unsigned long long* p);
// Tail kernel's quad capacity per block (rays integrated at once).
constexpr int TAIL_RAYS_PER_BLOCK = 256 / 4;

// Work-order probe: steps of one ray per 8x8 tile of `wl` (rectangle mode), capped.
// quad (Kerr-Schild only): each probe ray on a quad of lanes (probe_quad_kernel), same keys.
hipError_t launch_probe(int geometry, const DevScene* d_scene, const WorkList& wl, uint32_t n_tiles, uint32_t cap,
                        uint32_t* d_steps, bool quad, hipStream_t stream);
// Schwarzschild work-order keys without a probe pass: predicted steps per 8x8 tile of
// `wl` from the impact parameter of the tile's probe pixel (impact_key_kernel).
hipError_t launch_impact_keys(const DevScene* d_scene, const WorkList& wl, uint32_t n_tiles, uint32_t* d_keys,
                              hipStream_t stream);
// Tile queue order from the probe keys (schedule.hip): 3x3-dilated keys (edge tiles of a
// region of probes that reached `cap` boosted), sorted descending (stable).  `temp` /
// `temp_bytes`: scratch, query with temp == NULL.
hipError_t launch_tile_order(const uint32_t* d_probe, uint32_t tiles_x, uint32_t tiles_y, uint32_t cap, uint32_t* d_keys,
                             uint32_t* d_keys_sorted, uint32_t* d_idx, uint32_t* d_order, void* temp,
                             size_t* temp_bytes, hipStream_t stream);

// Whole trajectories (render-ray / render-ray-at): camera pixels (row, col) or explicit
// native-chart (position, momentum) pairs; record layout in trajectory_kernel.
struct TrajectoryList {
  uint64_t n;
  const double* row;  // camera mode: pixel coordinates (offsets allowed), both non-null
  const double* col;
  const double* pos;  // explicit mode: n x 4 each
  const double* mom;
  uint64_t cap;       // records stored per ray
  double* steps;      // n x cap x 9
  uint64_t* n_steps;  // steps produced per ray (step 0 included), even beyond cap
  uint8_t* stop;
  uint8_t* status;
};
// test hook: div_inrange / div2_inrange against the compiler's division on n random pairs
hipError_t launch_arith_map(uint32_t samples, uint64_t seed, uint8_t* d_map, uint8_t* d_zmap, uint8_t* d_smap,
                            hipStream_t stream);
hipError_t launch_rhs_check(int geometry, const DevScene* d_scene, const double* d_states, const double* d_consts,
                            uint64_t n, double* d_out, uint8_t* d_pred, hipStream_t stream);
#if GRT_PATH_COUNT
hipError_t path_read(unsigned long long* out, bool reset);  // 16 words
#endif
// The same trace compiled with FMA contraction (geodesic_fused.hip, grt_set_arithmetic(1)):
// every geometry but Kerr-Schild (hipErrorInvalidValue for it).
namespace fused {
hipError_t launch_trace(int geometry, const DevScene* d_scene, const WorkList& wl, const Workspace& ws,
                        const Outputs& out, unsigned long long* d_counter, unsigned long long* d_stats,
                        int blocks, int threads, bool vol, const TailList& tl, int tail_blocks,
                        hipStream_t stream);
}  // namespace fused
// The exact KerrBL trace (geodesic_kerr_bl.hip: the same code compiled without machine
// loop-invariant code motion, which hoisted ~100 VGPRs of polynomial constants out of the
// loops and made the 3-wave integrate kernel spill; C3 -2%, its raymarch -7%, profiles/r06p).
namespace kerr_bl {
hipError_t launch_trace(int geometry, const DevScene* d_scene, const WorkList& wl, const Workspace& ws,
                        const Outputs& out, unsigned long long* d_counter, unsigned long long* d_stats,
                        int blocks, int threads, bool vol, const TailList& tl, int tail_blocks,
                        hipStream_t stream);
hipError_t set_ray_times(unsigned long long* p);
#if GRT_PATH_COUNT
hipError_t path_read(unsigned long long* out, bool reset);
#endif
}  // namespace kerr_bl
hipError_t launch_trajectories(int geometry, const DevScene* d_scene, const TrajectoryList& tl, hipStream_t stream);

// Invariant monitors of the n = rows x cols rays of a rectangle (health_kernel):
// d_out n x 5 doubles, d_status n bytes.
hipError_t launch_health(int geometry, const DevScene* d_scene, const WorkList& wl, uint64_t n, double* d_out,
                         uint8_t* d_status, hipStream_t stream);

// Adaptive supersampling helpers (raytracer.rs:91-159, :320-458).
struct AdaptiveParams {
  uint32_t w, h;  // section size
  int32_t exclude_background_contrast;
  int32_t _pad;
  double min_lum;
  double luminance_contrast_threshold;
  double opacity_contrast_threshold;
};
// d_min_lum (nullable): the luminance floor on the device, else p.min_lum.
hipError_t launch_select(const double* d_xyza64, const uint8_t* d_cls, const AdaptiveParams& p,
                         const double* d_min_lum, uint8_t* d_flags, hipStream_t stream);
// The index-th of n luminances d_y[stride * i] in f64::total_cmp order, on the device
// (radix sort; n <= INT_MAX).  Call with d_mem == NULL for the scratch size.
// luminance_order_stat returns the value to the host; luminance_floor_device writes
// 1e-3 x the value (resolve_minimum_luminance) to *d_min_lum without a host copy.
hipError_t luminance_order_stat(const double* d_y, uint32_t stride, uint64_t n, uint64_t index, void* d_mem,
                                size_t* mem_bytes, double* value, hipStream_t stream);
hipError_t luminance_floor_device(const double* d_y, uint32_t stride, uint64_t n, uint64_t index, void* d_mem,
                                  size_t* mem_bytes, double* d_min_lum, hipStream_t stream);
// Indices i < n with d_flags[i] != 0, in order, and their count (n <= INT_MAX).
// Call with d_temp == NULL for *temp_bytes.
hipError_t compact_flags(const uint8_t* d_flags, uint64_t n, uint32_t* d_out, unsigned long long* d_count, void* d_temp,
                         size_t* temp_bytes, hipStream_t stream);
hipError_t launch_select_shard(const double* d_ya, const uint8_t* d_cls, const AdaptiveParams& p,
                               const double* d_min_lum, uint32_t band_rows, uint32_t shard, uint32_t n_shards,
                               uint32_t local_rows, uint8_t* d_flags, hipStream_t stream);
// The supersample helpers take a chunk of the selected list: n_sel entries starting at
// position `base` of a list of *d_count entries (d_count NULL: all n_sel present).
hipError_t launch_make_offsets(const uint32_t* d_sel, uint64_t n_sel, const unsigned long long* d_count, uint64_t base,
                               uint32_t spa, uint32_t row0, uint32_t col0, uint32_t w, uint32_t* d_pix, double* d_dx,
                               double* d_dy, hipStream_t stream);
// Failed sub-samples of the supersample pass (device side; count NULL: not recorded).
struct SubsampleFailures {
  unsigned long long* count;
  uint64_t* key;      // pixel * spa^2 + stratum
  uint8_t* status;
  uint64_t cap;
  // with `stop` set, the list also takes the sub-rays without an error that ended on NaN
  // coordinates or without a terminal event (status 0), with their stop reason and steps
  uint8_t* stop;
  uint32_t* steps;
  const uint8_t* ray_stop;    // the sub-ray trace's stop reasons / step counts
  const uint32_t* ray_steps;
};
hipError_t launch_average(const uint32_t* d_sel_out, const uint32_t* d_sel_px, uint64_t n_sel,
                          const unsigned long long* d_count, uint64_t base, uint32_t spa, const double* d_samples,
                          const uint8_t* d_status, double* d_out, const SubsampleFailures& f, hipStream_t stream);
hipError_t launch_paint(const uint32_t* d_sel, uint64_t n_sel, const unsigned long long* d_count, const double* mask,
                        double* d_out, hipStream_t stream);
// live[c] = sub-rays of chunk c (P selected pixels per chunk, `per` sub-rays each)
hipError_t launch_chunk_live(const unsigned long long* d_count, uint32_t n_chunks, uint64_t P, uint32_t per,
                             unsigned long long* d_live, hipStream_t stream);
hipError_t launch_frame_index(const uint32_t* d_sel_local, const unsigned long long* d_count, uint64_t n_max, uint32_t w,
                              uint32_t band_rows, uint32_t shard, uint32_t n_shards, uint32_t* d_sel_frame,
                              hipStream_t stream);
// Work order of the supersample pass: the first *d_count of d_sel (pixel indices of a
// w x h rect, n_max entries of room) into d_out, longest expected sub-rays first -- by
// the 1-spp step counts d_steps (rect order) around each pixel -- ties in selection
// order.  Call with d_temp == NULL for *temp_bytes (n_max <= INT_MAX).
hipError_t order_selection(const uint32_t* d_sel, const unsigned long long* d_count, uint64_t n_max,
                           const uint32_t* d_steps, uint32_t w, uint32_t h, uint32_t* d_out, void* d_temp,
                           size_t* temp_bytes, hipStream_t stream);

}  // namespace grt
