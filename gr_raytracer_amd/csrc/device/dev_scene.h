// dev_scene.h — device-resident scene layout for the gfx950 geodesic kernels.
//
// Built once per frame (per GPU) from grt_scene_desc by api.hip.  Every field is
// read wave-uniformly, so the compiler serves it from the scalar cache (s_load);
// textures and LUTs live in HBM behind plain pointers.
#pragma once
#include <stdint.h>

// Window candidates a ray keeps in workspace slots before the hit pool (grt_api.h
// GRT_MAX_HITS).  Overridable at build time: a build with very few slots sends nearly
// every candidate through the pool, which the parity tests then cover.
#ifndef GRT_WS_SLOTS
#define GRT_WS_SLOTS GRT_MAX_HITS
#endif

namespace grt {

struct DevTexture {
  int32_t kind;  // grt_texture_kind
  uint32_t width, height;
  uint32_t _pad;
  double beaming;
  const uint32_t* rgba;  // RGBA8 texels, row-major
  double cw, ch;         // checker cell counts
  double c1[4], c2[4];   // checker colours, XYZA
};

struct DevObject {
  int32_t kind;       // grt_object_kind
  int32_t temp_kind;  // grt_temperature_kind
  double radius, R2;  // sphere radius and radius.powi(2)
  double cx, cy, cz;  // sphere centre
  double temperature; // sphere constant temperature
  double rin, rout, rin2, rout2;  // disc annulus
  double temp_constant, r_isco;
  // far-field filter (integrate_kernel): a sphere cannot be hit from a window whose two
  // ends have Cartesian radius outside [shell_lo, shell_hi] (margins 1e-9, see api.hip)
  double shell_lo, shell_hi;
  const double* lut_r;
  const double* lut_t;
  uint32_t lut_n;
  uint32_t _pad;
  DevTexture tex;
  // VolumetricDisc (volumetric_disc.rs:21-95), derived on the host (api.hip)
  double ax[3], e1[3], e2[3];  // normalised axis and in-plane frame (:61-73)
  double thickness, cap_h;     // Gaussian sigma; capture half-height thickness * 3.0 (:454)
  double m_step, m_maxdist;    // raymarch step; step_size * max_steps as f64 (:173)
  uint64_t m_max;              // raymarch samples per intersection
  double dens_mult, bref, sig_a, sig_s, noff, g_fbm;  // g_fbm = (-0.5).exp2() (:331), host libm
  double ns[3];                // noise_scale
  uint32_t octaves, perm_slot; // fBm octaves; index of this object's table in DevScene::perm
  // exact far-field window filter for the capture region (geodesic.hip window_far):
  // vol_far_r = 2 * |capture corner| * (1 + 1e-6); vol_rmax bounds the radii it is
  // used at; vol_slab_h = cap_h * (1 + 1e-6) + 1e-12 (axis == z only, vol_slab_ok)
  double vol_far_r, vol_rmax, vol_slab_h;
  double vol_h_cut;            // |h| beyond which the vertical falloff is < 0.001: 2.62826 thickness (1 + 1e-6)
  int32_t vol_slab_ok, _pad2;
};

struct DevCamera {
  double pos[4];
  double vel[4];
  double tet[4][4];  // rows e_t, e_x, e_y, e_z
  double tan_half_alpha;
  double rows, cols;  // as f64 (camera.rs uses `as f64`)
  double sig_s;       // spatial signature
  double hand;        // spatial handedness
  double sin_theta, cos_theta;  // of pos[2], host libm
};

struct DevScene {
  int32_t geometry;
  uint32_t n_objects;
  double radius, a, horizon_epsilon;
  // horizon test thresholds, evaluated on the host exactly as the reference does
  double horizon_r;     // Schwarzschild: radius + eps; Kerr/KerrBL: r_plus + eps
  int32_t has_horizon;  // Kerr/KerrBL: |a| <= M
  int32_t div_fast;     // radius > 0 (and a) in range: the range-free divisions may run (api.hip)
  double ks_cap;        // Kerr-Schild: coordinate bound of ks_fd_ok, a power of two in 2^10 .. 2^32 (api.hip)
  uint64_t max_steps;
  double max_radius_sq, step_size, epsilon;
  double trapped_radius;  // TRAPPED_ORBIT_RADIUS_FACTOR * radius
  // far-field filter: Cartesian radius of a state is within [r, r + far_a]; the
  // celestial test |x|^2 > max_radius^2 is decided from r outside [cel_lo2, cel_hi2]
  int32_t far_ok;         // geometry has a curvilinear chart (Schwarzschild / KerrBL)
  int32_t div_share;      // radius is a moderate normal: x / r divisions may share 1 / r
  // step controller thresholds (host, 1e-9 margins): err below pow_skip_err proves
  // eps/err > 1800; err below small_lo / above small_hi decides err/eps < 1e-5
  double pow_skip_err, small_lo, small_hi, tiny_err_sq;
  double far_a, cel_lo2, cel_hi2;
  DevCamera cam;
  DevTexture celestial;
  double celestial_temperature;
  double hit_threshold;   // object_hit_opacity_threshold
  double cos_half_pi, sin_half_pi;  // host libm cos(pi/2), sin(pi/2)
  const double* bb_log_t;
  const double* bb_xyz;
  uint32_t bb_n;
  uint32_t _pad1;
  const double* srgb_lin;  // 256 entries
  int32_t has_vol;         // any GRT_OBJ_VOLUMETRIC_DISC: integrate records chord directions and
  int32_t _pad2;           // the frequency data (p_t, p_phi), the shade pass raymarches
  DevObject obj[8];
  uint8_t perm[8][256];    // Perlin permutation tables (noise 0.9.0 PermutationTable), per object
};

// Work description for one launch.
struct WorkList {
  uint32_t row0, col0, rows, cols;  // rows = local rows (this shard's rows when sharded)
  uint32_t tiles_x;       // ceil(cols / 8)
  uint32_t band_rows;     // row-band sharding (grt_row_shard); n_shards <= 1: no sharding
  uint32_t shard, n_shards;
  uint64_t n_items;       // padded tile items, or offset count
  const uint32_t* pixel_index;  // offsets mode (NULL = rectangle mode)
  const double* dx;
  const double* dy;
  const uint32_t* tile_order;   // rectangle mode: queue position -> tile (NULL = row-major)
  // offsets mode, count decided on the device (the adaptive pass): the items actually
  // present are min(*n_live, n_items); n_items is the launch's capacity (NULL = n_items)
  const unsigned long long* n_live;
  // Two-ended queue (probe-ordered traces, n_items < 2^31): the work counter packs the
  // items claimed from the front (low 32 bits) and from the back (high 32 bits).  Of
  // the waves sharing a SIMD, the one in an even hardware wave slot takes the longest
  // predicted items from the front at raised issue priority; the others take the
  // shortest from the back (integrate_kernel).
  uint32_t two_ended;
  uint32_t _pad;
};

// Window candidates of a ray beyond its GRT_WS_SLOTS workspace slots (the reference keeps
// every window's intersection, scene.rs:139-152).  The integrate / tail kernels append
// one record per candidate (one atomic each; rays with more than GRT_WS_SLOTS candidates
// are rare) and link a ray's records in window order through `next`; the shade kernel
// walks that list after the workspace slots.  Structure of arrays with stride `cap`.
// A trace that needs more than `cap` records loses the rest: the pixel gets
// GRT_FLAG_HIT_OVERFLOW and the synchronous entry points grow the pool and trace again.
// The descriptor lives in device memory (Workspace::pool): the kernels load its fields
// only on the rare paths that use them, so the persistent integrate kernels carry one
// pointer for it, not a dozen (their scalar registers are scarce).
constexpr uint32_t HIT_NIL = 0xffffffffu;
struct HitPool {
  uint64_t cap;              // records (< 2^31)
  unsigned long long* count; // [0] records requested by this trace (may exceed cap),
                             // [1] the largest [0] of the traces since the host reset it
  uint32_t* win;             // [cap] window (accepted-step) index
  uint8_t* obj;              // [cap] object index
  double* p;                 // [4][cap] lerped momentum
  double* pt;                // [3][cap] hit point
  uint32_t* next;            // [cap] the ray's next record
  double* hcol;              // [4][cap] shade kernel: colour of a window-nearest hit
  uint32_t* hprev;           // [cap] shade kernel: the ray's previous window-nearest pool record
  double* dir;               // [3][cap] volumetric scenes: chord direction
  double* vcol;              // [4][cap] volumetric scenes: raymarched colour
  uint32_t* head;            // [n] per ray: pool record of candidate GRT_WS_SLOTS
  uint32_t* last;            // [n] per ray: pool record of the last candidate appended,
                             //     HIT_NIL once one was lost
};

// A window candidate in a workspace slot: 64 B, written whole (four 16-B stores) by the
// lane that records it.
struct CandRec {
  double p[4];   // momentum lerped to the hit (objects.rs:27-44)
  double pt[3];  // hit point (sphere-local for spheres)
  uint32_t win;  // window (accepted-step) index
  uint32_t obj;  // object index
};
static_assert(sizeof(CandRec) == 64, "candidate record: one 64-B line");

// Hand-off from the integrate kernel to the shade kernel, n = number of output slots of
// the launch.  Per ray, written once by the lane that ends it, as one 64-B record of
// whole 16-B stores (not one 8-B store per field into structure-of-arrays slots, nor a
// second small record: rays end one by one in probe order, so lines shared by several
// rays were written back part-filled, once per ray): the final state, the constants the
// shade needs, the candidate count, stop reason and status (fin; layout and KerrBL's
// 16-B meta record in geodesic.hip fin_put).  The window candidates: the first GRT_WS_SLOTS in slots (slot-major: slot k
// of ray i at k*n + i, one 64-B record each), the rest in the hit pool.
struct Workspace {
  uint64_t n;
  double* fin;        // [n][8] ray record (64 B, 64-B aligned)
  uint32_t* meta;     // KerrBL: [n][4] steps, candidates, stop | status << 8, 0
  double* rc;         // volumetric scenes only: [6][n] ray constants (observer energy, E, L_z,
                      // Q, p_t, p_phi) written at the ray's start, for the raymarch
  CandRec* rec;       // [MAX][n] candidate records, slot j of ray i at j * n + i
  // volumetric scenes only (NULL otherwise)
  double* rec_dir;    // [3][MAX][n] chord direction y_end - y_start (volumetric candidates)
  double* vcol;       // [4][MAX][n] raymarched colour of volumetric candidate slots
  uint64_t* jobs;     // [MAX * n + pool.cap] raymarch jobs: (ray << 8) | candidate slot, or
                      // JOB_POOL | ray << 31 | pool record
  unsigned long long* march;  // [0] job count, [1] job cursor, [2] samples, [3] jobs (cumulative),
                              // [4] samples that evaluated the noise, [5] samples that emitted
  // rays present when the count is decided on the device: min(*n_live, n) (NULL = n);
  // n stays the SoA stride
  const unsigned long long* n_live;
  const HitPool* pool;  // device memory
  uint32_t* steps;      // optional per-pixel step counts (Outputs::steps), written at the ray's end
};
constexpr uint64_t JOB_POOL = 1ull << 63;

// Local row -> frame row under cyclic row-band sharding: band k of shard s is frame
// band k * n_shards + s (grt_api.h, grt_row_shard).
#if defined(__HIPCC__)
__host__ __device__
#endif
inline uint32_t shard_frame_row(uint32_t band_rows, uint32_t shard, uint32_t n_shards, uint32_t local) {
  if (n_shards <= 1) return local;
  return ((local / band_rows) * n_shards + shard) * band_rows + local % band_rows;
}

#ifndef GRT_INTEGRATE_WAVES
#define GRT_INTEGRATE_WAVES 2  // waves per SIMD of the Kerr-Schild and volumetric integrate kernels
#endif
#ifndef GRT_INTEGRATE_WAVES_LIGHT
#define GRT_INTEGRATE_WAVES_LIGHT 3  // the other integrate kernels (<= 168 VGPRs)
#endif
// Waves per SIMD of integrate_kernel<geometry, vol> (its __launch_bounds__; the launch
// puts twice that many blocks of 256 threads on each CU).  Kerr-Schild's RHS needs ~250
// registers, the volumetric window records more; the Schwarzschild, KerrBL and flat
// kernels fit 168 (measured: C2 -2%, C3 -10% at 3 waves).
#if defined(__HIPCC__)
__host__ __device__
#endif
constexpr int integrate_waves(int geometry, bool vol) {
  return (geometry == 2 /* GRT_GEOM_KERR */ || vol) ? GRT_INTEGRATE_WAVES : GRT_INTEGRATE_WAVES_LIGHT;
}
#ifndef GRT_TAIL_WAVES
#define GRT_TAIL_WAVES 1  // waves per SIMD of the tail kernel: a lone wave owns its SIMD's issue slots
#endif

// Long-ray hand-off (Kerr-Schild).  Once the tile queue is drained and at most
// `threshold` rays are still being integrated, the integrate kernel's waves write their
// rays' loop state here and exit; tail_kernel continues each ray on the 4 lanes of a
// quad (the three acceleration components of the Kerr-Schild RHS in parallel), one
// wave per SIMD.  The split changes who computes a value, never its operations, so every
// result is identical to integrating the ray on one lane (tests/test_tail.py).

struct TailList {
  // [0] live rays (started - ended), [1] rays handed off, [2] tail claim cursor; timeline
  // (s_memrealtime, 100 MHz): [3] integrate start, [4] queue drained, [5] first hand-off,
  // [6] tail kernel end
  unsigned long long* ctl;  // 16 words
  uint64_t cap;             // entries of st (0: hand-off disabled)
  uint64_t threshold;       // hand off once the queue is drained and live <= threshold
  // [16][cap] 64-bit words per entry: y[0..7], c[0..2], h, h_cur, i, output slot,
  // nrec | retries << 32 | c_valid << 48 (no ray constant: only Kerr-Schild hands off,
  // and its RHS, momentum and records read none; the shade kernel recomputes the
  // observer energy from the pixel)
  unsigned long long* st;
};

struct Outputs {
  float* xyza;        // 4 floats per sample
  uint8_t* cls;
  uint8_t* status;
  double* xyza64;     // optional
  uint32_t* steps;    // optional
  uint8_t* stop;      // optional
  uint32_t* hits;     // optional: windows with an intersection (scene.rs:148, before any error)
};

}  // namespace grt
