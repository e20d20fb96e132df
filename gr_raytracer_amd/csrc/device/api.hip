// api.hip — C ABI of the device hot path (include/grt_api.h).
//
// grt_scene_create deep-copies the caller's POD descriptor (textures and LUTs
// included); each GPU receives its own device copy the first time it renders.
// grt_render_pixels replaces Raytracer::render_section_to_cie_buffer_raw
// (raytracer.rs:195-244) and supersample (:320-384); grt_render_section replaces
// render_section_to_cie_buffer[_supersampled] (:177-318).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "grt_api.h"
#include "../host/host_internal.h"
#include "dev_scene.h"
#include "kernels.h"

namespace {

// Process-wide tuning knobs (grt_set_*).  The library is called from one host thread per
// device (grt_render_frame_multi, or a host of its own), so a setter may run beside renders
// on other threads: the knobs are atomics, and a trace reads them once, into a Knobs
// snapshot, so that one call never sees two settings.
std::atomic<long long> g_launch{256};  // grt_set_launch_config: blocks per CU << 16 | threads per block
std::atomic<int> g_range_free{1};      // grt_debug_range_free: 0 = every division and sqrt in its IEEE form (tests)
std::atomic<int> g_schedule{-1};       // grt_set_schedule: -1 auto, 0 row-major tiles, 1 probe-ordered tiles
std::atomic<int> g_two_ended{1};       // grt_set_two_ended: probe-ordered traces take the queue from both ends
std::atomic<long long> g_tail{-1};     // grt_set_tail: -1 auto, 0 off, > 0 hand-off threshold (live rays)
std::atomic<int> g_arith{0};           // grt_set_arithmetic: 0 exact (reference bits), 1 fused (FMA contraction)
constexpr uint32_t PROBE_CAP = 32768;  // upper bound of the probe's step cap

struct Knobs {
  int blocks_per_cu, threads, schedule, two_ended;
  long long tail;
  int arith;
  static Knobs now() {
    const long long l = g_launch.load(std::memory_order_relaxed);
    return Knobs{(int)(l >> 16), (int)(l & 0xffff), g_schedule.load(std::memory_order_relaxed),
                 g_two_ended.load(std::memory_order_relaxed), g_tail.load(std::memory_order_relaxed),
                 g_arith.load(std::memory_order_relaxed)};
  }
};


int fail(int code, const std::string& msg) {
  grt_host::set_error(msg);
  return code;
}
#define HIP_TRY(expr)                                                                    \
  do {                                                                                   \
    hipError_t _e = (expr);                                                              \
    if (_e != hipSuccess) {                                                              \
      (void)hipGetLastError(); /* clear it: a later launch check must not see it */    \
      return fail(-EIO, std::string(#expr) + ": " + hipGetErrorString(_e));             \
    }                                                                                    \
  } while (0)

struct HostTexture {
  std::vector<uint32_t> rgba;
};

struct DeviceCopy {
  std::atomic<bool> ready{false};  // set (release) once the device copy below is complete
  grt::DevScene* d_scene = nullptr;
  std::vector<void*> allocations;
  unsigned long long* d_counter = nullptr;  // [0] work counter, [5..6] hit pool (HitPool::count)
  unsigned long long* d_stats = nullptr;    // [0..3] accepted, attempts, rays, overflows
  // [0] jobs, [1] job cursor, [2] samples, [3] jobs (cumulative), [4] noise samples,
  // [5] emitting samples, [8 + k] march_kernel's claim cursor of object k's pass
  unsigned long long* d_march = nullptr;
  bool vol = false;                         // the scene has VolumetricDiscs
  int cus = 0;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  std::mutex mu;  // calls on one device are serialised
  // the last stream that enqueued work into the shared scratch below (stream_order)
  hipEvent_t ev_busy = nullptr;
  hipStream_t busy_stream = nullptr;
  bool busy = false;
  // integrate -> shade hand-off buffers, grown on demand (bytes per ray: ~1.1 KB)
  uint64_t ws_cap = 0;
  bool ws_vol = false;  // the arena holds the volumetric arrays
  void* ws_mem = nullptr;
  // tile-order scratch (probe counts, keys, indices, order, radix-sort temp), grow-only
  uint64_t sched_tiles = 0;
  void* sched_mem = nullptr;
  // adaptive-pass scratch (section buffers, flags, selection, sort and sub-ray buffers),
  // grow-only: no allocation (and no implicit device synchronisation) between passes
  uint64_t ad_bytes = 0;
  void* ad_mem = nullptr;
  // long-ray hand-off (Kerr-Schild): [0] live, [1] handed off, [2] claim cursor; entries, grow-only
  unsigned long long* d_tail_ctl = nullptr;  // 16 words (TailList::ctl)
  uint64_t tail_cap = 0;
  unsigned long long* tail_mem = nullptr;
  // hit pool: window candidates past a ray's GRT_WS_SLOTS workspace slots, grow-only
  uint64_t pool_cap = 0;
  bool pool_vol = false;
  void* pool_mem = nullptr;
  uint64_t ws_jobs_pool = 0;  // pool capacity the workspace's raymarch job list was sized for
  uint32_t *ws_head = nullptr, *ws_last = nullptr;  // per-ray list ends, carved from the workspace
  grt::HitPool* d_pool = nullptr;  // the descriptor the kernels read (device memory)
  grt::HitPool pool_desc{};        // what *d_pool holds
};

constexpr uint64_t POOL_MIN = 1ull << 20;            // records
constexpr uint64_t POOL_MAX = (1ull << 31) - 1;      // job and list encodings hold 31 bits
std::atomic<uint64_t> g_pool_min{POOL_MIN};         // grt_set_hit_pool_min (tests force a full pool)
uint64_t pool_record_bytes(bool vol) { return 4 + 1 + 4 * 8 + 3 * 8 + 4 + 4 * 8 + 4 + (vol ? 3 * 8 + 4 * 8 : 0); }

// Grow the hit pool to at least `want` records (never shrinks).
int ensure_pool(DeviceCopy& dc, uint64_t want) {
  want = std::min(std::max(want, g_pool_min.load(std::memory_order_relaxed)), POOL_MAX);
  if (want <= dc.pool_cap && dc.pool_mem && (!dc.vol || dc.pool_vol)) return 0;
  want = std::max(want, dc.pool_cap);
  if (dc.pool_mem) {
    (void)hipDeviceSynchronize();  // earlier async launches may still use the old pool
    (void)hipFree(dc.pool_mem);
  }
  dc.pool_mem = nullptr;
  dc.pool_cap = 0;
  if (hipMalloc(&dc.pool_mem, want * pool_record_bytes(dc.vol) + 16 * 256) != hipSuccess) {
    (void)hipGetLastError();
    dc.pool_mem = nullptr;
    return fail(-ENOMEM, "cannot allocate the hit pool");
  }
  dc.pool_cap = want;
  dc.pool_vol = dc.vol;
  return 0;
}

// The scratch of a device (workspace, hit pool, tile order, tail list, adaptive arena) is
// one grow-only set per device and every call carves it from offset 0.  An async call
// on another stream than the previous one first waits for that stream's work in it
// (one event), so two streams never run in the same scratch at once; the call then
// records the event on its own stream (stream_done).
int stream_order(DeviceCopy& dc, hipStream_t st) {
  if (dc.busy && dc.busy_stream != st) HIP_TRY(hipStreamWaitEvent(st, dc.ev_busy, 0));
  return 0;
}
int stream_done(DeviceCopy& dc, hipStream_t st) {
  HIP_TRY(hipEventRecord(dc.ev_busy, st));
  dc.busy_stream = st;
  dc.busy = true;
  return 0;
}

grt::HitPool pool_view(const DeviceCopy& dc) {
  grt::HitPool hp;
  std::memset(&hp, 0, sizeof(hp));
  hp.head = dc.ws_head;
  hp.last = dc.ws_last;
  const uint64_t m = dc.pool_cap;
  char* p = (char*)dc.pool_mem;
  auto take = [&](uint64_t bytes) {
    char* r = p;
    p += (bytes + 255) & ~255ull;
    return (void*)r;
  };
  hp.cap = m;
  hp.count = dc.d_counter + 5;
  hp.p = (double*)take(4 * 8 * m);
  hp.pt = (double*)take(3 * 8 * m);
  hp.hcol = (double*)take(4 * 8 * m);
  hp.win = (uint32_t*)take(4 * m);
  hp.next = (uint32_t*)take(4 * m);
  hp.hprev = (uint32_t*)take(4 * m);
  hp.obj = (uint8_t*)take(m);
  if (dc.pool_vol) {
    hp.dir = (double*)take(3 * 8 * m);
    hp.vcol = (double*)take(4 * 8 * m);
  }
  return hp;
}

// Carve a Workspace for n rays out of the device's grow-only arena.
int ensure_workspace(DeviceCopy& dc, uint64_t n, grt::Workspace* ws) {
  const uint64_t M = GRT_WS_SLOTS;
  const bool vol = dc.vol;
  // ray record (64 B), KerrBL's meta record (16 B), pool list ends (8 B), candidate slots;
  // volumetric scenes: the ray constants (48 B), chord directions, raymarched colours, jobs
  const uint64_t per_ray = 64 + 16 + 8 + M * 64 + (vol ? 6 * 8 + M * (3 * 8 + 4 * 8 + 8) : 0);
  // volumetric scenes: the raymarch job list also holds one job per pool record
  const uint64_t jobs_extra = vol ? dc.pool_cap : 0;
  if (n > dc.ws_cap || (vol && !dc.ws_vol) || jobs_extra > dc.ws_jobs_pool) {
    if (dc.ws_mem) {
      (void)hipDeviceSynchronize();  // earlier async launches may still use the old arena
      (void)hipFree(dc.ws_mem);
    }
    dc.ws_mem = nullptr;
    uint64_t cap = std::max<uint64_t>(n, 1 << 16);
    if (hipMalloc(&dc.ws_mem, cap * per_ray + jobs_extra * 8 + 32 * 256) != hipSuccess) {  // + per-array alignment
      (void)hipGetLastError();
      dc.ws_mem = nullptr;
      dc.ws_cap = 0;
      return fail(-ENOMEM, "cannot allocate the integrate/shade workspace");
    }
    dc.ws_cap = cap;
    dc.ws_vol = vol;
    dc.ws_jobs_pool = jobs_extra;
  }
  uint64_t cap = dc.ws_cap;
  char* p = (char*)dc.ws_mem;
  auto take = [&](uint64_t bytes) {
    char* r = p;
    p += (bytes + 255) & ~255ull;
    return (void*)r;
  };
  ws->n = n;
  ws->fin = (double*)take(64 * cap);
  ws->meta = (uint32_t*)take(16 * cap);
  ws->steps = nullptr;  // launch_trace points it at Outputs::steps
  ws->rc = vol ? (double*)take(6 * 8 * cap) : nullptr;
  ws->rec = (grt::CandRec*)take(M * 64 * cap);
  dc.ws_head = (uint32_t*)take(4 * cap);
  dc.ws_last = (uint32_t*)take(4 * cap);
  ws->rec_dir = ws->vcol = nullptr;
  ws->jobs = nullptr;
  ws->march = dc.d_march;
  ws->n_live = nullptr;
  if (vol) {
    ws->rec_dir = (double*)take(3 * M * 8 * cap);
    ws->vcol = (double*)take(4 * M * 8 * cap);
    ws->jobs = (uint64_t*)take(M * 8 * cap + 8 * dc.ws_jobs_pool);
  }
  // the kernels index with the launch's n, which must not exceed the carved capacity
  if (n > cap) return fail(-ENOMEM, "workspace too small");
  return 0;
}

}  // namespace

struct grt_scene {
  grt_scene_desc desc;
  HostTexture celestial;
  HostTexture obj_tex[GRT_MAX_OBJECTS];
  std::vector<double> lut_r[GRT_MAX_OBJECTS], lut_t[GRT_MAX_OBJECTS];
  std::vector<double> bb_log_t, bb_xyz;
  // one device copy per GPU, created on first use (ensure_device).  Fixed slots, so that a
  // host thread looking up its device never sees the table move under it while another
  // thread creates a copy for its own device.
  static constexpr int MAX_DEVICES = 64;
  std::atomic<DeviceCopy*> devices[MAX_DEVICES] = {};
  std::mutex mu;  // creation of the slots' copies
};

namespace {

void copy_texture(const grt_texture_desc& t, HostTexture& out) {
  if (t.kind == GRT_TEX_BITMAP && t.rgba && t.width && t.height) {
    size_t n = (size_t)t.width * t.height;
    out.rgba.resize(n);
    std::memcpy(out.rgba.data(), t.rgba, n * 4);
  }
}

template <class T>
int upload(DeviceCopy& dc, const T* src, size_t n, T** dst) {
  *dst = nullptr;
  if (n == 0) return 0;
  void* p = nullptr;
  HIP_TRY(hipMalloc(&p, n * sizeof(T)));
  dc.allocations.push_back(p);
  HIP_TRY(hipMemcpy(p, src, n * sizeof(T), hipMemcpyHostToDevice));
  *dst = (T*)p;
  return 0;
}

void fill_dev_texture(const grt_texture_desc& t, grt::DevTexture& d) {
  d.kind = t.kind;
  d.width = t.width;
  d.height = t.height;
  d.beaming = t.beaming_exponent;
  d.rgba = nullptr;
  d.cw = t.checker_width;
  d.ch = t.checker_height;
  for (int k = 0; k < 4; ++k) {
    d.c1[k] = t.c1[k];
    d.c2[k] = t.c2[k];
  }
}

int init_device_copy(grt_scene* s, int device, DeviceCopy& dc);

// The scene's copy on `device`, uploaded on first use.  Safe from one host thread per device
// (and from several threads on one device: the first uploads, the others wait for it).
int ensure_device(grt_scene* s, int device, DeviceCopy** out) {
  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) return fail(-ENODEV, "invalid device ordinal");
  if (device >= grt_scene::MAX_DEVICES) return fail(-ENODEV, "device ordinal beyond the library's 64 slots");
  DeviceCopy* p = s->devices[device].load(std::memory_order_acquire);
  if (!p) {
    std::lock_guard<std::mutex> lk(s->mu);
    p = s->devices[device].load(std::memory_order_acquire);
    if (!p) {
      p = new DeviceCopy();
      s->devices[device].store(p, std::memory_order_release);
    }
  }
  DeviceCopy& dc = *p;
  *out = &dc;
  if (dc.ready.load(std::memory_order_acquire)) return 0;
  std::lock_guard<std::mutex> lk(dc.mu);
  if (dc.ready.load(std::memory_order_acquire)) return 0;
  return init_device_copy(s, device, dc);
}

// The device copy of a scene on `device` if one is complete, else nullptr.
DeviceCopy* find_device(const grt_scene* s, int device) {
  if (device < 0 || device >= grt_scene::MAX_DEVICES) return nullptr;
  DeviceCopy* p = s->devices[device].load(std::memory_order_acquire);
  return (p && p->ready.load(std::memory_order_acquire)) ? p : nullptr;
}

int init_device_copy(grt_scene* s, int device, DeviceCopy& dc) {
  HIP_TRY(hipSetDevice(device));
  const grt_scene_desc& d = s->desc;
  grt::DevScene ds;
  std::memset(&ds, 0, sizeof(ds));
  ds.geometry = d.geometry;
  ds.n_objects = d.n_objects;
  ds.radius = d.radius;
  ds.a = d.a;
  ds.horizon_epsilon = d.horizon_epsilon;
  // horizon thresholds exactly as schwarzschild.rs:181-183, kerr.rs:382-394, kerr_bl.rs:482-492
  if (d.geometry == GRT_GEOM_SCHWARZSCHILD) {
    ds.horizon_r = d.radius + d.horizon_epsilon;
    ds.has_horizon = 1;
  } else if (d.geometry == GRT_GEOM_KERR || d.geometry == GRT_GEOM_KERR_BL) {
    double m = d.geometry == GRT_GEOM_KERR ? 0.5 * d.radius : d.radius / 2.0;
    ds.has_horizon = !(std::fabs(d.a) > d.radius / 2.0);
    double disc = std::fmax(m * m - d.a * d.a, 0.0);
    double rp = m + std::sqrt(disc);
    ds.horizon_r = rp + d.horizon_epsilon;
  }
  ds.max_steps = d.max_steps;
  ds.max_radius_sq = d.max_radius * d.max_radius;
  ds.step_size = d.step_size;
  ds.epsilon = d.epsilon;
  ds.trapped_radius = 5.0 * d.radius;
  // Far-field filter bounds.  The margins (1e-9 relative) are ~1e6 x the rounding of
  // the Cartesian conversion and of the chord arithmetic, so every window the filter
  // skips would have been a miss in the reference too ("Exact skips").
  ds.far_ok = (d.geometry == GRT_GEOM_SCHWARZSCHILD || d.geometry == GRT_GEOM_KERR_BL ||
               d.geometry == GRT_GEOM_EUCLIDEAN_SPHERICAL) ? 1 : 0;
  ds.far_a = d.geometry == GRT_GEOM_KERR_BL ? std::fabs(d.a) : 0.0;
  ds.cel_lo2 = ds.max_radius_sq * (1.0 - 1e-9);
  ds.cel_hi2 = ds.max_radius_sq * (1.0 + 1e-9);
  if (!std::isfinite(ds.far_a) || !std::isfinite(ds.max_radius_sq)) ds.far_ok = 0;
  {
    int ex = 0;
    std::frexp(d.radius, &ex);
    ds.div_share = (std::fpclassify(d.radius) == FP_NORMAL && ex > -500 && ex < 500) ? 1 : 0;
    int ea = 0;
    std::frexp(d.a, &ea);
    // KerrBL: a normal |a| within 2^+-50; Kerr-Schild (ks_fd_ok): radius and a normal
    // within 2^+-20, or a == 0
    const int lim = d.geometry == GRT_GEOM_KERR ? 20 : 50;
    const bool a_mod = std::fpclassify(d.a) == FP_NORMAL && ea > -lim && ea < lim;
    const bool a_ok = d.geometry == GRT_GEOM_KERR_BL ? a_mod : (d.geometry != GRT_GEOM_KERR || a_mod || d.a == 0.0);
    ds.div_fast = (g_range_free.load(std::memory_order_relaxed) && std::fpclassify(d.radius) == FP_NORMAL && d.radius > 0.0 && ex > -lim && ex < lim &&
                   a_ok) ? 1 : 0;
    // ks_fd_ok's coordinate bound: 2^ceil(log2(2 max_radius)) covers every state of a ray
    // (it stops one step beyond max_radius), within the proven 2^10 .. 2^32
    int em = 0;
    const double mr2 = 2.0 * d.max_radius;
    const double m = std::isfinite(mr2) && mr2 > 0.0 ? std::frexp(mr2, &em) : 0.0;
    if (m == 0.5) em -= 1;  // an exact power of two is its own bound
    ds.ks_cap = std::ldexp(1.0, !std::isfinite(mr2) ? 32 : std::min(32, std::max(10, em)));
  }
  {  // exact controller shortcuts (geodesic.hip step_control); off unless epsilon is a moderate normal
    int ex = 0;
    std::frexp(d.epsilon, &ex);
    const bool ok = std::fpclassify(d.epsilon) == FP_NORMAL && d.epsilon > 0.0 && ex > -900 && ex < 900;
    ds.pow_skip_err = ok ? d.epsilon / 1800.0 * (1.0 - 1e-9) : 0.0;
    ds.small_lo = ok ? d.epsilon * 1e-5 * (1.0 - 1e-9) : 0.0;
    ds.small_hi = ok ? d.epsilon * 1e-5 * (1.0 + 1e-9) : HUGE_VAL;
    const double t = std::fmin(ds.pow_skip_err, ds.small_lo);
    ds.tiny_err_sq = (ok && t >= 1e-150) ? t * t * (1.0 - 1e-9) : 0.0;  // t^2 stays a normal
  }
  const grt_camera_desc& c = d.camera;
  for (int k = 0; k < 4; ++k) {
    ds.cam.pos[k] = c.position[k];
    ds.cam.vel[k] = c.velocity[k];
    for (int j = 0; j < 4; ++j) ds.cam.tet[k][j] = c.tetrad[k][j];
  }
  ds.cam.tan_half_alpha = c.tan_half_alpha;
  ds.cam.rows = (double)c.rows;
  ds.cam.cols = (double)c.cols;
  ds.cam.sig_s = c.spatial_signature;
  ds.cam.hand = c.spatial_handedness;
  ds.cam.sin_theta = c.sin_theta;
  ds.cam.cos_theta = c.cos_theta;
  fill_dev_texture(d.celestial, ds.celestial);
  ds.celestial_temperature = d.celestial_temperature;
  ds.hit_threshold = d.object_hit_opacity_threshold;
  ds.cos_half_pi = std::cos(1.57079632679489661923);
  ds.sin_half_pi = std::sin(1.57079632679489661923);
  int rc;
  uint32_t* tex = nullptr;
  if ((rc = upload(dc, s->celestial.rgba.data(), s->celestial.rgba.size(), &tex))) return rc;
  ds.celestial.rgba = tex;
  for (uint32_t k = 0; k < d.n_objects; ++k) {
    const grt_object_desc& o = d.objects[k];
    grt::DevObject& q = ds.obj[k];
    q.kind = o.kind;
    q.temp_kind = o.temp_kind;
    q.radius = o.radius;
    q.R2 = o.radius * o.radius;
    q.cx = o.center[0];
    q.cy = o.center[1];
    q.cz = o.center[2];
    q.temperature = o.temperature;
    q.rin = o.inner_radius;
    q.rout = o.outer_radius;
    q.rin2 = o.inner_radius * o.inner_radius;
    q.rout2 = o.outer_radius * o.outer_radius;
    {
      double cn = std::sqrt(o.center[0] * o.center[0] + o.center[1] * o.center[1] + o.center[2] * o.center[2]);
      double R = std::fabs(o.radius);
      q.shell_lo = (cn - R) * (1.0 - 1e-9) - 1e-9;
      q.shell_hi = (cn + R) * (1.0 + 1e-9) + 1e-9;
      if (!std::isfinite(q.shell_lo) || !std::isfinite(q.shell_hi)) ds.far_ok = 0;
    }
    q.temp_constant = o.temp_constant;
    q.r_isco = o.r_isco;
    q.lut_n = o.lut_n;
    double* lr = nullptr;
    double* lt = nullptr;
    if ((rc = upload(dc, s->lut_r[k].data(), s->lut_r[k].size(), &lr))) return rc;
    if ((rc = upload(dc, s->lut_t[k].data(), s->lut_t[k].size(), &lt))) return rc;
    q.lut_r = lr;
    q.lut_t = lt;
    if (o.kind == GRT_OBJ_VOLUMETRIC_DISC) {  // VolumetricDisc::new (volumetric_disc.rs:43-95)
      dc.vol = true;
      ds.has_vol = 1;
      grt_volumetric_frame(o.axis, q.ax, q.e1, q.e2);
      grt_perlin_permutation(o.perlin_seed, ds.perm[k]);
      q.perm_slot = k;
      q.thickness = o.thickness;
      q.cap_h = o.thickness * 3.0;
      q.m_step = o.march_step_size;
      q.m_max = o.march_max_steps;
      q.m_maxdist = o.march_step_size * (double)o.march_max_steps;
      q.dens_mult = o.density_multiplier;
      q.bref = o.brightness_reference_temperature;
      q.sig_a = o.absorption;
      q.sig_s = o.scattering;
      q.noff = o.noise_offset;
      q.g_fbm = std::exp2(-0.5);
      for (int i = 0; i < 3; ++i) q.ns[i] = o.noise_scale[i];
      q.octaves = o.num_octaves;
      // far-field filter bounds (geodesic.hip vol_far)
      const double corner = std::sqrt(o.outer_radius * o.outer_radius + q.cap_h * q.cap_h);
      q.vol_far_r = 2.0 * corner * (1.0 + 1e-6);
      q.vol_rmax = 1e6 * q.cap_h;
      q.vol_slab_h = q.cap_h * (1.0 + 1e-6) + 1e-12;
      q.vol_h_cut = std::sqrt(std::log(1000.0)) * o.thickness * (1.0 + 1e-6);  // exp(-(h/th)^2) < 0.001 beyond
      q.vol_slab_ok = (q.ax[0] == 0.0 && q.ax[1] == 0.0 && q.ax[2] == 1.0) ? 1 : 0;
      if (!std::isfinite(q.vol_far_r) || !std::isfinite(q.vol_rmax) || !(q.cap_h > 0.0)) {
        q.vol_far_r = HUGE_VAL;
        q.vol_rmax = 0.0;
        q.vol_slab_ok = 0;
      }
    }
    fill_dev_texture(o.texture, q.tex);
    uint32_t* ot = nullptr;
    if ((rc = upload(dc, s->obj_tex[k].rgba.data(), s->obj_tex[k].rgba.size(), &ot))) return rc;
    q.tex.rgba = ot;
  }
  double *bl = nullptr, *bx = nullptr, *sl = nullptr;
  if ((rc = upload(dc, s->bb_log_t.data(), s->bb_log_t.size(), &bl))) return rc;
  if ((rc = upload(dc, s->bb_xyz.data(), s->bb_xyz.size(), &bx))) return rc;
  if ((rc = upload(dc, d.srgb_to_linear, 256, &sl))) return rc;
  ds.bb_log_t = bl;
  ds.bb_xyz = bx;
  ds.bb_n = d.bb_n;
  ds.srgb_lin = sl;
  grt::DevScene* dsp = nullptr;
  if ((rc = upload(dc, &ds, 1, &dsp))) return rc;
  dc.d_scene = dsp;
  void* p = nullptr;
  HIP_TRY(hipMalloc(&p, (16 + 8 + GRT_MAX_OBJECTS) * sizeof(unsigned long long)));
  dc.allocations.push_back(p);
  HIP_TRY(hipMemset(p, 0, (16 + 8 + GRT_MAX_OBJECTS) * sizeof(unsigned long long)));
  dc.d_counter = (unsigned long long*)p;
  dc.d_stats = dc.d_counter + 1;
  dc.d_march = dc.d_counter + 8;
  HIP_TRY(hipMalloc(&p, 16 * sizeof(unsigned long long)));
  dc.allocations.push_back(p);
  HIP_TRY(hipMemset(p, 0, 16 * sizeof(unsigned long long)));
  dc.d_tail_ctl = (unsigned long long*)p;
  HIP_TRY(hipMalloc(&p, sizeof(grt::HitPool)));
  dc.allocations.push_back(p);
  HIP_TRY(hipMemset(p, 0, sizeof(grt::HitPool)));
  dc.d_pool = (grt::HitPool*)p;
  hipDeviceProp_t prop;
  HIP_TRY(hipGetDeviceProperties(&prop, device));
  dc.cus = prop.multiProcessorCount;
  int occ = 0;
  void (*kfn)() = nullptr;
  (void)kfn;
  HIP_TRY(hipEventCreate(&dc.ev0));
  HIP_TRY(hipEventCreate(&dc.ev1));
  HIP_TRY(hipEventCreateWithFlags(&dc.ev_busy, hipEventDisableTiming));
  (void)occ;
  dc.ready.store(true, std::memory_order_release);
  return 0;
}

grt::WorkList rect_worklist(uint32_t row0, uint32_t col0, uint32_t rows, uint32_t cols) {
  grt::WorkList wl;
  std::memset(&wl, 0, sizeof(wl));
  wl.row0 = row0;
  wl.col0 = col0;
  wl.rows = rows;
  wl.cols = cols;
  wl.tiles_x = (cols + 7) / 8;
  uint64_t tiles_y = (rows + 7) / 8;
  wl.n_items = (uint64_t)wl.tiles_x * tiles_y * 64;
  return wl;
}

// Step cap of the probe rays (scheduling only).  The pass lasts as long as its capped
// probes (horizon creepers) take to run the cap.  An escaping ray needs about max_radius
// accepted steps at H_MAX = 1 (C4: 15825-15900 for max_radius 15000), so the cap is
// 1.3 x max_radius, which tells them from the long rays.  A Kerr-Schild probe moving
// outward far from the hole ends at once with a key just below the cap (probe_escaped,
// round 5), so for Kerr-Schild the cap no longer has to outlast the escaping rays:
// 0.3 x max_radius (C4: 4,500 steps; C4 shard 2 0.51 -> 0.09 s before the integrate
// kernel, the integrate kernel's own time unchanged, profiles/r05aj, r05ak).  The other
// charts have no such shortcut and keep 1.3 x: with the short cap their escaping probes
// would end capped, keyed by their distance to the horizon, ahead of the long rays.
static uint32_t probe_cap(const grt_scene* s) {
  const double scale = s->desc.geometry == GRT_GEOM_KERR ? 0.3 : 1.3;
  const double c = scale * s->desc.max_radius;
  return c >= (double)PROBE_CAP ? PROBE_CAP : (c <= 4096.0 ? 4096u : (uint32_t)c);
}

// Probe-ordered tile queue (schedule.hip): worth its ~1/64 extra rays when a ray may run
// far longer than an escaping one (max_steps well above the probe cap) over many tiles,
// in the affine-parameter charts.  KerrBL integrates in Mino time, where even captured
// rays take ~1e3 steps (C3: max 1147), and Euclidean rays are straight lines: there the
// probe pass is pure overhead (measured +5% on C3), so automatic mode skips them.
bool schedule_wanted(const grt_scene* s, const grt::WorkList& wl, const Knobs& k) {
  if (wl.pixel_index || k.schedule == 0) return false;
  const uint64_t tiles = wl.n_items / 64;
  if (k.schedule == 1) return tiles > 1;
  const int g = s->desc.geometry;
  return (g == GRT_GEOM_KERR || g == GRT_GEOM_SCHWARZSCHILD) && s->desc.max_steps >= 8ull * PROBE_CAP &&
         tiles >= 1024;
}
// Schwarzschild frames the probe pass is not worth (automatic mode): the tile order from
// each tile's impact parameter instead (impact_key_kernel; no integration, ~0.1 ms).  C2
// one frame alone 1,280-1,282 -> 1,263-1,271 ms; two frames in flight unchanged
// (1,234-1,241 against 1,240 ms), and with the two-ended queue slower (1,253 ms); frames
// identical (profiles/r06x).
bool impact_wanted(const grt_scene* s, const grt::WorkList& wl, const Knobs& k) {
  return !wl.pixel_index && k.schedule == -1 && s->desc.geometry == GRT_GEOM_SCHWARZSCHILD &&
         wl.n_items / 64 >= 1024 && !schedule_wanted(s, wl, k);
}

// Enqueue the probe pass and the sort; returns the device tile order in *order.
// quad: the Kerr-Schild probe on quads, -1 automatic, 0 never, 1 always (grt_debug_probe_keys).
int enqueue_tile_order(grt_scene* s, DeviceCopy& dc, const grt::WorkList& wl, hipStream_t stream,
                       const uint32_t** order, int quad_mode = -1, bool impact = false) {
  const uint32_t tiles_x = wl.tiles_x, tiles_y = (uint32_t)(wl.n_items / 64 / wl.tiles_x);
  const uint64_t n = (uint64_t)tiles_x * tiles_y;
  size_t temp_bytes = 0;
  HIP_TRY(grt::launch_tile_order(nullptr, tiles_x, tiles_y, 0, nullptr, nullptr, nullptr, nullptr, nullptr,
                                 &temp_bytes, stream));
  const uint64_t need = 5 * ((n * 4 + 255) & ~255ull) + temp_bytes + 256;
  if (n > dc.sched_tiles || !dc.sched_mem) {
    if (dc.sched_mem) {
      (void)hipDeviceSynchronize();
      (void)hipFree(dc.sched_mem);
      dc.sched_mem = nullptr;
    }
    dc.sched_tiles = 0;
    // room for a frame of the same tile count with a larger radix-sort temp
    HIP_TRY(hipMalloc(&dc.sched_mem, need + (need >> 2)));
    dc.sched_tiles = n;
  }
  char* p = (char*)dc.sched_mem;
  auto take = [&](uint64_t bytes) {
    char* r = p;
    p += (bytes + 255) & ~255ull;
    return r;
  };
  uint32_t* probe = (uint32_t*)take(n * 4);
  uint32_t* keys = (uint32_t*)take(n * 4);
  uint32_t* keys_sorted = (uint32_t*)take(n * 4);
  uint32_t* idx = (uint32_t*)take(n * 4);
  uint32_t* ord = (uint32_t*)take(n * 4);
  void* temp = take(temp_bytes);
  if (impact) {  // predicted lengths, no probe rays; no key counts as capped
    HIP_TRY(grt::launch_impact_keys(dc.d_scene, wl, (uint32_t)n, probe, stream));
    HIP_TRY(grt::launch_tile_order(probe, tiles_x, tiles_y, 0xffffffffu, keys, keys_sorted, idx, ord, temp, &temp_bytes,
                                   stream));
    *order = ord;
    return 0;
  }
  const uint32_t cap = probe_cap(s);
  // Kerr-Schild probe rays on quads when they fill at most 2 waves per SIMD that way
  // (probe_quad_kernel: a C4 1/8 shard's 32,768 probes); above that the one-lane probe,
  // whose pass is then bound by its work, not by one probe's latency
  const bool quad = quad_mode > 0 || (quad_mode < 0 && n <= (uint64_t)dc.cus * 128);
  HIP_TRY(grt::launch_probe(s->desc.geometry, dc.d_scene, wl, (uint32_t)n, cap, probe, quad, stream));
  HIP_TRY(grt::launch_tile_order(probe, tiles_x, tiles_y, cap, keys, keys_sorted, idx, ord, temp, &temp_bytes, stream));
  *order = ord;
  return 0;
}

// Long-ray hand-off of a Kerr-Schild trace (TailList, dev_scene.h): the tail kernel runs
// one block of 4 waves per CU per GRT_TAIL_WAVES, 64 rays per block (a quad each); by
// default the integrate kernel hands off once the queue is drained and no more rays are
// live than the tail kernel integrates at once.  A lane holds at most one ray, so the
// entry arena needs one entry per integrate lane whatever the threshold.
int tail_list(const grt_scene* s, DeviceCopy& dc, uint64_t lanes, long long tail, grt::TailList* tl,
              int* tail_blocks) {
  std::memset(tl, 0, sizeof(*tl));
  *tail_blocks = 0;
  if (s->desc.geometry != GRT_GEOM_KERR || tail == 0) return 0;
  const int blocks = dc.cus * GRT_TAIL_WAVES;
  const uint64_t threshold = tail > 0 ? (uint64_t)tail : (uint64_t)blocks * grt::TAIL_RAYS_PER_BLOCK;
  const uint64_t cap = lanes;
  if (cap > dc.tail_cap) {
    if (dc.tail_mem) {
      (void)hipDeviceSynchronize();
      (void)hipFree(dc.tail_mem);
      dc.tail_mem = nullptr;
    }
    dc.tail_cap = 0;
    HIP_TRY(hipMalloc(&dc.tail_mem, cap * 16 * sizeof(unsigned long long)));
    dc.tail_cap = cap;
  }
  tl->ctl = dc.d_tail_ctl;
  tl->cap = dc.tail_cap;
  tl->threshold = threshold;
  tl->st = dc.tail_mem;
  *tail_blocks = blocks;
  return 0;
}

#if GRT_RAY_TIMES
// Diagnostic builds: the per-ray schedule record of the last trace ([6][n] words,
// geodesic.hip), one process-wide buffer (single-device diagnostics).
unsigned long long* g_rt = nullptr;
uint64_t g_rt_cap = 0, g_rt_n = 0;
uint64_t g_rt_trace = 0, g_rt_only = 0;  // record only trace g_rt_only since grt_debug_ray_times_only (0: each)
int ray_times_reserve(uint64_t n, hipStream_t stream) {
  ++g_rt_trace;
  if (g_rt_only && g_rt_trace != g_rt_only) {  // another trace: it records nothing
    HIP_TRY(hipDeviceSynchronize());          // the recorded kernel may still be running
    HIP_TRY(grt::set_ray_times(nullptr));
    return 0;
  }
  if (n > g_rt_cap) {
    if (g_rt) {
      (void)hipDeviceSynchronize();
      (void)hipFree(g_rt);
    }
    g_rt = nullptr;
    g_rt_cap = 0;
    HIP_TRY(hipMalloc(&g_rt, n * 6 * 8));
    g_rt_cap = n;
  }
  g_rt_n = n;
  HIP_TRY(hipMemsetAsync(g_rt, 0, n * 6 * 8, stream));
  HIP_TRY(grt::set_ray_times(g_rt));
  return 0;
}
#endif

// Enqueue one trace over `wl` on `stream`; counters are zeroed first.
int enqueue_trace(grt_scene* s, DeviceCopy& dc, const grt::WorkList& wl_in, const grt::Outputs& o,
                  unsigned long long* d_stats, hipStream_t stream) {
  grt::WorkList wl = wl_in;
  const Knobs k = Knobs::now();
  if (int rc0 = stream_order(dc, stream)) return rc0;
  if (schedule_wanted(s, wl, k)) {
    int rc0 = enqueue_tile_order(s, dc, wl, stream, &wl.tile_order);
    if (rc0) return rc0;
    // longest tiles to the priority wave of each SIMD, shortest to the others (WorkList)
    wl.two_ended = (k.two_ended != 0 && wl.n_items < (1ull << 31)) ? 1u : 0u;
  } else if (impact_wanted(s, wl, k)) {
    int rc0 = enqueue_tile_order(s, dc, wl, stream, &wl.tile_order, -1, true);
    if (rc0) return rc0;
  }
  HIP_TRY(hipMemsetAsync(dc.d_counter, 0, sizeof(unsigned long long), stream));
  if (dc.vol) {  // jobs, cursor; the march passes' cursors
    HIP_TRY(hipMemsetAsync(dc.d_march, 0, 2 * sizeof(unsigned long long), stream));
    HIP_TRY(hipMemsetAsync(dc.d_march + 8, 0, GRT_MAX_OBJECTS * sizeof(unsigned long long), stream));
  }
  int threads = k.threads ? k.threads : 256;
  int blocks = k.blocks_per_cu > 0 ? dc.cus * k.blocks_per_cu
                                   : dc.cus * 2 * grt::integrate_waves(s->desc.geometry, dc.vol);
  // never launch more lanes than there is work for
  uint64_t max_blocks = (wl.n_items + threads - 1) / threads;
  if ((uint64_t)blocks > max_blocks) blocks = (int)std::max<uint64_t>(1, max_blocks);
  uint64_t n_out = wl.pixel_index ? wl.n_items : (uint64_t)wl.rows * wl.cols;
  grt::Workspace ws;
  // the pool starts at its minimum (grt_set_hit_pool_min) and only grows from a trace's
  // measured need: the synchronous calls' re-trace of flagged pixels, grt_hit_pool_reserve
  int rc = ensure_pool(dc, 0);
  if (rc) return rc;
  rc = ensure_workspace(dc, n_out, &ws);
  if (rc) return rc;
  ws.n_live = wl.n_live;
  {  // the pool descriptor changes only when the pool or the workspace arena moved
    const grt::HitPool hp = pool_view(dc);
    if (std::memcmp(&hp, &dc.pool_desc, sizeof(hp)) != 0) {
      HIP_TRY(hipDeviceSynchronize());  // no kernel in flight reads the old one
      HIP_TRY(hipMemcpy(dc.d_pool, &hp, sizeof(hp), hipMemcpyHostToDevice));
      dc.pool_desc = hp;
    }
  }
  ws.pool = dc.d_pool;
  HIP_TRY(hipMemsetAsync(dc.pool_desc.count, 0, sizeof(unsigned long long), stream));
#if GRT_RAY_TIMES
  if ((rc = ray_times_reserve(n_out, stream))) return rc;
#endif
  grt::TailList tl;
  int tail_blocks = 0;
  rc = tail_list(s, dc, blocks * (uint64_t)threads, k.tail, &tl, &tail_blocks);
  if (rc) return rc;
  if (tl.cap) HIP_TRY(hipMemsetAsync(dc.d_tail_ctl, 0, 16 * sizeof(unsigned long long), stream));
  // grt_set_arithmetic(1): the light charts' kernels built with FMA contraction
  // (geodesic_fused.hip); Kerr-Schild always runs the exact ones
  const bool fused = k.arith == 1 && s->desc.geometry != GRT_GEOM_KERR;
  const auto launch = fused ? grt::fused::launch_trace
                            : (s->desc.geometry == GRT_GEOM_KERR_BL ? grt::kerr_bl::launch_trace : grt::launch_trace);
  // the exact KerrBL kernels are a unit of their own (geodesic_kerr_bl.hip)
  HIP_TRY(launch(s->desc.geometry, dc.d_scene, wl, ws, o, dc.d_counter, d_stats, blocks, threads, dc.vol, tl,
                 tail_blocks, stream));
  return stream_done(dc, stream);
}

struct DevBuf {
  void* p = nullptr;
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
  int alloc(size_t n) {
    if (n == 0) n = 16;
    HIP_TRY(hipMalloc(&p, n));
    return 0;
  }
};

int validate_desc(const grt_scene_desc* d) {
  if (!d) return fail(-EINVAL, "null scene descriptor");
  if (d->abi_version != GRT_ABI_VERSION) return fail(-EINVAL, "grt_scene_desc ABI version mismatch");
  if (d->geometry < GRT_GEOM_EUCLIDEAN || d->geometry > GRT_GEOM_EUCLIDEAN_SPHERICAL)
    return fail(-EINVAL, "unknown geometry");
  if (d->n_objects > GRT_MAX_OBJECTS) return fail(-EINVAL, "too many objects");
  auto check_tex = [&](const grt_texture_desc& t) -> int {
    if (t.kind == GRT_TEX_BITMAP && (!t.rgba || !t.width || !t.height)) return fail(-EINVAL, "bitmap texture without texels");
    if (t.kind == GRT_TEX_BLACKBODY && (d->bb_n < 2 || !d->bb_log_t || !d->bb_xyz))
      return fail(-EINVAL, "blackbody texture without LUT");
    if (t.kind < GRT_TEX_BITMAP || t.kind > GRT_TEX_BLACKBODY) return fail(-EINVAL, "unknown texture kind");
    return 0;
  };
  int rc;
  if ((rc = check_tex(d->celestial))) return rc;
  for (uint32_t k = 0; k < d->n_objects; ++k) {
    const grt_object_desc& o = d->objects[k];
    if (o.kind != GRT_OBJ_SPHERE && o.kind != GRT_OBJ_DISC && o.kind != GRT_OBJ_VOLUMETRIC_DISC)
      return fail(-EINVAL, "unknown object kind");
    if ((rc = check_tex(o.texture))) return rc;
    if (o.kind != GRT_OBJ_SPHERE && o.temp_kind == GRT_TEMP_KERR_LUT && (o.lut_n < 2 || !o.lut_r || !o.lut_t))
      return fail(-EINVAL, "disc temperature LUT missing");
    if (o.kind == GRT_OBJ_VOLUMETRIC_DISC &&
        (!(o.outer_radius > o.inner_radius) || !(o.thickness > 0.0) || o.march_max_steps == 0 ||
         !(o.march_step_size > 0.0) || !(o.brightness_reference_temperature > 0.0) || !(o.absorption >= 0.0) ||
         !(o.scattering >= 0.0)))
      return fail(-EINVAL, "invalid VolumetricDisc parameters (cli/shared.rs:238-284)");
  }
  if (d->camera.rows <= 0 || d->camera.cols <= 0) return fail(-EINVAL, "camera has no pixels");
  return 0;
}

}  // namespace

namespace grt_host {
void scene_frame_size(const grt_scene* s, int64_t* rows, int64_t* cols) {
  *rows = s->desc.camera.rows;
  *cols = s->desc.camera.cols;
}
}  // namespace grt_host

extern "C" {

int grt_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int grt_set_launch_config(int blocks_per_cu, int threads_per_block) {
  if (blocks_per_cu < 0 || threads_per_block < 0 || threads_per_block % 64 != 0 || threads_per_block > 256)
    return fail(-EINVAL, "launch config: threads must be a multiple of 64 and <= 256");
  g_launch.store(((long long)blocks_per_cu << 16) | (threads_per_block ? threads_per_block : 256));
  return 0;
}

int grt_set_tail(long long threshold) {
  if (threshold < -1) return fail(-EINVAL, "tail threshold must be -1 (auto), 0 (off) or a ray count");
  g_tail.store(threshold);
  return 0;
}

int grt_tail_handoffs(grt_scene* scene, int device, uint64_t* handed_off) {
  return grt_tail_report(scene, device, handed_off, nullptr, nullptr, nullptr, 0);
}

int grt_tail_report(grt_scene* scene, int device, uint64_t* handed_off, double timeline_s[3], uint64_t* slot,
                    uint64_t* step, uint64_t capacity) {
  if (!scene || !handed_off) return fail(-EINVAL, "null argument");
  *handed_off = 0;
  if (timeline_s) timeline_s[0] = timeline_s[1] = timeline_s[2] = 0.0;
  DeviceCopy* dcp = find_device(scene, device);
  if (!dcp) return 0;
  DeviceCopy& dc = *dcp;
  std::lock_guard<std::mutex> lock(dc.mu);
  HIP_TRY(hipSetDevice(device));
  unsigned long long v[16];
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpy(v, dc.d_tail_ctl, sizeof(v), hipMemcpyDeviceToHost));
  *handed_off = v[1];
  if (timeline_s) {  // s_memrealtime ticks at 100 MHz
    auto since = [&](unsigned long long t) { return (t && v[3]) ? (double)(long long)(t - v[3]) * 1e-8 : 0.0; };
    timeline_s[0] = since(v[4]);
    timeline_s[1] = since(v[5]);
    timeline_s[2] = since(v[6]);
  }
  const uint64_t n = std::min<uint64_t>(std::min<uint64_t>(v[1], dc.tail_cap), capacity);
  if (n && dc.tail_mem) {
    if (slot) HIP_TRY(hipMemcpy(slot, dc.tail_mem + 14 * dc.tail_cap, n * 8, hipMemcpyDeviceToHost));
    if (step) HIP_TRY(hipMemcpy(step, dc.tail_mem + 13 * dc.tail_cap, n * 8, hipMemcpyDeviceToHost));
  }
  return 0;
}

#if GRT_RAY_TIMES
// Diagnostic builds only (not in grt_api.h): the probe pass and tile order of a row-band
// shard, without the trace: probe keys (n_tiles) and the queue order (n_tiles).
int grt_debug_probe_order(grt_scene* s, int device, const grt_row_shard* sh, uint32_t* probe_out,
                          uint32_t* order_out, uint64_t n_tiles) {
  if (!s || !sh || !probe_out || !order_out) return fail(-EINVAL, "null argument");
  DeviceCopy* dc;
  int rc;
  if ((rc = ensure_device(s, device, &dc))) return rc;
  HIP_TRY(hipSetDevice(device));
  grt::WorkList wl = rect_worklist(0, 0, grt_shard_row_count((uint32_t)s->desc.camera.rows, sh),
                                   (uint32_t)s->desc.camera.cols);
  wl.band_rows = sh->band_rows;
  wl.shard = sh->shard;
  wl.n_shards = sh->n_shards;
  if (wl.n_items / 64 != n_tiles) return fail(-EINVAL, "tile count differs");
  const uint32_t* order = nullptr;
  if ((rc = enqueue_tile_order(s, *dc, wl, nullptr, &order))) return rc;
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpy(probe_out, dc->sched_mem, n_tiles * 4, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(order_out, order, n_tiles * 4, hipMemcpyDeviceToHost));
  return 0;
}

// Diagnostic builds only (not in grt_api.h): record the schedule of the k-th trace from
// now on (and of no other), or of every trace (k = 0): C5's supersample chunk is trace 2.
int grt_debug_ray_times_only(uint64_t k) {
  g_rt_only = k;
  g_rt_trace = 0;
  return 0;
}

// Diagnostic builds only (not in grt_api.h): the last trace's per-ray schedule record,
// [6][n] words (start, hand-off, end, hardware place, integrate / tail attempts), and
// the integrate kernel's start (s_memrealtime) in *t0.
int grt_debug_ray_times(grt_scene* scene, int device, uint64_t* out, uint64_t n, uint64_t* t0) {
  if (!scene || !out || !t0) return fail(-EINVAL, "null argument");
  if (n != g_rt_n || !g_rt) return fail(-EINVAL, "ray count differs from the last trace");
  DeviceCopy* dcp = find_device(scene, device);
  if (!dcp) return fail(-EINVAL, "no trace on this device");
  DeviceCopy& dc = *dcp;
  HIP_TRY(hipSetDevice(device));
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpy(out, g_rt, n * 6 * 8, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(t0, dc.d_tail_ctl + 3, 8, hipMemcpyDeviceToHost));
  return 0;
}
#endif

// Test hook (not in grt_api.h): the probe keys (probe_kernel / probe_quad_kernel) of a
// row-band shard with the probe forced onto quads (quad = 1) or onto one lane per ray (0),
// or the Schwarzschild impact-parameter keys (quad = 2, impact_key_kernel).
int grt_debug_probe_keys(grt_scene* s, int device, const grt_row_shard* sh, int quad, uint32_t* keys_out,
                         uint64_t n_tiles) {
  if (!s || !sh || !keys_out || quad < 0 || quad > 2) return fail(-EINVAL, "probe keys: bad argument");
  if (quad == 2 && s->desc.geometry != GRT_GEOM_SCHWARZSCHILD) return fail(-EINVAL, "impact keys: Schwarzschild only");
  DeviceCopy* dc;
  int rc;
  if ((rc = ensure_device(s, device, &dc))) return rc;
  std::lock_guard<std::mutex> lk(dc->mu);
  HIP_TRY(hipSetDevice(device));
  grt::WorkList wl = rect_worklist(0, 0, grt_shard_row_count((uint32_t)s->desc.camera.rows, sh),
                                   (uint32_t)s->desc.camera.cols);
  wl.band_rows = sh->band_rows;
  wl.shard = sh->shard;
  wl.n_shards = sh->n_shards;
  if (wl.n_items / 64 != n_tiles || wl.n_items % 64 != 0) return fail(-EINVAL, "tile count differs");
  const uint32_t* order = nullptr;
  if ((rc = enqueue_tile_order(s, *dc, wl, nullptr, &order, quad == 2 ? -1 : quad, quad == 2))) return rc;
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpy(keys_out, dc->sched_mem, n_tiles * 4, hipMemcpyDeviceToHost));
  return 0;
}

// Test hook (not in grt_api.h): the range-free divisions and square root (geodesic.hip
// div_inrange, div2_inrange, div_fx, sqrt_fx) against the compiler's over the exponent
// plane (arith_map_kernel): map[2047 * 2047], zmap[2047], smap[2047] flag bytes.
int grt_debug_arith_map(int device, uint32_t samples, uint64_t seed, uint8_t* map, uint8_t* zmap, uint8_t* smap) {
  if (!map || !zmap || !smap || samples == 0 || samples > 4096) return fail(-EINVAL, "arith map: 1 <= samples <= 4096");
  HIP_TRY(hipSetDevice(device));
  const size_t nm = 2047u * 2047u;
  DevBuf b;
  int rc = b.alloc(nm + 2 * 2047);
  if (rc) return rc;
  uint8_t* d = (uint8_t*)b.p;
  HIP_TRY(hipMemset(d, 0, nm + 2 * 2047));
  HIP_TRY(grt::launch_arith_map(samples, seed, d, d + nm, d + nm + 2047, nullptr));
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpy(map, d, nm, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(zmap, d + nm, 2047, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(smap, d + nm + 2047, 2047, hipMemcpyDeviceToHost));
  return 0;
}

// Test hook (not in grt_api.h): the scene's RHS in its range-free and IEEE forms on n
// host states (8 doubles each; KerrBL: e, l_z, q per state in consts), out[16 n], pred[n]
// (rhs_check_kernel).
int grt_debug_rhs_check(grt_scene* s, int device, uint64_t n, const double* states, const double* consts,
                        double* out, uint8_t* pred) {
  if (!s || !states || !out || !pred || n == 0 || n > (1ull << 26)) return fail(-EINVAL, "rhs check: 1 <= n <= 2^26");
  const int g = s->desc.geometry;
  if (g != GRT_GEOM_SCHWARZSCHILD && g != GRT_GEOM_KERR && g != GRT_GEOM_KERR_BL)
    return fail(-EINVAL, "rhs check: Schwarzschild, Kerr-Schild or KerrBL");
  if (g == GRT_GEOM_KERR_BL && !consts) return fail(-EINVAL, "rhs check: KerrBL needs e, l_z, q per state");
  DeviceCopy* dc;
  int rc = ensure_device(s, device, &dc);
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(dc->mu);
  HIP_TRY(hipSetDevice(device));
  DevBuf b_st, b_c, b_out, b_pred;
  if ((rc = b_st.alloc(n * 64)) || (rc = b_c.alloc(n * 24)) || (rc = b_out.alloc(n * 128)) || (rc = b_pred.alloc(n)))
    return rc;
  HIP_TRY(hipMemcpy(b_st.p, states, n * 64, hipMemcpyHostToDevice));
  if (consts) HIP_TRY(hipMemcpy(b_c.p, consts, n * 24, hipMemcpyHostToDevice));
  HIP_TRY(grt::launch_rhs_check(g, dc->d_scene, (const double*)b_st.p, (const double*)b_c.p, n, (double*)b_out.p,
                                (uint8_t*)b_pred.p, nullptr));
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpy(out, b_out.p, n * 128, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(pred, b_pred.p, n, hipMemcpyDeviceToHost));
  return 0;
}

#if GRT_PATH_COUNT
// Diagnostic builds only (not in grt_api.h): the integrate kernels' path counters since the
// last reset (geodesic.hip path_count): out[16], [k] wave-level, [8 + k] lane-level.
int grt_debug_path_counts(uint64_t* out, int reset) {
  if (!out) return fail(-EINVAL, "null argument");
  HIP_TRY(grt::path_read((unsigned long long*)out, reset != 0));
  return 0;
}
#endif

// Test hook (not in grt_api.h): 0 makes the device copies of scenes created (first rendered)
// afterwards run every division and square root of the RHS in the compiler's IEEE form
// (DevScene::div_fast = 0), so a test can hold the range-free forms to them end to end.
int grt_debug_range_free(int on) {
  if (on != 0 && on != 1) return fail(-EINVAL, "range-free arithmetic: 0 or 1");
  g_range_free.store(on);
  return 0;
}

int grt_set_arithmetic(int mode) {
  if (mode != 0 && mode != 1) return fail(-EINVAL, "arithmetic: 0 (exact) or 1 (fused)");
  g_arith.store(mode);
  return 0;
}

int grt_get_arithmetic(void) { return g_arith.load(); }

int grt_set_two_ended(int on) {
  if (on != 0 && on != 1) return fail(-EINVAL, "two-ended queue: 0 or 1");
  g_two_ended.store(on);
  return 0;
}

int grt_set_schedule(int mode) {
  if (mode < -1 || mode > 1) return fail(-EINVAL, "schedule mode must be -1 (auto), 0 or 1");
  g_schedule.store(mode);
  return 0;
}

int grt_scene_create(const grt_scene_desc* desc, grt_scene** out) {
  if (!out) return fail(-EINVAL, "null output pointer");
  int rc = validate_desc(desc);
  if (rc) return rc;
  grt_scene* s = new grt_scene();
  s->desc = *desc;
  copy_texture(desc->celestial, s->celestial);
  for (uint32_t k = 0; k < desc->n_objects; ++k) {
    const grt_object_desc& o = desc->objects[k];
    copy_texture(o.texture, s->obj_tex[k]);
    if (o.lut_n) {
      s->lut_r[k].assign(o.lut_r, o.lut_r + o.lut_n);
      s->lut_t[k].assign(o.lut_t, o.lut_t + o.lut_n);
    }
  }
  if (desc->bb_n) {
    s->bb_log_t.assign(desc->bb_log_t, desc->bb_log_t + desc->bb_n);
    s->bb_xyz.assign(desc->bb_xyz, desc->bb_xyz + 3 * (size_t)desc->bb_n);
  }
  // the copy owns its arrays now
  s->desc.celestial.rgba = nullptr;
  for (uint32_t k = 0; k < desc->n_objects; ++k) {
    s->desc.objects[k].texture.rgba = nullptr;
    s->desc.objects[k].lut_r = nullptr;
    s->desc.objects[k].lut_t = nullptr;
  }
  s->desc.bb_log_t = nullptr;
  s->desc.bb_xyz = nullptr;
  *out = s;
  return 0;
}

int grt_scene_destroy(grt_scene* s) {
  if (!s) return 0;
  for (int dev = 0; dev < grt_scene::MAX_DEVICES; ++dev) {
    DeviceCopy* dc = s->devices[dev].load(std::memory_order_acquire);
    if (!dc) continue;
    (void)hipSetDevice((int)dev);
    for (void* p : dc->allocations) (void)hipFree(p);
    if (dc->ws_mem) (void)hipFree(dc->ws_mem);
    if (dc->sched_mem) (void)hipFree(dc->sched_mem);
    if (dc->ad_mem) (void)hipFree(dc->ad_mem);
    if (dc->tail_mem) (void)hipFree(dc->tail_mem);
    if (dc->pool_mem) (void)hipFree(dc->pool_mem);
    if (dc->ev0) (void)hipEventDestroy(dc->ev0);
    if (dc->ev1) (void)hipEventDestroy(dc->ev1);
    if (dc->ev_busy) (void)hipEventDestroy(dc->ev_busy);
    delete dc;
  }
  delete s;
  return 0;
}

static int check_rect(const grt_scene* s, uint64_t row0, uint64_t col0, uint64_t rows, uint64_t cols) {
  if (row0 + rows > (uint64_t)s->desc.camera.rows || col0 + cols > (uint64_t)s->desc.camera.cols)
    return fail(-EINVAL, "rectangle outside the camera frame");
  return 0;
}

// Synchronous calls: after the work has finished, whether some trace needed more hit-pool
// records than it had.  If so the pool is grown to that size (*again = true): the call
// traces again, and the deterministic trace then keeps every candidate.
static int pool_check(DeviceCopy& dc, bool* again) {
  unsigned long long need = 0;
  HIP_TRY(hipMemcpy(&need, dc.d_counter + 6, sizeof(need), hipMemcpyDeviceToHost));
  *again = need > dc.pool_cap && dc.pool_cap < POOL_MAX;
  if (*again) return ensure_pool(dc, need + need / 4);
  return 0;
}

// Device outputs of one synchronous trace of n slots (the aux ones when asked for).
struct HostTrace {
  DevBuf xyza, cls, status, x64, steps, stop, hits;
  grt::Outputs o{};
  int alloc(uint64_t n, const grt_aux_out* aux) {
    int rc;
    if ((rc = xyza.alloc(n * 16)) || (rc = cls.alloc(n)) || (rc = status.alloc(n))) return rc;
    if (aux && aux->xyza64 && (rc = x64.alloc(n * 32))) return rc;
    if (aux && aux->steps && (rc = steps.alloc(n * 4))) return rc;
    if (aux && aux->stop_reason && (rc = stop.alloc(n))) return rc;
    if (aux && aux->hits && (rc = hits.alloc(n * 4))) return rc;
    o = grt::Outputs{(float*)xyza.p, (uint8_t*)cls.p, (uint8_t*)status.p, (double*)x64.p, (uint32_t*)steps.p,
                     (uint8_t*)stop.p, (uint32_t*)hits.p};
    return 0;
  }
};

// One trace of `wl` on the null stream, waited for.  Adds its counters to acc ([0..3]
// accepted, attempts, rays, overflows; [4..7] march jobs, samples, noise, emitting
// samples) and its event time to *ms; *need = hit-pool records it asked for.
static int trace_sync(grt_scene* s, DeviceCopy& dc, const grt::WorkList& wl, const grt::Outputs& o,
                      unsigned long long acc[8], float* ms, unsigned long long* need) {
  hipStream_t st = nullptr;
  HIP_TRY(hipMemsetAsync(dc.d_stats, 0, 4 * sizeof(unsigned long long), st));
  HIP_TRY(hipMemsetAsync(dc.d_march, 0, 8 * sizeof(unsigned long long), st));
  HIP_TRY(hipMemsetAsync(dc.d_counter + 6, 0, sizeof(unsigned long long), st));
  HIP_TRY(hipEventRecord(dc.ev0, st));
  if (int rc = enqueue_trace(s, dc, wl, o, dc.d_stats, st)) return rc;
  HIP_TRY(hipEventRecord(dc.ev1, st));
  HIP_TRY(hipEventSynchronize(dc.ev1));
  unsigned long long h[4], m[8];
  HIP_TRY(hipMemcpy(h, dc.d_stats, sizeof(h), hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(m, dc.d_march, sizeof(m), hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(need, dc.d_counter + 6, sizeof(*need), hipMemcpyDeviceToHost));
  float t = 0;
  HIP_TRY(hipEventElapsedTime(&t, dc.ev0, dc.ev1));
  for (int k = 0; k < 4; ++k) acc[k] += h[k];
  acc[4] += m[3];
  acc[5] += m[2];
  acc[6] += m[4];
  acc[7] += m[5];
  *ms += t;
  return 0;
}

// Trace `wl` (n output slots) into device scratch, wait, copy to the host arrays.  When the
// hit pool was too small (the trace asked for more records than it had), only the pixels
// that lost candidates (GRT_FLAG_HIT_OVERFLOW) are traced again, as a pixel list at their
// centres (get_ray_for_offset at (0.5, 0.5) is get_ray_for, camera.rs:338-363), with the
// pool grown once that subset alone does not fit; their outputs replace the flagged ones.
// `offs` (host, nullable): the offsets list wl was built from.  The stats count the work
// done, the re-traced rays included.
static int run_to_host(grt_scene* s, DeviceCopy* dc_, const grt::WorkList& wl, uint64_t n, const grt_offsets* offs,
                       float* xyza_out, uint8_t* class_out, uint8_t* status_out, const grt_aux_out* aux,
                       grt_stats* stats) {
  int rc;
  DeviceCopy& dc = *dc_;
  unsigned long long acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  float ms = 0;
  unsigned long long need = 0;
  {
    HostTrace T;
    if ((rc = T.alloc(n, aux)) || (rc = trace_sync(s, dc, wl, T.o, acc, &ms, &need))) return rc;
    HIP_TRY(hipMemcpy(xyza_out, T.xyza.p, n * 16, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(class_out, T.cls.p, n, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(status_out, T.status.p, n, hipMemcpyDeviceToHost));
    if (T.o.xyza64) HIP_TRY(hipMemcpy(aux->xyza64, T.x64.p, n * 32, hipMemcpyDeviceToHost));
    if (T.o.steps) HIP_TRY(hipMemcpy(aux->steps, T.steps.p, n * 4, hipMemcpyDeviceToHost));
    if (T.o.stop) HIP_TRY(hipMemcpy(aux->stop_reason, T.stop.p, n, hipMemcpyDeviceToHost));
    if (T.o.hits) HIP_TRY(hipMemcpy(aux->hits, T.hits.p, n * 4, hipMemcpyDeviceToHost));
  }
  // the flagged pixels, traced again until none is left (a round either fits or grows the
  // pool to its own subset's need, which the next round's subset cannot exceed)
  for (int round = 0; need > dc.pool_cap && round < 8; ++round) {
    std::vector<uint64_t> lost;
    for (uint64_t k = 0; k < n; ++k)
      if (status_out[k] & GRT_FLAG_HIT_OVERFLOW) lost.push_back(k);
    if (lost.empty()) break;
    if (round > 0) {
      if (dc.pool_cap >= POOL_MAX) break;  // cannot grow: the pixels stay flagged
      if ((rc = ensure_pool(dc, need + need / 4))) return rc;
    }
    const uint64_t m = lost.size();
    std::vector<uint32_t> pix(m);
    std::vector<double> dx(m, 0.5), dy(m, 0.5);
    grt::WorkList wo;
    std::memset(&wo, 0, sizeof(wo));
    wo.col0 = wl.col0;
    wo.cols = wl.cols;
    wo.n_items = m;
    if (offs) {  // an offsets trace: the same (pixel, dx, dy) items
      wo.row0 = wl.row0;
      wo.rows = wl.rows;
      for (uint64_t j = 0; j < m; ++j) {
        pix[j] = offs->pixel_index[lost[j]];
        dx[j] = offs->dx[lost[j]];
        dy[j] = offs->dy[lost[j]];
      }
    } else if (wl.n_shards > 1) {  // a row-band shard: frame rows of the local ones
      wo.row0 = 0;
      wo.rows = (uint32_t)s->desc.camera.rows;
      for (uint64_t j = 0; j < m; ++j) {
        const uint32_t lr = (uint32_t)(lost[j] / wl.cols), c = (uint32_t)(lost[j] % wl.cols);
        pix[j] = grt::shard_frame_row(wl.band_rows, wl.shard, wl.n_shards, lr) * wl.cols + c;
      }
    } else {
      wo.row0 = wl.row0;
      wo.rows = wl.rows;
      for (uint64_t j = 0; j < m; ++j) pix[j] = (uint32_t)lost[j];
    }
    DevBuf b_pix, b_dx, b_dy;
    if ((rc = b_pix.alloc(m * 4)) || (rc = b_dx.alloc(m * 8)) || (rc = b_dy.alloc(m * 8))) return rc;
    HIP_TRY(hipMemcpy(b_pix.p, pix.data(), m * 4, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(b_dx.p, dx.data(), m * 8, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(b_dy.p, dy.data(), m * 8, hipMemcpyHostToDevice));
    wo.pixel_index = (const uint32_t*)b_pix.p;
    wo.dx = (const double*)b_dx.p;
    wo.dy = (const double*)b_dy.p;
    HostTrace T;
    acc[3] = 0;  // the overflows of the last round are the ones left
    if ((rc = T.alloc(m, aux)) || (rc = trace_sync(s, dc, wo, T.o, acc, &ms, &need))) return rc;
    std::vector<float> x(m * 4);
    std::vector<uint8_t> c(m), st(m), sp(T.o.stop ? m : 0);
    std::vector<double> x64(T.o.xyza64 ? m * 4 : 0);
    std::vector<uint32_t> ns(T.o.steps ? m : 0), nh(T.o.hits ? m : 0);
    HIP_TRY(hipMemcpy(x.data(), T.xyza.p, m * 16, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(c.data(), T.cls.p, m, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(st.data(), T.status.p, m, hipMemcpyDeviceToHost));
    if (T.o.xyza64) HIP_TRY(hipMemcpy(x64.data(), T.x64.p, m * 32, hipMemcpyDeviceToHost));
    if (T.o.steps) HIP_TRY(hipMemcpy(ns.data(), T.steps.p, m * 4, hipMemcpyDeviceToHost));
    if (T.o.stop) HIP_TRY(hipMemcpy(sp.data(), T.stop.p, m, hipMemcpyDeviceToHost));
    if (T.o.hits) HIP_TRY(hipMemcpy(nh.data(), T.hits.p, m * 4, hipMemcpyDeviceToHost));
    for (uint64_t j = 0; j < m; ++j) {
      const uint64_t k = lost[j];
      std::memcpy(xyza_out + 4 * k, &x[4 * j], 16);
      class_out[k] = c[j];
      status_out[k] = st[j];
      if (T.o.xyza64) std::memcpy(aux->xyza64 + 4 * k, &x64[4 * j], 32);
      if (T.o.steps) aux->steps[k] = ns[j];
      if (T.o.stop) aux->stop_reason[k] = sp[j];
      if (T.o.hits) aux->hits[k] = nh[j];
    }
  }
  if (stats) {
    stats->accepted_steps = acc[0];
    stats->attempts = acc[1];
    stats->rays = acc[2];
    stats->hit_overflows = acc[3];
    stats->kernel_ms = ms;
    stats->march_jobs = acc[4];
    stats->march_samples = acc[5];
    stats->march_noise_samples = acc[6];
    stats->march_emit_samples = acc[7];
  }
  return 0;
}

int grt_render_pixels_async(grt_scene* s, int device, void* stream, uint32_t row0, uint32_t col0,
                            uint32_t rows, uint32_t cols, float* d_xyza, uint8_t* d_class,
                            uint8_t* d_status, double* d_xyza64, uint32_t* d_steps, uint8_t* d_stop,
                            uint64_t* d_stats) {
  if (!s || !d_xyza || !d_class || !d_status || !d_stats) return fail(-EINVAL, "null argument");
  if (rows == 0 || cols == 0) return 0;
  int rc = check_rect(s, row0, col0, rows, cols);
  if (rc) return rc;
  DeviceCopy* dc;
  rc = ensure_device(s, device, &dc);
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(dc->mu);
  HIP_TRY(hipSetDevice(device));
  grt::WorkList wl = rect_worklist(row0, col0, rows, cols);
  grt::Outputs o{d_xyza, d_class, d_status, d_xyza64, d_steps, d_stop};
  return enqueue_trace(s, *dc, wl, o, (unsigned long long*)d_stats, (hipStream_t)stream);
}

int grt_render_pixels(grt_scene* s, int device, uint32_t row0, uint32_t col0, uint32_t rows, uint32_t cols,
                      const grt_offsets* offsets, float* xyza_out, uint8_t* class_out, uint8_t* status_out,
                      const grt_aux_out* aux, grt_stats* stats) {
  if (!s || !xyza_out || !class_out || !status_out) return fail(-EINVAL, "null argument");
  int rc = check_rect(s, row0, col0, rows, cols);
  if (rc) return rc;
  DeviceCopy* dc;
  rc = ensure_device(s, device, &dc);
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(dc->mu);
  HIP_TRY(hipSetDevice(device));
  uint64_t n = offsets ? offsets->count : (uint64_t)rows * cols;
  if (stats) std::memset(stats, 0, sizeof(*stats));
  if (n == 0) return 0;
  grt::WorkList wl;
  DevBuf b_pix, b_dx, b_dy;
  if (offsets) {
    if (!offsets->pixel_index || !offsets->dx || !offsets->dy) return fail(-EINVAL, "incomplete offsets");
    if (cols == 0) return fail(-EINVAL, "offsets need the rectangle width");
    for (uint64_t k = 0; k < n; ++k)
      if (offsets->pixel_index[k] >= (uint64_t)rows * cols) return fail(-EINVAL, "offset pixel outside rectangle");
    std::memset(&wl, 0, sizeof(wl));
    wl.row0 = row0;
    wl.col0 = col0;
    wl.rows = rows;
    wl.cols = cols;
    wl.n_items = n;
    if ((rc = b_pix.alloc(n * 4)) || (rc = b_dx.alloc(n * 8)) || (rc = b_dy.alloc(n * 8))) return rc;
    HIP_TRY(hipMemcpy(b_pix.p, offsets->pixel_index, n * 4, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(b_dx.p, offsets->dx, n * 8, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(b_dy.p, offsets->dy, n * 8, hipMemcpyHostToDevice));
    wl.pixel_index = (const uint32_t*)b_pix.p;
    wl.dx = (const double*)b_dx.p;
    wl.dy = (const double*)b_dy.p;
  } else {
    wl = rect_worklist(row0, col0, rows, cols);
  }
  return run_to_host(s, dc, wl, n, offsets, xyza_out, class_out, status_out, aux, stats);
}

// Shared body of grt_trace_pixels / grt_trace_rays: a, b are (row, col) or (pos, mom).
static int trace_common(grt_scene* s, int device, uint64_t n, bool camera, const double* a, const double* b,
                        uint64_t capacity, double* steps_out, uint64_t* n_steps, uint8_t* stop_out,
                        uint8_t* status_out) {
  if (!s || !n_steps || !stop_out || !status_out || (n && (!a || !b)) || (capacity && !steps_out))
    return fail(-EINVAL, "null argument");
  if (n == 0) return 0;
  if (capacity > (1ull << 40) / 72 / n) return fail(-EINVAL, "trajectory buffer too large");
  DeviceCopy* dc;
  int rc = ensure_device(s, device, &dc);
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(dc->mu);
  HIP_TRY(hipSetDevice(device));
  const uint64_t in_bytes = n * 8 * (camera ? 1 : 4);
  DevBuf b_a, b_b, b_steps, b_n, b_stop, b_status;
  if ((rc = b_a.alloc(in_bytes)) || (rc = b_b.alloc(in_bytes)) || (rc = b_steps.alloc(n * capacity * 72)) ||
      (rc = b_n.alloc(n * 8)) || (rc = b_stop.alloc(n)) || (rc = b_status.alloc(n)))
    return rc;
  HIP_TRY(hipMemcpy(b_a.p, a, in_bytes, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(b_b.p, b, in_bytes, hipMemcpyHostToDevice));
  grt::TrajectoryList tl;
  std::memset(&tl, 0, sizeof(tl));
  tl.n = n;
  if (camera) {
    tl.row = (const double*)b_a.p;
    tl.col = (const double*)b_b.p;
  } else {
    tl.pos = (const double*)b_a.p;
    tl.mom = (const double*)b_b.p;
  }
  tl.cap = capacity;
  tl.steps = (double*)b_steps.p;
  tl.n_steps = (uint64_t*)b_n.p;
  tl.stop = (uint8_t*)b_stop.p;
  tl.status = (uint8_t*)b_status.p;
  HIP_TRY(grt::launch_trajectories(s->desc.geometry, dc->d_scene, tl, nullptr));
  HIP_TRY(hipDeviceSynchronize());
  if (capacity) HIP_TRY(hipMemcpy(steps_out, b_steps.p, n * capacity * 72, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(n_steps, b_n.p, n * 8, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(stop_out, b_stop.p, n, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(status_out, b_status.p, n, hipMemcpyDeviceToHost));
  return 0;
}

int grt_health_pixels(grt_scene* s, int device, uint32_t row0, uint32_t col0, uint32_t rows, uint32_t cols,
                      grt_health* out, double* per_ray) {
  if (!s || !out) return fail(-EINVAL, "null argument");
  std::memset(out, 0, sizeof(*out));
  out->n_constants = s->desc.geometry == GRT_GEOM_KERR_BL ? 3u : 2u;
  if ((uint64_t)row0 + rows > (uint64_t)s->desc.camera.rows || (uint64_t)col0 + cols > (uint64_t)s->desc.camera.cols)
    return fail(-EINVAL, "rectangle outside the frame");
  const uint64_t n = (uint64_t)rows * cols;
  if (n == 0) return 0;
  DeviceCopy* dc;
  int rc = ensure_device(s, device, &dc);
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(dc->mu);
  HIP_TRY(hipSetDevice(device));
  DevBuf b_out, b_status;
  if ((rc = b_out.alloc(n * 5 * 8)) || (rc = b_status.alloc(n))) return rc;
  grt::WorkList wl = rect_worklist(row0, col0, rows, cols);
  HIP_TRY(grt::launch_health(s->desc.geometry, dc->d_scene, wl, n, (double*)b_out.p, (uint8_t*)b_status.p, nullptr));
  HIP_TRY(hipDeviceSynchronize());
  std::vector<double> v(n * 5);
  std::vector<uint8_t> st(n);
  HIP_TRY(hipMemcpy(v.data(), b_out.p, n * 5 * 8, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(st.data(), b_status.p, n, hipMemcpyDeviceToHost));
  // scene.rs:116-124 (error above 1e-10 for every ray) and report_drifts (integrator.rs:176-201,
  // warnings above 1e-4 for the rays whose integration returned Ok)
  for (uint64_t k = 0; k < n; ++k) {
    const double* o = &v[k * 5];
    out->rays++;
    if (!(o[0] < 1e-10)) out->null_violations++;
    out->max_null = std::fmax(out->max_null, o[0]);
    if (st[k] != GRT_OK) {
      out->failed++;
      continue;
    }
    if (o[1] > 1e-4) out->kk_drift_rays++;
    out->max_kk_drift = std::fmax(out->max_kk_drift, o[1]);
    for (uint32_t c = 0; c < out->n_constants; ++c) {
      if (o[2 + c] > 1e-4) out->constant_drift_rays[c]++;
      out->max_constant_drift[c] = std::fmax(out->max_constant_drift[c], o[2 + c]);
    }
  }
  if (per_ray) std::memcpy(per_ray, v.data(), n * 5 * 8);
  return 0;
}

int grt_trace_pixels(grt_scene* s, int device, uint64_t n, const double* rows, const double* cols,
                     uint64_t capacity, double* steps_out, uint64_t* n_steps, uint8_t* stop_out,
                     uint8_t* status_out) {
  return trace_common(s, device, n, true, rows, cols, capacity, steps_out, n_steps, stop_out, status_out);
}

int grt_trace_rays(grt_scene* s, int device, uint64_t n, const double* positions, const double* momenta,
                   uint64_t capacity, double* steps_out, uint64_t* n_steps, uint8_t* stop_out,
                   uint8_t* status_out) {
  return trace_common(s, device, n, false, positions, momenta, capacity, steps_out, n_steps, stop_out,
                      status_out);
}

// ------------------------------------------------------------- adaptive pass ----
// Bump allocator over the device's grow-only adaptive arena.  Plan the whole call's
// buffers first (ad_plan), then carve them (ad_take): growing the arena happens before
// any kernel of the call is enqueued.
struct AdArena {
  char* base = nullptr;
  uint64_t off = 0;
  void* take(uint64_t bytes) {
    void* r = base ? base + off : nullptr;
    off += (bytes + 255) & ~255ull;
    return r;
  }
};
static int ad_reserve(DeviceCopy& dc, uint64_t bytes) {
  if (bytes <= dc.ad_bytes && dc.ad_mem) return 0;
  if (dc.ad_mem) {
    (void)hipDeviceSynchronize();  // earlier async launches may still use the old arena
    (void)hipFree(dc.ad_mem);
    dc.ad_mem = nullptr;
    dc.ad_bytes = 0;
  }
  const uint64_t cap = bytes + (bytes >> 3);
  if (hipMalloc(&dc.ad_mem, cap) != hipSuccess) {
    (void)hipGetLastError();
    dc.ad_mem = nullptr;
    return fail(-ENOMEM, "cannot allocate the adaptive-pass scratch");
  }
  dc.ad_bytes = cap;
  return 0;
}

constexpr uint64_t SUB_CHUNK = 1ull << 21;  // sub-rays per supersample trace launch
std::atomic<uint64_t> g_sub_chunk{SUB_CHUNK};  // grt_set_sub_chunk (tests force several chunks)

// Buffers of the supersample pass over at most n_max selected pixels.
struct SuperBufs {
  uint64_t chunk_pix = 0, cap = 0;
  uint32_t n_chunks = 0, per = 0;
  uint32_t* pix = nullptr;
  double *dx = nullptr, *dy = nullptr, *x64 = nullptr;
  float* xyza = nullptr;
  uint8_t *cls = nullptr, *status = nullptr, *stop = nullptr;
  uint32_t* steps = nullptr;
  unsigned long long* live = nullptr;
  // sub_chunk: grt_set_sub_chunk's value, read once per call (the plan and the carve of
  // one call must agree)
  void carve(AdArena& A, uint64_t n_max, uint32_t spa, uint64_t sub_chunk) {
    per = spa * spa;
    chunk_pix = std::max<uint64_t>(1, std::min<uint64_t>(n_max, sub_chunk / per));
    n_chunks = (uint32_t)((n_max + chunk_pix - 1) / chunk_pix);
    cap = chunk_pix * per;
    pix = (uint32_t*)A.take(cap * 4);
    dx = (double*)A.take(cap * 8);
    dy = (double*)A.take(cap * 8);
    xyza = (float*)A.take(cap * 16);
    cls = (uint8_t*)A.take(cap);
    status = (uint8_t*)A.take(cap);
    x64 = (double*)A.take(cap * 32);
    stop = (uint8_t*)A.take(cap);
    steps = (uint32_t*)A.take(cap * 4);
    live = (unsigned long long*)A.take((uint64_t)n_chunks * 8);
  }
};

// supersample (raytracer.rs:320-384) over a selection that lives on the device: entries
// j < *d_count <= n_max of sel_px (pixel index in the rect row0/col0/rows/cols: camera
// ray and jitter hash) and sel_out (index into d_out64).  The sub-rays go through the
// trace in chunks of g_sub_chunk; the integrate / shade kernels read each chunk's live
// count from the device, so nothing waits for the host between the passes.
static int enqueue_supersample(grt_scene* s, DeviceCopy& dc, hipStream_t st, const SuperBufs& B, uint32_t row0,
                        uint32_t col0, uint32_t rows, uint32_t cols, const uint32_t* sel_px, const uint32_t* sel_out,
                        const unsigned long long* d_count, uint32_t spa, double* d_out64, unsigned long long* d_stats,
                        const grt::SubsampleFailures& fails_in) {
  grt::SubsampleFailures fails = fails_in;
  fails.ray_stop = B.stop;
  fails.ray_steps = B.steps;
  HIP_TRY(grt::launch_chunk_live(d_count, B.n_chunks, B.chunk_pix, B.per, B.live, st));
  for (uint32_t c = 0; c < B.n_chunks; ++c) {
    const uint64_t base = (uint64_t)c * B.chunk_pix;
    HIP_TRY(grt::launch_make_offsets(sel_px + base, B.chunk_pix, d_count, base, spa, row0, col0, cols, B.pix, B.dx,
                                     B.dy, st));
    grt::WorkList wo;
    std::memset(&wo, 0, sizeof(wo));
    wo.row0 = row0;
    wo.col0 = col0;
    wo.rows = rows;
    wo.cols = cols;
    wo.n_items = B.cap;
    wo.pixel_index = B.pix;
    wo.dx = B.dx;
    wo.dy = B.dy;
    wo.n_live = B.live + c;
    grt::Outputs so{B.xyza, B.cls, B.status, B.x64, B.steps, B.stop};
    int rc = enqueue_trace(s, dc, wo, so, d_stats, st);
    if (rc) return rc;
    HIP_TRY(grt::launch_average(sel_out + base, sel_px + base, B.chunk_pix, d_count, base, spa, B.x64, B.status,
                                d_out64, fails, st));
  }
  return 0;
}

// resolve_minimum_luminance's relative floor (raytracer.rs:118-129): 1e-3 x the element
// at ((n - 1) * 0.99) as usize in f64::total_cmp order (select_nth_unstable_by selects
// the same element as nth_element under the same total order).  Reorders `lum`.
static double relative_min_luminance(std::vector<double>& lum) {
  if (lum.empty()) return 0.0;
  uint64_t index = (uint64_t)((double)(lum.size() - 1) * 0.99);
  auto key = [](double v) {
    int64_t b;
    std::memcpy(&b, &v, 8);
    return b ^ (int64_t)((uint64_t)(b >> 63) >> 1);
  };
  std::nth_element(lum.begin(), lum.begin() + index, lum.end(), [&](double a, double b) { return key(a) < key(b); });
  return 1e-3 * lum[index];
}

static uint64_t floor_index(uint64_t n) { return (uint64_t)((double)(n - 1) * 0.99); }

int grt_adaptive_min_luminance_device(int device, void* stream, const double* d_y, uint32_t stride, uint64_t n,
                                      const grt_adaptive_config* cfg, double* out) {
  if (!out || (n && (!d_y || stride == 0))) return fail(-EINVAL, "null argument");
  if (cfg && cfg->has_minimum_luminance) {
    *out = cfg->minimum_luminance;
    return 0;
  }
  if (n == 0) {
    *out = 0.0;
    return 0;
  }
  if (n > (uint64_t)INT_MAX) return fail(-EOVERFLOW, "more than INT_MAX luminances");
  HIP_TRY(hipSetDevice(device));
  size_t bytes = 0;
  HIP_TRY(grt::luminance_order_stat(d_y, stride, n, floor_index(n), nullptr, &bytes, nullptr, (hipStream_t)stream));
  DevBuf b;
  int rc = b.alloc(bytes);
  if (rc) return rc;
  double v = 0.0;
  HIP_TRY(grt::luminance_order_stat(d_y, stride, n, floor_index(n), b.p, &bytes, &v, (hipStream_t)stream));
  *out = 1e-3 * v;
  return 0;
}

double grt_adaptive_min_luminance(const double* lum, uint64_t n, const grt_adaptive_config* cfg) {
  if (cfg && cfg->has_minimum_luminance) return cfg->minimum_luminance;
  if (!lum || n == 0) return 0.0;
  std::vector<double> v(lum, lum + n);
  return relative_min_luminance(v);
}

// The recorded failed sub-samples, sorted by (pixel, stratum): the reference logs them
// from a parallel loop (raytracer.rs:357-362), in no particular order.
static int copy_failures(const grt::SubsampleFailures& f, uint64_t count, uint32_t spa, grt_subsample_failures* out) {
  const uint64_t m = std::min<uint64_t>(count, f.cap);
  if (m == 0) return 0;
  std::vector<uint64_t> key(m);
  std::vector<uint8_t> st(m), sp(f.stop ? m : 0);
  std::vector<uint32_t> ns(f.stop ? m : 0);
  HIP_TRY(hipMemcpy(key.data(), f.key, m * 8, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(st.data(), f.status, m, hipMemcpyDeviceToHost));
  if (f.stop) {
    HIP_TRY(hipMemcpy(sp.data(), f.stop, m, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(ns.data(), f.steps, m * 4, hipMemcpyDeviceToHost));
  }
  std::vector<uint64_t> order(m);
  for (uint64_t i = 0; i < m; ++i) order[i] = i;
  std::sort(order.begin(), order.end(), [&](uint64_t a, uint64_t b) { return key[a] < key[b]; });
  const uint64_t per = (uint64_t)spa * spa;
  for (uint64_t i = 0; i < m; ++i) {
    out->pixel[i] = (uint32_t)(key[order[i]] / per);
    if (out->sample) out->sample[i] = (uint32_t)(key[order[i]] % per);
    out->status[i] = st[order[i]];
    if (f.stop) {
      out->stop[i] = sp[order[i]];
      if (out->steps) out->steps[i] = ns[order[i]];
    }
  }
  return 0;
}

int grt_render_section_ex(grt_scene* s, int device, uint32_t from_row, uint32_t from_col, uint32_t to_row,
                          uint32_t to_col, const grt_adaptive_config* cfg, const double* mask_xyza, double* xyza_out,
                          uint8_t* class_out, uint64_t* n_supersampled, grt_stats* stats, uint8_t* status_out,
                          grt_subsample_failures* failures, uint8_t* stop_out, uint32_t* steps_out) {
  if (!s || !cfg || !xyza_out) return fail(-EINVAL, "null argument");
  if (to_row < from_row || to_col < from_col) return fail(-EINVAL, "empty section");
  if (cfg->samples_per_axis == 0) return fail(-EINVAL, "adaptive_sampling.samples_per_axis must be greater than zero");
  int rc = check_rect(s, from_row, from_col, to_row - from_row, to_col - from_col);
  if (rc) return rc;
  DeviceCopy* dc;
  rc = ensure_device(s, device, &dc);
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(dc->mu);
  HIP_TRY(hipSetDevice(device));
  uint32_t w = to_col - from_col, h = to_row - from_row;
  uint64_t n = (uint64_t)w * h;
  if (stats) std::memset(stats, 0, sizeof(*stats));
  if (n_supersampled) *n_supersampled = 0;
  if (failures) failures->count = 0;
  if (n == 0) return 0;
  const bool supersampled = cfg->enabled || mask_xyza != nullptr;
  const bool device_floor = supersampled && !cfg->has_minimum_luminance;
  if (supersampled && n > (uint64_t)INT_MAX) return fail(-EOVERFLOW, "section larger than INT_MAX pixels");
  const uint32_t spa = cfg->samples_per_axis;
  const uint64_t sub_chunk = g_sub_chunk.load(std::memory_order_relaxed);
  // plan: section buffers, selection, floor, sort / compaction scratch, sub-ray buffers
  size_t sort_bytes = 0, select_bytes = 0;
  if (device_floor) HIP_TRY(grt::luminance_floor_device(nullptr, 4, n, floor_index(n), nullptr, &sort_bytes, nullptr, 0));
  if (supersampled) HIP_TRY(grt::compact_flags(nullptr, n, nullptr, nullptr, nullptr, &select_bytes, 0));
  // the supersample pass's work order (longest sub-rays first) reads the 1-spp step counts
  const bool ordered = supersampled && !mask_xyza;
  size_t order_bytes = 0;
  if (ordered) HIP_TRY(grt::order_selection(nullptr, nullptr, n, nullptr, w, h, nullptr, nullptr, &order_bytes, 0));
  const uint64_t fail_cap = (failures && failures->pixel && failures->status) ? failures->capacity : 0;
  const bool want_events = fail_cap && failures->stop;
  grt::SubsampleFailures fails{nullptr, nullptr, nullptr, fail_cap};
  uint8_t* b_stop = nullptr;
  uint32_t *b_steps = nullptr, *b_order = nullptr;
  void* b_order_tmp = nullptr;
  auto carve = [&](AdArena& A, float** xyza, uint8_t** cls, uint8_t** status, double** x64, uint8_t** flags,
                   uint32_t** sel, unsigned long long** cnt, double** floor, void** sort, void** select,
                   SuperBufs* B) {
    *xyza = (float*)A.take(n * 16);
    *cls = (uint8_t*)A.take(n);
    *status = (uint8_t*)A.take(n);
    *x64 = (double*)A.take(n * 32);
    if (stop_out) b_stop = (uint8_t*)A.take(n);
    if (steps_out || ordered) b_steps = (uint32_t*)A.take(n * 4);
    if (!supersampled) return;
    if (ordered) {
      b_order = (uint32_t*)A.take(n * 4);
      b_order_tmp = A.take(order_bytes);
    }
    *flags = (uint8_t*)A.take(n);
    *sel = (uint32_t*)A.take(n * 4);
    *cnt = (unsigned long long*)A.take(16);  // [0] selected pixels, [1] failed sub-samples
    *floor = (double*)A.take(8);
    *sort = A.take(sort_bytes);
    *select = A.take(select_bytes);
    if (!mask_xyza) B->carve(A, n, spa, sub_chunk);
    fails.key = (uint64_t*)A.take(fail_cap * 8);
    fails.status = (uint8_t*)A.take(fail_cap);
    if (want_events) {  // NaN / no-terminal-event sub-rays too (scene.rs:178-183, :196-202)
      fails.stop = (uint8_t*)A.take(fail_cap);
      fails.steps = (uint32_t*)A.take(fail_cap * 4);
    }
  };
  float* b_xyza = nullptr;
  uint8_t *b_cls = nullptr, *b_status = nullptr, *b_flags = nullptr;
  double *b_x64 = nullptr, *d_floor = nullptr;
  uint32_t* b_sel = nullptr;
  unsigned long long* d_cnt = nullptr;
  void *b_sort = nullptr, *b_select = nullptr;
  SuperBufs B;
  {
    AdArena plan;
    carve(plan, &b_xyza, &b_cls, &b_status, &b_x64, &b_flags, &b_sel, &d_cnt, &d_floor, &b_sort, &b_select, &B);
    if ((rc = ad_reserve(*dc, plan.off))) return rc;
    AdArena A{(char*)dc->ad_mem, 0};
    carve(A, &b_xyza, &b_cls, &b_status, &b_x64, &b_flags, &b_sel, &d_cnt, &d_floor, &b_sort, &b_select, &B);
  }
  hipStream_t st = nullptr;
  for (bool again = true; again;) {
  HIP_TRY(hipMemsetAsync(dc->d_stats, 0, 4 * sizeof(unsigned long long), st));
  HIP_TRY(hipMemsetAsync(dc->d_march, 0, 8 * sizeof(unsigned long long), st));
  HIP_TRY(hipMemsetAsync(dc->d_counter + 6, 0, sizeof(unsigned long long), st));
  if (supersampled) HIP_TRY(hipMemsetAsync(d_cnt, 0, 16, st));
  HIP_TRY(hipEventRecord(dc->ev0, st));
  grt::WorkList wl = rect_worklist(from_row, from_col, h, w);
  grt::Outputs o{b_xyza, b_cls, b_status, b_x64, b_steps, b_stop};
  if ((rc = enqueue_trace(s, *dc, wl, o, dc->d_stats, st))) return rc;
  if (supersampled) {
    // resolve_minimum_luminance (raytracer.rs:118-129): the exact 99th percentile in
    // f64::total_cmp order, selected on the device from the 1-spp buffer
    if (device_floor)
      HIP_TRY(grt::luminance_floor_device(b_x64 + 1, 4, n, floor_index(n), b_sort, &sort_bytes, d_floor, st));
    grt::AdaptiveParams ap;
    ap.w = w;
    ap.h = h;
    ap.exclude_background_contrast = cfg->exclude_background_contrast;
    ap.min_lum = cfg->minimum_luminance;
    ap.luminance_contrast_threshold = cfg->luminance_contrast_threshold;
    ap.opacity_contrast_threshold = cfg->opacity_contrast_threshold;
    // collect_pixels_to_supersample (:386-458): stencil, then the selected pixels in
    // order by a device stream compaction
    HIP_TRY(grt::launch_select(b_x64, b_cls, ap, device_floor ? d_floor : nullptr, b_flags, st));
    HIP_TRY(grt::compact_flags(b_flags, n, b_sel, d_cnt, b_select, &select_bytes, st));
    if (mask_xyza) {  // raytracer.rs:285-295: paint instead of supersampling
      HIP_TRY(grt::launch_paint(b_sel, n, d_cnt, mask_xyza, b_x64, st));
    } else {
      fails.count = d_cnt + 1;
      HIP_TRY(grt::order_selection(b_sel, d_cnt, n, b_steps, w, h, b_order, b_order_tmp, &order_bytes, st));
      if ((rc = enqueue_supersample(s, *dc, st, B, from_row, from_col, h, w, b_order, b_order, d_cnt, spa, b_x64,
                                    dc->d_stats, fails)))
        return rc;
    }
  }
  HIP_TRY(hipEventRecord(dc->ev1, st));
  HIP_TRY(hipEventSynchronize(dc->ev1));
  if ((rc = pool_check(*dc, &again))) return rc;
  }
  HIP_TRY(hipMemcpy(xyza_out, b_x64, n * 32, hipMemcpyDeviceToHost));
  if (class_out) HIP_TRY(hipMemcpy(class_out, b_cls, n, hipMemcpyDeviceToHost));
  if (status_out) HIP_TRY(hipMemcpy(status_out, b_status, n, hipMemcpyDeviceToHost));
  if (stop_out) HIP_TRY(hipMemcpy(stop_out, b_stop, n, hipMemcpyDeviceToHost));
  if (steps_out) HIP_TRY(hipMemcpy(steps_out, b_steps, n * 4, hipMemcpyDeviceToHost));
  if (supersampled) {
    unsigned long long cnt[2] = {0, 0};
    HIP_TRY(hipMemcpy(cnt, d_cnt, sizeof(cnt), hipMemcpyDeviceToHost));
    if (n_supersampled) *n_supersampled = cnt[0];
    if (failures) {
      failures->count = cnt[1];
      if (int frc = copy_failures(fails, cnt[1], spa, failures)) return frc;
    }
  }
  if (stats) {
    unsigned long long hs[4];
    HIP_TRY(hipMemcpy(hs, dc->d_stats, sizeof(hs), hipMemcpyDeviceToHost));
    float ms = 0;
    HIP_TRY(hipEventElapsedTime(&ms, dc->ev0, dc->ev1));
    stats->accepted_steps = hs[0];
    stats->attempts = hs[1];
    stats->rays = hs[2];
    stats->hit_overflows = hs[3];
    stats->kernel_ms = ms;
    unsigned long long m[8];
    HIP_TRY(hipMemcpy(m, dc->d_march, sizeof(m), hipMemcpyDeviceToHost));
    stats->march_jobs = m[3];
    stats->march_samples = m[2];
    stats->march_noise_samples = m[4];
    stats->march_emit_samples = m[5];
  }
  return 0;
}

int grt_render_section(grt_scene* s, int device, uint32_t from_row, uint32_t from_col, uint32_t to_row,
                       uint32_t to_col, const grt_adaptive_config* cfg, const double* mask_xyza,
                       double* xyza_out, uint8_t* class_out, uint64_t* n_supersampled, grt_stats* stats,
                       uint8_t* status_out) {
  return grt_render_section_ex(s, device, from_row, from_col, to_row, to_col, cfg, mask_xyza, xyza_out, class_out,
                               n_supersampled, stats, status_out, nullptr, nullptr, nullptr);
}


// ------------------------------------------------------------- row-band shards ----
static int check_shard(const grt_row_shard* sh) {
  if (!sh) return fail(-EINVAL, "null shard");
  if (sh->n_shards == 0 || sh->shard >= sh->n_shards) return fail(-EINVAL, "shard index out of range");
  if (sh->band_rows == 0) return fail(-EINVAL, "band_rows must be >= 1");
  return 0;
}

uint32_t grt_shard_row_count(uint32_t frame_rows, const grt_row_shard* sh) {
  if (!sh || sh->n_shards == 0 || sh->band_rows == 0 || sh->shard >= sh->n_shards) return 0;
  if (sh->n_shards == 1) return frame_rows;
  uint64_t bands = ((uint64_t)frame_rows + sh->band_rows - 1) / sh->band_rows;
  uint64_t mine = bands > sh->shard ? (bands - sh->shard + sh->n_shards - 1) / sh->n_shards : 0;
  if (mine == 0) return 0;
  uint64_t last_band = sh->shard + (mine - 1) * sh->n_shards;
  uint64_t last_rows = std::min<uint64_t>(sh->band_rows, frame_rows - last_band * sh->band_rows);
  return (uint32_t)((mine - 1) * sh->band_rows + last_rows);
}

uint32_t grt_shard_frame_row(uint32_t local_row, const grt_row_shard* sh) {
  if (!sh) return local_row;
  return grt::shard_frame_row(sh->band_rows, sh->shard, sh->n_shards, local_row);
}

static grt::WorkList shard_worklist(const grt_scene* s, const grt_row_shard* sh) {
  uint32_t rows = grt_shard_row_count((uint32_t)s->desc.camera.rows, sh);
  grt::WorkList wl = rect_worklist(0, 0, rows, (uint32_t)s->desc.camera.cols);
  wl.band_rows = sh->band_rows;
  wl.shard = sh->shard;
  wl.n_shards = sh->n_shards;
  return wl;
}

int grt_render_shard(grt_scene* s, int device, const grt_row_shard* sh, float* xyza_out, uint8_t* class_out,
                     uint8_t* status_out, const grt_aux_out* aux, grt_stats* stats) {
  if (!s || !xyza_out || !class_out || !status_out) return fail(-EINVAL, "null argument");
  int rc = check_shard(sh);
  if (rc) return rc;
  if (stats) std::memset(stats, 0, sizeof(*stats));
  grt::WorkList wl = shard_worklist(s, sh);
  uint64_t n = (uint64_t)wl.rows * wl.cols;
  if (n == 0) return 0;
  DeviceCopy* dc;
  if ((rc = ensure_device(s, device, &dc))) return rc;
  std::lock_guard<std::mutex> lk(dc->mu);
  HIP_TRY(hipSetDevice(device));
  return run_to_host(s, dc, wl, n, nullptr, xyza_out, class_out, status_out, aux, stats);
}

int grt_set_sub_chunk(uint64_t sub_rays) {
  if (sub_rays > (1ull << 31)) return fail(-EINVAL, "sub-ray chunk larger than 2^31");
  g_sub_chunk.store(sub_rays ? sub_rays : SUB_CHUNK);
  return 0;
}

int grt_set_hit_pool_min(uint64_t records) {
  if (records == 0 || records > POOL_MAX) return fail(-EINVAL, "hit pool minimum must be in [1, 2^31)");
  g_pool_min.store(records);
  return 0;
}

int grt_hit_pool_reserve(grt_scene* s, int device, uint64_t records, uint64_t* capacity) {
  if (!s) return fail(-EINVAL, "null argument");
  DeviceCopy* dc;
  int rc = ensure_device(s, device, &dc);
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(dc->mu);
  HIP_TRY(hipSetDevice(device));
  if (records == 0) {  // the largest need since the last reset, once the device is idle
    HIP_TRY(hipDeviceSynchronize());
    unsigned long long need = 0;
    HIP_TRY(hipMemcpy(&need, dc->d_counter + 6, sizeof(need), hipMemcpyDeviceToHost));
    HIP_TRY(hipMemset(dc->d_counter + 6, 0, sizeof(need)));
    records = need + need / 4;
  }
  if (records > POOL_MAX) return fail(-ENOMEM, "hit pool larger than 2^31 records");
  if ((rc = ensure_pool(*dc, records))) return rc;
  if (capacity) *capacity = dc->pool_cap;
  return 0;
}

int grt_render_shard_async(grt_scene* s, int device, void* stream, const grt_row_shard* sh, float* d_xyza,
                           uint8_t* d_class, uint8_t* d_status, double* d_xyza64, uint32_t* d_steps,
                           uint8_t* d_stop, uint64_t* d_stats) {
  if (!s || !d_xyza || !d_class || !d_status || !d_stats) return fail(-EINVAL, "null argument");
  int rc = check_shard(sh);
  if (rc) return rc;
  grt::WorkList wl = shard_worklist(s, sh);
  if ((uint64_t)wl.rows * wl.cols == 0) return 0;
  DeviceCopy* dc;
  if ((rc = ensure_device(s, device, &dc))) return rc;
  std::lock_guard<std::mutex> lk(dc->mu);
  HIP_TRY(hipSetDevice(device));
  grt::Outputs o{d_xyza, d_class, d_status, d_xyza64, d_steps, d_stop};
  return enqueue_trace(s, *dc, wl, o, (unsigned long long*)d_stats, (hipStream_t)stream);
}

}  // extern "C"

namespace grt_host {
// grt_supersample_shard_device; d_local_steps (nullable): the shard's 1-spp step counts in
// local order, for the sub-rays' longest-first work order (order_selection).
int supersample_shard(grt_scene* s, int device, void* stream, const grt_row_shard* sh,
                                const grt_adaptive_config* cfg, double min_lum, const double* d_min_lum,
                                const double* d_frame_ya, const uint8_t* d_frame_class,
                                const double* sampling_mask_xyza, double* d_xyza64, const uint32_t* d_local_steps,
                                uint64_t* d_n_supersampled, uint64_t* d_stats, grt_subsample_failures* failures) {
  if (!s || !cfg || !d_frame_ya || !d_frame_class || !d_xyza64 || !d_stats) return fail(-EINVAL, "null argument");
  if (cfg->samples_per_axis == 0) return fail(-EINVAL, "adaptive_sampling.samples_per_axis must be greater than zero");
  int rc = check_shard(sh);
  if (rc) return rc;
  if (failures) failures->count = 0;
  const uint32_t frame_rows = (uint32_t)s->desc.camera.rows, w = (uint32_t)s->desc.camera.cols;
  const uint32_t local_rows = grt_shard_row_count(frame_rows, sh);
  const uint64_t n_local = (uint64_t)local_rows * w;
  DeviceCopy* dc;
  if ((rc = ensure_device(s, device, &dc))) return rc;
  std::lock_guard<std::mutex> lk(dc->mu);
  HIP_TRY(hipSetDevice(device));
  hipStream_t st = (hipStream_t)stream;
  if (n_local == 0) {
    if (d_n_supersampled) HIP_TRY(hipMemsetAsync(d_n_supersampled, 0, 8, st));
    return 0;
  }
  if (n_local > (uint64_t)INT_MAX) return fail(-EOVERFLOW, "shard larger than INT_MAX pixels");
  const uint32_t spa = cfg->samples_per_axis;
  const uint64_t sub_chunk = g_sub_chunk.load(std::memory_order_relaxed);
  const uint64_t fail_cap = (failures && failures->pixel && failures->status) ? failures->capacity : 0;
  const bool want_events = fail_cap && failures->stop;
  size_t select_bytes = 0, order_bytes = 0;
  HIP_TRY(grt::compact_flags(nullptr, n_local, nullptr, nullptr, nullptr, &select_bytes, 0));
  const bool ordered = d_local_steps && !sampling_mask_xyza;
  if (ordered)
    HIP_TRY(grt::order_selection(nullptr, nullptr, n_local, nullptr, w, local_rows, nullptr, nullptr, &order_bytes, 0));
  uint8_t* b_flags = nullptr;
  uint32_t *sel_local = nullptr, *sel_frame = nullptr, *sel_order = nullptr;
  unsigned long long* d_cnt = nullptr;
  void *b_select = nullptr, *b_order_tmp = nullptr;
  SuperBufs B;
  grt::SubsampleFailures fails{nullptr, nullptr, nullptr, fail_cap};
  auto carve = [&](AdArena& A) {
    b_flags = (uint8_t*)A.take(n_local);
    sel_local = (uint32_t*)A.take(n_local * 4);
    sel_frame = (uint32_t*)A.take(n_local * 4);
    d_cnt = (unsigned long long*)A.take(16);  // [0] selected pixels, [1] failed sub-samples
    b_select = A.take(select_bytes);
    if (ordered) {
      sel_order = (uint32_t*)A.take(n_local * 4);
      b_order_tmp = A.take(order_bytes);
    }
    if (!sampling_mask_xyza) B.carve(A, n_local, spa, sub_chunk);
    fails.key = (uint64_t*)A.take(fail_cap * 8);
    fails.status = (uint8_t*)A.take(fail_cap);
    if (want_events) {  // NaN / no-terminal-event sub-rays too (scene.rs:178-183, :196-202)
      fails.stop = (uint8_t*)A.take(fail_cap);
      fails.steps = (uint32_t*)A.take(fail_cap * 4);
    }
  };
  {
    AdArena plan;
    carve(plan);
    if ((rc = ad_reserve(*dc, plan.off))) return rc;
    AdArena A{(char*)dc->ad_mem, 0};
    carve(A);
  }
  if ((rc = stream_order(*dc, st))) return rc;
  HIP_TRY(hipMemsetAsync(d_cnt, 0, 16, st));
  // collect_pixels_to_supersample (raytracer.rs:386-458) over this shard's pixels, with
  // the whole frame's 1-spp buffer as the neighbourhood
  grt::AdaptiveParams ap;
  ap.w = w;
  ap.h = frame_rows;
  ap.exclude_background_contrast = cfg->exclude_background_contrast;
  ap.min_lum = min_lum;
  ap.luminance_contrast_threshold = cfg->luminance_contrast_threshold;
  ap.opacity_contrast_threshold = cfg->opacity_contrast_threshold;
  HIP_TRY(grt::launch_select_shard(d_frame_ya, d_frame_class, ap, d_min_lum, sh->band_rows, sh->shard, sh->n_shards,
                                   local_rows, b_flags, st));
  // selected pixels in frame order (shard rows increase with local rows): local index
  // for the output, frame index for the jitter hash and the camera ray
  HIP_TRY(grt::compact_flags(b_flags, n_local, sel_local, d_cnt, b_select, &select_bytes, st));
  if (ordered) {  // longest sub-rays first (the 3 x 3 neighbourhood in the shard's own rows)
    HIP_TRY(grt::order_selection(sel_local, d_cnt, n_local, d_local_steps, w, local_rows, sel_order, b_order_tmp,
                                 &order_bytes, st));
    sel_local = sel_order;
  }
  HIP_TRY(grt::launch_frame_index(sel_local, d_cnt, n_local, w, sh->band_rows, sh->shard, sh->n_shards, sel_frame,
                                  st));
  if (sampling_mask_xyza) {  // raytracer.rs:285-295: paint instead of supersampling
    HIP_TRY(grt::launch_paint(sel_local, n_local, d_cnt, sampling_mask_xyza, d_xyza64, st));
  } else {
    fails.count = d_cnt + 1;
    if ((rc = enqueue_supersample(s, *dc, st, B, 0, 0, frame_rows, w, sel_frame, sel_local, d_cnt, spa, d_xyza64,
                                  (unsigned long long*)d_stats, fails)))
      return rc;
  }
  if (d_n_supersampled) HIP_TRY(hipMemcpyAsync(d_n_supersampled, d_cnt, 8, hipMemcpyDeviceToDevice, st));
  if ((rc = stream_done(*dc, st))) return rc;
  if (failures) {
    unsigned long long cnt[2] = {0, 0};
    HIP_TRY(hipMemcpyAsync(cnt, d_cnt, sizeof(cnt), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    failures->count = cnt[1];
    if ((rc = copy_failures(fails, cnt[1], spa, failures))) return rc;
  }
  return 0;
}

}  // namespace grt_host

extern "C" {

int grt_supersample_shard_device(grt_scene* s, int device, void* stream, const grt_row_shard* sh,
                                 const grt_adaptive_config* cfg, double min_lum, const double* d_min_lum,
                                 const double* d_frame_ya, const uint8_t* d_frame_class,
                                 const double* sampling_mask_xyza, double* d_xyza64,
                                 uint64_t* d_n_supersampled, uint64_t* d_stats, grt_subsample_failures* failures) {
  return grt_host::supersample_shard(s, device, stream, sh, cfg, min_lum, d_min_lum, d_frame_ya, d_frame_class,
                                     sampling_mask_xyza, d_xyza64, nullptr, d_n_supersampled, d_stats, failures);
}

int grt_supersample_shard(grt_scene* s, int device, void* stream, const grt_row_shard* sh,
                          const grt_adaptive_config* cfg, double min_lum, const double* d_frame_ya,
                          const uint8_t* d_frame_class, const double* sampling_mask_xyza, double* d_xyza64,
                          uint64_t* n_supersampled, uint64_t* d_stats) {
  if (n_supersampled) *n_supersampled = 0;
  if (!s) return fail(-EINVAL, "null argument");
  DeviceCopy* dc;
  int rc = ensure_device(s, device, &dc);
  if (rc) return rc;
  HIP_TRY(hipSetDevice(device));
  DevBuf cnt;
  if ((rc = cnt.alloc(8))) return rc;
  HIP_TRY(hipMemsetAsync(cnt.p, 0, 8, (hipStream_t)stream));
  if ((rc = grt_supersample_shard_device(s, device, stream, sh, cfg, min_lum, nullptr, d_frame_ya, d_frame_class,
                                         sampling_mask_xyza, d_xyza64, (uint64_t*)cnt.p, d_stats, nullptr)))
    return rc;
  uint64_t v = 0;
  HIP_TRY(hipMemcpyAsync(&v, cnt.p, 8, hipMemcpyDeviceToHost, (hipStream_t)stream));
  HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
  if (n_supersampled) *n_supersampled = v;
  return 0;
}

// The luminance floor written to device memory (no host round trip): the multi-GPU
// adaptive pass hands it to grt_supersample_shard_device.  Scratch from the scene's
// grow-only arena on `device`, stream-ordered.
int grt_adaptive_floor_device(grt_scene* s, int device, void* stream, const double* d_y, uint32_t stride, uint64_t n,
                              double* d_min_lum) {
  if (!s || !d_min_lum || (n && (!d_y || stride == 0))) return fail(-EINVAL, "null argument");
  if (n > (uint64_t)INT_MAX) return fail(-EOVERFLOW, "more than INT_MAX luminances");
  DeviceCopy* dc;
  int rc = ensure_device(s, device, &dc);
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(dc->mu);
  HIP_TRY(hipSetDevice(device));
  hipStream_t st = (hipStream_t)stream;
  if (n == 0) {
    HIP_TRY(hipMemsetAsync(d_min_lum, 0, 8, st));  // +0.0
    return 0;
  }
  size_t bytes = 0;
  HIP_TRY(grt::luminance_floor_device(d_y, stride, n, floor_index(n), nullptr, &bytes, nullptr, st));
  if ((rc = ad_reserve(*dc, bytes))) return rc;
  if ((rc = stream_order(*dc, st))) return rc;
  HIP_TRY(grt::luminance_floor_device(d_y, stride, n, floor_index(n), dc->ad_mem, &bytes, d_min_lum, st));
  return stream_done(*dc, st);
}

}  // extern "C"
