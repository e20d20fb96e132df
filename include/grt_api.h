/*
 * grt_api.h — C ABI of the MI355X-native geodesic ray tracer (gr_raytracer_amd).
 *
 * This is the drop-in boundary for the hot path of mdreem/gr_raytracer:
 *
 *   Raytracer::render_section_to_cie_buffer_raw   (src/rendering/raytracer.rs:195-244)
 *   Raytracer::supersample                         (src/rendering/raytracer.rs:320-384)
 *     -> Scene::color_of_ray                       (src/rendering/scene.rs:114-220)
 *        -> Integrator::integrate / rkf45          (src/rendering/integrator.rs:78-268,
 *                                                   src/rendering/runge_kutta.rs:86-182)
 *        -> Objects::intersects (Sphere / Disc)    (src/scene_objects/objects.rs:65-120)
 *        -> redshift / texture / blend shade       (src/rendering/{redshift,texture,color}.rs)
 *
 * The reference binds these through Rust traits (`RenderableGeometry`, `Geometry`,
 * `GeodesicSolver`, `Hittable`, `TextureMap`, `TemperatureComputer`); see
 * src/geometry/geometry.rs:15-153.  Here the scene is flattened to a plain-old-data
 * descriptor (grt_scene_desc) built once per frame on the host (camera tetrad and
 * look-up tables included, exactly like `create_scene`, src/cli/shared.rs:131-321),
 * and the per-pixel work runs in hand-written HIP kernels for gfx950.
 *
 * All signatures use plain C types only.  Every function returns 0 on success or a
 * negative errno-style code; grt_last_error() returns the text of the last failure
 * on the calling thread.
 */
#ifndef GRT_API_H
#define GRT_API_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GRT_ABI_VERSION 3

/* ---- enums (values are part of the ABI) -------------------------------------- */

/* configuration.rs:111-129 GeometryType. */
enum grt_geometry_kind {
  GRT_GEOM_EUCLIDEAN = 0,     /* geometry/euclidean.rs, Cartesian chart, (+,-,-,-)   */
  GRT_GEOM_SCHWARZSCHILD = 1, /* geometry/schwarzschild.rs, spherical chart, (+,-,-,-) */
  GRT_GEOM_KERR = 2,          /* geometry/kerr.rs, Kerr-Schild Cartesian, (-,+,+,+)   */
  GRT_GEOM_KERR_BL = 3,       /* geometry/kerr_bl.rs, Boyer-Lindquist, (-,+,+,+)      */
  GRT_GEOM_EUCLIDEAN_SPHERICAL = 4 /* geometry/euclidean_spherical.rs, flat space in the
                                      spherical chart, (+,-,-,-)                        */
};

/* configuration.rs:162-177 TextureConfig. */
enum grt_texture_kind {
  GRT_TEX_BITMAP = 0,   /* texture.rs:41-102  TextureMapper (bilinear)           */
  GRT_TEX_CHECKER = 1,  /* texture.rs:212-257 CheckerMapper                      */
  GRT_TEX_BLACKBODY = 2 /* texture.rs:104-210 BlackBodyMapper (LUT over log10 T) */
};

/* configuration.rs:188-219 ObjectsConfig. */
enum grt_object_kind {
  GRT_OBJ_SPHERE = 0,          /* scene_objects/sphere.rs                           */
  GRT_OBJ_DISC = 1,            /* scene_objects/disc.rs                             */
  GRT_OBJ_VOLUMETRIC_DISC = 2  /* scene_objects/volumetric_disc.rs (Perlin fBm gas,
                                  constant-step raymarch per intersection)          */
};

/* rendering/temperature.rs: ConstantTemperatureComputer / KerrTemperatureComputer. */
enum grt_temperature_kind {
  GRT_TEMP_CONSTANT = 0,
  GRT_TEMP_KERR_LUT = 1
};

/* scene.rs:25-30 RayClass. */
enum grt_ray_class { GRT_CLASS_ESCAPED = 0, GRT_CLASS_CAPTURED = 1, GRT_CLASS_HIT = 2 };

/* color.rs:16-21 ToneMappingMethod. */
enum grt_tone_mapping { GRT_TONE_REINHARD = 0, GRT_TONE_GLOBAL_LINEAR = 1 };

/* Per-pixel status: which RaytracerError (raytracer.rs:20-52) aborted the pixel.
 * A pixel with a non-zero status keeps the reference default {(0,0,0,1), Escaped}
 * (raytracer.rs:204-210, :232-239).  Bit 7 flags are informational. */
enum grt_status {
  GRT_OK = 0,
  GRT_ERR_MAX_STEPS_REACHED = 1,     /* runge_kutta.rs:179-181 (100 retries)           */
  GRT_ERR_NO_CIRCULAR_ORBIT = 2,     /* circular_orbit.rs:93-101                        */
  GRT_ERR_BELOW_RISCO = 3,           /* temperature.rs:204-217                          */
  GRT_ERR_NON_FINITE_RADIUS = 4,     /* temperature.rs:199-202                          */
  GRT_FLAG_HIT_OVERFLOW = 0x80       /* the device hit pool was full: this ray's candidates
                                        past GRT_MAX_HITS are missing.  The *_async
                                        calls return it (grt_hit_pool_reserve, then trace
                                        again); the synchronous calls trace the flagged
                                        pixels again, growing the pool to their need, and
                                        return it only past 2^31 - 1 records.            */
};

/* Stop reason of the integration (integrator.rs:22-27), recorded per pixel. */
enum grt_stop_reason {
  GRT_STOP_NONE = 0, /* step budget exhausted, no terminal event */
  GRT_STOP_HORIZON = 1,
  GRT_STOP_CELESTIAL = 2,
  GRT_STOP_NAN = 3,
  GRT_STOP_CLOSED_ORBIT = 4
};

#define GRT_MAX_OBJECTS 8
/* Window candidates a ray keeps in its fixed workspace slots; any further ones go to a
 * device-wide hit pool, so every window's intersection reaches the pixel as in the
 * reference (scene.rs:139-152, :206-210).  An implementation constant, not a limit. */
#define GRT_MAX_HITS 16

/* ---- POD scene descriptor ------------------------------------------------------ */

typedef struct grt_texture_desc {
  int32_t kind;            /* grt_texture_kind */
  int32_t _pad;
  double beaming_exponent; /* apply_beaming exponent (color.rs:72-80)              */
  /* GRT_TEX_BITMAP: caller-owned RGBA8 texels, row-major, width*height*4 bytes.    */
  const uint8_t* rgba;
  uint32_t width, height;
  /* GRT_TEX_CHECKER: cell counts and the two colours already in CIE XYZA          */
  double checker_width, checker_height;
  double c1[4], c2[4];
} grt_texture_desc;

typedef struct grt_object_desc {
  int32_t kind;          /* grt_object_kind */
  int32_t temp_kind;     /* grt_temperature_kind (Disc only)                       */
  /* Sphere: radius, Cartesian centre, constant temperature (sphere.rs:14-35).     */
  double radius;
  double center[3];
  double temperature;
  /* Disc: annulus in the z = 0 plane (disc.rs:335-356).                            */
  double inner_radius, outer_radius;
  /* Disc temperature model: constant, or the KerrTemperatureComputer LUT
   * (temperature.rs:29-118): r_isco, and n (r, T) pairs strictly increasing in r. */
  double temp_constant;
  double r_isco;
  const double* lut_r;
  const double* lut_t;
  uint32_t lut_n;
  uint32_t _pad2;
  grt_texture_desc texture;
  /* GRT_OBJ_VOLUMETRIC_DISC (volumetric_disc.rs:21-95, configuration.rs:200-217).
   * inner/outer radius, the temperature model and the texture are the Disc fields
   * above (cli/shared.rs:219-307 builds it like a Disc).  The axis is the configured
   * one, (0,0,1) when absent; grt_scene_create normalises it and derives e1, e2
   * exactly as VolumetricDisc::new (:61-73) and the Perlin permutation table from
   * perlin_seed (noise 0.9.0 PermutationTable::new, see grt_perlin_permutation). */
  double axis[3];
  double thickness;                        /* Gaussian sigma; capture slab 3x this  */
  double march_step_size;                  /* raymarch step (config step_size)      */
  double density_multiplier;
  double brightness_reference_temperature;
  double absorption, scattering;           /* sigma_a, sigma_s                      */
  double noise_scale[3];
  double noise_offset;
  uint64_t march_max_steps;                /* raymarch samples per intersection     */
  uint32_t num_octaves;
  uint32_t perlin_seed;                    /* config perlin_seed, default 1         */
} grt_object_desc;

/* The camera after Camera::new (camera.rs:151-196): position and velocity in the
 * geometry's native chart, the rotated + Lorentz-boosted tetrad rows t, x, y, z,
 * and the scalars used by get_direction_for (camera.rs:214-232). */
typedef struct grt_camera_desc {
  double position[4];
  double velocity[4];
  double tetrad[4][4];       /* tetrad[0]=e_t, [1]=e_x, [2]=e_y, [3]=e_z (components) */
  double alpha;              /* vertical field of view (pi/4 for the CLI, shared.rs:162) */
  double tan_half_alpha;     /* tan(alpha/2), host libm                                  */
  int64_t rows, cols;
  double spatial_signature;  /* signature[3]                                             */
  double spatial_handedness; /* camera.rs:134-148                                        */
  /* sin/cos of the camera's polar angle (position[2]) for the spherical and BL charts,
   * evaluated once on the host (libm) like every other per-frame constant.            */
  double sin_theta, cos_theta;
} grt_camera_desc;

typedef struct grt_scene_desc {
  uint32_t abi_version;      /* = GRT_ABI_VERSION */
  int32_t geometry;          /* grt_geometry_kind */
  double radius;             /* r_s (Schwarzschild radius)                      */
  double a;                  /* spin parameter (Kerr, KerrBL)                   */
  double horizon_epsilon;
  /* IntegrationConfiguration (integrator.rs:46-67), from GlobalOpts (cli.rs:5-47). */
  uint64_t max_steps;
  double max_radius;
  double step_size;
  double epsilon;
  grt_camera_desc camera;
  grt_texture_desc celestial;
  double celestial_temperature;
  uint32_t n_objects;        /* <= GRT_MAX_OBJECTS, tested in config order     */
  uint32_t _pad;
  grt_object_desc objects[GRT_MAX_OBJECTS];
  /* BlackBodyMapper LUT (texture.rs:120-138): n entries of (log10 T, X, Y, Z).    */
  const double* bb_log_t;
  const double* bb_xyz;      /* 3*n, interleaved X,Y,Z                          */
  uint32_t bb_n;
  uint32_t _pad3;
  /* Inverse sRGB companding (color.rs:301-308) of the 256 8-bit codes.            */
  double srgb_to_linear[256];
  /* AdaptiveSamplingConfig.object_hit_opacity_threshold (configuration.rs:36).    */
  double object_hit_opacity_threshold;
} grt_scene_desc;

/* ---- host-side scene setup (the Rust host's create_scene, cli/shared.rs) -------- */

/* GlobalOpts (cli.rs:5-47). */
typedef struct grt_global_opts {
  int64_t width, height;
  double step_size;
  uint64_t max_steps;
  double max_radius;
  double epsilon;
  double camera_position[3];
  double phi, theta, psi;
  int32_t tone_mapping;       /* 0 Reinhard, 1 GlobalLinear (color.rs:16-21) */
  int32_t show_sampling_mask;
  uint8_t sampling_mask_color[3];
  uint8_t _pad[5];
} grt_global_opts;

/* AdaptiveSamplingConfig (configuration.rs:21-94). */
typedef struct grt_adaptive_config {
  int32_t enabled;
  uint32_t samples_per_axis;
  double luminance_contrast_threshold;
  double opacity_contrast_threshold;
  int32_t has_minimum_luminance;
  int32_t exclude_background_contrast;
  double minimum_luminance;
  double object_hit_opacity_threshold;
} grt_adaptive_config;

typedef struct grt_host_scene grt_host_scene; /* owns textures + LUTs + desc */

void grt_default_global_opts(grt_global_opts* opts);
void grt_default_adaptive_config(grt_adaptive_config* cfg);

/* Parse a scene TOML (configuration.rs schema) and build the frame exactly like
 * `main.rs:80-116` + `cli/<geometry>.rs::create_scene_internal` + `create_scene`.
 * Texture paths are resolved relative to `resource_root` (NULL = cwd). */
int grt_host_scene_load(const char* toml_path, const char* resource_root,
                        const grt_global_opts* opts, grt_host_scene** out);
/* Geometry and integration configuration only (no camera, textures or objects): what
 * `render-ray-at` uses (main.rs:143-168 builds the geometry, not a scene). */
int grt_host_geometry_load(const char* toml_path, const grt_global_opts* opts,
                           grt_host_scene** out);
const grt_scene_desc* grt_host_scene_desc(const grt_host_scene* s);
/* The info-level lines the reference logs while it builds this scene, one per line, in
 * order (today the temperature LUT's, KerrTemperatureComputer::new, temperature.rs:55-102:
 * the r_isco clamp, "Computed r_isco: ...", "Max f: ...", "Computed m_dot: ..."; numbers
 * in Rust's f64 Display form).  Owned by the scene; "" when there are none. */
const char* grt_host_scene_log(const grt_host_scene* s);
void grt_host_scene_adaptive(const grt_host_scene* s, grt_adaptive_config* out);
int grt_host_scene_destroy(grt_host_scene* s);

/* Camera::new (camera.rs:151-196) for an explicit position/velocity in the native
 * chart of `geometry` (radius, a as in grt_scene_desc).  Fails with -EDOM when a
 * tetrad is not orthonormal (TetradValidator, tetrad.rs:60-131). */
int grt_camera_build(int32_t geometry, double radius, double a,
                     const double position[4], const double velocity[4], double alpha,
                     int64_t rows, int64_t cols, double phi, double theta, double psi,
                     grt_camera_desc* out);

/* Per-geometry support quantities used by the host to place the camera. */
int grt_stationary_velocity(int32_t geometry, double radius, double a,
                            const double position[4], double out[4]);
int grt_zamo_velocity(int32_t geometry, double radius, double a,
                      const double position[4], double out[4]);
/* Chart conversions (spherical_coordinates_helper.rs:5-61). */
void grt_cartesian_to_spherical(const double in[4], double out[4]);
void grt_cartesian_to_boyer_lindquist(double a, const double in[4], double out[4]);

/* KerrTemperatureComputer::new (temperature.rs:45-118): fills n (r, T) pairs.
 * Returns -ERANGE on DenominatorCloseToZero / NoCircularOrbitPossible. */
int grt_kerr_temperature_lut(double temperature, double outer_radius, double a,
                             double radius, uint32_t n, double* lut_r, double* lut_t,
                             double* r_isco);
double grt_r_isco(double radius, double a);
/* BlackBodyMapper::new (texture.rs:121-138): n entries of (log10 T, XYZ). */
int grt_blackbody_lut(uint32_t n, double* log_t, double* xyz);
/* integrate_blackbody_xyz (black_body_radiation.rs:18-41). */
void grt_blackbody_xyz(double temperature, double redshift, double out_xyz[3]);
/* srgb_to_xyz (color.rs:310-332), alpha := a/255 (CIETristimulus::from_color). */
void grt_srgb_to_xyza(uint8_t r, uint8_t g, uint8_t b, uint8_t a, double out[4]);
/* Perlin::new(seed) of the `noise` crate 0.9.0 (volumetric_disc.rs:83), restated from
 * its published source (the crate is not vendored): PermutationTable::new seeds
 * rand_xorshift 0.3's XorShiftRng with the words [1, seed, seed, seed] and shuffles
 * 0..=255 with rand 0.8's SliceRandom::shuffle (Fisher-Yates, gen_range by widening
 * multiply + rejection).  out[i] = values[i]. */
void grt_perlin_permutation(uint32_t seed, uint8_t out[256]);
/* VolumetricDisc::new's frame (volumetric_disc.rs:61-73): the normalised axis
 * ((0,0,1) when |axis|^2 <= f64::EPSILON) and the in-plane unit vectors e1, e2. */
void grt_volumetric_frame(const double axis_in[3], double axis[3], double e1[3], double e2[3]);
/* xyz_to_srgb (color.rs:225-241): one XYZ colour -> sRGB8, linear * exposure, no
 * tone mapping (the `blackbody` subcommand, cli/blackbody.rs:7-25). */
void grt_xyz_to_srgb(const double xyz[3], double exposure, uint8_t rgb_out[3]);
/* run_blackbody_spectrum (cli/blackbody.rs:27-95): width x height RGBA8 image of
 * integrate_blackbody_xyz(T, z), T linear in x over [min, max] temperature, z linear
 * in y over [min, max] redshift, tone-mapped like a render (exposure 1), alpha 255. */
int grt_blackbody_spectrum(double min_temperature, double max_temperature, double min_redshift,
                           double max_redshift, uint32_t width, uint32_t height,
                           int32_t tone_mapping, uint8_t* rgba_out);
/* xyz -> tone-mapped sRGB8 (color.rs:204-298), whole buffer = grt_linear_max (only for
 * GlobalLinear) + grt_tonemap.  Split so that a frame spread over several processes
 * can reduce the three channel maxima (MAX) before mapping its own rows. */
void grt_linear_max(const double* xyza, size_t n, double exposure, double max3[3]);
int grt_tonemap(const double* xyza, size_t n, int32_t tone_mapping, double exposure,
                const double max3[3], uint8_t* rgb_out);
int grt_xyz_to_srgb8(const double* xyza, size_t n, int32_t tone_mapping, double exposure,
                     uint8_t* rgb_out);

/* ---- device hot path -------------------------------------------------------- */

typedef struct grt_scene grt_scene; /* device-resident copy, one per GPU on demand */

typedef struct grt_stats {
  uint64_t accepted_steps; /* iterations of integrator.rs:100 that produced a step     */
  uint64_t attempts;       /* rkf45_step evaluations (6 RHS each)                      */
  uint64_t rays;
  uint64_t hit_overflows;  /* pixels flagged GRT_FLAG_HIT_OVERFLOW: for the synchronous calls
                              0 unless the pool would need more than 2^31 - 1 records     */
  double kernel_ms;        /* hipEvent time of the integration kernel(s)               */
  /* VolumetricDisc raymarches (volumetric_disc.rs:199-328): one per window-nearest
   * volumetric intersection whose colour reaches the composite, and their samples. */
  uint64_t march_jobs;
  uint64_t march_samples;
  uint64_t march_noise_samples; /* samples inside the density's support (fBm evaluated) */
  uint64_t march_emit_samples;  /* samples with density > 0 that emitted                */
} grt_stats;

/* Optional per-sample sub-pixel offsets (get_ray_for_offset, camera.rs:247-254):
 * sample k traces pixel (row0 + pix[k] / cols, col0 + pix[k] % cols) at (dx[k], dy[k]). */
typedef struct grt_offsets {
  uint64_t count;
  const uint32_t* pixel_index;
  const double* dx;
  const double* dy;
} grt_offsets;

/* Optional extra per-sample outputs for parity work (any pointer may be NULL). */
typedef struct grt_aux_out {
  double* xyza64;       /* 4 doubles per sample: the f64 colour before the f32 cast   */
  uint32_t* steps;      /* accepted steps per sample                                  */
  uint8_t* stop_reason; /* grt_stop_reason per sample                                 */
  uint32_t* hits;       /* windows with an intersection per sample: intersections.len()
                           of scene.rs:141-152 before the terminal colour (for a pixel
                           aborted by a window error, the windows before it)           */
} grt_aux_out;

int grt_scene_create(const grt_scene_desc* desc, grt_scene** out);
int grt_scene_destroy(grt_scene* scene);
const char* grt_last_error(void);
int grt_device_count(void);
/* SHA-256 (64 hex digits) of the sources this library was built from
 * (gr_raytracer_amd/source_hash.py; "unstamped" for a copy built outside the checkout).
 * No reference counterpart: it ties a prebuilt library to its checkout. */
const char* grt_source_hash(void);

/* Trace a rows x cols rectangle at 1 spp (or the offset list) on `device`.
 * Host output arrays, row-major over the rectangle (or per offset entry). */
int grt_render_pixels(grt_scene* scene, int device, uint32_t row0, uint32_t col0,
                      uint32_t rows, uint32_t cols, const grt_offsets* offsets,
                      float* xyza_out, uint8_t* class_out, uint8_t* status_out,
                      const grt_aux_out* aux, grt_stats* stats);

/* Same, but every output pointer is a DEVICE pointer on `device` and the work is
 * enqueued on `stream` (a hipStream_t, NULL = default stream) without a host sync.
 * `device_stats` is a device buffer of 4 uint64 counters (accepted, attempts, rays,
 * overflows) that the kernel accumulates into (caller zeroes it). */
int grt_render_pixels_async(grt_scene* scene, int device, void* stream,
                            uint32_t row0, uint32_t col0, uint32_t rows, uint32_t cols,
                            float* d_xyza, uint8_t* d_class, uint8_t* d_status,
                            double* d_xyza64, uint32_t* d_steps, uint8_t* d_stop,
                            uint64_t* d_stats);

/* Whole section with the reference's adaptive supersampling
 * (render_section_to_cie_buffer[_supersampled], raytracer.rs:177-318), fully on the
 * device: 1-spp pass, exact 99th-percentile floor, 8-neighbour selection, 16 jittered
 * rays per selected pixel, ordered average.  Output: f64 XYZA per pixel. */
int grt_render_section(grt_scene* scene, int device, uint32_t from_row, uint32_t from_col,
                       uint32_t to_row, uint32_t to_col, const grt_adaptive_config* cfg,
                       const double* sampling_mask_xyza, double* xyza_out,
                       uint8_t* class_out, uint64_t* n_supersampled, grt_stats* stats,
                       uint8_t* status_out /* nullable: grt_status of each pixel's 1-spp ray, the
                                              error the reference logs at raytracer.rs:232-239 */);

/* Failed sub-samples of the supersample pass (supersample's Err arm, raytracer.rs:357-362,
 * which the reference logs as "Unable to compute color for ray at pixel (col, row)").
 * The caller provides `capacity` entries; `count` returns how many failed (it may exceed
 * the capacity).  Entries are sorted by (pixel, sample). */
typedef struct grt_subsample_failures {
  uint64_t capacity;
  uint32_t* pixel;   /* pixel index, row-major in the section (shard: in the frame)      */
  uint32_t* sample;  /* nullable: stratum index stratum_row * spa + stratum_col          */
  uint8_t* status;   /* grt_status of the failed sub-sample ray                         */
  uint64_t count;    /* out                                                             */
  /* Nullable.  When set, the list also holds the sub-rays that ended without an error
   * but on NaN coordinates or without a terminal event (status 0, stop GRT_STOP_NAN /
   * GRT_STOP_NONE), which the reference logs from color_of_ray (scene.rs:178-183,
   * :196-202); every entry then carries its stop reason and accepted steps.          */
  uint8_t* stop;
  uint32_t* steps;   /* nullable */
} grt_subsample_failures;

/* grt_render_section plus the failed sub-samples (nullable) and the 1-spp rays' stop
 * reasons and accepted steps per section pixel (nullable; the reference's color_of_ray
 * logs the NaN and no-terminal-event rays, scene.rs:178-183, :196-202).  The whole
 * section stays on the device between the 1-spp pass and the supersample pass: the
 * luminance floor, the selection, its compaction and count, and the sub-ray launches'
 * sizes are decided there (no host round trip). */
int grt_render_section_ex(grt_scene* scene, int device, uint32_t from_row, uint32_t from_col,
                          uint32_t to_row, uint32_t to_col, const grt_adaptive_config* cfg,
                          const double* sampling_mask_xyza, double* xyza_out, uint8_t* class_out,
                          uint64_t* n_supersampled, grt_stats* stats, uint8_t* status_out,
                          grt_subsample_failures* failures, uint8_t* stop_out, uint32_t* steps_out);

/* Row-band sharding of one frame across GPUs (multi-GPU render).
 * The frame's rows are cut into bands of `band_rows` rows (the last may be short);
 * shard s of n owns the bands b with b % n == s.  Its output is the full-width rows of
 * those bands, packed in increasing frame order ("local rows").  Cyclic bands balance
 * the cost, which is concentrated around the shadow and the disc.  The reference has
 * one process rendering everything (raytracer.rs:195-244); the per-pixel results of a
 * shard are identical to rendering the same rows through grt_render_pixels. */
typedef struct grt_row_shard {
  uint32_t band_rows; /* >= 1; a multiple of 8 keeps the 8x8 pixel tiles inside a band */
  uint32_t shard;     /* < n_shards */
  uint32_t n_shards;  /* >= 1 */
} grt_row_shard;

/* Number of local rows of shard `sh` in a frame of `frame_rows` rows. */
uint32_t grt_shard_row_count(uint32_t frame_rows, const grt_row_shard* sh);
/* Frame row of local row `local_row` of shard `sh`. */
uint32_t grt_shard_frame_row(uint32_t local_row, const grt_row_shard* sh);

/* Trace all local rows of a shard (full frame width) at 1 spp: host outputs,
 * local-row-major, like grt_render_pixels. */
int grt_render_shard(grt_scene* scene, int device, const grt_row_shard* sh, float* xyza_out,
                     uint8_t* class_out, uint8_t* status_out, const grt_aux_out* aux,
                     grt_stats* stats);
/* Same with device outputs on `stream`, like grt_render_pixels_async. */
int grt_render_shard_async(grt_scene* scene, int device, void* stream, const grt_row_shard* sh,
                           float* d_xyza, uint8_t* d_class, uint8_t* d_status, double* d_xyza64,
                           uint32_t* d_steps, uint8_t* d_stop, uint64_t* d_stats);

/* ---- one frame across several GPUs of this process (north_star) ----
 * The north-star layout behind the C ABI: the frame's rows in cyclic bands of band_rows
 * (band b -> devices[b % n_devices], grt_row_shard), one host thread per device tracing
 * its bands (grt_render_shard_async), and ONE RCCL gather (grouped send / receive over
 * xGMI, one communicator per device from ncclCommInitAll) of every device's pixel records
 * to devices[0], where a kernel de-interleaves them into frame order.  With supersampling
 * (cfg->enabled, or a sampling mask) one RCCL allgather of each pixel's (Y, alpha, class)
 * (17 B) comes first: the selection stencil reads neighbours in other devices' bands and
 * the luminance floor is a percentile of the whole frame; each device then supersamples
 * its own pixels (grt_supersample_shard_device).  Replaces the single-process frame
 * driver of the `render` command: render_section_to_cie_buffer[_raw|_supersampled]
 * (raytracer.rs:195-318) as Raytracer::render_section calls it (:460-497, main.rs:80-116).
 * Every pixel equals grt_render_pixels / grt_render_section_ex of the same frame on one
 * device.  The communicators, streams and device scratch are created on the first call
 * for a device list and kept (grt_multi_release frees them). */
#define GRT_MULTI_MAX_DEVICES 16

/* Host outputs in frame order (camera rows x cols); a NULL field is not gathered.  The
 * gather moves 2 B per pixel (class, status) plus the requested fields: f32 XYZA + class
 * + status is the 18-B pixel record of the 1-spp frame. */
typedef struct grt_frame_out {
  float* xyza;         /* f32 XYZA (1-spp frames only: NULL with supersampling)          */
  double* xyza64;      /* f64 XYZA, the supersampled colour where selected (required with
                          supersampling)                                                  */
  uint8_t* ray_class;  /* RayClass of the 1-spp ray                                       */
  uint8_t* status;     /* grt_status of the 1-spp ray (raytracer.rs:232-239)              */
  uint8_t* stop;       /* grt_stop_reason of the 1-spp ray                                */
  uint32_t* steps;     /* accepted steps of the 1-spp ray                                 */
} grt_frame_out;

typedef struct grt_multi_report {
  uint32_t n_devices;
  uint32_t record_bytes;     /* bytes per pixel the gather moved                                */
  uint32_t attempts;         /* traces of the frame (more than 1 when a hit pool had to grow)   */
  uint32_t _pad;
  double wall_ms;            /* the whole call, host clock                                      */
  double gather_ms;          /* last trace: RCCL gather + de-interleave on devices[0] (events)  */
  double allgather_ms;       /* supersampling: the (Y, alpha, class) allgather, max over devices */
  double trace_ms[GRT_MULTI_MAX_DEVICES];        /* per device: its trace (+ supersample pass)   */
  uint64_t accepted_steps[GRT_MULTI_MAX_DEVICES];
  uint64_t rows[GRT_MULTI_MAX_DEVICES];          /* frame rows each device traced                */
} grt_multi_report;

/* Render the whole camera frame over n_devices distinct GPUs (1 <= n <= 16; n = 1 runs the
 * same RCCL path with a one-rank communicator).  cfg (nullable): the scene's adaptive
 * configuration (grt_host_scene_adaptive), NULL or !enabled = 1 spp; sampling_mask_xyza
 * (nullable): paint the selected pixels instead (--show-sampling-mask).  stats: summed
 * counters, kernel_ms the slowest device's trace.  failures (nullable): every device's
 * failed sub-samples, frame pixel indices, sorted by (pixel, sample).  A trace that lost
 * hit candidates grows the pools and traces the frame again (at most 3 traces; after
 * that the pixels keep GRT_FLAG_HIT_OVERFLOW and stats->hit_overflows counts them). */
int grt_render_frame_multi(grt_scene* scene, int n_devices, const int* devices, uint32_t band_rows,
                           const grt_adaptive_config* cfg, const double* sampling_mask_xyza,
                           const grt_frame_out* out, uint64_t* n_supersampled, grt_stats* stats,
                           grt_subsample_failures* failures, grt_multi_report* report);
/* Free the communicators, streams and scratch grt_render_frame_multi keeps (no frame may
 * be in flight). */
void grt_multi_release(void);

/* The device hit pool that keeps the window candidates past a ray's GRT_MAX_HITS slots
 * (no reference counterpart: the reference's per-ray Vec grows, scene.rs:139-152).
 * A trace starts with the pool at its minimum (grt_set_hit_pool_min, 2^20 records) or
 * the size a measured need grew it to; a trace that needs more flags the pixels it could
 * not keep (GRT_FLAG_HIT_OVERFLOW, grt_stats.hit_overflows).  The synchronous calls then
 * trace those pixels again (growing the pool to their need).  After an *_async call whose
 * d_stats[3] is non-zero, call this with records = 0 (waits for the device, then sizes
 * the pool for the largest trace since the last call) or with an explicit record count,
 * and trace again.  *capacity (nullable) returns the pool size in records. */
int grt_hit_pool_reserve(grt_scene* scene, int device, uint64_t records, uint64_t* capacity);
/* Smallest pool a trace allocates (default 2^20 records; tests lower it to exercise a
 * full pool).  Applies to pools allocated or grown afterwards. */
int grt_set_hit_pool_min(uint64_t records);
/* Sub-rays per supersample trace launch (default 0 = 2^21; at least one pixel's spa^2
 * sub-rays per launch).  The supersample pass runs the selected pixels in chunks of
 * this many sub-rays, each chunk's live count read on the device.  Scheduling only:
 * results are identical for every chunk size (tests force several partly filled ones). */
int grt_set_sub_chunk(uint64_t sub_rays);

/* ---- adaptive supersampling of a frame split across GPUs -------
 * render_section_to_cie_buffer_supersampled (raytracer.rs:257-318) with the frame's
 * rows spread over processes.  Per rank:
 *   1. grt_render_shard_async(..., d_xyza64, ...): the 1-spp pass of its row bands;
 *   2. allgather of every pixel's (Y, alpha) and class, frame order (17 B per pixel:
 *      the selection stencil reads its 8 neighbours, which may belong to other ranks,
 *      and the luminance floor is a percentile over the whole frame);
 *   3. grt_adaptive_min_luminance over the frame's Y: identical on every rank;
 *   4. grt_supersample_shard: selection of the shard's pixels, samples_per_axis^2
 *      jittered rays per selected pixel, ordered average into the shard's f64 XYZA.
 * The result is identical to grt_render_section over the whole frame. */

/* resolve_minimum_luminance (raytracer.rs:118-129): cfg->minimum_luminance when set,
 * else 1e-3 x the ((n-1) * 0.99)-th luminance in f64::total_cmp order (0 when n = 0). */
double grt_adaptive_min_luminance(const double* lum, uint64_t n, const grt_adaptive_config* cfg);
/* The same value from n DEVICE luminances d_y[stride * i] on `device`, selected on the
 * GPU (radix sort in total_cmp order; synchronises `stream`).  Returns 0 or -errno. */
int grt_adaptive_min_luminance_device(int device, void* stream, const double* d_y, uint32_t stride, uint64_t n,
                                      const grt_adaptive_config* cfg, double* out);

/* collect_pixels_to_supersample (raytracer.rs:386-458) over the local pixels of shard
 * `sh` + supersample (:320-384), on `device`, enqueued on `stream` and synchronised
 * before returning (the selection count sizes the second trace).
 * d_frame_ya: (Y, alpha) per frame pixel, 2 f64, frame order; d_frame_class: RayClass
 * per frame pixel; d_xyza64: the shard's 1-spp f64 XYZA (local rows, grt_render_shard
 * order), overwritten in place for the selected pixels; sampling_mask_xyza (host,
 * 4 f64, nullable): paint the selected pixels instead (--show-sampling-mask,
 * raytracer.rs:285-295).  d_stats: 4 uint64 device counters, accumulated. */
int grt_supersample_shard(grt_scene* scene, int device, void* stream, const grt_row_shard* sh,
                          const grt_adaptive_config* cfg, double min_lum, const double* d_frame_ya,
                          const uint8_t* d_frame_class, const double* sampling_mask_xyza,
                          double* d_xyza64, uint64_t* n_supersampled, uint64_t* d_stats);
/* The same, asynchronous on `stream` with everything on the device: the floor is
 * *d_min_lum when d_min_lum is non-null (grt_adaptive_floor_device), else min_lum; the
 * selection count goes to *d_n_supersampled (device uint64, nullable).  failures
 * (nullable) synchronises `stream` to return the failed sub-samples (frame pixel
 * indices). */
int grt_supersample_shard_device(grt_scene* scene, int device, void* stream, const grt_row_shard* sh,
                                 const grt_adaptive_config* cfg, double min_lum, const double* d_min_lum,
                                 const double* d_frame_ya, const uint8_t* d_frame_class,
                                 const double* sampling_mask_xyza, double* d_xyza64,
                                 uint64_t* d_n_supersampled, uint64_t* d_stats,
                                 grt_subsample_failures* failures);
/* resolve_minimum_luminance's relative floor of n DEVICE luminances d_y[stride * i],
 * written to *d_min_lum (device double) on `stream` without a host copy (n <= INT_MAX;
 * n = 0 gives +0.0).  A configured minimum_luminance is the caller's constant instead. */
int grt_adaptive_floor_device(grt_scene* scene, int device, void* stream, const double* d_y, uint32_t stride,
                              uint64_t n, double* d_min_lum);

/* The image files of Raytracer::render_section (raytracer.rs:460-497): an 8-bit RGB
 * PNG, and the Radiance .hdr that stores XYZ as its RGB channels (f32, RGBE). */
int grt_write_png_rgb(const char* path, const uint8_t* rgb, uint32_t width, uint32_t height);
int grt_write_hdr_xyz(const char* path, const double* xyza, uint32_t width, uint32_t height);

/* ---- whole trajectories (render-ray / render-ray-at) ------ */
/* Integrator::integrate keeping every Step (integrator.rs:78-174), as
 * Raytracer::integrate_ray_at_point (raytracer.rs:499-507, `render-ray`) and
 * integrate_and_save_ray (cli/shared.rs:107-129, `render-ray-at`) use it.  Ray k's
 * records are steps_out[(k * capacity + i) * 9 + f], i = 0 .. min(n_steps[k], capacity)
 * - 1, f = 0: affine parameter t; 1..4: position x^mu in the geometry's own chart;
 * 5..8: momentum_from_state p^mu.  Record 0 is the initial state.  n_steps[k] counts
 * every step, also those beyond `capacity`; stop_out is a grt_stop_reason, status_out a
 * grt_status (GRT_ERR_MAX_STEPS_REACHED: rkf45's Err, the reference writes no CSV). */
int grt_trace_pixels(grt_scene* scene, int device, uint64_t n, const double* rows,
                     const double* cols, uint64_t capacity, double* steps_out,
                     uint64_t* n_steps, uint8_t* stop_out, uint8_t* status_out);
/* Rays given by position and contravariant momentum in the geometry's chart (n x 4). */
int grt_trace_rays(grt_scene* scene, int device, uint64_t n, const double* positions,
                   const double* momenta, uint64_t capacity, double* steps_out,
                   uint64_t* n_steps, uint8_t* stop_out, uint8_t* status_out);

/* ---- invariant monitors (off the render path) --------------------------------- */
/* The reference's per-ray health checks over a rows x cols rectangle, re-integrating
 * each ray with the monitors on:
 *  - the null condition of the camera ray: Scene::color_of_ray logs an error when
 *    |k.k| >= 1e-10 (scene.rs:116-124);
 *  - the debug-build drift monitors of Integrator::integrate (integrator.rs:91-146): the
 *    largest |k.k| over the accepted steps and the largest drift of each constant of
 *    motion (get_constants_of_motion: E, L_z, and Carter's Q for KerrBL) from its value at
 *    step 0, relative when |initial| > 1e-12, warned above 1e-4 (report_drifts, :176-201).
 *    Rays whose rkf45 fails return Err before report_drifts and report no drift. */
typedef struct grt_health {
  uint64_t rays;
  uint64_t failed;                 /* rkf45 Err (MaxStepsReached): no drift report          */
  uint64_t null_violations;        /* camera rays with |k.k| >= 1e-10                        */
  double max_null;                 /* largest |k.k| of a camera ray                         */
  uint64_t kk_drift_rays;          /* rays whose largest |k.k| along the path > 1e-4         */
  double max_kk_drift;
  uint32_t n_constants;            /* 2 (E, L_z) or 3 (KerrBL: E, L_z, Q)                    */
  uint32_t _pad;
  uint64_t constant_drift_rays[3]; /* rays whose drift of constant c > 1e-4                  */
  double max_constant_drift[3];
} grt_health;
/* per_ray (nullable): rows*cols x 5 doubles -- |k.k| of the camera ray, largest |k.k| along
 * the path, largest drift of E, L_z, Q (0 where not defined). */
int grt_health_pixels(grt_scene* scene, int device, uint32_t row0, uint32_t col0, uint32_t rows,
                      uint32_t cols, grt_health* out, double* per_ray);

/* render_ray_at's initial ray (cli/{euclidean,schwarzschild,kerr,kerr_bl}.rs): the unit
 * spatial `direction` in the local tetrad at the Cartesian `position` (t = 0), as a
 * native-chart position and contravariant momentum for grt_trace_rays.  -EINVAL when
 * the direction is degenerate or the momentum is not future-directed
 * (assert_future_directed, cli/shared.rs:79-86). */
int grt_ray_at(int32_t geometry, double radius, double a, const double position[3],
               const double direction[3], double position_out[4], double momentum_out[4]);
/* IntegratedRay::save (ray.rs:35-54): "i,t,tau,x,y,z" then one line per record
 * (step, t, Cartesian x^0..x^3), f64 printed like Rust's Display. */
int grt_write_trajectory_csv(const char* path, int32_t geometry, double a, const double* steps,
                             uint64_t n_records);
/* Rust Display of one f64 into buf (NUL-terminated, truncated to cap); returns its length. */
size_t grt_format_f64(double v, char* buf, size_t cap);

/* ---- device output stage ------------------------------- */
/* Replaces xyz_to_linear_srgb_buffer + linear_srgb_to_srgb_buffer (color.rs:204-298),
 * called by Raytracer::render_section for non-HDR files (raytracer.rs:460-497).
 * GlobalLinear needs the per-channel maxima of (linear sRGB * exposure) over the WHOLE
 * frame, folded from 0.0 (color.rs:238-258): grt_linear_max_async writes them to
 * d_max3 (3 doubles, device); a frame split across GPUs allreduces them (MAX) before
 * grt_tonemap_async.  Byte-identical to the reference (glibc pow restated on device).
 * d_xyza: n x 4 f64 (the render's xyza64 output); d_rgb: n x 3 u8.  Async on `stream`. */
int grt_linear_max_async(int device, void* stream, const double* d_xyza, uint64_t n,
                         double exposure, double* d_max3);
int grt_tonemap_async(int device, void* stream, const double* d_xyza, uint64_t n,
                      int32_t tone_mapping, double exposure, const double* d_max3,
                      uint8_t* d_rgb);
/* Host buffers in and out, same result as grt_xyz_to_srgb8, computed on `device`. */
int grt_xyz_to_srgb8_device(int device, const double* xyza, size_t n, int32_t tone_mapping,
                            double exposure, uint8_t* rgb_out);

/* Floating-point contraction of the trace (no reference counterpart: the reference's Rust
 * never fuses a*b + c).  0 = exact (default): every multiply and add rounded separately in
 * the reference's order, so pixels are bit-identical to the reference's wherever the libm
 * calls are.  1 = fused: the light charts (Euclidean, Schwarzschild,
 * KerrBL, EuclideanSpherical) run kernels compiled with FMA contraction -- the same
 * algorithm and operation order, one rounding per fused pair -- which is faster (C2 -17%,
 * C3 -13%) and keeps every robust pixel within the north-star 1e-4 relative per channel
 * (tests/test_fused.py), but no longer bit-identical; Kerr-Schild always runs exact (its
 * finite-difference metric turns the changed roundings into other step sequences).
 * It applies to frame traces (grt_render_*, grt_supersample_shard*, grt_render_frame_multi);
 * trajectories (grt_trace_*), monitors and the work-order probe always run exact.
 * Process-wide; each trace reads it once when it is enqueued. */
int grt_set_arithmetic(int mode);
int grt_get_arithmetic(void);

/* Kernel launch geometry knobs (persistent grid). 0 = library default: 256 threads per
 * block, 2w blocks per CU for an integrate kernel that keeps w waves per SIMD resident
 * (w = 3 for Schwarzschild, KerrBL and the flat charts; 2 for Kerr-Schild and scenes with
 * a VolumetricDisc).  Scheduling only: results are identical for every shape. */
int grt_set_launch_config(int blocks_per_cu, int threads_per_block);
/* Tile queue order of rectangle / shard traces: 0 = row-major 8x8 tiles; 1 = a probe
 * pass (one capped ray per tile) then the tiles with the longest predicted rays first;
 * -1 = automatic (default: probe order for Kerr-Schild / Schwarzschild when
 * max_steps >= 262144 over >= 1024 tiles; KerrBL's Mino-time rays are all short).
 * Scheduling only: every pixel's result is identical in all modes. */
int grt_set_schedule(int mode);
/* Probe-ordered traces (above) hand the queue out from both ends: on every SIMD the wave
 * in an even hardware slot takes the tiles with the longest predicted rays, at raised
 * issue priority, the others take the shortest (1 = default); 0 = one end, longest
 * first, for every wave.  Scheduling only: results are identical in both modes. */
int grt_set_two_ended(int on);
/* Long-ray hand-off of Kerr-Schild traces: once the tile queue is drained and at most
 * `threshold` rays are still integrating, they continue in a tail kernel that splits each
 * RHS evaluation over 4 lanes (one wave per SIMD).  -1 = automatic (default: on, threshold
 * = the rays the tail kernel integrates at once, 64 per CU); 0 = off; > 0 = explicit
 * threshold.  Scheduling only: every pixel's result is identical in all modes. */
int grt_set_tail(long long threshold);
/* Rays the last Kerr-Schild trace on `device` handed to the tail kernel (synchronises the
 * device; 0 before the first trace).  A diagnostic of the scheduling above. */
int grt_tail_handoffs(grt_scene* scene, int device, uint64_t* handed_off);
/* The same plus the last trace's timeline in seconds since the integrate kernel started
 * (queue drained, first hand-off, tail kernel end; 0 when not reached), and for the first
 * min(handed_off, capacity) handed-off rays their output slot and the accepted steps
 * they had taken (any pointer nullable). */
int grt_tail_report(grt_scene* scene, int device, uint64_t* handed_off, double timeline_s[3], uint64_t* slot,
                    uint64_t* step, uint64_t capacity);

#ifdef __cplusplus
}
#endif
#endif /* GRT_API_H */
