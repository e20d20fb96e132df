// host_internal.h — internal declarations shared by the host-side C++ files.
#pragma once
#include <cstddef>
#include <cstdint>
#include <map>
#include <memory>
#include <algorithm>
#include <string>
#include <thread>
#include <vector>

#include "grt_api.h"

namespace grt_host {

void set_error(const std::string& msg);
// fn(i) for i in [0, n) on up to 16 host threads (interleaved); fn must only write its own i.
// Setup loops whose entries are independent (LUTs), so every entry is the same value as in
// a sequential loop.
template <class F>
void parallel_for(uint64_t n, F&& fn) {
  const unsigned hw = std::thread::hardware_concurrency();
  const unsigned nt = (unsigned)std::min<uint64_t>(n, std::max(1u, std::min(16u, hw)));
  if (nt <= 1) {
    for (uint64_t i = 0; i < n; ++i) fn(i);
    return;
  }
  std::vector<std::thread> pool;
  for (unsigned k = 0; k < nt; ++k)
    pool.emplace_back([&, k] {
      for (uint64_t i = k; i < n; i += nt) fn(i);
    });
  for (auto& t : pool) t.join();
}
// The camera frame of a device scene (grt_scene_desc.camera rows x cols; api.hip).
void scene_frame_size(const grt_scene* s, int64_t* rows, int64_t* cols);
// grt_supersample_shard_device with the shard's 1-spp step counts (d_local_steps, local
// order, nullable) for the sub-rays' longest-first work order (api.hip).
int supersample_shard(grt_scene* s, int device, void* stream, const grt_row_shard* sh, const grt_adaptive_config* cfg,
                      double min_lum, const double* d_min_lum, const double* d_frame_ya, const uint8_t* d_frame_class,
                      const double* sampling_mask_xyza, double* d_xyza64, const uint32_t* d_local_steps,
                      uint64_t* d_n_supersampled, uint64_t* d_stats, grt_subsample_failures* failures);
double rclamp_pub(double v, double lo, double hi);
int camera_build(int geometry, double radius, double a, const double position[4], const double velocity[4],
                 double alpha, int64_t rows, int64_t cols, double phi, double theta, double psi,
                 grt_camera_desc* out);
bool future_directed(int geometry, double radius, double a, const double position[4], const double v[4]);
double inner(int geometry, double radius, double a, const double position[4], const double v[4], const double w[4]);
double signature0(int geometry);
double r_isco(double r_s, double a);
// log (nullable): the reference's info! lines of KerrTemperatureComputer::new
// (temperature.rs:55-102), appended one per line
int kerr_temperature_lut(double temperature, double outer_radius, double a, double radius, uint32_t n,
                         double* lut_r, double* lut_t, double* r_isco_out, std::string* log = nullptr);
void blackbody_xyz(double temperature, double redshift, double out[3]);
int blackbody_lut(uint32_t n, double* log_t, double* xyz);
double inv_compand_srgb(double u);
void srgb_to_xyza(uint8_t r8, uint8_t g8, uint8_t b8, uint8_t a8, double out[4]);
int xyz_to_srgb8(const double* xyza, size_t n, int tone, double exposure, uint8_t* rgb);
void xyz_to_srgb(const double* xyz, double exposure, uint8_t* rgb);
void linear_max(const double* xyza, size_t n, double exposure, double* max3);
int tonemap(const double* xyza, size_t n, int tone, double exposure, const double* max3, uint8_t* rgb);
int stationary(int geometry, double radius, double a, const double position[4], double out[4]);
int zamo(int geometry, double radius, double a, const double position[4], double out[4]);
int ray_at(int geometry, double radius, double a, const double position[3], const double direction[3],
           double pos_out[4], double mom_out[4], std::string& err);
std::string rust_display_f64(double v);
int blackbody_spectrum(double t_min, double t_max, double z_min, double z_max, uint32_t w, uint32_t h, int tone,
                       uint8_t* rgba);

// ---- minimal TOML (the subset the reference's scene files use) ----
struct TomlValue;
using TomlTable = std::map<std::string, std::shared_ptr<TomlValue>>;
struct TomlValue {
  enum Kind { Float, Int, Bool, String, Array, Table, TableArray } kind = Table;
  double f = 0.0;
  int64_t i = 0;
  bool b = false;
  std::string s;
  std::vector<std::shared_ptr<TomlValue>> arr;
  TomlTable table;
  double number() const { return kind == Int ? (double)i : f; }
};
bool toml_parse(const std::string& text, TomlTable& root, std::string& err);

// ---- PNG (8-bit, non-interlaced) ----
bool png_decode_rgba(const std::string& path, std::vector<uint8_t>& rgba, uint32_t& w, uint32_t& h,
                     std::string& err);
bool png_encode_rgb(const std::string& path, const uint8_t* rgb, uint32_t w, uint32_t h, std::string& err);
bool png_encode_rgba(const std::string& path, const uint8_t* rgba, uint32_t w, uint32_t h, std::string& err);
bool hdr_encode_rgb(const std::string& path, const float* rgb, uint32_t w, uint32_t h, std::string& err);

}  // namespace grt_host
