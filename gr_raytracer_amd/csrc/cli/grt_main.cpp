// grt_main.cpp — `grt`, the command line of the MI355X build, flag-compatible with
// the reference's clap CLI (src/cli/cli.rs:5-113, src/main.rs:21-178) for `render`:
//
//   grt [--width N] [--height N] [--step-size H] [--max-steps N] [--max-radius R]
//       [--epsilon E] [--camera-position x,y,z] [--phi A] [--theta A] [--psi A]
//       [--tone-mapping reinhard|global-linear] [--show-sampling-mask]
//       [--sampling-mask-color r,g,b] --config-file scene.toml
//       render [--filename out.png|out.hdr] [--from-row N] [--from-col N]
//              [--to-row N] [--to-col N]
//     | render-ray -r ROW -c COL [--filename rendered-ray.csv]
//     | render-ray-at -p x,y,z -d x,y,z [--filename rendered-ray-at.csv]
//     | blackbody -t T [-r Z]
//     | blackbody-spectrum [--min-temperature T] [--max-temperature T] [--min-redshift Z]
//                          [--max-redshift Z] [--width N] [--height N] [-f FILE]
//
// Global options go before the subcommand, subcommand options after it (clap).
// Extra (not in the reference): --device N selects the GPU, --resource-root DIR
// resolves texture paths, --raw-out FILE dumps the f64 XYZA buffer; --gpus N (GPUs
// 0..N-1) or --devices A,B,... renders the whole frame over several GPUs of this process
// (grt_render_frame_multi: cyclic row bands of --band-rows rows, default 16, one RCCL
// gather), --gpus 1 included; --arithmetic exact|fused selects grt_set_arithmetic (exact,
// the reference's roundings, by default).
#include <algorithm>
#include <charconv>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cctype>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "grt_api.h"

namespace grt_host {
bool png_encode_rgb(const std::string& path, const uint8_t* rgb, uint32_t w, uint32_t h, std::string& err);
bool png_encode_rgba(const std::string& path, const uint8_t* rgba, uint32_t w, uint32_t h, std::string& err);
std::string rust_display_f64(double v);
bool hdr_encode_rgb(const std::string& path, const float* rgb, uint32_t w, uint32_t h, std::string& err);
}

static int usage(const char* msg) {
  std::fprintf(stderr,
               "error: %s\nusage: grt [global options] --config-file FILE render [--filename F]\n"
               "       grt [global options] --config-file FILE render-ray -r ROW -c COL [--filename F]\n"
               "       grt [global options] --config-file FILE render-ray-at -p X,Y,Z -d X,Y,Z [--filename F]\n"
               "       grt [global options] blackbody -t T [-r Z]\n"
               "       grt [global options] blackbody-spectrum [--min-temperature T] [--max-temperature T]\n"
               "           [--min-redshift Z] [--max-redshift Z] [--width N] [--height N] [-f FILE]\n",
               msg);
  return 2;
}

// Debug form of the RaytracerError behind a grt_status (raytracer.rs:20-52).
static const char* error_debug_name(int status) {
  switch (status) {
    case GRT_ERR_MAX_STEPS_REACHED: return "IntegrationError(MaxStepsReached)";
    case GRT_ERR_NO_CIRCULAR_ORBIT: return "NoCircularOrbitPossible";
    case GRT_ERR_BELOW_RISCO: return "BelowRISCO";
    case GRT_ERR_NON_FINITE_RADIUS: return "NonFiniteRadius";
    default: return "Unknown";
  }
}

// clap's value parsers for the flag types of cli.rs:5-113: the whole string must be a
// number of the field's type (f64 / i64 / u32 / usize); anything else is an error.
static bool parse_f64(const std::string& v, double* out) {
  if (v.empty() || std::isspace((unsigned char)v[0])) return false;
  char* end = nullptr;
  *out = std::strtod(v.c_str(), &end);
  return *end == 0;
}
static bool parse_i64(const std::string& v, long long lo, unsigned long long hi, long long* out) {
  if (v.empty() || std::isspace((unsigned char)v[0])) return false;
  const bool neg = v[0] == '-';
  const std::string d = (v[0] == '+' || neg) ? v.substr(1) : v;
  if (d.empty() || d.find_first_not_of("0123456789") != std::string::npos || d.size() > 19) return false;
  const unsigned long long m = std::strtoull(d.c_str(), nullptr, 10);
  if (neg ? (lo >= 0 ? m != 0 : m > (unsigned long long)(-(lo + 1)) + 1) : m > hi) return false;
  *out = neg ? -(long long)(m - 1) - 1 : (long long)m;
  return true;
}

// impl FromStr for Color (color.rs:151-170): three comma-separated components, each
// trimmed and parsed as u8 (optional '+', decimal digits, at most 255).
static bool parse_rgb(const std::string& s, uint8_t out[3]) {
  int n = 0;
  size_t p = 0;
  while (true) {
    size_t q = s.find(',', p);
    std::string tok = s.substr(p, q == std::string::npos ? std::string::npos : q - p);
    size_t b = tok.find_first_not_of(" \t\n\r\f\v"), e = tok.find_last_not_of(" \t\n\r\f\v");
    if (b == std::string::npos) return false;
    tok = tok.substr(b, e - b + 1);
    if (tok[0] == '+') tok = tok.substr(1);
    if (tok.empty() || tok.size() > 3 || tok.find_first_not_of("0123456789") != std::string::npos) return false;
    int v = std::atoi(tok.c_str());
    if (v > 255 || n >= 3) return false;
    out[n++] = (uint8_t)v;
    if (q == std::string::npos) break;
    p = q + 1;
  }
  return n == 3;
}

static bool split_csv(const std::string& s, std::vector<double>& out) {
  out.clear();
  size_t p = 0;
  while (p <= s.size()) {
    size_t q = s.find(',', p);
    if (q == std::string::npos) q = s.size();
    std::string tok = s.substr(p, q - p);
    char* end = nullptr;
    double v = std::strtod(tok.c_str(), &end);
    if (tok.empty() || *end) return false;
    out.push_back(v);
    p = q + 1;
  }
  return true;
}

// scene.rs:178-183, :196-202: color_of_ray's lines for an error-free ray that ended on NaN
// coordinates or without a terminal event.  The Ray's Debug form is cut to its pixel
// (row, col); steps.len() = accepted steps + the initial step.
static void log_ray_event(unsigned row, unsigned col, int stop, uint32_t accepted) {
  const unsigned long long len = (unsigned long long)accepted + 1;
  if (stop == GRT_STOP_NAN)
    std::fprintf(stderr, "[grt] ERROR Ray hit NaN coordinates: Ray { row: %u, col: %u, .. } with %llu steps.\n", row,
                 col, len);
  else if (stop == GRT_STOP_NONE)
    std::fprintf(stderr, "[grt] ERROR Ray did not hit anything: Ray { row: %u, col: %u, .. } at Some(Step { .. }) "
                 "with %llu steps.\n", row, col, len);
}

// Rust's Debug form of an f64 ({:?}): Display's shortest digits, with ".0" on integral
// values and exponential notation outside 1e-4 <= |v| < 1e16 (core::fmt::float).
static std::string rust_debug_f64(double v) {
  if (std::isnan(v) || std::isinf(v)) return grt_host::rust_display_f64(v);
  const double a = std::fabs(v);
  if (a != 0.0 && (a < 1e-4 || a >= 1e16)) {
    char buf[64];
    auto res = std::to_chars(buf, buf + sizeof(buf), v, std::chars_format::scientific);  // shortest digits
    std::string sci(buf, res.ptr);
    const size_t e = sci.find('e');
    return sci.substr(0, e) + "e" + std::to_string(std::atoi(sci.c_str() + e + 1));
  }
  std::string d = grt_host::rust_display_f64(v);
  if (d.find('.') == std::string::npos) d += ".0";
  return d;
}

// CoordinateSystem's Debug form for the geometry (geometry/*.rs coordinate_system, point.rs:11)
static std::string coordinate_system_debug(const grt_scene_desc* d) {
  switch (d->geometry) {
    case GRT_GEOM_SCHWARZSCHILD:
    case GRT_GEOM_EUCLIDEAN_SPHERICAL: return "Spherical";
    case GRT_GEOM_KERR_BL: return "BoyerLindquist { a: " + rust_debug_f64(d->a) + " }";
    default: return "Cartesian";  // Euclidean, Kerr (Kerr-Schild)
  }
}

// A Duration's Debug form with two decimals ({:.2?}, core::time: the largest unit of s /
// ms / us / ns with a non-zero integer part; the dropped digits round half up).
static std::string rust_duration_2(double secs) {
  const unsigned long long ns = (unsigned long long)std::llround(secs * 1e9);
  unsigned long long div;
  const char* unit;
  if (ns >= 1000000000ull) { div = 1000000000ull; unit = "s"; }
  else if (ns >= 1000000ull) { div = 1000000ull; unit = "ms"; }
  else if (ns >= 1000ull) { div = 1000ull; unit = "\u00b5s"; }
  else { div = 1ull; unit = "ns"; }
  if (div == 1) return std::to_string(ns) + ".00" + unit;
  const unsigned long long hundredths = (ns * 100 + div / 2) / div;
  char buf[64];
  std::snprintf(buf, sizeof(buf), "%llu.%02llu%s", hundredths / 100, hundredths % 100, unit);
  return buf;
}

static const char* stop_name(int s) {  // integrator.rs StopReason, as logged by the reference
  switch (s) {
    case GRT_STOP_HORIZON: return "Some(HorizonReached)";
    case GRT_STOP_CELESTIAL: return "Some(CelestialSphereReached)";
    case GRT_STOP_NAN: return "Some(CoordinateIsNan)";
    case GRT_STOP_CLOSED_ORBIT: return "Some(ClosedOrbitDetected)";
    default: return "None";
  }
}

// render-ray / render-ray-at: integrate one ray on the GPU and save its trajectory
// (main.rs:117-171).  The file is created before integrating, as the reference does.
static int trace_and_save(grt_scene* scene, int device, const grt_scene_desc* d, bool camera, const double* a,
                          const double* b, const std::string& filename) {
  FILE* f = std::fopen(filename.c_str(), "wb");
  if (!f) {
    std::fprintf(stderr, "Error: cannot create %s\n", filename.c_str());
    return 1;
  }
  std::fclose(f);
  const uint64_t cap = d->max_steps > 0 ? d->max_steps : 1;  // steps 0 .. max_steps-1
  std::vector<double> steps(cap * 9);
  uint64_t n = 0;
  uint8_t stop = 0, status = 0;
  int rc = camera ? grt_trace_pixels(scene, device, 1, a, b, cap, steps.data(), &n, &stop, &status)
                  : grt_trace_rays(scene, device, 1, a, b, cap, steps.data(), &n, &stop, &status);
  if (rc) {
    std::fprintf(stderr, "Error: %s\n", grt_last_error());
    return 1;
  }
  if (status != GRT_OK) {
    std::fprintf(stderr, "Error: %s\n", status == GRT_ERR_MAX_STEPS_REACHED ? "Max steps reached" : "integration failed");
    return 1;
  }
  std::fprintf(stderr, "[grt] INFO Stop reason: %s\n", stop_name(stop));
  if (grt_write_trajectory_csv(filename.c_str(), d->geometry, d->a, steps.data(), n < cap ? n : cap)) {
    std::fprintf(stderr, "Error: %s\n", grt_last_error());
    return 1;
  }
  std::fprintf(stderr, "[grt] INFO Saved integrated ray to %s\n", filename.c_str());
  return 0;
}

int main(int argc, char** argv) {
  auto t_start = std::chrono::steady_clock::now();
  grt_global_opts opts;
  grt_default_global_opts(&opts);
  std::string config_file, action, filename, resource_root, raw_out;
  long from_row = -1, from_col = -1, to_row = -1, to_col = -1;
  long long ray_row = 0, ray_col = 0;
  bool have_row = false, have_col = false;
  std::vector<double> ray_position, ray_direction;
  bool have_position = false, have_direction = false;
  // blackbody / blackbody-spectrum (cli.rs:88-110 defaults)
  double bb_temperature = 0.0, bb_redshift = 1.0, bb_tmin = 1000.0, bb_tmax = 10000.0, bb_zmin = 0.5, bb_zmax = 2.0;
  uint32_t bb_w = 1000, bb_h = 1000;
  bool have_temperature = false;
  int device = 0;
  std::vector<int> multi_devices;  // --gpus / --devices: the multi-GPU frame
  uint32_t band_rows = 16;
  std::vector<std::string> args(argv + 1, argv + argc);
  for (size_t i = 0; i < args.size(); ++i) {
    std::string a = args[i], val;
    bool has_eq = false;
    size_t eq = a.find('=');
    if (a.rfind("--", 0) == 0 && eq != std::string::npos) {
      val = a.substr(eq + 1);
      a = a.substr(0, eq);
      has_eq = true;
    }
    auto next = [&](std::string& v) -> bool {
      if (has_eq) {
        v = val;
        return true;
      }
      if (i + 1 >= args.size()) return false;
      v = args[++i];
      return true;
    };
    std::string v;
    if (action.empty() && (a == "render" || a == "render-ray" || a == "render-ray-at" || a == "blackbody" ||
                           a == "blackbody-spectrum")) {
      action = a;
      continue;
    }
    if (action.empty() && a == "--show-sampling-mask") { opts.show_sampling_mask = 1; continue; }
    if (!next(v)) return usage(("missing value for " + a).c_str());
    std::vector<double> nums;
    auto bad = [&]() { return usage(("invalid value '" + v + "' for '" + a + "'").c_str()); };
    auto f64 = [&](double* out) { return parse_f64(v, out); };
    auto int_in = [&](long long lo, unsigned long long hi, long long* out) { return parse_i64(v, lo, hi, out); };
    long long iv = 0;
    // extras accepted anywhere
    if (a == "--device") { device = std::atoi(v.c_str()); continue; }
    if (a == "--gpus") {
      if (!int_in(1, GRT_MULTI_MAX_DEVICES, &iv)) return bad();
      multi_devices.clear();
      for (long long k = 0; k < iv; ++k) multi_devices.push_back((int)k);
      continue;
    }
    if (a == "--devices") {
      std::vector<double> ds;
      if (!split_csv(v, ds) || ds.empty() || ds.size() > GRT_MULTI_MAX_DEVICES) return bad();
      multi_devices.clear();
      for (double x : ds) {
        if (x < 0 || x != (double)(int)x) return bad();
        multi_devices.push_back((int)x);
      }
      continue;
    }
    if (a == "--arithmetic") {
      if (v != "exact" && v != "fused") return bad();
      (void)grt_set_arithmetic(v == "fused" ? 1 : 0);
      continue;
    }
    if (a == "--band-rows") {
      if (!int_in(1, 4294967295ull, &iv)) return bad();
      band_rows = (uint32_t)iv;
      continue;
    }
    if (a == "--resource-root") { resource_root = v; continue; }
    if (a == "--raw-out") { raw_out = v; continue; }
    if (!action.empty()) {  // subcommand options
      if (a == "--filename") filename = v;
      else if (action == "render" && (a == "--from-row" || a == "--from-col" || a == "--to-row" || a == "--to-col")) {
        if (!int_in(0, 4294967295ull, &iv)) return bad();  // Option<u32>
        (a == "--from-row" ? from_row : a == "--from-col" ? from_col : a == "--to-row" ? to_row : to_col) = (long)iv;
      } else if (action == "render-ray" && (a == "-r" || a == "--row")) {
        if (!int_in(INT64_MIN, INT64_MAX, &iv)) return bad();  // i64
        ray_row = iv;
        have_row = true;
      } else if (action == "render-ray" && (a == "-c" || a == "--col")) {
        if (!int_in(INT64_MIN, INT64_MAX, &iv)) return bad();
        ray_col = iv;
        have_col = true;
      }
      else if (action == "render-ray-at" && (a == "-p" || a == "--position")) {
        if (!split_csv(v, ray_position)) return usage("invalid position");
        have_position = true;
      } else if (action == "render-ray-at" && (a == "-d" || a == "--direction")) {
        if (!split_csv(v, ray_direction)) return usage("invalid direction");
        have_direction = true;
      } else if (action == "blackbody" && (a == "-t" || a == "--temperature")) {
        if (!f64(&bb_temperature)) return bad();
        have_temperature = true;
      } else if (action == "blackbody" && (a == "-r" || a == "--redshift")) {
        if (!f64(&bb_redshift)) return bad();
      } else if (action == "blackbody-spectrum" && a == "--min-temperature") {
        if (!f64(&bb_tmin)) return bad();
      } else if (action == "blackbody-spectrum" && a == "--max-temperature") {
        if (!f64(&bb_tmax)) return bad();
      } else if (action == "blackbody-spectrum" && a == "--min-redshift") {
        if (!f64(&bb_zmin)) return bad();
      } else if (action == "blackbody-spectrum" && a == "--max-redshift") {
        if (!f64(&bb_zmax)) return bad();
      } else if (action == "blackbody-spectrum" && (a == "--width" || a == "--height")) {
        if (!int_in(0, 4294967295ull, &iv)) return bad();  // u32
        (a == "--width" ? bb_w : bb_h) = (uint32_t)iv;
      }
      else if (action == "blackbody-spectrum" && a == "-f") filename = v;
      else return usage(("unknown argument " + a + " for " + action).c_str());
      continue;
    }
    if (a == "--width" || a == "--height") {
      if (!int_in(INT64_MIN, INT64_MAX, &iv)) return bad();  // i64
      (a == "--width" ? opts.width : opts.height) = iv;
    } else if (a == "--max-steps") {  // usize
      const std::string d = (!v.empty() && v[0] == '+') ? v.substr(1) : v;
      if (d.empty() || d.find_first_not_of("0123456789") != std::string::npos) return bad();
      errno = 0;
      opts.max_steps = std::strtoull(d.c_str(), nullptr, 10);
      if (errno == ERANGE) return bad();
    } else if (a == "--step-size") { if (!f64(&opts.step_size)) return bad(); }
    else if (a == "--max-radius") { if (!f64(&opts.max_radius)) return bad(); }
    else if (a == "--epsilon") { if (!f64(&opts.epsilon)) return bad(); }
    else if (a == "--phi") { if (!f64(&opts.phi)) return bad(); }
    else if (a == "--theta") { if (!f64(&opts.theta)) return bad(); }
    else if (a == "--psi") { if (!f64(&opts.psi)) return bad(); }
    else if (a == "--camera-position") {
      if (!split_csv(v, nums) || nums.size() != 3) return usage("Camera position must be a vector of length 3");
      for (int k = 0; k < 3; ++k) opts.camera_position[k] = nums[k];
    } else if (a == "--tone-mapping") {
      if (v == "reinhard") opts.tone_mapping = GRT_TONE_REINHARD;
      else if (v == "global-linear") opts.tone_mapping = GRT_TONE_GLOBAL_LINEAR;
      else return usage("tone mapping must be reinhard or global-linear");
    } else if (a == "--sampling-mask-color") {
      uint8_t rgb[3];
      if (!parse_rgb(v, rgb)) return usage(("invalid RGB color '" + v + "'; expected R,G,B").c_str());
      for (int k = 0; k < 3; ++k) opts.sampling_mask_color[k] = rgb[k];
    } else if (a == "-c" || a == "--config-file") config_file = v;
    else return usage(("unknown argument " + a).c_str());
  }
  if (action.empty()) return usage("missing subcommand (render, render-ray, render-ray-at, blackbody, blackbody-spectrum)");
  if (action == "blackbody") {  // run_blackbody (cli/blackbody.rs:7-25): no scene needed
    if (!have_temperature) return usage("blackbody needs --temperature");
    double xyz[3];
    uint8_t c[3];
    grt_blackbody_xyz(bb_temperature, bb_redshift, xyz);
    grt_xyz_to_srgb(xyz, 1.0, c);
    std::printf("Blackbody color at T=%sK (redshift=%s):\n", grt_host::rust_display_f64(bb_temperature).c_str(),
                grt_host::rust_display_f64(bb_redshift).c_str());
    std::printf("XYZ:  %.4f, %.4f, %.4f\n", xyz[0], xyz[1], xyz[2]);
    std::printf("sRGB: R=%u, G=%u, B=%u\n", c[0], c[1], c[2]);
    std::printf("sRGB: R=%.4f, G=%.4f, B=%.4f\n", c[0] / 255.0, c[1] / 255.0, c[2] / 255.0);
    std::printf("Color block: \x1b[48;2;%u;%u;%um      \x1b[0m\n", c[0], c[1], c[2]);
    return 0;
  }
  if (action == "blackbody-spectrum") {  // run_blackbody_spectrum (cli/blackbody.rs:27-95)
    if (filename.empty()) filename = "blackbody_spectrum.png";
    std::vector<uint8_t> rgba((size_t)bb_w * bb_h * 4);
    if (grt_blackbody_spectrum(bb_tmin, bb_tmax, bb_zmin, bb_zmax, bb_w, bb_h, opts.tone_mapping, rgba.data())) {
      std::fprintf(stderr, "Error: %s\n", grt_last_error());
      return 1;
    }
    std::string err;
    if (!grt_host::png_encode_rgba(filename, rgba.data(), bb_w, bb_h, err)) {
      std::fprintf(stderr, "Failed to save spectrum image: %s\n", err.c_str());
      return 1;
    }
    std::printf("Saved blackbody spectrum to %s\n", filename.c_str());
    return 0;
  }
  if (action == "render-ray" && !(have_row && have_col)) return usage("render-ray needs --row and --col");
  if (action == "render-ray-at" && !(have_position && have_direction))
    return usage("render-ray-at needs --position and --direction");
  if (filename.empty())
    filename = action == "render" ? "render.png" : (action == "render-ray" ? "rendered-ray.csv" : "rendered-ray-at.csv");
  if (config_file.empty()) return usage("Config file is required for this action");

  if (action == "render" && !multi_devices.empty() &&
      (from_row > 0 || from_col > 0 || (to_row >= 0 && to_row != (long long)opts.height) ||
       (to_col >= 0 && to_col != (long long)opts.width)))
    return usage("--gpus / --devices render whole frames (no --from-row/--from-col/--to-row/--to-col)");

  // The HIP runtime's start-up (driver and device enumeration) runs beside the scene load
  // below: the first HIP call of the process does it, wherever it is made.
  std::thread hip_init([] { (void)grt_device_count(); });
  // on every way out of main from here: the start-up thread joined, then the multi-GPU
  // frame's RCCL set-up waited for and torn down (a communicator still being created when
  // the process exits brings the exit down)
  struct Joiner {
    std::thread& t;
    bool multi;
    ~Joiner() {
      if (t.joinable()) t.join();
      if (multi) grt_multi_release();
    }
  } hip_init_join{hip_init, !multi_devices.empty()};
  // phase times of a render (printed on one [grt] line at the end; not in the reference)
  using clk = std::chrono::steady_clock;
  auto ms_since = [](clk::time_point t) { return std::chrono::duration<double, std::milli>(clk::now() - t).count(); };
  double ph_load = 0, ph_create = 0, ph_init = 0, ph_render = 0, ph_output = 0, ph_write = 0;
  auto t_phase = clk::now();
  grt_host_scene* hs = nullptr;
  if (action == "render-ray-at" ? grt_host_geometry_load(config_file.c_str(), &opts, &hs)
                                : grt_host_scene_load(config_file.c_str(),
                                                      resource_root.empty() ? nullptr : resource_root.c_str(), &opts,
                                                      &hs)) {
    std::fprintf(stderr, "Error: %s\n", grt_last_error());
    return 1;
  }
  grt_adaptive_config ac;
  grt_host_scene_adaptive(hs, &ac);
  ph_load = ms_since(t_phase);
  t_phase = clk::now();
  grt_scene* scene = nullptr;
  if (grt_scene_create(grt_host_scene_desc(hs), &scene)) {
    std::fprintf(stderr, "Error: %s\n", grt_last_error());
    return 1;
  }
  ph_create = ms_since(t_phase);
  t_phase = clk::now();
  hip_init.join();  // what is left of the HIP runtime's start-up after the load
  ph_init = ms_since(t_phase);
  const grt_scene_desc* d = grt_host_scene_desc(hs);
  auto elapsed = [&]() {  // main.rs:175-176
    const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t_start).count();
    std::fprintf(stderr, "[grt] INFO Elapsed time: %s\n", rust_duration_2(secs).c_str());
  };
  if (action == "render")  // main.rs:100-103
    std::fprintf(stderr, "[grt] INFO Using coordinate system: %s\n", coordinate_system_debug(d).c_str());
  {  // the scene setup's info lines (KerrTemperatureComputer::new, temperature.rs:55-102)
    const std::string log = grt_host_scene_log(hs);
    for (size_t p = 0; p < log.size();) {
      size_t q = log.find('\n', p);
      if (q == std::string::npos) q = log.size();
      std::fprintf(stderr, "[grt] INFO %s\n", log.substr(p, q - p).c_str());
      p = q + 1;
    }
  }
  if (action != "render") {
    int rc;
    if (action == "render-ray") {  // Raytracer::integrate_ray_at_point (raytracer.rs:499-507)
      const double row = (double)ray_row, col = (double)ray_col;
      rc = trace_and_save(scene, device, d, true, &row, &col, filename);
    } else {
      if (ray_position.size() != 3) {
        std::fprintf(stderr, "Error: Position must be a vector of length 3, got %zu values\n", ray_position.size());
        return 1;
      }
      if (ray_direction.size() != 3) {
        std::fprintf(stderr, "Error: Direction must be a vector of length 3, got %zu values\n", ray_direction.size());
        return 1;
      }
      double pos[4], mom[4];
      if (grt_ray_at(d->geometry, d->radius, d->a, ray_position.data(), ray_direction.data(), pos, mom)) {
        std::fprintf(stderr, "Error: %s\n", grt_last_error());
        return 1;
      }
      rc = trace_and_save(scene, device, d, false, pos, mom, filename);
    }
    grt_scene_destroy(scene);
    grt_host_scene_destroy(hs);
    if (rc == 0) elapsed();
    return rc;
  }
  uint32_t r0 = from_row < 0 ? 0 : (uint32_t)from_row, c0 = from_col < 0 ? 0 : (uint32_t)from_col;
  uint32_t r1 = to_row < 0 ? (uint32_t)opts.height : (uint32_t)to_row;
  uint32_t c1 = to_col < 0 ? (uint32_t)opts.width : (uint32_t)to_col;
  uint32_t w = c1 - c0, h = r1 - r0;
  std::vector<double> xyza((size_t)w * h * 4);
  double mask[4];
  const double* maskp = nullptr;
  if (opts.show_sampling_mask) {
    grt_srgb_to_xyza(opts.sampling_mask_color[0], opts.sampling_mask_color[1], opts.sampling_mask_color[2], 255, mask);
    maskp = mask;
  }
  grt_stats st;
  uint64_t nsel = 0;
  std::vector<uint8_t> status((size_t)w * h);
  // failed supersample sub-rays (raytracer.rs:357-362), up to 1M logged
  const uint64_t fail_cap = 1u << 20;
  std::vector<uint32_t> fail_pix(fail_cap), fail_sample(fail_cap);
  std::vector<uint8_t> fail_status(fail_cap), fail_stop(fail_cap);
  std::vector<uint32_t> fail_steps(fail_cap);
  grt_subsample_failures fails{fail_cap, fail_pix.data(), fail_sample.data(), fail_status.data(), 0,
                               fail_stop.data(), fail_steps.data()};
  std::vector<uint8_t> stop((size_t)w * h);
  std::vector<uint32_t> steps((size_t)w * h);
  const bool supersampled = ac.enabled || maskp;
  const bool hdr = filename.size() >= 4 && filename.compare(filename.size() - 4, 4, ".hdr") == 0;
  if (hdr) {  // raytracer.rs:468-469, :481-483
    std::fprintf(stderr, "[grt] INFO Creating HDR image\n");
  } else {
    std::fprintf(stderr, "[grt] INFO Creating non-HDR image\n");
    std::fprintf(stderr, "[grt] INFO Tone mapping method: %s\n",
                 opts.tone_mapping == GRT_TONE_GLOBAL_LINEAR ? "GlobalLinear" : "Reinhard");
  }
  const bool multi = !multi_devices.empty();
  if (supersampled)  // raytracer.rs:264-267
    std::fprintf(stderr, "[grt] INFO Rendering section from (%u, %u) to (%u, %u) with supersampling\n", r0, c0, r1,
                 c1);
  t_phase = clk::now();
  grt_multi_report mrep;
  if (multi) {
    // the frame over several GPUs: cyclic row bands, one host thread per device, one RCCL
    // gather of f64 XYZA + class + status + stop + steps (39 B per pixel) to the first
    grt_frame_out fo{nullptr, xyza.data(), nullptr, status.data(), stop.data(), steps.data()};
    if (grt_render_frame_multi(scene, (int)multi_devices.size(), multi_devices.data(), band_rows, &ac, maskp, &fo,
                               &nsel, &st, &fails, &mrep)) {
      std::fprintf(stderr, "Error: %s\n", grt_last_error());
      return 1;
    }
  } else if (grt_render_section_ex(scene, device, r0, c0, r1, c1, &ac, maskp, xyza.data(), nullptr, &nsel, &st,
                                   status.data(), &fails, stop.data(), steps.data())) {
    std::fprintf(stderr, "Error: %s\n", grt_last_error());
    return 1;
  }
  ph_render = ms_since(t_phase);
  // The 1-spp pass, in pixel order (the reference logs from its parallel loop):
  //  * raytracer.rs:232-239: a pixel whose color_of_ray failed (Debug form of the
  //    RaytracerError); it keeps the default colour;
  //  * scene.rs:178-183 / :196-202: an error-free ray that ended on NaN coordinates or
  //    without a terminal event (steps.len() counts the initial step too).
  for (size_t i = 0; i < status.size(); ++i) {
    const unsigned col = (unsigned)(c0 + i % w), row = (unsigned)(r0 + i / w);
    if (status[i] & 0x7f)
      std::fprintf(stderr, "[grt] ERROR Unable to compute color for ray at pixel (%u, %u): %s\n", col, row,
                   error_debug_name(status[i] & 0x7f));
    else
      log_ray_event(row, col, stop[i], steps[i]);
  }
  if (supersampled && !maskp) {  // supersample (raytracer.rs:325), then its sub-rays' lines
    std::fprintf(stderr, "[grt] INFO Supersampling %llu pixels\n", (unsigned long long)nsel);
    // :357-362: the same error line for each failed sub-sample ray of a supersampled pixel
    for (uint64_t k = 0; k < std::min<uint64_t>(fails.count, fail_cap); ++k) {
      const unsigned col = (unsigned)(c0 + fail_pix[k] % w), row = (unsigned)(r0 + fail_pix[k] / w);
      if (fail_status[k])
        std::fprintf(stderr, "[grt] ERROR Unable to compute color for ray at pixel (%u, %u): %s\n", col, row,
                     error_debug_name(fail_status[k]));
      else
        log_ray_event(row, col, fail_stop[k], fail_steps[k]);
    }
    if (fails.count > fail_cap)
      std::fprintf(stderr, "[grt] ERROR %llu more failed or unterminated sub-sample rays not listed\n",
                   (unsigned long long)(fails.count - fail_cap));
  }
  if (supersampled)  // raytracer.rs:313-316
    std::fprintf(stderr, "[grt] INFO Finished rendering section from (%u, %u) to (%u, %u)\n", r0, c0, r1, c1);
  std::fprintf(stderr, "[grt] %llu rays, %llu accepted steps, %llu attempts, %llu supersampled pixels, kernel %.1f ms "
               "(%.3e steps/s)\n",
               (unsigned long long)st.rays, (unsigned long long)st.accepted_steps, (unsigned long long)st.attempts,
               (unsigned long long)nsel, st.kernel_ms, st.accepted_steps / (st.kernel_ms * 1e-3));
  if (multi) {
    std::string per;
    for (uint32_t k = 0; k < mrep.n_devices; ++k) {
      char b[96];
      std::snprintf(b, sizeof(b), "%s%d: %llu rows %.1f ms", k ? ", " : "", multi_devices[k],
                    (unsigned long long)mrep.rows[k], mrep.trace_ms[k]);
      per += b;
    }
    std::fprintf(stderr, "[grt] %u GPU(s) [%s]; allgather %.2f ms, gather %.2f ms (%u B per pixel), %u trace(s)\n",
                 mrep.n_devices, per.c_str(), mrep.allgather_ms, mrep.gather_ms, mrep.record_bytes, mrep.attempts);
  }
  if (st.march_jobs)
    std::fprintf(stderr, "[grt] VolumetricDisc: %llu raymarches, %llu samples (%llu with noise, %llu emitting)\n",
                 (unsigned long long)st.march_jobs, (unsigned long long)st.march_samples,
                 (unsigned long long)st.march_noise_samples, (unsigned long long)st.march_emit_samples);
  std::string err;
  bool ok;
  t_phase = clk::now();
  if (hdr) {
    std::vector<float> rgb((size_t)w * h * 3);
    for (size_t i = 0; i < (size_t)w * h; ++i)
      for (int k = 0; k < 3; ++k) rgb[3 * i + k] = (float)xyza[4 * i + k];
    ok = grt_host::hdr_encode_rgb(filename, rgb.data(), w, h, err);
  } else {
    std::vector<uint8_t> rgb((size_t)w * h * 3);
    // output stage on the GPU (color.rs:204-298 via output.hip), exposure 1 as in
    // render_section (raytracer.rs:485)
    if (grt_xyz_to_srgb8_device(multi ? multi_devices[0] : device, xyza.data(), (size_t)w * h, opts.tone_mapping,
                                1.0, rgb.data())) {
      std::fprintf(stderr, "Error: %s\n", grt_last_error());
      return 1;
    }
    ph_output = ms_since(t_phase);
    t_phase = clk::now();
    ok = grt_host::png_encode_rgb(filename, rgb.data(), w, h, err);
  }
  if (!ok) {
    std::fprintf(stderr, "Error: %s\n", err.c_str());
    return 1;
  }
  if (!raw_out.empty()) {
    FILE* f = std::fopen(raw_out.c_str(), "wb");
    if (f) {
      std::fwrite(xyza.data(), 8, xyza.size(), f);
      std::fclose(f);
    }
  }
  ph_write = ms_since(t_phase);
  std::fprintf(stderr, "[grt] INFO saved image to %s\n", filename.c_str());  // raytracer.rs:494
  // where the wall time went: TOML + texture decode + LUTs; the descriptor copy; the render
  // call (device upload on first use, trace, supersampling, D2H); tone map; encode + write
  std::fprintf(stderr, "[grt] phases (ms): load %.1f, create %.1f, hip init %.1f, render %.1f, output %.1f, "
               "write %.1f, since start %.1f\n", ph_load, ph_create, ph_init, ph_render, ph_output, ph_write,
               ms_since(t_start));
  elapsed();
  // teardown after the reference's measured span (main.rs:175-176 logs before its drops;
  // the multi-GPU set-up is released by hip_init_join)
  grt_scene_destroy(scene);
  grt_host_scene_destroy(hs);
  return 0;
}
