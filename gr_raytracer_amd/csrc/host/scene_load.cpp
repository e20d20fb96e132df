// scene_load.cpp — TOML scene + GlobalOpts -> grt_scene_desc, i.e. the reference's
//   main.rs:74-116                      (read TOML, camera position, pick geometry)
//   configuration.rs:1-230              (RenderConfig schema and validation)
//   cli/{euclidean,schwarzschild,kerr,kerr_bl}.rs::create_scene_internal
//                                       (camera chart conversion, camera velocity)
//   cli/shared.rs:48-321                (resolve_camera_velocity, assert_future_directed,
//                                        create_scene: textures, Camera::new, objects)
// The result is an owned grt_host_scene whose descriptor the device API consumes.
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <future>
#include <memory>
#include <map>
#include <sstream>
#include <string>
#include <vector>

#include "host_internal.h"

struct CachedTexture {
  uint32_t w = 0, h = 0;
  double beaming = 0.0;
  std::vector<uint8_t> rgba;
  // the PNG decode, started when the texture is first named and waited for at the end of
  // grt_host_scene_load (the textures decode beside each other and beside the LUTs);
  // the decode's error text, "" when it succeeded
  std::shared_future<std::string> decoded;
};
// A texture descriptor waiting for its bitmap's size and texels.
struct TexturePatch {
  grt_texture_desc* d;
  CachedTexture* ct;
};
struct grt_host_scene {
  grt_scene_desc desc;
  grt_adaptive_config adaptive;
  std::map<std::string, std::unique_ptr<CachedTexture>> textures;  // TextureMapperFactory cache (by path)
  std::vector<double> lut_r[GRT_MAX_OBJECTS], lut_t[GRT_MAX_OBJECTS];
  std::vector<double> bb_log_t, bb_xyz;
  std::string error;
  std::string info_log;  // the reference's info! lines of the scene setup, one per line
};

namespace grt_host {
namespace {

int fail(const std::string& m) {
  set_error(m);
  return -EINVAL;
}

const TomlValue* get(const TomlTable& t, const std::string& k) {
  auto it = t.find(k);
  return it == t.end() ? nullptr : it->second.get();
}
bool num(const TomlTable& t, const std::string& k, double* out, std::string& err) {
  const TomlValue* v = get(t, k);
  if (!v || (v->kind != TomlValue::Float && v->kind != TomlValue::Int)) {
    err = "missing or non-numeric field `" + k + "`";
    return false;
  }
  *out = v->number();
  return true;
}
bool uint_field(const TomlTable& t, const std::string& k, uint64_t* out, std::string& err) {  // serde usize / u32
  const TomlValue* v = get(t, k);
  if (!v || v->kind != TomlValue::Int || v->i < 0) {
    err = "missing or non-integer field `" + k + "`";
    return false;
  }
  *out = (uint64_t)v->i;
  return true;
}
bool triple(const TomlTable& t, const std::string& k, double out[3], std::string& err) {
  const TomlValue* v = get(t, k);
  if (!v || v->kind != TomlValue::Array || v->arr.size() != 3) {
    err = "field `" + k + "` must be an array of 3 numbers";
    return false;
  }
  for (int i = 0; i < 3; ++i) {
    const TomlValue* e = v->arr[i].get();
    if (e->kind != TomlValue::Float && e->kind != TomlValue::Int) {
      err = "field `" + k + "` must be numeric";
      return false;
    }
    out[i] = e->number();
  }
  return true;
}
// serde externally-tagged enum in TOML: either "Variant" or { Variant = {...} }
bool variant(const TomlValue* v, std::string& name, const TomlTable** body) {
  static const TomlTable empty;
  if (!v) return false;
  if (v->kind == TomlValue::String) {
    name = v->s;
    *body = &empty;
    return true;
  }
  if (v->kind == TomlValue::Table && v->table.size() == 1) {
    name = v->table.begin()->first;
    const TomlValue* b = v->table.begin()->second.get();
    if (b->kind != TomlValue::Table) return false;
    *body = &b->table;
    return true;
  }
  return false;
}

struct TexSpec {
  int kind;
  double beaming;
  std::string path;
  double cw, ch;
  uint8_t c1[3], c2[3];
};
bool parse_texture(const TomlValue* v, TexSpec& t, std::string& err) {  // configuration.rs:162-177
  std::string name;
  const TomlTable* b;
  if (!variant(v, name, &b)) {
    err = "texture must be one of Bitmap / Checker / BlackBody";
    return false;
  }
  if (!num(*b, "beaming_exponent", &t.beaming, err)) return false;
  if (name == "Bitmap") {
    const TomlValue* p = get(*b, "path");
    if (!p || p->kind != TomlValue::String) {
      err = "Bitmap texture needs `path`";
      return false;
    }
    t.kind = GRT_TEX_BITMAP;
    t.path = p->s;
    return true;
  }
  if (name == "Checker") {
    t.kind = GRT_TEX_CHECKER;
    double c1[3], c2[3];
    if (!num(*b, "width", &t.cw, err) || !num(*b, "height", &t.ch, err) || !triple(*b, "color1", c1, err) ||
        !triple(*b, "color2", c2, err))
      return false;
    for (int i = 0; i < 3; ++i) {
      if (c1[i] < 0 || c1[i] > 255 || c2[i] < 0 || c2[i] > 255) {
        err = "checker colours must be 0..255";
        return false;
      }
      t.c1[i] = (uint8_t)c1[i];
      t.c2[i] = (uint8_t)c2[i];
    }
    return true;
  }
  if (name == "BlackBody") {
    t.kind = GRT_TEX_BLACKBODY;
    return true;
  }
  err = "unknown texture variant `" + name + "`";
  return false;
}

std::string join_path(const char* root, const std::string& p) {
  if (!root || !*root || (!p.empty() && p[0] == '/')) return p;
  std::string r(root);
  if (r.back() != '/') r += '/';
  return r + p;
}

}  // namespace
}  // namespace grt_host

using namespace grt_host;

static int fill_texture(grt_host_scene* hs, const TexSpec& t, const char* root, grt_texture_desc& d, bool* need_bb,
                        std::vector<TexturePatch>* patches) {
  std::memset(&d, 0, sizeof(d));
  d.kind = t.kind;
  d.beaming_exponent = t.beaming;
  if (t.kind == GRT_TEX_BITMAP) {
    // TextureMapperFactory caches by file name only (texture.rs:278-295): the first
    // beaming exponent seen for a path wins.
    auto it = hs->textures.find(t.path);
    if (it == hs->textures.end()) {
      std::unique_ptr<CachedTexture> ct(new CachedTexture());
      CachedTexture* c = ct.get();
      const std::string path = join_path(root, t.path);
      c->decoded = std::async(std::launch::async, [c, path]() {
                     std::string err;
                     return png_decode_rgba(path, c->rgba, c->w, c->h, err) ? std::string() : err;
                   }).share();
      ct->beaming = t.beaming;
      it = hs->textures.emplace(t.path, std::move(ct)).first;
    }
    // size and texels once the decode is done (grt_host_scene_load's end)
    patches->push_back(TexturePatch{&d, it->second.get()});
    d.beaming_exponent = it->second->beaming;
  } else if (t.kind == GRT_TEX_CHECKER) {
    d.checker_width = t.cw;
    d.checker_height = t.ch;
    double c[4];
    grt_srgb_to_xyza(t.c1[0], t.c1[1], t.c1[2], 255, c);
    c[3] = 1.0;  // CheckerMapper uses srgb_to_xyz (alpha 1.0)
    std::memcpy(d.c1, c, sizeof(c));
    grt_srgb_to_xyza(t.c2[0], t.c2[1], t.c2[2], 255, c);
    c[3] = 1.0;
    std::memcpy(d.c2, c, sizeof(c));
  } else {
    *need_bb = true;
  }
  return 0;
}

extern "C" {

void grt_default_global_opts(grt_global_opts* o) {  // cli.rs:5-47 defaults
  std::memset(o, 0, sizeof(*o));
  o->width = 500;
  o->height = 500;
  o->step_size = 0.01;
  o->max_steps = 20000;
  o->max_radius = 15000.0;
  o->epsilon = 0.00001;
  o->camera_position[0] = 18.0;
  o->camera_position[1] = 0.0;
  o->camera_position[2] = 0.8;
  o->tone_mapping = 0;
  o->show_sampling_mask = 0;
  o->sampling_mask_color[0] = 255;
  o->sampling_mask_color[1] = 0;
  o->sampling_mask_color[2] = 255;
}

void grt_default_adaptive_config(grt_adaptive_config* c) {  // configuration.rs:46-57
  std::memset(c, 0, sizeof(*c));
  c->enabled = 1;
  c->samples_per_axis = 4;
  c->luminance_contrast_threshold = 0.15;
  c->opacity_contrast_threshold = 0.1;
  c->has_minimum_luminance = 0;
  c->minimum_luminance = 0.0;
  c->object_hit_opacity_threshold = 0.5;
  c->exclude_background_contrast = 1;
}

// Read the TOML file, then geometry_type (configuration.rs:111-158) and the integration
// configuration from GlobalOpts into a fresh descriptor.
static int load_geometry(const char* toml_path, const grt_global_opts* opts, TomlTable& root, grt_scene_desc& d) {
  std::ifstream f(toml_path);
  if (!f) return fail(std::string("Config file not found: ") + toml_path);
  std::stringstream ss;
  ss << f.rdbuf();
  std::string err;
  if (!toml_parse(ss.str(), root, err)) return fail("TOML error: " + err);
  std::memset(&d, 0, sizeof(d));
  d.abi_version = GRT_ABI_VERSION;
  std::string gname;
  const TomlTable* gb;
  if (!variant(get(root, "geometry_type"), gname, &gb)) return fail("missing or invalid `geometry_type`");
  if (gname == "Euclidean") {
    d.geometry = GRT_GEOM_EUCLIDEAN;
  } else if (gname == "EuclideanSpherical") {
    d.geometry = GRT_GEOM_EUCLIDEAN_SPHERICAL;
  } else if (gname == "Schwarzschild") {
    d.geometry = GRT_GEOM_SCHWARZSCHILD;
    if (!num(*gb, "radius", &d.radius, err) || !num(*gb, "horizon_epsilon", &d.horizon_epsilon, err)) return fail(err);
  } else if (gname == "Kerr" || gname == "KerrBL") {
    d.geometry = gname == "Kerr" ? GRT_GEOM_KERR : GRT_GEOM_KERR_BL;
    if (!num(*gb, "radius", &d.radius, err) || !num(*gb, "a", &d.a, err) ||
        !num(*gb, "horizon_epsilon", &d.horizon_epsilon, err))
      return fail(err);
  } else {
    return fail("unknown geometry `" + gname + "`");
  }
  d.max_steps = opts->max_steps;
  d.max_radius = opts->max_radius;
  d.step_size = opts->step_size;
  d.epsilon = opts->epsilon;
  for (int i = 0; i < 256; ++i) d.srgb_to_linear[i] = inv_compand_srgb((double)i / 255.0);
  d.object_hit_opacity_threshold = 0.5;
  return 0;
}

int grt_host_geometry_load(const char* toml_path, const grt_global_opts* opts, grt_host_scene** out) {
  if (!toml_path || !opts || !out) return fail("null argument");
  std::unique_ptr<grt_host_scene> hs(new grt_host_scene());
  TomlTable root;
  int rc = load_geometry(toml_path, opts, root, hs->desc);
  if (rc) return rc;
  grt_default_adaptive_config(&hs->adaptive);
  grt_scene_desc& d = hs->desc;
  // no camera, no objects: a 1x1 placeholder frame and a constant black sky
  d.camera.rows = d.camera.cols = 1;
  d.celestial.kind = GRT_TEX_CHECKER;
  d.celestial.checker_width = d.celestial.checker_height = 1.0;
  d.celestial.c1[3] = d.celestial.c2[3] = 1.0;
  *out = hs.release();
  return 0;
}

int grt_host_scene_load(const char* toml_path, const char* resource_root, const grt_global_opts* opts,
                        grt_host_scene** out) {
  if (!toml_path || !opts || !out) return fail("null argument");
  std::unique_ptr<grt_host_scene> hs(new grt_host_scene());
  grt_scene_desc& d = hs->desc;
  TomlTable root;
  std::string err;
  int rc0 = load_geometry(toml_path, opts, root, d);
  if (rc0) return rc0;

  // adaptive_sampling (configuration.rs:21-94), serde(default) per field
  grt_adaptive_config& ac = hs->adaptive;
  grt_default_adaptive_config(&ac);
  if (const TomlValue* a = get(root, "adaptive_sampling")) {
    if (a->kind != TomlValue::Table) return fail("`adaptive_sampling` must be a table");
    const TomlTable& t = a->table;
    if (const TomlValue* v = get(t, "enabled")) ac.enabled = v->b;
    if (const TomlValue* v = get(t, "samples_per_axis")) {
      if (v->kind != TomlValue::Int || v->i < 0) return fail("adaptive_sampling.samples_per_axis must be an integer");
      ac.samples_per_axis = (uint32_t)v->i;
    }
    if (get(t, "luminance_contrast_threshold") && !num(t, "luminance_contrast_threshold", &ac.luminance_contrast_threshold, err)) return fail(err);
    if (get(t, "opacity_contrast_threshold") && !num(t, "opacity_contrast_threshold", &ac.opacity_contrast_threshold, err)) return fail(err);
    if (get(t, "object_hit_opacity_threshold") && !num(t, "object_hit_opacity_threshold", &ac.object_hit_opacity_threshold, err)) return fail(err);
    if (get(t, "minimum_luminance")) {
      if (!num(t, "minimum_luminance", &ac.minimum_luminance, err)) return fail(err);
      ac.has_minimum_luminance = 1;
    }
    if (const TomlValue* v = get(t, "exclude_background_contrast")) ac.exclude_background_contrast = v->b;
  }
  // AdaptiveSamplingConfig::validate (configuration.rs:60-93)
  if (ac.samples_per_axis == 0) return fail("adaptive_sampling.samples_per_axis must be greater than zero");
  const double ths[3] = {ac.luminance_contrast_threshold, ac.opacity_contrast_threshold, ac.object_hit_opacity_threshold};
  const char* thn[3] = {"luminance_contrast_threshold", "opacity_contrast_threshold", "object_hit_opacity_threshold"};
  for (int i = 0; i < 3; ++i)
    if (!std::isfinite(ths[i]) || !(ths[i] >= 0.0 && ths[i] <= 1.0))
      return fail(std::string("adaptive_sampling.") + thn[i] + " must be finite and between 0 and 1");
  if (ac.has_minimum_luminance && (!std::isfinite(ac.minimum_luminance) || ac.minimum_luminance < 0.0))
    return fail("adaptive_sampling.minimum_luminance must be finite and non-negative");
  d.object_hit_opacity_threshold = ac.object_hit_opacity_threshold;

  // camera position in the geometry's native chart (cli/<geometry>.rs)
  double cart[4] = {0.0, opts->camera_position[0], opts->camera_position[1], opts->camera_position[2]};
  double pos[4];
  if (d.geometry == GRT_GEOM_SCHWARZSCHILD || d.geometry == GRT_GEOM_EUCLIDEAN_SPHERICAL)
    grt_cartesian_to_spherical(cart, pos);
  else if (d.geometry == GRT_GEOM_KERR_BL) grt_cartesian_to_boyer_lindquist(d.a, cart, pos);
  else std::memcpy(pos, cart, sizeof(pos));

  // resolve_camera_velocity (cli/shared.rs:48-77)
  double vel[4];
  std::string vname = "StaticObserver";
  const TomlTable* vb = nullptr;
  if (const TomlValue* cv = get(root, "camera_velocity")) {
    if (!variant(cv, vname, &vb)) return fail("invalid `camera_velocity`");
  }
  if (vname == "StaticObserver") {
    grt_stationary_velocity(d.geometry, d.radius, d.a, pos, vel);
  } else if (vname == "Zamo") {
    grt_zamo_velocity(d.geometry, d.radius, d.a, pos, vel);
  } else if (vname == "Explicit") {
    const TomlValue* c = vb ? get(*vb, "components") : nullptr;
    if (!c || c->kind != TomlValue::Array || c->arr.size() != 4) return fail("Explicit camera_velocity needs 4 components");
    for (int i = 0; i < 4; ++i) vel[i] = c->arr[i]->number();
    double norm = inner(d.geometry, d.radius, d.a, pos, vel, vel);
    if (std::fabs(norm - signature0(d.geometry)) > 1e-6) return fail("Explicit camera_velocity is not normalized");
  } else {
    return fail("unknown camera_velocity `" + vname + "`");
  }
  if (!future_directed(d.geometry, d.radius, d.a, pos, vel)) return fail("camera four-velocity has wrong time orientation");

  // celestial texture + Camera::new (alpha = pi/4, rows = height, cols = width)
  bool need_bb = false;
  TexSpec ct;
  if (!parse_texture(get(root, "celestial_texture"), ct, err)) return fail("celestial_texture: " + err);
  std::vector<TexturePatch> patches;
  int rc = fill_texture(hs.get(), ct, resource_root, d.celestial, &need_bb, &patches);
  if (rc) return rc;
  if (!num(root, "celestial_temperature", &d.celestial_temperature, err)) return fail(err);
  rc = grt_camera_build(d.geometry, d.radius, d.a, pos, vel, 3.14159265358979323846 / 4.0, opts->height, opts->width,
                        opts->phi, opts->theta, opts->psi, &d.camera);
  if (rc) return fail("Camera error: Tetrad is not orthonormal");

  // objects, in config order (cli/shared.rs:176-308)
  const TomlValue* objs = get(root, "objects");
  if (!objs || objs->kind != TomlValue::TableArray) return fail("missing `objects` array");
  if (objs->arr.size() > GRT_MAX_OBJECTS) return fail("too many objects");
  for (size_t k = 0; k < objs->arr.size(); ++k) {
    std::string oname;
    const TomlTable* ob;
    const TomlValue* ov = objs->arr[k].get();
    if (ov->kind != TomlValue::Table || ov->table.size() != 1) return fail("each [[objects]] needs one variant table");
    if (!variant(ov, oname, &ob)) return fail("invalid object");
    grt_object_desc& o = d.objects[d.n_objects];
    std::memset(&o, 0, sizeof(o));
    TexSpec tex;
    if (!parse_texture(get(*ob, "texture"), tex, err)) return fail(oname + ".texture: " + err);
    if (oname == "Sphere") {
      o.kind = GRT_OBJ_SPHERE;
      if (!num(*ob, "radius", &o.radius, err) || !triple(*ob, "position", o.center, err) ||
          !num(*ob, "temperature", &o.temperature, err))
        return fail("Sphere: " + err);
    } else if (oname == "Disc" || oname == "VolumetricDisc") {
      const bool vol = oname == "VolumetricDisc";
      o.kind = vol ? GRT_OBJ_VOLUMETRIC_DISC : GRT_OBJ_DISC;
      double temperature;
      if (!num(*ob, "inner_radius", &o.inner_radius, err) || !num(*ob, "outer_radius", &o.outer_radius, err) ||
          !num(*ob, "temperature", &temperature, err))
        return fail(oname + ": " + err);
      if (vol) {  // configuration.rs:200-217, validated as cli/shared.rs:238-284
        uint64_t octaves, msteps, seed = 1;
        if (!uint_field(*ob, "num_octaves", &octaves, err) || !uint_field(*ob, "max_steps", &msteps, err) ||
            !num(*ob, "step_size", &o.march_step_size, err) || !num(*ob, "thickness", &o.thickness, err) ||
            !num(*ob, "density_multiplier", &o.density_multiplier, err) ||
            !num(*ob, "brightness_reference_temperature", &o.brightness_reference_temperature, err) ||
            !num(*ob, "absorption", &o.absorption, err) || !num(*ob, "scattering", &o.scattering, err) ||
            !triple(*ob, "noise_scale", o.noise_scale, err) || !num(*ob, "noise_offset", &o.noise_offset, err))
          return fail("VolumetricDisc: " + err);
        if (get(*ob, "perlin_seed") && (!uint_field(*ob, "perlin_seed", &seed, err) || seed > 0xffffffffull))
          return fail("VolumetricDisc: field `perlin_seed` must be a u32");
        o.axis[0] = 0.0;
        o.axis[1] = 0.0;
        o.axis[2] = 1.0;
        if (get(*ob, "axis") && !triple(*ob, "axis", o.axis, err)) return fail("VolumetricDisc: " + err);
        o.num_octaves = (uint32_t)(octaves > 0xffffffffull ? 0xffffffffull : octaves);
        o.march_max_steps = msteps;
        o.perlin_seed = (uint32_t)seed;
        char buf[256];
        auto bad = [&](const char* what, double v) {
          snprintf(buf, sizeof buf, "Invalid configuration: VolumetricDisc requires %s (got %s=%g).", what,
                   what, v);
          return fail(buf);
        };
        if (o.outer_radius <= o.inner_radius) {
          snprintf(buf, sizeof buf,
                   "Invalid configuration: VolumetricDisc requires outer_radius > inner_radius (got "
                   "outer_radius=%g, inner_radius=%g).",
                   o.outer_radius, o.inner_radius);
          return fail(buf);
        }
        if (o.thickness <= 0.0) return bad("thickness > 0", o.thickness);
        if (msteps == 0) return fail("Invalid configuration: VolumetricDisc requires max_steps > 0 (got max_steps=0).");
        if (o.march_step_size <= 0.0) return bad("step_size > 0", o.march_step_size);
        if (o.brightness_reference_temperature <= 0.0)
          return bad("brightness_reference_temperature > 0", o.brightness_reference_temperature);
        if (o.absorption < 0.0) return bad("absorption >= 0", o.absorption);
        if (o.scattering < 0.0) return bad("scattering >= 0", o.scattering);
      }
      // geometry.get_temperature_computer (euclidean.rs:219-226, schwarzschild.rs:267-279,
      // kerr.rs:498-510, kerr_bl.rs:412-424)
      if (d.geometry == GRT_GEOM_EUCLIDEAN || d.geometry == GRT_GEOM_EUCLIDEAN_SPHERICAL) {
        o.temp_kind = GRT_TEMP_CONSTANT;
        o.temp_constant = temperature;
      } else {
        o.temp_kind = GRT_TEMP_KERR_LUT;
        hs->lut_r[k].resize(1000);
        hs->lut_t[k].resize(1000);
        double spin = d.geometry == GRT_GEOM_SCHWARZSCHILD ? 0.0 : d.a;
        if (grt_host::kerr_temperature_lut(temperature, o.outer_radius, spin, d.radius, 1000, hs->lut_r[k].data(),
                                           hs->lut_t[k].data(), &o.r_isco, &hs->info_log))
          return fail(oname + " temperature LUT: DenominatorCloseToZero / NoCircularOrbitPossible");
        o.lut_r = hs->lut_r[k].data();
        o.lut_t = hs->lut_t[k].data();
        o.lut_n = 1000;
      }
    } else {
      return fail("unknown object `" + oname + "`");
    }
    rc = fill_texture(hs.get(), tex, resource_root, o.texture, &need_bb, &patches);
    if (rc) return rc;
    d.n_objects++;
  }
  if (need_bb) {
    hs->bb_log_t.resize(1000);
    hs->bb_xyz.resize(3000);
    grt_blackbody_lut(1000, hs->bb_log_t.data(), hs->bb_xyz.data());
    d.bb_log_t = hs->bb_log_t.data();
    d.bb_xyz = hs->bb_xyz.data();
    d.bb_n = 1000;
  }
  // the bitmaps, in the order the scene names them (the first decode error is reported)
  for (const TexturePatch& p : patches) {
    const std::string& err = p.ct->decoded.get();
    if (!err.empty()) return fail(err);
    p.d->width = p.ct->w;
    p.d->height = p.ct->h;
    p.d->rgba = p.ct->rgba.data();
  }
  *out = hs.release();
  return 0;
}

const grt_scene_desc* grt_host_scene_desc(const grt_host_scene* s) { return s ? &s->desc : nullptr; }
const char* grt_host_scene_log(const grt_host_scene* s) { return s ? s->info_log.c_str() : ""; }
void grt_host_scene_adaptive(const grt_host_scene* s, grt_adaptive_config* out) {
  if (s && out) *out = s->adaptive;
}
int grt_host_scene_destroy(grt_host_scene* s) {
  delete s;
  return 0;
}

}  // extern "C"
