// png.cpp — PNG decode/encode for textures and output images (the `image` crate's
// role in rendering/texture.rs:46-59 and raytracer.rs:468-495).  Decodes 8-bit,
// non-interlaced greyscale / grey+alpha / RGB / RGBA / palette images (every texture
// in the reference's resources/ is 8-bit RGB or RGBA, non-interlaced) to RGBA8 the
// way DynamicImage::get_pixel does (missing alpha = 255).  Encodes RGB8.  Also writes
// Radiance .hdr (RGBE) for the `.hdr` output path.
#include <zlib.h>

#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iterator>

#include "host_internal.h"

namespace grt_host {

static uint32_t be32(const uint8_t* p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }

static uint8_t paeth(int a, int b, int c) {
  int p = a + b - c;
  int pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
  if (pa <= pb && pa <= pc) return (uint8_t)a;
  if (pb <= pc) return (uint8_t)b;
  return (uint8_t)c;
}

bool png_decode_rgba(const std::string& path, std::vector<uint8_t>& rgba, uint32_t& w, uint32_t& h,
                     std::string& err) {
  std::ifstream f(path, std::ios::binary);
  if (!f) {
    err = "cannot open texture '" + path + "'";
    return false;
  }
  std::vector<uint8_t> data((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  static const uint8_t sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
  if (data.size() < 8 || std::memcmp(data.data(), sig, 8) != 0) {
    err = "not a PNG file: '" + path + "'";
    return false;
  }
  size_t p = 8;
  int bit_depth = 0, color_type = -1, interlace = 0;
  std::vector<uint8_t> idat, palette, trns;
  while (p + 8 <= data.size()) {
    uint32_t len = be32(&data[p]);
    std::string type((const char*)&data[p + 4], 4);
    if (p + 12 + (size_t)len > data.size()) break;
    const uint8_t* d = &data[p + 8];
    if (type == "IHDR") {
      w = be32(d);
      h = be32(d + 4);
      bit_depth = d[8];
      color_type = d[9];
      interlace = d[12];
    } else if (type == "PLTE") {
      palette.assign(d, d + len);
    } else if (type == "tRNS") {
      trns.assign(d, d + len);
    } else if (type == "IDAT") {
      idat.insert(idat.end(), d, d + len);
    } else if (type == "IEND") {
      break;
    }
    p += 12 + len;
  }
  if (bit_depth != 8 || interlace != 0) {
    err = "unsupported PNG (need 8-bit, non-interlaced): '" + path + "'";
    return false;
  }
  int channels;
  switch (color_type) {
    case 0: channels = 1; break;
    case 2: channels = 3; break;
    case 3: channels = 1; break;
    case 4: channels = 2; break;
    case 6: channels = 4; break;
    default:
      err = "unsupported PNG colour type: '" + path + "'";
      return false;
  }
  size_t stride = (size_t)w * channels;
  std::vector<uint8_t> raw((stride + 1) * h);
  uLongf raw_len = (uLongf)raw.size();
  if (uncompress(raw.data(), &raw_len, idat.data(), (uLong)idat.size()) != Z_OK || raw_len != raw.size()) {
    err = "corrupt PNG data: '" + path + "'";
    return false;
  }
  std::vector<uint8_t> img(stride * h);
  for (uint32_t y = 0; y < h; ++y) {
    uint8_t ft = raw[y * (stride + 1)];
    const uint8_t* src = &raw[y * (stride + 1) + 1];
    uint8_t* dst = &img[y * stride];
    const uint8_t* prev = y ? &img[(y - 1) * stride] : nullptr;
    for (size_t x = 0; x < stride; ++x) {
      int a = x >= (size_t)channels ? dst[x - channels] : 0;
      int b = prev ? prev[x] : 0;
      int c = (prev && x >= (size_t)channels) ? prev[x - channels] : 0;
      int v = src[x];
      switch (ft) {
        case 0: break;
        case 1: v += a; break;
        case 2: v += b; break;
        case 3: v += (a + b) / 2; break;
        case 4: v += paeth(a, b, c); break;
        default:
          err = "bad PNG filter: '" + path + "'";
          return false;
      }
      dst[x] = (uint8_t)v;
    }
  }
  rgba.resize((size_t)w * h * 4);
  for (size_t i = 0; i < (size_t)w * h; ++i) {
    uint8_t* o = &rgba[4 * i];
    const uint8_t* s = &img[i * channels];
    switch (color_type) {
      case 0: o[0] = o[1] = o[2] = s[0]; o[3] = 255; break;
      case 2: o[0] = s[0]; o[1] = s[1]; o[2] = s[2]; o[3] = 255; break;
      case 4: o[0] = o[1] = o[2] = s[0]; o[3] = s[1]; break;
      case 6: o[0] = s[0]; o[1] = s[1]; o[2] = s[2]; o[3] = s[3]; break;
      case 3: {
        size_t k = s[0];
        if (3 * k + 2 >= palette.size()) {
          err = "PNG palette index out of range: '" + path + "'";
          return false;
        }
        o[0] = palette[3 * k];
        o[1] = palette[3 * k + 1];
        o[2] = palette[3 * k + 2];
        o[3] = k < trns.size() ? trns[k] : 255;
        break;
      }
    }
  }
  return true;
}

static void put32(std::vector<uint8_t>& v, uint32_t x) {
  v.push_back(x >> 24);
  v.push_back(x >> 16);
  v.push_back(x >> 8);
  v.push_back(x);
}
static void chunk(std::vector<uint8_t>& out, const char* type, const std::vector<uint8_t>& d) {
  put32(out, (uint32_t)d.size());
  std::vector<uint8_t> td(type, type + 4);
  td.insert(td.end(), d.begin(), d.end());
  out.insert(out.end(), td.begin(), td.end());
  put32(out, (uint32_t)crc32(0, td.data(), (uInt)td.size()));
}

// 8-bit RGB (colour type 2) or RGBA (6), no interlace, filter 0 on every row.
static bool png_encode(const std::string& path, const uint8_t* px, uint32_t w, uint32_t h, uint32_t channels,
                       std::string& err) {
  const size_t row = (size_t)w * channels;
  std::vector<uint8_t> raw((row + 1) * h);
  for (uint32_t y = 0; y < h; ++y) {
    raw[y * (row + 1)] = 0;
    std::memcpy(&raw[y * (row + 1) + 1], px + (size_t)y * row, row);
  }
  uLongf zl = compressBound((uLong)raw.size());
  std::vector<uint8_t> z(zl);
  if (compress2(z.data(), &zl, raw.data(), (uLong)raw.size(), 6) != Z_OK) {
    err = "zlib compression failed";
    return false;
  }
  z.resize(zl);
  std::vector<uint8_t> out = {137, 80, 78, 71, 13, 10, 26, 10};
  std::vector<uint8_t> ihdr;
  put32(ihdr, w);
  put32(ihdr, h);
  ihdr.insert(ihdr.end(), {8, (uint8_t)(channels == 4 ? 6 : 2), 0, 0, 0});
  chunk(out, "IHDR", ihdr);
  chunk(out, "IDAT", z);
  chunk(out, "IEND", {});
  std::ofstream f(path, std::ios::binary);
  if (!f) {
    err = "cannot write '" + path + "'";
    return false;
  }
  f.write((const char*)out.data(), (std::streamsize)out.size());
  return (bool)f;
}

bool png_encode_rgb(const std::string& path, const uint8_t* rgb, uint32_t w, uint32_t h, std::string& err) {
  return png_encode(path, rgb, w, h, 3, err);
}
bool png_encode_rgba(const std::string& path, const uint8_t* rgba, uint32_t w, uint32_t h, std::string& err) {
  return png_encode(path, rgba, w, h, 4, err);
}

bool hdr_encode_rgb(const std::string& path, const float* rgb, uint32_t w, uint32_t h, std::string& err) {
  std::ofstream f(path, std::ios::binary);
  if (!f) {
    err = "cannot write '" + path + "'";
    return false;
  }
  f << "#?RADIANCE\nFORMAT=32-bit_rle_rgbe\n\n-Y " << h << " +X " << w << "\n";
  std::vector<uint8_t> row((size_t)w * 4);
  for (uint32_t y = 0; y < h; ++y) {
    for (uint32_t x = 0; x < w; ++x) {
      const float* c = rgb + 3 * ((size_t)y * w + x);
      float m = std::fmax(c[0], std::fmax(c[1], c[2]));
      uint8_t* o = &row[4 * x];
      if (!(m > 1e-32f)) {
        o[0] = o[1] = o[2] = o[3] = 0;
      } else {
        int e;
        float s = std::frexp(m, &e) * 256.0f / m;
        o[0] = (uint8_t)(c[0] * s);
        o[1] = (uint8_t)(c[1] * s);
        o[2] = (uint8_t)(c[2] * s);
        o[3] = (uint8_t)(e + 128);
      }
    }
    f.write((const char*)row.data(), (std::streamsize)row.size());
  }
  return (bool)f;
}

}  // namespace grt_host

// ---- C ABI: the image files Raytracer::render_section writes (raytracer.rs:460-497) ----
extern "C" int grt_write_png_rgb(const char* path, const uint8_t* rgb, uint32_t width, uint32_t height) {
  if (!path || (!rgb && width && height)) {
    grt_host::set_error("null argument");
    return -EINVAL;
  }
  std::string err;
  if (!grt_host::png_encode_rgb(path, rgb, width, height, err)) {
    grt_host::set_error(err);
    return -EIO;
  }
  return 0;
}

extern "C" int grt_write_hdr_xyz(const char* path, const double* xyza, uint32_t width, uint32_t height) {
  if (!path || (!xyza && width && height)) {
    grt_host::set_error("null argument");
    return -EINVAL;
  }
  // XYZ stored as the RGB channels of an f32 Radiance image (raytracer.rs:468-480)
  std::vector<float> rgb((size_t)width * height * 3);
  for (size_t i = 0; i < (size_t)width * height; ++i)
    for (int k = 0; k < 3; ++k) rgb[3 * i + k] = (float)xyza[4 * i + k];
  std::string err;
  if (!grt_host::hdr_encode_rgb(path, rgb.data(), width, height, err)) {
    grt_host::set_error(err);
    return -EIO;
  }
  return 0;
}
