// output.hip — the reference's output stage on the device:
// CIE XYZ -> linear sRGB -> tone mapping -> sRGB compand -> u8, i.e.
// xyz_to_linear_srgb_buffer + linear_srgb_to_srgb_buffer (color.rs:204-298) as called
// by Raytracer::render_section for non-HDR files (raytracer.rs:460-497, exposure 1).
//
// Two kernels, both HBM-bound streams over the f64 XYZA framebuffer (32 B in, 3 B out
// per pixel):
//   linear_max_kernel  GlobalLinear only: per-channel max of (M * xyz) * exposure,
//                      folded from 0.0 like the reference's fold(0.0, f64::max).  Every
//                      contributing value is > 0, and positive doubles order like their
//                      bit patterns, so the cross-block combine is an exact u64 atomicMax.
//                      A multi-GPU frame allreduces the 3 maxima (MAX) before tonemap.
//   tonemap_kernel     per pixel, in the reference's operation order; powf(1/2.4) is
//                      glibc's pow bit for bit (glibc_math.h), so the bytes equal the
//                      reference's.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cerrno>
#include <string>

#include "grt_api.h"
#include "../host/host_internal.h"
#include "glibc_math.h"

namespace grt {
namespace {

#define ODEV __device__ __forceinline__

// 2003 IEC inverse matrix (color.rs:211-223), nalgebra gemv order
ODEV void xyz_to_linear(const double* c, double* lin) {
  lin[0] = 3.2406255 * c[0];
  lin[0] = -1.5372080 * c[1] + lin[0];
  lin[0] = -0.4986286 * c[2] + lin[0];
  lin[1] = -0.9689307 * c[0];
  lin[1] = 1.8757561 * c[1] + lin[1];
  lin[1] = 0.0415175 * c[2] + lin[1];
  lin[2] = 0.0557101 * c[0];
  lin[2] = -0.2040211 * c[1] + lin[2];
  lin[2] = 1.0569959 * c[2] + lin[2];
}

ODEV double opow(double x, double y) {
  double r;
  if (glibc::pow_fast(x, y, &r)) return r;
  return pow(x, y);
}

// compand_srgb (color.rs:193-202)
ODEV double compand(double linear) {
  const double sign = linear < 0.0 ? -1.0 : 1.0;
  const double a = fabs(linear);
  const double enc = a <= 0.0031308 ? 12.92 * a : 1.055 * opow(a, 1.0 / 2.4) - 0.055;
  double v = sign * enc;  // f64::clamp(0, 1)
  if (v < 0.0) v = 0.0;
  if (v > 1.0) v = 1.0;
  return v;
}

// (x * 255.0).round() as u8: round half away from zero, saturating cast (NaN -> 0)
ODEV uint8_t to_u8(double v) {
  const double r = round(v * 255.0);
  if (!(r > 0.0)) return 0;
  if (r >= 255.0) return 255;
  return (uint8_t)r;
}

__global__ void __launch_bounds__(256) linear_max_kernel(const double* __restrict__ xyza, uint64_t n,
                                                         double exposure, unsigned long long* __restrict__ max3) {
  double m[3] = {0.0, 0.0, 0.0};
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const double4 c4 = reinterpret_cast<const double4*>(xyza)[i];
    const double c[3] = {c4.x, c4.y, c4.z};
    double lin[3];
    xyz_to_linear(c, lin);
#pragma unroll
    for (int k = 0; k < 3; ++k) m[k] = fmax(m[k], lin[k] * exposure);  // fmax drops NaN like f64::max
  }
#pragma unroll
  for (int k = 0; k < 3; ++k)
    for (int off = 32; off > 0; off >>= 1) m[k] = fmax(m[k], __shfl_down(m[k], off));
  __shared__ double part[3][4];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0)
    for (int k = 0; k < 3; ++k) part[k][wave] = m[k];
  __syncthreads();
  if (threadIdx.x < 3) {
    double v = 0.0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) v = fmax(v, part[threadIdx.x][w]);
    if (v > 0.0) atomicMax(max3 + threadIdx.x, (unsigned long long)__double_as_longlong(v));
  }
}

__global__ void __launch_bounds__(256) tonemap_kernel(const double* __restrict__ xyza, uint64_t n, int tone,
                                                      double exposure, const double* __restrict__ max3,
                                                      uint8_t* __restrict__ rgb) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double4 c4 = reinterpret_cast<const double4*>(xyza)[i];
  const double xyz[3] = {c4.x, c4.y, c4.z};
  double c[3];
  xyz_to_linear(xyz, c);
#pragma unroll
  for (int k = 0; k < 3; ++k) c[k] = c[k] * exposure;
  if (tone == GRT_TONE_REINHARD) {
    const double l_in = 0.2126 * c[0] + 0.7152 * c[1] + 0.0722 * c[2];
    if (l_in > 0.0) {
      const double l_out = l_in / (1.0 + l_in);
      const double f = l_out / l_in;
#pragma unroll
      for (int k = 0; k < 3; ++k) c[k] = c[k] * f;
    }
  } else {
    const double mc = fmax(fmax(max3[0], max3[1]), max3[2]);
    const double scale = mc > 0.0 ? 1.0 / mc : 1.0;
#pragma unroll
    for (int k = 0; k < 3; ++k) c[k] = scale * c[k];
  }
#pragma unroll
  for (int k = 0; k < 3; ++k) rgb[3 * i + k] = to_u8(compand(fmax(c[k], 0.0)));
}

int fail(int code, const std::string& msg) {
  grt_host::set_error(msg);
  return code;
}
#define OUT_TRY(expr)                                                                    \
  do {                                                                                   \
    hipError_t _e = (expr);                                                              \
    if (_e != hipSuccess) return grt::fail(-EIO, std::string(#expr) + ": " + hipGetErrorString(_e)); \
  } while (0)

int grid_for(uint64_t n, int cap) {
  uint64_t b = (n + 255) / 256;
  return (int)(b < (uint64_t)cap ? (b ? b : 1) : cap);
}

}  // namespace
}  // namespace grt

extern "C" {

int grt_linear_max_async(int device, void* stream, const double* d_xyza, uint64_t n, double exposure,
                         double* d_max3) {
  if (!d_max3 || (n && !d_xyza)) return grt::fail(-EINVAL, "grt_linear_max_async: null buffer");
  OUT_TRY(hipSetDevice(device));
  hipStream_t s = (hipStream_t)stream;
  OUT_TRY(hipMemsetAsync(d_max3, 0, 3 * sizeof(double), s));
  if (n == 0) return 0;
  hipLaunchKernelGGL(grt::linear_max_kernel, dim3(grt::grid_for(n, 4096)), dim3(256), 0, s, d_xyza, n, exposure,
                     reinterpret_cast<unsigned long long*>(d_max3));
  OUT_TRY(hipGetLastError());
  return 0;
}

int grt_tonemap_async(int device, void* stream, const double* d_xyza, uint64_t n, int32_t tone_mapping,
                      double exposure, const double* d_max3, uint8_t* d_rgb) {
  if (tone_mapping != GRT_TONE_REINHARD && tone_mapping != GRT_TONE_GLOBAL_LINEAR)
    return grt::fail(-EINVAL, "unknown tone mapping");
  if (tone_mapping == GRT_TONE_GLOBAL_LINEAR && !d_max3)
    return grt::fail(-EINVAL, "GlobalLinear tone mapping needs the channel maxima");
  if (n && (!d_xyza || !d_rgb)) return grt::fail(-EINVAL, "grt_tonemap_async: null buffer");
  if (n == 0) return 0;
  OUT_TRY(hipSetDevice(device));
  const uint64_t blocks = (n + 255) / 256;
  if (blocks > 0x7fffffffull) return grt::fail(-EINVAL, "grt_tonemap_async: too many pixels");
  hipLaunchKernelGGL(grt::tonemap_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, d_xyza, n,
                     (int)tone_mapping, exposure, d_max3, d_rgb);
  OUT_TRY(hipGetLastError());
  return 0;
}

int grt_xyz_to_srgb8_device(int device, const double* xyza, size_t n, int32_t tone_mapping, double exposure,
                            uint8_t* rgb_out) {
  if (n && (!xyza || !rgb_out)) return grt::fail(-EINVAL, "grt_xyz_to_srgb8_device: null buffer");
  if (tone_mapping != GRT_TONE_REINHARD && tone_mapping != GRT_TONE_GLOBAL_LINEAR)
    return grt::fail(-EINVAL, "unknown tone mapping");
  if (n == 0) return 0;
  OUT_TRY(hipSetDevice(device));
  void *d_in = nullptr, *d_rgb = nullptr, *d_max = nullptr;
  int rc = 0;
  hipError_t e = hipMalloc(&d_in, n * 4 * sizeof(double));
  if (e == hipSuccess) e = hipMalloc(&d_rgb, n * 3);
  if (e == hipSuccess) e = hipMalloc(&d_max, 3 * sizeof(double));
  if (e == hipSuccess) e = hipMemcpy(d_in, xyza, n * 4 * sizeof(double), hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    rc = grt::fail(-EIO, std::string("grt_xyz_to_srgb8_device: ") + hipGetErrorString(e));
  } else {
    if (tone_mapping == GRT_TONE_GLOBAL_LINEAR)
      rc = grt_linear_max_async(device, nullptr, (const double*)d_in, n, exposure, (double*)d_max);
    if (!rc) rc = grt_tonemap_async(device, nullptr, (const double*)d_in, n, tone_mapping, exposure,
                                    (const double*)d_max, (uint8_t*)d_rgb);
    if (!rc && (e = hipMemcpy(rgb_out, d_rgb, n * 3, hipMemcpyDeviceToHost)) != hipSuccess)
      rc = grt::fail(-EIO, std::string("grt_xyz_to_srgb8_device: ") + hipGetErrorString(e));
  }
  if (d_in) (void)hipFree(d_in);
  if (d_rgb) (void)hipFree(d_rgb);
  if (d_max) (void)hipFree(d_max);
  return rc;
}

}  // extern "C"
