// fp64_peak.hip — measures the sustained FP64 vector FMA rate of the device, to pin
// the roofline peak used by bench.py (MI355X FP64 vector spec: 78.6 TFLOP/s).
#include <hip/hip_runtime.h>
#include <cstdio>

template <int CHAINS>
__global__ void __launch_bounds__(256) fma_kernel(double* out, double a, double b, int iters) {
  double x[CHAINS];
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) x[c] = threadIdx.x * 1e-3 + c;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) x[c] = __fma_rn(x[c], a, b);
  }
  double s = 0;
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) s += x[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  int dev = 0;
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, dev);
  int blocks = p.multiProcessorCount * 8, threads = 256, iters = 20000;
  double* out;
  hipMalloc(&out, (size_t)blocks * threads * sizeof(double));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(fma_kernel<16>, dim3(blocks), dim3(threads), 0, 0, out, 0.999999, 1e-7, 100);
  hipDeviceSynchronize();
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    hipEventRecord(e0);
    hipLaunchKernelGGL(fma_kernel<16>, dim3(blocks), dim3(threads), 0, 0, out, 0.999999, 1e-7, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    if (ms < best) best = ms;
  }
  double flops = 2.0 * 16 * (double)iters * blocks * threads;
  printf("{\"fp64_fma_tflops\": %.2f, \"cus\": %d, \"clock_khz\": %d, \"ms\": %.3f}\n", flops / (best * 1e-3) / 1e12,
         p.multiProcessorCount, p.clockRate, best);
  return 0;
}
