// Start-up probe: time of the process's first HIP call (hipGetDeviceCount), built with and
// without librccl linked (-DWITH_RCCL), to price RCCL's presence at process start.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#ifdef WITH_RCCL
#include <rccl/rccl.h>
#endif
int main() {
  auto t0 = std::chrono::steady_clock::now();
  int n = 0;
  (void)hipGetDeviceCount(&n);
  auto t1 = std::chrono::steady_clock::now();
  void* p = nullptr;
  (void)hipMalloc(&p, 1 << 20);
  (void)hipFree(p);
  auto t2 = std::chrono::steady_clock::now();
#ifdef WITH_RCCL
  int v = 0;
  (void)ncclGetVersion(&v);
#endif
  std::printf("{\"rccl\": %d, \"devices\": %d, \"get_device_count_ms\": %.1f, \"first_malloc_ms\": %.1f}\n",
#ifdef WITH_RCCL
              1,
#else
              0,
#endif
              n, std::chrono::duration<double, std::milli>(t1 - t0).count(),
              std::chrono::duration<double, std::milli>(t2 - t1).count());
  return 0;
}
