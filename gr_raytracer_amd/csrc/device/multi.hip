// multi.hip — one frame over several GPUs of one process (grt_render_frame_multi,
// include/grt_api.h): the north-star layout behind the C ABI.  The frame's rows are cut
// into cyclic bands (band b -> device b mod N, grt_row_shard), one host thread per device
// traces its bands (grt_render_shard_async on the device's own stream), and ONE grouped
// RCCL send/recv moves every device's pixel records to devices[0] over xGMI, where
// deinterleave_kernel puts them in frame order.  With the reference's adaptive
// supersampling, one RCCL allgather of (Y, alpha, class) per pixel comes first: the
// selection stencil reads neighbours in other devices' bands and the luminance floor is a
// percentile of the whole frame (raytracer.rs:91-129, :386-458).
//
// The reference renders a frame in one process (render_section_to_cie_buffer_raw,
// raytracer.rs:195-244, called from main.rs:80-116 via Raytracer::render_section
// :460-497); every pixel here is identical to grt_render_pixels / grt_render_section of
// the same frame on one device (tests/test_multi.py).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cerrno>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <future>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <type_traits>
#include <vector>

#include "grt_api.h"
#include "../host/host_internal.h"
#include "dev_scene.h"

namespace grt {

// Fields of a pixel record, in the order they sit in a device's send block (8-byte fields
// first).  Bit f of a field mask selects field f.
enum RecField { RF_XYZA64 = 0, RF_XYZA32 = 1, RF_STEPS = 2, RF_CLASS = 3, RF_STATUS = 4, RF_STOP = 5, RF_N = 6 };
#if defined(__HIPCC__)
__host__ __device__
#endif
constexpr uint32_t rec_field_bytes(int f) { return f == RF_XYZA64 ? 32 : f == RF_XYZA32 ? 16 : f == RF_STEPS ? 4 : 1; }

constexpr int MULTI_MAX = GRT_MULTI_MAX_DEVICES;

// Where the gathered buffer holds each shard's fields, and the frame they go to.
struct GatherLayout {
  uint32_t cols, band_rows, n_shards, n_fields;
  uint64_t n_pixels;                 // frame pixels, rows x cols
  uint32_t elem[RF_N];               // bytes per pixel of gathered field k
  uint64_t src[MULTI_MAX][RF_N];     // byte offset of shard s's field k in the gathered buffer
};
struct GatherDst {
  uint8_t* p[RF_N];  // frame-order output of gathered field k
};

// Frame row -> (shard, local row): the inverse of shard_frame_row (dev_scene.h).
__host__ __device__ inline void frame_row_source(uint32_t band_rows, uint32_t n_shards, uint32_t row,
                                                 uint32_t* shard, uint32_t* local) {
  if (n_shards <= 1) {
    *shard = 0;
    *local = row;
    return;
  }
  const uint32_t band = row / band_rows;
  *shard = band % n_shards;
  *local = (band / n_shards) * band_rows + row % band_rows;
}

// Byte offset in the gathered buffer of frame pixel p's field k.
__host__ __device__ inline uint64_t gather_source(const GatherLayout& L, int k, uint64_t p) {
  const uint32_t row = (uint32_t)(p / L.cols), col = (uint32_t)(p % L.cols);
  uint32_t s, lr;
  frame_row_source(L.band_rows, L.n_shards, row, &s, &lr);
  return L.src[s][k] + ((uint64_t)lr * L.cols + col) * L.elem[k];
}

// De-interleave: blockIdx.y = field, a grid-stride loop over the frame's pixels.  Reads
// are coalesced within a band row (consecutive pixels of one row are consecutive in their
// shard), writes always.  Every field offset is 256-B aligned, so the 32- and 16-B
// fields move as 16-B vectors.  An HBM stream: (read + write) x record bytes per pixel.
__global__ void __launch_bounds__(256) deinterleave_kernel(GatherLayout L, const uint8_t* __restrict__ g,
                                                           GatherDst d) {
  const int k = blockIdx.y;
  const uint32_t e = L.elem[k];
  uint8_t* __restrict__ out = d.p[k];
  for (uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; p < L.n_pixels;
       p += (uint64_t)gridDim.x * blockDim.x) {
    const uint8_t* s = g + gather_source(L, k, p);
    uint8_t* t = out + p * e;
    if (e == 32) {
      const uint4 a = ((const uint4*)s)[0], b = ((const uint4*)s)[1];
      ((uint4*)t)[0] = a;
      ((uint4*)t)[1] = b;
    } else if (e == 16) {
      *(uint4*)t = *(const uint4*)s;
    } else if (e == 4) {
      *(uint32_t*)t = *(const uint32_t*)s;
    } else {
      for (uint32_t b = 0; b < e; ++b) t[b] = s[b];
    }
  }
}

// The adaptive pass's neighbourhood record of each local pixel: (Y, alpha) of the 1-spp
// f64 XYZA, and the class (should_supersample_pair, raytracer.rs:91-108; the floor,
// resolve_minimum_luminance :118-129, reads Y).
__global__ void __launch_bounds__(256) pack_ya_kernel(const double* __restrict__ x64, const uint8_t* __restrict__ cls,
                                                      uint64_t n, double* __restrict__ ya, uint8_t* __restrict__ c_out) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const double y = x64[4 * i + 1], a = x64[4 * i + 3];
    ya[2 * i] = y;
    ya[2 * i + 1] = a;
    c_out[i] = cls[i];
  }
}

}  // namespace grt

namespace {

int fail(int code, const std::string& msg) {
  grt_host::set_error(msg);
  return code;
}

// RCCL is bound at the first multi-GPU frame (dlopen of librccl.so.1), not linked: a
// process that never renders over several GPUs (the single-GPU CLI, the Python host) does
// not load the 570 MB library at start-up, and libgrt.so loads where RCCL is absent.
struct Rccl {
  decltype(&ncclCommInitAll) CommInitAll = nullptr;
  decltype(&ncclCommDestroy) CommDestroy = nullptr;
  decltype(&ncclGetErrorString) GetErrorString = nullptr;
  decltype(&ncclAllGather) AllGather = nullptr;
  decltype(&ncclGroupStart) GroupStart = nullptr;
  decltype(&ncclGroupEnd) GroupEnd = nullptr;
  decltype(&ncclSend) Send = nullptr;
  decltype(&ncclRecv) Recv = nullptr;
  std::string error;  // why binding failed, or empty
};
const Rccl& rccl() {
  static const Rccl r = [] {
    Rccl x;
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) {
      const char* e = dlerror();
      x.error = std::string("cannot load librccl.so.1: ") + (e ? e : "unknown error");
      return x;
    }
    auto get = [&](auto& fn, const char* name) {
      fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
      if (!fn && x.error.empty()) x.error = std::string("librccl.so.1 has no ") + name;
    };
    get(x.CommInitAll, "ncclCommInitAll");
    get(x.CommDestroy, "ncclCommDestroy");
    get(x.GetErrorString, "ncclGetErrorString");
    get(x.AllGather, "ncclAllGather");
    get(x.GroupStart, "ncclGroupStart");
    get(x.GroupEnd, "ncclGroupEnd");
    get(x.Send, "ncclSend");
    get(x.Recv, "ncclRecv");
    return x;
  }();
  return r;
}
#define HIP_TRY(expr)                                                                    \
  do {                                                                                   \
    hipError_t _e = (expr);                                                              \
    if (_e != hipSuccess) {                                                              \
      (void)hipGetLastError();                                                           \
      return fail(-EIO, std::string(#expr) + ": " + hipGetErrorString(_e));             \
    }                                                                                    \
  } while (0)
#define NCCL_TRY(expr)                                                                   \
  do {                                                                                   \
    ncclResult_t _r = (expr);                                                            \
    if (_r != ncclSuccess) return fail(-EIO, std::string(#expr) + ": " + rccl().GetErrorString(_r)); \
  } while (0)

constexpr uint64_t align256(uint64_t b) { return (b + 255) & ~255ull; }

// Byte offset of field f in a block of n pixels holding the fields of `mask`; f = RF_N
// gives the block's size.  Each field starts 256-B aligned.
uint64_t field_offset(uint32_t mask, uint64_t n, int f) {
  uint64_t off = 0;
  for (int g = 0; g < f; ++g)
    if (mask & (1u << g)) off += align256(n * grt::rec_field_bytes(g));
  return off;
}

// Per device: its stream, events and a grow-only scratch arena.
struct MultiDev {
  int device = 0;
  hipStream_t st = nullptr;
  hipEvent_t ev[6] = {};  // trace start / end, allgather start / end, gather start / end
  void* mem = nullptr;
  uint64_t bytes = 0;
};

// One RCCL communicator per device of a device list (ncclCommInitAll), created on first
// use and cached for the process: a frame after the first pays no setup.  `mu` serialises
// frames on one device list (a communicator is driven by one thread at a time).
// RCCL's start-up takes seconds (1.6-5.8 s for one device on the pool's boxes, most of it
// loading its device code), and while it runs a kernel launch of the process can wait for
// it; so the communicators are created on a thread of their own (`comm_ready`) started
// once every device has enqueued its first frame's trace (note_launched), and a device
// waits for them only before its first collective.
struct MultiCtx {
  std::vector<int> devs;
  std::vector<ncclComm_t> comms;
  std::vector<MultiDev> d;
  std::mutex mu;
  std::mutex cm;  // the three below
  std::condition_variable cv;
  int launched = 0;
  bool started = false;
  std::shared_future<std::string> comm_ready;  // "" once the communicators exist, else the error

  // A device thread of the first frame has enqueued its trace (or failed before): the
  // last of them starts the communicators' creation.
  void note_launched() {
    std::lock_guard<std::mutex> lk(cm);
    if (started || ++launched < (int)devs.size()) return;
    started = true;
    MultiCtx* cp = this;
    comm_ready = std::async(std::launch::async, [cp]() -> std::string {
                   const Rccl& R = rccl();
                   if (!R.error.empty()) return R.error;
                   const ncclResult_t r = R.CommInitAll(cp->comms.data(), (int)cp->devs.size(), cp->devs.data());
                   return r == ncclSuccess ? std::string() : std::string("ncclCommInitAll: ") + R.GetErrorString(r);
                 }).share();
    cv.notify_all();
  }
};
std::mutex g_ctx_mu;
std::vector<std::unique_ptr<MultiCtx>> g_ctx;

int get_ctx(const std::vector<int>& devs, MultiCtx** out) {
  std::lock_guard<std::mutex> lk(g_ctx_mu);
  for (auto& c : g_ctx)
    if (c->devs == devs) {
      *out = c.get();
      return 0;
    }
  auto c = std::make_unique<MultiCtx>();
  c->devs = devs;
  c->comms.resize(devs.size());
  c->d.resize(devs.size());
  for (size_t i = 0; i < devs.size(); ++i) {
    MultiDev& m = c->d[i];
    m.device = devs[i];
    HIP_TRY(hipSetDevice(devs[i]));
    HIP_TRY(hipStreamCreateWithFlags(&m.st, hipStreamNonBlocking));
    for (auto& e : m.ev) HIP_TRY(hipEventCreate(&e));
  }
  *out = c.get();
  g_ctx.push_back(std::move(c));
  return 0;
}

// A device list: 1..GRT_MULTI_MAX_DEVICES distinct, valid ordinals.
int check_devices(int n_devices, const int* devices, std::vector<int>* out) {
  if (!devices) return fail(-EINVAL, "null argument");
  if (n_devices < 1 || n_devices > grt::MULTI_MAX) return fail(-EINVAL, "n_devices must be in 1..GRT_MULTI_MAX_DEVICES");
  std::vector<int> devs(devices, devices + n_devices);
  for (int a = 0; a < n_devices; ++a)
    for (int b = a + 1; b < n_devices; ++b)
      if (devs[a] == devs[b]) return fail(-EINVAL, "a device appears twice (one RCCL rank per GPU)");
  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev));
  for (int d : devs)
    if (d < 0 || d >= ndev) return fail(-ENODEV, "invalid device ordinal");
  *out = std::move(devs);
  return 0;
}

// The communicators of C, waited for (created beside the first frame's traces).
int comms_ready(MultiCtx& C) {
  std::shared_future<std::string> f;
  {
    std::unique_lock<std::mutex> lk(C.cm);
    C.cv.wait(lk, [&] { return C.started; });
    f = C.comm_ready;
  }
  const std::string err = f.get();
  return err.empty() ? 0 : fail(-EIO, err);
}

// A reusable barrier of the device threads.  arrive(ok) returns false on every thread
// when any thread arrived with ok == false: no thread then enters the next collective
// (a peer that never joins would leave the others waiting in RCCL).
struct Barrier {
  std::mutex mu;
  std::condition_variable cv;
  int n, waiting = 0;
  uint64_t gen = 0;
  bool failed = false;
  explicit Barrier(int n_) : n(n_) {}
  bool arrive(bool ok) {
    std::unique_lock<std::mutex> lk(mu);
    if (!ok) failed = true;
    const uint64_t g = gen;
    if (++waiting == n) {
      waiting = 0;
      ++gen;
      cv.notify_all();
    } else {
      cv.wait(lk, [&] { return gen != g; });
    }
    return !failed;
  }
};

// The plan of one frame: which fields move, each device's rows and buffers.
struct Plan {
  uint32_t rows = 0, cols = 0, band = 0, n_dev = 0;
  uint32_t mask = 0;          // fields each device sends
  bool super = false;         // adaptive supersampling (or the sampling-mask paint)
  uint64_t n_local[grt::MULTI_MAX] = {};
  uint64_t block[grt::MULTI_MAX] = {};   // send block bytes
  uint64_t block_off[grt::MULTI_MAX + 1] = {};  // offsets in the gathered buffer
  uint64_t max_local = 0;
  uint64_t ag_bytes = 0;      // per-device allgather block: (Y, alpha) then class, padded to max_local
};

struct DevResult {
  int rc = 0;
  std::string err;
  unsigned long long stats[4] = {0, 0, 0, 0};
  uint64_t n_sel = 0;
  float trace_ms = 0, ag_ms = 0, gather_ms = 0;
  std::vector<uint32_t> f_pix, f_smp, f_steps;
  std::vector<uint8_t> f_status, f_stop;
  uint64_t f_count = 0;
};

// Carve a device's scratch (AdArena style: plan with base == nullptr, then carve).
struct Carve {
  char* base = nullptr;
  uint64_t off = 0;
  void* take(uint64_t b) {
    void* r = base ? base + off : nullptr;
    off += align256(b);
    return r;
  }
};
struct DevBufs {
  unsigned long long* stats = nullptr;  // [0..3] trace counters, [4] selected pixels
  double* floor = nullptr;
  uint8_t* block = nullptr;             // send block (fields of plan.mask)
  float* x32 = nullptr;                 // f32 XYZA when the plan does not send it
  double* x64 = nullptr;                // f64 XYZA when the plan does not send it (supersampling sends it)
  uint32_t* steps = nullptr;            // 1-spp step counts when supersampling and the plan does not send them
  uint8_t *ag_send = nullptr, *ag_recv = nullptr;
  double* frame_ya = nullptr;
  uint8_t* frame_cls = nullptr;
  uint8_t* gathered = nullptr;          // devices[0]: every block
  uint8_t* frame = nullptr;             // devices[0]: frame-order fields
};
void carve(Carve& A, const Plan& P, int i, DevBufs& B) {
  const uint64_t n = P.n_local[i];
  const uint64_t F = (uint64_t)P.rows * P.cols;
  B.stats = (unsigned long long*)A.take(8 * 8);
  B.floor = (double*)A.take(8);
  B.block = (uint8_t*)A.take(P.block[i]);
  if (!(P.mask & (1u << grt::RF_XYZA32))) B.x32 = (float*)A.take(n * 16);
  if (P.super) {
    if (!(P.mask & (1u << grt::RF_STEPS))) B.steps = (uint32_t*)A.take(n * 4);
    B.ag_send = (uint8_t*)A.take(P.ag_bytes);
    B.ag_recv = (uint8_t*)A.take(P.ag_bytes * P.n_dev);
    B.frame_ya = (double*)A.take(F * 16);
    B.frame_cls = (uint8_t*)A.take(F);
  }
  if (i == 0) {
    B.gathered = (uint8_t*)A.take(P.block_off[P.n_dev]);
    B.frame = (uint8_t*)A.take(field_offset(P.mask, F, grt::RF_N));
  }
}

uint8_t* field_ptr(uint8_t* block, uint32_t mask, uint64_t n, int f) {
  return (mask & (1u << f)) ? block + field_offset(mask, n, f) : nullptr;
}

grt::GatherLayout gather_layout(const Plan& P) {
  grt::GatherLayout L;
  std::memset(&L, 0, sizeof(L));
  L.cols = P.cols;
  L.band_rows = P.band;
  L.n_shards = P.n_dev;
  L.n_pixels = (uint64_t)P.rows * P.cols;
  for (int f = 0; f < grt::RF_N; ++f) {
    if (!(P.mask & (1u << f))) continue;
    const uint32_t k = L.n_fields++;
    L.elem[k] = grt::rec_field_bytes(f);
    for (uint32_t s = 0; s < P.n_dev; ++s) L.src[s][k] = P.block_off[s] + field_offset(P.mask, P.n_local[s], f);
  }
  return L;
}

int launch_deinterleave(const grt::GatherLayout& L, const uint8_t* g, const grt::GatherDst& d, hipStream_t st) {
  if (L.n_pixels == 0 || L.n_fields == 0) return 0;
  const uint64_t want = (L.n_pixels + 255) / 256;
  const unsigned gx = (unsigned)std::min<uint64_t>(want, 8192);
  hipLaunchKernelGGL(grt::deinterleave_kernel, dim3(gx, L.n_fields), dim3(256), 0, st, L, g, d);
  HIP_TRY(hipGetLastError());
  return 0;
}

// One device's part of one frame.  Every collective is entered only after a barrier that
// all threads pass with no error so far.
void device_part(grt_scene* scene, MultiCtx& C, const Plan& P, int i, const grt_adaptive_config* cfg,
                 const double* mask_xyza, const grt_frame_out* out, grt_subsample_failures* want_fail,
                 Barrier& bar, DevResult& R) {
  MultiDev& M = C.d[i];
  const int dev = M.device;
  // every thread arrives at each of the frame's barriers exactly once (a failed thread
  // arrives at the ones it has not reached with ok = false, below)
  const int n_barriers = P.super ? 2 : 1;
  int passed = 0;
  bool noted = false;  // C.note_launched() called
  auto barrier = [&]() -> bool {
    ++passed;
    return bar.arrive(true);
  };
  auto run = [&]() -> int {
    HIP_TRY(hipSetDevice(dev));
    Carve plan;
    DevBufs B;
    carve(plan, P, i, B);
    if (plan.off > M.bytes) {
      if (M.mem) {
        HIP_TRY(hipStreamSynchronize(M.st));
        HIP_TRY(hipFree(M.mem));
        M.mem = nullptr;
        M.bytes = 0;
      }
      HIP_TRY(hipMalloc(&M.mem, plan.off));
      M.bytes = plan.off;
    }
    Carve A{(char*)M.mem, 0};
    carve(A, P, i, B);
    const uint64_t n = P.n_local[i];
    const hipStream_t st = M.st;
    HIP_TRY(hipMemsetAsync(B.stats, 0, 8 * 8, st));
    HIP_TRY(hipEventRecord(M.ev[0], st));
    grt_row_shard sh{P.band, (uint32_t)i, P.n_dev};
    float* x32 = (P.mask & (1u << grt::RF_XYZA32)) ? (float*)field_ptr(B.block, P.mask, n, grt::RF_XYZA32) : B.x32;
    double* x64 = (double*)field_ptr(B.block, P.mask, n, grt::RF_XYZA64);
    uint8_t* cls = field_ptr(B.block, P.mask, n, grt::RF_CLASS);
    uint8_t* status = field_ptr(B.block, P.mask, n, grt::RF_STATUS);
    // the supersample pass orders its sub-rays by the 1-spp step counts: traced always then
    uint32_t* steps = (P.mask & (1u << grt::RF_STEPS)) ? (uint32_t*)field_ptr(B.block, P.mask, n, grt::RF_STEPS)
                                                       : B.steps;
    uint8_t* stop = field_ptr(B.block, P.mask, n, grt::RF_STOP);
    if (n) {
      int rc = grt_render_shard_async(scene, dev, st, &sh, x32, cls, status, x64, steps, stop, (uint64_t*)B.stats);
      if (rc) return rc;
    }
    noted = true;
    C.note_launched();
    if (P.super) {
      // (Y, alpha) and class of every local pixel, then ONE allgather: every device gets
      // the whole frame's neighbourhood records, de-interleaved into frame order
      if (n) {
        const unsigned gx = (unsigned)std::min<uint64_t>((n + 255) / 256, 8192);
        hipLaunchKernelGGL(grt::pack_ya_kernel, dim3(gx), dim3(256), 0, st, x64, cls, n, (double*)B.ag_send,
                           B.ag_send + align256(P.max_local * 16));
        HIP_TRY(hipGetLastError());
      }
      HIP_TRY(hipStreamSynchronize(st));
      if (int rc = comms_ready(C)) return rc;
      if (!barrier()) return fail(-ECANCELED, "another device failed");
      HIP_TRY(hipEventRecord(M.ev[2], st));
      NCCL_TRY(rccl().AllGather(B.ag_send, B.ag_recv, P.ag_bytes, ncclUint8, C.comms[i], st));
      grt::GatherLayout L;
      std::memset(&L, 0, sizeof(L));
      L.cols = P.cols;
      L.band_rows = P.band;
      L.n_shards = P.n_dev;
      L.n_pixels = (uint64_t)P.rows * P.cols;
      L.n_fields = 2;
      L.elem[0] = 16;
      L.elem[1] = 1;
      for (uint32_t s = 0; s < P.n_dev; ++s) {
        L.src[s][0] = s * P.ag_bytes;
        L.src[s][1] = s * P.ag_bytes + align256(P.max_local * 16);
      }
      grt::GatherDst d{};
      d.p[0] = (uint8_t*)B.frame_ya;
      d.p[1] = B.frame_cls;
      if (int rc = launch_deinterleave(L, B.ag_recv, d, st)) return rc;
      HIP_TRY(hipEventRecord(M.ev[3], st));
      // the frame's exact 99th-percentile floor (or the configured minimum), then this
      // device's selection and sub-rays (grt_supersample_shard_device, longest first)
      const bool dev_floor = !cfg->has_minimum_luminance;
      if (dev_floor) {
        int rc = grt_adaptive_floor_device(scene, dev, st, B.frame_ya, 2, L.n_pixels, B.floor);
        if (rc) return rc;
      }
      grt_subsample_failures fl{};
      grt_subsample_failures* flp = nullptr;
      if (want_fail && want_fail->capacity && want_fail->pixel && want_fail->status) {
        const uint64_t cap = want_fail->capacity;
        R.f_pix.resize(cap);
        R.f_smp.resize(cap);
        R.f_status.resize(cap);
        fl.capacity = cap;
        fl.pixel = R.f_pix.data();
        fl.sample = R.f_smp.data();
        fl.status = R.f_status.data();
        if (want_fail->stop) {
          R.f_stop.resize(cap);
          R.f_steps.resize(cap);
          fl.stop = R.f_stop.data();
          fl.steps = R.f_steps.data();
        }
        flp = &fl;
      }
      int rc = grt_host::supersample_shard(scene, dev, st, &sh, cfg, cfg->minimum_luminance,
                                           dev_floor ? B.floor : nullptr, B.frame_ya, B.frame_cls, mask_xyza, x64,
                                           steps, (uint64_t*)(B.stats + 4), (uint64_t*)B.stats, flp);
      if (rc) return rc;
      R.f_count = flp ? fl.count : 0;
    }
    HIP_TRY(hipEventRecord(M.ev[1], st));
    HIP_TRY(hipStreamSynchronize(st));
    // ONE gather: every device sends its block to devices[0] (grouped send / receive;
    // devices[0] sends to itself too, so every frame takes the same RCCL path)
    if (int rc = comms_ready(C)) return rc;
    if (!barrier()) return fail(-ECANCELED, "another device failed");
    HIP_TRY(hipEventRecord(M.ev[4], st));
    NCCL_TRY(rccl().GroupStart());
    NCCL_TRY(rccl().Send(B.block, P.block[i], ncclUint8, 0, C.comms[i], st));
    if (i == 0)
      for (uint32_t s = 0; s < P.n_dev; ++s)
        NCCL_TRY(rccl().Recv(B.gathered + P.block_off[s], P.block[s], ncclUint8, (int)s, C.comms[i], st));
    NCCL_TRY(rccl().GroupEnd());
    if (i == 0) {
      const grt::GatherLayout L = gather_layout(P);
      grt::GatherDst d{};
      const uint64_t F = L.n_pixels;
      for (int f = 0, k = 0; f < grt::RF_N; ++f)
        if (P.mask & (1u << f)) d.p[k++] = B.frame + field_offset(P.mask, F, f);
      if (int rc = launch_deinterleave(L, B.gathered, d, st)) return rc;
    }
    HIP_TRY(hipEventRecord(M.ev[5], st));
    if (i == 0) {  // frame-order fields to the caller
      const uint64_t F = (uint64_t)P.rows * P.cols;
      auto d2h = [&](void* host, int f) -> int {
        if (host && F) HIP_TRY(hipMemcpyAsync(host, B.frame + field_offset(P.mask, F, f), F * grt::rec_field_bytes(f),
                                              hipMemcpyDeviceToHost, st));
        return 0;
      };
      int rc;
      if ((rc = d2h(out->xyza64, grt::RF_XYZA64)) || (rc = d2h(out->xyza, grt::RF_XYZA32)) ||
          (rc = d2h(out->steps, grt::RF_STEPS)) || (rc = d2h(out->ray_class, grt::RF_CLASS)) ||
          (rc = d2h(out->status, grt::RF_STATUS)) || (rc = d2h(out->stop, grt::RF_STOP)))
        return rc;
    }
    HIP_TRY(hipStreamSynchronize(st));
    unsigned long long h[5];
    HIP_TRY(hipMemcpy(h, B.stats, sizeof(h), hipMemcpyDeviceToHost));
    for (int k = 0; k < 4; ++k) R.stats[k] = h[k];
    R.n_sel = h[4];
    HIP_TRY(hipEventElapsedTime(&R.trace_ms, M.ev[0], M.ev[1]));
    if (P.super) HIP_TRY(hipEventElapsedTime(&R.ag_ms, M.ev[2], M.ev[3]));
    HIP_TRY(hipEventElapsedTime(&R.gather_ms, M.ev[4], M.ev[5]));
    return 0;
  };
  R.rc = run();
  if (!noted) C.note_launched();  // failed before its trace: the others must not wait
  if (R.rc) {
    R.err = grt_last_error();
    // the barriers this thread has not reached: the other threads stop there instead of
    // entering a collective this device will not join
    for (; passed < n_barriers; ++passed) bar.arrive(false);
  }
}

}  // namespace

extern "C" {

int grt_render_frame_multi(grt_scene* scene, int n_devices, const int* devices, uint32_t band_rows,
                           const grt_adaptive_config* cfg, const double* sampling_mask_xyza, const grt_frame_out* out,
                           uint64_t* n_supersampled, grt_stats* stats, grt_subsample_failures* failures,
                           grt_multi_report* report) {
  const auto t0 = std::chrono::steady_clock::now();
  if (stats) std::memset(stats, 0, sizeof(*stats));
  if (n_supersampled) *n_supersampled = 0;
  if (failures) failures->count = 0;
  if (!scene || !devices || !out) return fail(-EINVAL, "null argument");
  if (band_rows == 0) return fail(-EINVAL, "band_rows must be >= 1");
  std::vector<int> devs;
  if (int rc = check_devices(n_devices, devices, &devs)) return rc;
  Plan P;
  P.n_dev = (uint32_t)n_devices;
  P.band = band_rows;
  {
    int64_t r = 0, c = 0;
    grt_host::scene_frame_size(scene, &r, &c);
    if (r <= 0 || c <= 0 || r > (int64_t)UINT32_MAX || c > (int64_t)UINT32_MAX)
      return fail(-EINVAL, "camera frame size out of range");
    P.rows = (uint32_t)r;
    P.cols = (uint32_t)c;
  }
  P.super = (cfg && cfg->enabled) || sampling_mask_xyza != nullptr;
  if (P.super) {
    if (!cfg) return fail(-EINVAL, "supersampling needs the adaptive configuration");
    if (cfg->samples_per_axis == 0) return fail(-EINVAL, "adaptive_sampling.samples_per_axis must be greater than zero");
    if (!out->xyza64) return fail(-EINVAL, "a supersampled frame is f64: pass out->xyza64");
    if (out->xyza) return fail(-EINVAL, "a supersampled frame has no f32 XYZA (pass out->xyza = NULL)");
  }
  P.mask = (1u << grt::RF_CLASS) | (1u << grt::RF_STATUS);
  if (out->xyza64 || P.super) P.mask |= 1u << grt::RF_XYZA64;
  if (out->xyza) P.mask |= 1u << grt::RF_XYZA32;
  if (out->steps) P.mask |= 1u << grt::RF_STEPS;
  if (out->stop) P.mask |= 1u << grt::RF_STOP;
  uint64_t off = 0;
  for (uint32_t s = 0; s < P.n_dev; ++s) {
    grt_row_shard sh{band_rows, s, P.n_dev};
    P.n_local[s] = (uint64_t)grt_shard_row_count(P.rows, &sh) * P.cols;
    P.max_local = std::max(P.max_local, P.n_local[s]);
    P.block[s] = field_offset(P.mask, P.n_local[s], grt::RF_N);
    P.block_off[s] = off;
    off += P.block[s];
  }
  P.block_off[P.n_dev] = off;
  P.ag_bytes = align256(P.max_local * 16) + align256(P.max_local);
  if (P.super && (uint64_t)P.rows * P.cols > (uint64_t)INT32_MAX) return fail(-EOVERFLOW, "frame larger than INT_MAX pixels");
  MultiCtx* C;
  if (int rc = get_ctx(devs, &C)) return rc;
  std::lock_guard<std::mutex> lk(C->mu);
  std::vector<DevResult> R;
  uint32_t attempt = 0;
  // a trace that lost hit candidates (a device's hit pool too small) grows that device's
  // pool from the trace's measured need and the frame is traced again, at most 3 times
  for (;;) {
    ++attempt;
    R.assign(P.n_dev, DevResult());
    Barrier bar(n_devices);
    std::vector<std::thread> th;
    for (int i = 1; i < n_devices; ++i)
      th.emplace_back(device_part, scene, std::ref(*C), std::cref(P), i, cfg, sampling_mask_xyza, out, failures,
                      std::ref(bar), std::ref(R[i]));
    device_part(scene, *C, P, 0, cfg, sampling_mask_xyza, out, failures, bar, R[0]);
    for (auto& t : th) t.join();
    {  // no communicator is still being created when this call returns (a frame that
       // failed before its collectives has not waited for them)
      std::shared_future<std::string> f;
      {
        std::lock_guard<std::mutex> l2(C->cm);
        if (C->started) f = C->comm_ready;
      }
      if (f.valid()) (void)f.get();
    }
    for (uint32_t i = 0; i < P.n_dev; ++i)
      if (R[i].rc && R[i].rc != -ECANCELED) return fail(R[i].rc, "device " + std::to_string(devs[i]) + ": " + R[i].err);
    for (uint32_t i = 0; i < P.n_dev; ++i)
      if (R[i].rc) return fail(R[i].rc, R[i].err);
    uint64_t lost = 0;
    for (uint32_t i = 0; i < P.n_dev; ++i) lost += R[i].stats[3];
    if (lost == 0 || attempt == 3) break;
    for (uint32_t i = 0; i < P.n_dev; ++i)
      if (R[i].stats[3])
        if (int rc = grt_hit_pool_reserve(scene, devs[i], 0, nullptr)) return rc;
  }
  uint64_t nsel = 0;
  if (stats) {
    for (uint32_t i = 0; i < P.n_dev; ++i) {
      stats->accepted_steps += R[i].stats[0];
      stats->attempts += R[i].stats[1];
      stats->rays += R[i].stats[2];
      stats->hit_overflows += R[i].stats[3];
      stats->kernel_ms = std::max(stats->kernel_ms, (double)R[i].trace_ms);
    }
  }
  for (uint32_t i = 0; i < P.n_dev; ++i) nsel += R[i].n_sel;
  if (n_supersampled) *n_supersampled = nsel;
  if (failures && failures->capacity && failures->pixel && failures->status) {
    // every device's failed sub-samples (frame pixel indices), sorted by (pixel, sample)
    struct E {
      uint32_t pix, smp, steps;
      uint8_t status, stop;
    };
    std::vector<E> all;
    uint64_t count = 0;
    for (uint32_t i = 0; i < P.n_dev; ++i) {
      count += R[i].f_count;
      const uint64_t m = std::min<uint64_t>(R[i].f_count, R[i].f_pix.size());
      for (uint64_t k = 0; k < m; ++k)
        all.push_back(E{R[i].f_pix[k], R[i].f_smp[k], R[i].f_steps.empty() ? 0u : R[i].f_steps[k], R[i].f_status[k],
                        R[i].f_stop.empty() ? (uint8_t)0 : R[i].f_stop[k]});
    }
    std::sort(all.begin(), all.end(), [](const E& a, const E& b) { return a.pix != b.pix ? a.pix < b.pix : a.smp < b.smp; });
    const uint64_t m = std::min<uint64_t>(all.size(), failures->capacity);
    for (uint64_t k = 0; k < m; ++k) {
      failures->pixel[k] = all[k].pix;
      if (failures->sample) failures->sample[k] = all[k].smp;
      failures->status[k] = all[k].status;
      if (failures->stop) failures->stop[k] = all[k].stop;
      if (failures->steps) failures->steps[k] = all[k].steps;
    }
    failures->count = count;
  }
  if (report) {
    std::memset(report, 0, sizeof(*report));
    report->n_devices = P.n_dev;
    uint32_t rb = 0;
    for (int f = 0; f < grt::RF_N; ++f)
      if (P.mask & (1u << f)) rb += grt::rec_field_bytes(f);
    report->record_bytes = rb;
    report->attempts = attempt;
    report->gather_ms = R[0].gather_ms;
    for (uint32_t i = 0; i < P.n_dev; ++i) {
      report->trace_ms[i] = R[i].trace_ms;
      report->accepted_steps[i] = R[i].stats[0];
      report->rows[i] = P.cols ? P.n_local[i] / P.cols : 0;
      report->allgather_ms = std::max(report->allgather_ms, (double)R[i].ag_ms);
    }
    report->wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  }
  return 0;
}

void grt_multi_release(void) {
  std::lock_guard<std::mutex> lk(g_ctx_mu);
  for (auto& c : g_ctx) {
    std::lock_guard<std::mutex> l2(c->mu);
    const bool have_comms = c->started && c->comm_ready.get().empty();
    for (auto& m : c->d) {
      (void)hipSetDevice(m.device);
      if (m.st) (void)hipStreamSynchronize(m.st);
      if (m.mem) (void)hipFree(m.mem);
      for (auto& e : m.ev)
        if (e) (void)hipEventDestroy(e);
      if (m.st) (void)hipStreamDestroy(m.st);
    }
    if (have_comms)
      for (auto& cm : c->comms) (void)rccl().CommDestroy(cm);
  }
  g_ctx.clear();
}

// Test hook (not in grt_api.h): the de-interleave of deinterleave_kernel run on the host
// with the same per-pixel source function (gather_source), so that a CPU test can hold
// the frame-order assembly of n_shards gathered blocks to distributed.shard_frame_rows.
// gathered: the blocks of shards 0..n-1 back to back, each laid out for `mask`
// (grt_debug_gather_block_bytes); dst[f] (nullable): frame-order output of field f.
int grt_debug_deinterleave_host(uint32_t rows, uint32_t cols, uint32_t band_rows, uint32_t n_shards, uint32_t mask,
                                const uint8_t* gathered, uint8_t* const* dst) {
  if (!gathered || !dst || n_shards == 0 || n_shards > (uint32_t)grt::MULTI_MAX || band_rows == 0 || mask >= 64u)
    return fail(-EINVAL, "deinterleave: bad argument");
  Plan P;
  P.rows = rows;
  P.cols = cols;
  P.band = band_rows;
  P.n_dev = n_shards;
  P.mask = mask;
  uint64_t off = 0;
  for (uint32_t s = 0; s < n_shards; ++s) {
    grt_row_shard sh{band_rows, s, n_shards};
    P.n_local[s] = (uint64_t)grt_shard_row_count(rows, &sh) * cols;
    P.block[s] = field_offset(mask, P.n_local[s], grt::RF_N);
    P.block_off[s] = off;
    off += P.block[s];
  }
  P.block_off[n_shards] = off;
  const grt::GatherLayout L = gather_layout(P);
  for (int f = 0, k = 0; f < grt::RF_N; ++f) {
    if (!(mask & (1u << f))) continue;
    const uint32_t e = L.elem[k];
    if (dst[f])
      for (uint64_t p = 0; p < L.n_pixels; ++p) std::memcpy(dst[f] + p * e, gathered + grt::gather_source(L, k, p), e);
    ++k;
  }
  return 0;
}

// Test hook (not in grt_api.h): bytes of a device's send block of n pixels for `mask`,
// and each field's offset in it (offsets[6], ~0 for a field not in the mask).
uint64_t grt_debug_gather_block_bytes(uint32_t mask, uint64_t n, uint64_t* offsets) {
  for (int f = 0; f < grt::RF_N; ++f)
    if (offsets) offsets[f] = (mask & (1u << f)) ? field_offset(mask, n, f) : ~0ull;
  return field_offset(mask, n, grt::RF_N);
}

}  // extern "C"
