// SDMA copies between HBM and pinned host memory, issued through ROCr.
//
// hipMemcpyAsync(DeviceToHost) into pinned memory runs as the runtime's
// `__amd_rocclr_copyBuffer` blit KERNEL on this ROCm (rocprofv3 kernel trace,
// profiles/dma/): it occupies CUs and floods the L2 -> fabric queues with
// host-bound writes for the whole drain, which is what a training step running
// next to an async snapshot pays for.  The copy engines (SDMA) move the same
// bytes without touching the CUs.  ROCr exposes them through
// hsa_amd_memory_async_copy[_on_engine]; HIP does not, so this file binds the
// already-loaded libhsa-runtime64 at run time (dlopen NOLOAD + dlsym: no link
// dependency, and the one ROCr instance torch's HIP runtime uses).
//
// Ordering: the caller has synchronised the producer (the bytes are final);
// before reading HBM the SDMA engine must see them at system scope, so a
// hipEventReleaseToSystem event is recorded and waited on the copy stream
// first (writes back dirty L2 lines).  Host -> device copies (restores) go
// only into uncached device memory, which no L2 line can shadow, so the
// kernels that read them need no system-scope acquire (see the end of this
// file).
//
// By default a copy is one request on the engine ROCr assigns; optionally it
// is split into pieces over the engines ROCr reports as free for the GPU ->
// CPU direction, each piece on its own completion signal.  The call returns
// when all pieces are done (or reports the first failure).

#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <mutex>
#include <vector>

namespace {

struct HsaApi {
  decltype(&hsa_iterate_agents) iterate_agents = nullptr;
  decltype(&hsa_agent_get_info) agent_get_info = nullptr;
  decltype(&hsa_signal_create) signal_create = nullptr;
  decltype(&hsa_signal_destroy) signal_destroy = nullptr;
  decltype(&hsa_signal_store_screlease) signal_store = nullptr;
  decltype(&hsa_signal_wait_scacquire) signal_wait = nullptr;
  decltype(&hsa_amd_memory_async_copy) async_copy = nullptr;
  decltype(&hsa_amd_memory_async_copy_on_engine) async_copy_on_engine = nullptr;
  decltype(&hsa_amd_memory_copy_engine_status) engine_status = nullptr;
  bool ok = false;
};

struct DevInfo {
  hsa_agent_t gpu{0};
  hsa_agent_t cpu{0};
  uint32_t engines = 0;  // free SDMA engine mask for GPU -> CPU copies
  uint32_t h2d_engines = 0;  // ... and for CPU -> GPU copies
  bool ok = false;
};

std::once_flag g_once;
HsaApi g_api;
std::mutex g_mu;
std::vector<DevInfo> g_devs;
char g_err[256];

template <typename F>
bool bind(void* h, const char* name, F* out) {
  *out = reinterpret_cast<F>(dlsym(h, name));
  return *out != nullptr;
}

void load_api() {
  void* h = dlopen("libhsa-runtime64.so.1", RTLD_NOW | RTLD_NOLOAD);
  if (!h) h = dlopen("libhsa-runtime64.so", RTLD_NOW | RTLD_NOLOAD);
  if (!h) {
    snprintf(g_err, sizeof(g_err), "libhsa-runtime64 is not loaded in this process");
    return;
  }
  HsaApi a;
  a.ok = bind(h, "hsa_iterate_agents", &a.iterate_agents) &&
         bind(h, "hsa_agent_get_info", &a.agent_get_info) &&
         bind(h, "hsa_signal_create", &a.signal_create) &&
         bind(h, "hsa_signal_destroy", &a.signal_destroy) &&
         bind(h, "hsa_signal_store_screlease", &a.signal_store) &&
         bind(h, "hsa_signal_wait_scacquire", &a.signal_wait) &&
         bind(h, "hsa_amd_memory_async_copy", &a.async_copy) &&
         bind(h, "hsa_amd_memory_async_copy_on_engine", &a.async_copy_on_engine) &&
         bind(h, "hsa_amd_memory_copy_engine_status", &a.engine_status);
  if (!a.ok) snprintf(g_err, sizeof(g_err), "libhsa-runtime64 lacks the async copy API");
  g_api = a;
}

struct AgentScan {
  std::vector<hsa_agent_t> gpus;
  std::vector<hsa_agent_t> cpus;
};

hsa_status_t scan_agent(hsa_agent_t a, void* data) {
  auto* s = static_cast<AgentScan*>(data);
  hsa_device_type_t t;
  if (g_api.agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS)
    return HSA_STATUS_SUCCESS;
  if (t == HSA_DEVICE_TYPE_GPU) s->gpus.push_back(a);
  if (t == HSA_DEVICE_TYPE_CPU) s->cpus.push_back(a);
  return HSA_STATUS_SUCCESS;
}

// The HSA agent of HIP device `dev`, matched by PCI bus/device (HIP may hide
// devices through HIP_VISIBLE_DEVICES, so the indices need not agree).
DevInfo* dev_info(int dev) {
  std::call_once(g_once, load_api);
  if (!g_api.ok) return nullptr;
  std::lock_guard<std::mutex> g(g_mu);
  if (dev < 0) return nullptr;
  if (int(g_devs.size()) <= dev) g_devs.resize(dev + 1);
  DevInfo& d = g_devs[dev];
  if (d.ok) return &d;
  int bus = -1, devno = -1, dom = -1;
  if (hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, dev) != hipSuccess ||
      hipDeviceGetAttribute(&devno, hipDeviceAttributePciDeviceId, dev) != hipSuccess ||
      hipDeviceGetAttribute(&dom, hipDeviceAttributePciDomainId, dev) != hipSuccess) {
    snprintf(g_err, sizeof(g_err), "hipDeviceGetAttribute(PCI) failed for device %d", dev);
    return nullptr;
  }
  AgentScan scan;
  g_api.iterate_agents(scan_agent, &scan);
  if (scan.cpus.empty()) {
    snprintf(g_err, sizeof(g_err), "no HSA CPU agent");
    return nullptr;
  }
  for (hsa_agent_t a : scan.gpus) {
    uint32_t bdf = 0, adom = 0;
    if (g_api.agent_get_info(a, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_BDFID), &bdf) !=
        HSA_STATUS_SUCCESS)
      continue;
    if (g_api.agent_get_info(a, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_DOMAIN),
                             &adom) != HSA_STATUS_SUCCESS)
      adom = uint32_t(dom);
    if (int((bdf >> 8) & 0xff) == bus && int((bdf >> 3) & 0x1f) == devno && int(adom) == dom) {
      d.gpu = a;
      d.cpu = scan.cpus[0];
      uint32_t mask = 0;
      if (g_api.engine_status(d.cpu, d.gpu, &mask) != HSA_STATUS_SUCCESS) mask = 0;
      d.engines = mask;
      mask = 0;
      if (g_api.engine_status(d.gpu, d.cpu, &mask) != HSA_STATUS_SUCCESS) mask = 0;
      d.h2d_engines = mask;
      d.ok = true;
      return &d;
    }
  }
  snprintf(g_err, sizeof(g_err), "no HSA GPU agent matches HIP device %d (bus %d dev %d)", dev,
           bus, devno);
  return nullptr;
}

thread_local std::vector<hsa_signal_t> t_signals;

hsa_signal_t take_signal() {
  if (!t_signals.empty()) {
    hsa_signal_t s = t_signals.back();
    t_signals.pop_back();
    return s;
  }
  hsa_signal_t s{0};
  if (g_api.signal_create(1, 0, nullptr, &s) != HSA_STATUS_SUCCESS) s.handle = 0;
  return s;
}

void give_signal(hsa_signal_t s) {
  if (t_signals.size() < 16) t_signals.push_back(s);
  else g_api.signal_destroy(s);
}

}  // namespace

extern "C" {

const char* hsg_sdma_last_error() { return g_err; }

// Number of SDMA engines usable for device -> host copies of `dev` (0: the
// SDMA path is unavailable; callers use hipMemcpyAsync).
int hsg_sdma_engines(int dev) {
  DevInfo* d = dev_info(dev);
  if (!d) return 0;
  return __builtin_popcount(d->engines);
}

// Blocking device -> pinned-host copy of n bytes on the SDMA engines
// (`max_engines` 0 = one request on the engine ROCr assigns).  `stream` =
// the HIP stream whose queued work produced `src` (the copy is ordered
// after it).  Returns 0, or < 0 on failure (nothing is left
// in flight on failure: every issued piece is waited for).
int hsg_sdma_d2h(int dev, void* dst, const void* src, uint64_t n, int max_engines, void* stream) {
  DevInfo* d = dev_info(dev);
  if (!d) return -1;
  if (n == 0) return 0;
  hipError_t e = hipSetDevice(dev);
  if (e != hipSuccess) return -2;
  {
    // producer work done AND written back to system scope before SDMA reads
    hipEvent_t ev;
    if (hipEventCreateWithFlags(&ev, hipEventDisableTiming | hipEventReleaseToSystem) !=
        hipSuccess)
      return -3;
    e = hipEventRecord(ev, static_cast<hipStream_t>(stream));
    if (e == hipSuccess) e = hipEventSynchronize(ev);
    hipEventDestroy(ev);
    if (e != hipSuccess) {
      snprintf(g_err, sizeof(g_err), "release event: %s", hipGetErrorString(e));
      return -4;
    }
  }
  // max_engines 0: one request, ROCr picks the engine (it spreads concurrent
  // requests from several staging threads over its engines and never
  // conflicts with copies the HIP runtime issues itself); > 0: split over
  // that many explicitly chosen free engines
  std::vector<int> engines;
  if (max_engines > 0)
    for (int b = 0; b < 32; ++b)
      if (d->engines & (1u << b)) engines.push_back(b);
  int k = int(engines.size());
  if (k > max_engines) k = max_engines;
  // pieces >= 64 MiB: fewer, larger DMA requests per engine
  const uint64_t min_piece = 64ull << 20;
  if (k > 1 && n / uint64_t(k) < min_piece) k = int(std::max<uint64_t>(1, n / min_piece));
  std::vector<hsa_signal_t> sigs;
  int rc = 0;
  const uint64_t step = (n + uint64_t(std::max(k, 1)) - 1) / uint64_t(std::max(k, 1));
  for (int i = 0; i < std::max(k, 1); ++i) {
    const uint64_t off = uint64_t(i) * step;
    if (off >= n) break;
    const uint64_t len = std::min(step, n - off);
    hsa_signal_t s = take_signal();
    if (s.handle == 0) {
      rc = -5;
      break;
    }
    g_api.signal_store(s, 1);
    hsa_status_t st;
    char* dp = static_cast<char*>(dst) + off;
    const char* sp = static_cast<const char*>(src) + off;
    if (k >= 1 && !engines.empty())
      st = g_api.async_copy_on_engine(dp, d->cpu, sp, d->gpu, len, 0, nullptr, s,
                                      static_cast<hsa_amd_sdma_engine_id_t>(1u << engines[i]),
                                      true);
    else
      st = g_api.async_copy(dp, d->cpu, sp, d->gpu, len, 0, nullptr, s);
    if (st != HSA_STATUS_SUCCESS) {
      give_signal(s);
      snprintf(g_err, sizeof(g_err), "hsa_amd_memory_async_copy: status 0x%x", unsigned(st));
      rc = -6;
      break;
    }
    sigs.push_back(s);
  }
  for (hsa_signal_t s : sigs) {
    const hsa_signal_value_t v =
        g_api.signal_wait(s, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_BLOCKED);
    if (v < 0 && rc == 0) {
      snprintf(g_err, sizeof(g_err), "SDMA copy reported an error (%ld)", long(v));
      rc = -7;
    }
    give_signal(s);
  }
  return rc;
}

// Asynchronous form of hsg_sdma_d2h with one request: orders the copy after
// `stream` (system-scope release, as above), submits it and returns at once
// with *handle naming its completion signal.  The caller must pass the
// handle to hsg_sdma_wait exactly once (the source and destination must stay
// valid until then).  Staging workers submit a blob's copy and go on to
// encode the next one while the engine works through its queue.
int hsg_sdma_d2h_submit(int dev, void* dst, const void* src, uint64_t n, void* stream,
                        uint64_t* handle) {
  *handle = 0;
  DevInfo* d = dev_info(dev);
  if (!d) return -1;
  if (n == 0) return 0;
  hipError_t e = hipSetDevice(dev);
  if (e != hipSuccess) return -2;
  {
    hipEvent_t ev;
    if (hipEventCreateWithFlags(&ev, hipEventDisableTiming | hipEventReleaseToSystem) !=
        hipSuccess)
      return -3;
    e = hipEventRecord(ev, static_cast<hipStream_t>(stream));
    if (e == hipSuccess) e = hipEventSynchronize(ev);
    hipEventDestroy(ev);
    if (e != hipSuccess) {
      snprintf(g_err, sizeof(g_err), "release event: %s", hipGetErrorString(e));
      return -4;
    }
  }
  hsa_signal_t s = take_signal();
  if (s.handle == 0) return -5;
  g_api.signal_store(s, 1);
  const hsa_status_t st = g_api.async_copy(dst, d->cpu, src, d->gpu, n, 0, nullptr, s);
  if (st != HSA_STATUS_SUCCESS) {
    give_signal(s);
    snprintf(g_err, sizeof(g_err), "hsa_amd_memory_async_copy: status 0x%x", unsigned(st));
    return -6;
  }
  *handle = s.handle;
  return 0;
}

// One system-scope release on `stream` (writes back the L2s), for a caller
// that then submits many copies of memory nothing writes any more: the
// async-take drain of a frozen arena.  Per-copy release events (above) cost
// an event create/record/sync/destroy each -- ~1.3 ms per 32 MiB chunk when
// the trainer's launches contend for the same runtime (profiles/r3/s2/overlap).
int hsg_sdma_release(int dev, void* stream) {
  if (hipSetDevice(dev) != hipSuccess) return -2;
  hipEvent_t ev;
  if (hipEventCreateWithFlags(&ev, hipEventDisableTiming | hipEventReleaseToSystem) != hipSuccess)
    return -3;
  hipError_t e = hipEventRecord(ev, static_cast<hipStream_t>(stream));
  if (e == hipSuccess) e = hipEventSynchronize(ev);
  hipEventDestroy(ev);
  if (e != hipSuccess) {
    snprintf(g_err, sizeof(g_err), "release event: %s", hipGetErrorString(e));
    return -4;
  }
  return 0;
}

// hsg_sdma_d2h_submit without the per-copy release (after hsg_sdma_release).
int hsg_sdma_d2h_submit_released(int dev, void* dst, const void* src, uint64_t n,
                                 uint64_t* handle) {
  *handle = 0;
  DevInfo* d = dev_info(dev);
  if (!d) return -1;
  if (n == 0) return 0;
  hsa_signal_t s = take_signal();
  if (s.handle == 0) return -5;
  g_api.signal_store(s, 1);
  const hsa_status_t st = g_api.async_copy(dst, d->cpu, src, d->gpu, n, 0, nullptr, s);
  if (st != HSA_STATUS_SUCCESS) {
    give_signal(s);
    snprintf(g_err, sizeof(g_err), "hsa_amd_memory_async_copy: status 0x%x", unsigned(st));
    return -6;
  }
  *handle = s.handle;
  return 0;
}

// ---- host -> device into uncached device memory -----------------------------
//
// hipMemcpyAsync(HostToDevice) calls issued by several restore threads block
// inside the HIP runtime for milliseconds each before the copy is submitted
// (rocprofv3 --hip-runtime-trace, profiles/r4/restore_trace/): the PCIe link
// idles meanwhile.  The SDMA engines take the same copy through ROCr with no
// such stall.  An SDMA write into HBM is not ordered with the GPU's L2, so the
// destination is memory the GPU never caches (hipDeviceMallocUncached): no L2
// line of it can be stale when a kernel reads it after the copy, and no
// system-scope acquire is needed.  The restore uploads encoded HSZ1 frames
// there; the decode kernel reads them once.

// Blocking pinned-host -> device copy of n bytes on an SDMA engine.  `dst`
// must be uncached device memory (hsg_uncached_acquire); `src` pinned.
int hsg_sdma_h2d(int dev, void* dst, const void* src, uint64_t n) {
  DevInfo* d = dev_info(dev);
  if (!d) return -1;
  if (n == 0) return 0;
  hsa_signal_t s = take_signal();
  if (s.handle == 0) return -5;
  g_api.signal_store(s, 1);
  const hsa_status_t st = g_api.async_copy(dst, d->gpu, src, d->cpu, n, 0, nullptr, s);
  if (st != HSA_STATUS_SUCCESS) {
    give_signal(s);
    snprintf(g_err, sizeof(g_err), "hsa_amd_memory_async_copy (h2d): status 0x%x", unsigned(st));
    return -6;
  }
  const hsa_signal_value_t v =
      g_api.signal_wait(s, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_BLOCKED);
  give_signal(s);
  if (v < 0) {
    snprintf(g_err, sizeof(g_err), "SDMA h2d copy reported an error (%ld)", long(v));
    return -7;
  }
  return 0;
}

// Asynchronous hsg_sdma_h2d: submits the copy and returns at once with
// *handle naming its completion signal (pass it to hsg_sdma_wait exactly
// once; `src` and `dst` stay valid until then).  The native restore keeps
// several uploads queued so the link never idles between them.
int hsg_sdma_h2d_submit_on(int dev, void* dst, const void* src, uint64_t n, int engine,
                           uint64_t* handle);

int hsg_sdma_h2d_submit(int dev, void* dst, const void* src, uint64_t n, uint64_t* handle) {
  return hsg_sdma_h2d_submit_on(dev, dst, src, n, -1, handle);
}

// Free SDMA engines for host -> device copies of `dev` (bit mask).
uint32_t hsg_sdma_h2d_engine_mask(int dev) {
  DevInfo* d = dev_info(dev);
  return d ? d->h2d_engines : 0;
}

// hsg_sdma_h2d_submit on SDMA engine `engine` (-1: the one ROCr picks).
int hsg_sdma_h2d_submit_on(int dev, void* dst, const void* src, uint64_t n, int engine,
                           uint64_t* handle) {
  *handle = 0;
  DevInfo* d = dev_info(dev);
  if (!d) return -1;
  if (n == 0) return 0;
  hsa_signal_t s = take_signal();
  if (s.handle == 0) return -5;
  g_api.signal_store(s, 1);
  const hsa_status_t st =
      engine >= 0 ? g_api.async_copy_on_engine(dst, d->gpu, src, d->cpu, n, 0, nullptr, s,
                                               static_cast<hsa_amd_sdma_engine_id_t>(1u << engine),
                                               true)
                  : g_api.async_copy(dst, d->gpu, src, d->cpu, n, 0, nullptr, s);
  if (st != HSA_STATUS_SUCCESS) {
    give_signal(s);
    snprintf(g_err, sizeof(g_err), "hsa_amd_memory_async_copy (h2d): status 0x%x", unsigned(st));
    return -6;
  }
  *handle = s.handle;
  return 0;
}

// Wait for a copy submitted by hsg_sdma_d2h_submit; 0 = done, < 0 = the
// engine reported an error (the copy did not complete).  handle 0: no-op.
int hsg_sdma_wait(uint64_t handle) {
  if (handle == 0) return 0;
  hsa_signal_t s;
  s.handle = handle;
  const hsa_signal_value_t v =
      g_api.signal_wait(s, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_BLOCKED);
  give_signal(s);
  if (v < 0) {
    snprintf(g_err, sizeof(g_err), "SDMA copy reported an error (%ld)", long(v));
    return -7;
  }
  return 0;
}

}  // extern "C"
