// hshost: the HIP runtime calls of the host engines (hsrestore.cpp,
// hsdrain.cpp) behind a C ABI.  Those engines are plain C++ threads, slot and
// ring bookkeeping around device operations; keeping every HIP call here lets
// them build without HIP against the stubs of tests/native/engine_stubs.cpp,
// where ThreadSanitizer and AddressSanitizer check their concurrency on the
// CPU (GPU sanitizers are not available on the MI355X pool).

#include <hip/hip_runtime.h>
#include <unistd.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <atomic>
#include <mutex>
#include <unordered_map>

namespace {

// The last failed runtime call of these hooks, with HIP's error name: the
// engines' "device work" errors carry it (a bare EIO named nothing).
std::mutex g_rt_mu;
char g_rt_err[200] = {0};

void note(const char* what, hipError_t e) {
  std::lock_guard<std::mutex> g(g_rt_mu);
  snprintf(g_rt_err, sizeof(g_rt_err), "%s: %s (%d)", what, hipGetErrorName(e), int(e));
}

// Pool trace (hsg_rt_set_trace(1), from Python native.set_pool_trace): one
// stderr line per device allocation and free of the engines' pools and per
// restore upload (pid, microseconds, address, bytes, kind), so a failing
// multi-process restore can be laid against which process held which range.
std::atomic<int> g_trace{0};

int trace_on() { return g_trace.load(std::memory_order_relaxed); }

uint64_t now_us() {
  return static_cast<uint64_t>(std::chrono::duration_cast<std::chrono::microseconds>(
      std::chrono::steady_clock::now().time_since_epoch()).count());
}

}  // namespace

extern "C" {

const char* hsg_rt_last_error() { return g_rt_err; }

int hsg_rt_trace_on() { return trace_on(); }

void hsg_rt_set_trace(int on) { g_trace.store(on ? 1 : 0); }

void hsg_rt_trace(const char* what, const void* p, uint64_t n, int kind) {
  if (!trace_on()) return;
  fprintf(stderr, "[hs-pool] pid=%d t=%llu %s p=%p n=%llu kind=%d\n", int(getpid()),
          (unsigned long long)now_us(), what, p, (unsigned long long)n, kind);
}

int hsg_rt_set_device(int dev) { return hipSetDevice(dev) == hipSuccess ? 0 : -1; }

// `nbytes` of device memory on `dev`: device-uncached (hipDeviceMallocUncached:
// SDMA upload targets the kernels read without an acquire) or plain.  Null on
// failure (the error is cleared: callers trim their pools and retry).
void* hsg_rt_dev_alloc(int dev, uint64_t nbytes, int uncached) {
  if (hipSetDevice(dev) != hipSuccess) return nullptr;
  void* p = nullptr;
  const hipError_t e = uncached ? hipExtMallocWithFlags(&p, nbytes, hipDeviceMallocUncached)
                                : hipMalloc(&p, nbytes);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  hsg_rt_trace("alloc", p, nbytes, uncached);
  return p;
}

void hsg_rt_dev_free(void* p) {
  if (!p) return;
  hsg_rt_trace("free", p, 0, -1);
  const hipError_t e = hipFree(p);
  if (e != hipSuccess) {
    note("hipFree", e);
    (void)hipGetLastError();
  }
}

// ---- device memory at addresses that are never handed out twice -----------
//
// A process that hipFree's both uncached and plain device memory is NOT safe
// on this pool: the blocks it allocates next are used by its kernels through
// stale translations -- writes land in, reads come from, physical memory the
// driver has meanwhile given to another allocation or another process, while
// SDMA copies see the new mapping (scripts/probes/pool_churn_mp.py: 466 of 600
// iterations wrong in one process; profiles/r6/trim/).  The engines' freeable
// blocks come from the virtual memory API instead: each gets a virtual range
// reserved for it alone; freeing unmaps and releases the physical memory
// (other processes and torch may use it at once) but keeps the range
// reserved, so no later mapping of this process ever reuses it.  With these
// blocks the same churn ran 0 wrong in 4 and 8 processes.  The leaked
// reservations cost virtual address space only.
namespace {
struct VmmBlock {
  hipMemGenericAllocationHandle_t handle;
  size_t size;
};
std::mutex g_vmm_mu;
std::unordered_map<void*, VmmBlock> g_vmm;
std::atomic<uint64_t> g_vmm_retired{0};  // bytes of virtual ranges kept reserved
}  // namespace

void* hsg_rt_vmm_alloc(int dev, uint64_t nbytes, int uncached) {
  if (hipSetDevice(dev) != hipSuccess) return nullptr;
  hipMemAllocationProp prop = {};
  prop.type = uncached ? hipMemAllocationTypeUncached : hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = dev;
  size_t gran = 0;
  hipError_t e = hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityMinimum);
  if (e != hipSuccess || gran == 0) gran = size_t(2) << 20;
  const size_t size = (std::max<uint64_t>(nbytes, 1) + gran - 1) / gran * gran;
  hipMemGenericAllocationHandle_t h{};
  e = hipMemCreate(&h, size, &prop, 0);
  if (e != hipSuccess) {
    note("hipMemCreate", e);
    (void)hipGetLastError();
    return nullptr;
  }
  void* p = nullptr;
  e = hipMemAddressReserve(&p, size, gran, nullptr, 0);
  if (e == hipSuccess) {
    e = hipMemMap(p, size, 0, h, 0);
    if (e == hipSuccess) {
      hipMemAccessDesc acc = {};
      acc.location.type = hipMemLocationTypeDevice;
      acc.location.id = dev;
      acc.flags = hipMemAccessFlagsProtReadWrite;
      e = hipMemSetAccess(p, size, &acc, 1);
      if (e != hipSuccess) (void)hipMemUnmap(p, size);
    }
    if (e != hipSuccess) (void)hipMemAddressFree(p, size);  // never mapped: safe to return
  }
  if (e != hipSuccess) {
    note("hipMemMap", e);
    (void)hipGetLastError();
    (void)hipMemRelease(h);
    return nullptr;
  }
  {
    std::lock_guard<std::mutex> g(g_vmm_mu);
    g_vmm[p] = VmmBlock{h, size};
  }
  hsg_rt_trace("vmm-alloc", p, size, uncached);
  return p;
}

// Unmap and release the block's memory; its virtual range stays reserved.
// The caller has finished every use (kernels, SDMA) of it.  Returns -1 if `p`
// is not a block of hsg_rt_vmm_alloc.
int hsg_rt_vmm_free(void* p) {
  VmmBlock b{};
  {
    std::lock_guard<std::mutex> g(g_vmm_mu);
    auto it = g_vmm.find(p);
    if (it == g_vmm.end()) return -1;
    b = it->second;
    g_vmm.erase(it);
  }
  hsg_rt_trace("vmm-free", p, b.size, -1);
  // nothing of this process may still be reading or writing it
  hipError_t e = hipDeviceSynchronize();
  if (e == hipSuccess) e = hipMemUnmap(p, b.size);
  if (e == hipSuccess) e = hipMemRelease(b.handle);
  if (e != hipSuccess) {
    note("hipMemUnmap", e);
    (void)hipGetLastError();
    return -2;
  }
  g_vmm_retired.fetch_add(b.size);
  return 0;
}

uint64_t hsg_rt_vmm_retired_bytes() { return g_vmm_retired.load(); }

// A new event recorded on `stream` (null on failure).
void* hsg_rt_event_record(void* stream) {
  hipEvent_t ev = nullptr;
  if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  if (hipEventRecord(ev, static_cast<hipStream_t>(stream)) != hipSuccess) {
    (void)hipGetLastError();
    (void)hipEventDestroy(ev);
    return nullptr;
  }
  return ev;
}

int hsg_rt_event_sync(void* ev) {
  const hipError_t e = hipEventSynchronize(static_cast<hipEvent_t>(ev));
  if (e == hipSuccess) return 0;
  note("hipEventSynchronize", e);
  return -1;
}

void hsg_rt_event_free(void* ev) {
  if (ev) (void)hipEventDestroy(static_cast<hipEvent_t>(ev));
}

// Work queued on `waiter` from now on runs after everything already queued on
// `producer`.
int hsg_rt_stream_after(void* waiter, void* producer) {
  void* ev = hsg_rt_event_record(producer);
  if (!ev) return -1;
  const hipError_t e =
      hipStreamWaitEvent(static_cast<hipStream_t>(waiter), static_cast<hipEvent_t>(ev), 0);
  hsg_rt_event_free(ev);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return -1;
  }
  return 0;
}

int hsg_rt_stream_sync(void* stream) {
  const hipError_t e = hipStreamSynchronize(static_cast<hipStream_t>(stream));
  if (e == hipSuccess) return 0;
  note("hipStreamSynchronize", e);
  return -1;
}

// Blocking device -> host copy of n bytes (small result arrays).
int hsg_rt_memcpy_d2h(void* dst, const void* src, uint64_t n) {
  if (hipMemcpy(dst, src, n, hipMemcpyDeviceToHost) != hipSuccess) {
    (void)hipGetLastError();
    return -1;
  }
  return 0;
}

}  // extern "C"
