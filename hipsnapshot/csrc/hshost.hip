// hshost: the HIP runtime calls of the host engines (hsrestore.cpp,
// hsdrain.cpp) behind a C ABI.  Those engines are plain C++ threads, slot and
// ring bookkeeping around device operations; keeping every HIP call here lets
// them build without HIP against the stubs of tests/native/engine_stubs.cpp,
// where ThreadSanitizer and AddressSanitizer check their concurrency on the
// CPU (GPU sanitizers are not available on the MI355X pool).

#include <hip/hip_runtime.h>

#include <cstdint>

extern "C" {

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
  return p;
}

void hsg_rt_dev_free(void* p) {
  if (p) (void)hipFree(p);
}

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
  return hipEventSynchronize(static_cast<hipEvent_t>(ev)) == hipSuccess ? 0 : -1;
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
  return hipStreamSynchronize(static_cast<hipStream_t>(stream)) == hipSuccess ? 0 : -1;
}

// Register / unregister host memory (a file mapping: csrc/hsfmap.cpp) so the
// SDMA engines can write it.
int hsg_rt_host_register(void* p, uint64_t n) {
  if (hipHostRegister(p, n, hipHostRegisterDefault) != hipSuccess) {
    (void)hipGetLastError();
    return -1;
  }
  return 0;
}

int hsg_rt_host_unregister(void* p) {
  if (hipHostUnregister(p) != hipSuccess) {
    (void)hipGetLastError();
    return -1;
  }
  return 0;
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
