// CPU stand-ins for every device hook the host engines (hipsnapshot/csrc/
// hsrestore.cpp, hsdrain.cpp) call, so those engines run under ThreadSanitizer
// and AddressSanitizer without a GPU (tests/test_native_sanitizers.py).
//
// The stubs keep the asynchrony the engines must cope with:
//   * streams are worker threads running their queue in order; events are
//     markers on them; hsg_rt_stream_after makes one stream wait for another;
//   * SDMA copies run on two "engine" threads after a random delay and are
//     waited for by handle;
//   * decode / copy launches run on their stream; a copy launch stamps its
//     pinned stage and device workspace with a tag at launch and checks the
//     tags when it runs -- a range handed to another launch before this one
//     ran (a ring reused too early) is reported as corruption;
//   * injected failures: every Nth upload / device-to-host copy fails, and
//     device allocations fail above a byte cap.

#include "engine_stubs.h"

#include <sys/mman.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <random>
#include <thread>
#include <unordered_map>
#include <vector>

namespace stub {

std::atomic<int> fail_upload_every{0};
std::atomic<int> fail_d2h_every{0};
std::atomic<uint64_t> dev_cap{UINT64_MAX};
std::atomic<uint64_t> dev_live{0};
std::atomic<int> pinned_live{0};
std::atomic<int> corruption{0};
std::atomic<int> max_delay_us{200};

namespace {

std::atomic<uint64_t> g_uploads{0}, g_d2h{0};

void jitter() {
  thread_local std::mt19937 rng(
      static_cast<unsigned>(std::hash<std::thread::id>()(std::this_thread::get_id())));
  const int m = max_delay_us.load();
  if (m <= 0) return;
  const int us = int(rng() % unsigned(m));
  if (us < m / 2)
    std::this_thread::yield();
  else
    std::this_thread::sleep_for(std::chrono::microseconds(us));
}

// An in-order work queue on its own thread (a HIP stream / an SDMA engine).
struct Queue {
  std::mutex mu;
  std::condition_variable cv;
  std::deque<std::function<void()>> q;
  uint64_t pushed = 0, finished = 0;
  bool stop = false;
  std::thread th;

  Queue() : th([this] { run(); }) {}
  ~Queue() {
    {
      std::lock_guard<std::mutex> g(mu);
      stop = true;
    }
    cv.notify_all();
    th.join();
  }
  void run() {
    for (;;) {
      std::function<void()> f;
      {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return stop || !q.empty(); });
        if (q.empty()) return;
        f = std::move(q.front());
        q.pop_front();
      }
      jitter();
      f();
      {
        std::lock_guard<std::mutex> g(mu);
        ++finished;
      }
      cv.notify_all();
    }
  }
  void push(std::function<void()> f) {
    {
      std::lock_guard<std::mutex> g(mu);
      q.push_back(std::move(f));
      ++pushed;
    }
    cv.notify_all();
  }
  void sync() {
    std::unique_lock<std::mutex> lk(mu);
    const uint64_t want = pushed;
    cv.wait(lk, [&] { return finished >= want; });
  }
};

struct Flag {
  std::mutex mu;
  std::condition_variable cv;
  bool done = false;
  int rc = 0;
  uint64_t value = 0;
  void set(int r, uint64_t v = 0) {
    {
      std::lock_guard<std::mutex> g(mu);
      done = true;
      rc = r;
      value = v;
    }
    cv.notify_all();
  }
  void wait() {
    std::unique_lock<std::mutex> lk(mu);
    cv.wait(lk, [&] { return done; });
  }
};

std::mutex g_mu;
std::map<int, std::unique_ptr<Queue>>* g_streams = nullptr;
std::unique_ptr<Queue>* g_engines = nullptr;  // two SDMA engines
std::unordered_map<uint64_t, std::shared_ptr<Flag>>* g_handles = nullptr;
std::unordered_map<void*, uint64_t>* g_dev_sizes = nullptr;
uint64_t g_next_handle = 1;

void ensure() {
  if (g_streams) return;
  g_streams = new std::map<int, std::unique_ptr<Queue>>();
  g_engines = new std::unique_ptr<Queue>[2];
  g_engines[0].reset(new Queue());
  g_engines[1].reset(new Queue());
  g_handles = new std::unordered_map<uint64_t, std::shared_ptr<Flag>>();
  g_dev_sizes = new std::unordered_map<void*, uint64_t>();
}

Queue* stream_of(void* s) { return static_cast<Queue*>(s); }

uint64_t new_handle(std::shared_ptr<Flag> f) {
  std::lock_guard<std::mutex> g(g_mu);
  ensure();
  const uint64_t h = g_next_handle++;
  (*g_handles)[h] = std::move(f);
  return h;
}

std::shared_ptr<Flag> take_handle(uint64_t h) {
  std::lock_guard<std::mutex> g(g_mu);
  ensure();
  auto it = g_handles->find(h);
  if (it == g_handles->end()) return nullptr;
  auto f = it->second;
  g_handles->erase(it);
  return f;
}

int copy_async(void* dst, const void* src, uint64_t n, bool fail) {
  (void)dst;
  auto f = std::make_shared<Flag>();
  const uint64_t h = new_handle(f);
  Queue* e;
  {
    std::lock_guard<std::mutex> g(g_mu);
    e = g_engines[h & 1].get();
  }
  e->push([=] {
    if (!fail) memcpy(dst, src, n);
    f->set(fail ? -1 : 0);
  });
  return int(h);  // caller stores it
}

// a stamp that identifies one launch
std::atomic<uint32_t> g_tag{1};

uint64_t fnv(const uint8_t* p, uint64_t n) {
  uint64_t h = 1469598103934665603ull;
  for (uint64_t i = 0; i < n; ++i) h = (h ^ p[i]) * 1099511628211ull;
  return h;
}

}  // namespace

uint64_t hash_bytes(const void* p, uint64_t n) { return fnv(static_cast<const uint8_t*>(p), n); }

void shutdown() {
  std::map<int, std::unique_ptr<Queue>>* s;
  std::unique_ptr<Queue>* e;
  {
    std::lock_guard<std::mutex> g(g_mu);
    s = g_streams;
    e = g_engines;
    g_streams = nullptr;
    g_engines = nullptr;
    delete g_handles;
    g_handles = nullptr;
    delete g_dev_sizes;
    g_dev_sizes = nullptr;
  }
  delete s;
  delete[] e;
}

void* new_stream() {
  std::lock_guard<std::mutex> g(g_mu);
  ensure();
  const int key = -1 - int(g_streams->size());
  auto& q = (*g_streams)[key];
  q.reset(new Queue());
  return q.get();
}

}  // namespace stub

using namespace stub;

extern "C" {

// ---- HIP runtime hooks (hshost.hip) -------------------------------------------

int hsg_rt_set_device(int dev) { return dev == 0 ? 0 : -1; }

const char* hsg_rt_last_error() { return "stub"; }

void hsg_rt_trace(const char* what, const void* p, uint64_t n, int kind) {
  (void)what;
  (void)p;
  (void)n;
  (void)kind;
}

void* hsg_rt_dev_alloc(int dev, uint64_t nbytes, int uncached) {
  (void)dev;
  (void)uncached;
  if (dev_live.load() + nbytes > dev_cap.load()) return nullptr;
  void* p = aligned_alloc(4096, (nbytes + 4095) / 4096 * 4096);
  if (!p) return nullptr;
  dev_live.fetch_add(nbytes);
  std::lock_guard<std::mutex> g(g_mu);
  ensure();
  (*g_dev_sizes)[p] = nbytes;
  return p;
}

void hsg_rt_dev_free(void* p) {
  if (!p) return;
  {
    std::lock_guard<std::mutex> g(g_mu);
    ensure();
    auto it = g_dev_sizes->find(p);
    if (it != g_dev_sizes->end()) {
      dev_live.fetch_sub(it->second);
      g_dev_sizes->erase(it);
    }
  }
  free(p);
}

// The engines' pools allocate through the VMM hooks (hshost.hip), whose
// promise is that a freed block's address range is never handed out again.
// The stand-in keeps it: blocks are anonymous mappings, and a free replaces
// the range with an inaccessible reservation -- the memory goes back, the
// addresses stay taken, and any later use of the block (a kernel or copy the
// engine still had queued on it) faults at once, as a GPU access to an
// unmapped range does.
void* hsg_rt_vmm_alloc(int dev, uint64_t nbytes, int uncached) {
  (void)dev;
  (void)uncached;
  const uint64_t n = (std::max<uint64_t>(nbytes, 1) + 4095) / 4096 * 4096;
  if (dev_live.load() + n > dev_cap.load()) return nullptr;
  void* p = mmap(nullptr, n, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  if (p == MAP_FAILED) return nullptr;
  dev_live.fetch_add(n);
  std::lock_guard<std::mutex> g(g_mu);
  ensure();
  (*g_dev_sizes)[p] = n;
  return p;
}

std::atomic<uint64_t> g_vmm_retired{0};

int hsg_rt_vmm_free(void* p) {
  uint64_t n = 0;
  {
    std::lock_guard<std::mutex> g(g_mu);
    ensure();
    auto it = g_dev_sizes->find(p);
    if (it == g_dev_sizes->end()) {
      fprintf(stderr, "stub: vmm free of %p, which is not a live block\n", p);
      abort();
    }
    n = it->second;
    g_dev_sizes->erase(it);
  }
  void* q = mmap(p, n, PROT_NONE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_FIXED | MAP_NORESERVE, -1, 0);
  if (q != p) {
    fprintf(stderr, "stub: retiring %p failed\n", p);
    abort();
  }
  dev_live.fetch_sub(n);
  g_vmm_retired.fetch_add(n);
  return 0;
}

uint64_t hsg_rt_vmm_retired_bytes() { return g_vmm_retired.load(); }

struct StubEvent {
  std::shared_ptr<Flag> f;
};

void* hsg_rt_event_record(void* stream) {
  auto* ev = new StubEvent{std::make_shared<Flag>()};
  auto f = ev->f;
  stream_of(stream)->push([f] { f->set(0); });
  return ev;
}

int hsg_rt_event_sync(void* ev) {
  static_cast<StubEvent*>(ev)->f->wait();
  return 0;
}

void hsg_rt_event_free(void* ev) { delete static_cast<StubEvent*>(ev); }

int hsg_rt_stream_after(void* waiter, void* producer) {
  auto f = std::make_shared<Flag>();
  stream_of(producer)->push([f] { f->set(0); });
  stream_of(waiter)->push([f] { f->wait(); });
  return 0;
}

int hsg_rt_stream_sync(void* stream) {
  stream_of(stream)->sync();
  return 0;
}

int hsg_rt_memcpy_d2h(void* dst, const void* src, uint64_t n) {
  memcpy(dst, src, n);
  return 0;
}

// ---- streams, pinned memory (hsgpu.hip) -----------------------------------------

void* hsg_copy_stream(int dev, int slot) {
  (void)dev;
  std::lock_guard<std::mutex> g(g_mu);
  ensure();
  auto& q = (*g_streams)[slot];
  if (!q) q.reset(new Queue());
  return q.get();
}

int hsg_stream_priority(int dev, int slot, int high) {
  (void)dev;
  (void)slot;
  (void)high;
  return 0;
}

void* hsg_pinned_acquire(uint64_t nbytes) {
  void* p = aligned_alloc(4096, (std::max<uint64_t>(nbytes, 1) + 4095) / 4096 * 4096);
  if (p) pinned_live.fetch_add(1);
  return p;
}

int hsg_pinned_release(void* p) {
  if (!p) return 0;
  pinned_live.fetch_sub(1);
  free(p);
  return 0;
}

// ---- SDMA (hsdma.hip) -------------------------------------------------------------

uint32_t hsg_sdma_h2d_engine_mask(int dev) {
  (void)dev;
  return 3u;
}

int hsg_sdma_h2d_submit_on(int dev, void* dst, const void* src, uint64_t n, int engine,
                           uint64_t* handle) {
  (void)dev;
  (void)engine;
  const int every = fail_upload_every.load();
  const bool fail = every > 0 && (g_uploads.fetch_add(1) + 1) % uint64_t(every) == 0;
  *handle = uint64_t(copy_async(dst, src, n, fail));
  return 0;
}

int hsg_sdma_release(int dev, void* stream) {
  (void)dev;
  stream_of(stream)->sync();
  return 0;
}

int hsg_sdma_d2h_submit_released(int dev, void* dst, const void* src, uint64_t n,
                                 uint64_t* handle) {
  (void)dev;
  const int every = fail_d2h_every.load();
  const bool fail = every > 0 && (g_d2h.fetch_add(1) + 1) % uint64_t(every) == 0;
  *handle = uint64_t(copy_async(dst, src, n, fail));
  return 0;
}

int hsg_sdma_d2h_submit(int dev, void* dst, const void* src, uint64_t n, void* stream,
                        uint64_t* handle) {
  (void)stream;
  return hsg_sdma_d2h_submit_released(dev, dst, src, n, handle);
}

int hsg_sdma_wait(uint64_t handle) {
  auto f = take_handle(handle);
  if (!f) return -1;
  f->wait();
  return f->rc;
}

// ---- hashing (hsgpu.hip hs_hash64) ----------------------------------------------------

int hsg_hash64(int dev, int slot, int after_slot, const void* p, uint64_t n, uint64_t first_word,
               int max_grid, int* handle) {
  (void)after_slot;
  (void)first_word;
  (void)max_grid;
  auto f = std::make_shared<Flag>();
  const uint64_t h = new_handle(f);
  static_cast<Queue*>(hsg_copy_stream(dev, slot))->push([=] { f->set(0, hash_bytes(p, n)); });
  *handle = int(h);
  return 0;
}

int hsg_hash64_into(int dev, void* stream, const void* p, uint64_t n, uint64_t first_word,
                    int max_grid, void* acc) {
  (void)dev;
  (void)first_word;
  (void)max_grid;
  stream_of(stream)->push([=] { *static_cast<uint64_t*>(acc) = hash_bytes(p, n); });
  return 0;
}

int hsg_hash64_result(int dev, int slot, int handle, uint64_t* out) {
  (void)dev;
  (void)slot;
  auto f = take_handle(uint64_t(handle));
  if (!f) return -1;
  f->wait();
  *out = f->value;
  return f->rc;
}

// ---- decode (hsz.hip) and region copies (hsgpu.hip) ------------------------------------

// Stub HSZ1 frames: a 32-byte frame header, then the frame's logical bytes
// stored as they are (the host engine validates the container, not the
// entropy coding).
int hsg_hsz_decode(int dev, const void* frames, const void* offsets, uint32_t first,
                   uint32_t count, uint64_t logical, int w, uint32_t frame_bytes, void* out,
                   void* stream, void* err) {
  (void)dev;
  (void)w;
  stream_of(stream)->push([=] {
    const uint8_t* base = static_cast<const uint8_t*>(frames);
    const uint64_t* offs = static_cast<const uint64_t*>(offsets);
    for (uint32_t f = first; f < first + count; ++f) {
      const uint64_t lo = uint64_t(f) * frame_bytes;
      const uint64_t len = std::min<uint64_t>(frame_bytes, logical - lo);
      if (offs[f + 1] - offs[f] < 32 + len) {
        *static_cast<volatile uint32_t*>(err) = 1;
        continue;
      }
      memcpy(static_cast<uint8_t*>(out) + lo, base + offs[f] + 32, len);
    }
  });
  return 0;
}

uint64_t hsg_desc_size() { return sizeof(StubDesc); }

uint64_t hsg_copy_workspace_bytes(const void* descs, int n) {
  (void)descs;
  return 64 * uint64_t(n) + 256;
}

int hsg_copy_nd(int dev, const void* descs, int n, void* workspace, uint64_t ws_bytes,
                void* pinned_stage, void* stream, int sync) {
  (void)dev;
  std::vector<StubDesc> d(static_cast<const StubDesc*>(descs),
                          static_cast<const StubDesc*>(descs) + n);
  // the launch writes its tables into the pinned stage now (host side) ...
  const uint32_t tag = g_tag.fetch_add(1);
  uint32_t* st = static_cast<uint32_t*>(pinned_stage);
  const uint64_t words = ws_bytes / 4;
  for (uint64_t k = 0; k < words; ++k) st[k] = tag;
  Queue* q = stream_of(stream);
  q->push([=] {
    // ... and the stream reads them later: nobody may have reused the stage
    for (uint64_t k = 0; k < words; ++k)
      if (st[k] != tag) {
        corruption.fetch_add(1);
        break;
      }
    uint32_t* ws = static_cast<uint32_t*>(workspace);
    for (uint64_t k = 0; k < words; ++k) ws[k] = tag;
    for (const StubDesc& x : d)
      memcpy(reinterpret_cast<void*>(x.dst), reinterpret_cast<const void*>(x.src), x.nbytes);
    for (uint64_t k = 0; k < words; ++k)
      if (ws[k] != tag) {
        corruption.fetch_add(1);
        break;
      }
  });
  if (sync) q->sync();
  return 0;
}

}  // extern "C"
