// hsdrain: native drain of an async_take's frozen HBM arena to local files.
//
// After `Snapshot.async_take` froze the device state into one HBM arena
// (engine/hbm_staging.py lays every blob out contiguously there, slab members
// at their slab offsets with zeroed gaps), the background commit has to move
// each blob arena -> host -> file.  Driven from Python, that took ~1 ms of
// interpreter work per blob on staging threads that contend for the GIL with
// the training loop, and a training step slowed by +68 % while a drain ran
// (profiles/overlap/session4).  Here the whole drain is ONE call:
//
//   dma thread     per blob: one narrow-grid hs64 hash launch (hs_hash64 on
//                  its own stream, beside the copies); per chunk of the blob
//                  (<= slot size): take a free pinned slot, submit the SDMA
//                  device->host copy (ROCr copy engine, no CUs), queue it;
//   wait thread    waits the copies in submission order, hands chunks to
//                  the writers;
//   writers        pwrite() chunks at their file offsets (page cache, or
//                  O_DIRECT straight from the pinned slot), return slots;
//                  the last chunk of a blob trims the file to size,
//                  optionally fdatasync()s it and closes it.
//
// No Python runs until the caller collects the result: the trainer keeps the
// GIL and the GPU's compute units (copies run on the SDMA engines, the hash on
// a few workgroups).  Reference behaviour being replaced:
// `/root/reference/torchsnapshot/scheduler.py:194-217` (drain of pending
// writes) and `storage_plugins/fs.py:34-36` (file writes).
//
// Host code only (device work goes through the C hooks below), so the
// engine also builds against the stubs of tests/native/engine_stubs.cpp
// under ThreadSanitizer and AddressSanitizer (tests/test_native_sanitizers.py).

#include <fcntl.h>
#include <sched.h>
#include <sys/resource.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <sys/types.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cerrno>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

extern "C" {
int hsg_sdma_d2h_submit(int dev, void* dst, const void* src, uint64_t n, void* stream,
                        uint64_t* handle);
int hsg_sdma_wait(uint64_t handle);
int hsg_sdma_release(int dev, void* stream);
int hsg_sdma_d2h_submit_released(int dev, void* dst, const void* src, uint64_t n,
                                 uint64_t* handle);
void* hsg_copy_stream(int dev, int slot);
int hsg_stream_priority(int dev, int slot, int high);
int hsg_hash64(int dev, int slot, int after_slot, const void* p, uint64_t n,
               uint64_t first_word, int max_grid, int* handle);
int hsg_hash64_result(int dev, int slot, int handle, uint64_t* out);
void* hsg_pinned_acquire(uint64_t nbytes);
int hsg_pinned_release(void* p);
int hsg_rt_set_device(int dev);
}

namespace {

constexpr int kDrainCopySlot = 1000;  // idle stream the SDMA submits order after
constexpr int kDrainHashSlot = 1001;     // high priority
constexpr int kDrainHashSlotLow = 1002;  // default priority (kFlagHashLowPrio)
constexpr int kHashLag = 256;         // results collected this many blobs behind
constexpr int kFlagSync = 1;
constexpr int kFlagHash = 2;
constexpr int kFlagDirect = 4;  // O_DIRECT: the engines' slots go to the device, no CPU copy
constexpr int kFlagHashLowPrio = 8;  // keep the hash stream at default priority
constexpr uint64_t kDirectAlign = 4096;
constexpr int kNiceShift = 8;  // flags bits 8..15: nice increment of the drain threads
constexpr int kParkedShift = 16;  // flags bits 16..23: parked writers (hsg_drain_boost)

// Lower this thread's CPU priority by `inc` (Linux: per-thread nice).  The
// drain's threads then yield a shared core to the trainer's launch thread
// instead of taking half of it; an unprivileged process may always do this.
void lower_priority(int inc) {
  if (inc <= 0) return;
  const pid_t tid = static_cast<pid_t>(syscall(SYS_gettid));
  errno = 0;
  const int cur = getpriority(PRIO_PROCESS, tid);
  if (errno != 0) return;
  setpriority(PRIO_PROCESS, tid, std::min(cur + inc, 19));
}

int mkdirs(const std::string& path) {
  // parent directories of `path`
  for (size_t i = 1; i < path.size(); ++i) {
    if (path[i] != '/') continue;
    std::string d = path.substr(0, i);
    if (mkdir(d.c_str(), 0755) != 0 && errno != EEXIST) return -errno;
  }
  return 0;
}

struct Blob {
  uint64_t src;
  uint64_t nbytes;
  std::string path;
  int fd = -1;
  bool direct = false;
  std::atomic<int> chunks_left{0};
  uint64_t sum = 0;
  int hash_handle = -1;
};

struct Chunk {
  int blob;
  uint64_t off;
  uint64_t n;
  int slot;
  uint64_t handle;
};

// Where a drain's time goes (seconds, summed over the threads doing it):
// returned by hsg_drain_wait for the bench / timeline.
enum Stat {
  kSlotWait,     // dma thread waiting for a free pinned slot (writers behind)
  kHashCollect,  // dma thread waiting for hash results
  kHashLaunch,   // dma thread launching hashes
  kSubmit,       // dma thread submitting SDMA copies
  kSdmaWait,     // wait thread waiting for copies (engines behind)
  kPwrite,       // writers in pwrite
  kClose,        // writers trimming / syncing / closing files
  kOpen,         // dma thread creating directories and opening files
  kWall,
  kNumStats
};

uint64_t now_ns() {
  return static_cast<uint64_t>(std::chrono::duration_cast<std::chrono::nanoseconds>(
      std::chrono::steady_clock::now().time_since_epoch()).count());
}

struct Job {
  std::atomic<uint64_t> ns[kNumStats] = {};
  uint64_t t_start = 0;
  void add(Stat k, uint64_t t0) { ns[k].fetch_add(now_ns() - t0); }
  int dev;
  int flags;
  int max_hash_grid;
  uint64_t slot_bytes;
  std::vector<Blob> blobs;
  std::vector<void*> slots;

  std::mutex mu;
  std::condition_variable cv;
  std::vector<int> free_slots;
  std::deque<Chunk> inflight;   // submitted copies, in order
  std::deque<Chunk> to_write;
  bool submit_done = false;
  bool wait_done = false;
  std::atomic<int> err{0};
  char errmsg[256] = {0};
  std::atomic<uint64_t> bytes_written{0};
  std::atomic<int> blobs_left{0};

  std::vector<std::thread> threads;
  bool finished = false;
  bool boost = false;  // parked writers may work (the caller waits for the drain)

  void fail(int code, const char* what, const std::string& path) {
    int expected = 0;
    if (err.compare_exchange_strong(expected, code)) {
      std::lock_guard<std::mutex> g(mu);
      snprintf(errmsg, sizeof(errmsg), "%s %s: %s", what, path.c_str(),
               code < 0 ? strerror(-code) : "error");
    }
    cv.notify_all();
  }
};

void close_blob(Job* j, Blob& b) {
  if (b.fd < 0) return;
  const uint64_t t0 = now_ns();
  struct stat st;
  if (fstat(b.fd, &st) == 0 && uint64_t(st.st_size) != b.nbytes) {
    if (ftruncate(b.fd, off_t(b.nbytes)) != 0) j->fail(-errno, "ftruncate", b.path);
  }
  if ((j->flags & kFlagSync) && fdatasync(b.fd) != 0) j->fail(-errno, "fdatasync", b.path);
  close(b.fd);
  b.fd = -1;
  j->add(kClose, t0);
}

void dma_thread(Job* j) {
  lower_priority((j->flags >> kNiceShift) & 0xff);
  // hashes run at high stream priority: a narrow grid that must not wait
  // for a training step's workgroups to drain (hsg_stream_priority)
  const int hash_slot = (j->flags & kFlagHashLowPrio) ? kDrainHashSlotLow : kDrainHashSlot;
  if (hash_slot == kDrainHashSlot) hsg_stream_priority(j->dev, kDrainHashSlot, 1);
  void* stream = hsg_copy_stream(j->dev, kDrainCopySlot);
  // the arena is frozen (the caller waited for the freeze): ONE system-scope
  // release makes it visible to the copy engines, no per-chunk event
  {
    const uint64_t t0 = now_ns();
    if (hsg_sdma_release(j->dev, stream) != 0) j->fail(-EIO, "release", "");
    j->add(kSubmit, t0);
  }
  int hashed = 0, collected = 0;
  const int nb = static_cast<int>(j->blobs.size());
  auto collect = [&](int upto) {
    const uint64_t t0 = now_ns();
    for (; collected < upto && collected < hashed; ++collected) {
      Blob& b = j->blobs[collected];
      if (b.hash_handle < 0) continue;
      if (hsg_hash64_result(j->dev, hash_slot, b.hash_handle, &b.sum) != 0)
        j->fail(-EIO, "hash result", b.path);
    }
    j->add(kHashCollect, t0);
  };
  for (int i = 0; i < nb && !j->err.load(); ++i) {
    Blob& b = j->blobs[i];
    uint64_t t0 = now_ns();
    int r = mkdirs(b.path);
    if (r == 0 && (j->flags & kFlagDirect)) {
      b.fd = open(b.path.c_str(), O_WRONLY | O_CREAT | O_CLOEXEC | O_DIRECT, 0644);
      b.direct = b.fd >= 0;  // EINVAL: the filesystem has no O_DIRECT (tmpfs)
    }
    if (r == 0 && b.fd < 0) {
      b.fd = open(b.path.c_str(), O_WRONLY | O_CREAT | O_CLOEXEC, 0644);
      if (b.fd < 0) r = -errno;
    }
    j->add(kOpen, t0);
    if (r != 0) {
      j->fail(r, "open", b.path);
      break;
    }
    t0 = now_ns();
    if (j->flags & kFlagHash) {
      if (hsg_hash64(j->dev, hash_slot, -1, reinterpret_cast<const void*>(b.src),
                     b.nbytes, 0, j->max_hash_grid, &b.hash_handle) != 0) {
        j->fail(-EIO, "hash launch", b.path);
        break;
      }
    }
    j->add(kHashLaunch, t0);
    hashed = i + 1;
    collect(hashed - kHashLag);
    const uint64_t nchunks = b.nbytes ? (b.nbytes + j->slot_bytes - 1) / j->slot_bytes : 0;
    b.chunks_left.store(static_cast<int>(nchunks));
    if (nchunks == 0) {
      close_blob(j, b);
      j->blobs_left.fetch_sub(1);
      continue;
    }
    for (uint64_t c = 0; c < nchunks && !j->err.load(); ++c) {
      int slot;
      uint64_t tw = now_ns();
      {
        std::unique_lock<std::mutex> lk(j->mu);
        j->cv.wait(lk, [&] { return !j->free_slots.empty() || j->err.load(); });
        if (j->err.load()) break;
        slot = j->free_slots.back();
        j->free_slots.pop_back();
      }
      j->add(kSlotWait, tw);
      tw = now_ns();
      const uint64_t off = c * j->slot_bytes;
      const uint64_t n = std::min(j->slot_bytes, b.nbytes - off);
      uint64_t h = 0;
      r = hsg_sdma_d2h_submit_released(j->dev, j->slots[slot],
                                       reinterpret_cast<const void*>(b.src + off), n, &h);
      j->add(kSubmit, tw);
      if (r != 0) {
        j->fail(-EIO, "sdma submit", b.path);
        break;
      }
      {
        std::lock_guard<std::mutex> g(j->mu);
        j->inflight.push_back(Chunk{i, off, n, slot, h});
      }
      j->cv.notify_all();
    }
  }
  collect(hashed);
  {
    std::lock_guard<std::mutex> g(j->mu);
    j->submit_done = true;
  }
  j->cv.notify_all();
}

void wait_thread(Job* j) {
  lower_priority((j->flags >> kNiceShift) & 0xff);
  for (;;) {
    Chunk c;
    {
      std::unique_lock<std::mutex> lk(j->mu);
      j->cv.wait(lk, [&] { return !j->inflight.empty() || j->submit_done; });
      if (j->inflight.empty()) break;
      c = j->inflight.front();
      j->inflight.pop_front();
    }
    // every submitted copy is waited for, even after an error: the engine
    // must be done with a slot before it is reused or freed
    const uint64_t t0 = now_ns();
    if (hsg_sdma_wait(c.handle) != 0) j->fail(-EIO, "sdma copy", j->blobs[c.blob].path);
    j->add(kSdmaWait, t0);
    {
      std::lock_guard<std::mutex> g(j->mu);
      j->to_write.push_back(c);
    }
    j->cv.notify_all();
  }
  {
    std::lock_guard<std::mutex> g(j->mu);
    j->wait_done = true;
  }
  j->cv.notify_all();
}

// Run this thread on the CPUs of the process's main thread (the caller's
// own mask; the drain's threads start on a narrower one that keeps off the
// training thread's core).
void widen_affinity() {
  cpu_set_t set;
  CPU_ZERO(&set);
  if (sched_getaffinity(getpid(), sizeof(set), &set) == 0)
    (void)sched_setaffinity(0, sizeof(set), &set);
}

// A parked writer (`parked`) takes no chunk before hsg_drain_boost: beside a
// training loop the drain uses few writers (their page-cache copies slow a
// launch-bound step), and all of them once the caller blocks on the drain.
// Nothing trains then, so a parked writer keeps its normal priority and, once
// woken, the caller's whole CPU mask: on the ZeRO-3 OPT-shape save (40 GB)
// the drain ran at 44.7 GB/s with 16 niced writers off the caller's core, at
// 49.5 GB/s without those restrictions (profiles/r5/zero3_ab/).
void writer_thread(Job* j, bool parked) {
  if (!parked) lower_priority((j->flags >> kNiceShift) & 0xff);
  bool widened = false;
  for (;;) {
    Chunk c;
    {
      std::unique_lock<std::mutex> lk(j->mu);
      j->cv.wait(lk, [&] {
        return ((!parked || j->boost) && !j->to_write.empty()) || j->wait_done;
      });
      if (j->to_write.empty() || (parked && !j->boost)) break;
      c = j->to_write.front();
      j->to_write.pop_front();
    }
    if (parked && !widened) {
      widened = true;
      widen_affinity();
    }
    Blob& b = j->blobs[c.blob];
    if (!j->err.load()) {
      const char* p = static_cast<const char*>(j->slots[c.slot]);
      // O_DIRECT writes whole 4 KiB blocks: the tail chunk is padded with
      // slot bytes past its end, which the blob's final ftruncate drops
      const uint64_t len = b.direct ? (c.n + kDirectAlign - 1) / kDirectAlign * kDirectAlign : c.n;
      uint64_t done = 0;
      const uint64_t t0 = now_ns();
      while (done < len) {
        const ssize_t w = pwrite(b.fd, p + done, len - done, off_t(c.off + done));
        if (w < 0) {
          if (errno == EINTR) continue;
          if (errno == EINVAL && b.direct) {
            // the device wants a larger alignment: continue buffered
            const int fl = fcntl(b.fd, F_GETFL);
            if (fl >= 0 && fcntl(b.fd, F_SETFL, fl & ~O_DIRECT) == 0) continue;
          }
          j->fail(-errno, "pwrite", b.path);
          break;
        }
        done += uint64_t(w);
      }
      j->add(kPwrite, t0);
      j->bytes_written.fetch_add(std::min(done, c.n));
    }
    {
      std::lock_guard<std::mutex> g(j->mu);
      j->free_slots.push_back(c.slot);
    }
    j->cv.notify_all();
    if (b.chunks_left.fetch_sub(1) == 1) {
      close_blob(j, b);
      j->blobs_left.fetch_sub(1);
    }
  }
}

}  // namespace

extern "C" {

// Start draining `n` blobs: blob i is device bytes [srcs[i], srcs[i] +
// sizes[i]) -> file paths[i] (created with parent directories, overwritten
// in place, trimmed to size).  `nslots` pinned slots of `slot_bytes` move
// the data; `nwriters` threads write it.  flags: 1 = fdatasync every file,
// 2 = hs64 hash every blob on the GPU (narrow grid `max_hash_grid`), 4 =
// O_DIRECT files (the pinned slots go to the device with no CPU copy and no
// page cache; buffered where the filesystem refuses it), 8 = hash stream at
// default instead of high priority, bits 8..15 = nice
// increment of every drain thread, bits 16..23 = parked writers that start
// on hsg_drain_boost.
// Returns a handle (> 0) for hsg_drain_wait, or 0 with *err set.
void* hsg_drain_start(int dev, int n, const uint64_t* srcs, const uint64_t* sizes,
                      const char* const* paths, uint64_t slot_bytes, int nslots, int nwriters,
                      int flags, int max_hash_grid, int* err) {
  *err = 0;
  if (hsg_rt_set_device(dev) != 0) {
    *err = -1;
    return nullptr;
  }
  Job* j = new Job();
  j->dev = dev;
  j->flags = flags;
  j->max_hash_grid = max_hash_grid;
  j->slot_bytes = (std::max<uint64_t>(slot_bytes, 1 << 20) + kDirectAlign - 1) / kDirectAlign *
                  kDirectAlign;
  j->blobs = std::vector<Blob>(n);
  for (int i = 0; i < n; ++i) {
    j->blobs[i].src = srcs[i];
    j->blobs[i].nbytes = sizes[i];
    j->blobs[i].path = paths[i];
  }
  j->blobs_left.store(n);
  nslots = std::max(nslots, 2);
  for (int s = 0; s < nslots; ++s) {
    void* p = hsg_pinned_acquire(j->slot_bytes);
    if (!p) {
      for (void* q : j->slots) hsg_pinned_release(q);
      delete j;
      *err = -2;
      return nullptr;
    }
    j->slots.push_back(p);
    j->free_slots.push_back(s);
    if (reinterpret_cast<uintptr_t>(p) % kDirectAlign) j->flags &= ~kFlagDirect;
  }
  j->t_start = now_ns();
  j->threads.emplace_back(dma_thread, j);
  j->threads.emplace_back(wait_thread, j);
  for (int w = 0; w < std::max(nwriters, 1); ++w) j->threads.emplace_back(writer_thread, j, false);
  for (int w = 0; w < ((flags >> kParkedShift) & 0xff); ++w)
    j->threads.emplace_back(writer_thread, j, true);
  return j;
}

// Let the parked writers work (the caller now waits for the drain).
void hsg_drain_boost(void* handle) {
  Job* j = static_cast<Job*>(handle);
  {
    std::lock_guard<std::mutex> g(j->mu);
    j->boost = true;
  }
  j->cv.notify_all();
}

// Wait for the drain (blocking; Python calls it without the GIL).  Returns 0
// or the first error (negative errno); `sums` (n entries, may be null)
// receives each blob's hs64 partial sum; `msg` (>= 256 bytes, may be null)
// the error text; `stats` (kNumStats doubles, may be null) the seconds per
// Stat.  Frees the job: call exactly once per handle.
int hsg_drain_wait(void* handle, uint64_t* sums, uint64_t* bytes_written, char* msg,
                   double* stats) {
  Job* j = static_cast<Job*>(handle);
  for (auto& t : j->threads) t.join();
  j->add(kWall, j->t_start);
  if (stats)
    for (int k = 0; k < kNumStats; ++k) stats[k] = 1e-9 * double(j->ns[k].load());
  for (auto& b : j->blobs)
    if (b.fd >= 0) close(b.fd);
  for (void* p : j->slots) hsg_pinned_release(p);
  const int e = j->err.load();
  if (sums)
    for (size_t i = 0; i < j->blobs.size(); ++i) sums[i] = j->blobs[i].sum;
  if (bytes_written) *bytes_written = j->bytes_written.load();
  if (msg) snprintf(msg, 256, "%s", j->errmsg);
  delete j;
  return e;
}

// Non-blocking progress: blobs not yet on storage (-1: bad handle).
int hsg_drain_pending(void* handle) {
  Job* j = static_cast<Job*>(handle);
  return j ? j->blobs_left.load() : -1;
}

}  // extern "C"
