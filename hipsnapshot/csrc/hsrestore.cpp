// hsrestore: native restore of local-FS blobs into HBM.
//
// The Python read pipeline (engine/scheduler.py execute_read_reqs) spends
// ~1 ms of interpreter work per blob -- pinned destinations, the header
// parse, upload and decode launches, region descriptors -- on consumer
// threads that contend for the GIL; at one rank's share of an 8-GPU
// Llama-3-8B restore that was a third of the restore and the PCIe link ran
// at 46 GB/s of its 57 (profiles/r4/restore_native/).  Here every blob whose
// bytes all land in HBM is restored by ONE call:
//
//   readers      claim the next chunk (<= slot bytes) of the plan in order,
//                pread() it from the page cache into a free pinned slot and
//                submit its SDMA upload into the blob's uncached device
//                block (csrc/hsdma.hip; several uploads stay queued, so the
//                link does not idle between chunks or blobs);
//   completion   waits the uploads in submission order, returns slots; when
//                a blob's last chunk has landed it validates the blob's HSZ1
//                frame table (kept from its first chunk) and launches the
//                device work on one of two streams: the HSZ1 decode
//                (csrc/hsz.hip) straight into the destination or into a
//                scratch block, then ONE hs_copy_nd launch (csrc/hsgpu.hip)
//                writing every destination view (strided / narrowed / cast);
//   retire       waits each blob's completion event and returns its device
//                blocks, so the HBM the pipeline holds stays within a budget.
//
// The uncached upload target needs no acquire before the kernels read it
// (see hsg_sdma_h2d); the kernels write the destinations through the L2 like
// any other kernel, ordered after the destinations' producer streams.
// Reference behaviour being replaced: `/root/reference/torchsnapshot/
// scheduler.py:384-444` (read pipeline) and `io_preparers/tensor.py:294-346`
// (buffer consumers copying into the target tensors).
//
// Host code only: every device operation goes through a C hook -- SDMA,
// decode and copy launches in hsdma.hip / hsz.hip / hsgpu.hip, the HIP
// runtime calls (device, memory, events, streams) in hshost.hip -- so this
// engine also builds without HIP, against the stubs of
// tests/native/engine_stubs.cpp, under ThreadSanitizer and AddressSanitizer
// (tests/test_native_sanitizers.py).

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

extern "C" {
int hsg_sdma_h2d_submit_on(int dev, void* dst, const void* src, uint64_t n, int engine,
                           uint64_t* handle);
uint32_t hsg_sdma_h2d_engine_mask(int dev);
int hsg_sdma_wait(uint64_t handle);
void* hsg_pinned_acquire(uint64_t nbytes);
int hsg_pinned_release(void* p);
int hsg_hsz_decode(int dev, const void* frames, const void* offsets, uint32_t first,
                   uint32_t count, uint64_t logical, int w, uint32_t frame_bytes, void* out,
                   void* stream, void* err);
uint64_t hsg_copy_workspace_bytes(const void* descs, int n);
int hsg_copy_nd(int dev, const void* descs, int n, void* workspace, uint64_t ws_bytes,
                void* pinned_stage, void* stream, int sync);
uint64_t hsg_desc_size();
void* hsg_copy_stream(int dev, int slot);
int hsg_rt_set_device(int dev);
void* hsg_rt_vmm_alloc(int dev, uint64_t nbytes, int uncached);
int hsg_rt_vmm_free(void* p);
uint64_t hsg_rt_vmm_retired_bytes();
void* hsg_rt_event_record(void* stream);
int hsg_rt_event_sync(void* ev);
void hsg_rt_event_free(void* ev);
int hsg_rt_stream_after(void* waiter, void* producer);
int hsg_rt_stream_sync(void* stream);
int hsg_rt_memcpy_d2h(void* dst, const void* src, uint64_t n);
int hsg_hash64_into(int dev, void* stream, const void* p, uint64_t n, uint64_t first_word,
                    int max_grid, void* acc);
const char* hsg_rt_last_error();
void hsg_rt_trace(const char* what, const void* p, uint64_t n, int kind);
}

namespace {

constexpr uint64_t kGranule = uint64_t(2) << 20;
constexpr uint64_t kHszHeader = 64;
constexpr uint64_t kHszFrameHeader = 32;
constexpr int kCodecRaw = 0;
constexpr int kCodecHsz = 1;
constexpr int kRestoreSlot = 2000;  // persistent streams (dev, 2000 + s), s = 0, 1

uint64_t now_ns() {
  return static_cast<uint64_t>(std::chrono::duration_cast<std::chrono::nanoseconds>(
      std::chrono::steady_clock::now().time_since_epoch()).count());
}

uint64_t align16(uint64_t n) { return (n + 15) & ~uint64_t(15); }

// ---- device block pools (uncached upload targets, plain scratch) -----------
//
// Cached per device by size (best fit up to 2x, 2 MiB granules) across
// restores; hsg_restore_trim() frees the idle ones.  Blocks come from
// hsg_rt_vmm_alloc (hshost.hip): a freed block's virtual range is never
// handed out again.  With hipMalloc / hipExtMallocWithFlags blocks, freeing
// uncached and plain blocks left the process's next blocks used through stale
// translations: wrong bytes and hipErrorIllegalAddress faults whenever the
// pools were trimmed (profiles/r6/trim/).
//
// Freed ranges stay reserved (virtual address space only); past this many
// bytes of them a trim keeps its blocks instead.
constexpr uint64_t kMaxRetiredVa = uint64_t(64) << 40;
struct DevPool {
  std::mutex mu;
  std::map<int, std::multimap<uint64_t, void*>> free_blocks;
  std::unordered_map<void*, std::pair<int, uint64_t>> live;
  uint64_t idle_bytes = 0;
  int uncached;  // device-uncached blocks (SDMA upload targets)

  explicit DevPool(int u) : uncached(u) {}

  void* acquire(int dev, uint64_t nbytes) {
    const uint64_t want = (std::max<uint64_t>(nbytes, 1) + kGranule - 1) / kGranule * kGranule;
    {
      std::lock_guard<std::mutex> g(mu);
      auto& fl = free_blocks[dev];
      auto it = fl.lower_bound(want);
      if (it != fl.end() && it->first <= 2 * want) {
        void* p = it->second;
        live[p] = {dev, it->first};
        idle_bytes -= it->first;
        hsg_rt_trace("reuse", p, it->first, uncached);
        fl.erase(it);
        return p;
      }
    }
    void* p = nullptr;
    for (int attempt = 0; attempt < 2; ++attempt) {
      p = hsg_rt_vmm_alloc(dev, want, uncached);
      if (p) break;
      if (attempt == 0) trim(dev, 0);  // drop this device's idle blocks and retry
    }
    if (!p) return nullptr;
    std::lock_guard<std::mutex> g(mu);
    live[p] = {dev, want};
    return p;
  }

  void release(void* p) {
    if (!p) return;
    std::lock_guard<std::mutex> g(mu);
    auto it = live.find(p);
    if (it == live.end()) return;
    free_blocks[it->second.first].emplace(it->second.second, p);
    idle_bytes += it->second.second;
    live.erase(it);
  }

  // bytes of `dev`'s blocks (-1: every device): idle ones, ones in use
  void bytes(int dev, uint64_t* idle_out, uint64_t* live_out) {
    std::lock_guard<std::mutex> g(mu);
    uint64_t idle = 0, used = 0;
    for (auto& dv : free_blocks) {
      if (dev >= 0 && dv.first != dev) continue;
      for (auto& kv : dv.second) idle += kv.first;
    }
    for (auto& kv : live)
      if (dev < 0 || kv.second.first == dev) used += kv.second.second;
    *idle_out = idle;
    *live_out = used;
  }

  // idle blocks of `dev`: (address, bytes) pairs, at most `max`
  int idle(int dev, uint64_t* ptrs, uint64_t* sizes, int max) {
    std::lock_guard<std::mutex> g(mu);
    int n = 0;
    auto it = free_blocks.find(dev);
    if (it == free_blocks.end()) return 0;
    for (auto& kv : it->second) {
      if (n >= max) break;
      ptrs[n] = reinterpret_cast<uint64_t>(kv.second);
      sizes[n] = kv.first;
      ++n;
    }
    return n;
  }

  // free idle blocks of `dev` (-1: all devices) until at most `keep` idle
  // bytes remain (largest first); returns the bytes freed
  uint64_t trim(int dev, uint64_t keep) {
    std::vector<void*> drop;
    uint64_t freed = 0;
    if (hsg_rt_vmm_retired_bytes() > kMaxRetiredVa) return 0;
    {
      std::lock_guard<std::mutex> g(mu);
      for (auto& dv : free_blocks) {
        if (dev >= 0 && dv.first != dev) continue;
        auto& fl = dv.second;
        while (!fl.empty() && idle_bytes > keep) {
          auto it = std::prev(fl.end());
          drop.push_back(it->second);
          idle_bytes -= it->first;
          freed += it->first;
          fl.erase(it);
        }
      }
    }
    for (void* q : drop) (void)hsg_rt_vmm_free(q);
    return freed;
  }
};

DevPool g_upload_pool(1);
DevPool g_scratch_pool(0);

// A job's device memory: one block per kind (uncached upload targets, decode
// scratch) carved into per-item ranges in plan order and returned in any
// order; a range is reusable once every range before it came back.  One
// allocation per job instead of one per blob (the first restore of a
// checkpoint paid a hipMalloc per blob).
struct Ring {
  char* base = nullptr;
  uint64_t cap = 0;
  uint64_t head = 0, tail = 0;  // virtual byte counters (offset = v % cap)
  struct Range {
    uint64_t v0, v1;
    bool released;
  };
  std::deque<Range> live;

  bool fits(uint64_t n) const {
    uint64_t start = head;
    const uint64_t phys = start % cap;
    if (phys + n > cap) start += cap - phys;  // wrap: the tail end stays unused
    return start + n - tail <= cap;
  }
  // caller checked fits(n); returns the range's virtual start (its id)
  uint64_t alloc(uint64_t n, char** p) {
    const uint64_t v0 = head;
    uint64_t start = head;
    const uint64_t phys = start % cap;
    if (phys + n > cap) start += cap - phys;
    live.push_back(Range{v0, start + n, false});
    head = start + n;
    *p = base + start % cap;
    return v0;
  }
  void release(uint64_t v0) {
    for (auto& r : live)
      if (r.v0 == v0) {
        r.released = true;
        break;
      }
    while (!live.empty() && live.front().released) {
      tail = live.front().v1;
      live.pop_front();
    }
    // empty: restart at a physical offset of 0.  Otherwise a range longer
    // than both the space after the old head and the space before it would
    // never fit an empty ring, and its reader would wait for a release that
    // cannot come.
    if (live.empty()) head = tail = (head + cap - 1) / cap * cap;
  }
};

uint64_t align4k(uint64_t n) { return (n + 4095) & ~uint64_t(4095); }

// ---- the job -----------------------------------------------------------------

struct Item {
  std::string path;
  uint64_t file_lo = 0;    // first file byte to read
  uint64_t nbytes = 0;     // bytes to read (the whole stored blob for HSZ1)
  int codec = kCodecRaw;
  uint64_t logical = 0;    // HSZ1: expected logical size
  uint64_t direct = 0;     // HSZ1: decode straight into this device address
  uint64_t base_off = 0;   // region sources start here in the decoded / raw bytes
  int64_t desc_off = 0;    // first descriptor in the job's table
  int desc_n = 0;
  bool hash = false;       // hs64 the uploaded (stored) bytes: restore(verify=True)

  // runtime
  std::mutex mu;
  int fd = -1;
  int pieces_read = 0;     // pieces read so far (the last one closes fd)
  int npieces = 0;
  void* block = nullptr;   // uncached upload target
  void* scratch = nullptr; // HSZ1 decode output when not direct
  void* ws = nullptr;      // copy descriptor / tile workspace
  void* stage = nullptr;   // pinned stage of the workspace tables
  bool allocated = false;  // block (and scratch) assigned
  bool pooled = false;     // from the pools (larger than a ring), not a ring
  uint64_t up_v = 0, sc_v = 0;  // ring range ids
  bool ws_ring = false;    // ws / stage carved from the job's small rings
  uint64_t ws_v = 0, st_v = 0;
  int nchunks = 0;
  std::atomic<int> chunks_left{0};
  std::vector<uint8_t> head;  // HSZ1 header + frame table (from chunk 0)
  void* done = nullptr;  // completion event of the item's device work
};

struct Chunk {
  int item;
  int index;
  uint64_t off;  // within the item
  uint64_t n;
  int slot;
  uint64_t handle;
};

// A pinned slot being filled: one upload unit (<= slot bytes of one item),
// read by several readers in pieces; the reader finishing the last piece
// submits the upload.
struct SlotFill {
  int item = -1;
  int chunk = -1;
  uint64_t off = 0;  // within the item
  uint64_t n = 0;
  int pieces = 0;
  int next_piece = 0;
  std::atomic<int> left{0};
};

enum Stat {
  kRead,         // readers in pread
  kSlotWait,     // readers waiting for a free pinned slot
  kBudgetWait,   // readers waiting for ring space (earlier blobs to retire)
  kAlloc,        // readers acquiring device blocks
  kSubmit,       // readers submitting uploads
  kUploadWait,   // completion thread waiting for uploads
  kLaunch,       // completion thread validating + launching device work
  kRetireWait,   // retire thread waiting for device work
  kFirstUpload,  // start -> first upload submitted
  kUploadBusy,   // time with at least one upload in flight
  kWall,
  kNumStats
};

struct Job {
  int dev = 0;
  uint64_t slot_bytes = 0;
  uint64_t budget = 0;
  int engine = -1;  // SDMA engine of the uploads (-1: ROCr's choice)
  std::vector<Item> items;
  std::vector<uint8_t> descs;  // packed CopyDesc table (sources relative)
  uint64_t desc_size = 0;
  uint32_t* err_words = nullptr;  // host-mapped, one per item
  void* streams[2] = {nullptr, nullptr};
  int hash_grid = 64;
  uint64_t* hash_acc = nullptr;   // device: one hs64 partial sum per item


  std::vector<void*> slots;
  std::unique_ptr<SlotFill[]> fills;
  uint64_t piece_bytes = 0;
  int filling = -1;  // the slot readers currently claim pieces of
  std::mutex mu;
  std::condition_variable cv;
  std::vector<int> free_slots;
  std::deque<Chunk> inflight;
  std::deque<int> retire;
  // upload units in plan order: the job's first is small (the link starts
  // early), the rest up to slot bytes (few, large SDMA requests: each costs a
  // fixed ~0.1 ms on the engine, profiles/r4/restore_native/)
  struct Span {
    int item;
    int index;
    uint64_t off;
    uint64_t n;
  };
  std::vector<Span> spans;
  size_t cursor = 0;
  int readers_left = 0;
  bool completion_done = false;
  Ring up_ring, sc_ring;
  void* up_base = nullptr;  // pool blocks behind the rings
  void* sc_base = nullptr;
  // copy-launch tables: descriptors + tiles in HBM, staged through pinned
  // memory; carved per blob from one block each (a first restore in a
  // process paid a hipMalloc and a pinned registration per slab blob)
  Ring ws_ring, st_ring;
  void* ws_base = nullptr;
  void* st_base = nullptr;
  int pooled_live = 0;      // items on pool blocks (one at a time, rings empty)
  int launched = 0;
  uint64_t busy_since = 0;  // outstanding went non-zero at (kUploadBusy)
  int outstanding = 0;      // uploads submitted and not yet waited for

  std::atomic<int> err{0};
  int err_item = -1;
  char errmsg[320] = {0};
  std::atomic<uint64_t> ns[kNumStats] = {};
  std::atomic<uint64_t> bytes_read{0};
  std::atomic<bool> first_upload{false};
  uint64_t t_start = 0;
  std::vector<std::thread> threads;

  void add(Stat k, uint64_t t0) { ns[k].fetch_add(now_ns() - t0); }

  void fail(int code, int item, const char* what) {
    int expected = 0;
    if (err.compare_exchange_strong(expected, code)) {
      std::lock_guard<std::mutex> g(mu);
      err_item = item;
      snprintf(errmsg, sizeof(errmsg), "%s %s: %s%s%s", what,
               item >= 0 ? items[item].path.c_str() : "",
               code < 0 && code > -4096 ? strerror(-code) : "error",
               code == -EIO ? " -- " : "", code == -EIO ? hsg_rt_last_error() : "");
    }
    cv.notify_all();
  }
};


// Device memory of item i (upload target, decode scratch), assigned when
// its first span starts filling, under j->mu and in plan order (the rings
// are then released roughly in order).  Returns 0 = assigned, 1 = wait for
// earlier items to retire, -1 = out of device memory.  An item larger than
// a ring gets pool blocks, once nothing else holds device memory.
int alloc_item_locked(Job* j, int i) {
  Item& it = j->items[i];
  if (it.allocated) return 0;
  const uint64_t nu = align4k(it.nbytes);
  const uint64_t ns = (it.codec == kCodecHsz && !it.direct) ? align4k(it.logical) : 0;
  const bool ring_ok = j->up_ring.base && nu <= j->up_ring.cap &&
                       (ns == 0 || (j->sc_ring.base && ns <= j->sc_ring.cap));
  if (ring_ok) {
    if (j->pooled_live > 0 || !j->up_ring.fits(nu) || (ns && !j->sc_ring.fits(ns))) return 1;
    char* p = nullptr;
    it.up_v = j->up_ring.alloc(nu, &p);
    it.block = p;
    if (ns) {
      it.sc_v = j->sc_ring.alloc(ns, &p);
      it.scratch = p;
    }
    it.allocated = true;
    return 0;
  }
  if (j->pooled_live > 0 || !j->up_ring.live.empty() || !j->sc_ring.live.empty()) return 1;
  const uint64_t t0 = now_ns();
  it.block = g_upload_pool.acquire(j->dev, it.nbytes);
  if (it.block && ns) it.scratch = g_scratch_pool.acquire(j->dev, it.logical);
  j->add(kAlloc, t0);
  it.pooled = true;
  it.allocated = true;
  ++j->pooled_live;
  return (it.block && (ns == 0 || it.scratch)) ? 0 : -1;
}

int pieces_of(const Job* j, uint64_t n) { return int((n + j->piece_bytes - 1) / j->piece_bytes); }

void reader_thread(Job* j) {
  (void)hsg_rt_set_device(j->dev);
  for (;;) {
    int s, i;
    uint64_t poff, pn;
    {
      std::unique_lock<std::mutex> lk(j->mu);
      bool finished = false;
      int nomem = -1;
      for (;;) {
        if (j->err.load()) {
          finished = true;
          break;
        }
        if (j->filling >= 0 && j->fills[j->filling].next_piece < j->fills[j->filling].pieces)
          break;
        if (j->cursor >= j->spans.size()) {
          finished = true;
          break;
        }
        if (j->free_slots.empty()) {
          const uint64_t t0 = now_ns();
          j->cv.wait(lk);
          j->add(kSlotWait, t0);
          continue;
        }
        // start filling a free slot with the plan's next span; an item's
        // first span gets its device memory first
        const Job::Span& nx = j->spans[j->cursor];
        if (nx.index == 0) {
          const uint64_t t0 = now_ns();
          const int a = alloc_item_locked(j, nx.item);
          if (a == 1) {
            j->cv.wait(lk);
            j->add(kBudgetWait, t0);
            continue;
          }
          if (a < 0) {
            nomem = nx.item;
            finished = true;
            break;
          }
        }
        const int fs = j->free_slots.back();
        j->free_slots.pop_back();
        const Job::Span& sp = j->spans[j->cursor++];
        SlotFill& f = j->fills[fs];
        f.item = sp.item;
        f.chunk = sp.index;
        f.off = sp.off;
        f.n = sp.n;
        f.pieces = pieces_of(j, f.n);
        f.next_piece = 0;
        f.left.store(f.pieces);
        j->filling = fs;
      }
      if (finished) {
        lk.unlock();
        if (nomem >= 0) j->fail(-ENOMEM, nomem, "device block");
        break;
      }
      s = j->filling;
      SlotFill& f = j->fills[s];
      const int k = f.next_piece++;
      i = f.item;
      poff = uint64_t(k) * j->piece_bytes;
      pn = std::min(j->piece_bytes, f.n - poff);
    }
    // other readers may claim the slot's remaining pieces at once
    j->cv.notify_all();
    SlotFill& f = j->fills[s];
    Item& it = j->items[i];
    {
      std::lock_guard<std::mutex> g(it.mu);
      if (it.fd < 0 && it.pieces_read < it.npieces) {
        it.fd = open(it.path.c_str(), O_RDONLY | O_CLOEXEC);
        if (it.fd < 0) {
          j->fail(-errno, i, "open");
          break;
        }
      }
    }
    char* p = static_cast<char*>(j->slots[s]) + poff;
    uint64_t t0 = now_ns();
    uint64_t done = 0;
    int rerr = 0;
    while (done < pn) {
      const ssize_t r = pread(it.fd, p + done, pn - done, off_t(it.file_lo + f.off + poff + done));
      if (r < 0) {
        if (errno == EINTR) continue;
        rerr = -errno;
        break;
      }
      if (r == 0) {
        rerr = -ENODATA;  // the file is shorter than the manifest says
        break;
      }
      done += uint64_t(r);
    }
    j->add(kRead, t0);
    {
      std::lock_guard<std::mutex> g(it.mu);
      if (++it.pieces_read == it.npieces && it.fd >= 0) {
        close(it.fd);
        it.fd = -1;
      }
    }
    if (rerr) {
      j->fail(rerr, i, "read");
      break;
    }
    j->bytes_read.fetch_add(pn);
    if (f.left.fetch_sub(1) != 1) continue;
    // the slot is full: upload it
    const char* sp = static_cast<const char*>(j->slots[s]);
    if (f.chunk == 0 && it.codec == kCodecHsz) {
      // header + frame table: validated once every chunk has landed
      uint64_t nf = 0;
      memcpy(&nf, sp + 24, 4);
      const uint64_t hb = std::min<uint64_t>(f.n, kHszHeader + 8 * (nf + 1));
      it.head.assign(sp, sp + hb);
    }
    t0 = now_ns();
    uint64_t h = 0;
    hsg_rt_trace("upload", static_cast<char*>(it.block) + f.off, f.n, i);
    const int r = hsg_sdma_h2d_submit_on(j->dev, static_cast<char*>(it.block) + f.off, sp, f.n,
                                         j->engine, &h);
    if (!j->first_upload.exchange(true)) j->ns[kFirstUpload].store(now_ns() - j->t_start);
    j->add(kSubmit, t0);
    if (r != 0) {
      j->fail(-EIO, i, "sdma upload");
      break;
    }
    {
      std::lock_guard<std::mutex> g(j->mu);
      if (j->outstanding++ == 0) j->busy_since = now_ns();
      j->inflight.push_back(Chunk{i, f.chunk, f.off, f.n, s, h});
    }
    j->cv.notify_all();
  }
  {
    std::lock_guard<std::mutex> g(j->mu);
    --j->readers_left;
  }
  j->cv.notify_all();
}

// Validate item i's HSZ1 header + frame table (what codec.validate_offsets
// checks in Python) before any kernel walks the frames.
bool hsz_header_ok(const Item& it, int* w, uint32_t* fb, uint32_t* nf) {
  const std::vector<uint8_t>& h = it.head;
  if (h.size() < kHszHeader || memcmp(h.data(), "HSZ1", 4) != 0) return false;
  uint32_t version, width, frame_bytes, n_frames;
  uint64_t logical;
  memcpy(&version, h.data() + 4, 4);
  memcpy(&logical, h.data() + 8, 8);
  memcpy(&width, h.data() + 16, 4);
  memcpy(&frame_bytes, h.data() + 20, 4);
  memcpy(&n_frames, h.data() + 24, 4);
  if (version != 1 && version != 2) return false;
  if (logical != it.logical) return false;
  if (!(width == 1 || width == 2 || width == 4 || width == 8)) return false;
  if (frame_bytes == 0 || frame_bytes % 16 || frame_bytes % width) return false;
  const uint64_t want_nf = std::max<uint64_t>(1, (logical + frame_bytes - 1) / frame_bytes);
  if (n_frames != want_nf) return false;
  if (h.size() < kHszHeader + 8 * (uint64_t(n_frames) + 1)) return false;
  const uint64_t* offs = reinterpret_cast<const uint64_t*>(h.data() + kHszHeader);
  if (offs[0] < kHszHeader + 8 * (uint64_t(n_frames) + 1) || offs[n_frames] > it.nbytes)
    return false;
  for (uint32_t f = 0; f < n_frames; ++f) {
    const uint64_t lo = uint64_t(f) * frame_bytes;
    const uint64_t len = std::min<uint64_t>(frame_bytes, logical - std::min(lo, logical));
    if (offs[f + 1] < offs[f] + kHszFrameHeader ||
        offs[f + 1] - offs[f] > align16(kHszFrameHeader + len))
      return false;
  }
  *w = int(width);
  *fb = frame_bytes;
  *nf = n_frames;
  return true;
}

// Decode / copy launches for item i on stream s; records it.done.
int launch_item(Job* j, int i, void* s) {
  Item& it = j->items[i];
  char* base = static_cast<char*>(it.block);
  // the stored bytes as they landed, before anything reads them
  if (it.hash && hsg_hash64_into(j->dev, s, it.block, it.nbytes, 0, j->hash_grid,
                                 j->hash_acc + i) != 0) {
    j->fail(-EIO, i, "hash launch");
    return -1;
  }
  if (it.codec == kCodecHsz) {
    int w;
    uint32_t fb, nf;
    if (!hsz_header_ok(it, &w, &fb, &nf)) {
      j->fail(-EBADMSG, i, "corrupt HSZ1 header or frame table in");
      return -1;
    }
    void* out = it.direct ? reinterpret_cast<void*>(it.direct) : it.scratch;
    if (hsg_hsz_decode(j->dev, it.block, base + kHszHeader, 0, nf, it.logical, w, fb, out, s,
                       j->err_words + i) != 0) {
      j->fail(-EIO, i, "decode launch");
      return -1;
    }
    base = static_cast<char*>(out);
  }
  if (it.desc_n > 0) {
    std::vector<uint8_t> d(j->descs.begin() + it.desc_off * int64_t(j->desc_size),
                           j->descs.begin() + (it.desc_off + it.desc_n) * int64_t(j->desc_size));
    const uint64_t src_base = reinterpret_cast<uint64_t>(base) + it.base_off;
    for (int k = 0; k < it.desc_n; ++k) {
      uint64_t v;
      memcpy(&v, d.data() + uint64_t(k) * j->desc_size, 8);
      v += src_base;
      memcpy(d.data() + uint64_t(k) * j->desc_size, &v, 8);
    }
    const uint64_t wsb = hsg_copy_workspace_bytes(d.data(), it.desc_n);
    {
      std::lock_guard<std::mutex> g(j->mu);
      const uint64_t n = align4k(wsb);
      if (j->ws_ring.base && j->st_ring.base && n <= j->ws_ring.cap && n <= j->st_ring.cap &&
          j->ws_ring.fits(n) && j->st_ring.fits(n)) {
        char* p = nullptr;
        it.ws_v = j->ws_ring.alloc(n, &p);
        it.ws = p;
        it.st_v = j->st_ring.alloc(n, &p);
        it.stage = p;
        it.ws_ring = true;
      }
    }
    if (!it.ws_ring) {  // full or too large: pool blocks
      it.ws = g_scratch_pool.acquire(j->dev, wsb);
      it.stage = hsg_pinned_acquire(wsb);
    }
    if (!it.ws || !it.stage) {
      j->fail(-ENOMEM, i, "copy workspace");
      return -1;
    }
    if (hsg_copy_nd(j->dev, d.data(), it.desc_n, it.ws, wsb, it.stage, s, 0) != 0) {
      j->fail(-EIO, i, "copy launch");
      return -1;
    }
  }
  it.done = hsg_rt_event_record(s);
  if (!it.done) {
    j->fail(-EIO, i, "completion event");
    return -1;
  }
  return 0;
}

void release_item(Job* j, Item& it) {
  if (!it.ws_ring) {
    g_scratch_pool.release(it.ws);
    if (it.stage) hsg_pinned_release(it.stage);
  }
  if (it.done) {
    hsg_rt_event_free(it.done);
    it.done = nullptr;
  }
  {
    std::lock_guard<std::mutex> g(j->mu);
    if (it.allocated) {
      if (it.pooled) {
        g_upload_pool.release(it.block);
        g_scratch_pool.release(it.scratch);
        --j->pooled_live;
      } else {
        j->up_ring.release(it.up_v);
        if (it.scratch) j->sc_ring.release(it.sc_v);
      }
    }
    if (it.ws_ring) {
      j->ws_ring.release(it.ws_v);
      j->st_ring.release(it.st_v);
    }
    it.allocated = it.pooled = it.ws_ring = false;
    it.block = it.scratch = it.ws = it.stage = nullptr;
  }
  j->cv.notify_all();
}

void completion_thread(Job* j) {
  (void)hsg_rt_set_device(j->dev);
  for (;;) {
    Chunk c;
    {
      std::unique_lock<std::mutex> lk(j->mu);
      j->cv.wait(lk, [&] { return !j->inflight.empty() || j->readers_left == 0; });
      if (j->inflight.empty()) break;
      c = j->inflight.front();
      j->inflight.pop_front();
    }
    // every submitted upload is waited for, even after an error: the engine
    // must be done with a slot and a block before they are reused
    uint64_t t0 = now_ns();
    const int r = hsg_sdma_wait(c.handle);
    j->add(kUploadWait, t0);
    {
      std::lock_guard<std::mutex> g(j->mu);
      j->free_slots.push_back(c.slot);
      if (--j->outstanding == 0) j->ns[kUploadBusy].fetch_add(now_ns() - j->busy_since);
    }
    j->cv.notify_all();
    if (r != 0) j->fail(-EIO, c.item, "sdma upload");
    Item& it = j->items[c.item];
    if (it.chunks_left.fetch_sub(1) != 1 || j->err.load()) continue;
    t0 = now_ns();
    const int rc = launch_item(j, c.item, j->streams[j->launched++ & 1]);
    j->add(kLaunch, t0);
    std::lock_guard<std::mutex> g(j->mu);
    if (rc == 0) j->retire.push_back(c.item);
    j->cv.notify_all();
  }
  std::lock_guard<std::mutex> g(j->mu);
  j->completion_done = true;
  j->cv.notify_all();
}

void retire_thread(Job* j) {
  (void)hsg_rt_set_device(j->dev);
  for (;;) {
    int i;
    {
      std::unique_lock<std::mutex> lk(j->mu);
      j->cv.wait(lk, [&] { return !j->retire.empty() || j->completion_done; });
      if (j->retire.empty()) break;
      i = j->retire.front();
      j->retire.pop_front();
    }
    const uint64_t t0 = now_ns();
    if (hsg_rt_event_sync(j->items[i].done) != 0) j->fail(-EIO, i, "device work");
    j->add(kRetireWait, t0);
    release_item(j, j->items[i]);
  }
}

}  // namespace

extern "C" {

// Start restoring `n` items.  Item i: read file bytes [file_lo[i], file_lo[i]
// + nbytes[i]) of paths[i]; codec[i] 0 = raw bytes, 1 = a whole HSZ1 blob of
// logical[i] logical bytes (decoded into direct[i] when nonzero, else into a
// scratch block); then descriptors [desc_off[i], desc_off[i] + desc_n[i]) of
// `descs` (CopyDesc rows whose `src` is an offset into the raw / decoded
// bytes, relative to base_off[i]) copy the bytes into their destinations.
// Device work is ordered after every stream in `producers`.  `err_words`:
// host-mapped uint32 per item (decoders flag corrupt frames there).
// `hash_items` (nullable): items whose stored bytes are hs64-hashed in HBM
// on their stream before anything reads them (grid <= `hash_grid`
// workgroups); hsg_restore_wait returns the partial sums.
// Returns a handle for hsg_restore_wait, or null with *err set.
void* hsg_restore_start(int dev, int n, const char* const* paths, const uint64_t* file_lo,
                        const uint64_t* nbytes, const int* codec, const uint64_t* logical,
                        const uint64_t* direct, const uint64_t* base_off, const int64_t* desc_off,
                        const int* desc_n, const void* descs, int64_t n_descs,
                        const uint64_t* producers, int n_producers, uint32_t* err_words,
                        uint64_t slot_bytes, uint64_t first_bytes, uint64_t piece_bytes,
                        int nslots, int nreaders, uint64_t budget, int engine,
                        const int* hash_items, int hash_grid, int* err) {
  *err = 0;
  if (hsg_rt_set_device(dev) != 0) {
    *err = -1;
    return nullptr;
  }
  Job* j = new Job();
  j->dev = dev;
  j->slot_bytes = (std::max<uint64_t>(slot_bytes, 1 << 20) + 4095) / 4096 * 4096;
  first_bytes = std::max<uint64_t>(first_bytes, 1 << 20);
  j->piece_bytes = std::min<uint64_t>(j->slot_bytes,
                                      (std::max<uint64_t>(piece_bytes, 256 << 10) + 4095) / 4096 * 4096);
  j->budget = std::max<uint64_t>(budget, kGranule);
  // engine -2: the lowest free host -> device engine; >= 0 as given if free
  const uint32_t emask = hsg_sdma_h2d_engine_mask(dev);
  if (engine == -2) engine = emask ? __builtin_ctz(emask) : -1;
  j->engine = (engine >= 0 && engine < 32 && (emask & (1u << engine))) ? engine : -1;
  j->desc_size = hsg_desc_size();
  j->err_words = err_words;
  j->descs.assign(static_cast<const uint8_t*>(descs),
                  static_cast<const uint8_t*>(descs) + n_descs * int64_t(j->desc_size));
  j->items = std::vector<Item>(n);
  for (int i = 0; i < n; ++i) {
    Item& it = j->items[i];
    it.path = paths[i];
    it.file_lo = file_lo[i];
    it.nbytes = nbytes[i];
    it.codec = codec[i];
    it.logical = logical[i];
    it.direct = direct[i];
    it.base_off = base_off[i];
    it.desc_off = desc_off[i];
    it.desc_n = desc_n[i];
    it.hash = hash_items != nullptr && hash_items[i] != 0;
    for (uint64_t off = 0; off < it.nbytes;) {
      const uint64_t cap = j->spans.empty() ? std::min(j->slot_bytes, first_bytes) : j->slot_bytes;
      const uint64_t n = std::min(cap, it.nbytes - off);
      j->spans.push_back(Job::Span{i, it.nchunks++, off, n});
      it.npieces += pieces_of(j, n);
      off += n;
    }
    it.chunks_left.store(it.nchunks);
    if (desc_off[i] < 0 || desc_off[i] + desc_n[i] > n_descs || it.nchunks == 0 ||
        (it.codec == kCodecHsz && it.nbytes < kHszHeader)) {
      delete j;
      *err = -3;
      return nullptr;
    }
  }
  j->hash_grid = hash_grid;
  // persistent streams (creating one costs ~1 ms of HIP runtime time)
  for (int s = 0; s < 2; ++s) {
    j->streams[s] = hsg_copy_stream(dev, kRestoreSlot + s);
    if (!j->streams[s]) {
      delete j;
      *err = -4;
      return nullptr;
    }
  }
  // the destinations' producers: their queued work finishes before ours (a
  // failure here would let the copies race it: the job does not start)
  for (int p = 0; p < n_producers; ++p) {
    bool ok = true;
    for (int s = 0; ok && s < 2; ++s)
      ok = hsg_rt_stream_after(j->streams[s], reinterpret_cast<void*>(producers[p])) == 0;
    if (!ok) {
      delete j;
      *err = -5;
      return nullptr;
    }
  }
  // the rings: at most `budget` bytes each, no more than the job needs
  uint64_t need_up = 0, need_sc = 0;
  for (const Item& it : j->items) {
    need_up += align4k(it.nbytes);
    if (it.codec == kCodecHsz && !it.direct) need_sc += align4k(it.logical);
  }
  const uint64_t cap_up = std::min(j->budget, need_up), cap_sc = std::min(j->budget, need_sc);
  if (cap_up) j->up_base = g_upload_pool.acquire(dev, cap_up);
  if (cap_sc) j->sc_base = g_scratch_pool.acquire(dev, cap_sc);
  if (j->up_base) {
    j->up_ring.base = static_cast<char*>(j->up_base);
    j->up_ring.cap = cap_up;
  }
  if (j->sc_base) {
    j->sc_ring.base = static_cast<char*>(j->sc_base);
    j->sc_ring.cap = cap_sc;
  }
  bool any_desc = false;
  for (const Item& it : j->items) any_desc |= it.desc_n > 0;
  if (any_desc) {
    // a quarter of a slot (the pinned stage counts against the read's budget)
    const uint64_t kTables = std::min<uint64_t>(uint64_t(32) << 20,
                                                std::max<uint64_t>(1 << 20, j->slot_bytes / 4));
    j->ws_base = g_scratch_pool.acquire(dev, kTables);
    j->st_base = hsg_pinned_acquire(kTables);
    if (j->ws_base && j->st_base) {
      j->ws_ring.base = static_cast<char*>(j->ws_base);
      j->ws_ring.cap = kTables;
      j->st_ring.base = static_cast<char*>(j->st_base);
      j->st_ring.cap = kTables;
    }
  }
  nslots = std::max(nslots, 2);
  j->fills.reset(new SlotFill[nslots]);
  j->slots.assign(nslots, nullptr);
  bool any_hash = false;
  for (const Item& it : j->items) any_hash |= it.hash;
  if (any_hash) j->hash_acc = static_cast<uint64_t*>(g_scratch_pool.acquire(dev, 8 * uint64_t(n)));
  // two slots now, the rest from a helper thread while the readers start:
  // a first use of pinned memory in the process registers it (~10 ms/GiB)
  for (int s = 0; s < 2; ++s) {
    void* p = (any_hash && !j->hash_acc) ? nullptr : hsg_pinned_acquire(j->slot_bytes);
    if (!p) {
      g_scratch_pool.release(j->hash_acc);
      for (void* q : j->slots)
        if (q) hsg_pinned_release(q);
      g_upload_pool.release(j->up_base);
      g_scratch_pool.release(j->sc_base);
      g_scratch_pool.release(j->ws_base);
      if (j->st_base) hsg_pinned_release(j->st_base);
      delete j;
      *err = -2;
      return nullptr;
    }
    j->slots[s] = p;
    j->free_slots.push_back(1 - s);
  }
  j->t_start = now_ns();
  hsg_rt_trace("job-start", j, uint64_t(n), dev);
  if (nslots > 2)
    j->threads.emplace_back([j, nslots] {
      for (int s = 2; s < nslots && !j->err.load(); ++s) {
        {
          std::lock_guard<std::mutex> g(j->mu);
          if (j->cursor >= j->spans.size()) break;  // every span already has a slot
        }
        void* p = hsg_pinned_acquire(j->slot_bytes);
        if (!p) break;  // fewer slots, not an error
        {
          std::lock_guard<std::mutex> g(j->mu);
          j->slots[s] = p;
          j->free_slots.insert(j->free_slots.begin(), s);
        }
        j->cv.notify_all();
      }
    });
  nreaders = std::max(nreaders, 1);
  j->readers_left = nreaders;
  for (int r = 0; r < nreaders; ++r) j->threads.emplace_back(reader_thread, j);
  j->threads.emplace_back(completion_thread, j);
  j->threads.emplace_back(retire_thread, j);
  return j;
}

// Wait for the restore (blocking; Python calls it without the GIL).  Returns
// 0 or the first error (negative errno); *err_item = the item it concerns
// (-1: none); `msg` (>= 320 bytes) its text; `stats` (kNumStats doubles:
// seconds) where the time went; *bytes_read the bytes read from files;
// `sums` (n entries, nullable) the hs64 partial sums of the hashed items'
// stored bytes (0 for the others).
// Everything launched has finished when this returns (decode error words
// are final).  Frees the job: call exactly once per handle.
int hsg_restore_wait(void* handle, int* err_item, char* msg, double* stats,
                     uint64_t* bytes_read, uint64_t* sums) {
  Job* j = static_cast<Job*>(handle);
  for (auto& t : j->threads) t.join();
  for (int s = 0; s < 2; ++s) {
    if (hsg_rt_stream_sync(j->streams[s]) != 0) j->fail(-EIO, -1, "device work");
  }
  if (j->hash_acc) {
    const size_t n = j->items.size();
    if (sums && hsg_rt_memcpy_d2h(sums, j->hash_acc, 8 * n) != 0)
      j->fail(-EIO, -1, "hash results");
    g_scratch_pool.release(j->hash_acc);
    j->hash_acc = nullptr;
  }
  j->add(kWall, j->t_start);
  for (auto& it : j->items) {
    if (it.fd >= 0) close(it.fd);
    if (it.allocated || it.ws || it.stage || it.done) release_item(j, it);
  }
  g_upload_pool.release(j->up_base);
  g_scratch_pool.release(j->sc_base);
  g_scratch_pool.release(j->ws_base);
  if (j->st_base) hsg_pinned_release(j->st_base);
  for (void* p : j->slots)
    if (p) hsg_pinned_release(p);
  if (stats)
    for (int k = 0; k < kNumStats; ++k) stats[k] = 1e-9 * double(j->ns[k].load());
  if (bytes_read) *bytes_read = j->bytes_read.load();
  const int e = j->err.load();
  hsg_rt_trace("job-end", j, uint64_t(-e), j->err_item);
  if (err_item) *err_item = j->err_item;
  if (msg) snprintf(msg, 320, "%s", j->errmsg);
  delete j;
  return e;
}

// Warm the pools a restore job is about to draw from, beside the caller's
// planning (a process's first restore paid ~5 ms of uncached / pinned
// allocation in hsg_restore_start and ~7 ms before its first upload):
// `up_bytes` / `sc_bytes` device ring blocks (0: skip), `nslots` pinned slots
// of `slot_bytes`, the copy-table blocks of `table_bytes`, and one small SDMA
// upload (the engine path's first use).  Everything goes back to the pools.
// Returns 0, or -1 if an allocation failed (the job then allocates itself).
int hsg_restore_prewarm(int dev, uint64_t up_bytes, uint64_t sc_bytes, uint64_t slot_bytes,
                        int nslots, uint64_t table_bytes) {
  if (hsg_rt_set_device(dev) != 0) return -1;
  int rc = 0;
  void* up = up_bytes ? g_upload_pool.acquire(dev, up_bytes) : nullptr;
  void* sc = sc_bytes ? g_scratch_pool.acquire(dev, sc_bytes) : nullptr;
  if ((up_bytes && !up) || (sc_bytes && !sc)) rc = -1;
  void* ws = table_bytes ? g_scratch_pool.acquire(dev, table_bytes) : nullptr;
  void* st = table_bytes ? hsg_pinned_acquire(table_bytes) : nullptr;
  std::vector<void*> slots;
  const uint64_t sb = (std::max<uint64_t>(slot_bytes, 1 << 20) + 4095) / 4096 * 4096;
  for (int s = 0; s < nslots; ++s) {
    void* p = hsg_pinned_acquire(sb);
    if (!p) {
      rc = -1;
      break;
    }
    slots.push_back(p);
  }
  void* probe = up ? up : g_upload_pool.acquire(dev, kGranule);
  if (probe && !slots.empty()) {
    uint64_t h = 0;
    if (hsg_sdma_h2d_submit_on(dev, probe, slots[0], 64 << 10, -1, &h) == 0) (void)hsg_sdma_wait(h);
  }
  if (probe != up) g_upload_pool.release(probe);
  for (void* p : slots) hsg_pinned_release(p);
  if (st) hsg_pinned_release(st);
  g_scratch_pool.release(ws);
  g_scratch_pool.release(sc);
  g_upload_pool.release(up);
  return rc;
}

// Free idle device blocks of the restore pools until at most `keep` idle
// bytes remain in each (per call; -1 device = all).  Returns bytes freed.
uint64_t hsg_restore_trim(int dev, uint64_t keep) {
  return g_upload_pool.trim(dev, keep) + g_scratch_pool.trim(dev, keep);
}

// The idle blocks of both pools on `dev` (upload first), at most `max`
// (address, bytes) pairs; returns how many.  For tests that overwrite what a
// restore left in them (a later restore must not depend on those bytes).
int hsg_restore_idle_blocks(int dev, uint64_t* ptrs, uint64_t* sizes, int max) {
  const int n = g_upload_pool.idle(dev, ptrs, sizes, max);
  return n + g_scratch_pool.idle(dev, ptrs + n, sizes + n, max - n);
}

// Device bytes the restore pools hold on `dev` (-1: all devices): out[0..3] =
// upload idle, upload in use, scratch idle, scratch in use.
void hsg_restore_pool_bytes(int dev, uint64_t* out) {
  g_upload_pool.bytes(dev, out, out + 1);
  g_scratch_pool.bytes(dev, out + 2, out + 3);
}

// The same per pool: uncached upload blocks / plain scratch blocks.
uint64_t hsg_restore_trim_pools(int dev, uint64_t keep_upload, uint64_t keep_scratch) {
  return g_upload_pool.trim(dev, keep_upload) + g_scratch_pool.trim(dev, keep_scratch);
}

}  // extern "C"
