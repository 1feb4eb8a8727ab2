// hsio: native file I/O engine for hipsnapshot.
//
// Replaces the reference's aiofiles-based FS plugin
// (/root/reference/torchsnapshot/storage_plugins/fs.py:19-56, one Python thread
// hop per write/read) with a C++ worker pool that issues large pwrite/pread
// calls straight from caller-owned buffers (pinned host staging slots or CPU
// tensor storage) with the GIL never involved.  Completion is reported through
// an eventfd that the Python asyncio loop watches (loop.add_reader), so a
// snapshot with thousands of blobs costs one syscall per blob plus one wakeup
// per batch of completions.
//
// Features:
//   * mkdir -p of parent directories with a directory cache,
//   * optional O_DIRECT for the 4 KiB-aligned body of a write/read (tail goes
//     through a buffered fd), falling back to buffered I/O when the filesystem
//     refuses O_DIRECT (tmpfs, overlayfs),
//   * optional fdatasync for durable checkpoints (the reference never fsyncs),
//   * ranged reads into caller buffers (no intermediate bytes object).
//
// C ABI only (loaded with ctypes) so that it builds without torch headers.

#include <atomic>
#include <cerrno>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <deque>
#include <fcntl.h>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <cstdlib>
#include <sched.h>
#include <sys/eventfd.h>
#include <sys/resource.h>
#include <sys/syscall.h>
#include <sys/stat.h>
#include <sys/types.h>
#include <thread>
#include <unistd.h>
#include <unordered_set>
#include <utility>
#include <vector>

namespace {

constexpr int kFlagDirect = 1;   // try O_DIRECT for the aligned body
constexpr int kFlagSync = 2;     // fdatasync before completing a write
constexpr int kFlagMkdirs = 4;   // create parent directories
constexpr int kFlagAppend = 8;   // write at offset without truncating
// bits 16..23: NUMA node + 1 whose CPUs run the job (0: any).  A blob
// written straight from host pages (a host-resident UVM table) is copied into
// the page cache by the worker's CPU: a worker on the pages' node reads them
// locally.  Unbound, the workers landed on either socket and an 8 GB DLRM
// UVM save spread 36-69 GB/s; bound to the wrong node it ran 30-43
// (profiles/r6/dlrm_var/).
constexpr int kNodeShift = 16;
constexpr size_t kAlign = 4096;
constexpr size_t kMaxIo = size_t(1) << 30;  // keep single syscalls < 2 GiB

enum class Op { kWrite, kRead, kDelete };

// A large read split into sub-reads that run on several workers; the request
// completes (one Completion with the summed byte count, or the first error)
// when its last part finishes.  Buffered reads of one file proceed in
// parallel in the kernel (no exclusive inode lock, unlike buffered writes), so
// with a FIFO queue the first file of a restore arrives at the aggregate
// page-cache bandwidth instead of 1/Nth of it -- consumers (H2D) start early
// and completions are staggered in submission order.
struct Group {
  int64_t id;
  std::atomic<int> remaining;
  std::atomic<int64_t> err{0};
  std::atomic<int64_t> bytes{0};
  Group(int64_t i, int n) : id(i), remaining(n) {}
};

struct Job {
  int64_t id;
  Op op;
  std::string path;
  char* buf;
  size_t nbytes;
  size_t offset;
  int flags;
  std::shared_ptr<Group> group;
};

struct Completion {
  int64_t id;
  int64_t result;  // >=0 bytes transferred, <0 = -errno
};

int64_t full_pwrite(int fd, const char* p, size_t n, size_t off) {
  size_t done = 0;
  while (done < n) {
    size_t chunk = n - done < kMaxIo ? n - done : kMaxIo;
    ssize_t r = ::pwrite(fd, p + done, chunk, static_cast<off_t>(off + done));
    if (r < 0) {
      if (errno == EINTR) continue;
      return -errno;
    }
    if (r == 0) return -EIO;
    done += static_cast<size_t>(r);
  }
  return static_cast<int64_t>(done);
}

int64_t full_pread(int fd, char* p, size_t n, size_t off) {
  size_t done = 0;
  while (done < n) {
    size_t chunk = n - done < kMaxIo ? n - done : kMaxIo;
    ssize_t r = ::pread(fd, p + done, chunk, static_cast<off_t>(off + done));
    if (r < 0) {
      if (errno == EINTR) continue;
      return -errno;
    }
    if (r == 0) break;  // EOF
    done += static_cast<size_t>(r);
  }
  return static_cast<int64_t>(done);
}

class Engine {
 public:
  explicit Engine(int nthreads) {
    CPU_ZERO(&base_mask_);
    have_base_ = ::sched_getaffinity(0, sizeof(base_mask_), &base_mask_) == 0;
    efd_ = ::eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
    if (nthreads < 1) nthreads = 1;
    for (int i = 0; i < nthreads; ++i)
      workers_.emplace_back([this] {
        Run();
      });
  }

  ~Engine() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : workers_) t.join();
    if (efd_ >= 0) ::close(efd_);
  }

  int64_t Submit(Op op, const char* path, char* buf, size_t n, size_t off, int flags) {
    const int64_t id = next_id_.fetch_add(1);
    const size_t split = read_split_.load();
    if (op == Op::kRead && split >= kAlign && n > split + split / 2) {
      const size_t parts = (n + split - 1) / split;
      auto grp = std::make_shared<Group>(id, static_cast<int>(parts));
      {
        std::lock_guard<std::mutex> g(mu_);
        for (size_t i = 0; i < parts; ++i) {
          const size_t lo = i * split;
          const size_t len = (lo + split > n) ? n - lo : split;
          queue_.push_back(Job{0, op, std::string(path), buf + lo, len, off + lo, flags, grp});
        }
      }
      cv_.notify_all();
      return id;
    }
    {
      std::lock_guard<std::mutex> g(mu_);
      queue_.push_back(Job{id, op, std::string(path), buf, n, off, flags, nullptr});
    }
    cv_.notify_one();
    return id;
  }

  void SetReadSplit(size_t bytes) { read_split_.store(bytes / kAlign * kAlign); }

  int Poll(int64_t* ids, int64_t* results, int max) {
    uint64_t v;
    (void)!::read(efd_, &v, sizeof(v));  // reset the counter (non-blocking)
    std::lock_guard<std::mutex> g(cmu_);
    int k = 0;
    while (k < max && !done_.empty()) {
      ids[k] = done_.front().id;
      results[k] = done_.front().result;
      done_.pop_front();
      ++k;
    }
    if (!done_.empty()) {
      uint64_t one = 1;
      (void)!::write(efd_, &one, sizeof(one));  // more left: keep fd readable
    }
    return k;
  }

  int eventfd() const { return efd_; }

  int64_t RunSync(Op op, const char* path, char* buf, size_t n, size_t off, int flags) {
    Job j{0, op, std::string(path), buf, n, off, flags, nullptr};
    return Execute(j);
  }

 private:
  void Run() {
    for (;;) {
      Job j;
      {
        std::unique_lock<std::mutex> g(mu_);
        cv_.wait(g, [this] { return stop_ || !queue_.empty(); });
        if (stop_ && queue_.empty()) return;
        j = std::move(queue_.front());
        queue_.pop_front();
      }
      PlaceFor(((j.flags >> kNodeShift) & 0xff) - 1);
      int64_t r = Execute(j);
      int64_t id = j.id;
      if (j.group) {
        Group& grp = *j.group;
        if (r < 0) {
          int64_t zero = 0;
          grp.err.compare_exchange_strong(zero, r);
        } else {
          grp.bytes.fetch_add(r);
        }
        if (grp.remaining.fetch_sub(1) != 1) continue;  // not the last part
        id = grp.id;
        r = grp.err.load() < 0 ? grp.err.load() : grp.bytes.load();
      }
      {
        std::lock_guard<std::mutex> g(cmu_);
        done_.push_back({id, r});
      }
      uint64_t one = 1;
      (void)!::write(efd_, &one, sizeof(one));
    }
  }

  // Run this worker on `node`'s CPUs (within the engine's original mask), or
  // back on the original mask for node -1.  Kept until a job asks otherwise.
  void PlaceFor(int node) {
    thread_local int placed = -1;
    if (node == placed || !have_base_) return;
    cpu_set_t m;
    if (node < 0) {
      m = base_mask_;
    } else {
      if (!NodeMask(node, &m)) return;
      CPU_AND(&m, &m, &base_mask_);
      if (CPU_COUNT(&m) == 0) return;
    }
    if (::sched_setaffinity(0, sizeof(m), &m) == 0) placed = node;
  }

  bool NodeMask(int node, cpu_set_t* out) {
    std::lock_guard<std::mutex> g(nmu_);
    auto it = node_masks_.find(node);
    if (it == node_masks_.end()) {
      cpu_set_t m;
      CPU_ZERO(&m);
      char path[96];
      snprintf(path, sizeof(path), "/sys/devices/system/node/node%d/cpulist", node);
      bool ok = false;
      if (FILE* f = fopen(path, "r")) {
        char buf[4096];
        if (fgets(buf, sizeof(buf), f)) {
          ok = true;
          for (char* tok = strtok(buf, ",\n"); tok; tok = strtok(nullptr, ",\n")) {
            int a = -1, b = -1;
            if (sscanf(tok, "%d-%d", &a, &b) == 2) {
              for (int c = a; c <= b && c < CPU_SETSIZE; ++c) CPU_SET(c, &m);
            } else if (sscanf(tok, "%d", &a) == 1 && a >= 0 && a < CPU_SETSIZE) {
              CPU_SET(a, &m);
            }
          }
        }
        fclose(f);
      }
      it = node_masks_.emplace(node, std::make_pair(ok, m)).first;
    }
    *out = it->second.second;
    return it->second.first;
  }

  int MkdirsFor(const std::string& path) {
    size_t slash = path.rfind('/');
    if (slash == std::string::npos || slash == 0) return 0;
    std::string dir = path.substr(0, slash);
    {
      std::lock_guard<std::mutex> g(dmu_);
      if (dirs_.count(dir)) return 0;
    }
    std::string cur;
    size_t pos = 0;
    while (pos != std::string::npos) {
      pos = dir.find('/', pos + 1);
      cur = dir.substr(0, pos);
      if (cur.empty()) continue;
      if (::mkdir(cur.c_str(), 0755) != 0 && errno != EEXIST) return -errno;
    }
    std::lock_guard<std::mutex> g(dmu_);
    dirs_.insert(dir);
    return 0;
  }

  void ForgetDirOf(const std::string& path) {
    size_t slash = path.rfind('/');
    if (slash == std::string::npos) return;
    std::lock_guard<std::mutex> g(dmu_);
    dirs_.erase(path.substr(0, slash));
  }

  int64_t Execute(const Job& j) {
    switch (j.op) {
      case Op::kWrite: return DoWrite(j);
      case Op::kRead: return DoRead(j);
      case Op::kDelete: return ::unlink(j.path.c_str()) == 0 ? 0 : -errno;
    }
    return -EINVAL;
  }

  int64_t DoWrite(const Job& j) {
    if (j.flags & kFlagMkdirs) {
      int r = MkdirsFor(j.path);
      if (r < 0) return r;
    }
    // Overwrite in place instead of O_TRUNC: re-taking a snapshot to the same
    // path then rewrites the page-cache pages it already owns (truncating and
    // re-allocating 16 GB of page cache costs ~1 s per take on a 3 TB host);
    // the stale tail, if any, is cut with ftruncate below.
    int oflags = O_WRONLY | O_CREAT | O_CLOEXEC;
    int fd = ::open(j.path.c_str(), oflags, 0644);
    if (fd < 0 && errno == ENOENT && (j.flags & kFlagMkdirs)) {
      // the cached parent was removed since (e.g. a directory of a previous
      // take deleted by its successor): forget it, recreate, retry once
      ForgetDirOf(j.path);
      int r = MkdirsFor(j.path);
      if (r < 0) return r;
      fd = ::open(j.path.c_str(), oflags, 0644);
    }
    if (fd < 0) return -errno;
    int64_t res = 0;
    size_t body = 0;
    bool aligned = (reinterpret_cast<uintptr_t>(j.buf) % kAlign == 0) && (j.offset % kAlign == 0);
    if ((j.flags & kFlagDirect) && aligned && j.nbytes >= kAlign) {
      body = j.nbytes / kAlign * kAlign;
      int dfd = ::open(j.path.c_str(), O_WRONLY | O_CLOEXEC | O_DIRECT);
      if (dfd >= 0) {
        res = full_pwrite(dfd, j.buf, body, j.offset);
        ::close(dfd);
        if (res < 0) body = 0;  // retry everything buffered below
      } else {
        body = 0;  // filesystem without O_DIRECT support
      }
    }
    res = full_pwrite(fd, j.buf + body, j.nbytes - body, j.offset + body);
    if (res >= 0 && !(j.flags & kFlagAppend) && j.offset == 0) {
      struct stat st;
      if (::fstat(fd, &st) == 0 && static_cast<size_t>(st.st_size) != j.nbytes) {
        if (::ftruncate(fd, static_cast<off_t>(j.nbytes)) != 0) res = -errno;
      }
    }
    if (res >= 0 && (j.flags & kFlagSync)) {
      if (::fdatasync(fd) != 0) res = -errno;
    }
    ::close(fd);
    return res < 0 ? res : static_cast<int64_t>(j.nbytes);
  }

  int64_t DoRead(const Job& j) {
    int fd = ::open(j.path.c_str(), O_RDONLY | O_CLOEXEC);
    if (fd < 0) return -errno;
    size_t body = 0;
    int64_t got = 0;
    bool aligned = (reinterpret_cast<uintptr_t>(j.buf) % kAlign == 0) && (j.offset % kAlign == 0);
    if ((j.flags & kFlagDirect) && aligned && j.nbytes >= kAlign) {
      body = j.nbytes / kAlign * kAlign;
      int dfd = ::open(j.path.c_str(), O_RDONLY | O_CLOEXEC | O_DIRECT);
      if (dfd >= 0) {
        got = full_pread(dfd, j.buf, body, j.offset);
        ::close(dfd);
        if (got < 0 || static_cast<size_t>(got) != body) { body = 0; got = 0; }
      } else {
        body = 0;
      }
    }
    int64_t r = full_pread(fd, j.buf + body, j.nbytes - body, j.offset + body);
    ::close(fd);
    if (r < 0) return r;
    return static_cast<int64_t>(body) + r;
  }

  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<Job> queue_;
  bool stop_ = false;
  std::vector<std::thread> workers_;
  std::atomic<int64_t> next_id_{1};
  std::atomic<size_t> read_split_{size_t(8) << 20};
  std::mutex cmu_;
  std::deque<Completion> done_;
  std::mutex dmu_;
  std::unordered_set<std::string> dirs_;
  cpu_set_t base_mask_;  // the creating thread's CPUs (the workers' default)
  bool have_base_ = false;
  std::mutex nmu_;
  std::map<int, std::pair<bool, cpu_set_t>> node_masks_;
  int efd_ = -1;
};

}  // namespace

extern "C" {

void* hsio_create(int nthreads) { return new Engine(nthreads); }
void hsio_destroy(void* e) { delete static_cast<Engine*>(e); }
int hsio_eventfd(void* e) { return static_cast<Engine*>(e)->eventfd(); }

// Reads larger than 1.5x this many bytes are split across workers (0 = never).
void hsio_set_read_split(void* e, uint64_t bytes) {
  static_cast<Engine*>(e)->SetReadSplit(bytes);
}

int64_t hsio_submit_write(void* e, const char* path, const void* buf, uint64_t n,
                          uint64_t off, int flags) {
  return static_cast<Engine*>(e)->Submit(Op::kWrite, path,
                                         const_cast<char*>(static_cast<const char*>(buf)),
                                         n, off, flags);
}

int64_t hsio_submit_read(void* e, const char* path, void* buf, uint64_t n, uint64_t off,
                         int flags) {
  return static_cast<Engine*>(e)->Submit(Op::kRead, path, static_cast<char*>(buf), n, off,
                                         flags);
}

int64_t hsio_submit_delete(void* e, const char* path) {
  return static_cast<Engine*>(e)->Submit(Op::kDelete, path, nullptr, 0, 0, 0);
}

int hsio_poll(void* e, int64_t* ids, int64_t* results, int max) {
  return static_cast<Engine*>(e)->Poll(ids, results, max);
}

// Blocking variants (used by the synchronous metadata path and tests).
int64_t hsio_write_sync(void* e, const char* path, const void* buf, uint64_t n,
                        uint64_t off, int flags) {
  return static_cast<Engine*>(e)->RunSync(
      Op::kWrite, path, const_cast<char*>(static_cast<const char*>(buf)), n, off, flags);
}

int64_t hsio_read_sync(void* e, const char* path, void* buf, uint64_t n, uint64_t off,
                       int flags) {
  return static_cast<Engine*>(e)->RunSync(Op::kRead, path, static_cast<char*>(buf), n, off,
                                          flags);
}

int64_t hsio_file_size(const char* path) {
  struct stat st;
  if (::stat(path, &st) != 0) return -errno;
  return static_cast<int64_t>(st.st_size);
}

// Page-aligned anonymous host allocation for CPU-only staging (no HIP needed).
void* hsio_alloc_aligned(uint64_t n) {
  void* p = nullptr;
  if (posix_memalign(&p, kAlign, n ? n : kAlign) != 0) return nullptr;
  return p;
}
void hsio_free_aligned(void* p) { free(p); }

// Multi-threaded memcpy for large host->host staging copies (async snapshot of
// CPU tensors); a single core tops out around 10-12 GB/s.
void hsio_parallel_memcpy(void* dst, const void* src, uint64_t n, int nthreads) {
  if (nthreads <= 1 || n < (uint64_t(32) << 20)) {
    std::memcpy(dst, src, n);
    return;
  }
  std::vector<std::thread> ts;
  uint64_t per = (n / nthreads + 4095) / 4096 * 4096;
  for (int i = 0; i < nthreads; ++i) {
    uint64_t lo = per * i;
    if (lo >= n) break;
    uint64_t len = (lo + per > n) ? n - lo : per;
    ts.emplace_back([=] {
      std::memcpy(static_cast<char*>(dst) + lo, static_cast<const char*>(src) + lo, len);
    });
  }
  for (auto& t : ts) t.join();
}

}  // extern "C"
