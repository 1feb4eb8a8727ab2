// hsfmap: checkpoint files the GPU's copy engines write directly.
//
// A buffered write of a blob costs the host one CPU copy of every stored
// byte -- SDMA into a pinned buffer, then pwrite() copies it into the page
// cache: three passes over DRAM and ~80-100 ms of CPU per GiB
// (profiles/r5/filemap/).  With N ranks per node that copy, not the PCIe
// links, bounds a checkpoint.  The page cache pages of a file can instead be
// mapped (MAP_SHARED) and registered with the GPU (hipHostRegister): the
// SDMA engines then write the blob into the file pages themselves, at the
// PCIe rate, and the host only re-dirties each page afterwards (a DMA write
// does not mark a page dirty for writeback): ~3 ms per GiB.
//
// Registration costs ~30 ms per GiB for a file whose pages are cached and
// 100-180 ms for a new file (the kernel allocates and zeroes every page),
// more than pwrite's copy, so only EXISTING files of the blob's exact size
// are mapped -- the rewrite a training job does every checkpoint into the
// same path -- and mappings are kept across takes: a later take pays only
// the DMA and the re-dirty pass.  A cached mapping is reused only while the
// path still names the same, unmodified file (device, inode, size, and the
// change time recorded after our own last commit: any write or truncate by
// someone else invalidates it); anything else drops it.  Mappings are bounded
// by a byte budget (least recently used go first).
//
// Host code only (the HIP registration sits behind hshost.hip hooks), so it
// builds against the CPU stubs of tests/native/engine_stubs.cpp too.

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <cstdint>
#include <cstring>
#include <list>
#include <mutex>
#include <string>
#include <unordered_map>

extern "C" {
int hsg_rt_host_register(void* p, uint64_t n);
int hsg_rt_host_unregister(void* p);
}

namespace {

constexpr uint64_t kPage = 4096;

bool same_time(const struct timespec& a, const struct timespec& b) {
  return a.tv_sec == b.tv_sec && a.tv_nsec == b.tv_nsec;
}

// the path still names the mapped file, unmodified since our last commit
bool unchanged(const struct stat& st, const struct Mapping* m);

struct Mapping {
  std::string path;
  int fd = -1;
  char* addr = nullptr;
  uint64_t size = 0;
  dev_t dev = 0;
  ino_t ino = 0;
  struct timespec ctim = {0, 0};  // st_ctim after our last commit
  int busy = 0;  // acquired and not yet committed / abandoned
};

struct Cache {
  std::mutex mu;
  std::list<Mapping*> lru;  // front = most recently used
  std::unordered_map<std::string, std::list<Mapping*>::iterator> by_path;
  std::unordered_map<void*, Mapping*> by_addr;
  uint64_t bytes = 0;
  uint64_t budget = uint64_t(64) << 30;
  uint64_t hits = 0, maps = 0, drops = 0, misses = 0;
};

Cache g;

bool unchanged(const struct stat& st, const Mapping* m) {
  return S_ISREG(st.st_mode) && st.st_dev == m->dev && st.st_ino == m->ino &&
         uint64_t(st.st_size) == m->size && same_time(st.st_ctim, m->ctim);
}

void unmap(Mapping* m) {
  if (m->addr) {
    (void)hsg_rt_host_unregister(m->addr);
    munmap(m->addr, m->size);
  }
  if (m->fd >= 0) close(m->fd);
  delete m;
}

// caller holds g.mu; unlinks m from the cache and returns it for unmap()
Mapping* detach_locked(std::unordered_map<std::string, std::list<Mapping*>::iterator>::iterator it) {
  Mapping* m = *it->second;
  g.lru.erase(it->second);
  g.by_path.erase(it);
  g.by_addr.erase(m->addr);
  g.bytes -= m->size;
  ++g.drops;
  return m;
}

// Drop idle mappings, least recently used first, until `need` more bytes fit.
void evict_for(uint64_t need, std::list<Mapping*>* out) {
  auto it = g.lru.end();
  while (g.bytes + need > g.budget && it != g.lru.begin()) {
    --it;
    Mapping* m = *it;
    if (m->busy) continue;
    auto after = std::next(it);  // stays valid when `it` is erased
    out->push_back(detach_locked(g.by_path.find(m->path)));
    it = after;
  }
}

}  // namespace

extern "C" {

// A GPU-writable mapping of the existing file `path` if it is exactly
// `nbytes` long: returns its address (and marks it busy until
// hsg_fmap_commit / hsg_fmap_abandon), or null when the file is missing,
// has another size, nbytes == 0, or mapping / registering failed -- the
// caller then writes the blob the buffered way.
void* hsg_fmap_acquire(const char* path, uint64_t nbytes) {
  if (nbytes == 0) return nullptr;
  struct stat st;
  const bool exists = stat(path, &st) == 0 && S_ISREG(st.st_mode);
  std::list<Mapping*> drop;
  void* out = nullptr;
  {
    std::lock_guard<std::mutex> lk(g.mu);
    auto it = g.by_path.find(path);
    if (it != g.by_path.end()) {
      Mapping* m = *it->second;
      if (m->busy) {
        ++g.misses;
        return nullptr;  // another writer of this path is in flight
      }
      if (exists && m->size == nbytes && unchanged(st, m)) {
        g.lru.splice(g.lru.begin(), g.lru, it->second);
        m->busy = 1;
        ++g.hits;
        return m->addr;
      }
      drop.push_back(detach_locked(it));  // the path names another file now
    }
    if (!exists || uint64_t(st.st_size) != nbytes || nbytes > g.budget) {
      ++g.misses;
      for (Mapping* m : drop) unmap(m);
      return nullptr;
    }
    evict_for(nbytes, &drop);
  }
  for (Mapping* m : drop) unmap(m);
  // map and register outside the lock (tens of ms per GiB)
  Mapping* m = new Mapping();
  m->path = path;
  m->size = nbytes;
  m->fd = open(path, O_RDWR | O_CLOEXEC);
  struct stat fst;
  if (m->fd < 0 || fstat(m->fd, &fst) != 0 || uint64_t(fst.st_size) != nbytes) {
    unmap(m);
    return nullptr;
  }
  m->dev = fst.st_dev;
  m->ino = fst.st_ino;
  m->ctim = fst.st_ctim;
  void* p = mmap(nullptr, nbytes, PROT_READ | PROT_WRITE, MAP_SHARED, m->fd, 0);
  if (p == MAP_FAILED) {
    unmap(m);
    return nullptr;
  }
  m->addr = static_cast<char*>(p);
  if (hsg_rt_host_register(m->addr, nbytes) != 0) {
    munmap(m->addr, nbytes);
    m->addr = nullptr;
    unmap(m);
    return nullptr;
  }
  m->busy = 1;
  {
    std::lock_guard<std::mutex> lk(g.mu);
    if (g.by_path.count(path)) {  // raced with another acquire of the same path
      m->busy = 0;
      drop.clear();
      drop.push_back(m);
    } else {
      g.lru.push_front(m);
      g.by_path[m->path] = g.lru.begin();
      g.by_addr[m->addr] = m;
      g.bytes += nbytes;
      ++g.maps;
      out = m->addr;
    }
  }
  if (!out)
    for (Mapping* d : drop) unmap(d);
  return out;
}

// The copy into `addr` (from hsg_fmap_acquire) has completed: mark every page
// of the file dirty (one CPU store per page of the byte it already holds) so
// writeback persists what the DMA wrote, optionally fdatasync() the file, and
// release the mapping for later takes.  Returns 0 or -errno.
int hsg_fmap_commit(void* addr, int sync) {
  Mapping* m = nullptr;
  {
    std::lock_guard<std::mutex> lk(g.mu);
    auto it = g.by_addr.find(addr);
    if (it != g.by_addr.end() && it->second->busy) m = it->second;
  }
  if (!m) return -EINVAL;
  volatile char* p = m->addr;
  for (uint64_t off = 0; off < m->size; off += kPage) p[off] = p[off];
  int rc = 0;
  if (sync && fdatasync(m->fd) != 0) rc = -errno;
  struct stat st;
  const bool ok = fstat(m->fd, &st) == 0;
  std::lock_guard<std::mutex> lk(g.mu);
  if (ok)
    m->ctim = st.st_ctim;  // our own stores changed it
  else
    m->ctim = {0, 0};  // unknown: the next acquire remaps
  m->busy = 0;
  return rc;
}

// The copy into `addr` failed or was never started: release the mapping (the
// file keeps whatever it held; the caller writes the blob another way).
void hsg_fmap_abandon(void* addr) {
  std::lock_guard<std::mutex> lk(g.mu);
  auto it = g.by_addr.find(addr);
  if (it != g.by_addr.end()) it->second->busy = 0;
}

// Unmap every idle mapping (all = 1: every mapping; call only with no copy in
// flight).  Returns the bytes released.
uint64_t hsg_fmap_release(int all) {
  std::list<Mapping*> drop;
  uint64_t freed = 0;
  {
    std::lock_guard<std::mutex> lk(g.mu);
    for (auto it = g.by_path.begin(); it != g.by_path.end();) {
      Mapping* m = *it->second;
      if (m->busy && !all) {
        ++it;
        continue;
      }
      freed += m->size;
      auto nx = std::next(it);
      drop.push_back(detach_locked(it));
      it = nx;
    }
  }
  for (Mapping* m : drop) unmap(m);
  return freed;
}

// Drop idle mappings whose path no longer names their file (deleted,
// replaced or resized): their pinned pages would otherwise outlive the file.
uint64_t hsg_fmap_prune() {
  std::list<Mapping*> drop;
  uint64_t freed = 0;
  {
    std::lock_guard<std::mutex> lk(g.mu);
    for (auto it = g.by_path.begin(); it != g.by_path.end();) {
      Mapping* m = *it->second;
      struct stat st;
      const bool same = stat(m->path.c_str(), &st) == 0 && unchanged(st, m);
      if (m->busy || same) {
        ++it;
        continue;
      }
      freed += m->size;
      auto nx = std::next(it);
      drop.push_back(detach_locked(it));
      it = nx;
    }
  }
  for (Mapping* m : drop) unmap(m);
  return freed;
}

void hsg_fmap_set_budget(uint64_t bytes) {
  std::list<Mapping*> drop;
  {
    std::lock_guard<std::mutex> lk(g.mu);
    g.budget = bytes;
    evict_for(0, &drop);
  }
  for (Mapping* m : drop) unmap(m);
}

// [bytes mapped, mappings, hits, new mappings, drops, misses]
void hsg_fmap_stats(uint64_t* out) {
  std::lock_guard<std::mutex> lk(g.mu);
  out[0] = g.bytes;
  out[1] = g.lru.size();
  out[2] = g.hits;
  out[3] = g.maps;
  out[4] = g.drops;
  out[5] = g.misses;
}

}  // extern "C"
