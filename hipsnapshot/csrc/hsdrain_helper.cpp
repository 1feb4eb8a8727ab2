// hsdrain_helper: a drain process beside the trainer.
//
// The in-process native drain (hsdrain.hip) already moves an async take's
// frozen HBM arena to files without Python, but its SDMA submits, hash
// launches, pinned-slot management and pwrite() memcpy still run inside the
// trainer's process: they share its HIP runtime (device/stream locks taken
// by every kernel launch), its allocator arenas and its address space with
// a launch-bound training loop.  A step at seq 512 (~200 ms, launch-bound)
// ran 3-8 % slower while a drain was in flight, where the same bytes drained
// from ANOTHER process cost the trainer ~1.6 % (profiles/overlap_iso).
//
// This program is that other process.  The trainer's Python side
// (engine/drain_process.py) starts it once, as a child, and sends it drain
// jobs over a pipe:
//
//   * the arena's allocation is exported with hipIpcGetMemHandle (dmabuf
//     IPC) and mapped here once; the mapping is cached while the trainer
//     keeps the arena between takes, and closed when the trainer says so;
//   * the job (blob offsets / sizes / paths and the drain settings) runs
//     through the SAME hsg_drain_start / hsg_drain_wait code as in process;
//   * the reply carries the per-blob hs64 partial sums, bytes written, the
//     per-phase seconds and any error text.
//
// No HIP headers here: the HIP runtime the trainer uses (its path is argv[1],
// read from the trainer's /proc/self/maps) is dlopen'ed RTLD_GLOBAL before
// _hsgpu.so (argv[2]), exactly as torch + ctypes do in the trainer, so both
// processes run the same runtime and kernels.
//
// Wire format (native endianness, one request -> one reply):
//   request: u32 magic 'HSDH', u32 op
//     op 1 DRAIN: i32 dev, u32 hlen, u8 handle[hlen], u64 slot_bytes,
//                 i32 nslots, i32 nwriters, i32 flags, i32 max_hash_grid,
//                 u32 close_after, u32 n, n x {u64 offset, u64 nbytes,
//                 u32 plen, char path[plen]}
//       replies:  i32 mapped (0, or -10000: the arena could not be mapped),
//                 then i32 rc, u64 written, u32 n, u64 sums[n], u32 nstats,
//                 f64 stats[nstats], f64 map_s, u32 mlen, char msg[mlen]
//     op 2 CLOSE: u32 hlen, u8 handle[hlen]        reply: i32 rc
//     op 3 PING:                                   reply: i32 0, i32 pid
//   EOF on stdin (the trainer exited or closed the pipe) ends the process.
//
// Reference behaviour this serves: the background commit of an async
// snapshot, `/root/reference/torchsnapshot/snapshot.py:891-933`.

#include <dlfcn.h>
#include <unistd.h>

#include <chrono>
#include <cstdlib>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <vector>

namespace {

constexpr uint32_t kMagic = 0x48534448;  // "HSDH"
constexpr int kNumStats = 9;             // hsdrain.hip: enum Stat

using drain_start_t = void* (*)(int, int, const uint64_t*, const uint64_t*, const char* const*,
                                uint64_t, int, int, int, int, int*);
using drain_wait_t = int (*)(void*, uint64_t*, uint64_t*, char*, double*);
using ipc_open_t = void* (*)(int, const void*);
using ipc_close_t = int (*)(void*);
using last_error_t = const char* (*)();
using init_device_t = int (*)(int);

drain_start_t drain_start;
drain_wait_t drain_wait;
ipc_open_t ipc_open;
ipc_close_t ipc_close;
last_error_t last_error;
init_device_t init_device;
int g_ready_dev = -1;  // device whose runtime context is up

bool read_all(void* p, size_t n) {
  char* c = static_cast<char*>(p);
  while (n) {
    const ssize_t r = read(0, c, n);
    if (r <= 0) return false;
    c += r;
    n -= static_cast<size_t>(r);
  }
  return true;
}

struct Out {
  std::vector<char> buf;
  template <class T>
  void put(const T& v) {
    const char* c = reinterpret_cast<const char*>(&v);
    buf.insert(buf.end(), c, c + sizeof(T));
  }
  void put_bytes(const void* p, size_t n) {
    const char* c = static_cast<const char*>(p);
    buf.insert(buf.end(), c, c + n);
  }
  bool flush() {
    const char* c = buf.data();
    size_t n = buf.size();
    while (n) {
      const ssize_t w = write(1, c, n);
      if (w <= 0) return false;
      c += w;
      n -= static_cast<size_t>(w);
    }
    buf.clear();
    return true;
  }
};

template <class T>
bool get(T* v) {
  return read_all(v, sizeof(T));
}

bool get_string(std::string* s) {
  uint32_t n = 0;
  if (!get(&n) || n > (1u << 20)) return false;
  s->resize(n);
  return n == 0 || read_all(&(*s)[0], n);
}

std::map<std::string, std::pair<int, void*>> g_maps;  // handle bytes -> (dev, base)

void* mapping(int dev, const std::string& handle) {
  auto it = g_maps.find(handle);
  if (it != g_maps.end()) return it->second.second;
  void* base = ipc_open(dev, handle.data());
  if (base) g_maps[handle] = {dev, base};
  return base;
}

void unmap(const std::string& handle) {
  auto it = g_maps.find(handle);
  if (it == g_maps.end()) return;
  ipc_close(it->second.second);
  g_maps.erase(it);
}

bool g_debug = false;  // HIPSNAPSHOT_DRAIN_HELPER_DEBUG: stage markers on stderr

void dbg(const char* what) {
  if (g_debug) {
    fprintf(stderr, "hsdrain_helper[%d]: %s\n", static_cast<int>(getpid()), what);
    fflush(stderr);
  }
}

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

bool do_drain(Out* out) {
  int32_t dev = 0, nslots = 0, nwriters = 0, flags = 0, grid = 0;
  uint64_t slot_bytes = 0;
  uint32_t close_after = 0, n = 0;
  std::string handle;
  if (!get(&dev) || !get_string(&handle) || !get(&slot_bytes) || !get(&nslots) ||
      !get(&nwriters) || !get(&flags) || !get(&grid) || !get(&close_after) || !get(&n))
    return false;
  std::vector<uint64_t> offs(n), sizes(n);
  std::vector<std::string> paths(n);
  for (uint32_t i = 0; i < n; ++i)
    if (!get(&offs[i]) || !get(&sizes[i]) || !get_string(&paths[i])) return false;

  if (g_ready_dev != dev) {
    dbg("drain: runtime init");
    if (init_device(dev) == 0) g_ready_dev = dev;
    dbg("drain: runtime ready");
  }
  dbg("drain: mapping the arena");
  const double t0 = now_s();
  void* base = mapping(dev, handle);
  const double map_s = now_s() - t0;
  dbg(base ? "drain: mapped, starting" : "drain: mapping failed");
  // interim reply: the mapping outcome, before the (long) drain runs -- the
  // trainer bounds this wait separately and drains in process on a stall
  out->put(static_cast<int32_t>(base ? 0 : -10000));
  if (!out->flush()) return false;
  int32_t rc = 0;
  uint64_t written = 0;
  std::vector<uint64_t> sums(n, 0);
  double stats[kNumStats] = {0};
  char msg[256] = {0};
  if (!base) {
    rc = -10000;
    snprintf(msg, sizeof(msg), "drain helper: mapping the arena failed: %s", last_error());
  } else {
    std::vector<uint64_t> srcs(n);
    std::vector<const char*> cpaths(n);
    for (uint32_t i = 0; i < n; ++i) {
      srcs[i] = reinterpret_cast<uint64_t>(base) + offs[i];
      cpaths[i] = paths[i].c_str();
    }
    int err = 0;
    void* job = drain_start(dev, static_cast<int>(n), srcs.data(), sizes.data(), cpaths.data(),
                            slot_bytes, nslots, nwriters, flags, grid, &err);
    if (!job) {
      rc = -10001;
      snprintf(msg, sizeof(msg), "drain helper: hsg_drain_start failed (%d): %s", err,
               last_error());
    } else {
      dbg("drain: started, waiting");
      rc = drain_wait(job, sums.data(), &written, msg, stats);
      dbg("drain: done");
    }
  }
  if (close_after) unmap(handle);
  out->put(rc);
  out->put(written);
  out->put(n);
  out->put_bytes(sums.data(), n * sizeof(uint64_t));
  out->put(static_cast<uint32_t>(kNumStats));
  out->put_bytes(stats, sizeof(stats));
  out->put(map_s);
  const uint32_t mlen = static_cast<uint32_t>(strnlen(msg, sizeof(msg)));
  out->put(mlen);
  out->put_bytes(msg, mlen);
  return out->flush();
}

template <class F>
bool sym(void* lib, const char* name, F* fn) {
  *fn = reinterpret_cast<F>(dlsym(lib, name));
  if (!*fn) fprintf(stderr, "hsdrain_helper: missing symbol %s\n", name);
  return *fn != nullptr;
}

}  // namespace

int main(int argc, char** argv) {
  g_debug = getenv("HIPSNAPSHOT_DRAIN_HELPER_DEBUG") != nullptr;
  dbg("started");
  if (argc < 3) {
    fprintf(stderr, "usage: hsdrain_helper <libamdhip64 path> <_hsgpu.so path>\n");
    return 2;
  }
  if (!dlopen(argv[1], RTLD_NOW | RTLD_GLOBAL)) {
    fprintf(stderr, "hsdrain_helper: %s\n", dlerror());
    return 2;
  }
  dbg("HIP runtime loaded");
  void* lib = dlopen(argv[2], RTLD_NOW);
  if (!lib) {
    fprintf(stderr, "hsdrain_helper: %s\n", dlerror());
    return 2;
  }
  if (!sym(lib, "hsg_drain_start", &drain_start) || !sym(lib, "hsg_drain_wait", &drain_wait) ||
      !sym(lib, "hsg_ipc_open", &ipc_open) || !sym(lib, "hsg_ipc_close", &ipc_close) ||
      !sym(lib, "hsg_last_error", &last_error) || !sym(lib, "hsg_init_device", &init_device))
    return 2;
  dbg("libraries loaded, serving");
  Out out;
  for (;;) {
    uint32_t magic = 0, op = 0;
    if (!get(&magic) || !get(&op)) break;  // EOF: the trainer is gone
    if (magic != kMagic) {
      fprintf(stderr, "hsdrain_helper: bad request magic %08x\n", magic);
      return 3;
    }
    bool ok = true;
    if (op == 1) {
      ok = do_drain(&out);
    } else if (op == 2) {
      std::string handle;
      ok = get_string(&handle);
      if (ok) {
        unmap(handle);
        out.put(static_cast<int32_t>(0));
        ok = out.flush();
      }
    } else if (op == 3) {
      out.put(static_cast<int32_t>(0));
      out.put(static_cast<int32_t>(getpid()));
      ok = out.flush();
    } else {
      fprintf(stderr, "hsdrain_helper: unknown op %u\n", op);
      return 3;
    }
    if (!ok) break;
  }
  for (auto& kv : g_maps) ipc_close(kv.second.second);
  return 0;
}
