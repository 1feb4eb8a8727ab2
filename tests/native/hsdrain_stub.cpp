// Host-only stand-in for the _hsgpu.so entry points the drain helper
// (hipsnapshot/csrc/hsdrain_helper.cpp) binds, so the helper's request
// parsing, mapping cache and reply framing can run under ASan/UBSan on a
// machine without a GPU (tests/test_native_sanitizers.py):
//   * hsg_ipc_open maps a handle whose first byte is 0xAB to a 1 MiB host
//     buffer holding byte i = i * 7 + 3 (anything else: no mapping);
//   * hsg_drain_start writes each "device" range to its file synchronously
//     and records the byte sum as the blob's hash; hsg_drain_wait reports it.

#include <fcntl.h>
#include <unistd.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

namespace {

constexpr uint64_t kArena = 1 << 20;
uint8_t* g_arena = nullptr;
int g_open_maps = 0;

struct Job {
  std::vector<uint64_t> sums;
  uint64_t written = 0;
  int err = 0;
};

}  // namespace

extern "C" {

const char* hsg_last_error() { return "stub: no such mapping"; }

int hsg_init_device(int) { return 0; }

void* hsg_ipc_open(int, const void* handle) {
  if (static_cast<const uint8_t*>(handle)[0] != 0xAB) return nullptr;
  if (!g_arena) {
    g_arena = new uint8_t[kArena];
    for (uint64_t i = 0; i < kArena; ++i) g_arena[i] = static_cast<uint8_t>(i * 7 + 3);
  }
  ++g_open_maps;
  return g_arena;
}

int hsg_ipc_close(void* p) {
  if (p != g_arena || g_open_maps <= 0) return -1;
  if (--g_open_maps == 0) {
    delete[] g_arena;
    g_arena = nullptr;
  }
  return 0;
}

void* hsg_drain_start(int, int n, const uint64_t* srcs, const uint64_t* sizes,
                      const char* const* paths, uint64_t, int, int, int, int, int* err) {
  *err = 0;
  Job* j = new Job();
  j->sums.assign(n, 0);
  for (int i = 0; i < n; ++i) {
    const uint8_t* p = reinterpret_cast<const uint8_t*>(srcs[i]);
    if (p < g_arena || p + sizes[i] > g_arena + kArena) {
      j->err = -14;  // EFAULT: outside the mapped arena
      continue;
    }
    const int fd = open(paths[i], O_WRONLY | O_CREAT | O_TRUNC, 0644);
    if (fd < 0) {
      j->err = -2;
      continue;
    }
    uint64_t s = 0;
    for (uint64_t k = 0; k < sizes[i]; ++k) s += p[k];
    j->sums[i] = s;
    const ssize_t w = write(fd, p, sizes[i]);
    close(fd);
    if (w != static_cast<ssize_t>(sizes[i])) j->err = -5;
    else j->written += sizes[i];
  }
  return j;
}

int hsg_drain_wait(void* handle, uint64_t* sums, uint64_t* bytes_written, char* msg,
                   double* stats) {
  Job* j = static_cast<Job*>(handle);
  if (sums)
    for (size_t i = 0; i < j->sums.size(); ++i) sums[i] = j->sums[i];
  if (bytes_written) *bytes_written = j->written;
  if (msg) snprintf(msg, 256, "%s", j->err ? "stub drain failed" : "");
  if (stats)
    for (int k = 0; k < 9; ++k) stats[k] = 0.001 * k;
  const int e = j->err;
  delete j;
  return e;
}

}  // extern "C"
