// HBM -> HBM contiguous copy: the freeze kernel's byte path (hs_copy_nd,
// flags & 1: 1 MiB tiles, persistent grid, 4 x 16-B loads in flight per lane)
// against variants -- non-temporal loads / stores, 8 loads in flight, a
// larger grid.  Standalone (no torch): 2 x 8 GiB buffers, best of 5 event-timed
// runs per variant.
//
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/copy_variants scripts/probes/copy_variants.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

constexpr int kBlock = 256;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int INFLIGHT, bool NT>
__global__ void __launch_bounds__(kBlock)
copy_tiles(const u32x4* __restrict__ src, u32x4* __restrict__ dst, int64_t nvec,
           int64_t tile_vec) {
  const int64_t ntiles = (nvec + tile_vec - 1) / tile_vec;
  for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int64_t b = t * tile_vec;
    const int64_t e = b + tile_vec < nvec ? b + tile_vec : nvec;
    const u32x4* s = src + b;
    u32x4* d = dst + b;
    const int64_t n = e - b;
    int64_t i = threadIdx.x;
    for (; i + (INFLIGHT - 1) * kBlock < n; i += INFLIGHT * kBlock) {
      u32x4 r[INFLIGHT];
#pragma unroll
      for (int k = 0; k < INFLIGHT; ++k)
        r[k] = NT ? __builtin_nontemporal_load(s + i + k * kBlock) : s[i + k * kBlock];
#pragma unroll
      for (int k = 0; k < INFLIGHT; ++k) {
        if (NT) __builtin_nontemporal_store(r[k], d + i + k * kBlock);
        else d[i + k * kBlock] = r[k];
      }
    }
    for (; i < n; i += kBlock) d[i] = s[i];
  }
}

template <int INFLIGHT, bool NT>
float run(const u32x4* s, u32x4* d, int64_t nvec, int64_t tile_vec, int grid, hipStream_t st) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  float best = 1e30f;
  for (int it = 0; it < 6; ++it) {
    CK(hipEventRecord(a, st));
    hipLaunchKernelGGL((copy_tiles<INFLIGHT, NT>), dim3(grid), dim3(kBlock), 0, st, s, d, nvec,
                       tile_vec);
    CK(hipGetLastError());
    CK(hipEventRecord(b, st));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    if (it > 0) best = std::min(best, ms);
  }
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return best;
}

int main() {
  const int64_t bytes = 16060522496LL / 2 / 16 * 16 * 2;  // the 8B model's 16.06 GB
  const int64_t nvec = bytes / 16;
  u32x4 *s = nullptr, *d = nullptr;
  CK(hipMalloc(&s, bytes));
  CK(hipMalloc(&d, bytes));
  CK(hipMemset(s, 0x5a, bytes));
  CK(hipMemset(d, 0, bytes));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  const int64_t tile = (1 << 20) / 16;
  struct R { const char* name; float ms; };
  R r[] = {
      {"plain_x4_grid2048 (hs_copy_nd today)", run<4, false>(s, d, nvec, tile, 2048, st)},
      {"plain_x8_grid2048", run<8, false>(s, d, nvec, tile, 2048, st)},
      {"nt_x4_grid2048", run<4, true>(s, d, nvec, tile, 2048, st)},
      {"nt_x8_grid2048", run<8, true>(s, d, nvec, tile, 2048, st)},
      {"plain_x4_grid4096", run<4, false>(s, d, nvec, tile, 4096, st)},
      {"nt_x4_grid4096", run<4, true>(s, d, nvec, tile, 4096, st)},
      {"plain_x4_grid1024", run<4, false>(s, d, nvec, tile, 1024, st)},
      {"nt_x4_grid1024", run<4, true>(s, d, nvec, tile, 1024, st)},
      {"plain_x4_tile4M_grid2048", run<4, false>(s, d, nvec, tile * 4, 2048, st)},
  };
  // the copy must be right: spot-check the destination
  unsigned char probe[64];
  CK(hipMemcpy(probe, reinterpret_cast<char*>(d) + bytes - 64, 64, hipMemcpyDeviceToHost));
  for (int i = 0; i < 64; ++i)
    if (probe[i] != 0x5a) { fprintf(stderr, "copy mismatch\n"); return 2; }
  printf("{\"bytes\": %lld", (long long)bytes);
  for (const R& x : r)
    printf(", \"%s\": {\"ms\": %.3f, \"payload_TBps\": %.3f}", x.name, x.ms, bytes / x.ms / 1e9);
  printf("}\n");
  CK(hipFree(s));
  CK(hipFree(d));
  return 0;
}
