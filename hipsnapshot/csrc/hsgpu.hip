// hsgpu: MI355X (gfx950 / CDNA4) data plane for hipsnapshot.
//
// What the reference does through ATen on the GPU
// (/root/reference/torchsnapshot/io_preparers/tensor.py:247-254 pageable
// .to("cpu") in a 4-thread pool; batcher.py:141-156 slab alloc + per-member
// DtoD + .cpu(); tensor.py:329-358 and sharded_tensor.py:278-309 host copy_ +
// narrow for restore/resharding) is re-designed here as:
//
//   * a caching PINNED host pool (THP-backed registered memory, 2 MiB granularity, reused
//     across snapshots) so every DtoH/HtoD is a DMA into page-locked memory,
//   * per-(device, slot) non-blocking copy streams ordered after the producer
//     stream with an event (no device-wide sync, no default-stream stalls),
//   * ONE batched strided copy/cast kernel (hs_copy_nd) that serves as
//       K2  strided -> contiguous pack,
//       K3  multi-tensor slab gather (descriptor table, one launch),
//       K6  contiguous -> strided scatter with dtype conversion on restore,
//       K7  resharding: every saved-shard x local-shard overlap in one launch,
//     and can target host-mapped pinned memory directly (kernel stores over
//     PCIe, "pack-to-host") or HBM (async-snapshot arena),
//   * K5/K9 blockwise OCP-fp8 (e4m3fn) quantize / dequantize kernels.
//
// Work decomposition: every descriptor is cut into tiles of a fixed number of
// elements; a tile table is built on the host and the grid walks it with a
// grid-stride loop (grid capped at 256 CUs x 8), so thousands of tiny tensors
// and a few huge ones share one launch and fill all 256 CUs.  Each lane moves
// 16 bytes per access (dwordx4) wherever alignment allows (CDNA guide,
// Guideline 13).  Wave size is 64 everywhere.
//
// C ABI (ctypes); no torch headers.

#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <type_traits>
#include <vector>

namespace {

constexpr int kMaxDims = 8;
constexpr int kBlock = 256;            // 4 waves of 64
constexpr int64_t kTileBytes = 1 << 20;  // 1 MiB of output per tile
constexpr size_t kPinnedGranule = size_t(2) << 20;

// dtype codes shared with python (hipsnapshot/ops/native.py)
enum DType : int32_t {
  kRaw1 = 0, kRaw2 = 1, kRaw4 = 2, kRaw8 = 3, kRaw16 = 4,  // same-type copies
  kF16 = 10, kBF16 = 11, kF32 = 12, kF64 = 13,
};

struct CopyDesc {
  const char* src;
  char* dst;
  int64_t numel;
  int32_t ndim;
  int32_t src_dtype;
  int32_t dst_dtype;
  int32_t flags;  // bit0: both fully contiguous & same type -> byte copy
  int64_t sizes[kMaxDims];
  int64_t src_strides[kMaxDims];  // in elements
  int64_t dst_strides[kMaxDims];
};

struct Tile {
  int32_t desc;
  int32_t pad;
  int64_t begin;  // element (or byte for flag-0 byte copies) range
  int64_t end;
};

thread_local char g_err[512];

void set_err(const char* what, hipError_t e) {
  snprintf(g_err, sizeof(g_err), "%s: %s", what, hipGetErrorString(e));
}

#define HS_CHECK(expr)                      \
  do {                                      \
    hipError_t _e = (expr);                 \
    if (_e != hipSuccess) {                 \
      set_err(#expr, _e);                   \
      return -static_cast<int>(_e) - 1;     \
    }                                       \
  } while (0)

__device__ __forceinline__ int elem_size(int32_t dt) {
  switch (dt) {
    case kRaw1: return 1;
    case kRaw2: case kF16: case kBF16: return 2;
    case kRaw4: case kF32: return 4;
    case kRaw8: case kF64: return 8;
    default: return 16;
  }
}

__device__ __forceinline__ float bf16_to_f32(uint16_t v) {
  return __uint_as_float(static_cast<uint32_t>(v) << 16);
}

__device__ __forceinline__ uint16_t f32_to_bf16(float f) {
  // round-to-nearest-even, NaN preserved (matches torch's c10::BFloat16)
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return static_cast<uint16_t>((u >> 16) | 0x40);
  u += 0x7fffu + ((u >> 16) & 1u);
  return static_cast<uint16_t>(u >> 16);
}

__device__ __forceinline__ double load_as_f64(const char* p, int32_t dt) {
  switch (dt) {
    case kF16: return static_cast<double>(static_cast<float>(*reinterpret_cast<const _Float16*>(p)));
    case kBF16: return static_cast<double>(bf16_to_f32(*reinterpret_cast<const uint16_t*>(p)));
    case kF32: return static_cast<double>(*reinterpret_cast<const float*>(p));
    default: return *reinterpret_cast<const double*>(p);
  }
}

__device__ __forceinline__ float load_as_f32(const char* p, int32_t dt) {
  switch (dt) {
    case kF16: return static_cast<float>(*reinterpret_cast<const _Float16*>(p));
    case kBF16: return bf16_to_f32(*reinterpret_cast<const uint16_t*>(p));
    case kF32: return *reinterpret_cast<const float*>(p);
    default: return static_cast<float>(*reinterpret_cast<const double*>(p));
  }
}

__device__ __forceinline__ void store_from_f32(char* p, int32_t dt, float v) {
  switch (dt) {
    case kF16: {
      // the empty asm pins v as an f32: otherwise a caller's f32 multiply and
      // this fptrunc may be fused into one mixed-precision FMA (a single
      // rounding to f16), which differs from torch's f32 -> f16 in rare ties
      asm volatile("" : "+v"(v));
      *reinterpret_cast<_Float16*>(p) = static_cast<_Float16>(v);
      break;
    }
    case kBF16: *reinterpret_cast<uint16_t*>(p) = f32_to_bf16(v); break;
    case kF32: *reinterpret_cast<float*>(p) = v; break;
    default: *reinterpret_cast<double*>(p) = static_cast<double>(v); break;
  }
}

__device__ __forceinline__ void store_from_f64(char* p, int32_t dt, double v) {
  switch (dt) {
    // f64 -> f16 goes through f32 (two RNE roundings) exactly like torch's
    // copy_ on ROCm (c10::Half is constructed from float); measured on MI355X:
    // a single-rounding conversion differs from torch in ~1e-4 of values.
    case kF16: {
      // the empty asm pins the f32 intermediate: without it LLVM folds the two
      // fptruncs into one f64->f16 rounding, which torch does not do
      float f = static_cast<float>(v);
      asm volatile("" : "+v"(f));
      *reinterpret_cast<_Float16*>(p) = static_cast<_Float16>(f);
      break;
    }
    case kBF16: *reinterpret_cast<uint16_t*>(p) = f32_to_bf16(static_cast<float>(v)); break;
    case kF32: *reinterpret_cast<float*>(p) = static_cast<float>(v); break;
    default: *reinterpret_cast<double*>(p) = v; break;
  }
}

// Contiguous same-type byte copy of [begin, end) bytes: dwordx4 body when both
// pointers are 16-B aligned at the tile start, byte loop otherwise.
__device__ void copy_bytes(const char* __restrict__ src, char* __restrict__ dst,
                           int64_t begin, int64_t end) {
  const char* s = src + begin;
  char* d = dst + begin;
  int64_t n = end - begin;
  if (((reinterpret_cast<uintptr_t>(s) | reinterpret_cast<uintptr_t>(d)) & 15) == 0) {
    const int64_t nv = n >> 4;
    const uint4* sv = reinterpret_cast<const uint4*>(s);
    uint4* dv = reinterpret_cast<uint4*>(d);
    int64_t i = threadIdx.x;
    // 4 independent 16-B loads in flight per lane before the stores
    for (; i + 3 * kBlock < nv; i += 4 * kBlock) {
      uint4 a = sv[i], b = sv[i + kBlock], c = sv[i + 2 * kBlock], e = sv[i + 3 * kBlock];
      dv[i] = a; dv[i + kBlock] = b; dv[i + 2 * kBlock] = c; dv[i + 3 * kBlock] = e;
    }
    for (; i < nv; i += kBlock) dv[i] = sv[i];
    for (int64_t j = (nv << 4) + threadIdx.x; j < n; j += kBlock) d[j] = s[j];
  } else if (((reinterpret_cast<uintptr_t>(s) | reinterpret_cast<uintptr_t>(d)) & 3) == 0) {
    const int64_t nv = n >> 2;
    const uint32_t* sv = reinterpret_cast<const uint32_t*>(s);
    uint32_t* dv = reinterpret_cast<uint32_t*>(d);
    for (int64_t i = threadIdx.x; i < nv; i += kBlock) dv[i] = sv[i];
    for (int64_t j = (nv << 2) + threadIdx.x; j < n; j += kBlock) d[j] = s[j];
  } else {
    for (int64_t j = threadIdx.x; j < n; j += kBlock) d[j] = s[j];
  }
}

template <int ES>
struct RawT;
template <> struct RawT<1> { using T = uint8_t; };
template <> struct RawT<2> { using T = uint16_t; };
template <> struct RawT<4> { using T = uint32_t; };
template <> struct RawT<8> { using T = uint64_t; };
template <> struct RawT<16> { using T = uint4; };

// Each lane owns kRun consecutive logical elements: decode the N-d index once,
// then walk with carry propagation (one divide chain per run instead of per
// element).  ND is a template parameter so the coordinate arrays stay in VGPRs
// (a runtime-indexed array would spill to scratch -- CDNA guide 5.4 rule 20);
// the host collapses mergeable dims first so ND <= 4 covers practically every
// view (narrow/transpose/column shard).
constexpr int kRun = 8;

template <int ND>
__device__ __forceinline__ void decode(const CopyDesc& d, int64_t linear, int64_t* coord,
                                       int64_t* soff, int64_t* doff) {
  int64_t s = 0, t = 0;
#pragma unroll
  for (int k = ND - 1; k >= 0; --k) {
    const int64_t sz = d.sizes[k];
    int64_t c;
    if (k == 0) {
      c = linear;
    } else {
      c = linear % sz;
      linear /= sz;
    }
    coord[k] = c;
    s += c * d.src_strides[k];
    t += c * d.dst_strides[k];
  }
  *soff = s;
  *doff = t;
}

template <int ND>
__device__ __forceinline__ void advance(const CopyDesc& d, int64_t* coord, int64_t* soff,
                                        int64_t* doff) {
#pragma unroll
  for (int k = ND - 1; k >= 0; --k) {
    coord[k] += 1;
    *soff += d.src_strides[k];
    *doff += d.dst_strides[k];
    if (k == 0 || coord[k] < d.sizes[k]) return;
    *soff -= coord[k] * d.src_strides[k];
    *doff -= coord[k] * d.dst_strides[k];
    coord[k] = 0;
  }
}

template <int ND, int ES>
__device__ void copy_strided_same(const CopyDesc& d, int64_t begin, int64_t end) {
  using T = typename RawT<ES>::T;
  const T* __restrict__ src = reinterpret_cast<const T*>(d.src);
  T* __restrict__ dst = reinterpret_cast<T*>(d.dst);
  for (int64_t base = begin + int64_t(threadIdx.x) * kRun; base < end;
       base += int64_t(kBlock) * kRun) {
    int64_t coord[ND];
    int64_t so, dof;
    decode<ND>(d, base, coord, &so, &dof);
    const int64_t cnt = min(int64_t(kRun), end - base);
    T buf[kRun];
    int64_t doffs[kRun];
#pragma unroll
    for (int r = 0; r < kRun; ++r) {
      if (r < cnt) {
        buf[r] = src[so];
        doffs[r] = dof;
        advance<ND>(d, coord, &so, &dof);
      }
    }
#pragma unroll
    for (int r = 0; r < kRun; ++r) {
      if (r < cnt) dst[doffs[r]] = buf[r];
    }
  }
}

template <int ND>
__device__ void copy_strided_cast(const CopyDesc& d, int64_t begin, int64_t end) {
  const int ses = elem_size(d.src_dtype);
  const int des = elem_size(d.dst_dtype);
  const bool wide = (d.src_dtype == kF64) || (d.dst_dtype == kF64);
  for (int64_t base = begin + int64_t(threadIdx.x) * kRun; base < end;
       base += int64_t(kBlock) * kRun) {
    int64_t coord[ND];
    int64_t so, dof;
    decode<ND>(d, base, coord, &so, &dof);
    const int64_t lim = min(base + kRun, end);
    for (int64_t e = base; e < lim; ++e) {
      const char* sp = d.src + so * ses;
      char* dp = d.dst + dof * des;
      if (wide) store_from_f64(dp, d.dst_dtype, load_as_f64(sp, d.src_dtype));
      else store_from_f32(dp, d.dst_dtype, load_as_f32(sp, d.src_dtype));
      advance<ND>(d, coord, &so, &dof);
    }
  }
}

// Contiguous -> contiguous cast between f16 / bf16 / f32 (the restore of an
// fp32 checkpoint into a bf16 model, and back): 8 elements per lane per step
// with 16-B vector loads and stores, same conversions as store_from_f32(
// load_as_f32()) (bit-identical to torch's copy_).  Unaligned tiles and the
// tail take the scalar path.
template <int DT>
__device__ __forceinline__ void load8_f32(const char* p, float* f) {
  if constexpr (DT == kF32) {
    const uint4 a = reinterpret_cast<const uint4*>(p)[0];
    const uint4 b = reinterpret_cast<const uint4*>(p)[1];
    f[0] = __uint_as_float(a.x); f[1] = __uint_as_float(a.y);
    f[2] = __uint_as_float(a.z); f[3] = __uint_as_float(a.w);
    f[4] = __uint_as_float(b.x); f[5] = __uint_as_float(b.y);
    f[6] = __uint_as_float(b.z); f[7] = __uint_as_float(b.w);
  } else {
    const uint4 a = reinterpret_cast<const uint4*>(p)[0];
    const uint32_t w[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint16_t lo = static_cast<uint16_t>(w[i] & 0xffffu);
      const uint16_t hi = static_cast<uint16_t>(w[i] >> 16);
      if constexpr (DT == kBF16) {
        f[2 * i] = bf16_to_f32(lo);
        f[2 * i + 1] = bf16_to_f32(hi);
      } else {
        _Float16 x, y;
        __builtin_memcpy(&x, &lo, 2);
        __builtin_memcpy(&y, &hi, 2);
        f[2 * i] = static_cast<float>(x);
        f[2 * i + 1] = static_cast<float>(y);
      }
    }
  }
}

template <int DT>
__device__ __forceinline__ void store8_f32(char* p, const float* f) {
  if constexpr (DT == kF32) {
    reinterpret_cast<uint4*>(p)[0] = make_uint4(__float_as_uint(f[0]), __float_as_uint(f[1]),
                                                __float_as_uint(f[2]), __float_as_uint(f[3]));
    reinterpret_cast<uint4*>(p)[1] = make_uint4(__float_as_uint(f[4]), __float_as_uint(f[5]),
                                                __float_as_uint(f[6]), __float_as_uint(f[7]));
  } else {
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      uint16_t lo, hi;
      if constexpr (DT == kBF16) {
        lo = f32_to_bf16(f[2 * i]);
        hi = f32_to_bf16(f[2 * i + 1]);
      } else {
        const _Float16 a = static_cast<_Float16>(f[2 * i]);
        const _Float16 b = static_cast<_Float16>(f[2 * i + 1]);
        __builtin_memcpy(&lo, &a, 2);
        __builtin_memcpy(&hi, &b, 2);
      }
      w[i] = uint32_t(lo) | (uint32_t(hi) << 16);
    }
    reinterpret_cast<uint4*>(p)[0] = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

template <int SD, int DD>
__device__ void copy_contig_cast(const CopyDesc& d, int64_t begin, int64_t end) {
  constexpr int SES = (SD == kF32) ? 4 : 2;
  constexpr int DES = (DD == kF32) ? 4 : 2;
  const char* s = d.src + begin * SES;
  char* o = d.dst + begin * DES;
  const int64_t n = end - begin;
  int64_t done = 0;
  if (((reinterpret_cast<uintptr_t>(s) | reinterpret_cast<uintptr_t>(o)) & 15) == 0) {
    const int64_t nv = n / 8;
    for (int64_t i = threadIdx.x; i < nv; i += kBlock) {
      float f[8];
      load8_f32<SD>(s + i * 8 * SES, f);
      store8_f32<DD>(o + i * 8 * DES, f);
    }
    done = nv * 8;
  }
  for (int64_t j = done + threadIdx.x; j < n; j += kBlock)
    store_from_f32(o + j * DES, DD, load_as_f32(s + j * SES, SD));
}

template <int ND>
__device__ __forceinline__ bool try_contig_cast(const CopyDesc& d, int64_t b, int64_t e) {
  if constexpr (ND != 1) {
    return false;
  } else {
    if (d.src_strides[0] != 1 || d.dst_strides[0] != 1) return false;
    const int sd = d.src_dtype, dd = d.dst_dtype;
#define HS_CAST_CASE(S, D) \
    if (sd == S && dd == D) { copy_contig_cast<S, D>(d, b, e); return true; }
    HS_CAST_CASE(kF32, kBF16) HS_CAST_CASE(kBF16, kF32)
    HS_CAST_CASE(kF32, kF16) HS_CAST_CASE(kF16, kF32)
    HS_CAST_CASE(kBF16, kF16) HS_CAST_CASE(kF16, kBF16)
#undef HS_CAST_CASE
    return false;
  }
}

template <int ND>
__device__ __forceinline__ void copy_tile_nd(const CopyDesc& d, int64_t b, int64_t e) {
  if (d.src_dtype == d.dst_dtype || d.src_dtype < kF16) {
    switch (elem_size(d.src_dtype)) {
      case 1: copy_strided_same<ND, 1>(d, b, e); break;
      case 2: copy_strided_same<ND, 2>(d, b, e); break;
      case 4: copy_strided_same<ND, 4>(d, b, e); break;
      case 8: copy_strided_same<ND, 8>(d, b, e); break;
      default: copy_strided_same<ND, 16>(d, b, e); break;
    }
  } else if (!try_contig_cast<ND>(d, b, e)) {
    copy_strided_cast<ND>(d, b, e);
  }
}

// ---- rows mode (flags & 2): 2-D copy whose inner dim is contiguous on both
// sides (column shards, narrowed views).  Work unit = one vector of `vw` bytes
// (vw = flags >> 8, the widest power of two dividing the row length, both row
// strides and both base addresses); the tile range indexes the flattened
// (row, vector) space so long and short rows balance the same way.
template <int VW>
__device__ void copy_rows(const CopyDesc& d, int64_t begin, int64_t end, int es) {
  using V = typename RawT<VW>::T;
  const int64_t vpr = d.sizes[1] * es / VW;  // vectors per row
  const int64_t s_row = d.src_strides[0] * es, d_row = d.dst_strides[0] * es;
  for (int64_t v = begin + threadIdx.x; v < end; v += kBlock) {
    const int64_t r = v / vpr, c = v - r * vpr;
    const V* s = reinterpret_cast<const V*>(d.src + r * s_row) + c;
    V* o = reinterpret_cast<V*>(d.dst + r * d_row) + c;
    *o = *s;
  }
}

// ---- transpose mode (flags & 4): canonical [B, I, J] with src contiguous along
// I and dst contiguous along J.  64x64 tiles staged through LDS (padded to 65
// words per row: conflict-free column reads), loads coalesced along I, stores
// coalesced along J.  A tile range is a range of 64x64 blocks.
template <int ES>
__device__ void transpose_blocks(const CopyDesc& d, int64_t begin, int64_t end, char* lds_raw) {
  using T = typename RawT<ES>::T;
  using W = typename std::conditional<ES == 8, uint64_t, uint32_t>::type;
  W(*lds)[65] = reinterpret_cast<W(*)[65]>(lds_raw);
  const int64_t I = d.sizes[1], J = d.sizes[2];
  const int64_t ti_n = (I + 63) / 64, tj_n = (J + 63) / 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int64_t blk = begin; blk < end; ++blk) {
    const int64_t b = blk / (ti_n * tj_n);
    const int64_t rr = blk - b * (ti_n * tj_n);
    const int64_t i0 = (rr / tj_n) * 64, j0 = (rr % tj_n) * 64;
    const T* src = reinterpret_cast<const T*>(d.src) + b * d.src_strides[0];
    T* dst = reinterpret_cast<T*>(d.dst) + b * d.dst_strides[0];
    const int64_t sj = d.src_strides[2], di = d.dst_strides[1];
#pragma unroll 4
    for (int jj = ty; jj < 64; jj += kBlock / 64) {
      const int64_t i = i0 + tx, j = j0 + jj;
      if (i < I && j < J) lds[jj][tx] = static_cast<W>(src[i + j * sj]);
    }
    __syncthreads();
#pragma unroll 4
    for (int ii = ty; ii < 64; ii += kBlock / 64) {
      const int64_t i = i0 + ii, j = j0 + tx;
      if (i < I && j < J) dst[i * di + j] = static_cast<T>(lds[tx][ii]);
    }
    __syncthreads();
  }
}

__global__ void __launch_bounds__(kBlock)
hs_copy_nd(const CopyDesc* __restrict__ descs, const Tile* __restrict__ tiles, int64_t ntiles) {
  extern __shared__ __attribute__((aligned(16))) char lds_raw[];
  for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const Tile tile = tiles[t];
    const CopyDesc& d = descs[tile.desc];
    if (d.flags & 1) {
      copy_bytes(d.src, d.dst, tile.begin, tile.end);
    } else if (d.flags & 2) {
      const int es = elem_size(d.src_dtype);
      switch (d.flags >> 8) {
        case 16: copy_rows<16>(d, tile.begin, tile.end, es); break;
        case 8: copy_rows<8>(d, tile.begin, tile.end, es); break;
        case 4: copy_rows<4>(d, tile.begin, tile.end, es); break;
        case 2: copy_rows<2>(d, tile.begin, tile.end, es); break;
        default: copy_rows<1>(d, tile.begin, tile.end, es); break;
      }
    } else if (d.flags & 4) {
      switch (elem_size(d.src_dtype)) {
        case 1: transpose_blocks<1>(d, tile.begin, tile.end, lds_raw); break;
        case 2: transpose_blocks<2>(d, tile.begin, tile.end, lds_raw); break;
        case 4: transpose_blocks<4>(d, tile.begin, tile.end, lds_raw); break;
        default: transpose_blocks<8>(d, tile.begin, tile.end, lds_raw); break;
      }
    } else {
      switch (d.ndim) {
        case 1: copy_tile_nd<1>(d, tile.begin, tile.end); break;
        case 2: copy_tile_nd<2>(d, tile.begin, tile.end); break;
        case 3: copy_tile_nd<3>(d, tile.begin, tile.end); break;
        case 4: copy_tile_nd<4>(d, tile.begin, tile.end); break;
        case 5: copy_tile_nd<5>(d, tile.begin, tile.end); break;
        case 6: copy_tile_nd<6>(d, tile.begin, tile.end); break;
        case 7: copy_tile_nd<7>(d, tile.begin, tile.end); break;
        default: copy_tile_nd<8>(d, tile.begin, tile.end); break;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// fp8 (OCP e4m3fn) blockwise quantization.  One 64-lane wave owns one block of
// `block` elements (block = 64 * VPT); amax via 64-wide xor-shuffle reduction,
// scale = amax / 448, payload via v_cvt_pk_fp8_f32 (gfx950: OCP encoding).
// ---------------------------------------------------------------------------

constexpr float kFp8Max = 448.0f;

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Non-finite inputs of the blockwise (f32-scale) formats, as in the MX ones:
// they do not set their block's scale (|x| of inf / nan counts as 0), and
// their code is the e4m3fn NaN with the input's sign (torch's cast).  So one
// inf no longer turns every element of its block into NaN, and the GPU codes
// equal ops/quant.py's reference for every input.
__device__ __forceinline__ float finite_abs(float x) {
  const float a = fabsf(x);
  return a < __builtin_huge_valf() ? a : 0.f;
}

// `word` holds the codes of x[0..3] (byte j <- x[j]); j >= nvalid are left as is
__device__ __forceinline__ uint32_t fp8_fix_nonfinite(uint32_t word, const float* x,
                                                      int nvalid = 4) {
  uint32_t fix = 0, mask = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (j >= nvalid) break;
    const uint32_t b = __float_as_uint(x[j]);
    if ((b & 0x7f800000u) == 0x7f800000u) {
      mask |= 0xffu << (8 * j);
      fix |= ((b >> 31) ? 0xffu : 0x7fu) << (8 * j);
    }
  }
  return (word & ~mask) | fix;
}

template <int VPT>
__global__ void __launch_bounds__(kBlock)
hs_fp8_quant(const char* __restrict__ src, int32_t src_dtype, int64_t n,
             uint8_t* __restrict__ out, float* __restrict__ scales) {
  constexpr int kBlk = 64 * VPT;
  const int lane = threadIdx.x & 63;
  const int64_t nblocks = (n + kBlk - 1) / kBlk;
  const int64_t wave0 = (int64_t(blockIdx.x) * kBlock + threadIdx.x) >> 6;
  const int64_t nwaves = (int64_t(gridDim.x) * kBlock) >> 6;
  const int ses = (src_dtype == kF32) ? 4 : 2;
  for (int64_t b = wave0; b < nblocks; b += nwaves) {
    const int64_t e0 = b * kBlk + int64_t(lane) * VPT;
    float v[VPT];
    float amax = 0.f;
#pragma unroll
    for (int j = 0; j < VPT; ++j) {
      const int64_t e = e0 + j;
      v[j] = (e < n) ? load_as_f32(src + e * ses, src_dtype) : 0.f;
      amax = fmaxf(amax, finite_abs(v[j]));
    }
    amax = wave_max(amax);
    // two correctly rounded divisions per BLOCK (scale, then its reciprocal)
    // and one multiply per element -- the torch reference (ops/quant.py
    // _scale_and_quant) applies the same rule, so payloads are bit-identical;
    // a division per element made this kernel VALU-bound (profiles/pmc_r2)
    const float scale = amax > 0.f ? amax / kFp8Max : 1.f;
    const float inv = 1.f / scale;
    if (lane == 0) scales[b] = scale;
    uint32_t words[(VPT + 3) / 4];
#pragma unroll
    for (int w = 0; w < (VPT + 3) / 4; ++w) {
      float a0 = fminf(fmaxf(v[4 * w + 0] * inv, -kFp8Max), kFp8Max);
      float a1 = (4 * w + 1 < VPT) ? fminf(fmaxf(v[4 * w + 1] * inv, -kFp8Max), kFp8Max) : 0.f;
      float a2 = (4 * w + 2 < VPT) ? fminf(fmaxf(v[4 * w + 2] * inv, -kFp8Max), kFp8Max) : 0.f;
      float a3 = (4 * w + 3 < VPT) ? fminf(fmaxf(v[4 * w + 3] * inv, -kFp8Max), kFp8Max) : 0.f;
      int word = __builtin_amdgcn_cvt_pk_fp8_f32(a0, a1, 0, false);
      word = __builtin_amdgcn_cvt_pk_fp8_f32(a2, a3, word, true);
      words[w] = fp8_fix_nonfinite(static_cast<uint32_t>(word), v + 4 * w,
                                   VPT - 4 * w < 4 ? VPT - 4 * w : 4);
    }
    if (e0 + VPT <= n && (VPT % 4) == 0) {
#pragma unroll
      for (int w = 0; w < VPT / 4; ++w)
        reinterpret_cast<uint32_t*>(out + e0)[w] = words[w];
    } else {
      for (int j = 0; j < VPT; ++j)
        if (e0 + j < n) out[e0 + j] = static_cast<uint8_t>(words[j >> 2] >> (8 * (j & 3)));
    }
  }
}

template <int VPT>
__global__ void __launch_bounds__(kBlock)
hs_fp8_dequant(const uint8_t* __restrict__ q, const float* __restrict__ scales, int64_t n,
               char* __restrict__ dst, int32_t dst_dtype) {
  constexpr int kBlk = 64 * VPT;
  const int des = (dst_dtype == kF32) ? 4 : (dst_dtype == kF64 ? 8 : 2);
  const int64_t nthreads = int64_t(gridDim.x) * kBlock;
  for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i * 4 < n; i += nthreads) {
    const int64_t e0 = i * 4;
    uint32_t word;
    if (e0 + 4 <= n) {
      word = reinterpret_cast<const uint32_t*>(q)[i];
    } else {
      word = 0;
      for (int j = 0; j < 4 && e0 + j < n; ++j) word |= uint32_t(q[e0 + j]) << (8 * j);
    }
    const float s = scales[e0 / kBlk];
    float f[4];
    f[0] = __builtin_amdgcn_cvt_f32_fp8(static_cast<int>(word), 0);
    f[1] = __builtin_amdgcn_cvt_f32_fp8(static_cast<int>(word), 1);
    f[2] = __builtin_amdgcn_cvt_f32_fp8(static_cast<int>(word), 2);
    f[3] = __builtin_amdgcn_cvt_f32_fp8(static_cast<int>(word), 3);
    for (int j = 0; j < 4 && e0 + j < n; ++j) store_from_f32(dst + (e0 + j) * des, dst_dtype, f[j] * s);
  }
}

// ---------------------------------------------------------------------------
// MX fp8: OCP e4m3fn elements + one E8M0 (power-of-two) scale byte per
// 32-element block.  Scale 2^k with the smallest k such that amax <= 448*2^k
// (exact, from frexp: amax = m*2^e, k = e-9 if m <= 0.875 else e-8), so
// x * 2^-k is exact (v_ldexp_f32, no division, no clamp needed) and restore is
// q * 2^k, exact in f32.  Streaming layout for the HBM roof:
//   * every 16-B load instruction is contiguous across the wave (lane l
//     reads bytes [16 l, 16 l + 16) of a 1 KiB wave segment), U = 4 of them in
//     flight per lane;
//   * a 32-element block spans LPB = 32 / (16 / es) lanes (4 for bf16/f16, 8
//     for f32): amax is an in-register max over the lane's 16 B then a
//     log2(LPB)-step xor-shuffle;
//   * fp8 bytes leave as one 8-B (bf16) / 4-B (f32) store per lane per load,
//     again contiguous across the wave.
// ---------------------------------------------------------------------------

constexpr int kMxBlock = 32;
typedef unsigned int mx_u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int mx_u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float fp8_byte_to_f32(uint32_t w, int b) {
  switch (b) {  // the byte select must be an immediate
    case 0: return __builtin_amdgcn_cvt_f32_fp8(static_cast<int>(w), 0);
    case 1: return __builtin_amdgcn_cvt_f32_fp8(static_cast<int>(w), 1);
    case 2: return __builtin_amdgcn_cvt_f32_fp8(static_cast<int>(w), 2);
    default: return __builtin_amdgcn_cvt_f32_fp8(static_cast<int>(w), 3);
  }
}

__device__ __forceinline__ int mx_exp(float amax) {
  if (!(amax > 0.f) || !(amax < __builtin_huge_valf())) return 0;  // zero / inf / nan
  int e;
  const float m = frexpf(amax, &e);
  const int k = (m <= 0.875f) ? e - 9 : e - 8;
  return k < -127 ? -127 : (k > 127 ? 127 : k);
}

template <int DT>
__device__ __forceinline__ float mx_unpack(uint32_t w, int half) {
  if constexpr (DT == kBF16) return __uint_as_float(half ? (w & 0xffff0000u) : (w << 16));
  else {
    _Float16 h;
    const uint16_t b = static_cast<uint16_t>(half ? (w >> 16) : (w & 0xffffu));
    __builtin_memcpy(&h, &b, 2);
    return static_cast<float>(h);
  }
}

template <int DT>
__global__ void __launch_bounds__(kBlock)
hs_mx8_quant(const char* __restrict__ src, int64_t n, int64_t payload,
             uint8_t* __restrict__ out, uint8_t* __restrict__ scales) {
  constexpr int ES = (DT == kF32) ? 4 : 2;
  constexpr int EPL = 16 / ES;
  constexpr int LPB = kMxBlock / EPL;
  constexpr int U = 4;
  constexpr int64_t kChunk = 64LL * EPL * U;
  const int lane = threadIdx.x & 63;
  const int64_t wave0 = (int64_t(blockIdx.x) * kBlock + threadIdx.x) >> 6;
  const int64_t nwaves = (int64_t(gridDim.x) * kBlock) >> 6;
  const int64_t nchunks = (n + kChunk - 1) / kChunk;
  for (int64_t c = wave0; c < nchunks; c += nwaves) {
    const int64_t base = c * kChunk;
    const bool full = base + kChunk <= n;
    uint4 raw[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t e0 = base + (int64_t(u) * 64 + lane) * EPL;
      if (full) {
        const mx_u32x4 t =
            __builtin_nontemporal_load(reinterpret_cast<const mx_u32x4*>(src + e0 * ES));
        raw[u] = make_uint4(t.x, t.y, t.z, t.w);
      } else {
        uint32_t w[4] = {0, 0, 0, 0};
        for (int j = 0; j < EPL; ++j) {
          if (e0 + j >= n) break;
          uint32_t bits;
          if constexpr (ES == 4) bits = *reinterpret_cast<const uint32_t*>(src + (e0 + j) * 4);
          else bits = *reinterpret_cast<const uint16_t*>(src + (e0 + j) * 2);
          w[(j * ES) >> 2] |= bits << (((j * ES) & 3) * 8);
        }
        raw[u] = make_uint4(w[0], w[1], w[2], w[3]);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t ws[4] = {raw[u].x, raw[u].y, raw[u].z, raw[u].w};
      float v[EPL];
#pragma unroll
      for (int j = 0; j < EPL; ++j) {
        if constexpr (ES == 4) v[j] = __uint_as_float(ws[j]);
        else v[j] = mx_unpack<DT>(ws[j >> 1], j & 1);
      }
      float amax = 0.f;  // over the finite elements (inf / nan do not set the scale)
#pragma unroll
      for (int j = 0; j < EPL; ++j) {
        const float a = fabsf(v[j]);
        amax = fmaxf(amax, a < __builtin_huge_valf() ? a : 0.f);
      }
#pragma unroll
      for (int o = 1; o < LPB; o <<= 1) amax = fmaxf(amax, __shfl_xor(amax, o, 64));
      const int k = mx_exp(amax);
      const int64_t e0 = base + (int64_t(u) * 64 + lane) * EPL;
      if ((lane % LPB) == 0 && e0 < n) scales[e0 / kMxBlock] = static_cast<uint8_t>(k + 127);
      uint32_t q[EPL / 4];
#pragma unroll
      for (int w = 0; w < EPL / 4; ++w) {
        int word = __builtin_amdgcn_cvt_pk_fp8_f32(ldexpf(v[4 * w], -k), ldexpf(v[4 * w + 1], -k),
                                                   0, false);
        word = __builtin_amdgcn_cvt_pk_fp8_f32(ldexpf(v[4 * w + 2], -k),
                                               ldexpf(v[4 * w + 3], -k), word, true);
        // non-finite elements: e4m3fn NaN with the element's sign (torch's cast)
        uint32_t fix = 0, fixmask = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const uint32_t b = __float_as_uint(v[4 * w + j]);
          if ((b & 0x7f800000u) == 0x7f800000u) {
            fixmask |= 0xffu << (8 * j);
            fix |= ((b >> 31) ? 0xffu : 0x7fu) << (8 * j);
          }
        }
        q[w] = (static_cast<uint32_t>(word) & ~fixmask) | fix;
      }
      if (full) {
        if constexpr (EPL == 8) {
          mx_u32x2 t;
          t.x = q[0];
          t.y = q[1];
          __builtin_nontemporal_store(t, reinterpret_cast<mx_u32x2*>(out + e0));
        } else
          __builtin_nontemporal_store(q[0], reinterpret_cast<uint32_t*>(out + e0));
      } else {
        for (int j = 0; j < EPL; ++j) {
          const int64_t e = e0 + j;
          if (e < payload) out[e] = e < n ? static_cast<uint8_t>(q[j >> 2] >> (8 * (j & 3))) : 0;
        }
      }
    }
  }
}

template <int DT>
__device__ __forceinline__ void mx_store(char* p, const float* f) {
  // 16 B of output: 8 x bf16/f16, 4 x f32 or 2 x f64
  if constexpr (DT == kF32) {
    *reinterpret_cast<float4*>(p) = make_float4(f[0], f[1], f[2], f[3]);
  } else if constexpr (DT == kF64) {
    *reinterpret_cast<double2*>(p) = make_double2(static_cast<double>(f[0]),
                                                  static_cast<double>(f[1]));
  } else {
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      uint16_t lo, hi;
      if constexpr (DT == kBF16) {
        lo = f32_to_bf16(f[2 * i]);
        hi = f32_to_bf16(f[2 * i + 1]);
      } else {
        const _Float16 a = static_cast<_Float16>(f[2 * i]), b = static_cast<_Float16>(f[2 * i + 1]);
        __builtin_memcpy(&lo, &a, 2);
        __builtin_memcpy(&hi, &b, 2);
      }
      w[i] = uint32_t(lo) | (uint32_t(hi) << 16);
    }
    *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

template <int DT>
__global__ void __launch_bounds__(kBlock)
hs_mx8_dequant(const uint8_t* __restrict__ q, const uint8_t* __restrict__ scales, int64_t n,
               char* __restrict__ dst) {
  constexpr int DES = (DT == kF32) ? 4 : (DT == kF64 ? 8 : 2);
  constexpr int EPL = 16 / DES;  // fp8 bytes per lane per step = one 16-B store
  constexpr int U = 4;
  constexpr int64_t kChunk = 64LL * EPL * U;
  const int lane = threadIdx.x & 63;
  const int64_t wave0 = (int64_t(blockIdx.x) * kBlock + threadIdx.x) >> 6;
  const int64_t nwaves = (int64_t(gridDim.x) * kBlock) >> 6;
  const int64_t nchunks = (n + kChunk - 1) / kChunk;
  for (int64_t c = wave0; c < nchunks; c += nwaves) {
    const int64_t base = c * kChunk;
    const bool full = base + kChunk <= n;
    uint32_t raw[U][(EPL + 3) / 4];
    uint8_t sb[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t e0 = base + (int64_t(u) * 64 + lane) * EPL;
      if (full) {
        if constexpr (EPL == 8) {
          const uint2 t = *reinterpret_cast<const uint2*>(q + e0);
          raw[u][0] = t.x;
          raw[u][1] = t.y;
        } else if constexpr (EPL == 4) {
          raw[u][0] = *reinterpret_cast<const uint32_t*>(q + e0);
        } else {
          raw[u][0] = *reinterpret_cast<const uint16_t*>(q + e0);
        }
      } else {
        for (int w = 0; w < (EPL + 3) / 4; ++w) raw[u][w] = 0;
        for (int j = 0; j < EPL && e0 + j < n; ++j)
          raw[u][j >> 2] |= uint32_t(q[e0 + j]) << (8 * (j & 3));
      }
      sb[u] = e0 < n ? scales[e0 / kMxBlock] : 127;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t e0 = base + (int64_t(u) * 64 + lane) * EPL;
      const int k = int(sb[u]) - 127;
      float f[EPL];
#pragma unroll
      for (int j = 0; j < EPL; ++j)
        f[j] = ldexpf(fp8_byte_to_f32(raw[u][j >> 2], j & 3), k);
      if (full) {
        mx_store<DT>(dst + e0 * DES, f);
      } else {
        for (int j = 0; j < EPL && e0 + j < n; ++j) store_from_f32(dst + (e0 + j) * DES, DT, f[j]);
      }
    }
  }
}

// Blockwise fp8 restore in the same streaming layout (hs_mx8_dequant's):
// lane l reads EPL = 16 / dst-element-size codes and writes 16 B, U = 4 in
// flight; x = f32(q) * scale[e / BLK] (the scale is per lane: BLK % EPL == 0).
template <int DT, int BLK>
__global__ void __launch_bounds__(kBlock)
hs_fp8_dequant_v(const uint8_t* __restrict__ q, const float* __restrict__ scales, int64_t n,
                 char* __restrict__ dst) {
  constexpr int DES = (DT == kF32) ? 4 : (DT == kF64 ? 8 : 2);
  constexpr int EPL = 16 / DES;
  constexpr int U = 4;
  constexpr int64_t kChunk = 64LL * EPL * U;
  const int lane = threadIdx.x & 63;
  const int64_t wave0 = (int64_t(blockIdx.x) * kBlock + threadIdx.x) >> 6;
  const int64_t nwaves = (int64_t(gridDim.x) * kBlock) >> 6;
  const int64_t nchunks = (n + kChunk - 1) / kChunk;
  for (int64_t c = wave0; c < nchunks; c += nwaves) {
    const int64_t base = c * kChunk;
    const bool full = base + kChunk <= n;
    uint32_t raw[U][(EPL + 3) / 4];
    float sc[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t e0 = base + (int64_t(u) * 64 + lane) * EPL;
      if (full) {
        if constexpr (EPL == 8) {
          const uint2 t = *reinterpret_cast<const uint2*>(q + e0);
          raw[u][0] = t.x;
          raw[u][1] = t.y;
        } else if constexpr (EPL == 4) {
          raw[u][0] = *reinterpret_cast<const uint32_t*>(q + e0);
        } else {
          raw[u][0] = *reinterpret_cast<const uint16_t*>(q + e0);
        }
      } else {
        for (int w = 0; w < (EPL + 3) / 4; ++w) raw[u][w] = 0;
        for (int j = 0; j < EPL && e0 + j < n; ++j)
          raw[u][j >> 2] |= uint32_t(q[e0 + j]) << (8 * (j & 3));
      }
      sc[u] = e0 < n ? scales[e0 / BLK] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t e0 = base + (int64_t(u) * 64 + lane) * EPL;
      float f[EPL];
#pragma unroll
      for (int j = 0; j < EPL; ++j) f[j] = fp8_byte_to_f32(raw[u][j >> 2], j & 3) * sc[u];
      if (full) {
        mx_store<DT>(dst + e0 * DES, f);
      } else {
        for (int j = 0; j < EPL && e0 + j < n; ++j) store_from_f32(dst + (e0 + j) * DES, DT, f[j]);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Blockwise fp8 (f32 scale per BLK elements, format "fp8_e4m3fn_block") in the
// streaming layout of hs_mx8_quant: lane l of a wave reads 16 contiguous bytes
// (EPL elements) of a 1 KiB wave segment, U = 4 segments in flight per lane,
// a block spans LPB = BLK / EPL adjacent lanes (amax: log2(LPB) xor shuffles),
// and each lane stores its EPL fp8 codes with one vector store.  Same numerics
// as hs_fp8_quant: scale = amax / 448 (1 if amax == 0), q = cvt(clamp(x * (1 /
// scale))).  hs_fp8_quant (one block per wave, two 2-B loads per lane) ran at
// 1.9 TB/s: too little in flight per wave.
// ---------------------------------------------------------------------------

template <int DT, int BLK>
__global__ void __launch_bounds__(kBlock)
hs_fp8_quant_v(const char* __restrict__ src, int64_t n, uint8_t* __restrict__ out,
               float* __restrict__ scales) {
  constexpr int ES = (DT == kF32) ? 4 : 2;
  constexpr int EPL = 16 / ES;
  constexpr int LPB = BLK / EPL;
  static_assert(LPB >= 1 && LPB <= 64 && (64 % LPB) == 0, "block must fit a wave");
  constexpr int U = 4;
  constexpr int64_t kChunk = 64LL * EPL * U;
  const int lane = threadIdx.x & 63;
  const int64_t wave0 = (int64_t(blockIdx.x) * kBlock + threadIdx.x) >> 6;
  const int64_t nwaves = (int64_t(gridDim.x) * kBlock) >> 6;
  const int64_t nchunks = (n + kChunk - 1) / kChunk;
  for (int64_t c = wave0; c < nchunks; c += nwaves) {
    const int64_t base = c * kChunk;
    const bool full = base + kChunk <= n;
    uint4 raw[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t e0 = base + (int64_t(u) * 64 + lane) * EPL;
      if (full) {
        const mx_u32x4 t =
            __builtin_nontemporal_load(reinterpret_cast<const mx_u32x4*>(src + e0 * ES));
        raw[u] = make_uint4(t.x, t.y, t.z, t.w);
      } else {
        uint32_t w[4] = {0, 0, 0, 0};
        for (int j = 0; j < EPL; ++j) {
          if (e0 + j >= n) break;
          uint32_t bits;
          if constexpr (ES == 4) bits = *reinterpret_cast<const uint32_t*>(src + (e0 + j) * 4);
          else bits = *reinterpret_cast<const uint16_t*>(src + (e0 + j) * 2);
          w[(j * ES) >> 2] |= bits << (((j * ES) & 3) * 8);
        }
        raw[u] = make_uint4(w[0], w[1], w[2], w[3]);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t ws[4] = {raw[u].x, raw[u].y, raw[u].z, raw[u].w};
      float v[EPL];
#pragma unroll
      for (int j = 0; j < EPL; ++j) {
        if constexpr (ES == 4) v[j] = __uint_as_float(ws[j]);
        else v[j] = mx_unpack<DT>(ws[j >> 1], j & 1);
      }
      float amax = 0.f;
#pragma unroll
      for (int j = 0; j < EPL; ++j) amax = fmaxf(amax, finite_abs(v[j]));
#pragma unroll
      for (int o = 1; o < LPB; o <<= 1) amax = fmaxf(amax, __shfl_xor(amax, o, 64));
      const float scale = amax > 0.f ? amax / kFp8Max : 1.f;
      const float inv = 1.f / scale;
      const int64_t e0 = base + (int64_t(u) * 64 + lane) * EPL;
      if ((lane % LPB) == 0 && e0 < n) scales[e0 / BLK] = scale;
      uint32_t q[EPL / 4];
#pragma unroll
      for (int w = 0; w < EPL / 4; ++w) {
        int word = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(v[4 * w] * inv, -kFp8Max), kFp8Max),
                                                   fminf(fmaxf(v[4 * w + 1] * inv, -kFp8Max), kFp8Max),
                                                   0, false);
        word = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(v[4 * w + 2] * inv, -kFp8Max), kFp8Max),
                                               fminf(fmaxf(v[4 * w + 3] * inv, -kFp8Max), kFp8Max),
                                               word, true);
        q[w] = fp8_fix_nonfinite(static_cast<uint32_t>(word), v + 4 * w);
      }
      if (full) {
        if constexpr (EPL == 8) {
          mx_u32x2 t;
          t.x = q[0];
          t.y = q[1];
          __builtin_nontemporal_store(t, reinterpret_cast<mx_u32x2*>(out + e0));
        } else {
          __builtin_nontemporal_store(q[0], reinterpret_cast<uint32_t*>(out + e0));
        }
      } else {
        for (int j = 0; j < EPL && e0 + j < n; ++j)
          out[e0 + j] = static_cast<uint8_t>(q[j >> 2] >> (8 * (j & 3)));
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Hadamard-rotated fp8 (MFMA).  The flat tensor is viewed as rows of 32
// ("groups"); every group is rotated by the 32x32 Sylvester Hadamard matrix H
// (entries +-1, H*H = 32 I) before blockwise e4m3 quantization, which spreads
// outliers across the group and cuts fp8 error on heavy-tailed weights.
//
// One wave owns a tile of 32 groups (1024 elements) and computes
// Y[32x32] = X[32x32] * H with 16 x v_mfma_f32_32x32x2_f32 (exact f32 inputs,
// k-ordered fmaf chain -> bit-reproducible by a sequential fp32 reference).
// Operand maps (CDNA guide 3): lane l, r = l&31, h = l>>5:
//   A[i=r][k=h] per instruction t -> X[row r][2t+h];  B[k=h][j=r] -> H[2t+h][r]
//   C/D reg i -> row (i&3) + 8(i>>2) + 4h, col r
// so register quad g4 of lane-half h is exactly quantization block 2*g4+h of
// the tile (4 rows x 32 cols = 128 elements): amax = 4 regs + xor-shuffle over
// the 32 lanes of the half.  Restore inverts with X = (Y' * H) / 32.
// ---------------------------------------------------------------------------

typedef float floatx16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ float hada(int k, int c) {
  return (__popc(k & c) & 1) ? -1.f : 1.f;
}

// Half-row operand layout: lane (r, h) owns X[r][16h .. 16h + 15] -- 32 B
// (bf16/f16) or 64 B (f32) contiguous in memory, loaded with 16-B vector
// loads -- and MFMA step t contracts k = t (h = 0 lanes) and k = 16 + t
// (h = 1 lanes): the accumulation order is k = 0, 16, 1, 17, ..., 15, 31
// (``ops/quant.py`` HADAMARD_K_ORDER; the torch reference sums in the same
// order, so the blobs stay bit-identical).
template <int DT>
__device__ __forceinline__ void load_half_row(const char* src, int64_t e0, int64_t n, float* x) {
  constexpr int ES = (DT == kF32) ? 4 : 2;
  if (e0 + 16 <= n && ((reinterpret_cast<uintptr_t>(src + e0 * ES) & 15) == 0)) {
    const uint4* v = reinterpret_cast<const uint4*>(src + e0 * ES);
    if constexpr (ES == 4) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint4 w = v[q];
        x[4 * q] = __uint_as_float(w.x);
        x[4 * q + 1] = __uint_as_float(w.y);
        x[4 * q + 2] = __uint_as_float(w.z);
        x[4 * q + 3] = __uint_as_float(w.w);
      }
    } else {
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const uint4 w = v[q];
        const uint32_t ws[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          x[8 * q + 2 * i] = mx_unpack<DT>(ws[i], 0);
          x[8 * q + 2 * i + 1] = mx_unpack<DT>(ws[i], 1);
        }
      }
    }
  } else {
#pragma unroll
    for (int t = 0; t < 16; ++t)
      x[t] = (e0 + t < n) ? load_as_f32(src + (e0 + t) * ES, DT) : 0.f;
  }
}

// max over the 32 lanes of a wave half: quad xor-1 / xor-2 and the 8- and
// 16-lane mirrors on DPP (no LDS traffic), one ds_bpermute for lane ^ 16
__device__ __forceinline__ float max_over_32(float v) {
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false)));
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, false)));
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x141, 0xF, 0xF, false)));
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x140, 0xF, 0xF, false)));
  return fmaxf(v, __shfl_xor(v, 16, 64));
}

template <int DT>
__global__ void __launch_bounds__(kBlock)
hs_fp8_hadamard_quant(const char* __restrict__ src, int64_t n, int64_t n_pad,
                      uint8_t* __restrict__ out, float* __restrict__ scales) {
  const int lane = threadIdx.x & 63;
  const int r = lane & 31, h = lane >> 5;
  const int64_t ntiles = (n_pad + 1023) / 1024;
  const int64_t nblocks = (n_pad + 127) / 128;
  const int64_t wave0 = (int64_t(blockIdx.x) * kBlock + threadIdx.x) >> 6;
  const int64_t nwaves = (int64_t(gridDim.x) * kBlock) >> 6;
  // (prefetching the next tile's half rows before the MFMA chain was tried:
  // 100 VGPRs instead of 48, no faster -- profiles/r3/s2/fp8_host_timed_callE.jsonl)
  for (int64_t tile = wave0; tile < ntiles; tile += nwaves) {
    float x[16];
    load_half_row<DT>(src, (tile * 32 + r) * 32 + 16 * h, n, x);
    floatx16 acc = {};
#pragma unroll
    for (int t = 0; t < 16; ++t)
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(x[t], hada(16 * h + t, r), acc, 0, 0, 0);
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      float amax = fmaxf(fmaxf(finite_abs(acc[4 * g4]), finite_abs(acc[4 * g4 + 1])),
                         fmaxf(finite_abs(acc[4 * g4 + 2]), finite_abs(acc[4 * g4 + 3])));
      amax = max_over_32(amax);
      const float scale = amax > 0.f ? amax / kFp8Max : 1.f;
      const float inv = 1.f / scale;
      const int64_t blk = tile * 8 + 2 * g4 + h;
      if (r == 0 && blk < nblocks) scales[blk] = scale;
      float v[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = fminf(fmaxf(acc[4 * g4 + q] * inv, -kFp8Max), kFp8Max);
      // byte q of `w` = row q + 8 g4 + 4 h, column r.  A 4x4 byte transpose
      // over each quad of lanes (two DPP quad-perm exchanges + v_perm_b32)
      // leaves lane r with row (r & 3) + 8 g4 + 4 h, columns (r & ~3) .. +3:
      // one 4-B store per lane, 256 contiguous bytes per wave instruction,
      // instead of 4 one-byte stores.
      uint32_t w = static_cast<uint32_t>(__builtin_amdgcn_cvt_pk_fp8_f32(v[0], v[1], 0, false));
      w = static_cast<uint32_t>(__builtin_amdgcn_cvt_pk_fp8_f32(v[2], v[3], static_cast<int>(w), true));
      {
        const float a4[4] = {acc[4 * g4], acc[4 * g4 + 1], acc[4 * g4 + 2], acc[4 * g4 + 3]};
        w = fp8_fix_nonfinite(w, a4);
      }
      uint32_t o = static_cast<uint32_t>(
          __builtin_amdgcn_mov_dpp(static_cast<int>(w), 0xB1, 0xF, 0xF, false));  // lane ^ 1
      w = __builtin_amdgcn_perm(o, w, (r & 1) ? 0x03070105u : 0x06020400u);
      o = static_cast<uint32_t>(
          __builtin_amdgcn_mov_dpp(static_cast<int>(w), 0x4E, 0xF, 0xF, false));  // lane ^ 2
      w = __builtin_amdgcn_perm(o, w, (r & 2) ? 0x03020706u : 0x05040100u);
      const int64_t row0 = (tile * 32 + (r & 3) + 8 * g4 + 4 * h) * 32;
      if (row0 < n_pad) *reinterpret_cast<uint32_t*>(out + row0 + (r & ~3)) = w;
    }
  }
}

// 16-bit inputs (bf16 / f16): the same rotation on the 16-bit MFMA,
// v_mfma_f32_32x32x16_{bf16,f16}: K = 16 per instruction, so a 32x32 tile
// takes 2 MFMAs instead of 16 f32 ones (~64 matrix-pipe cycles per KiB of
// output instead of ~256, which no longer hide under the tile's HBM traffic).
// The +-1 entries and the 16-bit inputs are exact; the products are summed
// inside the MFMA in fp32, in the hardware's own order, so a result can differ
// from the k-ordered fp32 reference in its last bit (tests bound the fp8 codes).
// Operand maps (CDNA guide 3, 32x32x16): lane l, r = l&31, h = l>>5 holds
//   A[row r][k = 8h + j], B[k = 8h + j][col r], j = 0..7, per K-step s (+16 s)
// i.e. the A fragment of step s is the 16 contiguous bytes X[r][16s + 8h ..+7]:
// one 16-B load, and the two loads of a wave cover the tile's 2 KiB exactly.
// C/D is the f32 form's map, so the epilogue is the one above.
typedef short hs_i16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 hs_bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 hs_f16x8 __attribute__((ext_vector_type(8)));

template <int DT>
__device__ __forceinline__ floatx16 mfma16(hs_i16x8 a, hs_i16x8 b, floatx16 c) {
  if constexpr (DT == kBF16)
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(hs_bf16x8, a),
                                                   __builtin_bit_cast(hs_bf16x8, b), c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(hs_f16x8, a),
                                                  __builtin_bit_cast(hs_f16x8, b), c, 0, 0, 0);
}

template <int DT>
__device__ __forceinline__ hs_i16x8 load_a_frag(const char* src, int64_t e0, int64_t n) {
  hs_i16x8 a;
  if (e0 + 8 <= n && ((reinterpret_cast<uintptr_t>(src + e0 * 2) & 15) == 0)) {
    const mx_u32x4 t = __builtin_nontemporal_load(reinterpret_cast<const mx_u32x4*>(src + e0 * 2));
    a = __builtin_bit_cast(hs_i16x8, t);
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j)
      a[j] = (e0 + j < n) ? *reinterpret_cast<const short*>(src + (e0 + j) * 2) : short(0);
  }
  return a;
}

// Epilogue of one rotated tile: blockwise scales + e4m3 codes (see above).
__device__ __forceinline__ void hadamard_tile_store(const floatx16& acc, int64_t tile, int r,
                                                    int h, int64_t n_pad, int64_t nblocks,
                                                    uint8_t* __restrict__ out,
                                                    float* __restrict__ scales) {
#pragma unroll
  for (int g4 = 0; g4 < 4; ++g4) {
    float amax = fmaxf(fmaxf(finite_abs(acc[4 * g4]), finite_abs(acc[4 * g4 + 1])),
                       fmaxf(finite_abs(acc[4 * g4 + 2]), finite_abs(acc[4 * g4 + 3])));
    amax = max_over_32(amax);
    const float scale = amax > 0.f ? amax / kFp8Max : 1.f;
    const float inv = 1.f / scale;
    const int64_t blk = tile * 8 + 2 * g4 + h;
    if (r == 0 && blk < nblocks) scales[blk] = scale;
    float v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = fminf(fmaxf(acc[4 * g4 + q] * inv, -kFp8Max), kFp8Max);
    uint32_t w = static_cast<uint32_t>(__builtin_amdgcn_cvt_pk_fp8_f32(v[0], v[1], 0, false));
    w = static_cast<uint32_t>(__builtin_amdgcn_cvt_pk_fp8_f32(v[2], v[3], static_cast<int>(w), true));
    {
      const float a4[4] = {acc[4 * g4], acc[4 * g4 + 1], acc[4 * g4 + 2], acc[4 * g4 + 3]};
      w = fp8_fix_nonfinite(w, a4);
    }
    uint32_t o = static_cast<uint32_t>(
        __builtin_amdgcn_mov_dpp(static_cast<int>(w), 0xB1, 0xF, 0xF, false));  // lane ^ 1
    w = __builtin_amdgcn_perm(o, w, (r & 1) ? 0x03070105u : 0x06020400u);
    o = static_cast<uint32_t>(
        __builtin_amdgcn_mov_dpp(static_cast<int>(w), 0x4E, 0xF, 0xF, false));  // lane ^ 2
    w = __builtin_amdgcn_perm(o, w, (r & 2) ? 0x03020706u : 0x05040100u);
    const int64_t row0 = (tile * 32 + (r & 3) + 8 * g4 + 4 * h) * 32;
    if (row0 < n_pad) __builtin_nontemporal_store(w, reinterpret_cast<uint32_t*>(out + row0 + (r & ~3)));
  }
}

// U tiles per iteration (2 A-fragment loads each): 2U 16-B loads in flight
// per lane before the first MFMA (one tile per iteration ran at 4.2 TB/s,
// latency-bound with 2 loads in flight).
template <int DT, int U>
__global__ void __launch_bounds__(kBlock)
hs_fp8_hadamard_quant16(const char* __restrict__ src, int64_t n, int64_t n_pad,
                        uint8_t* __restrict__ out, float* __restrict__ scales) {
  const int lane = threadIdx.x & 63;
  const int r = lane & 31, h = lane >> 5;
  const int64_t ntiles = (n_pad + 1023) / 1024;
  const int64_t nblocks = (n_pad + 127) / 128;
  const int64_t wave0 = (int64_t(blockIdx.x) * kBlock + threadIdx.x) >> 6;
  const int64_t nwaves = (int64_t(gridDim.x) * kBlock) >> 6;
  // B fragments: H[16 s + 8 h + j][r] as 16-bit +-1 (bf16 0x3F80/0xBF80, f16 0x3C00/0xBC00)
  const short one = (DT == kBF16) ? short(0x3F80) : short(0x3C00);
  hs_i16x8 b0, b1;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    b0[j] = (__popc((8 * h + j) & r) & 1) ? short(one | 0x8000) : one;
    b1[j] = (__popc((16 + 8 * h + j) & r) & 1) ? short(one | 0x8000) : one;
  }
  // wave-uniform fast path: every load of the U tiles in bounds and 16-B
  // aligned -> 2U vector loads issued back to back (a per-load bounds branch
  // made the compiler wait for each load before the next one)
  const bool aligned = (reinterpret_cast<uintptr_t>(src) & 15) == 0;
  for (int64_t t0 = wave0 * U; t0 < ntiles; t0 += nwaves * U) {
    hs_i16x8 a[U][2];
    if (aligned && (t0 + U) * 1024 <= n) {
      const mx_u32x4* p = reinterpret_cast<const mx_u32x4*>(src) + ((t0 * 32 + r) * 32 + 8 * h) / 8;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        a[u][0] = __builtin_bit_cast(hs_i16x8, __builtin_nontemporal_load(p + u * 128));
        a[u][1] = __builtin_bit_cast(hs_i16x8, __builtin_nontemporal_load(p + u * 128 + 2));
      }
    } else {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t e0 = ((t0 + u) * 32 + r) * 32 + 8 * h;  // past the end: zeros
        a[u][0] = load_a_frag<DT>(src, e0, n);
        a[u][1] = load_a_frag<DT>(src, e0 + 16, n);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (t0 + u >= ntiles) break;
      floatx16 acc = {};
      acc = mfma16<DT>(a[u][0], b0, acc);
      acc = mfma16<DT>(a[u][1], b1, acc);
      hadamard_tile_store(acc, t0 + u, r, h, n_pad, nblocks, out, scales);
    }
  }
}

// Dequantization on the matrix cores: X = (Q H) * s / 32 with Q the e4m3
// codes widened to bf16 (exact: 3 mantissa bits, exponents -9..8) and fed to
// v_mfma_f32_32x32x16_bf16 (2 per tile).  Every e4m3 value is a multiple of
// 2^-9 below 448, so a row sum of 32 of them (|sum| < 2^14) is exact in fp32
// whatever order the MFMA adds in: the only rounding is the product with the
// block scale (the /32 is exact) -- ``ops/quant.py`` computes the same, so GPU
// and CPU restores of a blob are bit-identical.  (The fp8 MFMA,
// v_mfma_f32_32x32x16_fp8_fp8, is not used: on a 65 613-element test its
// sums differed from the exact ones in the last bit -- subnormal e4m3 inputs
// are the suspect.)
// Operands (lane l, r = l&31, h = l>>5): the lane's 16 contiguous codes of
// row r, k = 16h .. 16h+15, are its A fragments of steps 0 and 1 (k = 16h +
// 8s + j); B holds H[16h + 8s + j][r] (bf16 +-1).  C/D as the quant kernels:
// register quad g4 = rows 8g4 + 4h + 0..3, column r, one block scale.
// 16-bit destinations leave through a 4x4 lane-quad transpose (3 DPP moves
// per quad) as 8-B stores, 256 contiguous bytes per wave instruction.
// 8 e4m3 codes (two words) -> 8 bf16 (exact: the f32 value's upper half)
__device__ __forceinline__ hs_i16x8 fp8x8_to_bf16x8(uint32_t w0, uint32_t w1) {
  hs_i16x8 o;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    o[j] = static_cast<short>(__float_as_uint(fp8_byte_to_f32(w0, j)) >> 16);
    o[4 + j] = static_cast<short>(__float_as_uint(fp8_byte_to_f32(w1, j)) >> 16);
  }
  return o;
}

template <int DT>
__device__ __forceinline__ uint32_t pack16(float lo, float hi) {
  uint32_t a, b;
  if constexpr (DT == kBF16) {
    a = f32_to_bf16(lo);
    b = f32_to_bf16(hi);
  } else {
    asm volatile("" : "+v"(lo), "+v"(hi));  // f32 products, then RNE (store_from_f32)
    a = __builtin_bit_cast(uint16_t, static_cast<_Float16>(lo));
    b = __builtin_bit_cast(uint16_t, static_cast<_Float16>(hi));
  }
  return a | (b << 16);
}

template <int DT, int U>
__global__ void __launch_bounds__(kBlock)
hs_fp8_hadamard_dequant8(const uint8_t* __restrict__ q, const float* __restrict__ scales,
                         int64_t n, int64_t n_pad, char* __restrict__ dst) {
  constexpr int DES = (DT == kF32) ? 4 : (DT == kF64 ? 8 : 2);
  const int lane = threadIdx.x & 63;
  const int r = lane & 31, h = lane >> 5;
  const int64_t ntiles = (n_pad + 1023) / 1024;
  const int64_t wave0 = (int64_t(blockIdx.x) * kBlock + threadIdx.x) >> 6;
  const int64_t nwaves = (int64_t(gridDim.x) * kBlock) >> 6;
  hs_i16x8 b0, b1;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    b0[j] = (__popc((16 * h + j) & r) & 1) ? short(0xBF80) : short(0x3F80);
    b1[j] = (__popc((16 * h + 8 + j) & r) & 1) ? short(0xBF80) : short(0x3F80);
  }
  const bool vec_out = (DES == 2) && (reinterpret_cast<uintptr_t>(dst) & 7) == 0;
  for (int64_t t0 = wave0 * U; t0 < ntiles; t0 += nwaves * U) {
    mx_u32x4 a[U];
    float sc[U][4];
#pragma unroll
    for (int u = 0; u < U; ++u) {  // q holds n_pad bytes (a multiple of 32)
      const int64_t e0 = ((t0 + u) * 32 + r) * 32 + 16 * h;
      a[u] = (e0 + 16 <= n_pad) ? __builtin_nontemporal_load(reinterpret_cast<const mx_u32x4*>(q + e0))
                                : mx_u32x4{0, 0, 0, 0};
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int64_t blk = (t0 + u) * 8 + 2 * g4 + h;
        sc[u][g4] = (blk * 128 < n_pad) ? scales[blk] : 0.f;
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t tile = t0 + u;
      if (tile >= ntiles) break;
      floatx16 acc = {};
      acc = mfma16<kBF16>(fp8x8_to_bf16x8(a[u].x, a[u].y), b0, acc);
      acc = mfma16<kBF16>(fp8x8_to_bf16x8(a[u].z, a[u].w), b1, acc);
      if (vec_out && (tile + 1) * 1024 <= n) {
        if constexpr (DES == 2) {
#pragma unroll
          for (int g4 = 0; g4 < 4; ++g4) {
            const float s = sc[u][g4] * (1.f / 32.f);
            // lane slot i = row 8 g4 + 4 h + i, column r (two 16-bit rows per word)
            uint32_t A = pack16<DT>(acc[4 * g4] * s, acc[4 * g4 + 1] * s);
            uint32_t B = pack16<DT>(acc[4 * g4 + 2] * s, acc[4 * g4 + 3] * s);
            // stage 1 (lanes ^ 1): 2x2 transposes of 16-bit elements
            const uint32_t A1 = static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(A), 0xB1, 0xF, 0xF, false));
            const uint32_t B1 = static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(B), 0xB1, 0xF, 0xF, false));
            if (r & 1) {
              A = __builtin_amdgcn_perm(A, A1, 0x07060302u);  // (partner.hi, mine.hi)
              B = __builtin_amdgcn_perm(B, B1, 0x07060302u);
            } else {
              A = __builtin_amdgcn_perm(A1, A, 0x05040100u);  // (mine.lo, partner.lo)
              B = __builtin_amdgcn_perm(B1, B, 0x05040100u);
            }
            // stage 2 (lanes ^ 2): swap 32-bit words
            const uint32_t X = (r & 2) ? A : B;
            const uint32_t R = static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(X), 0x4E, 0xF, 0xF, false));
            if (r & 2) A = R; else B = R;
            const int64_t row = tile * 32 + 8 * g4 + 4 * h + (r & 3);
            mx_u32x2 w;
            w.x = A;
            w.y = B;
            __builtin_nontemporal_store(w, reinterpret_cast<mx_u32x2*>(dst + (row * 32 + (r & ~3)) * 2));
          }
        }
      } else {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int row = (i & 3) + 8 * (i >> 2) + 4 * h;
          const int64_t e = (tile * 32 + row) * 32 + r;
          if (e < n) store_from_f32(dst + e * DES, DT, acc[i] * (sc[u][i >> 2] * (1.f / 32.f)));
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// ---- hs64 blob checksum (definition: csrc/hschk.cpp) -------------------------
// Grid-stride over the blob's 64-bit words; each lane mixes its words with
// their global index, a wave reduces with shuffles and adds its partial sum
// to one device accumulator (a vector atomic per wave).  Memory-bound: a
// staged blob is hashed in HBM right before its DMA to the host.
constexpr uint64_t kHsM1 = 0x9E3779B97F4A7C15ull;

__device__ __forceinline__ uint64_t hs_mix64(uint64_t x) {
  x ^= x >> 30;
  x *= 0xBF58476D1CE4E5B9ull;
  x ^= x >> 27;
  x *= 0x94D049BB133111EBull;
  x ^= x >> 31;
  return x;
}

__global__ void __launch_bounds__(kBlock)
hs_hash64(const uint8_t* __restrict__ p, uint64_t n, uint64_t first_word,
          unsigned long long* __restrict__ acc) {
  const uint64_t nw = n / 8;
  const uint64_t tid = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  const uint64_t nthr = uint64_t(gridDim.x) * blockDim.x;
  uint64_t s = 0;
  uint64_t done = 0;  // words covered by the vector loop
  if ((reinterpret_cast<uintptr_t>(p) & 15) == 0) {
    // 16 B per lane per load; the position keys advance by adding a
    // constant instead of a 64-bit multiply per word
    // (four independent loads in flight per lane: the launch is kept narrow
    // on purpose, see hsg_hash64, so each lane must cover latency itself)
    const uint64_t npair = nw / 2;
    const ulonglong2* v = reinterpret_cast<const ulonglong2*>(p);
    uint64_t key = (first_word + 2 * tid + 1) * kHsM1;
    const uint64_t dkey = 2 * nthr * kHsM1;
    uint64_t j = tid;
    for (; j + 3 * nthr < npair; j += 4 * nthr, key += 4 * dkey) {
      const ulonglong2 w0 = v[j], w1 = v[j + nthr], w2 = v[j + 2 * nthr], w3 = v[j + 3 * nthr];
      s += hs_mix64(w0.x ^ key) + hs_mix64(w0.y ^ (key + kHsM1));
      s += hs_mix64(w1.x ^ (key + dkey)) + hs_mix64(w1.y ^ (key + dkey + kHsM1));
      s += hs_mix64(w2.x ^ (key + 2 * dkey)) + hs_mix64(w2.y ^ (key + 2 * dkey + kHsM1));
      s += hs_mix64(w3.x ^ (key + 3 * dkey)) + hs_mix64(w3.y ^ (key + 3 * dkey + kHsM1));
    }
    for (; j < npair; j += nthr, key += dkey) {
      const ulonglong2 w = v[j];
      s += hs_mix64(w.x ^ key) + hs_mix64(w.y ^ (key + kHsM1));
    }
    done = 2 * npair;
  } else if ((reinterpret_cast<uintptr_t>(p) & 7) == 0) {
    const uint64_t* w = reinterpret_cast<const uint64_t*>(p);
    uint64_t key = (first_word + tid + 1) * kHsM1;
    const uint64_t dkey = nthr * kHsM1;
    for (uint64_t i = tid; i < nw; i += nthr, key += dkey) s += hs_mix64(w[i] ^ key);
    done = nw;
  } else {
    for (uint64_t i = tid; i < nw; i += nthr) {
      uint64_t w = 0;
#pragma unroll
      for (int k = 0; k < 8; ++k) w |= uint64_t(p[8 * i + k]) << (8 * k);
      s += hs_mix64(w ^ ((first_word + i + 1) * kHsM1));
    }
    done = nw;
  }
  if (tid == 0) {
    // the odd word after the pairs, then the zero-padded tail
    for (uint64_t i = done; i < nw; ++i) {
      uint64_t w = 0;
      for (int k = 0; k < 8; ++k) w |= uint64_t(p[8 * i + k]) << (8 * k);
      s += hs_mix64(w ^ ((first_word + i + 1) * kHsM1));
    }
    const uint64_t tail = n - 8 * nw;
    if (tail) {
      uint64_t w = 0;
      for (uint64_t k = 0; k < tail; ++k) w |= uint64_t(p[8 * nw + k]) << (8 * k);
      s += hs_mix64(w ^ ((first_word + nw + 1) * kHsM1));
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
  if ((threadIdx.x & 63) == 0) atomicAdd(acc, static_cast<unsigned long long>(s));
}

// Host-side state: pinned pool, copy streams, launch helpers.
// ---------------------------------------------------------------------------

struct PinnedPool {
  std::mutex mu;
  std::multimap<size_t, void*> free_blocks;      // size -> ptr
  std::unordered_map<void*, size_t> live;       // ptr -> size
  size_t cached_bytes = 0;                        // total allocated (live + free)
  size_t in_use_bytes = 0;
  std::unordered_map<void*, int> node;            // blocks bound to a NUMA node
};
PinnedPool g_pool;

struct StreamKey {
  int dev, slot;
  bool operator<(const StreamKey& o) const { return dev != o.dev ? dev < o.dev : slot < o.slot; }
};
std::mutex g_stream_mu;
std::map<StreamKey, hipStream_t> g_streams;
std::map<StreamKey, hipEvent_t> g_events;

std::map<StreamKey, int> g_stream_prio;  // slots created with a priority (hsg_stream_priority)

int get_stream(int dev, int slot, hipStream_t* out, hipEvent_t* ev) {
  std::lock_guard<std::mutex> g(g_stream_mu);
  StreamKey k{dev, slot};
  auto it = g_streams.find(k);
  if (it == g_streams.end()) {
    HS_CHECK(hipSetDevice(dev));
    // default priority: lowest-priority copy streams made a concurrent
    // training step 45 % slower instead of 18 % (profiles/overlap/priority.md)
    hipStream_t s;
    auto pr = g_stream_prio.find(k);
    if (pr != g_stream_prio.end())
      HS_CHECK(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, pr->second));
    else
      HS_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t e;
    HS_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    g_streams[k] = s;
    g_events[k] = e;
    it = g_streams.find(k);
  }
  *out = it->second;
  *ev = g_events[k];
  return 0;
}

// Build the tile table for a descriptor batch.  Tile size adapts to the
// batch so that a launch always has >= ~4096 tiles when there is enough work
// (>> 256 CUs: every CU gets several 4-wave workgroups and enough loads in
// flight to reach HBM / PCIe bandwidth), and never below 32 KiB (tile-table
// overhead) or above 1 MiB.
int elem_bytes_host(int32_t dt) {
  switch (dt) {
    case kRaw1: return 1;
    case kRaw2: case kF16: case kBF16: return 2;
    case kRaw4: case kF32: return 4;
    case kRaw8: case kF64: return 8;
    default: return 16;
  }
}

void build_tiles(const CopyDesc* descs, int n, std::vector<Tile>* tiles) {
  int64_t total_bytes = 0;
  for (int i = 0; i < n; ++i) total_bytes += descs[i].numel * elem_bytes_host(descs[i].src_dtype);
  int64_t tile_bytes = total_bytes / 4096;
  tile_bytes = (tile_bytes + 16383) / 16384 * 16384;
  tile_bytes = std::max<int64_t>(32 << 10, std::min<int64_t>(kTileBytes, tile_bytes));
  for (int i = 0; i < n; ++i) {
    const CopyDesc& d = descs[i];
    const int es = elem_bytes_host(d.src_dtype);
    int64_t total, step;
    if (d.flags & 1) {
      total = d.numel * es;  // bytes
      step = tile_bytes;
    } else if (d.flags & 2) {
      const int vw = d.flags >> 8;
      total = d.sizes[0] * (d.sizes[1] * es / vw);  // vectors
      step = std::max<int64_t>(kBlock, tile_bytes / vw);
    } else if (d.flags & 4) {
      total = d.sizes[0] * ((d.sizes[1] + 63) / 64) * ((d.sizes[2] + 63) / 64);  // 64x64 blocks
      step = std::max<int64_t>(1, tile_bytes / (64 * 64 * es));
    } else {
      total = d.numel;
      // elements per tile on the strided/cast path (multiple of the per-block run)
      step = std::max<int64_t>(kBlock * 8, tile_bytes / es / (kBlock * 8) * (kBlock * 8));
    }
    for (int64_t b = 0; b < total; b += step) {
      tiles->push_back(Tile{i, 0, b, std::min(total, b + step)});
    }
  }
}

}  // namespace

extern "C" {

const char* hsg_last_error() { return g_err; }

int hsg_device_count() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

// PCI domain / bus / device of HIP device `dev` (three attribute queries:
// hipGetDeviceProperties, behind torch.cuda.get_device_properties, took
// ~130 ms the first time in a process).  0 on success.
int hsg_pci_location(int dev, int* domain, int* bus, int* device) {
  if (hipDeviceGetAttribute(domain, hipDeviceAttributePciDomainId, dev) != hipSuccess ||
      hipDeviceGetAttribute(bus, hipDeviceAttributePciBusId, dev) != hipSuccess ||
      hipDeviceGetAttribute(device, hipDeviceAttributePciDeviceId, dev) != hipSuccess)
    return -1;
  return 0;
}

// ---- pinned pool ----------------------------------------------------------
//
// Pool blocks are anonymous memory backed by transparent huge pages and
// registered with the GPU (hipHostRegister), not hipHostMalloc blocks: the
// copy engines see both the same (SDMA device -> host 56.9 GB/s, host ->
// device 57.5 GB/s), but the CPU side -- pread()s of a restore into the
// block, pwrite()s of a take out of it -- runs ~1.5x faster on 2 MiB pages
// (pread into hipHostMalloc memory 88 GB/s, into THP-backed memory 131 GB/s,
// 16 threads; scripts/probes/pinned_thp_probe.py, profiles/pinned/).  Registering
// pre-faulted huge pages costs ~2 ms per GiB, once per pool block.  Any
// failure falls back to hipHostMalloc.

struct MappedBlock {
  void* base;
  size_t len;
};
std::mutex g_mapped_mu;
std::unordered_map<void*, MappedBlock> g_mapped;  // registered block -> its mapping

void* alloc_thp_registered(size_t want, int node = -1) {
  constexpr size_t kHuge = size_t(2) << 20;
  const size_t len = want + kHuge;
  void* base = mmap(nullptr, len, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  if (base == MAP_FAILED) return nullptr;
  char* p = reinterpret_cast<char*>((reinterpret_cast<uintptr_t>(base) + kHuge - 1) & ~(kHuge - 1));
  if (node >= 0 && node < 64) {
    // pages on `node` whichever CPU touches them first (MPOL_BIND = 2)
    unsigned long mask = 1ul << node;
    if (syscall(SYS_mbind, p, want, 2, &mask, 65ul, 0u) != 0) {
      munmap(base, len);
      return nullptr;
    }
  }
  (void)madvise(p, want, MADV_HUGEPAGE);
  // fault every page in now (a huge page per 2 MiB where the kernel grants
  // one): registration then maps resident pages, and no copy pays a fault.
  // The kernel zeroes each page on its first touch; a large block is split
  // over 4 threads so a cold process's first blocks -- a restore's first
  // reads -- wait less.
  const size_t kSplit = size_t(32) << 20;
  const int nt = static_cast<int>(std::min<size_t>(4, std::max<size_t>(1, want / kSplit)));
  auto touch = [p](size_t lo, size_t hi) {
    for (size_t off = lo; off < hi; off += 4096) p[off] = 0;
  };
  if (nt <= 1) {
    touch(0, want);
  } else {
    const size_t per = (want / nt + kHuge - 1) / kHuge * kHuge;
    std::vector<std::thread> th;
    for (int i = 1; i < nt; ++i) {
      const size_t lo = std::min(want, per * i), hi = std::min(want, per * (i + 1));
      if (lo >= hi) continue;
      try {
        th.emplace_back(touch, lo, hi);
      } catch (...) {  // no thread to be had: touch this part here
        touch(lo, hi);
      }
    }
    touch(0, std::min(want, per));
    for (auto& t : th) t.join();
  }
  if (hipHostRegister(p, want, hipHostRegisterDefault) != hipSuccess) {
    (void)hipGetLastError();
    munmap(base, len);
    return nullptr;
  }
  std::lock_guard<std::mutex> g(g_mapped_mu);
  g_mapped[p] = MappedBlock{base, len};
  return p;
}

void free_pinned_block(void* p) {
  {
    std::lock_guard<std::mutex> g(g_pool.mu);
    g_pool.node.erase(p);
  }
  MappedBlock mb{nullptr, 0};
  {
    std::lock_guard<std::mutex> g(g_mapped_mu);
    auto it = g_mapped.find(p);
    if (it != g_mapped.end()) {
      mb = it->second;
      g_mapped.erase(it);
    }
  }
  if (mb.base != nullptr) {
    (void)hipHostUnregister(p);
    munmap(mb.base, mb.len);
  } else {
    (void)hipHostFree(p);
  }
}

void* hsg_pinned_acquire(uint64_t nbytes) {
  size_t want = (std::max<size_t>(nbytes, 1) + kPinnedGranule - 1) / kPinnedGranule * kPinnedGranule;
  {
    std::lock_guard<std::mutex> g(g_pool.mu);
    auto it = g_pool.free_blocks.lower_bound(want);
    // best fit, but do not hand out a block more than 2x the request
    if (it != g_pool.free_blocks.end() && it->first <= 2 * want) {
      void* p = it->second;
      size_t sz = it->first;
      g_pool.free_blocks.erase(it);
      g_pool.live[p] = sz;
      g_pool.in_use_bytes += sz;
      return p;
    }
  }
  void* p = alloc_thp_registered(want);
  hipError_t e = hipSuccess;
  if (p == nullptr) e = hipHostMalloc(&p, want, hipHostMallocDefault);
  if (e != hipSuccess) {
    // out of pinnable memory: drop the cache and retry once
    std::vector<void*> drop;
    {
      std::lock_guard<std::mutex> g(g_pool.mu);
      for (auto& kv : g_pool.free_blocks) { drop.push_back(kv.second); g_pool.cached_bytes -= kv.first; }
      g_pool.free_blocks.clear();
    }
    for (void* q : drop) free_pinned_block(q);
    p = alloc_thp_registered(want);
    e = p != nullptr ? hipSuccess : hipHostMalloc(&p, want, hipHostMallocDefault);
    if (e != hipSuccess) {
      set_err("hipHostMalloc", e);
      return nullptr;
    }
  }
  std::lock_guard<std::mutex> g(g_pool.mu);
  g_pool.live[p] = want;
  g_pool.cached_bytes += want;
  g_pool.in_use_bytes += want;
  return p;
}

// Blocks released while the pool caches more than this are returned to the
// driver instead of being kept (bounds pinned host memory per process).
uint64_t g_pool_limit = ~uint64_t(0);

void hsg_pinned_set_limit(uint64_t bytes) { g_pool_limit = bytes; }

// A pinned block whose pages are bound to NUMA `node` (an async take's UVM
// capture copies a table into a block on the table's own node, then writes
// it from there: engine/uvm_capture.py).  Cached separately from the
// unplaced blocks; node < 0 is hsg_pinned_acquire.
void* hsg_pinned_acquire_on(uint64_t nbytes, int node) {
  if (node < 0) return hsg_pinned_acquire(nbytes);
  const size_t want =
      (std::max<size_t>(nbytes, 1) + kPinnedGranule - 1) / kPinnedGranule * kPinnedGranule;
  {
    std::lock_guard<std::mutex> g(g_pool.mu);
    for (auto it = g_pool.free_blocks.lower_bound(want);
         it != g_pool.free_blocks.end() && it->first <= 2 * want; ++it) {
      auto nd = g_pool.node.find(it->second);
      if (nd == g_pool.node.end() || nd->second != node) continue;
      void* p = it->second;
      const size_t sz = it->first;
      g_pool.free_blocks.erase(it);
      g_pool.live[p] = sz;
      g_pool.in_use_bytes += sz;
      return p;
    }
  }
  void* p = alloc_thp_registered(want, node);
  if (p == nullptr) return nullptr;  // the caller falls back to an unplaced block
  std::lock_guard<std::mutex> g(g_pool.mu);
  g_pool.live[p] = want;
  g_pool.node[p] = node;
  g_pool.cached_bytes += want;
  g_pool.in_use_bytes += want;
  return p;
}

int hsg_pinned_release(void* p) {
  void* drop = nullptr;
  {
    std::lock_guard<std::mutex> g(g_pool.mu);
    auto it = g_pool.live.find(p);
    if (it == g_pool.live.end()) return -1;
    g_pool.in_use_bytes -= it->second;
    if (g_pool.cached_bytes > g_pool_limit) {
      g_pool.cached_bytes -= it->second;
      drop = p;
    } else {
      g_pool.free_blocks.emplace(it->second, p);
    }
    g_pool.live.erase(it);
  }
  if (drop) free_pinned_block(drop);
  return 0;
}

void hsg_pinned_stats(uint64_t* cached, uint64_t* in_use) {
  std::lock_guard<std::mutex> g(g_pool.mu);
  *cached = g_pool.cached_bytes;
  *in_use = g_pool.in_use_bytes;
}

uint64_t hsg_pinned_trim() {
  std::vector<std::pair<size_t, void*>> drop;
  {
    std::lock_guard<std::mutex> g(g_pool.mu);
    for (auto& kv : g_pool.free_blocks) drop.emplace_back(kv.first, kv.second);
    g_pool.free_blocks.clear();
    for (auto& kv : drop) g_pool.cached_bytes -= kv.first;
  }
  uint64_t freed = 0;
  for (auto& kv : drop) { free_pinned_block(kv.second); freed += kv.first; }
  return freed;
}

int hsg_restore_idle_blocks(int dev, uint64_t* ptrs, uint64_t* sizes, int max);

// Test hook: overwrite every idle block of the restore's device pools (on
// `dev`) and of the pinned host pool with `byte`, so a test can show that no
// restore reads bytes an earlier one left behind.  Returns the blocks written.
int hsg_poison_idle_pools(int dev, int byte) {
  std::vector<uint64_t> ptrs(4096), sizes(4096);
  const int n = hsg_restore_idle_blocks(dev, ptrs.data(), sizes.data(), 4096);
  HS_CHECK(hipSetDevice(dev));
  for (int i = 0; i < n; ++i)
    HS_CHECK(hipMemset(reinterpret_cast<void*>(ptrs[i]), byte, sizes[i]));
  HS_CHECK(hipDeviceSynchronize());
  int m = 0;
  std::lock_guard<std::mutex> g(g_pool.mu);
  for (auto& kv : g_pool.free_blocks) {
    std::memset(kv.second, byte, kv.first);
    ++m;
  }
  return n + m;
}

// ---- DMA copies on side streams --------------------------------------------

// Copy `n` bytes between host and device on copy stream (dev, slot), ordered
// after all work already queued on `producer` when `has_producer` is set (a
// torch stream; handle 0 = the legacy default stream).
// kind: 0 = D2H, 1 = H2D, 2 = D2D.  If `sync` is nonzero the call blocks until
// the copy is done (ctypes releases the GIL around it).
// ---- uncached device blocks (SDMA upload targets, csrc/hsdma.hip) ----------
//
// hipDeviceMallocUncached memory, cached per device by size (best fit up to
// 2x, 2 MiB granules): the restore's encoded frames are uploaded into it by
// SDMA and read once by the decode kernel, never through a stale L2 line.
extern "C" void* hsg_rt_vmm_alloc(int dev, uint64_t nbytes, int uncached);
extern "C" int hsg_rt_vmm_free(void* p);
extern "C" const char* hsg_rt_last_error();

struct UncachedPool {
  std::mutex mu;
  std::map<int, std::multimap<size_t, void*>> free_blocks;  // dev -> size -> block
  std::unordered_map<void*, std::pair<int, size_t>> live;
  size_t cached_bytes = 0;
};
UncachedPool g_upool;

void* hsg_uncached_acquire(int dev, uint64_t nbytes) {
  constexpr size_t kGranule = size_t(2) << 20;
  const size_t want = (std::max<size_t>(nbytes, 1) + kGranule - 1) / kGranule * kGranule;
  {
    std::lock_guard<std::mutex> g(g_upool.mu);
    auto& fl = g_upool.free_blocks[dev];
    auto it = fl.lower_bound(want);
    if (it != fl.end() && it->first <= 2 * want) {
      void* p = it->second;
      g_upool.live[p] = {dev, it->first};
      fl.erase(it);
      return p;
    }
  }
  // hsg_rt_vmm_alloc (hshost.hip): a freed block's address is never handed
  // out again (re-used addresses of freed uncached blocks were written
  // through stale translations, profiles/r6/trim/)
  void* p = hsg_rt_vmm_alloc(dev, want, 1);
  if (p == nullptr) {
    // drop this device's idle blocks and retry once
    std::vector<void*> drop;
    {
      std::lock_guard<std::mutex> g(g_upool.mu);
      auto& fl = g_upool.free_blocks[dev];
      for (auto& kv : fl) { drop.push_back(kv.second); g_upool.cached_bytes -= kv.first; }
      fl.clear();
    }
    for (void* q : drop) (void)hsg_rt_vmm_free(q);
    p = hsg_rt_vmm_alloc(dev, want, 1);
    if (p == nullptr) {
      snprintf(g_err, sizeof(g_err), "uncached block of %zu bytes: %s", want, hsg_rt_last_error());
      return nullptr;
    }
  }
  std::lock_guard<std::mutex> g(g_upool.mu);
  g_upool.live[p] = {dev, want};
  g_upool.cached_bytes += want;
  return p;
}

// Bytes the uncached pool holds (idle + in use, every device).
uint64_t hsg_uncached_bytes() {
  std::lock_guard<std::mutex> g(g_upool.mu);
  return g_upool.cached_bytes;
}

int hsg_uncached_release(void* p) {
  std::lock_guard<std::mutex> g(g_upool.mu);
  auto it = g_upool.live.find(p);
  if (it == g_upool.live.end()) return -1;
  g_upool.free_blocks[it->second.first].emplace(it->second.second, p);
  g_upool.live.erase(it);
  return 0;
}

// Free every idle uncached block; returns the bytes freed.
uint64_t hsg_uncached_trim() {
  std::vector<std::pair<int, void*>> drop;
  uint64_t freed = 0;
  {
    std::lock_guard<std::mutex> g(g_upool.mu);
    for (auto& dv : g_upool.free_blocks) {
      for (auto& kv : dv.second) {
        drop.emplace_back(dv.first, kv.second);
        freed += kv.first;
      }
      dv.second.clear();
    }
    g_upool.cached_bytes -= freed;
  }
  for (auto& d : drop) (void)hsg_rt_vmm_free(d.second);
  return freed;
}

int hsg_memcpy(int dev, int slot, void* dst, const void* src, uint64_t n, int kind,
               void* producer, int has_producer, int sync) {
  HS_CHECK(hipSetDevice(dev));
  hipStream_t s;
  hipEvent_t ev;
  int r = get_stream(dev, slot, &s, &ev);
  if (r) return r;
  // producer may be the legacy null stream (handle 0, torch's default stream):
  // the copy streams are non-blocking, so it must be joined explicitly too
  if (has_producer) {
    HS_CHECK(hipEventRecord(ev, static_cast<hipStream_t>(producer)));
    HS_CHECK(hipStreamWaitEvent(s, ev, 0));
  }
  hipMemcpyKind k = kind == 0 ? hipMemcpyDeviceToHost
                  : kind == 1 ? hipMemcpyHostToDevice : hipMemcpyDeviceToDevice;
  if (n) HS_CHECK(hipMemcpyAsync(dst, src, n, k, s));
  if (sync) HS_CHECK(hipStreamSynchronize(s));
  return 0;
}

// Make `consumer` (torch stream) wait for everything queued on copy stream
// (dev, slot) -- used after H2D restores so the trainer sees the data.
int hsg_stream_join(int dev, int slot, void* consumer) {
  HS_CHECK(hipSetDevice(dev));
  hipStream_t s;
  hipEvent_t ev;
  int r = get_stream(dev, slot, &s, &ev);
  if (r) return r;
  HS_CHECK(hipEventRecord(ev, s));
  HS_CHECK(hipStreamWaitEvent(static_cast<hipStream_t>(consumer), ev, 0));
  return 0;
}

int hsg_stream_sync(int dev, int slot) {
  HS_CHECK(hipSetDevice(dev));
  hipStream_t s;
  hipEvent_t ev;
  int r = get_stream(dev, slot, &s, &ev);
  if (r) return r;
  HS_CHECK(hipStreamSynchronize(s));
  return 0;
}

// Grid cap for the calling thread's launches (0 = none).  The async-take
// drain runs its staging threads with a cap so its kernels (HSZ1 encode,
// slab gathers) occupy only that many CUs while training continues: at full
// width the encoder made a concurrent Llama-3-8B training step ~30 % slower
// (profiles/overlap_iso/), and the drain is PCIe-bound anyway.
thread_local int t_grid_cap = 0;

int hsg_set_thread_grid_cap(int cap) {
  const int old = t_grid_cap;
  t_grid_cap = cap < 0 ? 0 : cap;
  return old;
}

int hsg_thread_grid_cap() { return t_grid_cap; }

// ---- hs64 on the copy streams -------------------------------------------------
// A ring of 8-byte device accumulators (+ pinned landing words) per device.
// Every hash takes the next ring entry, so threads that share a copy stream
// never share an accumulator; an entry comes round again only after
// kHashRing later hashes, long after its result was read (each thread has at
// most one hash in flight).
constexpr int kHashRing = 4096;
struct HashRing {
  unsigned long long* acc = nullptr;
  uint64_t* host = nullptr;
  std::atomic<uint32_t> next{0};
};
std::mutex g_hash_mu;
std::map<int, HashRing> g_hash_rings;

int hash_ring(int dev, HashRing** out) {
  std::lock_guard<std::mutex> g(g_hash_mu);
  HashRing& h = g_hash_rings[dev];
  if (h.acc == nullptr) {
    HS_CHECK(hipSetDevice(dev));
    HS_CHECK(hipMalloc(reinterpret_cast<void**>(&h.acc), kHashRing * sizeof(unsigned long long)));
    HS_CHECK(hipHostMalloc(reinterpret_cast<void**>(&h.host), kHashRing * sizeof(uint64_t),
                           hipHostMallocDefault));
  }
  *out = &h;
  return 0;
}

// Enqueue hs64's partial sum of device bytes [p, p + n) (first word index
// `first_word`) on stream (dev, slot), ordered after everything queued so far
// on stream (dev, after_slot) when after_slot >= 0: the hash of a blob then
// runs beside its device->host copy (both only read it) instead of in front.
// Nothing is synchronised; *handle names the result for hsg_hash64_result.
//
// `max_grid` bounds the launch (<= 0: whole chip).  A full-width hash reads
// HBM at ~4 TB/s and slows concurrent SDMA reads of HBM by ~20 %
// (scripts/probes/hash_probe.py), while blobs only need hashing at the PCIe rate;
// the staging path therefore launches it narrow.
int hsg_hash64(int dev, int slot, int after_slot, const void* p, uint64_t n,
               uint64_t first_word, int max_grid, int* handle) {
  HS_CHECK(hipSetDevice(dev));
  hipStream_t s;
  hipEvent_t ev;
  int r = get_stream(dev, slot, &s, &ev);
  if (r) return r;
  if (after_slot >= 0 && after_slot != slot) {
    hipStream_t a;
    hipEvent_t aev;
    r = get_stream(dev, after_slot, &a, &aev);
    if (r) return r;
    HS_CHECK(hipEventRecord(aev, a));
    HS_CHECK(hipStreamWaitEvent(s, aev, 0));
  }
  HashRing* h;
  r = hash_ring(dev, &h);
  if (r) return r;
  const int k = static_cast<int>(h->next.fetch_add(1) % kHashRing);
  HS_CHECK(hipMemsetAsync(h->acc + k, 0, sizeof(unsigned long long), s));
  const uint64_t words = n / 8 + 1;
  int grid = static_cast<int>(std::min<uint64_t>((words + kBlock - 1) / kBlock, 256 * 8));
  if (max_grid > 0) grid = std::min(grid, max_grid);
  if (t_grid_cap > 0) grid = std::min(grid, t_grid_cap);
  hipLaunchKernelGGL(hs_hash64, dim3(std::max(grid, 1)), dim3(kBlock), 0, s,
                     static_cast<const uint8_t*>(p), n, first_word, h->acc + k);
  HS_CHECK(hipGetLastError());
  *handle = k;
  return 0;
}

// hs64's partial sum of device bytes [p, p + n) into the caller's device
// accumulator `acc` (one u64, zeroed here), on the caller's `stream`: the
// native restore hashes every uploaded blob on the stream that decodes it,
// into one accumulator per blob of its own (no shared ring to outrun).
int hsg_hash64_into(int dev, void* stream, const void* p, uint64_t n, uint64_t first_word,
                    int max_grid, void* acc) {
  HS_CHECK(hipSetDevice(dev));
  hipStream_t s = static_cast<hipStream_t>(stream);
  auto* a = static_cast<unsigned long long*>(acc);
  HS_CHECK(hipMemsetAsync(a, 0, sizeof(unsigned long long), s));
  const uint64_t words = n / 8 + 1;
  int grid = static_cast<int>(std::min<uint64_t>((words + kBlock - 1) / kBlock, 256 * 8));
  if (max_grid > 0) grid = std::min(grid, max_grid);
  hipLaunchKernelGGL(hs_hash64, dim3(std::max(grid, 1)), dim3(kBlock), 0, s,
                     static_cast<const uint8_t*>(p), n, first_word, a);
  HS_CHECK(hipGetLastError());
  return 0;
}

// The partial sum of hash `handle`, started on stream (dev, slot); waits for it.
int hsg_hash64_result(int dev, int slot, int handle, uint64_t* out) {
  HS_CHECK(hipSetDevice(dev));
  if (handle < 0 || handle >= kHashRing) return hipErrorInvalidValue;
  hipStream_t s;
  hipEvent_t ev;
  int r = get_stream(dev, slot, &s, &ev);
  if (r) return r;
  HashRing* h;
  r = hash_ring(dev, &h);
  if (r) return r;
  HS_CHECK(hipMemcpyAsync(h->host + handle, h->acc + handle, sizeof(uint64_t),
                          hipMemcpyDeviceToHost, s));
  HS_CHECK(hipStreamSynchronize(s));
  *out = h->host[handle];
  return 0;
}

// Create stream (dev, slot) at the device's highest priority (high != 0)
// when it is first used.  The native drain's hash stream: its tiny hs64
// launches and 8-byte read-backs otherwise queue behind a saturating
// training step's workgroups -- a GEMM loop on another stream cut a drain
// with hashing from 36 to 13.5 GB/s, without hashing it kept 35.6 GB/s
// (scripts/probes/drain_contention_probe.py, profiles/r3/drain_probe/).  Returns
// 1 if the stream already existed (its priority is unchanged).
int hsg_stream_priority(int dev, int slot, int high) {
  std::lock_guard<std::mutex> g(g_stream_mu);
  StreamKey k{dev, slot};
  if (g_streams.count(k)) return 1;
  int least = 0, greatest = 0;
  HS_CHECK(hipSetDevice(dev));
  HS_CHECK(hipDeviceGetStreamPriorityRange(&least, &greatest));
  g_stream_prio[k] = high ? greatest : least;
  return 0;
}

void* hsg_copy_stream(int dev, int slot) {
  hipStream_t s;
  hipEvent_t ev;
  if (get_stream(dev, slot, &s, &ev)) return nullptr;
  return s;
}

int hsg_sync_stream_handle(void* stream) {
  HS_CHECK(hipStreamSynchronize(static_cast<hipStream_t>(stream)));
  return 0;
}

uint64_t hsg_desc_size() { return sizeof(CopyDesc); }

// Load this library's code object on `dev` now (the runtime loads it at the
// first kernel launch otherwise: ~3 ms that fell into the first async_take's
// freeze launch).  Called from a helper thread while a first take plans.
int hsg_prewarm_module(int dev) {
  HS_CHECK(hipSetDevice(dev));
  hipFuncAttributes attr;
  HS_CHECK(hipFuncGetAttributes(&attr, reinterpret_cast<const void*>(&hs_copy_nd)));
  return 0;
}

// Batched strided copy / cast.  `descs` is a host array of `n` CopyDesc (see
// hipsnapshot/ops/native.py for the packing); `scratch` is a device (or
// host-mapped) workspace of at least hsg_copy_workspace_bytes() bytes used for
// the descriptor + tile tables (copied H2D on `stream`, so the host arrays may
// be reused as soon as this returns).  `stream` == null -> copy stream (dev,slot).
uint64_t hsg_copy_workspace_bytes(const void* descs, int n) {
  std::vector<Tile> tiles;
  build_tiles(static_cast<const CopyDesc*>(descs), n, &tiles);
  return sizeof(CopyDesc) * n + sizeof(Tile) * tiles.size() + 256;
}

int hsg_copy_nd(int dev, const void* descs, int n, void* workspace, uint64_t ws_bytes,
                void* pinned_stage, void* stream, int sync) {
  HS_CHECK(hipSetDevice(dev));
  if (n <= 0) return 0;
  std::vector<Tile> tiles;
  const CopyDesc* d = static_cast<const CopyDesc*>(descs);
  build_tiles(d, n, &tiles);
  if (tiles.empty()) return 0;
  const size_t dbytes = sizeof(CopyDesc) * n;
  const size_t tbytes = sizeof(Tile) * tiles.size();
  const size_t toff = (dbytes + 255) / 256 * 256;
  if (toff + tbytes > ws_bytes) {
    snprintf(g_err, sizeof(g_err), "workspace too small: need %zu have %llu", toff + tbytes,
             (unsigned long long)ws_bytes);
    return -1000;
  }
  hipStream_t s = static_cast<hipStream_t>(stream);
  // stage tables through pinned memory so the H2D is a true async DMA
  char* stage = static_cast<char*>(pinned_stage);
  std::memcpy(stage, d, dbytes);
  std::memcpy(stage + toff, tiles.data(), tbytes);
  char* ws = static_cast<char*>(workspace);
  HS_CHECK(hipMemcpyAsync(ws, stage, toff + tbytes, hipMemcpyHostToDevice, s));
  const int64_t ntiles = static_cast<int64_t>(tiles.size());
  int grid = static_cast<int>(std::min<int64_t>(ntiles, 256 * 8));
  if (t_grid_cap > 0) grid = std::min(grid, t_grid_cap);
  // dynamic LDS only when a transpose descriptor is present (64x65 words)
  size_t lds = 0;
  for (int i = 0; i < n; ++i) {
    if (d[i].flags & 4) {
      const size_t w = elem_bytes_host(d[i].src_dtype) == 8 ? 8 : 4;
      lds = std::max(lds, 64 * 65 * w);
    }
  }
  hipLaunchKernelGGL(hs_copy_nd, dim3(grid), dim3(kBlock), lds, s,
                     reinterpret_cast<const CopyDesc*>(ws),
                     reinterpret_cast<const Tile*>(ws + toff), ntiles);
  HS_CHECK(hipGetLastError());
  if (sync) HS_CHECK(hipStreamSynchronize(s));
  return 0;
}

// fp8 quantize: src (bf16/f16/f32, contiguous, device) -> out fp8 bytes [n] +
// scales fp32 [ceil(n/block)], block = 64*vpt with vpt in {2,4,8,16}.
int hsg_fp8_quantize(int dev, const void* src, int src_dtype, int64_t n, void* out,
                     void* scales, int vpt, void* stream) {
  HS_CHECK(hipSetDevice(dev));
  if (n <= 0) return 0;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int64_t blk = 64LL * vpt;
  const int64_t nblocks = (n + blk - 1) / blk;
  const int64_t waves_per_wg = kBlock / 64;
  const int grid = static_cast<int>(std::min<int64_t>((nblocks + waves_per_wg - 1) / waves_per_wg, 256 * 8));
  const char* sp = static_cast<const char*>(src);
  uint8_t* op = static_cast<uint8_t*>(out);
  float* sc = static_cast<float*>(scales);
  // streaming kernel: 16-B aligned source, 8-B aligned payload, a block
  // within one wave (bf16/f16 blocks of 128..512, f32 of 128..256)
  const bool aligned = (reinterpret_cast<uintptr_t>(src) % 16) == 0 &&
                       (reinterpret_cast<uintptr_t>(out) % 8) == 0;
  if (aligned && (src_dtype == kBF16 || src_dtype == kF16 || src_dtype == kF32)) {
    const int epl = src_dtype == kF32 ? 4 : 8;
    const int64_t chunk = 64LL * epl * 4;
    const int vgrid = static_cast<int>(std::max<int64_t>(
        1, std::min<int64_t>((n + chunk - 1) / chunk / waves_per_wg + 1, 256 * 16)));
#define HS_FP8V(DT, B)                                                                     \
  hipLaunchKernelGGL((hs_fp8_quant_v<DT, B>), dim3(vgrid), dim3(kBlock), 0, s, sp, n, op, sc); \
  HS_CHECK(hipGetLastError());                                                             \
  return 0
    if (src_dtype == kBF16) {
      if (vpt == 2) { HS_FP8V(kBF16, 128); }
      if (vpt == 4) { HS_FP8V(kBF16, 256); }
      if (vpt == 8) { HS_FP8V(kBF16, 512); }
    } else if (src_dtype == kF16) {
      if (vpt == 2) { HS_FP8V(kF16, 128); }
      if (vpt == 4) { HS_FP8V(kF16, 256); }
      if (vpt == 8) { HS_FP8V(kF16, 512); }
    } else {
      if (vpt == 2) { HS_FP8V(kF32, 128); }
      if (vpt == 4) { HS_FP8V(kF32, 256); }
    }
#undef HS_FP8V
  }
  switch (vpt) {
    case 2: hipLaunchKernelGGL(hs_fp8_quant<2>, dim3(grid), dim3(kBlock), 0, s, sp, src_dtype, n, op, sc); break;
    case 4: hipLaunchKernelGGL(hs_fp8_quant<4>, dim3(grid), dim3(kBlock), 0, s, sp, src_dtype, n, op, sc); break;
    case 8: hipLaunchKernelGGL(hs_fp8_quant<8>, dim3(grid), dim3(kBlock), 0, s, sp, src_dtype, n, op, sc); break;
    case 16: hipLaunchKernelGGL(hs_fp8_quant<16>, dim3(grid), dim3(kBlock), 0, s, sp, src_dtype, n, op, sc); break;
    default: snprintf(g_err, sizeof(g_err), "unsupported vpt %d", vpt); return -1001;
  }
  HS_CHECK(hipGetLastError());
  return 0;
}

int hsg_fp8_dequantize(int dev, const void* q, const void* scales, int64_t n, void* dst,
                       int dst_dtype, int vpt, void* stream) {
  HS_CHECK(hipSetDevice(dev));
  if (n <= 0) return 0;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int64_t words = (n + 3) / 4;
  const int grid = static_cast<int>(std::min<int64_t>((words + kBlock - 1) / kBlock, 256 * 8));
  const uint8_t* qp = static_cast<const uint8_t*>(q);
  const float* sc = static_cast<const float*>(scales);
  char* dp = static_cast<char*>(dst);
  // streaming kernel: 8-B aligned codes, 16-B aligned destination
  if ((reinterpret_cast<uintptr_t>(q) % 8) == 0 && (reinterpret_cast<uintptr_t>(dst) % 16) == 0 &&
      (vpt == 2 || vpt == 4 || vpt == 8 || vpt == 16) &&
      (dst_dtype == kBF16 || dst_dtype == kF16 || dst_dtype == kF32 || dst_dtype == kF64)) {
    const int64_t epl = (dst_dtype == kF32) ? 4 : (dst_dtype == kF64 ? 2 : 8);
    const int64_t waves = (n + 64 * epl * 4 - 1) / (64 * epl * 4);
    const int vgrid = static_cast<int>(std::min<int64_t>((waves + 3) / 4, 256 * 16));
#define HS_FP8DV(DT)                                                                          \
  switch (vpt) {                                                                              \
    case 2: hipLaunchKernelGGL((hs_fp8_dequant_v<DT, 128>), dim3(vgrid), dim3(kBlock), 0, s, qp, sc, n, dp); break; \
    case 4: hipLaunchKernelGGL((hs_fp8_dequant_v<DT, 256>), dim3(vgrid), dim3(kBlock), 0, s, qp, sc, n, dp); break; \
    case 8: hipLaunchKernelGGL((hs_fp8_dequant_v<DT, 512>), dim3(vgrid), dim3(kBlock), 0, s, qp, sc, n, dp); break; \
    default: hipLaunchKernelGGL((hs_fp8_dequant_v<DT, 1024>), dim3(vgrid), dim3(kBlock), 0, s, qp, sc, n, dp); break; \
  }
    switch (dst_dtype) {
      case kBF16: HS_FP8DV(kBF16); break;
      case kF16: HS_FP8DV(kF16); break;
      case kF32: HS_FP8DV(kF32); break;
      default: HS_FP8DV(kF64); break;
    }
#undef HS_FP8DV
    HS_CHECK(hipGetLastError());
    return 0;
  }
  switch (vpt) {
    case 2: hipLaunchKernelGGL(hs_fp8_dequant<2>, dim3(grid), dim3(kBlock), 0, s, qp, sc, n, dp, dst_dtype); break;
    case 4: hipLaunchKernelGGL(hs_fp8_dequant<4>, dim3(grid), dim3(kBlock), 0, s, qp, sc, n, dp, dst_dtype); break;
    case 8: hipLaunchKernelGGL(hs_fp8_dequant<8>, dim3(grid), dim3(kBlock), 0, s, qp, sc, n, dp, dst_dtype); break;
    case 16: hipLaunchKernelGGL(hs_fp8_dequant<16>, dim3(grid), dim3(kBlock), 0, s, qp, sc, n, dp, dst_dtype); break;
    default: snprintf(g_err, sizeof(g_err), "unsupported vpt %d", vpt); return -1001;
  }
  HS_CHECK(hipGetLastError());
  return 0;
}

// MX fp8: src (bf16/f16/f32, contiguous) -> out [payload = round_up(n, 16)
// bytes; [n, payload) zero-filled] + scales [ceil(n / 32) E8M0 bytes].  Every
// output byte is written (the blob needs no zero-fill).
int hsg_mx8_quantize(int dev, const void* src, int src_dtype, int64_t n, void* out,
                     void* scales, void* stream) {
  HS_CHECK(hipSetDevice(dev));
  if (n <= 0) return 0;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int64_t payload = (n + 15) / 16 * 16;
  const int64_t chunk = (src_dtype == kF32) ? 64 * 4 * 4 : 64 * 8 * 4;
  const int64_t waves = (n + chunk - 1) / chunk;
  const int grid = static_cast<int>(std::min<int64_t>((waves + 3) / 4, 256 * 16));
  const char* sp = static_cast<const char*>(src);
  uint8_t* op = static_cast<uint8_t*>(out);
  uint8_t* sc = static_cast<uint8_t*>(scales);
  switch (src_dtype) {
    case kBF16: hipLaunchKernelGGL(hs_mx8_quant<kBF16>, dim3(grid), dim3(kBlock), 0, s, sp, n, payload, op, sc); break;
    case kF16: hipLaunchKernelGGL(hs_mx8_quant<kF16>, dim3(grid), dim3(kBlock), 0, s, sp, n, payload, op, sc); break;
    case kF32: hipLaunchKernelGGL(hs_mx8_quant<kF32>, dim3(grid), dim3(kBlock), 0, s, sp, n, payload, op, sc); break;
    default: snprintf(g_err, sizeof(g_err), "unsupported mx8 source dtype %d", src_dtype); return -1002;
  }
  HS_CHECK(hipGetLastError());
  return 0;
}

int hsg_mx8_dequantize(int dev, const void* q, const void* scales, int64_t n, void* dst,
                       int dst_dtype, void* stream) {
  HS_CHECK(hipSetDevice(dev));
  if (n <= 0) return 0;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int64_t epl = (dst_dtype == kF32) ? 4 : (dst_dtype == kF64 ? 2 : 8);
  const int64_t waves = (n + 64 * epl * 4 - 1) / (64 * epl * 4);
  const int grid = static_cast<int>(std::min<int64_t>((waves + 3) / 4, 256 * 16));
  const uint8_t* qp = static_cast<const uint8_t*>(q);
  const uint8_t* sc = static_cast<const uint8_t*>(scales);
  char* dp = static_cast<char*>(dst);
  switch (dst_dtype) {
    case kBF16: hipLaunchKernelGGL(hs_mx8_dequant<kBF16>, dim3(grid), dim3(kBlock), 0, s, qp, sc, n, dp); break;
    case kF16: hipLaunchKernelGGL(hs_mx8_dequant<kF16>, dim3(grid), dim3(kBlock), 0, s, qp, sc, n, dp); break;
    case kF32: hipLaunchKernelGGL(hs_mx8_dequant<kF32>, dim3(grid), dim3(kBlock), 0, s, qp, sc, n, dp); break;
    case kF64: hipLaunchKernelGGL(hs_mx8_dequant<kF64>, dim3(grid), dim3(kBlock), 0, s, qp, sc, n, dp); break;
    default: snprintf(g_err, sizeof(g_err), "unsupported mx8 dest dtype %d", dst_dtype); return -1002;
  }
  HS_CHECK(hipGetLastError());
  return 0;
}

// Hadamard-rotated fp8: payload `out` has n_pad = round_up(n, 32) bytes,
// `scales` ceil(n_pad / 128) floats.
int hsg_fp8_hadamard_quantize(int dev, const void* src, int src_dtype, int64_t n, void* out,
                              void* scales, void* stream) {
  HS_CHECK(hipSetDevice(dev));
  if (n <= 0) return 0;
  const int64_t n_pad = (n + 31) / 32 * 32;
  const int64_t ntiles = (n_pad + 1023) / 1024;
  const int grid = static_cast<int>(std::min<int64_t>((ntiles + 3) / 4, 256 * 8));
  constexpr int kHadU = 2;
  const int grid16 = static_cast<int>(std::min<int64_t>((ntiles + 4 * kHadU - 1) / (4 * kHadU), 256 * 8));
  hipStream_t st = static_cast<hipStream_t>(stream);
  const char* sp = static_cast<const char*>(src);
  uint8_t* op = static_cast<uint8_t*>(out);
  float* sc = static_cast<float*>(scales);
  switch (src_dtype) {
    case kBF16: hipLaunchKernelGGL((hs_fp8_hadamard_quant16<kBF16, kHadU>), dim3(grid16), dim3(kBlock), 0, st, sp, n, n_pad, op, sc); break;
    case kF16: hipLaunchKernelGGL((hs_fp8_hadamard_quant16<kF16, kHadU>), dim3(grid16), dim3(kBlock), 0, st, sp, n, n_pad, op, sc); break;
    case kF32: hipLaunchKernelGGL(hs_fp8_hadamard_quant<kF32>, dim3(grid), dim3(kBlock), 0, st, sp, n, n_pad, op, sc); break;
    default: snprintf(g_err, sizeof(g_err), "unsupported hadamard source dtype %d", src_dtype); return -1002;
  }
  HS_CHECK(hipGetLastError());
  return 0;
}

int hsg_fp8_hadamard_dequantize(int dev, const void* q, const void* scales, int64_t n, void* dst,
                                int dst_dtype, void* stream) {
  HS_CHECK(hipSetDevice(dev));
  if (n <= 0) return 0;
  const int64_t n_pad = (n + 31) / 32 * 32;
  const int64_t ntiles = (n_pad + 1023) / 1024;
  constexpr int U = 2;
  const int grid = static_cast<int>(std::min<int64_t>((ntiles + 4 * U - 1) / (4 * U), 256 * 8));
  hipStream_t st = static_cast<hipStream_t>(stream);
  const uint8_t* qp = static_cast<const uint8_t*>(q);
  const float* sp = static_cast<const float*>(scales);
  char* dp = static_cast<char*>(dst);
  switch (dst_dtype) {
    case kBF16: hipLaunchKernelGGL((hs_fp8_hadamard_dequant8<kBF16, U>), dim3(grid), dim3(kBlock), 0, st, qp, sp, n, n_pad, dp); break;
    case kF16: hipLaunchKernelGGL((hs_fp8_hadamard_dequant8<kF16, U>), dim3(grid), dim3(kBlock), 0, st, qp, sp, n, n_pad, dp); break;
    case kF32: hipLaunchKernelGGL((hs_fp8_hadamard_dequant8<kF32, U>), dim3(grid), dim3(kBlock), 0, st, qp, sp, n, n_pad, dp); break;
    case kF64: hipLaunchKernelGGL((hs_fp8_hadamard_dequant8<kF64, U>), dim3(grid), dim3(kBlock), 0, st, qp, sp, n, n_pad, dp); break;
    default: snprintf(g_err, sizeof(g_err), "unsupported hadamard dest dtype %d", dst_dtype); return -1002;
  }
  HS_CHECK(hipGetLastError());
  return 0;
}

// ---- managed (UVM) memory helpers (fbgemm uvm_to_cpu equivalent, K11) --------

int hsg_is_managed(const void* p) {
  hipPointerAttribute_t attr;
  if (hipPointerGetAttributes(&attr, p) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return attr.isManaged ? 1 : 0;
}

void* hsg_managed_alloc(int dev, uint64_t n) {
  if (hipSetDevice(dev) != hipSuccess) return nullptr;
  void* p = nullptr;
  hipError_t e = hipMallocManaged(&p, n, hipMemAttachGlobal);
  if (e != hipSuccess) { set_err("hipMallocManaged", e); return nullptr; }
  return p;
}

int hsg_managed_free(void* p) {
  HS_CHECK(hipFree(p));
  return 0;
}

// ---- stream gates (engine/uvm_capture.py) ------------------------------------
//
// An async take of host-resident UVM tables copies them on the CPU (threads on
// the pages' NUMA node: ~160-200 GB/s vs ~55 GB/s for the HBM freeze kernel
// reading them over PCIe, profiles/r6/uvmcap/) while the trainer's stream
// waits on a host word: hipStreamWaitValue32(word >= v) armed on the stream,
// released by the CPU once the copy is done.  One word per device, values
// increase per take, and a release only ever raises the word (an older
// take's late release cannot re-block a newer gate).

struct GateWord {
  uint32_t* word = nullptr;
  uint32_t next = 0;
};
std::mutex g_gate_mu;
std::map<int, GateWord> g_gates;

// 1 if hipStreamWaitValue32 works on `dev` (else the HBM freeze is used).
int hsg_gate_supported(int dev) {
  int v = 0;
  if (hipDeviceGetAttribute(&v, hipDeviceAttributeCanUseStreamWaitValue, dev) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return v ? 1 : 0;
}

// Arm a gate on `stream`: work queued on it from now on waits until the
// gate's value is released.  *value gets the value to release (> 0).
int hsg_gate_arm(int dev, void* stream, uint32_t* value) {
  HS_CHECK(hipSetDevice(dev));
  std::lock_guard<std::mutex> g(g_gate_mu);
  GateWord& gw = g_gates[dev];
  if (gw.word == nullptr) {
    void* p = nullptr;
    // signal memory: the command processor polls it, the CPU stores into it;
    // allocated once per device and never freed
    HS_CHECK(hipExtMallocWithFlags(&p, 8, hipMallocSignalMemory));
    gw.word = static_cast<uint32_t*>(p);
    __atomic_store_n(gw.word, 0u, __ATOMIC_SEQ_CST);
  }
  const uint32_t v = ++gw.next;
  HS_CHECK(hipStreamWaitValue32(static_cast<hipStream_t>(stream), gw.word, v,
                                hipStreamWaitValueGte, 0xffffffffu));
  *value = v;
  return 0;
}

// Release every gate of `dev` armed with a value <= `value`.
int hsg_gate_release(int dev, uint32_t value) {
  uint32_t* w;
  {
    std::lock_guard<std::mutex> g(g_gate_mu);
    auto it = g_gates.find(dev);
    if (it == g_gates.end() || it->second.word == nullptr) return -1;
    w = it->second.word;
  }
  uint32_t cur = __atomic_load_n(w, __ATOMIC_ACQUIRE);
  while (cur < value && !__atomic_compare_exchange_n(w, &cur, value, false, __ATOMIC_SEQ_CST,
                                                     __ATOMIC_ACQUIRE)) {
  }
  return 0;
}

// The gate word's current value (tests).
uint32_t hsg_gate_value(int dev) {
  std::lock_guard<std::mutex> g(g_gate_mu);
  auto it = g_gates.find(dev);
  if (it == g_gates.end() || it->second.word == nullptr) return 0;
  return __atomic_load_n(it->second.word, __ATOMIC_ACQUIRE);
}

// Advised placement of a managed range: *preferred / *last_prefetch get a
// device index, -1 (hipCpuDeviceId: host DRAM) or -2 (never set).
int hsg_managed_location(const void* p, uint64_t n, int* preferred, int* last_prefetch) {
  int v = -2;
  if (hipMemRangeGetAttribute(&v, sizeof(v), hipMemRangeAttributePreferredLocation,
                              const_cast<void*>(p), n) != hipSuccess) {
    (void)hipGetLastError();
    v = -2;
  }
  *preferred = v;
  v = -2;
  if (hipMemRangeGetAttribute(&v, sizeof(v), hipMemRangeAttributeLastPrefetchLocation,
                              const_cast<void*>(p), n) != hipSuccess) {
    (void)hipGetLastError();
    v = -2;
  }
  *last_prefetch = v;
  return 0;
}

// Place a managed range: preferred location `loc` (device index, or -1 for
// host DRAM) and an asynchronous prefetch there on `stream`.
int hsg_managed_place(int dev, const void* p, uint64_t n, int loc, void* stream) {
  HS_CHECK(hipSetDevice(dev));
  HS_CHECK(hipMemAdvise(p, n, hipMemAdviseSetPreferredLocation, loc));
  HS_CHECK(hipMemPrefetchAsync(p, n, loc, static_cast<hipStream_t>(stream)));
  return 0;
}

}  // extern "C"
