// hsz: HSZ1 lossless exponent-entropy codec on gfx950 (format: hipsnapshot/ops/codec.py).
//
// Encode (before D2H) = 4 launches on the caller's stream:
//   hsz_analyze<W>  one workgroup per 256 KiB frame: LDS histogram of a 2048-
//                   element sample (64 coalesced runs of 32) -> 15-entry
//                   dictionary (wave-wide argmax), then a full pass over the
//                   frame.  For 2-/4-byte elements that pass keeps one 16-bin
//                   index histogram per lane in LDS; wave 0 builds the
//                   length-limited Huffman code in registers (one node per
//                   lane, shuffle argmins) and every lane sizes its own
//                   stream, so the frame mode (raw / nibble / huffman) and the
//                   exact coded size are known before anything is written
//   hsz_layout      one workgroup: exclusive scan of frame sizes, blob header +
//                   frame table, total size for the host
//   hsz_encode<W>   modes 0/1, one workgroup per frame: 8 elements per lane per
//                   step, coalesced 16-B loads, nibble codes via an LDS code
//                   table, low-byte plane stores; the rare escapes go to an LDS
//                   list and are written in element order by rank
//   hsz_encode2<W>  mode 2: lane t packs the codes of element groups t, t+256,
//                   ... into its own bit stream in LDS (stream offsets from a
//                   block scan of the analyze pass's lane sizes) while the
//                   low-byte plane streams out with 8-B stores; the finished
//                   streams leave LDS with coalesced 4-B stores
//   hsz_encode2x<2> mode 2 for bf16/fp16: the same stream layout, packed by
//                   1024 threads, 4 per lane stream (each piece's bit offset
//                   comes from per-piece byte counters in the analyze pass)
// Decode (after H2D) = 2 launches, one workgroup per frame each:
//   hsz_decode<W>   modes 0/1 (escape positions are collected from the nibble
//                   plane first, then every element is rebuilt)
//   hsz_decode2g<W, P>  mode 2 (default): the frame's streams are staged in
//                   LDS, lane t decodes its stream through a 2048-entry LDS
//                   lookup table and stores its groups as 16-B vectors
//                   (adjacent lanes -> adjacent groups, so the stores
//                   coalesce); escapes are patched in element order after a
//                   barrier (round 4 rewrite of the round-3 LDS decoder,
//                   which it replaced: profiles/r4/decode_pmc/)
//
// A frame is one workgroup (4 waves): a 512 MiB blob has 2048 frames, 8x the
// CU count, so the grid fills the chip; all traffic is streaming HBM
// (read 2 B + write ~1.34 B per bf16 element encoded).

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <cstdlib>
#include <cstdio>

extern "C" int hsg_thread_grid_cap();  // hsgpu.hip

namespace {

constexpr int kThreads = 256;
constexpr int kLanes = 256;  // mode-2 lane streams per frame == threads per workgroup
constexpr int kSample = 2048;
constexpr int kRun = 32;  // dictionary sample = kSample / kRun runs (codec.sample_indices)
constexpr int kMaxEsc = 1024;
constexpr int kHeader = 64;
constexpr int kFrameHeader = 32;
constexpr int kEsc = 15;
constexpr int kMaxLen = 11;
constexpr int kLut = 1 << kMaxLen;
constexpr uint32_t kMaxCoded = 65535;
constexpr int kLaneTable = 2 * kLanes;
constexpr int kSub = 4;                    // hsz_encode2x: pieces (threads) per lane stream
constexpr int kThreadsX = kLanes * kSub;   // 1024

struct FrameMeta {
  uint32_t mode;
  uint32_t n_esc;
  uint32_t nsel;   // dictionary entries actually selected (rest are 0 padding)
  uint32_t coded;  // mode 2: total stream bytes
  uint8_t dict[16];
  uint8_t lens[16];  // mode 2 code lengths
  uint64_t size;     // padded frame bytes
  uint64_t offset;   // absolute offset in the blob
};
// meta buffer = FrameMeta[n_frames], then uint16 lane_bytes[n_frames][256], then
// uint32 piece_bits[n_frames][kSub - 1][256]: bits of lane t's stream up to the
// end of its piece s (hsz_encode2x splits every stream into kSub pieces)

__device__ __forceinline__ uint64_t align16(uint64_t n) { return (n + 15) & ~uint64_t(15); }

// bf16/fp16 high bytes come in +/- pairs 128 apart (sign bit), which land on
// the same LDS bank; the lookup tables shift the upper half by one dword so
// that v and v ^ 0x80 are served in the same cycle (PMC: SQ_LDS_BANK_CONFLICT).
__device__ __forceinline__ uint32_t cslot(uint32_t v) { return v + ((v >> 7) << 2); }  // u8 tables
__device__ __forceinline__ uint32_t eslot(uint32_t v) { return v + (v >> 7); }         // u32 tables

__device__ __forceinline__ int block_sum(int v, int* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int wid = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) red[wid] = v;
  __syncthreads();
  int t = red[0] + red[1] + red[2] + red[3];
  __syncthreads();
  return t;
}

// Exclusive prefix sum over the 256 threads; *total receives the sum.
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* wsum, uint32_t* total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) wsum[wid] = x;
  __syncthreads();
  uint32_t base = 0;
  for (int i = 0; i < wid; ++i) base += wsum[i];
  if (threadIdx.x == 0) *total = wsum[0] + wsum[1] + wsum[2] + wsum[3];
  __syncthreads();
  return base + x - v;
}

// The 15 most frequent values of hist (count desc, value asc); zero counts are
// never chosen.  Runs on wave 0; results in dict / code_of (LDS).
__device__ void build_dict(const uint32_t* hist, uint8_t* dict, uint8_t* code_of, int* nsel) {
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    uint64_t key[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int v = lane * 4 + j;
      key[j] = (uint64_t(hist[v]) << 8) | uint64_t(255 - v);
    }
    int k = 0;
    for (; k < 15; ++k) {
      uint64_t best = key[0];
#pragma unroll
      for (int j = 1; j < 4; ++j) best = key[j] > best ? key[j] : best;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const uint64_t other = __shfl_xor(best, o, 64);
        best = other > best ? other : best;
      }
      if ((best >> 8) == 0) break;
      const int v = 255 - int(best & 255);
      if (lane == 0) dict[k] = uint8_t(v);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (v == lane * 4 + j) key[j] = 0;
    }
    if (lane == 0) *nsel = k;
    for (int j = k + lane; j < 16; j += 64) dict[j] = 0;
  }
  __syncthreads();
  for (int v = threadIdx.x; v < 256; v += kThreads) code_of[cslot(v)] = kEsc;
  __syncthreads();
  if (threadIdx.x < *nsel) code_of[cslot(dict[threadIdx.x])] = uint8_t(threadIdx.x);
  __syncthreads();
}

__device__ __forceinline__ uint64_t wave_min_u64(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint64_t x = __shfl_xor(v, o, 64);
    v = x < v ? x : v;
  }
  return v;
}

__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint64_t x = __shfl_xor(v, o, 64);
    v = x > v ? x : v;
  }
  return v;
}

__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Huffman code length of index `lane` (mirror of codec.huffman_lengths), built
// by one whole wave: lane i holds node i (leaves 0..15 = index values, merged
// nodes 16.. in creation order), each merge is two wave-wide argmins over
// (weight, node) -- the same tie-break as the reference -- and depths are
// found by chasing parent links with lane shuffles.  `cnt` is the index's
// count in lanes 0..15 (ignored elsewhere); returns its length (0 = unused).
// Everything stays in registers: no LDS round trips on a serial path.
__device__ uint32_t wave_huffman_len(uint32_t cnt) {
  const int lane = threadIdx.x & 63;
  const bool used = lane < 16 && cnt != 0;
  const int k = __popcll(__ballot(used));
  if (k <= 1) return used ? 1u : 0u;
  uint64_t w = used ? cnt : 0;
  bool alive = used;
  int par = -1;
  for (int step = 0; step < k - 1; ++step) {
    const int m = 16 + step;
    const uint64_t a = wave_min_u64(alive ? (w << 8) | uint64_t(lane) : ~0ull);
    if (lane == int(a & 255)) { alive = false; par = m; }
    const uint64_t b = wave_min_u64(alive ? (w << 8) | uint64_t(lane) : ~0ull);
    if (lane == int(b & 255)) { alive = false; par = m; }
    if (lane == m) { w = (a >> 8) + (b >> 8); alive = true; }
  }
  int j = lane;
  uint32_t d = 0;
  for (int it = 0; it < k - 1; ++it) {  // depth <= k - 1
    const int p = __shfl(par, j, 64);
    if (p >= 0) { j = p; ++d; }
  }
  uint32_t len = used ? d : 0;
  if (wave_max_u64(len) <= uint64_t(kMaxLen)) return len;
  if (len > uint32_t(kMaxLen)) len = kMaxLen;
  for (;;) {  // Kraft fix: lengthen the longest code below the limit (rarer, then larger index)
    const uint32_t kraft = wave_sum_u32(used ? 1u << (kMaxLen - len) : 0u);
    if (kraft <= (1u << kMaxLen)) break;
    const uint64_t key = (used && len < uint32_t(kMaxLen))
                             ? (uint64_t(len) << 56) | (uint64_t(0xffffffffu - cnt) << 8) | uint64_t(lane)
                             : 0;
    if (lane == int(wave_max_u64(key) & 255)) ++len;
  }
  return len;
}

// Bit-reversed canonical codeword of index `lane` (mirror of
// codec.canonical_codes), one wave: the code of a symbol is the Kraft sum of
// the symbols before it in (length, index) order, scaled to its length.
// `len` = the index's code length in lanes 0..15 (<= kMaxLen).
__device__ uint32_t wave_canonical_code(uint32_t len) {
  const int lane = threadIdx.x & 63;
  uint32_t kr = 0;
#pragma unroll
  for (int s = 0; s < 16; ++s) {
    const uint32_t ls = __shfl(len, s, 64);
    if (ls && (ls < len || (ls == len && s < lane))) kr += 1u << (kMaxLen - ls);
  }
  if (lane >= 16 || len == 0) return 0;
  return __builtin_bitreverse32(kr >> (kMaxLen - len)) >> (32 - len);
}

// Element group g (elements 8g..8g+7, W = 2 or 4 bytes each) as 2W
// little-endian words: W / 2 coalesced 16-B loads per lane.
template <int W>
__device__ __forceinline__ void load_group(const uint8_t* s, uint64_t g, bool aligned,
                                           uint32_t wd[2 * W]) {
  if (aligned) {
#pragma unroll
    for (int k = 0; k < W / 2; ++k) {
      const uint4 v = reinterpret_cast<const uint4*>(s)[g * (W / 2) + k];
      wd[4 * k] = v.x; wd[4 * k + 1] = v.y; wd[4 * k + 2] = v.z; wd[4 * k + 3] = v.w;
    }
  } else {
    const uint8_t* p = s + 8 * W * g;
#pragma unroll
    for (int q = 0; q < 2 * W; ++q)
      wd[q] = uint32_t(p[4 * q]) | (uint32_t(p[4 * q + 1]) << 8) | (uint32_t(p[4 * q + 2]) << 16) |
              (uint32_t(p[4 * q + 3]) << 24);
  }
}

// Element e of a loaded group (e must be a compile-time constant after unrolling).
template <int W>
__device__ __forceinline__ uint32_t group_elem(const uint32_t* wd, int e) {
  if constexpr (W == 2) return (wd[e >> 1] >> (16 * (e & 1))) & 0xffffu;
  else return wd[e];
}

// The low (W-1) bytes of the 8 elements of a group form 8(W-1) contiguous
// bytes of the low-byte plane, held as W-1 u64 words.  put_lo takes the
// whole element and keeps its low bytes.
template <int W>
__device__ __forceinline__ void put_lo(uint64_t* lw, int e, uint32_t v) {
  constexpr int L = 8 * (W - 1);
  const int bp = L * e;
  const uint64_t x = v & ((1u << L) - 1);  // drop the high byte
  lw[bp >> 6] |= x << (bp & 63);
  if ((bp & 63) + L > 64) lw[(bp >> 6) + 1] |= x >> (64 - (bp & 63));
}

// The W-1 low-byte words of group g from the low-byte plane.
template <int W>
__device__ __forceinline__ void load_lo(const uint8_t* lo, uint64_t g, bool aligned,
                                        uint64_t lw[W - 1]) {
#pragma unroll
  for (int k = 0; k < W - 1; ++k) {
    if (aligned) {
      lw[k] = reinterpret_cast<const uint64_t*>(lo)[g * (W - 1) + k];
    } else {
      lw[k] = 0;
#pragma unroll
      for (int b = 0; b < 8; ++b) lw[k] |= uint64_t(lo[8 * ((W - 1) * g + k) + b]) << (8 * b);
    }
  }
}

template <int W>
__device__ __forceinline__ uint32_t get_lo(const uint64_t* lw, int e) {
  constexpr int L = 8 * (W - 1);
  const int bp = L * e;
  uint64_t x = lw[bp >> 6] >> (bp & 63);
  if ((bp & 63) + L > 64) x |= lw[(bp >> 6) + 1] << (64 - (bp & 63));
  return uint32_t(x) & ((1u << L) - 1);
}

// A lane's count of one index: the column word, or with per-piece byte
// counters (hsz_analyze's "packed" mode) the sum of its 4 bytes.
__device__ __forceinline__ uint32_t col_count(uint32_t w, bool packed) {
  return packed ? (w & 255) + ((w >> 8) & 255) + ((w >> 16) & 255) + (w >> 24) : w;
}

template <int W>
__device__ inline void
hsz_analyze_frame(const uint64_t f, const uint8_t* __restrict__ src, uint64_t logical, uint32_t frame_bytes,
            FrameMeta* __restrict__ meta, uint16_t* __restrict__ lane_bytes_all,
            uint32_t* __restrict__ piece_bits_all) {
  __shared__ uint32_t hist[256];
  __shared__ uint8_t dict[16];
  __shared__ uint8_t code_of[260];  // indexed through cslot()
  __shared__ int nsel;
  __shared__ int red[4];
  const uint64_t base = f * frame_bytes;
  const uint64_t len = min(uint64_t(frame_bytes), logical - base);
  const uint64_t n = len / W;
  const uint8_t* s = src + base;
  for (int v = threadIdx.x; v < 256; v += kThreads) hist[v] = 0;
  __syncthreads();
  // half a wave reads one run of kRun consecutive elements (coalesced)
  const uint64_t step = n / (kSample / kRun);
  for (int i = threadIdx.x; i < kSample; i += kThreads) {
    const uint64_t idx = n <= uint64_t(kSample) ? uint64_t(i) : uint64_t(i / kRun) * step + i % kRun;
    if (idx < n) atomicAdd(&hist[s[idx * W + W - 1]], 1u);
  }
  __syncthreads();
  build_dict(hist, dict, code_of, &nsel);
  const uint64_t tail = len - n * W;
  const uint64_t coded1 = kFrameHeader + (n + 1) / 2 + uint64_t(W - 1) * n + tail;  // + escapes
  const uint64_t raw = kFrameHeader + len;
  if constexpr (W == 2 || W == 4) {
    if (n > 0 && n % 8 == 0) {
      // mode-2 sizing: one 16-bin histogram per lane (lane t owns groups t, t+256, ...)
      __shared__ uint32_t lcnt[16 * kLanes];
      __shared__ uint32_t fcnt[16];
      __shared__ uint8_t hlen[16];
      for (int i = threadIdx.x; i < 16 * kLanes; i += kThreads) lcnt[i] = 0;
      __syncthreads();
      const uint64_t groups = n / 8;
      const bool aligned = (reinterpret_cast<uintptr_t>(s) & 15) == 0;
      // the next group's load is in flight while this one is counted, and
      // each count is one ds_add (no read-modify-write round trip per element:
      // the thread owns its column, so nothing contends)
      // encode2x splits lane t's stream into kSub pieces of pq consecutive
      // groups and needs each piece's bit offset: while a piece has < 256
      // elements ("packed"), the count of piece p lives in byte p of the
      // column word (one ds_add of 1 << 8p), so the same pass yields them
      const uint32_t pq = uint32_t((groups + kLanes - 1) / kLanes + kSub - 1) / kSub;
      const bool packed = pq * 8 < 256;
      uint32_t left = pq, inc = 1;
      uint32_t nx[2 * W];
      if (threadIdx.x < groups) load_group<W>(s, threadIdx.x, aligned, nx);
      for (uint64_t g = threadIdx.x; g < groups; g += kThreads) {
        uint32_t wd[2 * W];
#pragma unroll
        for (int q = 0; q < 2 * W; ++q) wd[q] = nx[q];
        if (g + kThreads < groups) load_group<W>(s, g + kThreads, aligned, nx);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const uint32_t c = code_of[cslot(group_elem<W>(wd, e) >> (8 * (W - 1)))];
          atomicAdd(&lcnt[c * kLanes + threadIdx.x], inc);
        }
        if (--left == 0) {
          left = pq;
          if (packed) inc <<= 8;
        }
      }
      __syncthreads();
      {  // frame histogram: wave q sums the lane columns of indices 4q..4q+3
        const int lane = threadIdx.x & 63, q = threadIdx.x >> 6;
#pragma unroll
        for (int c = 4 * q; c < 4 * q + 4; ++c) {
          uint32_t v = 0;
#pragma unroll
          for (int r = 0; r < kLanes; r += 64) v += col_count(lcnt[c * kLanes + r + lane], packed);
          v = wave_sum_u32(v);
          if (lane == 0) fcnt[c] = v;
        }
      }
      __syncthreads();
      if (threadIdx.x < 64) {
        const uint32_t len = wave_huffman_len(threadIdx.x < 16 ? fcnt[threadIdx.x] : 0u);
        if (threadIdx.x < 16) hlen[threadIdx.x] = uint8_t(len);
      }
      __syncthreads();
      uint32_t bits = 0;
      uint32_t pbits[kSub - 1];  // bits up to the end of piece sp
#pragma unroll
      for (int sp = 0; sp < kSub - 1; ++sp) pbits[sp] = 0;
#pragma unroll 1
      for (int c = 0; c < 16; ++c) {
        const uint32_t w = lcnt[c * kLanes + threadIdx.x];
        const uint32_t hl = hlen[c];
        bits += col_count(w, packed) * hl;
        uint32_t cum = 0;
#pragma unroll
        for (int sp = 0; sp < kSub - 1; ++sp) {
          cum += (w >> (8 * sp)) & 255;
          pbits[sp] += cum * hl;
        }
      }
      const uint32_t lb = (bits + 7) / 8;
      lane_bytes_all[f * kLanes + threadIdx.x] = uint16_t(lb < 65535u ? lb : 65535u);
      if (packed) {
#pragma unroll
        for (int sp = 0; sp < kSub - 1; ++sp)
          piece_bits_all[(f * (kSub - 1) + sp) * kLanes + threadIdx.x] = pbits[sp];
      }
      const int c_bytes = block_sum(int(lb), red);
      if (threadIdx.x == 0) {
        const uint32_t esc = fcnt[kEsc];
        const uint64_t size1 = coded1 + esc;
        const uint64_t size2 = kFrameHeader + uint64_t(W - 1) * n + kLaneTable + uint64_t(c_bytes) + esc + tail;
        FrameMeta m;
        m.mode = 0;
        if (esc <= uint32_t(kMaxEsc)) {
          if (uint32_t(c_bytes) <= kMaxCoded && size2 < size1 && size2 < raw) m.mode = 2;
          else if (size1 < raw) m.mode = 1;
        }
        m.n_esc = m.mode ? esc : 0;
        m.nsel = m.mode ? nsel : 0;
        m.coded = m.mode == 2 ? uint32_t(c_bytes) : 0;
        for (int j = 0; j < 16; ++j) {
          m.dict[j] = m.mode ? dict[j] : 0;
          m.lens[j] = m.mode == 2 ? hlen[j] : 0;
        }
        m.size = align16(m.mode == 2 ? size2 : (m.mode == 1 ? size1 : raw));
        m.offset = 0;
        meta[f] = m;
      }
      return;
    }
  }
  int esc = 0;
  if (((reinterpret_cast<uintptr_t>(s)) & 15) == 0) {
    const uint64_t nv = (n * W) / 16;  // whole 16-B vectors of elements
    const uint4* sv = reinterpret_cast<const uint4*>(s);
    for (uint64_t i = threadIdx.x; i < nv; i += kThreads) {
      const uint4 v = sv[i];
      const uint32_t wd[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int p = W - 1; p < 16; p += W) esc += code_of[cslot((wd[p >> 2] >> (8 * (p & 3))) & 255)] == kEsc;
    }
    for (uint64_t e = nv * 16 / W + threadIdx.x; e < n; e += kThreads)
      esc += code_of[cslot(s[e * W + W - 1])] == kEsc;
  } else {
    for (uint64_t e = threadIdx.x; e < n; e += kThreads) esc += code_of[cslot(s[e * W + W - 1])] == kEsc;
  }
  const int total = block_sum(esc, red);
  if (threadIdx.x == 0) {
    const uint64_t coded = coded1 + total;
    FrameMeta m;
    m.mode = (total <= kMaxEsc && coded < raw && n > 0) ? 1 : 0;
    m.n_esc = m.mode ? total : 0;
    m.nsel = m.mode ? nsel : 0;
    m.coded = 0;
    for (int j = 0; j < 16; ++j) {
      m.dict[j] = m.mode ? dict[j] : 0;
      m.lens[j] = 0;
    }
    m.size = align16(m.mode ? coded : raw);
    m.offset = 0;
    meta[f] = m;
  }
}

// One workgroup per frame; with a grid smaller than the frame count (a
// background drain caps it, hsg_set_thread_grid_cap) each workgroup walks
// several frames, so the encoder occupies only that many CUs.
template <int W>
__global__ void __launch_bounds__(kThreads, 8)  // 8 waves / SIMD: what LDS allows (8 workgroups / CU)
hsz_analyze(const uint8_t* __restrict__ src, uint64_t logical, uint32_t frame_bytes,
            FrameMeta* __restrict__ meta, uint16_t* __restrict__ lane_bytes_all,
            uint32_t* __restrict__ piece_bits_all, uint32_t nf) {
  for (uint64_t f = blockIdx.x; f < nf; f += gridDim.x) {
    hsz_analyze_frame<W>(f, src, logical, frame_bytes, meta, lane_bytes_all, piece_bits_all);
    __syncthreads();  // the next frame reuses this workgroup's LDS
  }
}

__global__ void __launch_bounds__(1024)
hsz_layout(FrameMeta* __restrict__ meta, uint32_t n_frames, uint8_t* __restrict__ out,
           uint64_t logical, uint32_t w, uint32_t frame_bytes, uint64_t* __restrict__ total) {
  __shared__ uint64_t part[1024];
  __shared__ uint64_t carry;
  const uint64_t start = align16(kHeader + 8ull * (n_frames + 1));
  if (threadIdx.x == 0) carry = start;
  __syncthreads();
  uint64_t* table = reinterpret_cast<uint64_t*>(out + kHeader);
  for (uint32_t c = 0; c < n_frames; c += 1024) {
    const uint32_t i = c + threadIdx.x;
    const uint64_t v = i < n_frames ? meta[i].size : 0;
    part[threadIdx.x] = v;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {  // Hillis-Steele inclusive scan
      const uint64_t add = threadIdx.x >= uint32_t(o) ? part[threadIdx.x - o] : 0;
      __syncthreads();
      part[threadIdx.x] += add;
      __syncthreads();
    }
    if (i < n_frames) {
      const uint64_t off = carry + part[threadIdx.x] - v;
      meta[i].offset = off;
      table[i] = off;
    }
    __syncthreads();
    if (threadIdx.x == 1023) carry += part[1023];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    table[n_frames] = carry;
    *total = carry;
    uint32_t* h32 = reinterpret_cast<uint32_t*>(out);
    h32[0] = 0x315a5348u;  // "HSZ1"
    h32[1] = 2;            // format version
    *reinterpret_cast<uint64_t*>(out + 8) = logical;
    h32[4] = w;
    h32[5] = frame_bytes;
    h32[6] = n_frames;
    for (int j = 7; j < 16; ++j) h32[j] = 0;
    for (uint64_t p = kHeader + 8ull * (n_frames + 1); p < start; ++p) out[p] = 0;
  }
}

// Writes frame f's escape values in element order: entries (idx, value) were
// appended in arbitrary order; each one's rank = #entries with a smaller idx.
template <int NT = kThreads>
__device__ void write_escapes(const uint32_t* eidx, const uint8_t* evals, int n_esc,
                              uint8_t* dst) {
  for (int i = threadIdx.x; i < n_esc; i += NT) {
    const uint32_t me = eidx[i];
    int rank = 0;
    for (int j = 0; j < n_esc; ++j) rank += eidx[j] < me;
    dst[rank] = evals[i];
  }
}

// Frame header bytes 0..31 (mode, n_esc, dict, mode-2 code lengths).
__device__ __forceinline__ void write_frame_header(const FrameMeta& m, uint8_t* fr) {
  if (threadIdx.x < kFrameHeader) {
    uint8_t b = 0;
    const int t = threadIdx.x;
    if (t == 0) b = uint8_t(m.mode);
    else if (t >= 4 && t < 8) b = uint8_t(m.n_esc >> (8 * (t - 4)));
    else if (t >= 8 && t < 24) b = m.dict[t - 8];
    else if (t >= 24) b = uint8_t(m.lens[2 * (t - 24)] | (m.lens[2 * (t - 24) + 1] << 4));
    fr[t] = b;
  }
}

template <int W>
__device__ inline void
hsz_encode_frame(const uint64_t f, const uint8_t* __restrict__ src, uint64_t logical, uint32_t frame_bytes,
           const FrameMeta* __restrict__ meta, uint8_t* __restrict__ out) {
  __shared__ uint8_t code_of[260];  // indexed through cslot()
  __shared__ uint32_t eidx[kMaxEsc];
  __shared__ uint8_t evals[kMaxEsc];
  __shared__ int ecount;
  const FrameMeta& m = meta[f];  // arrays indexed at run time: read from memory
  if (m.mode == 2) return;  // hsz_encode2
  const uint64_t base = f * frame_bytes;
  const uint64_t len = min(uint64_t(frame_bytes), logical - base);
  const uint64_t n = len / W;
  const uint8_t* s = src + base;
  uint8_t* fr = out + m.offset;
  write_frame_header(m, fr);
  uint8_t* body = fr + kFrameHeader;
  const uint64_t padded_end = m.size - kFrameHeader;  // body bytes incl. padding
  if (m.mode == 0) {
    if ((((reinterpret_cast<uintptr_t>(s)) | reinterpret_cast<uintptr_t>(body)) & 15) == 0) {
      const uint64_t nv = len / 16;
      const uint4* sv = reinterpret_cast<const uint4*>(s);
      uint4* dv = reinterpret_cast<uint4*>(body);
      for (uint64_t i = threadIdx.x; i < nv; i += kThreads) dv[i] = sv[i];
      for (uint64_t j = nv * 16 + threadIdx.x; j < padded_end; j += kThreads)
        body[j] = j < len ? s[j] : 0;
    } else {
      for (uint64_t j = threadIdx.x; j < padded_end; j += kThreads) body[j] = j < len ? s[j] : 0;
    }
    return;
  }
  for (int v = threadIdx.x; v < 256; v += kThreads) code_of[cslot(v)] = kEsc;
  if (threadIdx.x == 0) ecount = 0;
  __syncthreads();
  if (threadIdx.x < m.nsel) code_of[cslot(m.dict[threadIdx.x])] = uint8_t(threadIdx.x);
  __syncthreads();
  uint8_t* nib = body;
  const uint64_t nb = (n + 1) / 2;
  uint8_t* lo = body + nb;
  uint8_t* escp = lo + uint64_t(W - 1) * n;
  const bool fast = (reinterpret_cast<uintptr_t>(s) & 15) == 0 &&
                    ((reinterpret_cast<uintptr_t>(nib) | reinterpret_cast<uintptr_t>(lo)) & 7) == 0 &&
                    (n % 8) == 0;
  uint64_t done = 0;
  if (fast && W == 2) {
    // 8 elements (16 B) per lane per step -> 4 B of nibbles + 8 B of low bytes
    const uint64_t groups = n / 8;
    const uint4* sv = reinterpret_cast<const uint4*>(s);
    uint32_t* nv = reinterpret_cast<uint32_t*>(nib);
    uint64_t* lv = reinterpret_cast<uint64_t*>(lo);
    for (uint64_t g = threadIdx.x; g < groups; g += kThreads) {
      const uint4 v = sv[g];
      const uint32_t wd[4] = {v.x, v.y, v.z, v.w};
      uint32_t codes = 0;
      uint64_t lob = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int e = q * 2 + h;
          const uint32_t hi = (wd[q] >> (16 * h + 8)) & 255;
          const uint32_t c = code_of[cslot(hi)];
          codes |= c << (4 * e);
          lob |= uint64_t((wd[q] >> (16 * h)) & 255) << (8 * e);
          if (c == kEsc) {
            const int k = atomicAdd(&ecount, 1);
            if (k < kMaxEsc) { eidx[k] = uint32_t(g * 8 + e); evals[k] = uint8_t(hi); }
          }
        }
      }
      nv[g] = codes;
      lv[g] = lob;
    }
    done = n;
  } else if (fast && W == 4) {
    const uint64_t groups = n / 8;  // 32 B in, 4 B nibbles + 24 B low bytes
    const uint4* sv = reinterpret_cast<const uint4*>(s);
    uint32_t* nv = reinterpret_cast<uint32_t*>(nib);
    for (uint64_t g = threadIdx.x; g < groups; g += kThreads) {
      const uint4 a = sv[2 * g], b = sv[2 * g + 1];
      const uint32_t wd[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
      uint32_t codes = 0;
      uint8_t lob[24];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const uint32_t hi = wd[e] >> 24;
        const uint32_t c = code_of[cslot(hi)];
        codes |= c << (4 * e);
        lob[3 * e] = wd[e] & 255;
        lob[3 * e + 1] = (wd[e] >> 8) & 255;
        lob[3 * e + 2] = (wd[e] >> 16) & 255;
        if (c == kEsc) {
          const int k = atomicAdd(&ecount, 1);
          if (k < kMaxEsc) { eidx[k] = uint32_t(g * 8 + e); evals[k] = uint8_t(hi); }
        }
      }
      nv[g] = codes;
      uint64_t* lv = reinterpret_cast<uint64_t*>(lo + 24 * g);
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        uint64_t x = 0;
#pragma unroll
        for (int b8 = 0; b8 < 8; ++b8) x |= uint64_t(lob[8 * q + b8]) << (8 * b8);
        lv[q] = x;
      }
    }
    done = n;
  }
  if (done < n) {
    // generic path: one element pair per lane step (partial / unaligned frames)
    for (uint64_t p = threadIdx.x; p < nb; p += kThreads) {
      uint8_t byte = 0;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const uint64_t e = 2 * p + h;
        if (e >= n) break;
        const uint8_t* el = s + e * W;
        const uint32_t hi = el[W - 1];
        const uint32_t c = code_of[cslot(hi)];
        byte |= uint8_t(c << (4 * h));
        for (int b = 0; b < W - 1; ++b) lo[e * (W - 1) + b] = el[b];
        if (c == kEsc) {
          const int k = atomicAdd(&ecount, 1);
          if (k < kMaxEsc) { eidx[k] = uint32_t(e); evals[k] = uint8_t(hi); }
        }
      }
      nib[p] = byte;
    }
  }
  __syncthreads();
  write_escapes(eidx, evals, min(ecount, kMaxEsc), escp);
  // tail bytes + zero padding
  uint8_t* tail = escp + m.n_esc;
  const uint64_t tail_len = len - n * W;
  const uint64_t used = uint64_t(tail - body);
  for (uint64_t j = threadIdx.x; used + j < padded_end; j += kThreads)
    tail[j] = j < tail_len ? s[n * W + j] : 0;
}

// One workgroup per frame; with a grid smaller than the frame count (a
// background drain caps it, hsg_set_thread_grid_cap) each workgroup walks
// several frames, so the encoder occupies only that many CUs.
template <int W>
__global__ void __launch_bounds__(kThreads)
hsz_encode(const uint8_t* __restrict__ src, uint64_t logical, uint32_t frame_bytes,
           const FrameMeta* __restrict__ meta, uint8_t* __restrict__ out, uint32_t nf) {
  for (uint64_t f = blockIdx.x; f < nf; f += gridDim.x) {
    hsz_encode_frame<W>(f, src, logical, frame_bytes, meta, out);
    __syncthreads();  // the next frame reuses this workgroup's LDS
  }
}

// Mode-2 encoder (W = 2 or 4).  LDS: 64 KiB stream buffer + escapes.
template <int W>
__device__ inline void
hsz_encode2_frame(const uint64_t f, const uint8_t* __restrict__ src, uint64_t logical, uint32_t frame_bytes,
            const FrameMeta* __restrict__ meta, const uint16_t* __restrict__ lane_bytes_all,
            uint8_t* __restrict__ out) {
  // lane streams as 32-bit words; a word shared by two lanes' streams is
  // assembled with LDS atomic ORs (the buffer starts zeroed)
  __shared__ uint32_t coded32[(kMaxCoded + 1 + 8 + 3) / 4];
  __shared__ uint8_t code_of[260];  // indexed through cslot()
  __shared__ uint32_t enc_tab[257];  // eslot(high byte) -> codeword | len << 16 | escape << 31
  __shared__ uint16_t hcode[16];
  __shared__ uint8_t hlen[16];
  __shared__ uint32_t eidx[kMaxEsc];
  __shared__ uint8_t evals[kMaxEsc];
  __shared__ uint32_t wsum[4];
  __shared__ uint32_t ctotal;
  __shared__ int ecount;
  const FrameMeta& m = meta[f];  // arrays indexed at run time: read from memory
  if (m.mode != 2) return;
  const uint64_t base = f * frame_bytes;
  const uint64_t len = min(uint64_t(frame_bytes), logical - base);
  const uint64_t n = len / W;
  const uint8_t* s = src + base;
  uint8_t* fr = out + m.offset;
  write_frame_header(m, fr);
  for (int v = threadIdx.x; v < 256; v += kThreads) code_of[cslot(v)] = kEsc;
  const uint32_t c_words = (m.coded + 3) / 4;
  for (uint32_t i = threadIdx.x; i < c_words; i += kThreads) coded32[i] = 0;
  if (threadIdx.x < 64) {
    const uint32_t l = threadIdx.x < 16 ? m.lens[threadIdx.x] : 0u;
    const uint32_t code = wave_canonical_code(l);
    if (threadIdx.x < 16) {
      hlen[threadIdx.x] = uint8_t(l);
      hcode[threadIdx.x] = uint16_t(code);
    }
    if (threadIdx.x == 0) ecount = 0;
  }
  __syncthreads();
  if (threadIdx.x < m.nsel) code_of[cslot(m.dict[threadIdx.x])] = uint8_t(threadIdx.x);
  __syncthreads();
  {  // one LDS lookup per element instead of three
    const uint32_t c = code_of[cslot(threadIdx.x)];
    enc_tab[eslot(threadIdx.x)] = uint32_t(hcode[c]) | (uint32_t(hlen[c]) << 16) |
                           (c == kEsc ? 0x80000000u : 0u);
  }
  const uint32_t lb = lane_bytes_all[f * kLanes + threadIdx.x];
  const uint32_t loff = block_excl_scan(lb, wsum, &ctotal);  // syncs: enc_tab is ready
  uint8_t* body = fr + kFrameHeader;
  uint8_t* lo = body;
  const uint64_t nlo = uint64_t(W - 1) * n;
  uint16_t* table = reinterpret_cast<uint16_t*>(body + nlo);  // n % 8 == 0: aligned
  table[threadIdx.x] = uint16_t(lb);
  uint8_t* streams = body + nlo + kLaneTable;
  const uint64_t groups = n / 8;
  const bool aligned = (reinterpret_cast<uintptr_t>(s) & 15) == 0;
  const bool lo_aligned = (reinterpret_cast<uintptr_t>(lo) & 7) == 0;
  // bit cursor: word wpos, nb pending bits in acc; the stream starts at byte
  // loff, i.e. (loff & 3) * 8 zero bits into word loff / 4
  uint32_t wpos = loff >> 2;
  uint64_t acc = 0;
  int nb = int(loff & 3) * 8;
  // software-pipelined: the next group's load is in flight while this one is
  // coded (2 waves/SIMD at this LDS size cannot hide HBM latency otherwise)
  uint32_t nx[2 * W];
  if (threadIdx.x < groups) load_group<W>(s, threadIdx.x, aligned, nx);
  for (uint64_t g = threadIdx.x; g < groups; g += kThreads) {
    uint32_t wd[2 * W];
#pragma unroll
    for (int q = 0; q < 2 * W; ++q) wd[q] = nx[q];
    if (g + kThreads < groups) load_group<W>(s, g + kThreads, aligned, nx);
    uint64_t lw[W - 1];
#pragma unroll
    for (int k = 0; k < W - 1; ++k) lw[k] = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int e = q * 2 + h;
        const uint32_t v = group_elem<W>(wd, e);
        const uint32_t hi = v >> (8 * (W - 1));
        put_lo<W>(lw, e, v);
        const uint32_t ent = enc_tab[eslot(hi)];
        if (ent >> 31) {
          const int k = atomicAdd(&ecount, 1);
          if (k < kMaxEsc) { eidx[k] = uint32_t(g * 8 + e); evals[k] = uint8_t(hi); }
        }
        acc |= uint64_t(ent & 0xffffu) << nb;
        nb += (ent >> 16) & 31;
      }
      // after 2 codes acc holds <= 31 + 22 = 53 bits: emit a full 32-bit
      // word when there is one (predicated per lane, no divergent loop)
      if (nb >= 32) {
        atomicOr(&coded32[wpos], uint32_t(acc));
        ++wpos;
        acc >>= 32;
        nb -= 32;
      }
    }
#pragma unroll
    for (int k = 0; k < W - 1; ++k) {
      if (lo_aligned) {
        reinterpret_cast<uint64_t*>(lo)[g * (W - 1) + k] = lw[k];
      } else {
#pragma unroll
        for (int b = 0; b < 8; ++b) lo[8 * ((W - 1) * g + k) + b] = uint8_t(lw[k] >> (8 * b));
      }
    }
  }
  if (nb > 0) atomicOr(&coded32[wpos], uint32_t(acc));  // < 32 bits left
  __syncthreads();
  const uint8_t* coded = reinterpret_cast<const uint8_t*>(coded32);
  const uint32_t c_bytes = m.coded;
  if ((reinterpret_cast<uintptr_t>(streams) & 3) == 0) {
    const uint32_t nw = c_bytes / 4;
    const uint32_t* cw = reinterpret_cast<const uint32_t*>(coded);
    uint32_t* sw = reinterpret_cast<uint32_t*>(streams);
    for (uint32_t i = threadIdx.x; i < nw; i += kThreads) sw[i] = cw[i];
    for (uint32_t j = nw * 4 + threadIdx.x; j < c_bytes; j += kThreads) streams[j] = coded[j];
  } else {
    for (uint32_t j = threadIdx.x; j < c_bytes; j += kThreads) streams[j] = coded[j];
  }
  uint8_t* escp = streams + c_bytes;
  write_escapes(eidx, evals, min(ecount, kMaxEsc), escp);
  uint8_t* tail = escp + m.n_esc;
  const uint64_t tail_len = len - W * n;
  const uint64_t used = uint64_t(tail - body);
  const uint64_t padded_end = m.size - kFrameHeader;
  for (uint64_t j = threadIdx.x; used + j < padded_end; j += kThreads)
    tail[j] = j < tail_len ? s[W * n + j] : 0;
}

// One workgroup per frame; with a grid smaller than the frame count (a
// background drain caps it, hsg_set_thread_grid_cap) each workgroup walks
// several frames, so the encoder occupies only that many CUs.
template <int W>
__global__ void __launch_bounds__(kThreads)
hsz_encode2(const uint8_t* __restrict__ src, uint64_t logical, uint32_t frame_bytes,
            const FrameMeta* __restrict__ meta, const uint16_t* __restrict__ lane_bytes_all,
            uint8_t* __restrict__ out, uint32_t nf) {
  for (uint64_t f = blockIdx.x; f < nf; f += gridDim.x) {
    hsz_encode2_frame<W>(f, src, logical, frame_bytes, meta, lane_bytes_all, out);
    __syncthreads();  // the next frame reuses this workgroup's LDS
  }
}

// Mode-2 encoder, split streams (W = 2 or 4): kSub threads per lane stream.
//
// hsz_encode2 gives each of the frame's 256 lane streams ONE thread, which
// codes its groups in one serial chain, and its 64 KiB LDS stream buffer caps
// the CU at 2 such workgroups (8 waves): the chains' load and LDS latencies
// are barely hidden.  Here a 1024-thread workgroup splits every lane's groups
// into kSub consecutive pieces.  The analyze pass already recorded each
// piece's bit offset inside its stream, so every thread streams its piece
// (next group's load in flight) and packs its codes at that offset with the
// same LDS atomic-OR word assembly -- 32 waves per CU (2 workgroups), chains
// a quarter as long.  The output is byte-identical to hsz_encode2.
template <int W>
__device__ inline void
hsz_encode2x_frame(const uint64_t f, const uint8_t* __restrict__ src, uint64_t logical,
                   uint32_t frame_bytes, const FrameMeta* __restrict__ meta,
                   const uint16_t* __restrict__ lane_bytes_all,
                   const uint32_t* __restrict__ piece_bits_all, uint8_t* __restrict__ out) {
  __shared__ uint32_t coded32[(kMaxCoded + 1 + 8 + 3) / 4];
  __shared__ uint8_t code_of[260];   // indexed through cslot()
  __shared__ uint32_t enc_tab[257];  // eslot(high byte) -> codeword | len << 16 | escape << 31
  __shared__ uint16_t hcode[16];
  __shared__ uint8_t hlen[16];
  __shared__ uint32_t eidx[kMaxEsc];
  __shared__ uint8_t evals[kMaxEsc];
  __shared__ uint32_t loffs[kLanes];  // byte offset of each lane stream
  __shared__ uint32_t wsum[4];
  __shared__ int ecount;
  const FrameMeta& m = meta[f];  // arrays indexed at run time: read from memory
  if (m.mode != 2) return;
  const int tid = threadIdx.x;
  const int lane = tid & (kLanes - 1);
  const int sub = tid >> 8;
  const uint64_t base = f * frame_bytes;
  const uint64_t len = min(uint64_t(frame_bytes), logical - base);
  const uint64_t n = len / W;
  const uint8_t* s = src + base;
  uint8_t* fr = out + m.offset;
  write_frame_header(m, fr);
  if (tid < 256) code_of[cslot(tid)] = kEsc;
  const uint32_t c_words = (m.coded + 3) / 4;
  for (uint32_t i = tid; i < c_words; i += kThreadsX) coded32[i] = 0;
  if (tid < 64) {
    const uint32_t l = tid < 16 ? m.lens[tid] : 0u;
    const uint32_t code = wave_canonical_code(l);
    if (tid < 16) {
      hlen[tid] = uint8_t(l);
      hcode[tid] = uint16_t(code);
    }
    if (tid == 0) ecount = 0;
  }
  // this thread's piece: groups lane + 256 k for k in [k0, k0 + pq); the
  // first load is issued before the table setup
  const uint64_t groups = n / 8;
  const uint32_t pq = uint32_t((groups + kLanes - 1) / kLanes + kSub - 1) / kSub;
  const uint64_t g0 = uint64_t(lane) + uint64_t(kLanes) * (uint64_t(sub) * pq);
  const uint64_t g_end = min(groups, g0 + uint64_t(kLanes) * pq);
  const bool aligned = (reinterpret_cast<uintptr_t>(s) & 15) == 0;
  uint32_t nx[2 * W];
  if (g0 < g_end) load_group<W>(s, g0, aligned, nx);
  uint32_t start = 0;  // bit offset of the piece inside the lane stream
  if (sub > 0) start = piece_bits_all[(f * (kSub - 1) + (sub - 1)) * kLanes + lane];
  __syncthreads();
  if (tid < m.nsel) code_of[cslot(m.dict[tid])] = uint8_t(tid);
  uint32_t lb = 0, x = 0;
  if (tid < kLanes) {  // waves 0-3: exclusive scan of the lane stream sizes
    lb = lane_bytes_all[f * kLanes + tid];
    x = lb;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(x, o, 64);
      if ((tid & 63) >= o) x += y;
    }
    if ((tid & 63) == 63) wsum[tid >> 6] = x;
  }
  __syncthreads();
  if (tid < kLanes) {
    const uint32_t c = code_of[cslot(tid)];
    enc_tab[eslot(tid)] = uint32_t(hcode[c]) | (uint32_t(hlen[c]) << 16) |
                          (c == kEsc ? 0x80000000u : 0u);
    uint32_t b = 0;
    for (int i = 0; i < (tid >> 6); ++i) b += wsum[i];
    loffs[tid] = b + x - lb;
  }
  uint8_t* body = fr + kFrameHeader;
  uint8_t* lo = body;
  const uint64_t nlo = uint64_t(W - 1) * n;
  uint16_t* table = reinterpret_cast<uint16_t*>(body + nlo);  // n % 8 == 0: aligned
  if (tid < kLanes) table[tid] = uint16_t(lb);
  uint8_t* streams = body + nlo + kLaneTable;
  __syncthreads();  // enc_tab, loffs ready
  // bit cursor: word wpos, nb pending bits in acc (the low nb are placeholders
  // for bits owned by the piece or lane before this one: OR-ed in LDS)
  start += loffs[lane] * 8;
  uint32_t wpos = start >> 5;
  uint64_t acc = 0;
  int nb = int(start & 31);
  const bool lo_aligned = (reinterpret_cast<uintptr_t>(lo) & 7) == 0;
  for (uint64_t g = g0; g < g_end; g += kLanes) {
    uint32_t wd[2 * W];
#pragma unroll
    for (int q = 0; q < 2 * W; ++q) wd[q] = nx[q];
    if (g + kLanes < g_end) load_group<W>(s, g + kLanes, aligned, nx);
    // the group's 8 table lookups are issued together (one LDS wait), and
    // the rare escapes take one branch per group, not one per element
    uint32_t ent[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) ent[e] = enc_tab[eslot(group_elem<W>(wd, e) >> (8 * (W - 1)))];
    uint64_t lw[W - 1];
#pragma unroll
    for (int k = 0; k < W - 1; ++k) lw[k] = 0;
    uint32_t esc = 0;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      put_lo<W>(lw, e, group_elem<W>(wd, e));
      esc |= (ent[e] >> 31) << e;
    }
    if (esc) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        if ((esc >> e) & 1) {
          const int k = atomicAdd(&ecount, 1);
          if (k < kMaxEsc) {
            eidx[k] = uint32_t(g * 8 + e);
            evals[k] = uint8_t(group_elem<W>(wd, e) >> (8 * (W - 1)));
          }
        }
      }
    }
#pragma unroll
    for (int p = 0; p < 4; ++p) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const uint32_t en = ent[p * 2 + h];
        acc |= uint64_t(en & 0xffffu) << nb;
        nb += (en >> 16) & 31;
      }
      if (nb >= 32) {  // <= 31 + 22 bits after two codes: at most one full word
        atomicOr(&coded32[wpos], uint32_t(acc));
        ++wpos;
        acc >>= 32;
        nb -= 32;
      }
    }
#pragma unroll
    for (int k = 0; k < W - 1; ++k) {
      if (lo_aligned) {
        reinterpret_cast<uint64_t*>(lo)[g * (W - 1) + k] = lw[k];
      } else {
#pragma unroll
        for (int b = 0; b < 8; ++b) lo[8 * ((W - 1) * g + k) + b] = uint8_t(lw[k] >> (8 * b));
      }
    }
  }
  if (nb > 0) atomicOr(&coded32[wpos], uint32_t(acc));  // < 32 bits left
  __syncthreads();
  const uint8_t* coded = reinterpret_cast<const uint8_t*>(coded32);
  const uint32_t c_bytes = m.coded;
  if ((reinterpret_cast<uintptr_t>(streams) & 3) == 0) {
    const uint32_t nw = c_bytes / 4;
    const uint32_t* cw = reinterpret_cast<const uint32_t*>(coded);
    uint32_t* sw = reinterpret_cast<uint32_t*>(streams);
    for (uint32_t i = tid; i < nw; i += kThreadsX) sw[i] = cw[i];
    for (uint32_t j = nw * 4 + tid; j < c_bytes; j += kThreadsX) streams[j] = coded[j];
  } else {
    for (uint32_t j = tid; j < c_bytes; j += kThreadsX) streams[j] = coded[j];
  }
  uint8_t* escp = streams + c_bytes;
  write_escapes<kThreadsX>(eidx, evals, min(ecount, kMaxEsc), escp);
  uint8_t* tail = escp + m.n_esc;
  const uint64_t tail_len = len - W * n;
  const uint64_t used = uint64_t(tail - body);
  const uint64_t padded_end = m.size - kFrameHeader;
  for (uint64_t j = tid; used + j < padded_end; j += kThreadsX)
    tail[j] = j < tail_len ? s[W * n + j] : 0;
}

template <int W>
__global__ void __launch_bounds__(kThreadsX, W == 2 ? 8 : 4)  // bf16: 2 workgroups / CU (<= 64 VGPRs)
hsz_encode2x(const uint8_t* __restrict__ src, uint64_t logical, uint32_t frame_bytes,
             const FrameMeta* __restrict__ meta, const uint16_t* __restrict__ lane_bytes_all,
             const uint32_t* __restrict__ piece_bits_all, uint8_t* __restrict__ out,
             uint32_t nf) {
  for (uint64_t f = blockIdx.x; f < nf; f += gridDim.x) {
    hsz_encode2x_frame<W>(f, src, logical, frame_bytes, meta, lane_bytes_all, piece_bits_all,
                          out);
    __syncthreads();  // the next frame reuses this workgroup's LDS
  }
}

// hsz_encode2x needs the analyze pass's piece offsets, recorded while a
// piece holds < 256 elements (byte counters): frames up to ~1 MiB of bf16.
__host__ __device__ constexpr bool encode2x_fits(int w, uint64_t frame_bytes) {
  return ((frame_bytes / uint64_t(w) / 8 + kLanes - 1) / kLanes + kSub - 1) / kSub * 8 < 256;
}

// A rejected (corrupt / truncated) frame is reported through `err` (host-
// mapped pinned word, may be null): one plain store of 1 -- every writer
// stores the same value -- read by the host after the stream sync, so a bad
// blob raises like the host decoder's -74 instead of restoring stale bytes.
__device__ __forceinline__ void flag_corrupt(uint32_t* err) {
  if (err != nullptr) *reinterpret_cast<volatile uint32_t*>(err) = 1u;
}

template <int W>
__global__ void __launch_bounds__(kThreads)
hsz_decode(const uint8_t* __restrict__ frames, const uint64_t* __restrict__ offsets,
           uint32_t first_frame, uint64_t logical, uint32_t frame_bytes,
           uint8_t* __restrict__ out, uint32_t* err) {
  __shared__ uint32_t eidx[kMaxEsc];
  __shared__ uint32_t sorted[kMaxEsc];
  __shared__ int ecount;
  __shared__ uint8_t dict[16];
  const uint64_t fl = blockIdx.x;             // local frame index
  const uint64_t f = first_frame + fl;         // global frame index
  const uint64_t base = f * frame_bytes;
  const uint64_t len = min(uint64_t(frame_bytes), logical - base);
  const uint64_t n = len / W;
  const uint8_t* fr = frames + offsets[fl];
  const uint64_t extent = offsets[fl + 1] - offsets[fl];
  // every early return below depends only on the frame: uniform per block
  if (offsets[fl + 1] < offsets[fl] + kFrameHeader) {
    if (threadIdx.x == 0) flag_corrupt(err);
    return;
  }
  uint8_t* o = out + fl * uint64_t(frame_bytes);
  const int mode = fr[0];
  const uint8_t* body = fr + kFrameHeader;
  if (mode == 2) {  // hsz_decode2 (element widths 2 and 4 only)
    if (W != 2 && W != 4 && threadIdx.x == 0) flag_corrupt(err);
    return;
  }
  if (mode == 0 && kFrameHeader + len > extent) {
    if (threadIdx.x == 0) flag_corrupt(err);
    return;
  }
  if (mode == 0) {
    if ((((reinterpret_cast<uintptr_t>(o)) | reinterpret_cast<uintptr_t>(body)) & 15) == 0) {
      const uint64_t nv = len / 16;
      const uint4* sv = reinterpret_cast<const uint4*>(body);
      uint4* dv = reinterpret_cast<uint4*>(o);
      for (uint64_t i = threadIdx.x; i < nv; i += kThreads) dv[i] = sv[i];
      for (uint64_t j = nv * 16 + threadIdx.x; j < len; j += kThreads) o[j] = body[j];
    } else {
      for (uint64_t j = threadIdx.x; j < len; j += kThreads) o[j] = body[j];
    }
    return;
  }
  const uint32_t n_esc = *reinterpret_cast<const uint32_t*>(fr + 4);
  const uint64_t nb = (n + 1) / 2;
  if (mode != 1 || n_esc > uint32_t(kMaxEsc) ||
      kFrameHeader + nb + uint64_t(W - 1) * n + n_esc + (len - n * W) > extent) {
    if (threadIdx.x == 0) flag_corrupt(err);
    return;
  }
  if (threadIdx.x < 16) dict[threadIdx.x] = fr[8 + threadIdx.x];
  if (threadIdx.x == 0) ecount = 0;
  __syncthreads();
  const uint8_t* nib = body;
  const uint8_t* lo = body + nb;
  const uint8_t* escv = lo + uint64_t(W - 1) * n;
  if (n_esc > 0) {
    // collect escape element indices (nibble value 15), then sort them by rank
    for (uint64_t p = threadIdx.x; p < nb; p += kThreads) {
      const uint8_t b = nib[p];
      if ((b & 15) == kEsc && 2 * p < n) {
        const int k = atomicAdd(&ecount, 1);
        if (k < kMaxEsc) eidx[k] = uint32_t(2 * p);
      }
      if ((b >> 4) == kEsc && 2 * p + 1 < n) {
        const int k = atomicAdd(&ecount, 1);
        if (k < kMaxEsc) eidx[k] = uint32_t(2 * p + 1);
      }
    }
    __syncthreads();
    const int ne = min(ecount, kMaxEsc);
    for (int i = threadIdx.x; i < ne; i += kThreads) {
      const uint32_t me = eidx[i];
      int rank = 0;
      for (int j = 0; j < ne; ++j) rank += eidx[j] < me;
      sorted[rank] = me;
    }
    __syncthreads();
  }
  const int n_found = min(min(ecount, kMaxEsc), int(n_esc));
  auto esc_value = [&](uint32_t e) -> uint8_t {
    int lo_i = 0, hi_i = n_found - 1;
    if (hi_i < 0) return 0;
    while (lo_i < hi_i) {
      const int mid = (lo_i + hi_i) >> 1;
      if (sorted[mid] < e) lo_i = mid + 1; else hi_i = mid;
    }
    return escv[lo_i];
  };
  const bool fast = (reinterpret_cast<uintptr_t>(o) & 15) == 0 &&
                    ((reinterpret_cast<uintptr_t>(nib) | reinterpret_cast<uintptr_t>(lo)) & 7) == 0 &&
                    (n % 8) == 0;
  uint64_t done = 0;
  if (fast && W == 2) {
    const uint64_t groups = n / 8;
    const uint32_t* nv = reinterpret_cast<const uint32_t*>(nib);
    const uint64_t* lv = reinterpret_cast<const uint64_t*>(lo);
    uint4* ov = reinterpret_cast<uint4*>(o);
    for (uint64_t g = threadIdx.x; g < groups; g += kThreads) {
      const uint32_t codes = nv[g];
      const uint64_t lob = lv[g];
      uint32_t wd[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        uint32_t x = 0;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int e = q * 2 + h;
          const uint32_t c = (codes >> (4 * e)) & 15;
          const uint32_t hi = c == kEsc ? esc_value(uint32_t(g * 8 + e)) : dict[c];
          x |= ((uint32_t((lob >> (8 * e)) & 255)) | (hi << 8)) << (16 * h);
        }
        wd[q] = x;
      }
      ov[g] = make_uint4(wd[0], wd[1], wd[2], wd[3]);
    }
    done = n;
  } else if (fast && W == 4) {
    const uint64_t groups = n / 8;
    const uint32_t* nv = reinterpret_cast<const uint32_t*>(nib);
    uint4* ov = reinterpret_cast<uint4*>(o);
    for (uint64_t g = threadIdx.x; g < groups; g += kThreads) {
      const uint32_t codes = nv[g];
      const uint64_t* lv = reinterpret_cast<const uint64_t*>(lo + 24 * g);
      const uint64_t l0 = lv[0], l1 = lv[1], l2 = lv[2];
      uint32_t wd[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const uint32_t c = (codes >> (4 * e)) & 15;
        const uint32_t hi = c == kEsc ? esc_value(uint32_t(g * 8 + e)) : dict[c];
        uint32_t b[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          const int bi = 3 * e + k;
          const uint64_t src = bi < 8 ? l0 : (bi < 16 ? l1 : l2);
          b[k] = uint32_t((src >> (8 * (bi & 7))) & 255);
        }
        wd[e] = b[0] | (b[1] << 8) | (b[2] << 16) | (hi << 24);
      }
      ov[2 * g] = make_uint4(wd[0], wd[1], wd[2], wd[3]);
      ov[2 * g + 1] = make_uint4(wd[4], wd[5], wd[6], wd[7]);
    }
    done = n;
  }
  if (done < n) {
    for (uint64_t e = threadIdx.x; e < n; e += kThreads) {
      const uint32_t c = (nib[e >> 1] >> (4 * (e & 1))) & 15;
      const uint8_t hi = c == kEsc ? esc_value(uint32_t(e)) : dict[c];
      for (int b = 0; b < W - 1; ++b) o[e * W + b] = lo[e * (W - 1) + b];
      o[e * W + W - 1] = hi;
    }
  }
  const uint8_t* tail = escv + n_esc;
  for (uint64_t j = threadIdx.x; j < len - n * W; j += kThreads) o[n * W + j] = tail[j];
}

// Branch-free bit-buffer refill to 56..63 valid bits: the 8 stream bytes at
// byte `pos` come from two aligned 8-B LDS reads and a funnel shift.  Bits of
// a byte that only partly fits are OR-ed in again (same values) next time.
__device__ __forceinline__ void refill(const uint64_t* coded64, uint32_t& pos, uint64_t& acc,
                                       int& nb) {
  const uint32_t q = pos >> 3, sh = (pos & 7) * 8;
  const uint64_t a = coded64[q], b = coded64[q + 1];
  const uint64_t bits = sh ? (a >> sh) | (b << (64 - sh)) : a;
  acc |= bits << nb;
  const int k = (63 - nb) >> 3;
  pos += k;
  nb += 8 * k;
}

// LUT entry of the lean decoder: code length (bits 0-3; bit 4 is 0, so the
// entry itself is a valid v_alignbit / v_lshrrev shift amount), escape (5),
// invalid code (6; length kMaxLen so a corrupt lane still advances by a
// bounded amount), decoded high byte (8-15).
constexpr uint32_t kEntEsc = 0x20u, kEntBad = 0x40u;

// Lean mode-2 decoder (it replaced the round-3 LDS decoder).  Measured (profiles/r4/decode_pmc/): a frame's
// decode is latency-bound -- one frame alone on a CU takes as long as 2 per
// CU, so neither LDS bank conflicts nor issue rate set the pace, but the
// serial chain of each lane stream (512 symbols per lane for bf16) and the
// HBM round trips inside it.  So:
//   * the LUT entry carries the decoded high byte itself and its length in
//     the bits a shift reads: one LDS read per symbol, no dictionary read,
//     escapes and invalid codes are OR-ed into a per-group flag word and
//     handled off the chain;
//   * the bit window is kept pre-shifted by one bit as two 32-bit halves:
//     the chain per symbol is LUT read -> v_alignbit (by the entry) -> v_and
//     -> next LUT read (the 64-bit shift, the length extraction and the
//     index scaling are off it);
//   * the window is refilled from the LDS-staged streams twice per 8 symbols
//     (>= 56 bits cover 5 codes), and the staging copy has all of a thread's
//     16-B loads in flight at once;
//   * P > 0: the low-byte plane is loaded P groups ahead;
//   * bf16 pairs are assembled with v_perm.
// A frame whose fields do not fit its stored extent, or whose lane streams
// decode invalid codes or overrun, is flagged through `err` (the host
// validated the frame table itself).
template <int W, int P>
__global__ void __launch_bounds__(kThreads)
hsz_decode2g(const uint8_t* __restrict__ frames, const uint64_t* __restrict__ offsets,
             uint32_t first_frame, uint64_t logical, uint32_t frame_bytes,
             uint8_t* __restrict__ out, uint32_t* err) {
  // the LUT at the start of the big LDS array: its reads need no base add
  // (a base past 64 KB does not fit the ds_read offset field)
  __shared__ uint64_t smem[kLut / 4 + (kMaxCoded + 1 + 16 + 7) / 8];
  uint16_t* lut = reinterpret_cast<uint16_t*>(smem);
  uint64_t* coded64 = smem + kLut / 4;
  __shared__ uint16_t hcode[16];
  __shared__ uint8_t hlen[16];
  __shared__ uint8_t dict[16];
  __shared__ uint32_t eidx[kMaxEsc];
  __shared__ uint32_t sorted[kMaxEsc];
  __shared__ uint32_t wsum[4];
  __shared__ uint32_t ctotal;
  __shared__ int ecount;
  __shared__ int valid;
  const uint64_t fl = blockIdx.x;
  const uint64_t f = first_frame + fl;
  const uint64_t base = f * frame_bytes;
  const uint64_t len = min(uint64_t(frame_bytes), logical - base);
  const uint64_t n = len / W;
  const uint64_t nlo = uint64_t(W - 1) * n;
  const uint8_t* fr = frames + offsets[fl];
  const uint64_t extent = offsets[fl + 1] - offsets[fl];
  if (offsets[fl + 1] < offsets[fl] + kFrameHeader || fr[0] != 2) return;
  uint8_t* o = out + fl * uint64_t(frame_bytes);
  const uint32_t n_esc = *reinterpret_cast<const uint32_t*>(fr + 4);
  if (threadIdx.x < 16) {
    dict[threadIdx.x] = fr[8 + threadIdx.x];
    hlen[threadIdx.x] = (fr[24 + threadIdx.x / 2] >> (4 * (threadIdx.x & 1))) & 15;
  }
  if (threadIdx.x == 0) ecount = 0;
  // the lane table's load overlaps the header's (bounds checked here; the
  // frame is rejected below when it is short)
  const uint8_t* body = fr + kFrameHeader;
  const uint8_t* lo = body;
  uint32_t lb = 0;
  if (kFrameHeader + nlo + kLaneTable <= extent)
    lb = reinterpret_cast<const uint16_t*>(body + nlo)[threadIdx.x];
  __syncthreads();
  if (threadIdx.x < 64) {
    const uint32_t l = threadIdx.x < 16 ? hlen[threadIdx.x] : 0u;
    const bool long_code = __ballot(l > uint32_t(kMaxLen)) != 0;
    const uint32_t code = wave_canonical_code(l < uint32_t(kMaxLen) ? l : uint32_t(kMaxLen));
    if (threadIdx.x < 16) hcode[threadIdx.x] = uint16_t(code);
    if (threadIdx.x == 0)
      valid = !long_code && n % 8 == 0 && n_esc <= uint32_t(kMaxEsc) &&
              kFrameHeader + nlo + kLaneTable <= extent;
  }
  __syncthreads();
  if (!valid) {
    if (threadIdx.x == 0) flag_corrupt(err);
    return;
  }
  const uint32_t loff = block_excl_scan(lb, wsum, &ctotal);
  const uint32_t c_bytes = ctotal;
  const uint64_t tail_len = len - W * n;
  if (c_bytes > kMaxCoded ||
      kFrameHeader + nlo + kLaneTable + c_bytes + n_esc + tail_len > extent) {
    if (threadIdx.x == 0) flag_corrupt(err);
    return;  // uniform across the workgroup (ctotal is shared)
  }
  const uint8_t* streams = body + nlo + kLaneTable;
  const uint64_t groups = n / 8;
  const bool vec = ((reinterpret_cast<uintptr_t>(o) & 15) | (reinterpret_cast<uintptr_t>(lo) & 7)) == 0;
  // the streams' 16-B loads (all of a thread's in flight at once) are issued
  // before the LUT is built and land in LDS after it: the HBM round trip
  // hides behind the LUT's VALU work
  uint8_t* coded = reinterpret_cast<uint8_t*>(coded64);
  const bool s16_ok = (reinterpret_cast<uintptr_t>(streams) & 15) == 0;
  const uint32_t n16 = s16_ok ? c_bytes / 16 : 0;
  const uint4* s16 = reinterpret_cast<const uint4*>(streams);
  uint4 t[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const uint32_t i = threadIdx.x + q * kThreads;
    t[q] = i < n16 ? s16[i] : make_uint4(0u, 0u, 0u, 0u);
  }
  for (int x = threadIdx.x; x < kLut; x += kThreads) {
    uint32_t ent = kEntBad | uint32_t(kMaxLen);
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      const uint32_t l = hlen[c];
      if (l && (uint32_t(x) & ((1u << l) - 1)) == hcode[c])
        ent = (c == kEsc ? kEntEsc : uint32_t(dict[c]) << 8) | l;
    }
    lut[x] = uint16_t(ent);
  }
  {
    uint4* d16 = reinterpret_cast<uint4*>(coded);
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const uint32_t i = threadIdx.x + q * kThreads;
      if (i < n16) d16[i] = t[q];
    }
    for (uint32_t j = n16 * 16 + threadIdx.x; j < c_bytes; j += kThreads) coded[j] = streams[j];
    if (threadIdx.x < 16) coded[c_bytes + threadIdx.x] = 0;
    __syncthreads();  // orders the LUT and the staged streams before any read
  }
  // window = stream bits << 1 (bit 0 is always 0, so `lo & 0xffe` is the
  // LUT's byte offset); nb = valid stream bits in it
  uint32_t wlo = 0, whi = 0;
  int nb = 0;
  uint32_t pos = loff;
  uint32_t allfl = 0;
  const uint8_t* lut8 = reinterpret_cast<const uint8_t*>(lut);
  auto group = [&](uint64_t g, const uint64_t* lw, auto vec_tag) {
    constexpr bool kVec = decltype(vec_tag)::value;
    uint32_t ent[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      if (e == 0 || e == 5) {  // every lane at the same points: top up to >= 56 bits
        const uint32_t q = pos >> 3, sh = (pos & 7) * 8;
        const uint64_t a = coded64[q], b = coded64[q + 1];
        const uint64_t bits = sh ? (a >> sh) | (b << (64 - sh)) : a;
        // nb <= 60 here (>= 3 bits went since the last refill), so nb + 1 < 64
        const uint64_t w = ((uint64_t(whi) << 32) | wlo) | (bits << (nb + 1));
        wlo = uint32_t(w);
        whi = uint32_t(w >> 32);
        const int k = (63 - nb) >> 3;
        pos += k;
        nb += 8 * k;
      }
      ent[e] = *reinterpret_cast<const uint16_t*>(lut8 + (wlo & (2 * kLut - 2)));
      wlo = __builtin_amdgcn_alignbit(whi, wlo, ent[e]);  // (uses bits 0-4)
      whi >>= ent[e] & 31;
      nb -= int(ent[e] & 15);
    }
    const uint32_t fl8 = ent[0] | ent[1] | ent[2] | ent[3] | ent[4] | ent[5] | ent[6] | ent[7];
    allfl |= fl8;
    if (fl8 & kEntEsc) {
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (ent[e] & kEntEsc) {
          const int k = atomicAdd(&ecount, 1);
          if (k < kMaxEsc) eidx[k] = uint32_t(g * 8 + e);
        }
    }
    uint32_t wd[2 * W];
    if constexpr (W == 2) {
      // dword q = [lo 2q, hi 2q, lo 2q+1, hi 2q+1]
      const uint32_t lw0 = uint32_t(lw[0]), lw1 = uint32_t(lw[0] >> 32);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint32_t hh = __builtin_amdgcn_perm(ent[2 * q + 1], ent[2 * q], 0x0c0c0501u);
        wd[q] = __builtin_amdgcn_perm(hh, q < 2 ? lw0 : lw1, (q & 1) ? 0x05030402u : 0x05010400u);
      }
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) wd[e] = get_lo<W>(lw, e) | (((ent[e] >> 8) & 255u) << (8 * (W - 1)));
    }
    if constexpr (kVec) {
#pragma unroll
      for (int k = 0; k < W / 2; ++k)
        reinterpret_cast<uint4*>(o)[g * (W / 2) + k] =
            make_uint4(wd[4 * k], wd[4 * k + 1], wd[4 * k + 2], wd[4 * k + 3]);
    } else {
#pragma unroll
      for (int q = 0; q < 2 * W; ++q)
#pragma unroll
        for (int b = 0; b < 4; ++b) o[8 * W * g + 4 * q + b] = uint8_t(wd[q] >> (8 * b));
    }
  };
  auto run = [&](auto vec_tag) {
    constexpr bool kVec = decltype(vec_tag)::value;
    // P > 0: the low bytes of group g + P * kThreads load while group g
    // decodes (a group's 8 symbols are ~1/4 of an HBM round trip).  Taken when
    // every lane has a multiple of P groups (all full frames): the loop then
    // has no branch around its loads, so each wait covers exactly its load.
    if constexpr (P > 0) {
      if (groups % (uint64_t(P) * kThreads) == 0) {
        uint64_t buf[P][W - 1];
#pragma unroll
        for (int b = 0; b < P; ++b) load_lo<W>(lo, threadIdx.x + uint64_t(b) * kThreads, kVec, buf[b]);
        for (uint64_t g0 = threadIdx.x; g0 < groups; g0 += uint64_t(P) * kThreads) {
#pragma unroll
          for (int b = 0; b < P; ++b) {
            const uint64_t g = g0 + uint64_t(b) * kThreads;
            uint64_t lw[W - 1];
#pragma unroll
            for (int k = 0; k < W - 1; ++k) lw[k] = buf[b][k];
            load_lo<W>(lo, min(g + uint64_t(P) * kThreads, groups - 1), kVec, buf[b]);
            group(g, lw, vec_tag);
          }
        }
        return;
      }
    }
    for (uint64_t g = threadIdx.x; g < groups; g += kThreads) {
      uint64_t lw[W - 1];
      load_lo<W>(lo, g, kVec, lw);
      group(g, lw, vec_tag);
    }
  };
  if (vec) run(std::true_type{});
  else run(std::false_type{});
  // a lane may not read past its own stream (host decoder: same check)
  if ((allfl & kEntBad) || uint64_t(pos - loff) * 8 - uint64_t(nb) > uint64_t(lb) * 8)
    flag_corrupt(err);
  __syncthreads();
  const uint8_t* escv = streams + c_bytes;
  const int ne = min(min(ecount, kMaxEsc), int(n_esc));
  for (int i = threadIdx.x; i < ne; i += kThreads) {
    const uint32_t me = eidx[i];
    int rank = 0;
    for (int j = 0; j < ne; ++j) rank += eidx[j] < me;
    sorted[rank] = me;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < ne; i += kThreads) o[W * uint64_t(sorted[i]) + W - 1] = escv[i];
  if (threadIdx.x < tail_len) o[W * n + threadIdx.x] = escv[n_esc + threadIdx.x];
}

thread_local char g_hsz_err[256];

int fail(const char* what, hipError_t e) {
  snprintf(g_hsz_err, sizeof(g_hsz_err), "%s: %s", what, hipGetErrorString(e));
  return -static_cast<int>(e) - 1;
}

}  // namespace

extern "C" {

const char* hsg_hsz_last_error() { return g_hsz_err; }

uint64_t hsg_hsz_meta_bytes(uint32_t n_frames) {
  return uint64_t(n_frames) *
         (sizeof(FrameMeta) + sizeof(uint16_t) * kLanes + sizeof(uint32_t) * (kSub - 1) * kLanes);
}

// Encode `logical` bytes at device `src` (16-B aligned) into device `out`
// (capacity >= max_encoded_bytes).  `meta` = device scratch of
// hsg_hsz_meta_bytes(n_frames); `total` = device u64 receiving the blob size.
// Everything is enqueued on `stream`; nothing synchronises.
int hsg_hsz_encode(int dev, const void* src, uint64_t logical, int w, uint32_t frame_bytes,
                   void* out, void* meta, void* total, void* stream) {
  hipError_t e = hipSetDevice(dev);
  if (e != hipSuccess) return fail("hipSetDevice", e);
  if (frame_bytes % 16 || frame_bytes % w) return -1000;
  const uint32_t nf = logical ? uint32_t((logical + frame_bytes - 1) / frame_bytes) : 1;
  hipStream_t s = static_cast<hipStream_t>(stream);
  auto* src8 = static_cast<const uint8_t*>(src);
  auto* m = static_cast<FrameMeta*>(meta);
  auto* lanes = reinterpret_cast<uint16_t*>(m + nf);
  auto* o = static_cast<uint8_t*>(out);
  const int cap = hsg_thread_grid_cap();
  const uint32_t g = cap > 0 ? std::min<uint32_t>(nf, uint32_t(cap)) : nf;
  auto* pbits = reinterpret_cast<uint32_t*>(lanes + uint64_t(nf) * kLanes);
  switch (w) {
    case 1: hipLaunchKernelGGL(hsz_analyze<1>, dim3(g), dim3(kThreads), 0, s, src8, logical, frame_bytes, m, lanes, pbits, nf); break;
    case 2: hipLaunchKernelGGL(hsz_analyze<2>, dim3(g), dim3(kThreads), 0, s, src8, logical, frame_bytes, m, lanes, pbits, nf); break;
    case 4: hipLaunchKernelGGL(hsz_analyze<4>, dim3(g), dim3(kThreads), 0, s, src8, logical, frame_bytes, m, lanes, pbits, nf); break;
    case 8: hipLaunchKernelGGL(hsz_analyze<8>, dim3(g), dim3(kThreads), 0, s, src8, logical, frame_bytes, m, lanes, pbits, nf); break;
    default: return -1001;
  }
  hipLaunchKernelGGL(hsz_layout, dim3(1), dim3(1024), 0, s, m, nf, o, logical, uint32_t(w),
                     frame_bytes, static_cast<uint64_t*>(total));
  switch (w) {
    case 1: hipLaunchKernelGGL(hsz_encode<1>, dim3(g), dim3(kThreads), 0, s, src8, logical, frame_bytes, m, o, nf); break;
    case 2: hipLaunchKernelGGL(hsz_encode<2>, dim3(g), dim3(kThreads), 0, s, src8, logical, frame_bytes, m, o, nf); break;
    case 4: hipLaunchKernelGGL(hsz_encode<4>, dim3(g), dim3(kThreads), 0, s, src8, logical, frame_bytes, m, o, nf); break;
    default: hipLaunchKernelGGL(hsz_encode<8>, dim3(g), dim3(kThreads), 0, s, src8, logical, frame_bytes, m, o, nf); break;
  }
  // bf16/fp16: split-stream encoder (802 -> 420 us per GiB); fp32 stays on
  // hsz_encode2 (449 us vs 525 us: twice the bytes per group under the split
  // kernel's 64-VGPR budget) -- profiles/codec_r2/split_encode.md
  if (w == 2 && encode2x_fits(w, frame_bytes))
    hipLaunchKernelGGL(hsz_encode2x<2>, dim3(g), dim3(kThreadsX), 0, s, src8, logical,
                       frame_bytes, m, lanes, pbits, o, nf);
  else if (w == 2)
    hipLaunchKernelGGL(hsz_encode2<2>, dim3(g), dim3(kThreads), 0, s, src8, logical, frame_bytes,
                       m, lanes, o, nf);
  else if (w == 4)
    hipLaunchKernelGGL(hsz_encode2<4>, dim3(g), dim3(kThreads), 0, s, src8, logical, frame_bytes,
                       m, lanes, o, nf);
  e = hipGetLastError();
  return e == hipSuccess ? 0 : fail("hsz encode launch", e);
}

// Decode `count` frames starting at global frame `first` into `out` (logical
// bytes of those frames).  `offsets` (device, count + 1 entries) are byte
// offsets of each frame relative to `frames`, then the end of the last one.
// `err` (nullable): host-mapped pinned uint32 set to 1 when any frame is
// rejected; read it after synchronising `stream`.
int hsg_hsz_decode(int dev, const void* frames, const void* offsets, uint32_t first,
                   uint32_t count, uint64_t logical, int w, uint32_t frame_bytes, void* out,
                   void* stream, void* err) {
  hipError_t e = hipSetDevice(dev);
  if (e != hipSuccess) return fail("hipSetDevice", e);
  if (count == 0) return 0;
  hipStream_t s = static_cast<hipStream_t>(stream);
  auto* fr = static_cast<const uint8_t*>(frames);
  auto* off = static_cast<const uint64_t*>(offsets);
  auto* o = static_cast<uint8_t*>(out);
  auto* ew = static_cast<uint32_t*>(err);
  switch (w) {
    case 1: hipLaunchKernelGGL(hsz_decode<1>, dim3(count), dim3(kThreads), 0, s, fr, off, first, logical, frame_bytes, o, ew); break;
    case 2: hipLaunchKernelGGL(hsz_decode<2>, dim3(count), dim3(kThreads), 0, s, fr, off, first, logical, frame_bytes, o, ew); break;
    case 4: hipLaunchKernelGGL(hsz_decode<4>, dim3(count), dim3(kThreads), 0, s, fr, off, first, logical, frame_bytes, o, ew); break;
    case 8: hipLaunchKernelGGL(hsz_decode<8>, dim3(count), dim3(kThreads), 0, s, fr, off, first, logical, frame_bytes, o, ew); break;
    default: return -1001;
  }
  if (w == 2)
    hipLaunchKernelGGL((hsz_decode2g<2, 8>), dim3(count), dim3(kThreads), 0, s, fr, off, first,
                       logical, frame_bytes, o, ew);
  else if (w == 4)
    hipLaunchKernelGGL((hsz_decode2g<4, 8>), dim3(count), dim3(kThreads), 0, s, fr, off, first,
                       logical, frame_bytes, o, ew);
  e = hipGetLastError();
  return e == hipSuccess ? 0 : fail("hsz decode launch", e);
}

}  // extern "C"
