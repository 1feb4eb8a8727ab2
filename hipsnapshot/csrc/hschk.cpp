// hs64: the blob checksum of hipsnapshot snapshots (host side).
//
// Definition (also implemented by the gfx950 kernel `hs_hash64` in hsgpu.hip
// and by the NumPy reference in hipsnapshot/ops/checksum.py):
//
//   words w_i = little-endian uint64 of bytes [8i, 8i+8), the last one
//               zero-padded;
//   S  = sum_i mix64(w_i ^ ((i + 1) * 0x9E3779B97F4A7C15))   (mod 2^64)
//   hs64(blob) = mix64(S ^ n_bytes)
//
// mix64 is the SplitMix64 finalizer.  Every word is mixed with its own index,
// so the sum is order-sensitive yet splits over any 8-byte-aligned ranges:
// the GPU sums ranges in parallel (one atomic add per wave), the host sums
// ranges on several threads, and a reader can check a blob it fetched in
// pieces.  It detects corruption (bit flips, truncation, misplaced blocks);
// it is not a cryptographic hash.

#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

namespace {

constexpr uint64_t kM1 = 0x9E3779B97F4A7C15ull;

inline uint64_t mix64(uint64_t x) {
  x ^= x >> 30;
  x *= 0xBF58476D1CE4E5B9ull;
  x ^= x >> 27;
  x *= 0x94D049BB133111EBull;
  x ^= x >> 31;
  return x;
}

// Sum over `nw` whole words.  One plain loop the compiler vectorises; the
// clones give it 64-bit vector multiplies (AVX-512DQ vpmullq) or AVX2 where
// the CPU has them, picked at load time (the .so is built once, here, and
// runs on whichever host the GPU box has).
__attribute__((target_clones("arch=skylake-avx512", "avx2", "default")))
uint64_t words_sum(const uint8_t* p, uint64_t nw, uint64_t w0) {
  uint64_t s = 0;
  for (uint64_t i = 0; i < nw; ++i) {
    uint64_t a;
    std::memcpy(&a, p + 8 * i, 8);
    s += mix64(a ^ ((w0 + i + 1) * kM1));
  }
  return s;
}

// Sum over the bytes [p, p + n) whose first word has global index `w0`.
uint64_t partial(const uint8_t* p, uint64_t n, uint64_t w0) {
  const uint64_t nw = n / 8;
  uint64_t s = words_sum(p, nw, w0);
  const uint64_t tail = n - 8 * nw;
  if (tail) {
    uint64_t t = 0;
    std::memcpy(&t, p + 8 * nw, tail);
    s += mix64(t ^ ((w0 + nw + 1) * kM1));
  }
  return s;
}

}  // namespace

extern "C" {

// Partial sum S over [p, p + n), p being at byte offset 8 * first_word of the
// blob; split across up to `nthreads` threads for large ranges.
uint64_t hs64_partial(const void* p, uint64_t n, uint64_t first_word, int nthreads) {
  const auto* b = static_cast<const uint8_t*>(p);
  const uint64_t per_min = uint64_t(16) << 20;
  if (nthreads <= 1 || n < 2 * per_min) return partial(b, n, first_word);
  uint64_t per = (n / 8 + uint64_t(nthreads) - 1) / uint64_t(nthreads) * 8;
  if (per < per_min) per = per_min;
  std::vector<uint64_t> sums((n + per - 1) / per, 0);
  std::vector<std::thread> ts;
  for (size_t k = 0; k < sums.size(); ++k) {
    const uint64_t lo = k * per;
    const uint64_t len = lo + per > n ? n - lo : per;
    ts.emplace_back([&, k, lo, len] { sums[k] = partial(b + lo, len, first_word + lo / 8); });
  }
  for (auto& t : ts) t.join();
  uint64_t s = 0;
  for (uint64_t v : sums) s += v;
  return s;
}

uint64_t hs64_finish(uint64_t sum, uint64_t n_bytes) { return mix64(sum ^ n_bytes); }

}  // extern "C"
