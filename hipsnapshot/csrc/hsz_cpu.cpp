// HSZ1 codec on the host (format: hipsnapshot/ops/codec.py; GPU: hsz.hip).
//
// Used for CPU tensors on save and for CPU destinations on restore.  Frames
// are independent, so a blob is split across threads by frame; within a frame
// the loops are plain byte loops the compiler vectorises.

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

namespace {

constexpr int kSample = 2048;
constexpr uint32_t kMaxEsc = 1024;
constexpr uint64_t kHeader = 64;
constexpr uint64_t kFrameHeader = 32;
constexpr uint8_t kEsc = 15;

inline uint64_t align16(uint64_t n) { return (n + 15) & ~uint64_t(15); }

struct Plan {
  uint8_t mode = 0;
  uint32_t n_esc = 0;
  int nsel = 0;
  uint8_t dict[16] = {0};
  uint8_t code_of[256];
  uint64_t size = 0;
};

void plan_frame(const uint8_t* s, uint64_t len, int w, Plan* p) {
  const uint64_t n = len / w;
  uint32_t hist[256] = {0};
  const uint64_t stride = n / kSample > 0 ? n / kSample : 1;
  for (uint64_t i = 0; i < kSample; ++i) {
    const uint64_t idx = i * stride;
    if (idx >= n) break;
    ++hist[s[idx * w + w - 1]];
  }
  int order[256];
  for (int v = 0; v < 256; ++v) order[v] = v;
  std::stable_sort(order, order + 256, [&](int a, int b) { return hist[a] > hist[b]; });
  int k = 0;
  for (; k < 15 && hist[order[k]] > 0; ++k) p->dict[k] = uint8_t(order[k]);
  p->nsel = k;
  std::memset(p->code_of, kEsc, 256);
  for (int j = 0; j < k; ++j) p->code_of[p->dict[j]] = uint8_t(j);
  uint64_t esc = 0;
  for (uint64_t e = 0; e < n; ++e) esc += p->code_of[s[e * w + w - 1]] == kEsc;
  const uint64_t coded = kFrameHeader + (n + 1) / 2 + uint64_t(w - 1) * n + esc + (len - n * w);
  const uint64_t raw = kFrameHeader + len;
  if (n > 0 && esc <= kMaxEsc && coded < raw) {
    p->mode = 1;
    p->n_esc = uint32_t(esc);
    p->size = align16(coded);
  } else {
    p->mode = 0;
    p->n_esc = 0;
    p->nsel = 0;
    std::memset(p->dict, 0, 16);
    p->size = align16(raw);
  }
}

void encode_frame(const uint8_t* s, uint64_t len, int w, const Plan& p, uint8_t* fr) {
  std::memset(fr, 0, kFrameHeader);
  fr[0] = p.mode;
  std::memcpy(fr + 4, &p.n_esc, 4);
  std::memcpy(fr + 8, p.dict, 16);
  uint8_t* body = fr + kFrameHeader;
  const uint64_t body_cap = p.size - kFrameHeader;
  if (p.mode == 0) {
    std::memcpy(body, s, len);
    std::memset(body + len, 0, body_cap - len);
    return;
  }
  const uint64_t n = len / w;
  const uint64_t nb = (n + 1) / 2;
  uint8_t* nib = body;
  uint8_t* lo = body + nb;
  uint8_t* esc = lo + uint64_t(w - 1) * n;
  uint32_t ne = 0;
  for (uint64_t pr = 0; pr < nb; ++pr) {
    uint8_t byte = 0;
    for (int h = 0; h < 2; ++h) {
      const uint64_t e = 2 * pr + h;
      if (e >= n) break;
      const uint8_t* el = s + e * w;
      const uint8_t c = p.code_of[el[w - 1]];
      byte |= uint8_t(c << (4 * h));
      if (c == kEsc) esc[ne++] = el[w - 1];
    }
    nib[pr] = byte;
  }
  if (w == 2) {
    for (uint64_t e = 0; e < n; ++e) lo[e] = s[2 * e];
  } else {
    for (uint64_t e = 0; e < n; ++e) std::memcpy(lo + e * (w - 1), s + e * w, w - 1);
  }
  uint8_t* tail = esc + ne;
  const uint64_t tail_len = len - n * w;
  std::memcpy(tail, s + n * w, tail_len);
  const uint64_t used = uint64_t(tail - body) + tail_len;
  std::memset(body + used, 0, body_cap - used);
}

void decode_frame(const uint8_t* fr, uint64_t len, int w, uint8_t* o) {
  const uint8_t* body = fr + kFrameHeader;
  if (fr[0] == 0) {
    std::memcpy(o, body, len);
    return;
  }
  uint32_t n_esc;
  std::memcpy(&n_esc, fr + 4, 4);
  const uint8_t* dict = fr + 8;
  const uint64_t n = len / w;
  const uint64_t nb = (n + 1) / 2;
  const uint8_t* nib = body;
  const uint8_t* lo = body + nb;
  const uint8_t* esc = lo + uint64_t(w - 1) * n;
  uint32_t ne = 0;
  for (uint64_t e = 0; e < n; ++e) {
    const uint8_t c = (nib[e >> 1] >> (4 * (e & 1))) & 15;
    uint8_t hi;
    if (c == kEsc) hi = ne < n_esc ? esc[ne++] : 0;
    else hi = dict[c];
    uint8_t* d = o + e * w;
    if (w == 2) {
      d[0] = lo[e];
    } else {
      std::memcpy(d, lo + e * (w - 1), w - 1);
    }
    d[w - 1] = hi;
  }
  std::memcpy(o + n * w, esc + n_esc, len - n * w);
}

template <typename F>
void parallel_frames(uint32_t nf, int nthreads, F fn) {
  nthreads = std::max(1, std::min<int>(nthreads, int(nf)));
  if (nthreads == 1) {
    for (uint32_t f = 0; f < nf; ++f) fn(f);
    return;
  }
  std::atomic<uint32_t> next{0};
  std::vector<std::thread> ts;
  for (int t = 0; t < nthreads; ++t)
    ts.emplace_back([&] {
      for (uint32_t f; (f = next.fetch_add(1)) < nf;) fn(f);
    });
  for (auto& t : ts) t.join();
}

}  // namespace

extern "C" {

uint64_t hsz_max_encoded_bytes(uint64_t logical, uint32_t frame_bytes) {
  const uint64_t nf = logical ? (logical + frame_bytes - 1) / frame_bytes : 1;
  return align16(kHeader + 8 * (nf + 1)) + nf * align16(kFrameHeader + frame_bytes);
}

// Returns the encoded size (out must hold hsz_max_encoded_bytes), or < 0.
int64_t hsz_encode_cpu(const void* src, uint64_t logical, int w, uint32_t frame_bytes,
                       void* out, int nthreads) {
  if (w < 1 || w > 8 || frame_bytes % 16 || frame_bytes % w) return -22;
  const auto* s = static_cast<const uint8_t*>(src);
  auto* o = static_cast<uint8_t*>(out);
  const uint32_t nf = logical ? uint32_t((logical + frame_bytes - 1) / frame_bytes) : 1;
  std::vector<Plan> plans(nf);
  auto flen = [&](uint32_t f) {
    const uint64_t lo = uint64_t(f) * frame_bytes;
    return std::min<uint64_t>(frame_bytes, logical - lo);
  };
  parallel_frames(nf, nthreads, [&](uint32_t f) {
    plan_frame(s + uint64_t(f) * frame_bytes, flen(f), w, &plans[f]);
  });
  std::vector<uint64_t> offs(nf + 1);
  const uint64_t start = align16(kHeader + 8 * (uint64_t(nf) + 1));
  offs[0] = start;
  for (uint32_t f = 0; f < nf; ++f) offs[f + 1] = offs[f] + plans[f].size;
  std::memset(o, 0, start);
  std::memcpy(o, "HSZ1", 4);
  const uint32_t ver = 1;
  std::memcpy(o + 4, &ver, 4);
  std::memcpy(o + 8, &logical, 8);
  const uint32_t w32 = uint32_t(w);
  std::memcpy(o + 16, &w32, 4);
  std::memcpy(o + 20, &frame_bytes, 4);
  std::memcpy(o + 24, &nf, 4);
  std::memcpy(o + kHeader, offs.data(), 8 * (nf + 1));
  parallel_frames(nf, nthreads, [&](uint32_t f) {
    encode_frame(s + uint64_t(f) * frame_bytes, flen(f), w, plans[f], o + offs[f]);
  });
  return int64_t(offs[nf]);
}

// Decode frames [first, first+count) of a blob whose frame bytes start at
// `frames`; offsets[i] = byte offset of frame first+i relative to `frames`.
// Output = the logical bytes of those frames.  Returns 0 or < 0.
int hsz_decode_cpu(const void* frames, const uint64_t* offsets, uint32_t first, uint32_t count,
                   uint64_t logical, int w, uint32_t frame_bytes, void* out, int nthreads) {
  if (w < 1 || w > 8) return -22;
  const auto* fr = static_cast<const uint8_t*>(frames);
  auto* o = static_cast<uint8_t*>(out);
  parallel_frames(count, nthreads, [&](uint32_t i) {
    const uint64_t f = uint64_t(first) + i;
    const uint64_t lo = f * frame_bytes;
    const uint64_t len = std::min<uint64_t>(frame_bytes, logical - lo);
    decode_frame(fr + offsets[i], len, w, o + uint64_t(i) * frame_bytes);
  });
  return 0;
}

}  // extern "C"
