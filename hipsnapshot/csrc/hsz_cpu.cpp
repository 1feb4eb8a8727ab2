// HSZ1 codec on the host (format: hipsnapshot/ops/codec.py; GPU: hsz.hip).
//
// Used for CPU tensors on save and for CPU destinations on restore.  Frames
// are independent, so a blob is split across threads by frame; within a frame
// the loops are plain byte loops the compiler vectorises.  Mode 2 (Huffman
// coded indices, 2-byte elements) follows the NumPy reference bit for bit:
// same code-length construction, same 256-lane stream split.

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

namespace {

constexpr int kSample = 2048;
constexpr int kRun = 32;
constexpr uint32_t kMaxEsc = 1024;
constexpr uint64_t kHeader = 64;
constexpr uint64_t kFrameHeader = 32;
constexpr uint8_t kEsc = 15;
constexpr int kLanes = 256;
constexpr uint64_t kLaneTable = 2 * kLanes;
constexpr int kMaxLen = 11;
constexpr uint64_t kMaxCoded = 65535;

inline uint64_t align16(uint64_t n) { return (n + 15) & ~uint64_t(15); }

// Code lengths of the 16 indices (mirror of codec.huffman_lengths).
void huffman_lengths(const uint64_t cnt[16], uint8_t lens[16]) {
  std::memset(lens, 0, 16);
  int k = 0;
  for (int c = 0; c < 16; ++c) k += cnt[c] != 0;
  if (k == 0) return;
  if (k == 1) {
    for (int c = 0; c < 16; ++c)
      if (cnt[c]) lens[c] = 1;
    return;
  }
  // nodes 0..15 are the leaves (dead when unused), merged nodes from 16 on:
  // the same relative order as the reference's numbering, so ties agree
  uint64_t w[32];
  int par[32];  // -1 live root, -2 unused leaf, >= 0 parent
  for (int c = 0; c < 16; ++c) {
    w[c] = cnt[c];
    par[c] = cnt[c] ? -1 : -2;
  }
  int m = 16;
  for (int step = 0; step < k - 1; ++step) {
    int a = -1, b = -1;
    for (int i = 0; i < m; ++i)
      if (par[i] == -1 && (a < 0 || w[i] < w[a])) a = i;
    par[a] = -3;
    for (int i = 0; i < m; ++i)
      if (par[i] == -1 && (b < 0 || w[i] < w[b])) b = i;
    w[m] = w[a] + w[b];
    par[m] = -1;
    par[a] = m;
    par[b] = m;
    ++m;
  }
  int maxl = 0;
  for (int c = 0; c < 16; ++c) {
    if (!cnt[c]) continue;
    int d = 0;
    for (int j = c; par[j] >= 0; j = par[j]) ++d;
    lens[c] = uint8_t(d);
    maxl = std::max(maxl, d);
  }
  if (maxl <= kMaxLen) return;
  for (int c = 0; c < 16; ++c)
    if (lens[c] > kMaxLen) lens[c] = kMaxLen;
  for (;;) {
    uint32_t kraft = 0;
    for (int c = 0; c < 16; ++c)
      if (cnt[c]) kraft += 1u << (kMaxLen - lens[c]);
    if (kraft <= (1u << kMaxLen)) break;
    int s = -1;
    for (int c = 0; c < 16; ++c) {
      if (!cnt[c] || lens[c] >= kMaxLen) continue;
      if (s < 0 || lens[c] > lens[s] || (lens[c] == lens[s] && cnt[c] <= cnt[s])) s = c;
    }
    ++lens[s];
  }
}

// Bit-reversed canonical codewords (mirror of codec.canonical_codes).
void canonical_codes(const uint8_t lens[16], uint16_t codes[16]) {
  std::memset(codes, 0, 16 * sizeof(uint16_t));
  uint32_t code = 0;
  int prev = 0;
  bool first = true;
  for (int l = 1; l <= kMaxLen; ++l)
    for (int c = 0; c < 16; ++c) {
      if (lens[c] != l) continue;
      if (!first) code = (code + 1) << (l - prev);
      first = false;
      prev = l;
      uint32_t rev = 0;
      for (int b = 0; b < l; ++b) rev |= ((code >> b) & 1u) << (l - 1 - b);
      codes[c] = uint16_t(rev);
    }
}

struct Plan {
  uint8_t mode = 0;
  uint32_t n_esc = 0;
  int nsel = 0;
  uint8_t dict[16] = {0};
  uint8_t code_of[256];
  uint8_t lens[16] = {0};
  uint16_t lane_bytes[kLanes] = {0};
  uint64_t coded = 0;  // mode 2 stream bytes
  uint64_t size = 0;
};

void plan_frame(const uint8_t* s, uint64_t len, int w, Plan* p) {
  const uint64_t n = len / w;
  uint32_t hist[256] = {0};
  // sample: every element up to kSample, else kSample / kRun runs of kRun
  // consecutive elements evenly spread over the frame (codec.sample_indices)
  if (n <= uint64_t(kSample)) {
    for (uint64_t i = 0; i < n; ++i) ++hist[s[i * w + w - 1]];
  } else {
    const uint64_t step = n / (kSample / kRun);
    for (uint64_t i = 0; i < uint64_t(kSample); ++i) {
      const uint64_t idx = (i / kRun) * step + i % kRun;
      ++hist[s[idx * w + w - 1]];
    }
  }
  int order[256];
  for (int v = 0; v < 256; ++v) order[v] = v;
  std::stable_sort(order, order + 256, [&](int a, int b) { return hist[a] > hist[b]; });
  int k = 0;
  for (; k < 15 && hist[order[k]] > 0; ++k) p->dict[k] = uint8_t(order[k]);
  p->nsel = k;
  std::memset(p->code_of, kEsc, 256);
  for (int j = 0; j < k; ++j) p->code_of[p->dict[j]] = uint8_t(j);
  const bool m2 = (w == 2 || w == 4) && n > 0 && n % 8 == 0;
  uint64_t esc = 0;
  std::vector<uint32_t> lane_cnt;  // [lane][16]
  uint64_t cnt[16] = {0};
  if (m2) {
    lane_cnt.assign(size_t(kLanes) * 16, 0);
    for (uint64_t e = 0; e < n; ++e) {
      const uint8_t c = p->code_of[s[e * w + w - 1]];
      ++lane_cnt[((e >> 3) & (kLanes - 1)) * 16 + c];
    }
    for (int l = 0; l < kLanes; ++l)
      for (int c = 0; c < 16; ++c) cnt[c] += lane_cnt[size_t(l) * 16 + c];
    esc = cnt[kEsc];
  } else {
    for (uint64_t e = 0; e < n; ++e) esc += p->code_of[s[e * w + w - 1]] == kEsc;
  }
  const uint64_t tail = len - n * w;
  const uint64_t coded1 = kFrameHeader + (n + 1) / 2 + uint64_t(w - 1) * n + esc + tail;
  const uint64_t raw = kFrameHeader + len;
  p->mode = 0;
  if (n > 0 && esc <= kMaxEsc) {
    if (m2) {
      huffman_lengths(cnt, p->lens);
      uint64_t c_bytes = 0;
      for (int l = 0; l < kLanes; ++l) {
        uint64_t bits = 0;
        for (int c = 0; c < 16; ++c) bits += uint64_t(lane_cnt[size_t(l) * 16 + c]) * p->lens[c];
        const uint64_t b = (bits + 7) / 8;
        p->lane_bytes[l] = uint16_t(std::min<uint64_t>(b, 65535));
        c_bytes += b;
      }
      const uint64_t size2 = kFrameHeader + uint64_t(w - 1) * n + kLaneTable + c_bytes + esc + tail;
      if (c_bytes <= kMaxCoded && size2 < coded1 && size2 < raw) {
        p->mode = 2;
        p->coded = c_bytes;
        p->size = align16(size2);
      }
    }
    if (p->mode == 0 && coded1 < raw) {
      p->mode = 1;
      p->size = align16(coded1);
    }
  }
  if (p->mode == 0) {
    p->n_esc = 0;
    p->nsel = 0;
    std::memset(p->dict, 0, 16);
    p->size = align16(raw);
  } else {
    p->n_esc = uint32_t(esc);
  }
  if (p->mode != 2) std::memset(p->lens, 0, 16);
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
  uint8_t* esc;
  uint32_t ne = 0;
  if (p.mode == 2) {
    for (int j = 0; j < 8; ++j) fr[24 + j] = uint8_t(p.lens[2 * j] | (p.lens[2 * j + 1] << 4));
    uint16_t codes[16];
    canonical_codes(p.lens, codes);
    uint8_t* lo = body;
    if (w == 2) {
      for (uint64_t e = 0; e < n; ++e) lo[e] = s[2 * e];
    } else {
      for (uint64_t e = 0; e < n; ++e) std::memcpy(lo + e * (w - 1), s + e * w, w - 1);
    }
    uint8_t* table = body + uint64_t(w - 1) * n;
    std::memcpy(table, p.lane_bytes, kLaneTable);  // little-endian host
    uint8_t* streams = table + kLaneTable;
    const uint64_t groups = n / 8;
    uint32_t enc[256];  // high byte -> codeword | length << 16 (one lookup per element)
    for (int v = 0; v < 256; ++v) {
      const uint8_t c = p.code_of[v];
      enc[v] = uint32_t(codes[c]) | (uint32_t(p.lens[c]) << 16);
    }
    uint64_t pos = 0;
    for (int l = 0; l < kLanes; ++l) {
      // whole 32-bit words of the lane's stream are stored as they fill
      // (LSB-first, so the bytes equal a byte-at-a-time emission); after two
      // codes at most 31 + 22 bits are pending
      uint64_t acc = 0;
      int nb = 0;
      for (uint64_t g = uint64_t(l); g < groups; g += kLanes) {
        const uint8_t* hi = s + 8 * g * w + (w - 1);
        for (int e = 0; e < 8; e += 2) {
          const uint32_t t0 = enc[hi[e * w]], t1 = enc[hi[(e + 1) * w]];
          acc |= uint64_t(t0 & 0xffff) << nb;
          nb += int(t0 >> 16);
          acc |= uint64_t(t1 & 0xffff) << nb;
          nb += int(t1 >> 16);
          if (nb >= 32) {
            const uint32_t word = uint32_t(acc);
            std::memcpy(streams + pos, &word, 4);  // little-endian host
            pos += 4;
            acc >>= 32;
            nb -= 32;
          }
        }
      }
      for (; nb > 0; nb -= 8) {
        streams[pos++] = uint8_t(acc);
        acc >>= 8;
      }
    }
    esc = streams + p.coded;
    if (p.n_esc)
      for (uint64_t e = 0; e < n; ++e)
        if (p.code_of[s[e * w + w - 1]] == kEsc) esc[ne++] = s[e * w + w - 1];
  } else {
    const uint64_t nb = (n + 1) / 2;
    uint8_t* nib = body;
    uint8_t* lo = body + nb;
    esc = lo + uint64_t(w - 1) * n;
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
  }
  uint8_t* tail = esc + ne;
  const uint64_t tail_len = len - n * w;
  std::memcpy(tail, s + n * w, tail_len);
  const uint64_t used = uint64_t(tail - body) + tail_len;
  std::memset(body + used, 0, body_cap - used);
}

// Mode-2 frame body -> logical bytes.  `extent` = the frame's stored size.
int decode_frame2(const uint8_t* fr, uint64_t extent, uint64_t len, int w, uint8_t* o) {
  uint32_t n_esc;
  std::memcpy(&n_esc, fr + 4, 4);
  const uint8_t* dict = fr + 8;
  uint8_t lens[16];
  for (int c = 0; c < 16; ++c) lens[c] = (fr[24 + c / 2] >> (4 * (c & 1))) & 15;
  for (int c = 0; c < 16; ++c)
    if (lens[c] > kMaxLen) return -74;
  const uint64_t n = len / w;
  const uint64_t nlo = uint64_t(w - 1) * n;
  if (n % 8 || n_esc > kMaxEsc) return -74;
  const uint8_t* body = fr + kFrameHeader;
  if (kFrameHeader + nlo + kLaneTable > extent) return -74;
  const uint8_t* lo = body;
  uint16_t lane_bytes[kLanes];
  std::memcpy(lane_bytes, body + nlo, kLaneTable);
  uint64_t c_bytes = 0;
  for (int l = 0; l < kLanes; ++l) c_bytes += lane_bytes[l];
  const uint64_t tail = len - n * w;
  if (kFrameHeader + nlo + kLaneTable + c_bytes + n_esc + tail > extent) return -74;
  const uint8_t* streams = body + nlo + kLaneTable;
  const uint8_t* escv = streams + c_bytes;
  uint16_t codes[16];
  canonical_codes(lens, codes);
  uint16_t lut[1 << kMaxLen];
  std::memset(lut, 0, sizeof(lut));
  for (int c = 0; c < 16; ++c) {  // code c fills every entry whose low lens[c] bits are its code
    if (!lens[c]) continue;
    const uint16_t ent = uint16_t(c | (lens[c] << 8));
    for (uint32_t k = 0; k < (1u << (kMaxLen - lens[c])); ++k) lut[codes[c] | (k << lens[c])] = ent;
  }
  std::vector<uint8_t> idx(n);
  const uint64_t groups = n / 8;
  // bytes readable from `streams` on: the rest of the frame's stored extent
  const uint64_t avail = extent - (kFrameHeader + nlo + kLaneTable);
  const uint64_t full = groups / kLanes;  // rounds every lane has
  const uint64_t extra = groups % kLanes;  // lanes l < extra have one more group
  constexpr uint32_t kMask = (1u << kMaxLen) - 1;
  // One code of lane k: refill to 56..63 bits (an 8-byte load while the
  // frame has 8 bytes left; the byte at `pos` always belongs at bit `nb`, so
  // the bits above `nb` are stream data, not zeros; refills may read past the
  // lane's own stream, which the per-lane check below bounds), LUT lookup,
  // consume.
#define HSZ_DECODE_ONE(k, dst)                                                      \
  do {                                                                              \
    if (pos[k] + 8 <= avail) {                                                      \
      /* unconditional: re-OR-ing bits already held is harmless, and it */          \
      /* avoids a data-dependent branch per code */                                 \
      uint64_t v;                                                                   \
      std::memcpy(&v, streams + pos[k], 8);                                         \
      acc[k] |= v << nb[k];                                                         \
      pos[k] += (63 - nb[k]) >> 3;                                                  \
      nb[k] |= 56;                                                                  \
    } else {                                                                        \
      for (; nb[k] <= 56 && pos[k] < avail; nb[k] += 8)                             \
        acc[k] |= uint64_t(streams[pos[k]++]) << nb[k];                             \
    }                                                                               \
    const uint16_t ent = lut[acc[k] & kMask];                                       \
    const int ln = ent >> 8;                                                        \
    if (ln == 0 || ln > nb[k]) return -74;                                          \
    acc[k] >>= ln;                                                                  \
    nb[k] -= ln;                                                                    \
    (dst) = uint8_t(ent & 15);                                                      \
  } while (0)
  // Lanes are independent streams: decode 4 side by side so the out-of-order
  // core overlaps their serial refill -> lookup -> shift chains (measured
  // single-thread: 0.29 GB/s one lane at a time).
  constexpr int kIlv = 4;
  uint64_t lane_start = 0;
  for (int l0 = 0; l0 < kLanes; l0 += kIlv) {
    uint64_t pos[kIlv], acc[kIlv], st[kIlv];
    int nb[kIlv];
#pragma GCC unroll 4
    for (int k = 0; k < kIlv; ++k) {
      st[k] = pos[k] = lane_start;
      lane_start += lane_bytes[l0 + k];
      acc[k] = 0;
      nb[k] = 0;
    }
    for (uint64_t j = 0; j < full; ++j) {
      uint8_t* base = idx.data() + 8 * (uint64_t(l0) + j * kLanes);
      for (int e = 0; e < 8; ++e) {
        HSZ_DECODE_ONE(0, base[e]);
        HSZ_DECODE_ONE(1, base[8 + e]);
        HSZ_DECODE_ONE(2, base[16 + e]);
        HSZ_DECODE_ONE(3, base[24 + e]);
      }
    }
    // the ragged last round, then: the lane's codes must lie inside its own
    // stream (constant indices only, so the lane state stays in registers)
#define HSZ_LANE_END(k)                                                              \
  do {                                                                              \
    if (uint64_t(l0 + k) < extra) {                                                 \
      uint8_t* base = idx.data() + 8 * (uint64_t(l0 + k) + full * kLanes);          \
      for (int e = 0; e < 8; ++e) HSZ_DECODE_ONE(k, base[e]);                       \
    }                                                                               \
    if ((pos[k] - st[k]) * 8 - uint64_t(nb[k]) > uint64_t(lane_bytes[l0 + k]) * 8)  \
      return -74;                                                                   \
  } while (0)
    HSZ_LANE_END(0);
    HSZ_LANE_END(1);
    HSZ_LANE_END(2);
    HSZ_LANE_END(3);
#undef HSZ_LANE_END
  }
#undef HSZ_DECODE_ONE
  uint32_t ne = 0;
  for (uint64_t e = 0; e < n; ++e) {
    const uint8_t c = idx[e];
    uint8_t* d = o + e * w;
    if (w == 2) {
      d[0] = lo[e];
    } else {
      std::memcpy(d, lo + e * (w - 1), w - 1);
    }
    d[w - 1] = c == kEsc ? (ne < n_esc ? escv[ne++] : 0) : dict[c];
  }
  if (tail) std::memcpy(o + n * w, escv + n_esc, tail);
  return 0;
}

int decode_frame(const uint8_t* fr, uint64_t extent, uint64_t len, int w, uint8_t* o) {
  const uint8_t* body = fr + kFrameHeader;
  if (fr[0] == 0) {
    if (kFrameHeader + len > extent) return -74;
    std::memcpy(o, body, len);
    return 0;
  }
  if (fr[0] == 2) return w == 2 || w == 4 ? decode_frame2(fr, extent, len, w, o) : -74;
  if (fr[0] != 1) return -74;
  uint32_t n_esc;
  std::memcpy(&n_esc, fr + 4, 4);
  const uint8_t* dict = fr + 8;
  const uint64_t n = len / w;
  const uint64_t nb = (n + 1) / 2;
  if (kFrameHeader + nb + uint64_t(w - 1) * n + uint64_t(n_esc) + (len - n * w) > extent)
    return -74;
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
  return 0;
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
  const uint32_t ver = 2;
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
// `frames`; offsets[i] (i <= count) = byte offset of frame first+i relative to
// `frames`, offsets[count] = end of the last frame.  Output = the logical
// bytes of those frames.  Returns 0, or < 0 for a corrupt frame.
int hsz_decode_cpu(const void* frames, const uint64_t* offsets, uint32_t first, uint32_t count,
                   uint64_t logical, int w, uint32_t frame_bytes, void* out, int nthreads) {
  if (w < 1 || w > 8) return -22;
  const auto* fr = static_cast<const uint8_t*>(frames);
  auto* o = static_cast<uint8_t*>(out);
  std::atomic<int> err{0};
  parallel_frames(count, nthreads, [&](uint32_t i) {
    const uint64_t f = uint64_t(first) + i;
    const uint64_t lo = f * frame_bytes;
    const uint64_t len = std::min<uint64_t>(frame_bytes, logical - lo);
    if (offsets[i + 1] < offsets[i] + kFrameHeader) {
      err = -74;
      return;
    }
    const int r = decode_frame(fr + offsets[i], offsets[i + 1] - offsets[i], len, w,
                               o + uint64_t(i) * frame_bytes);
    if (r) err = r;
  });
  return err.load();
}

}  // extern "C"
