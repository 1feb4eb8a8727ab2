// HSZ1 CPU decoder on corrupted frames, built with -fsanitize=address,undefined
// (tests/test_native_sanitizers.py).  Each frame buffer is exactly its stored
// extent, so any read the decoder makes past it is reported.  A corrupted
// frame may decode to wrong bytes or be rejected (-74); nothing else.
#include "../../hipsnapshot/csrc/hsz_cpu.cpp"

#include <cstdio>
#include <random>

int main() {
  std::mt19937 rng(7);
  std::normal_distribution<float> nd(0.f, 1.f / 64);
  int decoded = 0, rejected = 0, other = 0;
  for (int trial = 0; trial < 3000; ++trial) {
    const int w = (trial & 1) ? 4 : 2;
    const uint64_t len = (trial % 7 == 0) ? 32003 : 65536;  // with / without a tail
    std::vector<uint8_t> src(len);
    for (uint64_t i = 0; i + 4 <= len; i += 4) {
      const float f = nd(rng);
      std::memcpy(&src[i], &f, 4);
    }
    Plan p;
    plan_frame(src.data(), len, w, &p);
    std::vector<uint8_t> fr(p.size);
    encode_frame(src.data(), len, w, p, fr.data());
    if (trial % 10 == 0) {  // clean frames must round-trip
      std::vector<uint8_t> out(len);
      if (decode_frame(fr.data(), fr.size(), len, w, out.data()) != 0 || out != src) {
        std::printf("clean frame %d did not round-trip\n", trial);
        return 1;
      }
    }
    for (int k = 0; k < 1 + trial % 8; ++k) fr[rng() % fr.size()] ^= uint8_t(1u << (rng() % 8));
    std::vector<uint8_t> out(len);
    const int r = decode_frame(fr.data(), fr.size(), len, w, out.data());
    if (r == 0) ++decoded;
    else if (r == -74) ++rejected;
    else ++other;
  }
  std::printf("decoded %d rejected %d other %d\n", decoded, rejected, other);
  if (other) return 1;
  std::printf("ok\n");
  return 0;
}
