// Stress driver for the native I/O engine, built with ASan/UBSan and TSan
// (tests/test_native_sanitizers.py).  Many threads submit writes/reads/deletes
// concurrently while another thread polls completions through the eventfd.
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <poll.h>
#include <string>
#include <thread>
#include <vector>

extern "C" {
void* hsio_create(int);
void hsio_destroy(void*);
int hsio_eventfd(void*);
int64_t hsio_submit_write(void*, const char*, const void*, uint64_t, uint64_t, int);
int64_t hsio_submit_read(void*, const char*, void*, uint64_t, uint64_t, int);
int hsio_poll(void*, int64_t*, int64_t*, int);
int64_t hsio_write_sync(void*, const char*, const void*, uint64_t, uint64_t, int);
int64_t hsio_read_sync(void*, const char*, void*, uint64_t, uint64_t, int);
void hsio_parallel_memcpy(void*, const void*, uint64_t, int);
void hsio_set_read_split(void*, uint64_t);
uint64_t hsz_max_encoded_bytes(uint64_t, uint32_t);
int64_t hsz_encode_cpu(const void*, uint64_t, int, uint32_t, void*, int);
int hsz_decode_cpu(const void*, const uint64_t*, uint32_t, uint32_t, uint64_t, int, uint32_t,
                   void*, int);
}

int main(int argc, char** argv) {
  const std::string dir = argc > 1 ? argv[1] : "/tmp/hsio_stress";
  void* eng = hsio_create(8);
  const int kFiles = 64;
  std::vector<std::vector<char>> bufs(kFiles);
  for (int i = 0; i < kFiles; ++i) {
    bufs[i].resize(4096 * (i + 1) + i);
    for (size_t j = 0; j < bufs[i].size(); ++j) bufs[i][j] = char((i * 31 + j) & 0xff);
  }
  std::atomic<int> submitted{0};
  std::vector<std::thread> producers;
  for (int t = 0; t < 4; ++t) {
    producers.emplace_back([&, t] {
      for (int i = t; i < kFiles; i += 4) {
        std::string p = dir + "/d" + std::to_string(i % 5) + "/f" + std::to_string(i);
        hsio_submit_write(eng, p.c_str(), bufs[i].data(), bufs[i].size(), 0, 4 | (i % 2));
        submitted.fetch_add(1);
      }
    });
  }
  int done = 0;
  int64_t ids[64], res[64];
  pollfd pfd{hsio_eventfd(eng), POLLIN, 0};
  while (done < kFiles) {
    poll(&pfd, 1, 100);
    int k = hsio_poll(eng, ids, res, 64);
    for (int j = 0; j < k; ++j) {
      if (res[j] < 0) { std::fprintf(stderr, "write failed %lld\n", (long long)res[j]); return 1; }
    }
    done += k;
  }
  for (auto& th : producers) th.join();
  for (int i = 0; i < kFiles; ++i) {
    std::string p = dir + "/d" + std::to_string(i % 5) + "/f" + std::to_string(i);
    std::vector<char> back(bufs[i].size());
    int64_t r = hsio_read_sync(eng, p.c_str(), back.data(), back.size(), 0, 0);
    if (r != (int64_t)back.size() || std::memcmp(back.data(), bufs[i].data(), back.size())) {
      std::fprintf(stderr, "mismatch in file %d\n", i);
      return 1;
    }
  }
  // split reads: every file read back asynchronously in 4 KiB parts, all in
  // flight at once (groups complete out of order on 8 workers)
  hsio_set_read_split(eng, 4096);
  std::vector<std::vector<char>> backs(kFiles);
  std::vector<int64_t> rid(kFiles);
  for (int i = 0; i < kFiles; ++i) {
    std::string p = dir + "/d" + std::to_string(i % 5) + "/f" + std::to_string(i);
    backs[i].assign(bufs[i].size(), 0);
    rid[i] = hsio_submit_read(eng, p.c_str(), backs[i].data(), backs[i].size(), 0, 0);
  }
  done = 0;
  while (done < kFiles) {
    poll(&pfd, 1, 100);
    int k = hsio_poll(eng, ids, res, 64);
    for (int j = 0; j < k; ++j) {
      int i = 0;
      while (rid[i] != ids[j]) ++i;
      if (res[j] != (int64_t)bufs[i].size()) { std::fprintf(stderr, "split read %d: %lld\n", i, (long long)res[j]); return 1; }
    }
    done += k;
  }
  for (int i = 0; i < kFiles; ++i)
    if (std::memcmp(backs[i].data(), bufs[i].data(), bufs[i].size())) { std::fprintf(stderr, "split mismatch %d\n", i); return 1; }
  // HSZ1 codec round trip, multi-threaded, odd length + all element widths
  for (int w : {1, 2, 4, 8}) {
    const uint64_t n = (3u << 20) + 13;
    std::vector<uint8_t> src(n);
    uint32_t x = 12345;
    for (uint64_t i = 0; i < n; ++i) {
      x = x * 1103515245u + 12345u;
      src[i] = (i % w == uint64_t(w - 1)) ? uint8_t(60 + ((x >> 16) % 5)) : uint8_t(x >> 24);
    }
    std::vector<uint8_t> enc(hsz_max_encoded_bytes(n, 65536));
    int64_t sz = hsz_encode_cpu(src.data(), n, w, 65536, enc.data(), 8);
    if (sz <= 0 || uint64_t(sz) > enc.size()) { std::fprintf(stderr, "encode w=%d: %lld\n", w, (long long)sz); return 1; }
    uint32_t nf;
    std::memcpy(&nf, enc.data() + 24, 4);
    std::vector<uint64_t> offs(nf + 1);
    std::memcpy(offs.data(), enc.data() + 64, 8 * (nf + 1));
    std::vector<uint8_t> dec(n);
    if (hsz_decode_cpu(enc.data(), offs.data(), 0, nf, n, w, 65536, dec.data(), 8) != 0 ||
        std::memcmp(dec.data(), src.data(), n)) { std::fprintf(stderr, "decode w=%d\n", w); return 1; }
  }
  std::vector<char> a(64 << 20, 7), b(64 << 20, 0);
  hsio_parallel_memcpy(b.data(), a.data(), a.size(), 8);
  if (std::memcmp(a.data(), b.data(), a.size())) return 1;
  hsio_destroy(eng);
  std::puts("ok");
  return 0;
}
