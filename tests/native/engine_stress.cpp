// Stress driver of the native restore and drain engines on the CPU device
// stubs (engine_stubs.cpp), built by tests/test_native_sanitizers.py with
// -fsanitize=thread and with -fsanitize=address,undefined.
//
//   engine_stress restore <dir> <rounds>  random restore plans: raw blobs read
//       with a prefix (slab members), HSZ1 blobs decoded straight into their
//       destination or into scratch and copied out, budgets below one blob
//       (pool blocks), 2..6 slots, 1..8 readers; every 4th round injects a
//       failure (upload error, missing file, short file, corrupt HSZ1 header,
//       no device memory) that must end the job with an error, not a hang
//   engine_stress drain <dir> <rounds>    random drains: empty / small / multi-
//       slot blobs, 2..8 slots, 1..6 writers plus parked ones boosted from
//       another thread, buffered or O_DIRECT; injected copy failures and
//       unwritable paths
//   engine_stress ringwrap <dir>          the c026ee7 case: a blob longer than
//       both free ends of an emptied upload ring (waited forever before the
//       ring restarted at offset 0)
//   engine_stress restore-trim <dir> <rounds>  three restore loops at once
//       on the shared device pools while a fourth thread frees every idle
//       pool block again and again (release_restore_memory() from another
//       thread, and the round-5 trim-to-0 after every job): every byte must
//       arrive, and no freed block may be touched again (the stubs retire a
//       freed block's addresses, so a late use faults)
//
// Prints "ok" and exits 0 when every check held.

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "engine_stubs.h"

using stub::StubDesc;

namespace {

uint64_t seed0() { return getenv("STRESS_SEED") ? strtoull(getenv("STRESS_SEED"), nullptr, 10) : 12345; }

// per thread (restore-trim runs several restore loops at once)
thread_local std::mt19937_64 rng(seed0());

uint64_t rnd(uint64_t lo, uint64_t hi) {  // [lo, hi]
  return lo + rng() % (hi - lo + 1);
}

#define CHECK(cond, ...)                                   \
  do {                                                     \
    if (!(cond)) {                                         \
      fprintf(stderr, "CHECK failed %s:%d: %s: ", __FILE__, __LINE__, #cond); \
      fprintf(stderr, __VA_ARGS__);                        \
      fprintf(stderr, "\n");                               \
      exit(1);                                             \
    }                                                      \
  } while (0)

std::vector<uint8_t> random_bytes(uint64_t n) {
  std::vector<uint8_t> v(n);
  for (uint64_t i = 0; i < n; ++i) v[i] = uint8_t(rng() >> 13);
  return v;
}

void write_file(const std::string& path, const std::vector<uint8_t>& data) {
  FILE* f = fopen(path.c_str(), "wb");
  CHECK(f, "open %s", path.c_str());
  if (!data.empty())
    CHECK(fwrite(data.data(), 1, data.size(), f) == data.size(), "write %s", path.c_str());
  fclose(f);
}

uint64_t align16(uint64_t n) { return (n + 15) & ~uint64_t(15); }

// a stub HSZ1 blob: header, frame offsets, frames of (32-byte header, logical bytes)
std::vector<uint8_t> hsz_blob(const std::vector<uint8_t>& logical, uint32_t fb) {
  const uint64_t L = logical.size();
  const uint32_t nf = uint32_t(std::max<uint64_t>(1, (L + fb - 1) / fb));
  std::vector<uint64_t> offs(nf + 1);
  offs[0] = 64 + 8 * (uint64_t(nf) + 1);
  for (uint32_t f = 0; f < nf; ++f) {
    const uint64_t len = std::min<uint64_t>(fb, L - std::min<uint64_t>(uint64_t(f) * fb, L));
    offs[f + 1] = offs[f] + align16(32 + len);
  }
  std::vector<uint8_t> b(offs[nf], 0);
  memcpy(b.data(), "HSZ1", 4);
  const uint32_t version = 1, width = 2;
  memcpy(b.data() + 4, &version, 4);
  memcpy(b.data() + 8, &L, 8);
  memcpy(b.data() + 16, &width, 4);
  memcpy(b.data() + 20, &fb, 4);
  memcpy(b.data() + 24, &nf, 4);
  memcpy(b.data() + 64, offs.data(), 8 * offs.size());
  for (uint32_t f = 0; f < nf; ++f) {
    const uint64_t lo = uint64_t(f) * fb;
    const uint64_t len = std::min<uint64_t>(fb, L - std::min(lo, L));
    if (len) memcpy(b.data() + offs[f] + 32, logical.data() + lo, len);
  }
  return b;
}

struct RestorePlan {
  std::vector<std::string> paths;
  std::vector<uint64_t> lo, nb, logical, direct, base_off;
  std::vector<int> codec, dn;
  std::vector<int64_t> doff;
  std::vector<StubDesc> descs;
  std::vector<std::vector<uint8_t>> dest;      // destination buffers
  std::vector<std::vector<uint8_t>> expected;  // what they must hold
  std::vector<std::string> files;
  std::vector<std::vector<uint8_t>> file_data;
  std::vector<int> hash;                       // items hashed in the job
  int first_hsz = -1;
};

// item of `L` logical bytes; kind 0 raw, 1 HSZ1 direct, 2 HSZ1 via scratch
void add_item(RestorePlan& p, uint64_t L, int kind) {
  const int i = int(p.nb.size());
  const size_t fi = p.files.size() ? rnd(0, p.files.size() - 1) : 0;
  std::vector<uint8_t>& file = p.file_data[fi];
  file.resize(file.size() + rnd(0, 8191), 0x5a);  // gap before the blob
  std::vector<uint8_t> content = random_bytes(L);
  p.dest.emplace_back(L, 0);
  p.expected.push_back(content);
  uint8_t* dst = p.dest.back().data();
  p.paths.push_back(p.files[fi]);
  p.doff.push_back(int64_t(p.descs.size()));
  if (kind == 0) {
    const uint64_t prefix = rnd(0, 4096);
    std::vector<uint8_t> pre = random_bytes(prefix);
    p.lo.push_back(file.size());
    file.insert(file.end(), pre.begin(), pre.end());
    file.insert(file.end(), content.begin(), content.end());
    p.nb.push_back(prefix + L);
    p.codec.push_back(0);
    p.logical.push_back(0);
    p.direct.push_back(0);
    p.base_off.push_back(prefix);
  } else {
    const uint32_t fbs[] = {64u << 10, 256u << 10, 1u << 20};
    std::vector<uint8_t> blob = hsz_blob(content, fbs[rnd(0, 2)]);
    p.lo.push_back(file.size());
    file.insert(file.end(), blob.begin(), blob.end());
    p.nb.push_back(blob.size());
    p.codec.push_back(1);
    p.logical.push_back(L);
    p.direct.push_back(kind == 1 ? reinterpret_cast<uint64_t>(dst) : 0);
    p.base_off.push_back(0);
    if (p.first_hsz < 0) p.first_hsz = i;
  }
  int n = 0;
  if (kind != 1) {
    // 1..3 region copies covering the item, in random order of pieces
    const int pieces = int(rnd(1, 3));
    uint64_t cut[4] = {0, 0, 0, L};
    for (int k = 1; k < pieces; ++k) cut[k] = rnd(0, L);
    std::sort(cut, cut + pieces);
    cut[pieces] = L;
    for (int k = 0; k < pieces; ++k) {
      if (cut[k + 1] == cut[k]) continue;
      p.descs.push_back(StubDesc{cut[k], reinterpret_cast<uint64_t>(dst + cut[k]),
                                 cut[k + 1] - cut[k], 0});
      ++n;
    }
  }
  p.dn.push_back(n);
  p.hash.push_back(int(rnd(0, 2) == 0));
}

int run_restore(RestorePlan& p, uint64_t slot, uint64_t first, uint64_t piece, int nslots,
                int readers, uint64_t budget, std::string* msg) {
  for (size_t f = 0; f < p.files.size(); ++f) write_file(p.files[f], p.file_data[f]);
  const int n = int(p.nb.size());
  std::vector<const char*> cpaths;
  for (auto& s : p.paths) cpaths.push_back(s.c_str());
  std::vector<uint32_t> err_words(std::max(n, 1), 0);
  std::vector<uint64_t> sums(std::max(n, 1), 0);
  p.hash.resize(n, 0);
  std::vector<uint64_t> producers;
  for (int k = int(rnd(0, 2)); k > 0; --k) producers.push_back(reinterpret_cast<uint64_t>(stub::new_stream()));
  int err = 0;
  void* h = hsg_restore_start(0, n, cpaths.data(), p.lo.data(), p.nb.data(), p.codec.data(),
                              p.logical.data(), p.direct.data(), p.base_off.data(), p.doff.data(),
                              p.dn.data(), p.descs.data(), int64_t(p.descs.size()),
                              producers.data(), int(producers.size()), err_words.data(), slot,
                              first, piece, nslots, readers, budget, -1, p.hash.data(), 64,
                              &err);
  if (!h) {
    *msg = "start failed " + std::to_string(err);
    return -1000 + err;
  }
  int item = -1;
  char text[320];
  double stats[16];
  uint64_t nread = 0;
  const int rc = hsg_restore_wait(h, &item, text, stats, &nread, sums.data());
  *msg = text;
  for (int i = 0; rc == 0 && i < n; ++i) {
    CHECK(err_words[i] == 0, "decode flagged item %d", i);
    if (!p.hash[i]) continue;
    // the hash covers the stored bytes of the item as read from its file
    const std::vector<uint8_t>* file = nullptr;
    for (size_t f = 0; f < p.files.size(); ++f)
      if (p.files[f] == p.paths[i]) file = &p.file_data[f];
    CHECK(file, "item %d file", i);
    CHECK(sums[i] == stub::hash_bytes(file->data() + p.lo[i], p.nb[i]), "item %d hash", i);
  }
  return rc;
}

RestorePlan make_restore_plan(const std::string& dir, int round, int nitems, uint64_t max_item) {
  RestorePlan p;
  const int nfiles = std::max(1, nitems / 3);
  for (int f = 0; f < nfiles; ++f) {
    p.files.push_back(dir + "/r" + std::to_string(round) + "_f" + std::to_string(f));
    p.file_data.emplace_back();
  }
  for (int i = 0; i < nitems; ++i) {
    const uint64_t L = rng() % 4 == 0 ? rnd(1, 4096) : rnd(1, max_item);
    add_item(p, L, int(rnd(0, 9)) < 6 ? 0 : int(rnd(1, 2)));
  }
  return p;
}

void restore_mode(const std::string& dir, int rounds) {
  CHECK(hsg_restore_prewarm(0, 4 << 20, 4 << 20, 1 << 20, 3, 1 << 20) == 0, "prewarm");
  for (int r = 0; r < rounds; ++r) {
    const bool inject = r % 4 == 3;
    const int nitems = int(rnd(1, 14));
    RestorePlan p = make_restore_plan(dir, r, nitems, rng() % 3 == 0 ? (12u << 20) : (3u << 20));
    const uint64_t slot = rnd(1, 3) << 20;
    const uint64_t first = rnd(1, 2) << 20;
    const uint64_t piece = rnd(64, 1024) << 10;
    const int nslots = int(rnd(2, 6));
    const int readers = int(rnd(1, 8));
    // budgets from below one blob (pool blocks) to plenty
    const uint64_t budget = rnd(1, 24) << 20;
    int want = 0;
    if (inject) {
      switch (rnd(0, 4)) {
        case 0: {
          // the 2nd upload fails when there are two, else the only one
          uint64_t total = 0;
          for (uint64_t x : p.nb) total += x;
          stub::fail_upload_every.store(total > first ? 2 : 1);
          want = -EIO;
          break;
        }
        case 1:
          p.paths[rnd(0, p.paths.size() - 1)] = dir + "/does_not_exist";
          want = -ENOENT;
          break;
        case 2: {
          // the last item's file ends before it does
          const int i = nitems - 1;
          for (size_t f = 0; f < p.files.size(); ++f)
            if (p.files[f] == p.paths[i]) p.file_data[f].resize(p.lo[i] + p.nb[i] / 2);
          want = -ENODATA;
          break;
        }
        case 3:
          if (p.first_hsz < 0) add_item(p, rnd(1, 1 << 20), 1);
          for (size_t f = 0; f < p.files.size(); ++f)
            if (p.files[f] == p.paths[p.first_hsz]) p.file_data[f][p.lo[p.first_hsz]] ^= 0xff;
          want = -EBADMSG;
          break;
        default:
          hsg_restore_trim(-1, 0);
          stub::dev_cap.store(1 << 20);
          want = -ENOMEM;
      }
    }
    std::string msg;
    const int rc = run_restore(p, slot, first, piece, nslots, readers, budget, &msg);
    stub::fail_upload_every.store(0);
    stub::dev_cap.store(UINT64_MAX);
    CHECK(stub::pinned_live.load() == 0, "round %d: %d pinned blocks not released",
          r, stub::pinned_live.load());
    CHECK(stub::corruption.load() == 0, "round %d: a copy launch's tables were reused early", r);
    if (!inject) {
      CHECK(rc == 0, "round %d: rc %d (%s)", r, rc, msg.c_str());
      for (size_t i = 0; i < p.dest.size(); ++i)
        CHECK(p.dest[i] == p.expected[i], "round %d: item %zu restored wrong bytes", r, i);
    } else {
      // out of device memory may already fail the start (its small blocks:
      // the hash accumulators come from the 2 MiB-granule scratch pool)
      const bool nomem_at_start = want == -ENOMEM && rc == -1000 - 2;
      CHECK(rc == want || nomem_at_start, "round %d: injected %d, got %d (%s)", r, want, rc,
            msg.c_str());
    }
    hsg_restore_trim(-1, rnd(0, 1) ? 0 : (8u << 20));
    for (auto& f : p.files) unlink(f.c_str());
  }
  hsg_restore_trim(-1, 0);
  CHECK(stub::dev_live.load() == 0, "%llu device bytes leaked",
        (unsigned long long)stub::dev_live.load());
}

// c026ee7: ring of 10 MiB, blob A (5 MiB) then B (6 MiB).  B cannot start
// while A holds [0, 5); once A retires the ring is empty, and B only fits if
// the ring restarts at offset 0 (from offset 5 it would need 11 MiB).
void ringwrap_mode(const std::string& dir) {
  RestorePlan p;
  p.files.push_back(dir + "/ring");
  p.file_data.emplace_back();
  const uint64_t sizes[2] = {5u << 20, 6u << 20};
  for (uint64_t L : sizes) {
    std::vector<uint8_t> content = random_bytes(L);
    p.dest.emplace_back(L, 0);
    p.expected.push_back(content);
    p.paths.push_back(p.files[0]);
    p.lo.push_back(p.file_data[0].size());
    p.file_data[0].insert(p.file_data[0].end(), content.begin(), content.end());
    p.nb.push_back(L);
    p.codec.push_back(0);
    p.logical.push_back(0);
    p.direct.push_back(0);
    p.base_off.push_back(0);
    p.doff.push_back(int64_t(p.descs.size()));
    p.descs.push_back(StubDesc{0, reinterpret_cast<uint64_t>(p.dest.back().data()), L, 0});
    p.dn.push_back(1);
  }
  std::string msg;
  const int rc = run_restore(p, 1 << 20, 1 << 20, 1 << 20, 2, 2, 10u << 20, &msg);
  CHECK(rc == 0, "rc %d (%s)", rc, msg.c_str());
  for (size_t i = 0; i < p.dest.size(); ++i) CHECK(p.dest[i] == p.expected[i], "item %zu", i);
  hsg_restore_trim(-1, 0);
}

std::vector<uint8_t> read_file(const std::string& path) {
  std::vector<uint8_t> v;
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) return v;
  uint8_t buf[1 << 16];
  size_t k;
  while ((k = fread(buf, 1, sizeof(buf), f)) > 0) v.insert(v.end(), buf, buf + k);
  fclose(f);
  return v;
}

void drain_mode(const std::string& dir, int rounds) {
  for (int r = 0; r < rounds; ++r) {
    const bool inject = r % 4 == 3;
    const int n = int(rnd(1, 30));
    std::vector<std::vector<uint8_t>> src;
    std::vector<uint64_t> srcs, sizes;
    std::vector<std::string> paths;
    for (int i = 0; i < n; ++i) {
      const int kind = int(rnd(0, 9));
      const uint64_t len = kind == 0 ? 0 : kind < 5 ? rnd(1, 64 << 10) : rnd(1, 3u << 20);
      src.push_back(random_bytes(len));
      paths.push_back(dir + "/d" + std::to_string(r) + "/s" + std::to_string(i % 3) + "/b" +
                      std::to_string(i));
    }
    for (int i = 0; i < n; ++i) {
      srcs.push_back(reinterpret_cast<uint64_t>(src[i].data()));
      sizes.push_back(src[i].size());
    }
    int want_fail = 0;
    if (inject) {
      if (rnd(0, 1)) {
        stub::fail_d2h_every.store(2);
      } else {
        // a regular file where a directory must go
        const std::string blocker = dir + "/d" + std::to_string(r) + "_blocker";
        write_file(blocker, {1, 2, 3});
        paths[rnd(0, n - 1)] = blocker + "/x/b";
      }
      want_fail = 1;
    }
    std::vector<const char*> cpaths;
    for (auto& s : paths) cpaths.push_back(s.c_str());
    const int parked = int(rnd(0, 4));
    const int flags = 2 | (rnd(0, 1) ? 4 : 0) | (rng() % 8 == 0 ? 1 : 0) | (parked << 16);
    int err = 0;
    void* h = hsg_drain_start(0, n, srcs.data(), sizes.data(), cpaths.data(), 1 << 20,
                              int(rnd(2, 8)), int(rnd(1, 6)), flags, 64, &err);
    CHECK(h, "drain start failed %d", err);
    std::thread booster([h] {
      std::this_thread::sleep_for(std::chrono::microseconds(rnd(0, 3000)));
      CHECK(hsg_drain_pending(h) >= 0, "pending");
      hsg_drain_boost(h);
    });
    booster.join();  // a boost must not outlive the job (hsg_drain_wait frees it)
    std::vector<uint64_t> sums(n, 0);
    uint64_t written = 0;
    char msg[256];
    double stats[16];
    const int rc = hsg_drain_wait(h, sums.data(), &written, msg, stats);
    stub::fail_d2h_every.store(0);
    CHECK(stub::pinned_live.load() == 0, "round %d: pinned slots not released", r);
    if (want_fail) {
      CHECK(rc != 0, "round %d: injected failure not reported", r);
      continue;
    }
    CHECK(rc == 0, "round %d: rc %d (%s)", r, rc, msg);
    uint64_t total = 0;
    for (int i = 0; i < n; ++i) {
      CHECK(read_file(paths[i]) == src[i], "round %d: blob %d has wrong bytes", r, i);
      CHECK(sums[i] == stub::hash_bytes(src[i].data(), src[i].size()), "round %d: blob %d sum",
            r, i);
      total += src[i].size();
    }
    CHECK(written == total, "round %d: %llu bytes written of %llu", r,
          (unsigned long long)written, (unsigned long long)total);
  }
}

}  // namespace

void restore_trim_mode(const std::string& dir, int rounds) {
  std::atomic<bool> stop{false};
  std::atomic<uint64_t> trims{0};
  std::thread trimmer([&] {
    while (!stop.load()) {
      hsg_restore_trim(-1, 0);
      trims.fetch_add(1);
      std::this_thread::sleep_for(std::chrono::microseconds(int(rnd(20, 400))));
    }
  });
  std::vector<std::thread> loops;
  for (int t = 0; t < 3; ++t)
    loops.emplace_back([&, t] {
      rng.seed(seed0() + 1000 * uint64_t(t + 1));
      const std::string sub = dir + "/t" + std::to_string(t);
      mkdir(sub.c_str(), 0755);
      for (int r = 0; r < rounds; ++r) {
        RestorePlan p = make_restore_plan(sub, r, int(rnd(1, 10)),
                                          rng() % 3 == 0 ? (6u << 20) : (2u << 20));
        std::string msg;
        // budgets from below one blob (pool blocks) to several (rings)
        const int rc = run_restore(p, rnd(1, 2) << 20, 1 << 20, rnd(64, 512) << 10,
                                   int(rnd(2, 4)), int(rnd(1, 4)), rnd(1, 8) << 20, &msg);
        CHECK(rc == 0, "thread %d round %d: rc %d (%s)", t, r, rc, msg.c_str());
        for (size_t i = 0; i < p.dest.size(); ++i)
          CHECK(p.dest[i] == p.expected[i], "thread %d round %d: item %zu restored wrong bytes",
                t, r, i);
        if (rnd(0, 1)) hsg_restore_trim(-1, 0);  // the round-5 trim after every job
        for (auto& f : p.files) unlink(f.c_str());
      }
    });
  for (auto& th : loops) th.join();
  stop.store(true);
  trimmer.join();
  CHECK(stub::corruption.load() == 0, "a copy launch's tables were reused early");
  CHECK(stub::pinned_live.load() == 0, "%d pinned blocks not released", stub::pinned_live.load());
  CHECK(trims.load() > 0, "the trimmer never ran");
  hsg_restore_trim(-1, 0);
  CHECK(stub::dev_live.load() == 0, "%llu device bytes leaked",
        (unsigned long long)stub::dev_live.load());
}

int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: %s restore|drain|ringwrap <dir> [rounds]\n", argv[0]);
    return 2;
  }
  const std::string mode = argv[1], dir = argv[2];
  const int rounds = argc > 3 ? atoi(argv[3]) : 24;
  mkdir(dir.c_str(), 0755);
  if (mode == "restore")
    restore_mode(dir, rounds);
  else if (mode == "drain")
    drain_mode(dir, rounds);
  else if (mode == "ringwrap")
    ringwrap_mode(dir);
  else if (mode == "restore-trim")
    restore_trim_mode(dir, rounds);
  else
    return 2;
  stub::shutdown();
  printf("ok\n");
  return 0;
}
