// Controls of the CPU device stubs (engine_stubs.cpp) and the entry points of
// the host engines they stand under (hipsnapshot/csrc/hsrestore.cpp,
// hsdrain.cpp).
#pragma once

#include <atomic>
#include <cstdint>

namespace stub {

// the stub's region-copy descriptor (hsg_desc_size): `src` first, as the
// restore engine rebases the first 8 bytes of every row
struct StubDesc {
  uint64_t src;
  uint64_t dst;
  uint64_t nbytes;
  uint64_t pad;
};

extern std::atomic<int> fail_upload_every;  // every Nth host -> device upload fails (0: none)
extern std::atomic<int> fail_d2h_every;     // every Nth device -> host copy fails
extern std::atomic<uint64_t> dev_cap;       // device allocations fail above this many live bytes
extern std::atomic<uint64_t> dev_live;
extern std::atomic<int> pinned_live;        // pinned blocks not released
extern std::atomic<int> corruption;         // copy launches whose stage / workspace was reused early
extern std::atomic<int> max_delay_us;       // random delay before each queued operation

uint64_t hash_bytes(const void* p, uint64_t n);
void* new_stream();  // a stream of the caller's (a "producer" of restore destinations)
void shutdown();     // joins every stub thread

}  // namespace stub

extern "C" {
void* hsg_restore_start(int dev, int n, const char* const* paths, const uint64_t* file_lo,
                        const uint64_t* nbytes, const int* codec, const uint64_t* logical,
                        const uint64_t* direct, const uint64_t* base_off, const int64_t* desc_off,
                        const int* desc_n, const void* descs, int64_t n_descs,
                        const uint64_t* producers, int n_producers, uint32_t* err_words,
                        uint64_t slot_bytes, uint64_t first_bytes, uint64_t piece_bytes,
                        int nslots, int nreaders, uint64_t budget, int engine,
                        const int* hash_items, int hash_grid, int* err);
int hsg_restore_wait(void* handle, int* err_item, char* msg, double* stats,
                     uint64_t* bytes_read, uint64_t* sums);
int hsg_restore_prewarm(int dev, uint64_t up_bytes, uint64_t sc_bytes, uint64_t slot_bytes,
                        int nslots, uint64_t table_bytes);
uint64_t hsg_restore_trim(int dev, uint64_t keep);

void* hsg_drain_start(int dev, int n, const uint64_t* srcs, const uint64_t* sizes,
                      const char* const* paths, uint64_t slot_bytes, int nslots, int nwriters,
                      int flags, int max_hash_grid, int* err);
void hsg_drain_boost(void* handle);
int hsg_drain_wait(void* handle, uint64_t* sums, uint64_t* bytes_written, char* msg,
                   double* stats);
int hsg_drain_pending(void* handle);

}
