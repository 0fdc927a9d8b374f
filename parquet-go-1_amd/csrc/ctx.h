// ctx.h — the device context shared by the batch API (host.cpp) and the streaming pipeline
// (pipeline.cpp).
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <mutex>
#include <utility>
#include <vector>

struct pqgpu_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  hipStream_t side = nullptr;  // values kernels run here concurrently with k_levels (speculative mode)
  hipStream_t copy = nullptr;  // PLAIN / BOOLEAN copies (k_values_copy) beside both
  hipStream_t delta = nullptr; // DELTA_BINARY_PACKED pages (k_values_delta) beside all three
  hipStream_t aux = nullptr;   // repetition-stream level kernels beside the definition streams', then
                               // the nested arrays (k_nest_tile) beside the values path
  // Device scratch of the page index builds, kept between calls (hipMalloc'd: kernel stores into
  // stream-ordered hipMallocAsync memory from workgroups off the first XCD were observed never to
  // reach a later device-to-host copy of it)
  std::mutex scratch_m;
  std::atomic<uint32_t> ix_gen{0};  // page index builds: completion-marker generation (never 0)
  uint32_t next_ix_gen() {
    uint32_t g;
    do g = ++ix_gen; while (g == 0);
    return g;
  }
  std::vector<std::pair<void *, size_t>> scratch_free;

  void *scratch_get(size_t want, size_t *cap) {
    {
      std::lock_guard<std::mutex> lk(scratch_m);
      for (size_t k = 0; k < scratch_free.size(); k++)
        if (scratch_free[k].second >= want) {
          void *p = scratch_free[k].first;
          *cap = scratch_free[k].second;
          scratch_free.erase(scratch_free.begin() + (long)k);
          return p;
        }
    }
    size_t c = 1 << 16;
    while (c < want) c *= 2;
    void *p = nullptr;
    if (hipMalloc(&p, c) != hipSuccess) return nullptr;
    *cap = c;
    return p;
  }
  void scratch_put(void *p, size_t cap) {
    if (!p) return;
    std::lock_guard<std::mutex> lk(scratch_m);
    if (scratch_free.size() < 16) {
      scratch_free.emplace_back(p, cap);
      return;
    }
    (void)hipFree(p);
  }
  void scratch_release() {
    std::lock_guard<std::mutex> lk(scratch_m);
    for (auto &b : scratch_free) (void)hipFree(b.first);
    scratch_free.clear();
  }
};
