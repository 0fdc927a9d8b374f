// ctx.h — the device context shared by the batch API (host.cpp) and the streaming pipeline
// (pipeline.cpp).
#pragma once
#include <hip/hip_runtime.h>

#include <mutex>
#include <utility>
#include <vector>

struct pqgpu_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  hipStream_t side = nullptr;  // values kernels run here concurrently with k_levels (speculative mode)
  // page-locked staging kept between calls (small DMA tables of the page index build):
  // hipHostMalloc costs far more than the copies it serves
  std::mutex pin_m;
  std::vector<std::pair<void *, size_t>> pin_free;

  void *pin_get(size_t want, size_t *cap) {
    {
      std::lock_guard<std::mutex> lk(pin_m);
      for (size_t k = 0; k < pin_free.size(); k++)
        if (pin_free[k].second >= want) {
          void *p = pin_free[k].first;
          *cap = pin_free[k].second;
          pin_free.erase(pin_free.begin() + (long)k);
          return p;
        }
    }
    size_t c = 4096;
    while (c < want) c *= 2;
    void *p = nullptr;
    if (hipHostMalloc(&p, c, hipHostMallocCoherent) != hipSuccess) return nullptr;
    *cap = c;
    return p;
  }
  void pin_put(void *p, size_t cap) {
    if (!p) return;
    std::lock_guard<std::mutex> lk(pin_m);
    if (pin_free.size() < 16) {
      pin_free.emplace_back(p, cap);
      return;
    }
    (void)hipHostFree(p);
  }
  void pin_release() {
    std::lock_guard<std::mutex> lk(pin_m);
    for (auto &b : pin_free) (void)hipHostFree(b.first);
    pin_free.clear();
  }
};
