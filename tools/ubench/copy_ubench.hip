// copy_ubench.hip — calibration of the PLAIN fixed-width copy (experiment tool, not product).
// cfg2's DOUBLE column is 1,024 pages of ~59,000 non-null values; every page's value section sits
// at an arbitrary byte alignment in the stage buffer and goes to an 8-B aligned place in the
// values array. This times, on the same buffers:
//   ideal  : a grid-stride float4 copy of one contiguous range (the chip's copy ceiling)
//   items  : one workgroup per work item of S bytes through copy_bytes / copy_bytes_u<U>
//            (dev_util.h, the product's copy), sources misaligned as in cfg2 or aligned
// Rates count read + write bytes. Build: make -C tools/ubench; run: tools/ubench/copy_ubench
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../parquet-go-1_amd/csrc/dev_util.h"

using namespace pq;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(2); } } while (0)

struct Item { const uint8_t *src; uint8_t *dst; uint64_t n; };

__global__ void __launch_bounds__(256) k_ideal(const uint4 *__restrict__ s, uint4 *__restrict__ d, uint64_t n16) {
  const uint64_t nt = (uint64_t)gridDim.x * 256, t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  uint64_t i = t;
  for (; i + 3 * nt < n16; i += 4 * nt) {
    uint4 a = s[i], b = s[i + nt], c = s[i + 2 * nt], e = s[i + 3 * nt];
    d[i] = a; d[i + nt] = b; d[i + 2 * nt] = c; d[i + 3 * nt] = e;
  }
  for (; i < n16; i += nt) d[i] = s[i];
}

template <uint32_t U>
__global__ void __launch_bounds__(256) k_items(const Item *items) {
  const Item it = gp(items)[blockIdx.x];
  if constexpr (U == 0) copy_bytes(gp(it.dst), gp(it.src), it.n, threadIdx.x, 256);
  else copy_bytes_u<U>(gp(it.dst), gp(it.src), it.n, threadIdx.x, 256);
}

// the same as a persistent grid: workgroup g takes items g, g + G, ...
template <uint32_t U>
__global__ void __launch_bounds__(256) k_items_persist(const Item *items, uint32_t nitems) {
  for (uint32_t k = blockIdx.x; k < nitems; k += gridDim.x) {
    const Item it = gp(items)[k];
    copy_bytes_u<U>(gp(it.dst), gp(it.src), it.n, threadIdx.x, 256);
  }
}

int main(int argc, char **argv) {
  const uint32_t pages = 1024, vals = 59000;
  const uint64_t page_bytes = (uint64_t)vals * 8;
  const uint64_t page_stride = (page_bytes + 2048 + 15) & ~15ull;
  uint8_t *src, *dst;
  CK(hipMalloc(&src, page_stride * pages + 4096));
  CK(hipMalloc(&dst, page_bytes * pages + 4096));
  CK(hipMemset(src, 1, page_stride * pages + 4096));
  CK(hipMemset(dst, 0, page_bytes * pages + 4096));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const uint64_t total = page_bytes * pages;
  auto timeit = [&](const char *name, auto launch) {
    for (int w = 0; w < 3; w++) launch();
    CK(hipDeviceSynchronize());
    std::vector<float> ms;
    for (int r = 0; r < 5; r++) {  // 10 launches back to back per event pair (no launch gap in the figure)
      CK(hipEventRecord(e0, 0));
      for (int k = 0; k < 10; k++) launch();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float t;
      CK(hipEventElapsedTime(&t, e0, e1));
      ms.push_back(t / 10);
    }
    std::sort(ms.begin(), ms.end());
    const float med = ms[ms.size() / 2];
    printf("{\"case\": \"%s\", \"ms\": %.4f, \"TBps_rw\": %.3f}\n", name, med, 2.0 * total / (med * 1e-3) / 1e12);
    fflush(stdout);
  };
  // ideal: one contiguous range of the same byte count
  for (uint32_t gmul : {4u, 8u, 16u}) {
    char nm[64];
    snprintf(nm, sizeof nm, "ideal_grid%ux256", gmul);
    timeit(nm, [&] { k_ideal<<<256 * gmul, 256>>>((const uint4 *)src, (uint4 *)dst, total / 16); });
  }
  Item *ditems;
  CK(hipMalloc(&ditems, sizeof(Item) * pages * 64));
  for (int aligned = 0; aligned < 2; aligned++) {
    for (uint32_t per : {8192u, 16384u, 32768u, 65536u}) {  // values per work item
      std::vector<Item> items;
      for (uint32_t p = 0; p < pages; p++) {
        const uint32_t off = aligned ? 1024 : 1024 + (p * 7 + 3) % 16;  // value section offset in the page
        for (uint32_t v0 = 0; v0 < vals; v0 += per) {
          const uint32_t v1 = std::min(vals, v0 + per);
          items.push_back({src + p * page_stride + off + (uint64_t)v0 * 8, dst + (uint64_t)p * page_bytes + (uint64_t)v0 * 8,
                           (uint64_t)(v1 - v0) * 8});
        }
      }
      CK(hipMemcpy(ditems, items.data(), sizeof(Item) * items.size(), hipMemcpyHostToDevice));
      const uint32_t ni = (uint32_t)items.size();
      char nm[96];
      snprintf(nm, sizeof nm, "items%s_per%u_u0", aligned ? "_al" : "", per);
      timeit(nm, [&] { k_items<0><<<ni, 256>>>(ditems); });
      snprintf(nm, sizeof nm, "items%s_per%u_u4", aligned ? "_al" : "", per);
      timeit(nm, [&] { k_items<4><<<ni, 256>>>(ditems); });
      snprintf(nm, sizeof nm, "items%s_per%u_u8", aligned ? "_al" : "", per);
      timeit(nm, [&] { k_items<8><<<ni, 256>>>(ditems); });
      snprintf(nm, sizeof nm, "persist%s_per%u_u4_g2048", aligned ? "_al" : "", per);
      timeit(nm, [&] { k_items_persist<4><<<2048, 256>>>(ditems, ni); });
    }
  }
  return 0;
}
