// copy_shapes.hip — which copy shape reaches the guide's 6.29 TB/s (MI355X_MICROARCH.md: float4
// copy) on this box, against the product's PLAIN copy (dev_util.h copy_bytes_u, one workgroup per
// 16 Ki-value work item). Experiment tool, not product. Rates count read + write bytes.
//   flat1      one uint4 per thread, one grid over the range (no loop)
//   flat4      four uint4 per thread (wave-contiguous 1 KiB per instruction), no loop
//   gs4        grid-stride loop, 4 pieces per lane per round (load 4, store 4)
//   gs4_pipe   the same with the next round's loads issued before this round's stores
//   *_nt       non-temporal loads and stores
//   items_u4   the product copy (copy_bytes_u<4>) over cfg2-shaped work items, misaligned sources
//   items_p4   a pipelined item copy (next round's loads before this round's stores), misaligned
//   d2d        hipMemcpyAsync device to device
//   items_ua*  the item copy with unaligned 16-B loads (global_load_dwordx4 at any byte address; no
//              funnel shifts or lane shuffles), 16-B aligned stores; _nt: non-temporal; _d8: the
//              destinations only 8-B aligned as well (unaligned 16-B stores)
// Build: make -C tools/ubench copy_shapes; run: tools/ubench/copy_shapes
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../parquet-go-1_amd/csrc/dev_util.h"

using namespace pq;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(2); } } while (0)

template <bool NT>
DEV uint4 ld(const uint4 *p) {
  if (NT) { const nt_v4u32 v = __builtin_nontemporal_load((const nt_v4u32 *)p); return make_uint4(v.x, v.y, v.z, v.w); }
  return *p;
}
template <bool NT>
DEV void st(uint4 *p, uint4 v) {
  if (NT) __builtin_nontemporal_store(nt_v4u32{v.x, v.y, v.z, v.w}, (nt_v4u32 *)p);
  else *p = v;
}

template <bool NT>
__global__ void __launch_bounds__(256) k_flat1(const uint4 *__restrict__ s, uint4 *__restrict__ d, uint64_t n16) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n16) st<NT>(&d[i], ld<NT>(&s[i]));
}

template <bool NT>
__global__ void __launch_bounds__(256) k_flat4(const uint4 *__restrict__ s, uint4 *__restrict__ d, uint64_t n16) {
  const uint64_t base = (uint64_t)blockIdx.x * 1024 + (threadIdx.x >> 6) * 256 + (threadIdx.x & 63);
  uint4 a[4];
#pragma unroll
  for (int u = 0; u < 4; u++) if (base + 64 * u < n16) a[u] = ld<NT>(&s[base + 64 * u]);
#pragma unroll
  for (int u = 0; u < 4; u++) if (base + 64 * u < n16) st<NT>(&d[base + 64 * u], a[u]);
}

template <bool NT>
__global__ void __launch_bounds__(256) k_gs4(const uint4 *__restrict__ s, uint4 *__restrict__ d, uint64_t n16) {
  const uint64_t nt = (uint64_t)gridDim.x * 256, t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  uint64_t i = t;
  for (; i + 3 * nt < n16; i += 4 * nt) {
    uint4 a = ld<NT>(&s[i]), b = ld<NT>(&s[i + nt]), c = ld<NT>(&s[i + 2 * nt]), e = ld<NT>(&s[i + 3 * nt]);
    st<NT>(&d[i], a); st<NT>(&d[i + nt], b); st<NT>(&d[i + 2 * nt], c); st<NT>(&d[i + 3 * nt], e);
  }
  for (; i < n16; i += nt) st<NT>(&d[i], ld<NT>(&s[i]));
}

// next round's loads before this round's stores (vmcnt counts both in issue order: the wait for
// round r + 1's loads then leaves round r's stores in flight)
template <bool NT>
__global__ void __launch_bounds__(256) k_gs4_pipe(const uint4 *__restrict__ s, uint4 *__restrict__ d, uint64_t n16) {
  const uint64_t nt = (uint64_t)gridDim.x * 256, t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  const uint64_t rounds = n16 / (4 * nt);
  uint4 a[4];
  uint64_t i = t;
  if (rounds) {
#pragma unroll
    for (int u = 0; u < 4; u++) a[u] = ld<NT>(&s[i + u * nt]);
  }
  for (uint64_t r = 0; r < rounds; r++, i += 4 * nt) {
    uint4 b[4];
    const bool more = r + 1 < rounds;
    if (more) {
#pragma unroll
      for (int u = 0; u < 4; u++) b[u] = ld<NT>(&s[i + 4 * nt + u * nt]);
    }
#pragma unroll
    for (int u = 0; u < 4; u++) st<NT>(&d[i + u * nt], a[u]);
#pragma unroll
    for (int u = 0; u < 4; u++) a[u] = b[u];
  }
  for (i = rounds * 4 * nt + t; i < n16; i += nt) st<NT>(&d[i], ld<NT>(&s[i]));
}

struct Item { const uint8_t *src; uint8_t *dst; uint64_t n; };

__global__ void __launch_bounds__(256) k_items_u4(const Item *items) {
  const Item it = gp(items)[blockIdx.x];
  copy_bytes_u<4>(gp(it.dst), gp(it.src), it.n, threadIdx.x, 256);
}

// copy_bytes_u<4>'s layout, software-pipelined: round r + 1's four loads are issued before round r's
// funnel shifts and stores
DEV void copy_bytes_p4(uint8_t *dst, const uint8_t *src, uint64_t n, uint32_t tid, uint32_t nt) {
  constexpr uint32_t U = 4;
  if (n == 0) return;
  uintptr_t da = (uintptr_t)dst;
  uint64_t head = (16 - (da & 15)) & 15;
  if (head > n) head = n;
  if (tid < head) dst[tid] = src[tid];
  const uint64_t body = (n - head) & ~(uint64_t)15;
  uint4 *d = (uint4 *)(dst + head);
  const uint8_t *sp = src + head;
  const uint32_t sa = (uint32_t)((uintptr_t)sp & 15);
  const uint4 *sb = (const uint4 *)(sp - sa);
  const uint64_t pieces = body >> 4;
  const uint32_t lane = tid & 63u, wv = tid >> 6;
  const int nxt = (int)(((lane + 1) & 63u) * 4);
  auto shd = [nxt](uint32_t v) { return (uint32_t)__builtin_amdgcn_ds_bpermute(nxt, (int)v); };
  const uint64_t per = (uint64_t)nt * U;
  const uint64_t rounds = pieces / per;
  uint4 a[U], e = make_uint4(0u, 0u, 0u, 0u);
  uint64_t i = (uint64_t)wv * 64 * U + lane;
  if (rounds) {
#pragma unroll
    for (uint32_t u = 0; u < U; u++) a[u] = cp_ld16(&sb[i + 64 * u]);
    if (sa && lane == 63) e = sb[i + 64 * (U - 1) + 1];
  }
  for (uint64_t r = 0; r < rounds; r++, i += per) {
    uint4 c[U], e2 = make_uint4(0u, 0u, 0u, 0u);
    if (r + 1 < rounds) {
#pragma unroll
      for (uint32_t u = 0; u < U; u++) c[u] = cp_ld16(&sb[i + per + 64 * u]);
      if (sa && lane == 63) e2 = sb[i + per + 64 * (U - 1) + 1];
    }
    if (sa) {
#pragma unroll
      for (uint32_t u = 0; u < U; u++) {
        const uint4 o = (lane == 0 && u + 1 < U) ? a[u + 1] : a[u];
        uint4 b = make_uint4(shd(o.x), shd(o.y), shd(o.z), shd(o.w));
        if (lane == 63 && u + 1 == U) b = e;
        cp_st16(&d[i + 64 * u], funnel16(a[u], b, sa));
      }
    } else {
#pragma unroll
      for (uint32_t u = 0; u < U; u++) cp_st16(&d[i + 64 * u], a[u]);
    }
#pragma unroll
    for (uint32_t u = 0; u < U; u++) a[u] = c[u];
    e = e2;
  }
  for (uint64_t k = rounds * per + tid; k < pieces; k += nt) d[k] = sa ? funnel16(sb[k], sb[k + 1], sa) : sb[k];
  const uint64_t tail = n - head - body;
  if (tid < tail) dst[head + body + tid] = sp[body + tid];
}

__global__ void __launch_bounds__(256) k_items_p4(const Item *items) {
  const Item it = gp(items)[blockIdx.x];
  copy_bytes_p4(gp(it.dst), gp(it.src), it.n, threadIdx.x, 256);
}

typedef uint32_t ua_v4u32 __attribute__((ext_vector_type(4), aligned(1)));
template <bool NT>
DEV uint4 ld_ua(const uint8_t *p) {
  ua_v4u32 v;
  if (NT) v = __builtin_nontemporal_load((const ua_v4u32 *)p);
  else v = *(const ua_v4u32 *)p;
  return make_uint4(v.x, v.y, v.z, v.w);
}
template <bool NT>
DEV void st_ua(uint8_t *p, uint4 v) {
  const ua_v4u32 x = {v.x, v.y, v.z, v.w};
  if (NT) __builtin_nontemporal_store(x, (ua_v4u32 *)p);
  else *(ua_v4u32 *)p = x;
}
// dst[0..n) = src[0..n): 16-B pieces of the destination from its first 16-B aligned byte (A16) or its
// first byte (unaligned stores), four per lane per round, unaligned 16-B loads
template <bool NT, bool A16>
DEV void copy_ua(uint8_t *dst, const uint8_t *src, uint64_t n, uint32_t tid, uint32_t nt) {
  uint64_t head = A16 ? ((16 - ((uintptr_t)dst & 15)) & 15) : 0;
  if (head > n) head = n;
  if (tid < head) dst[tid] = src[tid];
  const uint64_t pieces = (n - head) >> 4;
  uint8_t *d = dst + head;
  const uint8_t *sp = src + head;
  const uint32_t lane = tid & 63u, wv = tid >> 6;
  const uint64_t per = (uint64_t)nt * 4;
  uint64_t r0 = 0;
  for (; r0 + per <= pieces; r0 += per) {
    const uint64_t i = r0 + (uint64_t)wv * 256 + lane;
    uint4 a[4];
#pragma unroll
    for (int u = 0; u < 4; u++) a[u] = ld_ua<NT>(sp + 16 * (i + 64 * u));
#pragma unroll
    for (int u = 0; u < 4; u++) {
      if (A16) st_ua<NT>(d + 16 * (i + 64 * u), a[u]);
      else st_ua<NT>(d + 16 * (i + 64 * u), a[u]);
    }
  }
  for (uint64_t i = r0 + tid; i < pieces; i += nt) st_ua<NT>(d + 16 * i, ld_ua<NT>(sp + 16 * i));
  const uint64_t tail = n - head - 16 * pieces;
  if (tid < tail) d[16 * pieces + tid] = sp[16 * pieces + tid];
}
template <bool NT, bool A16>
__global__ void __launch_bounds__(256) k_items_ua(const Item *items) {
  const Item it = gp(items)[blockIdx.x];
  copy_ua<NT, A16>(gp(it.dst), gp(it.src), it.n, threadIdx.x, 256);
}

int main() {
  const uint32_t pages = 1024, vals = 59000;  // cfg2's DOUBLE column: ~59,000 non-null values per page
  const uint64_t page_bytes = (uint64_t)vals * 8;
  const uint64_t page_stride = (page_bytes + 2048 + 15) & ~15ull;
  const uint64_t total = page_bytes * pages;
  uint8_t *src, *dst;
  CK(hipMalloc(&src, page_stride * pages + 4096));
  CK(hipMalloc(&dst, total + 4096));
  CK(hipMemset(src, 1, page_stride * pages + 4096));
  CK(hipMemset(dst, 0, total + 4096));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timeit = [&](const char *name, auto launch) {
    for (int w = 0; w < 3; w++) launch();
    CK(hipDeviceSynchronize());
    std::vector<float> ms;
    for (int r = 0; r < 7; r++) {
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
  const uint64_t n16 = total / 16;
  const uint4 *s4 = (const uint4 *)src;
  uint4 *d4 = (uint4 *)dst;
  timeit("flat1", [&] { k_flat1<false><<<(n16 + 255) / 256, 256>>>(s4, d4, n16); });
  timeit("flat1_nt", [&] { k_flat1<true><<<(n16 + 255) / 256, 256>>>(s4, d4, n16); });
  timeit("flat4", [&] { k_flat4<false><<<(n16 + 1023) / 1024, 256>>>(s4, d4, n16); });
  timeit("flat4_nt", [&] { k_flat4<true><<<(n16 + 1023) / 1024, 256>>>(s4, d4, n16); });
  for (uint32_t g : {1024u, 2048u, 4096u, 8192u}) {
    char nm[64];
    snprintf(nm, sizeof nm, "gs4_g%u", g);
    timeit(nm, [&] { k_gs4<false><<<g, 256>>>(s4, d4, n16); });
    snprintf(nm, sizeof nm, "gs4_nt_g%u", g);
    timeit(nm, [&] { k_gs4<true><<<g, 256>>>(s4, d4, n16); });
    snprintf(nm, sizeof nm, "gs4_pipe_g%u", g);
    timeit(nm, [&] { k_gs4_pipe<false><<<g, 256>>>(s4, d4, n16); });
    snprintf(nm, sizeof nm, "gs4_pipe_nt_g%u", g);
    timeit(nm, [&] { k_gs4_pipe<true><<<g, 256>>>(s4, d4, n16); });
  }
  timeit("d2d", [&] { CK(hipMemcpyAsync(dst, src, total, hipMemcpyDeviceToDevice, 0)); });
  Item *ditems;
  CK(hipMalloc(&ditems, sizeof(Item) * pages * 64));  // (>= 59,000 / 2,048 items per page)
  for (uint32_t per : {2048u, 4096u, 16384u, 32768u}) {
    std::vector<Item> items;
    for (uint32_t p = 0; p < pages; p++) {
      const uint32_t off = 1024 + (p * 7 + 3) % 16;  // value sections at arbitrary byte alignment
      for (uint32_t v0 = 0; v0 < vals; v0 += per) {
        const uint32_t v1 = std::min(vals, v0 + per);
        items.push_back({src + p * page_stride + off + (uint64_t)v0 * 8, dst + (uint64_t)p * page_bytes + (uint64_t)v0 * 8,
                         (uint64_t)(v1 - v0) * 8});
      }
    }
    CK(hipMemcpy(ditems, items.data(), sizeof(Item) * items.size(), hipMemcpyHostToDevice));
    const uint32_t ni = (uint32_t)items.size();
    char nm[96];
    snprintf(nm, sizeof nm, "items_u4_per%u", per);
    timeit(nm, [&] { k_items_u4<<<ni, 256>>>(ditems); });
    snprintf(nm, sizeof nm, "items_p4_per%u", per);
    timeit(nm, [&] { k_items_p4<<<ni, 256>>>(ditems); });
    snprintf(nm, sizeof nm, "items_ua_per%u", per);
    timeit(nm, [&] { k_items_ua<false, true><<<ni, 256>>>(ditems); });
    snprintf(nm, sizeof nm, "items_ua_nt_per%u", per);
    timeit(nm, [&] { k_items_ua<true, true><<<ni, 256>>>(ditems); });
  }
  for (uint32_t per : {2048u, 16384u}) {  // destinations 8-B aligned only (as int64 / double outputs at odd bases)
    std::vector<Item> items;
    for (uint32_t p = 0; p < pages; p++) {
      const uint32_t off = 1024 + (p * 7 + 3) % 16;
      for (uint32_t v0 = 0; v0 < vals; v0 += per) {
        const uint32_t v1 = std::min(vals, v0 + per);
        items.push_back({src + p * page_stride + off + (uint64_t)v0 * 8, dst + 8 + (uint64_t)p * page_bytes + (uint64_t)v0 * 8,
                         (uint64_t)(v1 - v0) * 8});
      }
    }
    CK(hipMemcpy(ditems, items.data(), sizeof(Item) * items.size(), hipMemcpyHostToDevice));
    const uint32_t ni = (uint32_t)items.size();
    char nm[96];
    snprintf(nm, sizeof nm, "items_u4_d8_per%u", per);
    timeit(nm, [&] { k_items_u4<<<ni, 256>>>(ditems); });
    snprintf(nm, sizeof nm, "items_ua_nt_d8_per%u", per);
    timeit(nm, [&] { k_items_ua<true, false><<<ni, 256>>>(ditems); });
    snprintf(nm, sizeof nm, "items_ua_nt_d8a16_per%u", per);
    timeit(nm, [&] { k_items_ua<true, true><<<ni, 256>>>(ditems); });
  }
  return 0;
}
