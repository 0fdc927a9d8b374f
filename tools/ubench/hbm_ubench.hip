// hbm_ubench.hip — what streaming shapes reach on this chip (experiment tool, not product):
// read-only, write-only and copy kernels over buffers of 0.5-2 GB, each workgroup owning a
// contiguous chunk (C bytes) swept in rounds of 256 lanes x U pieces of 16 B, with default or
// nontemporal loads/stores. Timed as 10 back-to-back launches between two events.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(2); } } while (0)

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) v4u guint4;

template <uint32_t U, bool NT>
__global__ void __launch_bounds__(256) k_copy(const uint4 *s_, uint4 *d_, uint64_t n16, uint64_t chunk16) {
  const guint4 *s = (const guint4 *)s_;
  guint4 *d = (guint4 *)d_;
  const uint64_t c0 = (uint64_t)blockIdx.x * chunk16, c1 = std::min(n16, c0 + chunk16);
  for (uint64_t r = c0; r < c1; r += 256 * U) {
    v4u v[U];
#pragma unroll
    for (uint32_t u = 0; u < U; u++) {
      const uint64_t i = r + u * 256 + threadIdx.x;
      if (i < c1) v[u] = NT ? __builtin_nontemporal_load(&s[i]) : s[i];
    }
#pragma unroll
    for (uint32_t u = 0; u < U; u++) {
      const uint64_t i = r + u * 256 + threadIdx.x;
      if (i < c1) {
        if (NT) __builtin_nontemporal_store(v[u], &d[i]);
        else d[i] = v[u];
      }
    }
  }
}

template <uint32_t U>
__global__ void __launch_bounds__(256) k_read(const uint4 *s_, uint64_t n16, uint64_t chunk16, uint32_t *out) {
  const guint4 *s = (const guint4 *)s_;
  const uint64_t c0 = (uint64_t)blockIdx.x * chunk16, c1 = std::min(n16, c0 + chunk16);
  uint32_t acc = 0;
  for (uint64_t r = c0; r < c1; r += 256 * U) {
    v4u v[U];
#pragma unroll
    for (uint32_t u = 0; u < U; u++) {
      const uint64_t i = r + u * 256 + threadIdx.x;
      v[u] = i < c1 ? s[i] : v4u{0, 0, 0, 0};
    }
#pragma unroll
    for (uint32_t u = 0; u < U; u++) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

template <uint32_t U>
__global__ void __launch_bounds__(256) k_write(uint4 *d_, uint64_t n16, uint64_t chunk16) {
  guint4 *d = (guint4 *)d_;
  const uint64_t c0 = (uint64_t)blockIdx.x * chunk16, c1 = std::min(n16, c0 + chunk16);
  for (uint64_t r = c0; r < c1; r += 256 * U) {
#pragma unroll
    for (uint32_t u = 0; u < U; u++) {
      const uint64_t i = r + u * 256 + threadIdx.x;
      if (i < c1) d[i] = v4u{(uint32_t)i, 1, 2, 3};
    }
  }
}

int main() {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  uint32_t *out;
  CK(hipMalloc(&out, 64));
  const uint64_t maxb = 2ull << 30;
  uint8_t *a, *b;
  CK(hipMalloc(&a, maxb));
  CK(hipMalloc(&b, maxb));
  CK(hipMemset(a, 1, maxb));
  CK(hipMemset(b, 2, maxb));
  auto timeit = [&](const char *name, uint64_t bytes_moved, auto launch) {
    launch();
    CK(hipDeviceSynchronize());
    std::vector<float> v;
    for (int r = 0; r < 5; r++) {
      CK(hipEventRecord(e0, 0));
      for (int k = 0; k < 10; k++) launch();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float t;
      CK(hipEventElapsedTime(&t, e0, e1));
      v.push_back(t / 10);
    }
    std::sort(v.begin(), v.end());
    printf("{\"case\": \"%s\", \"ms\": %.4f, \"TBps\": %.3f}\n", name, v[2], bytes_moved / (v[2] * 1e-3) / 1e12);
    fflush(stdout);
  };
  char nm[128];
  for (uint64_t sz : {512ull << 20, 2ull << 30}) {
    const uint64_t n16 = sz / 16;
    for (uint64_t chunk : {64ull << 10, 256ull << 10, 1ull << 20}) {
      const uint32_t grid = (uint32_t)((sz + chunk - 1) / chunk);
      const uint64_t c16 = chunk / 16;
      snprintf(nm, sizeof nm, "read_%lluMB_chunk%lluK_u8", (unsigned long long)(sz >> 20), (unsigned long long)(chunk >> 10));
      timeit(nm, sz, [&] { k_read<8><<<grid, 256>>>((const uint4 *)a, n16, c16, out); });
      snprintf(nm, sizeof nm, "write_%lluMB_chunk%lluK_u8", (unsigned long long)(sz >> 20), (unsigned long long)(chunk >> 10));
      timeit(nm, sz, [&] { k_write<8><<<grid, 256>>>((uint4 *)b, n16, c16); });
      snprintf(nm, sizeof nm, "copy_%lluMB_chunk%lluK_u4", (unsigned long long)(sz >> 20), (unsigned long long)(chunk >> 10));
      timeit(nm, 2 * sz, [&] { k_copy<4, false><<<grid, 256>>>((const uint4 *)a, (uint4 *)b, n16, c16); });
      snprintf(nm, sizeof nm, "copy_%lluMB_chunk%lluK_u8", (unsigned long long)(sz >> 20), (unsigned long long)(chunk >> 10));
      timeit(nm, 2 * sz, [&] { k_copy<8, false><<<grid, 256>>>((const uint4 *)a, (uint4 *)b, n16, c16); });
      snprintf(nm, sizeof nm, "copy_%lluMB_chunk%lluK_u16", (unsigned long long)(sz >> 20), (unsigned long long)(chunk >> 10));
      timeit(nm, 2 * sz, [&] { k_copy<16, false><<<grid, 256>>>((const uint4 *)a, (uint4 *)b, n16, c16); });
      snprintf(nm, sizeof nm, "copy_nt_%lluMB_chunk%lluK_u8", (unsigned long long)(sz >> 20), (unsigned long long)(chunk >> 10));
      timeit(nm, 2 * sz, [&] { k_copy<8, true><<<grid, 256>>>((const uint4 *)a, (uint4 *)b, n16, c16); });
    }
  }
  return 0;
}
