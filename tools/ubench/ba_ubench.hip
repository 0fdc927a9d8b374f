// ba_ubench.hip — where the time of a BYTE_ARRAY dictionary gather goes (experiment tool, not
// product; bytearray.hip k_ba_emit_slots is the product kernel). cfg3's shape: 8 dictionaries of
// 65,536 entries of 4-28 bytes in 32-B slots [u32 length | bytes | zero pad] (one per XCD, as the
// product's per-XCD tile queues place them), 33,554,432 u16 indices in 4,096-value tiles, an 8-wave
// workgroup per tile, wave w owning 512 values in 8 rounds of 64. Tile bases are precomputed (no
// look-back, no run tables: plain u16 index arrays), so each mode isolates one phase:
//   0 index reads only               1 + length gathers (slot word 0)     2 + offsets stores
//   3 + both slot pieces gathered (no payload stores)
//   4 + LDS assembly (ds_or) and aligned 16-B payload stores: the product's pass B
//   5 pass B loads by lane pairs (lanes 2k, 2k+1: pieces 0, 1 of one value: one cache line per value)
//   6 the first piece loaded in pass A (length from it), pass B loads only piece 1
//   7 pass A loads whole slots by lane pairs and keeps them; pass B loads nothing
// Modes 4-7 write the payload and offsets, checked against the host's.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(2); } } while (0)

constexpr uint32_t kDict = 65536, kTile = 4096, kWaves = 8, kR = 8, kChunks = 8;
constexpr uint32_t kWaveBuf = 2048, kWaveVec = kWaveBuf / 16 + 2;

__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }
__device__ __forceinline__ void wave_lds_sync() { __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront"); __builtin_amdgcn_wave_barrier(); __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront"); }
template <int CTRL, int ROWS = 0xf>
__device__ __forceinline__ uint32_t dpp0(uint32_t x) { return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, ROWS, 0xf, false); }
__device__ __forceinline__ uint32_t scan32(uint32_t x) {
  x += dpp0<0x111>(x); x += dpp0<0x112>(x); x += dpp0<0x114>(x); x += dpp0<0x118>(x);
  x += dpp0<0x142, 0xa>(x); x += dpp0<0x143, 0xc>(x);
  return x;
}
__device__ __forceinline__ uint32_t rdlane(uint32_t v, uint32_t l) { return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)l); }
typedef uint32_t v4u __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint32_t bperm(uint32_t v, uint32_t src_lane) { return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src_lane * 4), (int)v); }

// bytes of one 16-B piece (entry bytes [e0, e0 + 16) held in x as dwords; zero past the entry) OR-ed
// into the LDS buffer at byte d, n valid bytes (n <= 16)
template <int F = 0>
__device__ __forceinline__ void or_piece(uint32_t *lw, uint32_t d, const uint32_t (&W)[5], uint32_t n) {
  if (F & 2) return;
  if (F & 4) {  // 8-B granules: the piece shifted to d's 8-B alignment, then ds_or_b64
    const uint32_t sh8 = d & 7u, q0 = d >> 3, end8 = sh8 + n;
    uint32_t X[7];  // W shifted up by sh8 bytes, dword-granular
    const uint32_t sw = sh8 >> 2, sb = sh8 & 3u;
#pragma unroll
    for (int m = 0; m < 7; m++) {
      const int i = m - (int)sw;
      const uint32_t hi = (i >= 0 && i < 5) ? W[i] : 0u, lo = (i - 1 >= 0 && i - 1 < 5) ? W[i - 1] : 0u;
      X[m] = sb ? __builtin_amdgcn_alignbyte(hi, lo, 4 - sb) : hi;
    }
    unsigned long long *l8 = (unsigned long long *)lw;
#pragma unroll
    for (int m = 0; m < 3; m++) {
      if (8u * m >= end8) break;
      atomicOr(&l8[q0 + m], ((unsigned long long)X[2 * m + 1] << 32) | X[2 * m]);
    }
    return;
  }
  const uint32_t sh = d & 3u, d0 = d >> 2, end = sh + n;
#pragma unroll
  for (int m = 0; m < 5; m++) {
    if (4u * m >= end) break;
    const uint32_t prev = m ? W[m - 1] : 0u;
    const uint32_t word = sh ? __builtin_amdgcn_alignbyte(W[m], prev, 4 - sh) : W[m];
    atomicOr(&lw[d0 + m], word);
  }
}

// F (modes 4-7): 1 no payload stores, 2 no LDS assembly, 4 ds_or_b64 assembly, 8 non-temporal payload
// stores, 16 no buffer zeroing (timing only: the payload is then wrong)
template <int MODE, int F = 0>
__global__ void __launch_bounds__(64 * kWaves) __attribute__((amdgpu_waves_per_eu(MODE == 7 ? 4 : 6)))
k_emit(const uint16_t *__restrict__ idx, const uint4 *__restrict__ slots, const uint64_t *__restrict__ tbase,
       int32_t *__restrict__ offs, uint8_t *__restrict__ P, uint32_t *__restrict__ dummy, uint32_t tpc) {
  __shared__ uint4 wbuf[kWaves][kWaveVec];
  __shared__ uint32_t wtot[kWaves];
  const uint32_t q = blockIdx.x & 7u, tt = blockIdx.x >> 3;
  const uint32_t t = q * tpc + tt;  // chunk q's tile tt
  const uint4 *sl = slots + (uint64_t)q * kDict * 2;
  const uint32_t *slw = (const uint32_t *)sl;
  const uint32_t lane = lane_id(), wv = threadIdx.x >> 6;
  const uint64_t seg0 = (uint64_t)t * kTile + wv * 64 * kR;
  uint32_t id[kR], len[kR];
  uint4 p0[MODE == 6 ? kR : 1];
  uint4 pk[MODE == 7 ? kR : 1][2];
#pragma unroll
  for (uint32_t r = 0; r < kR; r++) id[r] = idx[seg0 + r * 64 + lane];
  uint32_t acc = 0;
#pragma unroll
  for (uint32_t r = 0; r < kR; r++) {
    if (MODE == 0) len[r] = 4 + (id[r] & 15);
    else if (MODE == 6) { p0[r] = sl[2 * id[r]]; len[r] = p0[r].x; }
    else if (MODE == 7) {
      // lane l loads piece (l & 1) of value (l >> 1) + 32 h of this round, h = 0, 1
#pragma unroll
      for (uint32_t h = 0; h < 2; h++) {
        const uint32_t v = bperm(id[r], (lane >> 1) + 32 * h);
        pk[r][h] = sl[2 * v + (lane & 1)];
      }
      // the length of this lane's own value: word 0 of piece 0 of value `lane`, held by lane 2 lane mod 64 of half lane / 32
      const uint32_t src = (2 * lane) & 63u;
      const uint32_t a = bperm(pk[r][0].x, src), b2 = bperm(pk[r][1].x, src);
      len[r] = lane < 32 ? a : b2;
    } else len[r] = slw[8 * id[r]];
  }
  if (MODE <= 3) {
    uint32_t wt = 0;
#pragma unroll
    for (uint32_t r = 0; r < kR; r++) {
      const uint32_t incl = scan32(len[r]);
      if (MODE >= 2) offs[seg0 + r * 64 + lane + 1] = (int32_t)(incl + wt);
      wt += rdlane(incl, 63);
      if (MODE == 3) {
        const uint4 a = sl[2 * id[r]], b2 = sl[2 * id[r] + 1];
        acc ^= a.y ^ b2.w;
      }
      acc += len[r];
    }
    if (acc == 0x12345678u) dummy[blockIdx.x] = acc;
    return;
  }
  // wave totals and the wave's base
  uint32_t mine = 0;
#pragma unroll
  for (uint32_t r = 0; r < kR; r++) mine += len[r];
  uint32_t wt = mine;
#pragma unroll
  for (int o = 32; o; o >>= 1) wt += (uint32_t)__shfl_xor((int)wt, o);
  uint4 *wb = &wbuf[wv][0];
  for (uint32_t k = lane; k < kWaveVec; k += 64) wb[k] = make_uint4(0u, 0u, 0u, 0u);
  if (lane == 0) wtot[wv] = wt;
  __syncthreads();
  uint64_t wbase = tbase[t];
  for (uint32_t k = 0; k < wv; k++) wbase += wtot[k];
  wave_lds_sync();
  uint8_t *lb = (uint8_t *)wb;
  uint32_t *lw = (uint32_t *)wb;
  uint8_t *gblk = P + wbase - ((uintptr_t)(P + wbase) & 15u);
  uint32_t cur = (uint32_t)((uintptr_t)(P + wbase) & 15u), own = cur;
  constexpr uint32_t G = 2;
#pragma unroll
  for (uint32_t g = 0; g < kR / G; g++) {
    uint4 s[G][2];
#pragma unroll
    for (uint32_t rr = 0; rr < G; rr++) {
      const uint32_t r = g * G + rr;
      if (MODE == 4) {
        s[rr][0] = sl[2 * id[r]];
        s[rr][1] = len[r] > 12 ? sl[2 * id[r] + 1] : make_uint4(0u, 0u, 0u, 0u);
      } else if (MODE == 5) {
#pragma unroll
        for (uint32_t h = 0; h < 2; h++) {
          const uint32_t v = bperm(id[r], (lane >> 1) + 32 * h);
          s[rr][h] = sl[2 * v + (lane & 1)];
        }
      } else if (MODE == 6) {
        s[rr][0] = p0[r];
        s[rr][1] = len[r] > 12 ? sl[2 * id[r] + 1] : make_uint4(0u, 0u, 0u, 0u);
      } else {
        s[rr][0] = pk[r][0];
        s[rr][1] = pk[r][1];
      }
    }
#pragma unroll
    for (uint32_t rr = 0; rr < G; rr++) {
      const uint32_t r = g * G + rr;
      const uint32_t l = len[r];
      const uint32_t incl = scan32(l);
      const uint32_t T = rdlane(incl, 63);
      const uint32_t ex = incl - l;
      offs[seg0 + r * 64 + lane + 1] = (int32_t)(wbase + incl);
      if (cur + T > kWaveBuf) { if (lane == 0) dummy[blockIdx.x] = 1; return; }  // (never with 4-28 B values)
      if (MODE == 4 || MODE == 6) {
        if (l) {  // the slot's bytes: words 1..7 of the two pieces (zero past the entry)
          const uint4 a = s[rr][0], b2 = s[rr][1];
          const uint32_t W0[5] = {a.y, a.z, a.w, b2.x, 0u};
          or_piece<F>(lw, cur + ex, W0, min(l, 16u));
          if (l > 16) {
            const uint32_t W1[5] = {b2.y, b2.z, b2.w, 0u, 0u};
            or_piece<F>(lw, cur + ex + 16, W1, l - 16);
          }
        }
      } else {
        // lane holds piece (lane & 1) of values (lane >> 1) and (lane >> 1) + 32
#pragma unroll
        for (uint32_t h = 0; h < 2; h++) {
          const uint32_t v = (lane >> 1) + 32 * h, pc = lane & 1;
          const uint32_t lv = bperm(l, v), ev = bperm(ex, v);
          const uint4 x = s[rr][h];
          if (pc == 0) {  // entry bytes [0, 12): slot words 1..3
            const uint32_t W0[5] = {x.y, x.z, x.w, 0u, 0u};
            const uint32_t n = min(lv, 12u);
            if (n) or_piece<F>(lw, cur + ev, W0, n);
          } else if (lv > 12) {  // entry bytes [12, 28): slot words 4..7
            const uint32_t W1[5] = {x.x, x.y, x.z, x.w, 0u};
            or_piece<F>(lw, cur + ev + 12, W1, lv - 12);
          }
        }
      }
      wave_lds_sync();
      const uint32_t end = cur + T, full = end >> 4;
      const uint32_t k0 = own ? 1u : 0u;
      if (!(F & 1))
        for (uint32_t k = k0 + lane; k < full; k += 64) {
          if (F & 8) {
            const uint4 x = wb[k];
            __builtin_nontemporal_store(v4u{x.x, x.y, x.z, x.w}, (v4u *)(gblk + 16 * k));
          } else {
            *(uint4 *)(gblk + 16 * k) = wb[k];
          }
        }
      if (own && full && lane >= own && lane < 16) gblk[lane] = lb[lane];
      wave_lds_sync();
      if (full) {
        if (lane == 0) wb[0] = wb[full];
        wave_lds_sync();
        if (!(F & 16))
          for (uint32_t k = 1 + lane; k <= full; k += 64) wb[k] = make_uint4(0u, 0u, 0u, 0u);
        wave_lds_sync();
        gblk += 16 * full;
        own = 0;
      }
      cur = end & 15u;
      wbase += T;
    }
  }
  if (lane >= own && lane < cur) gblk[lane] = lb[lane];
}

int main(int argc, char **argv) {
  const uint64_t N = 33554432ull, ntiles = N / kTile, tpc = ntiles / kChunks;
  std::mt19937_64 rng(4);
  std::vector<uint32_t> hslots((size_t)kChunks * kDict * 8, 0u);
  std::vector<uint8_t> hlen((size_t)kChunks * kDict);
  for (uint32_t c = 0; c < kChunks; c++)
    for (uint32_t e = 0; e < kDict; e++) {
      const uint32_t L = 4 + (uint32_t)(rng() % 25);
      hlen[(size_t)c * kDict + e] = (uint8_t)L;
      uint32_t *w = &hslots[((size_t)c * kDict + e) * 8];
      w[0] = L;
      uint8_t *by = (uint8_t *)(w + 1);
      for (uint32_t k = 0; k < L; k++) by[k] = (uint8_t)(97 + rng() % 26);
    }
  std::vector<uint16_t> hidx(N);
  for (uint64_t i = 0; i < N; i++) hidx[i] = (uint16_t)(rng() & 0xffff);
  // per-tile bases over the whole output (tiles of chunk c are contiguous: chunk-major)
  std::vector<uint64_t> tb(ntiles);
  std::vector<int32_t> hoff(N + 1);
  uint64_t tot = 0;
  for (uint64_t t = 0; t < ntiles; t++) {
    tb[t] = tot;
    const uint32_t c = (uint32_t)(t / tpc);
    for (uint32_t k = 0; k < kTile; k++) tot += hlen[(size_t)c * kDict + hidx[t * kTile + k]];
  }
  printf("payload %.1f MB, offsets %.1f MB, indices %.1f MB\n", tot / 1e6, N * 4 / 1e6, N * 2 / 1e6);
  uint16_t *didx; uint4 *dsl; uint64_t *dtb; int32_t *doff; uint8_t *dP; uint32_t *ddum;
  CK(hipMalloc(&didx, N * 2)); CK(hipMalloc(&dsl, hslots.size() * 4)); CK(hipMalloc(&dtb, ntiles * 8));
  CK(hipMalloc(&doff, (N + 1) * 4)); CK(hipMalloc(&dP, tot + 64)); CK(hipMalloc(&ddum, 1 << 20));
  CK(hipMemcpy(didx, hidx.data(), N * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dsl, hslots.data(), hslots.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dtb, tb.data(), ntiles * 8, hipMemcpyHostToDevice));
  // the reference payload for the checks
  std::vector<uint8_t> ref(tot);
  {
    uint64_t o = 0;
    for (uint64_t i = 0; i < N; i++) {
      const uint32_t c = (uint32_t)(i / kTile / tpc);
      const uint32_t *w = &hslots[((size_t)c * kDict + hidx[i]) * 8];
      memcpy(&ref[o], w + 1, w[0]);
      o += w[0];
    }
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto run = [&](int mode, int F, const char *name) {
    auto launch = [&]() {
      const dim3 g((uint32_t)ntiles), bl(64 * kWaves);
#define L(M, FF) if (mode == M && F == FF) hipLaunchKernelGGL((k_emit<M, FF>), g, bl, 0, 0, didx, dsl, dtb, doff, dP, ddum, (uint32_t)tpc)
      L(1, 0); L(2, 0); L(3, 0); L(4, 0); L(5, 0); L(6, 0); L(7, 0);
      L(4, 1); L(4, 2); L(4, 3); L(4, 4); L(4, 8); L(4, 16); L(7, 1); L(7, 2); L(7, 4); L(7, 8); L(6, 4); L(7, 20);
#undef L
    };
    CK(hipMemset(dP, 0, tot));
    launch();
    CK(hipDeviceSynchronize());
    const int reps = 20;
    CK(hipEventRecord(e0, 0));
    for (int k = 0; k < reps; k++) launch();
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= reps;
    const double bytes = (double)N * 2 + (mode >= 2 ? (double)N * 4 : 0) + (mode >= 4 ? (double)tot : 0);
    const bool check = mode >= 4 && !(F & 19);
    bool ok = true;
    if (check) {
      std::vector<uint8_t> got(tot);
      CK(hipMemcpy(got.data(), dP, tot, hipMemcpyDeviceToHost));
      ok = memcmp(got.data(), ref.data(), tot) == 0;
      if (!ok) {
        uint64_t i = 0;
        while (got[i] == ref[i]) i++;
        printf("  first payload mismatch at %llu\n", (unsigned long long)i);
      }
    }
    printf("%-34s mode %d F %2d: %.4f ms  %.0f GB/s of output+index bytes%s\n", name, mode, F, ms, bytes / ms / 1e6, check ? (ok ? "  payload OK" : "  PAYLOAD MISMATCH") : "");
  };
  struct Cfg { int m, f; const char *name; };
  const Cfg cfgs[] = {{1, 0, "index + length gather"}, {2, 0, "+ offsets"}, {3, 0, "+ both pieces gathered"},
                      {4, 0, "product pass B"}, {4, 1, "product, no payload stores"}, {4, 2, "product, no assembly"},
                      {4, 3, "product, neither"}, {4, 16, "product, no zeroing"}, {4, 4, "product, ds_or_b64"},
                      {4, 8, "product, nt stores"}, {5, 0, "pair loads in pass B"}, {6, 0, "P0"}, {6, 4, "P0, ds_or_b64"},
                      {7, 0, "pair loads in pass A, kept"}, {7, 1, "  .. no payload stores"}, {7, 2, "  .. no assembly"},
                      {7, 4, "  .. ds_or_b64"}, {7, 8, "  .. nt stores"}, {7, 20, "  .. ds_or_b64, no zeroing"}};
  for (const Cfg &c : cfgs) run(c.m, c.f, c.name);
  return 0;
}
