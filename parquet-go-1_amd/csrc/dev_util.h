// dev_util.h — device helpers shared by the gfx950 kernels (kernels.hip, dict.hip):
// unaligned loads from the padded stage, LSB-first bit extraction, global address-space
// casts, LDS-only workgroup barriers, wave/workgroup scans, error reporting, byte copies.
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/pqgpu.h"
#include "kernels.h"

namespace pq {

#define DEV __device__ __forceinline__

// ---------------------------------------------------------------------------
// Unaligned little-endian loads from the (padded) staging buffer.
// ---------------------------------------------------------------------------
DEV uint32_t ld32(const uint8_t *p) {
  uintptr_t a = (uintptr_t)p;
  const uint32_t *q = (const uint32_t *)(p - (a & 3));  // pointer arithmetic keeps the address space
  uint32_t lo = q[0], hi = q[1];
  return __builtin_amdgcn_alignbyte(hi, lo, (uint32_t)(a & 3));
}
DEV uint64_t ld64(const uint8_t *p) {
  uintptr_t a = (uintptr_t)p;
  const uint32_t *q = (const uint32_t *)(p - (a & 3));
  uint32_t s = (uint32_t)(a & 3);
  uint32_t w0 = q[0], w1 = q[1], w2 = q[2];
  uint32_t lo = __builtin_amdgcn_alignbyte(w1, w0, s);
  uint32_t hi = __builtin_amdgcn_alignbyte(w2, w1, s);
  return ((uint64_t)hi << 32) | lo;
}
// bw (<= 32) bits at bit offset `bo` of stream p, LSB-first (bitpack_gen.go:19-59).
DEV uint32_t bits32(const uint8_t *p, uint64_t bo, uint32_t bw) {
  uint64_t x = ld64(p + (bo >> 3)) >> (bo & 7);
  return bw >= 32 ? (uint32_t)x : (uint32_t)x & ((1u << bw) - 1u);
}
// bw (<= 64) bits at bit offset bo.
DEV uint64_t bits64(const uint8_t *p, uint64_t bo, uint32_t bw) {
  if (bw == 0) return 0;
  const uint8_t *q = p + (bo >> 3);
  uint32_t sh = (uint32_t)(bo & 7);
  uint64_t x = ld64(q) >> sh;
  if (sh && bw > 64 - sh) x |= (uint64_t)q[8] << (64 - sh);
  return bw >= 64 ? x : x & ((1ull << bw) - 1ull);
}

// Same, but bytes at or past the stream end `n` read as zero (the reference's
// bit-packed groups are read with a bare Read into a zeroed buffer: a short final
// group is zero-filled, hybrid_decoder.go:132-140).
DEV uint32_t bits32c(const uint8_t *p, uint32_t n, uint64_t bo, uint32_t bw) {
  uint64_t by = bo >> 3;
  if (by >= n) return 0;
  uint64_t x = ld64(p + by);
  uint64_t avail = n - by;
  if (avail < 8) x &= (1ull << (8 * avail)) - 1ull;
  x >>= (bo & 7);
  return bw >= 32 ? (uint32_t)x : (uint32_t)x & ((1u << bw) - 1u);
}
DEV uint64_t bits64c(const uint8_t *p, uint32_t n, uint64_t bo, uint32_t nb) {  // nb <= 57
  uint64_t by = bo >> 3;
  if (by >= n) return 0;
  uint64_t x = ld64(p + by);
  uint64_t avail = n - by;
  if (avail < 8) x &= (1ull << (8 * avail)) - 1ull;
  x >>= (bo & 7);
  return nb >= 64 ? x : x & ((1ull << nb) - 1ull);
}

DEV uint32_t lane_id() { return __lane_id(); }

// Global-memory pointers. Device addresses travel in descriptors as integers and in BatchDev
// as generic pointers, which compile to FLAT instructions; a FLAT access counts in both vmcnt
// and lgkmcnt, so every LDS wait (lgkmcnt) would also wait for all outstanding loads and
// stores. Casting each pointer's origin to address space 1 lets the compiler emit global_*
// instructions along every use.
#define PQ_GLOBAL __attribute__((address_space(1)))
template <class T>
DEV T *gp(T *p) { return (T *)(PQ_GLOBAL T *)p; }
template <class T>
DEV T *gp_u64(uint64_t a) { return (T *)(PQ_GLOBAL T *)(uintptr_t)a; }
DEV BatchDev global_view(BatchDev b) {
  b.pages = gp(b.pages); b.chunks = gp(b.chunks); b.chunk_err = gp(b.chunk_err);
  b.page_nn = gp(b.page_nn); b.page_nn_v = gp(b.page_nn_v); b.spec_mismatch = gp(b.spec_mismatch);
  b.page_rec = gp(b.page_rec); b.page_vbase = gp(b.page_vbase); b.page_rbase = gp(b.page_rbase);
  b.nest_cnt = gp(b.nest_cnt); b.nest_base = gp(b.nest_base); b.nest_tot = gp(b.nest_tot); b.nest_done = gp(b.nest_done);
  b.runs = gp(b.runs); b.run_base = gp(b.run_base); b.run_count = gp(b.run_count);
  b.tile_first = gp(b.tile_first); b.tile_desc = gp(b.tile_desc); b.tile_base = gp(b.tile_base); b.ba_tile_sum = gp(b.ba_tile_sum);
  b.ba_tile_page = gp(b.ba_tile_page); b.ba_tile_order = gp(b.ba_tile_order);
  b.ba_state = gp(b.ba_state); b.ba_totals = gp(b.ba_totals);
  b.dblk = gp(b.dblk); b.dblk_base = gp(b.dblk_base); b.dblk_n = gp(b.dblk_n); b.dblk_sum = gp(b.dblk_sum);
  b.ba_delta = gp(b.ba_delta);
  b.lv_runs = gp(b.lv_runs); b.lv_run_base = gp(b.lv_run_base); b.lv_meta = gp(b.lv_meta);
  b.lv_tile_run = gp(b.lv_tile_run); b.lv_tile0 = gp(b.lv_tile0);
  if (b.dbg) b.dbg = gp(b.dbg);
  return b;
}

// Workgroup barrier for LDS hand-offs. __syncthreads() is a workgroup-scope release/acquire
// over every address space, so it waits for all of the wave's outstanding global loads and
// stores (vmcnt(0)) before s_barrier: prefetched windows and the previous batch's stores
// would be drained at every barrier. Every barrier in this file orders LDS accesses only
// (global results are never read back by another thread of the same workgroup), so the
// fences are restricted to LDS and only lgkmcnt is waited for.
// LDS writes of this wave visible to its own later LDS reads (no workgroup barrier).
DEV void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
}

DEV void wg_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// Diagnostic phase stamps: per-wave cycle sums added to b.dbg. Compiled in only for the
// diagnostic library (make diag -> lib/libpqgpu_diag.so, -DPQ_DIAG_STAMPS) and active there
// when PQ_DEBUG_STAMPS=1; the production kernels carry no stamp code or registers.
#ifdef PQ_DIAG_STAMPS
DEV uint64_t stamp() { return __builtin_amdgcn_s_memtime(); }
struct Stamps {
  unsigned long long *dbg;
  uint64_t t, acc[8];
  DEV void begin() { if (dbg) t = stamp(); }
  DEV void lap(int k) {
    if (dbg) { uint64_t n = stamp(); acc[k] += n - t; t = n; }
  }
  DEV void flush(int base) {
    if (dbg && __lane_id() == 0)
      for (int k = 0; k < 8; k++) if (acc[k]) atomicAdd(&dbg[base + k], (unsigned long long)acc[k]);
  }
  DEV void count(int k) { if (dbg) acc[k]++; }
  DEV void add(int k, uint64_t v) { if (dbg) acc[k] += v; }
};
#define PQ_STAMPS(name, dbgp) Stamps name{dbgp, 0, {0, 0, 0, 0, 0, 0, 0, 0}}
#define PQ_ABLATE(b, bit) (((b).ablate >> (bit)) & 1u)
#else
#define PQ_ABLATE(b, bit) 0u
struct Stamps {
  DEV void begin() {}
  DEV void lap(int) {}
  DEV void flush(int) {}
  DEV void count(int) {}
  DEV void add(int, uint64_t) {}
};
#define PQ_STAMPS(name, dbgp) Stamps name
#endif
DEV uint32_t rdlane(uint32_t v, uint32_t l) { return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)l); }

DEV uint32_t wave_excl_scan(uint32_t v) {
  uint32_t x = v;
  const uint32_t lane = lane_id();
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint32_t y = __shfl_up(x, d, 64);
    if (lane >= (uint32_t)d) x += y;
  }
  return x - v;
}
DEV uint64_t wave_incl_scan64(uint64_t v) {
  const uint32_t lane = lane_id();
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint64_t y = __shfl_up(v, d, 64);
    if (lane >= (uint32_t)d) v += y;
  }
  return v;
}
// wave64 inclusive prefix sum with DPP row shifts and row broadcasts (GFX9 DPP)
template <int CTRL, int ROWS = 0xf>
DEV uint32_t dpp0(uint32_t x) { return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, ROWS, 0xf, false); }
DEV uint32_t wave_incl_scan32(uint32_t x) {
  x += dpp0<0x111>(x);       // row_shr:1
  x += dpp0<0x112>(x);       // row_shr:2
  x += dpp0<0x114>(x);       // row_shr:4
  x += dpp0<0x118>(x);       // row_shr:8
  x += dpp0<0x142, 0xa>(x);  // row_bcast:15 -> rows 1, 3
  x += dpp0<0x143, 0xc>(x);  // row_bcast:31 -> rows 2, 3
  return x;
}
// wave64 inclusive scan of 64-bit values (wrapping) with DPP row shifts / broadcasts
DEV uint64_t wave_incl_scan64_dpp(uint64_t v) {
  uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
#define PQ_SCAN_STEP(CTRL, ROWS)                                                  \
  {                                                                               \
    const uint32_t l2 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)lo, CTRL, ROWS, 0xf, false); \
    const uint32_t h2 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)hi, CTRL, ROWS, 0xf, false); \
    const uint64_t s = (((uint64_t)hi << 32) | lo) + (((uint64_t)h2 << 32) | l2); \
    lo = (uint32_t)s; hi = (uint32_t)(s >> 32);                                   \
  }
  PQ_SCAN_STEP(0x111, 0xf)
  PQ_SCAN_STEP(0x112, 0xf)
  PQ_SCAN_STEP(0x114, 0xf)
  PQ_SCAN_STEP(0x118, 0xf)
  PQ_SCAN_STEP(0x142, 0xa)
  PQ_SCAN_STEP(0x143, 0xc)
#undef PQ_SCAN_STEP
  return ((uint64_t)hi << 32) | lo;
}

DEV uint64_t wave_sum64(uint64_t v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
  return v;
}

DEV void report(const BatchDev &b, uint32_t chunk, uint32_t phase, uint32_t page, uint32_t stage, uint32_t pos,
                uint32_t code) {
  atomicMin(&b.chunk_err[chunk], (unsigned long long)err_key(phase, page, stage, pos, code));
}

// Byte-range copy dst[0..n) = src[0..n) with arbitrary alignments. The destination is
// walked in 16-B aligned pieces, one per lane; each piece is assembled from the two
// 16-B aligned source blocks that cover it (dwordx4 loads; the second block is the
// next lane's first, so the pair costs no extra HBM traffic) with v_alignbyte funnel
// shifts. Four pieces per lane are kept in flight.
DEV uint4 funnel16(uint4 a, uint4 b, uint32_t s) {  // bytes [s, s+16) of the 32-byte pair (a, b)
  uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
  uint32_t q = s >> 2, r = s & 3;
  uint4 o;
  switch (q) {  // wave-uniform (same source alignment for every lane)
    case 0: o.x = __builtin_amdgcn_alignbyte(w[1], w[0], r); o.y = __builtin_amdgcn_alignbyte(w[2], w[1], r);
            o.z = __builtin_amdgcn_alignbyte(w[3], w[2], r); o.w = __builtin_amdgcn_alignbyte(w[4], w[3], r); break;
    case 1: o.x = __builtin_amdgcn_alignbyte(w[2], w[1], r); o.y = __builtin_amdgcn_alignbyte(w[3], w[2], r);
            o.z = __builtin_amdgcn_alignbyte(w[4], w[3], r); o.w = __builtin_amdgcn_alignbyte(w[5], w[4], r); break;
    case 2: o.x = __builtin_amdgcn_alignbyte(w[3], w[2], r); o.y = __builtin_amdgcn_alignbyte(w[4], w[3], r);
            o.z = __builtin_amdgcn_alignbyte(w[5], w[4], r); o.w = __builtin_amdgcn_alignbyte(w[6], w[5], r); break;
    default: o.x = __builtin_amdgcn_alignbyte(w[4], w[3], r); o.y = __builtin_amdgcn_alignbyte(w[5], w[4], r);
             o.z = __builtin_amdgcn_alignbyte(w[6], w[5], r); o.w = __builtin_amdgcn_alignbyte(w[7], w[6], r); break;
  }
  return o;
}

DEV void copy_bytes(uint8_t *dst, const uint8_t *src, uint64_t n, uint32_t tid, uint32_t nt) {
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
  uint64_t i = tid;
  if (sa == 0) {
    for (; i + 3 * (uint64_t)nt < pieces; i += 4 * (uint64_t)nt) {
      uint4 v0 = sb[i], v1 = sb[i + nt], v2 = sb[i + 2 * nt], v3 = sb[i + 3 * nt];
      d[i] = v0; d[i + nt] = v1; d[i + 2 * nt] = v2; d[i + 3 * nt] = v3;
    }
    for (; i < pieces; i += nt) d[i] = sb[i];
  } else {
    for (; i + 3 * (uint64_t)nt < pieces; i += 4 * (uint64_t)nt) {
      uint4 a0 = sb[i], b0 = sb[i + 1], a1 = sb[i + nt], b1 = sb[i + nt + 1];
      uint4 a2 = sb[i + 2 * nt], b2 = sb[i + 2 * nt + 1], a3 = sb[i + 3 * nt], b3 = sb[i + 3 * nt + 1];
      d[i] = funnel16(a0, b0, sa);
      d[i + nt] = funnel16(a1, b1, sa);
      d[i + 2 * nt] = funnel16(a2, b2, sa);
      d[i + 3 * nt] = funnel16(a3, b3, sa);
    }
    for (; i < pieces; i += nt) d[i] = funnel16(sb[i], sb[i + 1], sa);
  }
  const uint64_t tail = n - head - body;
  if (tid < tail) dst[head + body + tid] = sp[body + tid];
}

// The same with U pieces per lane in flight and one load per piece. Per round the workgroup takes
// nt * U consecutive pieces, wave w the 64 * U of them from w * 64 * U, lane l piece u * 64 + l of
// those (so every store instruction writes 1 KiB contiguous). A lane's second source block is the
// next piece: lane l + 1's block (lane 63: lane 0's next block) by one lane shuffle, and only lane
// 63's last piece loads its own.
#ifndef PQ_COPY_NT
// copy_bytes_u (PLAIN copies) and k_values_delta's transposed output: 2 non-temporal loads and
// stores, 1 stores only, 0 neither. Streams read or written once need no L2 residency; cfg2 step
// 0.478 -> 0.453 ms with 2, 0.464 ms with 1, on one box (profiles/r05_s5_probe_copy_nt.txt)
#define PQ_COPY_NT 2
#endif
typedef uint32_t nt_v4u32 __attribute__((ext_vector_type(4)));
DEV uint4 cp_ld16(const uint4 *p) {
  if (PQ_COPY_NT >= 2) {
    const nt_v4u32 v = __builtin_nontemporal_load((const nt_v4u32 *)p);
    return make_uint4(v.x, v.y, v.z, v.w);
  }
  return *p;
}
DEV void cp_st16(uint4 *p, uint4 v) {
  if (PQ_COPY_NT >= 1) __builtin_nontemporal_store(nt_v4u32{v.x, v.y, v.z, v.w}, (nt_v4u32 *)p);
  else *p = v;
}
// The same store at any 4-B aligned address (gfx950 splits an unaligned 16-B store in the memory
// pipeline; tools/ubench/copy_shapes: 8-B aligned destinations copied at 5.9 TB/s this way against
// 5.3 TB/s with aligned pieces behind dword head stores)
typedef uint32_t nt_v4u32_a4 __attribute__((ext_vector_type(4), aligned(4)));
DEV void cp_st16_ua(uint8_t *p, uint4 v) {
  if (PQ_COPY_NT >= 1) __builtin_nontemporal_store(nt_v4u32_a4{v.x, v.y, v.z, v.w}, (nt_v4u32_a4 *)p);
  else *(nt_v4u32_a4 *)p = nt_v4u32_a4{v.x, v.y, v.z, v.w};
}
template <uint32_t U>
DEV void copy_bytes_u(uint8_t *dst, const uint8_t *src, uint64_t n, uint32_t tid, uint32_t nt) {
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
  uint64_t r0 = 0;
  const uint64_t per = (uint64_t)nt * U;
  for (; r0 + per <= pieces; r0 += per) {
    const uint64_t i = r0 + (uint64_t)wv * 64 * U + lane;
    uint4 a[U];
#pragma unroll
    for (uint32_t u = 0; u < U; u++) a[u] = cp_ld16(&sb[i + 64 * u]);
    if (sa) {
      uint4 e = make_uint4(0u, 0u, 0u, 0u);
      if (lane == 63) e = sb[i + 64 * (U - 1) + 1];
#pragma unroll
      for (uint32_t u = 0; u < U; u++) {
        const uint4 o = (lane == 0 && u + 1 < U) ? a[u + 1] : a[u];  // what lane l - 1 takes from this lane
        uint4 b = make_uint4(shd(o.x), shd(o.y), shd(o.z), shd(o.w));
        if (lane == 63 && u + 1 == U) b = e;
        cp_st16(&d[i + 64 * u], funnel16(a[u], b, sa));
      }
    } else {
#pragma unroll
      for (uint32_t u = 0; u < U; u++) cp_st16(&d[i + 64 * u], a[u]);
    }
  }
  for (uint64_t i = r0 + tid; i < pieces; i += nt) d[i] = sa ? funnel16(sb[i], sb[i + 1], sa) : sb[i];
  const uint64_t tail = n - head - body;
  if (tid < tail) dst[head + body + tid] = sp[body + tid];
}

// Workgroup exclusive scan of one 64-bit value per thread (blockDim.x a multiple of 64;
// wsum: LDS scratch of blockDim.x / 64 entries). *total = the workgroup sum.
DEV uint64_t block_excl_scan64(uint64_t v, uint64_t *wsum, uint64_t *total) {
  const uint32_t lane = lane_id(), wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const uint64_t incl = wave_incl_scan64_dpp(v);
  if (lane == 63) wsum[wv] = incl;
  __syncthreads();
  uint64_t before = 0, tot = 0;
  for (uint32_t q = 0; q < nw; q++) {
    const uint64_t t = wsum[q];
    before += q < wv ? t : 0ull;
    tot += t;
  }
  __syncthreads();
  *total = tot;
  return before + incl - v;
}

// bits at bit offset bo (relative to the stage start) of the LDS stage, width <= 64
DEV uint64_t lds_bits64(const uint32_t *win, uint32_t bo, uint32_t w) {
  if (w == 0) return 0;
  uint32_t wi = bo >> 5, sh = bo & 31;
  uint64_t lo = (uint64_t)win[wi] | ((uint64_t)win[wi + 1] << 32);
  uint64_t x = lo >> sh;
  if (sh && w > 64 - sh) x |= (uint64_t)win[wi + 2] << (64 - sh);
  return w >= 64 ? x : x & ((1ull << w) - 1ull);
}

DEV uint32_t lds_ld32(const uint32_t *stg, uint32_t off) {
  uint32_t w = off >> 2, s = off & 3;
  return __builtin_amdgcn_alignbyte(stg[w + 1], stg[w], s);
}
DEV uint32_t sgpr(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }

// True when page `pd`'s chunk already failed at or before this page (phase 0: a readPages-level
// error — nothing of the chunk is read; phase 1: a readValues error of page k — pages >= k).
DEV bool ba_page_failed(const BatchDev &b, const PageDesc &pd) {
  const unsigned long long key = __hip_atomic_load(&b.chunk_err[pd.chunk], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (key == ~0ull) return false;
  if ((key >> 62) == 0) return true;
  return pd.page_in_chunk >= (uint32_t)((key >> 40) & 0x3fffffu);
}

}  // namespace pq
