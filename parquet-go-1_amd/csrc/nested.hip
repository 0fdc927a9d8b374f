// nested.hip — Arrow-style nested arrays of a repeated leaf from its decoded levels: for every
// REPEATED node on the leaf's path (list level k, outermost first) the lists' offsets into the
// next level's entries (or, innermost, into the leaf's element slots) and their validity, and the
// leaf elements' validity. This is the step after the hot path that the reference performs as
// record assembly (ColumnStore.get data_store.go:262-309, Column.getData schema.go:216-312: a
// value with rLevel < maxR starts a new object, dLevel < maxD is a null / absent value); here it
// produces the columnar form an Arrow consumer reads instead of per-record Go values.
//
// Per slot (rep r, def d), with D0 = 0, Dk = list_def[k-1] (an element of a level-k list exists
// from Dk on) and Nk = list_null_def[k-1] (the level-k list is non-null from Nk on):
//   a level-k list starts          iff r < k and d >= D(k-1)
//   it is non-null                 iff d >= Nk
//   a level-k list gains a child   iff r <= k and d >= Dk  (= a level-(k+1) list starts; for the
//                                      innermost level, a leaf element slot exists)
//   a leaf element is non-null     iff d == maxD
// Three launches over 4,096-slot tiles of the chunks: counts per tile (k_nest_count), per-chunk
// exclusive scans over tiles (k_nest_scan), then the outputs (k_nest_emit), which also writes the
// chunk's record offsets.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "dev_util.h"

namespace pq {

DEV uint32_t slot_def(const ChunkDesc &cd, const uint8_t *dl, const uint32_t *valid, uint64_t slot) {
  if (dl) return dl[slot];
  if (valid) return (valid[slot >> 5] >> (slot & 31)) & 1u;  // max_def == 1: the bit is the level
  return 0;
}

// Counter j of slot (rep r, def d): j < R: a level-(j+1) list starts; j == R: a leaf element.
DEV bool nest_flag(const ChunkDesc &cd, uint32_t j, uint32_t r, uint32_t d) {
  const uint32_t R = cd.nest;
  if (j < R) return r < j + 1 && d >= (j ? cd.list_def[j - 1] : 0u);
  return d >= cd.list_def[R - 1];
}

constexpr uint32_t kNestTile = 4096;  // slots per tile (a chunk's slots are cut into tiles)
constexpr uint32_t kNestWaveSlots = kNestTile / 4;

struct NestTile {
  const ChunkDesc *cd;
  uint32_t chunk, local;  // tile index within the chunk
  uint64_t s0, s1;        // chunk slots [s0, s1)
};

DEV NestTile nest_tile(const BatchDev &b, const uint32_t *tile_chunk, uint32_t t) {
  NestTile x;
  x.chunk = tile_chunk[t];
  x.cd = &b.chunks[x.chunk];
  x.local = t - x.cd->nest_tile0;
  x.s0 = (uint64_t)x.local * kNestTile;
  x.s1 = min(x.s0 + kNestTile, x.cd->num_slots);
  return x;
}

// Per tile: how many entries of each counter (lists of levels 1..R, then leaf elements). A
// thread takes 16 consecutive slots with one 16-byte load per level array (the level arrays
// are 16-byte padded; a tile starts on a multiple of 4,096 slots).
__global__ void __launch_bounds__(256) k_nest_count(BatchDev b_in, const uint32_t *tile_chunk) {
  const BatchDev b = global_view(b_in);
  const uint32_t t = blockIdx.x;
  const NestTile x = nest_tile(b, tile_chunk, t);
  const ChunkDesc &cd = *x.cd;
  const uint8_t *rl = gp_u64<const uint8_t>(cd.rep_levels);
  const uint8_t *dl = gp_u64<const uint8_t>(cd.def_levels);
  const uint32_t *vb = gp_u64<const uint32_t>(cd.validity);
  __shared__ uint32_t part[kNestCnt][4];
  const uint32_t R = cd.nest, lane = lane_id(), wv = threadIdx.x >> 6;
  uint32_t c[kNestCnt] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  const uint64_t s = x.s0 + 16 * (uint64_t)threadIdx.x;
  if (s < x.s1) {
    const uint32_t ns = (uint32_t)min((uint64_t)16, x.s1 - s);
    const uint4 rv = *reinterpret_cast<const uint4 *>(rl + s);
    uint4 dv = make_uint4(0, 0, 0, 0);
    uint32_t vbits = 0;
    if (dl) dv = *reinterpret_cast<const uint4 *>(dl + s);
    else if (vb) vbits = vb[s >> 5] >> (s & 31);  // max_def == 1: the bit is the level
    const uint32_t rw[4] = {rv.x, rv.y, rv.z, rv.w}, dw[4] = {dv.x, dv.y, dv.z, dv.w};
#pragma unroll
    for (uint32_t q = 0; q < 16; q++) {
      const uint32_t r = (rw[q >> 2] >> (8 * (q & 3))) & 0xffu;
      const uint32_t d = dl ? (dw[q >> 2] >> (8 * (q & 3))) & 0xffu : (vbits >> q) & 1u;
      const bool in = q < ns;
#pragma unroll
      for (uint32_t j = 0; j < kNestCnt; j++)
        if (j <= R) c[j] += in && nest_flag(cd, j, r, d);
    }
  }
#pragma unroll
  for (uint32_t j = 0; j < kNestCnt; j++) {
    const uint32_t v = (uint32_t)wave_sum64(c[j]);
    if (lane == 0) part[j][wv] = v;
  }
  wg_barrier();
  if (threadIdx.x < kNestCnt)
    b.nest_cnt[(uint64_t)t * kNestCnt + threadIdx.x] =
        part[threadIdx.x][0] + part[threadIdx.x][1] + part[threadIdx.x][2] + part[threadIdx.x][3];
}

// One 256-thread workgroup per chunk: thread i takes a contiguous run of the chunk's tiles, sums
// its counters, one workgroup scan per counter gives the run's bases, and a second pass over the
// run writes every tile's base (a chunk of 4 M records has ~5,000 tiles: a serial scan of them
// cost ~0.5 ms).
__global__ void __launch_bounds__(256) k_nest_scan(BatchDev b_in, const uint32_t *chunks) {
  const BatchDev b = global_view(b_in);
  __shared__ uint64_t wsum[4];
  const uint32_t c = chunks[blockIdx.x];
  const ChunkDesc &cd = b.chunks[c];
  const uint32_t nt = (uint32_t)((cd.num_slots + kNestTile - 1) / kNestTile);
  const uint32_t per = (nt + blockDim.x - 1) / blockDim.x;
  const uint32_t k0 = min(nt, threadIdx.x * per), k1 = min(nt, k0 + per);
  const uint32_t *cnt = b.nest_cnt + (uint64_t)cd.nest_tile0 * kNestCnt;
  uint64_t *base = b.nest_base + (uint64_t)cd.nest_tile0 * kNestCnt;
  uint64_t acc[kNestCnt];
#pragma unroll
  for (uint32_t j = 0; j < kNestCnt; j++) acc[j] = 0;
  for (uint32_t k = k0; k < k1; k++)
#pragma unroll
    for (uint32_t j = 0; j < kNestCnt; j++) acc[j] += cnt[(uint64_t)k * kNestCnt + j];
#pragma unroll
  for (uint32_t j = 0; j < kNestCnt; j++) {
    uint64_t tot;
    acc[j] = block_excl_scan64(acc[j], wsum, &tot);
    if (threadIdx.x == 0) b.nest_tot[(uint64_t)c * kNestCnt + j] = tot;
  }
  for (uint32_t k = k0; k < k1; k++)
#pragma unroll
    for (uint32_t j = 0; j < kNestCnt; j++) {
      base[(uint64_t)k * kNestCnt + j] = acc[j];
      acc[j] += cnt[(uint64_t)k * kNestCnt + j];
    }
}

// Bits of x at the positions set in m, packed towards bit 0 (Hacker's Delight 7-4, compress).
DEV uint32_t compress32(uint32_t x, uint32_t m) {
  x &= m;
  uint32_t mk = ~m << 1;
#pragma unroll
  for (uint32_t i = 0; i < 5; i++) {
    uint32_t mp = mk ^ (mk << 1);
    mp ^= mp << 2;
    mp ^= mp << 4;
    mp ^= mp << 8;
    mp ^= mp << 16;
    const uint32_t mv = mp & m;
    m = (m ^ mv) | (mv >> (1u << i));
    const uint32_t t = x & mv;
    x = (x ^ t) | (t >> (1u << i));
    mk &= ~mp;
  }
  return x;
}

// nbits bits of the wave's LDS row (from bit 0) to bitmap bits [off, off + nbits): lane k writes
// destination word k of the range; the first and the last word may be shared with neighbouring
// ranges and are OR-ed atomically, the others are owned and stored.
DEV void nest_put_bits(uint32_t *bm, uint64_t off, const uint32_t *row, uint32_t nbits, uint32_t lane) {
  if (!nbits) return;
  const uint32_t sh = (uint32_t)(off & 31);
  const uint64_t w0 = off >> 5;
  const uint32_t nw = (uint32_t)(((off + nbits + 31) >> 5) - w0);
  for (uint32_t k = lane; k < nw; k += 64) {
    const uint32_t v = (row[k] << sh) | (k && sh ? row[k - 1] >> (32 - sh) : 0u);
    if (k == 0 || k == nw - 1) {
      if (v) atomicOr(&bm[w0 + k], v);
    } else {
      bm[w0 + k] = v;
    }
  }
}

// Per tile: wave w owns 1,024 consecutive slots, lane i sixteen of them (one 16-byte load per
// level array). Per counter j a lane holds the 16-bit mask of its flagged slots; wave prefix
// sums of their counts (and one workgroup exchange of the wave totals) give every entry its
// index. List offsets (the child counter's index at the list's first slot) and record offsets
// (counter 0: a level-1 list starts at rep == 0, ColumnStore.get's record split) are staged in a
// per-wave LDS row in entry order and leave as contiguous stores; the entries' validity bits are
// compressed out of the lane's slot mask, placed at their index in a per-wave LDS bit row and
// written with a funnel shift to their place in the bitmap.
// R: the chunks' list levels (the launch covers the tiles of chunks with nest == R, so every
// per-counter array is indexed by compile-time constants and stays in registers).
template <uint32_t R>
__global__ void __launch_bounds__(256) k_nest_emit(BatchDev b_in, const uint32_t *tile_chunk, uint32_t first) {
  constexpr uint32_t C = R + 1;
  const BatchDev b = global_view(b_in);
  const uint32_t t = first + blockIdx.x;
  const NestTile x = nest_tile(b, tile_chunk, t);
  const ChunkDesc &cd = *x.cd;
  const uint8_t *rl = gp_u64<const uint8_t>(cd.rep_levels);
  const uint8_t *dl = gp_u64<const uint8_t>(cd.def_levels);
  const uint32_t *vb = gp_u64<const uint32_t>(cd.validity);
  int32_t *rec = gp_u64<int32_t>(cd.list_offsets);
  const uint32_t maxd = (uint32_t)cd.max_def;
  __shared__ uint32_t wtot[C][4];
  __shared__ uint32_t ent[4][kNestWaveSlots];
  __shared__ uint32_t brow[4][kNestWaveSlots / 32 + 1];
  const uint32_t lane = lane_id(), wv = threadIdx.x >> 6;
  const uint64_t s = x.s0 + (uint64_t)wv * kNestWaveSlots + 16 * (uint64_t)lane;
  const uint32_t ns = s < x.s1 ? (uint32_t)min((uint64_t)16, x.s1 - s) : 0u;
  uint4 rv = make_uint4(0, 0, 0, 0), dv = make_uint4(0, 0, 0, 0);
  uint32_t vbits = 0;
  if (ns) {
    rv = *reinterpret_cast<const uint4 *>(rl + s);
    if (dl) dv = *reinterpret_cast<const uint4 *>(dl + s);
    else if (vb) vbits = vb[s >> 5] >> (s & 31);  // max_def == 1: the bit is the level
  }
  // the lane's flag and validity masks per counter
  uint32_t f[C], vm[C];
#pragma unroll
  for (uint32_t j = 0; j < C; j++) f[j] = vm[j] = 0;
  {
    const uint32_t rw[4] = {rv.x, rv.y, rv.z, rv.w}, dw[4] = {dv.x, dv.y, dv.z, dv.w};
#pragma unroll
    for (uint32_t q = 0; q < 16; q++) {
      const uint32_t r = (rw[q >> 2] >> (8 * (q & 3))) & 0xffu;
      const uint32_t d = dl ? (dw[q >> 2] >> (8 * (q & 3))) & 0xffu : (vbits >> q) & 1u;
      const uint32_t in = q < ns ? 1u : 0u;
#pragma unroll
      for (uint32_t j = 0; j < C; j++) {
        f[j] |= (in & (uint32_t)nest_flag(cd, j, r, d)) << q;
        vm[j] |= (uint32_t)(j < R ? d >= cd.list_null_def[j] : d == maxd) << q;
      }
    }
  }
  // entry indices: wave prefix sums, then the waves before this one in the tile
  uint32_t P[C], T[C];
#pragma unroll
  for (uint32_t j = 0; j < C; j++) {
    const uint32_t c = (uint32_t)__popc(f[j]);
    const uint32_t incl = (uint32_t)wave_incl_scan64_dpp(c);
    P[j] = incl - c;
    T[j] = (uint32_t)__shfl(incl, 63);
    if (lane == 0) wtot[j][wv] = T[j];
  }
  wg_barrier();
  uint64_t run[C];
#pragma unroll
  for (uint32_t j = 0; j < C; j++) {
    uint64_t v = b.nest_base[(uint64_t)t * kNestCnt + j];
    for (uint32_t q = 0; q < wv; q++) v += wtot[j][q];
    run[j] = v;
  }
  uint32_t *row = ent[wv];
  // list offsets of each level, then the record offsets (level-1 list starts)
#pragma unroll
  for (uint32_t j = 0; j <= R; j++) {
    const uint32_t lv = j < R ? j : 0;  // j == R: record offsets
    if (j == R && !rec) break;
    if (PQ_ABLATE(b, 16)) break;  // diagnostic bit 16: no offset stores
    uint32_t m = f[lv], k = P[lv];
    const uint32_t cb = (uint32_t)(run[lv + 1] + P[lv + 1]);  // children before this lane's slots
    while (m) {
      const uint32_t i = __builtin_ctz(m);
      m &= m - 1;
      row[k++] = j < R ? cb + (uint32_t)__popc(f[lv + 1] & ((1u << i) - 1u)) : (uint32_t)(s + i);
    }
    wave_lds_sync();
    int32_t *dst = j < R ? gp_u64<int32_t>(cd.lvl_offsets[j]) + run[j] : rec + run[0];
    for (uint32_t e = lane; e < T[lv]; e += 64) dst[e] = (int32_t)row[e];
    wave_lds_sync();
  }
  // validity bits of every counter's entries
  uint32_t *bits = brow[wv];
#pragma unroll
  for (uint32_t j = 0; j < C; j++) {
    if (PQ_ABLATE(b, 17)) break;  // diagnostic bit 17: no bitmaps
    if (lane <= kNestWaveSlots / 32) bits[lane] = 0;
    wave_lds_sync();
    const uint32_t c = (uint32_t)__popc(f[j]);
    if (c) {
      const uint32_t comp = compress32(vm[j], f[j]), p = P[j], sh = p & 31;
      atomicOr(&bits[p >> 5], comp << sh);
      if (sh && sh + c > 32) atomicOr(&bits[(p >> 5) + 1], comp >> (32 - sh));
    }
    wave_lds_sync();
    nest_put_bits(gp_u64<uint32_t>(j < R ? cd.lvl_validity[j] : cd.elem_validity), run[j], bits, T[j], lane);
    wave_lds_sync();
  }
  // struct validity of the OPTIONAL groups that own a bitmap (Column.getNextData schema.go:216-260:
  // a group is non-nil iff a child is defined at or below it, def >= group_def): its entries are
  // those of counter group_depth (the level-(depth + 1) lists, or the leaf's element slots), so the
  // bits go where that counter's validity goes
  for (uint32_t g = 0; g < cd.ngroups; g++) {
    uint32_t *gv = gp_u64<uint32_t>(cd.group_validity[g]);
    if (!gv) continue;  // shares list / element validity (workgroup-uniform)
    const uint32_t j = cd.group_depth[g], dg = cd.group_def[g];
    uint32_t fj = 0, pj = 0, tj = 0;
    uint64_t rj = 0;
#pragma unroll
    for (uint32_t q = 0; q < C; q++)  // selects: a dynamic index would put the arrays in scratch
      if (q == j) { fj = f[q]; pj = P[q]; tj = T[q]; rj = run[q]; }
    uint32_t vg = 0;
    {
      const uint32_t dw[4] = {dv.x, dv.y, dv.z, dv.w};
#pragma unroll
      for (uint32_t q = 0; q < 16; q++) {
        const uint32_t d = dl ? (dw[q >> 2] >> (8 * (q & 3))) & 0xffu : (vbits >> q) & 1u;
        vg |= (uint32_t)(d >= dg) << q;
      }
    }
    if (lane <= kNestWaveSlots / 32) bits[lane] = 0;
    wave_lds_sync();
    const uint32_t c = (uint32_t)__popc(fj);
    if (c) {
      const uint32_t comp = compress32(vg, fj), sh = pj & 31;
      atomicOr(&bits[pj >> 5], comp << sh);
      if (sh && sh + c > 32) atomicOr(&bits[(pj >> 5) + 1], comp >> (32 - sh));
    }
    wave_lds_sync();
    nest_put_bits(gv, rj, bits, tj, lane);
    wave_lds_sync();
  }
  // the chunk's last tile closes every level's offsets and the record offsets
  const uint32_t nt = (uint32_t)((cd.num_slots + kNestTile - 1) / kNestTile);
  if (x.local == nt - 1 && threadIdx.x < R) {
    const uint64_t *tot = b.nest_tot + (uint64_t)x.chunk * kNestCnt;
    gp_u64<int32_t>(cd.lvl_offsets[threadIdx.x])[tot[threadIdx.x]] = (int32_t)tot[threadIdx.x + 1];
    if (threadIdx.x == 0 && rec) rec[tot[0]] = (int32_t)cd.num_slots;
  }
}

// Struct validity of the OPTIONAL groups of a leaf with max_rep == 0: entries are the leaf's slots,
// bit s = def[s] >= group_def (u8 definition levels: max_def > 1 whenever such a group owns a
// bitmap). One thread per 32 slots, one word per group; tiles start on multiples of kGrpTile slots.
constexpr uint32_t kGrpTile = kGrpTileHost;
__global__ void __launch_bounds__(256) k_group_flat(BatchDev b_in, const uint32_t *tiles) {
  const BatchDev b = global_view(b_in);
  const uint32_t c = gp(tiles)[blockIdx.x];
  const ChunkDesc &cd = b.chunks[c];
  const uint64_t s = (uint64_t)(blockIdx.x - cd.grp_tile0) * kGrpTile + 32 * (uint64_t)threadIdx.x;
  if (s >= cd.num_slots) return;
  const uint32_t ns = (uint32_t)min((uint64_t)32, cd.num_slots - s);
  const uint8_t *dl = gp_u64<const uint8_t>(cd.def_levels) + s;
  uint32_t w[8];
  if (ns == 32) {
    const uint4 a = *reinterpret_cast<const uint4 *>(dl), b2 = *reinterpret_cast<const uint4 *>(dl + 16);
    w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w; w[4] = b2.x; w[5] = b2.y; w[6] = b2.z; w[7] = b2.w;
  } else {
#pragma unroll
    for (uint32_t k = 0; k < 8; k++) w[k] = 0;
    for (uint32_t q = 0; q < ns; q++) w[q >> 2] |= (uint32_t)dl[q] << (8 * (q & 3));
  }
  for (uint32_t g = 0; g < cd.ngroups; g++) {
    uint32_t *gv = gp_u64<uint32_t>(cd.group_validity[g]);
    if (!gv) continue;
    const uint32_t dg = cd.group_def[g];
    uint32_t bitsw = 0;
#pragma unroll
    for (uint32_t q = 0; q < 32; q++) bitsw |= (uint32_t)(((w[q >> 2] >> (8 * (q & 3))) & 0xffu) >= dg) << q;
    if (ns < 32) bitsw &= (1u << ns) - 1u;
    gv[s >> 5] = bitsw;
  }
}

__global__ void __launch_bounds__(256) k_words_differ(const uint32_t *a_in, const uint32_t *b_in, uint64_t n,
                                                      uint32_t *flag) {
  const uint32_t *a = gp(a_in), *b = gp(b_in);
  bool d = false;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    d |= a[i] != b[i];
  if (__ballot(d) && lane_id() == 0) atomicOr(gp(flag), 1u);
}
hipError_t launch_words_differ(const uint32_t *a, const uint32_t *b, uint64_t n, uint32_t *flag, hipStream_t s) {
  if (!n) return hipSuccess;
  const uint32_t grid = (uint32_t)std::min<uint64_t>(2048, (n + 255) / 256);
  hipLaunchKernelGGL(k_words_differ, dim3(grid), dim3(256), 0, s, a, b, n, flag);
  return hipGetLastError();
}

hipError_t launch_group_flat(const BatchDev &b, const LaunchLists &l, hipStream_t s) {
  if (!l.n_grp_tiles) return hipSuccess;
  hipLaunchKernelGGL(k_group_flat, dim3(l.n_grp_tiles), dim3(256), 0, s, b, l.grp_tiles);
  return hipGetLastError();
}

hipError_t launch_nest_count(const BatchDev &b, const LaunchLists &l, hipStream_t s) {
  if (!l.n_nest_tiles) return hipSuccess;
  hipLaunchKernelGGL(k_nest_count, dim3(l.n_nest_tiles), dim3(256), 0, s, b, l.nest_tiles);
  return hipGetLastError();
}
hipError_t launch_nest_scan(const BatchDev &b, const LaunchLists &l, hipStream_t s) {
  if (!l.n_nest_chunks) return hipSuccess;
  hipLaunchKernelGGL(k_nest_scan, dim3(l.n_nest_chunks), dim3(256), 0, s, b, l.nest_chunks);
  return hipGetLastError();
}
template <uint32_t R>
static void launch_emit_r(const BatchDev &b, const LaunchLists &l, hipStream_t s) {
  const uint32_t n = l.nest_first[R + 1] - l.nest_first[R];
  if (n) hipLaunchKernelGGL(k_nest_emit<R>, dim3(n), dim3(256), 0, s, b, l.nest_tiles, l.nest_first[R]);
}
hipError_t launch_nest_emit(const BatchDev &b, const LaunchLists &l, hipStream_t s) {
  if (!l.n_nest_tiles) return hipSuccess;
  // tiles are grouped by list levels (host.cpp): one instantiation per group
  launch_emit_r<1>(b, l, s);
  launch_emit_r<2>(b, l, s);
  launch_emit_r<3>(b, l, s);
  launch_emit_r<4>(b, l, s);
  launch_emit_r<5>(b, l, s);
  launch_emit_r<6>(b, l, s);
  launch_emit_r<7>(b, l, s);
  launch_emit_r<8>(b, l, s);
  return hipGetLastError();
}

}  // namespace pq
