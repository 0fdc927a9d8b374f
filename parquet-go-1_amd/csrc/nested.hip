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

// Per tile: how many entries of each counter (lists of levels 1..R, then leaf elements).
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
  for (uint64_t s = x.s0 + threadIdx.x; s < x.s1; s += blockDim.x) {
    const uint32_t r = rl[s], d = slot_def(cd, dl, vb, s);
#pragma unroll
    for (uint32_t j = 0; j < kNestCnt; j++)
      if (j <= R) c[j] += nest_flag(cd, j, r, d);
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

// One wave per chunk: lane j scans counter j over the chunk's tiles.
__global__ void __launch_bounds__(64) k_nest_scan(BatchDev b_in, const uint32_t *chunks) {
  const BatchDev b = global_view(b_in);
  const uint32_t c = chunks[blockIdx.x];
  const ChunkDesc &cd = b.chunks[c];
  const uint32_t j = threadIdx.x;
  if (j >= kNestCnt) return;
  const uint32_t nt = (uint32_t)((cd.num_slots + kNestTile - 1) / kNestTile);
  uint64_t acc = 0;
  for (uint32_t k = 0; k < nt; k++) {
    const uint64_t t = (uint64_t)cd.nest_tile0 + k;
    b.nest_base[t * kNestCnt + j] = acc;
    acc += b.nest_cnt[t * kNestCnt + j];
  }
  b.nest_tot[(uint64_t)c * kNestCnt + j] = acc;
}

// Bitmap writer of one wave over a contiguous range of entries: bits are appended in order and
// whole 32-bit words leave as plain stores (the wave alone owns them); the first and the last
// word of the range may be shared with the neighbouring ranges and are OR-ed atomically.
struct BitRun {
  uint32_t *bm;
  uint64_t word;   // index of the word being filled
  uint32_t acc;    // its bits so far
  uint32_t nbits;  // bits filled (from the word's bit 0)
  bool first;      // the range's first word (shared with the previous range)
  DEV void start(uint32_t *b, uint64_t at) {
    bm = b;
    word = at >> 5;
    nbits = (uint32_t)(at & 31);
    acc = 0;
    first = true;
  }
  DEV void flush_word() {
    if (first) atomicOr(&bm[word], acc);
    else bm[word] = acc;
    first = false;
    ++word;
    acc = 0;
    nbits = 0;
  }
  DEV void append(uint64_t m, uint32_t n) {  // the low n bits of m (n <= 64)
    while (n) {
      const uint32_t take = min(n, 32u - nbits);
      const uint32_t part = (uint32_t)(take == 64 ? m : (m & ((1ull << take) - 1)));
      acc |= part << nbits;
      nbits += take;
      m = take >= 64 ? 0 : m >> take;
      n -= take;
      if (nbits == 32) flush_word();
    }
  }
  DEV void finish() {
    if (nbits) atomicOr(&bm[word], acc);  // shared with the next range
  }
};

// Per tile: wave w owns 1,024 consecutive slots. Pass 1 counts each counter per wave (ballots);
// one barrier gives every wave its first entry index; pass 2 walks the slots again 64 at a time
// with a running index per counter: a level's lists in 64 slots are consecutive entries. Their
// validity bits: each flagged lane writes its bit at its rank into a per-wave LDS row, a ballot
// over the row reads them back packed, and a wave-uniform BitRun appends them to the bitmap.
// List offsets are the child counter's index at the list's first slot. Counter 0 (a level-1
// list starts: rep == 0) also gives the record offsets (ColumnStore.get's record split).
// R: the chunks' list levels (the launch covers the tiles of chunks with nest == R, so every
// per-counter array is indexed by compile-time constants and stays in registers).
template <uint32_t R>
__global__ void __launch_bounds__(256) k_nest_emit(BatchDev b_in, const uint32_t *tile_chunk, uint32_t first) {
  const BatchDev b = global_view(b_in);
  const uint32_t t = first + blockIdx.x;
  const NestTile x = nest_tile(b, tile_chunk, t);
  const ChunkDesc &cd = *x.cd;
  const uint8_t *rl = gp_u64<const uint8_t>(cd.rep_levels);
  const uint8_t *dl = gp_u64<const uint8_t>(cd.def_levels);
  const uint32_t *vb = gp_u64<const uint32_t>(cd.validity);
  int32_t *rec = gp_u64<int32_t>(cd.list_offsets);
  const uint32_t maxd = (uint32_t)cd.max_def;
  __shared__ uint32_t wcnt[R + 1][4];
  __shared__ uint8_t vrow[4][R + 1][64];
  const uint32_t lane = lane_id(), wv = threadIdx.x >> 6;
  const uint64_t lt = (1ull << lane) - 1;
  const uint64_t w0 = x.s0 + (uint64_t)wv * kNestWaveSlots, w1 = min(w0 + kNestWaveSlots, x.s1);
  // the wave's 16 x 64 slots' levels, loaded once (all loads in flight together), packed r | d << 8
  constexpr uint32_t kSteps = kNestWaveSlots / 64;
  uint32_t rd[kSteps];
#pragma unroll
  for (uint32_t k = 0; k < kSteps; k++) {
    const uint64_t sl = w0 + 64 * k + lane;
    rd[k] = sl < w1 ? (uint32_t)rl[sl] | (slot_def(cd, dl, vb, sl) << 8) : 0u;
  }
  // pass 1: this wave's entries per counter
  uint32_t cnt[R + 1] = {};
#pragma unroll
  for (uint32_t k = 0; k < kSteps; k++) {
    const uint64_t sl = w0 + 64 * k + lane;
    const uint32_t r = rd[k] & 0xffu, d = rd[k] >> 8;
#pragma unroll
    for (uint32_t j = 0; j <= R; j++) cnt[j] += (uint32_t)__popcll(__ballot(sl < w1 && nest_flag(cd, j, r, d)));
  }
  if (lane == 0) {
#pragma unroll
    for (uint32_t j = 0; j <= R; j++) wcnt[j][wv] = cnt[j];
  }
  wg_barrier();
  uint64_t run[R + 1];
  BitRun bits[R + 1];
#pragma unroll
  for (uint32_t j = 0; j <= R; j++) {
    uint64_t v = b.nest_base[(uint64_t)t * kNestCnt + j];
    for (uint32_t q = 0; q < wv; q++) v += wcnt[j][q];
    run[j] = v;
    bits[j].start(gp_u64<uint32_t>(j < R ? cd.lvl_validity[j] : cd.elem_validity), v);
  }
  // pass 2
#pragma unroll 1
  for (uint32_t k = 0; k < (PQ_ABLATE(b, 18) ? 0u : kSteps); k++) {  // diagnostic bit 18: no pass 2
    const uint64_t my = w0 + 64 * k + lane;
    if (w0 + 64 * k >= w1) break;  // wave-uniform
    const uint32_t r = rd[k] & 0xffu, d = rd[k] >> 8;
    uint64_t mask[R + 1];
#pragma unroll
    for (uint32_t j = 0; j <= R; j++) {
      mask[j] = __ballot(my < w1 && nest_flag(cd, j, r, d));
      if ((mask[j] >> lane) & 1ull)
        vrow[wv][j][__popcll(mask[j] & lt)] = (uint8_t)(j < R ? d >= cd.list_null_def[j] : d == maxd);
    }
#pragma unroll
    for (uint32_t j = 0; j < R; j++) {
      if (((mask[j] >> lane) & 1ull) && !PQ_ABLATE(b, 16)) {  // diagnostic bit 16: no offset stores
        const uint32_t q = (uint32_t)__popcll(mask[j] & lt);
        const uint32_t qc = (uint32_t)__popcll(mask[j + 1] & lt);  // children before this slot
        gp_u64<int32_t>(cd.lvl_offsets[j])[run[j] + q] = (int32_t)(run[j + 1] + qc);
        if (j == 0 && rec) rec[run[0] + q] = (int32_t)my;  // a record starts at this slot
      }
    }
    wave_lds_sync();
#pragma unroll
    for (uint32_t j = 0; j <= R; j++) {
      const uint32_t m = (uint32_t)__popcll(mask[j]);
      const uint64_t v = __ballot(lane < m && vrow[wv][j][lane]);
      if (!PQ_ABLATE(b, 17)) bits[j].append(v, m);  // diagnostic bit 17: no bitmaps
      run[j] += m;
    }
    wave_lds_sync();
  }
#pragma unroll
  for (uint32_t j = 0; j <= R; j++)
    if (!PQ_ABLATE(b, 17)) bits[j].finish();
  // the chunk's last tile closes every level's offsets and the record offsets
  const uint32_t nt = (uint32_t)((cd.num_slots + kNestTile - 1) / kNestTile);
  if (x.local == nt - 1 && threadIdx.x < R) {
    const uint64_t *tot = b.nest_tot + (uint64_t)x.chunk * kNestCnt;
    gp_u64<int32_t>(cd.lvl_offsets[threadIdx.x])[tot[threadIdx.x]] = (int32_t)tot[threadIdx.x + 1];
    if (threadIdx.x == 0 && rec) rec[tot[0]] = (int32_t)cd.num_slots;
  }
}

hipError_t launch_nest_count(const BatchDev &b, const LaunchLists &l, hipStream_t s) {
  if (!l.n_nest_tiles) return hipSuccess;
  hipLaunchKernelGGL(k_nest_count, dim3(l.n_nest_tiles), dim3(256), 0, s, b, l.nest_tiles);
  return hipGetLastError();
}
hipError_t launch_nest_scan(const BatchDev &b, const LaunchLists &l, hipStream_t s) {
  if (!l.n_nest_chunks) return hipSuccess;
  hipLaunchKernelGGL(k_nest_scan, dim3(l.n_nest_chunks), dim3(64), 0, s, b, l.nest_chunks);
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
