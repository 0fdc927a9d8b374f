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
// Three launches over the fill tiles of the chunks' pages (level_fill.h: kLfTile slots aligned on
// the chunk's slot index, one per page that holds slots of it), each cut into two 4,096-slot
// halves: counts per half (k_nest_count, whose last tile per chunk scans the chunk's halves),
// then the outputs (k_nest_emit): u8 levels, slot validity, list / record offsets and bitmaps.
// Both tile kernels expand the two level streams from the run tables the level kernels wrote
// (reading the compressed streams, ~0.4 B per slot) and keep the levels of their slots in
// registers: no level array is read back.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "dev_util.h"
#include "level_fill.h"

namespace pq {

// Counter j of slot (rep r, def d): j < R: a level-(j+1) list starts; j == R: a leaf element.
DEV bool nest_flag(const ChunkDesc &cd, uint32_t j, uint32_t r, uint32_t d) {
  const uint32_t R = cd.nest;
  if (j < R) return r < j + 1 && d >= (j ? cd.list_def[j - 1] : 0u);
  return d >= cd.list_def[R - 1];
}

constexpr uint32_t kNestHalf = 4096;               // slots per counting unit (half a fill tile)
constexpr uint32_t kNestWaveSlots = kNestHalf / 4;  // a wave's slots of a half (16 per lane)
static_assert(2 * kNestHalf == kLfTile, "a fill tile is two counting units");

// The fill tile of a nested tile descriptor (host-built, so the kernels start from one load:
// {global fill tile t, page, tile k of the page, chunk}): the page's slots [lo, hi) it covers,
// t0 = the page value index of its first (aligned) slot.
struct NestFill {
  uint32_t t, pi, k, chunk, lo, hi, ntiles;
  int64_t t0;
  uint64_t sbase;
};
DEV NestFill nest_fill(const BatchDev &b, uint4 d) {
  NestFill x;
  x.t = d.x;
  x.pi = d.y;
  x.k = d.z;
  x.chunk = d.w;
  const PageDesc &pd = b.pages[x.pi];
  x.sbase = pd.slot_base;
  const uint32_t ns = pd.num_slots, a = (uint32_t)(x.sbase & (kLfTile - 1));
  x.ntiles = lf_tiles(x.sbase, ns);
  x.t0 = (int64_t)x.k * kLfTile - a;
  x.lo = (uint32_t)max(x.t0, (int64_t)0);
  x.hi = (uint32_t)min(x.t0 + kLfTile, (int64_t)ns);
  return x;
}

// One level stream of a fill tile: its runs from the one holding the tile's first value, staged
// in LDS (`L`, kNfRuns entries) when they fit; `end`: the tile's values the stream covers end
// there (a failed stream covers none). Workgroup-uniform; the caller synchronises after it.
constexpr uint32_t kNfRuns = 1024;          // runs per stream staged by the nested tile kernels
constexpr uint32_t kNfGroups = kLfTile / 8;  // groups of eight values per fill tile
struct LfStream {
  const uint2 *runs;
  const uint8_t *src;
  uint32_t m, n, bw, cmp, end;
  bool staged, on;
};
DEV LfStream lf_stream(const BatchDev &b, const PageDesc &pd, const ChunkDesc &cd, const NestFill &x, uint32_t which,
                       uint2 *L, uint32_t tid) {
  LfStream S;
  const bool rep = which == 0;
  S.on = false;
  S.end = x.lo;
  S.m = 0;
  S.staged = false;
  S.runs = nullptr;
  S.src = nullptr;
  S.n = S.bw = S.cmp = 0;
  if (rep ? cd.max_rep == 0 : cd.max_def == 0) return S;
  const uint32_t nr = b.lv_meta[4 * x.pi + 2 * which], cov = b.lv_meta[4 * x.pi + 2 * which + 1];
  S.end = min(x.hi, cov);
  if (x.lo >= S.end || nr == 0) {
    S.end = x.lo;
    return S;
  }
  const uint2 *runs = b.lv_runs + b.lv_run_base[2 * x.pi + which];
  const uint32_t *trun = b.lv_tile_run + 2 * (uint64_t)x.t + which;
  const uint32_t r0 = trun[0];
  const bool more = x.k + 1 < x.ntiles && x.t0 + (int64_t)kLfTile < (int64_t)cov;
  S.m = (more ? trun[2] : nr - 1) - r0 + 1;
  S.runs = runs + r0;
  S.staged = S.m <= kNfRuns;
  if (S.staged)
    for (uint32_t i = tid; i < S.m; i += 256) L[i] = S.runs[i];
  S.src = gp_u64<const uint8_t>(pd.data) + (rep ? pd.rep_off : pd.def_off);
  S.n = rep ? pd.rep_len : pd.def_len;
  S.bw = (uint32_t)(rep ? cd.rep_bw : cd.def_bw);
  S.cmp = rep ? 0u : (uint32_t)cd.max_def;
  S.on = true;
  return S;
}
// Thread tid's group q (q = 2 h + e) of a fill tile: 16 consecutive slots per thread and half;
// its index among the tile's groups is h * 512 + 2 tid + e.
DEV int64_t nest_group(const NestFill &x, uint32_t tid, uint32_t q) {
  return x.t0 + (int64_t)((q >> 1) * kNestHalf + 16 * tid + 8 * (q & 1));
}
// Mask of the slots [g, g + n) that lie in [lo, end)
DEV uint32_t nest_inmask(int64_t g, uint32_t n, uint32_t lo, uint32_t end) {
  const int64_t vs = max(g, (int64_t)lo), ve = min(g + (int64_t)n, (int64_t)end);
  return vs < ve ? (uint32_t)(((1ull << (ve - vs)) - 1ull) << (vs - g)) : 0u;
}
DEV uint32_t wave_incl_max(uint32_t v, uint32_t lane) {
#pragma unroll
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const uint32_t o = __shfl_up(v, d);
    if (lane >= d) v = max(v, o);
  }
  return v;
}

// LDS of the expansion: both streams' staged runs and, per group of the tile, the last run that
// starts at or before the group (marked by the runs, then a workgroup prefix maximum), so that a
// group finds its run with one LDS read instead of a binary search.
struct NestStage {
  uint2 run[2][kNfRuns];
  uint16_t grun[2][kNfGroups];
  uint32_t wmax[2][2][4];
  uint32_t cnt[2][4];
};

// Both streams of the thread's four groups expanded: lw[0] repetition, lw[1] definition levels
// (bytes), eqd[q] the groups' definition == max_def masks; the u8 level arrays the chunk has are
// written and the pages' counts (records, non-null values) added once per tile.
DEV void nest_expand(const BatchDev &b, const PageDesc &pd, const ChunkDesc &cd, const NestFill &x, NestStage &T,
                     uint32_t tid, uint64_t (&lw)[2][4], uint32_t (&eqd)[4], uint32_t &end_d, Stamps &st,
                     bool count_pages = true) {
  const uint32_t lane = lane_id(), wv = tid >> 6;
  LfStream S[2];
  S[0] = lf_stream(b, pd, cd, x, 0, T.run[0], tid);
  S[1] = lf_stream(b, pd, cd, x, 1, T.run[1], tid);
  end_d = S[1].end;
  reinterpret_cast<uint2 *>(T.grun[0])[tid] = make_uint2(0, 0);
  reinterpret_cast<uint2 *>(T.grun[1])[tid] = make_uint2(0, 0);
  wg_barrier();
  st.lap(0);
  // run r > 0 starts in group ceil((x_r - t0) / 8) at the latest: the groups from there on begin in
  // it or later; of the runs that mark one group the last one writes (no atomics)
#pragma unroll
  for (uint32_t w = 0; w < 2; w++)
    if (S[w].staged)
      for (uint32_t r = 1 + tid; r < S[w].m; r += 256) {
        const int64_t gs = ((int64_t)T.run[w][r].x - x.t0 + 7) >> 3;
        const int64_t gn = r + 1 < S[w].m ? ((int64_t)T.run[w][r + 1].x - x.t0 + 7) >> 3 : (int64_t)kNfGroups;
        if (gs > 0 && gs < (int64_t)kNfGroups && gn != gs) T.grun[w][gs] = (uint16_t)r;
      }
  wg_barrier();
  // prefix maximum in group order: the thread's groups 2 tid, 2 tid + 1 (first half), 512 + 2 tid, + 1
  uint32_t e[2][4], ex[2][2];
#pragma unroll
  for (uint32_t w = 0; w < 2; w++) {
    const uint32_t p0 = reinterpret_cast<const uint32_t *>(T.grun[w])[tid];
    const uint32_t p1 = reinterpret_cast<const uint32_t *>(T.grun[w] + kNfGroups / 2)[tid];
    e[w][0] = p0 & 0xffffu; e[w][1] = max(p0 & 0xffffu, p0 >> 16); e[w][2] = p1 & 0xffffu; e[w][3] = max(p1 & 0xffffu, p1 >> 16);
#pragma unroll
    for (uint32_t h = 0; h < 2; h++) {
      const uint32_t incl = wave_incl_max(e[w][2 * h + 1], lane);
      const uint32_t prev = __shfl_up(incl, 1);
      ex[w][h] = lane ? prev : 0u;
      if (lane == 63) T.wmax[w][h][wv] = incl;
    }
  }
  wg_barrier();
#pragma unroll
  for (uint32_t w = 0; w < 2; w++) {
    uint32_t before0 = 0, before1 = 0, tot0 = 0;
#pragma unroll
    for (uint32_t q = 0; q < 4; q++) {
      tot0 = max(tot0, T.wmax[w][0][q]);
      if (q < wv) { before0 = max(before0, T.wmax[w][0][q]); before1 = max(before1, T.wmax[w][1][q]); }
    }
    const uint32_t c0 = max(before0, ex[w][0]), c1 = max(tot0, max(before1, ex[w][1]));
    e[w][0] = max(e[w][0], c0); e[w][1] = max(e[w][1], c0);
    e[w][2] = max(e[w][2], c1); e[w][3] = max(e[w][3], c1);
  }
  st.lap(1);
  uint32_t nc[2] = {0, 0};
#pragma unroll
  for (uint32_t w = 0; w < 2; w++) {
    const LfStream &Sw = S[w];
    uint8_t *out = gp_u64<uint8_t>(w ? cd.def_levels : cd.rep_levels);
#pragma unroll
    for (uint32_t q = 0; q < 4; q++) {
      const int64_t g = nest_group(x, tid, q);
      uint64_t word = 0;
      uint32_t eq = 0;
      const uint32_t vs = (uint32_t)max(g, (int64_t)x.lo), ve = (uint32_t)max(min(g + 8, (int64_t)Sw.end), (int64_t)vs);
      if (Sw.on && !PQ_ABLATE(b, 18)) {
        if (Sw.staged)
          lf_group_from([&](uint32_t i) { return T.run[w][i]; }, Sw.m, e[w][q], Sw.src, Sw.n, Sw.bw, Sw.cmp, g, vs, ve, word, eq);
        else
          lf_group([&](uint32_t i) { return Sw.runs[i]; }, Sw.m, Sw.src, Sw.n, Sw.bw, Sw.cmp, g, vs, ve, word, eq);
      }
      lw[w][q] = word;
      if (w) eqd[q] = eq;
      nc[w] += __popc(eq);
      if (out && vs < ve) {
        uint8_t *o = out + x.sbase;
        if (vs == g && ve == g + 8 && !(reinterpret_cast<uintptr_t>(o + g) & 7))
          *reinterpret_cast<uint2 *>(o + g) = make_uint2((uint32_t)word, (uint32_t)(word >> 32));
        else
          for (uint32_t v = vs; v < ve; v++) o[v] = (uint8_t)(word >> (8 * (v - (uint32_t)g)));
      }
    }
  }
  st.lap(2);
#pragma unroll
  for (uint32_t w = 0; w < 2; w++) {  // page counts: one atomic per tile and stream
    const uint32_t wc = (uint32_t)wave_sum64(nc[w]);
    if (lane == 0) T.cnt[w][wv] = wc;
  }
  wg_barrier();  // cnt complete
  if (count_pages && tid < 2 && (tid ? S[1].on : S[0].on)) {
    const uint32_t c = T.cnt[tid][0] + T.cnt[tid][1] + T.cnt[tid][2] + T.cnt[tid][3];
    if (c) atomicAdd(tid ? &b.page_nn[x.pi] : &b.page_rec[x.pi], c);
  }
  st.lap(3);
}

// A chunk's scan by one 256-thread workgroup: thread i takes a contiguous run of the chunk's
// counting units (two per fill tile), sums its counters, one workgroup scan per counter gives the
// run's bases, and a second pass over the run writes every unit's base. The chunk's totals close
// every level's offsets and the record offsets. Run by the chunk's last tile of k_nest_count to
// finish (k_nest_scan: chunks without tiles).
DEV void nest_scan_chunk(const BatchDev &b, uint32_t c, uint64_t *wsum) {
  const ChunkDesc &cd = b.chunks[c];
  const uint32_t nt = 2 * cd.nest_ntiles;
  const uint32_t per = (nt + blockDim.x - 1) / blockDim.x;
  const uint32_t k0 = min(nt, threadIdx.x * per), k1 = min(nt, k0 + per);
  uint32_t *cnt = b.nest_cnt + 2 * (uint64_t)cd.nest_tile0 * kNestCnt;  // (published by atomics)
  uint64_t *base = b.nest_base + 2 * (uint64_t)cd.nest_tile0 * kNestCnt;
  const uint32_t C = cd.nest + 1;  // counters in use (lists of levels 1..R, elements)
  uint64_t acc[kNestCnt], tot[kNestCnt];
#pragma unroll
  for (uint32_t j = 0; j < kNestCnt; j++) acc[j] = 0;
  for (uint32_t k = k0; k < k1; k++)
#pragma unroll
    for (uint32_t j = 0; j < kNestCnt; j++)
      if (j < C) acc[j] += __hip_atomic_load(&cnt[(uint64_t)k * kNestCnt + j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
  for (uint32_t j = 0; j < kNestCnt; j++) {
    tot[j] = 0;
    if (j < C) {  // workgroup-uniform
      acc[j] = block_excl_scan64(acc[j], wsum, &tot[j]);
      if (threadIdx.x == 0) b.nest_tot[(uint64_t)c * kNestCnt + j] = tot[j];
    }
  }
  for (uint32_t k = k0; k < k1; k++)
#pragma unroll
    for (uint32_t j = 0; j < kNestCnt; j++)
      if (j < C) {
        base[(uint64_t)k * kNestCnt + j] = acc[j];
        acc[j] += __hip_atomic_load(&cnt[(uint64_t)k * kNestCnt + j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
  // closing entries: offsets[num_lists] = the next level's entries (elements), records -> slots
  int32_t *rec = gp_u64<int32_t>(cd.list_offsets);
#pragma unroll
  for (uint32_t j = 0; j + 1 < kNestCnt; j++)
    if (threadIdx.x == j && j < cd.nest) gp_u64<int32_t>(cd.lvl_offsets[j])[tot[j]] = (int32_t)tot[j + 1];
  if (threadIdx.x == 0 && rec) rec[tot[0]] = (int32_t)cd.num_slots;
}

__global__ void __launch_bounds__(256) k_nest_scan(BatchDev b_in, const uint32_t *chunks) {
  const BatchDev b = global_view(b_in);
  __shared__ uint64_t wsum[4];
  nest_scan_chunk(b, chunks[blockIdx.x], wsum);
}

// The nested pages' counts from the level run tables alone: records (repetition level 0) and
// non-null values (definition level max_def) among the slots each stream covers — the counts
// k_nest_count / k_nest_tile otherwise add while expanding, so that k_bases (value and record bases:
// ColumnStore.readNextPage's per-page split) does not wait for the nested arrays. One workgroup per
// page: threads 0-127 the repetition stream, 128-255 the definition stream, a run per thread and
// step; RLE runs count whole, bit-packed runs 64 bits at a time (fields equal to the level by SWAR).
__global__ void __launch_bounds__(256) k_nest_pcount(BatchDev b_in, const uint32_t *pages) {
  const BatchDev b = global_view(b_in);
  __shared__ uint32_t part[4];
  const uint32_t pi = gp(pages)[blockIdx.x], tid = threadIdx.x, w = tid >> 7, t = tid & 127;
  const PageDesc &pd = b.pages[pi];
  const ChunkDesc &cd = b.chunks[pd.chunk];
  const uint32_t nr = b.lv_meta[4 * pi + 2 * w], cov = b.lv_meta[4 * pi + 2 * w + 1];
  const uint32_t end = min(cov, pd.num_slots);
  const uint32_t bw = w ? (uint32_t)cd.def_bw : (uint32_t)cd.rep_bw, cmp = w ? (uint32_t)cd.max_def : 0u;
  const bool on = (w ? cd.max_def : cd.max_rep) != 0;
  uint32_t c = 0;
  if (on && nr && end && bw) {
    const uint2 *runs = b.lv_runs + b.lv_run_base[2 * pi + w];
    const uint8_t *src = gp_u64<const uint8_t>(pd.data) + (w ? pd.def_off : pd.rep_off);
    const uint32_t n = w ? pd.def_len : pd.rep_len;
    const uint32_t k = 56 / bw;  // fields per 64-bit read (bw <= 8: k >= 7)
    uint64_t lo = 0, rc = 0;     // the field pattern: bit 0 of every field; the level in every field
    for (uint32_t i = 0; i < k; i++) { lo |= 1ull << (i * bw); }
    rc = lo * cmp;
    for (uint32_t r = t; r < nr; r += 128) {
      const uint2 run = runs[r];
      const uint32_t x0 = run.x, x1 = min(r + 1 < nr ? runs[r + 1].x : end, end);
      if (x0 >= x1) continue;
      if (!(run.y >> 31)) {  // RLE
        c += run.y == cmp ? x1 - x0 : 0u;
        continue;
      }
      const uint64_t pb = (uint64_t)(run.y & 0x7fffffffu) * 8;
      for (uint32_t v = x0; v < x1; v += k) {
        const uint32_t m = min(k, x1 - v);
        const uint64_t y = bits64c(src, n, pb + (uint64_t)(v - x0) * bw, m * bw) ^ (rc & ((m * bw >= 64) ? ~0ull : ((1ull << (m * bw)) - 1ull)));
        uint64_t z = y;  // a field is zero (equal to the level) iff no bit of it is set
        for (uint32_t q = 1; q < bw; q++) z |= y >> q;
        const uint64_t fm = lo & ((m * bw >= 64) ? ~0ull : ((1ull << (m * bw)) - 1ull));
        c += (uint32_t)__popcll(~z & fm);
      }
    }
  }
  c = (uint32_t)wave_sum64(c);
  if (lane_id() == 0) part[tid >> 6] = c;
  wg_barrier();
  if (tid == 0) {
    if (cd.max_rep) b.page_rec[pi] = part[0] + part[1];
    b.page_nn[pi] = part[2] + part[3];
  }
}

// The slots' flag masks, 32 bits per thread (bits 8q..8q+7: group q; 0-15 the first half's sixteen
// slots, 16-31 the second's), from the thread's expanded levels lw: kind 0, the slots where counter j
// counts (a level-(j+1) list starts, j < R; a leaf element slot, j == R); kind 1, the validity of
// those entries (list j non-null; the element non-null); kind 2, group g's validity (def >=
// group_def). Eight levels per 64-bit word are compared at once (SWAR: levels below 128; wider
// levels take the byte loop).
template <uint32_t R>
DEV uint32_t nest_mask(const ChunkDesc &cd, const uint64_t (&lw)[2][4], bool swar, uint32_t kind, uint32_t j, uint32_t g) {
  constexpr uint64_t H = 0x8080808080808080ull, L1 = 0x0101010101010101ull;
  auto ge = [&](uint64_t v, uint32_t t) -> uint64_t { return ((v | H) - L1 * t) & H; };  // bytes v >= t
  auto pack8 = [](uint64_t hx) -> uint32_t {  // the high bits of the eight bytes, in byte order
    const uint32_t lo = (uint32_t)hx >> 7, hi = (uint32_t)(hx >> 32) >> 7;
    return ((lo * 0x01020408u) >> 24) | (((hi * 0x01020408u) >> 24) << 4);
  };
  uint32_t m = 0;
  if (swar) {
#pragma unroll
    for (uint32_t q = 0; q < 4; q++) {
      const uint64_t rw = lw[0][q], dw = lw[1][q];
      uint64_t f;
      if (kind == 0) f = j < R ? ge(dw, j ? cd.list_def[j - 1] : 0u) & ~ge(rw, j + 1) : ge(dw, cd.list_def[R - 1]);
      else if (kind == 1) f = j < R ? ge(dw, cd.list_null_def[j]) : ge(dw, cd.max_def) & ~ge(dw, cd.max_def + 1);
      else f = ge(dw, cd.group_def[g]);
      m |= pack8(f) << (8 * q);
    }
  } else {
#pragma unroll 1
    for (uint32_t i = 0; i < 32; i++) {
      const uint32_t r = (uint32_t)(lw[0][i >> 3] >> (8 * (i & 7))) & 0xffu, d = (uint32_t)(lw[1][i >> 3] >> (8 * (i & 7))) & 0xffu;
      const bool bit = kind == 0 ? nest_flag(cd, j, r, d)
                       : kind == 1 ? (j < R ? d >= cd.list_null_def[j] : d == (uint32_t)cd.max_def)
                                   : d >= cd.group_def[g];
      m |= (uint32_t)bit << i;
    }
  }
  return m;
}
// The thread's slots that both level streams cover (a failing stream covers none past its error).
DEV uint32_t nest_cover_mask(const BatchDev &b, const PageDesc &pd, const ChunkDesc &cd, const NestFill &x, uint32_t tid) {
  const uint32_t cov_r = b.lv_meta[4 * x.pi + 1], cov_d = cd.max_def ? b.lv_meta[4 * x.pi + 3] : pd.num_slots;
  const uint32_t endc = min(x.hi, min(cov_r, cov_d));
  uint32_t inm = 0;
#pragma unroll
  for (uint32_t q = 0; q < 4; q++) inm |= nest_inmask(nest_group(x, tid, q), 8, x.lo, endc) << (8 * q);
  return inm;
}

// Pass 1 over the nested chunks' fill tiles: both level streams expanded (the u8 level arrays,
// the slot validity and the pages' record / non-null counts written from registers), the slots'
// flag masks for pass 2 (cd.nest_masks: which counters count at a slot, the entries' validity,
// the groups' validity), and per 4,096-slot half how many entries of each counter (lists of
// levels 1..R starting, then leaf elements), stored at the tile's position in the launch list
// (every half is written: no zeroing).
struct NestCountLDS {
  NestStage st;
  uint32_t vb[kLfTile / 32];  // slot validity of the tile (16 bits per thread and half)
  uint32_t part[2][kNestCnt][4];
  uint64_t wsum[4];
  uint32_t last;
};
// R: the chunks' list levels (one launch per group of tiles, as k_nest_emit).
template <uint32_t R>
__global__ void __launch_bounds__(256) k_nest_count(BatchDev b_in, const uint4 *tiles, uint32_t first) {
  constexpr uint32_t C = R + 1;
  const BatchDev b = global_view(b_in);
  __shared__ NestCountLDS L;
  const uint32_t pos = first + blockIdx.x, tid = threadIdx.x, lane = lane_id(), wv = tid >> 6;
  const NestFill x = nest_fill(b, gp(tiles)[pos]);
  const PageDesc &pd = b.pages[x.pi];
  const ChunkDesc &cd = b.chunks[x.chunk];
  // diagnostic build (tools/diag_nest.py): 0 run staging, 1 group marks, 2 expansion, 3 page counts,
  // 4 packed levels, 5 counters, 6 validity
  PQ_STAMPS(st, b.dbg);
  st.begin();
  uint64_t lw[2][4];
  uint32_t eqd[4], end_d = 0;
  nest_expand(b, pd, cd, x, L.st, tid, lw, eqd, end_d, st);
  // slot validity (definition level == max_def) of the definition stream's covered values
  uint32_t *vbits = gp_u64<uint32_t>(cd.validity);
  if (vbits && x.lo < end_d) {  // workgroup-uniform
    reinterpret_cast<uint16_t *>(L.vb)[tid] = (uint16_t)(eqd[0] | (eqd[1] << 8));
    reinterpret_cast<uint16_t *>(L.vb)[256 + tid] = (uint16_t)(eqd[2] | (eqd[3] << 8));
  }
  // The slots' flag masks for k_nest_emit, 32 bits per thread (bits 8q..8q+7: group q; 0-15 the first
  // half's sixteen slots, 16-31 the second's): mask j < C, the covered slots where counter j counts
  // (a level-(j+1) list starts, j < R; a leaf element slot, j == R); C + j the validity of those
  // entries (list j non-null; the element non-null); 2C + g, group g's validity (def >= group_def).
  // Eight levels per 64-bit word are compared at once (SWAR: levels below 128; wider levels take
  // the byte loop). The counters per half are the masks' popcounts, in 5-bit fields (at most 16
  // slots per thread and half).
  const bool swar = cd.max_def < 128;
  const uint32_t inm = nest_cover_mask(b, pd, cd, x, tid);
  const uint32_t M = cd.nest_nmask;  // 2 C + the groups
  uint32_t *mk = gp_u64<uint32_t>(cd.nest_masks) + (uint64_t)(pos - cd.nest_tile0) * M * 256 + tid;
  uint64_t pa = 0, pb = 0;
  // mask k < 2 C + ngroups: kind 0 (flag j = k), 1 (validity j = k - C) or 2 (group g = k - 2 C)
  auto mask_of = [&](uint32_t kind, uint32_t j, uint32_t g) -> uint32_t { return nest_mask<R>(cd, lw, swar, kind, j, g); };
#pragma unroll
  for (uint32_t j = 0; j < C; j++) {
    const uint32_t m = mask_of(0, j, 0) & inm;
    pa += (uint64_t)__popc(m & 0xffffu) << (5 * j);
    pb += (uint64_t)__popc(m >> 16) << (5 * j);
    mk[(uint64_t)j * 256] = m;
  }
#pragma unroll
  for (uint32_t j = 0; j < C; j++) mk[(uint64_t)(C + j) * 256] = mask_of(1, j, 0);
#pragma unroll 1
  for (uint32_t g = 0; g + 2 * C < M; g++) mk[(uint64_t)(2 * C + g) * 256] = mask_of(2, 0, g);
  st.lap(4);
#pragma unroll
  for (uint32_t j = 0; j < C; j++) {
    const uint32_t a2 = (uint32_t)wave_sum64((pa >> (5 * j)) & 31u), b2 = (uint32_t)wave_sum64((pb >> (5 * j)) & 31u);
    if (lane == 0) { L.part[0][j][wv] = a2; L.part[1][j][wv] = b2; }
  }
  wg_barrier();
  static_assert(2 * kNestCnt <= 64, "wave 0 publishes the counts");
  // The chunk's last tile to finish scans its counts (no launch of its own, no order assumed:
  // whichever tile arrives last finds every other tile's counts). The counts are published by
  // agent-scope atomics whose results the arrival count waits for (an agent-scope release fence
  // per tile would write back the XCD's whole L2: 0.39 -> 1.16 ms), and read by atomic loads.
  if (wv == 0) {
    uint32_t seen = 0;
    if (tid < 2 * kNestCnt && tid % kNestCnt < C) {  // (the scan reads counters j < C)
      const uint32_t h = tid / kNestCnt, j = tid % kNestCnt;
      const uint32_t v = L.part[h][j][0] + L.part[h][j][1] + L.part[h][j][2] + L.part[h][j][3];
      seen = __hip_atomic_exchange(&b.nest_cnt[(2 * (uint64_t)pos + h) * kNestCnt + j], v, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("; the exchanges have returned: %0" ::"v"(seen));  // (a use: the wave waits for them)
    if (lane == 0)
      L.last = __hip_atomic_fetch_add(&b.nest_done[x.chunk], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1 ==
               cd.nest_ntiles;
  }
  wg_barrier();
  if (L.last) nest_scan_chunk(b, x.chunk, L.wsum);  // workgroup-uniform
  st.lap(5);
  if (vbits && x.lo < end_d) {
    const uint32_t w = tid;  // kLfTile / 32 = 256 words: one per thread
    const int64_t w0 = x.t0 + 32 * (int64_t)w;
    if (w0 + 32 > (int64_t)x.lo && w0 < (int64_t)end_d) {
      const uint32_t v = L.vb[w];
      uint32_t *dst = vbits + ((x.sbase + (uint64_t)w0) >> 5);
      if (w0 >= (int64_t)x.lo && w0 + 32 <= (int64_t)end_d) *dst = v;  // the tile owns the whole word
      else if (v) atomicOr(dst, v);                                     // shared with a neighbouring page
    }
  }
  st.lap(6);
  st.flush(24);
}

// Bits of x at the positions set in m, packed towards bit 0 (Hacker's Delight 7-4, compress), for
// masks of at most 16 bits -- the emission's per-half masks: no bit moves 16 places, so four rounds,
// and the prefix XOR needs no 16-place step (cfg4 k_nest_tile 0.608 -> 0.605 ms against the 32-bit
// form, profiles/r05_s48_probe_compress16.txt).
DEV uint32_t compress16(uint32_t x, uint32_t m) {
  x &= m;
  uint32_t mk = ~m << 1;
#pragma unroll
  for (uint32_t i = 0; i < 4; i++) {
    uint32_t mp = mk ^ (mk << 1);
    mp ^= mp << 2;
    mp ^= mp << 4;
    mp ^= mp << 8;
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

// Pass 2: per fill tile and 4,096-slot half, from the levels k_nest_count packed: wave w owns
// 1,024 consecutive slots, lane i sixteen of them. Per counter j a lane holds the 16-bit mask of
// its flagged slots; wave prefix sums of their counts (and one workgroup exchange of the wave
// totals) give every entry its index. List offsets (the child counter's index at the list's first
// slot) and record offsets (counter 0: a level-1 list starts at rep == 0, ColumnStore.get's record
// split) are staged in a per-wave LDS row in entry order and leave as contiguous stores; the
// entries' validity bits are compressed out of the lane's slot mask, placed at their index in a
// per-wave LDS bit row and written with a funnel shift to their place in the bitmap.
// R: the chunks' list levels (the launch covers the tiles of chunks with nest == R, so every
// per-counter array is indexed by compile-time constants and stays in registers).
template <uint32_t R>
struct NestEmitLDS {
  uint32_t ent[4][kNestWaveSlots + 4];  // per-wave entry rows (shifted to the destination's 16-B phase)
  uint32_t wtot[2][R + 1][4];
  uint32_t brow[4][kNestWaveSlots / 32 + 1];
};
// Half h of a tile's outputs (see k_nest_emit): f[j] / vm[j], the thread's 16-bit flag and validity
// masks of counter j in this half; base[j], the half's first entry of counter j in the chunk;
// gown, the groups with a bitmap of their own; gmask(gi), group gi's 16-bit validity mask.
template <uint32_t R, class GM>
DEV void nest_emit_half(const BatchDev &b, const ChunkDesc &cd, const NestFill &x, uint32_t tid, uint32_t h,
                        const uint32_t (&f)[R + 1], const uint32_t (&vm)[R + 1], const uint64_t (&base)[R + 1],
                        uint32_t gown, GM gmask, NestEmitLDS<R> &L, Stamps &st) {
  constexpr uint32_t C = R + 1;
  const uint32_t lane = lane_id(), wv = tid >> 6;
  int32_t *rec = gp_u64<int32_t>(cd.list_offsets);
  uint32_t *row = L.ent[wv];
  uint32_t *bits = L.brow[wv];
  const int64_t g = nest_group(x, tid, 2 * h);
  const uint64_t s = (uint64_t)((int64_t)x.sbase + g);  // the chunk slot of the lane's first slot
  st.lap(0);
  // entry indices: wave prefix sums, then the waves before this one in the half
  uint32_t P[C], T[C];
#pragma unroll
  for (uint32_t j = 0; j < C; j++) {
    const uint32_t c = (uint32_t)__popc(f[j]);
    const uint32_t incl = (uint32_t)wave_incl_scan64_dpp(c);
    P[j] = incl - c;
    T[j] = (uint32_t)__shfl(incl, 63);
    if (lane == 0) L.wtot[h][j][wv] = T[j];
  }
  wg_barrier();  // wtot[h] complete (double-buffered: no barrier before the next half's stores)
  uint64_t run[C];
#pragma unroll
  for (uint32_t j = 0; j < C; j++) {
    uint64_t v = base[j];
    for (uint32_t q = 0; q < wv; q++) v += L.wtot[h][j][q];
    run[j] = v;
  }
  st.lap(1);
  // list offsets of each level, then the record offsets (level-1 list starts)
#pragma unroll
  for (uint32_t j = 0; j <= R; j++) {
    const uint32_t lv = j < R ? j : 0;  // j == R: record offsets
    if (j == R && !rec) break;
    if (PQ_ABLATE(b, 16)) break;  // diagnostic bit 16: no offset stores
    int32_t *dst = j < R ? gp_u64<int32_t>(cd.lvl_offsets[j]) + run[j] : rec + run[0];
    // the row holds entry e at row[a + e], a = dst's dword phase in its 16-B piece, so that the body
    // leaves as aligned 16-B LDS reads and stores (head and tail entries one by one)
    const uint32_t a = (uint32_t)((uintptr_t)dst >> 2) & 3u;
    uint32_t m = f[lv], k = a + P[lv];
    const uint32_t cb = (uint32_t)(run[lv + 1] + P[lv + 1]);  // children before this lane's slots
    while (m) {
      const uint32_t i = __builtin_ctz(m);
      m &= m - 1;
      row[k++] = j < R ? cb + (uint32_t)__popc(f[lv + 1] & ((1u << i) - 1u)) : (uint32_t)(s + i);
    }
    wave_lds_sync();
    const uint32_t tn = T[lv], head = min(tn, (4u - a) & 3u), nb = (tn - head) >> 2, t0 = head + 4 * nb;
    if (lane < head) dst[lane] = (int32_t)row[a + lane];
    const uint4 *r4 = reinterpret_cast<const uint4 *>(row + a + head);  // (a + head is 0 or 4)
    uint4 *d4 = reinterpret_cast<uint4 *>(dst + head);
    for (uint32_t q = lane; q < nb; q += 64) d4[q] = r4[q];
    if (lane < tn - t0) dst[t0 + lane] = (int32_t)row[a + t0 + lane];
    wave_lds_sync();
  }
  st.lap(2);
  // validity bits of every counter's entries
#pragma unroll
  for (uint32_t j = 0; j < C; j++) {
    if (PQ_ABLATE(b, 17)) break;  // diagnostic bit 17: no bitmaps
    if (lane <= kNestWaveSlots / 32) bits[lane] = 0;
    wave_lds_sync();
    const uint32_t c = (uint32_t)__popc(f[j]);
    if (c) {
      const uint32_t comp = compress16(vm[j], f[j]), p = P[j], sh = p & 31;
      atomicOr(&bits[p >> 5], comp << sh);
      if (sh && sh + c > 32) atomicOr(&bits[(p >> 5) + 1], comp >> (32 - sh));
    }
    wave_lds_sync();
    nest_put_bits(gp_u64<uint32_t>(j < R ? cd.lvl_validity[j] : cd.elem_validity), run[j], bits, T[j], lane);
    wave_lds_sync();
  }
  st.lap(3);
  // struct validity of the OPTIONAL groups that own a bitmap (Column.getNextData schema.go:216-260:
  // a group is non-nil iff a child is defined at or below it, def >= group_def): its entries are
  // those of counter group_depth (the level-(depth + 1) lists, or the leaf's element slots), so the
  // bits go where that counter's validity goes
  for (uint32_t gm = gown; gm; gm &= gm - 1) {  // (groups that share list / element validity: none)
    const uint32_t gi = (uint32_t)__builtin_ctz(gm);
    uint32_t *gv = gp_u64<uint32_t>(cd.group_validity[gi]);
    const uint32_t j = cd.group_depth[gi];
    uint32_t fj = 0, pj = 0, tj = 0;
    uint64_t rj = 0;
#pragma unroll
    for (uint32_t q = 0; q < C; q++)  // selects: a dynamic index would put the arrays in scratch
      if (q == j) { fj = f[q]; pj = P[q]; tj = T[q]; rj = run[q]; }
    const uint32_t vg = gmask(gi);
    if (lane <= kNestWaveSlots / 32) bits[lane] = 0;
    wave_lds_sync();
    const uint32_t c = (uint32_t)__popc(fj);
    if (c) {
      const uint32_t comp = compress16(vg, fj), sh = pj & 31;
      atomicOr(&bits[pj >> 5], comp << sh);
      if (sh && sh + c > 32) atomicOr(&bits[(pj >> 5) + 1], comp >> (32 - sh));
    }
    wave_lds_sync();
    nest_put_bits(gv, rj, bits, tj, lane);
    wave_lds_sync();
  }
  st.lap(4);
}
DEV uint32_t nest_groups_owned(const ChunkDesc &cd) {  // the groups with a bitmap of their own
  uint32_t gown = 0;
  for (uint32_t gi = 0; gi < cd.ngroups; gi++) gown |= (cd.group_validity[gi] != 0 ? 1u : 0u) << gi;
  return gown;
}

// Pass 2: per fill tile and 4,096-slot half, from the levels k_nest_count packed: wave w owns
// 1,024 consecutive slots, lane i sixteen of them. Per counter j a lane holds the 16-bit mask of
// its flagged slots; wave prefix sums of their counts (and one workgroup exchange of the wave
// totals) give every entry its index. List offsets (the child counter's index at the list's first
// slot) and record offsets (counter 0: a level-1 list starts at rep == 0, ColumnStore.get's record
// split) are staged in a per-wave LDS row in entry order and leave as contiguous stores; the
// entries' validity bits are compressed out of the lane's slot mask, placed at their index in a
// per-wave LDS bit row and written with a funnel shift to their place in the bitmap.
// R: the chunks' list levels (the launch covers the tiles of chunks with nest == R, so every
// per-counter array is indexed by compile-time constants and stays in registers).
template <uint32_t R>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(R == 1 ? 8 : R <= 3 ? 4 : 2))) k_nest_emit(BatchDev b_in, const uint4 *tiles, uint32_t first) {
  constexpr uint32_t C = R + 1;
  const BatchDev b = global_view(b_in);
  __shared__ NestEmitLDS<R> L;
  const uint32_t pos = first + blockIdx.x, tid = threadIdx.x;
  const NestFill x = nest_fill(b, gp(tiles)[pos]);
  const ChunkDesc &cd = b.chunks[x.chunk];
  // the thread's flag and validity masks (k_nest_count): bits 16 h .. 16 h + 15 for half h
  const uint32_t *mk = gp_u64<const uint32_t>(cd.nest_masks) + (uint64_t)(pos - cd.nest_tile0) * cd.nest_nmask * 256 + tid;
  uint32_t fm[C], vmm[C];
#pragma unroll
  for (uint32_t j = 0; j < C; j++) {
    fm[j] = mk[j * 256];
    vmm[j] = mk[(C + j) * 256];
  }
  uint64_t base0[C], base1[C];  // the halves' entry bases (k_nest_count's scan), loaded up front
#pragma unroll
  for (uint32_t j = 0; j < C; j++) {
    base0[j] = b.nest_base[(2 * (uint64_t)pos) * kNestCnt + j];
    base1[j] = b.nest_base[(2 * (uint64_t)pos + 1) * kNestCnt + j];
  }
  const uint32_t gown = nest_groups_owned(cd);
  // diagnostic build (tools/diag_nest.py): 0 masks, 1 entry indices, 2 offsets, 3 validity, 4 groups
  PQ_STAMPS(st, b.dbg);
  st.begin();
#pragma unroll 1
  for (uint32_t h = 0; h < 2; h++) {
    uint32_t f[C], vm[C];
#pragma unroll
    for (uint32_t j = 0; j < C; j++) {
      f[j] = (fm[j] >> (16 * h)) & 0xffffu;
      vm[j] = (vmm[j] >> (16 * h)) & 0xffffu;
    }
    auto gmask = [&](uint32_t gi) -> uint32_t { return (mk[(2 * C + gi) * 256] >> (16 * h)) & 0xffffu; };
    nest_emit_half<R>(b, cd, x, tid, h, f, vm, h ? base1 : base0, gown, gmask, L, st);
  }
  st.flush(32);
}

// ---------------------------------------------------------------------------
// k_nest_tile: both passes in one launch. A tile expands its levels and computes its flag masks and
// per-half counts as k_nest_count does, publishes the tile's counts, finds its entry bases by a
// decoupled look-back over the chunk's earlier tiles (wave 0; one 64-bit word per counter carrying
// its own state: aggregate, then inclusive prefix), and emits as k_nest_emit does from the masks it
// holds in registers: no flag masks, counts or bases go through memory, no per-chunk scan and no
// second launch. The chunk's last tile writes the chunk totals and the closing offsets. A tile waits
// only for tiles of its chunk with lower block indices (dispatched before it).
// ---------------------------------------------------------------------------
constexpr uint32_t kNsStride = 16;  // u64 per tile: one 128-B line (no two tiles' atomics share a line)
#ifndef PQ_NS_WIN
#define PQ_NS_WIN 16
#endif
constexpr uint32_t kNsWin = PQ_NS_WIN;  // predecessors read per look-back round trip (one per lane)
constexpr uint64_t kNsAgg = 1ull << 62, kNsIncl = 2ull << 62, kNsMask = (1ull << 62) - 1;
constexpr uint32_t kNsMaxPolls = 1u << 22;  // look-back polls before giving up (seconds: a bound, not a wait)

#ifndef PQ_NS_SLEEP
#define PQ_NS_SLEEP 2  // s_sleep between the polls of a predecessor that has not published
#endif
// A tile's counter words (wave 0): its aggregates, or, for the chunk's first tile, its inclusive
// prefixes (lane q < C writes word q; selects, no dynamic register index).
template <uint32_t C>
DEV void nest_publish(const BatchDev &b, uint32_t pos, uint64_t flag, const uint64_t (&v)[C]) {
  const uint32_t lane = lane_id();
  uint64_t w = 0;
#pragma unroll
  for (uint32_t q = 0; q < C; q++)
    if (lane == q) w = flag | v[q];
#ifdef PQ_DIAG_STAMPS
  // diagnostic build, PQ_ABLATE bit 26 (tests/test_nested.py::test_gpu_lookback_torn_publish): the
  // words go out one by one in reverse order, ~27 us apart, so a successor that polls meanwhile
  // finds this tile half-way between its aggregates and its inclusive prefixes (the state the
  // look-back must read again, nest_resolve) — certain, not a rare interleaving
  if (PQ_ABLATE(b, 26)) {
    for (int32_t q = (int32_t)C - 1; q >= 0; q--) {
      if (lane == (uint32_t)q)
        __hip_atomic_exchange(&b.nest_state[(uint64_t)pos * kNsStride + lane], w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      for (int i = 0; i < 8; i++) __builtin_amdgcn_s_sleep(127);
    }
    return;
  }
#endif
  if (lane < C)
    __hip_atomic_exchange(&b.nest_state[(uint64_t)pos * kNsStride + lane], w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// The tile's exclusive prefixes `pre` (wave 0), its aggregates already published (nest_publish), then
// its inclusive prefixes published. Returns the look-back's round trips.
template <uint32_t C>
DEV uint32_t nest_resolve(const BatchDev &b, const ChunkDesc &cd, uint32_t pos, const uint64_t (&agg)[C], uint64_t (&pre)[C]) {
  uint64_t *st = b.nest_state;
  const uint32_t lane = lane_id();
#pragma unroll
  for (uint32_t q = 0; q < C; q++) pre[q] = 0;
  if (pos == cd.nest_tile0) return 0;  // (published its inclusive prefixes already)
  int64_t k = (int64_t)pos - 1;  // the nearest tile not yet added
  uint32_t polls = 0;
  for (;;) {
    if (++polls > kNsMaxPolls) {  // never (a predecessor that does not publish): prefixes past any
#pragma unroll                   // chunk's slots make the caller write nothing and report it
      for (uint32_t q = 0; q < C; q++) pre[q] = kNsMask;
      return polls;
    }
    const int64_t my = k - (int64_t)lane;
    const bool win = lane < kNsWin, valid = win && my >= (int64_t)cd.nest_tile0;
    uint64_t s[C];
    bool set = true, any_agg = false, any_inc = false;
#pragma unroll
    for (uint32_t q = 0; q < C; q++) {
      // past the chunk's first tile: an inclusive prefix of 0
      s[q] = valid ? __hip_atomic_load(&st[(uint64_t)my * kNsStride + q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : kNsIncl;
      set &= s[q] != 0;
      any_agg |= (s[q] & ~kNsMask) == kNsAgg;
      any_inc |= (s[q] & ~kNsMask) == kNsIncl;
    }
    // a predecessor's C words become visible one by one: one caught between its aggregates and its
    // inclusive prefixes (some of each) is read again, like one not yet published
    bool rdy = set && !(any_agg && any_inc);
    const bool inc = rdy && !any_agg;
#ifdef PQ_DIAG_STAMPS
    if (PQ_ABLATE(b, 26)) {  // torn-state injection (nest_publish): wait for the predecessors'
      // inclusive prefixes instead of taking their aggregates (for up to 2^16 polls), so the reader
      // is polling while they go out word by word
      if (b.dbg && lane == 0 && __ballot(win && set && any_agg && any_inc))
        atomicAdd(&b.dbg[20], 1ull);  // torn predecessors seen, read again (slot 20: no stamp uses it)
      if (polls < (1u << 16)) rdy = inc;
    }
#endif
    const uint64_t incl = __ballot(win && inc), hole = __ballot(win && !rdy);
    const uint32_t stop = incl ? (uint32_t)__builtin_ctzll(incl) : 64u;
    const uint32_t h = hole ? (uint32_t)__builtin_ctzll(hole) : 64u;
    const uint32_t upto = min(min(stop + 1, h), kNsWin);  // lanes [0, upto) are added
#pragma unroll
    for (uint32_t q = 0; q < C; q++) pre[q] += wave_sum64(lane < upto ? (s[q] & kNsMask) : 0);
    if (stop < h) break;  // reached an inclusive prefix (or the chunk's first tile)
    k -= upto;
    if (h < 64 && PQ_NS_SLEEP) __builtin_amdgcn_s_sleep(PQ_NS_SLEEP);
  }
  uint64_t inc[C];
#pragma unroll
  for (uint32_t q = 0; q < C; q++) inc[q] = pre[q] + agg[q];
  nest_publish<C>(b, pos, kNsIncl, inc);
  return polls;
}

constexpr uint32_t kNestTiles = 1;  // tiles per k_nest_tile workgroup (2, the second counting while the
                                    // first looks back: cfg4 0.63 -> 0.73 ms, profiles/r05_s36_probe_nest_pairs.txt)
template <uint32_t R>
struct NestTileLDS {
  union {
    struct {
      NestStage st;
      uint32_t vb[kLfTile / 32];  // slot validity of the tile (16 bits per thread and half)
    } a;                          // counting
    NestEmitLDS<R> e;             // emission
  } u;
  uint32_t part[2][R + 1][4];
  uint32_t gmk[PQGPU_MAX_NEST][256];  // the owned groups' validity masks (the levels are not kept)
  uint32_t h0[kNestTiles][R + 1];     // per tile: the first half's entries of each counter
  uint32_t h1[kNestTiles][R + 1];     // the second half's
  uint64_t base[R + 1];               // the tile being emitted: its first entry of each counter
  uint32_t bad;                       // its prefixes exceed the chunk's slots (never: it writes nothing)
};
// One tile's counting half (k_nest_count's work, without the flag masks leaving registers): the
// levels expanded, u8 levels / slot validity / page counts written, the masks fm / vmm, the owned
// groups' masks in L.gmk, the per-half counts in L.h0[q] / L.h1[q], and the tile's aggregates
// published (wave 0).
template <uint32_t R>
DEV void nest_tile_count(const BatchDev &b, const NestFill &x, uint32_t pos, uint32_t q, bool counted, bool based,
                         NestTileLDS<R> &L, uint32_t (&fm)[R + 1], uint32_t (&vmm)[R + 1], Stamps &st) {
  constexpr uint32_t C = R + 1;
  const uint32_t tid = threadIdx.x, lane = lane_id(), wv = tid >> 6;
  const PageDesc &pd = b.pages[x.pi];
  const ChunkDesc &cd = b.chunks[x.chunk];
  uint64_t lw[2][4];
  uint32_t eqd[4], end_d = 0;
  nest_expand(b, pd, cd, x, L.u.a.st, tid, lw, eqd, end_d, st, !counted);  // (counted: k_nest_pcount's)
  uint32_t *vbits = gp_u64<uint32_t>(cd.validity);
  const bool vtile = vbits && x.lo < end_d;  // workgroup-uniform
  if (vtile) {
    reinterpret_cast<uint16_t *>(L.u.a.vb)[tid] = (uint16_t)(eqd[0] | (eqd[1] << 8));
    reinterpret_cast<uint16_t *>(L.u.a.vb)[256 + tid] = (uint16_t)(eqd[2] | (eqd[3] << 8));
  }
  const bool swar = cd.max_def < 128;
  const uint32_t inm = nest_cover_mask(b, pd, cd, x, tid);
  for (uint32_t gm = nest_groups_owned(cd); gm; gm &= gm - 1) {
    const uint32_t gi = (uint32_t)__builtin_ctz(gm);
    L.gmk[gi][tid] = nest_mask<R>(cd, lw, swar, 2, 0, gi);
  }
#pragma unroll
  for (uint32_t j = 0; j < C; j++) {
    fm[j] = nest_mask<R>(cd, lw, swar, 0, j, 0) & inm;
    vmm[j] = nest_mask<R>(cd, lw, swar, 1, j, 0);
    const uint32_t a2 = (uint32_t)wave_sum64((uint32_t)__popc(fm[j] & 0xffffu)), b2 = (uint32_t)wave_sum64((uint32_t)__popc(fm[j] >> 16));
    if (lane == 0) { L.part[0][j][wv] = a2; L.part[1][j][wv] = b2; }
  }
  wg_barrier();  // part and vb complete
  st.lap(4);
  // slot validity (definition level == max_def) of the definition stream's covered values
  if (vtile) {
    const uint32_t w = tid;  // kLfTile / 32 = 256 words: one per thread
    const int64_t w0 = x.t0 + 32 * (int64_t)w;
    if (w0 + 32 > (int64_t)x.lo && w0 < (int64_t)end_d) {
      const uint32_t v = L.u.a.vb[w];
      uint32_t *dst = vbits + ((x.sbase + (uint64_t)w0) >> 5);
      if (w0 >= (int64_t)x.lo && w0 + 32 <= (int64_t)end_d) *dst = v;  // the tile owns the whole word
      else if (v) atomicOr(dst, v);                                     // shared with a neighbouring page
    }
  }
  if (wv == 0) {
    uint64_t agg[C];
#pragma unroll
    for (uint32_t j = 0; j < C; j++) {
      const uint32_t a0 = L.part[0][j][0] + L.part[0][j][1] + L.part[0][j][2] + L.part[0][j][3];
      const uint32_t a1 = L.part[1][j][0] + L.part[1][j][1] + L.part[1][j][2] + L.part[1][j][3];
      agg[j] = a0 + a1;
      if (lane == j) { L.h0[q][j] = a0; L.h1[q][j] = a1; }
    }
    if (!based) nest_publish<C>(b, pos, pos == cd.nest_tile0 ? kNsIncl : kNsAgg, agg);
  }
  st.lap(6);
}
// One tile's second half: its bases by the look-back (wave 0), the chunk's totals and closing
// entries from its last tile, then the outputs (nest_emit_half). The caller synchronises after it.
template <uint32_t R>
DEV void nest_tile_emit(const BatchDev &b, const NestFill &x, uint32_t pos, uint32_t q, bool based, NestTileLDS<R> &L,
                        const uint32_t (&fm)[R + 1], const uint32_t (&vmm)[R + 1], Stamps &st, Stamps &se) {
  constexpr uint32_t C = R + 1;
  const uint32_t tid = threadIdx.x, lane = lane_id(), wv = tid >> 6;
  const PageDesc &pd = b.pages[x.pi];
  const ChunkDesc &cd = b.chunks[x.chunk];
  st.lap(7);
  if (wv == 0) {
    uint64_t agg[C], pre[C];
#pragma unroll
    for (uint32_t j = 0; j < C; j++) agg[j] = (uint64_t)L.h0[q][j] + L.h1[q][j];
    bool over = false;  // a counter's entries are at most the chunk's slots (the arrays' capacity)
    if (based) {  // k_nest_tcount + k_nest_scan: the bases are known, and the counts must be this tile's
#pragma unroll
      for (uint32_t j = 0; j < C; j++) {
        pre[j] = b.nest_base[(2 * (uint64_t)pos) * kNestCnt + j];
        over |= b.nest_cnt[(2 * (uint64_t)pos) * kNestCnt + j] != L.h0[q][j] ||
                b.nest_cnt[(2 * (uint64_t)pos + 1) * kNestCnt + j] != L.h1[q][j];
      }
    } else {
      const uint32_t polls = nest_resolve<C>(b, cd, pos, agg, pre);
      st.add(3, polls);  // (diagnostic build: look-back round trips, in place of the page counts' slot)
    }
#pragma unroll
    for (uint32_t j = 0; j < C; j++) {
      over |= pre[j] > cd.num_slots || pre[j] + agg[j] > cd.num_slots;
      if (lane == j) L.base[j] = pre[j];
    }
    if (lane == 0) {
      L.bad = over;
      if (over) report(b, x.chunk, 1, pd.page_in_chunk, ST_VALUES, 0, PQ_ERR_UNSUPPORTED);  // internal error
#ifdef PQ_DIAG_STAMPS
      if (over && PQ_ABLATE(b, 26) && b.dbg) atomicAdd(&b.dbg[20], 1ull << 40);  // the guard fired (high bits)
#endif
    }
    if (!based && pos - cd.nest_tile0 == cd.nest_ntiles - 1 && !over) {  // the chunk's last tile: totals, closing entries
      uint64_t tot[C];
#pragma unroll
      for (uint32_t j = 0; j < C; j++) {
        tot[j] = pre[j] + agg[j];
        if (lane == j) b.nest_tot[(uint64_t)x.chunk * kNestCnt + j] = tot[j];
      }
      int32_t *rec = gp_u64<int32_t>(cd.list_offsets);
#pragma unroll
      for (uint32_t j = 0; j < R; j++)
        if (lane == j) gp_u64<int32_t>(cd.lvl_offsets[j])[tot[j]] = (int32_t)tot[j + 1];
      if (lane == 0 && rec) rec[tot[0]] = (int32_t)cd.num_slots;
    }
  }
  wg_barrier();  // base complete; the counting LDS is free for the emission
  st.lap(5);
  if (L.bad) return;  // workgroup-uniform
  se.begin();
  uint64_t base0[C], base1[C];
#pragma unroll
  for (uint32_t j = 0; j < C; j++) {
    base0[j] = L.base[j];
    base1[j] = base0[j] + L.h0[q][j];
  }
  const uint32_t gown = nest_groups_owned(cd);
#pragma unroll 1
  for (uint32_t h = 0; h < 2; h++) {
    uint32_t f[C], vm[C];
#pragma unroll
    for (uint32_t j = 0; j < C; j++) {
      f[j] = (fm[j] >> (16 * h)) & 0xffffu;
      vm[j] = (vmm[j] >> (16 * h)) & 0xffffu;
    }
    auto gmask = [&](uint32_t gi) -> uint32_t { return (L.gmk[gi][tid] >> (16 * h)) & 0xffffu; };
    nest_emit_half<R>(b, cd, x, tid, h, f, vm, h ? base1 : base0, gown, gmask, L.u.e, se);
  }
  se.lap(5);
}

// Fields >= D among the bw-bit fields of x (zero past its last field): the even fields, then the odd
// ones moved onto the even positions, each with a field's width of zero bits above it, so that
// field + (2^bw - D) carries into that gap exactly when field >= D. fm / ad / cb: every even position
// below 56 / bw fields -- the field mask, the addend and the carry bits.
struct FieldsGe {
  uint64_t fm, ad, cb;
  uint32_t bw;
  DEV FieldsGe(uint32_t w, uint32_t D) : fm(0), ad(0), cb(0), bw(w) {
    const uint32_t k = 56 / w;
    for (uint32_t i = 0; i < k; i += 2) {
      fm |= ((1ull << w) - 1ull) << (i * w);
      ad |= (uint64_t)((1u << w) - D) << (i * w);
      cb |= 1ull << (i * w + w);
    }
  }
  DEV uint32_t operator()(uint64_t x) const {
    return (uint32_t)__popcll(((x & fm) + ad) & cb) + (uint32_t)__popcll((((x >> bw) & fm) + ad) & cb);
  }
};

// k_nest_tcount (chunks with one list level): each nested tile's counts per 4,096-slot half straight
// from the level run tables -- counter 0, the list starts (repetition level 0), from the repetition
// stream; counter 1, the element slots (definition level >= list_def[0]), from the definition
// stream; both over the slots both streams cover, as k_nest_tile's masks count them. RLE runs count
// whole, bit-packed runs 64 bits at a time (fields_ge). One wave per tile, a run per lane and step.
// k_nest_scan then turns the counts into every half's bases, so k_nest_tile looks back on nothing.
__global__ void __launch_bounds__(256) k_nest_tcount(BatchDev b_in, const uint4 *tiles, uint32_t first, uint32_t n) {
  const BatchDev b = global_view(b_in);
  const uint32_t w = blockIdx.x * 4 + (threadIdx.x >> 6), lane = lane_id();
  if (w >= n) return;  // wave-uniform
  const uint32_t pos = first + w;
  const NestFill x = nest_fill(b, gp(tiles)[pos]);
  const PageDesc &pd = b.pages[x.pi];
  const ChunkDesc &cd = b.chunks[x.chunk];
  const uint32_t cov_r = b.lv_meta[4 * x.pi + 1], cov_d = cd.max_def ? b.lv_meta[4 * x.pi + 3] : pd.num_slots;
  const uint32_t endc = min(x.hi, min(cov_r, cov_d));
  const int64_t hmid = x.t0 + (int64_t)kNestHalf;  // the halves: [lo, mid) and [mid, endc)
  const uint32_t mid = (uint32_t)min(max(hmid, (int64_t)x.lo), (int64_t)max(endc, x.lo));
  uint32_t cnt[2][2] = {{0, 0}, {0, 0}};  // [counter][half]
  if (x.lo < endc) {
#pragma unroll
    for (uint32_t s2 = 0; s2 < 2; s2++) {  // stream 0: repetition (counter 0), 1: definition (counter 1)
      const uint32_t nr = b.lv_meta[4 * x.pi + 2 * s2];
      if (!nr) continue;
      const uint2 *runs = b.lv_runs + b.lv_run_base[2 * x.pi + s2];
      const uint32_t r0 = b.lv_tile_run[2 * (uint64_t)x.t + s2];
      const uint8_t *src = gp_u64<const uint8_t>(pd.data) + (s2 ? pd.def_off : pd.rep_off);
      const uint32_t slen = s2 ? pd.def_len : pd.rep_len;
      const uint32_t bw = s2 ? (uint32_t)cd.def_bw : (uint32_t)cd.rep_bw;
      const uint32_t D = s2 ? (uint32_t)cd.list_def[0] : 1u;  // rep: count the fields below 1
      const uint32_t k = 56 / bw;
      const FieldsGe ge(bw, D);
      for (uint32_t r = r0 + lane; r < nr; r += 64) {
        const uint2 run = runs[r];
        const uint32_t x0 = max(run.x, x.lo), x1 = min(r + 1 < nr ? runs[r + 1].x : endc, endc);
        if (run.x >= endc) break;  // (lanes past the tile: their runs start later still)
        if (x0 >= x1) continue;
#pragma unroll
        for (uint32_t h = 0; h < 2; h++) {
          const uint32_t a = h ? max(x0, mid) : x0, e = h ? x1 : min(x1, mid);
          if (a >= e) continue;
          uint32_t c = 0;
          if (!(run.y >> 31)) {  // RLE
            c = run.y >= D ? e - a : 0u;
          } else {
            uint64_t bo = (uint64_t)(run.y & 0x7fffffffu) * 8 + (uint64_t)(a - run.x) * bw;
            for (uint32_t v = a; v < e; v += k, bo += (uint64_t)k * bw) {
              const uint32_t m = min(k, e - v);
              c += ge(bits64c(src, slen, bo, m * bw));
            }
          }
          cnt[s2][h] += s2 ? c : (e - a) - c;  // rep: the fields below 1 (list starts)
        }
      }
    }
  }
#pragma unroll
  for (uint32_t j = 0; j < 2; j++)
#pragma unroll
    for (uint32_t h = 0; h < 2; h++) {
      const uint32_t t = (uint32_t)wave_sum64(cnt[j][h]);
      if (lane == 0) b.nest_cnt[(2 * (uint64_t)pos + h) * kNestCnt + j] = t;
    }
}

// k_nest_tile<R>: one tile per workgroup (block-order position from `order`): its counting half,
// publishing its aggregates, then its look-back and outputs.
template <uint32_t R>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(R == 1 ? 5 : R <= 3 ? 4 : 2))) k_nest_tile(BatchDev b_in, const uint4 *tiles, uint32_t first,
                                                                                                                  uint32_t n, uint32_t counted, const uint32_t *order, uint32_t based) {
  constexpr uint32_t C = R + 1;  // (R = 1: 96 VGPRs)
  const BatchDev b = global_view(b_in);
  __shared__ NestTileLDS<R> L;
  // diagnostic build (tools/diag_nest.py): slots 24-31 -- 0 run staging, 1 group marks, 2 expansion,
  // 3 look-back round trips (count), 4 flag masks and counts, 5 look-back (wave 0) and its barrier,
  // 6 slot validity and the aggregates, 7 between the counts and the look-back; slots 32-39, the
  // emission as k_nest_emit's
  PQ_STAMPS(st, b.dbg);
  PQ_STAMPS(se, b.dbg);
  st.begin();
  if (blockIdx.x < n) {  // (workgroup-uniform)
    uint32_t fm[C], vmm[C];
    const uint32_t pos = gp(order)[first + blockIdx.x];
    const NestFill x = nest_fill(b, gp(tiles)[pos]);
    nest_tile_count<R>(b, x, pos, 0, counted != 0, based != 0, L, fm, vmm, st);
    nest_tile_emit<R>(b, x, pos, 0, based != 0, L, fm, vmm, st, se);
  }
  st.flush(24);
  se.flush(32);
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
// The per-decode resets in one launch: [z, z + zn) to zero and [f, f + fn) to 0xff bytes (both
// 16-B aligned, sizes multiples of 16), instead of two fill launches.
__global__ void __launch_bounds__(256) k_reset(uint4 *z, uint64_t zn, uint4 *f, uint64_t fn) {
  z = gp(z);
  f = gp(f);
  const uint64_t nz = zn / 16, nf = fn / 16, stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nz + nf; i += stride) {
    if (i < nz) z[i] = make_uint4(0u, 0u, 0u, 0u);
    else f[i - nz] = make_uint4(~0u, ~0u, ~0u, ~0u);
  }
}
hipError_t launch_reset(void *z, uint64_t zn, void *f, uint64_t fn, hipStream_t s) {
  const uint64_t n = (zn + fn) / 16;
  if (!n) return hipSuccess;
  const uint32_t grid = (uint32_t)std::min<uint64_t>(2048, (n + 255) / 256);
  hipLaunchKernelGGL(k_reset, dim3(grid), dim3(256), 0, s, (uint4 *)z, zn, (uint4 *)f, fn);
  return hipGetLastError();
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

template <uint32_t R>
static void launch_count_r(const BatchDev &b, const LaunchLists &l, hipStream_t s) {
  const uint32_t n = l.nest_first[R + 1] - l.nest_first[R];
  if (n) hipLaunchKernelGGL(k_nest_count<R>, dim3(n), dim3(256), 0, s, b, l.nest_desc, l.nest_first[R]);
}
hipError_t launch_nest_count(const BatchDev &b, const LaunchLists &l, hipStream_t s) {
  if (!l.n_nest_tiles) return hipSuccess;
  // tiles are grouped by list levels (host.cpp): one instantiation per group
  launch_count_r<1>(b, l, s);
  launch_count_r<2>(b, l, s);
  launch_count_r<3>(b, l, s);
  launch_count_r<4>(b, l, s);
  launch_count_r<5>(b, l, s);
  launch_count_r<6>(b, l, s);
  launch_count_r<7>(b, l, s);
  launch_count_r<8>(b, l, s);
  return hipGetLastError();
}
hipError_t launch_nest_scan(const BatchDev &b, const LaunchLists &l, hipStream_t s) {
  if (!l.n_nest_empty) return hipSuccess;  // (chunks with tiles are scanned by k_nest_count)
  hipLaunchKernelGGL(k_nest_scan, dim3(l.n_nest_empty), dim3(256), 0, s, b, l.nest_chunks);
  return hipGetLastError();
}
template <uint32_t R>
static void launch_emit_r(const BatchDev &b, const LaunchLists &l, hipStream_t s) {
  const uint32_t n = l.nest_first[R + 1] - l.nest_first[R];
  if (n) hipLaunchKernelGGL(k_nest_emit<R>, dim3(n), dim3(256), 0, s, b, l.nest_desc, l.nest_first[R]);
}
template <uint32_t R>
static void launch_tile_r(const BatchDev &b, const LaunchLists &l, hipStream_t s, uint32_t counted, uint32_t based) {
  const uint32_t n = l.nest_first[R + 1] - l.nest_first[R];
  if (n) hipLaunchKernelGGL(k_nest_tile<R>, dim3(n), dim3(256), 0, s, b, l.nest_desc, l.nest_first[R], n,
                            counted, l.nest_order, based);
}
// (based: every tile's bases from k_nest_tcount + k_nest_scan, chunks with one list level only)
hipError_t launch_nest_tile(const BatchDev &b, const LaunchLists &l, hipStream_t s, bool counted, bool based) {
  if (!l.n_nest_tiles) return hipSuccess;
  // tiles are grouped by list levels (host.cpp): one instantiation per group; a chunk's tiles are
  // contiguous and in slot order within one launch (the look-back's predecessors)
  const uint32_t c = counted ? 1u : 0u;
  launch_tile_r<1>(b, l, s, c, based ? 1u : 0u);
  launch_tile_r<2>(b, l, s, c, 0u);
  launch_tile_r<3>(b, l, s, c, 0u);
  launch_tile_r<4>(b, l, s, c, 0u);
  launch_tile_r<5>(b, l, s, c, 0u);
  launch_tile_r<6>(b, l, s, c, 0u);
  launch_tile_r<7>(b, l, s, c, 0u);
  launch_tile_r<8>(b, l, s, c, 0u);
  return hipGetLastError();
}
// the R = 1 tiles' counts (k_nest_tcount), then every nested chunk's scan (k_nest_scan: bases, totals
// and closing entries; chunks without tiles too)
hipError_t launch_nest_tcount(const BatchDev &b, const LaunchLists &l, hipStream_t s) {
  const uint32_t n = l.nest_first[2] - l.nest_first[1];
  if (n) hipLaunchKernelGGL(k_nest_tcount, dim3((n + 3) / 4), dim3(256), 0, s, b, l.nest_desc, l.nest_first[1], n);
  if (l.n_nest_chunks) hipLaunchKernelGGL(k_nest_scan, dim3(l.n_nest_chunks), dim3(256), 0, s, b, l.nest_chunks);
  return hipGetLastError();
}
hipError_t launch_nest_pcount(const BatchDev &b, const LaunchLists &l, hipStream_t s) {
  if (!l.n_pc_pages) return hipSuccess;
  hipLaunchKernelGGL(k_nest_pcount, dim3(l.n_pc_pages), dim3(256), 0, s, b, l.pc_pages);
  return hipGetLastError();
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
