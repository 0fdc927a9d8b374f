// bytearray.hip — byte-array outputs (BYTE_ARRAY, and FIXED_LEN_BYTE_ARRAY chunks laid out as
// byte arrays): int32 offsets + one contiguous payload per chunk, the layout of the
// reference's []interface{} of []byte values (type_bytearray.go:24-55 PLAIN, type_dict.go:40-60
// dictionary, :98-240 DELTA_LENGTH / DELTA_BYTE_ARRAY) without one allocation per value.
//
// Work unit: the byte-array tile, 2,048 consecutive values of one page (class 3: 4,096; a tile lies
// inside one dictionary tile). Per decode:
//   k_dict_slots  every byte-array dictionary whose entries are at most 60 bytes is copied
//                 into 16/32/64-byte slots [u32 length | bytes | zero pad], so ONE aligned
//                 16-B load gives a value's length and its first 12 bytes (page_dict.go:35-72:
//                 the dictionary page's materialisation, redone every decode).
//   k_ba_emit     per tile, single pass. Wave w owns 512 values of the tile (class 3: 256) in rounds of
//                 64 consecutive values: their lengths (dictionary pages: indices decoded from
//                 the run table, dict_tile.h; an index outside the dictionary fails the page,
//                 type_dict.go:52-54; other pages: the lengths their value kernels wrote);
//                 the tile's payload base by a decoupled look-back over the chunk's earlier
//                 tiles (wave 0); then offsets[v + 1] and the payload bytes. A round's offsets
//                 are one coalesced store; its bytes are assembled in a per-wave LDS buffer at
//                 their final byte alignment and leave it as aligned 16-B stores.
//   Chunks whose payload has no upload-time bound (DELTA_BYTE_ARRAY pages) take two more
//   launches before k_ba_emit: k_ba_sums (per-tile payload bytes) and k_ba_scan (per chunk),
//   after which the host sizes the payload; their tiles read the scanned base.
// Tiles are laid out per class (see ba_emit) in eight interleaved queues: block b takes tile
// b / 8 of queue b mod 8, chunk c's tiles in order in queue c mod 8, so a chunk's tiles run on
// one XCD (blocks are dispatched round-robin over the XCDs) and its dictionary, slots and index
// streams stay in that XCD's L2. A tile's predecessors have lower block indices; the look-back
// never depends on the order blocks are dispatched in, though: a predecessor that has not
// published its sum after a while has it computed by the waiting tile (tile_aggregate).
// Pages from the chunk's first failing page on write nothing (the reference stops reading the
// chunk there: the outputs of the pages before it stay valid), but still publish their sums.
#include <hip/hip_runtime.h>

#include "dev_util.h"
#include "dict_slots.h"
#include "dict_tile.h"

namespace pq {

constexpr uint32_t kWaveBuf = 2048;               // payload bytes per wave round staged in LDS
constexpr uint32_t kWaveVec = kWaveBuf / 16 + 2;  // uint4 of one wave's LDS buffer
#ifndef PQ_BA_LBWIN
#define PQ_BA_LBWIN 16
#endif
constexpr uint32_t kLbWin = PQ_BA_LBWIN;  // look-back window (predecessors read per round trip)
constexpr uint32_t kStStride = 16;  // u64 per look-back state word: one per 128-B line (no two
                                    // tiles' atomics serialise on a line)
constexpr uint64_t kStAgg = 1ull << 62, kStIncl = 2ull << 62, kStMask = (1ull << 62) - 1;
#ifndef PQ_BA_HELP
#define PQ_BA_HELP 24
#endif
constexpr uint32_t kHelpSpins = PQ_BA_HELP;       // look-back polls of a silent predecessor before computing its sum
// Waves of a k_ba_emit workgroup: 4 for classes 0-2 (a 2,048-value tile is 8 rounds of 64 values per
// wave; with 256 LDS runs a workgroup takes 28 KB, so five are resident per CU and their phases --
// tile load, gathers, look-back, emission -- overlap: cfg3 0.344 -> 0.336 ms against 4,096-value tiles
// in 8-wave workgroups); 8 for class 3, whose 16 KB LDS slot table per workgroup would otherwise
// seat fewer waves (cfg4 k_ba_emit_lds 0.255 ms; 4-wave workgroups 0.407 ms)
constexpr uint32_t kEmitWaves = 4;
constexpr uint32_t kEmitWavesLds = 8;
constexpr uint32_t kRounds = 8;  // 64-value rounds per wave: kBaTile = 64 kRounds kEmitWaves, kBaTileLds likewise
static_assert(kBaTile == 64 * kRounds * kEmitWaves && kBaTileLds == 64 * kRounds * kEmitWavesLds, "tile = rounds x waves");
DEV uint32_t ba_tile_vals(const ChunkDesc &cd) { return (cd.flags & CF_BA_TILE4K) ? kBaTileLds : kBaTile; }

DEV uint64_t block_sum64(uint64_t v, uint64_t *wsum) {
  v = wave_sum64(v);
  if (lane_id() == 0) wsum[threadIdx.x >> 6] = v;
  wg_barrier();
  uint64_t t = 0;
  for (uint32_t q = 0; q < (blockDim.x >> 6); q++) t += wsum[q];
  return t;
}

// Bytes [src, src + len) of global memory to LDS bytes [d, d + len): aligned dword stores in
// the middle (ld32 funnels the unaligned source), byte stores at the two edges.
DEV void lds_put(uint8_t *lb, uint32_t d, const uint8_t *src, uint32_t len) {
  uint32_t k = 0;
  const uint32_t head = min(len, (4u - (d & 3u)) & 3u);
  if (head) {
    const uint32_t x = ld32(src);
    for (; k < head; k++) lb[d + k] = (uint8_t)(x >> (8 * k));
  }
  for (; k + 4 <= len; k += 4) *(uint32_t *)&lb[d + k] = ld32(src + k);
  if (k < len) {
    const uint32_t x = ld32(src + k);
    for (uint32_t j = 0; k < len; k++, j++) lb[d + k] = (uint8_t)(x >> (8 * j));
  }
}

// A slot's bytes (slot words 1 .. NW-1 of its first NP 16-B pieces, in registers; len + 4 <=
// 16 NP) to LDS bytes [d, d + len): dword-aligned funnel shifts and ds_or into the zeroed buffer
// (the first and last words are shared with the neighbouring values). A slot's bytes past the
// entry are zero (k_dict_slots), and so are the pieces not loaded, so the words need no masks:
// the funnel shift brings zeros below the first byte and the padding supplies them past the last.
template <int NP>
DEV void lds_put_slot(uint32_t *lw, uint32_t d, const uint4 *sl, uint32_t len) {
  constexpr int NW = 4 * NP;
  uint32_t W[NW];  // W[0 .. NW-2] = the entry's bytes, W[NW-1] = 0 (funnel tail)
#pragma unroll
  for (int q = 0; q < NW / 4; q++) {
    const uint32_t x[4] = {sl[q].x, sl[q].y, sl[q].z, sl[q].w};
#pragma unroll
    for (int i = 0; i < 4; i++)
      if (4 * q + i >= 1) W[4 * q + i - 1] = x[i];
  }
  W[NW - 1] = 0;
  const uint32_t sh = d & 3u, d0 = d >> 2, end = sh + len;
#pragma unroll
  for (int m = 0; m < NW; m++) {
    if (4u * m >= end) break;
    const uint32_t prev = m ? W[m - 1] : 0u;
    const uint32_t word = sh ? __builtin_amdgcn_alignbyte(W[m], prev, 4 - sh) : W[m];
    if (NP == 2) {  // (64-B slots keep the masks: without them the 16-word loop is not unrolled)
      atomicOr(&lw[d0 + m], word);
    } else {
      const uint32_t lo = max(sh, 4u * m) - 4u * m, hi = min(end, 4u * m + 4) - 4u * m;  // valid bytes [lo, hi)
      const uint32_t mask = (hi >= 4 ? ~0u : ((1u << (8 * hi)) - 1u)) & ~((1u << (8 * lo)) - 1u);
      atomicOr(&lw[d0 + m], word & mask);
    }
  }
}

// Non-temporal 16-B payload stores: the written stream does not displace the dictionary's slot table
// from L2, which every value of the tile gathers from (tools/ubench/ba_ubench.hip: cfg3-shaped emit
// 0.433 -> 0.350 ms); the offsets stores keep the default policy.
typedef uint32_t v4u32 __attribute__((ext_vector_type(4)));
DEV void st_payload16(uint8_t *p, uint4 v) { __builtin_nontemporal_store(v4u32{v.x, v.y, v.z, v.w}, (v4u32 *)p); }
DEV void st_offset(int32_t *p, int32_t v) { *p = v; }
// lds_put's bytes straight to global memory (rounds whose bytes exceed the LDS buffer).
DEV void global_put(uint8_t *dst, const uint8_t *src, uint32_t len) {
  uint32_t k = 0;
  const uint32_t head = min(len, (uint32_t)((4u - ((uintptr_t)dst & 3u)) & 3u));
  for (; k < head; k++) dst[k] = src[k];
  for (; k + 4 <= len; k += 4) *(uint32_t *)(dst + k) = ld32(src + k);
  for (; k < len; k++) dst[k] = src[k];
}

// ---------------------------------------------------------------------------
// Dictionary slots (dict_slots.h); blockIdx.y = the chunk (list of chunks with a slot table).
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_dict_slots(BatchDev b_in, const uint32_t *chunks) {
  const BatchDev b = global_view(b_in);
  dict_slots_block(b, chunks[blockIdx.y], blockIdx.x, gridDim.x);
}

// ---------------------------------------------------------------------------
// Chunks without an upload-time payload bound (CF_BA_SYNC): per-tile payload bytes, then a
// per-chunk scan; the host then sizes the payload and k_ba_emit reads the scanned bases.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_ba_sums(BatchDev b_in) {
  const BatchDev b = global_view(b_in);
  __shared__ DictTileLDS lds;
  __shared__ uint64_t wsum[4];
  const uint32_t t = blockIdx.x, p = b.ba_tile_page[t];
  const PageDesc &pd = b.pages[p];
  const ChunkDesc &cd = b.chunks[pd.chunk];
  if (!(cd.flags & (CF_BA_SYNC | CF_BA_PRESUM))) return;  // workgroup-uniform
  const uint32_t nn = b.page_nn_v[p];
  const uint32_t tv = ba_tile_vals(cd), v0 = (t - pd.ba_tile) * tv, v1 = min(v0 + tv, nn);
  uint64_t sum = 0;
  if (v0 < v1 && !ba_page_failed(b, pd)) {
    if (pd.vkind == VK_DICT) {
      DictTile tl;
      if (dict_tile_load(b, pd, p, v0, v1, nn, lds, tl)) {
        const uint2 *ent = gp_u64<const uint2>(cd.dict_offsets);
        const uint32_t lane = lane_id(), seg0 = v0 + (threadIdx.x >> 6) * 1024;
        DictCursor rc = dict_cursor(tl, max(seg0 + lane, tl.v0));
        for (uint32_t r = 0; r < 16; r++) {
          const uint32_t v = seg0 + r * 64 + lane;
          if (v < tl.v0 || v >= tl.v1) continue;
          const uint32_t idx = dict_cursor_value(tl, lds, rc, v);
          if (idx < cd.dict_count) sum += ent[idx].y;  // out of range: k_ba_emit reports it
        }
      }
    } else {
      const int32_t *len = gp_u64<const int32_t>(cd.offsets) + b.page_vbase[p] + 1;
      for (uint32_t v = v0 + threadIdx.x; v < v1; v += blockDim.x) sum += (uint32_t)len[v];
    }
  }
  const uint64_t tot = block_sum64(sum, wsum);
  if (threadIdx.x == 0) b.ba_tile_sum[t] = tot;
}

__global__ void __launch_bounds__(256) k_ba_scan(BatchDev b_in, const uint32_t *chunks) {
  const BatchDev b = global_view(b_in);
  __shared__ uint64_t wsum[4];
  const uint32_t c = chunks[blockIdx.x];
  const ChunkDesc &cd = b.chunks[c];
  if (!(cd.flags & (CF_BA_SYNC | CF_BA_PRESUM))) return;
  uint64_t *ts = b.ba_tile_sum + cd.ba_tile0;
  uint64_t carry = 0;
  for (uint32_t t0 = 0; t0 < cd.ba_ntiles; t0 += blockDim.x) {
    const uint32_t k = t0 + threadIdx.x;
    const uint64_t v = k < cd.ba_ntiles ? ts[k] : 0;
    uint64_t tot;
    const uint64_t ex = block_excl_scan64(v, wsum, &tot);
    if (k < cd.ba_ntiles) ts[k] = carry + ex;
    carry += tot;
  }
  if (threadIdx.x == 0) b.ba_totals[c] = carry;
}

// ---------------------------------------------------------------------------
// k_ba_emit
// ---------------------------------------------------------------------------
template <uint32_t NR, uint32_t EW>
struct EmitLDST {
  static constexpr uint32_t kWaves = EW;
  DictTileLDST<NR> tile;
  uint4 wbuf[EW][kWaveVec];
  uint64_t wtot[EW];  // the waves' payload bytes
  uint64_t base;      // the tile's payload base
};
using EmitLDS = EmitLDST<kDictRuns, kEmitWaves>;
// Class 3: the first 16-B piece of every slot (length and the first 12 bytes) of a dictionary of at
// most kLdsSlots entries in 16- or 32-B slots is copied into LDS per tile, so pass A's lengths and
// pass B's first pieces are LDS reads instead of random gathers through the texture path (cfg4's
// 1,024 map keys of 6-14 bytes); only entries longer than 12 bytes load their second piece. 256
// runs per tile in LDS keep three workgroups per CU.
constexpr uint32_t kLdsSlots = 1024;
struct EmitLDSSlots {
  EmitLDST<kDictRuns, kEmitWavesLds> e;
  uint4 slots[kLdsSlots];
};

// The tile of block `blk` in class `cls` (~0u: padding of a shorter queue).
DEV uint32_t tile_of_block(const BatchDev &b, uint32_t cls, uint32_t blk) {
  return b.ba_tile_order[b.ba_class_off[cls] + blk];
}

// Payload bytes of tile t, computed by one wave without LDS (a look-back that found tile t
// silent): the same sum tile t's own workgroup publishes (values the run scan did not validate,
// and dictionary indices out of range, count 0).
template <class TL>
DEV uint64_t tile_aggregate(const BatchDev &b, uint32_t t, const TL &unstaged) {
  const uint32_t p = b.ba_tile_page[t], lane = lane_id();
  const PageDesc &pd = b.pages[p];
  const ChunkDesc &cd = b.chunks[pd.chunk];
  const uint32_t nn = b.page_nn_v[p];
  const uint32_t tv = ba_tile_vals(cd), v0 = (t - pd.ba_tile) * tv, v1 = min(v0 + tv, nn);
  uint64_t sum = 0;
  if (v0 < v1) {
    if (pd.vkind == VK_DICT) {
      DictTile tl;
      uint32_t r0, r1;
      if (dict_tile_open(b, pd, p, v0, v1, nn, tl, r0, r1)) {
        const uint2 *ent = gp_u64<const uint2>(cd.dict_offsets);
        uint32_t ri = dict_tile_seek(tl, tl.v0 + lane);
        for (uint32_t v = tl.v0 + lane; v < tl.v1; v += 64) {
          const uint32_t x = dict_tile_value(tl, unstaged, ri, v);  // not staged: global reads only
          if (x < cd.dict_count) sum += ent[x].y;
        }
      }
    } else {
      const int32_t *len = gp_u64<const int32_t>(cd.offsets) + b.page_vbase[p] + 1;
      for (uint32_t v = v0 + lane; v < v1; v += 64) sum += (uint32_t)len[v];
    }
  }
  return wave_sum64(sum);
}

// The tile's payload base: exclusive prefix of the chunk's tile sums, by decoupled look-back,
// run by one wave. Every tile publishes its sum (kStAgg) at once and its inclusive prefix
// (kStIncl) when known; a state word is written by agent-scope atomics and read by agent-scope
// loads, and carries its own data (no separate payload to order). Those go to memory, so the
// wave reads kLbWin predecessors at a time (the nearest inclusive prefix is usually among
// them); a predecessor still silent after kHelpSpins polls has its sum computed here, so the
// wait is bounded whatever the dispatch order.
template <class TL>
DEV uint64_t lookback(const BatchDev &b, const ChunkDesc &cd, uint32_t c, uint32_t t, uint64_t agg,
                      const TL &lds, Stamps &sp) {
  uint64_t *st = b.ba_state;
  const uint32_t lane = lane_id(), j = t - cd.ba_tile0;
  if (j == 0) {
    if (lane == 0) {
      __hip_atomic_exchange(&st[(uint64_t)t * kStStride], kStIncl | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (cd.ba_ntiles == 1) b.ba_totals[c] = agg;
    }
    return 0;
  }
  if (lane == 0) __hip_atomic_exchange(&st[(uint64_t)t * kStStride], kStAgg | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  uint64_t base = 0;
  int64_t k = (int64_t)t - 1;  // the nearest tile not yet added
  uint32_t spins = 0;
  for (;;) {
    const int64_t my = k - (int64_t)lane;
    const bool valid = lane < kLbWin && my >= (int64_t)cd.ba_tile0;
    uint64_t s = kStIncl;  // past the chunk's first tile: an inclusive prefix of 0
    if (lane < kLbWin) {
      s = valid ? __hip_atomic_load(&st[(uint64_t)my * kStStride], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : kStIncl;
      if (PQ_ABLATE(b, 12) && valid) s = 0;  // diagnostic: every predecessor silent (self-help only)
    }
    const uint64_t win = lane < kLbWin;
    const uint64_t incl = __ballot(win && (s & ~kStMask) == kStIncl), zero = __ballot(win && s == 0);
    const uint32_t stop = incl ? (uint32_t)__builtin_ctzll(incl) : 64u;
    const uint32_t hole = zero ? (uint32_t)__builtin_ctzll(zero) : 64u;
    const uint32_t upto = min(min(stop + 1, hole), kLbWin);  // lanes [0, upto) are added
    base += wave_sum64(lane < upto ? (s & kStMask) : 0);
    sp.count(6);
    if (stop < hole) break;  // reached an inclusive prefix (or the chunk's first tile)
    k -= upto;
    if (hole < 64) {
      if (upto) spins = 0;
      if (++spins > kHelpSpins || PQ_ABLATE(b, 12)) {  // tile k is silent: compute its sum
        base += tile_aggregate(b, (uint32_t)k, lds);
        sp.count(5);
        if (k == (int64_t)cd.ba_tile0) break;
        k--;
        spins = 0;
        continue;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  if (lane == 0) {
    __hip_atomic_exchange(&st[(uint64_t)t * kStStride], kStIncl | (base + agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (j == cd.ba_ntiles - 1) b.ba_totals[c] = base + agg;
  }
  return base;
}

// One tile (see the file comment). SLOT: a dictionary page whose entries are read from the
// slot table (any slot size: a value loads the 16-B pieces its entry occupies), else bytes are
// read from their source (dictionaries without slots, PLAIN / DELTA pages). Pass B works in
// groups of G rounds: the G rounds' loads are issued together.
// (Tried and removed: pass A loading every value's whole 32-B slot by lane pairs and keeping the
// pieces in registers -- 0.288 ms in tools/ubench/ba_ubench.hip, but 128 VGPRs with spills in the
// product kernel, 0.428 against 0.352 ms, profiles/r05_s4_probe_ba_emit.txt; the second pieces by
// LDS-DMA, profiles/r06_t_probe_ba_dma.txt.)
// P0 (16- and 32-B slots): pass A loads every value's first slot piece (its length and first 12
// bytes) instead of the length word, and keeps it; pass B loads only the second piece of entries
// longer than 12 bytes: 1 + P(len > 12) texture requests per value instead of 2 + P(len > 12).
// At 5 waves per SIMD (96 VGPRs) cfg3's k_ba_emit 0.358 -> 0.346 ms (profiles/r05_s29_probe_ba_p0.txt;
// at 6 the pieces spill, at 4 it measured the same as 5).
#ifndef PQ_BA_P0
#define PQ_BA_P0 1
#endif
#ifndef PQ_BA_G
#define PQ_BA_G 2  // pass B: rounds whose slot pieces are loaded together
#endif
template <bool SLOT, uint32_t SV = SLOT ? 4 : 1, bool LS = false, class EL, bool P0 = false>
DEV void emit_tile(const BatchDev &b, const PageDesc &pd, const ChunkDesc &cd, uint32_t t, uint32_t p, uint32_t v0,
                   uint32_t lo, uint32_t hi, bool is_dict, bool have, DictTile &tl, EL &L, Stamps &st,
                   const uint4 *lslots = nullptr) {
  // SV: uint4 per slot (at most)
  constexpr uint32_t G = PQ_BA_G;        // rounds per load group
  const uint32_t s4 = cd.slot_shift - 4; // SLOT: uint4 per slot = 1 << s4
  constexpr uint32_t R = kRounds;
  const uint64_t vb = b.page_vbase[p];
  int32_t *offs = gp_u64<int32_t>(cd.offsets) + vb;
  uint8_t *P = gp_u64<uint8_t>(cd.payload);
  const uint32_t lane = lane_id(), wv = threadIdx.x >> 6, seg0 = v0 + wv * 64 * R;
  const uint2 *ent = gp_u64<const uint2>(cd.dict_offsets);
  const uint64_t *srcs = gp_u64<const uint64_t>(cd.ba_index) + vb;
  const uint8_t *draw = gp_u64<const uint8_t>(cd.dict_raw);
  const uint4 *slots = gp_u64<const uint4>(cd.dict_slots);
  // ---- pass A: indices (LDS), then the lengths (slot word 0) for all rounds at once
  uint32_t idx[R];
  uint32_t first_err = 0xffffffffu;
  DictCursor rc = (is_dict && have) ? dict_cursor(tl, max(seg0 + lane, lo)) : DictCursor{0, 0, 0, 0, 0xffffffffu};
#pragma unroll
  for (uint32_t r = 0; r < R; r++) {
    const uint32_t v = seg0 + r * 64 + lane;
    idx[r] = ~0u;
    if (have && v >= lo && v < hi) {
      if (is_dict) {
        const uint32_t x = dict_cursor_value(tl, L.tile, rc, v);
        if (x < cd.dict_count) idx[r] = x;
        else first_err = min(first_err, v);
      } else {
        idx[r] = v;
      }
    }
  }
  uint32_t pos[R];  // S == 0 dictionaries: the entry's position in the dictionary page
  uint32_t len[R];
  uint4 p0[P0 ? R : 1];     // P0: the values' first slot pieces
#pragma unroll
  for (uint32_t r = 0; r < R; r++) {
    pos[r] = 0;
    len[r] = 0;
    if constexpr (P0) {
      p0[r] = idx[r] != ~0u ? slots[(uint64_t)idx[r] << s4] : make_uint4(0u, 0u, 0u, 0u);
      len[r] = p0[r].x;  // (0 where there is no value)
      continue;
    }
    if (idx[r] != ~0u) {
      if (PQ_ABLATE(b, 11)) {  // diagnostic: no length loads
        len[r] = 16;
      } else if (LS) {
        len[r] = lslots[idx[r]].x;  // LDS copy of the slot table (16-B slots)
      } else if (SLOT) {
        len[r] = ((const uint32_t *)slots)[(uint64_t)idx[r] << (s4 + 2)];
      } else if (is_dict) {
        const uint2 e = ent[idx[r]];
        pos[r] = e.x;
        len[r] = e.y;
      } else {
        len[r] = (uint32_t)offs[idx[r] + 1];
      }
    }
  }
  uint64_t mine = 0;
#pragma unroll
  for (uint32_t r = 0; r < R; r++) mine += len[r];
  bool fail = false;
  if (__ballot(first_err != 0xffffffffu)) {  // the page fails at its first bad index
    for (int o = 32; o; o >>= 1) first_err = min(first_err, (uint32_t)__shfl_xor((int)first_err, o));
    if (lane == 0) report(b, pd.chunk, 1, pd.page_in_chunk, ST_VALUES, first_err, PQ_ERR_DICT_INDEX);
    fail = true;
  }
  const uint64_t wt = wave_sum64(mine);
  st.lap(1);
  uint4 *wb = &L.wbuf[wv][0];
  for (uint32_t k = lane; k < kWaveVec; k += 64) wb[k] = make_uint4(0u, 0u, 0u, 0u);
  if (lane == 0) L.wtot[wv] = wt;
  wg_barrier();
  st.lap(2);
  // ---- the tile's base: k_ba_scan's (CF_BA_SYNC chunks) or the look-back's (wave 0)
  if (wv == 0) {
    uint64_t agg = 0;
    for (uint32_t q = 0; q < EL::kWaves; q++) agg += L.wtot[q];
    const uint64_t base = (cd.flags & (CF_BA_SYNC | CF_BA_PRESUM)) ? b.ba_tile_sum[t]
                          : PQ_ABLATE(b, 8) ? 0  // diagnostic: no look-back
                                            : lookback(b, cd, pd.chunk, t, agg, L.tile, st);
    if (lane == 0) L.base = base;
    st.lap(3);
  }
  wg_barrier();
  st.lap(4);
  uint64_t wbase = L.base;
  for (uint32_t q = 0; q < wv; q++) wbase += L.wtot[q];
  // write nothing for a failed page, or past the payload bound (a corrupt length); from here on
  // the wave works alone (no workgroup barrier)
  fail |= ba_page_failed(b, pd) || wbase + wt > cd.payload_capacity;
  if (fail || !P || PQ_ABLATE(b, 9)) return;  // wave-uniform (diagnostic: no pass B)
  wave_lds_sync();
  uint8_t *lb = (uint8_t *)wb;
  uint32_t *lw = (uint32_t *)wb;
  // ---- pass B: the wave's bytes form one contiguous range of the payload. They are assembled
  // in the LDS buffer at their final 16-B alignment: LDS byte 0 is the global byte gblk; whole
  // 16-B pieces leave as aligned stores, the unfinished last piece is carried to the next
  // round; bytes of the first piece before `own` belong to the previous range.
  uint8_t *gblk = P + wbase - ((uintptr_t)(P + wbase) & 15u);
  uint32_t cur = (uint32_t)((uintptr_t)(P + wbase) & 15u), own = cur;
#pragma unroll
  for (uint32_t g = 0; g < R / G; g++) {
    uint4 sl[G][SV];
    const uint8_t *src[G];  // S == 0: the values' bytes
#pragma unroll
    for (uint32_t rr = 0; rr < G; rr++) {
      const uint32_t r = g * G + rr;
      src[rr] = nullptr;
      if (!SLOT && idx[r] != ~0u) src[rr] = is_dict ? draw + pos[r] : gp_u64<const uint8_t>(srcs[idx[r]]);
    }
    if constexpr (SLOT) {
#pragma unroll
      for (uint32_t rr = 0; rr < G; rr++) {
        const uint32_t r = g * G + rr;
#pragma unroll
        for (uint32_t q = 0; q < SV; q++)  // the slot pieces holding bytes of the entry (none: no value)
          sl[rr][q] = (P0 && q == 0) ? p0[r]
                      : len[r] && len[r] + 4 > 16 * q && !(q && PQ_ABLATE(b, 14))  // (diagnostic: no later pieces)
                          ? ((LS && q == 0) ? lslots[idx[r]] : slots[((uint64_t)idx[r] << s4) + q])
                          : make_uint4(0u, 0u, 0u, 0u);
      }
    }
#pragma unroll
    for (uint32_t rr = 0; rr < G; rr++) {
      const uint32_t r = g * G + rr;
      const uint32_t v = seg0 + r * 64 + lane;
      const uint32_t l = len[r];
      const uint32_t incl = wave_incl_scan32(l);
      const uint32_t T = rdlane(incl, 63);
      const uint32_t ex = incl - l;
      if (v >= lo && v < hi && !PQ_ABLATE(b, 13)) st_offset(&offs[v + 1], (int32_t)(wbase + incl));  // (diagnostic: no stores)
      if (!T) continue;
      if (cur + T <= kWaveBuf) {
        if (l) {
          if constexpr (SLOT) {
            lds_put_slot<SV>(lw, cur + ex, sl[rr], l);
          } else if (src[rr]) {
            lds_put(lb, cur + ex, src[rr], l);
          }
        }
        wave_lds_sync();
        const uint32_t end = cur + T, full = end >> 4;
        const uint32_t k0 = own ? 1u : 0u;
        if (!PQ_ABLATE(b, 13)) {
          for (uint32_t k = k0 + lane; k < full; k += 64) st_payload16(gblk + 16 * k, wb[k]);
          if (own && full && lane >= own && lane < 16) gblk[lane] = lb[lane];
        }
        wave_lds_sync();
        if (full) {
          if (lane == 0) wb[0] = wb[full];  // the unfinished piece becomes piece 0
          wave_lds_sync();
          for (uint32_t k = 1 + lane; k <= full; k += 64) wb[k] = make_uint4(0u, 0u, 0u, 0u);
          wave_lds_sync();
          gblk += 16 * full;
          own = 0;
        }
        cur = end & 15u;
      } else {
        // bytes beyond the LDS buffer: flush what is buffered, then each lane writes its value
        if (lane >= own && lane < cur) gblk[lane] = lb[lane];
        if (l) {
          const uint8_t *from = SLOT ? (const uint8_t *)(slots + ((uint64_t)idx[r] << s4)) + 4
                                  : src[rr];
          if (from) global_put(P + wbase + ex, from, l);
        }
        const uint64_t e = wbase + T;
        gblk = P + e - ((uintptr_t)(P + e) & 15u);
        cur = own = (uint32_t)((uintptr_t)(P + e) & 15u);
        wave_lds_sync();
        if (lane == 0) wb[0] = make_uint4(0u, 0u, 0u, 0u);
        wave_lds_sync();
      }
      wbase += T;
    }
  }
  if (lane >= own && lane < cur) gblk[lane] = lb[lane];  // the last, unfinished piece
  st.lap(5);
}

// Classes: chunks whose pages are all dictionary pages with a slot table of 16/32-byte (class 0)
// or 64-byte slots (class 1), compiled without the source path; class 2: any page; class 3: as
// class 0 with at most kLdsSlots entries, their first slot pieces read from LDS.
template <uint32_t CLS, class EL>
DEV void ba_emit(const BatchDev &b, EL &L, const uint4 *lslots = nullptr) {
  PQ_STAMPS(st, b.dbg);
  st.begin();
  const uint32_t t = tile_of_block(b, CLS, blockIdx.x);
  if (t == ~0u) return;  // queue padding (workgroup-uniform)
  const uint32_t p = b.ba_tile_page[t];
  const PageDesc &pd = b.pages[p];
  const ChunkDesc &cd = b.chunks[pd.chunk];
  const uint32_t nn = b.page_nn_v[p];
  const uint32_t tv = ba_tile_vals(cd), v0 = (t - pd.ba_tile) * tv, v1 = min(v0 + tv, nn);
  if (b.page_vbase[p] + v0 == 0 && threadIdx.x == 0 && cd.offsets) gp_u64<int32_t>(cd.offsets)[0] = 0;
  const bool is_dict = pd.vkind == VK_DICT;
  DictTile tl;
  uint32_t lo = v0, hi = v1;
  bool have = v0 < v1;
  if (is_dict && have) {
    have = dict_tile_load(b, pd, p, v0, v1, nn, L.tile, tl);
    lo = tl.v0;
    hi = tl.v1;
  }
  st.lap(0);
  if (CLS == 3) emit_tile<true, 2, true>(b, pd, cd, t, p, v0, lo, hi, is_dict, have, tl, L, st, lslots);
  else if (CLS == 0) emit_tile<true, 2, false, EL, PQ_BA_P0 != 0>(b, pd, cd, t, p, v0, lo, hi, is_dict, have, tl, L, st);
  else if (CLS == 1 || (is_dict && cd.slot_shift)) emit_tile<true>(b, pd, cd, t, p, v0, lo, hi, is_dict, have, tl, L, st);
  else emit_tile<false>(b, pd, cd, t, p, v0, lo, hi, is_dict, have, tl, L, st);
  st.count(7);
  st.flush(40);
}

// class 0: with the first pieces in registers (PQ_BA_P0) <= 96 VGPRs (five 4-wave workgroups per CU)
#ifndef PQ_BA_WPE
#define PQ_BA_WPE (PQ_BA_P0 ? 5 : 6)
#endif
__global__ void __launch_bounds__(64 * kEmitWaves) __attribute__((amdgpu_waves_per_eu(PQ_BA_WPE))) k_ba_emit_slots(BatchDev b_in) {
  const BatchDev b = global_view(b_in);
  __shared__ EmitLDS L;
  ba_emit<0>(b, L);
}
__global__ void __launch_bounds__(64 * kEmitWaves) k_ba_emit_slots64(BatchDev b_in) {
  const BatchDev b = global_view(b_in);
  __shared__ EmitLDS L;
  ba_emit<1>(b, L);
}
__global__ void __launch_bounds__(64 * kEmitWaves) k_ba_emit(BatchDev b_in) {
  const BatchDev b = global_view(b_in);
  __shared__ EmitLDS L;
  ba_emit<2>(b, L);
}
__global__ void __launch_bounds__(64 * kEmitWavesLds) __attribute__((amdgpu_waves_per_eu(6))) k_ba_emit_lds(BatchDev b_in) {
  const BatchDev b = global_view(b_in);
  __shared__ EmitLDSSlots L;
  const uint32_t t = tile_of_block(b, 3, blockIdx.x);
  if (t == ~0u) return;  // queue padding (workgroup-uniform)
  const ChunkDesc &cd = b.chunks[b.pages[b.ba_tile_page[t]].chunk];
  const uint4 *gs = gp_u64<const uint4>(cd.dict_slots);
  const uint32_t s4 = cd.slot_shift - 4;
  for (uint32_t k = threadIdx.x; k < cd.dict_count; k += blockDim.x) L.slots[k] = gs[(uint64_t)k << s4];
  wg_barrier();
  ba_emit<3>(b, L.e, L.slots);
}

hipError_t launch_dict_slots(const BatchDev &b, const LaunchLists &l, hipStream_t s) {
  if (!l.n_slot_chunks) return hipSuccess;
  hipLaunchKernelGGL(k_dict_slots, dim3(l.slot_grid_x, l.n_slot_chunks), dim3(256), 0, s, b, l.slot_chunks);
  return hipGetLastError();
}
hipError_t launch_ba_sums(const BatchDev &b, const LaunchLists &l, hipStream_t s) {
  if (!l.n_ba_tiles) return hipSuccess;
  hipLaunchKernelGGL(k_ba_sums, dim3(l.n_ba_tiles), dim3(256), 0, s, b);
  return hipGetLastError();
}
hipError_t launch_ba_scan(const BatchDev &b, const LaunchLists &l, hipStream_t s) {
  if (!l.n_ba_chunks) return hipSuccess;
  hipLaunchKernelGGL(k_ba_scan, dim3(l.n_ba_chunks), dim3(256), 0, s, b, l.ba_chunks);
  return hipGetLastError();
}
hipError_t launch_ba_emit(const BatchDev &b, const LaunchLists &l, hipStream_t s) {
  // the two classes never share a chunk, so no look-back crosses the launches
  if (l.n_ba_class[0]) hipLaunchKernelGGL(k_ba_emit_slots, dim3(l.n_ba_class[0]), dim3(64 * kEmitWaves), 0, s, b);
  if (l.n_ba_class[1]) hipLaunchKernelGGL(k_ba_emit_slots64, dim3(l.n_ba_class[1]), dim3(64 * kEmitWaves), 0, s, b);
  if (l.n_ba_class[2]) hipLaunchKernelGGL(k_ba_emit, dim3(l.n_ba_class[2]), dim3(64 * kEmitWaves), 0, s, b);
  if (l.n_ba_class[3]) hipLaunchKernelGGL(k_ba_emit_lds, dim3(l.n_ba_class[3]), dim3(64 * kEmitWavesLds), 0, s, b);
  return hipGetLastError();
}

}  // namespace pq
