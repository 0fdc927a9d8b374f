// level_fill.h — fill tiles of the generic level streams: k_levels / k_levels_segw write a run
// table per stream (first value index, bit-packed flag | payload position, or the RLE value) and
// the run holding every fill tile's first value; k_level_fill (flat and non-nested chunks),
// k_nest_count and k_nest_emit (nested chunks, nested.hip) expand them tile by tile.
#pragma once
#include "dev_util.h"

namespace pq {

constexpr uint32_t kLfTile = kLfTileHost;  // values per fill tile (aligned on the chunk's slots)
constexpr uint32_t kLfRuns = 2048;         // runs of a tile's stream staged in LDS
// Fill tiles of a page: the kLfTile-slot blocks of the chunk that hold any of its slots.
DEV uint32_t lf_tiles(uint64_t slot_base, uint32_t ns) {
  return ns ? (uint32_t)((slot_base + ns - 1) / kLfTile - slot_base / kLfTile + 1) : 0u;
}

// The eight values of the group [g, g + 8) that lie in [vs, ve), from run table `R` (m runs):
// one step per run the values cross (usually one, at a run boundary two), each step an RLE
// broadcast or one read of the bit-packed payload, so the lanes of a wave stay converged.
// lf_group_from: the same from run j, the run of a value at or before vs (it advances to vs's run).
template <class RT>
DEV void lf_group_from(const RT &R, uint32_t m, uint32_t j, const uint8_t *src, uint32_t n, uint32_t bw, uint32_t cmp,
                       int64_t g, uint32_t vs, uint32_t ve, uint64_t &word, uint32_t &eq) {
  word = 0;
  eq = 0;
  if (vs >= ve) return;
  while (j + 1 < m && R(j + 1).x <= vs) j++;
  const uint32_t bmask = (1u << bw) - 1u;
  for (uint32_t v = vs; v < ve; j++) {
    const uint2 r = R(j);
    const uint32_t se = j + 1 < m ? min(ve, R(j + 1).x) : ve;  // this run's part of the group
    const uint32_t cnt = se - v, sh = v - (uint32_t)g;
    uint64_t pk;
    uint32_t e;
    if (!(r.y >> 31)) {  // RLE
      pk = 0x0101010101010101ull * (uint64_t)(r.y & 0xffu);
      e = r.y == cmp ? 0xffu : 0u;
    } else if (bw == 1) {  // bit-packed, 1-bit levels: nibble -> bytes by one multiply (SWAR; cfg4
      // k_nest_tile 0.632 -> 0.607 ms with the 2-bit case below, profiles/r05_s46_probe_lf_swar.txt)
      // (x * 0x204081 places bit k of a nibble at 8k and its other copies at 7k'..: no two overlap)
      const uint32_t x = (uint32_t)bits64c(src, n, (uint64_t)(r.y & 0x7fffffffu) * 8 + (uint64_t)(v - r.x), cnt);
      const uint32_t lo = ((x & 0xfu) * 0x00204081u) & 0x01010101u, hi = (((x >> 4) & 0xfu) * 0x00204081u) & 0x01010101u;
      pk = ((uint64_t)hi << 32) | lo;
      e = cmp == 1 ? x : cmp == 0 ? ~x : 0u;
    } else if (bw == 2) {  // bit-packed, 2-bit levels: fields -> bytes by two shift-or steps
      const uint32_t x = (uint32_t)bits64c(src, n, (uint64_t)(r.y & 0x7fffffffu) * 8 + (uint64_t)(v - r.x) * 2, cnt * 2);
      uint32_t lo = x & 0xffu, hi = (x >> 8) & 0xffu;
      lo = (lo | (lo << 12)) & 0x000f000fu;
      hi = (hi | (hi << 12)) & 0x000f000fu;
      lo = (lo | (lo << 6)) & 0x03030303u;
      hi = (hi | (hi << 6)) & 0x03030303u;
      pk = ((uint64_t)hi << 32) | lo;
      // fields equal to cmp: zero 2-bit fields of x ^ cmp..., their low bits compressed to one bit each
      const uint32_t t = x ^ (cmp * 0x5555u);
      uint32_t z = ~(t | (t >> 1)) & 0x5555u;
      z = (z | (z >> 1)) & 0x3333u;
      z = (z | (z >> 2)) & 0x0f0fu;
      e = cmp < 4 ? (z | (z >> 4)) & 0xffu : 0u;  // (no 2-bit field equals a larger cmp)
    } else if (bw <= 7) {  // bit-packed: one read for the segment
      const uint64_t x = bits64c(src, n, (uint64_t)(r.y & 0x7fffffffu) * 8 + (uint64_t)(v - r.x) * bw, cnt * bw);
      pk = 0;
      e = 0;
#pragma unroll
      for (uint32_t q = 0; q < 8; q++) {
        const uint32_t lv = (uint32_t)(x >> (q * bw)) & bmask;
        pk |= (uint64_t)lv << (8 * q);
        e |= (uint32_t)(lv == cmp) << q;
      }
    } else {  // wide levels (max level >= 128): value by value
      pk = 0;
      e = 0;
      for (uint32_t q = 0; q < cnt; q++) {
        const uint32_t lv = bits32c(src, n, (uint64_t)(r.y & 0x7fffffffu) * 8 + (uint64_t)(v + q - r.x) * bw, bw);
        pk |= (uint64_t)(lv & 0xffu) << (8 * q);
        e |= (uint32_t)(lv == cmp) << q;
      }
    }
    const uint64_t bm = cnt >= 8 ? ~0ull : ((1ull << (8 * cnt)) - 1ull);
    word |= (pk & bm) << (8 * sh);
    eq |= (e & ((1u << cnt) - 1u)) << sh;
    v = se;
  }
}

template <class RT>
DEV void lf_group(const RT &R, uint32_t m, const uint8_t *src, uint32_t n, uint32_t bw, uint32_t cmp, int64_t g,
                  uint32_t vs, uint32_t ve, uint64_t &word, uint32_t &eq) {
  word = 0;
  eq = 0;
  if (vs >= ve) return;
  uint32_t j = 0;
  for (uint32_t step = 1u << (31 - __builtin_clz(m)); step; step >>= 1)
    if (j + step < m && R(j + step).x <= vs) j += step;
  lf_group_from(R, m, j, src, n, bw, cmp, g, vs, ve, word, eq);
}

}  // namespace pq
