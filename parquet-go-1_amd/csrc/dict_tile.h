// dict_tile.h — the values of one tile of a hybrid-encoded VALUE stream (dictionary indices,
// type_dict.go:40-60; boolean RLE, type_boolean.go:109-120), for the kernels that consume
// them (k_values WI_DICT, k_ba_sums, k_ba_emit).
//
// k_scan_runs has already walked the page's run-header chain (hybrid_decoder.go:142-165) into
// a run table (HybRun: first value, payload position, RLE value / bit-packed flag) with the run
// covering the first value of every kDictTile-value tile. A tile load copies the tile's runs to
// LDS and stages the stream bytes the tile's bit-packed values occupy (one coalesced sweep of
// 16-B loads; bytes at or past the stream end read as zero, the short-final-group zero fill of
// hybrid_decoder.go:132-140). Values are then read by lanes in any order: a per-lane run cursor
// advances monotonically, and each bit-packed value is one LDS funnel read.
#pragma once
#include "dev_util.h"

namespace pq {

#ifndef PQ_DICT_RUNS
#define PQ_DICT_RUNS 256
#endif
#ifndef PQ_DICT_WPE
#define PQ_DICT_WPE 8
#endif
constexpr uint32_t kTileRuns = 1024;          // runs held in LDS (a tile with more reads the run table)
constexpr uint32_t kDictRuns = PQ_DICT_RUNS;  // the same for k_values_dict (smaller: 8 workgroups per CU)
constexpr uint32_t kTileStageB = 16896;       // staged stream bytes (a wider tile reads global memory)
template <uint32_t NR>
struct DictTileLDST {
  HybRun runs[NR];
  uint32_t stage[kTileStageB / 4 + 8];
};
using DictTileLDS = DictTileLDST<kTileRuns>;

struct DictTile {
  const uint8_t *s;      // value stream (after the bit-width byte)
  uint32_t n, bw;        // stream bytes, index bit width
  const HybRun *runs;    // the tile's runs: LDS copy, or the run table in global memory
  uint32_t nr;           // number of runs
  uint64_t sbit;         // stream bit of stage[0] (staged)
  uint32_t v0, v1;       // tile values [v0, v1) after clipping to the runs the scan validated
  uint32_t lo, hi;       // stream bytes of the tile's bit-packed values (from the descriptor)
  bool staged;
};

// Open tile [v0, v1) of page `page` (values within the page; a whole kDictTile tile, clipped to the
// page's values) without staging: one read of the tile's descriptor, written by k_scan_runs after its
// walk ({first run, last run, stream bytes [lo, hi)}, {values the valid runs cover, valid}); the
// runs are then read from the run table in global memory. Returns false when no value of the tile
// is decodable (the scan failed before it: the error is already reported at the right value
// position). Any lane may call it.
DEV bool dict_tile_open(const BatchDev &b, const PageDesc &pd, uint32_t page, uint32_t v0, uint32_t v1, uint32_t nn,
                        DictTile &t, uint32_t &r0, uint32_t &r1) {
  (void)nn;
  t.s = gp_u64<const uint8_t>(pd.data) + pd.val_off;
  t.n = pd.val_len;
  t.bw = pd.dict_bw;
  t.nr = 0;
  t.staged = false;
  t.runs = nullptr;
  t.sbit = 0;
  t.v0 = v0;
  t.v1 = v1;
  t.lo = t.hi = 0;
  if (t.bw == 0) return v0 < v1;  // bit width 0: every index is 0 and no stream is read
  const uint64_t di = 2 * ((uint64_t)pd.dict_tile0 + v0 / kDictTile);
  const uint4 D = b.tile_desc[di], E = b.tile_desc[di + 1];
  if (E.y != 1u) return false;  // 1 = written valid by this decode's k_scan_runs (the region is 0xff-filled)
  r0 = D.x;
  r1 = D.y;
  t.v1 = min(v1, E.x);  // values covered by valid runs
  if (t.v0 >= t.v1) return false;
  t.nr = r1 - r0 + 1;
  t.runs = b.runs + b.run_base[page] + r0;
  t.lo = D.z;
  t.hi = D.w;
  return true;
}

// Stage stream bytes [lo, hi) of tile t's stream in L.stage (one coalesced sweep of 16-B loads; bytes
// at or past the stream end read as zero) when they fit with `reserve` bytes left at the stage's end.
template <uint32_t NR>
DEV void dict_tile_stage(DictTileLDST<NR> &L, DictTile &t, uint64_t lo, uint64_t hi, uint32_t reserve) {
  const uintptr_t ga = ((uintptr_t)(t.s + lo)) & ~(uintptr_t)15;  // 16-B aligned global start
  const uint64_t sb = (uint64_t)(ga - (uintptr_t)t.s);             // its stream offset (may be "negative")
  const uint64_t span = hi > lo ? (hi + 8) - (lo & ~(uint64_t)15) + 16 : 0;
  if (span + reserve > kTileStageB) return;  // reserve: bytes at the stage's end the caller keeps
  t.staged = true;
  t.sbit = sb * 8;
  const uint4 *src = (const uint4 *)gp_u64<const uint8_t>((uint64_t)ga);
  const uint32_t nv = (uint32_t)((span + 15) / 16);
  for (uint32_t k = threadIdx.x; k < nv; k += blockDim.x) {
    uint4 x = src[k];
    // zero the bytes at or past the stream end (stream offset sb + 16k + j >= n)
    const int64_t rel = (int64_t)t.n - (int64_t)(sb + 16ull * k);  // stream bytes left at this block
    if (rel < 16) {
      uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const int64_t r = rel - 4 * q;
        w[q] = r >= 4 ? w[q] : (r <= 0 ? 0u : (w[q] & ((1u << (8 * r)) - 1u)));
      }
      x = make_uint4(w[0], w[1], w[2], w[3]);
    }
    *(uint4 *)&L.stage[4 * k] = x;
  }
  if (threadIdx.x < 8) L.stage[4 * nv + threadIdx.x] = 0;  // funnel reads past the last block
}

// Load tile [v0, v1) of page `page`: dict_tile_open, then the runs (up to NR) and the
// stream bytes of the tile's bit-packed values are staged in LDS. Every thread of the workgroup
// calls it; it ends with a barrier unless it returns false or the bit width is 0 (both
// workgroup-uniform).
template <uint32_t NR>
DEV bool dict_tile_load(const BatchDev &b, const PageDesc &pd, uint32_t page, uint32_t v0, uint32_t v1, uint32_t nn,
                        DictTileLDST<NR> &L, DictTile &t, uint32_t reserve = 0) {
  uint32_t r0 = 0, r1 = 0;
  if (!dict_tile_open(b, pd, page, v0, v1, nn, t, r0, r1)) return false;
  if (t.bw == 0) return true;
  const HybRun *rg = t.runs;
  if (t.nr <= NR) {
    for (uint32_t k = threadIdx.x; k < t.nr; k += blockDim.x) L.runs[k] = rg[k];
    t.runs = L.runs;
  }
  dict_tile_stage(L, t, t.lo, t.hi, reserve);  // the descriptor's [lo, hi)
  wg_barrier();
  return true;
}

// Up to N consecutive tiles of one page ([v0, v1) cut at kDictTile boundaries) loaded together:
// every descriptor is read at once, and the union of their runs (contiguous in the run table,
// neighbours share at most one) and of their stream bytes is staged under ONE barrier, so a
// workgroup pays the tile-load latency chain once for all of them. nt = the tiles loaded (a prefix:
// a tile is never valid after an invalid one, since the scan validates runs in stream order).
// Ends with a barrier iff nt > 0 and the bit width is not 0 (workgroup-uniform).
template <uint32_t N, uint32_t NR>
DEV void dict_tile_loadn(const BatchDev &b, const PageDesc &pd, uint32_t page, uint32_t v0, uint32_t v1, uint32_t nn,
                         DictTileLDST<NR> &L, DictTile (&t)[N], uint32_t &nt, uint32_t reserve = 0) {
  uint32_t r0[N], r1[N];
  bool ok[N];
#pragma unroll
  for (uint32_t k = 0; k < N; k++) {
    const uint32_t a = v0 + k * kDictTile;
    ok[k] = a < v1 && dict_tile_open(b, pd, page, a, min(a + kDictTile, v1), nn, t[k], r0[k], r1[k]);
  }
  nt = 0;
#pragma unroll
  for (uint32_t k = 0; k < N; k++)
    if (ok[k] && nt == k) nt = k + 1;
  if (nt == 0 || t[0].bw == 0) return;
  uint32_t rl = r1[0];
  uint64_t lo = t[0].lo, hi = t[0].hi;
#pragma unroll
  for (uint32_t k = 1; k < N; k++)
    if (k < nt) {
      rl = r1[k];
      lo = min(lo, (uint64_t)t[k].lo);
      hi = max(hi, (uint64_t)t[k].hi);
    }
  const uint32_t nr = rl - r0[0] + 1;  // the union of the runs
  if (nr <= NR) {
    const HybRun *rg = t[0].runs;
    for (uint32_t k = threadIdx.x; k < nr; k += blockDim.x) L.runs[k] = rg[k];
#pragma unroll
    for (uint32_t k = 0; k < N; k++) t[k].runs = L.runs + (r0[k] - r0[0]);
  }
  dict_tile_stage(L, t[0], lo, hi, reserve);
#pragma unroll
  for (uint32_t k = 1; k < N; k++) {
    t[k].staged = t[0].staged;
    t[k].sbit = t[0].sbit;
  }
  wg_barrier();
}

// The run of value v: binary search over the tile's runs (first value of a lane).
DEV uint32_t dict_tile_seek(const DictTile &t, uint32_t v) {
  if (t.bw == 0) return 0;
  uint32_t lo = 0, hi = t.nr;
  while (hi - lo > 1) {
    const uint32_t m = (lo + hi) >> 1;
    if (t.runs[m].value_start <= v) lo = m; else hi = m;
  }
  return lo;
}

// Index of value v (v inside [t.v0, t.v1)); `ri` is the lane's run cursor (values visited by a
// lane must not decrease).
template <class L_>
DEV uint32_t dict_tile_value(const DictTile &t, const L_ &L, uint32_t &ri, uint32_t v) {
  if (t.bw == 0) return 0;
  while (ri + 1 < t.nr && t.runs[ri + 1].value_start <= v) ri++;
  const HybRun r = t.runs[ri];
  if (!(r.info & 0x80000000u)) return r.info;
  const uint64_t bo = (uint64_t)r.payload_off * 8 + (uint64_t)(v - r.value_start) * t.bw;
  if (t.staged) return (uint32_t)lds_bits64(L.stage, (uint32_t)(bo - t.sbit), t.bw);
  return bits32c(t.s, t.n, bo, t.bw);
}

// A lane's run cursor with the run in registers: the run's first value, payload offset and info,
// and the next run's first value, so the values of one run (most of a lane's values: a bit-packed
// run is up to 504 values long) cost no run-table reads. Values visited must not decrease.
#ifndef PQ_DICT_BYTE
#define PQ_DICT_BYTE 1
#endif
struct DictCursor {
  uint32_t ri, start, off, info, next;
};
DEV void dict_cursor_load(const DictTile &t, DictCursor &c) {
  const HybRun r = t.runs[c.ri];
  c.start = r.value_start;
  c.off = r.payload_off;
  c.info = r.info;
  c.next = c.ri + 1 < t.nr ? t.runs[c.ri + 1].value_start : 0xffffffffu;
}
DEV DictCursor dict_cursor(const DictTile &t, uint32_t v) {  // the run of value v
  DictCursor c{0, 0, 0, 0, 0xffffffffu};
  if (t.bw == 0) return c;
  c.ri = dict_tile_seek(t, v);
  dict_cursor_load(t, c);
  return c;
}
template <class L_>
DEV uint32_t dict_cursor_value(const DictTile &t, const L_ &L, DictCursor &c, uint32_t v) {
  if (t.bw == 0) return 0;
  if (v >= c.next) {
    do c.ri++; while (c.ri + 1 < t.nr && t.runs[c.ri + 1].value_start <= v);
    dict_cursor_load(t, c);
  }
  if (!(c.info & 0x80000000u)) return c.info;
  if (PQ_DICT_BYTE && t.bw == 8 && t.staged)  // (uniform) byte-wide indices: one LDS byte read
    return ((const uint8_t *)L.stage)[c.off + (v - c.start) - (uint32_t)(t.sbit >> 3)];
  const uint64_t bo = (uint64_t)c.off * 8 + (uint64_t)(v - c.start) * t.bw;
  if (t.staged) return (uint32_t)lds_bits64(L.stage, (uint32_t)(bo - t.sbit), t.bw);
  return bits32c(t.s, t.n, bo, t.bw);
}

}  // namespace pq
