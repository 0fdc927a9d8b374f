// kernels.h — launch interface of the gfx950 decode kernels (kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pq_device.h"

namespace pq {

// Device view of one batch; passed by value to every kernel.
struct BatchDev {
  const PageDesc *pages;
  const ChunkDesc *chunks;
  unsigned long long *chunk_err;  // [nchunks] first-error key (atomicMin), init ~0
  unsigned long long *err_next;   // DELTA-major decodes: the key buffer of the next decode, which
                                  // k_values_delta's first workgroup resets (else null)
  uint32_t *page_nn;              // [npages] decoded non-null count (written by k_levels)
  uint32_t *page_nn_v;            // [npages] non-null count the values kernels use: a copy of
                                  // page_nn (serial mode, k_bases) or the page header's count
                                  // (speculative mode, uploaded; k_bases verifies it)
  uint32_t *spec_mismatch;        // speculative mode: set when a header count differs from page_nn
  uint32_t *page_rec;             // [npages] records (rep == 0) per page
  uint64_t *page_vbase;           // [npages] value base within chunk
  uint64_t *page_rbase;           // [npages] record base within chunk
  uint32_t *nest_cnt;             // [nested tiles][2][kNestCnt] lists starting per level, then elements, per half tile
  uint64_t *nest_base;            // [nested tiles][2][kNestCnt] their exclusive prefix within the chunk
  uint64_t *nest_tot;             // [nchunks][kNestCnt] chunk totals
  uint32_t *nest_done;            // [nchunks] k_nest_count tiles finished (zeroed per decode)
  uint64_t *nest_state;           // [nested tiles][16] k_nest_tile look-back words, one 128-B line per
                                  // tile (zeroed per decode)
  HybRun *runs;                   // run tables of hybrid value streams
  const uint64_t *run_base;       // [npages] first entry of each page's run table
  uint32_t *run_count;            // [npages]
  uint32_t *tile_first;           // dict tiles: first run index per tile
  uint4 *tile_desc;               // dict tiles: 2 x uint4 per tile written by k_scan_runs ({r0, r1, lo, hi},
                                  // {values covered, valid}): dict_tile.h reads one descriptor instead of
                                  // the run count, two tile_first entries and two runs one after another
  const uint64_t *tile_base;      // [npages] first tile-table entry per page
  uint64_t *ba_tile_sum;          // byte-array tiles: payload bytes per tile, then (k_ba_scan) its
                                  // exclusive base within the chunk
  const uint32_t *ba_tile_page;   // byte-array tile -> global page index
  const uint32_t *ba_tile_order;  // k_ba_emit block -> byte-array tile, per class (~0u: padding)
  uint32_t ba_class_off[4];       // class k's blocks: ba_tile_order[ba_class_off[k] ..]
  uint64_t *ba_state;             // [tiles] look-back state of each tile (zeroed per decode)
  uint64_t *ba_totals;            // [nchunks] payload bytes of each byte-array chunk (k_ba_scan)
  DeltaBlk *dblk;                 // DELTA block tables of all tiled DELTA pages
  const uint64_t *dblk_base;      // [npages] first DeltaBlk of the page
  uint32_t *dblk_n;               // [npages] blocks the header walk produced
  unsigned long long *dblk_sum;   // [total blocks] sum of each block's deltas (wrapping)
  const BaDelta *ba_delta;         // DELTA_LENGTH / DELTA_BYTE_ARRAY pages
  // generic level streams (k_levels walk -> k_level_fill)
  uint2 *lv_runs;                 // run tables: (first value index, bit-packed flag | payload position or RLE value)
  const uint64_t *lv_run_base;    // [npages][2] first entry of the repetition / definition stream's table
  uint32_t *lv_meta;              // [npages][4] repetition entries, values covered, definition entries, values covered
  uint32_t *lv_tile_run;          // [fill tiles][2] run of the tile's first value (repetition, definition)
  const uint32_t *lv_tile0;       // [npages] the page's first fill tile
  unsigned long long *dbg;        // diagnostic counters (PQ_DEBUG_STAMPS=1), else null
  uint32_t npages, nchunks;
  uint32_t spec;                  // 1: value bases came from the page headers (see k_bases)
  uint32_t ablate;                // diagnostic build only (PQ_ABLATE): skip phases to time them
};

constexpr uint32_t kDictTile = 4096;   // values per dictionary tile (tile table granularity)
constexpr uint32_t kNestCnt = 9;       // nested counters per page: lists of levels 1..8, then elements
constexpr uint32_t kPlainTile = 16384; // values per BOOLEAN PLAIN tile
// bytes per fixed-width PLAIN tile (a workgroup's copy): the copies come out of one round or two
// of 16-B pieces per lane instead of a loop, and more of them fill the CUs beside the DELTA pages
// (cfg2 k_values_delta alone 0.306 -> 0.287 ms against 128 KiB tiles; tools/ubench/copy_shapes:
// 16 KiB items 6.3 TB/s, 128 KiB items 5.0 TB/s)
constexpr uint32_t kPlainTileBytes = 32768;
constexpr uint32_t kDictEarlyHost = 4096;  // kernels.hip kDictEarly: dictionaries staged with their tile
constexpr uint32_t kDictGroupHost = 2;     // kernels.hip kDictGroup: tiles per WI_DICT2 item (at most)
// The pages whose dictionary tiles may be grouped into WI_DICT2 items: host.cpp groups only these and
// kernels.hip do_dict2 decodes only these (a grouped item outside it is reported, never dropped).
__host__ __device__ constexpr inline bool dict2_eligible(uint32_t vkind, uint32_t value_width, uint64_t dict_count) {
  return vkind == VK_DICT && value_width == 4 && dict_count * 4 <= kDictEarlyHost;
}
// Values per byte-array tile (page-aligned, inside one dictionary tile): kBaTile for emission classes
// 0-2 (4-wave workgroups), kBaTileLds for class 3 (the LDS slot table; 8-wave workgroups, chunks
// flagged CF_BA_TILE4K); bytearray.hip kEmitWaves
constexpr uint32_t kBaTile = 2048;
constexpr uint32_t kBaTileLds = 4096;
static_assert(kDictTile % kBaTile == 0 && kDictTile % kBaTileLds == 0, "a byte-array tile lies inside one dictionary tile");

struct LaunchLists {
  const uint32_t *level_pages; uint32_t n_level_pages;   // generic level streams: page << 1 | (0 rep, 1 def)
  const uint32_t *lv_tiles; uint32_t n_lv_tiles;         // page of every fill tile
  const uint32_t *lf_list; uint32_t n_lf_list;           // fill tiles of the non-nested chunks (k_level_fill)
  const uint32_t *level_pages_bw1; uint32_t n_level_pages_bw1;  // flat OPTIONAL pages (max_def 1, no rep)
  uint32_t n_level_pages_seg;  // the first n of them go to k_levels_seg (def stream fits its LDS stage)
  uint32_t seg_grid;           // k_levels_seg's wavefronts (0: one per page)
  uint32_t n_level_units_seg;  // the first n level_pages units go to k_levels_segw (stream fits its stage)
  uint32_t n_level_units_hyb;  // the next n (repetition streams) to k_levels_hyb, the rest to k_levels
  uint32_t n_ba_delta;                                   // BaDelta entries (one workgroup each)
  const uint32_t *scan_pages; uint32_t n_scan_pages;     // pages with hybrid value streams (dict / rle bool)
  const uint32_t *base_chunks; uint32_t n_base_chunks;   // chunks needing value/record bases
  const WorkItem *items; uint32_t n_items;               // values work items (LDS kinds: DELTA, dictionary)
  const WorkItem *copy_items; uint32_t n_copy_items;     // PLAIN / BOOLEAN copies (k_values_copy, no LDS)
  const uint32_t *ba_chunks; uint32_t n_ba_chunks;       // chunks with byte-array output
  uint32_t n_ba_tiles;
  uint32_t n_ba_class[4];  // k_ba_emit tiles per class (bytearray.hip ba_emit)                                   // byte-array tiles (BatchDev::ba_tile_page)
  const uint32_t *slot_chunks; uint32_t n_slot_chunks;   // chunks whose dictionary gets a slot table
  uint32_t slot_grid_x;
  const uint32_t *rec_pages; uint32_t n_rec_pages;       // pages of chunks with max_rep > 0
  const uint32_t *pc_pages; uint32_t n_pc_pages;         // pages of the nested chunks (k_nest_pcount)
  const uint4 *nest_desc; uint32_t n_nest_tiles;         // fill tiles of the nested chunks (k_nest_count / k_nest_emit):
                                                         // {global fill tile, page, tile of the page, chunk}
  uint32_t nest_first[10];        // tiles of chunks with R list levels: [nest_first[R], nest_first[R + 1])
  const uint32_t *nest_order;     // k_nest_tile: block nest_first[R] + i of group R takes tile position
                                  // nest_order[nest_first[R] + i] (the group's chunks interleaved)
  const uint32_t *nest_chunks; uint32_t n_nest_chunks, n_nest_empty;  // nested chunks, those without tiles first
  const uint32_t *grp_tiles; uint32_t n_grp_tiles;       // chunk of every k_group_flat tile
  const uint32_t *delta_pages; uint32_t n_delta_pages;   // tiled DELTA pages (header walk, block scan)
  uint32_t n_delta_tiles;                                // the first n_delta_tiles items are WI_DELTA_TILE
};

// s2 (when given): the generic streams past k_levels_segw's (k_levels_hyb, k_levels) go there
hipError_t launch_levels(const BatchDev &b, const LaunchLists &l, hipStream_t s, hipStream_t s2 = nullptr);
hipError_t launch_level_fill(const BatchDev &b, const LaunchLists &l, hipStream_t s);  // generic level run tables
constexpr uint32_t kLfTileHost = 8192;  // k_level_fill tile (kernels.hip kLfTile)
constexpr uint32_t kSgStageHost = 10240;  // k_levels_seg's LDS stage (kernels.hip kSgStage)
constexpr uint32_t kSgImageSlotsHost = 65536;  // slots of a 32-aligned page k_levels_seg's bitmap image holds whole
constexpr uint32_t kSgwStageHost = 57344; // k_levels_segw's LDS stage (kernels.hip kSgwStage)
hipError_t launch_bases(const BatchDev &b, const LaunchLists &l, hipStream_t s);
hipError_t launch_scan_runs(const BatchDev &b, const LaunchLists &l, hipStream_t s);
hipError_t launch_scan_slots(const BatchDev &b, const LaunchLists &l, hipStream_t s);  // k_scan_runs + k_dict_slots
hipError_t launch_values(const BatchDev &b, const LaunchLists &l, hipStream_t s);
hipError_t launch_values_copy(const BatchDev &b, const LaunchLists &l, hipStream_t s);
hipError_t launch_values_delta(const BatchDev &b, const WorkItem *items, uint32_t n, hipStream_t s);  // DELTA items only
// WI_DICT2 (grouped) items [0, n_pair), then WI_DICT items [n_pair, n)
hipError_t launch_values_dict(const BatchDev &b, const WorkItem *items, uint32_t n_pair, uint32_t n, hipStream_t s);
// byte-array outputs (bytearray.hip): per-tile payload sums, per-chunk scan of the tile sums,
// offsets + payload of every tile
hipError_t launch_dict_slots(const BatchDev &b, const LaunchLists &l, hipStream_t s);
hipError_t launch_ba_sums(const BatchDev &b, const LaunchLists &l, hipStream_t s);
hipError_t launch_ba_scan(const BatchDev &b, const LaunchLists &l, hipStream_t s);
hipError_t launch_ba_emit(const BatchDev &b, const LaunchLists &l, hipStream_t s);
hipError_t launch_records(const BatchDev &b, const LaunchLists &l, hipStream_t s);
hipError_t launch_nest_count(const BatchDev &b, const LaunchLists &l, hipStream_t s);
hipError_t launch_nest_scan(const BatchDev &b, const LaunchLists &l, hipStream_t s);
hipError_t launch_nest_emit(const BatchDev &b, const LaunchLists &l, hipStream_t s);
// the two passes in one (count, look-back over the chunk's earlier tiles, emit): k_nest_tile
hipError_t launch_nest_tile(const BatchDev &b, const LaunchLists &l, hipStream_t s, bool counted, bool based = false);
// the one-list-level tiles' counts from the run tables and every nested chunk's scan (k_nest_tcount,
// k_nest_scan): k_nest_tile then takes its bases from them instead of looking back
hipError_t launch_nest_tcount(const BatchDev &b, const LaunchLists &l, hipStream_t s);
// the nested pages' record and non-null counts from the level run tables (k_nest_pcount)
hipError_t launch_nest_pcount(const BatchDev &b, const LaunchLists &l, hipStream_t s);
constexpr uint32_t kGrpTileHost = 8192;  // nested.hip kGrpTile: slots per k_group_flat workgroup
hipError_t launch_group_flat(const BatchDev &b, const LaunchLists &l, hipStream_t s);
// *flag |= 1 when the n words at a and b differ (pqgpu_batch_share_ancestors)
hipError_t launch_words_differ(const uint32_t *a, const uint32_t *b, uint64_t n, uint32_t *flag, hipStream_t s);
// the per-decode resets: zn bytes at z to 0, fn bytes at f to 0xff (16-B aligned, multiples of 16)
hipError_t launch_reset(void *z, uint64_t zn, void *f, uint64_t fn, hipStream_t s);
hipError_t launch_ba_delta(const BatchDev &b, const LaunchLists &l, hipStream_t s);      // DLBA / DBA values
hipError_t launch_dba_gather(const BatchDev &b, const LaunchLists &l, hipStream_t s);    // DBA payloads
hipError_t launch_snappy(const BatchDev &b, const SnappyJob *jobs, uint32_t njobs, hipStream_t s);  // SNAPPY pages
hipError_t launch_delta_prep(const BatchDev &b, const LaunchLists &l, hipStream_t s);  // walk + sums + prefix
// PLAIN BYTE_ARRAY pages (plainba.hip): speculative segment walks, verified per page
struct PbaLists {
  const uint32_t *pages; uint32_t n_pages;  // PLAIN BYTE_ARRAY pages with values
  const uint32_t *seg0;                     // [n_pages + 1] first segment of each page
  const uint32_t *seg_page;                 // [n_segs] the page-list index of each segment
  uint4 *segs;                              // [n_segs] entry, exit, values, error -> first value
  uint32_t *limit;                          // [n_pages] values written per page
  uint32_t n_segs;
};
constexpr uint32_t kPbaSegHost = 256;  // plainba.hip kPbaSeg
hipError_t launch_plain_ba(const BatchDev &b, const PbaLists &l, hipStream_t s);
// on-device page index (pagewalk.hip): header walk of every chunk (+ CRC32 of every checksummed
// block), and the upload-time gather of resident UNCOMPRESSED page bodies
// The chunk table is host memory: it reaches the walk in the kernel arguments, kIxArgChunks chunks
// per launch (never through a DMA copy the walk would read); res[c] = (status, npages, fail_page, 0).
constexpr uint32_t kIxArgChunks = 64;
// res[c].w = `gen` once chunk c's walk has reported: a per-build generation (never 0, the value
// k_page_walk_init writes), so a marker left in reused scratch by an earlier build never passes.
hipError_t launch_page_walk(const uint8_t *buf, int64_t len, int64_t file_off, const PageIxChunk *chunks,
                            uint32_t nchunks, uint4 *res, PageIxEntry *table, uint32_t *table_n, uint32_t table_cap,
                            int validate_crc, uint32_t gen, hipStream_t s);
hipError_t launch_page_gather(const GatherJob *jobs, uint32_t njobs, hipStream_t s);

// Names of the kernels, for the timing hook.
extern const char *kValuesKernelName;

}  // namespace pq
