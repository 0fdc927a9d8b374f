// pq_device.h — descriptor tables shared by the host planner and the gfx950
// kernels. Plain structs (no pointers to host memory); device pointers are
// stored as uint64_t so the layout is identical on both sides.
//
// HBM layout of one batch (see DESIGN.md "Data layout in HBM"):
//   stage    : every page's (decompressed) payload, each page 16-B aligned,
//              followed by 64 B of zero padding so unaligned dword reads at a
//              section end stay in bounds;
//   pages[]  : PageDesc, one per data page, grouped by chunk;
//   chunks[] : ChunkDesc, one per column chunk;
//   outputs  : per chunk values / levels / validity / offsets / payload.
#pragma once
#include <stdint.h>

namespace pq {

// parquet.Encoding
enum : uint8_t {
  ENC_PLAIN = 0, ENC_PLAIN_DICTIONARY = 2, ENC_RLE = 3, ENC_BIT_PACKED = 4, ENC_DELTA_BINARY_PACKED = 5,
  ENC_DELTA_LENGTH_BYTE_ARRAY = 6, ENC_DELTA_BYTE_ARRAY = 7, ENC_RLE_DICTIONARY = 8,
};
// parquet.Type
enum : int32_t { T_BOOLEAN = 0, T_INT32 = 1, T_INT64 = 2, T_INT96 = 3, T_FLOAT = 4, T_DOUBLE = 5,
                 T_BYTE_ARRAY = 6, T_FLBA = 7 };

// Value-decoder kind chosen by getValuesDecoder (chunk_reader.go:106-159).
enum : uint8_t {
  VK_PLAIN_FIXED = 0,  // INT32/INT64/FLOAT/DOUBLE/FLBA PLAIN: byte copy
  VK_PLAIN_INT96 = 1,  // INT96 PLAIN (12-B copy)
  VK_PLAIN_BOOL = 2,   // BOOLEAN PLAIN: LSB-first bits -> 1 B per value
  VK_RLE_BOOL = 3,     // BOOLEAN RLE: hybrid bw=1
  VK_DICT = 4,         // RLE_DICTIONARY / PLAIN_DICTIONARY: hybrid indices -> gather
  VK_DELTA32 = 5,      // DELTA_BINARY_PACKED INT32
  VK_DELTA64 = 6,      // DELTA_BINARY_PACKED INT64
  VK_PLAIN_BA = 7,     // BYTE_ARRAY PLAIN (length-prefixed)
  VK_DLBA = 8,         // BYTE_ARRAY DELTA_LENGTH_BYTE_ARRAY: DELTA lengths + concatenated payload
  VK_DBA = 9,          // BYTE_ARRAY DELTA_BYTE_ARRAY: DELTA prefix lengths + DLBA suffixes
};

// Page flags
enum : uint16_t {
  PF_REP = 1,        // rep stream present (V1 with maxR>0, or V2 rep length > 0)
  PF_DEF = 2,        // def stream present
  PF_V2 = 4,
  PF_BASE_KNOWN = 8, // value_base computed on host (required column or V2 num_nulls)
  PF_DELTA_SLOW = 16,// DELTA page outside the tiled pipeline's shapes (miniblock not a multiple of 8
                     // values, block size not dividing kDeltaTileVals, > 8 miniblocks): exact scalar path
  PF_DEV_SNAPPY = 32,// host only: `data` is an offset into the device decompression region (k_snappy)
  PF_DEV_GATHER = 64,// host only: `data` is a gather-job index (page body copied from resident file bytes)
};

// Error staging key (64 bit, smaller = reported first):
//   [63:62] phase   0 = readPages (chunk-level, e.g. dictionary decode), 1 = readValues
//   [61:40] page    data-page index within chunk (0 for phase 0)
//   [39:36] stage   0 = dictionary, 1 = rep levels, 2 = def levels, 3 = values
//   [35:4]  pos     value / slot position within the stage
//   [3:0]   code    pqgpu_status error class
__host__ __device__ inline uint64_t err_key(uint32_t phase, uint32_t page, uint32_t stage, uint32_t pos,
                                            uint32_t code) {
  return ((uint64_t)(phase & 3) << 62) | ((uint64_t)(page & 0x3fffff) << 40) | ((uint64_t)(stage & 15) << 36) |
         ((uint64_t)pos << 4) | (uint64_t)(code & 15);
}
enum : uint32_t { ST_DICT = 0, ST_REP = 1, ST_DEF = 2, ST_VALUES = 3 };  // ST_DECOMP = 4 below

struct PageDesc {        // 104 B
  uint64_t data;         // device address of the page payload (decompressed)
  uint32_t rep_off, rep_len;  // hybrid streams, relative to data (no length prefix)
  uint32_t def_off, def_len;
  uint32_t val_off, val_len;  // values section (dict: after the bit-width byte)
  uint32_t num_slots;    // DataPageHeader(V2).num_values
  uint32_t chunk;        // owning chunk index
  uint32_t page_in_chunk;
  uint16_t flags;
  uint8_t vkind;         // VK_*
  uint8_t dict_bw;       // VK_DICT: index bit width (0..32); VK_RLE_BOOL: 1
  uint64_t slot_base;    // first level slot of this page within its chunk
  uint64_t value_base;   // first non-null value index within its chunk
  uint32_t expect_nn;    // non-null count the host expects (PF_BASE_KNOWN), else 0
  uint32_t delta_first_mb; // DELTA: offset (rel. to data) of the first miniblock header
  int64_t delta_first;   // DELTA: first value from the block header
  int32_t delta_count;   // DELTA: valuesCount from the block header
  uint16_t delta_mbc;    // DELTA: miniblocks per block
  uint16_t pad0;
  uint32_t delta_mbvc;   // DELTA: values per miniblock
  uint32_t ba_delta;     // VK_DLBA / VK_DBA: index of the page's BaDelta entry
  uint32_t ba_tile;      // byte-array chunks: global index of the page's first BA tile (ba_tile_vals values)
  uint32_t dict_tile0;   // VK_DICT / VK_RLE_BOOL with a run scan: the page's first entry of the tile tables
};

struct ChunkDesc {       // 480 B (static_assert below; copied to the device as is)
  int32_t type, type_length, max_def, max_rep;
  int32_t def_bw, rep_bw, value_width, flags;
  uint32_t first_page, num_pages;
  uint64_t num_slots;
  uint64_t nn_capacity;  // values buffer capacity (values)
  // dictionary (decoded on device into an aligned buffer)
  uint64_t dict_raw;     // device address of the dictionary page payload
  uint32_t dict_raw_len, dict_count;
  uint64_t dict_values;  // fixed-width values (== dict_raw)
  uint64_t dict_offsets; // byte-array layout: uint2[dict_count] (position of the entry's bytes in
                         // dict_raw, length), built by the host's dictionary-page walk
  // outputs
  uint64_t values;       // fixed width
  uint64_t def_levels;   // uint8 or 0
  uint64_t rep_levels;   // uint8 or 0
  uint64_t validity;     // uint32 words or 0
  uint64_t offsets;      // BYTE_ARRAY int32[nn+1]
  uint64_t payload;      // BYTE_ARRAY bytes
  uint64_t list_offsets; // int32[records+1]
  uint64_t ba_index;     // scratch: int32 dictionary index per value (BYTE_ARRAY dict)
  uint64_t payload_capacity;  // BYTE_ARRAY payload bytes allocated (k_ba_emit writes no more)
  uint64_t page_nn;      // device uint32[num_pages]: decoded non-null counts
  uint64_t page_rec;     // device uint32[num_pages]: records (rep==0) per page
  uint64_t page_vbase;   // device uint64[num_pages]: value bases (copied from / checked against PageDesc)
  uint64_t page_rbase;   // device uint64[num_pages]: record bases
  uint32_t ba_tile0, ba_ntiles;  // byte-array chunks: the chunk's BA tiles [ba_tile0, +ba_ntiles)
  uint32_t dict_max_len;         // longest dictionary entry (byte-array layout)
  uint32_t slot_shift;           // byte-array dictionary materialised in 2^slot_shift-byte slots
                                 // [u32 length | bytes] (4, 5 or 6; 0: entries over 60 bytes, no table)
  uint64_t dict_slots;           // device address of the slot table (k_dict_slots, every decode)
  // nested (Arrow-style) output, max_rep > 0: nest = number of list levels (0: not produced)
  uint32_t nest, nest_tile0;      // list levels; the chunk's first entry of the nested tile list
  uint32_t nest_ntiles;           // the chunk's fill tiles (nested.hip: two counting units each)
  uint32_t nest_nmask;            // flag masks per slot: 2 (nest + 1) + ngroups (k_nest_count -> k_nest_emit)
  uint8_t list_null_def[8], list_def[8];  // per REPEATED node: non-null from / has an element from
  uint64_t lvl_offsets[8];       // int32[num_lists + 1] per level
  uint64_t lvl_validity[8];      // uint32 bitmap per level
  uint64_t elem_validity;        // uint32 bitmap over the leaf's element slots
  // struct (OPTIONAL group) validity, per group on the path: entries of list depth group_depth
  // (records / a max_rep == 0 leaf's slots at 0), bit = def >= group_def; 0 = shares a bitmap above
  uint32_t ngroups, grp_tile0;    // k_group_flat: the chunk's first tile
  uint8_t group_def[8], group_depth[8];
  uint64_t group_validity[8];
  uint64_t nest_masks;            // device u32 [nest_ntiles][nest_nmask][256]: a thread's 32 slots per mask
                                  // (two-pass nested mode only; 0 with k_nest_tile)
};
static_assert(sizeof(ChunkDesc) == 480, "ChunkDesc layout: host and device share it byte for byte");

// Chunk flags
enum : int32_t { CF_DICT = 1, CF_BASE_ON_DEVICE = 2, CF_BA_DICT = 4, CF_FAILED = 8,
                 CF_BA_SYNC = 16,    // byte-array payload without an upload-time bound: sized after the scan
                 CF_BA_PRESUM = 32,  // byte-array tile bases from k_ba_sums + k_ba_scan (no look-back)
                 CF_NN_SPEC = 64,    // serial batch: non-null counts speculated from PLAIN value bytes (k_bases checks)
                 CF_BA_TILE4K = 128 };  // byte-array chunk of emission class 3: kBaTileLds-value tiles

// Work items of the values kernel.
enum : uint8_t { WI_PLAIN = 0, WI_BOOL = 1, WI_DICT = 2, WI_DELTA = 3, WI_PLAIN_BA = 4, WI_DICT_BA_LEN = 5,
                 WI_DELTA_TILE = 6, WI_DELTA_PAGE = 7, WI_DLENS = 8,
                 WI_DICT2 = 9 };  // 2-3 consecutive dictionary tiles of one page (k_values_dict2)

// DELTA_BINARY_PACKED block table entry (one per block of a page), written by the header
// walk (k_delta_walk), completed by the per-page scan of block sums (k_delta_prefix).
constexpr uint32_t kDeltaTileVals = 2048;  // values per DELTA tile (256 groups of 8)
struct DeltaBlk {        // 32 B
  int64_t min_delta;     // the block's minDelta (zigzag varint, deltabp_decoder.go:125-128)
  uint64_t widths;       // miniblock bit widths, 8 bits each (<= 8 miniblocks)
  int64_t base;          // value before the block's first delta (first + all earlier deltas)
  uint32_t pos;          // stream offset of the block's first miniblock payload byte
  uint32_t sum_lo;       // scratch: low half of the block's delta sum (k_delta_sums); unused
};
// DELTA_BINARY_PACKED page decoder (WI_DELTA_PAGE): the stream is staged through an LDS
// window of kDeltaWinLoad bytes; a block (header + payload) must fit in it with 48 bytes of
// slack (host check, else PF_DELTA_SLOW). At most kDeltaMaxBlk blocks are walked per window.
#ifndef PQ_DELTA_WIN
#define PQ_DELTA_WIN 8000  // kDeltaWinLoad + 32 <= 8 KiB: two 16-B loads per thread
#endif
constexpr uint32_t kDeltaWin = PQ_DELTA_WIN;
constexpr uint32_t kDeltaWinLoad = kDeltaWin + 128;
constexpr uint32_t kDeltaMaxBlk = kDeltaWin > 8192 ? 256 : 128;
// DELTA_LENGTH_BYTE_ARRAY / DELTA_BYTE_ARRAY page (type_bytearray.go:98-240). The host walks
// the DELTA lengths streams' headers at init (the reference decodes every length in init():
// its errors and where the payload starts follow from the stream layout alone, SURVEY.md
// App. A Q1/Q2); the GPU decodes the lengths (WI_DLENS) into scratch, then k_ba_delta turns
// them into value lengths, sources and the reference's value errors.
struct BaDeltaStream {   // a DELTA INT32 lengths stream
  uint32_t off;          // stream start, relative to the page data
  uint32_t len;          // bytes up to the end of the page data
  uint32_t hdr;          // first miniblock header, relative to the stream start
  int32_t first, count;  // first value, valuesCount
  uint16_t mbc, slow;    // miniblocks per block; 1: exact scalar decode (shape outside the page kernel's)
  uint32_t mbvc;
};
struct BaDelta {
  BaDeltaStream st[2];   // [0] lengths (DLBA) / suffix lengths (DBA); [1] prefix lengths (DBA)
  uint64_t scratch;      // device int32[3 * cap]: suffix lengths, prefix lengths, DBA ancestor links
  uint32_t cap;          // lengths decoded per stream: min(count, num_values)
  uint32_t pay_off, pay_len;  // payload (suffix bytes), relative to the page data
  uint32_t page;         // global page index
};
// SNAPPY data page decompressed on the device (compress.go:42-48,
// :102-123, golang/snappy decode.go). The stage holds the raw block after its length preamble
// (followed by >= 128 zero bytes); k_snappy writes the page — `raw` bytes (V2 level sections,
// which are not compressed, page_v2.go:112-127), then the decompressed bytes, then 64 zero
// bytes — at `dst`, the page data address every later kernel reads.
struct SnappyJob {       // 48 B
  uint64_t src;          // device address of the first element tag
  uint64_t raw;          // device address of the raw prefix (16-B aligned)
  uint64_t dst;          // device address of the page data (16-B aligned)
  uint32_t src_len;      // element bytes
  uint32_t raw_len;
  uint32_t dlen;         // decoded length from the preamble (== the page's decompressed size)
  uint32_t chunk;
  uint32_t page_in_chunk;
  uint32_t lead;         // 0, or direct output: 1 + (dst & 15). A REQUIRED PLAIN fixed-width page whose
                         // decoded bytes are exactly its values (no level sections, num_values x width
                         // == dlen) is written straight into the chunk's values array at its value base,
                         // without the 64-B pad; no k_values item copies it again (the
                         // decompressed body IS the output, page_v1.go:87-122, type_*.go PLAIN)
};
#ifndef PQ_SNAPPY_RING
#define PQ_SNAPPY_RING 16384
#endif
constexpr uint32_t kSnappyRing = PQ_SNAPPY_RING;  // LDS window of the most recent output bytes per page
enum : uint32_t { ST_DECOMP = 4 };       // err_key stage of a device decompression error

// On-device page index (pagewalk.hip): readPages' header loop
// (chunk_reader.go:182-263) over column-chunk bytes resident in HBM, the Thrift compact decode of
// every PageHeader (readThrift helpers.go:103-109) and the CRC32 check of readPageBlock
// (chunk_reader.go:173-177). The walk covers the valid case only: anything the walk cannot take
// (a Thrift error, a negative size, a page reaching past the buffer, a full table) marks the chunk
// IX_FALLBACK and the host planner walks that chunk itself, so every error keeps the host's
// (i.e. the reference's) class, message and position.
enum : uint32_t { IX_OK = 0, IX_FALLBACK = 1 };
struct PageIxChunk {     // 48 B: walk input (start .. total) and result (status, npages)
  int64_t start;         // file offset of the first header (dictionary page offset, else data page offset)
  int64_t data_off;      // DataPageOffset: the seek target after a dictionary page (chunk_reader.go:220-226)
  int64_t dict_off;      // DictionaryPageOffset, -1 when unset
  int64_t total;         // TotalCompressedSize: the loop bound (chunk_reader.go:190)
  uint32_t status;       // IX_OK / IX_FALLBACK
  uint32_t npages;       // entries the walk wrote for this chunk
  uint32_t fail_page;    // IX_FALLBACK: the page the walk stopped at
  uint32_t pad;
};
// Entry flags
enum : uint32_t { IXF_CRC = 1, IXF_DPH = 2, IXF_DICT = 4, IXF_DPH2 = 8, IXF_COMPRESSED = 16,
                  IXF_CRC_CHECKED = 32, IXF_CRC_OK = 64 };
struct PageIxEntry {     // 96 B: one PageHeader (format.h) and where it lies
  int64_t hdr_off;       // file offset of the header
  int32_t hdr_len;       // Thrift bytes consumed
  int32_t type, usize, csize, crc;
  uint32_t flags;        // IXF_*
  int32_t dph[4];        // DataPageHeader: num_values, encoding, def_enc, rep_enc
  int32_t dict[2];       // DictionaryPageHeader: num_values, encoding
  int32_t dph2[6];       // DataPageHeaderV2: num_values, num_nulls, num_rows, encoding, def_len, rep_len
  uint32_t chunk, seq;   // walk input chunk, page position in its chunk (dictionary page included)
  uint32_t gen;          // the build's generation (ctx next_ix_gen): an entry left in reused scratch by
                         // an earlier build carries another and is dropped by the host
  uint32_t pad;
};
// Device-to-device copy of an UNCOMPRESSED page body from the resident file bytes into the
// batch's page region (16-B aligned, 64 zero bytes after it), done once at upload.
struct GatherJob { uint64_t src, dst, len; };

struct WorkItem {        // 16 B
  uint32_t page;         // global page index
  uint32_t v0;           // first value (within page) of this tile
  uint32_t v1;           // end value bound (clamped to the decoded NN in kernel)
  uint8_t kind;
  uint8_t pad[3];
};

// Hybrid run table entry written by the scan kernel for dictionary-index streams.
struct HybRun {          // 12 B
  uint32_t value_start;  // index of the run's first value within the stream
  uint32_t payload_off;  // byte offset of the run payload (after the header) within the stream
  uint32_t info;         // bit 31: bit-packed; bits 0..30: RLE value (bit-packed: 0)
};

}  // namespace pq
