// host.cpp — C ABI of the MI355X Parquet column-chunk decoder (include/pqgpu.h).
//
// Host side of the boundary: walks Thrift page headers and validates them
// exactly as the reference's readChunk/readPages/page read() do
// (chunk_reader.go:182-362, page_v1.go:87-122, page_v2.go:79-131), stages the
// page sections (decompressing SNAPPY/GZIP pages on host threads), builds the
// flat page/work descriptor tables and drives the gfx950 kernels
// (kernels.hip). There is no CPU decode path: every value, level, offset and
// payload byte is produced on the GPU; if the HIP runtime or device is
// missing, pqgpu_ctx_create fails with PQ_ERR_HIP.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>

#include <algorithm>
#include <cassert>
#include <chrono>
#include <functional>
#include <memory>
#include <numeric>
#include <string>
#include <tuple>
#include <string>
#include <thread>
#include <vector>

#include "../../include/pqgpu.h"
#include "ctx.h"
#include "format.h"
#include "kernels.h"
#include "pq_device.h"

using namespace pq;

static void set_err(pqgpu_error *e, int code, int chunk, int page, const std::string &msg) {
  if (!e) return;
  e->code = code;
  e->chunk = chunk;
  e->page = page;
  snprintf(e->msg, sizeof(e->msg), "%s", msg.c_str());
}
static void clear_err(pqgpu_error *e) {
  if (e) set_err(e, PQ_OK, -1, -1, "");
}

#define HIPCHECK(expr, errp)                                                                           \
  do {                                                                                                 \
    hipError_t _e = (expr);                                                                            \
    if (_e != hipSuccess) {                                                                            \
      set_err(errp, PQ_ERR_HIP, -1, -1, std::string(#expr) + ": " + hipGetErrorString(_e));           \
      return PQ_ERR_HIP;                                                                               \
    }                                                                                                  \
  } while (0)


struct pqgpu_file {
  FileMeta meta;
  const uint8_t *buf = nullptr;
  int64_t len = 0;
};

namespace {

// Go-semantics varint readers over a byte range (helpers.go:151-208, Go 1.17 binary.ReadUvarint).
struct GoReader {
  const uint8_t *p;
  int64_t n, i = 0;
  int uvarint(uint64_t *out) {
    uint64_t x = 0;
    unsigned s = 0;
    for (int k = 0;; k++) {
      if (i >= n) { *out = x; return PQ_ERR_EOF; }
      uint8_t b = p[i++];
      if (b < 0x80) {
        if (k > 9 || (k == 9 && b > 1)) return PQ_ERR_RANGE;
        if (s < 64) x |= (uint64_t)b << s;
        *out = x;
        return PQ_OK;
      }
      if (s < 64) x |= (uint64_t)(b & 0x7f) << s;
      s += 7;
    }
  }
  int uvariant32(int32_t *out) {
    uint64_t v;
    int e = uvarint(&v);
    if (e) return e;
    if (v > 0x7fffffffULL) return PQ_ERR_RANGE;
    *out = (int32_t)v;
    return PQ_OK;
  }
  int varint64(int64_t *out) {
    uint64_t u;
    int e = uvarint(&u);
    int64_t x = (int64_t)(u >> 1);
    if (u & 1) x = ~x;
    *out = x;
    return e;
  }
  int variant32(int32_t *out) {
    int64_t v;
    int e = varint64(&v);
    if (e) return e;
    if (v > 2147483647LL || v < -2147483648LL) return PQ_ERR_RANGE;
    *out = (int32_t)v;
    return PQ_OK;
  }
  int readfull(int64_t k) {  // io.ReadFull semantics, bytes skipped
    if (k <= 0) return PQ_OK;
    if (i >= n) return PQ_ERR_EOF;
    if (n - i < k) { i = n; return PQ_ERR_UNEXPECTED_EOF; }
    i += k;
    return PQ_OK;
  }
};

// deltaBitPackDecoder32.init + decodeInt32 of all valuesCount values, as the DELTA_LENGTH /
// DELTA_BYTE_ARRAY decoders run it at init (type_bytearray.go:104-115, :195-214;
// deltabp_decoder.go:35-174; helpers.go:121-131) — structure only: block and miniblock
// headers, group reads (io.ReadFull: EOF / ErrUnexpectedEOF), the look-ahead (Q1) and the
// padding skip after the last group (Q2, skip errors ignored). The reader ends where the
// next section starts. Groups between miniblock checks are consumed in one step.
struct DeltaWalk { int64_t hdr; int32_t first, count, mbc, mbvc, bs; };
int delta32_walk(GoReader &r, DeltaWalk *w, std::string *msg) {
  int e;
  int32_t bs, mbc, vc, f32;
  if ((e = r.uvariant32(&bs))) { *msg = "failed to read block size"; return e; }
  if ((e = r.uvariant32(&mbc))) { *msg = "failed to read number of mini blocks"; return e; }
  if (mbc <= 0 || bs % mbc != 0) { *msg = "int/delta: invalid number of mini blocks"; return PQ_ERR_INVALID; }
  const int32_t mbvc = bs / mbc;
  if (mbvc == 0) { *msg = "invalid mini block value count, it can't be zero"; return PQ_ERR_INVALID; }
  if ((e = r.uvariant32(&vc))) { *msg = "failed to read total value count"; return e; }
  if ((e = r.variant32(&f32))) { *msg = "failed to read first value"; return e; }
  if (mbc > 65535) { *msg = "more than 65535 miniblocks per block"; return PQ_ERR_UNSUPPORTED; }
  w->hdr = r.i; w->first = f32; w->count = vc; w->mbc = mbc; w->mbvc = mbvc; w->bs = bs;
  const uint8_t *widths = nullptr;  // the current block's width bytes, in place
  auto mb_header = [&]() -> int {
    int32_t m32;
    int er;
    if ((er = r.variant32(&m32))) { *msg = "failed to read min delta"; return er; }
    const int64_t ws = r.i;
    if ((er = r.readfull(mbc))) { *msg = "not enough data to read all miniblock bit widths"; return er; }
    widths = r.p + ws;
    for (int32_t k = 0; k < mbc; k++)
      if (widths[k] > 32) { *msg = "invalid miniblock bit width"; return PQ_ERR_INVALID; }
    return PQ_OK;
  };
  if ((e = mb_header())) return e;
  const int64_t l8 = (int64_t)std::lcm<int64_t>(8, mbvc);  // group starts where next() checks the miniblock
  const int64_t last = vc > 0 ? ((int64_t)(vc - 1) / 8) * 8 : 0;  // start of the group holding value vc-1
  int64_t pos = 0, cur_w = 0, mb_pos = 0;
  int32_t cur_mb = 0;
  while (pos < vc) {
    if (pos % mbvc == 0) {
      if (cur_mb >= mbc) {
        if ((e = mb_header())) return e;
        cur_mb = 0;
      }
      cur_w = widths[cur_mb];
      mb_pos = 0;
      cur_mb++;
    }
    int64_t g = 1;  // groups read before the next rule applies (a miniblock check or the last group)
    if (pos < last) g = std::max<int64_t>(1, std::min((last - pos) / 8, ((pos / l8 + 1) * l8 - pos) / 8));
    if (cur_w > 0) {
      const int64_t avail = r.n - r.i, need = g * cur_w;
      if (avail < need) {
        const int64_t rem = avail - (avail / cur_w) * cur_w;  // bytes of the first group cut short
        *msg = "delta lengths";
        return rem == 0 ? PQ_ERR_EOF : PQ_ERR_UNEXPECTED_EOF;
      }
      r.i += need;
      mb_pos += need;
    }
    if (pos + 8 * (g - 1) == last) {  // the last group: skip the padding (:149-164)
      const int64_t l = (int64_t)(mbvc / 8) * cur_w - mb_pos;
      if (l < 0) { *msg = "invalid stream"; return PQ_ERR_INVALID; }
      r.i += std::min(l, r.n - r.i);
      for (int32_t i = cur_mb; i < mbc; i++) {
        const int64_t w2 = widths[cur_mb];  // sic: the reference indexes currentMiniBlock (Q2)
        if (w2) r.i += std::min((int64_t)(mbvc / 8) * w2, r.n - r.i);
      }
    }
    pos += 8 * g;
  }
  return PQ_OK;
}

// dictPageReader.read (page_dict.go:35-72) -> byteArrayPlainDecoder.decodeValues of `count`
// entries (type_bytearray.go:24-55): a u32 length read with io.ReadFull (EOF when no byte is
// left, else ErrUnexpectedEOF), a negative length is "len is negative", then io.ReadFull of the
// bytes (a zero-length entry reads nothing). Records (position, length) of every entry; the
// whole dictionary is read when the chunk is (readPages), so a failure is the chunk's error.
int walk_ba_dict(const uint8_t *p, int64_t n, uint32_t count, int32_t fixed, std::vector<uint32_t> *ent,
                 uint32_t *max_len, std::string *msg) {
  ent->assign(2 * (size_t)count, 0);
  int64_t i = 0;
  uint32_t mx = 0;
  auto fail = [&](uint32_t v, int code) {
    *msg = "expected " + std::to_string(count) + " values, read " + std::to_string(v) + " values: " +
           (code == PQ_ERR_EOF ? "EOF" : code == PQ_ERR_UNEXPECTED_EOF ? "unexpected EOF" : "bytearray/plain: len is negative");
    return code;
  };
  for (uint32_t v = 0; v < count; v++) {
    int64_t l = fixed;
    if (fixed == 0) {
      if (i >= n) return fail(v, PQ_ERR_EOF);
      if (i + 4 > n) return fail(v, PQ_ERR_UNEXPECTED_EOF);
      int32_t x;
      memcpy(&x, p + i, 4);
      i += 4;
      if (x < 0) return fail(v, PQ_ERR_INVALID);
      l = x;
    }
    if (l > 0 && i >= n) return fail(v, PQ_ERR_EOF);
    if (i + l > n) return fail(v, PQ_ERR_UNEXPECTED_EOF);
    (*ent)[2 * (size_t)v] = (uint32_t)i;
    (*ent)[2 * (size_t)v + 1] = (uint32_t)l;
    mx = std::max<uint32_t>(mx, (uint32_t)l);
    i += l;
  }
  *max_len = mx;
  return PQ_OK;
}

struct HostChunk {
  pqgpu_column_info col{};
  pqgpu_chunk_meta meta{};
  pqgpu_error err{};  // readPages-level (host) error
  uint32_t first_page = 0, num_pages = 0;
  uint64_t num_slots = 0;
  int32_t value_width = 0;
  bool has_dict = false;
  uint64_t dict_off = 0;  // stage offset
  uint32_t dict_len = 0, dict_count = 0;
  // device outputs (offsets into the arena)
  uint64_t o_values = 0, o_def = 0, o_rep = 0, o_valid = 0, o_offsets = 0, o_lists = 0, o_ba_index = 0;
  bool valid_unzeroed = false;  // the validity bitmap is outside the per-decode zeroed region (k_levels_seg stores all of it)
  // nested (Arrow-style) output: list levels (0: none), per level offsets / validity, elements
  uint32_t nest = 0, nest_tile0 = 0, nest_ntiles = 0, nest_nmask = 0;
  uint64_t o_nest_mask = 0;
  uint64_t o_lvl_off[PQGPU_MAX_NEST] = {}, o_lvl_valid[PQGPU_MAX_NEST] = {}, o_elem_valid = 0;
  int64_t num_lists[PQGPU_MAX_NEST] = {}, num_elems = 0;
  // struct validity of the OPTIONAL groups on the path (pqgpu_chunk_result group_*): own bitmap
  // (grp_alias -1) or the same bits as list level k's validity (0..7), the element validity (8)
  // or the chunk validity (9)
  uint32_t ngroups = 0, grp_tile0 = 0;
  int8_t grp_alias[PQGPU_MAX_NEST] = {};
  uint64_t o_grp_valid[PQGPU_MAX_NEST] = {};
  // pqgpu_batch_share_ancestors: list levels [0, share_lists) and groups [0, share_groups) are
  // chunk share_from's (cleared by every decode)
  int32_t share_from = -1;
  int8_t ba_class = -1;  // k_ba_emit class (byte-array chunks)
  uint32_t ba_tile_vals = kBaTile;  // values per byte-array tile (class 3: kBaTileLds)
  bool ba_presum = false;  // tile bases from k_ba_sums + k_ba_scan instead of the look-back
  uint32_t share_lists = 0, share_groups = 0;
  // byte-array dictionaries: (position, length) of every entry, from the host's walk of the
  // dictionary page (page_dict.go:35-72 + byteArrayPlainDecoder type_bytearray.go:24-55)
  std::vector<uint32_t> dict_ent;
  uint64_t dict_ent_off = 0;  // stage offset of dict_ent
  uint32_t dict_max_len = 0;
  bool ba_sync = false;       // no upload-time payload bound: size it after the scan (host sync)
  uint64_t payload_off = 0;   // offset in the batch payload arena (bounded chunks)
  uint64_t payload_bound = 0; // its size (k_ba_emit writes nothing past it)
  // a chunk that failed in page k (readValues): the decoded prefix, pages [0, k)
  bool partial = false;
  int64_t part_slots = 0, part_nn = 0, part_records = 0, part_payload = 0;
  uint64_t payload_cap = 0;
  uint8_t *payload = nullptr;  // the chunk's payload (arena slice, or own allocation when ba_sync)
  bool payload_own = false;
  bool sync_err = false;      // ba_sync chunk whose payload exceeded 2 GiB at the last decode
  uint32_t slot_shift = 0;    // dictionary slot table (k_dict_slots): log2 slot bytes, 0 = none
  uint64_t o_slots = 0;
  // results after sync
  int64_t nn = 0, records = 0, payload_bytes = 0;
  pqgpu_error dev_err{};
};

// Value-decoder choice: getValuesDecoder chunk_reader.go:106-159.
int pick_vkind(int32_t enc, int32_t type, int32_t type_length, uint8_t *vk, std::string *msg) {
  if (enc == ENC_PLAIN_DICTIONARY) enc = ENC_RLE_DICTIONARY;
  auto unsup = [&](const char *what) {
    *msg = std::string("unsupported encoding ") + std::to_string(enc) + " for " + what;
    return PQ_ERR_UNSUPPORTED;
  };
  switch (type) {
    case T_BOOLEAN:
      if (enc == ENC_PLAIN) { *vk = VK_PLAIN_BOOL; return PQ_OK; }
      if (enc == ENC_RLE) { *vk = VK_RLE_BOOL; return PQ_OK; }
      return unsup("boolean");
    case T_BYTE_ARRAY:
      if (enc == ENC_PLAIN) { *vk = VK_PLAIN_BA; return PQ_OK; }
      if (enc == ENC_DELTA_LENGTH_BYTE_ARRAY) { *vk = VK_DLBA; return PQ_OK; }
      if (enc == ENC_DELTA_BYTE_ARRAY) { *vk = VK_DBA; return PQ_OK; }
      if (enc == ENC_RLE_DICTIONARY) { *vk = VK_DICT; return PQ_OK; }
      return unsup("binary");
    case T_FLBA:
      if (enc == ENC_PLAIN) { *vk = type_length == 0 ? VK_PLAIN_BA : VK_PLAIN_FIXED; return PQ_OK; }
      // byteArrayDeltaDecoder (chunk_reader.go:71-72): values of any length, so a chunk with
      // such a page is laid out as byte arrays (add_chunk_impl)
      if (enc == ENC_DELTA_BYTE_ARRAY) { *vk = VK_DBA; return PQ_OK; }
      if (enc == ENC_RLE_DICTIONARY) { *vk = VK_DICT; return PQ_OK; }
      return unsup("fixed_len_byte_array");
    case T_FLOAT: case T_DOUBLE:
      if (enc == ENC_PLAIN) { *vk = VK_PLAIN_FIXED; return PQ_OK; }
      if (enc == ENC_RLE_DICTIONARY) { *vk = VK_DICT; return PQ_OK; }
      return unsup("float/double");
    case T_INT96:
      if (enc == ENC_PLAIN) { *vk = VK_PLAIN_INT96; return PQ_OK; }
      if (enc == ENC_RLE_DICTIONARY) { *vk = VK_DICT; return PQ_OK; }
      return unsup("int96");
    case T_INT32: case T_INT64:
      if (enc == ENC_PLAIN) { *vk = VK_PLAIN_FIXED; return PQ_OK; }
      if (enc == ENC_DELTA_BINARY_PACKED) { *vk = type == T_INT32 ? VK_DELTA32 : VK_DELTA64; return PQ_OK; }
      if (enc == ENC_RLE_DICTIONARY) { *vk = VK_DICT; return PQ_OK; }
      return unsup("int32/int64");
  }
  *msg = "unsupported type";
  return PQ_ERR_UNSUPPORTED;
}

int value_width_of(int32_t type, int32_t type_length) {
  switch (type) {
    case T_BOOLEAN: return 1;
    case T_INT32: case T_FLOAT: return 4;
    case T_INT64: case T_DOUBLE: return 8;
    case T_INT96: return 12;
    case T_FLBA: return type_length;  // 0 -> length-prefixed (byte array layout)
  }
  return 0;  // BYTE_ARRAY
}

int bits_len16(int v) {
  int n = 0;
  while (v) { n++; v >>= 1; }
  return n;
}

uint64_t align_up(uint64_t x, uint64_t a) { return (x + a - 1) / a * a; }

}  // namespace

// PQ_DELTA_TILED=1: DELTA pages through the tiled pipeline (block walk kernel + 2048-value
// tiles) instead of the single-pass page decoder.
static bool delta_tiled() {
  const char *t = getenv("PQ_DELTA_TILED");
  return t && atoi(t) != 0;
}

static bool spec_disabled() {  // PQ_SPEC=0 or PQ_NO_SPEC=1: the reference's serial order
  const char *on = getenv("PQ_SPEC"), *off = getenv("PQ_NO_SPEC");
  if (off && atoi(off) != 0) return true;
  return on && atoi(on) == 0;
}

struct KernelTimer {
  bool enabled = false;
  struct Rec { int slot; hipEvent_t a, b; };
  std::vector<Rec> recs;          // pending launch records
  std::vector<hipEvent_t> pool;   // free events
  double total_ms[PQGPU_TIMER_SLOTS] = {0};
  int64_t launches[PQGPU_TIMER_SLOTS] = {0};
  hipEvent_t get() {
    if (!pool.empty()) { hipEvent_t e = pool.back(); pool.pop_back(); return e; }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
  }
  // Resolve pending records (the caller has synchronised the stream).
  void resolve() {
    for (auto &r : recs) {
      float ms = 0;
      if (hipEventElapsedTime(&ms, r.a, r.b) == hipSuccess) { total_ms[r.slot] += ms; launches[r.slot] += 1; }
      pool.push_back(r.a);
      pool.push_back(r.b);
    }
    recs.clear();
  }
  void destroy() {
    for (auto &r : recs) { pool.push_back(r.a); pool.push_back(r.b); }
    recs.clear();
    for (auto e : pool) (void)hipEventDestroy(e);
    pool.clear();
  }
};
static const char *kTimerNames[PQGPU_TIMER_SLOTS] = {
    "k_levels", "k_values_delta", "k_scan_runs", "k_bases", "k_ba_sums", "k_ba_scan",
    "k_ba_emit", "k_records", "k_values_dict", "k_values", "k_delta_prep", "k_snappy", "k_dict_slots",
    "k_nest_count", "k_nest_emit", "k_level_fill", "k_nest_scan", "k_pba", "k_ba_delta", "k_dba_gather",
    "k_values_copy", "k_group_flat", "k_nest_tile", "k_nest_pcount", "k_nest_tcount"};

// The staged page bytes of a batch: grows geometrically without zero-filling, and in a batch
// with a device context lives in pinned host memory, so upload's H2D copy reads it directly
// (no bounce copy). Capacity is kept across reset(): a reused batch (the pipeline's) plans
// into memory that is already pinned and touched.
struct StageBuf {
  uint8_t *p = nullptr;
  size_t n = 0, cap = 0;
  bool pinned = false;
  StageBuf() = default;
  StageBuf(const StageBuf &) = delete;
  StageBuf &operator=(const StageBuf &) = delete;
  ~StageBuf() { release(); }
  void release() {
    if (p) {
      if (pinned) (void)hipHostFree(p);
      else free(p);
    }
    p = nullptr;
    n = cap = 0;
  }
  bool reserve(size_t want) {
    if (want <= cap) return true;
    size_t c = std::max<size_t>(want, cap ? cap * 2 : (size_t)1 << 20);
    uint8_t *q = nullptr;
    if (pinned) {
      if (hipHostMalloc((void **)&q, c, hipHostMallocCoherent) != hipSuccess) q = nullptr;
    } else {
      q = (uint8_t *)malloc(c);
    }
    if (!q) return false;
    if (n) memcpy(q, p, n);
    uint8_t *old = p;
    const bool was = pinned;
    p = q;
    cap = c;
    if (old) {
      if (was) (void)hipHostFree(old);
      else free(old);
    }
    return true;
  }
  // new bytes are uninitialised unless `fill` >= 0
  void resize(size_t m, int fill = -1) {
    if (m > cap && !reserve(m)) throw std::bad_alloc();
    if (fill >= 0 && m > n) memset(p + n, fill, m - n);
    n = m;
  }
  size_t size() const { return n; }
  uint8_t *data() { return p; }
  const uint8_t *data() const { return p; }
  void clear() { n = 0; }
};

struct pqgpu_batch {
  pqgpu_ctx *ctx = nullptr;
  std::vector<HostChunk> chunks;
  std::vector<PageDesc> pages;
  std::vector<BaDelta> ba_delta;          // DELTA_LENGTH / DELTA_BYTE_ARRAY pages (PageDesc::ba_delta)
  std::vector<uint64_t> ba_delta_scratch; // arena offset of each entry's scratch
  uint64_t o_ba_delta = 0;
  StageBuf stage;
  hipStream_t last_stream = nullptr;  // the stream of the last upload (its H2D reads `stage`)
  // SNAPPY data pages decompressed on the device by k_snappy (default; PQ_HOST_SNAPPY=1
  // decompresses them on the host like GZIP). Pages carry PF_DEV_SNAPPY and `data` = job index
  // until upload, which places their output in a region after the stage.
  struct DevSnappy {
    uint64_t comp_off, raw_off;  // stage offsets: the block (then >= 128 zero bytes), the raw prefix
    int64_t comp_gather = -1;    // page index: the gather job that copies the resident block
                                 // device to device at upload (not staged on the host)
    uint32_t comp_len, vlen;     // block bytes, preamble bytes
    uint32_t raw_len, dlen;      // V2 level bytes, decoded length
    uint32_t page;               // global page index
    bool to_values = false;      // plan: k_snappy writes the page into the chunk's values (SnappyJob::lead)
  };
  bool snappy_direct = !(getenv("PQ_SNAPPY_DIRECT") && atoi(getenv("PQ_SNAPPY_DIRECT")) == 0);
  bool dev_snappy = !(getenv("PQ_HOST_SNAPPY") && atoi(getenv("PQ_HOST_SNAPPY")) != 0);
  std::vector<DevSnappy> snappy;
  std::vector<uint8_t> pagebuf;  // the planner's copy of a device-decompressed page's head
  // UNCOMPRESSED pages of chunks added from an on-device page index: the body is copied device to
  // device from the resident file bytes (k_page_gather, at upload) instead of through the stage.
  struct HostGather { uint64_t src, len; uint32_t page; };
  std::vector<HostGather> gathers;
  uint64_t o_gather = 0;
  // PLAIN BYTE_ARRAY pages (plainba.hip): page list, first segment per page, segment -> page
  std::vector<uint32_t> pba_pages, pba_seg0, pba_seg_page;
  uint64_t l_pba_pages = 0, l_pba_seg0 = 0, l_pba_seg_page = 0, o_pba_segs = 0, o_pba_limit = 0;
  uint64_t o_snappy = 0;
  std::vector<WorkItem> items;
  std::vector<uint32_t> level_pages_bw1;  // flat OPTIONAL pages: k_levels_seg's first, then the others
  uint32_t n_level_seg = 0, n_level_units_seg = 0, n_level_units_hyb = 0;
  std::vector<uint32_t> delta_pages;      // tiled DELTA pages
  std::vector<uint64_t> dblk_base;        // [np] first DeltaBlk of each page
  uint64_t dblk_total = 0;
  uint32_t n_delta_tiles = 0;
  std::vector<uint32_t> level_pages, scan_pages, base_chunks, ba_chunks, rec_pages, nest_chunks;
  std::vector<uint32_t> pc_pages;  // pages of the nested chunks (k_nest_pcount)
  std::vector<uint4> nest_tiles;  // nested fill tiles: {global fill tile, page, tile of the page, chunk}
  std::vector<uint32_t> grp_tiles;  // chunk of every k_group_flat tile (max_rep == 0 leaves with struct bitmaps)
  uint64_t l_grp_tiles = 0;
  uint64_t o_nest_cnt = 0, o_nest_base = 0, o_nest_tot = 0, l_nest_tiles = 0, l_nest_chunks = 0, l_nest_order = 0;
  // k_nest_tile's block order within each list-level group: the chunks' tiles interleaved (block
  // -> tile position), so that a tile's predecessor in its chunk was dispatched a chunk count of
  // blocks earlier and has usually published by the time the tile looks back
  std::vector<uint32_t> nest_order;
  uint64_t o_nest_done = 0;
  uint32_t n_nest_empty = 0;  // nested chunks without fill tiles (first in nest_chunks)
  uint32_t nest_first[PQGPU_MAX_NEST + 2] = {};
  std::vector<uint64_t> run_base, tile_base;
  uint64_t run_total = 0, tile_total = 0;
  // generic level streams: run tables ([np][2] bases) and k_level_fill tiles
  std::vector<uint64_t> lv_run_base;
  std::vector<uint32_t> lv_tile0, lv_tiles, lf_list;
  uint64_t lv_run_total = 0;
  uint64_t o_lv_runs = 0, o_lv_run_base = 0, o_lv_meta = 0, o_lv_tile_run = 0, o_lv_tile0 = 0, l_lv_tiles = 0, l_lf_list = 0;
  std::vector<uint32_t> page_nn_init;
  std::vector<uint64_t> page_vbase_out;  // after sync: per-page value bases / non-null counts
  std::vector<uint32_t> page_nn_out;
  std::vector<uint32_t> page_nn_spec;   // header non-null counts (speculative mode)
  std::vector<uint64_t> page_vbase_spec; // their per-chunk exclusive prefix
  bool spec = false;                     // this upload runs values concurrently with k_levels
  bool bases_known = false;              // flat REQUIRED batch: value bases uploaded, no k_bases
  // Serial batch whose unfused copies all belong to chunks of PLAIN fixed-width pages: a page's non-null
  // count is speculated as its value bytes / width (a well-formed page holds exactly its non-null
  // values), so k_values_copy starts beside the level kernels instead of after k_bases; k_bases checks
  // the decoded counts of those chunks (CF_NN_SPEC) and a miss re-decodes serially, as in spec mode.
  bool copies_early = false;
  std::vector<uint8_t> chunk_nn_spec;
  // Speculative concurrent schedule (values beside k_levels) whenever every page's non-null count
  // is known up front; PQ_SPEC=0 keeps the serial order. cfg2: 0.559 vs 0.595 ms per step.
  bool force_serial = spec_disabled();
  bool split_values = getenv("PQ_SPLIT_VALUES") && atoi(getenv("PQ_SPLIT_VALUES")) != 0;
  // PQ_ONE_STREAM=1 (profiling): every launch on the batch stream, so each kernel is timed alone
  bool one_stream = getenv("PQ_ONE_STREAM") && atoi(getenv("PQ_ONE_STREAM")) != 0;
  bool levels_first = getenv("PQ_LEVELS_FIRST") && atoi(getenv("PQ_LEVELS_FIRST")) != 0;
  // PQ_DICT_ONLY=0: dictionary-only batches take the generic speculative schedule (a reset launch
  // in front of every decode) instead of the two-launch one (decode_impl)
  bool dict_only_off = getenv("PQ_DICT_ONLY") && atoi(getenv("PQ_DICT_ONLY")) == 0;
  // Nested arrays in one pass (k_nest_tile: counts, a decoupled look-back over the chunk's earlier
  // tiles, then the outputs) instead of k_nest_count + k_nest_emit; PQ_NEST_FUSED=0: the two passes
  // The byte-array dictionaries' slot tables built by the run scan's launch (k_scan_slots) instead
  // of their own launch in front of k_ba_emit; PQ_SCAN_SLOTS=0: k_dict_slots
  bool scan_slots = !getenv("PQ_SCAN_SLOTS") || atoi(getenv("PQ_SCAN_SLOTS")) != 0;
  // Nested batches: the repetition streams' level kernels on the aux stream beside the definition
  // streams' (PQ_LV_SPLIT=0: one after the other; cfg4 1.47 -> 1.41 ms). PQ_NEST_PCOUNT=1: the nested
  // pages' counts by k_nest_pcount, so that k_bases and the values path go ahead while k_nest_tile
  // runs on the aux stream -- slower (cfg4 1.41 -> 1.64 ms: the byte-array path beside k_nest_tile
  // 0.38 -> 1.1 ms, profiles/r05_s30_probe_cfg4_sched.txt), so k_nest_tile counts them by default.
  bool level_split = !getenv("PQ_LV_SPLIT") || atoi(getenv("PQ_LV_SPLIT")) != 0;
  bool nest_pcount = getenv("PQ_NEST_PCOUNT") && atoi(getenv("PQ_NEST_PCOUNT")) != 0;
  // PQ_NEST_TCOUNT=1 (batches whose nested chunks all have one list level): every tile's counts from
  // the run tables (k_nest_tcount) and a per-chunk scan before k_nest_tile, which then takes its bases
  // from them instead of looking back over the chunk's earlier tiles. Off: k_nest_tile without the
  // look-back is only 0.63 -> 0.60 ms, and the counts cost 0.13 ms (cfg4 1.37 -> 1.47 ms,
  // profiles/r05_s38_probe_nest_tcount.txt): the look-back's waits overlap other workgroups' work.
  bool nest_tcount = getenv("PQ_NEST_TCOUNT") && atoi(getenv("PQ_NEST_TCOUNT")) != 0;
  // (cfg4: 1.59 -> 1.47 ms, profiles/r05_s29_probe_cfg4_fused.txt)
  bool nest_fused = !getenv("PQ_NEST_FUSED") || atoi(getenv("PQ_NEST_FUSED")) != 0;
  // PLAIN / BOOLEAN copies inside k_values (on the side stream, beside the level kernels and
  // k_values_delta) or as their own zero-LDS launch on the copy stream: fused in the speculative
  // schedule (cfg2: 0.51-0.53 ms fused against 0.56-0.58 split), split in the serial one.
  // PQ_COPY_FUSED=0/1 forces either (set per plan).
  bool copy_fused = false;
  uint32_t n_copy_items = 0;      // the last n_copy_items work items go to k_values_copy
  uint32_t n_dict_items = 0;      // the WI_DICT(2) items, after the n_delta_items: k_values_dict(2)
  uint32_t n_dict2_items = 0;     // the first of them: grouped (WI_DICT2)
  // PQ_COPY_MODE (speculative schedule): where k_values_copy waits — 0 from the start beside
  // everything, 1 after k_values on the side stream, 2 after the level kernels, 3 after both
  int copy_mode = getenv("PQ_COPY_MODE") ? atoi(getenv("PQ_COPY_MODE")) : 0;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr, ev_copy = nullptr, ev_copy_join = nullptr, ev_delta_join = nullptr;
  hipEvent_t ev_levels = nullptr, ev_nest_join = nullptr;
  hipEvent_t ev_lv_fork = nullptr, ev_lv_join = nullptr, ev_aux_fork = nullptr, ev_aux_join = nullptr;
  // Column-group pipeline (speculative batches of flat REQUIRED columns with device SNAPPY pages):
  // the chunks are cut into n_groups contiguous groups; group g's SNAPPY launch is followed on the
  // values streams by its run scan, dictionary tiles and DELTA pages while group g+1 decompresses.
  // Per group: [first, end) of the SNAPPY jobs, the scan pages, the work items, and the number of
  // work items of k_values_delta's launch at the group's start.
  static constexpr int kMaxGroups = 8;
  uint32_t n_groups = 0;
  uint32_t grp_job[kMaxGroups + 1] = {}, grp_scan[kMaxGroups + 1] = {}, grp_item[kMaxGroups + 1] = {},
           grp_delta[kMaxGroups] = {}, grp_dict[kMaxGroups] = {};
  hipEvent_t ev_snap[kMaxGroups] = {};
  std::vector<uint32_t> ba_tile_page;  // byte-array tile -> page
  std::vector<uint32_t> ba_tile_order; // tiles in 8 per-XCD queues (chunk c in queue c mod 8)
  uint32_t ba_class_off[4] = {0, 0, 0, 0};  // class k's blocks in ba_tile_order
  uint32_t n_ba_class[4] = {0, 0, 0, 0};  // tiles per k_ba_emit class
  std::vector<uint32_t> slot_chunks;   // byte-array dictionaries materialised in slots
  uint32_t slot_grid_x = 0;
  bool any_ba_sync = false;
  // byte-array tile bases: k_ba_emit's decoupled look-back (default), or k_ba_sums + k_ba_scan
  // before k_ba_emit (PQ_BA_PRESUM=1; cfg3: 0.16 ms of k_ba_sums for 0.02 ms less k_ba_emit)
  // PQ_BA_PRESUM=2: only the chunks of the LDS-slot class (k_ba_emit_lds) take the pre-pass.
  // Default: the pre-pass whenever nested arrays are emitted beside the values path (their kernels
  // hold CUs the look-back's predecessors wait for; cfg4: k_ba_emit 1.31 ms in the concurrent
  // schedule, 0.28 ms alone; step 2.38 -> 2.12 ms with the pre-pass), else the look-back.
  int ba_presum_mode = getenv("PQ_BA_PRESUM") ? atoi(getenv("PQ_BA_PRESUM")) : -1;
  bool ba_presum = false;  // some chunk of this upload takes the pre-pass
  uint8_t *d_payload = nullptr;         // payload arena of the bounded byte-array chunks
  size_t d_payload_cap = 0;
  // device
  uint8_t *d_stage = nullptr;
  size_t d_stage_cap = 0;
  uint8_t *d_arena = nullptr;
  size_t d_arena_cap = 0;
  uint64_t arena_size = 0;
  // arena offsets of batch-level arrays
  uint64_t o_nnv = 0, o_spec_flag = 0, o_dblk = 0, o_dblk_base = 0, o_dblk_n = 0, o_dblk_sum = 0, l_delta = 0;
  uint64_t o_pages = 0, o_chunks = 0, o_err = 0, o_nn = 0, o_rec = 0, o_vbase = 0, o_rbase = 0, o_runs = 0,
           o_run_base = 0, o_run_count = 0, o_tile_first = 0, o_tile_desc = 0, o_tile_base = 0, o_items = 0, o_lists = 0,
           o_ba_tile_sum = 0, o_ba_tile_page = 0, o_ba_tile_order = 0, o_ba_totals = 0, l_slot = 0,
           o_ba_state = 0, o_nest_state = 0;
  uint64_t l_level_bw1 = 0;
  uint64_t l_level = 0, l_scan = 0, l_base = 0, l_ba = 0, l_rec = 0, l_pc = 0;
  uint64_t z_begin = 0, z_end = 0, f_begin = 0, f_end = 0;  // per-decode reset regions
  // [z_begin, z_bm_end): the validity bitmaps OR-ed at shared edge words (zeroed by the first decode
  // after an upload only: every decode of an uploaded batch writes the same bits, so the words an
  // earlier decode left hold exactly what the OR adds); [z_bm_end, z_end): counters and look-back
  // states, zeroed every decode
  uint64_t z_bm_end = 0;
  bool bm_zeroed = false;
  // Chunk error keys. DELTA-major decodes (cfg2) run their two streams without a join per decode:
  // the values launch on the batch stream reports into o_err / o_err2 (alternately: the launch resets
  // the next decode's buffer itself, err_next), the level stream into o_err_ds (reset with the rest of
  // the per-decode state on that stream). So consecutive decodes put nothing but the values launches
  // on the batch stream -- no reset, no cross-stream wait in front of the critical path; the level
  // stream is joined when anything else needs the batch (join_deferred). sync takes the smaller key
  // of the batch stream's buffer and the level stream's. err_sel: the batch-stream buffer the last
  // decode reported into; err_ready[k]: buffer k's reset is enqueued and it has not been used since.
  uint64_t o_err2 = 0, o_err_ds = 0;
  uint32_t err_sel = 0;
  bool err_ready[2] = {false, false};
  bool ds_pending = false;  // the level stream's work of a DELTA-major decode is not joined yet
  bool ds_synced = false;   // the level stream has waited for the batch stream since the last upload
  uint32_t n_delta_items = 0;
  uint64_t o_dbg = 0;
  bool debug_stamps = getenv("PQ_DEBUG_STAMPS") && atoi(getenv("PQ_DEBUG_STAMPS")) != 0;
  std::vector<ChunkDesc> chunk_desc;
  bool uploaded = false, decoded = false;
  pqgpu_batch_stats stats{};
  KernelTimer timer;
  int64_t slot_bytes[PQGPU_TIMER_SLOTS] = {0};  // algorithmic bytes per launch of each timer slot
};

// ---------------------------------------------------------------------------
// Planning: readChunk / readPages on the host
// ---------------------------------------------------------------------------
static int chunk_fail(pqgpu_batch *b, HostChunk &hc, int32_t id, int code, int page, const std::string &msg,
                      pqgpu_error *err) {
  // SNAPPY blocks staged for the device were read (readPages order) before this failure: the
  // reference decompresses each as it reads it, so the first corrupt one is the chunk's error.
  // Error path only: the full host decode here decides which error the reference reports.
  std::string m = msg;
  for (const auto &j : b->snappy) {
    if (j.page < hc.first_page) continue;
    std::vector<uint8_t> tmp;
    if (!Decompress(1, b->stage.data() + j.comp_off, j.comp_len, &tmp).ok() || tmp.size() != j.dlen) {
      code = PQ_ERR_DECOMPRESS;
      page = (int)(j.page - hc.first_page);
      m = "decompression failed: snappy: corrupt input";
      break;
    }
  }
  set_err(&hc.err, code, id, page, m);
  if (err) *err = hc.err;
  // drop the pages staged for this chunk: the reference returns before any readValues
  b->pages.resize(hc.first_page);
  while (!b->ba_delta.empty() && b->ba_delta.back().page >= hc.first_page) b->ba_delta.pop_back();
  while (!b->snappy.empty() && b->snappy.back().page >= hc.first_page) b->snappy.pop_back();
  while (!b->gathers.empty() && b->gathers.back().page >= hc.first_page) b->gathers.pop_back();
  hc.num_pages = 0;
  return code;
}

static uint64_t stage_append(pqgpu_batch *b, const uint8_t *src, int64_t n) {
  const size_t end = b->stage.size();
  uint64_t off = align_up(end, 16);
  b->stage.resize(off + (size_t)n);
  if (off > end) memset(b->stage.data() + end, 0, off - end);  // alignment gap: zero, as before
  if (n) memcpy(b->stage.data() + off, src, (size_t)n);
  return off;
}

// A SNAPPY block left for k_snappy (read_block with `defer`): where it is and its decoded length.
struct SnappyDefer { const uint8_t *blk = nullptr; int64_t len = 0, dlen = 0; };

// readPageBlock (chunk_reader.go:161-180) + newBlockReader (compress.go:102-123) for a whole block.
// With `defer` a SNAPPY block whose preamble gives the expected size is not decompressed here
// (k_snappy does it; a corrupt body is found there); anything else decodes on the host, whose
// error is the reference's.
// With a page-index entry `ixe` (the on-device walk of this header) the CRC32 verdict comes from
// k_page_crc, and with `direct` an UNCOMPRESSED block is not copied: *direct points at it in the
// caller's file bytes (its body reaches the device through k_page_gather).
static int read_block(const uint8_t *file, int64_t flen, int64_t *off, int64_t *count, int32_t csize, int32_t usize,
                      int validate_crc, const PageHeader &ph, int32_t codec, std::vector<uint8_t> *out,
                      int64_t skip_levels, std::string *msg, SnappyDefer *defer = nullptr,
                      const PageIxEntry *ixe = nullptr, const uint8_t **direct = nullptr) {
  if (csize < 0 || usize < 0) { *msg = "invalid page data size"; return PQ_ERR_INVALID; }
  int64_t avail = *off >= flen ? 0 : flen - *off;
  int64_t take = std::min<int64_t>(csize, avail);
  const uint8_t *blk = file + std::min<int64_t>(*off, flen);
  *off += take;
  *count += take;
  if (validate_crc && ph.has_crc) {
    bool ok;
    if (ixe && (ixe->flags & IXF_CRC_CHECKED)) ok = (ixe->flags & IXF_CRC_OK) != 0;
    else ok = (uint32_t)crc32(0L, blk, (uInt)take) == (uint32_t)ph.crc;
    if (!ok) { *msg = "CRC32 check failed"; return PQ_ERR_CRC; }
  }
  if (direct && codec == 0 && take == csize && usize == csize && skip_levels <= take) {
    *direct = blk;
    return PQ_OK;
  }
  // V2: the level bytes are copied raw, only the values part goes through the codec (page_v2.go:112-127)
  if (skip_levels > 0) {
    if (skip_levels > take) { *msg = "slice bounds out of range"; return PQ_ERR_INVALID; }
    out->insert(out->end(), blk, blk + skip_levels);
    blk += skip_levels;
    take -= skip_levels;
    csize -= (int32_t)skip_levels;
    usize -= (int32_t)skip_levels;
    if (csize < 0 || usize < 0) { *msg = "invalid page data size"; return PQ_ERR_INVALID; }
  }
  if (take != csize) {
    *msg = "compressed data must be " + std::to_string(csize) + " byte but its " + std::to_string(take) + " byte";
    return PQ_ERR_INVALID;
  }
  if (defer && codec == 1) {
    int64_t dlen;
    if (SnappyDecodedLen(blk, take, &dlen) && dlen == usize && (int64_t)out->size() + dlen < (1ll << 31)) {
      defer->blk = blk;
      defer->len = take;
      defer->dlen = dlen;
      return PQ_OK;
    }
  }
  size_t before = out->size();
  Status st = Decompress(codec, blk, take, out);
  if (!st.ok()) { *msg = st.msg; return st.code; }
  if ((int64_t)(out->size() - before) != usize) {
    *msg = "decompressed data must be " + std::to_string(usize) + " byte but its " +
           std::to_string(out->size() - before) + " byte";
    return PQ_ERR_DECOMPRESS;
  }
  return PQ_OK;
}

// Values decoder init() (reference: valuesDecoder.init called from page read()).
// `ensure(k)`: page bytes [0, k) are readable (a device-decompressed page holds only its head
// on the host); false if the block is corrupt there.
static int init_values(const uint8_t *page, int64_t plen, int64_t vstart, uint8_t vk, PageDesc *pd, BaDelta *bd,
                       std::string *msg, const std::function<bool(int64_t)> &ensure) {
  GoReader r{page + vstart, plen - vstart};
  auto corrupt = [&] { *msg = "decompression failed: snappy: corrupt input"; return PQ_ERR_DECOMPRESS; };
  pd->val_off = (uint32_t)vstart;
  pd->val_len = (uint32_t)(plen - vstart);
  if (vk == VK_DICT) {  // dictDecoder.init type_dict.go:22-38
    if (!ensure(vstart + 1)) return corrupt();
    if (r.i >= r.n) { *msg = "EOF"; return PQ_ERR_EOF; }
    uint8_t w = r.p[0];
    if (w > 32) { *msg = "invalid bitwidth " + std::to_string(w); return PQ_ERR_INVALID; }
    pd->dict_bw = w;
    pd->val_off += 1;
    pd->val_len -= 1;
    return PQ_OK;
  }
  if (vk == VK_RLE_BOOL) {  // booleanRLEDecoder.init type_boolean.go:104-107 (hybrid initSize)
    if (!ensure(vstart + 4)) return corrupt();
    int e = r.readfull(4);
    if (e) { *msg = "boolean rle size"; return e; }
    uint32_t size;
    memcpy(&size, r.p, 4);
    int64_t rem = r.n - 4;
    pd->dict_bw = 1;
    pd->val_off += 4;
    pd->val_len = (uint32_t)std::min<int64_t>(size, rem);
    return PQ_OK;
  }
  if (vk == VK_DLBA || vk == VK_DBA) {  // byteArrayDeltaLengthDecoder / byteArrayDeltaDecoder init
    if (!ensure(plen)) return corrupt();
    *bd = BaDelta{};
    int e;
    auto stream = [&](BaDeltaStream *st, DeltaWalk *dw) {
      const int64_t start = r.i;
      GoReader rs{r.p + start, r.n - start};
      int er = delta32_walk(rs, dw, msg);
      st->off = (uint32_t)(vstart + start);
      st->len = (uint32_t)(r.n - start);
      st->hdr = (uint32_t)dw->hdr;
      st->first = dw->first;
      st->count = dw->count;
      st->mbc = (uint16_t)dw->mbc;
      st->mbvc = (uint32_t)dw->mbvc;
      const uint64_t max_blk = 10 + (uint64_t)dw->mbc + (uint64_t)dw->bs * 4;
      st->slow = (dw->mbvc % 8 == 0 && dw->mbc <= 8 && max_blk + 48 <= kDeltaWinLoad) ? 0 : 1;
      r.i = start + rs.i;
      return er;
    };
    DeltaWalk pw{}, sw{};
    if (vk == VK_DBA && (e = stream(&bd->st[1], &pw))) return e;  // prefix lengths first (:195-201)
    if ((e = stream(&bd->st[0], &sw))) return e;
    if (vk == VK_DBA && pw.count != sw.count) {
      *msg = "bytearray/delta: different number of suffixes and prefixes";
      return PQ_ERR_INVALID;
    }
    bd->pay_off = (uint32_t)(vstart + r.i);
    bd->pay_len = (uint32_t)(r.n - r.i);
    return PQ_OK;
  }
  if (vk == VK_DELTA32 || vk == VK_DELTA64) {  // deltaBitPackDecoder.init deltabp_decoder.go:35-111
    bool is64 = vk == VK_DELTA64;
    int32_t bs, mbc, vc;
    int e;
    if (!ensure(vstart + 64)) return corrupt();  // five varints at most 50 bytes
    if ((e = r.uvariant32(&bs))) { *msg = "failed to read block size"; return e; }
    if ((e = r.uvariant32(&mbc))) { *msg = "failed to read number of mini blocks"; return e; }
    if (mbc <= 0 || bs % mbc != 0) { *msg = "int/delta: invalid number of mini blocks"; return PQ_ERR_INVALID; }
    int32_t mbvc = bs / mbc;
    if (mbvc == 0) { *msg = "invalid mini block value count, it can't be zero"; return PQ_ERR_INVALID; }
    if ((e = r.uvariant32(&vc))) { *msg = "failed to read total value count"; return e; }
    int64_t first;
    if (is64) {
      if ((e = r.varint64(&first))) { *msg = "failed to read first value"; return e; }
    } else {
      int32_t f32;
      if ((e = r.variant32(&f32))) { *msg = "failed to read first value"; return e; }
      first = f32;
    }
    int64_t mb_start = r.i;
    int64_t md;
    if (is64) {
      if ((e = r.varint64(&md))) { *msg = "failed to read min delta"; return e; }
    } else {
      int32_t m32;
      if ((e = r.variant32(&m32))) { *msg = "failed to read min delta"; return e; }
    }
    int64_t wstart = r.i;
    if (!ensure(vstart + wstart + std::max(mbc, 0))) return corrupt();
    if ((e = r.readfull(mbc))) { *msg = "not enough data to read all miniblock bit widths"; return e; }
    for (int32_t k = 0; k < mbc; k++)
      if (r.p[wstart + k] > (is64 ? 64 : 32)) { *msg = "invalid miniblock bit width"; return PQ_ERR_INVALID; }
    pd->delta_first = first;
    pd->delta_count = vc;
    pd->delta_mbc = (uint16_t)mbc;  // <= 65535, checked below
    pd->delta_mbvc = (uint32_t)mbvc;
    pd->delta_first_mb = (uint32_t)(vstart + mb_start);
    // shapes of the parallel paths (kernels.hip): whole groups per miniblock, widths packed in
    // one 64-bit word; the page decoder needs a whole block (widest case) inside its LDS
    // window, the tiled pipeline blocks that tile kDeltaTileVals; anything else: exact scalar path
    const uint64_t max_blk = 10 + (uint64_t)mbc + (uint64_t)bs * (is64 ? 8 : 4);
    const bool shape_ok = mbvc % 8 == 0 && mbc <= 8 &&
                          (delta_tiled() ? (bs >= 128 && (int32_t)kDeltaTileVals % bs == 0)
                                         : max_blk + 48 <= kDeltaWinLoad);
    if (!shape_ok) pd->flags |= PF_DELTA_SLOW;
    if (mbc > 65535) { *msg = "more than 65535 miniblocks per block"; return PQ_ERR_UNSUPPORTED; }
    return PQ_OK;
  }
  return PQ_OK;
}

// A chunk's entries of an on-device page index (pagewalk.hip) and where its pages are resident.
struct IxChunkView {
  const PageIxEntry *e;  // page order
  uint32_t n;
  uint64_t dev;          // device address of file byte `file_off`
  int64_t file_off;
  int64_t len;           // resident bytes
};

static void ix_header(const PageIxEntry &x, PageHeader *ph) {
  *ph = PageHeader();
  ph->type = x.type;
  ph->usize = x.usize;
  ph->csize = x.csize;
  ph->crc = x.crc;
  ph->has_crc = x.flags & IXF_CRC;
  ph->has_dph = x.flags & IXF_DPH;
  ph->has_dict = x.flags & IXF_DICT;
  ph->has_dph2 = x.flags & IXF_DPH2;
  ph->dph = DataPageHeader{x.dph[0], x.dph[1], x.dph[2], x.dph[3]};
  ph->dict = DictPageHeader{x.dict[0], x.dict[1]};
  ph->dph2.num_values = x.dph2[0];
  ph->dph2.num_nulls = x.dph2[1];
  ph->dph2.num_rows = x.dph2[2];
  ph->dph2.encoding = x.dph2[3];
  ph->dph2.def_len = x.dph2[4];
  ph->dph2.rep_len = x.dph2[5];
  ph->dph2.is_compressed = x.flags & IXF_COMPRESSED;
}

// ---------------------------------------------------------------------------
// On-device page index (pagewalk.hip)
// ---------------------------------------------------------------------------
struct pqgpu_page_index {
  uint64_t dev = 0;        // device address of file byte `file_off`
  int64_t file_off = 0, len = 0;
  int validate_crc = 0;
  std::vector<pqgpu_chunk_meta> metas;
  std::vector<PageIxChunk> chunks;
  std::vector<PageIxEntry> entries;  // grouped by chunk, page order
  std::vector<uint32_t> first;       // [nchunks + 1] each chunk's entries
  double walk_ms = 0;                // walk (+ checksums) on the device, incl. the table read-back
  int32_t polls = 0;                 // result read-backs beyond the first (a chunk's marker was missing)
  int32_t unreported = 0;            // chunks whose walk never reported (kept with the host walk)
  int32_t overflowed = 0;            // 1: the table could not hold every header (every chunk falls back)
  int32_t stale = 0;                 // entries read back with another build's generation (dropped)
  uint32_t gen = 0;                  // generation of the build whose table was read
};

static void to_public(const PageIxEntry &x, pqgpu_page_header *o) {
  memset(o, 0, sizeof(*o));
  o->header_offset = x.hdr_off;
  o->header_len = x.hdr_len;
  o->type = x.type;
  o->uncompressed_page_size = x.usize;
  o->compressed_page_size = x.csize;
  o->crc = x.crc;
  o->flags = (int32_t)x.flags;
  for (int k = 0; k < 4; k++) o->data_page[k] = x.dph[k];
  for (int k = 0; k < 2; k++) o->dictionary_page[k] = x.dict[k];
  for (int k = 0; k < 6; k++) o->data_page_v2[k] = x.dph2[k];
}

static int add_chunk_impl(pqgpu_batch *b, const uint8_t *file, int64_t flen, const pqgpu_column_info *col,
                          const pqgpu_chunk_meta *meta, int validate_crc, int32_t *chunk_id, pqgpu_error *err,
                          const IxChunkView *ix = nullptr) {
  auto t0 = std::chrono::steady_clock::now();
  int32_t id = (int32_t)b->chunks.size();
  if (chunk_id) *chunk_id = id;
  b->chunks.emplace_back();
  HostChunk &hc = b->chunks.back();
  hc.col = *col;
  hc.meta = *meta;
  clear_err(&hc.err);
  hc.err.chunk = id;
  hc.first_page = (uint32_t)b->pages.size();
  hc.value_width = value_width_of(col->physical_type, col->type_length);
  b->uploaded = false;
  clear_err(err);
  if (meta->has_file_path) return chunk_fail(b, hc, id, PQ_ERR_UNSUPPORTED, -1, "nyi: data is in another file", err);
  if (meta->physical_type != col->physical_type)
    return chunk_fail(b, hc, id, PQ_ERR_INVALID, -1, "wrong type in Column chunk metadata", err);
  if (col->max_def > 255 || col->max_rep > 255)
    return chunk_fail(b, hc, id, PQ_ERR_UNSUPPORTED, -1, "levels deeper than 255 are not supported", err);
  int64_t off = meta->dictionary_page_offset >= 0 ? meta->dictionary_page_offset : meta->data_page_offset;
  if (off < 0) return chunk_fail(b, hc, id, PQ_ERR_INVALID, -1, "seek: negative position", err);
  const int max_rep = col->max_rep, max_def = col->max_def;
  int64_t count = 0;
  std::string msg;
  std::vector<uint8_t> block;
  double decomp_ms = 0;
  uint32_t ixk = 0;  // next page-index entry
  while (meta->total_compressed_size - count > 0) {
    PageHeader ph;
    int64_t consumed = 0;
    const PageIxEntry *ixe = nullptr;  // this header as the device walk decoded it
    bool ok;
    if (ix && ixk < ix->n && ix->e[ixk].hdr_off == off) {
      ixe = &ix->e[ixk++];
      ix_header(*ixe, &ph);
      consumed = ixe->hdr_len;
      ok = true;
    } else {
      ok = off < flen && ParsePageHeader(file + off, flen - off, &ph, &consumed);
    }
    off += consumed;
    count += consumed;
    if (!ok) return chunk_fail(b, hc, id, PQ_ERR_THRIFT, -1, "thrift: invalid page header", err);
    if (ph.type == 2) {  // DICTIONARY_PAGE page_dict.go:35-72
      if (hc.has_dict) return chunk_fail(b, hc, id, PQ_ERR_INVALID, -1, "there should be only one dictionary", err);
      if (col->physical_type == T_BOOLEAN)
        return chunk_fail(b, hc, id, PQ_ERR_UNSUPPORTED, -1, "type BOOLEAN is not supported for dict value encoder", err);
      if (!ph.has_dict) return chunk_fail(b, hc, id, PQ_ERR_INVALID, -1, "null DictionaryPageHeader", err);
      if (ph.dict.num_values < 0) return chunk_fail(b, hc, id, PQ_ERR_INVALID, -1, "negative NumValues in DICTIONARY_PAGE", err);
      if (ph.dict.encoding != ENC_PLAIN && ph.dict.encoding != ENC_PLAIN_DICTIONARY)
        return chunk_fail(b, hc, id, PQ_ERR_UNSUPPORTED, -1,
                          "only Encoding_PLAIN and Encoding_PLAIN_DICTIONARY is supported for dict values encoder", err);
      block.clear();
      auto d0 = std::chrono::steady_clock::now();
      int e = read_block(file, flen, &off, &count, ph.csize, ph.usize, validate_crc, ph, meta->codec, &block, 0, &msg,
                         nullptr, ixe);
      decomp_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - d0).count();
      if (e) return chunk_fail(b, hc, id, e, -1, msg, err);
      hc.has_dict = true;
      hc.dict_count = (uint32_t)ph.dict.num_values;
      hc.dict_len = (uint32_t)block.size();
      hc.dict_off = stage_append(b, block.data(), (int64_t)block.size());
      int w = hc.value_width;
      if (w == 0) {  // BYTE_ARRAY: byteArrayPlainDecoder.next per entry (type_bytearray.go:24-45)
        std::string dm;
        int de = walk_ba_dict(block.data(), (int64_t)block.size(), hc.dict_count, 0, &hc.dict_ent, &hc.dict_max_len, &dm);
        if (de) return chunk_fail(b, hc, id, de, -1, dm, err);
      }
      if (w > 0) {  // fixed width PLAIN dictionary: binary.Read per entry
        uint64_t need = (uint64_t)w * hc.dict_count;
        if (need > block.size()) {
          uint64_t rem = block.size() % (uint64_t)w;
          if (col->physical_type == T_INT96 && block.size() / 12 + 1 == hc.dict_count && rem)
            return chunk_fail(b, hc, id, PQ_ERR_INVALID, -1, "truncated INT96 dictionary entry (nil slot)", err);
          return chunk_fail(b, hc, id, rem == 0 ? PQ_ERR_EOF : PQ_ERR_UNEXPECTED_EOF, -1,
                            "expected " + std::to_string(hc.dict_count) + " values", err);
        }
      }
      if (meta->dictionary_page_offset >= 0 && meta->dictionary_page_offset != off) {
        int64_t np = meta->data_page_offset;
        if (np < 0) return chunk_fail(b, hc, id, PQ_ERR_INVALID, -1, "seek: negative position", err);
        count += np - off;
        off = np;
      }
      continue;
    }
    if (ph.type != 0 && ph.type != 3)
      return chunk_fail(b, hc, id, PQ_ERR_UNSUPPORTED, -1, "DATA_PAGE or DATA_PAGE_V2 type supported", err);
    int pi = (int)b->pages.size() - (int)hc.first_page;
    PageDesc pd;
    memset(&pd, 0, sizeof(pd));
    BaDelta bd{};
    pd.chunk = (uint32_t)id;
    pd.page_in_chunk = (uint32_t)pi;
    block.clear();
    uint8_t vk = 0;
    // SNAPPY data pages go to k_snappy unless their values decoder reads the whole page at
    // init (DELTA_LENGTH / DELTA_BYTE_ARRAY walk every length on the host)
    SnappyDefer sd;
    SnappyPrefix sp;
    bool can_defer = false;
    if (b->dev_snappy && meta->codec == 1 && (ph.type == 0 ? ph.has_dph : ph.has_dph2)) {
      uint8_t vk_peek = 0;
      std::string ignored;
      can_defer = pick_vkind(ph.type == 0 ? ph.dph.encoding : ph.dph2.encoding, col->physical_type, col->type_length,
                             &vk_peek, &ignored) == PQ_OK &&
                  vk_peek != VK_DLBA && vk_peek != VK_DBA;
    }
    // the page bytes the planner reads: the host-decoded block, or (deferred) the raw prefix
    // plus the decoded head in pagebuf, extended on demand
    const uint8_t *pg = nullptr;
    int64_t plen = 0, raw_len = 0;
    const uint8_t *direct = nullptr;  // resident UNCOMPRESSED block (page index): read in place
    const uint8_t **want_direct = ixe ? &direct : nullptr;
    auto bind_page = [&]() {
      if (direct) { pg = direct; plen = ph.csize; return; }
      if (!sd.blk) { pg = block.data(); plen = (int64_t)block.size(); return; }
      raw_len = (int64_t)block.size();
      plen = raw_len + sd.dlen;
      if ((int64_t)b->pagebuf.size() < plen + 64) b->pagebuf.resize((size_t)plen + 64);
      if (raw_len) memcpy(b->pagebuf.data(), block.data(), (size_t)raw_len);
      sp.Init(sd.blk, sd.len, b->pagebuf.data() + raw_len, sd.dlen);
      pg = b->pagebuf.data();
    };
    auto ensure = [&](int64_t upto) -> bool { return !sd.blk || upto <= raw_len || sp.Extend(upto - raw_len); };
    // stage the raw prefix and the block now: a later failure in this chunk checks the block
    auto stage_snappy = [&]() {
      pqgpu_batch::DevSnappy j;
      j.raw_off = stage_append(b, block.data(), (int64_t)block.size());
      j.raw_len = (uint32_t)block.size();
      j.comp_len = (uint32_t)sd.len;
      j.vlen = (uint32_t)(sp.src - sd.blk);
      j.dlen = (uint32_t)sd.dlen;
      j.page = (uint32_t)b->pages.size();
      const int64_t at = (int64_t)(sd.blk - file) - (ix ? ix->file_off : 0);
      if (ix && at >= 0 && at + sd.len <= ix->len) {
        // page index: the block is already in HBM; k_page_gather copies it into the batch at
        // upload (the resident bytes are needed only until then), with zero bytes after it
        j.comp_off = 0;
        j.comp_gather = (int64_t)b->gathers.size();
        b->gathers.push_back(pqgpu_batch::HostGather{ix->dev + (uint64_t)at, (uint64_t)sd.len, j.page});
      } else {
        j.comp_off = stage_append(b, sd.blk, sd.len);
        b->stage.resize(b->stage.size() + 128, 0);  // k_snappy reads up to 70 bytes past the block
      }
      b->snappy.push_back(j);
    };
    auto corrupt_fail = [&]() {
      return chunk_fail(b, hc, id, PQ_ERR_DECOMPRESS, pi, "decompression failed: snappy: corrupt input", err);
    };
    if (ph.type == 0) {
      // dataPageReaderV1.init page_v1.go:65-85 then read :87-122
      if (!ph.has_dph) return chunk_fail(b, hc, id, PQ_ERR_INVALID, pi, "page header is missing data page header", err);
      if (max_rep > 0 && ph.dph.rep_enc != ENC_RLE)
        return chunk_fail(b, hc, id, PQ_ERR_UNSUPPORTED, pi, "encoding is not supported for definition and repetition level", err);
      if (max_def > 0 && ph.dph.def_enc != ENC_RLE)
        return chunk_fail(b, hc, id, PQ_ERR_UNSUPPORTED, pi, "encoding is not supported for definition and repetition level", err);
      if (ph.dph.num_values < 0) return chunk_fail(b, hc, id, PQ_ERR_INVALID, pi, "negative NumValues in DATA_PAGE", err);
      auto d0 = std::chrono::steady_clock::now();
      int e = read_block(file, flen, &off, &count, ph.csize, ph.usize, validate_crc, ph, meta->codec, &block, 0, &msg,
                         can_defer ? &sd : nullptr, ixe, want_direct);
      if (!e) bind_page();
      decomp_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - d0).count();
      if (e) return chunk_fail(b, hc, id, e, pi, msg, err);
      if (sd.blk) stage_snappy();
      if ((e = pick_vkind(ph.dph.encoding, col->physical_type, col->type_length, &vk, &msg)))
        return chunk_fail(b, hc, id, e, pi, msg, err);
      pd.num_slots = (uint32_t)ph.dph.num_values;
      GoReader r{pg, plen};
      if (max_rep > 0) {  // hybridDecoder.initSize: u32 length, LimitReader, ReadAll (buffered)
        if (!ensure(r.i + 4)) return corrupt_fail();
        if ((e = r.readfull(4))) return chunk_fail(b, hc, id, e, pi, "read repetition level size", err);
        uint32_t sz;
        memcpy(&sz, pg + r.i - 4, 4);
        int64_t take = std::min<int64_t>(sz, r.n - r.i);
        pd.rep_off = (uint32_t)r.i;
        pd.rep_len = (uint32_t)take;
        pd.flags |= PF_REP;
        r.i += take;
      }
      if (max_def > 0) {
        if (!ensure(r.i + 4)) return corrupt_fail();
        if ((e = r.readfull(4))) return chunk_fail(b, hc, id, e, pi, "read definition level size", err);
        uint32_t sz;
        memcpy(&sz, pg + r.i - 4, 4);
        int64_t take = std::min<int64_t>(sz, r.n - r.i);
        pd.def_off = (uint32_t)r.i;
        pd.def_len = (uint32_t)take;
        pd.flags |= PF_DEF;
        r.i += take;
      }
      if ((e = init_values(pg, plen, r.i, vk, &pd, &bd, &msg, ensure))) return chunk_fail(b, hc, id, e, pi, msg, err);
    } else {
      // dataPageReaderV2.read page_v2.go:79-131
      if (!ph.has_dph2) return chunk_fail(b, hc, id, PQ_ERR_INVALID, pi, "null DataPageHeaderV2", err);
      if (ph.dph2.num_values < 0) return chunk_fail(b, hc, id, PQ_ERR_INVALID, pi, "negative NumValues in DATA_PAGE_V2", err);
      if (ph.dph2.rep_len < 0) return chunk_fail(b, hc, id, PQ_ERR_INVALID, pi, "invalid RepetitionLevelsByteLength", err);
      if (ph.dph2.def_len < 0) return chunk_fail(b, hc, id, PQ_ERR_INVALID, pi, "invalid DefinitionLevelsByteLength", err);
      int e;
      if ((e = pick_vkind(ph.dph2.encoding, col->physical_type, col->type_length, &vk, &msg)))
        return chunk_fail(b, hc, id, e, pi, msg, err);
      int64_t levels = (int64_t)ph.dph2.rep_len + ph.dph2.def_len;
      auto d0 = std::chrono::steady_clock::now();
      e = read_block(file, flen, &off, &count, ph.csize, ph.usize, validate_crc, ph, meta->codec, &block, levels, &msg,
                     can_defer ? &sd : nullptr, ixe, want_direct);
      if (!e) bind_page();
      decomp_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - d0).count();
      if (e) return chunk_fail(b, hc, id, e, pi, msg, err);
      if (sd.blk) stage_snappy();
      pd.num_slots = (uint32_t)ph.dph2.num_values;
      pd.flags |= PF_V2;
      if (ph.dph2.num_nulls >= 0 && ph.dph2.num_nulls <= ph.dph2.num_values) {
        // a hint only: the reference counts non-nulls from the definition levels
        // (page_v2.go:47-50); k_bases checks the hint against that count
        pd.flags |= PF_BASE_KNOWN;
        pd.expect_nn = (uint32_t)(ph.dph2.num_values - ph.dph2.num_nulls);
      }
      if (ph.dph2.rep_len > 0 && max_rep > 0) { pd.rep_off = 0; pd.rep_len = (uint32_t)ph.dph2.rep_len; pd.flags |= PF_REP; }
      if (ph.dph2.def_len > 0 && max_def > 0) {
        pd.def_off = (uint32_t)ph.dph2.rep_len;
        pd.def_len = (uint32_t)ph.dph2.def_len;
        pd.flags |= PF_DEF;
      }
      if ((e = init_values(pg, plen, levels, vk, &pd, &bd, &msg, ensure))) return chunk_fail(b, hc, id, e, pi, msg, err);
    }
    if (hc.num_slots + pd.num_slots > 0x7fffffffULL)
      return chunk_fail(b, hc, id, PQ_ERR_UNSUPPORTED, pi, "more than 2^31-1 level slots in one chunk", err);
    pd.vkind = vk;
    if (vk == VK_DLBA || vk == VK_DBA) {
      bd.page = (uint32_t)b->pages.size();
      pd.ba_delta = (uint32_t)b->ba_delta.size();
      b->ba_delta.push_back(bd);
    }
    if (sd.blk) {  // staged by stage_snappy(); k_snappy writes the page
      pd.flags |= PF_DEV_SNAPPY;
      pd.data = b->snappy.size() - 1;  // job index until upload
    } else if (direct) {  // resident: k_page_gather copies the block at upload
      pd.flags |= PF_DEV_GATHER;
      pd.data = b->gathers.size();  // gather-job index until upload
      b->gathers.push_back(pqgpu_batch::HostGather{ix->dev + (uint64_t)((direct - file) - ix->file_off),
                                                    (uint64_t)plen, (uint32_t)b->pages.size()});
    } else {
      pd.data = stage_append(b, block.data(), (int64_t)block.size());  // stage offset until upload
    }
    pd.slot_base = hc.num_slots;
    hc.num_slots += pd.num_slots;
    b->pages.push_back(pd);
    hc.num_pages++;
  }
  if (col->physical_type == T_FLBA && hc.value_width > 0) {
    // FIXED_LEN_BYTE_ARRAY with a DELTA_BYTE_ARRAY page: the reference's byteArrayDeltaDecoder
    // returns []byte values of any length (type_bytearray.go:216-240), so the whole chunk uses
    // the byte-array layout (offsets + payload); its PLAIN pages walk type_length-byte values
    bool any_dba = false;
    for (uint32_t p = hc.first_page; p < hc.first_page + hc.num_pages; p++) any_dba |= b->pages[p].vkind == VK_DBA;
    if (any_dba) {
      hc.value_width = 0;
      for (uint32_t p = hc.first_page; p < hc.first_page + hc.num_pages; p++)
        if (b->pages[p].vkind == VK_PLAIN_FIXED) b->pages[p].vkind = VK_PLAIN_BA;
      if (hc.has_dict) {  // entries of type_length bytes (validated above as a fixed-width dictionary)
        hc.dict_ent.resize(2 * (size_t)hc.dict_count);
        for (uint32_t k = 0; k < hc.dict_count; k++) {
          hc.dict_ent[2 * k] = k * (uint32_t)col->type_length;
          hc.dict_ent[2 * k + 1] = (uint32_t)col->type_length;
        }
        hc.dict_max_len = (uint32_t)col->type_length;
      }
    }
  }
  if (!hc.dict_ent.empty())
    hc.dict_ent_off = stage_append(b, (const uint8_t *)hc.dict_ent.data(), (int64_t)hc.dict_ent.size() * 4);
  b->stats.host_decompress_ms += decomp_ms;
  b->stats.host_plan_ms +=
      std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() - decomp_ms;
  return PQ_OK;
}

// ---------------------------------------------------------------------------
// Upload: arena layout, descriptors, work lists
// ---------------------------------------------------------------------------
static hipError_t join_deferred(pqgpu_batch *b, hipStream_t s);
// k_ba_emit class 3 (bytearray.hip k_ba_emit_lds): dictionary pages only (so no CF_BA_SYNC unless the
// payload bound passes 2 GiB), 16- / 32-B slots (entries of at most 28 bytes: slot_shift <= 5) of a
// dictionary of at most 1,024 entries, whose first slot pieces fit in LDS. Decided from the chunk's
// dictionary before the slot table and the payload bound are (build_and_upload: the tile size
// depends on it). PQ_BA_LDS_SLOTS=0: never (comparison runs).
static bool ba_lds_class(const pqgpu_batch *b, const HostChunk &hc) {
  const char *lsv = getenv("PQ_BA_LDS_SLOTS");
  if ((lsv && atoi(lsv) == 0) || !hc.has_dict || hc.dict_count == 0 || hc.dict_count > 1024 || hc.dict_max_len > 28)
    return false;
  uint64_t bound = 0;
  for (uint32_t p = hc.first_page; p < hc.first_page + hc.num_pages; p++) {
    if (b->pages[p].vkind != VK_DICT) return false;
    bound += (uint64_t)b->pages[p].num_slots * hc.dict_max_len;
  }
  return bound <= 0x7fffffffULL - 64;
}
static int build_and_upload(pqgpu_batch *b, hipStream_t s, pqgpu_error *err) {
  if (b->ctx) HIPCHECK(join_deferred(b, s), err);  // (the level stream may still read the stage)
  const uint32_t np = (uint32_t)b->pages.size(), nc = (uint32_t)b->chunks.size();
  b->items.clear();
  b->level_pages.clear();
  b->level_pages_bw1.clear();
  b->ba_delta_scratch.assign(b->ba_delta.size(), 0);
  b->delta_pages.clear();
  b->pba_pages.clear();
  b->pba_seg0.clear();
  b->pba_seg_page.clear();
  b->dblk_base.assign(np, 0);
  b->dblk_total = 0;
  b->scan_pages.clear();
  b->base_chunks.clear();
  b->ba_chunks.clear();
  b->rec_pages.clear();
  b->pc_pages.clear();
  b->nest_tiles.clear();
  b->nest_chunks.clear();
  b->grp_tiles.clear();
  b->run_base.assign(np, 0);
  b->tile_base.assign(np, 0);
  b->lv_run_base.assign(2 * (size_t)np, 0);
  b->lv_tile0.assign(np, 0);
  b->lv_tiles.clear();
  b->lf_list.clear();
  b->lv_run_total = 0;
  b->page_nn_init.assign(np, 0);
  b->ba_tile_page.clear();
  b->ba_tile_order.clear();
  b->slot_chunks.clear();
  b->slot_grid_x = 0;
  b->any_ba_sync = false;
  b->run_total = b->tile_total = 0;
  uint64_t payload_arena = 0;  // bytes of the bounded byte-array chunks' payload arena
  uint64_t a = 256;  // offset 0 is reserved: a zero offset means "not allocated"
  auto take = [&](uint64_t bytes) {
    uint64_t o = align_up(a, 256);
    a = o + align_up(std::max<uint64_t>(bytes, 1), 16);
    return o;
  };
  int64_t in_bytes = 0;
  // Region zeroed before every decode: the validity bitmaps, then per-page record/run counters.
  // A flat OPTIONAL chunk whose every page goes to k_levels_seg and covers whole bitmap words (slot
  // base and count multiples of 32, at most the kernel's LDS image) has every word of its bitmap
  // stored by that kernel each decode (a page that fails writes nothing, and the chunk reports the
  // error): its bitmap lies past the region (cfg2: 16 MB less zeroing per decode).
  const bool lv_seg = !(getenv("PQ_LV_SEG") && atoi(getenv("PQ_LV_SEG")) == 0) &&
                      !(getenv("PQ_LV_WAVE") && atoi(getenv("PQ_LV_WAVE")) == 1);  // (launch_levels' routing)
  auto seg_whole_words = [&](const HostChunk &hc) {
    if (!lv_seg || hc.err.code || hc.col.max_def != 1 || hc.col.max_rep != 0) return false;
    for (uint32_t p = hc.first_page; p < hc.first_page + hc.num_pages; p++) {
      const PageDesc &pd = b->pages[p];
      if (!(pd.flags & PF_DEF) || (uint64_t)pd.def_len + 24 > kSgStageHost || pd.slot_base % 32 || pd.num_slots % 32 ||
          pd.num_slots > kSgImageSlotsHost)
        return false;
    }
    return true;
  };
  b->z_begin = align_up(a, 256);
  for (uint32_t c = 0; c < nc; c++) {
    HostChunk &hc = b->chunks[c];
    hc.valid_unzeroed = hc.col.max_def > 0 && seg_whole_words(hc);
    hc.o_valid = (!hc.err.code && hc.col.max_def > 0 && !hc.valid_unzeroed) ? take(((hc.num_slots + 31) / 32 + 2) * 4) : 0;
    // nested output: list validity bitmaps and element validity (OR-ed by k_nest_emit)
    hc.nest = 0;
    if (!hc.err.code && hc.col.max_rep > 0 && hc.col.max_rep <= PQGPU_MAX_NEST) {
      bool ok = true;
      for (int k = 0; k < hc.col.max_rep; k++)
        ok &= hc.col.list_def[k] > 0 && hc.col.list_def[k] <= hc.col.max_def && hc.col.list_null_def[k] < hc.col.list_def[k];
      if (ok) hc.nest = (uint32_t)hc.col.max_rep;
    }
    const uint64_t words = ((hc.num_slots + 31) / 32 + 2) * 4;
    for (uint32_t k = 0; k < PQGPU_MAX_NEST; k++) hc.o_lvl_valid[k] = k < hc.nest ? take(words) : 0;
    hc.o_elem_valid = hc.nest ? take(words) : 0;
    // struct validity of the OPTIONAL groups (with the nested arrays, or for max_rep == 0 leaves);
    // a group whose bits equal an existing bitmap's shares it
    hc.ngroups = 0;
    for (uint32_t g = 0; g < PQGPU_MAX_NEST; g++) hc.o_grp_valid[g] = 0;
    const int R = hc.col.max_rep;
    if (!hc.err.code && (R == 0 || hc.nest) && hc.col.num_groups > 0 && hc.col.num_groups <= PQGPU_MAX_NEST) {
      bool ok = true;
      for (int g = 0; g < hc.col.num_groups; g++)
        ok &= hc.col.group_def[g] >= 1 && hc.col.group_def[g] <= hc.col.max_def && hc.col.group_depth[g] >= 0 &&
              hc.col.group_depth[g] <= R && (R > 0 || hc.col.max_def > 1 || hc.col.group_def[g] == hc.col.max_def);
      if (ok) hc.ngroups = (uint32_t)hc.col.num_groups;
    }
    for (uint32_t g = 0; g < hc.ngroups; g++) {
      const int j = hc.col.group_depth[g], dg = hc.col.group_def[g];
      hc.grp_alias[g] = -1;
      if (j < R && dg == hc.col.list_null_def[j]) hc.grp_alias[g] = (int8_t)j;
      else if (j == R && dg == hc.col.max_def) hc.grp_alias[g] = R ? 8 : 9;
      if (hc.grp_alias[g] < 0) hc.o_grp_valid[g] = take(words);
    }
  }
  b->z_bm_end = a;
  b->o_rec = take((uint64_t)np * 4);
  b->o_run_count = take((uint64_t)np * 4);
  b->o_spec_flag = take(4);
  b->o_nest_done = take((uint64_t)nc * 4);
  uint64_t n_ba_tiles = 0;  // byte-array tiles (for the look-back state, zeroed per decode)
  for (uint32_t c = 0; c < nc; c++) {
    HostChunk &hc = b->chunks[c];
    if (hc.err.code || hc.value_width != 0) continue;
    hc.ba_tile_vals = ba_lds_class(b, hc) ? kBaTileLds : kBaTile;
    for (uint32_t p = hc.first_page; p < hc.first_page + hc.num_pages; p++)
      n_ba_tiles += (b->pages[p].num_slots + hc.ba_tile_vals - 1) / hc.ba_tile_vals;
  }
  b->o_ba_state = take(n_ba_tiles * 128);  // one 128-B line per tile (bytearray.hip kStStride)
  uint64_t n_nest_tiles = 0;  // nested tiles (k_nest_tile's look-back state, zeroed per decode)
  for (uint32_t c = 0; c < nc; c++) {
    const HostChunk &hc = b->chunks[c];
    if (!hc.nest) continue;
    for (uint32_t p = hc.first_page; p < hc.first_page + hc.num_pages; p++) {
      const uint64_t sb = b->pages[p].slot_base, ns = b->pages[p].num_slots;
      n_nest_tiles += ns ? (sb + ns - 1) / kLfTileHost - sb / kLfTileHost + 1 : 0;
    }
  }
  b->o_nest_state = take(n_nest_tiles * 128);  // one 128-B line per tile (nested.hip kNsStride)
  b->z_end = a;
  for (uint32_t c = 0; c < nc; c++) {
    HostChunk &hc = b->chunks[c];
    if (hc.valid_unzeroed) hc.o_valid = take(((hc.num_slots + 31) / 32 + 2) * 4);
  }
  for (uint32_t c = 0; c < nc; c++) {
    HostChunk &hc = b->chunks[c];
    if (hc.err.code) continue;
    const int w = hc.value_width;
    const uint64_t ns = hc.num_slots;
    bool is_ba = w == 0;
    hc.o_values = is_ba ? 0 : take(ns * (uint64_t)w);
    hc.o_def = hc.col.max_def > 1 ? take(ns) : 0;
    hc.o_rep = hc.col.max_rep > 0 ? take(ns) : 0;
    hc.o_lists = hc.col.max_rep > 0 ? take((ns + 1) * 4) : 0;
    for (uint32_t k = 0; k < PQGPU_MAX_NEST; k++) hc.o_lvl_off[k] = k < hc.nest ? take((ns + 1) * 4) : 0;
    if (hc.nest) b->nest_chunks.push_back(c);
    hc.grp_tile0 = (uint32_t)b->grp_tiles.size();
    bool own_flat = false;
    for (uint32_t g = 0; g < hc.ngroups; g++) own_flat |= hc.col.max_rep == 0 && hc.grp_alias[g] < 0;
    if (own_flat)  // k_group_flat: one 256-thread workgroup per kGrpTile slots (32 per thread)
      b->grp_tiles.insert(b->grp_tiles.end(), (size_t)((ns + kGrpTileHost - 1) / kGrpTileHost), c);
    hc.o_offsets = is_ba ? take((ns + 1) * 4) : 0;
    hc.o_ba_index = 0;
    b->base_chunks.push_back(c);
    if (hc.has_dict) in_bytes += hc.dict_len;
    uint64_t bound = 0;  // byte-array payload upper bound (k_ba_emit writes no more)
    hc.ba_sync = false;
    if (is_ba) {
      b->ba_chunks.push_back(c);
      bool srcs = false;  // pages whose value kernels record a source address per value
      for (uint32_t p = hc.first_page; p < hc.first_page + hc.num_pages; p++) {
        PageDesc &pd = b->pages[p];
        pd.ba_tile = (uint32_t)b->ba_tile_page.size();
        for (uint32_t k = 0; k < (pd.num_slots + hc.ba_tile_vals - 1) / hc.ba_tile_vals; k++) b->ba_tile_page.push_back(p);
        switch (pd.vkind) {
          case VK_DICT: bound += (uint64_t)pd.num_slots * hc.dict_max_len; break;
          case VK_PLAIN_BA: bound += pd.val_len; srcs = true; break;
          case VK_DLBA: bound += b->ba_delta[pd.ba_delta].pay_len; srcs = true; break;
          default: hc.ba_sync = true; srcs = true; break;  // DELTA_BYTE_ARRAY: prefixes repeat bytes
        }
      }
      if (bound > 0x7fffffffULL - 64) hc.ba_sync = true;
      hc.o_ba_index = srcs ? take(ns * 8) : 0;
      hc.slot_shift = 0;
      hc.o_slots = 0;
      if (hc.has_dict && hc.dict_count && hc.dict_max_len <= 60) {  // slot table (k_dict_slots)
        hc.slot_shift = hc.dict_max_len <= 12 ? 4 : hc.dict_max_len <= 28 ? 5 : 6;  // [u32 len | bytes]
        hc.o_slots = take((uint64_t)hc.dict_count << hc.slot_shift);
        b->slot_chunks.push_back(c);
        b->slot_grid_x = std::max<uint32_t>(b->slot_grid_x, std::min<uint32_t>((hc.dict_count + 255) / 256, 1024));
      }
      if (!hc.ba_sync) {
        hc.payload_off = payload_arena;
        hc.payload_bound = bound;
        payload_arena = align_up(payload_arena + bound + 64, 256);
      }
      b->any_ba_sync |= hc.ba_sync;
    }
    for (uint32_t p = hc.first_page; p < hc.first_page + hc.num_pages; p++) {
      PageDesc &pd = b->pages[p];
      in_bytes += pd.rep_len + pd.def_len + pd.val_len;
      if (hc.col.max_def == 1 && hc.col.max_rep == 0) {
        b->level_pages_bw1.push_back(p);  // (ordered below: pages for k_levels_seg first)
      } else if (hc.col.max_def > 0 || hc.col.max_rep > 0) {
        // generic: one k_levels workgroup per stream (page << 1 | 0 rep, 1 def) writing a run
        // table of at most one entry per two stream bytes; k_level_fill tiles expand them
        if (hc.col.max_rep > 0) {
          b->level_pages.push_back(p << 1);
          b->lv_run_base[2 * (size_t)p] = b->lv_run_total;
          b->lv_run_total += pd.rep_len / 2 + 2;
        }
        if (hc.col.max_def > 0) {
          b->level_pages.push_back(p << 1 | 1);
          b->lv_run_base[2 * (size_t)p + 1] = b->lv_run_total;
          b->lv_run_total += pd.def_len / 2 + 2;
        } else {
          b->page_nn_init[p] = pd.num_slots;
        }
        b->lv_tile0[p] = (uint32_t)b->lv_tiles.size();
        const uint64_t sb = pd.slot_base, ns = pd.num_slots;
        const uint64_t nt = ns ? (sb + ns - 1) / kLfTileHost - sb / kLfTileHost + 1 : 0;
        b->lv_tiles.insert(b->lv_tiles.end(), nt, p);
      } else {
        b->page_nn_init[p] = pd.num_slots;
      }
      if (hc.col.max_rep > 0 && !hc.nest) b->rec_pages.push_back(p);  // nested chunks: k_nest_emit
      if (hc.nest && pd.num_slots) b->pc_pages.push_back(p);
      const uint32_t ns_p = pd.num_slots;
      const uint32_t plain_tile_b = getenv("PQ_PLAIN_TILE_B") ? (uint32_t)atoi(getenv("PQ_PLAIN_TILE_B")) : 0u;  // (probe)
      auto tiles = [&](uint8_t kind, uint32_t tile) {
        for (uint32_t v0 = 0; v0 < ns_p; v0 += tile) b->items.push_back(WorkItem{p, v0, std::min(v0 + tile, ns_p), kind, {0, 0, 0}});
      };
      if (pd.flags & PF_DEV_SNAPPY) {
        // a REQUIRED fixed-width PLAIN page whose decoded bytes are exactly its values: k_snappy
        // writes them into the values array itself and no k_values item copies them again
        pqgpu_batch::DevSnappy &j = b->snappy[pd.data];
        const int w = hc.value_width;
        j.to_values = b->snappy_direct && hc.col.max_def == 0 && hc.col.max_rep == 0 && w > 0 &&
                      (pd.vkind == VK_PLAIN_FIXED || pd.vkind == VK_PLAIN_INT96) && j.raw_len == 0 && pd.val_off == 0 &&
                      (uint64_t)pd.num_slots * (uint64_t)w == j.dlen && pd.val_len == j.dlen;
      }
      const bool snappy_values = (pd.flags & PF_DEV_SNAPPY) && b->snappy[pd.data].to_values;
      switch (pd.vkind) {
        case VK_PLAIN_FIXED: case VK_PLAIN_INT96:
          if (!snappy_values) tiles(WI_PLAIN, std::max<uint32_t>(1, (plain_tile_b ? plain_tile_b : kPlainTileBytes) / std::max(1, hc.value_width)));
          break;
        case VK_PLAIN_BOOL: tiles(WI_BOOL, kPlainTile); break;
        case VK_DICT: case VK_RLE_BOOL: {
          if (pd.dict_bw > 0 && ns_p > 0) {
            b->scan_pages.push_back(p);
            uint64_t cap = std::min<uint64_t>(ns_p, (uint64_t)pd.val_len / 2 + 1) + 1;
            b->run_base[p] = b->run_total;
            b->run_total += cap;
            b->tile_base[p] = b->tile_total;
            pd.dict_tile0 = (uint32_t)b->tile_total;
            b->tile_total += (ns_p + kDictTile - 1) / kDictTile;
          }
          if (!is_ba) tiles(WI_DICT, kDictTile);  // byte-array dictionaries: k_ba_sums / k_ba_emit
          break;
        }
        case VK_DELTA32: case VK_DELTA64:
          if (!ns_p) break;
          if (pd.flags & PF_DELTA_SLOW) {
            b->items.push_back(WorkItem{p, 0, ns_p, WI_DELTA, {0, 0, 0}});
          } else if (!delta_tiled()) {
            b->items.push_back(WorkItem{p, 0, ns_p, WI_DELTA_PAGE, {0, 0, 0}});
          } else {
            const uint32_t bs = (uint32_t)pd.delta_mbc * pd.delta_mbvc;
            b->delta_pages.push_back(p);
            b->dblk_base[p] = b->dblk_total;
            b->dblk_total += ((uint64_t)ns_p + bs - 1) / bs + 1;
            tiles(WI_DELTA_TILE, kDeltaTileVals);
          }
          break;
        case VK_PLAIN_BA:
          if (ns_p) {  // plainba.hip: 256-byte segments of the values section
            const uint32_t li = (uint32_t)b->pba_pages.size();
            b->pba_pages.push_back(p);
            b->pba_seg0.push_back((uint32_t)b->pba_seg_page.size());
            const uint32_t nseg = std::max<uint32_t>(1, (pd.val_len + kPbaSegHost - 1) / kPbaSegHost);
            b->pba_seg_page.insert(b->pba_seg_page.end(), nseg, li);
          }
          break;
        case VK_DLBA: case VK_DBA: {
          BaDelta &bd = b->ba_delta[pd.ba_delta];
          bd.cap = (uint32_t)std::min<int64_t>(std::max(bd.st[0].count, 0), (int64_t)ns_p);
          b->ba_delta_scratch[pd.ba_delta] = take((uint64_t)bd.cap * 16);  // suffix, prefix, offset, ancestor
          if (bd.cap) {
            b->items.push_back(WorkItem{p, 0, bd.cap, WI_DLENS, {0, 0, 0}});
            if (pd.vkind == VK_DBA) b->items.push_back(WorkItem{p, 1, bd.cap, WI_DLENS, {0, 0, 0}});
          }
          break;
        }
      }
    }
  }
  // fill tiles: the nested chunks' tiles (k_nest_count / k_nest_emit, nested.hip) grouped by the
  // chunks' list levels so that each k_nest_emit<R> launch covers one group, a chunk's tiles
  // contiguous and in slot order; the other chunks' tiles go to k_level_fill
  for (uint32_t t = 0; t < (uint32_t)b->lv_tiles.size(); t++)
    if (!b->chunks[b->pages[b->lv_tiles[t]].chunk].nest) b->lf_list.push_back(t);
  for (uint32_t r = 0; r <= PQGPU_MAX_NEST + 1; r++) b->nest_first[r] = 0;
  for (uint32_t r = 1; r <= PQGPU_MAX_NEST; r++) {
    b->nest_first[r] = (uint32_t)b->nest_tiles.size();
    for (uint32_t c : b->nest_chunks) {
      HostChunk &hc = b->chunks[c];
      if (hc.nest != r) continue;
      hc.nest_tile0 = (uint32_t)b->nest_tiles.size();
      for (uint32_t p = hc.first_page; p < hc.first_page + hc.num_pages; p++) {
        const uint64_t sb = b->pages[p].slot_base, ns = b->pages[p].num_slots;
        const uint64_t nt = ns ? (sb + ns - 1) / kLfTileHost - sb / kLfTileHost + 1 : 0;
        for (uint64_t k = 0; k < nt; k++) b->nest_tiles.push_back(make_uint4(b->lv_tile0[p] + (uint32_t)k, p, (uint32_t)k, c));
      }
      hc.nest_ntiles = (uint32_t)b->nest_tiles.size() - hc.nest_tile0;
    }
  }
  b->nest_first[PQGPU_MAX_NEST + 1] = (uint32_t)b->nest_tiles.size();
  b->nest_order.clear();
  for (uint32_t r = 1; r <= PQGPU_MAX_NEST; r++) {
    std::vector<uint32_t> cs;
    uint32_t most = 0;
    for (uint32_t c : b->nest_chunks)
      if (b->chunks[c].nest == r && b->chunks[c].nest_ntiles) {
        cs.push_back(c);
        most = std::max(most, b->chunks[c].nest_ntiles);
      }
    for (uint32_t k = 0; k < most; k++)
      for (uint32_t c : cs)
        if (k < b->chunks[c].nest_ntiles) b->nest_order.push_back(b->chunks[c].nest_tile0 + k);
  }
  // chunks with tiles are scanned by their last k_nest_count tile; the others by k_nest_scan
  std::stable_partition(b->nest_chunks.begin(), b->nest_chunks.end(), [&](uint32_t c) { return b->chunks[c].nest_ntiles == 0; });
  b->n_nest_empty = 0;
  for (uint32_t c : b->nest_chunks) b->n_nest_empty += b->chunks[c].nest_ntiles == 0;
  // k_ba_emit block order: class 0 / 1 = chunks whose pages are all dictionary pages with a
  // slot table of 16/32-byte / 64-byte slots, class 2 = the rest. Within a class, chunk c's
  // tiles (in order) go to queue c mod 8 and block b takes tile b / 8 of queue b mod 8: blocks
  // are dispatched round-robin over the 8 XCDs, so the chunk's dictionary, slot table and index
  // streams stay in one XCD's L2, and a tile's predecessors have lower block indices.
  b->n_ba_class[0] = b->n_ba_class[1] = b->n_ba_class[2] = b->n_ba_class[3] = 0;
  b->ba_presum = false;
  if (!b->ba_tile_page.empty()) {
    std::vector<std::vector<uint32_t>> q(32);
    std::vector<int8_t> cls(nc, -1);
    for (uint32_t c : b->ba_chunks) {
      const HostChunk &hc = b->chunks[c];
      bool slot_only = hc.slot_shift != 0 && !hc.ba_sync;
      for (uint32_t p = hc.first_page; p < hc.first_page + hc.num_pages; p++) slot_only &= b->pages[p].vkind == VK_DICT;
      cls[c] = ba_lds_class(b, hc) ? 3 : slot_only ? (hc.slot_shift <= 5 ? 0 : 1) : 2;
      assert((cls[c] == 3) == (hc.ba_tile_vals == kBaTileLds) && (cls[c] != 3 || (slot_only && hc.slot_shift <= 5)));
    }
    for (uint32_t c : b->ba_chunks) {
      HostChunk &hc = b->chunks[c];
      hc.ba_class = cls[c];
      // default: the pre-pass when nested arrays are emitted beside the byte-array path (k_nest_emit on
      // the DELTA stream, or k_nest_tile on the aux stream with k_nest_pcount), else the look-back
      const bool nest_beside = !b->one_stream && !b->nest_chunks.empty() && (!b->nest_fused || b->nest_pcount);
      const int mode = b->ba_presum_mode >= 0 ? b->ba_presum_mode : nest_beside ? 1 : 0;
      hc.ba_presum = !hc.ba_sync && (mode == 1 || (mode == 2 && cls[c] == 3));
      b->ba_presum |= hc.ba_presum;
    }
    // A class with fewer than 8 chunks would leave XCDs idle: chunk k of the class (in chunk order)
    // then gets 8 / n queues and its tiles go round-robin over them, still in block order (tile j
    // of the chunk at a lower block index than tile j + 1), so the look-back is unchanged.
    uint32_t ncls[4] = {0, 0, 0, 0};
    std::vector<uint32_t> qbase(nc, 0), qn(nc, 1), seen(nc, 0);
    for (uint32_t c : b->ba_chunks) qbase[c] = ncls[cls[c]]++;
    for (uint32_t c : b->ba_chunks) {
      const uint32_t n = ncls[cls[c]];
      if (n < 8) {
        qn[c] = 8 / n;
        qbase[c] = qbase[c] * qn[c];
      } else {
        qbase[c] = c % 8;
      }
    }
    for (uint32_t t = 0; t < (uint32_t)b->ba_tile_page.size(); t++) {
      const uint32_t c = b->pages[b->ba_tile_page[t]].chunk;
      q[8 * cls[c] + qbase[c] + seen[c]++ % qn[c]].push_back(t);
    }
    for (uint32_t k = 0; k < 4; k++) {
      size_t m = 0;
      for (uint32_t x = 0; x < 8; x++) m = std::max(m, q[8 * k + x].size());
      b->ba_class_off[k] = (uint32_t)b->ba_tile_order.size();
      b->n_ba_class[k] = (uint32_t)(8 * m);
      b->ba_tile_order.resize(b->ba_tile_order.size() + 8 * m, ~0u);
      for (uint32_t x = 0; x < 8; x++)
        for (size_t i = 0; i < q[8 * k + x].size(); i++) b->ba_tile_order[b->ba_class_off[k] + 8 * i + x] = q[8 * k + x][i];
    }
  }
  // Speculative mode: every page's non-null count is known from its header (or it has no
  // definition levels), so the values kernels need not wait for k_levels.
  b->spec = !b->force_serial && (!b->level_pages.empty() || !b->level_pages_bw1.empty());
  b->page_nn_spec.assign(np, 0);
  b->page_vbase_spec.assign(np, 0);
  for (uint32_t c = 0; c < nc && b->spec; c++) {
    HostChunk &hc = b->chunks[c];
    if (hc.err.code) continue;
    uint64_t base = 0;
    for (uint32_t p = hc.first_page; p < hc.first_page + hc.num_pages; p++) {
      const PageDesc &pd = b->pages[p];
      uint32_t nn;
      if (hc.col.max_def == 0 && hc.col.max_rep == 0) nn = pd.num_slots;
      else if (pd.flags & PF_BASE_KNOWN) nn = pd.expect_nn;
      else { b->spec = false; break; }
      b->page_nn_spec[p] = nn;
      b->page_vbase_spec[p] = base;
      base += nn;
    }
  }
  // A batch of flat REQUIRED chunks only (no level stream anywhere): a page's values are its slots,
  // so every value base is known now; they are uploaded with the descriptors and k_bases is not
  // launched (cfg1: 6 us of a 38 us step).
  b->bases_known = !b->spec && b->level_pages.empty() && b->level_pages_bw1.empty() && b->lv_tiles.empty() &&
                   b->rec_pages.empty() && b->nest_chunks.empty();
  for (uint32_t c = 0; c < nc && b->bases_known; c++) {
    const HostChunk &hc = b->chunks[c];
    if (!hc.err.code && (hc.col.max_def != 0 || hc.col.max_rep != 0)) b->bases_known = false;
  }
  if (b->bases_known) {
    for (uint32_t c = 0; c < nc; c++) {
      const HostChunk &hc = b->chunks[c];
      uint64_t base = 0;
      for (uint32_t p = hc.first_page; p < hc.first_page + hc.num_pages; p++) {
        b->page_nn_spec[p] = b->pages[p].num_slots;
        b->page_vbase_spec[p] = base;
        base += b->pages[p].num_slots;
      }
    }
    b->base_chunks.clear();
  }
  // Region set to 0xff before every decode: chunk error keys (the batch stream's two buffers first,
  // the level stream's last), dictionary tile table and descriptors.
  b->o_err = take((uint64_t)nc * 8);
  b->f_begin = b->o_err;
  b->o_err2 = take((uint64_t)nc * 8);
  b->o_tile_first = take(b->tile_total * 4);
  b->o_tile_desc = take(b->tile_total * 32);  // (filled too: a descriptor k_scan_runs did not write reads invalid)
  b->o_err_ds = take((uint64_t)nc * 8);
  b->f_end = a;
  b->ds_synced = false;
  b->err_sel = 0;
  b->err_ready[0] = b->err_ready[1] = false;
  b->bm_zeroed = false;
  // DELTA tiles first (k_delta_sums runs over exactly that prefix), then the scalar DELTA
  // pages (long-running), then the LDS-staged tiles, then the PLAIN / BOOLEAN copies (in the same
  // grid when fused, else their own zero-LDS launch, k_values_copy, on the copy stream)
  // column-group pipeline: only for batches whose pages are all flat REQUIRED (no level streams,
  // no byte-array or nested outputs: every value base is known at upload, k_bases can run before
  // the first SNAPPY launch) with device SNAPPY pages and no DELTA tiles; its copies are fused
  const char *cf = getenv("PQ_COPY_FUSED");
  b->n_groups = 0;
  {
    const char *ge = getenv("PQ_SNAPPY_GROUPS");
    const int want = ge ? atoi(ge) : 1;  // (default: off until measured)
    bool ok = want > 1 && !b->snappy.empty() && (!cf || atoi(cf) != 0) && b->level_pages.empty() &&
              b->level_pages_bw1.empty() && b->ba_chunks.empty() && nc >= 2;
    for (const auto &hc : b->chunks) ok = ok && hc.col.max_rep == 0 && hc.col.max_def == 0 && !hc.nest;
    for (const auto &it : b->items) ok = ok && it.kind != WI_DELTA_TILE && it.kind != WI_DLENS;
    if (ok) b->n_groups = (uint32_t)std::min<int>(std::min<int>(want, pqgpu_batch::kMaxGroups), (int)nc);
  }
  b->copy_fused = cf ? atoi(cf) != 0 : (b->spec || b->n_groups > 0);
  const bool fused = b->copy_fused;
  // Dictionary tiles of 4-byte values whose dictionary is staged with the tile (kernels.hip
  // do_dict2) go up to kDictGroupHost to a workgroup when the batch has many (dict_tile_loadn: one tile-load
  // latency chain per group), as many as fit the stage beside the dictionary: 12 KiB of index
  // stream, 24 / bw tiles. PQ_DICT_PAIR=<n>: group from n tiles on (0: never). Not with column
  // groups (their dictionary launches are per group).
  {
    const char *pe = getenv("PQ_DICT_PAIR");
    const size_t min_tiles = pe ? (size_t)atoll(pe) : 8192;
    const char *gm = getenv("PQ_DICT_GROUP");  // (comparison runs: at most this many tiles per item)
    const uint32_t gmax = gm && atoi(gm) > 0 ? std::min<uint32_t>((uint32_t)atoi(gm), kDictGroupHost) : kDictGroupHost;
    size_t nd = 0;
    for (const auto &it : b->items) nd += it.kind == WI_DICT;
    if (min_tiles && nd >= min_tiles && b->n_groups == 0) {
      std::vector<WorkItem> out;
      out.reserve(b->items.size());
      for (size_t i = 0; i < b->items.size(); i++) {
        WorkItem it = b->items[i];
        const PageDesc &pd = b->pages[it.page];
        const HostChunk &hc = b->chunks[pd.chunk];
        const bool small = it.kind == WI_DICT && dict2_eligible(pd.vkind, hc.value_width, hc.dict_count);
        const uint32_t g = small ? std::min<uint32_t>(gmax, pd.dict_bw ? 24u / pd.dict_bw : gmax) : 1;
        for (uint32_t k = 1; k < g && i + 1 < b->items.size(); k++) {
          const WorkItem &nx = b->items[i + 1];
          if (nx.kind != WI_DICT || nx.page != it.page || nx.v0 != it.v1) break;  // the page's next tile
          it.v1 = nx.v1;
          it.kind = WI_DICT2;
          i++;
        }
        out.push_back(it);
      }
      b->items.swap(out);
    }
  }
  // ranks: DELTA tiles, DELTA pages, fused PLAIN / BOOLEAN copies (these three are k_values_delta's
  // launch: latency-bound pages first, the bandwidth-bound copies fill the CUs around them), the
  // dictionary tiles (k_values_dict), the other LDS-staged kinds (k_values), unfused copies
  // (k_values_copy)
  auto rank = [fused](uint8_t k) {
    const bool copy = k == WI_PLAIN || k == WI_BOOL;
    return k == WI_DELTA_TILE ? 0 : (k == WI_DELTA || k == WI_DELTA_PAGE) ? 1 : copy ? (fused ? 2 : 5) : (k == WI_DICT || k == WI_DICT2) ? 3 : 4;
  };
  const uint32_t G = b->n_groups;
  auto grp = [&](uint32_t page) { return G ? b->pages[page].chunk * G / nc : 0u; };
  std::stable_sort(b->items.begin(), b->items.end(), [&](const WorkItem &x, const WorkItem &y) {
    const uint32_t gx = grp(x.page), gy = grp(y.page);
    if (gx != gy) return gx < gy;
    if (rank(x.kind) != rank(y.kind)) return rank(x.kind) < rank(y.kind);
    return x.kind == WI_DICT2 && y.kind != WI_DICT2;  // k_values_dict2's items first
  });
  b->n_delta_items = 0;
  b->n_dict_items = 0;
  b->n_dict2_items = 0;
  b->n_delta_tiles = 0;
  b->n_copy_items = 0;
  for (auto &it : b->items) {
    b->n_delta_items += rank(it.kind) <= 2;  // k_values_delta's launch
    b->n_dict_items += rank(it.kind) == 3;   // k_values_dict's launch (k_values_dict2's first)
    b->n_dict2_items += it.kind == WI_DICT2;
    b->n_delta_tiles += it.kind == WI_DELTA_TILE;
    b->n_copy_items += rank(it.kind) == 5;
  }
  b->copies_early = false;
  b->chunk_nn_spec.assign(nc, 0);
  if (!b->spec && !b->bases_known && !b->force_serial && !fused && b->n_copy_items && !b->one_stream &&
      !(getenv("PQ_COPY_EARLY") && atoi(getenv("PQ_COPY_EARLY")) == 0)) {
    bool ok = true;
    for (size_t i = b->items.size() - b->n_copy_items; i < b->items.size() && ok; i++) {
      const uint32_t c = b->pages[b->items[i].page].chunk;
      if (b->chunk_nn_spec[c]) continue;
      const HostChunk &hc = b->chunks[c];
      const int w = hc.value_width;
      ok = !hc.err.code && w > 0;
      uint64_t base = 0;
      for (uint32_t p = hc.first_page; p < hc.first_page + hc.num_pages && ok; p++) {
        const PageDesc &pd = b->pages[p];
        ok = (pd.vkind == VK_PLAIN_FIXED || pd.vkind == VK_PLAIN_INT96) && pd.val_len % (uint64_t)w == 0 &&
             pd.val_len / (uint64_t)w <= pd.num_slots;
        b->page_nn_spec[p] = ok ? (uint32_t)(pd.val_len / (uint64_t)w) : 0u;
        b->page_vbase_spec[p] = base;
        base += b->page_nn_spec[p];
      }
      b->chunk_nn_spec[c] = 1;
    }
    b->copies_early = ok;
    if (!ok) b->chunk_nn_spec.assign(nc, 0);
  }
  if (G) {
    for (uint32_t g = 0; g <= G; g++) b->grp_job[g] = b->grp_scan[g] = b->grp_item[g] = 0;
    for (uint32_t g = 0; g < G; g++) b->grp_delta[g] = b->grp_dict[g] = 0;
    // jobs, scan pages and items are in chunk order: group g's ranges are contiguous
    for (uint32_t j = 0; j < (uint32_t)b->snappy.size(); j++) b->grp_job[b->pages[b->snappy[j].page].chunk * G / nc + 1]++;
    for (uint32_t p : b->scan_pages) b->grp_scan[grp(p) + 1]++;
    for (auto &it : b->items) {
      b->grp_item[grp(it.page) + 1]++;
      b->grp_delta[grp(it.page)] += rank(it.kind) <= 2;
      b->grp_dict[grp(it.page)] += rank(it.kind) == 3;
    }
    for (uint32_t g = 0; g < G; g++) {
      b->grp_job[g + 1] += b->grp_job[g];
      b->grp_scan[g + 1] += b->grp_scan[g];
      b->grp_item[g + 1] += b->grp_item[g];
    }
  }
  // batch-level arrays
  b->o_pages = take((uint64_t)np * sizeof(PageDesc));
  b->o_chunks = take((uint64_t)nc * sizeof(ChunkDesc));
  b->o_nn = take((uint64_t)np * 4);
  b->o_nnv = take((uint64_t)np * 4);
  b->o_vbase = take((uint64_t)np * 8);
  b->o_rbase = take((uint64_t)np * 8);
  b->o_runs = take(b->run_total * sizeof(HybRun));
  b->o_lv_runs = take(b->lv_run_total * 8);
  b->o_lv_run_base = take((uint64_t)np * 16);
  b->o_lv_meta = take((uint64_t)np * 16);
  b->o_lv_tile_run = take((uint64_t)b->lv_tiles.size() * 8);
  b->o_lv_tile0 = take((uint64_t)np * 4);
  b->l_lv_tiles = take((uint64_t)b->lv_tiles.size() * 4);
  b->l_lf_list = take((uint64_t)b->lf_list.size() * 4);
  b->o_run_base = take((uint64_t)np * 8);
  b->o_tile_base = take((uint64_t)np * 8);
  b->o_items = take(b->items.size() * sizeof(WorkItem));
  b->o_ba_tile_sum = take(b->ba_tile_page.size() * 8);
  b->o_ba_tile_page = take(b->ba_tile_page.size() * 4);
  b->o_ba_tile_order = take(b->ba_tile_order.size() * 4);
  b->l_slot = take(b->slot_chunks.size() * 4);
  b->o_ba_totals = take((uint64_t)nc * 8);
  b->o_dbg = take(64 * 8);
  b->o_ba_delta = take(b->ba_delta.size() * sizeof(BaDelta));
  b->o_snappy = take(b->snappy.size() * sizeof(SnappyJob));
  b->o_gather = take(b->gathers.size() * sizeof(GatherJob));
  b->pba_seg0.push_back((uint32_t)b->pba_seg_page.size());  // [n_pages + 1]
  b->l_pba_pages = take(b->pba_pages.size() * 4);
  b->l_pba_seg0 = take(b->pba_seg0.size() * 4);
  b->l_pba_seg_page = take(b->pba_seg_page.size() * 4);
  b->o_pba_segs = take(b->pba_seg_page.size() * 16);
  b->o_pba_limit = take(b->pba_pages.size() * 4);
  b->o_dblk = take(b->dblk_total * sizeof(DeltaBlk));
  b->o_dblk_sum = take(b->dblk_total * 8);
  b->o_dblk_base = take((uint64_t)np * 8);
  b->o_dblk_n = take((uint64_t)np * 4);
  b->l_delta = take(b->delta_pages.size() * 4);
  b->l_level = take(b->level_pages.size() * 4);
  {  // k_levels_seg takes the pages whose definition stream fits its LDS stage (+ 16 B alignment slack)
    const char *lsg = getenv("PQ_LV_SEG");
    const bool seg = !(lsg && atoi(lsg) == 0);
    auto fits = [&](uint32_t p) { return seg && (uint64_t)b->pages[p].def_len + 24 <= kSgStageHost; };
    std::stable_partition(b->level_pages_bw1.begin(), b->level_pages_bw1.end(), fits);
    b->n_level_seg = 0;
    for (uint32_t p : b->level_pages_bw1) b->n_level_seg += fits(p);
  }
  {  // generic level streams: k_levels_segw (segment speculation) takes the definition streams that
     // fit its LDS stage (PQ_LV_SEGW=2, the default: Arrow's definition streams alternate 2-byte RLE
     // runs with short literal runs, cfg4 k_levels 0.377 -> 0.269 ms); the repetition streams are
     // maximal literal runs (64 B at bit width 1), which k_levels' stride prelude walks 64 at a time
     // and on which segment speculation fails (PQ_LV_SEGW=1, every stream: 1.01 ms). 0: none.
    const char *lsg = getenv("PQ_LV_SEGW");
    const int segm = lsg ? atoi(lsg) : 2;
    auto fits = [&](uint32_t u) {
      const PageDesc &pd = b->pages[u >> 1];
      return (segm == 1 || (segm == 2 && (u & 1))) && (uint64_t)((u & 1) ? pd.def_len : pd.rep_len) + 24 <= kSgwStageHost;
    };
    std::stable_partition(b->level_pages.begin(), b->level_pages.end(), fits);
    b->n_level_units_seg = 0;
    for (uint32_t u : b->level_pages) b->n_level_units_seg += fits(u);
    // then the repetition streams for k_levels_hyb (PQ_LV_HYB=0: the list ranking of k_levels)
    const char *lh = getenv("PQ_LV_HYB");
    const bool hyb = !(lh && atoi(lh) == 0);
    auto is_hyb = [&](uint32_t u) { return hyb && !(u & 1); };
    std::stable_partition(b->level_pages.begin() + b->n_level_units_seg, b->level_pages.end(), is_hyb);
    b->n_level_units_hyb = 0;
    for (size_t k = b->n_level_units_seg; k < b->level_pages.size(); k++) b->n_level_units_hyb += is_hyb(b->level_pages[k]);
  }
  b->l_level_bw1 = take(b->level_pages_bw1.size() * 4);
  b->l_scan = take(b->scan_pages.size() * 4);
  b->l_base = take(b->base_chunks.size() * 4);
  b->l_ba = take(b->ba_chunks.size() * 4);
  b->l_rec = take(b->rec_pages.size() * 4);
  b->l_pc = take(b->pc_pages.size() * 4);
  b->l_nest_tiles = take(b->nest_tiles.size() * 16);
  b->l_nest_order = take(b->nest_order.size() * 4);
  b->l_nest_chunks = take(b->nest_chunks.size() * 4);
  b->l_grp_tiles = take(b->grp_tiles.size() * 4);
  b->o_nest_cnt = take((uint64_t)b->nest_tiles.size() * 2 * kNestCnt * 4);  // every entry written by k_nest_count
  b->o_nest_base = take((uint64_t)b->nest_tiles.size() * 2 * kNestCnt * 8);
  for (uint32_t c : b->nest_chunks) {  // the slots' flag masks (written by k_nest_count; two-pass mode only)
    HostChunk &hc = b->chunks[c];
    hc.nest_nmask = 2 * (hc.nest + 1) + hc.ngroups;
    hc.o_nest_mask = b->nest_fused ? 0 : take((uint64_t)hc.nest_ntiles * hc.nest_nmask * 1024);
  }
  b->o_nest_tot = take((uint64_t)nc * kNestCnt * 8);
  b->arena_size = a;
  if (a > b->d_arena_cap) {
    if (b->d_arena) (void)hipFree(b->d_arena);
    b->d_arena = nullptr;
    b->d_arena_cap = 0;
    HIPCHECK(hipMalloc(&b->d_arena, a), err);
    b->d_arena_cap = a;
  }
  if (payload_arena > b->d_payload_cap) {
    if (b->d_payload) (void)hipFree(b->d_payload);
    b->d_payload = nullptr;
    b->d_payload_cap = 0;
    HIPCHECK(hipMalloc(&b->d_payload, payload_arena), err);
    b->d_payload_cap = payload_arena;
  }
  // stage: pinned host copy + device buffer (64 B zero pad); after it, the pages k_snappy
  // writes (each 256-B aligned, followed by 64 zero bytes like every staged section)
  size_t ssz = align_up(b->stage.size(), 16) + 64;
  const uint64_t dec_base = align_up(ssz, 256);
  std::vector<uint64_t> dec_off(b->snappy.size());
  uint64_t dec = 0;
  for (size_t k = 0; k < b->snappy.size(); k++) {
    dec_off[k] = dec;
    if (!b->snappy[k].to_values)  // direct pages need no region of their own
      dec = align_up(dec + align_up((uint64_t)b->snappy[k].raw_len + b->snappy[k].dlen, 16) + 64, 256);
  }
  // then the resident UNCOMPRESSED pages k_page_gather copies in (same layout)
  const uint64_t gat_base = align_up(dec_base + dec, 256);
  std::vector<uint64_t> gat_off(b->gathers.size());
  uint64_t gat = 0;
  for (size_t k = 0; k < b->gathers.size(); k++) {
    gat_off[k] = gat;
    gat = align_up(gat + align_up(b->gathers[k].len, 16) + 64, 256);
  }
  const size_t dsz = (size_t)(gat_base + gat);
  if (dsz > b->d_stage_cap) {
    if (b->d_stage) (void)hipFree(b->d_stage);
    b->d_stage = nullptr;
    b->d_stage_cap = 0;
    HIPCHECK(hipMalloc(&b->d_stage, dsz), err);
    b->d_stage_cap = dsz;
  }
  {
    // the stage is pinned host memory: the H2D copy reads it directly (64 zero bytes after it)
    const size_t used = b->stage.size();
    b->stage.resize(ssz, 0);
    memset(b->stage.data() + used, 0, ssz - used);
    b->stage.resize(used);
    HIPCHECK(hipMemcpyAsync(b->d_stage, b->stage.data(), ssz, hipMemcpyHostToDevice, s), err);
    b->last_stream = s;
  }

  uint8_t *A = b->d_arena;
  auto dp = [&](uint64_t o) { return (uint64_t)(A + o); };
  // chunk descriptors
  b->chunk_desc.assign(nc, ChunkDesc{});
  for (uint32_t c = 0; c < nc; c++) {
    HostChunk &hc = b->chunks[c];
    ChunkDesc &cd = b->chunk_desc[c];
    memset(&cd, 0, sizeof(cd));
    cd.type = hc.col.physical_type;
    cd.type_length = hc.col.type_length;
    cd.max_def = hc.col.max_def;
    cd.max_rep = hc.col.max_rep;
    cd.def_bw = bits_len16(hc.col.max_def);
    cd.rep_bw = bits_len16(hc.col.max_rep);
    cd.value_width = hc.value_width;
    cd.first_page = hc.first_page;
    cd.num_pages = hc.num_pages;
    cd.num_slots = hc.num_slots;
    cd.nn_capacity = hc.num_slots;
    if (hc.err.code) { cd.flags |= CF_FAILED; continue; }
    if (b->copies_early && b->chunk_nn_spec[c]) cd.flags |= CF_NN_SPEC;
    if (hc.has_dict) {
      cd.flags |= CF_DICT;
      cd.dict_raw = (uint64_t)(b->d_stage + hc.dict_off);
      cd.dict_raw_len = hc.dict_len;
      cd.dict_count = hc.dict_count;
      cd.dict_values = cd.dict_raw;
      cd.dict_offsets = hc.dict_ent.empty() ? 0 : (uint64_t)(b->d_stage + hc.dict_ent_off);
      cd.dict_max_len = hc.dict_max_len;
      cd.slot_shift = hc.slot_shift;
      cd.dict_slots = hc.o_slots ? dp(hc.o_slots) : 0;
    }
    if (hc.value_width == 0) {
      const PageDesc *fp = hc.num_pages ? &b->pages[hc.first_page] : nullptr;
      cd.ba_tile0 = fp ? fp->ba_tile : 0;
      cd.ba_ntiles = 0;
      for (uint32_t p = hc.first_page; p < hc.first_page + hc.num_pages; p++)
        cd.ba_ntiles += (b->pages[p].num_slots + hc.ba_tile_vals - 1) / hc.ba_tile_vals;
      if (hc.ba_presum) cd.flags |= CF_BA_PRESUM;
      if (hc.ba_tile_vals == kBaTileLds) cd.flags |= CF_BA_TILE4K;
      if (hc.ba_sync) {
        cd.flags |= CF_BA_SYNC;
        cd.payload = hc.payload ? (uint64_t)hc.payload : 0;  // (re)sized after the scan of each decode
      } else {
        if (hc.payload_own && hc.payload) (void)hipFree(hc.payload);
        hc.payload_own = false;
        hc.payload = b->d_payload + hc.payload_off;
        cd.payload = (uint64_t)hc.payload;
        cd.payload_capacity = hc.payload_bound;
      }
    }
    cd.values = hc.o_values ? dp(hc.o_values) : 0;
    cd.def_levels = hc.o_def ? dp(hc.o_def) : 0;
    cd.rep_levels = hc.o_rep ? dp(hc.o_rep) : 0;
    cd.validity = hc.o_valid ? dp(hc.o_valid) : 0;
    cd.list_offsets = hc.o_lists ? dp(hc.o_lists) : 0;
    cd.nest = hc.nest;
    cd.nest_tile0 = hc.nest_tile0;
    cd.nest_ntiles = hc.nest_ntiles;
    cd.nest_nmask = hc.nest ? hc.nest_nmask : 0u;
    cd.nest_masks = hc.nest && hc.o_nest_mask ? dp(hc.o_nest_mask) : 0;
    for (uint32_t k = 0; k < PQGPU_MAX_NEST; k++) {
      cd.list_def[k] = (uint8_t)(k < hc.nest ? hc.col.list_def[k] : 0);
      cd.list_null_def[k] = (uint8_t)(k < hc.nest ? hc.col.list_null_def[k] : 0);
      cd.lvl_offsets[k] = hc.o_lvl_off[k] ? dp(hc.o_lvl_off[k]) : 0;
      cd.lvl_validity[k] = hc.o_lvl_valid[k] ? dp(hc.o_lvl_valid[k]) : 0;
    }
    cd.elem_validity = hc.o_elem_valid ? dp(hc.o_elem_valid) : 0;
    cd.ngroups = hc.ngroups;
    cd.grp_tile0 = hc.grp_tile0;
    for (uint32_t g = 0; g < PQGPU_MAX_NEST; g++) {
      cd.group_def[g] = (uint8_t)(g < hc.ngroups ? hc.col.group_def[g] : 0);
      cd.group_depth[g] = (uint8_t)(g < hc.ngroups ? hc.col.group_depth[g] : 0);
      cd.group_validity[g] = hc.o_grp_valid[g] ? dp(hc.o_grp_valid[g]) : 0;  // 0: aliased, not written
    }
    cd.offsets = hc.o_offsets ? dp(hc.o_offsets) : 0;
    cd.ba_index = hc.o_ba_index ? dp(hc.o_ba_index) : 0;
  }
  std::vector<GatherJob> gjobs(b->gathers.size());
  for (size_t k = 0; k < gjobs.size(); k++)
    gjobs[k] = GatherJob{b->gathers[k].src, (uint64_t)(b->d_stage + gat_base + gat_off[k]), b->gathers[k].len};
  std::vector<SnappyJob> jobs(b->snappy.size());
  for (size_t k = 0; k < jobs.size(); k++) {
    const pqgpu_batch::DevSnappy &j = b->snappy[k];
    const PageDesc &pd = b->pages[j.page];
    const uint64_t comp = j.comp_gather >= 0 ? gjobs[(size_t)j.comp_gather].dst : (uint64_t)(b->d_stage + j.comp_off);
    jobs[k] = SnappyJob{comp + j.vlen, (uint64_t)(b->d_stage + j.raw_off), (uint64_t)(b->d_stage + dec_base + dec_off[k]),
                        j.comp_len - j.vlen, j.raw_len, j.dlen, pd.chunk, pd.page_in_chunk, 0};
    if (j.to_values) {  // straight into the values array at the page's first value (REQUIRED: slot base)
      const HostChunk &hc = b->chunks[pd.chunk];
      jobs[k].dst = (uint64_t)(b->d_arena + hc.o_values) + pd.slot_base * (uint64_t)hc.value_width;
      jobs[k].lead = 1 + (uint32_t)(jobs[k].dst & 15);
    }
  }
  std::vector<PageDesc> pages = b->pages;
  for (auto &pd : pages)
    pd.data = (pd.flags & PF_DEV_SNAPPY)   ? jobs[pd.data].dst
              : (pd.flags & PF_DEV_GATHER) ? gjobs[pd.data].dst
                                           : (uint64_t)(b->d_stage + pd.data);
  HIPCHECK(hipMemcpyAsync(A + b->o_snappy, jobs.data(), jobs.size() * sizeof(SnappyJob), hipMemcpyHostToDevice, s), err);
  if (!gjobs.empty()) {
    HIPCHECK(hipMemcpyAsync(A + b->o_gather, gjobs.data(), gjobs.size() * sizeof(GatherJob), hipMemcpyHostToDevice, s),
             err);
    HIPCHECK(launch_page_gather((const GatherJob *)(A + b->o_gather), (uint32_t)gjobs.size(), s), err);
  }
  auto up = [&](uint64_t o, const void *src, size_t n) -> hipError_t {
    if (!n) return hipSuccess;
    return hipMemcpyAsync(A + o, src, n, hipMemcpyHostToDevice, s);
  };
  HIPCHECK(up(b->o_pages, pages.data(), pages.size() * sizeof(PageDesc)), err);
  std::vector<BaDelta> bad = b->ba_delta;
  for (size_t k = 0; k < bad.size(); k++) bad[k].scratch = (uint64_t)(A + b->ba_delta_scratch[k]);
  HIPCHECK(up(b->o_ba_delta, bad.data(), bad.size() * sizeof(BaDelta)), err);
  HIPCHECK(up(b->o_chunks, b->chunk_desc.data(), b->chunk_desc.size() * sizeof(ChunkDesc)), err);
  HIPCHECK(up(b->o_run_base, b->run_base.data(), np * 8), err);
  HIPCHECK(up(b->o_nn, b->page_nn_init.data(), np * 4), err);
  if (b->spec || b->bases_known || b->copies_early) {  // (copies_early: only its chunks' entries are used)
    HIPCHECK(up(b->o_nnv, b->page_nn_spec.data(), np * 4), err);
    HIPCHECK(up(b->o_vbase, b->page_vbase_spec.data(), np * 8), err);
  }
  if (b->bases_known) HIPCHECK(hipMemsetAsync(A + b->o_rbase, 0, (size_t)np * 8, s), err);  // no records
  HIPCHECK(hipMemsetAsync(A + b->o_dbg, 0, 64 * 8, s), err);
  HIPCHECK(up(b->o_tile_base, b->tile_base.data(), np * 8), err);
  HIPCHECK(up(b->o_items, b->items.data(), b->items.size() * sizeof(WorkItem)), err);
  HIPCHECK(up(b->o_ba_tile_page, b->ba_tile_page.data(), b->ba_tile_page.size() * 4), err);
  HIPCHECK(up(b->o_ba_tile_order, b->ba_tile_order.data(), b->ba_tile_order.size() * 4), err);
  HIPCHECK(up(b->l_slot, b->slot_chunks.data(), b->slot_chunks.size() * 4), err);
  HIPCHECK(up(b->l_level, b->level_pages.data(), b->level_pages.size() * 4), err);
  HIPCHECK(up(b->l_level_bw1, b->level_pages_bw1.data(), b->level_pages_bw1.size() * 4), err);
  HIPCHECK(up(b->o_lv_run_base, b->lv_run_base.data(), b->lv_run_base.size() * 8), err);
  HIPCHECK(up(b->o_lv_tile0, b->lv_tile0.data(), b->lv_tile0.size() * 4), err);
  HIPCHECK(up(b->l_lv_tiles, b->lv_tiles.data(), b->lv_tiles.size() * 4), err);
  HIPCHECK(up(b->l_lf_list, b->lf_list.data(), b->lf_list.size() * 4), err);
  HIPCHECK(up(b->l_scan, b->scan_pages.data(), b->scan_pages.size() * 4), err);
  HIPCHECK(up(b->l_base, b->base_chunks.data(), b->base_chunks.size() * 4), err);
  HIPCHECK(up(b->l_ba, b->ba_chunks.data(), b->ba_chunks.size() * 4), err);
  HIPCHECK(up(b->l_rec, b->rec_pages.data(), b->rec_pages.size() * 4), err);
  HIPCHECK(up(b->l_pc, b->pc_pages.data(), b->pc_pages.size() * 4), err);
  HIPCHECK(up(b->l_nest_tiles, b->nest_tiles.data(), b->nest_tiles.size() * 16), err);
  HIPCHECK(up(b->l_nest_order, b->nest_order.data(), b->nest_order.size() * 4), err);
  HIPCHECK(up(b->l_nest_chunks, b->nest_chunks.data(), b->nest_chunks.size() * 4), err);
  HIPCHECK(up(b->l_grp_tiles, b->grp_tiles.data(), b->grp_tiles.size() * 4), err);
  HIPCHECK(up(b->o_dblk_base, b->dblk_base.data(), np * 8), err);
  HIPCHECK(up(b->l_delta, b->delta_pages.data(), b->delta_pages.size() * 4), err);
  HIPCHECK(up(b->l_pba_pages, b->pba_pages.data(), b->pba_pages.size() * 4), err);
  HIPCHECK(up(b->l_pba_seg0, b->pba_seg0.data(), b->pba_seg0.size() * 4), err);
  HIPCHECK(up(b->l_pba_seg_page, b->pba_seg_page.data(), b->pba_seg_page.size() * 4), err);
  // the host copies above read from std::vector memory: wait before those vectors change
  HIPCHECK(hipStreamSynchronize(s), err);
  b->stats.num_chunks = nc;
  b->stats.num_pages = np;
  b->stats.input_bytes = in_bytes;
  b->stats.staged_bytes = (int64_t)b->stage.size();
  b->stats.snappy_pages = (int64_t)b->snappy.size();
  b->stats.snappy_kernel_bytes = 0;
  for (const auto &j : b->snappy) b->stats.snappy_kernel_bytes += (int64_t)j.comp_len + 2 * (int64_t)j.raw_len + j.dlen;
  b->uploaded = true;
  return PQ_OK;
}

static BatchDev batch_dev(pqgpu_batch *b) {
  uint8_t *A = b->d_arena;
  BatchDev d{};  // (every field not set below is null: err_next, dbg, ...)
  d.pages = (const PageDesc *)(A + b->o_pages);
  d.chunks = (const ChunkDesc *)(A + b->o_chunks);
  d.chunk_err = (unsigned long long *)(A + b->o_err);
  d.page_nn = (uint32_t *)(A + b->o_nn);
  d.page_nn_v = (uint32_t *)(A + b->o_nnv);
  d.dblk = (DeltaBlk *)(A + b->o_dblk);
  d.dblk_base = (const uint64_t *)(A + b->o_dblk_base);
  d.dblk_n = (uint32_t *)(A + b->o_dblk_n);
  d.dblk_sum = (unsigned long long *)(A + b->o_dblk_sum);
  d.spec_mismatch = (uint32_t *)(A + b->o_spec_flag);
  d.spec = b->spec ? 1u : 0u;
  d.ablate = getenv("PQ_ABLATE") ? (uint32_t)atoi(getenv("PQ_ABLATE")) : 0u;
  d.page_rec = (uint32_t *)(A + b->o_rec);
  d.ba_delta = (const BaDelta *)(A + b->o_ba_delta);
  d.page_vbase = (uint64_t *)(A + b->o_vbase);
  d.page_rbase = (uint64_t *)(A + b->o_rbase);
  d.nest_cnt = (uint32_t *)(A + b->o_nest_cnt);
  d.nest_base = (uint64_t *)(A + b->o_nest_base);
  d.nest_tot = (uint64_t *)(A + b->o_nest_tot);
  d.nest_done = (uint32_t *)(A + b->o_nest_done);
  d.nest_state = (uint64_t *)(A + b->o_nest_state);
  d.runs = (HybRun *)(A + b->o_runs);
  d.lv_runs = (uint2 *)(A + b->o_lv_runs);
  d.lv_run_base = (const uint64_t *)(A + b->o_lv_run_base);
  d.lv_meta = (uint32_t *)(A + b->o_lv_meta);
  d.lv_tile_run = (uint32_t *)(A + b->o_lv_tile_run);
  d.lv_tile0 = (const uint32_t *)(A + b->o_lv_tile0);
  d.run_base = (const uint64_t *)(A + b->o_run_base);
  d.run_count = (uint32_t *)(A + b->o_run_count);
  d.tile_first = (uint32_t *)(A + b->o_tile_first);
  d.tile_desc = (uint4 *)(A + b->o_tile_desc);
  d.tile_base = (const uint64_t *)(A + b->o_tile_base);
  d.ba_tile_sum = (uint64_t *)(A + b->o_ba_tile_sum);
  d.ba_tile_page = (const uint32_t *)(A + b->o_ba_tile_page);
  d.ba_tile_order = (const uint32_t *)(A + b->o_ba_tile_order);
  for (int k = 0; k < 4; k++) d.ba_class_off[k] = b->ba_class_off[k];
  d.ba_state = (uint64_t *)(A + b->o_ba_state);
  d.ba_totals = (uint64_t *)(A + b->o_ba_totals);
  d.dbg = b->debug_stamps ? (unsigned long long *)(A + b->o_dbg) : nullptr;
  d.npages = (uint32_t)b->pages.size();
  d.nchunks = (uint32_t)b->chunks.size();
  return d;
}

static PbaLists pba_lists(pqgpu_batch *b) {
  uint8_t *A = b->d_arena;
  PbaLists l;
  l.pages = (const uint32_t *)(A + b->l_pba_pages);
  l.n_pages = (uint32_t)b->pba_pages.size();
  l.seg0 = (const uint32_t *)(A + b->l_pba_seg0);
  l.seg_page = (const uint32_t *)(A + b->l_pba_seg_page);
  l.segs = (uint4 *)(A + b->o_pba_segs);
  l.limit = (uint32_t *)(A + b->o_pba_limit);
  l.n_segs = (uint32_t)b->pba_seg_page.size();
  return l;
}

static LaunchLists launch_lists(pqgpu_batch *b) {
  uint8_t *A = b->d_arena;
  LaunchLists l;
  l.level_pages = (const uint32_t *)(A + b->l_level);
  l.n_level_pages = (uint32_t)b->level_pages.size();
  l.level_pages_bw1 = (const uint32_t *)(A + b->l_level_bw1);
  l.n_level_pages_bw1 = (uint32_t)b->level_pages_bw1.size();
  l.n_level_pages_seg = b->n_level_seg;
  l.seg_grid = 0;
  l.n_level_units_seg = b->n_level_units_seg;
  l.n_level_units_hyb = b->n_level_units_hyb;
  l.lv_tiles = (const uint32_t *)(A + b->l_lv_tiles);
  l.lf_list = (const uint32_t *)(A + b->l_lf_list);
  l.n_lf_list = (uint32_t)b->lf_list.size();
  l.n_lv_tiles = (uint32_t)b->lv_tiles.size();
  l.n_ba_delta = (uint32_t)b->ba_delta.size();
  l.scan_pages = (const uint32_t *)(A + b->l_scan);
  l.n_scan_pages = (uint32_t)b->scan_pages.size();
  l.base_chunks = (const uint32_t *)(A + b->l_base);
  l.n_base_chunks = (uint32_t)b->base_chunks.size();
  l.items = (const WorkItem *)(A + b->o_items);
  l.n_items = (uint32_t)b->items.size() - b->n_copy_items;
  l.copy_items = l.items + l.n_items;
  l.n_copy_items = b->n_copy_items;
  l.ba_chunks = (const uint32_t *)(A + b->l_ba);
  l.n_ba_chunks = (uint32_t)b->ba_chunks.size();
  l.n_ba_tiles = (uint32_t)b->ba_tile_page.size();
  for (int k = 0; k < 4; k++) l.n_ba_class[k] = b->n_ba_class[k];
  l.slot_chunks = (const uint32_t *)(A + b->l_slot);
  l.n_slot_chunks = (uint32_t)b->slot_chunks.size();
  l.slot_grid_x = b->slot_grid_x;
  l.rec_pages = (const uint32_t *)(A + b->l_rec);
  l.n_rec_pages = (uint32_t)b->rec_pages.size();
  l.pc_pages = (const uint32_t *)(A + b->l_pc);
  l.n_pc_pages = (uint32_t)b->pc_pages.size();
  l.nest_desc = (const uint4 *)(A + b->l_nest_tiles);
  l.nest_order = (const uint32_t *)(A + b->l_nest_order);
  l.n_nest_tiles = (uint32_t)b->nest_tiles.size();
  for (uint32_t r = 0; r < PQGPU_MAX_NEST + 2; r++) l.nest_first[r] = b->nest_first[r];
  l.nest_chunks = (const uint32_t *)(A + b->l_nest_chunks);
  l.n_nest_chunks = (uint32_t)b->nest_chunks.size();
  l.n_nest_empty = b->n_nest_empty;
  l.grp_tiles = (const uint32_t *)(A + b->l_grp_tiles);
  l.n_grp_tiles = (uint32_t)b->grp_tiles.size();
  l.delta_pages = (const uint32_t *)(A + b->l_delta);
  l.n_delta_pages = (uint32_t)b->delta_pages.size();
  l.n_delta_tiles = b->n_delta_tiles;
  return l;
}

// Launch with optional event timing on the launch stream.
// `n` = the launch's work units: nothing is launched (or timed) for an empty list.
template <class F>
static hipError_t timed(pqgpu_batch *b, int slot, hipStream_t s, uint64_t n, F f) {
  KernelTimer &t = b->timer;
  if (!n) return hipSuccess;
  if (!t.enabled) return f();
  hipEvent_t ea = t.get(), eb = t.get();
  if (!ea || !eb) return hipErrorOutOfMemory;
  hipError_t e = hipEventRecord(ea, s);
  if (e != hipSuccess) return e;
  e = f();
  if (e != hipSuccess) return e;
  e = hipEventRecord(eb, s);
  t.recs.push_back(KernelTimer::Rec{slot, ea, eb});
  return e;
}

// The level stream's work of DELTA-major decodes that no join has covered yet: s waits for it.
static hipError_t join_deferred(pqgpu_batch *b, hipStream_t s) {
  if (!b->ds_pending) return hipSuccess;
  b->ds_pending = false;
  return hipStreamWaitEvent(s, b->ev_delta_join, 0);
}

static int decode_impl(pqgpu_batch *b, hipStream_t s, pqgpu_error *err) {
  if (!b->uploaded) {
    int e = build_and_upload(b, s, err);
    if (e) return e;
  }
  uint8_t *A = b->d_arena;
  const uint32_t np = (uint32_t)b->pages.size(), nc = (uint32_t)b->chunks.size();
  for (auto &hc : b->chunks) hc.share_from = -1;  // shared ancestors are re-checked after a decode
  // per-decode state: two contiguous fills (validity bitmaps + counters; error keys + tile table).
  // page_nn of pages without level streams is constant and was uploaded with the descriptors.
  (void)np;
  BatchDev d = batch_dev(b);
  LaunchLists l = launch_lists(b);
  const PbaLists pl = pba_lists(b);
  const char *dside = getenv("PQ_DELTA_SIDE");  // 1: the DELTA stream in every batch (comparison runs)
  const bool side = dside && atoi(dside) != 0;
  const bool any_delta = b->n_delta_items || l.n_delta_pages;
  const bool any_nest = l.n_nest_chunks || l.n_nest_tiles || l.n_grp_tiles;
  // Speculative mode whose values path is the DELTA launch alone (with its fused copies; cfg2): see below
  // (n_delta_items > 0: k_values_delta launches and resets the other key buffer, see err_ready)
  const bool delta_major = b->n_groups == 0 && b->spec && b->n_delta_items > 0 && !any_nest && !b->one_stream &&
                           b->copy_mode == 0 && !b->levels_first && !l.n_scan_pages && !b->n_dict_items &&
                           l.n_items == b->n_delta_items && !pl.n_pages && !l.n_ba_delta && !l.n_copy_items &&
                           b->ba_chunks.empty() && !l.n_rec_pages && !side;
  // Dictionary-only schedule (flat REQUIRED dictionary / boolean-RLE columns, value bases known at
  // upload; cfg1): the run scan and the dictionary tiles, two launches on the batch stream and
  // nothing else per decode. k_scan_runs resets its pages' tile tables itself, the dictionary launch
  // resets the next decode's error keys (err_next, as k_values_delta does in the DELTA-major
  // schedule); the other per-decode state is written by no kernel of this schedule, so the first
  // decode's reset holds for the later ones.
  const bool lvl_any0 = l.n_level_pages + l.n_level_pages_bw1 + l.n_lv_tiles > 0;
  const bool dict_only = b->n_groups == 0 && (b->spec || b->bases_known) && b->snappy.empty() && !any_delta && !any_nest && !lvl_any0 &&
                         b->n_dict_items > 0 && l.n_items == b->n_dict_items && l.n_scan_pages > 0 &&
                         !l.n_copy_items && !pl.n_pages && !l.n_ba_delta && b->ba_chunks.empty() && !l.n_rec_pages &&
                         !l.n_base_chunks && !l.n_lf_list && b->copy_mode == 0 && !b->levels_first && !side &&
                         !b->dict_only_off;
  // the error keys of this decode (see err_sel): the DELTA-major schedule resets the state on its
  // level stream (below) and reports into the buffer its predecessor reset; the others reset all on s
  uint32_t eu = 0;
  // deferred joins only on the context's own stream: a caller's stream must hold the whole decode
  const bool defer = delta_major && s == b->ctx->stream;
  BatchDev dl = d;  // the level stream's view in a DELTA-major decode (its own error keys)
  if (dict_only) {
    HIPCHECK(join_deferred(b, s), err);
    eu = b->err_sel ^ 1u;
    if (!b->err_ready[eu]) {  // the first decode after an upload: the whole per-decode state, once
      HIPCHECK(launch_reset(A + b->z_begin, b->z_end - b->z_begin, A + b->f_begin, b->f_end - b->f_begin, s), err);
      b->bm_zeroed = true;
      b->ds_synced = false;
    }
    d.chunk_err = (unsigned long long *)(A + (eu ? b->o_err2 : b->o_err));
    d.err_next = (unsigned long long *)(A + (eu ? b->o_err : b->o_err2));  // reset by the dictionary launch
    b->err_ready[eu ^ 1u] = true;
  } else if (delta_major) {
    eu = b->err_sel ^ 1u;
    if (!b->err_ready[eu]) {  // (the first such decode): this buffer alone, in front
      const uint64_t o = eu ? b->o_err2 : b->o_err;
      HIPCHECK(launch_reset(nullptr, 0, A + o, align_up((uint64_t)nc * 8, 16), s), err);
    }
    d.chunk_err = (unsigned long long *)(A + (eu ? b->o_err2 : b->o_err));
    d.err_next = (unsigned long long *)(A + (eu ? b->o_err : b->o_err2));  // reset by k_values_delta
    dl.chunk_err = (unsigned long long *)(A + b->o_err_ds);
    b->err_ready[eu ^ 1u] = true;
  } else {
    HIPCHECK(join_deferred(b, s), err);
    const uint64_t z0 = b->bm_zeroed ? b->z_bm_end : b->z_begin;  // (the bitmaps: first decode only)
    HIPCHECK(launch_reset(A + z0, b->z_end - z0, A + b->f_begin, b->f_end - b->f_begin, s), err);
    b->bm_zeroed = true;
    b->err_ready[1] = true;  // (o_err2 is inside the region)
    b->ds_synced = false;
  }
  b->err_sel = eu;
  b->err_ready[eu] = false;
  // SNAPPY pages first: every later kernel reads page data (column-group pipeline: one launch per
  // group, each followed by an event the group's values work waits for)
  const uint32_t G = b->n_groups;
  // the slot tables beside the run scan (one launch; never in the column-group pipeline, whose
  // scans go out per group)
  const bool slots_early = b->scan_slots && !G && l.n_slot_chunks && l.n_scan_pages;
  auto scan_runs = [&](hipStream_t st) -> hipError_t {
    if (slots_early) return timed(b, 2, st, l.n_scan_pages, [&] { return launch_scan_slots(d, l, st); });
    return timed(b, 2, st, l.n_scan_pages, [&] { return launch_scan_runs(d, l, st); });
  };
  if (G) {
    // flat REQUIRED pages only: k_bases needs no page data, and every group's values follow it
    HIPCHECK(timed(b, 3, s, l.n_base_chunks, [&] { return launch_bases(d, l, s); }), err);
    for (uint32_t g = 0; g < G; g++) {
      if (!b->ev_snap[g]) HIPCHECK(hipEventCreateWithFlags(&b->ev_snap[g], hipEventDisableTiming), err);
      const uint32_t j0 = b->grp_job[g], j1 = b->grp_job[g + 1];
      HIPCHECK(timed(b, 11, s, j1 - j0, [&] {
                 return launch_snappy(d, (const SnappyJob *)(A + b->o_snappy) + j0, j1 - j0, s);
               }),
               err);
      HIPCHECK(hipEventRecord(b->ev_snap[g], s), err);
    }
  } else if (!b->snappy.empty()) {
    HIPCHECK(timed(b, 11, s, b->snappy.size(), [&] {
               return launch_snappy(d, (const SnappyJob *)(A + b->o_snappy), (uint32_t)b->snappy.size(), s);
             }),
             err);
  }
  // DELTA work items and the other value work items go out as two launches (separately profiled).
  LaunchLists l1 = l, l2 = l;
  l1.n_items = b->n_delta_items;
  const WorkItem *dict_items = l.items + b->n_delta_items;
  const uint32_t n_dict = b->n_dict_items;
  l2.items = dict_items + n_dict;
  l2.n_items = l.n_items - b->n_delta_items - n_dict;
  // DELTA_BINARY_PACKED items (the first n_delta_items) go to k_values_delta on the DELTA stream,
  // beside the level kernels, the copies and the other values kinds; the default stream joins it
  // a batch without level streams and column groups keeps its DELTA pages on the batch stream: with
  // nothing to overlap but the other values kinds they only compete with them (cfg5 6.19 -> 6.08 ms)
  const bool lvl_any = l.n_level_pages + l.n_level_pages_bw1 + l.n_lv_tiles > 0;
  hipStream_t ds = b->one_stream || (!lvl_any && b->n_groups == 0 && !side) ? s : b->ctx->delta;
  if (!b->ev_delta_join) HIPCHECK(hipEventCreateWithFlags(&b->ev_delta_join, hipEventDisableTiming), err);
  // streams with nothing to run are neither forked nor joined (a cross-stream wait costs latency)
  auto fork_delta = [&](hipEvent_t after) -> hipError_t {
    if (!any_delta) return hipSuccess;
    hipError_t e = hipStreamWaitEvent(ds, after, 0);
    if (e == hipSuccess) e = timed(b, 10, ds, l.n_delta_pages, [&] { return launch_delta_prep(d, l, ds); });
    if (e == hipSuccess) e = timed(b, 1, ds, l1.n_items, [&] { return launch_values_delta(d, l1.items, l1.n_items, ds); });
    if (e == hipSuccess) e = hipEventRecord(b->ev_delta_join, ds);
    return e;
  };
  // Nested (Arrow-style) arrays and struct bitmaps need only the level run tables and the per-half
  // counts k_nest_count wrote (flat leaves' struct bitmaps: k_level_fill's u8 levels): they run on
  // the DELTA stream (after its DELTA pages) beside the values path, from the moment k_bases is
  // queued; the batch stream joins them at the end.
  if (!b->ev_levels) HIPCHECK(hipEventCreateWithFlags(&b->ev_levels, hipEventDisableTiming), err);
  if (!b->ev_nest_join) HIPCHECK(hipEventCreateWithFlags(&b->ev_nest_join, hipEventDisableTiming), err);
  // nested tiles on stream st: the fused pass (k_nest_tile), or k_nest_count (k_nest_emit in fork_nest)
  const bool pc_sched = b->nest_fused && b->nest_pcount && l.n_pc_pages && l.n_nest_tiles && !b->one_stream;
  bool aux_out = false;  // k_nest_tile on the aux stream, not yet joined
  auto launch_nest_pass = [&](hipStream_t st) -> hipError_t {
    if (pc_sched) {  // counts first (k_bases waits for them only), the arrays beside the rest
      hipError_t e = timed(b, 23, st, l.n_pc_pages, [&] { return launch_nest_pcount(d, l, st); });
      if (e == hipSuccess && !b->ev_aux_fork) e = hipEventCreateWithFlags(&b->ev_aux_fork, hipEventDisableTiming);
      if (e == hipSuccess && !b->ev_aux_join) e = hipEventCreateWithFlags(&b->ev_aux_join, hipEventDisableTiming);
      if (e == hipSuccess) e = hipEventRecord(b->ev_aux_fork, st);
      if (e == hipSuccess) e = hipStreamWaitEvent(b->ctx->aux, b->ev_aux_fork, 0);
      if (e == hipSuccess)
        e = timed(b, 22, b->ctx->aux, l.n_nest_tiles, [&] { return launch_nest_tile(d, l, b->ctx->aux, true); });
      if (e == hipSuccess) e = hipEventRecord(b->ev_aux_join, b->ctx->aux);
      aux_out = e == hipSuccess;
      return e;
    }
    if (b->nest_fused && b->nest_tcount && l.nest_first[2] == l.nest_first[PQGPU_MAX_NEST + 1]) {  // (all R = 1)
      hipError_t e = timed(b, 24, st, l.n_nest_tiles, [&] { return launch_nest_tcount(d, l, st); });
      if (e == hipSuccess) e = timed(b, 22, st, l.n_nest_tiles, [&] { return launch_nest_tile(d, l, st, false, true); });
      return e;
    }
    if (b->nest_fused) return timed(b, 22, st, l.n_nest_tiles, [&] { return launch_nest_tile(d, l, st, false); });
    return timed(b, 13, st, l.n_nest_tiles, [&] { return launch_nest_count(d, l, st); });
  };
  // the level kernels on st; with a split, the generic streams past k_levels_segw's on the aux stream
  const bool lv_split = b->level_split && !b->one_stream && l.n_level_units_seg && l.n_level_pages > l.n_level_units_seg;
  auto levels = [&](hipStream_t st) -> hipError_t {
    if (!lv_split) return timed(b, 0, st, l.n_level_pages + l.n_level_pages_bw1, [&] { return launch_levels(d, l, st); });
    hipError_t e = hipSuccess;
    if (!b->ev_lv_fork) e = hipEventCreateWithFlags(&b->ev_lv_fork, hipEventDisableTiming);
    if (e == hipSuccess && !b->ev_lv_join) e = hipEventCreateWithFlags(&b->ev_lv_join, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventRecord(b->ev_lv_fork, st);
    if (e == hipSuccess) e = hipStreamWaitEvent(b->ctx->aux, b->ev_lv_fork, 0);
    // (the timer slot brackets the launches on st: with the split it times k_levels_segw's part)
    if (e == hipSuccess)
      e = timed(b, 0, st, l.n_level_pages + l.n_level_pages_bw1, [&] { return launch_levels(d, l, st, b->ctx->aux); });
    if (e == hipSuccess) e = hipEventRecord(b->ev_lv_join, b->ctx->aux);
    if (e == hipSuccess) e = hipStreamWaitEvent(st, b->ev_lv_join, 0);
    return e;
  };
  auto fork_nest = [&]() -> hipError_t {
    if (!any_nest) return hipSuccess;
    hipError_t e = hipEventRecord(b->ev_levels, s);
    if (e == hipSuccess) e = hipStreamWaitEvent(ds, b->ev_levels, 0);
    if (e == hipSuccess) e = timed(b, 16, ds, l.n_nest_empty, [&] { return launch_nest_scan(d, l, ds); });
    if (e == hipSuccess && !b->nest_fused)
      e = timed(b, 14, ds, l.n_nest_tiles, [&] { return launch_nest_emit(d, l, ds); });
    if (e == hipSuccess) e = timed(b, 21, ds, l.n_grp_tiles, [&] { return launch_group_flat(d, l, ds); });  // flat leaves
    if (e == hipSuccess) e = hipEventRecord(b->ev_nest_join, ds);
    return e;
  };
  // PLAIN / BOOLEAN copies (k_values_copy) run on the copy stream beside everything else once
  // their value bases are known: at the start in speculative mode, after k_bases otherwise.
  hipStream_t cs = b->one_stream ? s : b->ctx->copy;
  if (!b->ev_copy) HIPCHECK(hipEventCreateWithFlags(&b->ev_copy, hipEventDisableTiming), err);
  if (!b->ev_copy_join) HIPCHECK(hipEventCreateWithFlags(&b->ev_copy_join, hipEventDisableTiming), err);
  bool copies_out = false;  // forked and not yet joined by the batch stream
  auto fork_copies = [&](hipStream_t from) -> hipError_t {
    if (!l.n_copy_items) return hipSuccess;
    copies_out = true;
    hipError_t e = hipEventRecord(b->ev_copy, from);
    if (e == hipSuccess) e = hipStreamWaitEvent(cs, b->ev_copy, 0);
    if (e == hipSuccess) e = timed(b, 20, cs, l.n_copy_items, [&] { return launch_values_copy(d, l, cs); });
    if (e == hipSuccess) e = hipEventRecord(b->ev_copy_join, cs);
    return e;
  };
  if (G) {
    // Column-group pipeline: group g's run scan and dictionary tiles (side stream) and its DELTA
    // pages and fused copies (DELTA stream) start when group g's SNAPPY launch is done, beside the
    // decompression of the later groups on the batch stream.
    hipStream_t v = b->one_stream ? s : b->ctx->side;
    if (!b->ev_join) HIPCHECK(hipEventCreateWithFlags(&b->ev_join, hipEventDisableTiming), err);
    for (uint32_t g = 0; g < G; g++) {
      LaunchLists lg = l;
      lg.scan_pages = l.scan_pages + b->grp_scan[g];
      lg.n_scan_pages = b->grp_scan[g + 1] - b->grp_scan[g];
      const WorkItem *it0 = l.items + b->grp_item[g];
      const uint32_t nd = b->grp_delta[g], nk = b->grp_dict[g], ni = b->grp_item[g + 1] - b->grp_item[g];
      lg.items = it0 + nd + nk;
      lg.n_items = ni - nd - nk;
      HIPCHECK(hipStreamWaitEvent(v, b->ev_snap[g], 0), err);
      HIPCHECK(timed(b, 2, v, lg.n_scan_pages, [&] { return launch_scan_runs(d, lg, v); }), err);
      HIPCHECK(timed(b, 8, v, nk, [&] { return launch_values_dict(d, it0 + nd, 0, nk, v); }), err);
      HIPCHECK(timed(b, 9, v, lg.n_items, [&] { return launch_values(d, lg, v); }), err);
      if (nd) {
        HIPCHECK(hipStreamWaitEvent(ds, b->ev_snap[g], 0), err);
        HIPCHECK(timed(b, 1, ds, nd, [&] { return launch_values_delta(d, it0, nd, ds); }), err);
      }
    }
    HIPCHECK(hipEventRecord(b->ev_join, v), err);
    HIPCHECK(hipEventRecord(b->ev_delta_join, ds), err);
    HIPCHECK(hipStreamWaitEvent(s, b->ev_join, 0), err);
    HIPCHECK(hipStreamWaitEvent(s, b->ev_delta_join, 0), err);
  } else if (delta_major) {
    // Speculative mode whose values path is the DELTA launch alone (with its fused copies; cfg2):
    // that launch is the critical path, so it runs on the batch stream right after the resets, and
    // the level kernels and k_bases go to the DELTA stream beside it. No stream waits on the
    // critical path but the final join of the (long finished) level stream: cfg2 lost ~20 us per
    // step between k_reset and k_values_delta and ~13 us after it to cross-stream waits.
    // The level stream reads only uploaded pages and writes only its own state: it waits for the
    // batch stream once after an upload (or a decode of another schedule), not per decode
    if (!b->ds_synced || !defer) {
      if (!b->ev_fork) HIPCHECK(hipEventCreateWithFlags(&b->ev_fork, hipEventDisableTiming), err);
      HIPCHECK(hipEventRecord(b->ev_fork, s), err);
      HIPCHECK(hipStreamWaitEvent(ds, b->ev_fork, 0), err);
      b->ds_synced = true;
    }
    // the per-decode state and the level stream's keys: [o_tile_first, o_err_ds end) of the 0xff region
    const uint64_t z0 = b->bm_zeroed ? b->z_bm_end : b->z_begin;  // (the bitmaps: first decode only)
    HIPCHECK(launch_reset(A + z0, b->z_end - z0, A + b->o_tile_first, b->f_end - b->o_tile_first, ds), err);
    b->bm_zeroed = true;
    // k_levels_seg beside the values launch: at most ~4 level waves per CU resident (each walks two
    // pages or more; cfg2's 2,048 pages: 1,024 waves, step 0.361 -> 0.346 ms; 768 or 1,536: slower)
    LaunchLists lv = l;
    lv.seg_grid = l.n_level_pages_seg > 1024 ? std::max<uint32_t>(1024, l.n_level_pages_seg / 2) : 0;
    HIPCHECK(timed(b, 0, ds, l.n_level_pages + l.n_level_pages_bw1, [&] { return launch_levels(dl, lv, ds); }), err);
    HIPCHECK(timed(b, 15, ds, l.n_lf_list, [&] { return launch_level_fill(dl, l, ds); }), err);
    HIPCHECK(timed(b, 3, ds, l.n_base_chunks, [&] { return launch_bases(dl, l, ds); }), err);
    HIPCHECK(hipEventRecord(b->ev_delta_join, ds), err);
    HIPCHECK(timed(b, 10, s, l.n_delta_pages, [&] { return launch_delta_prep(d, l, s); }), err);
    HIPCHECK(timed(b, 1, s, l1.n_items, [&] { return launch_values_delta(d, l1.items, l1.n_items, s); }), err);
    if (defer) b->ds_pending = true;  // joined by the next operation that needs it (join_deferred)
    else HIPCHECK(hipStreamWaitEvent(s, b->ev_delta_join, 0), err);
  } else if (b->spec) {
    // Speculative mode: the values path (dictionary pages, run tables, values) runs on the
    // side stream concurrently with the level decode; k_bases then checks the header counts
    // the values path used against the decoded ones (sync_impl re-runs serially on a miss).
    // no level streams in the batch (REQUIRED columns only): the values path runs on the batch stream
    const bool lvl = l.n_level_pages + l.n_level_pages_bw1 + l.n_lv_tiles > 0;
    hipStream_t v = lvl && !b->one_stream ? b->ctx->side : s;
    if (!b->ev_fork) HIPCHECK(hipEventCreateWithFlags(&b->ev_fork, hipEventDisableTiming), err);
    if (!b->ev_join) HIPCHECK(hipEventCreateWithFlags(&b->ev_join, hipEventDisableTiming), err);
    // PQ_COPY_MODE 4: the copies beside the level kernels, the values path after them;
    // 5: the copies beside the values path, the level kernels after it (profiling)
    const bool lv_then_val = b->copy_mode == 4, val_then_lv = b->copy_mode == 5;
    if (lv_then_val || val_then_lv) HIPCHECK(fork_copies(s), err);
    if (lv_then_val) HIPCHECK(levels(s), err);
    // (only when a stream waits for it: an event record on the batch stream costs ~6 us of idle GPU
    // in front of the next launch, cfg1 / cfg3 kernel traces)
    if (v != s || any_delta) HIPCHECK(hipEventRecord(b->ev_fork, s), err);
    if (b->levels_first)  // experiment (PQ_LEVELS_FIRST=1): the level kernels are dispatched first
      HIPCHECK(levels(s), err);
    if (v != s) HIPCHECK(hipStreamWaitEvent(v, b->ev_fork, 0), err);
    HIPCHECK(fork_delta(b->ev_fork), err);
    HIPCHECK(scan_runs(v), err);
    if (b->copy_mode == 0) HIPCHECK(fork_copies(s), err);
    if (b->copy_mode == 6)  // the copies first on the side stream, then the LDS kinds
      HIPCHECK(timed(b, 20, v, l.n_copy_items, [&] { return launch_values_copy(d, l, v); }), err);
    HIPCHECK(timed(b, 8, v, n_dict, [&] { return launch_values_dict(d, dict_items, b->n_dict2_items, n_dict, v); }), err);
    HIPCHECK(timed(b, 9, v, l2.n_items, [&] { return launch_values(d, l2, v); }), err);
    if (b->copy_mode == 1) HIPCHECK(fork_copies(v), err);
    HIPCHECK(timed(b, 17, v, pl.n_pages, [&] { return launch_plain_ba(d, pl, v); }), err);
    HIPCHECK(timed(b, 18, v, l.n_ba_delta, [&] { return launch_ba_delta(d, l, v); }), err);
    if (v != s) HIPCHECK(hipEventRecord(b->ev_join, v), err);
    if (val_then_lv && v != s) HIPCHECK(hipStreamWaitEvent(s, b->ev_join, 0), err);
    if (!b->levels_first && !lv_then_val) HIPCHECK(levels(s), err);
    HIPCHECK(timed(b, 15, s, l.n_lf_list, [&] { return launch_level_fill(d, l, s); }), err);
    HIPCHECK(launch_nest_pass(s), err);
    HIPCHECK(timed(b, 3, s, l.n_base_chunks, [&] { return launch_bases(d, l, s); }), err);
    HIPCHECK(fork_nest(), err);
    if (b->copy_mode == 2) HIPCHECK(fork_copies(s), err);
    if (v != s) HIPCHECK(hipStreamWaitEvent(s, b->ev_join, 0), err);
    if (b->copy_mode >= 3) HIPCHECK(fork_copies(s), err);
    // the byte-array path reads no copied values: it goes ahead of the copy stream's join (cfg4: it
    // waited ~140 us for the INT32 / INT64 copies)
    if (copies_out && b->ba_chunks.empty()) {
      HIPCHECK(hipStreamWaitEvent(s, b->ev_copy_join, 0), err);
      copies_out = false;
    }
    if (any_delta) HIPCHECK(hipStreamWaitEvent(s, b->ev_delta_join, 0), err);
  } else {
    // (bases speculated: the copies beside the level kernels. cfg4 1.30 -> 1.27-1.28 ms; enqueued after
    // the level kernels: equal; beside k_nest_tile: 1.33 ms, profiles/r06_z_probe_cfg4_copy_early.txt)
    if (b->copies_early) HIPCHECK(fork_copies(s), err);
    HIPCHECK(levels(s), err);
    HIPCHECK(timed(b, 15, s, l.n_lf_list, [&] { return launch_level_fill(d, l, s); }), err);
    HIPCHECK(launch_nest_pass(s), err);
    HIPCHECK(timed(b, 3, s, l.n_base_chunks, [&] { return launch_bases(d, l, s); }), err);
    if (b->copy_mode < 3 && !b->copies_early) HIPCHECK(fork_copies(s), err);
    if (!b->ev_fork) HIPCHECK(hipEventCreateWithFlags(&b->ev_fork, hipEventDisableTiming), err);
    if (any_delta && !b->split_values)  // (only when the DELTA stream waits for it)
      HIPCHECK(hipEventRecord(b->ev_fork, s), err);  // after k_bases: the value bases are known
    if (b->split_values) {  // PQ_SPLIT_VALUES=1: DELTA and the other work items one after the other (profiling)
      HIPCHECK(timed(b, 10, s, l.n_delta_pages, [&] { return launch_delta_prep(d, l, s); }), err);
      HIPCHECK(timed(b, 1, s, l1.n_items, [&] { return launch_values_delta(d, l1.items, l1.n_items, s); }), err);
      HIPCHECK(hipEventRecord(b->ev_delta_join, s), err);
    } else {
      HIPCHECK(fork_delta(b->ev_fork), err);
    }
    HIPCHECK(fork_nest(), err);  // on the DELTA stream after its pages
    // DELTA pages on the batch stream (no level streams; cfg5): the run scan and the dictionary tiles
    // beside them on the side stream (cfg5 5.67-5.68 -> 5.63 ms; the scan alone beside them: equal,
    // profiles/r06_ac_probe_cfg5_scan_side.txt). PQ_SCAN_SIDE=0: after them on the batch stream
    const bool side_dict = !(getenv("PQ_SCAN_SIDE") && atoi(getenv("PQ_SCAN_SIDE")) == 0) && ds == s && any_delta &&
                           !b->split_values && (l.n_scan_pages || n_dict) && !b->one_stream;
    hipStream_t vs = side_dict ? b->ctx->side : s;
    if (side_dict) {
      HIPCHECK(hipStreamWaitEvent(vs, b->ev_fork, 0), err);
      if (!b->ev_join) HIPCHECK(hipEventCreateWithFlags(&b->ev_join, hipEventDisableTiming), err);
    }
    HIPCHECK(scan_runs(vs), err);
    HIPCHECK(timed(b, 8, vs, n_dict, [&] { return launch_values_dict(d, dict_items, b->n_dict2_items, n_dict, vs); }), err);
    if (side_dict) {
      HIPCHECK(hipEventRecord(b->ev_join, vs), err);
      HIPCHECK(hipStreamWaitEvent(s, b->ev_join, 0), err);
    }
    HIPCHECK(timed(b, 9, s, l2.n_items, [&] { return launch_values(d, l2, s); }), err);
    HIPCHECK(timed(b, 17, s, pl.n_pages, [&] { return launch_plain_ba(d, pl, s); }), err);  // PLAIN BYTE_ARRAY chains
    HIPCHECK(timed(b, 18, s, l.n_ba_delta, [&] { return launch_ba_delta(d, l, s); }), err);  // DLBA / DBA lengths -> values
    if (b->copy_mode >= 3) HIPCHECK(fork_copies(s), err);  // PQ_COPY_MODE=3: after everything (profiling)
    if (copies_out && b->ba_chunks.empty()) {
      HIPCHECK(hipStreamWaitEvent(s, b->ev_copy_join, 0), err);
      copies_out = false;
    }
    if (any_delta && !b->split_values) HIPCHECK(hipStreamWaitEvent(s, b->ev_delta_join, 0), err);
  }
  if (!b->ba_chunks.empty()) {
    // byte-array outputs: tile payload sums, per-chunk scan, offsets + payload (bytearray.hip)
    if (!slots_early) HIPCHECK(timed(b, 12, s, l.n_slot_chunks, [&] { return launch_dict_slots(d, l, s); }), err);
    if (b->any_ba_sync || b->ba_presum) {
      HIPCHECK(timed(b, 4, s, l.n_ba_tiles, [&] { return launch_ba_sums(d, l, s); }), err);
      HIPCHECK(timed(b, 5, s, l.n_ba_chunks, [&] { return launch_ba_scan(d, l, s); }), err);
    }
    if (b->any_ba_sync) {
      // chunks without an upload-time payload bound (DELTA_BYTE_ARRAY pages): size them now
      std::vector<uint64_t> totals(nc);
      HIPCHECK(hipMemcpyAsync(totals.data(), A + b->o_ba_totals, (size_t)nc * 8, hipMemcpyDeviceToHost, s), err);
      HIPCHECK(hipStreamSynchronize(s), err);
      for (uint32_t c : b->ba_chunks) {
        HostChunk &hc = b->chunks[c];
        if (!hc.ba_sync) continue;
        ChunkDesc &cd = b->chunk_desc[c];
        hc.sync_err = totals[c] > 0x7fffffffULL - 64;
        if (hc.sync_err) {
          cd.payload = 0;  // k_ba_emit / k_dba_gather skip the chunk; sync reports it
        } else {
          if (totals[c] + 64 > hc.payload_cap) {
            if (hc.payload_own && hc.payload) (void)hipFree(hc.payload);
            hc.payload = nullptr;
            hc.payload_cap = 0;
            HIPCHECK(hipMalloc(&hc.payload, (size_t)totals[c] + 64), err);
            hc.payload_own = true;
            hc.payload_cap = totals[c] + 64;
          }
          cd.payload = (uint64_t)hc.payload;
          cd.payload_capacity = totals[c];
        }
        HIPCHECK(hipMemcpyAsync(A + b->o_chunks + (uint64_t)c * sizeof(ChunkDesc), &cd, sizeof(ChunkDesc),
                                hipMemcpyHostToDevice, s),
                 err);
      }
    }
    HIPCHECK(timed(b, 6, s, l.n_ba_tiles, [&] { return launch_ba_emit(d, l, s); }), err);
    HIPCHECK(timed(b, 19, s, l.n_ba_delta, [&] { return launch_dba_gather(d, l, s); }), err);
    if (b->any_ba_sync) HIPCHECK(hipStreamSynchronize(s), err);  // chunk_desc copies above read host memory
    if (copies_out) HIPCHECK(hipStreamWaitEvent(s, b->ev_copy_join, 0), err);  // (see above)
    copies_out = false;
  }
  HIPCHECK(timed(b, 7, s, l.n_rec_pages, [&] { return launch_records(d, l, s); }), err);
  // nested (Arrow-style) arrays of repeated leaves (nested.hip)
  // (k_nest_count counted the fill tiles' halves beside k_level_fill; k_nest_emit writes the levels)
  if (any_nest) HIPCHECK(hipStreamWaitEvent(s, b->ev_nest_join, 0), err);  // nested arrays (fork_nest)
  if (aux_out) HIPCHECK(hipStreamWaitEvent(s, b->ev_aux_join, 0), err);     // k_nest_tile (pc_sched)
  b->decoded = true;
  return PQ_OK;
}

// Key -> pqgpu_error (see err_key in pq_device.h).
static void decode_key(uint64_t key, int chunk, pqgpu_error *e) {
  uint32_t phase = (uint32_t)(key >> 62);
  uint32_t page = (uint32_t)((key >> 40) & 0x3fffff);
  uint32_t stage = (uint32_t)((key >> 36) & 15);
  uint32_t pos = (uint32_t)((key >> 4) & 0xffffffffu);
  uint32_t code = (uint32_t)(key & 15);
  static const char *stages[] = {"dictionary", "repetition levels", "definition levels", "values"};
  char msg[200];
  if (phase == 0 && stage == ST_DECOMP) {  // k_snappy: the page's readPages failure
    set_err(e, (int)code, chunk, (int)page, "decompression failed: snappy: corrupt input");
  } else if (phase == 0) {
    snprintf(msg, sizeof(msg), "%s decode failed at entry %u: %s", stages[stage & 3], pos, pqgpu_status_string((int)code));
    set_err(e, (int)code, chunk, -1, msg);
  } else {
    snprintf(msg, sizeof(msg), "read %s from page failed at position %u: %s", stages[stage & 3], pos,
             pqgpu_status_string((int)code));
    set_err(e, (int)code, chunk, (int)page, msg);
  }
}

static int sync_impl(pqgpu_batch *b, hipStream_t s, pqgpu_error *err) {
  clear_err(err);
  HIPCHECK(join_deferred(b, s), err);
  HIPCHECK(hipStreamSynchronize(s), err);
  if (!b->decoded) return PQ_OK;
  if (b->spec || b->copies_early) {
    uint32_t miss = 0;
    HIPCHECK(hipMemcpy(&miss, b->d_arena + b->o_spec_flag, 4, hipMemcpyDeviceToHost), err);
    if (miss) {  // a page header's non-null count was wrong: decode again in serial order
      b->force_serial = true;
      b->uploaded = false;
      int e = decode_impl(b, s, err);
      if (e) return e;
      HIPCHECK(hipStreamSynchronize(s), err);
    }
  }
  const uint32_t np = (uint32_t)b->pages.size(), nc = (uint32_t)b->chunks.size();
  std::vector<uint64_t> keys(nc), vbase(np), rbase(np);
  std::vector<uint32_t> nn(np), rec(np);
  uint8_t *A = b->d_arena;
  if (nc) {
    HIPCHECK(hipMemcpy(keys.data(), A + (b->err_sel ? b->o_err2 : b->o_err), nc * 8, hipMemcpyDeviceToHost), err);
    std::vector<uint64_t> kd(nc);  // the level stream's keys (0xff.. unless a DELTA-major decode reported)
    HIPCHECK(hipMemcpy(kd.data(), A + b->o_err_ds, nc * 8, hipMemcpyDeviceToHost), err);
    for (uint32_t c = 0; c < nc; c++) keys[c] = std::min(keys[c], kd[c]);
  }
  if (np) {
    HIPCHECK(hipMemcpy(vbase.data(), A + b->o_vbase, np * 8, hipMemcpyDeviceToHost), err);
    HIPCHECK(hipMemcpy(nn.data(), A + b->o_nn, np * 4, hipMemcpyDeviceToHost), err);
    HIPCHECK(hipMemcpy(rbase.data(), A + b->o_rbase, np * 8, hipMemcpyDeviceToHost), err);
    HIPCHECK(hipMemcpy(rec.data(), A + b->o_rec, np * 4, hipMemcpyDeviceToHost), err);
  }
  std::vector<uint64_t> nest_tot;
  if (!b->nest_chunks.empty()) {
    nest_tot.resize((size_t)nc * kNestCnt);
    HIPCHECK(hipMemcpy(nest_tot.data(), A + b->o_nest_tot, (size_t)nc * kNestCnt * 8, hipMemcpyDeviceToHost), err);
  }
  std::vector<uint64_t> ba_tot;
  if (!b->ba_chunks.empty()) {
    ba_tot.resize(nc);
    HIPCHECK(hipMemcpy(ba_tot.data(), A + b->o_ba_totals, (size_t)nc * 8, hipMemcpyDeviceToHost), err);
  }
  b->page_vbase_out = vbase;
  b->page_nn_out = nn;
  int first = PQ_OK;
  int64_t out_bytes = 0, slots = 0, values = 0, lvl_bytes = 0, val_bytes = 0, dl_bytes = 0, snappy_direct_bytes = 0,
          cp_bytes = 0, dict_bytes = 0;
  int64_t kb[PQGPU_TIMER_SLOTS] = {0};  // algorithmic bytes per launch slot
  for (uint32_t c = 0; c < nc; c++) {
    HostChunk &hc = b->chunks[c];
    clear_err(&hc.dev_err);
    hc.dev_err.chunk = (int)c;
    if (!hc.err.code && keys[c] != ~0ull) decode_key(keys[c], (int)c, &hc.dev_err);
    // a page's readValues error leaves the pages before it decoded (the reference's lazy page
    // reader returns their rows first, data_store.go:236-260); decompression and CRC errors are
    // readPages errors (chunk_reader.go:161-180): nothing of the chunk is returned
    hc.partial = !hc.err.code && hc.dev_err.code && hc.dev_err.page >= 0 && hc.dev_err.code != PQ_ERR_DECOMPRESS &&
                 hc.dev_err.code != PQ_ERR_CRC && (uint32_t)hc.dev_err.page < hc.num_pages;
    if (hc.partial) {
      const uint32_t fp = hc.first_page + (uint32_t)hc.dev_err.page;
      hc.part_slots = (int64_t)b->pages[fp].slot_base;
      hc.part_nn = (int64_t)vbase[fp];
      hc.part_records = (int64_t)rbase[fp];
      hc.part_payload = 0;
      if (hc.value_width == 0 && hc.part_nn > 0 && hc.o_offsets) {
        int32_t end = 0;
        HIPCHECK(hipMemcpy(&end, A + hc.o_offsets + 4 * (uint64_t)hc.part_nn, 4, hipMemcpyDeviceToHost), err);
        hc.part_payload = end;
      }
    }
    if (!hc.err.code && hc.sync_err && !hc.dev_err.code)
      set_err(&hc.dev_err, PQ_ERR_UNSUPPORTED, (int)c, -1, "BYTE_ARRAY chunk payload exceeds 2 GiB");
    if (!ba_tot.empty() && hc.value_width == 0) hc.payload_bytes = (int64_t)ba_tot[c];
    for (uint32_t k = 0; k < PQGPU_MAX_NEST; k++)
      hc.num_lists[k] = k < hc.nest ? (int64_t)nest_tot[(size_t)c * kNestCnt + k] : 0;
    hc.num_elems = hc.nest ? (int64_t)nest_tot[(size_t)c * kNestCnt + hc.nest] : 0;
    if (hc.num_pages) {
      uint32_t lp = hc.first_page + hc.num_pages - 1;
      hc.nn = (int64_t)(vbase[lp] + nn[lp]);
      hc.records = (int64_t)(rbase[lp] + rec[lp]);
    } else {
      hc.nn = 0;
      hc.records = 0;
    }
    const pqgpu_error &e = hc.err.code ? hc.err : hc.dev_err;
    if (e.code && !first) {
      first = e.code;
      if (err) *err = e;
    }
    if (!e.code) {
      slots += (int64_t)hc.num_slots;
      values += hc.nn;
      int w = hc.value_width;
      out_bytes += w ? hc.nn * w : (hc.nn + 1) * 4 + hc.payload_bytes;
      if (hc.o_def) out_bytes += (int64_t)hc.num_slots;
      if (hc.o_rep) out_bytes += (int64_t)hc.num_slots;
      if (hc.o_valid) out_bytes += (int64_t)(hc.num_slots + 7) / 8;
      if (hc.o_lists) out_bytes += (hc.records + 1) * 4;
      int64_t ba_dict_nn = 0, ba_other_nn = 0;
      for (uint32_t p = hc.first_page; p < hc.first_page + hc.num_pages; p++) {
        const PageDesc &pd = b->pages[p];
        lvl_bytes += pd.rep_len + pd.def_len;
        if (pd.vkind == VK_DELTA32 || pd.vkind == VK_DELTA64) dl_bytes += pd.val_len + (int64_t)nn[p] * w;
        if ((pd.vkind == VK_PLAIN_FIXED || pd.vkind == VK_PLAIN_INT96 || pd.vkind == VK_PLAIN_BOOL) &&
            !((pd.flags & PF_DEV_SNAPPY) && b->snappy[pd.data].to_values))
          cp_bytes += pd.val_len + (int64_t)nn[p] * (pd.vkind == VK_PLAIN_BOOL ? 1 : w);  // the copies' launch
        if (pd.vkind == VK_DICT || pd.vkind == VK_RLE_BOOL) kb[2] += pd.val_len;  // k_scan_runs: index streams
        if ((pd.vkind == VK_DICT && w > 0) || pd.vkind == VK_RLE_BOOL)
          dict_bytes += pd.val_len + (int64_t)nn[p] * (pd.vkind == VK_RLE_BOOL ? 1 : w);  // k_values_dict
        if (w == 0 && pd.vkind == VK_DICT) {
          if (hc.ba_sync || hc.ba_presum) kb[4] += pd.val_len;  // k_ba_sums re-reads the indices
          kb[6] += pd.val_len;
          ba_dict_nn += nn[p];
        } else if ((pd.flags & PF_DEV_SNAPPY) && b->snappy[pd.data].to_values) {
          snappy_direct_bytes += (int64_t)nn[p] * w;  // written by k_snappy into the values: no k_values work
        } else {
          val_bytes += pd.val_len;  // k_values reads the page's value section
          if (w == 0) ba_other_nn += nn[p];
        }
      }
      {
        // generic level streams: k_levels walks the streams (run tables), k_level_fill reads them
        // again and writes the outputs; flat OPTIONAL: k_levels_bw1 writes the validity
        int64_t lv_out = 0, lv_in = 0;
        for (uint32_t p = hc.first_page; p < hc.first_page + hc.num_pages; p++) lv_in += b->pages[p].rep_len + b->pages[p].def_len;
        if (hc.o_def) lv_out += (int64_t)hc.num_slots;
        if (hc.o_rep) lv_out += (int64_t)hc.num_slots;
        if (hc.o_valid) lv_out += (int64_t)(hc.num_slots + 7) / 8;
        if (hc.nest) {  // k_nest_count expands the streams and writes the levels (k_nest_emit: the nested arrays)
          kb[13] += lv_in + lv_out;
        } else if (hc.col.max_rep > 0 || hc.col.max_def > 1) {
          kb[15] += lv_in + lv_out;
        } else {
          lvl_bytes += lv_out;
        }
      }
      if (w) {
        val_bytes += hc.nn * w;  // (less the direct SNAPPY pages' values, below)
      } else {
        // lengths of the non-dictionary pages: read by k_ba_sums; read with their sources and
        // bytes by k_ba_emit, which writes every offset and the payload
        if (hc.ba_sync || hc.ba_presum) kb[4] += 4 * ba_other_nn;
        kb[6] += 4 * (hc.nn + 1) + hc.payload_bytes + 12 * ba_other_nn;
        kb[5] += 16 * (int64_t)b->chunk_desc[c].ba_ntiles;
        if (hc.slot_shift) kb[12] += (int64_t)hc.dict_len + 8 * (int64_t)hc.dict_count + ((int64_t)hc.dict_count << hc.slot_shift);
        (void)ba_dict_nn;
      }
      if (hc.o_lists && !hc.nest) kb[7] += (int64_t)hc.num_slots + 4 * (hc.records + 1);
      if (hc.nest) {  // offsets and bitmaps written by k_nest_emit
        kb[14] += (hc.num_elems + 7) / 8 + 4 * (hc.records + 1);  // + record offsets
        for (uint32_t k = 0; k < hc.nest; k++) kb[14] += 4 * (hc.num_lists[k] + 1) + (hc.num_lists[k] + 7) / 8;
        out_bytes += (hc.num_elems + 7) / 8;
        for (uint32_t k = 0; k < hc.nest; k++) out_bytes += 4 * (hc.num_lists[k] + 1) + (hc.num_lists[k] + 7) / 8;
      }
      for (uint32_t g = 0; g < hc.ngroups; g++) {  // struct bitmaps of their own (k_nest_emit / k_group_flat)
        if (hc.grp_alias[g] >= 0) continue;
        const int j = hc.col.group_depth[g];
        const int64_t ent = hc.col.max_rep == 0 ? (int64_t)hc.num_slots : (j < hc.col.max_rep ? hc.num_lists[j] : hc.num_elems);
        out_bytes += (ent + 7) / 8;
        // repeated leaves: k_nest_emit writes it; flat leaves: k_group_flat (+ the u8 levels it reads)
        if (hc.col.max_rep == 0) kb[21] += (ent + 7) / 8 + (int64_t)hc.num_slots;
        else kb[14] += (ent + 7) / 8;
      }
    }
  }
  kb[0] = lvl_bytes;
  if (b->scan_slots && !b->n_groups && !b->slot_chunks.empty() && !b->scan_pages.empty()) {  // k_scan_slots
    kb[2] += kb[12];
    kb[12] = 0;
  }
  if (b->nest_fused) {  // k_nest_tile: both passes' bytes (the flag masks between them never exist)
    kb[22] = kb[13] + kb[14];
    kb[13] = kb[14] = 0;
  }
  kb[20] = b->copy_fused ? 0 : cp_bytes;            // k_values_copy
  kb[1] = dl_bytes + (b->copy_fused ? cp_bytes : 0);  // k_values_delta: DELTA pages (+ the fused copies)
  val_bytes -= snappy_direct_bytes;
  kb[8] = dict_bytes;                                   // k_values_dict: dictionary tiles
  kb[9] = val_bytes - cp_bytes - dl_bytes - dict_bytes;  // k_values: the other LDS kinds
  kb[11] = b->stats.snappy_kernel_bytes;
  memcpy(b->slot_bytes, kb, sizeof(kb));
  b->stats.levels_kernel_bytes = lvl_bytes;
  b->stats.values_kernel_bytes = val_bytes;
  b->stats.delta_kernel_bytes = dl_bytes;
  b->stats.output_bytes = out_bytes;
  b->stats.num_slots = slots;
  b->stats.num_values = values;
  b->timer.resolve();
  return first;
}

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
extern "C" {

int pqgpu_abi_version(void) { return PQGPU_ABI_VERSION; }

const char *pqgpu_status_string(int code) {
  switch (code) {
    case PQ_OK: return "ok";
    case PQ_ERR_EOF: return "EOF";
    case PQ_ERR_UNEXPECTED_EOF: return "unexpected EOF";
    case PQ_ERR_INVALID: return "invalid data";
    case PQ_ERR_UNSUPPORTED: return "unsupported";
    case PQ_ERR_DICT_INDEX: return "dict: invalid index";
    case PQ_ERR_CRC: return "CRC32 check failed";
    case PQ_ERR_DECOMPRESS: return "decompression failed";
    case PQ_ERR_THRIFT: return "thrift decode error";
    case PQ_ERR_RANGE: return "int32 out of range";
    case PQ_ERR_NOMEM: return "out of memory";
    case PQ_ERR_ARG: return "invalid argument";
    case PQ_ERR_HIP: return "HIP runtime error";
  }
  return "unknown";
}

int pqgpu_ctx_create(int device, pqgpu_ctx **out, pqgpu_error *err) {
  clear_err(err);
  *out = nullptr;
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || n <= device || device < 0) {
    set_err(err, PQ_ERR_HIP, -1, -1, "no HIP device available for the MI355X decoder");
    return PQ_ERR_HIP;
  }
  HIPCHECK(hipSetDevice(device), err);
  pqgpu_ctx *c = new pqgpu_ctx();
  c->device = device;
  e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->copy, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->delta, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->aux, hipStreamNonBlocking);
  if (e != hipSuccess) {
    if (c->stream) (void)hipStreamDestroy(c->stream);
    if (c->side) (void)hipStreamDestroy(c->side);
    if (c->copy) (void)hipStreamDestroy(c->copy);
    if (c->delta) (void)hipStreamDestroy(c->delta);
    delete c;
    set_err(err, PQ_ERR_HIP, -1, -1, hipGetErrorString(e));
    return PQ_ERR_HIP;
  }
  *out = c;
  return PQ_OK;
}

void pqgpu_ctx_destroy(pqgpu_ctx *c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  if (c->side) (void)hipStreamDestroy(c->side);
  if (c->copy) (void)hipStreamDestroy(c->copy);
  if (c->delta) (void)hipStreamDestroy(c->delta);
  if (c->aux) (void)hipStreamDestroy(c->aux);
  c->scratch_release();
  delete c;
}

int pqgpu_file_open(const uint8_t *buf, size_t len, pqgpu_file **out, pqgpu_error *err) {
  clear_err(err);
  *out = nullptr;
  pqgpu_file *f = new pqgpu_file();
  Status st = OpenFile(buf, (int64_t)len, &f->meta);
  if (!st.ok()) {
    set_err(err, st.code, -1, -1, "reading file meta data failed: " + st.msg);
    delete f;
    return st.code;
  }
  f->buf = buf;
  f->len = (int64_t)len;
  *out = f;
  return PQ_OK;
}

void pqgpu_file_close(pqgpu_file *f) { delete f; }
const uint8_t *pqgpu_file_bytes(const pqgpu_file *f) { return f ? f->buf : nullptr; }
size_t pqgpu_file_len(const pqgpu_file *f) { return f ? (size_t)f->len : 0; }
int pqgpu_file_num_row_groups(const pqgpu_file *f) { return (int)f->meta.row_groups.size(); }
int pqgpu_file_num_columns(const pqgpu_file *f) { return (int)f->meta.leaves.size(); }
int64_t pqgpu_file_row_group_num_rows(const pqgpu_file *f, int rg) {
  if (rg < 0 || rg >= (int)f->meta.row_groups.size()) return -1;
  return f->meta.row_groups[(size_t)rg].num_rows;
}

int pqgpu_file_column(const pqgpu_file *f, int col, pqgpu_column_info *out) {
  if (col < 0 || col >= (int)f->meta.leaves.size()) return PQ_ERR_ARG;
  const Leaf &l = f->meta.leaves[(size_t)col];
  memset(out, 0, sizeof(*out));
  out->physical_type = l.type;
  out->type_length = l.type_length;
  out->max_def = l.max_def;
  out->max_rep = l.max_rep;
  out->repetition = l.rep;
  snprintf(out->path, sizeof(out->path), "%s", l.path.c_str());
  out->num_groups = (int32_t)std::min<size_t>(l.group_def.size(), PQGPU_MAX_NEST + 1);  // > MAX: not produced
  for (size_t g = 0; g < l.group_def.size() && g < PQGPU_MAX_NEST; g++) {
    out->group_def[g] = l.group_def[g];
    out->group_depth[g] = l.group_depth[g];
    out->group_node[g] = l.group_node[g];
  }
  for (size_t k = 0; k < l.list_def.size() && k < PQGPU_MAX_NEST; k++) {
    out->list_def[k] = l.list_def[k];
    out->list_null_def[k] = l.list_null_def[k];
    out->list_node[k] = l.list_node[k];
  }
  return PQ_OK;
}

int pqgpu_file_chunk_meta(const pqgpu_file *f, int rg, int col, pqgpu_chunk_meta *out, pqgpu_error *err) {
  clear_err(err);
  if (rg < 0 || rg >= (int)f->meta.row_groups.size() || col < 0 || col >= (int)f->meta.leaves.size()) {
    set_err(err, PQ_ERR_ARG, -1, -1, "row group or column out of range");
    return PQ_ERR_ARG;
  }
  const RowGroup &g = f->meta.row_groups[(size_t)rg];
  if ((int)g.cols.size() <= col) {  // readRowGroupData chunk_reader.go:383-385
    set_err(err, PQ_ERR_INVALID, -1, -1, "column index is out of bounds");
    return PQ_ERR_INVALID;
  }
  const ColumnChunkMeta &c = g.cols[(size_t)col];
  if (!c.has_meta) {
    set_err(err, PQ_ERR_INVALID, -1, -1, "missing meta data for Column");
    return PQ_ERR_INVALID;
  }
  memset(out, 0, sizeof(*out));
  out->physical_type = c.type;
  out->codec = c.codec;
  out->num_values = c.num_values;
  out->total_compressed_size = c.total_compressed;
  out->data_page_offset = c.data_page_offset;
  out->dictionary_page_offset = c.has_dict_offset ? c.dict_offset : -1;
  out->has_file_path = c.has_file_path;
  return PQ_OK;
}

int pqgpu_batch_create(pqgpu_ctx *ctx, pqgpu_batch **out, pqgpu_error *err) {
  clear_err(err);
  // ctx == NULL gives a plan-only batch: page headers are walked and
  // validated (add_chunk) but upload/decode report PQ_ERR_HIP.
  pqgpu_batch *b = new pqgpu_batch();
  b->ctx = ctx;
  b->stage.pinned = ctx != nullptr;  // plan-only batches stage in pageable memory
  *out = b;
  return PQ_OK;
}

static void free_payloads(pqgpu_batch *b) {
  for (auto &hc : b->chunks) {
    if (hc.payload_own && hc.payload) (void)hipFree(hc.payload);
    hc.payload = nullptr;
    hc.payload_cap = 0;
    hc.payload_own = false;
  }
}

void pqgpu_batch_destroy(pqgpu_batch *b) {
  if (!b) return;
  if (!b->ctx) { delete b; return; }
  (void)hipSetDevice(b->ctx->device);
  (void)hipStreamSynchronize(b->ctx->stream);
  (void)hipStreamSynchronize(b->ctx->side);
  (void)hipStreamSynchronize(b->ctx->copy);
  (void)hipStreamSynchronize(b->ctx->delta);  // an error return inside decode_impl can leave forked work here
  (void)hipStreamSynchronize(b->ctx->aux);
  free_payloads(b);
  if (b->ev_fork) (void)hipEventDestroy(b->ev_fork);
  if (b->ev_join) (void)hipEventDestroy(b->ev_join);
  if (b->ev_copy) (void)hipEventDestroy(b->ev_copy);
  if (b->ev_copy_join) (void)hipEventDestroy(b->ev_copy_join);
  if (b->ev_delta_join) (void)hipEventDestroy(b->ev_delta_join);
  if (b->ev_levels) (void)hipEventDestroy(b->ev_levels);
  for (auto &e : b->ev_snap)
    if (e) (void)hipEventDestroy(e);
  if (b->ev_nest_join) (void)hipEventDestroy(b->ev_nest_join);
  for (hipEvent_t ev : {b->ev_lv_fork, b->ev_lv_join, b->ev_aux_fork, b->ev_aux_join})
    if (ev) (void)hipEventDestroy(ev);
  if (b->d_arena) (void)hipFree(b->d_arena);
  if (b->d_payload) (void)hipFree(b->d_payload);
  if (b->d_stage) (void)hipFree(b->d_stage);
  b->timer.destroy();
  delete b;
}

int pqgpu_batch_reset(pqgpu_batch *b) {
  if (b->ctx) {
    (void)hipStreamSynchronize(b->ctx->stream);
    (void)hipStreamSynchronize(b->ctx->side);  // forked work of a decode that returned early
    (void)hipStreamSynchronize(b->ctx->copy);
    (void)hipStreamSynchronize(b->ctx->delta);
    (void)hipStreamSynchronize(b->ctx->aux);
    if (b->last_stream) (void)hipStreamSynchronize(b->last_stream);  // an H2D copy may still read the stage
    free_payloads(b);
  }
  b->ds_pending = false;
  b->chunks.clear();
  b->pages.clear();
  b->ba_delta.clear();
  b->snappy.clear();
  b->gathers.clear();
  b->stage.clear();
  b->uploaded = b->decoded = false;
  b->force_serial = spec_disabled();
  b->stats = pqgpu_batch_stats{};
  return PQ_OK;
}

int pqgpu_batch_add_chunk(pqgpu_batch *b, const uint8_t *file_bytes, size_t file_len, const pqgpu_column_info *col,
                          const pqgpu_chunk_meta *meta, int validate_crc, int32_t *chunk_id, pqgpu_error *err) {
  if (!b || !file_bytes || !col || !meta) {
    set_err(err, PQ_ERR_ARG, -1, -1, "null argument");
    return PQ_ERR_ARG;
  }
  return add_chunk_impl(b, file_bytes, (int64_t)file_len, col, meta, validate_crc, chunk_id, err);
}

int pqgpu_batch_add_file_chunk(pqgpu_batch *b, const pqgpu_file *f, int rg, int col, int validate_crc,
                               int32_t *chunk_id, pqgpu_error *err) {
  pqgpu_column_info ci;
  pqgpu_chunk_meta cm;
  if (pqgpu_file_column(f, col, &ci)) {
    set_err(err, PQ_ERR_ARG, -1, -1, "column out of range");
    return PQ_ERR_ARG;
  }
  int e = pqgpu_file_chunk_meta(f, rg, col, &cm, err);
  if (e) {
    // still assign a chunk id so the caller can query the error in batch order
    int32_t id = (int32_t)b->chunks.size();
    if (chunk_id) *chunk_id = id;
    b->chunks.emplace_back();
    HostChunk &hc = b->chunks.back();
    hc.col = ci;
    hc.first_page = (uint32_t)b->pages.size();
    if (err) { err->chunk = id; hc.err = *err; }
    return e;
  }
  // the chunk's staged bytes are about its compressed size (SNAPPY data pages stay compressed)
  b->stage.reserve(b->stage.size() + (size_t)std::max<int64_t>(cm.total_compressed_size, 0) + 4096);
  return add_chunk_impl(b, f->buf, f->len, &ci, &cm, validate_crc, chunk_id, err);
}

int pqgpu_parse_page_header(const uint8_t *buf, size_t len, pqgpu_page_header *out, int64_t *consumed) {
  PageHeader ph;
  int64_t c = 0;
  const bool ok = buf && ParsePageHeader(buf, (int64_t)len, &ph, &c);
  if (consumed) *consumed = c;
  if (!ok) return PQ_ERR_THRIFT;
  PageIxEntry x{};
  x.hdr_len = (int32_t)c;
  x.type = ph.type; x.usize = ph.usize; x.csize = ph.csize; x.crc = ph.crc;
  x.flags = (ph.has_crc ? IXF_CRC : 0) | (ph.has_dph ? IXF_DPH : 0) | (ph.has_dict ? IXF_DICT : 0) |
            (ph.has_dph2 ? IXF_DPH2 : 0) | (ph.dph2.is_compressed ? IXF_COMPRESSED : 0);
  x.dph[0] = ph.dph.num_values; x.dph[1] = ph.dph.encoding; x.dph[2] = ph.dph.def_enc; x.dph[3] = ph.dph.rep_enc;
  x.dict[0] = ph.dict.num_values; x.dict[1] = ph.dict.encoding;
  x.dph2[0] = ph.dph2.num_values; x.dph2[1] = ph.dph2.num_nulls; x.dph2[2] = ph.dph2.num_rows;
  x.dph2[3] = ph.dph2.encoding; x.dph2[4] = ph.dph2.def_len; x.dph2[5] = ph.dph2.rep_len;
  if (out) to_public(x, out);
  return PQ_OK;
}

int pqgpu_page_index_build(pqgpu_ctx *ctx, const void *dev_bytes, int64_t file_offset, int64_t len,
                           const pqgpu_chunk_meta *metas, int32_t n_chunks, int32_t validate_crc, void *stream,
                           pqgpu_page_index **out, pqgpu_error *err) {
  clear_err(err);
  if (!ctx || !out || (n_chunks > 0 && (!metas || !dev_bytes)) || n_chunks < 0 || len < 0 ||
      ((uintptr_t)dev_bytes & 15)) {
    set_err(err, PQ_ERR_ARG, -1, -1, "page index: bad argument (dev_bytes must be 16-byte aligned)");
    return PQ_ERR_ARG;
  }
  auto t0 = std::chrono::steady_clock::now();
  HIPCHECK(hipSetDevice(ctx->device), err);
  hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
  auto ix = std::make_unique<pqgpu_page_index>();
  ix->dev = (uint64_t)(uintptr_t)dev_bytes;
  ix->file_off = file_offset;
  ix->len = len;
  ix->validate_crc = validate_crc;
  ix->metas.assign(metas, metas + n_chunks);
  ix->chunks.resize(n_chunks);
  uint64_t cap = 4096;
  // test knobs (tests/test_page_index.py): PQ_IX_CAP forces the first table capacity (drives the
  // grow path; PQ_IX_NOGROW=1 the overflow path)
  const char *cap_env = getenv("PQ_IX_CAP");
  const bool no_grow = getenv("PQ_IX_NOGROW") && atoi(getenv("PQ_IX_NOGROW")) == 1;  // with PQ_IX_CAP
  for (int32_t c = 0; c < n_chunks; c++) {
    const pqgpu_chunk_meta &m = metas[c];
    PageIxChunk &k = ix->chunks[c];
    memset(&k, 0, sizeof(k));
    k.start = m.dictionary_page_offset >= 0 ? m.dictionary_page_offset : m.data_page_offset;
    k.data_off = m.data_page_offset;
    k.dict_off = m.dictionary_page_offset;
    k.total = m.has_file_path ? 0 : m.total_compressed_size;  // a chunk in another file: host error path
    cap += 64 + (uint64_t)std::max<int64_t>(k.total, 0) / 4096;
  }
  if (n_chunks == 0) { *out = ix.release(); return PQ_OK; }
  if (cap_env) cap = std::max<uint64_t>(1, strtoull(cap_env, nullptr, 10));
  // table capacity: a page per 4 KiB plus 64 per chunk; a walk that outgrows it is rerun larger.
  // The chunk table rides in the kernel arguments; the count, the per-chunk results and the table
  // come back by device-to-host copies after the stream has drained, from hipMalloc'd scratch.
  const size_t res_bytes = align_up((uint64_t)n_chunks * sizeof(uint4), 256);
  uint32_t n = 0;
  for (int attempt = 0;; attempt++) {
    cap = std::min<uint64_t>(cap, 1u << 26);
    size_t dcap = 0;
    const size_t bytes = 256 + res_bytes + cap * sizeof(PageIxEntry);
    void *d = ctx->scratch_get(bytes, &dcap);  // hipMalloc'd, never stream-ordered
    if (!d) HIPCHECK(hipErrorOutOfMemory, err);
    uint8_t *D = (uint8_t *)d;
    uint32_t *d_n = (uint32_t *)D;
    uint4 *d_res = (uint4 *)(D + 256);
    PageIxEntry *d_tab = (PageIxEntry *)(D + 256 + res_bytes);
    const uint32_t gen = ctx->next_ix_gen();
    ix->gen = gen;
    hipError_t he = launch_page_walk((const uint8_t *)dev_bytes, len, file_offset, ix->chunks.data(), (uint32_t)n_chunks,
                                     d_res, d_tab, d_n, (uint32_t)cap, validate_crc, gen, s);
    if (he == hipSuccess) he = hipStreamSynchronize(s);
    // Every chunk's walk must have reported (its result carries this build's generation) before the
    // count and the table are read. A missing marker is re-read after another drain of the stream,
    // a bounded number of times; the polls and the chunks that never reported are kept in the index
    // (pqgpu_page_index_stats), and such a chunk is walked by the host.
    std::vector<uint4> r((size_t)n_chunks);
    int polls = 0;
    for (;; polls++) {
      if (he == hipSuccess) he = hipMemcpyAsync(r.data(), d_res, (size_t)n_chunks * sizeof(uint4), hipMemcpyDeviceToHost, s);
      if (he == hipSuccess) he = hipStreamSynchronize(s);
      if (he != hipSuccess) break;
      bool all = true;
      for (int32_t c = 0; c < n_chunks && all; c++) all = r[c].w == gen;
      if (all || polls >= 20) break;
      std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
    ix->polls += polls;
    if (he == hipSuccess) he = hipMemcpyAsync(&n, d_n, 4, hipMemcpyDeviceToHost, s);
    if (he == hipSuccess) he = hipStreamSynchronize(s);
    const bool grow = he == hipSuccess && n > cap && cap < (1u << 26) && attempt < (no_grow ? 0 : 3);
    if (he == hipSuccess && !grow) {
      ix->unreported = 0;
      for (int32_t c = 0; c < n_chunks; c++) {
        const bool rep = r[c].w == gen;  // a chunk that never reported stays with the host
        ix->unreported += !rep;
        ix->chunks[c].status = rep ? r[c].x : IX_FALLBACK;
        ix->chunks[c].npages = rep ? r[c].y : 0;
        ix->chunks[c].fail_page = r[c].z;
      }
      if (n > cap) {
        // the table overflowed and cannot grow: slots reserved by failed flushes were never written,
        // so no entry is trusted and every chunk is walked by the host
        ix->overflowed = 1;
        ix->entries.clear();
        for (int32_t c = 0; c < n_chunks; c++) ix->chunks[c].status = IX_FALLBACK;
      } else {
        ix->entries.resize(n);
        if (n) he = hipMemcpyAsync(ix->entries.data(), d_tab, (size_t)n * sizeof(PageIxEntry), hipMemcpyDeviceToHost, s);
        if (he == hipSuccess) he = hipStreamSynchronize(s);
      }
    }
    if (he == hipSuccess) he = hipStreamSynchronize(s);  // the scratch is free for the next build
    ctx->scratch_put(d, dcap);
    HIPCHECK(he, err);
    if (!grow) break;
    cap = (uint64_t)n * 2 + 4096;
  }
  // entries stamped by another build (scratch reused: a slot this build reserved but whose store
  // never landed) or of a chunk id outside the build cannot come from this build's walk: dropped.
  // The per-chunk count check below then sends such a chunk to the host walk.
  {
    const uint32_t gen_ok = ix->gen;
    const size_t before = ix->entries.size();
    ix->entries.erase(std::remove_if(ix->entries.begin(), ix->entries.end(),
                                     [&](const PageIxEntry &x) { return x.gen != gen_ok || x.chunk >= (uint32_t)n_chunks; }),
                      ix->entries.end());
    ix->stale = (int32_t)(before - ix->entries.size());
  }
  // group by chunk in page order (a chunk's entries were reserved in increasing order)
  std::vector<PageIxEntry> &e = ix->entries;
  std::stable_sort(e.begin(), e.end(), [](const PageIxEntry &a, const PageIxEntry &b) {
    return a.chunk != b.chunk ? a.chunk < b.chunk : a.seq < b.seq;
  });
  ix->first.assign(n_chunks + 1, 0);
  for (const auto &x : e) ix->first[x.chunk + 1]++;
  for (int32_t c = 0; c < n_chunks; c++) ix->first[c + 1] += ix->first[c];
  for (int32_t c = 0; c < n_chunks; c++)  // a chunk that fell back mid-walk keeps no entries
    if (ix->chunks[c].status != IX_OK || ix->first[c + 1] - ix->first[c] != ix->chunks[c].npages)
      ix->chunks[c].status = IX_FALLBACK;
  ix->walk_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  *out = ix.release();
  return PQ_OK;
}

int pqgpu_page_index_chunk(const pqgpu_page_index *ix, int32_t chunk, int32_t *num_pages, int32_t *status) {
  if (!ix || chunk < 0 || chunk >= (int32_t)ix->chunks.size()) return PQ_ERR_ARG;
  const bool ok = ix->chunks[chunk].status == IX_OK;
  if (num_pages) *num_pages = ok ? (int32_t)(ix->first[chunk + 1] - ix->first[chunk]) : 0;
  if (status) *status = ok ? PQGPU_IX_OK : PQGPU_IX_FALLBACK;
  return PQ_OK;
}

int pqgpu_page_index_page(const pqgpu_page_index *ix, int32_t chunk, int32_t k, pqgpu_page_header *out) {
  int32_t np = 0, st = 0;
  if (pqgpu_page_index_chunk(ix, chunk, &np, &st) || k < 0 || k >= np || !out) return PQ_ERR_ARG;
  to_public(ix->entries[ix->first[chunk] + k], out);
  return PQ_OK;
}

double pqgpu_page_index_walk_ms(const pqgpu_page_index *ix) { return ix ? ix->walk_ms : 0.0; }

int pqgpu_page_index_stats(const pqgpu_page_index *ix, int32_t *polls, int32_t *unreported, int32_t *fallback_chunks,
                           int32_t *overflowed, int32_t *stale_entries) {
  if (!ix) return PQ_ERR_ARG;
  if (stale_entries) *stale_entries = ix->stale;
  int32_t fb = 0;
  for (const auto &k : ix->chunks) fb += k.status != IX_OK;
  if (polls) *polls = ix->polls;
  if (unreported) *unreported = ix->unreported;
  if (fallback_chunks) *fallback_chunks = fb;
  if (overflowed) *overflowed = ix->overflowed;
  return PQ_OK;
}

void pqgpu_page_index_destroy(pqgpu_page_index *ix) { delete ix; }

int pqgpu_batch_add_indexed_chunk(pqgpu_batch *b, const pqgpu_page_index *ix, int32_t ix_chunk,
                                  const uint8_t *file_bytes, size_t file_len, const pqgpu_column_info *col,
                                  int validate_crc, int32_t *chunk_id, pqgpu_error *err) {
  if (!b || !ix || !file_bytes || !col || ix_chunk < 0 || ix_chunk >= (int32_t)ix->chunks.size()) {
    set_err(err, PQ_ERR_ARG, -1, -1, "null argument or chunk out of range");
    return PQ_ERR_ARG;
  }
  const pqgpu_chunk_meta &cm = ix->metas[ix_chunk];
  b->stage.reserve(b->stage.size() + 4096);
  if (ix->chunks[ix_chunk].status != IX_OK)  // the walk did not take it: the host walks the chunk
    return add_chunk_impl(b, file_bytes, (int64_t)file_len, col, &cm, validate_crc, chunk_id, err);
  IxChunkView v{ix->entries.data() + ix->first[ix_chunk], ix->first[ix_chunk + 1] - ix->first[ix_chunk], ix->dev,
                ix->file_off, ix->len};
  return add_chunk_impl(b, file_bytes, (int64_t)file_len, col, &cm, validate_crc, chunk_id, err, &v);
}

int pqgpu_batch_add_indexed_file_chunk(pqgpu_batch *b, const pqgpu_page_index *ix, int32_t ix_chunk,
                                       const pqgpu_file *f, int col, int validate_crc, int32_t *chunk_id,
                                       pqgpu_error *err) {
  pqgpu_column_info ci;
  if (!f || pqgpu_file_column(f, col, &ci)) {
    set_err(err, PQ_ERR_ARG, -1, -1, "column out of range");
    return PQ_ERR_ARG;
  }
  return pqgpu_batch_add_indexed_chunk(b, ix, ix_chunk, f->buf, f->len, &ci, validate_crc, chunk_id, err);
}

#define NEED_CTX(b, err)                                                              \
  do {                                                                                \
    if (!(b)->ctx) {                                                                  \
      set_err(err, PQ_ERR_HIP, -1, -1, "plan-only batch: no device context");        \
      return PQ_ERR_HIP;                                                              \
    }                                                                                 \
  } while (0)

static hipStream_t pick_stream(pqgpu_batch *b, void *stream) {
  return stream ? (hipStream_t)stream : b->ctx->stream;
}

int pqgpu_batch_upload(pqgpu_batch *b, void *stream, pqgpu_error *err) {
  clear_err(err);
  NEED_CTX(b, err);
  HIPCHECK(hipSetDevice(b->ctx->device), err);
  return build_and_upload(b, pick_stream(b, stream), err);
}

int pqgpu_batch_decode(pqgpu_batch *b, void *stream, pqgpu_error *err) {
  clear_err(err);
  NEED_CTX(b, err);
  HIPCHECK(hipSetDevice(b->ctx->device), err);
  return decode_impl(b, pick_stream(b, stream), err);
}

int pqgpu_batch_wait(pqgpu_batch *b, void *stream, pqgpu_error *err) {
  clear_err(err);
  if (!b->ctx) return PQ_OK;  // plan-only: nothing runs on a device
  HIPCHECK(hipSetDevice(b->ctx->device), err);
  const hipStream_t s = pick_stream(b, stream);
  HIPCHECK(join_deferred(b, s), err);
  HIPCHECK(hipStreamSynchronize(s), err);
  return PQ_OK;
}

int pqgpu_batch_sync(pqgpu_batch *b, void *stream, pqgpu_error *err) {
  if (!b->ctx) {  // plan-only: report the first host-side (readPages) error
    clear_err(err);
    for (auto &hc : b->chunks)
      if (hc.err.code) { if (err) *err = hc.err; return hc.err.code; }
    return PQ_OK;
  }
  HIPCHECK(hipSetDevice(b->ctx->device), err);
  return sync_impl(b, pick_stream(b, stream), err);
}

int pqgpu_batch_num_chunks(const pqgpu_batch *b) { return (int)b->chunks.size(); }

int pqgpu_batch_chunk_status(const pqgpu_batch *b, int32_t id, pqgpu_error *err) {
  if (id < 0 || id >= (int32_t)b->chunks.size()) {
    set_err(err, PQ_ERR_ARG, -1, -1, "chunk id out of range");
    return PQ_ERR_ARG;
  }
  const HostChunk &hc = b->chunks[(size_t)id];
  const pqgpu_error &e = hc.err.code ? hc.err : hc.dev_err;
  if (err) *err = e;
  return e.code;
}

int pqgpu_batch_chunk_pages(const pqgpu_batch *b, int32_t id, int32_t *num_pages, int64_t *slot_first,
                            int64_t *slot_count, int64_t *value_first, int64_t *value_count, int32_t cap,
                            pqgpu_error *err) {
  clear_err(err);
  if (!b || id < 0 || id >= (int32_t)b->chunks.size() || !num_pages) {
    set_err(err, PQ_ERR_ARG, id, -1, "bad chunk id");
    return PQ_ERR_ARG;
  }
  if (!b->decoded || b->page_nn_out.size() != b->pages.size()) {
    set_err(err, PQ_ERR_ARG, id, -1, "batch not decoded and synced");
    return PQ_ERR_ARG;
  }
  const HostChunk &hc = b->chunks[id];
  *num_pages = (int32_t)hc.num_pages;
  if ((int64_t)hc.num_pages > cap) return PQ_OK;  // size query
  for (uint32_t k = 0; k < hc.num_pages; k++) {
    const uint32_t p = hc.first_page + k;
    if (slot_first) slot_first[k] = (int64_t)b->pages[p].slot_base;
    if (slot_count) slot_count[k] = (int64_t)b->pages[p].num_slots;
    if (value_first) value_first[k] = (int64_t)b->page_vbase_out[p];
    if (value_count) value_count[k] = (int64_t)b->page_nn_out[p];
  }
  return PQ_OK;
}

int pqgpu_batch_chunk_result(const pqgpu_batch *b, int32_t id, pqgpu_chunk_result *out, pqgpu_error *err) {
  int e = pqgpu_batch_chunk_status(b, id, err);
  memset(out, 0, sizeof(*out));
  if (e && (e == PQ_ERR_ARG || !b->chunks[(size_t)id].partial)) return e;
  const HostChunk &hc = b->chunks[(size_t)id];
  uint8_t *A = b->d_arena;
  out->num_slots = e ? hc.part_slots : (int64_t)hc.num_slots;
  out->num_values = e ? hc.part_nn : hc.nn;
  out->num_records = e ? hc.part_records : hc.records;
  out->payload_bytes = e ? hc.part_payload : hc.payload_bytes;
  out->physical_type = hc.col.physical_type;
  out->value_width = hc.value_width;
  out->max_def = hc.col.max_def;
  out->max_rep = hc.col.max_rep;
  out->values = hc.o_values ? A + hc.o_values : nullptr;
  out->offsets = hc.o_offsets ? (int32_t *)(A + hc.o_offsets) : nullptr;
  out->payload = hc.payload;
  out->def_levels = hc.o_def ? A + hc.o_def : nullptr;
  out->rep_levels = hc.o_rep ? A + hc.o_rep : nullptr;
  out->validity = hc.o_valid ? (uint32_t *)(A + hc.o_valid) : nullptr;
  out->list_offsets = hc.o_lists ? (int32_t *)(A + hc.o_lists) : nullptr;
  out->dictionary_page = hc.has_dict ? 1 : 0;
  out->nest_levels = e ? 0 : (int32_t)hc.nest;  // a failing chunk's prefix carries no nested arrays
  for (uint32_t k = 0; k < PQGPU_MAX_NEST && !e; k++) {
    out->num_lists[k] = hc.num_lists[k];
    out->lvl_offsets[k] = hc.o_lvl_off[k] ? (int32_t *)(A + hc.o_lvl_off[k]) : nullptr;
    out->lvl_validity[k] = hc.o_lvl_valid[k] ? (uint32_t *)(A + hc.o_lvl_valid[k]) : nullptr;
  }
  out->num_elements = e ? 0 : hc.num_elems;
  out->element_validity = (!e && hc.o_elem_valid) ? (uint32_t *)(A + hc.o_elem_valid) : nullptr;
  out->num_groups = e ? 0 : (int32_t)hc.ngroups;
  for (uint32_t g = 0; g < hc.ngroups && !e; g++) {
    const int j = hc.col.group_depth[g], a = hc.grp_alias[g];
    out->group_entries[g] = hc.col.max_rep == 0 ? (int64_t)hc.num_slots : (j < hc.col.max_rep ? hc.num_lists[j] : hc.num_elems);
    out->group_validity[g] = a < 0 ? (uint32_t *)(A + hc.o_grp_valid[g])
                             : a < 8 ? out->lvl_validity[a] : a == 8 ? out->element_validity : out->validity;
  }
  if (!e && hc.share_from >= 0) {  // common ancestors shared with another leaf (checked equal)
    pqgpu_chunk_result o;
    pqgpu_error e2;
    if (pqgpu_batch_chunk_result(b, hc.share_from, &o, &e2) == PQ_OK) {
      for (uint32_t k = 0; k < hc.share_lists; k++) {
        out->lvl_offsets[k] = o.lvl_offsets[k];
        out->lvl_validity[k] = o.lvl_validity[k];
      }
      for (uint32_t g = 0; g < hc.share_groups; g++) out->group_validity[g] = o.group_validity[g];
    }
  }
  return e;
}

int pqgpu_batch_copy_nested(const pqgpu_batch *b, int32_t id, int32_t level, int32_t *offsets, uint32_t *validity,
                            uint32_t *element_validity, pqgpu_error *err) {
  pqgpu_chunk_result r;
  const int e = pqgpu_batch_chunk_result(b, id, &r, err);
  if (e) return e;
  NEED_CTX(b, err);
  if (level < 0 || level >= r.nest_levels) {
    set_err(err, PQ_ERR_ARG, id, -1, "no such list level");
    return PQ_ERR_ARG;
  }
  HIPCHECK(hipSetDevice(b->ctx->device), err);
  const int64_t n = r.num_lists[level];
  if (offsets) HIPCHECK(hipMemcpy(offsets, r.lvl_offsets[level], (size_t)(n + 1) * 4, hipMemcpyDeviceToHost), err);
  if (validity) HIPCHECK(hipMemcpy(validity, r.lvl_validity[level], (size_t)((n + 31) / 32) * 4, hipMemcpyDeviceToHost), err);
  if (element_validity)
    HIPCHECK(hipMemcpy(element_validity, r.element_validity, (size_t)((r.num_elements + 31) / 32) * 4,
                       hipMemcpyDeviceToHost),
             err);
  return PQ_OK;
}

int pqgpu_batch_copy_group(const pqgpu_batch *b, int32_t id, int32_t group, uint32_t *validity, pqgpu_error *err) {
  pqgpu_chunk_result r;
  const int e = pqgpu_batch_chunk_result(b, id, &r, err);
  if (e) return e;
  NEED_CTX(b, err);
  if (group < 0 || group >= r.num_groups) {
    set_err(err, PQ_ERR_ARG, id, -1, "no such group");
    return PQ_ERR_ARG;
  }
  HIPCHECK(hipSetDevice(b->ctx->device), err);
  const size_t n = (size_t)((r.group_entries[group] + 31) / 32) * 4;
  if (validity && n) HIPCHECK(hipMemcpy(validity, r.group_validity[group], n, hipMemcpyDeviceToHost), err);
  return PQ_OK;
}

static std::vector<std::string> path_parts(const char *p) {
  std::vector<std::string> v;
  std::string cur;
  for (const char *c = p; *c; c++) {
    if (*c == '.') { v.push_back(cur); cur.clear(); }
    else cur += *c;
  }
  v.push_back(cur);
  return v;
}

int pqgpu_batch_share_ancestors(pqgpu_batch *b, int32_t ia, int32_t ib, int32_t *equal, pqgpu_error *err) {
  clear_err(err);
  if (equal) *equal = 0;
  if (ia == ib) {
    set_err(err, PQ_ERR_ARG, ib, -1, "a leaf cannot share ancestors with itself");
    return PQ_ERR_ARG;
  }
  pqgpu_chunk_result ra, rb;
  int e = pqgpu_batch_chunk_result(b, ia, &ra, err);
  if (!e) e = pqgpu_batch_chunk_result(b, ib, &rb, err);
  if (e) return e;
  NEED_CTX(b, err);
  HostChunk &ha = b->chunks[(size_t)ia], &hb = b->chunks[(size_t)ib];
  // the common ancestors: the shared prefix of the two paths, short of either leaf
  const auto pa = path_parts(ha.col.path), pb = path_parts(hb.col.path);
  int32_t m = 0;
  while ((size_t)m + 1 < pa.size() && (size_t)m + 1 < pb.size() && pa[(size_t)m] == pb[(size_t)m]) m++;
  auto count_below = [m](const int32_t *node, int32_t n) {
    int32_t c = 0;
    while (c < n && node[c] < m) c++;
    return c;
  };
  const int32_t La = count_below(ha.col.list_node, std::min(ha.col.max_rep, PQGPU_MAX_NEST));
  const int32_t Lb = count_below(hb.col.list_node, std::min(hb.col.max_rep, PQGPU_MAX_NEST));
  const int32_t Ga = count_below(ha.col.group_node, std::min(ha.col.num_groups, PQGPU_MAX_NEST));
  const int32_t Gb = count_below(hb.col.group_node, std::min(hb.col.num_groups, PQGPU_MAX_NEST));
  bool consistent = La == Lb && Ga == Gb && (La == 0 || (ra.nest_levels >= La && rb.nest_levels >= La)) &&
                    (Ga == 0 || (ra.num_groups >= Ga && rb.num_groups >= Ga));
  for (int32_t k = 0; k < La && consistent; k++)
    consistent = ha.col.list_node[k] == hb.col.list_node[k] && ha.col.list_def[k] == hb.col.list_def[k] &&
                 ha.col.list_null_def[k] == hb.col.list_null_def[k];
  for (int32_t g = 0; g < Ga && consistent; g++)
    consistent = ha.col.group_node[g] == hb.col.group_node[g] && ha.col.group_def[g] == hb.col.group_def[g];
  if (!consistent) {
    set_err(err, PQ_ERR_ARG, ib, -1, "the two leaves' common ancestors differ in the schema");
    return PQ_ERR_ARG;
  }
  // every array pair compared on the device (one flag); entry counts first, on the host
  bool same = true;
  std::vector<std::tuple<const uint32_t *, const uint32_t *, uint64_t>> cmp;
  for (int32_t k = 0; k < La && same; k++) {
    same = ra.num_lists[k] == rb.num_lists[k];
    cmp.emplace_back((const uint32_t *)ra.lvl_offsets[k], (const uint32_t *)rb.lvl_offsets[k], (uint64_t)ra.num_lists[k] + 1);
    cmp.emplace_back(ra.lvl_validity[k], rb.lvl_validity[k], (uint64_t)(ra.num_lists[k] + 31) / 32);
  }
  for (int32_t g = 0; g < Ga && same; g++) {
    same = ra.group_entries[g] == rb.group_entries[g];
    cmp.emplace_back(ra.group_validity[g], rb.group_validity[g], (uint64_t)(ra.group_entries[g] + 31) / 32);
  }
  if (same && !cmp.empty()) {
    HIPCHECK(hipSetDevice(b->ctx->device), err);
    hipStream_t s = b->ctx->stream;
    size_t cap = 0;
    uint32_t *flag = (uint32_t *)b->ctx->scratch_get(256, &cap);
    if (!flag) HIPCHECK(hipErrorOutOfMemory, err);
    hipError_t he = hipMemsetAsync(flag, 0, 4, s);
    for (auto &x : cmp)
      if (he == hipSuccess && std::get<0>(x) != std::get<1>(x)) he = launch_words_differ(std::get<0>(x), std::get<1>(x), std::get<2>(x), flag, s);
    uint32_t h = 1;
    if (he == hipSuccess) he = hipMemcpyAsync(&h, flag, 4, hipMemcpyDeviceToHost, s);
    if (he == hipSuccess) he = hipStreamSynchronize(s);
    b->ctx->scratch_put(flag, cap);
    HIPCHECK(he, err);
    same = h == 0;
  }
  if (same) {
    // link ib to the nearest chunk of ia's chain that resolves levels [0, La) and groups [0, Ga) itself:
    // a chunk that shares at least that many from its own link hands out its link's arrays, so ib
    // can point past it (leaves linked in order, a -> b, b -> c, ..., then all point at a and
    // chunk_result's recursion stays as deep as the number of distinct sharing depths, <= 8).
    // Then walk the rest of the chain to keep the links acyclic: when it already reaches ib, the
    // arrays are equal and nothing is linked.
    int32_t to = ia;
    for (int32_t hops = 0; hops <= (int32_t)b->chunks.size(); hops++) {
      const HostChunk &ht = b->chunks[(size_t)to];
      if (ht.share_from < 0 || ht.share_from == ib || (int32_t)ht.share_lists < La || (int32_t)ht.share_groups < Ga) break;
      to = ht.share_from;
    }
    int32_t at = to;
    for (int32_t hops = 0; at >= 0 && hops <= (int32_t)b->chunks.size(); hops++) {
      if (at == ib) {
        if (equal) *equal = 1;
        return PQ_OK;
      }
      at = b->chunks[(size_t)at].share_from;
    }
    hb.share_from = to;
    hb.share_lists = (uint32_t)La;
    hb.share_groups = (uint32_t)Ga;
    if (equal) *equal = 1;
  }
  return PQ_OK;
}

int pqgpu_batch_copy_chunk(const pqgpu_batch *b, int32_t id, void *values, int32_t *offsets, uint8_t *payload,
                           uint8_t *def_levels, uint8_t *rep_levels, uint32_t *validity, int32_t *list_offsets,
                           pqgpu_error *err) {
  pqgpu_chunk_result r;
  const int e = pqgpu_batch_chunk_result(b, id, &r, err);
  if (e && !r.num_slots) return e;  // nothing decoded (a failing chunk's prefix is copied)
  NEED_CTX(b, err);
  HIPCHECK(hipSetDevice(b->ctx->device), err);
  auto cp = [&](void *dst, const void *src, size_t n) -> hipError_t {
    if (!dst || !src || !n) return hipSuccess;
    return hipMemcpy(dst, src, n, hipMemcpyDeviceToHost);
  };
  HIPCHECK(cp(values, r.values, (size_t)r.num_values * (size_t)r.value_width), err);
  HIPCHECK(cp(offsets, r.offsets, r.offsets ? (size_t)(r.num_values + 1) * 4 : 0), err);
  HIPCHECK(cp(payload, r.payload, (size_t)r.payload_bytes), err);
  HIPCHECK(cp(def_levels, r.def_levels, (size_t)r.num_slots), err);
  HIPCHECK(cp(rep_levels, r.rep_levels, (size_t)r.num_slots), err);
  HIPCHECK(cp(validity, r.validity, (size_t)((r.num_slots + 31) / 32) * 4), err);
  HIPCHECK(cp(list_offsets, r.list_offsets, r.list_offsets ? (size_t)(r.num_records + 1) * 4 : 0), err);
  return e;
}

int pqgpu_dev_alloc(pqgpu_ctx *ctx, size_t bytes, void **out, pqgpu_error *err) {
  clear_err(err);
  if (!ctx || !out) { set_err(err, PQ_ERR_ARG, -1, -1, "null argument"); return PQ_ERR_ARG; }
  *out = nullptr;
  HIPCHECK(hipSetDevice(ctx->device), err);
  HIPCHECK(hipMalloc(out, std::max<size_t>(bytes, 1)), err);
  return PQ_OK;
}

void pqgpu_dev_free(pqgpu_ctx *ctx, void *p) {
  if (!ctx || !p) return;
  (void)hipSetDevice(ctx->device);
  (void)hipFree(p);
}

int pqgpu_copy(pqgpu_ctx *ctx, void *dst, const void *src, size_t bytes, pqgpu_error *err) {
  clear_err(err);
  if (!ctx) {
    set_err(err, PQ_ERR_ARG, -1, -1, "no device context");
    return PQ_ERR_ARG;
  }
  if (!bytes) return PQ_OK;
  HIPCHECK(hipSetDevice(ctx->device), err);
  HIPCHECK(hipMemcpy(dst, src, bytes, hipMemcpyDefault), err);
  HIPCHECK(hipDeviceSynchronize(), err);  // visible to kernels on every stream of the device
  return PQ_OK;
}

int pqgpu_batch_debug_counters(pqgpu_batch *b, uint64_t *out64, int reset) {
  if (!b->ctx || !b->d_arena) return PQ_ERR_ARG;
  (void)hipSetDevice(b->ctx->device);
  (void)join_deferred(b, b->ctx->stream);
  (void)hipStreamSynchronize(b->ctx->stream);
  if (hipMemcpy(out64, b->d_arena + b->o_dbg, 64 * 8, hipMemcpyDeviceToHost) != hipSuccess) return PQ_ERR_HIP;
  if (reset) (void)hipMemset(b->d_arena + b->o_dbg, 0, 64 * 8);
  return PQ_OK;
}

int pqgpu_batch_stats_get(const pqgpu_batch *b, pqgpu_batch_stats *out) {
  *out = b->stats;
  return PQ_OK;
}

int pqgpu_batch_kernel_timing(pqgpu_batch *b, int enable) {
  if (b->ctx) (void)join_deferred(b, b->ctx->stream);
  if (b->ctx) (void)hipStreamSynchronize(b->ctx->stream);
  b->timer.resolve();
  b->timer.enabled = enable != 0;
  for (int k = 0; k < PQGPU_TIMER_SLOTS; k++) { b->timer.total_ms[k] = 0; b->timer.launches[k] = 0; }
  return PQ_OK;
}

int pqgpu_batch_kernel_time(pqgpu_batch *b, double *avg_ms, int64_t *launches, char *name, size_t name_len) {
  (void)hipDeviceSynchronize();
  b->timer.resolve();
  const KernelTimer &t = b->timer;
  int best = -1;
  for (int k = 0; k < PQGPU_TIMER_SLOTS; k++)
    if (t.launches[k] && (best < 0 || t.total_ms[k] > t.total_ms[best])) best = k;
  if (best < 0) {
    if (avg_ms) *avg_ms = 0;
    if (launches) *launches = 0;
    if (name && name_len) name[0] = 0;
    return PQ_OK;
  }
  if (avg_ms) *avg_ms = t.total_ms[best] / (double)t.launches[best];
  if (launches) *launches = t.launches[best];
  if (name && name_len) snprintf(name, name_len, "%s", kTimerNames[best]);
  return PQ_OK;
}

int pqgpu_batch_kernel_bytes(const pqgpu_batch *b, int slot, int64_t *bytes) {
  if (!b || slot < 0 || slot >= PQGPU_TIMER_SLOTS || !bytes) return PQ_ERR_ARG;
  *bytes = b->slot_bytes[slot];
  return PQ_OK;
}

int pqgpu_batch_kernel_slot(pqgpu_batch *b, int slot, double *avg_ms, int64_t *launches, char *name,
                            size_t name_len) {
  if (!b || slot < 0 || slot >= PQGPU_TIMER_SLOTS) return PQ_ERR_ARG;
  (void)hipDeviceSynchronize();
  b->timer.resolve();
  const KernelTimer &t = b->timer;
  if (avg_ms) *avg_ms = t.launches[slot] ? t.total_ms[slot] / (double)t.launches[slot] : 0.0;
  if (launches) *launches = t.launches[slot];
  if (name && name_len) snprintf(name, name_len, "%s", kTimerNames[slot]);
  return PQ_OK;
}

}  // extern "C"
