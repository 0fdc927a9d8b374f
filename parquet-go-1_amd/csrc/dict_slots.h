// dict_slots.h — byte-array dictionary slot tables (k_dict_slots in bytearray.hip, and beside the
// run scan in k_scan_slots, kernels.hip): entry i at slots + (i << slot_shift) = [u32 length | bytes
// | zero pad], one thread per entry (page_dict.go:35-72: the dictionary page's materialisation,
// redone every decode).
#pragma once
#include "dev_util.h"
#include "kernels.h"

namespace pq {

// Block bx of gx blocks over chunk c's entries.
DEV void dict_slots_block(const BatchDev &b, uint32_t c, uint32_t bx, uint32_t gx) {
  const ChunkDesc &cd = b.chunks[c];
  const uint32_t S = cd.slot_shift;
  const uint2 *ent = gp_u64<const uint2>(cd.dict_offsets);
  const uint8_t *raw = gp_u64<const uint8_t>(cd.dict_raw);
  uint4 *slots = gp_u64<uint4>(cd.dict_slots);
  for (uint32_t i = bx * 256 + threadIdx.x; i < cd.dict_count; i += gx * 256) {
    const uint2 e = ent[i];
    const uint32_t n = e.y + 4;  // slot bytes in use; slot byte o holds entry byte o - 4
    for (uint32_t q = 0; q < (1u << S) / 16; q++) {
      uint32_t w[4];
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const uint32_t o = 16 * q + 4 * j;
        if (o == 0) { w[j] = e.y; continue; }
        const uint32_t x = o < n ? ld32(raw + e.x + (o - 4)) : 0u;
        w[j] = o + 4 <= n ? x : (o < n ? x & ((1u << (8 * (n - o))) - 1u) : 0u);
      }
      slots[((uint64_t)i << (S - 4)) + q] = make_uint4(w[0], w[1], w[2], w[3]);
    }
  }
}

}  // namespace pq
