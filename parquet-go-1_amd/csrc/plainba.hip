// plainba.hip — PLAIN BYTE_ARRAY pages (byteArrayPlainDecoder, type_bytearray.go:24-55): a page's
// values section is a chain of [u32 length | bytes] values, value k+1 starting where value k
// ends, so where any value starts is known only by walking the chain from the page start. This
// file walks it in parallel, by speculation verified afterwards:
//
//   k_pba_spec   one thread per 256-byte segment of a page's values section. The thread finds
//                the first position of its segment from which three consecutive values parse
//                (or one that ends exactly at the section end) — its guess of where the chain
//                enters the segment (segment 0 enters at 0) — and walks the values that START in
//                the segment from there, applying the reference's checks value by value (EOF,
//                short length, negative length, short payload). It records (entry, exit, values,
//                first error).
//   k_pba_fix    one wavefront per page: the true chain enters segment k where it left segment
//                k-1, so a segment is right iff its guessed entry equals its predecessor's exit
//                (or the chain jumps over the whole segment inside one long value). 64 segments
//                are checked at once; the first wrong one is re-walked from the true entry by the
//                wave, then the check resumes after it. Then a wave scan gives every segment's
//                first value index; the values before the page's limit (its non-null count, or
//                the first error on the true chain, reported with the reference's class at that
//                value) are the ones written.
//   k_pba_emit   one thread per segment again: walks its (verified) values and writes each one's
//                source address and length, which k_ba_emit turns into offsets and payload.
//
// Chains guessed from a wrong position almost always die within a value or two (a length read
// from inside a value's bytes points past the section), and a wrong guess only costs its
// segment a serial re-walk in k_pba_fix, never a wrong result. FIXED_LEN_BYTE_ARRAY pages laid
// out as byte arrays (type_length-byte values, no lengths) are written by k_pba_fix directly.
#include <hip/hip_runtime.h>

#include "dev_util.h"

namespace pq {

constexpr uint32_t kPbaSeg = 256;         // bytes per segment
constexpr uint32_t kPbaNone = 0xffffffffu;

struct PbaWalk {
  uint32_t exit;   // position after the last value that starts in the segment (or where it failed)
  uint32_t cnt;    // values that start in the segment and parse
  uint32_t err;    // 0, or the error class of the value after them
};

// The values starting in [pos, end) of section s[0, n) (the reference's loop body per value).
DEV PbaWalk pba_walk(const uint8_t *s, uint32_t n, uint32_t pos, uint32_t end) {
  PbaWalk w{pos, 0, 0};
  uint64_t p = pos;
  while (p < end) {
    if (p >= n) { w.err = PQ_ERR_EOF; break; }
    if (p + 4 > n) { w.err = PQ_ERR_UNEXPECTED_EOF; break; }
    const int32_t l = (int32_t)ld32(s + p);
    if (l < 0) { w.err = PQ_ERR_INVALID; break; }
    if (l > 0 && p + 4 >= n) { w.err = PQ_ERR_EOF; break; }
    if (p + 4 + (uint64_t)l > n) { w.err = PQ_ERR_UNEXPECTED_EOF; break; }
    p += 4 + (uint64_t)l;
    w.cnt++;
  }
  w.exit = (uint32_t)min<uint64_t>(p, 0xfffffff0ull);
  return w;
}

// Could the chain enter at q: three values parse from q, or the values from q end exactly at n.
DEV bool pba_candidate(const uint8_t *s, uint32_t n, uint32_t q) {
  uint64_t p = q;
  for (int h = 0; h < 3; h++) {
    if (p == n && h > 0) return true;
    if (p + 4 > n) return false;
    const int32_t l = (int32_t)ld32(s + p);
    if (l < 0 || p + 4 + (uint64_t)l > n) return false;
    p += 4 + (uint64_t)l;
  }
  return true;
}

struct PbaPage {
  const uint8_t *s;
  uint32_t n, k, nseg;
};

DEV PbaPage pba_page(const BatchDev &b, const uint32_t *pages, const uint32_t *seg0, uint32_t li, uint32_t seg) {
  const PageDesc &pd = b.pages[pages[li]];
  PbaPage x;
  x.s = gp_u64<const uint8_t>(pd.data) + pd.val_off;
  x.n = pd.val_len;
  x.k = seg - seg0[li];
  x.nseg = seg0[li + 1] - seg0[li];
  return x;
}

__global__ void __launch_bounds__(256) k_pba_spec(BatchDev b_in, const uint32_t *pages, const uint32_t *seg0,
                                                  const uint32_t *seg_page, uint4 *segs, uint32_t nseg) {
  const BatchDev b = global_view(b_in);
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= nseg) return;
  const uint32_t li = gp(seg_page)[g];
  const PbaPage x = pba_page(b, gp(pages), gp(seg0), li, g);
  const uint32_t lo = x.k * kPbaSeg, hi = lo + kPbaSeg;
  uint32_t c = x.k == 0 ? 0u : kPbaNone;
  for (uint32_t q = lo; c == kPbaNone && q < min(hi, x.n); q++)
    if (pba_candidate(x.s, x.n, q)) c = q;
  uint4 r = make_uint4(kPbaNone, 0u, 0u, 0u);
  if (c != kPbaNone) {
    const PbaWalk w = pba_walk(x.s, x.n, c, hi);
    r = make_uint4(c, w.exit, w.cnt, w.err);
  }
  gp(segs)[g] = r;
}

// One wave per PLAIN BYTE_ARRAY page: verify / repair the segments' entries, scan their value
// counts into first-value indices (segs[].w), report the first error on the true chain and
// store the page's limit (values to write).
__global__ void __launch_bounds__(64) k_pba_fix(BatchDev b_in, const uint32_t *pages_in, const uint32_t *seg0_in,
                                                uint4 *segs_in, uint32_t *limit) {
  const BatchDev b = global_view(b_in);
  const uint32_t *pages = gp(pages_in), *seg0 = gp(seg0_in);
  uint4 *segs = gp(segs_in);
  const uint32_t li = blockIdx.x, lane = lane_id(), p = pages[li];
  const PageDesc &pd = b.pages[p];
  const ChunkDesc &cd = b.chunks[pd.chunk];
  const uint8_t *s = gp_u64<const uint8_t>(pd.data) + pd.val_off;
  const uint32_t n = pd.val_len, nn = b.page_nn_v[p];
  const uint64_t vb = b.page_vbase[p];
  if (cd.type == T_FLBA && cd.type_length > 0) {  // fixed-length values: value v at v * type_length
    const uint32_t L = (uint32_t)cd.type_length;
    const uint32_t verr = n / L;  // the first value that does not fit: a partial one, or none left
    const uint32_t lim = min(nn, verr);
    if (verr < nn && lane == 0)
      report(b, pd.chunk, 1, pd.page_in_chunk, ST_VALUES, verr, n % L ? PQ_ERR_UNEXPECTED_EOF : PQ_ERR_EOF);
    for (uint32_t v = lane; v < lim; v += 64) {
      (gp_u64<uint64_t>(cd.ba_index))[vb + v] = (uint64_t)(s + (uint64_t)v * L);
      (gp_u64<int32_t>(cd.offsets))[vb + v + 1] = (int32_t)L;
    }
    if (lane == 0) limit[li] = lim;
    return;
  }
  const uint32_t base_seg = seg0[li], nseg = seg0[li + 1] - base_seg;
  uint32_t entry = 0;          // where the true chain enters the next window's first segment
  uint32_t v = 0;              // values on the true chain before it
  uint32_t lim = nn;           // values written
  bool done = false;
  for (uint32_t k0 = 0; k0 < nseg && !done; k0 += 64) {
    const uint32_t k = k0 + lane;
    const bool valid = k < nseg;
    uint4 r = valid ? segs[base_seg + k] : make_uint4(kPbaNone, 0u, 0u, 0u);
    const uint32_t hi = (k + 1) * kPbaSeg;
    uint32_t from = 0;  // first lane not yet known to be right
    for (;;) {
      // the true entry of each segment is its predecessor's exit (lane `from` uses `entry`)
      const uint32_t prev_exit = __shfl_up(r.y, 1);
      const uint32_t ent = lane == 0 ? entry : prev_exit;
      // right: the guess matches, or the chain passes over the segment inside one value
      const bool ok = lane < from || !valid ||
                      (ent >= hi ? (r.z == 0 && r.w == 0 && r.y == ent) : (r.x == ent));
      const uint64_t bad = __ballot(!ok);
      if (!bad) break;
      const uint32_t j = (uint32_t)__builtin_ctzll(bad);
      const uint32_t ej = sgpr(__shfl(ent, j));
      const uint32_t hj = (k0 + j + 1) * kPbaSeg;
      uint4 fix = make_uint4(ej, ej, 0u, 0u);
      if (ej < hj) {
        const PbaWalk w = pba_walk(s, n, ej, hj);
        fix = make_uint4(ej, w.exit, w.cnt, w.err);
      }
      if (lane == j) r = fix;
      from = j + 1;
      if (from >= 64 || fix.w) break;  // past a failing value the chain is over: later lanes do not matter
    }
    // first values and the first error on the true chain
    const uint32_t cnt = valid ? r.z : 0u;
    const uint32_t incl = wave_incl_scan32(cnt);
    const uint32_t first = v + incl - cnt;
    const uint32_t err = valid ? r.w : 0u;
    const uint32_t errv = err ? first + cnt : 0xffffffffu;
    uint32_t e0 = errv;
    for (int o = 32; o; o >>= 1) e0 = min(e0, (uint32_t)__shfl_xor((int)e0, o));
    if (e0 != 0xffffffffu) {
      const uint64_t eb = __ballot(errv == e0);
      const uint32_t jl = (uint32_t)__builtin_ctzll(eb);
      const uint32_t cls = sgpr(__shfl(err, jl));
      if (e0 < nn) {
        if (lane == 0) report(b, pd.chunk, 1, pd.page_in_chunk, ST_VALUES, e0, cls);
        lim = min(lim, e0);
      }
      done = true;
    }
    if (valid) segs[base_seg + k] = make_uint4(r.x, r.y, r.z, first);
    v += rdlane(incl, 63);
    entry = sgpr(__shfl(r.y, 63));
    if (v >= nn) done = true;
  }
  if (!done && v < nn) {  // the chain ended before nn values: the next read is past the section
    if (lane == 0) report(b, pd.chunk, 1, pd.page_in_chunk, ST_VALUES, v, PQ_ERR_EOF);
    lim = min(lim, v);
  }
  if (lane == 0) limit[li] = lim;
}

__global__ void __launch_bounds__(256) k_pba_emit(BatchDev b_in, const uint32_t *pages, const uint32_t *seg0,
                                                  const uint32_t *seg_page, const uint4 *segs, const uint32_t *limit,
                                                  uint32_t nseg) {
  const BatchDev b = global_view(b_in);
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= nseg) return;
  const uint32_t li = gp(seg_page)[g], p = gp(pages)[li];
  const PageDesc &pd = b.pages[p];
  const ChunkDesc &cd = b.chunks[pd.chunk];
  if (cd.type == T_FLBA && cd.type_length > 0) return;  // written by k_pba_fix
  const uint4 r = gp(segs)[g];
  const uint32_t lim = gp(limit)[li];
  if (r.x == kPbaNone || r.z == 0 || r.w >= lim) return;
  const uint8_t *s = gp_u64<const uint8_t>(pd.data) + pd.val_off;
  const uint64_t vb = b.page_vbase[p];
  uint64_t *src = gp_u64<uint64_t>(cd.ba_index) + vb;
  int32_t *len = gp_u64<int32_t>(cd.offsets) + vb + 1;
  uint64_t q = r.x;
  const uint32_t last = min(r.w + r.z, lim);
  for (uint32_t v = r.w; v < last; v++) {
    const int32_t l = (int32_t)ld32(s + q);
    src[v] = (uint64_t)(s + q + 4);
    len[v] = l;
    q += 4 + (uint64_t)l;
  }
}

hipError_t launch_plain_ba(const BatchDev &b, const PbaLists &l, hipStream_t s) {
  if (!l.n_pages) return hipSuccess;
  const uint32_t gb = (l.n_segs + 255) / 256;
  if (l.n_segs) hipLaunchKernelGGL(k_pba_spec, dim3(gb), dim3(256), 0, s, b, l.pages, l.seg0, l.seg_page, l.segs, l.n_segs);
  hipLaunchKernelGGL(k_pba_fix, dim3(l.n_pages), dim3(64), 0, s, b, l.pages, l.seg0, l.segs, l.limit);
  if (l.n_segs)
    hipLaunchKernelGGL(k_pba_emit, dim3(gb), dim3(256), 0, s, b, l.pages, l.seg0, l.seg_page, (const uint4 *)l.segs,
                       (const uint32_t *)l.limit, l.n_segs);
  return hipGetLastError();
}

}  // namespace pq
