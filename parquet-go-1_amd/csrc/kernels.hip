// kernels.hip — gfx950 (CDNA4) kernels of the Parquet column-chunk decoder.
//
// Everything here is integer / byte work bound by HBM bandwidth or by the
// latency of serial header chains; nothing is a contraction, so there is no
// MFMA. Design rules followed (cdna_hip_programming.md §6):
//  * wave64 everywhere: run headers are decoded speculatively by all 64 lanes
//    of a wave (one candidate byte position per lane) and the true header
//    chain is then followed with v_readlane hops in scalar registers;
//  * streams are staged through LDS in 4 KiB windows; bitmaps are built in
//    LDS and flushed with coalesced stores;
//  * bulk copies (PLAIN) move 16 B per lane with unaligned sources handled by
//    v_alignbyte funnel shifts, so every global access is a dword(x4) access;
//  * the staging buffer is padded so the 3-dword unaligned reads at a section
//    end never leave the allocation.
//
// Semantics (values, levels, errors) restate the reference decoders cited per
// kernel; tests/ compare every output bit-exactly with the oracle.
#include <hip/hip_runtime.h>

#include "../../include/pqgpu.h"
#include "dev_util.h"
#include "dict_slots.h"
#include "dict_tile.h"
#include "kernels.h"
#include "level_fill.h"

namespace pq {

const char *kValuesKernelName = "k_values";


// ---------------------------------------------------------------------------
// Hybrid RLE / bit-packing walker (hybrid_decoder.go:81-165), wave 0 of a workgroup.
//
// The walker keeps an LDS window of the stream (hyb_scan below). For the header at `pos`
// every lane decodes the header that WOULD start at pos+lane (uvarint,
// kind, count, payload length, Go error class). The true chain is then
// followed lane to lane with readlane hops; each visited lane is a run.
// Runs are handed to the sink with their first value index, clipped to the
// values still needed. Errors are reported at the value index where the
// reference's next() would fail:
//   header at EOF / truncated varint      -> io.EOF            (readUVariant32)
//   header > MaxInt32, varint overflow    -> "int32 out of range" / overflow
//   zero-count run                        -> "rle: empty ... run"
//   RLE value short                       -> EOF / ErrUnexpectedEOF
//   RLE value >= 2^bw                     -> "RLE run value is too large"
//   bit-packed group starting at EOF      -> io.EOF (a short group zero-fills)
// ---------------------------------------------------------------------------
constexpr uint32_t kSegSlots = 65536;  // bitmap slots staged in LDS per page

constexpr uint32_t kErrLongVarint = 15;  // internal: varint longer than 12 bytes, resolved lazily
DEV uint32_t resolve_long_varint(const uint8_t *s, uint32_t c, uint32_t n) {
  for (uint32_t q = c + 12; q < n; q++)
    if (s[q] < 0x80) return PQ_ERR_RANGE;
  return PQ_ERR_EOF;
}

struct Hdr {
  uint32_t err, nvals, okvals, value, adv, bp, cnt;
};

// Decode the run header that would start at stream position c (stage holds [sb, ...)):
// the readUVariant32 header (hybrid_decoder.go:77-99) and the run it announces.
// Branch-light: one round of four aligned LDS reads gives the 12 bytes from c; the
// varint terminator comes from a byte mask and the 7-bit groups are compacted with
// shifts (no per-byte loop). Go ReadUvarint semantics: a 10th byte > 1 or any 11th
// byte overflows; a value above 2^31-1 is out of range; no terminator within 12
// bytes is resolved lazily by the caller (kErrLongVarint).
DEV Hdr decode_hdr(const uint32_t *stg, uint32_t sb, const uint8_t *s, uint32_t c, uint32_t n, uint32_t bw,
                   uint32_t rs) {
  Hdr r{0, 0, 0, 0, 1, 0, 0};
  if (c >= n) { r.err = PQ_ERR_EOF; return r; }
  const uint32_t off = c - sb, a = off >> 2, sh = off & 3;
  const uint32_t w0 = stg[a], w1 = stg[a + 1], w2 = stg[a + 2], w3 = stg[a + 3];
  const uint32_t u0 = __builtin_amdgcn_alignbyte(w1, w0, sh), u1 = __builtin_amdgcn_alignbyte(w2, w1, sh),
                 u2 = __builtin_amdgcn_alignbyte(w3, w2, sh);
  const uint64_t lo = (uint64_t)u0 | ((uint64_t)u1 << 32);
  const uint64_t t_lo = ~lo & 0x8080808080808080ull;
  const uint32_t t_hi = ~u2 & 0x80808080u;
  // varint length L (bytes including the terminator); 13 = none within 12 bytes
  const uint32_t L = t_lo ? (uint32_t)(__builtin_ctzll(t_lo) >> 3) + 1
                          : (t_hi ? (uint32_t)(__builtin_ctz(t_hi) >> 3) + 9 : 13u);
  if (c + L > n) {  // the stream ends inside the varint (ReadByte at EOF)
    r.err = PQ_ERR_EOF;
    return r;
  }
  if (L == 13) { r.err = kErrLongVarint; return r; }
  if (L >= 11 || (L == 10 && ((u2 >> 8) & 0xffu) > 1)) { r.err = PQ_ERR_RANGE; return r; }
  uint64_t y = (L >= 8 ? lo : lo & ((1ull << (8 * L)) - 1ull)) & 0x7f7f7f7f7f7f7f7full;
  y = (y & 0x007f007f007f007full) | ((y & 0x7f007f007f007f00ull) >> 1);
  y = (y & 0x00003fff00003fffull) | ((y & 0x3fff00003fff0000ull) >> 2);
  uint64_t h = (y & 0x000000000fffffffull) | ((y & 0x0fffffff00000000ull) >> 4);
  if (L >= 9) h |= (uint64_t)(u2 & 0x7fu) << 56;
  if (L == 10) h |= (uint64_t)((u2 >> 8) & 1u) << 63;
  if (h > 0x7fffffffull) { r.err = PQ_ERR_RANGE; return r; }
  const uint32_t cnt = (uint32_t)(h >> 1);
  r.bp = (uint32_t)(h & 1);
  r.cnt = cnt;
  if (cnt == 0) { r.err = PQ_ERR_INVALID; return r; }
  const uint32_t hl = L;
  const uint32_t pay = c + hl;
  if (r.bp) {
    const uint64_t nv = (uint64_t)cnt * 8;
    r.nvals = nv > 0x7fffffffull ? 0x7fffffffu : (uint32_t)nv;
    const uint64_t pb = (uint64_t)cnt * bw;
    const uint64_t adv = hl + pb;
    r.adv = adv > 0x3fffffffull ? 0x3fffffffu : (uint32_t)adv;
    if ((uint64_t)pay + pb > n) {
      const uint64_t g = pay >= n ? 0 : ((uint64_t)(n - pay) + bw - 1) / bw;  // groups that start before EOF
      const uint64_t ok = g * 8;
      r.okvals = ok > r.nvals ? r.nvals : (uint32_t)ok;
    } else {
      r.okvals = r.nvals;
    }
    r.value = pay;
  } else {
    r.nvals = cnt;
    r.okvals = cnt;
    r.adv = hl + rs;
    if (pay >= n) r.err = PQ_ERR_EOF;
    else if (pay + rs > n) r.err = PQ_ERR_UNEXPECTED_EOF;
    else {
      // value bytes at offset L of the 12 register bytes (canonical headers: L <= 5)
      uint32_t v;
      if (L <= 8) {
        const uint64_t mid = ((uint64_t)u1 >> 0) | ((uint64_t)u2 << 32);  // bytes 4..11
        v = L < 4 ? __builtin_amdgcn_alignbyte(u1, u0, L) : (uint32_t)(mid >> (8 * (L - 4)));
      } else {
        v = lds_ld32(stg, pay - sb);
      }
      r.value = rs >= 4 ? v : (v & ((1u << (8 * rs)) - 1u));
      if (bw < 32 && (r.value >> bw) != 0) r.err = PQ_ERR_INVALID;
    }
  }
  return r;
}


// The walker over a whole stream, one 256-thread workgroup: the stream goes through an LDS
// window of kScanWin bytes (+ kScanOver bytes of look-ahead). All four waves load the next
// window into registers (16-B loads) while wave 0 walks the current one, so a long run of
// bit-packed values costs one step of the walk, not a load round trip.
constexpr uint32_t kScanWin = 16384;
constexpr uint32_t kScanOver = 256;
constexpr uint32_t kScanVec = (kScanWin + kScanOver) / 16;  // uint4 per window
constexpr uint32_t kScanPer = (kScanVec + 255) / 256;       // uint4 per thread
struct ScanLDS {
  uint32_t win[kScanVec * 4 + 8];
  uint32_t ctl_pos, ctl_done, ctl_stop;
};

constexpr uint32_t kPreGroups = 8;  // groups of 64 runs the stride prelude checks per step
// PRE: the stride prelude from global memory first (a stream that is one run shape throughout is
// then walked without staging it); without it every step of the walk reads the LDS window.
template <class Sink, bool PRE = true, int SB = 56>  // SB: first diagnostic counter slot
DEV uint32_t hyb_scan(ScanLDS &L, const uint8_t *s, uint32_t n, uint32_t bw, uint32_t need, Sink &sink,
                      unsigned long long *dbg = nullptr) {
  const uint32_t tid = threadIdx.x, lane = lane_id(), wv = tid >> 6;
  PQ_STAMPS(st, dbg);  // diagnostic build: 0 fast hops, 1 decode, 2 chain, 3 sink, 4 window wait, 5 hops#, 6 steps#
  st.begin();
  const uint32_t rs = (bw + 7) >> 3;
  // window w holds the bytes at 16-B aligned global addresses [s_al + w * kScanWin, + kScanWin + kScanOver)
  const uintptr_t s_al = (uintptr_t)s & ~(uintptr_t)15;
  const uint32_t sbase = (uint32_t)((uintptr_t)s - s_al);
  const uint4 *g = (const uint4 *)gp_u64<const uint8_t>((uint64_t)s_al);
  uint4 pre[kScanPer];
  auto fetch = [&](uint32_t w) {
#pragma unroll
    for (uint32_t j = 0; j < kScanPer; j++) {
      const uint32_t k = tid + j * 256;
      uint4 x = make_uint4(0u, 0u, 0u, 0u);
      const uint64_t ap = (uint64_t)w * kScanWin + 16ull * k;  // aligned position
      const int64_t rel = (int64_t)n + sbase - (int64_t)ap;       // stream bytes left at this block
      if (k < kScanVec && rel > 0) {
        x = g[ap >> 4];
        if (rel < 16) {  // bytes at or past the stream end read as zero
          uint32_t q[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
          for (int i = 0; i < 4; i++) {
            const int64_t r = rel - 4 * i;
            q[i] = r >= 4 ? q[i] : (r <= 0 ? 0u : (q[i] & ((1u << (8 * r)) - 1u)));
          }
          x = make_uint4(q[0], q[1], q[2], q[3]);
        }
      }
      pre[j] = x;
    }
  };
  auto store = [&]() {
#pragma unroll
    for (uint32_t j = 0; j < kScanPer; j++) {
      const uint32_t k = tid + j * 256;
      if (k < kScanVec) *(uint4 *)&L.win[4 * k] = pre[j];
    }
    if (tid < 8) L.win[kScanVec * 4 + tid] = 0;
  };
  uint32_t pos = 0, done = 0;
  // Prelude (wave 0): while the runs are long (>= 64 stream bytes) the chain is followed by stride
  // speculation straight from global memory — lane k reads the 8 header bytes k runs ahead — so a
  // stream of maximal literal runs is walked without staging its payload in LDS at all (a dictionary
  // page's payload is read later, by the tiles that decode it). Anything else (a short run, a run
  // that differs, the stream end, an error) stops the prelude; the windowed walk below takes over
  // at that position with the reference's exact semantics.
  if (PRE && wv == 0) {
    // Each step decodes the header at pos (the run shape), then reads the 8 header bytes of the
    // kPreGroups x 64 runs from pos on at once (lane k of group j: run 64 j + k, had every run this
    // shape) and keeps the longest prefix with that shape: those are exact chain nodes by induction,
    // and the first run that differs is the true next node, whose bytes a lane already holds (no
    // reload). A run that completes the values needed is taken whatever its length. One memory round
    // trip per 512 runs: a dictionary page of 1,600 maximal literal runs (cfg4's map keys) took 25
    // steps of two round trips each with one group.
    const uint8_t *sg = gp_u64<const uint8_t>((uint64_t)(uintptr_t)s);
    uint64_t hx = pos < n ? ld64(sg + pos) : 0;  // bytes past the stream end are never used (checks below)
    while (done < need && pos < n) {
      const uint32_t u0 = sgpr((uint32_t)hx), u1 = sgpr((uint32_t)(hx >> 32));
      const uint32_t tm = ~u0 & 0x80808080u;
      if (!tm) break;
      const uint32_t Lv = (uint32_t)(__builtin_ctz(tm) >> 3) + 1;
      const uint32_t y = (Lv >= 4 ? u0 : (u0 & ((1u << (8 * Lv)) - 1u))) & 0x7f7f7f7fu;
      const uint32_t h = (y & 0x7fu) | ((y >> 1) & 0x3f80u) | ((y >> 2) & 0x1fc000u) | ((y >> 3) & 0xfe00000u);
      const uint32_t cnt = h >> 1, isbp = h & 1u;
      const uint64_t adv = isbp ? Lv + (uint64_t)cnt * bw : (uint64_t)(Lv + rs);
      const uint32_t rv = (uint32_t)((((uint64_t)u1 << 32) | u0) >> (8 * Lv));
      const uint32_t val = isbp ? pos + Lv : (rs >= 4 ? rv : (rv & ((1u << (8 * rs)) - 1u)));
      const bool ok = cnt != 0 && (uint64_t)pos + adv <= n && (isbp || bw >= 32 || (val >> bw) == 0);
      const uint32_t nv = isbp ? cnt * 8 : cnt, rem = need - done;
      if (!(ok && (adv >= 64 || nv >= rem))) break;
      const uint32_t mneed = (uint32_t)(((uint64_t)rem + nv - 1) / nv);  // runs that cover rem
      uint64_t xk[kPreGroups];
      uint32_t vks[kPreGroups];
#pragma unroll
      for (uint32_t j = 0; j < kPreGroups; j++) {
        const uint64_t Pk = (uint64_t)pos + (uint64_t)(64 * j + lane) * adv;
        xk[j] = (64 * j + lane > 0 && 64 * j + lane < mneed && Pk < n) ? ld64(sg + Pk) : 0;
      }
      uint32_t F = 64 * kPreGroups;  // the first run (index from pos) without the shape
#pragma unroll
      for (uint32_t j = 0; j < kPreGroups; j++) {
        const uint64_t Pk = (uint64_t)pos + (uint64_t)(64 * j + lane) * adv;
        bool sm = j == 0 && lane == 0;
        uint32_t vk = val;
        if (!sm && Pk + adv <= n) {
          const uint32_t a0 = (uint32_t)xk[j];
          const uint32_t tk = ~a0 & 0x80808080u;
          const uint32_t Lk = (uint32_t)(__builtin_ctz(tk | 0x80000000u) >> 3) + 1;
          const uint32_t yk = (Lk >= 4 ? a0 : (a0 & ((1u << (8 * Lk)) - 1u))) & 0x7f7f7f7fu;
          const uint32_t hk = (yk & 0x7fu) | ((yk >> 1) & 0x3f80u) | ((yk >> 2) & 0x1fc000u) | ((yk >> 3) & 0xfe00000u);
          const uint32_t rk = (uint32_t)(xk[j] >> (8 * Lk));
          vk = isbp ? (uint32_t)Pk + Lk : (rs >= 4 ? rk : (rk & ((1u << (8 * rs)) - 1u)));
          sm = tk != 0 && Lk == Lv && hk == h && (isbp || bw >= 32 || (vk >> bw) == 0);
        }
        vks[j] = vk;
        const uint64_t nb = ~__ballot(sm);
        if (F == 64 * kPreGroups && nb) F = 64 * j + (uint32_t)__builtin_ctzll(nb);
      }
      const uint32_t M = min(F, mneed);  // runs of this step
#pragma unroll
      for (uint32_t j = 0; j < kPreGroups; j++) {
        if (64 * j >= M) break;
        const uint32_t g = 64 * j + lane;
        const uint64_t Pk = (uint64_t)pos + (uint64_t)g * adv;
        const uint32_t first = done + g * nv;  // < need for g < M
        sink.window(g < M, first, g < M ? min(nv, need - first) : 0u, isbp != 0, vks[j], (uint32_t)Pk, nullptr, 0u);
      }
      st.add(5, M);
      if (M == mneed) { done = need; break; }
      done += M * nv;
      pos += (uint32_t)(M * adv);
      if (F < 64 * kPreGroups) {  // the run that differs: its bytes are in lane F mod 64 of group F / 64
        if (pos >= n) break;
        uint64_t x = 0;
#pragma unroll
        for (uint32_t j = 0; j < kPreGroups; j++)
          if (j == F / 64) x = xk[j];
        hx = ((uint64_t)rdlane((uint32_t)(x >> 32), F & 63u) << 32) | rdlane((uint32_t)x, F & 63u);
      } else {
        hx = ld64(sg + pos);
      }
    }
  }
  if (PRE) {
    if (threadIdx.x == 0) { L.ctl_pos = pos; L.ctl_done = done; }
    wg_barrier();
    pos = L.ctl_pos;
    done = L.ctl_done;
  }
  if (done >= need) {
    if (wv == 0) st.flush(SB);
    return done;
  }
  uint32_t w = (pos + sbase) / kScanWin;  // the window holding the chain's position
  fetch(w);
  store();
  fetch(w + 1);
  wg_barrier();
  for (;;) {
    if (wv == 0) {
      const uint32_t sb = w * kScanWin - sbase;  // stream position of win[0] (mod 2^32)
      const uint32_t lim = (w + 1) * kScanWin - sbase;
      uint32_t stop = 0;
      while (done < need && pos < lim) {
        // ---- scalar fast path: a well-formed run of >= 64 stream bytes (long bit-packed runs;
        // one header per step, no speculation)
        {
          const uint32_t off = pos - sb;
          const uint32_t u0 = sgpr(lds_ld32(L.win, off)), u1 = sgpr(lds_ld32(L.win, off + 4));
          const uint32_t tm = ~u0 & 0x80808080u;
          if (tm && pos < n) {
            const uint32_t Lv = (uint32_t)(__builtin_ctz(tm) >> 3) + 1;
            const uint32_t y = (Lv >= 4 ? u0 : (u0 & ((1u << (8 * Lv)) - 1u))) & 0x7f7f7f7fu;
            const uint32_t h = (y & 0x7fu) | ((y >> 1) & 0x3f80u) | ((y >> 2) & 0x1fc000u) | ((y >> 3) & 0xfe00000u);
            const uint32_t cnt = h >> 1, isbp = h & 1u;
            const uint64_t adv = isbp ? Lv + (uint64_t)cnt * bw : (uint64_t)(Lv + rs);
            const uint32_t rv = (uint32_t)((((uint64_t)u1 << 32) | u0) >> (8 * Lv));
            const uint32_t val = isbp ? pos + Lv : (rs >= 4 ? rv : (rv & ((1u << (8 * rs)) - 1u)));
            const bool ok = cnt != 0 && (uint64_t)pos + adv <= n && (isbp || bw >= 32 || (val >> bw) == 0);
            if (ok && adv >= 64) {
              // Stride speculation: lane k decodes the header that would start k runs further on if
              // the next runs had this run's header (same varint length, kind and count: writers emit
              // maximal literal runs back to back). Lanes 0 .. m-1 with that header are exact chain
              // nodes by induction (lane j's position is true and its run is adv long); lane m's
              // position is the true next header whatever it holds.
              const uint32_t nv = isbp ? cnt * 8 : cnt, rem = need - done;
              const uint64_t Pk = (uint64_t)pos + (uint64_t)lane * adv;
              bool same = lane == 0;
              uint32_t vk = val;
              if (lane > 0 && Pk < lim && Pk < n) {
                const uint32_t o = (uint32_t)Pk - sb;
                const uint32_t a0 = lds_ld32(L.win, o), a1 = lds_ld32(L.win, o + 4);
                const uint32_t tk = ~a0 & 0x80808080u;
                const uint32_t Lk = (uint32_t)(__builtin_ctz(tk | 0x80000000u) >> 3) + 1;
                const uint32_t yk = (Lk >= 4 ? a0 : (a0 & ((1u << (8 * Lk)) - 1u))) & 0x7f7f7f7fu;
                const uint32_t hk = (yk & 0x7fu) | ((yk >> 1) & 0x3f80u) | ((yk >> 2) & 0x1fc000u) | ((yk >> 3) & 0xfe00000u);
                const uint32_t rk = (uint32_t)((((uint64_t)a1 << 32) | a0) >> (8 * Lk));
                vk = isbp ? (uint32_t)Pk + Lk : (rs >= 4 ? rk : (rk & ((1u << (8 * rs)) - 1u)));
                same = tk != 0 && Lk == Lv && hk == h && Pk + adv <= n && (isbp || bw >= 32 || (vk >> bw) == 0);
              }
              const uint64_t nb = ~__ballot(same);
              const uint32_t mneed = (uint32_t)(((uint64_t)rem + nv - 1) / nv);  // runs that cover rem
              const uint32_t m = min(nb ? (uint32_t)__builtin_ctzll(nb) : 64u, mneed);
              const uint32_t first = done + lane * nv;  // < need for lanes < m
              sink.window(lane < m, first, lane < m ? min(nv, need - first) : 0u, isbp != 0, vk, (uint32_t)Pk, L.win, sb);
              st.lap(0);
              st.add(5, m);
              if (m == mneed) { done = need; break; }
              done += m * nv;
              pos += (uint32_t)(m * adv);
              continue;
            }
          }
        }
        // ---- speculative header decode at c = pos + lane
        const uint32_t c = pos + lane;
        const Hdr h = decode_hdr(L.win, sb, s, c, n, bw, rs);
        st.lap(1);
        st.add(6, 1);
        // ---- follow the true chain lane to lane (scalar registers)
        uint64_t mask = 0;
        uint32_t cum = 0, p = 0, next_pos = pos;
        uint32_t stop_err = 0, stop_pos = 0;
        for (;;) {
          uint32_t e = rdlane(h.err, p);
          if (e == kErrLongVarint) e = sgpr(resolve_long_varint(s, pos + p, n));
          if (e) { stop = 1; stop_err = e; stop_pos = done + cum; break; }
          const uint32_t nv = rdlane(h.nvals, p), ok = rdlane(h.okvals, p);
          mask |= 1ull << p;
          const uint32_t rem = need - done - cum;
          if (ok < nv && ok < rem) { cum += ok; stop = 1; stop_err = PQ_ERR_EOF; stop_pos = done + cum; break; }
          if (nv >= rem) { cum += rem; stop = 1; break; }
          cum += nv;
          const uint32_t q = p + rdlane(h.adv, p);
          if (q >= 64) { next_pos = pos + q; break; }
          p = q;
        }
        st.lap(2);
        st.add(5, (uint64_t)__popcll(mask));
        // ---- the runs of this step
        const bool mine = (mask >> lane) & 1ull;
        const uint32_t first = wave_excl_scan(mine ? h.nvals : 0u);
        uint32_t cnt = 0;
        if (mine && first < cum) cnt = min(h.nvals, cum - first);
        sink.window(mine && cnt > 0, done + first, cnt, h.bp != 0, h.value, c, L.win, sb);
        st.lap(3);
        done = sgpr(done + cum);
        if (stop) {
          if (stop_err) sink.error(stop_pos, stop_err);
          break;
        }
        pos = sgpr(next_pos);
      }
      if (lane == 0) {
        L.ctl_pos = pos;
        L.ctl_done = done;
        L.ctl_stop = stop || done >= need;
      }
    }
    st.lap(3);
    wg_barrier();
    pos = L.ctl_pos;
    done = L.ctl_done;
    const uint32_t fin = L.ctl_stop;
    if (fin) break;
    const uint32_t nw = (pos + sbase) / kScanWin;
    if (nw == w + 1) {
      store();
      fetch(nw + 1);
    } else {  // a run longer than a window: that window was not prefetched
      fetch(nw);
      store();
      fetch(nw + 1);
    }
    w = nw;
    wg_barrier();
    st.lap(4);
  }
  if (wv == 0) st.flush(SB);
  return done;
}

// ---------------------------------------------------------------------------
// Level sink: rep/def levels -> uint8 levels, validity bits, counts.
// decodePackedArray helpers.go:133-149 (notNull = count(level == maxD)).
// ---------------------------------------------------------------------------
struct LevelSink {
  const uint8_t *s;
  uint32_t n;            // stream length
  uint32_t bw;
  uint8_t *out;          // uint8 levels at page start, or null
  uint32_t *bits_lds;    // LDS bitmap (page-relative slots [0, kSegSlots)) or null
  uint32_t *bits_glob;   // global bitmap of the chunk (slot_base applied by caller) or null
  uint64_t slot_base;    // chunk-relative slot of page start
  uint32_t cmp;          // level value that counts (maxD for def, 0 for rep)
  uint32_t count;        // lane-local count of (level == cmp)
  uint32_t err_code, err_pos;
  uint32_t stage_len;    // bytes held by the LDS stage passed to window()/piece()
  uint32_t ablate;       // diagnostic build: BatchDev::ablate
  // generic widths (run tables for k_level_fill)
  uint2 *runs;           // the stream's run table
  uint32_t *trun;        // first run of each of the page's fill tiles (stride 2)
  uint32_t tile_a;       // page slot_base mod kLfTile
  uint32_t ntiles;       // the page's fill tiles
  uint32_t covered;      // values the run table covers (num_values unless the stream failed)
  uint32_t nruns;        // run-table entries

  DEV static void or_bits(uint32_t *dst, uint64_t g, uint64_t m) {
    if (!m) return;
    uint32_t w = (uint32_t)(g >> 5), sh = (uint32_t)(g & 31);
    atomicOr(&dst[w], (uint32_t)(m << sh));
    uint64_t rest = sh ? (m >> (32 - sh)) : (m >> 32);
    if (rest) {
      atomicOr(&dst[w + 1], (uint32_t)rest);
      if (rest >> 32) atomicOr(&dst[w + 2], (uint32_t)(rest >> 32));
    }
  }
  // bits [slot, slot+nb) of the page: LDS segment for slots < kSegSlots, chunk bitmap beyond
  DEV void set_bits(uint32_t slot, uint64_t m, uint32_t nb) {
    if (!m) return;
    if (!bits_lds) {
      if (bits_glob) or_bits(gp(bits_glob), slot_base + slot, m);
      return;
    }
    if (slot + nb <= kSegSlots) { or_bits(bits_lds, slot, m); return; }
    if (slot >= kSegSlots) { or_bits(gp(bits_glob), slot_base + slot, m); return; }
    const uint32_t lo = kSegSlots - slot;  // split at the LDS segment end
    or_bits(bits_lds, slot, m & ((1ull << lo) - 1ull));
    or_bits(gp(bits_glob), slot_base + kSegSlots, m >> lo);
  }

  // Up to 64 values of one run, starting at value k of the run. `stg`/`sb`: the LDS stage.
  DEV void piece(bool bp, uint32_t value, uint32_t slot, uint32_t k, uint32_t nb, const uint32_t *stg, uint32_t sb) {
    uint64_t eq;
    if (bp) {
      const uint64_t bo = (uint64_t)value * 8 + (uint64_t)k * bw;   // stream bit offset
      const uint64_t be = bo + (uint64_t)nb * bw;
      const bool staged = stg && value >= sb && be + 64 <= (uint64_t)(sb + stage_len) * 8;
      if (bw == 1) {
        uint64_t raw;
        if (staged) raw = lds_bits64(stg, (uint32_t)(bo - (uint64_t)sb * 8), nb);
        else raw = nb > 56 ? (bits64c(s, n, bo, 32) | (bits64c(s, n, bo + 32, nb - 32) << 32)) : bits64c(s, n, bo, nb);
        eq = cmp ? raw : (~raw & (nb >= 64 ? ~0ull : ((1ull << nb) - 1)));
        if (out)
          for (uint32_t j = 0; j < nb; j++) out[slot + j] = (uint8_t)((raw >> j) & 1);
      } else {
        eq = 0;
        for (uint32_t j = 0; j < nb; j++) {
          const uint64_t b0 = bo + (uint64_t)j * bw;
          uint32_t lv = staged ? (uint32_t)lds_bits64(stg, (uint32_t)(b0 - (uint64_t)sb * 8), bw) : bits32c(s, n, b0, bw);
          if (out) out[slot + j] = (uint8_t)lv;
          eq |= (uint64_t)(lv == cmp) << j;
        }
      }
    } else {
      eq = value == cmp ? (nb >= 64 ? ~0ull : ((1ull << nb) - 1)) : 0;
      if (out)
        for (uint32_t j = 0; j < nb; j++) out[slot + j] = (uint8_t)value;
    }
    count += __popcll(eq);
    set_bits(slot, eq, nb);
  }

  DEV void window(bool active, uint32_t first, uint32_t cnt, bool bp, uint32_t value, uint32_t, const uint32_t *stg,
                  uint32_t sb) {
    // runs up to 4096 values: the owning lane, 64 values per step (payload from the LDS stage)
    const bool mine = active && cnt <= 4096;
    for (uint32_t k = 0; __ballot(mine && k < cnt); k += 64)
      if (mine && k < cnt) piece(bp, value, first + k, k, min(64u, cnt - k), stg, sb);
    // longer runs: the whole wave, 64 values per lane-step (payload read from global memory)
    uint64_t big = __ballot(active && cnt > 4096);
    while (big) {
      const uint32_t r = __builtin_ctzll(big);
      big &= big - 1;
      const uint32_t rf = rdlane(first, r), rc = rdlane(cnt, r), rv = rdlane(value, r);
      const bool rbp = rdlane(bp ? 1u : 0u, r) != 0;
      for (uint32_t k = lane_id() * 64; k < rc; k += 64 * 64) piece(rbp, rv, rf + k, k, min(64u, rc - k), nullptr, 0);
    }
  }
  DEV void error(uint32_t pos, uint32_t code) {
    if (!err_code) { err_code = code; err_pos = pos; }
  }
};

// ---------------------------------------------------------------------------
// Level decoder: one 256-thread workgroup per page with level streams.
//
// A hybrid stream (hybrid_decoder.go:81-165) is a chain of run headers: the position
// of run k+1 is known only once run k's header is decoded. The stream is processed in
// chunks of kLvChunk candidate header positions, staged in LDS with the bytes past the
// chunk end, by parallel list ranking:
//  P1  links: every position is decoded as if a run header started there (fast_hdr). A
//      header varint of at most 4 bytes whose run is well formed and complete inside the
//      stream links p -> p + adv (EXIT when that leaves the chunk); anything else (errors,
//      runs cut by EOF, longer varints) is a stop: a self-link.
//  P2  doubling: J[j+1][p] = J[j][J[j][p]] for j < kLvLevels (jumps of 2^j runs, saturating
//      at a stop or the chunk exit), in two ping-pong tables; J[0] is kept.
//  P3  one lane follows the true chain from the chunk entry by 2^kLvLevels-run jumps and
//      records each node it lands on: the checkpoints (at most 64: a run takes >= 2 bytes).
//  P4  wave 0, lane w: from checkpoint w, walk the next 2^kLvLevels runs over J[0] and mark
//      them: afterwards exactly the chain's nodes are marked.
//  P5  value indices: a workgroup prefix sum, in position order, of the marked runs' value
//      counts; the chain's last node gives the next chunk's entry.
//  P6  fill: every marked run is expanded by the thread that owns its position (bit width 1
//      with validity output only ORs whole 32-bit words of payload into an LDS bitmap; other
//      widths go through LevelSink::piece); runs longer than kLvLongRun values are expanded
//      by the whole workgroup.
// A stop on the chain is decoded exactly (decode_hdr, the reference's full header
// semantics): an error or a bit-packed run cut by EOF ends the stream; a valid run the
// fast form could not take (a long varint) is expanded and the next chunk starts after it.
// Runs past the one that reaches num_values are never read, as in the reference's
// decodePackedArray loop; results, error class and error value position are identical.
// The page's latency (not bandwidth) sets the kernel's time, so the workgroup's footprint
// is kept small (26 KB LDS, 80 VGPRs): six pages are resident per CU.
// ---------------------------------------------------------------------------
constexpr uint32_t kLvThreads = 256;
constexpr uint32_t kLvChunk = 2048;             // candidate header positions per chunk
#ifndef PQ_LV_LEVELS
#define PQ_LV_LEVELS 4
#endif
#ifndef PQ_LV_WPE
#define PQ_LV_WPE 6  // k_levels_bw1 waves per SIMD (= resident pages per CU)
#endif
constexpr uint32_t kLvLevels = PQ_LV_LEVELS;    // checkpoints every 2^kLvLevels runs
constexpr uint32_t kLvSeg = 1u << kLvLevels;    // runs per walker
constexpr uint32_t kLvMaxCkp = kLvChunk / 2 / kLvSeg;  // chain nodes <= kLvChunk / 2
static_assert(kLvMaxCkp <= 64, "one walker lane per checkpoint");
constexpr uint32_t kLvPer = kLvChunk / kLvThreads;  // positions per thread in P1
constexpr uint32_t kLvStageB = kLvChunk + 256;  // staged bytes: the chunk + headers / payload past its end
constexpr uint32_t kLvLongRun = 512;            // runs longer than this expand cooperatively
constexpr uint32_t kLvMaxLong = 64;
constexpr uint16_t kLvExit = 0xffff;
constexpr uint32_t kNoEntry = 0xffffffffu;
constexpr uint32_t kLvRunShift = 48;  // generic widths: run counts in the P5 scan's high bits
constexpr uint64_t kLvValMask = (1ull << kLvRunShift) - 1;
constexpr uint32_t kLvTileBuf = 64;
enum : uint32_t { LV_RUN = 0, LV_STOP_NEED = 1, LV_STOP_ERR = 2, LV_STOP_TRUNC = 3 };

struct LevelLDS {
  uint32_t stage[kLvStageB / 4 + 4];
  uint16_t J0[kLvChunk];                // J0[i]: chunk offset of the next run after i; i = stop; kLvExit
  uint16_t JA[kLvChunk], JB[kLvChunk];  // doubling ping-pong
  uint16_t ckp[kLvMaxCkp];
  uint8_t mark[kLvChunk];               // chain nodes of the chunk
  uint64_t wsum[kLvThreads / 64];
  uint32_t nckp;
  uint32_t long_f[kLvMaxLong], long_cnt[kLvMaxLong], long_bp[kLvMaxLong], long_val[kLvMaxLong];
  uint32_t nlong, nput, stop_kind, stop_code, stop_vpos, next_e;
  uint64_t total;
  uint64_t cnt[16];
  union {
    uint32_t bits[kSegSlots / 32];  // bit width 1: the page's first kSegSlots validity bits
    uint2 rbuf[kLvChunk / 2];       // generic widths: the chunk's run-table entries
  };
  uint32_t tb_k[kLvTileBuf], tb_r[kLvTileBuf], ntb;  // generic widths: fill-tile starts of the chunk
  uint32_t sp_e, sp_d, sp_r;                          // generic widths: the stride prelude's chain state
};

// Fast candidate at stream position c: a header varint of at most 4 bytes whose run is
// well formed and complete inside the stream (RLE value < 2^bw, bit-packed payload before
// EOF). Returns the next position's offset (adv; 0 marks a stop that decode_hdr resolves),
// the run's value count, its kind and its RLE value / payload position.
struct FastHdr { uint32_t adv, nvals, bp, value; };
DEV FastHdr fast_hdr(const uint32_t *stg, uint32_t sb, uint32_t c, uint32_t n, uint32_t bw, uint32_t rs) {
  FastHdr f{0, 0, 0, 0};
  if (c >= n) return f;
  const uint32_t o = c - sb, a = o >> 2, sh = o & 3;
  const uint32_t w0 = stg[a], w1 = stg[a + 1], w2 = stg[a + 2];
  const uint32_t u0 = __builtin_amdgcn_alignbyte(w1, w0, sh), u1 = __builtin_amdgcn_alignbyte(w2, w1, sh);
  const uint32_t t = ~u0 & 0x80808080u;  // varint terminators among bytes 0..3
  if (!t) return f;
  const uint32_t L = (uint32_t)(__builtin_ctz(t) >> 3) + 1;
  uint32_t y = L >= 4 ? u0 : (u0 & ((1u << (8 * L)) - 1u));
  y &= 0x7f7f7f7fu;
  const uint32_t h = (y & 0x7fu) | ((y >> 1) & 0x3f80u) | ((y >> 2) & 0x1fc000u) | ((y >> 3) & 0xfe00000u);
  const uint32_t cnt = h >> 1;
  if (cnt == 0) return f;
  if (h & 1) {
    const uint64_t adv = L + (uint64_t)cnt * bw;
    if (c + adv > n) return f;
    f.adv = (uint32_t)adv; f.nvals = cnt * 8; f.bp = 1; f.value = c + L;
  } else {
    const uint32_t adv = L + rs;
    if (c + adv > n) return f;
    const uint64_t x = ((uint64_t)u1 << 32) | u0;
    const uint32_t v = (uint32_t)(x >> (8 * L));
    const uint32_t val = rs >= 4 ? v : (v & ((1u << (8 * rs)) - 1u));
    if (bw < 32 && (val >> bw) != 0) return f;
    f.adv = adv; f.nvals = cnt; f.value = val;
  }
  return f;
}

// Bits [slot, slot + 32) (page-relative) of the validity bitmap, masked by m: the LDS
// segment for the first kSegSlots slots of the page, the chunk's global bitmap beyond.
DEV void lv_or_bits(LevelSink &sk, uint32_t slot, uint32_t m) {
  if (!m) return;
  if (slot + 32 <= kSegSlots) {
    const uint32_t w = slot >> 5, sh = slot & 31;
    atomicOr(&sk.bits_lds[w], m << sh);
    if (sh && (m >> (32 - sh))) atomicOr(&sk.bits_lds[w + 1], m >> (32 - sh));
  } else {
    sk.set_bits(slot, m, 32);
  }
}

DEV void stage_load_blk(uint32_t *stg, const uint8_t *s, uint32_t sb, uint32_t n, uint32_t words) {
  const uint8_t *src = s + sb;
  const uint32_t lim = n > sb ? n - sb : 0;
  for (uint32_t k = threadIdx.x; k < words; k += blockDim.x) {
    const uint32_t o = 4 * k;
    stg[k] = o + 4 <= lim ? ld32(src + o) : (o < lim ? ld32(src + o) & ((1u << (8 * (lim - o))) - 1u) : 0u);
  }
}

// Expand one run (first value index f, cnt values) into the sink, from one lane.
template <bool BW1>
DEV void lv_emit_run(LevelSink &sk, const uint32_t *stg, uint32_t sb, uint32_t send, uint32_t f, uint32_t cnt,
                     uint32_t bp, uint32_t value) {
  if (cnt == 0) return;
  if constexpr (BW1) {
    if (!bp) {  // RLE: a constant run of ones (value == maxD) or zeros
      if (value != sk.cmp) return;
      sk.count += cnt;
      for (uint32_t q = 0; q < cnt; q += 32) lv_or_bits(sk, f + q, cnt - q >= 32 ? ~0u : ((1u << (cnt - q)) - 1u));
      return;
    }
    // bit-packed, width 1: value k of the run is bit k of the payload (LSB first)
    for (uint32_t q = 0; q < cnt; q += 32) {
      const uint32_t by = value + (q >> 3);  // q is a multiple of 32: byte aligned
      uint32_t w;
      if (by >= sb && by + 4 <= send) w = lds_ld32(stg, by - sb);
      else w = bits32c(sk.s, sk.n, (uint64_t)by * 8, 32);
      if (cnt - q < 32) w &= (1u << (cnt - q)) - 1u;
      sk.count += __popc(w);
      lv_or_bits(sk, f + q, w);
    }
  } else {
    for (uint32_t q = 0; q < cnt; q += 64)
      sk.piece(bp != 0, value, f + q, q, min(64u, cnt - q), stg, sb);
  }
}

// A run of the fill: short runs expand right away, long ones are queued for the workgroup.
template <bool BW1>
DEV void lv_fill_run(LevelLDS &L, LevelSink &sk, uint32_t sb, uint32_t send, uint32_t f, uint32_t cnt, uint32_t bp,
                     uint32_t value) {
  if (PQ_ABLATE(sk, 2)) return;  // diagnostic: no expansion
  if (cnt > kLvLongRun && !(BW1 && !bp && value != sk.cmp)) {
    const uint32_t slot = atomicAdd(&L.nlong, 1u);
    if (slot < kLvMaxLong) {
      L.long_f[slot] = f; L.long_cnt[slot] = cnt; L.long_bp[slot] = bp; L.long_val[slot] = value;
      return;
    }
    atomicSub(&L.nlong, 1u);
  }
  lv_emit_run<BW1>(sk, L.stage, sb, send, f, cnt, bp, value);
}

// The stride prelude of lv_walk (generic widths; one wave, wave-uniform state): from chain position
// `entry` (value `done`, run-table entry `runs_done`), follow the chain up to 256 runs per step.
// Candidate k (four per lane) decodes the header k runs on, assuming the runs between have this
// run's header; the leading candidates with exactly that header are chain nodes by induction, and
// candidate m's position is the true next header whatever it holds. Writers emit maximal literal
// runs back to back (Arrow's repetition streams: 64 B at bit width 1), so a step takes many runs;
// a short run among them (an RLE run) is a step of its own. Each taken run goes straight to the
// run table, with the fill tiles whose first value it holds. A header the fast form does not take
// (long varint, zero count, run past the stream, RLE value >= 2^bw), kLvShortMax short-run steps
// in a row or the stream end stop it and the chunk walk takes the chain from there; runs past the
// one that reaches `need` are never read (decodePackedArray helpers.go:133-149).
// Software-pipelined: a step's loads bring the next step's first header too (candidate m's bytes,
// or candidate 0's, which reads 256 runs on), so the next step's loads are issued before this
// step's run-table stores, and each step waits for one load round trip (vmcnt counts stores too).
#ifndef PQ_LV_STRIDE
#define PQ_LV_STRIDE 1
#endif
constexpr uint32_t kLvStrideMin = 32;  // runs at least this long are "long"
constexpr uint32_t kLvShortMax = 1;    // consecutive steps of short runs before the chunk walk takes over
                                       // (each step is a memory round trip: repetition streams with RLE
                                       // runs among the literal ones take k_levels_hyb instead)
struct StrideHdr {
  uint32_t Lv, h, cnt, isbp, val, ok;
  uint64_t adv;
};
DEV StrideHdr stride_hdr(uint64_t x, uint32_t pos, uint32_t n, uint32_t bw, uint32_t rs) {
  StrideHdr H;
  const uint32_t u0 = (uint32_t)x;
  const uint32_t tm = ~u0 & 0x80808080u;
  H.Lv = (uint32_t)(__builtin_ctz(tm | 0x80000000u) >> 3) + 1;
  const uint32_t y = (H.Lv >= 4 ? u0 : (u0 & ((1u << (8 * H.Lv)) - 1u))) & 0x7f7f7f7fu;
  H.h = (y & 0x7fu) | ((y >> 1) & 0x3f80u) | ((y >> 2) & 0x1fc000u) | ((y >> 3) & 0xfe00000u);
  H.cnt = H.h >> 1;
  H.isbp = H.h & 1u;
  H.adv = H.isbp ? H.Lv + (uint64_t)H.cnt * bw : (uint64_t)(H.Lv + rs);
  const uint32_t rv = (uint32_t)(x >> (8 * H.Lv));
  H.val = H.isbp ? pos + H.Lv : (rs >= 4 ? rv : (rv & ((1u << (8 * rs)) - 1u)));
  H.ok = tm != 0 && H.cnt != 0 && (uint64_t)pos + H.adv <= n && (H.isbp || bw >= 32 || (H.val >> bw) == 0);
  return H;
}
constexpr uint32_t kLvStrideJ = 4;  // headers per lane per step: up to 256 runs per step
DEV void lv_stride(LevelSink &sk, uint32_t need, uint32_t &entry, uint32_t &done, uint32_t &runs_done) {
  constexpr uint32_t J = kLvStrideJ, NJ = 64 * J;
  const uint8_t *sg = sk.s;
  const uint32_t n = sk.n, bw = sk.bw, rs = (bw + 7) >> 3, lane = lane_id();
  uint32_t pos = entry, dn = done, rd = runs_done;
  if (dn < need && pos < n) {
    // candidate k = 64 j + lane reads the header k runs on; k = 0 (lane 0, j = 0) instead reads the
    // one NJ runs on: the next step's first header when every candidate matches
    auto load_lanes = [&](uint32_t at, uint64_t adv, uint64_t (&x)[J]) {
#pragma unroll
      for (uint32_t j = 0; j < J; j++) {
        const uint32_t k = 64 * j + lane;
        const uint64_t Pk = (uint64_t)at + (uint64_t)(k ? k : NJ) * adv;
        x[j] = Pk < n ? ld64(sg + Pk) : 0ull;  // bytes past the stream end are never used (checks below)
      }
    };
    const uint64_t x0 = ld64(sg + pos);
    StrideHdr H = stride_hdr(((uint64_t)sgpr((uint32_t)(x0 >> 32)) << 32) | sgpr((uint32_t)x0), pos, n, bw, rs);
    uint32_t shorts = 0;  // consecutive steps of short runs
    if (H.ok && H.adv >= kLvStrideMin) {
      uint64_t xk[J];
      load_lanes(pos, H.adv, xk);
      for (;;) {
        const uint32_t nv = H.isbp ? H.cnt * 8 : H.cnt, rem = need - dn;
        uint32_t vk[J];
        uint32_t m = NJ;  // the first candidate that is not a node of this run shape
#pragma unroll
        for (uint32_t j = 0; j < J; j++) {
          const uint32_t k = 64 * j + lane;
          const uint64_t Pk = (uint64_t)pos + (uint64_t)k * H.adv;
          bool same = k == 0;
          vk[j] = H.isbp ? (uint32_t)Pk + H.Lv : H.val;
          if (k > 0 && Pk + H.adv <= n) {
            const StrideHdr K = stride_hdr(xk[j], (uint32_t)Pk, n, bw, rs);
            vk[j] = K.val;
            same = K.ok && K.Lv == H.Lv && K.h == H.h;
          }
          const uint64_t nb = ~__ballot(same);
          if (m == NJ && nb) m = 64 * j + (uint32_t)__builtin_ctzll(nb);  // (wave-uniform)
        }
        const uint32_t mneed = (uint32_t)(((uint64_t)rem + nv - 1) / nv);  // runs that cover rem
        m = min(m, mneed);
        const bool fin = m == mneed;
        const uint32_t npos = pos + (uint32_t)(m * H.adv);
        // the next step's first header (candidate m's bytes; candidate 0's NJ runs on) and its loads
        const uint32_t jm = (m & (NJ - 1)) >> 6, lm = m & 63u;
        uint64_t xm = xk[0];
#pragma unroll
        for (uint32_t j = 1; j < J; j++) xm = jm == j ? xk[j] : xm;
        const uint64_t nx = ((uint64_t)rdlane((uint32_t)(xm >> 32), lm) << 32) | rdlane((uint32_t)xm, lm);
        const StrideHdr N = stride_hdr(nx, npos, n, bw, rs);
        // a short run (an RLE run among literal runs) is taken as a step of its own, while such steps
        // are rare: after kLvShortMax of them in a row the chunk walk takes over
        shorts = N.adv < kLvStrideMin ? shorts + 1 : 0;
        const bool go = !fin && npos < n && N.ok && shorts <= kLvShortMax;
        uint64_t nxk[J];
        if (go) load_lanes(npos, N.adv, nxk);
#pragma unroll
        for (uint32_t j = 0; j < J; j++) {  // this step's runs (stores issued after the next step's loads)
          const uint32_t k = 64 * j + lane;
          if (k >= m) continue;
          const uint32_t f = dn + k * nv, c = min(nv, need - f), idx = rd + k;
          sk.runs[idx] = make_uint2(f, H.isbp ? 0x80000000u | vk[j] : vk[j]);
          if (sk.ntiles) {  // fill tiles whose first value lies in [f, f + c): tile t > 0 starts at t * T - a
            const uint64_t a = sk.tile_a;
            uint64_t t = f == 0 ? 0 : ((uint64_t)f + a + kLfTile - 1) / kLfTile;
            const uint64_t thi = min(((uint64_t)f + c - 1 + a) / kLfTile, (uint64_t)sk.ntiles - 1);
            for (; t <= thi; t++) sk.trun[2 * t] = idx;
          }
        }
        rd += m;
        if (fin) { dn = need; break; }
        dn += m * nv;
        pos = npos;
        if (!go) break;
        H = N;
#pragma unroll
        for (uint32_t j = 0; j < J; j++) xk[j] = nxk[j];
      }
    }
  }
  entry = pos;
  done = dn;
  runs_done = rd;
}

// Decode `need` level values of one stream into the sink; every thread of the workgroup
// calls this (control flow outside per-lane work is workgroup-uniform). Chunks are fixed
// stream ranges [k * kLvChunk, (k + 1) * kLvChunk); the chain enters chunk k where it left
// chunk k - 1 (chunks a long run jumps over are skipped).
template <bool BW1>
DEV void lv_walk(LevelLDS &L, LevelSink &sk, uint32_t need, Stamps &st) {
  static_assert(kLvPer == 8, "8 positions per thread");
  const uint8_t *s = sk.s;
  const uint32_t n = sk.n, bw = sk.bw, rs = (bw + 7) >> 3;
  const uint32_t tid = threadIdx.x;
  const uint32_t i0 = tid * kLvPer;
  constexpr uint32_t kWords = kLvStageB / 4 + 4, kWpt = (kWords + kLvThreads - 1) / kLvThreads;
  uint32_t pre[kWpt];
  auto fetch = [&](uint32_t cs) {
    const uint8_t *src = s + cs;
    const uint32_t lim = n > cs ? n - cs : 0;
#pragma unroll
    for (uint32_t j = 0; j < kWpt; j++) {
      const uint32_t k = tid + j * kLvThreads, o = 4 * k;
      pre[j] = (k < kWords && o < lim) ? (o + 4 <= lim ? ld32(src + o) : ld32(src + o) & ((1u << (8 * (lim - o))) - 1u)) : 0u;
    }
  };
  uint32_t entry = 0, done = 0, fetched = 0;  // fetched: chunk start the registers hold
  uint32_t runs_done = 0;                      // generic widths: run-table entries written so far
  // Generic widths: a chunk's run-table entries and fill-tile starts are collected in LDS and
  // stored at the top of the next chunk, before its prefetch is issued. vmcnt counts stores too
  // and loads and stores complete out of order, so the wait for a prefetch is a wait for every
  // earlier store: stores issued late in a chunk would put their latency on the critical path.
  uint32_t pend_n = 0, pend_t = 0, pend_base = 0;
  auto flush = [&]() {
    if constexpr (!BW1) {
      for (uint32_t e = tid; e < pend_n; e += kLvThreads) sk.runs[pend_base + e] = L.rbuf[e];
      for (uint32_t e = tid; e < pend_t; e += kLvThreads) sk.trun[2 * L.tb_k[e]] = L.tb_r[e];
      pend_n = pend_t = 0;
    }
  };
  // Generic widths: run-table entry idx (chain order) and the fill tiles whose first value it holds
  auto put_run = [&](uint32_t idx, uint32_t f, uint32_t cnt, uint32_t bp, uint32_t value) {
    if constexpr (!BW1) {
      L.rbuf[idx - runs_done] = make_uint2(f, bp ? 0x80000000u | value : value);
      if (cnt && sk.ntiles) {  // fill tiles whose first value lies in [f, f + cnt): tile k > 0 starts at k * T - a
        const uint64_t a = sk.tile_a;
        uint64_t k = f == 0 ? 0 : ((uint64_t)f + a + kLfTile - 1) / kLfTile;
        const uint64_t khi = min(((uint64_t)f + cnt - 1 + a) / kLfTile, (uint64_t)sk.ntiles - 1);
        for (; k <= khi; k++) {
          const uint32_t q = atomicAdd(&L.ntb, 1u);
          if (q < kLvTileBuf) { L.tb_k[q] = (uint32_t)k; L.tb_r[q] = idx; }
          else sk.trun[2 * k] = idx;
        }
      }
      atomicAdd(&L.nput, 1u);
    }
  };
  bool try_stride = true;  // (generic widths) the stride prelude at the top of the next chunk
  if (BW1 || !PQ_LV_STRIDE) fetch(0);  // (with the stride prelude: fetched when the chunk walk needs it)
  else fetched = ~0u;
  for (;;) {
    if (done >= need) break;
    if (entry >= n) { sk.error(done, PQ_ERR_EOF); break; }  // next header read at EOF
    if constexpr (!BW1) {
      if (PQ_LV_STRIDE && try_stride) {  // (workgroup-uniform)
        // Stride prelude (wave 0, straight from global memory; the run-header chain of hyb_scan's
        // prelude): while the chain's runs are long (>= kLvStrideMin stream bytes) and alike, lane k
        // decodes the header that would start k runs on if the runs between had this run's header.
        // Writers emit maximal literal runs back to back (Arrow's level streams: 63 groups, 64 B
        // at bit width 1, 127 B at 2), so the leading lanes with that exact header are chain nodes
        // by induction: up to 64 runs per step go to the run table (and the fill-tile starts they
        // hold), with no LDS staging and no list ranking. Anything else stops the prelude and the
        // chunk walk below takes the chain from there with the exact semantics.
        uint32_t pe = entry, pdn = done, pr = runs_done;  // (wave 0's walk; every wave reads the result)
        if (tid < 64) lv_stride(sk, need, pe, pdn, pr);
        if (tid == 0) { L.sp_e = pe; L.sp_d = pdn; L.sp_r = pr; }
        wg_barrier();
        // workgroup-uniform: every thread compares the same LDS value with the same old count (a
        // chunk walk follows; the prelude is tried again only after one that took runs)
        try_stride = L.sp_r != runs_done;
        entry = L.sp_e;
        done = L.sp_d;
        runs_done = L.sp_r;
        sk.nruns = runs_done;
        sk.covered = min(done, need);
        if (done >= need) break;
        if (entry >= n) { sk.error(done, PQ_ERR_EOF); break; }
      }
    }
    const uint32_t cs = entry - entry % kLvChunk, e0 = entry - cs;
    const uint32_t clen = min(kLvChunk, n - cs), send = cs + kLvStageB;
    if (fetched != cs) { fetch(cs); fetched = cs; }
    wg_barrier();  // the previous chunk's stage readers are done
    st.lap(7);
#pragma unroll
    for (uint32_t j = 0; j < kWpt; j++) {
      const uint32_t k = tid + j * kLvThreads;
      if (k < kWords) L.stage[k] = pre[j];
    }
    if (tid == 0) { L.nlong = 0; L.nput = 0; L.ntb = 0; L.stop_kind = LV_RUN; L.next_e = kNoEntry; }
    flush();
    if (cs + kLvChunk < n) { fetch(cs + kLvChunk); fetched = cs + kLvChunk; }  // lands during this chunk
    wg_barrier();
    st.lap(0);
    // ---- P1: links of positions [i0, i0 + 8) from five staged words; value counts kept
    uint32_t nv[kLvPer];
    {
      uint32_t W[5];
      {  // two 8-B reads and a dword (lanes 8 B apart: no two lanes of a read share a bank)
        const uint2 A0 = *(const uint2 *)&L.stage[2 * tid], A1 = *(const uint2 *)&L.stage[2 * tid + 2];
        W[0] = A0.x; W[1] = A0.y; W[2] = A1.x; W[3] = A1.y; W[4] = L.stage[2 * tid + 4];
      }
      uint32_t jj[kLvPer];
#pragma unroll
      for (uint32_t k = 0; k < kLvPer; k++) {
        const uint32_t i = i0 + k, c = cs + i, a = k >> 2, sh = k & 3;
        const uint32_t u0 = __builtin_amdgcn_alignbyte(W[a + 1], W[a], sh), u1 = __builtin_amdgcn_alignbyte(W[a + 2], W[a + 1], sh);
        // fast_hdr on register bytes: varint of <= 4 bytes, well-formed run complete in the stream
        const uint32_t t = ~u0 & 0x80808080u;
        const uint32_t Lv = (uint32_t)(__builtin_ctz(t | 0x80000000u) >> 3) + 1;
        uint32_t y = (Lv >= 4 ? u0 : (u0 & ((1u << (8 * Lv)) - 1u))) & 0x7f7f7f7fu;
        const uint32_t h = (y & 0x7fu) | ((y >> 1) & 0x3f80u) | ((y >> 2) & 0x1fc000u) | ((y >> 3) & 0xfe00000u);
        const uint32_t cnt = h >> 1, isbp = h & 1;
        const uint64_t adv = isbp ? Lv + (uint64_t)cnt * bw : (uint64_t)(Lv + rs);
        const uint32_t rv = (uint32_t)((((uint64_t)u1 << 32) | u0) >> (8 * Lv));
        const uint32_t rval = rs >= 4 ? rv : (rv & ((1u << (8 * rs)) - 1u));
        const bool ok = i < clen && t != 0 && cnt != 0 && (uint64_t)c + adv <= n && (isbp || bw >= 32 || (rval >> bw) == 0);
        nv[k] = ok ? (isbp ? cnt * 8 : cnt) : 0u;
        jj[k] = !ok ? i : ((uint64_t)i + adv >= clen ? (uint32_t)kLvExit : i + (uint32_t)adv);
      }
      *(uint4 *)&L.J0[i0] = make_uint4(jj[0] | (jj[1] << 16), jj[2] | (jj[3] << 16), jj[4] | (jj[5] << 16), jj[6] | (jj[7] << 16));
      *(uint2 *)&L.mark[i0] = make_uint2(0u, 0u);
    }
    wg_barrier();
    st.lap(1);
    // ---- P2: doubling into the ping-pong tables
    const uint16_t *top = L.J0;
    for (uint32_t lv = 0; lv < kLvLevels; lv++) {
      uint16_t *dst = (lv & 1) ? L.JB : L.JA;
      const uint4 A = *(const uint4 *)&top[i0];
      const uint32_t a[8] = {A.x & 0xffffu, A.x >> 16, A.y & 0xffffu, A.y >> 16, A.z & 0xffffu, A.z >> 16, A.w & 0xffffu, A.w >> 16};
      uint32_t r[8];
#pragma unroll
      for (uint32_t k = 0; k < 8; k++) {
        const bool fix = a[k] == kLvExit || a[k] == i0 + k;
        const uint32_t b2 = top[fix ? i0 + k : a[k]];
        r[k] = fix ? a[k] : b2;
      }
      *(uint4 *)&dst[i0] = make_uint4(r[0] | (r[1] << 16), r[2] | (r[3] << 16), r[4] | (r[5] << 16), r[6] | (r[7] << 16));
      top = dst;
      wg_barrier();
    }
    st.lap(2);
    // ---- P3: the checkpoints, by 2^kLvLevels-run jumps (one lane)
    if (tid == 0) {
      __builtin_amdgcn_s_setprio(3);
      uint32_t p = e0, k = 0;
      for (;;) {
        L.ckp[k++] = (uint16_t)p;
        const uint32_t q = top[p];
        if (q == kLvExit || q == p || k == kLvMaxCkp) break;
        p = q;
      }
      L.nckp = k;
      __builtin_amdgcn_s_setprio(0);
    }
    wg_barrier();
    st.lap(3);
    // ---- P4 (wave 0): one walker per checkpoint marks its 2^kLvLevels runs
    if (tid < L.nckp) {
      uint32_t p = L.ckp[tid];
      for (uint32_t k = 0; k < kLvSeg; k++) {
        L.mark[p] = 1;
        const uint32_t q = L.J0[p];
        if (q == p || q == kLvExit) break;
        p = q;
      }
    }
    wg_barrier();
    st.lap(4);
    // ---- P5: value counts of this thread's marked runs, workgroup scan
    uint32_t mbits = 0;
    {
      const uint2 M = *(const uint2 *)&L.mark[i0];
      const uint64_t m = ((uint64_t)M.y << 32) | M.x;
#pragma unroll
      for (uint32_t k = 0; k < 8; k++) mbits |= ((m >> (8 * k)) & 0xffu) ? 1u << k : 0u;
    }
    Hdr sh{0, 0, 0, 0, 1, 0, 0};  // the chain's stop, when this thread owns it
    uint32_t sk_k = 32;
    uint64_t mine = 0;
#pragma unroll
    for (uint32_t k = 0; k < 8; k++) mine += (mbits >> k) & 1u ? nv[k] : 0u;
    // generic widths: the marked runs' count rides in bits 48.. of the scan (values < 2^41)
    if constexpr (!BW1) mine += (uint64_t)__popc(mbits) << kLvRunShift;
    for (uint32_t mm = mbits; mm; mm &= mm - 1) {
      const uint32_t k = __builtin_ctz(mm);
      if (L.J0[i0 + k] == i0 + k) {  // a stop on the chain: the exact decoder (hybrid_decoder.go:142-165)
        sk_k = k;
        sh = decode_hdr(L.stage, cs, s, cs + i0 + k, n, bw, rs);
        mine += sh.err ? 0u : min(sh.nvals, sh.okvals);
        break;
      }
    }
    const uint32_t lane = lane_id(), wv = tid >> 6;
    const uint64_t incl = wave_incl_scan64_dpp(mine);
    if (lane == 63) L.wsum[wv] = incl;
    wg_barrier();
    uint64_t before = 0, total = 0;
#pragma unroll
    for (uint32_t q = 0; q < kLvThreads / 64; q++) {
      const uint64_t t = L.wsum[q];
      before += q < wv ? t : 0ull;
      total += t;
    }
    uint64_t ex = before + incl - mine;
    uint32_t ri = 0;  // generic widths: this thread's first entry in the chunk's part of the run table
    if constexpr (!BW1) {
      ri = runs_done + (uint32_t)(ex >> kLvRunShift);
      ex &= kLvValMask;
      total &= kLvValMask;
    }
    if (tid == 0) L.total = total;
    uint64_t v = (uint64_t)done + ex;  // value index of this thread's first marked run
    // Generic widths: the marked runs go to the stream's run table in global memory, in chain
    // order (first value index; bit-packed flag | payload position, or the RLE value), and the
    // run holding each fill tile's first value is noted for k_level_fill. Runs past num_values
    // and an error stop come last in chain order and are not written.
    auto put = [&](uint32_t f, uint32_t cnt, uint32_t bp, uint32_t value) {
      if constexpr (BW1) {
        lv_fill_run<true>(L, sk, cs, send, f, cnt, bp, value);
      } else {
        put_run(ri++, f, cnt, bp, value);
      }
    };
    // ---- P6: fill (and the chain's end: exit position or the exact stop)
    while (mbits) {
      const uint32_t k = __builtin_ctz(mbits);
      mbits &= mbits - 1;
      const uint32_t p = cs + i0 + k;
      if (v >= need) break;  // runs past the one that reaches num_values are never read
      const uint32_t rem = (uint32_t)min((uint64_t)need - v, (uint64_t)0xffffffffu);
      if (k == sk_k) {  // the chain's stop
        if (sh.err) {
          L.stop_kind = LV_STOP_ERR; L.stop_vpos = (uint32_t)v;
          L.stop_code = sh.err == kErrLongVarint ? resolve_long_varint(s, p, n) : sh.err;
        } else {
          const uint32_t ok = min(sh.nvals, sh.okvals);
          put((uint32_t)v, min(ok, rem), sh.bp, sh.value);
          if (ok < sh.nvals && ok < rem) {
            L.stop_kind = LV_STOP_TRUNC; L.stop_vpos = (uint32_t)v + ok; L.stop_code = PQ_ERR_EOF;
          } else {
            L.next_e = p + sh.adv;  // a valid run the fast form could not take: continue after it
          }
        }
        break;
      }
      const FastHdr f = fast_hdr(L.stage, cs, p, n, bw, rs);
      uint32_t nvk = 0;  // nv[k] by selects: a dynamic index would put nv[] in scratch memory
#pragma unroll
      for (uint32_t q = 0; q < kLvPer; q++) nvk = q == k ? nv[q] : nvk;
      put((uint32_t)v, min(nvk, rem), f.bp, f.value);
      if (L.J0[i0 + k] == kLvExit) L.next_e = p + f.adv;  // the chain's last node
      v += nvk;
    }
    st.lap(5);
    wg_barrier();
    if constexpr (!BW1) {
      pend_base = runs_done;
      pend_n = L.nput;
      pend_t = min(L.ntb, kLvTileBuf);
      runs_done += pend_n;
    }
    // long runs (bit width 1): every thread expands 32-value pieces
    const uint32_t nlong = L.nlong;
    for (uint32_t r = 0; r < nlong; r++) {
      const uint32_t f = L.long_f[r], cnt = L.long_cnt[r], bp = L.long_bp[r], lval = L.long_val[r];
      constexpr uint32_t P = BW1 ? 32 : 64;
      for (uint32_t q = tid * P; q < cnt; q += kLvThreads * P) {
        const uint32_t m = min(P, cnt - q);
        if constexpr (BW1) lv_emit_run<true>(sk, L.stage, cs, send, f + q, m, bp, bp ? lval + q / 8 : lval);
        else sk.piece(bp != 0, lval, f + q, q, m, L.stage, cs);
      }
    }
    if (nlong) wg_barrier();
    st.lap(6);
    const uint32_t kind = L.stop_kind;
    const uint64_t ndone = (uint64_t)done + L.total;
    sk.covered = (uint32_t)min(ndone, (uint64_t)need);
    sk.nruns = runs_done;
    if (kind != LV_RUN) {
      if (kind == LV_STOP_ERR || kind == LV_STOP_TRUNC) sk.error(L.stop_vpos, L.stop_code);
      break;
    }
    if (ndone >= need) break;
    done = (uint32_t)ndone;
    entry = L.next_e;  // kNoEntry cannot happen: a chain that needs more values exits or stops
    if (entry == kNoEntry) { sk.error(done, PQ_ERR_INVALID); break; }
  }
  flush();  // the last chunk's entries (written before its final barrier)
}

// BW1: every level stream of the pages is a bit-width-1 definition stream with validity
// output only (flat OPTIONAL columns: max_def == 1, max_rep == 0).
template <bool BW1>
DEV void levels_page(const BatchDev &b, const uint32_t *pages, LevelLDS &lds) {
  const uint32_t pi = pages[blockIdx.x];
  const PageDesc pd = b.pages[pi];
  const ChunkDesc &cd = b.chunks[pd.chunk];
  const uint8_t *base = gp_u64<const uint8_t>(pd.data);
  const uint32_t tid = threadIdx.x, lane = lane_id(), wv = tid >> 6;
  const uint32_t ns = pd.num_slots;
  uint32_t *vbits = gp_u64<uint32_t>(cd.validity);
  for (uint32_t k = tid; k < kSegSlots / 32; k += blockDim.x) lds.bits[k] = 0;
  uint32_t nn = ns;  // constDecoder(0) == maxD(0): every slot is a value
  PQ_STAMPS(st, b.dbg);
  st.begin();
  for (uint32_t which = 0; which < 2; which++) {
    const bool rep = which == 0;
    if (rep ? cd.max_rep == 0 : cd.max_def == 0) continue;
    LevelSink sk;
    sk.s = base + (rep ? pd.rep_off : pd.def_off);
    sk.n = rep ? pd.rep_len : pd.def_len;
    sk.bw = (uint32_t)(rep ? cd.rep_bw : cd.def_bw);
    sk.out = rep ? gp_u64<uint8_t>(cd.rep_levels) + pd.slot_base
                 : (cd.def_levels ? gp_u64<uint8_t>(cd.def_levels) + pd.slot_base : nullptr);
    sk.bits_lds = rep ? nullptr : lds.bits;
    sk.bits_glob = rep ? nullptr : vbits;
    sk.slot_base = pd.slot_base;
    sk.cmp = rep ? 0u : (uint32_t)cd.max_def;
    sk.count = 0;
    sk.err_code = 0;
    sk.err_pos = 0;
    sk.stage_len = kLvStageB;
    sk.ablate = b.ablate;
    wg_barrier();
    if (!(pd.flags & (rep ? PF_REP : PF_DEF))) {
      if (ns) sk.error(0, PQ_ERR_INVALID);  // "reader is not initialized"
    } else {
      lv_walk<BW1>(lds, sk, ns, st);
    }
    const uint64_t wc = wave_sum64(sk.count);
    if (lane == 0) lds.cnt[wv] = wc;
    wg_barrier();
    uint64_t cntv = 0;
    for (uint32_t k = 0; k < (blockDim.x >> 6); k++) cntv += lds.cnt[k];
    if (sk.err_code) {  // workgroup-uniform
      if (tid == 0) {
        report(b, pd.chunk, 1, pd.page_in_chunk, rep ? ST_REP : ST_DEF, sk.err_pos, sk.err_code);
        b.page_nn[pi] = 0;
        if (rep) b.page_rec[pi] = (uint32_t)cntv;
      }
      st.flush(0);
      return;  // the reference fails the page at the first level error
    }
    if (rep) {
      if (tid == 0) b.page_rec[pi] = (uint32_t)cntv;
    } else {
      nn = (uint32_t)cntv;
    }
    wg_barrier();
  }
  if (cd.max_def > 0) {
    wg_barrier();
    // flush the LDS bitmap segment to the chunk bitmap
    const uint32_t seg = min(ns, kSegSlots);
    const uint32_t nw = (seg + 31) / 32;
    const uint32_t sh = (uint32_t)(pd.slot_base & 31);
    const uint64_t w0 = pd.slot_base >> 5;
    for (uint32_t k = tid; k < nw; k += blockDim.x) {
      uint32_t v = lds.bits[k];
      if (k == nw - 1 && (seg & 31)) v &= (1u << (seg & 31)) - 1u;
      if (sh == 0) {
        if (k == 0 || k == nw - 1) atomicOr(&vbits[w0 + k], v);
        else vbits[w0 + k] = v;
      } else if (v) {
        atomicOr(&vbits[w0 + k], v << sh);
        uint32_t hi = v >> (32 - sh);
        if (hi) atomicOr(&vbits[w0 + k + 1], hi);
      }
    }
  }
  st.lap(6);
  st.flush(0);
  if (tid == 0) b.page_nn[pi] = nn;
}

// ---------------------------------------------------------------------------
// k_levels_bw1w: flat OPTIONAL pages (definition levels of bit width 1, validity output), ONE
// wavefront per page (hybrid_decoder.go:81-165 through decodePackedArray helpers.go:133-149).
//
// The run-header chain is walked 64 stream positions per step: lane l decodes the header that
// would start at pos + l from a 1 KiB LDS ring of the stream (two 512-B halves; the next half is
// loaded into registers while the current one is walked), the true chain is followed lane to lane
// with one readlane per run, and the step's runs expand in parallel into an LDS bitmap of the
// page's first kSegSlots slots (the chunk bitmap beyond): RLE runs of ones set a bit range, bit-
// packed runs OR their payload words (bit k of the payload = value k). pyarrow's streams have
// runs of ~2.7 bytes, so a step covers ~24 runs; a page of 65,536 slots is ~150 steps of one wave
// and every page of a batch is resident at once (a 4-wave list-ranking workgroup per page held 27
// KB of LDS and 80 VGPRs, six pages per CU).
// A header the fast decode does not take (a varint of more than 4 bytes, a run reaching past the
// stream or 72 bytes, an RLE value >= 2, a zero count, EOF) is decoded exactly (decode_hdr, the
// reference's full header semantics) by the whole wave: an error ends the page at the value where
// next() fails, a valid run is expanded cooperatively and the chain continues after it. Runs past
// the one that reaches num_values are never read.
// ---------------------------------------------------------------------------
constexpr uint32_t kLwRing = 1024;             // LDS ring of stream bytes (two halves)
constexpr uint32_t kLwHalf = kLwRing / 2;
constexpr uint32_t kLwMaxAdv = 72;             // fast runs: header + payload within 72 bytes
constexpr uint32_t kLwLong = 512;              // runs longer than this expand with the whole wave
struct LevelWaveLDS {
  uint32_t bits[kSegSlots / 32];  // the page's first kSegSlots validity bits
  uint32_t ring[kLwRing / 4];     // stream dword k (of the 4-B aligned stream) in slot k mod 256
};

// 4 stream bytes at aligned offset ax (the ring holds aligned bytes [RA, RA + kLwRing))
DEV uint32_t lw_bytes4(const uint32_t *ring, uint32_t ax) {
  const uint32_t k = ax >> 2, sh = ax & 3;
  const uint32_t w0 = ring[k & (kLwRing / 4 - 1)], w1 = ring[(k + 1) & (kLwRing / 4 - 1)];
  return __builtin_amdgcn_alignbyte(w1, w0, sh);
}

// One half of the ring: aligned bytes [A, A + kLwHalf) of the stream (bytes at or past the stream
// end read as zero), two dwords per lane.
struct LwHalf { uint32_t d0, d1; };
DEV LwHalf lw_load(const uint32_t *sal, uint32_t A, uint32_t nal) {
  const uint32_t lane = lane_id();
  LwHalf h;
  uint32_t *o[2] = {&h.d0, &h.d1};
#pragma unroll
  for (uint32_t j = 0; j < 2; j++) {
    const uint32_t x = A + 4 * (lane + 64 * j);  // aligned byte offset of the dword
    uint32_t v = 0;
    if (x < nal) {
      v = sal[x >> 2];
      if (x + 4 > nal) v &= (1u << (8 * (nal - x))) - 1u;
    }
    *o[j] = v;
  }
  return h;
}
DEV void lw_store(uint32_t *ring, uint32_t A, const LwHalf &h) {
  const uint32_t lane = lane_id(), k = A >> 2;
  ring[(k + lane) & (kLwRing / 4 - 1)] = h.d0;
  ring[(k + lane + 64) & (kLwRing / 4 - 1)] = h.d1;
}

// Expand one run with the whole wave: values [0, take) of the run (RLE value `val`, or bit-packed
// with payload at stream byte `pay`, read from global memory with zero past the end).
DEV void lw_run_wave(LevelSink &sk, uint32_t first, uint32_t take, bool bp, uint32_t val, uint32_t pay) {
  for (uint32_t q = lane_id() * 32; q < take; q += 64 * 32) {
    const uint32_t m = take - q >= 32 ? ~0u : ((1u << (take - q)) - 1u);
    uint32_t w;
    if (bp) w = bits32c(sk.s, sk.n, (uint64_t)pay * 8 + q, 32) & m;
    else w = val == sk.cmp ? m : 0u;
    sk.count += __popc(w);
    lv_or_bits(sk, first + q, w);
  }
}

DEV void lw_walk(LevelSink &sk, uint32_t need, uint32_t *ring) {
  const uint32_t lane = lane_id();
  const uint8_t *s = sk.s;
  const uint32_t n = sk.n;
  const uint32_t sa = (uint32_t)((uintptr_t)s & 3u);
  const uint32_t *sal = (const uint32_t *)(s - sa);  // 4-B aligned view (pointer arithmetic keeps the space)
  const uint32_t nal = n + sa;
  // exact decodes read the stream straight from global memory (decode_hdr's "stage" = the aligned view)
  const uint32_t gsb = 0u - sa;
  uint32_t pos = 0, done = 0;
  uint32_t RA = 0;  // aligned offset of the ring's first half (a multiple of kLwHalf)
  lw_store(ring, 0, lw_load(sal, 0, nal));
  lw_store(ring, kLwHalf, lw_load(sal, kLwHalf, nal));
  LwHalf nxt = lw_load(sal, kLwRing, nal);
  wave_lds_sync();
  while (done < need) {
    // ---- keep pos in the ring's first half
    const uint32_t ap = pos + sa;
    if (ap >= RA + kLwHalf) {
      if (ap < RA + kLwRing) {
        lw_store(ring, RA + kLwRing, nxt);  // the dead first half takes [RA + 1024, RA + 1536)
        RA += kLwHalf;
      } else {  // jumped past the ring (a long run): restage
        RA = ap & ~(kLwHalf - 1);
        lw_store(ring, RA, lw_load(sal, RA, nal));
        lw_store(ring, RA + kLwHalf, lw_load(sal, RA + kLwHalf, nal));
      }
      nxt = lw_load(sal, RA + kLwRing, nal);
      wave_lds_sync();
    }
    // ---- fast decode of the header that would start at c = pos + lane (bit width 1: the RLE value
    // is one byte and must be 0 or 1; a bit-packed run of k groups has k payload bytes)
    const uint32_t c = pos + lane, ac = c + sa;
    const uint32_t u0 = lw_bytes4(ring, ac), u1 = lw_bytes4(ring, ac + 4);
    const uint32_t t = ~u0 & 0x80808080u;
    const uint32_t L = (uint32_t)(__builtin_ctz(t | 0x80000000u) >> 3) + 1;
    const uint32_t y = (L >= 4 ? u0 : (u0 & ((1u << (8 * L)) - 1u))) & 0x7f7f7f7fu;
    const uint32_t h = (y & 0x7fu) | ((y >> 1) & 0x3f80u) | ((y >> 2) & 0x1fc000u) | ((y >> 3) & 0xfe00000u);
    const uint32_t cnt = h >> 1, isbp = h & 1u;
    const uint32_t adv = isbp ? L + cnt : L + 1;
    const uint32_t v = (uint32_t)((((uint64_t)u1 << 32) | u0) >> (8 * L)) & 0xffu;
    const uint32_t nv = isbp ? cnt * 8 : cnt;
    const bool ok = t != 0 && cnt != 0 && adv <= kLwMaxAdv && (uint64_t)c + adv <= n && (isbp || v <= 1) &&
                    nv < (1u << 24);
    const uint32_t pk = ok ? adv | (nv << 8) : 0u;
    // ---- the true chain, lane to lane
    const uint32_t rem = need - done;
    uint64_t mask = 0;
    uint32_t cur = 0, cum = 0;
    bool stop = false, last = false;
    while (cur < 64) {
      const uint32_t pc = (uint32_t)__builtin_amdgcn_readlane((int)pk, (int)cur);
      if (!pc) { stop = true; break; }
      mask |= 1ull << cur;
      const uint32_t nvc = pc >> 8;
      if (nvc >= rem - cum) { cum = rem; last = true; break; }
      cum += nvc;
      cur += pc & 0xffu;
    }
    // ---- the step's runs expand in parallel
    const bool mine = (mask >> lane) & 1ull;
    const uint32_t first = wave_excl_scan(mine ? nv : 0u);
    const uint32_t take = mine ? min(nv, rem - first) : 0u;
    const uint32_t f = done + first;
    if (take && (isbp || take <= kLwLong)) {  // (a fast bit-packed run has at most 71 groups)
      if (isbp) {
        const uint32_t pay = ac + L;  // aligned offset of the payload
        for (uint32_t q = 0; q < take; q += 32) {
          const uint32_t m = take - q >= 32 ? ~0u : ((1u << (take - q)) - 1u);
          const uint32_t w = lw_bytes4(ring, pay + (q >> 3)) & m;
          sk.count += __popc(w);
          lv_or_bits(sk, f + q, w);
        }
      } else if (v == sk.cmp) {
        sk.count += take;
        for (uint32_t q = 0; q < take; q += 32) lv_or_bits(sk, f + q, take - q >= 32 ? ~0u : ((1u << (take - q)) - 1u));
      }
    }
    for (uint64_t big = __ballot(!isbp && take > kLwLong); big; big &= big - 1) {  // long RLE runs: the whole wave
      const uint32_t r = (uint32_t)__builtin_ctzll(big);
      lw_run_wave(sk, rdlane(f, r), rdlane(take, r), false, rdlane(v, r), 0);
    }
    done += cum;
    if (last) break;
    if (!stop) { pos += cur; continue; }
    // ---- the header at pos + cur, decoded exactly
    const uint32_t P = pos + cur;
    const Hdr eh = decode_hdr(sal, gsb, s, P, n, 1, 1);
    if (eh.err) {
      sk.error(done, eh.err == kErrLongVarint ? resolve_long_varint(s, P, n) : eh.err);
      break;
    }
    const uint32_t okv = min(eh.nvals, eh.okvals), r2 = need - done, tk = min(okv, r2);
    lw_run_wave(sk, done, tk, eh.bp != 0, eh.value, eh.value);
    if (okv < eh.nvals && okv < r2) {  // a bit-packed run cut by EOF: next() fails after its groups
      sk.error(done + okv, PQ_ERR_EOF);
      break;
    }
    done += tk;
    pos = P + eh.adv;
  }
}

__global__ void __launch_bounds__(64) k_levels_bw1w(BatchDev b_in, const uint32_t *pages) {
  const BatchDev b = global_view(b_in);
  __shared__ LevelWaveLDS L;
  const uint32_t pi = pages[blockIdx.x], lane = lane_id();
  const PageDesc pd = b.pages[pi];
  const ChunkDesc &cd = b.chunks[pd.chunk];
  const uint32_t ns = pd.num_slots;
  uint32_t *vbits = gp_u64<uint32_t>(cd.validity);
  for (uint32_t k = lane; k < kSegSlots / 32; k += 64) L.bits[k] = 0;
  LevelSink sk;
  sk.s = gp_u64<const uint8_t>(pd.data) + pd.def_off;
  sk.n = pd.def_len;
  sk.bw = 1;
  sk.out = nullptr;
  sk.bits_lds = L.bits;
  sk.bits_glob = vbits;
  sk.slot_base = pd.slot_base;
  sk.cmp = (uint32_t)cd.max_def;  // 1
  sk.count = 0;
  sk.err_code = 0;
  sk.err_pos = 0;
  sk.stage_len = 0;
  sk.ablate = b.ablate;
  wave_lds_sync();
  if (!(pd.flags & PF_DEF)) {
    if (ns) sk.error(0, PQ_ERR_INVALID);  // "reader is not initialized"
  } else if (ns) {
    lw_walk(sk, ns, L.ring);
  }
  const uint32_t cnt = (uint32_t)wave_sum64(sk.count);
  if (sk.err_code) {  // wave-uniform: the reference fails the page at the first level error
    if (lane == 0) {
      report(b, pd.chunk, 1, pd.page_in_chunk, ST_DEF, sk.err_pos, sk.err_code);
      b.page_nn[pi] = 0;
    }
    return;
  }
  wave_lds_sync();
  // the LDS bitmap segment to the chunk bitmap (the first and last words may be shared with the
  // neighbouring pages: OR-ed atomically)
  const uint32_t seg = min(ns, kSegSlots), nw = (seg + 31) / 32;
  const uint32_t sh = (uint32_t)(pd.slot_base & 31);
  const uint64_t w0 = pd.slot_base >> 5;
  for (uint32_t k = lane; k < nw; k += 64) {
    uint32_t x = L.bits[k];
    if (k == nw - 1 && (seg & 31)) x &= (1u << (seg & 31)) - 1u;
    if (sh == 0) {
      if (k == 0 || k == nw - 1) atomicOr(&vbits[w0 + k], x);
      else vbits[w0 + k] = x;
    } else if (x) {
      atomicOr(&vbits[w0 + k], x << sh);
      const uint32_t hi = x >> (32 - sh);
      if (hi) atomicOr(&vbits[w0 + k + 1], hi);
    }
  }
  if (lane == 0) b.page_nn[pi] = cnt;
}

// ---------------------------------------------------------------------------
// k_levels_seg: flat OPTIONAL pages (bit width 1 definition levels -> validity bitmap and non-null
// count; hybrid_decoder.go:81-165 through decodePackedArray helpers.go:133-149), ONE wavefront per
// page, by verified speculation over stream segments (no workgroup barrier, no list ranking).
//
// The run-header chain is serial: run k+1 starts where run k ends. The stream (staged in LDS) is
// cut into 64 segments [lo_i, hi_i), one per lane. Lane i starts kSg1Margin bytes before its
// segment at an arbitrary byte and walks run headers speculatively (a header that is not a
// well-formed run, or one that would jump more than kSg1Cap bytes, moves it one byte on); a chain
// started anywhere joins the true chain within a few runs. Measured offline on pyarrow's def-level
// streams (tools/sim_level_join.py): with hops capped at 16 bytes 99.6 % of the lanes of a 10 %-null
// stream are on the true chain before their segment starts, from 48 bytes ahead (round 5's 72-byte
// cap needed 128 bytes for 98.8 %: a garbage walker that takes long bit-packed "runs" out of payload
// bytes rarely lands back on the chain, one that steps byte by byte does). Its first position at or
// past lo_i is its ENTRY; from there it walks exactly (every fast run is taken, whatever its length)
// up to the first position at or past hi_i, its EXIT, counting the values of the runs it passed.
// Verification is exact: lane 0 starts at stream position 0; lane i's chain IS the true chain from
// its entry on iff entry_i == exit_(i-1) and lane i-1 is verified (chains are deterministic
// functions of a position). The first lane that fails (or stopped at a header the fast decoder does
// not take: a varint over 2 bytes, a run cut by EOF, an error) is re-walked from its predecessor's
// exit with the reference's full header semantics (decode_hdr), uniformly by the wave; then the
// next one, in lane order. A long run that jumps over whole segments leaves them empty.
// Then a wave scan of the lanes' value counts gives every run its first value index, and each lane
// walks its verified range again and writes its values' validity bits into the page's bitmap image
// in LDS: a lane's values are one contiguous bit range, assembled in a 64-bit register accumulator;
// words inside the range are plain LDS stores, the range's first and last words (shared with the
// neighbouring lanes) LDS atomic ORs; null runs only move the cursor. Runs of more than kSgLong values
// go to the whole wave. The image is then stored to the chunk bitmap with coalesced stores (atomic OR
// only for the page's two edge words, which the neighbouring pages share; slots past the image's
// kSg1Words words go to the chunk bitmap directly). Runs past the one that reaches num_values are
// never read; an error is the page's only if the reference's next() meets it before num_values (same
// class, same value position as decodePackedArray), and a failing page writes nothing.
// Round 6: the hop reads 4 bytes and decodes 1- and 2-byte varints only (the longer ones stop the
// lane for the exact re-walk, or take the general decoder on a verified range), the speculative hops
// are capped at 16 bytes, and the bitmap is assembled in LDS: round 5's loop spent ~23 K issued
// instructions per page beside the DELTA launch, and its scattered per-lane global stores moved 1.6x
// the bitmap's bytes.
// ---------------------------------------------------------------------------
constexpr uint32_t kSgStage = kSgStageHost;  // LDS stage; pages whose stream does not fit take k_levels_bw1
constexpr uint32_t kSgSlack = 128;    // zero bytes after the stage (reads of lanes past their range)
constexpr uint32_t kSgMargin = 128;   // k_levels_segw: bytes a lane walks speculatively before its segment
constexpr uint32_t kSgCap = 72;       // k_levels_segw: a speculative hop longer than this is not taken
constexpr uint32_t kSg1Margin = 48;   // k_levels_seg: the same two for bit width 1 streams
constexpr uint32_t kSg1Cap = 16;
constexpr uint32_t kSgLong = 1024;    // runs of more values (not null runs) expand with the whole wave
constexpr uint32_t kSgQueue = 64;
constexpr uint32_t kSg1Words = 2056;  // bitmap image: page bits [slot_base & ~31, + 32 * kSg1Words)
static_assert(kSgImageSlotsHost / 32 <= kSg1Words, "host: pages the image holds whole (unzeroed bitmaps)");
constexpr uint32_t kSg1Image = 2124;  // image words with one pad word per 32 (sg1_sw), a multiple of 4
enum : uint32_t { SG_OK = 0, SG_STOP = 1, SG_ERR = 2, SG_TRUNC = 3 };
struct LevelSegLDS {
  uint32_t stage[(kSgStage + kSgSlack) / 4];  // stream bytes from the 16-B aligned address below s
  uint32_t bm[kSg1Image];                     // the page's bitmap image (word w at sg1_sw(w))
  uint32_t qg[kSgQueue], qc[kSgQueue], qv[kSgQueue], nq;  // long runs: first bit, count, bp | payload / 1
};
// Image word w at w + w / 32: the lanes' current words are ~32 words apart (1,024 values each), which
// would put every lane of a store on one bank.
DEV uint32_t sg1_sw(uint32_t w) { return w + (w >> 5); }

// Bytes [p, p + 8) of the staged stream (stage byte o = stream byte o - sa; zero past the stream).
DEV uint64_t sg_bytes8(const uint32_t *stage, uint32_t o) {
  const uint32_t a = o >> 2, sh = o & 3;
  const uint32_t w0 = stage[a], w1 = stage[a + 1], w2 = stage[a + 2];
  return (uint64_t)__builtin_amdgcn_alignbyte(w1, w0, sh) | ((uint64_t)__builtin_amdgcn_alignbyte(w2, w1, sh) << 32);
}
DEV uint32_t sg_bytes4(const uint32_t *stage, uint32_t o) {
  const uint32_t a = o >> 2;
  return __builtin_amdgcn_alignbyte(stage[a + 1], stage[a], o & 3);
}

// The fast form of the header whose 8 bytes are x, at stream position p (bit width 1): a varint of
// at most 4 bytes announcing a well formed run complete inside the stream (RLE value 0 or 1; a
// bit-packed run of k groups has k payload bytes). adv == 0: not a fast header (decode_hdr decides).
struct SgHop { uint32_t adv, nv, bp, val, L; };
DEV SgHop sg_decode(uint64_t x, uint32_t p, uint32_t n) {
  const uint32_t u0 = (uint32_t)x;
  const uint32_t t = ~u0 & 0x80808080u;
  const uint32_t L = (uint32_t)(__builtin_ctz(t | 0x80000000u) >> 3) + 1;
  const uint32_t y = (L >= 4 ? u0 : (u0 & ((1u << (8 * L)) - 1u))) & 0x7f7f7f7fu;
  const uint32_t h = (y & 0x7fu) | ((y >> 1) & 0x3f80u) | ((y >> 2) & 0x1fc000u) | ((y >> 3) & 0xfe00000u);
  const uint32_t cnt = h >> 1, bp = h & 1u;
  const uint32_t adv = bp ? L + cnt : L + 1;
  const uint32_t v = (uint32_t)(x >> (8 * L)) & 0xffu;
  const bool ok = t != 0 && cnt != 0 && (uint64_t)p + adv <= n && (bp || v <= 1);
  SgHop r;
  r.adv = ok ? adv : 0u;
  r.nv = bp ? cnt * 8 : cnt;  // cnt < 2^27
  r.bp = bp;
  r.val = bp ? p + L : v;
  r.L = L;
  return r;
}
// The same for varints of 1 or 2 bytes (runs of fewer than 8,192 values or groups) from the 4 bytes
// x at p: the hop of k_levels_seg's walks. adv == 0: not taken here (sg_decode / decode_hdr).
// Branch-free (bitwise flags, selects): it is the body of the walk loops.
DEV SgHop sg_fast(uint32_t x, uint32_t p, uint32_t n) {
  const uint32_t two = (x >> 7) & 1u;  // a second varint byte
  const uint32_t h = (x & 0x7fu) | ((x >> 1) & (0x3f80u & (0u - two)));
  const uint32_t L = 1u + two;
  const uint32_t cnt = h >> 1, bp = h & 1u;
  const uint32_t adv = L + (bp ? cnt : 1u);
  const uint32_t v = __builtin_amdgcn_ubfe(x, 8u + 8u * two, 8u);  // RLE value byte
  const uint32_t ok = (((x >> 15) & two) ^ 1u) & (uint32_t)(cnt != 0) & (uint32_t)(p + adv <= n) &
                      (bp | (uint32_t)(v <= 1u));
  SgHop r;
  r.adv = ok ? adv : 0u;
  r.nv = bp ? cnt << 3 : cnt;
  r.bp = bp;
  r.val = bp ? p + L : v;
  r.L = L;
  return r;
}

// A lane's validity bits, in value order, into the page's bitmap image (LDS, pre-zeroed; words past
// the image: the chunk bitmap, pre-zeroed every decode): bits gather in a 64-bit accumulator and
// every finished or last word is OR-ed in (the first and last words of a lane's range are shared
// with the neighbouring lanes; on the zeroed image an OR is the store for the others).
struct SgBits {
  uint32_t *bm;  // LDS image
  uint32_t *vb;  // chunk bitmap from the image's word 0
  uint64_t acc;
  uint32_t w, o, ones;  // word of the accumulator's bit 0, bits in use, ones written
  bool nostore;  // diagnostic build: PQ_ABLATE bit 20 (no bitmap stores)
  DEV void start(uint32_t g) { w = g >> 5; o = g & 31; acc = 0; }
  DEV void put(uint32_t x) {
    if (x && !nostore) {
      if (w < kSg1Words) atomicOr(&bm[sg1_sw(w)], x);
      else atomicOr(&vb[w], x);
    }
  }
  DEV void step(uint32_t x, uint32_t k) {  // k values, bits x (x == 0 whenever k > 32)
    ones += __popc(x);
    acc |= (uint64_t)x << o;
    const uint32_t t = o + k;
    if (t >= 32) {  // (t >= 64 only for nulls: acc >> 32 is then 0 and the words between stay zero)
      put((uint32_t)acc);
      acc >>= 32;
      w += t >> 5;
    }
    o = t & 31;
  }
  DEV void end() {  // the range's last word, shared with whoever writes the bits after it
    if (o) put((uint32_t)acc);
    o = 0;
  }
};

// One long run (image bits [g, g + c)) by the whole wave: image word w takes run bits [32 w - g, +32),
// OR-ed in (the edge words are shared). Returns this lane's ones.
DEV uint32_t sg1_run_wave(LevelSegLDS &L, uint32_t *vb, uint32_t sa, uint32_t g, uint32_t c, bool bp,
                          uint32_t pay) {
  const uint32_t lane = lane_id();
  const uint32_t w0 = g >> 5, w1 = (g + c - 1) >> 5;
  uint32_t ones = 0;
  for (uint32_t w = w0 + lane; w <= w1; w += 64) {
    const int32_t r = (int32_t)(w * 32) - (int32_t)g;  // run bit at the word's bit 0 (negative: first word)
    const uint32_t lo = r < 0 ? (uint32_t)(-r) : 0u;   // word bits before the run
    const uint32_t rb = r > 0 ? (uint32_t)r : 0u;      // the word's first run bit
    const uint32_t nb = min(32u - lo, c - rb);
    uint32_t x = bp ? (uint32_t)(sg_bytes8(L.stage, pay + sa + (rb >> 3)) >> (rb & 7)) : ~0u;
    x &= nb == 32 ? ~0u : ((1u << nb) - 1u);
    x <<= lo;
    ones += __popc(x);
    if (x) {
      if (w < kSg1Words) atomicOr(&L.bm[sg1_sw(w)], x);
      else atomicOr(&vb[w], x);
    }
  }
  return ones;
}

DEV void levels_seg_page(const BatchDev &b, LevelSegLDS &L, const uint32_t pi) {
  const uint32_t lane = lane_id();
  const PageDesc pd = b.pages[pi];
  const ChunkDesc &cd = b.chunks[pd.chunk];
  const uint32_t ns = pd.num_slots;
  const uint32_t o0 = (uint32_t)(pd.slot_base & 31u);                        // image bit of the page's slot 0
  uint32_t *vbw = gp_u64<uint32_t>(cd.validity) + (uint32_t)(pd.slot_base >> 5);  // chunk word of image word 0
  const uint8_t *s = gp_u64<const uint8_t>(pd.data) + pd.def_off;
  const uint32_t n = pd.def_len;  // n + 24 <= kSgStage (host)
  // diagnostic build: 0 stage, 1 A, 2 B, 3 C+D, 4 image store; 5 B iterations, 6 A steps, 7 D steps
  PQ_STAMPS(stp, b.dbg);
  stp.begin();
  // ---- stage: the stream from the 16-B aligned address at or below s, zero at and past its end
  // (a short final group zero-fills; lanes past their range read zeros); the image zeroed
  const uint32_t sa = (uint32_t)((uintptr_t)s & 15u);
  {
    // the stream's 16-B blocks, four loads in flight per lane, then two zero blocks past its end
    // (reads past the stream: an 8-byte header read or a funnel at most 12 bytes on)
    const uint4 *g = (const uint4 *)(s - sa);
    const uint32_t lim = n + sa;
    const uint32_t nv = (lim + 15) / 16, nz = min(nv + 2, (kSgStage + kSgSlack) / 16);
    auto masked = [&](uint4 x, uint32_t k) {
      const int32_t rel = (int32_t)(lim - 16 * k);
      if (rel >= 16) return x;
      uint32_t q[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const int32_t r = rel - 4 * i;
        q[i] = r >= 4 ? q[i] : (r <= 0 ? 0u : (q[i] & ((1u << (8 * r)) - 1u)));
      }
      return make_uint4(q[0], q[1], q[2], q[3]);
    };
    for (uint32_t k0 = 0; k0 < nv; k0 += 256) {
      uint4 x[4];
#pragma unroll
      for (uint32_t u = 0; u < 4; u++) {
        const uint32_t k = k0 + 64 * u + lane;
        x[u] = k < nv ? g[k] : make_uint4(0u, 0u, 0u, 0u);
      }
#pragma unroll
      for (uint32_t u = 0; u < 4; u++) {
        const uint32_t k = k0 + 64 * u + lane;
        if (k < nv) *(uint4 *)&L.stage[4 * k] = masked(x[u], k);
      }
    }
    for (uint32_t k = nv + lane; k < nz; k += 64) *(uint4 *)&L.stage[4 * k] = make_uint4(0u, 0u, 0u, 0u);
    const uint32_t nimg = min(sg1_sw(min((o0 + ns + 31) >> 5, kSg1Words)) + 1, kSg1Image);
    for (uint32_t k = lane; 4 * k < nimg; k += 64) *(uint4 *)&L.bm[4 * k] = make_uint4(0u, 0u, 0u, 0u);
    if (lane == 0) L.nq = 0;
  }
  uint32_t err_pos = 0, err = 0, ones = 0;
  wave_lds_sync();
  stp.lap(0);
  const uint32_t need = ns;
  const uint32_t sa4 = (uint32_t)((uintptr_t)s & 3u);
  const uint32_t *s4 = (const uint32_t *)(s - sa4);  // decode_hdr's view: global memory
  if (!(pd.flags & PF_DEF)) {
    if (ns) err = PQ_ERR_INVALID;  // "reader is not initialized"
  } else if (ns) {
    // ---- A. speculative walks: segment [lo, hi) of lane i (branch-free body: every lane runs the
    // same instructions; a lane past its range only reads). A lane that starts at stream position 0
    // is on the chain from the start: its hops are not capped and a header it cannot take stops it.
    // segment bytes: an odd number of dwords, so the lanes' reads (about a segment apart) fall in
    // different LDS banks
    const uint32_t S = 4 * ((max((n + 63) / 64, 16u) + 3) / 8 * 2 + 1);
    const uint32_t lo = lane * S, hi = lo + S;
    const uint32_t lim = lo < n ? min(hi, n) : 0u;
    uint32_t p = (lane == 0 || lo <= kSg1Margin || lo >= n) ? 0u : lo - kSg1Margin;
    const uint32_t from0 = (uint32_t)(p == 0);
    uint32_t entry = lo < n ? (p >= lo ? p : ~0u) : n, cnt = 0, st = SG_OK;
    for (;;) {
      const bool act = st == SG_OK && p < lim;
      if (!__ballot(act)) break;
      stp.count(6);
      const SgHop h = sg_fast(sg_bytes4(L.stage, p + sa), p, n);
      const uint32_t spec = (uint32_t)(p < lo), exact = (spec ^ 1u) | from0, a = (uint32_t)act;
      const uint32_t take = (uint32_t)(h.adv != 0) & (exact | (uint32_t)(h.adv <= kSg1Cap));
      const uint32_t np = take ? p + h.adv : p + 1u;
      const uint32_t stop = a & exact & (take ^ 1u);  // (a stop does not move: st ends the walk)
      cnt += (a & (spec ^ 1u) & take) ? h.nv : 0u;
      entry = (a & spec & (uint32_t)(np >= lo)) ? np : entry;
      p = (a & (stop ^ 1u)) ? np : p;
      st = stop ? SG_STOP : st;
    }
    uint32_t exit = lo < n ? p : n;
    if (lo < n && entry == ~0u) entry = p;  // (a lane from 0 that stopped before its segment: fails B)
    stp.lap(1);
    // ---- B. verification in lane order; the first failing lane is re-walked exactly from its
    // predecessor's (verified) exit, uniformly by the wave
    uint32_t err_code = 0;
    auto bad_mask = [&]() {
      const uint32_t prev = __shfl_up(exit, 1, 64);
      const bool ok = st == SG_OK && (lane == 0 ? entry == 0 : entry == prev);
      return __ballot(!ok);
    };
    uint64_t bad = bad_mask();
    uint32_t f_dead = 64;  // lanes from here on hold no runs (the chain ended before them)
    while (bad) {
      const uint32_t f = (uint32_t)__builtin_ctzll(bad);
      stp.count(5);
      // values of the verified lanes before f: once they reach num_values, nothing after matters
      const uint32_t before = (uint32_t)wave_sum64(lane < f ? cnt : 0u);
      if (before >= need) { f_dead = f; break; }
      uint32_t P = f ? rdlane(exit, f - 1) : 0u;
      const uint32_t fhi = f * S + S;
      uint32_t c = 0, fst = SG_OK, fcode = 0;
      const uint32_t fentry = P;
      while (P < fhi && P < n && before + c < need) {
        const SgHop h = sg_decode(sg_bytes8(L.stage, P + sa), P, n);
        if (h.adv) { c += h.nv; P += h.adv; continue; }
        // the reference's full header semantics
        const Hdr eh = decode_hdr(s4, 0u - sa4, s, P, n, 1, 1);
        if (eh.err) {
          fst = SG_ERR;
          fcode = eh.err == kErrLongVarint ? resolve_long_varint(s, P, n) : eh.err;
          break;
        }
        const uint32_t okv = min(eh.nvals, eh.okvals);
        if (okv < eh.nvals) {  // a bit-packed run cut by EOF: next() fails after its groups
          c += okv;
          fst = SG_TRUNC;
          fcode = PQ_ERR_EOF;
          break;
        }
        c += eh.nvals;
        P += eh.adv;
      }
      if (lane == f) {
        entry = fentry;
        exit = P;
        cnt = c;
        st = fst;
        err_code = fcode;
      }
      if (fst != SG_OK || P >= n || before + c >= need) {
        f_dead = f + 1;  // the chain ends in lane f (error, EOF, stream end or num_values)
        break;
      }
      bad = bad_mask() & ~((2ull << f) - 1ull);  // lanes <= f are verified now
    }
    if (lane >= f_dead) { cnt = 0; st = SG_OK; }
    stp.lap(2);
    // ---- C. value bases; the reference's first failure before num_values
    const uint32_t base = wave_excl_scan(cnt);
    const uint32_t total = (uint32_t)wave_sum64(cnt);
    {
      const uint64_t em = __ballot((st == SG_ERR || st == SG_TRUNC) && base + cnt < need);
      if (em) {
        const uint32_t e = (uint32_t)__builtin_ctzll(em);
        err_pos = rdlane(base + cnt, e);
        err = rdlane(err_code, e);
      } else if (total < need) {
        err_pos = total;  // the chain ended at the stream end: next() reads a header at EOF
        err = PQ_ERR_EOF;
      }
    }
    // ---- D. every verified lane writes its values' validity bits into the image (a failing page
    // writes nothing). One uniform step per iteration: a lane whose run is spent takes the next
    // header, then every lane appends up to 32 values of its run (a null run all at once: the
    // cursor moves), so the wave runs one short path instead of a per-run-kind branch chain.
    if (!err && !PQ_ABLATE(b, 21)) {  // (diagnostic: bit 21 skips D)
      uint32_t P = entry, v = base;
      const bool mine = cnt > 0 && base < need;
      const uint32_t vend = min(base + cnt, need);
      SgBits out;
      out.bm = L.bm;
      out.vb = vbw;
      out.ones = 0;
      out.nostore = PQ_ABLATE(b, 20);
      out.start(o0 + base);
      uint32_t rem = 0, rpay = 0, kind = 0;  // the current run: values left, next payload byte (stage),
                                             // 0 nulls / 1 ones / 2 bit-packed
      // (software-pipelined: the bytes of the header after the current run are read in the step
      // before the one that decodes them, together with the step's payload piece: one LDS
      // latency per step instead of a header read, its decode, then the dependent payload read)
      uint32_t hx = sg_bytes4(L.stage, P + sa);
      for (;;) {
        const bool act = mine && (rem || (P < exit && v < vend));
        if (!__ballot(act)) break;
        stp.count(7);
        if (act && !rem) {
          SgHop h = sg_fast(hx, P, n);
          if (!h.adv) {  // a longer varint, or a run decode_hdr took in B
            h = sg_decode(sg_bytes8(L.stage, P + sa), P, n);
            if (!h.adv) {
              const Hdr eh = decode_hdr(s4, 0u - sa4, s, P, n, 1, 1);
              h.adv = eh.adv;
              h.nv = eh.nvals;
              h.bp = eh.bp;
              h.val = eh.value;
            }
          }
          rem = min(h.nv, vend - v);
          kind = h.bp ? 2u : (h.val ? 1u : 0u);
          rpay = h.val + sa;
          P += h.adv;
          if (rem > kSgLong && kind) {  // long: the whole wave (the accumulator restarts after it)
            const uint32_t q = atomicAdd(&L.nq, 1u);
            if (q < kSgQueue) {
              out.end();
              L.qg[q] = o0 + v;
              L.qc[q] = rem;
              L.qv[q] = kind == 2 ? 0x80000000u | h.val : 1u;
              v += rem;
              out.start(o0 + v);
              rem = 0;
            }
          }
        }
        const uint32_t px = sg_bytes4(L.stage, rpay);
        hx = sg_bytes4(L.stage, P + sa);
        if (act && rem) {
          const uint32_t k = kind ? min(rem, 32u) : rem;
          const uint32_t m = k >= 32 ? ~0u : ((1u << k) - 1u);
          const uint32_t x = kind == 2 ? px & m : (kind ? m : 0u);
          out.step(x, k);
          rpay += 4;
          rem -= k;
          v += k;
        }
      }
      // a bit-packed run cut by EOF ends the last lane's range: its readable values (zero filled)
      if (mine && st == SG_TRUNC && v < need) {
        const Hdr eh = decode_hdr(s4, 0u - sa4, s, P, n, 1, 1);
        uint32_t c = min(min(eh.okvals, eh.nvals), need - v), pay = eh.value;
        for (uint32_t q = 0; q < c; q += 32, pay += 4) {
          const uint32_t k = min(32u, c - q);
          out.step(sg_bytes4(L.stage, pay + sa) & (k == 32 ? ~0u : ((1u << k) - 1u)), k);
        }
      }
      if (mine) out.end();
      ones = out.ones;
      wave_lds_sync();
      const uint32_t nq = min(L.nq, kSgQueue);
      for (uint32_t q = 0; q < nq; q++) {
        const uint32_t qv = L.qv[q];
        ones += sg1_run_wave(L, vbw, sa, L.qg[q], L.qc[q], (qv >> 31) != 0, qv & 0x7fffffffu);
      }
      stp.lap(3);
      // ---- the image to the chunk bitmap: coalesced word stores, atomic OR for the page's edge words
      wave_lds_sync();
      if (!PQ_ABLATE(b, 20)) {
        const uint32_t nw = (o0 + ns + 31) >> 5, nl = min(nw, kSg1Words);
        const bool edge_hi = ((o0 + ns) & 31u) != 0;
        for (uint32_t w = lane; w < nl; w += 64) {
          const uint32_t x = L.bm[sg1_sw(w)];
          if ((w == 0 && o0) || (w == nw - 1 && edge_hi)) { if (x) atomicOr(&vbw[w], x); }
          else vbw[w] = x;
        }
      }
      stp.lap(4);
    } else {
      stp.lap(3);
    }
  }
  const uint32_t cntv = (uint32_t)wave_sum64(ones);
  if (lane == 0) {
    if (err) {  // the reference fails the page at the first level error
      report(b, pd.chunk, 1, pd.page_in_chunk, ST_DEF, err_pos, err);
      b.page_nn[pi] = 0;
    } else {
      b.page_nn[pi] = cntv;
    }
  }
  stp.flush(16);
}

// One wavefront walks pages k, k + gridDim.x, ... of the list: a grid smaller than the page count
// keeps fewer level waves resident beside the values launch (DELTA-major schedule), each for longer.
// The LDS is dynamic (sizeof(LevelSegLDS) at launch): with a static size the compiler sizes the
// register allocation to the occupancy the LDS allows (176 VGPRs for 64 used), and each of those
// registers is one the DELTA launch beside it cannot have.
__global__ void __launch_bounds__(64) k_levels_seg(BatchDev b_in, const uint32_t *pages, uint32_t npages) {
  const BatchDev b = global_view(b_in);
  extern __shared__ uint4 sg_dyn_lds[];
  LevelSegLDS &L = *reinterpret_cast<LevelSegLDS *>(sg_dyn_lds);
  for (uint32_t k = blockIdx.x; k < npages; k += gridDim.x) {
    wave_lds_sync();  // (the previous page's stage and image reads are done)
    levels_seg_page(b, L, pages[k]);
  }
}

// ---------------------------------------------------------------------------
// k_levels_segw: generic level streams (repetition levels; definition levels with max_def > 1) by
// the same verified segment speculation as k_levels_seg, one 512-thread workgroup per (page,
// stream) whose stream fits the LDS stage (kSgwStage; the rest take k_levels): 512 lanes walk
// 512 segments, verification runs in lane order across the waves (lane 0 of wave w checks against
// lane 63 of wave w - 1 through LDS), a failing lane is re-walked by wave 0 with decode_hdr's full
// semantics while the others wait, a workgroup scan gives every lane its first value and first run
// index, and each lane writes its runs to the stream's run table (first value; bit-packed flag |
// payload position, or the RLE value) together with the run of every k_level_fill tile whose first
// value it holds — the same table and markers k_levels writes, expanded chip-wide by k_level_fill.
// ---------------------------------------------------------------------------
constexpr uint32_t kSgwWaves = 8, kSgwLanes = 64 * kSgwWaves;
constexpr uint32_t kSgwStage = kSgwStageHost;  // stream bytes staged in LDS
struct LevelSegWLDS {
  uint32_t stage[(kSgwStage + kSgSlack) / 4];
  uint32_t E[kSgwLanes], X[kSgwLanes], C[kSgwLanes], NR[kSgwLanes], ST[kSgwLanes], EC[kSgwLanes];
  uint32_t wtot[kSgwWaves], wtot2[kSgwWaves], wst[kSgwWaves], wpos[kSgwWaves], wcode[kSgwWaves];
  uint32_t dead, err_pos, err;
};

// The fast form of the header whose 8 bytes are x at stream position p, bit width bw (rs = value
// bytes of an RLE run): a varint of at most 4 bytes announcing a well formed run complete inside the
// stream. adv == 0: not a fast header.
DEV SgHop sgg_decode(uint64_t x, uint32_t p, uint32_t n, uint32_t bw, uint32_t rs) {
  const uint32_t u0 = (uint32_t)x;
  const uint32_t t = ~u0 & 0x80808080u;
  const uint32_t L = (uint32_t)(__builtin_ctz(t | 0x80000000u) >> 3) + 1;
  const uint32_t y = (L >= 4 ? u0 : (u0 & ((1u << (8 * L)) - 1u))) & 0x7f7f7f7fu;
  const uint32_t h = (y & 0x7fu) | ((y >> 1) & 0x3f80u) | ((y >> 2) & 0x1fc000u) | ((y >> 3) & 0xfe00000u);
  const uint32_t cnt = h >> 1, bp = h & 1u;
  const uint64_t adv = bp ? L + (uint64_t)cnt * bw : (uint64_t)(L + rs);
  const uint32_t rv = (uint32_t)(x >> (8 * L));
  const uint32_t v = rs >= 4 ? rv : (rv & ((1u << (8 * rs)) - 1u));
  const bool ok = t != 0 && cnt != 0 && (uint64_t)p + adv <= n && (bp || bw >= 32 || (v >> bw) == 0);
  SgHop r;
  r.adv = ok ? (uint32_t)adv : 0u;
  r.nv = bp ? cnt * 8 : cnt;
  r.bp = bp;
  r.val = bp ? p + L : v;
  r.L = L;
  return r;
}

__global__ void __launch_bounds__(kSgwLanes) k_levels_segw(BatchDev b_in, const uint32_t *units) {
  const BatchDev b = global_view(b_in);
  __shared__ LevelSegWLDS L;
  const uint32_t u = units[blockIdx.x], pi = u >> 1, which = u & 1;
  const bool rep = which == 0;
  const PageDesc pd = b.pages[pi];
  const ChunkDesc &cd = b.chunks[pd.chunk];
  const uint32_t tid = threadIdx.x, lane = lane_id(), wv = tid >> 6, ns = pd.num_slots;
  const uint8_t *s = gp_u64<const uint8_t>(pd.data) + (rep ? pd.rep_off : pd.def_off);
  const uint32_t n = rep ? pd.rep_len : pd.def_len;  // n + 24 <= kSgwStage (host)
  const uint32_t bw = (uint32_t)(rep ? cd.rep_bw : cd.def_bw), rs = (bw + 7) >> 3;
  const uint32_t sa = (uint32_t)((uintptr_t)s & 15u);
  const uint32_t sa4 = (uint32_t)((uintptr_t)s & 3u);
  const uint32_t *s4 = (const uint32_t *)(s - sa4);  // decode_hdr's view: global memory
  uint2 *runs = b.lv_runs + b.lv_run_base[2 * pi + which];
  uint32_t *trun = b.lv_tile_run + 2 * (uint64_t)b.lv_tile0[pi] + which;
  const uint32_t tile_a = (uint32_t)(pd.slot_base & (kLfTile - 1)), ntiles = lf_tiles(pd.slot_base, ns);
  // ---- stage
  {
    const uint4 *g = (const uint4 *)(s - sa);
    const uint32_t lim = n + sa, nv = (lim + 15) / 16;
    for (uint32_t k = tid; k < (kSgwStage + kSgSlack) / 16; k += kSgwLanes) {
      uint4 x = make_uint4(0u, 0u, 0u, 0u);
      if (k < nv) {
        x = g[k];
        const int32_t rel = (int32_t)(lim - 16 * k);
        if (rel < 16) {
          uint32_t q[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
          for (int i = 0; i < 4; i++) {
            const int32_t r = rel - 4 * i;
            q[i] = r >= 4 ? q[i] : (r <= 0 ? 0u : (q[i] & ((1u << (8 * r)) - 1u)));
          }
          x = make_uint4(q[0], q[1], q[2], q[3]);
        }
      }
      *(uint4 *)&L.stage[4 * k] = x;
    }
    if (tid == 0) { L.dead = kSgwLanes; L.err = 0; L.err_pos = 0; }
  }
  if (!rep && tid == 0) b.page_nn[pi] = 0;  // k_level_fill adds the page's non-null count
  wg_barrier();
  const uint32_t need = ns;
  uint32_t nruns = 0, covered = 0;
  if (!(pd.flags & (rep ? PF_REP : PF_DEF))) {
    if (ns && tid == 0) { L.err = PQ_ERR_INVALID; L.err_pos = 0; }  // "reader is not initialized"
  } else if (ns) {
    // ---- A. speculative walks (as k_levels_seg), counting values and runs
    const uint32_t S = max((n + kSgwLanes - 1) / kSgwLanes, 16u);
    const uint32_t lo = tid * S, hi = lo + S;
    const uint32_t lim = lo < n ? min(hi, n) : 0u;
    const uint32_t twomax = rs >= 4 ? 0u : 4u - rs;  // a second hop fits the 8 bytes after a first of this length
    uint32_t p = (tid == 0 || lo <= kSgMargin || lo >= n) ? 0u : lo - kSgMargin;
    uint32_t entry = lo < n ? (p >= lo ? p : ~0u) : n, cnt = 0, nr = 0, st = SG_OK;
    for (;;) {
      const bool act = st == SG_OK && p < lim;
      if (!__ballot(act)) break;  // (each wave ends its walks alone; the barrier follows the loop)
      const uint64_t x = sg_bytes8(L.stage, p + sa);
      const SgHop h = sgg_decode(x, p, n, bw, rs);
      const bool spec = p < lo;
      const bool take = h.adv != 0 && (!spec || h.adv <= kSgCap);
      const uint32_t np = take ? p + h.adv : p + 1u;
      const SgHop h2 = sgg_decode(x >> (8 * min(h.adv, 3u)), np, n, bw, rs);
      const bool spec2 = np < lo;
      const bool take2 = take && h.adv <= twomax && np < lim && h2.adv != 0 && (!spec2 || h2.adv <= kSgCap);
      const uint32_t np2 = take2 ? np + h2.adv : np;
      if (act && !spec) {
        cnt += take ? h.nv : 0u;
        nr += take ? 1u : 0u;
        st = take ? SG_OK : SG_STOP;
      }
      if (act && take2 && !spec2) { cnt += h2.nv; nr++; }
      if (act && spec && np >= lo) entry = np;
      if (act && take2 && spec2 && np2 >= lo) entry = np2;
      if (act && (take || spec)) p = np2;
    }
    if (lo < n && entry == ~0u) entry = p;
    L.E[tid] = entry;
    L.X[tid] = lo < n ? p : n;
    L.C[tid] = cnt;
    L.NR[tid] = nr;
    L.ST[tid] = st;
    L.EC[tid] = 0;
    wg_barrier();
    // ---- B. verification in lane order (wave 0 over the workgroup's lanes, 64 at a time); the first
    // failing lane is re-walked exactly from its predecessor's exit
    if (wv == 0) {
      uint32_t before = 0, prevX = 0, dead = kSgwLanes;
      for (uint32_t w = 0; w < kSgwWaves && dead == kSgwLanes; w++) {
        const uint32_t t = w * 64 + lane;
        uint64_t bad;
        auto bad_mask = [&]() {
          const uint32_t x = L.X[t], pv = __shfl_up(x, 1, 64);
          const uint32_t prev = lane == 0 ? prevX : pv;
          const bool ok = L.ST[t] == SG_OK && (t == 0 ? L.E[t] == 0 : L.E[t] == prev);
          return __ballot(!ok);
        };
        bad = bad_mask();
        while (bad) {
          const uint32_t f = (uint32_t)__builtin_ctzll(bad), ft = w * 64 + f;
          const uint32_t bef = before + (uint32_t)wave_sum64(lane < f ? L.C[t] : 0u);
          if (bef >= need) { dead = ft; break; }
          uint32_t P = f ? L.X[ft - 1] : prevX;
          const uint32_t fhi = ft * S + S;
          uint32_t c = 0, k = 0, fst = SG_OK, fcode = 0;
          const uint32_t fentry = P;
          while (P < fhi && P < n && bef + c < need) {
            const SgHop h = sgg_decode(sg_bytes8(L.stage, P + sa), P, n, bw, rs);
            if (h.adv) { c += h.nv; k++; P += h.adv; continue; }
            const Hdr eh = decode_hdr(s4, 0u - sa4, s, P, n, bw, rs);
            if (eh.err) {
              fst = SG_ERR;
              fcode = eh.err == kErrLongVarint ? resolve_long_varint(s, P, n) : eh.err;
              break;
            }
            const uint32_t okv = min(eh.nvals, eh.okvals);
            if (okv < eh.nvals) {  // a bit-packed run cut by EOF: next() fails after its groups
              c += okv;
              k++;
              fst = SG_TRUNC;
              fcode = PQ_ERR_EOF;
              break;
            }
            c += eh.nvals;
            k++;
            P += eh.adv;
          }
          if (lane == 0) {
            L.E[ft] = fentry;
            L.X[ft] = P;
            L.C[ft] = c;
            L.NR[ft] = k;
            L.ST[ft] = fst;
            L.EC[ft] = fcode;
          }
          wave_lds_sync();
          if (fst != SG_OK || P >= n || bef + c >= need) { dead = ft + 1; break; }
          bad = bad_mask() & ~((2ull << f) - 1ull);  // lanes <= f are verified now
        }
        if (dead != kSgwLanes) break;
        before += (uint32_t)wave_sum64(L.C[t]);
        prevX = rdlane(L.X[t], 63);
        if (before >= need) dead = w * 64 + 64;  // nothing after this wave is read
      }
      if (lane == 0) L.dead = dead;
    }
    wg_barrier();
    const uint32_t dead = L.dead;
    cnt = tid < dead ? L.C[tid] : 0u;
    nr = tid < dead ? L.NR[tid] : 0u;
    st = tid < dead ? L.ST[tid] : SG_OK;
    entry = L.E[tid];
    const uint32_t exit = L.X[tid], ecode = L.EC[tid];
    wg_barrier();  // (the arrays are reused by the scans below)
    // ---- C. value bases and run indices: workgroup scans
    const uint32_t wi1 = wave_incl_scan32(cnt), wi2 = wave_incl_scan32(nr);
    if (lane == 63) { L.wtot[wv] = wi1; L.wtot2[wv] = wi2; }
    wg_barrier();
    uint32_t base = wi1 - cnt, rbase = wi2 - nr, total = 0;
    for (uint32_t q = 0; q < kSgwWaves; q++) {
      const uint32_t t1 = L.wtot[q], t2 = L.wtot2[q];
      base += q < wv ? t1 : 0u;
      rbase += q < wv ? t2 : 0u;
      total += t1;
    }
    // the reference's first failure before num_values: the first erroring lane (lane order)
    {
      const bool e = (st == SG_ERR || st == SG_TRUNC) && base + cnt < need;
      const uint64_t em = __ballot(e);
      if (lane == 0) L.wst[wv] = em ? 1u : 0u;
      if (em && lane == (uint32_t)__builtin_ctzll(em)) { L.wpos[wv] = base + cnt; L.wcode[wv] = ecode; }
    }
    wg_barrier();
    if (tid == 0) {
      uint32_t err = 0, epos = 0;
      for (uint32_t q = 0; q < kSgwWaves; q++)
        if (L.wst[q]) { err = L.wcode[q]; epos = L.wpos[q]; break; }
      if (!err && total < need) { err = PQ_ERR_EOF; epos = total; }  // a header read at EOF
      L.err = err;
      L.err_pos = epos;
    }
    wg_barrier();
    // ---- D. runs of every verified lane into the run table, with the fill tiles' first runs
    uint32_t wrote = 0;
    if (!L.err) {
      const bool mine = cnt > 0 && base < need;
      uint32_t P = entry, v = base, ri = rbase;
      auto put = [&](uint32_t f, uint32_t c, uint32_t info) {
        runs[ri] = make_uint2(f, info);
        if (c && ntiles) {  // fill tiles whose first value lies in [f, f + c): tile k > 0 starts at k * T - a
          uint64_t k = f == 0 ? 0 : ((uint64_t)f + tile_a + kLfTile - 1) / kLfTile;
          const uint64_t khi = min(((uint64_t)f + c - 1 + tile_a) / kLfTile, (uint64_t)ntiles - 1);
          for (; k <= khi; k++) trun[2 * k] = ri;
        }
        ri++;
        wrote++;
      };
      while (mine && P < exit && v < need) {
        SgHop h = sgg_decode(sg_bytes8(L.stage, P + sa), P, n, bw, rs);
        if (!h.adv) {
          const Hdr eh = decode_hdr(s4, 0u - sa4, s, P, n, bw, rs);
          h.adv = eh.adv;
          h.nv = eh.nvals;
          h.bp = eh.bp;
          h.val = eh.value;
        }
        put(v, min(h.nv, need - v), h.bp ? 0x80000000u | h.val : h.val);
        v += h.nv;
        P += h.adv;
      }
      if (mine && st == SG_TRUNC && v < need) {  // a bit-packed run cut by EOF: its readable values
        const Hdr eh = decode_hdr(s4, 0u - sa4, s, P, n, bw, rs);
        put(v, min(min(eh.okvals, eh.nvals), need - v), 0x80000000u | eh.value);
        v += eh.okvals;
      }
    }
    // the run count (runs before num_values) and the values they cover
    const uint32_t ww = (uint32_t)wave_sum64(wrote);
    if (lane == 0) L.wtot[wv] = ww;
    wg_barrier();
    for (uint32_t q = 0; q < kSgwWaves; q++) nruns += L.wtot[q];
    covered = min(total, need);
  }
  if (tid == 0) {
    const uint32_t err = L.err;
    b.lv_meta[4 * pi + 2 * which] = nruns;
    b.lv_meta[4 * pi + 2 * which + 1] = err ? 0u : covered;  // a failed page is not expanded
    if (err) report(b, pd.chunk, 1, pd.page_in_chunk, rep ? ST_REP : ST_DEF, L.err_pos, err);
  }
}

// The same walk for the generic level streams (repetition levels, definition levels of max > 1):
// one wavefront per (page, stream) writes the stream's run table (first value index; bit-packed
// flag | payload position, or the RLE value) and the run of every k_level_fill tile's first value,
// which k_level_fill expands chip-wide; the payload is not read here, so a fast run may reach up
// to 4 KiB past its header.
constexpr uint32_t kLwMaxAdvG = 4095;
DEV void lw_put_tiles(LevelSink &sk, uint32_t idx, uint32_t f, uint32_t cnt) {
  if (!cnt || !sk.ntiles) return;
  const uint64_t a = sk.tile_a;  // fill tiles whose first value lies in [f, f + cnt): tile k > 0 starts at k * T - a
  uint64_t k = f == 0 ? 0 : ((uint64_t)f + a + kLfTile - 1) / kLfTile;
  const uint64_t khi = min(((uint64_t)f + cnt - 1 + a) / kLfTile, (uint64_t)sk.ntiles - 1);
  for (; k <= khi; k++) sk.trun[2 * k] = idx;
}

DEV void lw_walk_gen(LevelSink &sk, uint32_t need, uint32_t *ring) {
  const uint32_t lane = lane_id();
  const uint8_t *s = sk.s;
  const uint32_t n = sk.n, bw = sk.bw, rs = (bw + 7) >> 3;
  const uint32_t sa = (uint32_t)((uintptr_t)s & 3u);
  const uint32_t *sal = (const uint32_t *)(s - sa);
  const uint32_t nal = n + sa, gsb = 0u - sa;
  uint32_t pos = 0, done = 0, nruns = 0, RA = 0;
  lw_store(ring, 0, lw_load(sal, 0, nal));
  lw_store(ring, kLwHalf, lw_load(sal, kLwHalf, nal));
  LwHalf nxt = lw_load(sal, kLwRing, nal);
  wave_lds_sync();
  while (done < need) {
    const uint32_t ap = pos + sa;
    if (ap >= RA + kLwHalf) {
      if (ap < RA + kLwRing) {
        lw_store(ring, RA + kLwRing, nxt);
        RA += kLwHalf;
      } else {
        RA = ap & ~(kLwHalf - 1);
        lw_store(ring, RA, lw_load(sal, RA, nal));
        lw_store(ring, RA + kLwHalf, lw_load(sal, RA + kLwHalf, nal));
      }
      nxt = lw_load(sal, RA + kLwRing, nal);
      wave_lds_sync();
    }
    const uint32_t c = pos + lane, ac = c + sa;
    const uint32_t u0 = lw_bytes4(ring, ac), u1 = lw_bytes4(ring, ac + 4);
    const uint32_t t = ~u0 & 0x80808080u;
    const uint32_t L = (uint32_t)(__builtin_ctz(t | 0x80000000u) >> 3) + 1;
    const uint32_t y = (L >= 4 ? u0 : (u0 & ((1u << (8 * L)) - 1u))) & 0x7f7f7f7fu;
    const uint32_t h = (y & 0x7fu) | ((y >> 1) & 0x3f80u) | ((y >> 2) & 0x1fc000u) | ((y >> 3) & 0xfe00000u);
    const uint32_t cnt = h >> 1, isbp = h & 1u;
    const uint64_t adv = isbp ? L + (uint64_t)cnt * bw : (uint64_t)(L + rs);
    const uint32_t rv = (uint32_t)((((uint64_t)u1 << 32) | u0) >> (8 * L));
    const uint32_t v = rs >= 4 ? rv : (rv & ((1u << (8 * rs)) - 1u));
    const uint32_t nv = isbp ? cnt * 8 : cnt;
    const bool ok = t != 0 && cnt != 0 && adv <= kLwMaxAdvG && (uint64_t)c + adv <= n &&
                    (isbp || bw >= 32 || (v >> bw) == 0) && nv < (1u << 20);
    const uint32_t pk = ok ? (uint32_t)adv | (nv << 12) : 0u;
    const uint32_t rem = need - done;
    uint64_t mask = 0;
    uint32_t cur = 0, cum = 0;
    bool stop = false, last = false;
    while (cur < 64) {
      const uint32_t pc = (uint32_t)__builtin_amdgcn_readlane((int)pk, (int)cur);
      if (!pc) { stop = true; break; }
      mask |= 1ull << cur;
      const uint32_t nvc = pc >> 12;
      if (nvc >= rem - cum) { cum = rem; last = true; break; }
      cum += nvc;
      cur += pc & 0xfffu;
    }
    const bool mine = (mask >> lane) & 1ull;
    const uint32_t first = wave_excl_scan(mine ? nv : 0u);
    const uint32_t ri = nruns + wave_excl_scan(mine ? 1u : 0u);
    if (mine) {
      const uint32_t f = done + first;
      sk.runs[ri] = make_uint2(f, isbp ? 0x80000000u | (c + L) : v);
      lw_put_tiles(sk, ri, f, min(nv, rem - first));
    }
    nruns += (uint32_t)__popcll(mask);
    done += cum;
    if (last) break;
    if (!stop) { pos += cur; continue; }
    const uint32_t P = pos + cur;
    const Hdr eh = decode_hdr(sal, gsb, s, P, n, bw, rs);
    if (eh.err) {
      sk.error(done, eh.err == kErrLongVarint ? resolve_long_varint(s, P, n) : eh.err);
      break;
    }
    const uint32_t okv = min(eh.nvals, eh.okvals), r2 = need - done, tk = min(okv, r2);
    if (tk) {
      if (lane == 0) sk.runs[nruns] = make_uint2(done, eh.bp ? 0x80000000u | eh.value : eh.value);
      // the tiles of a long run: lanes split the tile range
      if (sk.ntiles) {
        const uint64_t a = sk.tile_a;
        const uint64_t k0 = done == 0 ? 0 : ((uint64_t)done + a + kLfTile - 1) / kLfTile;
        const uint64_t khi = min(((uint64_t)done + tk - 1 + a) / kLfTile, (uint64_t)sk.ntiles - 1);
        for (uint64_t k = k0 + lane; k <= khi; k += 64) sk.trun[2 * k] = nruns;
      }
      nruns++;
    }
    if (okv < eh.nvals && okv < r2) {
      sk.error(done + okv, PQ_ERR_EOF);
      break;
    }
    done += tk;
    pos = P + eh.adv;
  }
  sk.nruns = nruns;
  sk.covered = min(done, need);
}

__global__ void __launch_bounds__(64) k_levels_w(BatchDev b_in, const uint32_t *units) {
  const BatchDev b = global_view(b_in);
  __shared__ uint32_t ring[kLwRing / 4];
  const uint32_t u = units[blockIdx.x], pi = u >> 1, which = u & 1, lane = lane_id();
  const bool rep = which == 0;
  const PageDesc pd = b.pages[pi];
  const ChunkDesc &cd = b.chunks[pd.chunk];
  const uint32_t ns = pd.num_slots;
  LevelSink sk;
  sk.s = gp_u64<const uint8_t>(pd.data) + (rep ? pd.rep_off : pd.def_off);
  sk.n = rep ? pd.rep_len : pd.def_len;
  sk.bw = (uint32_t)(rep ? cd.rep_bw : cd.def_bw);
  sk.out = nullptr;
  sk.bits_lds = nullptr;
  sk.bits_glob = nullptr;
  sk.slot_base = pd.slot_base;
  sk.cmp = rep ? 0u : (uint32_t)cd.max_def;
  sk.count = 0;
  sk.err_code = 0;
  sk.err_pos = 0;
  sk.stage_len = 0;
  sk.ablate = b.ablate;
  sk.runs = b.lv_runs + b.lv_run_base[2 * pi + which];
  sk.trun = b.lv_tile_run + 2 * (uint64_t)b.lv_tile0[pi] + which;
  sk.tile_a = (uint32_t)(pd.slot_base & (kLfTile - 1));
  sk.ntiles = lf_tiles(pd.slot_base, ns);
  sk.covered = 0;
  sk.nruns = 0;
  if (!rep && lane == 0) b.page_nn[pi] = 0;  // k_level_fill adds the page's non-null count
  if (!(pd.flags & (rep ? PF_REP : PF_DEF))) {
    if (ns) sk.error(0, PQ_ERR_INVALID);  // "reader is not initialized"
  } else if (ns) {
    lw_walk_gen(sk, ns, ring);
  }
  if (lane == 0) {
    b.lv_meta[4 * pi + 2 * which] = sk.nruns;
    b.lv_meta[4 * pi + 2 * which + 1] = sk.err_code ? 0u : sk.covered;  // a failed page is not expanded
    if (sk.err_code) report(b, pd.chunk, 1, pd.page_in_chunk, rep ? ST_REP : ST_DEF, sk.err_pos, sk.err_code);
  }
}

// Flat OPTIONAL columns (bit width 1, validity only): held to 80 VGPRs so six workgroups fit
// per CU (24 KB LDS each): the kernel is latency-bound per page, so resident pages set its time.
__global__ void __launch_bounds__(kLvThreads) __attribute__((amdgpu_waves_per_eu(PQ_LV_WPE))) k_levels_bw1(BatchDev b_in,
                                                                                               const uint32_t *pages) {
  const BatchDev b = global_view(b_in);
  __shared__ LevelLDS lds;
  levels_page<true>(b, pages, lds);
}
// Generic level streams (repetition levels, definition levels of max_def > 1): one workgroup
// per (page, stream) — unit = page << 1 | (0: repetition, 1: definition). The walk writes the
// stream's run table (and the run of every fill tile's first value); k_level_fill expands the
// tables into levels, validity and counts with the whole chip, so a long page is not expanded
// by one workgroup.
__global__ void __launch_bounds__(kLvThreads) __attribute__((amdgpu_waves_per_eu(PQ_LV_WPE))) k_levels(BatchDev b_in,
                                                                                          const uint32_t *units) {
  const BatchDev b = global_view(b_in);
  __shared__ LevelLDS lds;
  const uint32_t u = units[blockIdx.x], pi = u >> 1, which = u & 1;
  const bool rep = which == 0;
  const PageDesc pd = b.pages[pi];
  const ChunkDesc &cd = b.chunks[pd.chunk];
  const uint32_t tid = threadIdx.x, ns = pd.num_slots;
  PQ_STAMPS(st, b.dbg);
  st.begin();
  LevelSink sk;
  sk.s = gp_u64<const uint8_t>(pd.data) + (rep ? pd.rep_off : pd.def_off);
  sk.n = rep ? pd.rep_len : pd.def_len;
  sk.bw = (uint32_t)(rep ? cd.rep_bw : cd.def_bw);
  sk.out = nullptr;
  sk.bits_lds = nullptr;
  sk.bits_glob = nullptr;
  sk.slot_base = pd.slot_base;
  sk.cmp = rep ? 0u : (uint32_t)cd.max_def;
  sk.count = 0;
  sk.err_code = 0;
  sk.err_pos = 0;
  sk.stage_len = kLvStageB;
  sk.ablate = b.ablate;
  sk.runs = b.lv_runs + b.lv_run_base[2 * pi + which];
  sk.trun = b.lv_tile_run + 2 * (uint64_t)b.lv_tile0[pi] + which;
  sk.tile_a = (uint32_t)(pd.slot_base & (kLfTile - 1));
  sk.ntiles = lf_tiles(pd.slot_base, ns);
  sk.covered = 0;
  sk.nruns = 0;
  if (!rep && tid == 0) b.page_nn[pi] = 0;  // k_level_fill adds the page's non-null count
  if (!(pd.flags & (rep ? PF_REP : PF_DEF))) {
    if (ns) sk.error(0, PQ_ERR_INVALID);  // "reader is not initialized"
  } else {
    lv_walk<false>(lds, sk, ns, st);
  }
  if (tid == 0) {
    b.lv_meta[4 * pi + 2 * which] = sk.nruns;
    b.lv_meta[4 * pi + 2 * which + 1] = sk.err_code ? 0u : sk.covered;  // a failed page is not expanded
    if (sk.err_code) report(b, pd.chunk, 1, pd.page_in_chunk, rep ? ST_REP : ST_DEF, sk.err_pos, sk.err_code);
  }
  st.lap(6);
  st.flush(0);
}

// k_levels_hyb: generic level streams made of long literal runs (repetition streams: Arrow writes
// maximal literal runs, 64 B at bit width 1, with an RLE run now and then) walked by hyb_scan, the
// dictionary index walker of k_scan_runs, from its 16 KiB LDS windows: runs of 64 stream bytes or
// more by stride speculation (up to 64 per step), the others by speculative header decode 64
// stream bytes at a time — every step an LDS round trip, where k_levels' list ranking pays ~10
// workgroup barriers per 2 KiB and a walk from global memory a memory round trip per step. Writes
// the same run table and fill-tile markers as k_levels (hybrid_decoder.go:81-165 through
// decodePackedArray helpers.go:133-149: runs past the one that reaches num_values are never read,
// an error is the page's at the value where next() meets it).
struct LvRunSink {
  uint2 *runs;
  uint32_t *trun;
  uint32_t tile_a, ntiles;
  uint32_t nruns;  // uniform
  uint32_t err_code, err_pos;
  DEV void window(bool active, uint32_t first, uint32_t cnt, bool bp, uint32_t value, uint32_t, const uint32_t *,
                  uint32_t) {
    const uint64_t m = __ballot(active);
    if (active) {
      const uint32_t idx = nruns + (uint32_t)__popcll(m & ((1ull << lane_id()) - 1ull));
      runs[idx] = make_uint2(first, bp ? 0x80000000u | value : value);
      if (ntiles) {  // fill tiles whose first value lies in [first, first + cnt): tile k > 0 starts at k * T - a
        const uint64_t a = tile_a;
        uint64_t k = first == 0 ? 0 : ((uint64_t)first + a + kLfTile - 1) / kLfTile;
        const uint64_t khi = min(((uint64_t)first + cnt - 1 + a) / kLfTile, (uint64_t)ntiles - 1);
        for (; k <= khi; k++) trun[2 * k] = idx;
      }
    }
    nruns += (uint32_t)__popcll(m);
  }
  DEV void error(uint32_t pos, uint32_t code) {
    if (!err_code) { err_code = code; err_pos = pos; }
  }
};
__global__ void __launch_bounds__(256) k_levels_hyb(BatchDev b_in, const uint32_t *units) {
  const BatchDev b = global_view(b_in);
  __shared__ ScanLDS lds;
  const uint32_t u = units[blockIdx.x], pi = u >> 1, which = u & 1;
  const bool rep = which == 0;
  const PageDesc pd = b.pages[pi];
  const ChunkDesc &cd = b.chunks[pd.chunk];
  const uint32_t ns = pd.num_slots;
  LvRunSink sk{b.lv_runs + b.lv_run_base[2 * pi + which], b.lv_tile_run + 2 * (uint64_t)b.lv_tile0[pi] + which,
               (uint32_t)(pd.slot_base & (kLfTile - 1)), lf_tiles(pd.slot_base, ns), 0u, 0u, 0u};
  if (!rep && threadIdx.x == 0) b.page_nn[pi] = 0;  // the fill kernels add the page's non-null count
  uint32_t done = 0;
  if (!(pd.flags & (rep ? PF_REP : PF_DEF))) {
    if (ns) sk.error(0, PQ_ERR_INVALID);  // "reader is not initialized"
  } else if (ns) {
    done = hyb_scan<LvRunSink, true, 48>(lds,  // (stride prelude first: profiles/r06_u_probe_hyb_pre.txt)
                                          gp_u64<const uint8_t>(pd.data) + (rep ? pd.rep_off : pd.def_off),
                                          rep ? pd.rep_len : pd.def_len, (uint32_t)(rep ? cd.rep_bw : cd.def_bw), ns, sk,
                                          b.dbg);
  }
  if (threadIdx.x == 0) {  // wave 0 walked: its sink holds the run count and the error
    b.lv_meta[4 * pi + 2 * which] = sk.nruns;
    b.lv_meta[4 * pi + 2 * which + 1] = sk.err_code ? 0u : min(done, ns);  // a failed page is not expanded
    if (sk.err_code) report(b, pd.chunk, 1, pd.page_in_chunk, rep ? ST_REP : ST_DEF, sk.err_pos, sk.err_code);
  }
}

// k_level_fill: the run tables of the generic level streams expanded, one workgroup per fill
// tile (kLfTile slots aligned on the chunk's slot index, so tiles own whole words of the level
// arrays and of the validity bitmap). A thread expands kLfGroups groups of eight consecutive
// values (group q of thread i: slots [q * 2048 + 8 i, + 8) of the tile), each one independent
// of the others so that their loads overlap: the tile's runs are staged in LDS (or, past
// kLfRuns of them, searched in global memory), the run of a group's first value is found by
// binary search and the group advances from there. Outputs: u8 levels, validity (definition
// level == max_def) and the page's counts (records: repetition level == 0; non-null values),
// added atomically once per tile. Nested chunks' tiles go to k_nest_count / k_nest_emit
// (nested.hip), which expand both streams together and keep the levels in registers.
constexpr uint32_t kLfGroups = kLfTile / (8 * kLvThreads);
static_assert(kLfGroups * 8 * kLvThreads == kLfTile, "tile = groups x 8 values x threads");
struct LevelFillLDS {
  uint2 run[kLfRuns];
  uint32_t vb[kLfTile / 32];
  uint32_t cnt[kLvThreads / 64];
};
// lv_tiles: page of every fill tile; list: the fill tiles of this launch
__global__ void __launch_bounds__(kLvThreads) k_level_fill(BatchDev b_in, const uint32_t *lv_tiles, const uint32_t *list) {
  const BatchDev b = global_view(b_in);
  __shared__ LevelFillLDS L;
  const uint32_t t = list[blockIdx.x], pi = lv_tiles[t], tid = threadIdx.x, lane = lane_id(), wv = tid >> 6;
  const PageDesc &pd = b.pages[pi];
  const ChunkDesc &cd = b.chunks[pd.chunk];
  const uint64_t sbase = pd.slot_base;
  const uint32_t ns = pd.num_slots, a = (uint32_t)(sbase & (kLfTile - 1)), ntiles = lf_tiles(sbase, ns);
  const uint32_t k = t - b.lv_tile0[pi];
  const int64_t t0 = (int64_t)k * kLfTile - a;  // page value index of the tile's first (aligned) slot
  const uint32_t lo = (uint32_t)max(t0, (int64_t)0), hi = (uint32_t)min(t0 + kLfTile, (int64_t)ns);
  const uint8_t *page = gp_u64<const uint8_t>(pd.data);
  for (uint32_t which = 0; which < 2; which++) {
    const bool rep = which == 0;
    if (rep ? cd.max_rep == 0 : cd.max_def == 0) continue;
    const uint32_t nr = b.lv_meta[4 * pi + 2 * which], cov = b.lv_meta[4 * pi + 2 * which + 1];
    const uint32_t end = min(hi, cov);
    if (lo >= end || nr == 0) continue;  // workgroup-uniform
    const uint2 *runs = b.lv_runs + b.lv_run_base[2 * pi + which];
    const uint32_t *trun = b.lv_tile_run + 2 * (uint64_t)b.lv_tile0[pi] + which;
    const uint32_t r0 = trun[2 * k];
    const bool more = k + 1 < ntiles && (int64_t)(k + 1) * kLfTile - a < (int64_t)cov;
    const uint32_t m = (more ? trun[2 * (k + 1)] : nr - 1) - r0 + 1;
    const bool staged = m <= kLfRuns;
    if (staged)
      for (uint32_t i = tid; i < m; i += kLvThreads) L.run[i] = runs[r0 + i];
    wg_barrier();
    const uint8_t *src = page + (rep ? pd.rep_off : pd.def_off);
    const uint32_t n = rep ? pd.rep_len : pd.def_len, bw = (uint32_t)(rep ? cd.rep_bw : cd.def_bw);
    const uint32_t cmp = rep ? 0u : (uint32_t)cd.max_def;
    uint8_t *out = rep ? gp_u64<uint8_t>(cd.rep_levels) : gp_u64<uint8_t>(cd.def_levels);
    uint32_t *vbits = rep ? nullptr : gp_u64<uint32_t>(cd.validity);
    uint32_t nc = 0;
#pragma unroll 1
    for (uint32_t q = 0; q < kLfGroups; q++) {
      const int64_t g = t0 + (int64_t)(q * 8 * kLvThreads + 8 * tid);  // the group's values [g, g + 8)
      const uint32_t vs = (uint32_t)max(g, (int64_t)lo), ve = (uint32_t)max(min(g + 8, (int64_t)end), (int64_t)vs);
      uint64_t word;
      uint32_t eq;
      if (PQ_ABLATE(b, 2)) {
        word = 0; eq = 0;
      } else if (staged) {
        lf_group([&](uint32_t i) { return L.run[i]; }, m, src, n, bw, cmp, g, vs, ve, word, eq);
      } else {
        lf_group([&](uint32_t i) { return runs[r0 + i]; }, m, src, n, bw, cmp, g, vs, ve, word, eq);
      }
      if (out && vs < ve) {
        uint8_t *o = out + sbase;
        if (vs == g && ve == g + 8 && !(reinterpret_cast<uintptr_t>(o + g) & 7)) {
          *reinterpret_cast<uint2 *>(o + g) = make_uint2((uint32_t)word, (uint32_t)(word >> 32));
        } else {
          for (uint32_t v = vs; v < ve; v++) o[v] = (uint8_t)(word >> (8 * (v - (uint32_t)g)));
        }
      }
      nc += __popc(eq);
      if (vbits) reinterpret_cast<uint8_t *>(L.vb)[q * kLvThreads + tid] = (uint8_t)eq;
    }
    // counts: one atomic per tile
    const uint32_t wc = (uint32_t)wave_sum64(nc);
    if (lane == 0) L.cnt[wv] = wc;
    wg_barrier();
    if (tid == 0) {
      uint32_t c = 0;
      for (uint32_t q = 0; q < kLvThreads / 64; q++) c += L.cnt[q];
      if (c) atomicAdd(rep ? &b.page_rec[pi] : &b.page_nn[pi], c);
    }
    if (vbits) {
      for (uint32_t w = tid; w < kLfTile / 32; w += kLvThreads) {
        const int64_t w0 = t0 + 32 * (int64_t)w;  // the word's first value
        if (w0 + 32 <= (int64_t)lo || w0 >= (int64_t)end) continue;
        const uint32_t v = L.vb[w];
        uint32_t *dst = vbits + ((sbase + (uint64_t)w0) >> 5);
        if (w0 >= (int64_t)lo && w0 + 32 <= (int64_t)end) *dst = v;  // the tile owns the whole word
        else if (v) atomicOr(dst, v);                                 // shared with a neighbouring page
      }
    }
    wg_barrier();  // L is reused by the next stream
  }
}

// ---------------------------------------------------------------------------
// Value bases: exclusive scan of per-page non-null counts (and record counts)
// within each chunk. One workgroup per chunk (pages per chunk are few).
//
// Serial mode: the value bases and the counts the values kernels use come from
// k_levels (page_nn). Speculative mode (every page carries a non-null count in
// its header, e.g. DataPageHeaderV2.num_nulls): the host uploaded those counts
// and their bases, the values kernels ran concurrently with k_levels, and this
// kernel only checks that the header counts equal the decoded ones — the
// reference derives notNull from the definition levels (page_v1.go:49-52), so
// any difference sends the batch back through the serial path (host.cpp).
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_bases(BatchDev b_in, const uint32_t *chunks) {
  const BatchDev b = global_view(b_in);
  const ChunkDesc &cd = b.chunks[chunks[blockIdx.x]];
  __shared__ uint64_t carry_v, carry_r;
  __shared__ uint64_t part_v[256], part_r[256];
  if (threadIdx.x == 0) { carry_v = 0; carry_r = 0; }
  wg_barrier();
  for (uint32_t p0 = 0; p0 < cd.num_pages; p0 += 256) {
    uint32_t p = p0 + threadIdx.x;
    uint32_t gp = cd.first_page + p;
    uint64_t nv = p < cd.num_pages ? b.page_nn[gp] : 0;
    uint64_t nr = p < cd.num_pages ? b.page_rec[gp] : 0;
    if (p < cd.num_pages) {
      // speculated counts (spec mode: page headers; CF_NN_SPEC: PLAIN value bytes) are checked; a
      // CF_NN_SPEC chunk's copies read the uploaded ones, which an equal count leaves in place
      if ((b.spec || (cd.flags & CF_NN_SPEC)) && b.page_nn_v[gp] != (uint32_t)nv) atomicOr(b.spec_mismatch, 1u);
      if (!b.spec && !(cd.flags & CF_NN_SPEC)) b.page_nn_v[gp] = (uint32_t)nv;
    }
    part_v[threadIdx.x] = nv;
    part_r[threadIdx.x] = nr;
    wg_barrier();
    for (uint32_t d = 1; d < 256; d <<= 1) {
      uint64_t av = threadIdx.x >= d ? part_v[threadIdx.x - d] : 0;
      uint64_t ar = threadIdx.x >= d ? part_r[threadIdx.x - d] : 0;
      wg_barrier();
      part_v[threadIdx.x] += av;
      part_r[threadIdx.x] += ar;
      wg_barrier();
    }
    if (p < cd.num_pages) {
      if (!b.spec && !(cd.flags & CF_NN_SPEC)) b.page_vbase[gp] = carry_v + part_v[threadIdx.x] - nv;
      b.page_rbase[gp] = carry_r + part_r[threadIdx.x] - nr;
    }
    wg_barrier();
    if (threadIdx.x == 255) { carry_v += part_v[255]; carry_r += part_r[255]; }
    wg_barrier();
  }
}

// ---------------------------------------------------------------------------
// Run-table sink for hybrid VALUE streams (dictionary indices, boolean RLE):
// records every run and, per 4096-value tile, the run covering its first value.
// ---------------------------------------------------------------------------
struct RunSink {
  HybRun *runs;
  uint32_t *tile_first;
  uint32_t nruns;  // uniform
  uint32_t stream_base;  // not used
  uint32_t err_code, err_pos;

  DEV void window(bool active, uint32_t first, uint32_t cnt, bool bp, uint32_t value, uint32_t c, const uint32_t *,
                  uint32_t) {
    uint64_t m = __ballot(active);
    uint32_t rank = __popcll(m & ((1ull << lane_id()) - 1ull));
    if (active) {
      uint32_t idx = nruns + rank;
      HybRun r;
      r.value_start = first;
      r.payload_off = bp ? value : c;
      r.info = bp ? 0x80000000u : value;
      runs[idx] = r;
      // tiles whose first value falls inside [first, first+cnt)
      uint32_t t0 = (first + kDictTile - 1) / kDictTile, t1 = (first + cnt - 1) / kDictTile;
      for (uint32_t t = t0; t <= t1; t++) tile_first[t] = idx;
    }
    nruns += __popcll(m);
  }
  // One run found by the scalar fast path (every lane calls it with uniform arguments).
  DEV void one(uint32_t first, uint32_t cnt, bool bp, uint32_t value, uint32_t c) {
    const uint32_t idx = nruns;
    if (lane_id() == 0) {
      HybRun r;
      r.value_start = first;
      r.payload_off = bp ? value : c;
      r.info = bp ? 0x80000000u : value;
      runs[idx] = r;
    }
    const uint32_t t0 = (first + kDictTile - 1) / kDictTile, t1 = (first + cnt - 1) / kDictTile;
    for (uint32_t t = t0 + lane_id(); t <= t1; t += 64) tile_first[t] = idx;
    nruns = idx + 1;
  }
  DEV void error(uint32_t pos, uint32_t code) {
    if (!err_code) { err_code = code; err_pos = pos; }
  }
};

DEV void scan_runs_page(const BatchDev &b, uint32_t pi, ScanLDS &lds);
__global__ void __launch_bounds__(256) k_scan_runs(BatchDev b_in, const uint32_t *pages) {
  const BatchDev b = global_view(b_in);
  __shared__ ScanLDS lds;
  scan_runs_page(b, pages[blockIdx.x], lds);
}
// The run scan and the byte-array dictionaries' slot tables (dict_slots.h) in one launch: blocks
// [0, n_scan) scan pages, the next n_slot_chunks x gx blocks fill slots (no launch of their own, and
// the slot blocks fill the CUs the page walks leave idle).
__global__ void __launch_bounds__(256) k_scan_slots(BatchDev b_in, const uint32_t *pages, uint32_t n_scan,
                                                    const uint32_t *slot_chunks, uint32_t gx) {
  const BatchDev b = global_view(b_in);
  __shared__ ScanLDS lds;
  if (blockIdx.x < n_scan) {
    scan_runs_page(b, pages[blockIdx.x], lds);
  } else {
    const uint32_t k = blockIdx.x - n_scan;
    dict_slots_block(b, slot_chunks[k / gx], k % gx, gx);
  }
}
DEV void scan_runs_page(const BatchDev &b, uint32_t pi, ScanLDS &lds) {
  const PageDesc pd = b.pages[pi];
  const uint32_t nn = b.page_nn_v[pi];
  RunSink rs{b.runs + b.run_base[pi], b.tile_first + b.tile_base[pi], 0u, 0u, 0u, 0u};
  uint32_t done = 0;
  if (threadIdx.x < 64 && nn && pd.dict_bw > 0) {
    // the page's tile table reads ~0 where no run starts a tile (the dictionary-only schedule has no
    // reset launch); wave 0, which then writes the runs' entries, orders them after these
    const uint32_t ntile = (nn + kDictTile - 1) / kDictTile;
    for (uint32_t t = threadIdx.x; t < ntile; t += 64) rs.tile_first[t] = ~0u;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  }
  if (nn && pd.dict_bw > 0) {  // workgroup-uniform
    done = hyb_scan(lds, gp_u64<const uint8_t>(pd.data) + pd.val_off, pd.val_len, pd.dict_bw, nn, rs, b.dbg);
  }
  if (threadIdx.x == 0) {  // wave 0 walked: its sink holds the run count and the error
    b.run_count[pi] = rs.nruns;
    HybRun sentinel;
    sentinel.value_start = done;  // values covered by valid runs
    sentinel.payload_off = 0;
    sentinel.info = 0;
    rs.runs[rs.nruns] = sentinel;
    if (rs.err_code) report(b, pd.chunk, 1, pd.page_in_chunk, ST_VALUES, rs.err_pos, rs.err_code);
  }
  // Tile descriptors (wave 0, which wrote the run table and the tiles' first runs): for tile t the
  // runs [r0, r1] its values cross, the stream bytes [lo, hi) its bit-packed values occupy and the
  // values the valid runs cover — dict_tile.h reads this instead of chasing the table itself.
  if (threadIdx.x < 64 && nn && pd.dict_bw > 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");  // the lanes' run / tile stores
    const uint32_t nr = rs.nruns, bw = pd.dict_bw, ntile = (nn + kDictTile - 1) / kDictTile;
    const uint32_t *tf = b.tile_first + pd.dict_tile0;
    const HybRun *rg = rs.runs;
    uint4 *desc = b.tile_desc + 2 * (uint64_t)pd.dict_tile0;
    for (uint32_t t = threadIdx.x; t < ntile; t += 64) {
      const uint32_t v0 = t * kDictTile, v1 = min(min(v0 + kDictTile, nn), done);
      uint32_t r0 = tf[t], r1 = t + 1 < ntile ? tf[t + 1] : nr - 1;
      if (r1 >= nr) r1 = nr - 1;
      const bool ok = nr > 0 && r0 < nr && v0 < v1;
      uint32_t lo = 0, hi = 0;
      if (ok) {
        const HybRun f = rg[r0], l = rg[r1];
        const uint64_t a = (f.info & 0x80000000u) ? (uint64_t)f.payload_off + (((uint64_t)(v0 - f.value_start) * bw) >> 3)
                                                 : (uint64_t)f.payload_off;
        uint64_t z = (l.info & 0x80000000u) && v1 > l.value_start
                         ? (uint64_t)l.payload_off + (((uint64_t)(v1 - l.value_start) * bw + 7) >> 3)
                         : (uint64_t)l.payload_off + 8;
        z = min(z, (uint64_t)pd.val_len);
        lo = (uint32_t)a;
        hi = (uint32_t)z;
      }
      desc[2 * t] = make_uint4(r0, r1, lo, hi);
      desc[2 * t + 1] = make_uint4(done, ok ? 1u : 0u, 0u, 0u);
    }
  }
}

// ---------------------------------------------------------------------------
// Values kernel: one workgroup (256 threads) per work item.
// ---------------------------------------------------------------------------
struct DeltaTileLDS {
  uint64_t scan[260];        // per-group exclusive scan + per-wave totals
  uint32_t stage[(kDeltaTileVals * 8 + 8 * 24 + 64) / 4];  // the tile's payload bytes
};

// Reference fixed-width PLAIN error: binary.Read/io.ReadFull of w bytes per value
// (type_int32.go:21-31 ...): the first value that does not fit fails with EOF when
// no byte of it is left, else ErrUnexpectedEOF.
DEV uint32_t plain_err(uint64_t have, uint32_t w) { return (have % w) == 0 ? PQ_ERR_EOF : PQ_ERR_UNEXPECTED_EOF; }


// PLAIN fixed width (INT32/INT64/FLOAT/DOUBLE/INT96/FLBA): byte copy.
#ifndef PQ_FUSED_COPY_U
#define PQ_FUSED_COPY_U 4
#endif
// U: pieces per lane in flight (copy_bytes_u); 0: copy_bytes
template <uint32_t U = 0>
DEV void do_plain(const BatchDev &b, const WorkItem &wi, const PageDesc &pd, const ChunkDesc &cd, uint32_t nn) {
  const uint32_t w = (uint32_t)cd.value_width;
  const uint64_t vb = b.page_vbase[wi.page];
  // the tiles' inner boundaries moved to 16-B aligned destination bytes (4- and 8-byte values): a
  // boundary line written half by each of two workgroups costs a partial-line write each
  const uint32_t a = w == 8 ? (uint32_t)(vb & 1u) : (w == 4 ? (uint32_t)((4u - (uint32_t)(vb & 3u)) & 3u) : 0u);
  const uint32_t v0 = wi.v0 ? wi.v0 + a : 0u;
  uint32_t v1 = min(wi.v1 + a, nn);
  if (v0 >= v1) return;
  const uint64_t have = pd.val_len;
  uint64_t fit = have / w;  // values that fit
  uint32_t e1 = (uint32_t)min((uint64_t)v1, fit);
  if (e1 < v1 && threadIdx.x == 0) report(b, pd.chunk, 1, pd.page_in_chunk, ST_VALUES, (uint32_t)fit, plain_err(have, w));
  if (e1 <= v0) return;
  const uint8_t *src = gp_u64<const uint8_t>(pd.data) + pd.val_off + (uint64_t)v0 * w;
  uint8_t *dst = gp_u64<uint8_t>(cd.values) + (vb + v0) * w;
  if constexpr (U == 0) copy_bytes(dst, src, (uint64_t)(e1 - v0) * w, threadIdx.x, blockDim.x);
  else copy_bytes_u<U>(dst, src, (uint64_t)(e1 - v0) * w, threadIdx.x, blockDim.x);
}

// BOOLEAN PLAIN (type_boolean.go:46-69): bit i of byte i/8, LSB first, one byte read per 8 values.
DEV void do_bool(const BatchDev &b, const WorkItem &wi, const PageDesc &pd, const ChunkDesc &cd, uint32_t nn) {
  uint32_t v1 = min(wi.v1, nn);
  uint64_t fit = (uint64_t)pd.val_len * 8;
  if (v1 > fit && threadIdx.x == 0 && wi.v0 <= fit)
    report(b, pd.chunk, 1, pd.page_in_chunk, ST_VALUES, (uint32_t)fit, PQ_ERR_EOF);
  uint32_t e1 = (uint32_t)min((uint64_t)v1, fit);
  const uint8_t *src = gp_u64<const uint8_t>(pd.data) + pd.val_off;
  uint8_t *dst = gp_u64<uint8_t>(cd.values) + b.page_vbase[wi.page];
  for (uint32_t v = wi.v0 + threadIdx.x; v < e1; v += blockDim.x) dst[v] = (src[v >> 3] >> (v & 7)) & 1;
}

// Dictionary indices of a fixed-width column (type_dict.go:40-60: dst[i] = dict[idx], an index
// outside the dictionary fails the page with "dict: invalid index") and boolean RLE
// (type_boolean.go:109-120: value = index == 1), one kDictTile-value tile per workgroup, or
// kDictGroup of them (grouped items, do_dict2). The tile's runs and stream bytes are staged in LDS (dict_tile.h); wave w takes values
// [w * 1024, (w + 1) * 1024) of the tile in 16 rounds of 64 consecutive values, so every
// store instruction writes 64 consecutive outputs (256 B for 4-byte values).
#ifndef PQ_DICT_LDS
#define PQ_DICT_LDS 1
#endif
constexpr uint32_t kDictEarly = 4096;  // dictionaries up to this many bytes are staged with the tile
constexpr uint32_t kDictEarlyWord = (kTileStageB - kDictEarly) / 4;  // the early dictionary's first stage word

#ifndef PQ_DICT_CURSOR
#define PQ_DICT_CURSOR 1  // the run in registers (dict_tile.h DictCursor); 0: a run-table read per value
#endif
// This wave's 1024 values of tile t as 16 rounds of indices (LDS reads): idx ~0u where there is no
// value, or where the index is outside the dictionary (first_err: the first such value).
DEV void dict_tile_indices(const DictTile &t, const DictTileLDST<kDictRuns> &lds, uint32_t seg0, uint32_t dcount,
                           uint32_t (&idx)[16], uint32_t &first_err) {
  const uint32_t lane = lane_id();
  DictCursor c = dict_cursor(t, max(seg0 + lane, t.v0));
  uint32_t ri = PQ_DICT_CURSOR ? 0 : dict_tile_seek(t, max(seg0 + lane, t.v0));
#pragma unroll
  for (uint32_t r = 0; r < 16; r++) {
    const uint32_t v = seg0 + r * 64 + lane;
    idx[r] = ~0u;
    if (v >= t.v0 && v < t.v1) {
      const uint32_t x = PQ_DICT_CURSOR ? dict_cursor_value(t, lds, c, v) : dict_tile_value(t, lds, ri, v);
      if (x < dcount) idx[r] = x;
      else first_err = min(first_err, v);
    }
  }
}
// 4-byte values: all 16 gathers in flight at once, then the stores (out: the wave's first value
// of round 0 for this lane)
DEV void dict_store4(const BatchDev &b, uint32_t *out, const uint32_t *dv, const uint32_t (&idx)[16]) {
  uint32_t val[16];
#pragma unroll
  for (uint32_t r = 0; r < 16; r++) val[r] = idx[r] != ~0u ? (PQ_ABLATE(b, 24) ? idx[r] : dv[idx[r]]) : 0u;
#pragma unroll
  for (uint32_t r = 0; r < 16; r++)
    if (idx[r] != ~0u) out[r * 64] = val[r];
}

DEV void do_dict(const BatchDev &b, const WorkItem &wi, const PageDesc &pd, const ChunkDesc &cd, uint32_t nn,
                 DictTileLDST<kDictRuns> &lds) {
  const uint32_t v1 = min(wi.v1, nn);
  if (wi.v0 >= v1) return;
  DictTile t;
  const bool is_bool = pd.vkind == VK_RLE_BOOL;
  const uint32_t w = (uint32_t)cd.value_width;
  const uint32_t dcount = cd.dict_count;
  // a small dictionary (at most kDictEarly bytes) goes to the stage's end while the tile is staged,
  // under the same barrier: no barrier pair after the index decode
  const uint32_t dbytes = dcount * w;
  const bool early = PQ_DICT_LDS && !is_bool && w == 4 && dbytes <= kDictEarly;  // workgroup-uniform
  if (early) {
    const uint32_t *src = gp_u64<const uint32_t>(cd.dict_values);
    for (uint32_t k = threadIdx.x; k < dbytes / 4; k += blockDim.x) lds.stage[kDictEarlyWord + k] = src[k];
  }
  if (!dict_tile_load(b, pd, wi.page, wi.v0, v1, nn, lds, t, early ? kDictEarly + 64 : 0)) return;
  // dict_tile_load ends without a barrier at bit width 0 (workgroup-uniform): the early dictionary's
  // stores above must still be visible to every wave before the gathers
  if (early && t.bw == 0) wg_barrier();
  const uint64_t vb = b.page_vbase[wi.page];
  const uint32_t lane = lane_id(), wv = threadIdx.x >> 6;
  const uint32_t seg0 = t.v0 - t.v0 % kDictTile + wv * 1024;  // this wave's 1024 values
  uint32_t first_err = 0xffffffffu;
  if (!is_bool && (w == 4 || w == 8)) {
    // the 16 rounds' indices first (LDS), then all gathers in flight at once, then the stores
    uint32_t idx[16];
    dict_tile_indices(t, lds, seg0, dcount, idx, first_err);
    // a dictionary that fits the stage is gathered from LDS: once every wave has its indices, the
    // stage's stream bytes are dead and the dictionary takes their place (PQ_DICT_LDS=0: global)
    const bool ldict = PQ_DICT_LDS && (uint64_t)dcount * w <= kTileStageB;  // workgroup-uniform
    if (ldict && !early) {
      wg_barrier();  // every wave's reads of the staged stream are done
      const uint32_t *src = gp_u64<const uint32_t>(cd.dict_values);
      for (uint32_t k = threadIdx.x; k < dcount * (w / 4); k += blockDim.x) lds.stage[k] = src[k];
      wg_barrier();
    }
    if (w == 4) {
      const uint32_t *dv = early ? lds.stage + kDictEarlyWord : ldict ? lds.stage : gp_u64<const uint32_t>(cd.dict_values);
      dict_store4(b, gp_u64<uint32_t>(cd.values) + vb + seg0 + lane, dv, idx);
    } else {
      const uint64_t *dv = ldict ? (const uint64_t *)lds.stage : gp_u64<const uint64_t>(cd.dict_values);
      uint64_t *out = gp_u64<uint64_t>(cd.values) + vb + seg0 + lane;
#pragma unroll
      for (uint32_t h = 0; h < 16; h += 8) {
        uint64_t val[8];
#pragma unroll
        for (uint32_t r = 0; r < 8; r++) val[r] = idx[h + r] != ~0u ? dv[idx[h + r]] : 0ull;
#pragma unroll
        for (uint32_t r = 0; r < 8; r++)
          if (idx[h + r] != ~0u) out[(h + r) * 64] = val[r];
      }
    }
    if (first_err != 0xffffffffu) report(b, pd.chunk, 1, pd.page_in_chunk, ST_VALUES, first_err, PQ_ERR_DICT_INDEX);
    return;
  }
  uint32_t ri = dict_tile_seek(t, max(seg0 + lane, t.v0));
  for (uint32_t r = 0; r < 16; r++) {
    const uint32_t v = seg0 + r * 64 + lane;
    if (v < t.v0 || v >= t.v1) continue;
    const uint32_t idx = dict_tile_value(t, lds, ri, v);
    if (is_bool) {
      (gp_u64<uint8_t>(cd.values))[vb + v] = idx == 1;
      continue;
    }
    if (idx >= dcount) {
      first_err = min(first_err, v);
      continue;
    }
    {
      const uint8_t *src = gp_u64<const uint8_t>(cd.dict_values) + (uint64_t)idx * w;
      uint8_t *dst = gp_u64<uint8_t>(cd.values) + (vb + v) * w;
      for (uint32_t k = 0; k < w; k++) dst[k] = src[k];
    }
  }
  if (first_err != 0xffffffffu) report(b, pd.chunk, 1, pd.page_in_chunk, ST_VALUES, first_err, PQ_ERR_DICT_INDEX);
}

// A grouped item (WI_DICT2): up to kDictGroup consecutive tiles of one page loaded together
// (dict_tile_loadn), so the workgroup pays the tile-load latency chain (item, descriptors, runs and
// stream) once for all of them. host.cpp groups only dictionary pages of 4-byte values whose
// dictionary fits kDictEarly, and sizes the group so its stream bytes fit the stage beside the
// dictionary, which is staged with the tiles and stays there for all of them.
constexpr uint32_t kDictGroup = 2;  // (3 measured the same on cfg5: 0.661 against 0.662 ms)
static_assert(kDictGroup == kDictGroupHost, "host.cpp groups at most kDictGroupHost tiles");
DEV void do_dict2(const BatchDev &b, const WorkItem &wi, const PageDesc &pd, const ChunkDesc &cd, uint32_t nn,
                  DictTileLDST<kDictRuns> &lds) {
  const uint32_t v1 = min(wi.v1, nn);
  const uint32_t dcount = cd.dict_count;
  if (wi.v0 >= v1) return;
  static_assert(kDictEarly == kDictEarlyHost, "dict2_eligible sizes the dictionary by kDictEarlyHost");
  if (!dict2_eligible(pd.vkind, (uint32_t)cd.value_width, dcount)) {  // (workgroup-uniform) never grouped by host.cpp
    if (threadIdx.x == 0) report(b, pd.chunk, 1, pd.page_in_chunk, ST_VALUES, wi.v0, PQ_ERR_UNSUPPORTED);
    return;
  }
  PQ_STAMPS(st, b.dbg);
  st.begin();
  {
    const uint32_t *src = gp_u64<const uint32_t>(cd.dict_values);
    for (uint32_t k = threadIdx.x; k < dcount; k += blockDim.x) lds.stage[kDictEarlyWord + k] = src[k];
  }
  DictTile t[kDictGroup];
  uint32_t nt;
  dict_tile_loadn(b, pd, wi.page, wi.v0, v1, nn, lds, t, nt, kDictEarly + 64);
  if (nt == 0) return;
  if (t[0].bw == 0) wg_barrier();  // (no stream staged: the dictionary's stores still need one)
  st.lap(0);  // diagnostic stamps: item, descriptors, runs, stream and dictionary staged
  const uint64_t vb = b.page_vbase[wi.page];
  const uint32_t lane = lane_id(), wv = threadIdx.x >> 6;
  uint32_t first_err = 0xffffffffu;
#pragma unroll
  for (uint32_t k = 0; k < kDictGroup; k++) {
    if (k >= nt) break;
    const uint32_t seg0 = t[k].v0 - t[k].v0 % kDictTile + wv * 1024;  // this wave's 1024 values of the tile
    uint32_t idx[16];
    dict_tile_indices(t[k], lds, seg0, dcount, idx, first_err);
    st.lap(1);  // indices
    dict_store4(b, gp_u64<uint32_t>(cd.values) + vb + seg0 + lane, lds.stage + kDictEarlyWord, idx);
    st.lap(2);  // gathers and stores issued
  }
  if (first_err != 0xffffffffu) report(b, pd.chunk, 1, pd.page_in_chunk, ST_VALUES, first_err, PQ_ERR_DICT_INDEX);
#ifdef PQ_DIAG_STAMPS
  if (b.dbg) __builtin_amdgcn_s_waitcnt(0);  // (diagnostic: the stores' drain)
#endif
  st.lap(3);
  st.count(4);
  st.flush(32);
}

// DELTA_BINARY_PACKED (deltabp_decoder.go:113-174 / :272-333), one workgroup per page,
// single pass over the stream: the stream is staged through a 16 KiB LDS window
// (coalesced dwordx4 loads); thread 0 walks up to 8 block headers inside the window
// (minDelta zigzag varint + miniblock widths -> miniblock offsets); then every thread
// unpacks one group of 8 deltas from LDS, a wave64 shuffle scan plus a 4-entry
// cross-wave combine gives the running sums, and each thread writes its 8 values
// (64 contiguous bytes). Requires miniblock sizes that are multiples of 8 and at most
// 2048 values per block (else PF_DELTA_SLOW).
//
// Reference semantics reproduced exactly:
//  * value[i] = first + sum of (delta[k] + minDelta[block(k)]) for k < i, with the
//    look-ahead: returning value i reads the group holding delta i (Q1);
//  * next() at position p fails when p >= the header's valuesCount (io.EOF);
//  * a block header is read by next() at the block's first position; its errors
//    (varint EOF/overflow/range, short width bytes, width > 32/64) surface there;
//  * a group is read with io.ReadFull at its first position (EOF / ErrUnexpectedEOF).
// `s` may be an LDS view of the stream that is valid for 10 + mbc bytes from pos; `gs`
// is the stream in global memory, read only for varints longer than 10 bytes.
DEV bool delta_hdr(const uint8_t *s, const uint8_t *gs, uint32_t n, uint32_t pos, bool is64, uint32_t mbc,
                   int64_t *min_delta, uint8_t *w, uint32_t *hdr_len, uint32_t *err) {
  // minDelta: zigzag varint (readVariant32 / readVariant64), then mbc width bytes (io.ReadFull)
  uint64_t x = 0;
  unsigned sh = 0;
  uint32_t k = 0;
  for (;; k++) {
    if (pos + k >= n) { *err = PQ_ERR_EOF; return false; }
    if (k == 10) {  // Go keeps reading: a later terminator is an overflow, none is EOF
      for (uint32_t q = pos + 10; q < n; q++)
        if (gs[q] < 0x80) { *err = PQ_ERR_RANGE; return false; }
      *err = PQ_ERR_EOF;
      return false;
    }
    uint32_t by = s[pos + k];
    if (by < 0x80) {
      if (k > 9 || (k == 9 && by > 1)) { *err = PQ_ERR_RANGE; return false; }
      if (sh < 64) x |= (uint64_t)by << sh;
      break;
    }
    if (sh < 64) x |= (uint64_t)(by & 0x7f) << sh;
    sh += 7;
  }
  int64_t v = (int64_t)(x >> 1);
  if (x & 1) v = ~v;
  if (!is64 && (v > 2147483647ll || v < -2147483648ll)) { *err = PQ_ERR_RANGE; return false; }
  *min_delta = v;
  uint32_t p = pos + k + 1;
  if (p >= n && mbc > 0) { *err = PQ_ERR_EOF; return false; }
  if (p + mbc > n) { *err = PQ_ERR_UNEXPECTED_EOF; return false; }
  for (uint32_t i = 0; i < mbc; i++) {
    uint32_t wi = s[p + i];
    if (wi > (is64 ? 64u : 32u)) { *err = PQ_ERR_INVALID; return false; }
    if (w) w[i] = (uint8_t)wi;
  }
  *hdr_len = k + 1 + mbc;
  return true;
}



// ---------------------------------------------------------------------------
// DELTA_BINARY_PACKED, tiled pipeline (deltabp_decoder.go:113-174 / :272-333).
//
// The only serial part of the format is the chain of block headers (a block's
// position follows from the previous block's miniblock widths). It runs alone:
//  1. k_delta_walk: one workgroup per page streams the page through a 16 KiB LDS
//     window (the next window is loaded into registers while lane 0 walks the
//     current one, at issue priority 3) and writes one DeltaBlk per block: minDelta,
//     miniblock widths, payload position. Header errors are reported at the block's
//     first value position (next() reads the header there, :119-135).
//  2. k_delta_sums: one thread per group of 8 deltas, every tile of every page in
//     parallel: per-block sums of (delta + minDelta) (wrapping, LDS 64-bit atomics).
//  3. k_delta_prefix: per page, exclusive scan of the block sums from the first value.
//  4. WI_DELTA_TILE items of k_values (beside the PLAIN tiles): unpack, tile scan,
//     block base, 8 values per thread; group read errors (io.ReadFull EOF /
//     ErrUnexpectedEOF at the group's first position, :137-141) are reported here.
// Semantics: value i = first + sum_{k<i} (delta_k + minDelta(block(k))); returning
// value i reads the group (and at block starts the header) holding delta i (the Q1
// look-ahead); positions >= valuesCount fail with io.EOF. The first error in value
// order wins through the chunk's atomicMin error key.
// ---------------------------------------------------------------------------
constexpr uint32_t kDwWin = 16384;                     // walk window bytes
constexpr uint32_t kDwWinLoad = kDwWin + 64;           // + overlap for a header straddling the end

struct DeltaWalkLDS {
  uint32_t win[kDwWinLoad / 4 + 4];
  uint32_t pos, j, done, reload;
};

// Block header at stream position pos (readMiniBlockHeader :88-111 / :247-270) from the
// LDS window holding stream bytes [wa, wa + kDwWinLoad): zigzag minDelta varint, then
// mbc (<= 8) width bytes. Returns the error class (0 = ok).
DEV uint32_t delta_hdr_parse(const uint32_t *win, uint32_t wa, const uint8_t *gs, uint32_t n, uint32_t pos, bool is64,
                             uint32_t mbc, int64_t *md, uint64_t *widths, uint32_t *hlen) {
  const uint32_t off = pos - wa, a = off >> 2, sh = off & 3;
  const uint32_t w0 = win[a], w1 = win[a + 1], w2 = win[a + 2], w3 = win[a + 3], w4 = win[a + 4];
  const uint32_t u0 = __builtin_amdgcn_alignbyte(w1, w0, sh), u1 = __builtin_amdgcn_alignbyte(w2, w1, sh),
                 u2 = __builtin_amdgcn_alignbyte(w3, w2, sh), u3 = __builtin_amdgcn_alignbyte(w4, w3, sh);
  const uint64_t lo = (uint64_t)u0 | ((uint64_t)u1 << 32), hi = (uint64_t)u2 | ((uint64_t)u3 << 32);
  const uint64_t term = ~lo & 0x8080808080808080ull;
  uint64_t x = 0;
  uint32_t L = 0;
  if (term) {
    L = (uint32_t)(__builtin_ctzll(term) >> 3) + 1;
    if (pos + L > n) return PQ_ERR_EOF;  // the stream ends inside the varint (ReadByte at EOF)
    uint64_t y = lo & (L == 8 ? ~0ull : ((1ull << (8 * L)) - 1ull)) & 0x7f7f7f7f7f7f7f7full;
    y = (y & 0x007f007f007f007full) | ((y & 0x7f007f007f007f00ull) >> 1);
    y = (y & 0x00003fff00003fffull) | ((y & 0x3fff00003fff0000ull) >> 2);
    x = (y & 0x000000000fffffffull) | ((y & 0x0fffffff00000000ull) >> 4);
  } else {  // 9+ byte varint: Go's ReadUvarint byte by byte
    unsigned shv = 0;
    for (uint32_t k = 0;; k++) {
      if (pos + k >= n) return PQ_ERR_EOF;
      if (k == 10) return resolve_long_varint(gs, pos - 2, n) == PQ_ERR_RANGE ? PQ_ERR_RANGE : PQ_ERR_EOF;
      const uint32_t by = k < 8 ? (uint32_t)(lo >> (8 * k)) & 0xffu : (uint32_t)(hi >> (8 * (k - 8))) & 0xffu;
      if (by < 0x80) {
        if (k == 9 && by > 1) return PQ_ERR_RANGE;
        if (shv < 64) x |= (uint64_t)by << shv;
        L = k + 1;
        break;
      }
      if (shv < 64) x |= (uint64_t)(by & 0x7f) << shv;
      shv += 7;
    }
  }
  int64_t v = (int64_t)(x >> 1);
  if (x & 1) v = ~v;
  if (!is64 && (v > 2147483647ll || v < -2147483648ll)) return PQ_ERR_RANGE;
  const uint32_t p = pos + L;
  if (p >= n && mbc > 0) return PQ_ERR_EOF;
  if (p + mbc > n) return PQ_ERR_UNEXPECTED_EOF;
  // widths: bytes [L, L + mbc) of the 16 register bytes (L <= 10, mbc <= 8 -> within 18: use a
  // second funnel when L + mbc > 16)
  uint64_t wv;
  if (L + mbc <= 16) {
    wv = L == 8 ? hi : (L < 8 ? ((lo >> (8 * L)) | (hi << (64 - 8 * L))) : (hi >> (8 * (L - 8))));
  } else {
    wv = 0;
    for (uint32_t i = 0; i < mbc; i++) wv |= (uint64_t)(lds_ld32(win, off + L + i) & 0xffu) << (8 * i);
  }
  if (mbc < 8) wv &= (1ull << (8 * mbc)) - 1ull;
  const uint32_t lim = is64 ? 64u : 32u;
  uint64_t t = wv;
  for (uint32_t i = 0; i < mbc; i++, t >>= 8)
    if ((t & 0xffu) > lim) return PQ_ERR_INVALID;
  *md = v;
  *widths = wv;
  *hlen = L + mbc;
  return 0;
}

DEV uint32_t bytesum64(uint64_t w) {
  return __builtin_amdgcn_sad_u8((uint32_t)w, 0u, 0u) + __builtin_amdgcn_sad_u8((uint32_t)(w >> 32), 0u, 0u);
}
DEV uint32_t bytesum64_swar(uint64_t w) {  // scalar-friendly byte sum
  w = (w & 0x00ff00ff00ff00ffull) + ((w >> 8) & 0x00ff00ff00ff00ffull);
  w = (w & 0x0000ffff0000ffffull) + ((w >> 16) & 0x0000ffff0000ffffull);
  return (uint32_t)w + (uint32_t)(w >> 32);
}
DEV uint64_t sgpr64(uint64_t v) {
  return ((uint64_t)sgpr((uint32_t)(v >> 32)) << 32) | sgpr((uint32_t)v);
}

// Common-case block header hop (wave-uniform inputs and result): minDelta varint of at
// most 8 bytes, mbc <= 8 widths within the 16 bytes read, every width valid, header and
// widths inside the stream. Returns 0 when the exact parser (delta_hdr_parse) is needed.
DEV uint32_t delta_hdr_fast(const uint32_t *win, uint32_t wa, uint32_t n, uint32_t pos, uint32_t mbc, uint32_t wlim,
                            int64_t *md, uint64_t *widths) {
  const uint32_t off = pos - wa, a = off >> 2, sh = off & 3;
  const uint32_t w0 = sgpr(win[a]), w1 = sgpr(win[a + 1]), w2 = sgpr(win[a + 2]), w3 = sgpr(win[a + 3]),
                 w4 = sgpr(win[a + 4]);
  const uint32_t u0 = sgpr(__builtin_amdgcn_alignbyte(w1, w0, sh)), u1 = sgpr(__builtin_amdgcn_alignbyte(w2, w1, sh)),
                 u2 = sgpr(__builtin_amdgcn_alignbyte(w3, w2, sh)), u3 = sgpr(__builtin_amdgcn_alignbyte(w4, w3, sh));
  const uint64_t lo = (uint64_t)u0 | ((uint64_t)u1 << 32), hi = (uint64_t)u2 | ((uint64_t)u3 << 32);
  const uint64_t term = ~lo & 0x8080808080808080ull;
  if (!term) return 0;
  const uint32_t L = (uint32_t)(__builtin_ctzll(term) >> 3) + 1;
  if (L + mbc > 16 || pos + L + mbc > n) return 0;
  uint64_t y = lo & (L == 8 ? ~0ull : ((1ull << (8 * L)) - 1ull)) & 0x7f7f7f7f7f7f7f7full;
  y = (y & 0x007f007f007f007full) | ((y & 0x7f007f007f007f00ull) >> 1);
  y = (y & 0x00003fff00003fffull) | ((y & 0x3fff00003fff0000ull) >> 2);
  const uint64_t x = (y & 0x000000000fffffffull) | ((y & 0x0fffffff00000000ull) >> 4);
  int64_t v = (int64_t)(x >> 1);
  if (x & 1) v = ~v;
  if (wlim == 32 && (v > 2147483647ll || v < -2147483648ll)) return 0;
  uint64_t wv = L == 8 ? hi : ((lo >> (8 * L)) | (hi << (64 - 8 * L)));
  if (mbc < 8) wv &= (1ull << (8 * mbc)) - 1ull;
  // any width byte > wlim: (byte + (127 - wlim)) reaches bit 7, or the byte has it already
  const uint64_t add = (0x7full - wlim) * 0x0101010101010101ull;
  if (((wv + add) | wv) & 0x8080808080808080ull) return 0;
  *md = v;
  *widths = wv;
  return L + mbc;
}

DEV void delta_group_at(const DeltaBlk &B, uint32_t inb, uint32_t mbvc, uint32_t g8, uint32_t *goff, uint32_t *w);
DEV void delta_unpack8_lds(const uint32_t *stg, int32_t base, uint32_t goff, uint32_t w, bool is64, int64_t md,
                           uint64_t (&d)[8]);

// One workgroup per page: block index (walk), block sums and their scan, fused. Windows
// start at a block header and hold whole blocks (a block's payload is at most
// kDeltaTileVals * 8 bytes), so the blocks walked in a window are summed from LDS before
// the next window is loaded at the first block that did not fit.
constexpr uint32_t kDiWin = kDeltaTileVals * 8 + 1024;  // window bytes (>= the largest block + header)
constexpr uint32_t kDiMaxBlk = 256;                     // blocks per window
struct DeltaIndexLDS {
  uint32_t win[kDiWin / 4 + 8];
  int64_t md[kDiMaxBlk];
  uint64_t wd[kDiMaxBlk];
  uint32_t pos[kDiMaxBlk];
  unsigned long long acc[kDiMaxBlk];
  uint64_t wsum[4];
  uint32_t nblk, next, done;
};

__global__ void __launch_bounds__(256) k_delta_walk(BatchDev b_in, const uint32_t *pages) {
  const BatchDev b = global_view(b_in);
  __shared__ DeltaIndexLDS L;
  const uint32_t pi = pages[blockIdx.x];
  const PageDesc &pd = b.pages[pi];
  const uint32_t tid = threadIdx.x, lane = lane_id(), wv = tid >> 6;
  const uint32_t nn = b.page_nn_v[pi];
  const uint8_t *s = gp_u64<const uint8_t>(pd.data) + pd.val_off;
  const uint32_t n = pd.val_len;
  const bool is64 = pd.vkind == VK_DELTA64;
  const uint32_t mbc = pd.delta_mbc, mbvc = pd.delta_mbvc, bs = mbc * mbvc, g8 = mbvc / 8, gpb = bs / 8;
  DeltaBlk *tab = b.dblk + b.dblk_base[pi];
  uint32_t limit = nn;
  if ((uint32_t)pd.delta_count < nn) {
    limit = (uint32_t)pd.delta_count;
    if (tid == 0) report(b, pd.chunk, 1, pd.page_in_chunk, ST_VALUES, limit, PQ_ERR_EOF);  // next() past valuesCount
  }
  const uint32_t need = (uint32_t)(((uint64_t)limit + bs - 1) / bs);
  uint32_t pos = pd.delta_first_mb - pd.val_off, j = 0;
  uint64_t carry = (uint64_t)pd.delta_first;
  const uint32_t wlim = is64 ? 64u : 32u;
  const uint64_t wadd = (0x7full - wlim) * 0x0101010101010101ull;
  const uint64_t wmask = mbc >= 8 ? ~0ull : ((1ull << (8 * mbc)) - 1ull);
  bool stop = need == 0;
  while (!stop) {
    // ---- window at the next block header (16-B aligned address; wa may be a few bytes below 0)
    const int32_t wa = (int32_t)pos - (int32_t)(((uintptr_t)(s + pos)) & 15u);
    {
      const uint4 *src = (const uint4 *)(s + wa);
      const int64_t lim = (int64_t)n + 16 - wa;  // the page padding keeps 16 B past n readable
      uint4 *dst = (uint4 *)L.win;
      for (uint32_t q = tid; q < kDiWin / 16 + 1; q += 256) dst[q] = (int64_t)q * 16 < lim ? src[q] : make_uint4(0, 0, 0, 0);
    }
    wg_barrier();
    const int64_t wend = (int64_t)wa + kDiWin;  // bytes [wa, wend) are staged
    // ---- wave 0 walks the blocks that fit whole in the window
    if (wv == 0) {
      __builtin_amdgcn_s_setprio(3);
      uint32_t k = 0, done = 0;
      uint32_t p = pos, jj = j;
      while (jj < need && k < kDiMaxBlk) {
        int64_t md = 0;
        uint64_t wd = 0;
        uint32_t hl = 0;
        if (p >= n) {  // next() reads block jj's header at EOF
          if (lane == 0) report(b, pd.chunk, 1, pd.page_in_chunk, ST_VALUES, jj * bs, PQ_ERR_EOF);
          done = 1;
          break;
        }
        if ((int64_t)p + 32 > wend) break;  // header not staged: next window
        {  // common case: minDelta varint of <= 4 bytes, widths within the 8 bytes read
          const uint32_t off = (uint32_t)((int32_t)p - wa), a = off >> 2, sh = off & 3;
          const uint64_t x01 = ((uint64_t)L.win[a + 1] << 32) | L.win[a];
          const uint32_t x2 = L.win[a + 2];
          const uint64_t u = (x01 >> (8 * sh)) | (sh ? ((uint64_t)x2 << (64 - 8 * sh)) : 0ull);
          const uint32_t u0 = (uint32_t)u, t = ~u0 & 0x80808080u;
          const uint32_t Lv = t ? (uint32_t)(__builtin_ctz(t) >> 3) + 1 : 8u;
          if (Lv + mbc <= 8 && p + Lv + mbc <= n) {
            const uint32_t y = (Lv >= 4 ? u0 : (u0 & ((1u << (8 * Lv)) - 1u))) & 0x7f7f7f7fu;
            const uint32_t x = (y & 0x7fu) | ((y >> 1) & 0x3f80u) | ((y >> 2) & 0x1fc000u) | ((y >> 3) & 0xfe00000u);
            const uint64_t wvv = (u >> (8 * Lv)) & wmask;
            if (!(((wvv + wadd) | wvv) & 0x8080808080808080ull)) {
              md = (int64_t)(x >> 1) ^ -(int64_t)(x & 1);
              wd = wvv;
              hl = Lv + mbc;
            }
          }
        }
        if (!hl) {  // exact parse: longer varint, many miniblocks, or an error
          const uint32_t e = delta_hdr_parse(L.win, (uint32_t)wa, s, n, p, is64, mbc, &md, &wd, &hl);
          if (e) {  // the header of block jj is read by next() at position jj * bs
            if (lane == 0) report(b, pd.chunk, 1, pd.page_in_chunk, ST_VALUES, jj * bs, e);
            done = 1;
            break;
          }
        }
        const uint32_t blen = hl + g8 * bytesum64(wd);
        if ((int64_t)p + blen > wend && (int64_t)p + blen <= (int64_t)n + 0 && k > 0) break;  // next window
        if (lane == 0) { L.md[k] = md; L.wd[k] = wd; L.pos[k] = p + hl; }
        k++;
        jj++;
        p += blen;
      }
      if (lane == 0) { L.nblk = k; L.next = p; L.done = done; }
      __builtin_amdgcn_s_setprio(0);
    }
    wg_barrier();
    const uint32_t nb = L.nblk;
    // ---- block sums of the window's blocks (groups past the stream end contribute 0;
    // their read error is reported by the tile pass)
    for (uint32_t q = tid; q < nb; q += 256) L.acc[q] = 0;
    wg_barrier();
    for (uint32_t gi = tid; gi < nb * gpb; gi += 256) {
      const uint32_t k = gi / gpb, inb = (gi % gpb) * 8;
      if ((uint64_t)(j + k) * bs + inb >= limit) continue;
      DeltaBlk B;
      B.widths = L.wd[k];
      B.pos = L.pos[k];
      uint32_t goff, w;
      delta_group_at(B, inb, mbvc, g8, &goff, &w);
      if ((uint64_t)goff + w > n || (int64_t)goff + 24 > wend) continue;
      uint64_t d[8];
      delta_unpack8_lds(L.win, wa, goff, w, is64, L.md[k], d);
      uint64_t sum = 0;
#pragma unroll
      for (int e = 0; e < 8; e++) sum += d[e];
      atomicAdd(&L.acc[k], (unsigned long long)sum);
    }
    wg_barrier();
    // ---- scan of the block sums -> block base values; complete block records
    for (uint32_t k0 = 0; k0 < nb; k0 += 256) {
      const uint32_t k = k0 + tid;
      const uint64_t v = k < nb ? (uint64_t)L.acc[k] : 0;
      const uint64_t incl = wave_incl_scan64(v);
      if (lane == 63) L.wsum[wv] = incl;
      wg_barrier();
      uint64_t before = carry, total = 0;
      for (uint32_t q = 0; q < 4; q++) {
        if (q < wv) before += L.wsum[q];
        total += L.wsum[q];
      }
      if (k < nb) {
        DeltaBlk blk;
        blk.min_delta = L.md[k];
        blk.widths = L.wd[k];
        blk.base = (int64_t)(before + incl - v);
        blk.pos = L.pos[k];
        blk.sum_lo = 0;
        tab[j + k] = blk;
      }
      carry += total;
      wg_barrier();
    }
    j += nb;
    pos = L.next;
    stop = L.done || j >= need || (nb == 0 && pos >= n);
    wg_barrier();
  }
  if (tid == 0) b.dblk_n[pi] = j;
}

// Group g (8 deltas from position d0) of a page: payload offset and width.
DEV void delta_group_at(const DeltaBlk &B, uint32_t inb, uint32_t mbvc, uint32_t g8, uint32_t *goff, uint32_t *w) {
  const uint32_t m = inb / mbvc, o = inb % mbvc;
  const uint64_t below = m >= 8 ? B.widths : (B.widths & ((1ull << (8 * m)) - 1ull));
  *w = (uint32_t)(B.widths >> (8 * m)) & 0xffu;
  *goff = B.pos + g8 * bytesum64(below) + (o / 8) * *w;
}

// The 8 deltas (unpacked + minDelta, wrapping) of a group of width w at byte goff.
// A group is w bytes; widths <= 16 read 5 aligned dwords once, wider ones per value.
DEV void delta_unpack8(const uint8_t *s, uint32_t goff, uint32_t w, bool is64, int64_t md, uint64_t (&d)[8]) {
  if (w <= 16) {
    const uint32_t sh = (uint32_t)((uintptr_t)(s + goff) & 3);
    const uint32_t *q = (const uint32_t *)(s + goff - sh);
    const uint32_t x0 = q[0], x1 = q[1], x2 = q[2], x3 = q[3], x4 = q[4];
    const uint64_t lo = (uint64_t)__builtin_amdgcn_alignbyte(x1, x0, sh) | ((uint64_t)__builtin_amdgcn_alignbyte(x2, x1, sh) << 32);
    const uint64_t hi = (uint64_t)__builtin_amdgcn_alignbyte(x3, x2, sh) | ((uint64_t)__builtin_amdgcn_alignbyte(x4, x3, sh) << 32);
    const uint64_t mask = w >= 64 ? ~0ull : ((1ull << w) - 1ull);
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const uint32_t bo = k * w;
      uint64_t u = bo >= 64 ? (hi >> (bo - 64)) : ((lo >> bo) | (bo ? (hi << (64 - bo)) : 0ull));
      u &= mask;
      if (!is64) u = (uint64_t)(int64_t)(int32_t)(uint32_t)u;
      d[k] = u + (uint64_t)md;
    }
  } else {
#pragma unroll
    for (int k = 0; k < 8; k++) {
      uint64_t u = bits64(s, (uint64_t)goff * 8 + (uint64_t)k * w, w);
      if (!is64) u = (uint64_t)(int64_t)(int32_t)(uint32_t)u;
      d[k] = u + (uint64_t)md;
    }
  }
}

// Common geometry of a DELTA tile work item for thread tid.
struct DeltaGroup {
  bool valid;        // group holds a needed delta of a walked block
  uint32_t d0, j, goff, w, err;
};
DEV DeltaGroup delta_tile_group(const BatchDev &b, const WorkItem &wi, const PageDesc &pd, uint32_t limit,
                                uint32_t tid, DeltaBlk *B) {
  DeltaGroup g{false, wi.v0 + 8 * tid, 0, 0, 0, 0};
  const uint32_t mbvc = pd.delta_mbvc, bs = pd.delta_mbc * mbvc;
  if (g.d0 >= limit) return g;
  g.j = g.d0 / bs;
  if (g.j >= b.dblk_n[wi.page]) return g;
  *B = b.dblk[b.dblk_base[wi.page] + g.j];
  g.valid = true;
  delta_group_at(*B, g.d0 % bs, mbvc, mbvc / 8, &g.goff, &g.w);
  const uint32_t n = pd.val_len;
  if (g.w > 0 && g.goff >= n) g.err = PQ_ERR_EOF;  // io.ReadFull of the group (:137-141)
  else if ((uint64_t)g.goff + g.w > n) g.err = PQ_ERR_UNEXPECTED_EOF;
  return g;
}

// A DELTA tile's payload bytes (first to last walked block of the tile) staged in LDS with
// coalesced 16-B loads; returns the stream offset of LDS byte 0 (16-B aligned address, may
// be a few bytes below 0), or INT32_MIN when the tile has no walked block.
constexpr uint32_t kDtStageB = kDeltaTileVals * 8 + 8 * 24 + 64;  // 64-bit widths + headers + slack
DEV int32_t delta_stage_tile(const BatchDev &b, const WorkItem &wi, const PageDesc &pd, uint32_t *stg) {
  const uint32_t bs = pd.delta_mbc * pd.delta_mbvc, g8 = pd.delta_mbvc / 8, n = pd.val_len;
  const uint32_t j0 = wi.v0 / bs, nbt = kDeltaTileVals / bs, nb = b.dblk_n[wi.page];
  if (j0 >= nb) return INT32_MIN;
  const DeltaBlk *tab = b.dblk + b.dblk_base[wi.page];
  const uint32_t j1 = min(j0 + nbt, nb) - 1;
  const DeltaBlk last = tab[j1];
  const uint32_t lo = tab[j0].pos;
  const uint32_t hi = min((uint64_t)last.pos + (uint64_t)g8 * bytesum64(last.widths), (uint64_t)n);
  const uint8_t *s = gp_u64<const uint8_t>(pd.data) + pd.val_off;
  const int32_t base = (int32_t)lo - (int32_t)(((uintptr_t)(s + lo)) & 15u);
  const int32_t end = (int32_t)max(hi, lo) + 16;  // the page padding keeps 16 B past n readable
  const uint32_t nv = (uint32_t)(end - base + 15) / 16;
  const uint4 *src = (const uint4 *)(s + base);
  uint4 *dst = (uint4 *)stg;
  for (uint32_t k = threadIdx.x; k < nv && k < kDtStageB / 16; k += blockDim.x) dst[k] = src[k];
  return base;
}

// delta_unpack8 from the staged tile (group at stream offset goff, LDS byte 0 = offset base).
DEV void delta_unpack8_lds(const uint32_t *stg, int32_t base, uint32_t goff, uint32_t w, bool is64, int64_t md,
                           uint64_t (&d)[8]) {
  const uint32_t o = (uint32_t)((int32_t)goff - base);
  if (w <= 16) {
    const uint32_t a = o >> 2, sh = o & 3;
    const uint32_t x0 = stg[a], x1 = stg[a + 1], x2 = stg[a + 2], x3 = stg[a + 3], x4 = stg[a + 4];
    const uint64_t lo = (uint64_t)__builtin_amdgcn_alignbyte(x1, x0, sh) | ((uint64_t)__builtin_amdgcn_alignbyte(x2, x1, sh) << 32);
    const uint64_t hi = (uint64_t)__builtin_amdgcn_alignbyte(x3, x2, sh) | ((uint64_t)__builtin_amdgcn_alignbyte(x4, x3, sh) << 32);
    const uint64_t mask = (1ull << w) - 1ull;
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const uint32_t bo = k * w;
      uint64_t u = bo >= 64 ? (hi >> (bo - 64)) : ((lo >> bo) | (bo ? (hi << (64 - bo)) : 0ull));
      u &= mask;
      if (!is64) u = (uint64_t)(int64_t)(int32_t)(uint32_t)u;
      d[k] = u + (uint64_t)md;
    }
  } else {
#pragma unroll
    for (int k = 0; k < 8; k++) {
      uint64_t u = lds_bits64(stg, o * 8 + (uint32_t)k * w, w);
      if (!is64) u = (uint64_t)(int64_t)(int32_t)(uint32_t)u;
      d[k] = u + (uint64_t)md;
    }
  }
}

__global__ void __launch_bounds__(256) k_delta_sums(BatchDev b_in, const WorkItem *items) {
  const BatchDev b = global_view(b_in);
  __shared__ uint32_t stg[kDtStageB / 4];
  __shared__ unsigned long long acc[kDeltaTileVals / 128];
  const WorkItem wi = items[blockIdx.x];
  const PageDesc &pd = b.pages[wi.page];
  const uint32_t tid = threadIdx.x;
  const uint32_t bs = pd.delta_mbc * pd.delta_mbvc;
  const uint32_t nn = b.page_nn_v[wi.page];
  const uint32_t limit = min(nn, (uint32_t)max(pd.delta_count, 0));
  const uint32_t nbt = kDeltaTileVals / bs;  // blocks per tile (bs divides the tile)
  if (tid < nbt) acc[tid] = 0;
  if (wi.v0 >= limit) return;  // workgroup-uniform
  const int32_t base = delta_stage_tile(b, wi, pd, stg);
  wg_barrier();
  DeltaBlk B;
  const DeltaGroup g = delta_tile_group(b, wi, pd, limit, tid, &B);
  if (g.valid && !g.err) {
    uint64_t d[8];
    delta_unpack8_lds(stg, base, g.goff, g.w, pd.vkind == VK_DELTA64, B.min_delta, d);
    uint64_t sum = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) sum += d[k];
    atomicAdd(&acc[(g.d0 - wi.v0) / bs], (unsigned long long)sum);
  }
  wg_barrier();
  if (tid < nbt) {
    const uint32_t j = wi.v0 / bs + tid;
    if (j < b.dblk_n[wi.page]) b.dblk_sum[b.dblk_base[wi.page] + j] = acc[tid];
  }
}

__global__ void __launch_bounds__(256) k_delta_prefix(BatchDev b_in, const uint32_t *pages) {
  const BatchDev b = global_view(b_in);
  __shared__ uint64_t wsum[4];
  __shared__ uint64_t carry;
  const uint32_t pi = pages[blockIdx.x];
  const PageDesc &pd = b.pages[pi];
  const uint32_t tid = threadIdx.x, lane = lane_id(), wv = tid >> 6;
  const uint32_t nb = b.dblk_n[pi];
  DeltaBlk *tab = b.dblk + b.dblk_base[pi];
  const unsigned long long *sums = b.dblk_sum + b.dblk_base[pi];
  if (tid == 0) carry = (uint64_t)pd.delta_first;
  wg_barrier();
  for (uint32_t j0 = 0; j0 < nb; j0 += 256) {
    const uint32_t j = j0 + tid;
    const uint64_t v = j < nb ? sums[j] : 0;
    const uint64_t incl = wave_incl_scan64(v);
    if (lane == 63) wsum[wv] = incl;
    wg_barrier();
    uint64_t before = carry, total = 0;
    for (uint32_t k = 0; k < 4; k++) {
      if (k < wv) before += wsum[k];
      total += wsum[k];
    }
    if (j < nb) tab[j].base = (int64_t)(before + incl - v);
    wg_barrier();
    if (tid == 0) carry += total;
    wg_barrier();
  }
}

// WI_DELTA_TILE: 8 values per thread.
DEV void do_delta_tile(const BatchDev &b, const WorkItem &wi, const PageDesc &pd, const ChunkDesc &cd, uint32_t nn,
                       uint64_t *scan, uint32_t *stg) {
  const uint32_t tid = threadIdx.x, lane = lane_id(), wv = tid >> 6;
  const bool is64 = pd.vkind == VK_DELTA64;
  const uint32_t bs = pd.delta_mbc * pd.delta_mbvc;
  const uint32_t limit = min(nn, (uint32_t)max(pd.delta_count, 0));
  if (wi.v0 >= limit) return;  // workgroup-uniform
  const int32_t base = delta_stage_tile(b, wi, pd, stg);
  wg_barrier();
  DeltaBlk B;
  const DeltaGroup g = delta_tile_group(b, wi, pd, limit, tid, &B);
  uint64_t d[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t sum = 0;
  if (g.valid && g.err) report(b, pd.chunk, 1, pd.page_in_chunk, ST_VALUES, g.d0, g.err);
  if (g.valid && !g.err) {
    delta_unpack8_lds(stg, base, g.goff, g.w, is64, B.min_delta, d);
#pragma unroll
    for (int k = 0; k < 8; k++) sum += d[k];
  }
  // exclusive scan of group sums over the tile; a block's values restart from its base
  const uint64_t incl = wave_incl_scan64(sum);
  if (lane == 63) scan[256 + wv] = incl;
  wg_barrier();
  uint64_t before = 0;
  for (uint32_t k = 0; k < wv; k++) before += scan[256 + k];
  const uint64_t excl = before + incl - sum;
  scan[tid] = excl;
  wg_barrier();
  // values of this group, staged in LDS (the payload stage is free after the scan barrier)
  // and stored with coalesced 16-B writes: a thread's 8 values are 64 contiguous bytes, so
  // storing them directly would make every store instruction write partial cache lines
  uint64_t out[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (g.valid && !g.err) {
    const uint32_t gb = (g.j * bs - wi.v0) / 8;  // the block's first group in this tile
    uint64_t run = (uint64_t)B.base + (excl - scan[gb]);
#pragma unroll
    for (int k = 0; k < 8; k++) { out[k] = run; run += d[k]; }
  }
  if (is64) {
    uint4 *o = (uint4 *)stg + tid * 4;
#pragma unroll
    for (int k = 0; k < 4; k++)
      o[k] = make_uint4((uint32_t)out[2 * k], (uint32_t)(out[2 * k] >> 32), (uint32_t)out[2 * k + 1],
                        (uint32_t)(out[2 * k + 1] >> 32));
  } else {
    uint4 *o = (uint4 *)stg + tid * 2;
    o[0] = make_uint4((uint32_t)out[0], (uint32_t)out[1], (uint32_t)out[2], (uint32_t)out[3]);
    o[1] = make_uint4((uint32_t)out[4], (uint32_t)out[5], (uint32_t)out[6], (uint32_t)out[7]);
  }
  wg_barrier();
  const uint32_t w = is64 ? 8u : 4u;
  const uint32_t cnt = min(kDeltaTileVals, limit - wi.v0);  // values of this tile before the limit
  const uint64_t vb = b.page_vbase[wi.page];
  uint8_t *dst = gp_u64<uint8_t>(cd.values) + (vb + wi.v0) * w;
  const uint32_t bytes = cnt * w;
  if (((uintptr_t)dst & 15) == 0) {
    for (uint32_t q = tid; q < bytes / 16; q += blockDim.x) ((uint4 *)dst)[q] = ((const uint4 *)stg)[q];
    for (uint32_t q = (bytes & ~15u) / 4 + tid; q < bytes / 4; q += blockDim.x) ((uint32_t *)dst)[q] = stg[q];
  } else if (((uintptr_t)dst & 7) == 0) {
    for (uint32_t q = tid; q < bytes / 8; q += blockDim.x) ((uint2 *)dst)[q] = ((const uint2 *)stg)[q];
    for (uint32_t q = (bytes & ~7u) / 4 + tid; q < bytes / 4; q += blockDim.x) ((uint32_t *)dst)[q] = stg[q];
  } else {
    for (uint32_t q = tid; q < bytes / 4; q += blockDim.x) ((uint32_t *)dst)[q] = stg[q];
  }
}

// ---------------------------------------------------------------------------
// DELTA_BINARY_PACKED, one workgroup per page, single pass (WI_DELTA_PAGE;
// deltabp_decoder.go:113-174 / :272-333).
//
// The stream goes through an LDS window of kDeltaWinLoad bytes that starts at the next
// block header. Per window:
//  1. walk: wave 0 follows the block-header chain (position -> next position only:
//     varint length from a byte mask, widths summed with SWAR) in scalar registers;
//     headers the fast form cannot take go through the exact parser;
//  2. the next window's loads are issued into registers (they land during 3-4);
//  3. parse: one thread per walked block re-reads its header exactly (minDelta,
//     widths, Go error class) and finds the first group io.ReadFull cannot read whole;
//     the first error in value order (an LDS atomicMin over (position, class)) bounds the
//     values written;
//  4. batches of 256 groups of 8 deltas: unpack from LDS, wave64 DPP scan of the group
//     sums plus a 4-wave combine, 8 values per thread written as 16-B stores.
// Semantics as the tiled path above: value i = first + sum_{k<i} delta_k; returning value
// i reads the group (and at a block start the header) holding delta i (Q1); positions >=
// valuesCount fail with io.EOF.
// ---------------------------------------------------------------------------
struct DeltaPageLDS {
  uint32_t win[kDeltaWinLoad / 4 + 8];  // stream bytes [win0, win0 + kDeltaWinLoad + 32)
  uint32_t hpos[kDeltaMaxBlk];          // header position of each walked block
  uint32_t ppos[kDeltaMaxBlk];          // payload position
  int64_t md[kDeltaMaxBlk];
  uint64_t wd[kDeltaMaxBlk];            // miniblock widths, 8 bits each
  uint64_t wsum[2][4];                  // per-wave batch totals (double-buffered by batch parity)
  uint4 xpose[4][128];                  // per-wave output transpose (2 KiB of output at a time)
  unsigned long long stop;              // (value position << 4 | class) of the first error
  uint32_t nb, next;
};

union ValuesLDS {
  DeltaTileLDS dtile;        // WI_DELTA_TILE
  DeltaPageLDS dpage;        // WI_DELTA_PAGE

};

// Length of the block at stream position pos (scalar registers): header varint of at most
// 8 - mbc bytes, widths from the same 8 bytes. 0 = take the exact parser.
DEV uint32_t delta_blk_len_s(const uint32_t *win, int32_t win0, uint32_t pos, uint32_t mbc, uint32_t g8) {
  const uint32_t off = (uint32_t)((int32_t)pos - win0), a = off >> 2, sh = off & 3;
  const uint32_t w0 = sgpr(win[a]), w1 = sgpr(win[a + 1]), w2 = sgpr(win[a + 2]);
  const uint64_t lo = ((uint64_t)w1 << 32) | w0;
  const uint64_t x = sh ? ((lo >> (8 * sh)) | ((uint64_t)w2 << (64 - 8 * sh))) : lo;  // bytes pos .. pos+7
  const uint32_t t = ~(uint32_t)x & 0x80808080u;
  if (!t) return 0;
  const uint32_t L = (uint32_t)(__builtin_ctz(t) >> 3) + 1;
  if (L + mbc > 8) return 0;
  const uint64_t ww = (x >> (8 * L)) & ((1ull << (8 * mbc)) - 1ull);
  return L + mbc + g8 * bytesum64_swar(ww);
}

// The same on vector byte operations (wave-uniform inputs; the result goes back to a scalar
// register): varint terminator by mask + ffbl, widths by a 64-bit funnel and one SAD. mbc <= 4.
DEV uint32_t delta_blk_len_v(const uint32_t *win, int32_t win0, uint32_t pos, uint32_t mbc, uint32_t g8) {
  const uint32_t off = (uint32_t)((int32_t)pos - win0), a = off >> 2, sh = off & 3;
  uint32_t x0 = win[a], x1 = win[a + 1], x2 = win[a + 2];
  // keep the byte work on the vector unit: a uniform LDS load would otherwise be moved to
  // scalar registers word by word, and every VALU <-> SALU hand-off sits on the hop chain
  asm volatile("" : "+v"(x0), "+v"(x1), "+v"(x2));
  const uint32_t u0 = __builtin_amdgcn_alignbyte(x1, x0, sh), u1 = __builtin_amdgcn_alignbyte(x2, x1, sh);
  const uint32_t t = ~u0 & 0x80808080u;
  const uint32_t L = (uint32_t)(__builtin_ctz(t | 0x80000000u) >> 3) + 1;  // t == 0 -> 4: rejected below
  const uint32_t ww = (uint32_t)((((uint64_t)u1 << 32) | u0) >> (8 * L)) & (mbc >= 4 ? ~0u : ((1u << (8 * mbc)) - 1u));
  const uint32_t bl = __umul24(g8, __builtin_amdgcn_sad_u8(ww, 0u, 0u)) + L + mbc;
  const uint32_t ok = (uint32_t)(t != 0) & (uint32_t)(L + mbc <= 8);
  return sgpr(bl * ok);
}

// The same per lane (positions differ between lanes): 0 = not a fast block.
DEV uint32_t delta_blk_len_lane(const uint32_t *win, int32_t win0, uint32_t pos, uint32_t mbc, uint32_t g8) {
  const uint32_t off = (uint32_t)((int32_t)pos - win0), a = off >> 2, sh = off & 3;
  const uint32_t x0 = win[a], x1 = win[a + 1], x2 = win[a + 2];
  const uint32_t u0 = __builtin_amdgcn_alignbyte(x1, x0, sh), u1 = __builtin_amdgcn_alignbyte(x2, x1, sh);
  const uint32_t t = ~u0 & 0x80808080u;
  const uint32_t L = (uint32_t)(__builtin_ctz(t | 0x80000000u) >> 3) + 1;
  const uint32_t ww = (uint32_t)((((uint64_t)u1 << 32) | u0) >> (8 * L)) & (mbc >= 4 ? ~0u : ((1u << (8 * mbc)) - 1u));
  const uint32_t bl = __umul24(g8, __builtin_amdgcn_sad_u8(ww, 0u, 0u)) + L + mbc;
  return (t != 0 && L + mbc <= 8) ? bl : 0u;
}

// One DELTA_BINARY_PACKED stream to decode: an INT32/INT64 page's values section, or a
// lengths stream of a DELTA_LENGTH_BYTE_ARRAY / DELTA_BYTE_ARRAY page (validated on the host).
struct DeltaStream {
  const uint8_t *s;      // stream bytes
  uint32_t n;            // stream length
  uint32_t hdr;          // first miniblock header, relative to s
  int64_t first;         // first value (block header)
  int32_t count;         // valuesCount (block header)
  uint32_t mbc, mbvc;
  bool is64;
  uint8_t *out;          // value 0 of the output (int64 or int32 array)
  uint32_t chunk, page;  // error reporting: chunk index and data-page index within it
};

DEV DeltaStream page_stream(const BatchDev &b, const WorkItem &wi, const PageDesc &pd, const ChunkDesc &cd) {
  DeltaStream ds;
  ds.s = gp_u64<const uint8_t>(pd.data) + pd.val_off;
  ds.n = pd.val_len;
  ds.hdr = pd.delta_first_mb - pd.val_off;
  ds.first = pd.delta_first;
  ds.count = pd.delta_count;
  ds.mbc = pd.delta_mbc;
  ds.mbvc = pd.delta_mbvc;
  ds.is64 = pd.vkind == VK_DELTA64;
  ds.out = gp_u64<uint8_t>(cd.values) + b.page_vbase[wi.page] * (ds.is64 ? 8 : 4);
  ds.chunk = pd.chunk;
  ds.page = pd.page_in_chunk;
  return ds;
}

DEV void do_delta_page(const BatchDev &b, const DeltaStream &ds, uint32_t nn, DeltaPageLDS &L) {
  if (nn == 0) return;
  const uint8_t *s = ds.s;
  const uint32_t n = ds.n;
  const bool is64 = ds.is64;
  const uint32_t mbc = ds.mbc, mbvc = ds.mbvc, bs = mbc * mbvc, g8 = mbvc / 8, gpb = bs / 8;
  const uint32_t tid = threadIdx.x, lane = lane_id(), wv = tid >> 6;
  constexpr uint32_t NL = 256;  // threads that load a window
  const uint32_t lt = tid;
  uint32_t limit = nn;  // next() fails with io.EOF at positions >= the header's valuesCount
  bool final_eof = false;
  if ((uint32_t)max(ds.count, 0) < nn) { limit = (uint32_t)max(ds.count, 0); final_eof = true; }
  const uint32_t need = (uint32_t)(((uint64_t)limit + bs - 1) / bs);  // blocks holding deltas 0 .. limit-1
  uint64_t carry = (uint64_t)ds.first;
  uint32_t hdr = ds.hdr, blk = 0;
  const bool al16 = ((uintptr_t)ds.out & 15) == 0;  // 8 values of a group: 16-B aligned stores
  constexpr uint32_t kVec = (kDeltaWinLoad + 32 + 16 * NL - 1) / (16 * NL);
  uint4 pre[kVec];
  auto fetch = [&](int32_t w0) {
    const uint4 *src = (const uint4 *)(s + w0);
    const int64_t lim = (int64_t)n + 16 - w0;  // the page padding keeps 16 B past n readable (zeros)
#pragma unroll
    for (uint32_t j = 0; j < kVec; j++) {
      const uint32_t k = lt + j * NL;
      pre[j] = (int64_t)k * 16 < lim && k < (kDeltaWinLoad + 32) / 16 ? src[k] : make_uint4(0, 0, 0, 0);
    }
  };
  auto store = [&]() {
#pragma unroll
    for (uint32_t j = 0; j < kVec; j++) {
      const uint32_t k = lt + j * NL;
      if (k < (kDeltaWinLoad + 32) / 16) ((uint4 *)L.win)[k] = pre[j];
    }
  };
  PQ_STAMPS(st, b.dbg);
  st.begin();
  int32_t win0 = (int32_t)hdr - (int32_t)(((uintptr_t)(s + hdr)) & 15u);
  fetch(win0);
  store();
  if (tid == 0) L.stop = ~0ull;
  wg_barrier();
  st.lap(0);
  while (blk < need) {
    // ---- 1. walk (wave 0)
    if (wv == 0) {
      __builtin_amdgcn_s_setprio(3);
      st.lap(1);
      const int64_t lend = (int64_t)win0 + kDeltaWinLoad;
      const bool tail = (int64_t)n + 24 <= lend;  // the window holds the stream end (zeros past it)
      // a fast hop's block ends at or below lim: inside the stream, and the block plus the next
      // header are staged
      const uint32_t lim = tail ? n : (uint32_t)min((int64_t)n, lend - 24);
      const uint32_t kmax = min(kDeltaMaxBlk, need - blk);
      uint32_t p = sgpr(hdr), k = 0;
      for (;;) {
        // fast hops: position -> next position on vector byte ops (funnel shifts, SAD)
        while (mbc <= 4 && k < kmax) {
          const uint32_t bl = delta_blk_len_v(L.win, win0, p, mbc, g8);
          if (!bl || p + bl > lim) break;
          // stride speculation: lane j takes the block that starts j blocks on if the blocks between
          // have this block's length (writers with steady miniblock widths); lanes 0 .. m-1 whose
          // block has that length are true block starts by induction
          const uint64_t Pj = (uint64_t)p + (uint64_t)lane * bl;
          const uint32_t bj = lane == 0 ? bl : (Pj + bl <= lim ? delta_blk_len_lane(L.win, win0, (uint32_t)Pj, mbc, g8) : 0u);
          const uint64_t nb = ~__ballot(bj == bl);
          const uint32_t m = min(nb ? (uint32_t)__builtin_ctzll(nb) : 64u, kmax - k);
          if (lane < m) L.hpos[k + lane] = (uint32_t)Pj;
          k += m;
          p += m * bl;
        }
        // one block by the exact rules (or the end of the walk)
        if (k >= kmax) break;
        if (p >= n) {  // next() reads this block's header at EOF: the parse reports it
          if (lane == 0) L.hpos[k] = p;
          k++;
          break;
        }
        if (!tail && (int64_t)p + 24 > lend) break;
        int64_t md;
        uint64_t wdv;
        uint32_t hl;
        if (sgpr(delta_hdr_parse(L.win, (uint32_t)win0, s, n, p, is64, mbc, &md, &wdv, &hl))) {
          if (lane == 0) L.hpos[k] = p;  // header error: the parse reports it
          k++;
          break;
        }
        const uint32_t bl = sgpr(hl + g8 * bytesum64_swar(wdv));
        if (!tail && (int64_t)p + bl + 24 > lend && k > 0) break;  // block not staged whole
        if (lane == 0) L.hpos[k] = p;
        k++;
        if ((uint64_t)p + bl > n) break;  // the stream ends inside this block: the parse reports it
        p += bl;
      }
      if (lane == 0) { L.nb = k; L.next = p; }
      __builtin_amdgcn_s_setprio(0);
      st.lap(7);
      st.add(5, k);
    }
    wg_barrier();
    st.lap(1);
    const uint32_t nb = sgpr(L.nb);
    hdr = sgpr(L.next);
    const bool more = blk + nb < need && nb > 0;
    const int32_t nwin0 = (int32_t)hdr - (int32_t)(((uintptr_t)(s + hdr)) & 15u);
    if (more) fetch(nwin0);  // lands during the parse and the batches
    // ---- 3. parse: thread k re-reads block k's header exactly, finds its first unreadable group
    if (tid < nb) {
      const uint32_t p = L.hpos[tid], j = blk + tid;
      int64_t md = 0;
      uint64_t wdv = 0;
      uint32_t hl = 0;
      unsigned long long key = ~0ull;
      const uint32_t e = p >= n ? (uint32_t)PQ_ERR_EOF
                                : delta_hdr_parse(L.win, (uint32_t)win0, s, n, p, is64, mbc, &md, &wdv, &hl);
      if (e) {
        key = ((unsigned long long)j * bs << 4) | e;  // read by next() at the block's first position
      } else {
        uint64_t start = (uint64_t)p + hl;
        for (uint32_t m = 0; m < mbc; m++) {
          const uint32_t w = (uint32_t)(wdv >> (8 * m)) & 0xffu;
          const uint64_t mend = start + (uint64_t)g8 * w;
          if (w && mend > n) {  // io.ReadFull of group q (:137-141): EOF if no byte is left
            const uint32_t q = start >= n ? 0u : (uint32_t)((n - start) / w);
            const uint32_t ec = start + (uint64_t)q * w >= n ? PQ_ERR_EOF : PQ_ERR_UNEXPECTED_EOF;
            key = ((unsigned long long)((uint64_t)j * bs + m * mbvc + 8 * q) << 4) | ec;
            break;
          }
          start = mend;
        }
      }
      L.md[tid] = md;
      L.wd[tid] = wdv;
      L.ppos[tid] = p + hl;
      if (key != ~0ull) atomicMin(&L.stop, key);
    }
    wg_barrier();
    st.lap(6);
    const unsigned long long sk = sgpr64(L.stop);
    const uint64_t epos = sk >> 4;
    const uint32_t stop = (uint32_t)min((uint64_t)limit, epos);
    // ---- 4. batches of 256 groups
    const uint32_t ng = nb * gpb;
    uint32_t par = 0;
    for (uint32_t g0 = 0; g0 < ng; g0 += 256, par ^= 1) {
      const uint32_t g = g0 + tid;
      const uint32_t k = g / gpb, inb = (g - k * gpb) * 8;
      const uint32_t d0 = (blk + k) * bs + inb;
      const bool valid = g < ng && d0 < stop;
      uint64_t d[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      uint64_t sum = 0;
      if (valid && PQ_ABLATE(b, 1)) {  // diagnostic: no unpack
#pragma unroll
        for (int q = 0; q < 8; q++) d[q] = (uint64_t)L.md[k] + q;
        sum = d[0] * 8;
      } else if (valid) {
        const uint32_t m = inb / mbvc, o = inb - m * mbvc;
        const uint64_t wdv = L.wd[k];
        const uint32_t w = (uint32_t)(wdv >> (8 * m)) & 0xffu;
        const uint64_t below = m ? (wdv & ((1ull << (8 * m)) - 1ull)) : 0ull;
        const uint32_t goff = L.ppos[k] + g8 * bytesum64(below) + (o / 8) * w;
        delta_unpack8_lds(L.win, win0, goff, w, is64, L.md[k], d);
#pragma unroll
        for (int q = 0; q < 8; q++) sum += d[q];
      }
      st.lap(2);
      const uint64_t incl = wave_incl_scan64_dpp(sum);
      if (lane == 63) L.wsum[par][wv] = incl;
      wg_barrier();
      uint64_t before = 0, total = 0;
#pragma unroll
      for (uint32_t q = 0; q < 4; q++) {
        const uint64_t t = L.wsum[par][q];
        before += q < wv ? t : 0ull;
        total += t;
      }
      uint64_t run = carry + before + incl - sum;
      carry += total;
      st.lap(3);
      uint64_t *out = d;  // values in place of their deltas (registers)
#pragma unroll
      for (int q = 0; q < 8; q++) { const uint64_t t = d[q]; d[q] = run; run += t; }
      if (PQ_ABLATE(b, 0)) {  // diagnostic: no stores (kept live by an impossible condition)
        if (out[7] == 0x0123456789abcdefull && valid) ((uint64_t *)ds.out)[d0] = out[0];
      } else if (__ballot(valid && d0 + 8 <= stop) == ~0ull) {
        // the wave's 64 groups are 512 consecutive values: transpose through LDS so that every
        // store instruction writes 1 KiB contiguous (16 B per lane) instead of 64 B-strided pieces.
        // The output leaves in 2 KiB halves (int64: lanes 0-31, then lanes 32-63; int32: one half,
        // every lane). Piece e (16 B) of a half is held by lane e / vw as its piece e % vw; it sits
        // in LDS slot xsw(e): the piece index within the lane is XOR-swizzled with lane bits so that
        // the 16-B writes of 16 (int64) / 8 (int32) consecutive lanes cover all 64 banks (lanes
        // 64 B / 32 B apart would otherwise meet in the same banks, 4- / 2-way).
        uint4 *xw = L.xpose[wv];
        auto xsw = [&](uint32_t e) -> uint32_t {
          return is64 ? (e & ~3u) | ((e ^ (e >> 4)) & 3u) : (e & ~1u) | ((e ^ (e >> 4)) & 1u);
        };
        const uint32_t wd0 = rdlane(d0, 0);
        const uint32_t nhalf = is64 ? 2u : 1u;
        for (uint32_t h = 0; h < nhalf; h++) {
          if (is64) {
            if ((lane >> 5) == h) {
              const uint32_t l32 = lane & 31u;
#pragma unroll
              for (int q = 0; q < 4; q++)
                xw[xsw(l32 * 4 + q)] = make_uint4((uint32_t)out[2 * q], (uint32_t)(out[2 * q] >> 32),
                                                  (uint32_t)out[2 * q + 1], (uint32_t)(out[2 * q + 1] >> 32));
            }
          } else {
            xw[xsw(lane * 2)] = make_uint4((uint32_t)out[0], (uint32_t)out[1], (uint32_t)out[2], (uint32_t)out[3]);
            xw[xsw(lane * 2 + 1)] = make_uint4((uint32_t)out[4], (uint32_t)out[5], (uint32_t)out[6], (uint32_t)out[7]);
          }
          asm volatile("" ::: "memory");  // same wave: LDS executes its accesses in order
          uint8_t *dst0 = ds.out + (uint64_t)wd0 * (is64 ? 8 : 4) + 2048u * h;
          if (al16) {
            uint4 *dst = (uint4 *)dst0;
#pragma unroll
            for (uint32_t q = 0; q < 2; q++) cp_st16(&dst[q * 64 + lane], xw[xsw(q * 64 + lane)]);
          } else {  // 4-B aligned output: the same pieces, unaligned 16-B stores
#pragma unroll
            for (uint32_t q = 0; q < 2; q++) cp_st16_ua(dst0 + 16u * (q * 64 + lane), xw[xsw(q * 64 + lane)]);
          }
          asm volatile("" ::: "memory");  // this half's LDS reads precede the next half's writes
        }
      } else if (valid) {
        if (d0 + 8 <= stop && al16) {
          if (is64) {
            uint4 *o4 = (uint4 *)((uint64_t *)ds.out + d0);
#pragma unroll
            for (int q = 0; q < 4; q++)
              o4[q] = make_uint4((uint32_t)out[2 * q], (uint32_t)(out[2 * q] >> 32), (uint32_t)out[2 * q + 1],
                                 (uint32_t)(out[2 * q + 1] >> 32));
          } else {
            uint4 *o4 = (uint4 *)((uint32_t *)ds.out + d0);
            o4[0] = make_uint4((uint32_t)out[0], (uint32_t)out[1], (uint32_t)out[2], (uint32_t)out[3]);
            o4[1] = make_uint4((uint32_t)out[4], (uint32_t)out[5], (uint32_t)out[6], (uint32_t)out[7]);
          }
        } else {
#pragma unroll
          for (int q = 0; q < 8; q++) {
            if (d0 + q < stop) {
              if (is64) ((uint64_t *)ds.out)[d0 + q] = out[q];
              else ((uint32_t *)ds.out)[d0 + q] = (uint32_t)out[q];
            }
          }
        }
      }
      st.lap(4);
    }
    blk += nb;
    if (epos < limit) {  // the page fails at its first unreadable position
      if (tid == 0) report(b, ds.chunk, 1, ds.page, ST_VALUES, (uint32_t)epos, (uint32_t)(sk & 15));
      st.flush(8);
      return;
    }
    if (!more) break;
    // ---- 2'. the prefetched window replaces the current one (every read of it is behind
    // the last batch's barrier, or the parse barrier when there was no batch)
    win0 = nwin0;
    store();
    wg_barrier();
    st.lap(0);
  }
  st.flush(8);
  if (final_eof && tid == 0) report(b, ds.chunk, 1, ds.page, ST_VALUES, limit, PQ_ERR_EOF);
}

// Exact scalar restatement of deltaBitPackDecoder.next for pages whose miniblock
// value count is not a multiple of 8 (deltabp_decoder.go:113-174).
DEV void do_delta_slow(const BatchDev &b, const DeltaStream &ds, uint32_t nn) {
  if (threadIdx.x != 0 || nn == 0) return;
  const uint8_t *s = ds.s;
  const uint32_t n = ds.n;
  const bool is64 = ds.is64;
  const uint32_t mbc = ds.mbc, mbvc = ds.mbvc;
  uint32_t rpos = ds.hdr;
  int64_t md = 0;
  uint32_t hl, e = 0;
  // the miniblock widths are read in place from the stream (any miniblock count the reference
  // accepts): wpos = the current block's first width byte
  // init(): the first miniblock header was validated on the host; re-read it here
  if (!delta_hdr(s, s, n, rpos, is64, mbc, &md, nullptr, &hl, &e)) {
    report(b, ds.chunk, 0, 0, ST_VALUES, 0, e);
    return;
  }
  uint32_t wpos = rpos + hl - mbc;
  rpos += hl;
  uint32_t cur_mb = 0, cur_w = 0, mb_pos = 0;  // mb_pos: miniBlockPosition (bytes read in the miniblock)
  int64_t mbv[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t prev = (uint64_t)ds.first;
  const int32_t vcount = ds.count;
  for (uint32_t pos = 0; pos < nn; pos++) {
    if ((int32_t)pos >= vcount) { report(b, ds.chunk, 1, ds.page, ST_VALUES, pos, PQ_ERR_EOF); return; }
    if (pos % 8 == 0) {
      if (pos % mbvc == 0) {
        if (cur_mb >= mbc) {
          if (!delta_hdr(s, s, n, rpos, is64, mbc, &md, nullptr, &hl, &e)) {
            report(b, ds.chunk, 1, ds.page, ST_VALUES, pos, e);
            return;
          }
          wpos = rpos + hl - mbc;
          rpos += hl;
          cur_mb = 0;
        }
        cur_w = s[wpos + cur_mb];
        mb_pos = 0;
        cur_mb++;
      }
      if (cur_w > 0 && rpos >= n) { report(b, ds.chunk, 1, ds.page, ST_VALUES, pos, PQ_ERR_EOF); return; }
      if (rpos + cur_w > n) { report(b, ds.chunk, 1, ds.page, ST_VALUES, pos, PQ_ERR_UNEXPECTED_EOF); return; }
      for (int j = 0; j < 8; j++)
        mbv[j] = is64 ? (int64_t)bits64(s + rpos, (uint64_t)j * cur_w, cur_w)
                      : (int64_t)(int32_t)bits32(s + rpos, (uint64_t)j * cur_w, cur_w);
      rpos += cur_w;
      mb_pos += cur_w;
      // the padding skip after the last group (:149-164): it only moves the reader (nothing
      // follows an INT page), but a negative remainder — miniblocks of fewer than 8 values —
      // is "invalid stream"
      if ((int64_t)pos + 8 >= (int64_t)vcount && (int64_t)(mbvc / 8) * cur_w < (int64_t)mb_pos) {
        report(b, ds.chunk, 1, ds.page, ST_VALUES, pos, PQ_ERR_INVALID);
        return;
      }
    }
    uint64_t ret = prev;
    prev = prev + (uint64_t)mbv[pos % 8] + (uint64_t)md;
    if (!is64) prev = (uint64_t)(int64_t)(int32_t)(uint32_t)prev;
    if (is64) ((uint64_t *)ds.out)[pos] = ret;
    else ((uint32_t *)ds.out)[pos] = (uint32_t)ret;
  }
}

// PLAIN / BOOLEAN copies: no LDS, so their workgroups fit on a CU beside the DELTA pages'
// (39 KB of LDS each) and the level kernels' instead of queueing behind them.
__global__ void __launch_bounds__(256) k_values_copy(BatchDev b_in, const WorkItem *items) {
  const BatchDev b = global_view(b_in);
  const WorkItem wi = gp(items)[blockIdx.x];
  const PageDesc &pd = b.pages[wi.page];
  const ChunkDesc &cd = b.chunks[pd.chunk];
  const uint32_t nn = b.page_nn_v[wi.page];
  if (wi.kind == WI_PLAIN) do_plain<4>(b, wi, pd, cd, nn);  // (copy_shapes ubench: 4 pieces per lane, nt)
  else do_bool(b, wi, pd, cd, nn);
}

// DELTA_BINARY_PACKED work items (pages, tiles, the scalar path) in their own launch, followed in
// the speculative schedule by the PLAIN / BOOLEAN copies (the latency-bound pages are dispatched
// first and the bandwidth-bound copies fill the CUs around them): the kernel's registers and LDS
// are the DELTA decoder's, not the maximum over every work-item kind (dictionary tiles stay in
// k_values).
union DeltaLDS {
  DeltaTileLDS dtile;
  DeltaPageLDS dpage;
};
#ifndef PQ_DELTA_WPE
#define PQ_DELTA_WPE 5
#endif
DEV void values_delta(BatchDev b_in, const WorkItem *items, DeltaLDS &lds) {
  const BatchDev b = global_view(b_in);
  if (blockIdx.x == 0 && b.err_next)  // (DELTA-major decodes: the next decode's keys, on this stream)
    for (uint32_t c = threadIdx.x; c < b.nchunks; c += blockDim.x) gp(b.err_next)[c] = ~0ull;
  const WorkItem wi = items[blockIdx.x];
  const PageDesc &pd = b.pages[wi.page];
  const ChunkDesc &cd = b.chunks[pd.chunk];
  const uint32_t nn = b.page_nn_v[wi.page];
  switch (wi.kind) {
    case WI_DELTA: do_delta_slow(b, page_stream(b, wi, pd, cd), nn); break;
    case WI_DELTA_TILE: do_delta_tile(b, wi, pd, cd, nn, lds.dtile.scan, lds.dtile.stage); break;
    case WI_DELTA_PAGE: do_delta_page(b, page_stream(b, wi, pd, cd), nn, lds.dpage); break;
    case WI_PLAIN: do_plain<PQ_FUSED_COPY_U>(b, wi, pd, cd, nn); break;  // fused copies (registers to spare: more in flight)
    case WI_BOOL: do_bool(b, wi, pd, cd, nn); break;
  }
}
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(PQ_DELTA_WPE))) k_values_delta(BatchDev b_in, const WorkItem *items) {
  __shared__ DeltaLDS lds;
  values_delta(b_in, items, lds);
}

__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(5))) k_values(BatchDev b_in, const WorkItem *items) {
  const BatchDev b = global_view(b_in);
  __shared__ ValuesLDS lds;
  const WorkItem wi = items[blockIdx.x];
  const PageDesc &pd = b.pages[wi.page];
  const ChunkDesc &cd = b.chunks[pd.chunk];
  const uint32_t nn = b.page_nn_v[wi.page];
  switch (wi.kind) {
    case WI_PLAIN: do_plain(b, wi, pd, cd, nn); break;  // (only when PQ_COPY_FUSED=1 puts them here)
    case WI_BOOL: do_bool(b, wi, pd, cd, nn); break;
    case WI_DELTA: do_delta_slow(b, page_stream(b, wi, pd, cd), nn); break;
    case WI_DELTA_TILE: do_delta_tile(b, wi, pd, cd, nn, lds.dtile.scan, lds.dtile.stage); break;
    case WI_DELTA_PAGE: do_delta_page(b, page_stream(b, wi, pd, cd), nn, lds.dpage); break;
    case WI_DLENS: {  // a DELTA lengths stream of a DELTA_LENGTH / DELTA_BYTE_ARRAY page
      const BaDelta &bd = b.ba_delta[pd.ba_delta];
      const BaDeltaStream &st = bd.st[wi.v0];
      DeltaStream ds;
      ds.s = gp_u64<const uint8_t>(pd.data) + st.off;
      ds.n = st.len;
      ds.hdr = st.hdr;
      ds.first = st.first;
      ds.count = st.count;
      ds.mbc = st.mbc;
      ds.mbvc = st.mbvc;
      ds.is64 = false;
      ds.out = (uint8_t *)(gp_u64<int32_t>(bd.scratch) + (wi.v0 ? bd.cap : 0u));
      ds.chunk = pd.chunk;
      ds.page = pd.page_in_chunk;
      if (st.slow) do_delta_slow(b, ds, wi.v1);
      else do_delta_page(b, ds, wi.v1, lds.dpage);
      break;
    }
  }
}

// Dictionary tiles (WI_DICT) in a launch of their own: the registers and LDS are do_dict's alone
// (not the maximum over every work-item kind), so more tiles are resident per CU.
// (dictionary-only decodes: block 0 resets the next decode's error keys, err_next, on this stream)
DEV void reset_err_next(const BatchDev &b) {
  if (blockIdx.x == 0 && b.err_next)
    for (uint32_t c = threadIdx.x; c < b.nchunks; c += blockDim.x) gp(b.err_next)[c] = ~0ull;
}
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(PQ_DICT_WPE))) k_values_dict(BatchDev b_in, const WorkItem *items) {
  const BatchDev b = global_view(b_in);
  reset_err_next(b);
  __shared__ DictTileLDST<kDictRuns> lds;
  const WorkItem wi = items[blockIdx.x];
  const PageDesc &pd = b.pages[wi.page];
  do_dict(b, wi, pd, b.chunks[pd.chunk], b.page_nn_v[wi.page], lds);
}
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(PQ_DICT_WPE))) k_values_dict2(BatchDev b_in, const WorkItem *items) {
  const BatchDev b = global_view(b_in);
  reset_err_next(b);
  __shared__ DictTileLDST<kDictRuns> lds;
  const WorkItem wi = items[blockIdx.x];
  const PageDesc &pd = b.pages[wi.page];
  do_dict2(b, wi, pd, b.chunks[pd.chunk], b.page_nn_v[wi.page], lds);
}

// ---------------------------------------------------------------------------
// DELTA_LENGTH_BYTE_ARRAY / DELTA_BYTE_ARRAY values (type_bytearray.go:117-140, :216-240).
// The lengths streams were decoded into the page's scratch by WI_DLENS items (k_values);
// one workgroup per page turns them into value lengths (offsets[v+1], scanned later by the
// BYTE_ARRAY offsets kernels) and sources (ba_index), and finds the first error the
// reference's value loop meets:
//   value i >= len(lens)                      -> io.EOF            (next(), :118-120)
//   suffix length < 0                         -> invalid (Go: make() panics)
//   io.ReadFull of the suffix                 -> EOF / ErrUnexpectedEOF (:123-125)
//   DBA: prefix > length of value i-1         -> invalid (:227-230)
//   DBA: prefix < 0 and prefix + suffix < 0   -> invalid (Go: make() panics); a negative prefix
//        with a long enough suffix yields the suffix alone, as in the reference
// DELTA_BYTE_ARRAY values share bytes with their predecessors: value i = value(i-1)[:p_i] +
// suffix_i. Byte j < p_i of value i is byte j of the last earlier value whose suffix wrote it,
// so each value is rebuilt from the chain of previous-smaller-prefix values (a_1 = the last
// k < i with p_k < p_i, a_2 the same below a_1, ...: value a_t contributes [p_{a_t},
// p_{a_(t-1)}) from its suffix). The links come from pointer jumping over the page's values
// (k_ba_delta); k_dba_gather copies the pieces after the payload offsets are known.
// ---------------------------------------------------------------------------

__global__ void __launch_bounds__(256) k_ba_delta(BatchDev b_in) {
  const BatchDev b = global_view(b_in);
  __shared__ uint64_t wsum[4];
  __shared__ unsigned long long ekey;
  __shared__ uint32_t changed;
  const BaDelta &bd = b.ba_delta[blockIdx.x];
  const uint32_t pi = bd.page;
  const PageDesc &pd = b.pages[pi];
  const ChunkDesc &cd = b.chunks[pd.chunk];
  const bool dba = pd.vkind == VK_DBA;
  const uint32_t nn = b.page_nn_v[pi], cap = bd.cap, count = (uint32_t)max(bd.st[0].count, 0);
  const uint64_t vb = b.page_vbase[pi];
  int32_t *suf = gp_u64<int32_t>(bd.scratch), *pre = suf + cap, *anc = suf + 3 * (uint64_t)cap;
  uint32_t *soff = (uint32_t *)(suf + 2 * (uint64_t)cap);
  const uint8_t *pay = gp_u64<const uint8_t>(pd.data) + bd.pay_off;
  const uint64_t plen = bd.pay_len;
  int32_t *offs = gp_u64<int32_t>(cd.offsets);
  uint64_t *srcs = gp_u64<uint64_t>(cd.ba_index);
  const uint32_t tid = threadIdx.x;
  if (tid == 0) ekey = ~0ull;
  __syncthreads();
  const uint32_t nv = min(nn, cap);  // values with a decoded length
  constexpr uint32_t kPer = 8, kTile = 256 * kPer;
  // ---- pass 1: the first error in value order
  uint64_t carry = 0;
  for (uint32_t t0 = 0; t0 < nn; t0 += kTile) {
    const uint32_t i0 = t0 + tid * kPer;
    uint64_t mine = 0;
    for (uint32_t q = 0; q < kPer; q++) {
      const uint32_t i = i0 + q;
      if (i < nv) mine += (uint64_t)max(suf[i], 0);
    }
    uint64_t total;
    uint64_t off = carry + block_excl_scan64(mine, wsum, &total);
    carry += total;
    unsigned long long key = ~0ull;
    for (uint32_t q = 0; q < kPer && key == ~0ull; q++) {
      const uint32_t i = i0 + q;
      if (i >= nn) break;
      if (i >= count) { key = ((unsigned long long)i << 4) | PQ_ERR_EOF; break; }
      const int32_t sl = suf[i];
      if (sl < 0) key = ((unsigned long long)i << 4) | PQ_ERR_INVALID;
      else if (sl > 0 && off >= plen) key = ((unsigned long long)i << 4) | PQ_ERR_EOF;
      else if (off + (uint64_t)sl > plen) key = ((unsigned long long)i << 4) | PQ_ERR_UNEXPECTED_EOF;
      else if (dba) {
        const int64_t prev = i == 0 ? 0 : (int64_t)max(pre[i - 1], 0) + suf[i - 1];
        const int32_t p = pre[i];
        if (prev < p || (p < 0 && (int64_t)p + sl < 0)) key = ((unsigned long long)i << 4) | PQ_ERR_INVALID;
      }
      off += (uint64_t)max(sl, 0);
    }
    if (key != ~0ull) atomicMin(&ekey, key);
  }
  __syncthreads();
  const unsigned long long ek = ekey;
  const uint32_t stop = ek == ~0ull ? nn : (uint32_t)min((uint64_t)nn, (uint64_t)(ek >> 4));
  if (ek != ~0ull && tid == 0) report(b, pd.chunk, 1, pd.page_in_chunk, ST_VALUES, (uint32_t)(ek >> 4), (uint32_t)(ek & 15));
  // ---- pass 2: lengths and sources of the values before the error
  carry = 0;
  for (uint32_t t0 = 0; t0 < nn; t0 += kTile) {
    const uint32_t i0 = t0 + tid * kPer;
    uint64_t mine = 0;
    for (uint32_t q = 0; q < kPer; q++) {
      const uint32_t i = i0 + q;
      if (i < stop) mine += (uint64_t)suf[i];
    }
    uint64_t total;
    uint64_t off = carry + block_excl_scan64(mine, wsum, &total);
    carry += total;
    for (uint32_t q = 0; q < kPer; q++) {
      const uint32_t i = i0 + q;
      if (i >= nn) break;
      if (i < stop) {
        const int32_t sl = suf[i];
        const uint32_t len = dba ? (uint32_t)(max(pre[i], 0) + sl) : (uint32_t)sl;
        offs[vb + i + 1] = (int32_t)len;
        srcs[vb + i] = dba ? 0ull : (uint64_t)(pay + off);
        if (dba) soff[i] = (uint32_t)off;
        off += (uint64_t)sl;
      } else {
        offs[vb + i + 1] = 0;
        srcs[vb + i] = 0;
      }
    }
  }
  if (!dba) return;
  // ---- pass 3 (DBA): previous-smaller-prefix links by pointer jumping
  for (uint32_t i = tid; i < stop; i += blockDim.x) anc[i] = max(pre[i], 0) == 0 ? -1 : (int32_t)i - 1;
  for (;;) {
    __syncthreads();
    if (tid == 0) changed = 0;
    __syncthreads();
    uint32_t ch = 0;
    for (uint32_t i = tid; i < stop; i += blockDim.x) {
      const int32_t a = anc[i];
      if (a >= 0 && max(pre[a], 0) >= max(pre[i], 0)) { anc[i] = anc[a]; ch = 1; }
    }
    if (ch) changed = 1;
    __syncthreads();
    if (!changed) break;
  }
}

// DELTA_BYTE_ARRAY payload: one workgroup per page (chunks without a decode error).
__global__ void __launch_bounds__(256) k_dba_gather(BatchDev b_in) {
  const BatchDev b = global_view(b_in);
  const BaDelta &bd = b.ba_delta[blockIdx.x];
  const uint32_t pi = bd.page;
  const PageDesc &pd = b.pages[pi];
  if (pd.vkind != VK_DBA) return;
  const ChunkDesc &cd = b.chunks[pd.chunk];
  if (!cd.payload || ba_page_failed(b, pd)) return;
  const uint32_t nn = min(b.page_nn_v[pi], bd.cap), cap = bd.cap;
  const uint64_t vb = b.page_vbase[pi];
  const int32_t *pre = gp_u64<const int32_t>(bd.scratch) + cap, *anc = pre + 2 * (uint64_t)cap;
  const uint32_t *soff = (const uint32_t *)(pre + cap);
  const uint8_t *pay = gp_u64<const uint8_t>(pd.data) + bd.pay_off;
  const int32_t *offs = gp_u64<const int32_t>(cd.offsets);
  uint8_t *out = gp_u64<uint8_t>(cd.payload);
  for (uint32_t i = threadIdx.x; i < nn; i += blockDim.x) {
    const int32_t o0 = offs[vb + i], o1 = offs[vb + i + 1];
    uint8_t *dst = out + o0;
    const uint32_t p = (uint32_t)max(pre[i], 0), len = (uint32_t)(o1 - o0);
    const uint8_t *src = pay + soff[i];
    for (uint32_t k = p; k < len; k++) dst[k] = src[k - p];
    uint32_t hi = p;
    int32_t a = anc[i];
    while (hi > 0 && a >= 0) {
      const uint32_t lo = (uint32_t)max(pre[a], 0);
      const uint8_t *sa = pay + soff[a];
      for (uint32_t k = lo; k < hi; k++) dst[k] = sa[k - lo];
      hi = lo;
      a = anc[a];
    }
  }
}

// ---------------------------------------------------------------------------
// Record (list) offsets: list_offsets[r] = slot index of the r-th slot with
// rep == 0 (ColumnStore.get data_store.go:285-308: a new record starts when
// rl < maxR ... at rl == 0 for the top level). One workgroup per page.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_records(BatchDev b_in, const uint32_t *pages) {
  const BatchDev b = global_view(b_in);
  const uint32_t pi = pages[blockIdx.x];
  const PageDesc &pd = b.pages[pi];
  const ChunkDesc &cd = b.chunks[pd.chunk];
  const uint8_t *rep = gp_u64<const uint8_t>(cd.rep_levels) + pd.slot_base;
  int32_t *lo = gp_u64<int32_t>(cd.list_offsets);
  uint64_t rbase = b.page_rbase[pi];
  __shared__ uint32_t part[256];
  __shared__ uint64_t carry;
  if (threadIdx.x == 0) carry = 0;
  wg_barrier();
  for (uint32_t s0 = 0; s0 < pd.num_slots; s0 += 256 * 16) {
    uint32_t a = s0 + threadIdx.x * 16, e = min(a + 16, pd.num_slots);
    uint32_t c = 0;
    for (uint32_t s = a; s < e; s++) c += rep[s] == 0;
    part[threadIdx.x] = c;
    wg_barrier();
    for (uint32_t d = 1; d < 256; d <<= 1) {
      uint32_t x = threadIdx.x >= d ? part[threadIdx.x - d] : 0;
      wg_barrier();
      part[threadIdx.x] += x;
      wg_barrier();
    }
    uint64_t r = rbase + carry + part[threadIdx.x] - c;
    for (uint32_t s = a; s < e; s++)
      if (rep[s] == 0) lo[r++] = (int32_t)(pd.slot_base + s);
    wg_barrier();
    if (threadIdx.x == 255) carry += part[255];
    wg_barrier();
  }
  // last page of the chunk writes the terminating offset
  if (threadIdx.x == 0 && pd.page_in_chunk == cd.num_pages - 1) {
    uint64_t nrec = rbase + b.page_rec[pi];
    lo[nrec] = (int32_t)cd.num_slots;
  }
}

// ---------------------------------------------------------------------------
// k_snappy: a SNAPPY data page's raw block -> the page data, one wave per page
// (golang/snappy v0.0.1 decode_other.go / decode_amd64.s: any inconsistency is ErrCorrupt,
// which the reference reports as the page's readPages failure, compress.go:102-123).
//
// The element chain is walked 64 stream bytes at a time: every lane decodes the element that
// would start at its byte, the chain is followed lane to lane with readlane, then the chain's
// elements execute in order. Output goes through an LDS ring holding the most recent
// kSnappyRing page bytes (copy sources: both encoders keep offsets below 64 KiB, most below
// the ring) and is flushed to HBM in 16-B aligned pieces; copies reaching past the ring read
// the flushed output with L1-bypassing loads.
// ---------------------------------------------------------------------------
constexpr uint32_t kRingMask = kSnappyRing - 1;

struct SnappyOut {
  uint8_t *ring;      // LDS, 16-B aligned
  uint8_t *dst;       // page data (global, 16-B aligned)
  uint32_t flushed;   // page bytes [0, flushed) are in dst; a multiple of 16
  uint32_t lo, hi;    // the bytes of dst this page owns (direct output: [lead, lead + dlen); else all)
};

// Direct output (SnappyJob::lead): the page is written straight into a values array whose start
// need not be 16-B aligned; dst is rounded down and page byte P lives at dst + P, so the first
// and the last 16-B piece hold bytes of the neighbouring pages' values and are written bytewise.
DEV uint8_t *snappy_base(const SnappyJob &jb) { return gp_u64<uint8_t>(jb.dst) - (jb.lead ? jb.lead - 1 : 0u); }

DEV void snappy_flush(SnappyOut &o, uint32_t upto) {  // ring[flushed, upto) -> dst, upto % 16 == 0
  for (uint32_t x = o.flushed + lane_id() * 16; x < upto; x += 64 * 16) {
    const uint4 v = *(const uint4 *)(o.ring + (x & kRingMask));
    if (x >= o.lo && x + 16 <= o.hi) {
      *(uint4 *)(o.dst + x) = v;
    } else {
      const uint32_t vw[4] = {v.x, v.y, v.z, v.w};
      for (uint32_t i = 0; i < 16; i++)
        if (x + i >= o.lo && x + i < o.hi) o.dst[x + i] = (uint8_t)(vw[i >> 2] >> (8 * (i & 3)));
    }
  }
  o.flushed = upto;
}
// make room for page bytes [P, P + k) in the ring (k <= kSnappyRing - 16)
DEV void snappy_room(SnappyOut &o, uint32_t P, uint32_t k) {
  if (P + k - o.flushed > kSnappyRing) snappy_flush(o, P & ~15u);
}

// Global bytes S[0, len) -> page bytes [P, P + len), len <= kSnappyRing / 2. Whole ring words
// are assembled from two aligned dword loads (S's 4-B aligned floor is readable and the
// source is followed by zero padding); the partial words at either end go byte by byte.
DEV void snappy_put(SnappyOut &o, const uint8_t *S, uint32_t P, uint32_t len) {
  snappy_room(o, P, len);
  const uint32_t w1 = (P + len + 3) >> 2;
#pragma unroll 4
  for (uint32_t w = (P >> 2) + lane_id(); w < w1; w += 64) {
    const uint32_t lo = max(w * 4, P), hi = min(w * 4 + 4, P + len);
    if (hi - lo == 4) {
      const uint8_t *a = S + (lo - P);
      const uint32_t sh = (uint32_t)(uintptr_t)a & 3;
      const uint32_t *al = (const uint32_t *)(a - sh);
      *(uint32_t *)(o.ring + ((w * 4) & kRingMask)) = __builtin_amdgcn_alignbyte(al[1], al[0], sh);
    } else {
      for (uint32_t x = lo; x < hi; x++) o.ring[x & kRingMask] = S[x - P];
    }
  }
}

// A literal of `len` bytes (any length): the head goes through the ring up to a 16-B page
// boundary, the aligned body is copied global -> global by all kSnappyWaves waves of the
// workgroup (funnel16, 4 pieces of 16 B in flight per lane; pieces in the body's last
// kSnappyRing bytes also land in the ring, which must hold the most recent output for later
// copies), the tail goes through the ring again. Long literals dominate incompressible pages
// (one literal per 64 KiB encoder fragment).
#ifndef PQ_SNAPPY_WAVES
#define PQ_SNAPPY_WAVES 2
#endif
constexpr uint32_t kSnappyWaves = PQ_SNAPPY_WAVES;
constexpr uint32_t kSnappyDirect = 2048;  // bytes: shorter literals stay on the ring path
struct SnappyCmd {                         // LDS: wave 0 -> helper waves
  uint64_t src;                            // literal body source (global address)
  uint32_t P, pieces, ring_from, stop;
};

// Share of one long-literal body for wave `w` (all waves call it between two barriers).
// PQ_SNAPPY_ONELOAD: one load per 16-B piece (the funnel's second block is the next lane's first,
// taken by a lane shuffle as in copy_bytes_u; wave w's round covers 64 U consecutive pieces); 0: two
// loads per piece. cfg5 k_snappy 3.867 -> 3.834 ms; 8 pieces per lane 3.853 ms
// (profiles/r04_s19_probe_snappy_oneload.txt).
#ifndef PQ_SNAPPY_ONELOAD
#define PQ_SNAPPY_ONELOAD 1
#endif
#ifndef PQ_SNAPPY_U
#define PQ_SNAPPY_U 4
#endif
DEV void snappy_body(const SnappyCmd &c, uint8_t *ring, uint8_t *dst, uint32_t w) {
  const uint8_t *S = gp_u64<const uint8_t>(c.src);
  const uint32_t P = c.P, pieces = c.pieces, ring_from = c.ring_from;
  const uint32_t sa = (uint32_t)((uintptr_t)S & 15);
  const uint4 *sb = (const uint4 *)(S - sa);
  uint4 *d = (uint4 *)(dst + P);
  constexpr uint32_t NT = 64 * kSnappyWaves, U = 4;
  uint32_t i = w * 64 + lane_id();
  if (PQ_SNAPPY_ONELOAD) {
    const uint32_t lane = lane_id();
    const int nxt = (int)(((lane + 1) & 63u) * 4);
    auto shd = [nxt](uint32_t v) { return (uint32_t)__builtin_amdgcn_ds_bpermute(nxt, (int)v); };
    constexpr uint32_t U1 = PQ_SNAPPY_U;  // pieces per lane in flight
    uint32_t r0 = 0;
    for (; r0 + NT * U1 <= pieces; r0 += NT * U1) {
      const uint32_t j = r0 + w * 64 * U1 + lane;
      uint4 a[U1];
#pragma unroll
      for (uint32_t u = 0; u < U1; u++) a[u] = sb[j + 64 * u];
      uint4 e = make_uint4(0u, 0u, 0u, 0u);
      if (sa && lane == 63) e = sb[j + 64 * (U1 - 1) + 1];
#pragma unroll
      for (uint32_t u = 0; u < U1; u++) {
        uint4 v = a[u];
        if (sa) {
          const uint4 o = (lane == 0 && u + 1 < U1) ? a[u + 1] : a[u];  // what lane l - 1 takes from this lane
          uint4 nb = make_uint4(shd(o.x), shd(o.y), shd(o.z), shd(o.w));
          if (lane == 63 && u + 1 == U1) nb = e;
          v = funnel16(a[u], nb, sa);
        }
        d[j + 64 * u] = v;
        if (j + 64 * u >= ring_from) *(uint4 *)(ring + ((P + (j + 64 * u) * 16) & kRingMask)) = v;
      }
    }
    i = r0 + w * 64 + lane;
  }
  for (; i + (U - 1) * NT < pieces; i += U * NT) {
    uint4 a[U], e[U];
#pragma unroll
    for (uint32_t u = 0; u < U; u++) { a[u] = sb[i + u * NT]; e[u] = sb[i + u * NT + 1]; }
#pragma unroll
    for (uint32_t u = 0; u < U; u++) {
      const uint4 v = funnel16(a[u], e[u], sa);
      d[i + u * NT] = v;
      if (i + u * NT >= ring_from) *(uint4 *)(ring + ((P + (i + u * NT) * 16) & kRingMask)) = v;
    }
  }
  for (; i < pieces; i += NT) {
    const uint4 v = funnel16(sb[i], sb[i + 1], sa);
    d[i] = v;
    if (i >= ring_from) *(uint4 *)(ring + ((P + i * 16) & kRingMask)) = v;
  }
  __builtin_amdgcn_s_waitcnt(0);  // stores done before the barrier: wave 0 may read them back
}

DEV void snappy_literal(SnappyOut &o, SnappyCmd &cmd, const uint8_t *S, uint32_t P, uint32_t len) {
  if (len >= kSnappyDirect) {
    const uint32_t h = (16 - (P & 15)) & 15;
    if (h) snappy_put(o, S, P, h);
    S += h; P += h; len -= h;
    snappy_flush(o, P);  // ring [flushed, P) -> page, so the page is complete below P
    const uint32_t body = len & ~15u;
    if (lane_id() == 0) {
      cmd.src = (uint64_t)(uintptr_t)S;
      cmd.P = P;
      cmd.pieces = body >> 4;
      cmd.ring_from = body > kSnappyRing ? (body - kSnappyRing) >> 4 : 0;  // first piece kept
      cmd.stop = 0;
    }
    wg_barrier();
    snappy_body(cmd, o.ring, o.dst, 0);
    wg_barrier();
    o.flushed = P + body;
    S += body; P += body; len -= body;
  }
  for (uint32_t k = 0; k < len; k += kSnappyRing / 2)
    snappy_put(o, S + k, P + k, min(len - k, kSnappyRing / 2));
}

// Page bytes [P - off, ...) -> [P, P + len), len <= 64, 1 <= off <= P (overlap repeats the
// pattern: byte i comes from P - off + i % off).
DEV void snappy_copy(SnappyOut &o, uint32_t P, uint32_t off, uint32_t len) {
  snappy_room(o, P, 64);
  const uint32_t i = lane_id();
  uint32_t m = i;
  if (off < len) m = i - off * (uint32_t)(((float)i + 0.5f) * __builtin_amdgcn_rcpf((float)off));
  const uint32_t q = P - off + m;
  uint32_t v = 0;
  if (off <= kSnappyRing) {
    if (i < len) v = o.ring[q & kRingMask];
  } else {  // flushed long ago (flushed >= P + 64 - kSnappyRing > q): read HBM, bypassing L1
    __builtin_amdgcn_s_waitcnt(0);
    if (i < len) {
      const uint32_t *wp = (const uint32_t *)(o.dst + (q & ~3u));
      v = __hip_atomic_load(wp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >> (8 * (q & 3));
    }
  }
  if (i < len) o.ring[(P + i) & kRingMask] = (uint8_t)v;
}

// The elements of one 64-byte stream window whose output lies within reach, executed together
// (`batch`: chain lanes; every literal among them lies inside the window, so its bytes are in the
// lanes' `w` registers). Output byte j of the batch (page position P + j) gets a state: a resolved
// byte (literals; copy sources before the batch, read from the ring or, past it, from HBM) or a
// pointer to the earlier batch byte it copies (copy source inside the batch; an overlapping copy
// points into its own output). Pointer jumping resolves every byte in O(log T) rounds, then the
// batch lands in the ring at once — instead of executing one element after another, each waiting
// for the previous one's LDS writes. Returns false on a corrupt element (bounds as
// decode_other.go:63-95: literal past the stream or the decoded length, copy offset 0 or past
// the output start, copy past the decoded length).
constexpr uint32_t kSnappyBatch = 1536;  // bytes: elements starting in 64 stream bytes write at most
                                         // 22 copies x 64 = 1408 (2-byte-offset copies, 3 bytes each)
constexpr uint32_t kSnRes = 0x8000u;     // state: resolved | byte, else the batch index it copies
DEV bool snappy_batch(SnappyOut &o, uint16_t *st, uint64_t batch, uint32_t P, uint32_t op, uint32_t dlen, uint32_t n,
                      uint32_t pos, uint32_t t, uint32_t hdr, uint32_t val, uint32_t clen, uint32_t w, uint32_t &T) {
  const uint32_t lane = lane_id();
  const bool in = (batch >> lane) & 1ull;
  const uint32_t len = in ? (t == 0 ? val + 1 : clen) : 0u;  // literals in a batch are short: no overflow
  const uint32_t O = wave_excl_scan(len);
  T = sgpr(rdlane(O + len, 63));
  const uint32_t rel = lane + hdr;  // literal start within the window
  bool bad = false;
  if (in) {
    if (pos + rel > n) bad = true;
    else if (t == 0) bad = (uint64_t)len > (uint64_t)(dlen - (op + O)) || pos + rel + len > n;
    else bad = val == 0 || op + O < val || len > dlen - (op + O);
  }
  if (__ballot(bad) || T > kSnappyBatch) return false;
  snappy_room(o, P, T);
  // Byte-parallel fill: batch byte j belongs to the last lane e whose output start O_e <= j (a
  // lane outside the batch has the start of the next batch lane, so that lane is a batch lane),
  // found by binary search over the lanes' O (ds_bpermute); 4 bytes per lane in flight.
  const uint32_t pk2 = t | (rel << 2);
  bool far = false;  // some copy source is older than the ring
  auto bperm = [](uint32_t l, uint32_t v) {
    return (uint32_t)__builtin_amdgcn_ds_bpermute((int)((l & 63) * 4), (int)v);
  };
  for (uint32_t j0 = 0; j0 < T; j0 += 256) {
    uint32_t e[4];
#pragma unroll
    for (uint32_t k = 0; k < 4; k++) e[k] = 0;
#pragma unroll
    for (uint32_t step = 32; step; step >>= 1) {
#pragma unroll
      for (uint32_t k = 0; k < 4; k++) {
        const uint32_t c = e[k] + step;
        const uint32_t oc = bperm(c, O);
        if (c < 64 && oc <= j0 + 64 * k + lane) e[k] = c;
      }
    }
    uint32_t Oe[4], ve[4], pe[4], lb[4];
#pragma unroll
    for (uint32_t k = 0; k < 4; k++) {
      Oe[k] = bperm(e[k], O);
      ve[k] = bperm(e[k], val);
      pe[k] = bperm(e[k], pk2);
    }
#pragma unroll
    for (uint32_t k = 0; k < 4; k++) {
      const uint32_t j = j0 + 64 * k + lane;
      lb[k] = bperm((pe[k] >> 2) + (j - Oe[k]), w) & 0xffu;  // the literal's byte (literals lie in the window)
    }
#pragma unroll
    for (uint32_t k = 0; k < 4; k++) {
      const uint32_t j = j0 + 64 * k + lane;
      if (j < T) {
        uint32_t sv;
        if ((pe[k] & 3) == 0) {
          sv = kSnRes | lb[k];
        } else if (j >= ve[k]) {
          // an earlier byte of this batch; inside an overlapping copy (offset < its length) byte j
          // repeats byte Oe - d + (j - Oe) mod d, before the element: one hop instead of a chain
          const uint32_t d = ve[k], r = j - Oe[k];
          sv = (r >= d && Oe[k] >= d) ? Oe[k] - d + r % d : j - d;
        } else if (ve[k] + T <= kSnappyRing) {
          sv = kSnRes | o.ring[(P + j - ve[k]) & kRingMask];  // page byte before the batch, in the ring
        } else {
          sv = kSnRes;
          far = true;  // resolved below from HBM
        }
        st[j] = (uint16_t)sv;
      }
    }
  }
  if (__ballot(far)) {  // sources flushed long ago: read the page in HBM (L1 bypassed)
    __builtin_amdgcn_s_waitcnt(0);
    for (uint32_t i = 0;; i++) {
      const bool act = in && t != 0 && i < len && O + i < val && val + T > kSnappyRing;
      if (!__ballot(act)) break;
      if (act) {
        const uint32_t q = P + O + i - val;
        const uint32_t *wp = (const uint32_t *)(o.dst + (q & ~3u));
        st[O + i] = (uint16_t)(kSnRes | ((__hip_atomic_load(wp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >> (8 * (q & 3))) & 0xffu));
      }
    }
  }
  wave_lds_sync();
  for (;;) {  // pointer jumping: 8 bytes per lane per group, their LDS reads issued together
    bool open = false;
    for (uint32_t j0 = 0; j0 < T; j0 += 512) {
      uint32_t v[8], u[8];
#pragma unroll
      for (uint32_t k = 0; k < 8; k++) {
        const uint32_t j = j0 + 64 * k + lane;
        v[k] = j < T ? st[j] : kSnRes;
      }
#pragma unroll
      for (uint32_t k = 0; k < 8; k++) u[k] = (v[k] & kSnRes) ? v[k] : st[v[k]];
#pragma unroll
      for (uint32_t k = 0; k < 8; k++) {
        if (!(v[k] & kSnRes)) {
          st[j0 + 64 * k + lane] = (uint16_t)u[k];
          open |= !(u[k] & kSnRes);
        }
      }
    }
    wave_lds_sync();
    if (!__ballot(open)) break;
  }
  for (uint32_t j = lane; j < T; j += 64) o.ring[(P + j) & kRingMask] = (uint8_t)st[j];
  wave_lds_sync();
  return true;
}

// Wave 0 walks and executes the element chain; waves 1.. wait at barriers and join in the
// body copies of long literals (snappy_literal) until wave 0 raises `stop`.
DEV void snappy_page(const BatchDev &b, const SnappyJob &jb, uint8_t *ring, SnappyCmd &cmd, uint16_t *st) {
  const uint8_t *src = gp_u64<const uint8_t>(jb.src);
  const uint32_t n = sgpr(jb.src_len), raw = sgpr(jb.raw_len), dlen = sgpr(jb.dlen);
  const uint32_t lane = lane_id();
  // direct output: the page starts `lead` bytes into its aligned base (there is no raw prefix)
  const uint32_t direct = sgpr(jb.lead), base = direct ? direct - 1 : raw;
  SnappyOut o{ring, snappy_base(jb), 0, direct ? base : 0u, direct ? base + dlen : 0xffffffffu};
  for (uint32_t k = 0; k < raw; k += kSnappyRing / 2)  // V2: the uncompressed level sections first
    snappy_put(o, gp_u64<const uint8_t>(jb.raw) + k, k, min(raw - k, kSnappyRing / 2));
  uint32_t pos = 0, op = 0;  // stream position, decoded bytes
  bool bad = false;
  // The element stream is held in registers, 512 bytes at a time: lane k of W0 / W1 holds the
  // dword at aligned-stream offset wb + 4k / wb + 256 + 4k (aligned stream = src rounded down
  // to 4 B). W1 is loaded one window ahead, so the walk does not wait on HBM every 64 bytes.
  const uint32_t sa0 = (uint32_t)((uintptr_t)src & 3);
  const uint32_t *srcw = (const uint32_t *)(src - sa0);
  // bytes past the block read as zero whatever follows it (a staged block is followed by zero
  // padding; a resident one, page index, by the next page): the partial last dword is masked
  const uint32_t wlim = n + sa0;
  auto ldw = [&](uint32_t at) -> uint32_t {  // the dword at aligned offset at + 4 * lane
    const uint32_t k = at + 4 * lane;
    if (k >= wlim) return 0u;
    const uint32_t w = srcw[k >> 2];
    return k + 4 <= wlim ? w : w & ((1u << (8 * (wlim - k))) - 1u);
  };
  uint32_t wb = 0, W0 = ldw(0), W1 = ldw(256);
  PQ_STAMPS(sp, b.dbg);
  sp.begin();
  while (pos < n) {
    // the element that would start at pos + lane: tag, header bytes, literal length - 1 or
    // copy offset, copy length (decode_other.go:20-96)
    const uint32_t ap = pos + sa0;
    if (ap - wb >= 256) {
      if (ap - wb < 512) {
        W0 = W1; wb += 256; W1 = ldw(wb + 256);
      } else {  // jumped past a long literal
        wb = ap & ~3u; W0 = ldw(wb); W1 = ldw(wb + 256);
      }
    }
    const uint32_t off = ap - wb, r = off + lane, q = r >> 2, sh = r & 3;
    uint32_t d0 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(q * 4), (int)W0);
    uint32_t d1 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(q * 4 + 4), (int)W0);
    if (off >= 256 - 68) {  // some lane reads W1 (uniform)
      const uint32_t e0 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(q * 4), (int)W1);
      const uint32_t e1 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(q * 4 + 4), (int)W1);
      if (q >= 64) d0 = e0;
      if (q + 1 >= 64) d1 = e1;
    }
    const uint32_t w = __builtin_amdgcn_alignbyte(d1, d0, sh), b4 = (d1 >> (8 * sh)) & 0xff;
    const uint32_t tag = w & 0xff, x = tag >> 2, t = tag & 3;
    uint32_t hdr, val, clen = 0;
    if (t == 0) {
      hdr = x < 60 ? 1 : x - 58;
      val = x < 60 ? x : x == 60 ? (w >> 8) & 0xff : x == 61 ? (w >> 8) & 0xffff : x == 62 ? (w >> 8) & 0xffffff
                                                                                          : (w >> 8) | (b4 << 24);
    } else if (t == 1) {
      hdr = 2; clen = 4 + (x & 7); val = ((tag & 0xe0) << 3) | ((w >> 8) & 0xff);
    } else if (t == 2) {
      hdr = 3; clen = 1 + x; val = (w >> 8) & 0xffff;
    } else {
      hdr = 5; clen = 1 + x; val = (w >> 8) | (b4 << 24);
    }
    // stream bytes of the element (saturated: a literal that long fails its bounds check)
    const uint32_t esz = t == 0 ? (uint32_t)min<uint64_t>((uint64_t)hdr + val + 1, 0x7fffffffu) : hdr;
    const uint32_t pk = t | (hdr << 2) | (clen << 5);  // one readlane per element for type, header, length
    uint64_t chain = 0;
    uint32_t cur = 0;
    sp.lap(0);
    while (cur < 64 && pos + cur < n) {
      chain |= 1ull << cur;
      cur += (uint32_t)__builtin_amdgcn_readlane((int)esz, (int)cur);
    }
    sp.lap(1);
    sp.count(4);
    sp.add(5, __popcll(chain));
    // runs of short elements execute as batches; a literal reaching past the window (its bytes
    // are not in the registers) executes on its own, with the long-literal copy when it is long
    const bool lng = t == 0 && lane + hdr + (uint64_t)val + 1 > 64;
    const uint64_t longs = __ballot(lng) & chain;
    while (chain && !bad) {
      const uint64_t upto = longs & chain;
      const uint32_t fl = upto ? (uint32_t)__builtin_ctzll(upto) : 64u;
      const uint64_t batch = fl < 64 ? chain & ((1ull << fl) - 1ull) : chain;
      if (batch) {
        uint32_t T;
        if (!snappy_batch(o, st, batch, base + op, op, dlen, n, pos, t, hdr, val, clen, w, T)) { bad = true; break; }
        op += T;
        sp.lap(2);
        sp.add(6, T);
        chain &= ~batch;
      }
      if (fl < 64) {
        const uint32_t e = fl;
        chain &= chain - 1;  // fl is now the lowest element
        const uint32_t epk = (uint32_t)__builtin_amdgcn_readlane((int)pk, (int)e);
        const uint32_t eh = (epk >> 2) & 7;
        const uint32_t ev = (uint32_t)__builtin_amdgcn_readlane((int)val, (int)e);
        const uint32_t s = pos + e + eh;
        if (s > n) { bad = true; break; }
        const uint64_t len = (uint64_t)ev + 1;
        if (len > dlen - op || len > n - s) { bad = true; break; }
        snappy_literal(o, cmd, src + s, base + op, (uint32_t)len);
        op += (uint32_t)len;
        sp.lap(3);
      }
    }
    if (bad) break;
    pos += cur;
  }
  sp.lap(7);
  sp.flush(48);
  if (bad || op != dlen) {
    if (lane == 0) report(b, jb.chunk, 0, jb.page_in_chunk, ST_DECOMP, 0, PQ_ERR_DECOMPRESS);
    return;
  }
  // last piece: zeros past the page end, then the 64 B zero pad every page section carries (direct
  // output: the bytes past the end belong to the next page's values and are not written)
  const uint32_t end = base + dlen, end16 = (end + 15) & ~15u;
  snappy_room(o, end, 16);
  if (end + lane < end16) o.ring[(end + lane) & kRingMask] = 0;
  snappy_flush(o, end16);
  if (!direct && lane < 4) *(uint4 *)(o.dst + end16 + lane * 16) = uint4{0, 0, 0, 0};
}

__global__ void __launch_bounds__(64 * kSnappyWaves) k_snappy(BatchDev b_in, const SnappyJob *jobs) {
  const BatchDev b = global_view(b_in);
  __shared__ __attribute__((aligned(16))) uint8_t ring[kSnappyRing];
  __shared__ SnappyCmd cmd;
  __shared__ uint16_t st[kSnappyBatch];  // batch byte states (snappy_batch)
  const SnappyJob &jb = gp(jobs)[blockIdx.x];
  const uint32_t w = threadIdx.x / 64;
  if (w == 0) {
    snappy_page(b, jb, ring, cmd, st);
    if (lane_id() == 0) cmd.stop = 1;
    wg_barrier();
  } else {
    for (;;) {  // one round per long literal; exits when wave 0 is done (every path sets stop)
      wg_barrier();
      if (cmd.stop) break;
      snappy_body(cmd, ring, snappy_base(jb), w);
      wg_barrier();
    }
  }
}

// ---------------------------------------------------------------------------
// Launchers
// ---------------------------------------------------------------------------
hipError_t launch_snappy(const BatchDev &b, const SnappyJob *jobs, uint32_t njobs, hipStream_t s) {
  if (!njobs) return hipSuccess;
  hipLaunchKernelGGL(k_snappy, dim3(njobs), dim3(64 * kSnappyWaves), 0, s, b, jobs);
  return hipGetLastError();
}
hipError_t launch_levels(const BatchDev &b, const LaunchLists &l, hipStream_t s, hipStream_t s2) {
  if (!s2) s2 = s;
  if (l.n_level_pages_bw1) {
    // default: verified segment speculation (k_levels_seg); PQ_LV_SEG=0: the list-ranking workgroup
    // kernel; PQ_LV_WAVE=1: the lane-to-lane wave walk (both slower: DESIGN.md §5)
    const char *lw = getenv("PQ_LV_WAVE");
    if (lw && atoi(lw) == 1) {
      hipLaunchKernelGGL(k_levels_bw1w, dim3(l.n_level_pages_bw1), dim3(64), 0, s, b, l.level_pages_bw1);
    } else {
      const uint32_t nseg = l.n_level_pages_seg, nrest = l.n_level_pages_bw1 - nseg;
      const char *sg = getenv("PQ_SEG_GRID");  // (probe) wavefronts of k_levels_seg; 0: one per page
      const uint32_t want = sg && atoi(sg) > 0 ? (uint32_t)atoi(sg) : (l.seg_grid ? l.seg_grid : nseg);
      const uint32_t grid = want < nseg ? want : nseg;
      if (nseg) hipLaunchKernelGGL(k_levels_seg, dim3(grid), dim3(64), sizeof(LevelSegLDS), s, b, l.level_pages_bw1, nseg);
      if (nrest) hipLaunchKernelGGL(k_levels_bw1, dim3(nrest), dim3(kLvThreads), 0, s, b, l.level_pages_bw1 + nseg);
    }
  }
  if (l.n_level_pages) {
    const char *lw = getenv("PQ_LV_WAVE");
    if (lw && atoi(lw) == 1) {
      hipLaunchKernelGGL(k_levels_w, dim3(l.n_level_pages), dim3(64), 0, s, b, l.level_pages);
    } else {  // host order: streams that fit k_levels_segw's stage, repetition streams for k_levels_hyb,
              // then the list-ranking kernel
      const uint32_t nseg = l.n_level_units_seg, nhyb = l.n_level_units_hyb, nrest = l.n_level_pages - nseg - nhyb;
      if (nseg) hipLaunchKernelGGL(k_levels_segw, dim3(nseg), dim3(kSgwLanes), 0, s, b, l.level_pages);
      if (nhyb) hipLaunchKernelGGL(k_levels_hyb, dim3(nhyb), dim3(256), 0, s2, b, l.level_pages + nseg);
      if (nrest) hipLaunchKernelGGL(k_levels, dim3(nrest), dim3(kLvThreads), 0, s2, b, l.level_pages + nseg + nhyb);
    }
  }
  return hipGetLastError();
}
hipError_t launch_level_fill(const BatchDev &b, const LaunchLists &l, hipStream_t s) {
  if (l.n_lf_list)
    hipLaunchKernelGGL(k_level_fill, dim3(l.n_lf_list), dim3(kLvThreads), 0, s, b, l.lv_tiles, l.lf_list);
  return hipGetLastError();
}
hipError_t launch_bases(const BatchDev &b, const LaunchLists &l, hipStream_t s) {
  if (!l.n_base_chunks) return hipSuccess;
  hipLaunchKernelGGL(k_bases, dim3(l.n_base_chunks), dim3(256), 0, s, b, l.base_chunks);
  return hipGetLastError();
}
hipError_t launch_scan_runs(const BatchDev &b, const LaunchLists &l, hipStream_t s) {
  if (!l.n_scan_pages) return hipSuccess;
  hipLaunchKernelGGL(k_scan_runs, dim3(l.n_scan_pages), dim3(256), 0, s, b, l.scan_pages);
  return hipGetLastError();
}
hipError_t launch_scan_slots(const BatchDev &b, const LaunchLists &l, hipStream_t s) {
  const uint32_t n = l.n_scan_pages + l.n_slot_chunks * l.slot_grid_x;
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_scan_slots, dim3(n), dim3(256), 0, s, b, l.scan_pages, l.n_scan_pages, l.slot_chunks, l.slot_grid_x);
  return hipGetLastError();
}
hipError_t launch_values(const BatchDev &b, const LaunchLists &l, hipStream_t s) {
  if (!l.n_items) return hipSuccess;
  hipLaunchKernelGGL(k_values, dim3(l.n_items), dim3(256), 0, s, b, l.items);
  return hipGetLastError();
}
hipError_t launch_values_dict(const BatchDev &b, const WorkItem *items, uint32_t n_pair, uint32_t n, hipStream_t s) {
  if (n_pair) hipLaunchKernelGGL(k_values_dict2, dim3(n_pair), dim3(256), 0, s, b, items);  // grouped items first
  if (n > n_pair) hipLaunchKernelGGL(k_values_dict, dim3(n - n_pair), dim3(256), 0, s, b, items + n_pair);
  return hipGetLastError();
}
hipError_t launch_values_delta(const BatchDev &b, const WorkItem *items, uint32_t n, hipStream_t s) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_values_delta, dim3(n), dim3(256), 0, s, b, items);
  return hipGetLastError();
}
hipError_t launch_values_copy(const BatchDev &b, const LaunchLists &l, hipStream_t s) {
  if (!l.n_copy_items) return hipSuccess;
  hipLaunchKernelGGL(k_values_copy, dim3(l.n_copy_items), dim3(256), 0, s, b, l.copy_items);
  return hipGetLastError();
}
hipError_t launch_delta_prep(const BatchDev &b, const LaunchLists &l, hipStream_t s) {
  if (!l.n_delta_pages) return hipSuccess;
  hipLaunchKernelGGL(k_delta_walk, dim3(l.n_delta_pages), dim3(256), 0, s, b, l.delta_pages);
  return hipGetLastError();
}
hipError_t launch_ba_delta(const BatchDev &b, const LaunchLists &l, hipStream_t s) {
  if (!l.n_ba_delta) return hipSuccess;
  hipLaunchKernelGGL(k_ba_delta, dim3(l.n_ba_delta), dim3(256), 0, s, b);
  return hipGetLastError();
}
hipError_t launch_dba_gather(const BatchDev &b, const LaunchLists &l, hipStream_t s) {
  if (!l.n_ba_delta) return hipSuccess;
  hipLaunchKernelGGL(k_dba_gather, dim3(l.n_ba_delta), dim3(256), 0, s, b);
  return hipGetLastError();
}
hipError_t launch_records(const BatchDev &b, const LaunchLists &l, hipStream_t s) {
  if (!l.n_rec_pages) return hipSuccess;
  hipLaunchKernelGGL(k_records, dim3(l.n_rec_pages), dim3(256), 0, s, b, l.rec_pages);
  return hipGetLastError();
}

}  // namespace pq
