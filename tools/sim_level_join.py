"""Offline measurement behind k_levels_seg's speculative join: on cfg2's pyarrow
definition-level streams (bit width 1), how far does a run-header walk started at an arbitrary byte
go before it lands on a position of the true chain? A well-formed fast run moves the walk by its
length if that is at most `cap` bytes, anything else by one byte. Second table: k_levels_seg's lanes
(64 segments per page, each lane's walk from `margin` bytes before its segment with hops capped at
`cap` bytes): the share of lanes whose first position at or past their segment start is not the true
chain's, i.e. that verification sends to the exact re-walk. CPU only.

  python tools/sim_level_join.py [pages] [stride]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "parquet-go-1_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def streams(rows=1 << 20):
    import pqgpu
    import workloads as W
    data, _ = W.gen_cfg2(rows=rows, rg_rows=rows)
    f = pqgpu.File(data)
    out = []
    for c in range(f.num_columns):
        m = f.chunk_meta(0, c)
        off, end = m.data_page_offset, m.data_page_offset + m.total_compressed_size
        while off < end:
            h, n = pqgpu.parse_page_header(data[off:off + 4096])
            body = off + n
            dl, rl = h.data_page_v2[4], h.data_page_v2[5]
            out.append(np.frombuffer(data[body + rl: body + rl + dl], np.uint8))
            off = body + h.compressed_page_size
    return out


def hop(s, p, cap):
    """Next position after a fast bit-width-1 run at p, or -1 (not fast, or longer than cap)."""
    n, h, L = len(s), 0, 0
    for k in range(4):
        if p + k >= n:
            return -1
        b = int(s[p + k])
        h |= (b & 0x7f) << (7 * k)
        if b < 0x80:
            L = k + 1
            break
    else:
        return -1
    cnt = h >> 1
    if cnt == 0:
        return -1
    if h & 1:
        adv = L + cnt
    else:
        if p + L >= n or s[p + L] > 1:
            return -1
        adv = L + 1
    return -1 if p + adv > n or adv > cap else p + adv


def main():
    npages = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    stride = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    for cap in (72, 1 << 30):
        dist = []
        for s in streams()[:npages]:
            n, p, true = len(s), 0, np.zeros(len(s) + 1, bool)
            while 0 <= p < n:
                true[p] = True
                p = hop(s, p, 1 << 30)
            for st in range(0, n - 600, stride):
                p = st
                while p < n and not true[p]:
                    q = hop(s, p, cap)
                    p = p + 1 if q < 0 else q
                dist.append(p - st)
        d = np.array(dist)
        print(f"cap {cap}: {len(d)} starts; not joined within 64 / 128 / 256 bytes: "
              f"{(d > 64).mean():.4%} / {(d > 128).mean():.4%} / {(d > 256).mean():.4%}")
    ss = streams()[:npages]
    for margin, cap in ((128, 72), (48, 16), (48, 8), (64, 16), (32, 16)):
        lanes = fails = hops = 0
        for s in ss:
            n, p, true = len(s), 0, []
            while 0 <= p < n:
                true.append(p)
                p = hop(s, p, 1 << 30)
            S = max((n + 63) // 64, 16)
            for lane in range(1, 64):
                lo = lane * S
                if lo >= n:
                    break
                lanes += 1
                p = 0 if lo <= margin else lo - margin
                while p < lo:
                    q = hop(s, p, cap)
                    p = p + 1 if q < 0 else q
                    hops += 1
                fails += p != next((t for t in true if t >= lo), n)
        print(f"margin {margin} cap {cap}: {lanes} lanes, {fails / lanes:.3%} fail verification, "
              f"{hops / lanes:.1f} speculative hops per lane")


if __name__ == "__main__":
    main()
