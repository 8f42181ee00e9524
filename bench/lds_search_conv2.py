#!/usr/bin/env python3
"""Offline search for a conflict-free LDS layout of the LeNet conv2 forward A reads
(convpool_fwd_k<Geo<8,16,5,0,14,14>>: ds_read_b128, fragment rows = 4 pool windows x 4
positions, lane group g reads tap 4s+g).  Reports mean LDS-array cycles per read
(ideal 4) for linear row strides, per-row rotations / XOR swizzles, and x / y parity
splits of the 14x14x8 image.  Result (profiles/r2/lenet/head_s5/lds_layout_search.md):
the current linear WS = 24 (6.08) is already the best of every family tried."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from lds_sim import cycles  # noqa: E402

CIN, PW, NPIX, KS, KE = 8, 5, 100, 5, 200


def evaluate(L):
    tot = n = 0
    for fm in range(7):
        for s in range(7):
            addrs = []
            for lane in range(64):
                g, li = divmod(lane, 16)
                r = min(fm * 16 + li, NPIX - 1)
                w, d = r >> 2, r & 3
                ph, pw = divmod(w, PW)
                y, x = 2 * ph + (d >> 1), 2 * pw + (d & 1)
                k0 = 32 * s + 8 * g
                kh, kw = divmod(k0 // CIN, KS) if k0 < KE else (0, 0)
                addrs.append(16 * L(y + kh, x + kw))
            tot += cycles("b128", addrs)
            n += 1
    return tot / n


def bijective(f):
    return len({f(y, x) for y in range(14) for x in range(14)}) == 196


def main():
    res = []
    for WS in range(14, 41):
        res.append((evaluate(lambda y, x: y * WS + x), "linear", WS))
        for r in range(1, 16):
            res.append((evaluate(lambda y, x, r=r: y * WS + ((x + r * y) % WS)), "rotate", WS, r))
        for H in range(7, 17):
            f = lambda y, x, H=H: y * WS + (x % 2) * H + x // 2  # noqa: E731
            if bijective(f):
                res.append((evaluate(f), "x-parity", WS, H))
    res.sort()
    for r in res[:8]:
        print(r)


if __name__ == "__main__":
    main()
