#!/usr/bin/env python3
"""LDS bank-conflict model of the fused LeNet-5 backward kernel (csrc/kernels/lenet_bwd.hip).

Bank rules (MI355X_MICROARCH.md §LDS): a wave64 access is serviced per lane group, one
LDS cycle per group when conflict-free; extra distinct dwords on one bank add cycles.
  ds_read_b128       4 x 16 lanes (odd groups), bank (a/4) % 64
  ds_read_b64(_tr)   2 x 32 lanes,              bank (a/4) % 64
  ds_write_b64       4 x 16 contiguous lanes,   bank (a/4) % 32
  ds_write_b128      8 x 8 contiguous lanes,    bank (a/4) % 32
Prints the average cycles per group (1.0 = conflict-free) of every access pattern for
the strides given on the command line / the defaults the kernel uses, and searches the
image strides.

    python bench/lds_bwd.py [--search]
"""
import itertools
import sys

B128_GROUPS = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
               list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32)),
               list(range(32, 36)) + list(range(44, 48)) + list(range(52, 60)),
               list(range(36, 44)) + list(range(48, 52)) + list(range(60, 64))]


def cycles(addrs, nbytes, kind):
    """addrs: 64 byte addresses (None = lane inactive)."""
    if kind == "b128":
        groups, mod = B128_GROUPS, 64
    elif kind in ("b64", "tr"):
        groups, mod = [list(range(0, 32)), list(range(32, 64))], 64
    elif kind == "w64":
        groups, mod = [list(range(16 * i, 16 * i + 16)) for i in range(4)], 32
    elif kind == "w128":
        groups, mod = [list(range(8 * i, 8 * i + 8)) for i in range(8)], 32
    else:
        raise ValueError(kind)
    tot = 0
    for gl in groups:
        banks = {}
        for l in gl:
            a = addrs[l]
            if a is None:
                continue
            for dw in range(nbytes // 4):
                d = a // 4 + dw
                banks.setdefault(d % mod, set()).add(d)
        tot += max((len(v) for v in banks.values()), default=0)
    return tot / len(groups)


def kitem(g, rho, q):
    """(image, pixel / window offset) of MFMA K row 8g + 4rho + q inside a 32-item k-step:
    items are enumerated image-fastest, so the 32 lanes of one transposed read (fixed g >> 1
    and rho) cover the 8 images of one pixel."""
    return 4 * (g & 1) + q, 2 * (g >> 1) + rho


DEF = dict(DY2_IMG=4640, DY2_RS=384, P1_IMG=3168, DP1_IMG=3152, X_IMG=2592, X_RS=80)
# conv2 weight-gradient tiles: tap pairs (25 = the bias row, a broadcast ONES cell)
C2_TAPS = [(0, 1), (2, 3), (5, 6), (7, 8), (10, 11), (12, 13), (4, 9),
           (15, 16), (17, 18), (14, 19), (20, 21), (22, 23), (24, 25)]


def dgrad_b(S, dy=1, p=2, v=2):
    out = []
    for l in range(64):
        i, g = l & 15, l >> 4
        img, rr = i >> 1, i & 1
        y = 2 * p + rr - dy
        x = 2 * v + (g >> 1)
        out.append(img * S["DY2_IMG"] + (y + 1) * S["DY2_RS"] + x * 32 + 16 * (g & 1))
    return cycles(out, 16, "b128")


def dgrad_w(S, p=2, u=3):
    out = []
    for l in range(64):
        i, g = l & 15, l >> 4
        img, rr = i >> 1, i & 1
        xq = 2 * u + (g >> 1)
        out.append(img * S["DP1_IMG"] + ((2 * p + rr) * 14 + xq) * 16 + 8 * (g & 1))
    return cycles(out, 8, "w64")


def c2w(S, s, rho, t):
    """(A pool1 tr read of M-tile t, B dY2 tr read) of k-step s, read rho."""
    a, b = [], []
    for l in range(64):
        g, q, p = l >> 4, (l >> 2) & 3, l & 3
        img, sub = kitem(g, rho, q)
        pix = 4 * s + sub
        y, x = pix // 10, pix % 10
        tap = C2_TAPS[t][p >> 1]
        if tap == 25:
            a.append(100000 + 8 * (p & 1))     # ONES cell
        else:
            a.append(img * S["P1_IMG"] + ((y + tap // 5) * 14 + x + tap % 5) * 16 + 8 * (p & 1))
        b.append(img * S["DY2_IMG"] + (y + 1) * S["DY2_RS"] + x * 32 + 8 * p)
    return cycles(a, 8, "tr"), cycles(b, 8, "tr")


def c1w(S, sig, s, rho, t=0):
    a, b = [], []
    for l in range(64):
        g, q, p = l >> 4, (l >> 2) & 3, l & 3
        img, sub = kitem(g, rho, q)
        tw = min(4 * s + sub, 97)
        yp, xi = tw // 7, tw % 7
        xp = 2 * xi + sig
        a.append(img * S["X_IMG"] + (2 * yp + 2 * t + (p >> 1)) * S["X_RS"] + (4 * xi + 4 * (p & 1) + 4 * sig) * 2)
        b.append(img * S["DP1_IMG"] + (yp * 14 + xp) * 16 + 8 * (p & 1))
    return cycles(a, 8, "tr"), cycles(b, 8, "tr")


def report(S):
    r = {}
    r["dgrad_B_b128"] = sum(dgrad_b(S, dy, p, v) for dy in range(5) for p in range(1, 6) for v in range(5)) / 125
    r["dgrad_W_w64"] = sum(dgrad_w(S, p, u) for p in range(7) for u in range(7)) / 49
    ca = cb = 0
    n = 0
    for s in range(25):
        for rho in range(2):
            for t in range(13):
                x, y = c2w(S, s, rho, t)
                ca += x
                cb += y
                n += 1
    r["c2w_A_tr"] = ca / n
    r["c2w_B_tr"] = cb / n
    ca = cb = 0
    n = 0
    for sig in range(2):
        for s in range(25):
            for rho in range(2):
                for t in range(3):
                    x, y = c1w(S, sig, s, rho, t)
                    ca += x
                    cb += y
                    n += 1
    r["c1w_A_tr"] = ca / n
    r["c1w_B_tr"] = cb / n
    return r


def main():
    S = dict(DEF)
    for a in sys.argv[1:]:
        if "=" in a:
            k, v = a.split("=")
            S[k] = int(v)
    if "--search" in sys.argv:
        best = {}
        for name, keys, cands in [
                ("dY2", ["DY2_IMG"], [4608 + 16 * i for i in range(0, 32)]),
                ("p1", ["P1_IMG"], [3136 + 16 * i for i in range(0, 32)]),
                ("X", ["X_IMG", "X_RS"], [(xi, xr) for xr in (72, 80, 88, 96, 104) for xi in range(32 * xr, 32 * xr + 512, 16)]),
                ]:
            res = []
            for c in cands:
                T = dict(S)
                if len(keys) == 1:
                    T[keys[0]] = c
                else:
                    T.update(dict(zip(keys, c)))
                rr = report(T)
                key = {"dY2": rr["dgrad_B_b128"] + rr["c2w_B_tr"], "p1": rr["c2w_A_tr"],
                       "X": rr["c1w_A_tr"]}[name]
                res.append((key, c))
            res.sort()
            print(name, res[:5])
        return
    for k, v in report(S).items():
        print(f"{k:14s} {v:.3f}")


if __name__ == "__main__":
    main()
