#!/usr/bin/env python3
"""LDS bank-conflict model of the fused LeNet-5 backward kernel (csrc/kernels/lenet_bwd.hip).

Bank rules (MI355X_MICROARCH.md §LDS): a wave64 access is serviced per lane group, one
LDS cycle per group when conflict-free; extra distinct dwords on one bank add cycles.
  ds_read_b128       4 x 16 lanes (odd groups), bank (a/4) % 64
  ds_read_b64(_tr)   2 x 32 lanes,              bank (a/4) % 64
  ds_write_b64       4 x 16 contiguous lanes,   bank (a/4) % 32
  ds_write_b128      8 x 8 contiguous lanes,    bank (a/4) % 32
Prints the average cycles per group (1.0 = conflict-free) of every access pattern for
the strides given on the command line / the defaults the kernel uses.

    python bench/lds_bwd.py [NAME=value ...]
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


DEF = dict(DY2_IMG=3872, DY2_RS=384, P1_IMG=3808, P1_RS=272, D_IMG=3920, D_RS=280, X_IMG=2592, X_RS=80)
# conv2 weight-gradient tiles: (first tap, second-tap step): one pixel apart (+1) or one
# row apart (+5; tap 29 = discarded rows)
C2_TILES = [(0, 1), (2, 1), (5, 1), (7, 1), (10, 1), (12, 1), (15, 1), (17, 1), (20, 1), (22, 1),
            (4, 5), (14, 5), (24, 5)]


def dgrad_b(S, dy=1, p=2, v=2):
    out = []
    for l in range(64):
        i, g = l & 15, l >> 4
        img, rr = i >> 1, i & 1
        y = 2 * p + rr - dy
        x = 2 * v + (g >> 1)
        if 0 <= y <= 9:
            out.append(img * S["DY2_IMG"] + y * S["DY2_RS"] + x * 32 + 16 * (g & 1))
        else:
            out.append(10 ** 6 + x * 32 + 16 * (g & 1))   # the shared zero row
    return cycles(out, 16, "b128")


def dgrad_w(S, p=2, u=3):
    out = []
    for l in range(64):
        i, g = l & 15, l >> 4
        img, rr = i >> 1, i & 1
        xq = 2 * u + (g >> 1)
        out.append(img * S["D_IMG"] + (2 * p + rr) * S["D_RS"] + xq * 16 + 8 * (g & 1))
    return cycles(out, 8, "w64")


def c2w(S, s, rho, t):
    """(A pool1 tr read of M-tile t, B dY2 tr read) of k-step s (dY2 row s // 3, pixels
    4 (s % 3) .. + 3), read rho."""
    a, b = [], []
    y, x0 = s // 3, 4 * (s % 3)
    for l in range(64):
        g, q, p = l >> 4, (l >> 2) & 3, l & 3
        img, sub = kitem(g, rho, q)
        x = x0 + sub
        tap0, step = C2_TILES[t]
        tap = tap0 + (p >> 1) * step
        a.append(img * S["P1_IMG"] + (y + tap // 5) * S["P1_RS"] + (x + tap % 5) * 16 + 8 * (p & 1))
        b.append(img * S["DY2_IMG"] + y * S["DY2_RS"] + x * 32 + 8 * p)
    return cycles(a, 8, "tr"), cycles(b, 8, "tr")


def c1w(S, sig, s, rho, t=0):
    """(A input tr read of M-tile t, B dP1 / code tr read) of k-step s (window row s // 2,
    windows 4 (s % 2) .. + 3 of parity set sig)."""
    a, b = [], []
    yp, xi0 = s // 2, 4 * (s % 2)
    for l in range(64):
        g, q, p = l >> 4, (l >> 2) & 3, l & 3
        img, sub = kitem(g, rho, q)
        xi = xi0 + sub
        xp = 2 * xi + sig
        a.append(img * S["X_IMG"] + (2 * yp + 2 * t + (p >> 1)) * S["X_RS"] + (4 * xi + 4 * (p & 1) + 4 * sig) * 2)
        b.append(img * S["D_IMG"] + yp * S["D_RS"] + xp * 16 + 8 * (p & 1))
    return cycles(a, 8, "tr"), cycles(b, 8, "tr")


def stores(S, rotate=True):
    """Staging stores per tile: dY2 unpool (threads < 400: pooled pixel x 8 channels, 4
    window positions d; `rotate`: the d of instruction i is rotated per lane), pool1 and code
    windows (wave pair per image, lane r -> window r / r + 128), input quads."""
    r = {}
    tot = n = 0
    for w in range(7):
        for i in range(4):
            addrs = []
            for l in range(64):
                t = 64 * w + l
                if t >= 400:
                    addrs.append(None)
                    continue
                im, rr = t // 50, t % 50
                pw, hf = rr >> 1, rr & 1
                yp, xp = pw // 5, pw % 5
                d = (i ^ ((xp >> 1) & 1)) if rotate else i
                addrs.append(im * S["DY2_IMG"] + (2 * yp + (d >> 1)) * S["DY2_RS"] + (2 * xp + (d & 1)) * 32 + 16 * hf)
            tot += cycles(addrs, 16, "w128")
            n += 1
    r["dY2_w128"] = tot / n
    for name, rs, size, kind in (("P1_w128", S["P1_RS"], 16, "w128"), ("CD_w64x2", S["D_RS"], 8, "w64")):
        tot = n = 0
        for wp in range(2):
            for ch in range(2):
                addrs = []
                for l in range(64):
                    q = l + 64 * wp + 128 * ch
                    if q >= 196:
                        addrs.append(None)
                        continue
                    addrs.append((q // 14) * rs + (q % 14) * 16)
                tot += cycles(addrs, size, kind)
                n += 1
        r[name] = tot / n
    tot = n = 0
    for wp in range(2):
        for ch in range(2):
            addrs = []
            for l in range(64):
                q = l + 64 * wp + 128 * ch
                addrs.append(None if q >= 196 else (q // 7 + 2) * S["X_RS"] + (4 * (q % 7) + 4) * 2)
            tot += cycles(addrs, 8, "w64")
            n += 1
    r["X_w64"] = tot / n
    return r


def report(S):
    r = {}
    r["dgrad_B_b128"] = sum(dgrad_b(S, dy, p, v) for dy in range(5) for p in range(7) for v in range(5)) / 175
    r["dgrad_W_w64"] = sum(dgrad_w(S, p, u) for p in range(7) for u in range(7)) / 49
    ca = cb = 0
    n = 0
    for s in range(30):
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
        for s in range(28):
            for rho in range(2):
                for t in range(3):
                    x, y = c1w(S, sig, s, rho, t)
                    ca += x
                    cb += y
                    n += 1
    r["c1w_A_tr"] = ca / n
    r["c1w_B_tr"] = cb / n
    r.update(stores(S))
    return r


def main():
    S = dict(DEF)
    for a in sys.argv[1:]:
        if "=" in a:
            k, v = a.split("=")
            S[k] = int(v)
    for k, v in report(S).items():
        print(f"{k:14s} {v:.3f}")


if __name__ == "__main__":
    main()
