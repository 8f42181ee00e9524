#!/usr/bin/env python3
"""LDS bank-conflict model of the reference-CNN conv1 weight gradient
(csrc/kernels/refc1_wgrad.hip): the consumers' transposed A (input) and B (dP1 / codes)
reads of one k-step for every (parity set, channel group, A row tile), cycles per 32-lane
half (1.0 = conflict-free), for the strides on the command line or the kernel's; with
--search, the smallest conflict-free strides.  Bank rules: bench/lds_bwd.py.

    python bench/lds_refc1.py [X_RS=96 X_IMG=3192 D_RS=1040 D_IMG=14560] [--search]
"""
import sys

from lds_bwd import cycles

DEF = dict(X_RS=96, X_IMG=3192, D_RS=1040, D_IMG=14560)


def lane_item(l):
    gg, q, p = l >> 4, (l >> 2) & 3, l & 3
    return gg, q >> 1, q & 1, p >> 1, p & 1, 4 * (gg >> 1) + (gg & 1)   # gg, yr, img, hA, pc, xi


def a_read(S, sig, t):
    tot = 0
    for rho in (0, 1):
        out = []
        for l in range(64):
            gg, yr, img, hA, pc, xi = lane_item(l)
            out.append(img * S["X_IMG"] + (2 * yr + hA) * S["X_RS"] + (4 * xi + 4 * pc + 4 * sig) * 2 + 16 * rho
                       + 2 * t * S["X_RS"])
        tot += cycles(out, 8, "tr")
    return tot / 2


def b_read(S, sig, cg):
    tot = 0
    for rho in (0, 1):
        out = []
        for l in range(64):
            gg, yr, img, hA, pc, xi = lane_item(l)
            out.append(img * S["D_IMG"] + yr * S["D_RS"] + (2 * xi + sig) * 64 + 16 * cg + 8 * pc + 256 * rho)
        tot += cycles(out, 8, "tr")
    return tot / 2


def report(S):
    a = sum(a_read(S, s, t) for s in (0, 1) for t in range(3)) / 6
    b = sum(b_read(S, s, c) for s in (0, 1) for c in range(4)) / 8
    return a, b


def main():
    S = dict(DEF)
    search = "--search" in sys.argv
    for arg in sys.argv[1:]:
        if "=" in arg:
            k, v = arg.split("=")
            S[k] = int(v)
    a, b = report(S)
    print(f"A (input) reads {a:.2f}, B (dP1 / codes) reads {b:.2f} cycles per half  {S}")
    if search:
        for xr in range(80, 112, 8):
            for xi in range(32 * xr, 32 * xr + 256, 8):
                if report(dict(S, X_RS=xr, X_IMG=xi))[0] == 1.0:
                    print("A conflict-free:", xr, xi)
                    break
        for dr in range(1024, 1152, 16):
            for di in range(14 * dr, 14 * dr + 512, 16):
                if report(dict(S, D_RS=dr, D_IMG=di))[1] == 1.0:
                    print("B conflict-free:", dr, di)
                    break


if __name__ == "__main__":
    main()
