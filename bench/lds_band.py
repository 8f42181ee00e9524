#!/usr/bin/env python3
"""LDS bank-conflict model of the banded LeNet-5 forward (csrc/kernels/lenet_band.hip,
lenet_band_fwd_k): every LDS access pattern of one tile with its average cycles per lane
group (1.0 = conflict-free) and its issue count per tile, for the strides on the command
line or the kernel's defaults.  Bank rules as bench/lds_bwd.py (MI355X_MICROARCH.md §LDS);
b32 / ds_read2_b32: one 64-lane group, bank (a/4) % 64.

    python bench/lds_band.py [XIS=900 XPL=448 PIS=1584 PPL=792 PRW=112 PSK=8 ...] [--search]

The kernel's layout (PSK = 0, two 8-byte pool1 stores per pixel) models 34 % conflict cycles
(PMC: 31 %).  Round 4 tried PSK = 8 with one 16-byte store per pixel (conv1_store16): it
models 1.0 for the pool1 stores and the conv2 B reads (15 % overall) but measured 4 us slower
(profiles/r4/lenet_band/skew_ab.txt: the extra swaps land on the critical conv1 role).
"""
import sys

from lds_bwd import cycles

DEF = dict(XIS=900, XPL=448, XRW=32, PIS=1584, PPL=792, PRW=112, PSK=0, XSK=0)


def pib(S, i):
    """pool1 image base (elements): odd images skewed by PSK"""
    return i * S["PIS"] + (i & 1) * S["PSK"]


def xib(S, i):
    return i * S["XIS"] + (i & 1) * S["XSK"]


def b32(addrs):
    banks = {}
    for a in addrs:
        if a is None:
            continue
        banks.setdefault((a // 4) % 64, set()).add(a // 4)
    return max(len(v) for v in banks.values())


def conv1_b(S, u=3, yp0=2, p=1):
    """B fragment: 4 dwords from element xlane + yp0 XRW + 4u + p XRW (two ds_read2_b32)."""
    tot = 0
    for dw in range(4):
        out = []
        for l in range(64):
            col, h = l & 31, l >> 5
            img, half, xq = (col >> 1) & 7, col >> 4, col & 1
            e = xib(S, img) + h * S["XPL"] + (7 * half - 1) * S["XRW"] + 2 * xq + yp0 * S["XRW"] + 4 * u + p * S["XRW"]
            out.append(2 * e + 4 * dw + 4 * S["XRW"])
        tot += b32(out)
    return tot / 4


def conv1_store(S, u=3, yp0=2):
    out = []
    for l in range(64):
        col, h = l & 31, l >> 5
        img, half, xq = (col >> 1) & 7, col >> 4, col & 1
        row_even = S["PPL"] + 3 * S["PRW"] if half else 0
        row_odd = 4 * S["PRW"] if half else S["PPL"]
        off = (row_odd if yp0 & 1 else row_even) + (yp0 >> 1) * S["PRW"] + 16 * u
        out.append(2 * (pib(S, img) + 8 * xq + 4 * h + off))
    return cycles(out, 8, "w64")


def conv1_store16(S, u=3, yp0=2):
    """the pixel's 8 channels gathered into the h = 0 lane (permlane32 swap), one b128 store"""
    out = []
    for l in range(64):
        col, h = l & 31, l >> 5
        img, half, xq = (col >> 1) & 7, col >> 4, col & 1
        if h:
            out.append(None)
            continue
        row_even = S["PPL"] + 3 * S["PRW"] if half else 0
        row_odd = 4 * S["PRW"] if half else S["PPL"]
        off = (row_odd if yp0 & 1 else row_even) + (yp0 >> 1) * S["PRW"] + 16 * u
        out.append(2 * (pib(S, img) + 8 * xq + off))
    return cycles(out, 16, "w128")


def conv2_b(S, w2v=1, r=2, q=1):
    out = []
    for l in range(64):
        col, h = l & 31, l >> 5
        slot, im2 = (col >> 2) & 3, (col >> 4) | ((col & 3) << 1)
        f = min(4 * w2v + slot, 24)
        y2p, x2p = f // 5, f % 5
        e = pib(S, im2) + y2p * S["PRW"] + (2 * x2p + h) * 8 + (r & 1) * S["PPL"] + (r >> 1) * S["PRW"] + 16 * q
        out.append(2 * e)
    return cycles(out, 16, "b128")


def copy_out(S, wave=1, i=0):
    out = []
    for l in range(64):
        t = 64 * wave + l
        cp = (t + 192) & 255
        if cp >= 196:
            out.append(None)
            continue
        e = ((cp // 14) & 1) * S["PPL"] + ((cp // 14) >> 1) * S["PRW"] + (cp % 14) * 8 + pib(S, i)
        out.append(2 * e)
    return cycles(out, 16, "b128")


def xfill(S, wave=1, i=2):
    tot = 0
    for dw in range(2):
        out = []
        for l in range(64):
            t = 64 * wave + l
            r = (t & 31) + 32 * i
            if r >= 196:
                out.append(None)
                continue
            y, k = r // 7, r % 7
            e = xib(S, t >> 5) + 2 + (y & 1) * S["XPL"] + (y >> 1) * S["XRW"] + 4 * k
            out.append(2 * e + 4 * dw)
        tot += b32(out)
    return tot / 2


def avg(f, S, **grid):
    import itertools
    keys = list(grid)
    vals = [f(S, **dict(zip(keys, c))) for c in itertools.product(*grid.values())]
    return sum(vals) / len(vals)


def report(S):
    # issues per tile (per block): conv1 49 units x 3 k-steps x 2 read2, 49 stores; conv2
    # 7 units x 6 rows x 3 b128; copy-out 4 waves x 8 b128; fill 4 waves x 7 x write2
    rows = [("conv1 B (read2_b32 x2)", avg(conv1_b, S, u=range(7), yp0=range(7), p=range(3)), 49 * 3 * 2),
            ("conv1 pool1 store (w64)", avg(conv1_store, S, u=range(7), yp0=range(7)), 49),
            ("conv2 B (b128)", avg(conv2_b, S, w2v=range(4), r=range(6), q=range(3)), 7 * 6 * 3),
            ("copy-out (b128)", avg(copy_out, S, wave=range(4), i=range(8)), 4 * 8),
            ("input fill (write2_b32)", avg(xfill, S, wave=range(4), i=range(7)), 4 * 7)]
    tot_c = sum(c * n for _, c, n in rows)
    tot_n = sum(n for _, c, n in rows)
    for name, c, n in rows:
        print(f"{name:28s} {c:5.2f} cycles/group  x{n}")
    print(f"{'weighted':28s} {tot_c / tot_n:5.2f}  (conflict share {(1 - tot_n / tot_c) * 100:.0f} %)")
    return tot_c / tot_n


def main():
    S = dict(DEF)
    search = False
    for a in sys.argv[1:]:
        if a == "--search":
            search = True
        else:
            k, v = a.split("=")
            S[k] = int(v)
    report(S)
    if search:
        best = []
        import io
        import contextlib
        for pis in range(S["PPL"] * 2, S["PPL"] * 2 + 64, 4):
            for ppl in range(7 * S["PRW"], 7 * S["PRW"] + 64, 4):
                if pis < 2 * ppl:
                    continue
                T = dict(S, PIS=pis, PPL=ppl)
                with contextlib.redirect_stdout(io.StringIO()):
                    w = report(T)
                best.append((w, pis, ppl))
        best.sort()
        print("best (weighted, PIS, PPL):", best[:8])


if __name__ == "__main__":
    main()
