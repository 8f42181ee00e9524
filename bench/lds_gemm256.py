#!/usr/bin/env python3
"""Bank model of gemm256.hip's LDS images (CPU only; tests/test_lds_layouts.py runs it).

The LDS-DMA staging writes each 1 KB wave-instruction lane-linearly, so the bank swizzle of
the two operand images is an XOR on the 16-byte chunk index chosen per row (applied to the
global SOURCE chunk, undone on the read).  This searches every XOR-of-row-bits swizzle for
the one that makes the fragment reads conflict-free, with the gfx950 lane-group tables
(MI355X_MICROARCH.md §LDS):

  K-contiguous image  [256 rows][64 k] (128-byte rows), ds_read_b128: lane l reads row
      r0 + (l & 15), chunk 4 kh + (l >> 4); groups of 16 lanes, bank = (a / 4) mod 64
  MN-contiguous image [64 k][256 cols] (512-byte rows), ds_read_b64_tr_b16: lane 4q + p of
      16-lane group g reads row 32 kh + 8 g + 4 s + q, 8 bytes at column c0 + 4 p;
      half-waves of 32 lanes, bank = (a / 4) mod 64

    python bench/lds_gemm256.py
"""
import itertools

B128_GROUPS = [[0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27],
               [4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31]]
B128_GROUPS += [[l + 32 for l in g] for g in B128_GROUPS]
TR_GROUPS = [list(range(32)), list(range(32, 64))]


def kc_swz(r):      # gemm256.hip kc_swz
    return (r >> 1) & 7


def mn_swz(r):      # gemm256.hip mn_swz
    return ((r & 1) << 1) | (((r >> 1) & 1) << 2) | (((r >> 3) & 1) << 3)


def kc_worst(h):
    """Max lanes on one 16-byte bank slot over every ds_read_b128 group (1 = conflict-free)."""
    worst = 0
    for kh in range(2):
        for r0 in range(0, 256, 16):
            for g in B128_GROUPS:
                slots = {}
                for l in g:
                    r = r0 + (l & 15)
                    c = (4 * kh + (l >> 4)) ^ h(r)
                    s = ((r * 128 + c * 16) // 16) % 16
                    slots[s] = slots.get(s, 0) + 1
                worst = max(worst, max(slots.values()))
    return worst


def mn_worst(f):
    """Max accesses on one bank over every ds_read_b64_tr_b16 half-wave (1 = conflict-free)."""
    worst = 0
    for kh in range(2):
        for s in range(2):
            for c0 in range(0, 256, 16):
                for g in TR_GROUPS:
                    banks = {}
                    for l in g:
                        gg, q, p = (l >> 4) & 3, (l >> 2) & 3, l & 3
                        r = 32 * kh + 8 * gg + 4 * s + q
                        cb = 2 * (c0 + 4 * p)
                        a = r * 512 + 16 * ((cb >> 4) ^ f(r)) + (cb & 15)
                        for d in range(2):
                            b = (a // 4 + d) % 64
                            banks[b] = banks.get(b, 0) + 1
                    worst = max(worst, max(banks.values()))
    return worst


def xor_of_bits(masks):
    def h(r):
        v = 0
        for i, m in enumerate(masks):
            if (r >> i) & 1:
                v ^= m
        return v
    return h


def search():
    kc = min(itertools.product(range(8), repeat=4), key=lambda m: kc_worst(xor_of_bits(m)))
    mn = min(itertools.product(range(0, 16, 2), repeat=4), key=lambda m: mn_worst(xor_of_bits(m)))
    return kc, kc_worst(xor_of_bits(kc)), mn, mn_worst(xor_of_bits(mn))


def main():
    print("linear images: KC", kc_worst(lambda r: 0), "-way, MN", mn_worst(lambda r: 0), "-way")
    print("gemm256.hip swizzles: KC", kc_worst(kc_swz), "-way, MN", mn_worst(mn_swz), "-way")
    kc, kcw, mn, mnw = search()
    print("search: best KC masks", kc, kcw, "| best MN masks", mn, mnw)


if __name__ == "__main__":
    main()
