#!/usr/bin/env python3
"""LDS bank model of gemm.hip's K-contiguous operand images (kc_store / frag_kc): the staging
stores (two ds_write_b64 per 16-byte global vector, permuted k order) and the fragment reads
(ds_read_b128), per row stride, with and without the odd-row 16-byte-block swap the kernel
uses at 48-element rows.  Bank rules: bench/lds_bwd.py.

    python bench/lds_gemm_kc.py
"""
from lds_bwd import cycles


def kc_col(k):
    return 8 * ((k & 15) >> 2) + (k & 3) + 4 * (k >> 4)


def store(S, sw, second):
    out = []
    for l in range(64):
        r, vq = l // 4, l % 4
        col = kc_col(8 * vq + (4 if second else 0))
        if sw:
            col ^= (r & 1) << 3
        out.append(2 * (r * S + col))
    return cycles(out, 8, "w64")


def read(S, sw, r0=0):
    out = []
    for l in range(64):
        i, g = l & 15, l >> 4
        b = g ^ (i & 1) if sw else g
        out.append(2 * ((r0 + i) * S + 8 * b))
    return cycles(out, 16, "b128")


if __name__ == "__main__":
    for S in (40, 48, 56):
        for sw in (False, True):
            st = (store(S, sw, False) + store(S, sw, True)) / 2
            rd = sum(read(S, sw, r0) for r0 in (0, 16, 32, 48)) / 4
            print(f"row stride {S} swap {sw}: store {st:.2f}  read {rd:.2f} cycles per group")
