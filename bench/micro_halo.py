#!/usr/bin/env python3
"""Per-variant times of the conv_halo.hip forward / dgrad launches (reference CNN conv2:
14x14x32 -> 64, 5x5 SAME) at the benchmark batch, CUDA-event timed, best of 3 x 10 calls.

    python bench/micro_halo.py [--batch 16384] [--variants 0,6,7]
"""
import argparse
import math
import os
import sys

import torch

# MICRO_PKG_ROOT: import the package (and its built kernels) from another tree, for
# same-box A/B runs of two builds
sys.path.insert(0, os.environ.get("MICRO_PKG_ROOT") or os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributed_tensorflow_ibm_mnist_amd.ops import functional as Fk
from distributed_tensorflow_ibm_mnist_amd.ops._ext import kernels


def timed(fn, reps=10, rounds=3):
    fn()
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(rounds):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        torch.cuda.synchronize()
        best = min(best, a.elapsed_time(b) * 1000 / reps)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16384)
    ap.add_argument("--variants", default="0,6,7")
    a = ap.parse_args()
    K = kernels()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    B = a.batch
    x = torch.randn(B, 14, 14, 32, device=dev).to(torch.bfloat16)
    w = (torch.randn(5, 5, 32, 64, device=dev) / math.sqrt(800)).to(torch.bfloat16)
    b = torch.randn(64, device=dev)
    dy = torch.randn(B, 14, 14, 64, device=dev).to(torch.bfloat16)
    mask = torch.randn(B, 14, 14, 32, device=dev).relu().to(torch.bfloat16)
    flop = 2 * B * 196 * 64 * 800
    ref_y = ref_dx = None
    K.set_halo_variants(0, 0)   # warm the clocks / caches: the first timed variant ran 10-15 % slow
    for _ in range(20):
        Fk.conv2d(x, w, b, "SAME", relu=True)
        Fk.conv2d_dgrad(dy, w, (14, 14), "SAME", mask=mask)
    K.set_halo_variants(-1, -1)
    for v in [int(t) for t in a.variants.split(",")]:
        K.set_halo_variants(v, v)
        try:
            y = Fk.conv2d(x, w, b, "SAME", relu=True)
            dx = Fk.conv2d_dgrad(dy, w, (14, 14), "SAME", mask=mask)
            if ref_y is None:
                ref_y, ref_dx = y.float(), dx.float()
            ey = (y.float() - ref_y).abs().max().item()
            ed = (dx.float() - ref_dx).abs().max().item()
            tf = timed(lambda: Fk.conv2d(x, w, b, "SAME", relu=True))
            td = timed(lambda: Fk.conv2d_dgrad(dy, w, (14, 14), "SAME", mask=mask))
            print(f"variant {v}: fwd {tf:7.1f} us ({flop / tf / 1e6:6.1f} TFLOP/s)  dgrad {td:7.1f} us "
                  f"({flop / td / 1e6:6.1f} TFLOP/s)  max |diff| vs first: fwd {ey:.3g} dgrad {ed:.3g}", flush=True)
        finally:
            K.set_halo_variants(-1, -1)


if __name__ == "__main__":
    main()
