#!/usr/bin/env python3
"""Reference-CNN conv1 weight gradient with the norm1 backward folded in: refc1_wgrad.hip vs
the folded convpool_wgrad it replaces, at the benchmark batch (one JSON line).

    python bench/micro_refc1.py [--batch 16384] [--iters 50]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_tensorflow_ibm_mnist_amd.ops._ext import kernels  # noqa: E402

LRN = (1.0, 0.001 / 9.0, 0.75)


def timed(fn, iters):
    best = float("inf")
    for _ in range(3):
        fn()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(iters):
            fn()
        b.record()
        torch.cuda.synchronize()
        best = min(best, a.elapsed_time(b) * 1e3 / iters)
    return round(best, 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16384)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--cin", type=int, default=1, choices=(1, 3))
    args = ap.parse_args()
    K, dev, B, C = kernels(), torch.device("cuda:0"), args.batch, args.cin
    torch.manual_seed(0)
    x = (torch.rand(B, 28, 28, C, device=dev) - 0.5).to(torch.bfloat16)
    w = (torch.randn(5, 5, C, 32, device=dev) * 0.2).to(torch.bfloat16)
    b = torch.randn(32, device=dev) * 0.05
    P1 = torch.empty(B, 14, 14, 32, dtype=torch.bfloat16, device=dev)
    A1 = torch.empty(B, 14, 14, 32, dtype=torch.uint8, device=dev)
    K.convpool_fwd(x, w, b, 32, P1, A1, B, C, 32, 5, 2, 28, 28)
    dn = (torch.randn(B, 14, 14, 32, device=dev) * 0.1).to(torch.bfloat16)
    grid = K.refc1_wgrad_blocks(B)
    slab = torch.empty(grid * (48 if C == 1 else 80) * 32, device=dev)
    cgrid = K.convpool_wgrad_grid(C, 32, 5, 2, 28, 28)
    cslab = torch.empty(cgrid * K.convpool_rows(C, 32, 5, 2, 28, 28) * 32, device=dev)
    run = lambda: K.refc1_wgrad(x, dn, P1, A1, slab, grid, B, *LRN, cin=C)
    res = {"B": B, "cin": C, "grid": grid, "refc1_us": timed(run, args.iters),
           "convpool_fold_us": timed(lambda: K.convpool_wgrad(x, dn, A1, cslab, cgrid, B, C, 32, 5, 2, 28, 28, lrn_p=P1,
                                                              lrn_bias=LRN[0], lrn_alpha=LRN[1], lrn_beta=LRN[2],
                                                              lrn_r=4), args.iters)}
    # the HBM floor: dL/d norm1 + pool1 (bf16) + codes + the images, once each
    gb = B * (196 * 32 * 5 + 784 * 2 * C) / 1e9
    res["bytes_GB"] = round(gb, 3)
    res["refc1_TBps"] = round(gb / res["refc1_us"] * 1e-3 * 1e6, 2)
    # parts left out (experiment bits: 1 GEMM, 2 LRN math, 4 next-tile loads)
    skips = {}
    for s in (1, 2, 4, 3, 5, 6, 7):
        K.refc1_set_skip(s)
        skips[s] = timed(run, args.iters)
    K.refc1_set_skip(0)
    res["us_by_skip"] = skips
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
