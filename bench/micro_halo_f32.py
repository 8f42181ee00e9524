#!/usr/bin/env python3
"""fp32 conv_halo forward launches (reference CNN conv2, 14x14x32 -> 64, 5x5 SAME) at the
benchmark batch, interleaved in one process after a warm-up, CUDA-event timed (best of 3 x 5):
variant 0 = (row, fragment) units balanced over the SIMDs, 1 = the 7 two-row groups.

    python bench/micro_halo_f32.py [--batch 16384] [--order 1,0,1,0]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.environ.get("MICRO_PKG_ROOT") or os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_tensorflow_ibm_mnist_amd.ops._ext import kernels  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16384)
    ap.add_argument("--order", default="1,0,1,0,1,0")
    a = ap.parse_args()
    K = kernels()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    B = a.batch
    x = torch.randn(B, 14, 14, 32, device=dev)
    w = torch.randn(5, 5, 32, 64, device=dev) * 0.05
    b = torch.randn(64, device=dev)
    y = torch.empty(B, 14, 14, 64, device=dev)
    run = lambda: K.f32_conv_fwd(x, w, y, B, 14, 14, 32, 14, 14, 5, 5, 2, 2, 64, b, True)
    for _ in range(5):
        run()
    torch.cuda.synchronize()
    flop = 2 * B * 196 * 64 * 800
    for v in [int(t) for t in a.order.split(",")]:
        K.set_f32_halo_fwd_variant(v)
        run()
        torch.cuda.synchronize()
        best = float("inf")
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                run()
            e1.record()
            torch.cuda.synchronize()
            best = min(best, e0.elapsed_time(e1) * 1000 / 5)
        print(f"variant {v}: fwd {best:8.1f} us ({flop / best / 1e6:6.1f} TFLOP/s)", flush=True)
    K.set_f32_halo_fwd_variant(0)


if __name__ == "__main__":
    main()
