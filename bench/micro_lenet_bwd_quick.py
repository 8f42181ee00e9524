#!/usr/bin/env python3
"""Fused LeNet-5 conv backward alone at B = 65536 (median of rounds of 30 launches, us): a quick
single-number timing for env-knob A/Bs run as separate processes (bench/micro_lenet_bwd.py has
the full attribution).

    MNISTX_SOME_KNOB=1 python bench/micro_lenet_bwd_quick.py
"""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from distributed_tensorflow_ibm_mnist_amd.ops._ext import kernels
    K = kernels()
    dev = torch.device("cuda", 0)
    B = 65536
    torch.manual_seed(0)
    n = 60000
    ds = torch.randint(0, 256, (n, 784), device=dev, dtype=torch.uint8)
    idx = torch.randint(0, n, (B,), device=dev, dtype=torch.int64)
    w1 = torch.zeros(5, 5, 1, 8, device=dev)
    w1[..., :6] = torch.randn(5, 5, 1, 6, device=dev) / 5
    w2 = torch.zeros(5, 5, 8, 16, device=dev)
    w2[:, :, :6] = torch.randn(5, 5, 6, 16, device=dev) / 12
    w1, w2 = w1.to(torch.bfloat16), w2.to(torch.bfloat16)
    b1, b2 = torch.randn(6, device=dev) * 0.1, torch.randn(16, device=dev) * 0.1
    P1 = torch.empty(B, 196, 8, dtype=torch.bfloat16, device=dev)
    P2 = torch.empty(B, 5, 5, 16, dtype=torch.bfloat16, device=dev)
    A2 = torch.empty(B, 5, 5, 16, dtype=torch.uint8, device=dev)
    K.lenet_band_fwd(ds, w1, b1, 6, w2, b2, B, P2, A2, p1=P1, idx=idx)   # combined pool1 records
    dP2 = (torch.randn(B, 400, device=dev) * 1e-3).to(torch.bfloat16)
    grid = K.lenet_bwd_blocks(B)
    s1 = torch.zeros(grid * 32 * 8, device=dev)
    s2 = torch.zeros(grid * 208 * 16, device=dev)
    f = lambda: K.lenet_bwd(ds, P1, dP2, A2, w2, B, s1, s2, grid, idx=idx)
    for _ in range(200):
        f()
    ts = []
    for _ in range(9):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(30):
            f()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / 30 * 1e3)
    print(json.dumps({"lenet_bwd_us": round(statistics.median(ts), 1),
                      "min_us": round(min(ts), 1)}), flush=True)


if __name__ == "__main__":
    main()
