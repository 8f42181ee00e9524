#!/usr/bin/env python3
"""Why is lenet_bwd_k slower inside the step (~228 us in the kernel tables) than alone
(~196 us, bench/micro_lenet_bwd_quick.py)?  Times ONE launch (events around it, median of 40)
after three different predecessors:

  alone      the previous launch was lenet_bwd_k itself (the quick micro's situation)
  after_fwd  lenet_band_fwd_k just wrote the pool1 records the backward reads (the step's)
  after_fill a 768 MB fill just evicted every cache level (cold HBM)

The difference between after_fwd and after_fill says how much of the forward's output the
backward still finds in the memory-side cache.

    python bench/micro_lenet_bwd_ctx.py
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
    idx = torch.cat([torch.randperm(n, device=dev), torch.randperm(n, device=dev)])[:B].contiguous()
    w1 = torch.zeros(5, 5, 1, 8, device=dev)
    w1[..., :6] = torch.randn(5, 5, 1, 6, device=dev) / 5
    w2 = torch.zeros(5, 5, 8, 16, device=dev)
    w2[:, :, :6] = torch.randn(5, 5, 6, 16, device=dev) / 12
    w1, w2 = w1.to(torch.bfloat16), w2.to(torch.bfloat16)
    b1, b2 = torch.randn(6, device=dev) * 0.1, torch.randn(16, device=dev) * 0.1
    P1 = torch.empty(B, 196, 8, dtype=torch.bfloat16, device=dev)
    P2 = torch.empty(B, 5, 5, 16, dtype=torch.bfloat16, device=dev)
    A2 = torch.empty(B, 5, 5, 16, dtype=torch.uint8, device=dev)
    fwd = lambda: K.lenet_band_fwd(ds, w1, b1, 6, w2, b2, B, P2, A2, p1=P1, idx=idx)   # noqa: E731
    fwd()
    dP2 = (torch.randn(B, 400, device=dev) * 1e-3).to(torch.bfloat16)
    grid = K.lenet_bwd_blocks(B)
    s1 = torch.zeros(grid * 32 * 8, device=dev)
    s2 = torch.zeros(grid * 208 * 16, device=dev)
    bwd = lambda: K.lenet_bwd(ds, P1, dP2, A2, w2, B, s1, s2, grid, idx=idx)   # noqa: E731
    junk = torch.empty(768 << 20, dtype=torch.uint8, device=dev)
    fill = lambda: junk.fill_(1)   # noqa: E731
    pre = {"alone": bwd, "after_fwd": fwd, "after_fill": fill}
    for _ in range(50):
        fwd()
        bwd()
    out = {}
    for name, p in pre.items():
        ts = []
        for _ in range(40):
            p()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            bwd()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        out[name] = round(statistics.median(ts), 1)
        print(json.dumps({"pre": name, "lenet_bwd_us": out[name], "min_us": round(min(ts), 1)}), flush=True)
    # the forward the same way (after the backward, as in the step's next iteration)
    ts = []
    for _ in range(40):
        bwd()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fwd()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    print(json.dumps({"pre": "bwd", "lenet_band_fwd_us": round(statistics.median(ts), 1)}), flush=True)


if __name__ == "__main__":
    main()
