#!/usr/bin/env python3
"""Upper bound of VERDICT r4 ask 1(c) -- "stop writing pool1 and its codes; recompute them in
the backward": what the LeNet-5 step would save if pool1 (205 MB bf16) and its argmax codes
(51 MB) were never written by the band forward nor read by the fused backward, before paying
for any recompute.

    band forward with pool1 / codes written   vs   not written (the eval-path launch)
    fused backward (prof build)               vs   the same launch with the pool1 / code loads
                                                   skipped (MNISTX_BWD_SKIP=32; wrong results,
                                                   timing only)

Interleaved launches, median of rounds (us), B = 65536.

    python bench/micro_p1_ab.py [B]
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
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    torch.manual_seed(0)
    n = 60000
    ds = (torch.rand(n, 784, device=dev) - 0.5).to(torch.bfloat16)
    idx = torch.randint(0, n, (B,), device=dev, dtype=torch.int64)
    w1 = torch.zeros(5, 5, 1, 8, device=dev)
    w1[..., :6] = torch.randn(5, 5, 1, 6, device=dev) / 5
    w2 = torch.zeros(5, 5, 8, 16, device=dev)
    w2[:, :, :6] = torch.randn(5, 5, 6, 16, device=dev) / 12
    w1, w2 = w1.to(torch.bfloat16), w2.to(torch.bfloat16)
    b1, b2 = torch.randn(6, device=dev) * 0.1, torch.randn(16, device=dev) * 0.1
    P1 = torch.empty(B, 14, 14, 8, dtype=torch.bfloat16, device=dev)
    A1 = torch.empty(B, 14, 14, 4, dtype=torch.uint8, device=dev)
    P2 = torch.empty(B, 5, 5, 16, dtype=torch.bfloat16, device=dev)
    A2 = torch.empty(B, 5, 5, 16, dtype=torch.uint8, device=dev)
    dP2 = (torch.randn(B, 400, device=dev) * 1e-3).to(torch.bfloat16)
    grid = K.lenet_bwd_blocks(B)
    s1 = torch.zeros(grid * 32 * 8, device=dev)
    s2 = torch.zeros(grid * 208 * 16, device=dev)
    pr = torch.zeros(8, dtype=torch.int64, device=dev)

    def bwd(skip):
        def f():
            os.environ["MNISTX_BWD_SKIP"] = str(skip)
            K.lenet_bwd(ds, P1, dP2, A2, w2, B, s1, s2, grid, idx=idx, prof=pr)
        return f

    cases = {
        "band_fwd_p1": lambda: K.lenet_band_fwd(ds, w1, b1, 6, w2, b2, B, P2, A2, p1=P1, idx=idx),
        "band_fwd_no_p1": lambda: K.lenet_band_fwd(ds, w1, b1, 6, w2, b2, B, P2, A2, idx=idx),
        "bwd_prof": bwd(0),
        "bwd_prof_skip_p1_loads": bwd(32),
    }
    a = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
    for _ in range(150):
        a = (a @ a).clamp_(-1, 1)
    res = {k: [] for k in cases}
    for _ in range(9):
        for name, f in cases.items():
            for _ in range(3):
                f()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                f()
            e1.record()
            torch.cuda.synchronize()
            res[name].append(e0.elapsed_time(e1) / 10 * 1e3)
    os.environ.pop("MNISTX_BWD_SKIP", None)
    med = {k: round(statistics.median(v), 1) for k, v in res.items()}
    med["upper_bound_saving_us"] = round(med["band_fwd_p1"] - med["band_fwd_no_p1"] + med["bwd_prof"]
                                         - med["bwd_prof_skip_p1_loads"], 1)
    print(json.dumps({"B": B, **med}), flush=True)


if __name__ == "__main__":
    main()
