#!/usr/bin/env python3
"""Time the banded LeNet forward kernel alone (B = 65536) under ablation knobs.
Each MNISTX_BAND_DBG value runs in its own process (the launcher reads it once)."""
import json, os, subprocess, sys, time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run_one(p1: int, B: int, iters: int = 50):
    """p1: 0 = pool1 stays in LDS, 1 = pool1 + codes (convpool layouts), 2 = the combined
    16-byte records the training step writes (lenet_bwd_k reads them)."""
    import torch
    from distributed_tensorflow_ibm_mnist_amd.ops._ext import kernels
    K = kernels()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    n = 60000
    ds = (torch.rand(n, 784, device=dev) - 0.5).to(torch.bfloat16)
    idx = torch.randint(0, n, (B,), device=dev, dtype=torch.int64)
    w1 = torch.zeros(5, 5, 1, 8, device=dev); w1[..., :6] = torch.randn(5, 5, 1, 6, device=dev) / 5
    w2 = torch.zeros(5, 5, 8, 16, device=dev); w2[:, :, :6] = torch.randn(5, 5, 6, 16, device=dev) / 12
    w1, w2 = w1.to(torch.bfloat16), w2.to(torch.bfloat16)
    b1, b2 = torch.randn(6, device=dev) * 0.1, torch.randn(16, device=dev) * 0.1
    P1 = torch.empty(B, 14, 14, 8, dtype=torch.bfloat16, device=dev)
    A1 = torch.empty(B, 14, 14, 4, dtype=torch.uint8, device=dev)
    P2 = torch.empty(B, 5, 5, 16, dtype=torch.bfloat16, device=dev)
    A2 = torch.empty(B, 5, 5, 16, dtype=torch.uint8, device=dev)
    kw = dict(p1=P1, arg1=A1) if p1 == 1 else dict(p1=P1) if p1 == 2 else {}
    f = lambda: K.lenet_band_fwd(ds, w1, b1, 6, w2, b2, B, P2, A2, idx=idx, **kw)
    for _ in range(10):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        f()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / iters * 1e3
    prof = torch.zeros(4, dtype=torch.int64, device=dev)
    K.lenet_band_fwd(ds, w1, b1, 6, w2, b2, B, P2, A2, idx=idx, prof=prof, **kw)
    torch.cuda.synchronize()
    pr = prof.tolist()
    nw = 4 * K.lenet_band_fwd_grid() if hasattr(K, "lenet_band_fwd_grid") else 1
    print(json.dumps({"conv1_busy": pr[0], "conv2_busy": pr[1], "conv1_wait": pr[2], "conv2_wait": pr[3],
                      "conv1_busy_frac": pr[0] / max(1, pr[0] + pr[2]), "conv2_busy_frac": pr[1] / max(1, pr[1] + pr[3])}))
    return us


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "one":
        print(json.dumps({"us": run_one(int(sys.argv[2]), int(sys.argv[3]))}))
        sys.exit(0)
    B = int(os.environ.get("B", "65536"))
    for p1 in (1, 0):
        for dbg in (0, 0):
            env = dict(os.environ, MNISTX_BAND_DBG=str(dbg))
            out = subprocess.run([sys.executable, __file__, "one", str(p1), str(B)], env=env, capture_output=True,
                                 text=True, timeout=300)
            line = out.stdout.strip() if out.returncode == 0 else out.stderr[-300:]
            print(f"p1out={p1} dbg={dbg:2d}: {line}", flush=True)
