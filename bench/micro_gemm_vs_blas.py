#!/usr/bin/env python3
"""Reference-CNN local3 GEMMs (B=16384: 16384x3136 @ 3136x1024, its dgrad and wgrad):
the in-tree MFMA GEMM engine (gemm.hip / f32.hip) vs torch.matmul (hipBLASLt) on the
same shapes, bf16 and fp32.  Prints us per call."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_tensorflow_ibm_mnist_amd.ops import functional as Fk  # noqa: E402
from distributed_tensorflow_ibm_mnist_amd.ops._ext import kernels  # noqa: E402


def t(f, n=20):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        f()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1e3


def main():
    dev = torch.device("cuda", 0)
    torch.backends.cuda.matmul.allow_tf32 = False
    B, D, N = 16384, 3136, 1024
    K = kernels()
    for dt in (torch.bfloat16, torch.float32):
        x = torch.randn(B, D, device=dev).to(dt)
        w = (torch.randn(D, N, device=dev) * 0.02).to(dt)
        dy = torch.randn(B, N, device=dev).to(dt)
        bias = torch.zeros(N, device=dev)
        if dt == torch.bfloat16:
            out = torch.empty(B, N, dtype=dt, device=dev)
            ours = {"fwd": lambda: Fk.dense(x, w, bias, True, out=out),
                    "dgrad": lambda: Fk.dense_dgrad(dy, w),
                    "wgrad": lambda: Fk.dense_wgrad(x, dy, D, N)}
        else:
            y = torch.empty(B, N, device=dev)
            dx = torch.empty(B, D, device=dev)
            S = 3
            slab = torch.empty(S * (D + 1) * N, device=dev)
            ours = {"fwd": lambda: K.f32_dense_fwd(x, w, y, B, N, D, N, bias, True),
                    "dgrad": lambda: K.f32_dense_dgrad(dy, w, dx, B, D, N, None),
                    "wgrad": lambda: K.f32_dense_wgrad(x, dy, slab, B, D, N, S)}
        blas = {"fwd": lambda: torch.matmul(x, w), "dgrad": lambda: torch.matmul(dy, w.t()),
                "wgrad": lambda: torch.matmul(x.t(), dy)}
        for k in ("fwd", "dgrad", "wgrad"):
            us_o, us_b = t(ours[k]), t(blas[k])
            fl = 2.0 * B * D * N
            print(f"{str(dt)[6:]:9s} {k:6s} ours {us_o:8.1f} us ({fl / us_o / 1e6:6.0f} TF/s)   "
                  f"torch.matmul {us_b:8.1f} us ({fl / us_b / 1e6:6.0f} TF/s)", flush=True)


if __name__ == "__main__":
    main()
