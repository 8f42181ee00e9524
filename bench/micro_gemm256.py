#!/usr/bin/env python3
"""The reference CNN's local3 GEMMs at B = 16384 on gemm256.hip vs gemm.hip vs torch.matmul
(hipBLASLt), interleaved rounds in one process on random data; median us and TFLOP/s.

    python bench/micro_gemm256.py [B]
"""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_tensorflow_ibm_mnist_amd.ops._ext import kernels  # noqa: E402


def main():
    K = kernels()
    dev = torch.device("cuda", 0)
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    din, dout = 3136, 1024
    torch.manual_seed(0)
    x = torch.randn(B, din, device=dev).to(torch.bfloat16)
    w = (torch.randn(din, dout, device=dev) / din ** 0.5).to(torch.bfloat16)
    b = torch.randn(dout, device=dev) * 0.1
    dy = torch.randn(B, dout, device=dev).to(torch.bfloat16)
    y = torch.empty(B, dout, device=dev, dtype=torch.bfloat16)
    dx = torch.empty(B, din, device=dev, dtype=torch.bfloat16)
    flop = 2.0 * B * din * dout

    def fwd(on):
        def f():
            K.set_gemm256(on)
            K.dense_fwd(x, w, y, B, dout, din, din, dout, dout, b, dout, True, None, 0)
        return f

    def dgrad(on):
        def f():
            K.set_gemm256(on)
            K.dense_dgrad(dy, w, dx, B, din, dout, dout, dout, din, None, 0)
        return f

    S = 5   # the executor's slab capacity for local3 (ops/functional.py pick_splits)
    slab = torch.empty(S * (din + 1) * dout, device=dev)

    def wgrad(on):
        def f():
            K.set_gemm256(on)
            K.dense_wgrad(x, dy, slab, din, dout, B, din, dout, True, S)
        return f

    def dbg(f, bits):   # gemm256 experiment bits: 1 = no in-loop DMA (timing only), 2 = BK 64 ring
        def g():
            K.set_gemm256_debug(bits)
            f()
            K.set_gemm256_debug(0)
        return g

    cases = {"fwd_gemm256_no_dma": dbg(fwd(True), 1),
             "wgrad_gemm256": wgrad(True), "wgrad_gemm256_bk64": dbg(wgrad(True), 2),
             "wgrad_gemm256_rp": dbg(wgrad(True), 16), "fwd_gemm256_rp": dbg(fwd(True), 16),
             "dgrad_gemm256_rp": dbg(dgrad(True), 16),
             "wgrad_gemm_hip": wgrad(False), "wgrad_torch_matmul": lambda: torch.matmul(x.t(), dy),
             "fwd_gemm256": fwd(True), "fwd_gemm256_bk64": dbg(fwd(True), 2), "fwd_gemm_hip": fwd(False),
             "fwd_torch_matmul": lambda: torch.matmul(x, w, out=y),
             "dgrad_gemm256": dgrad(True), "dgrad_gemm256_bk64": dbg(dgrad(True), 2), "dgrad_gemm_hip": dgrad(False),
             "dgrad_torch_matmul": lambda: torch.matmul(dy, w.t(), out=dx)}
    # fp32 (--precision fp32): the same local3 GEMMs on gemm256.hip's fp32 kernel vs f32.hip
    xf, wf, dyf = x.float(), w.float(), dy.float()
    yf = torch.empty(B, dout, device=dev)
    dxf = torch.empty(B, din, device=dev)
    Sf = 8
    slabf = torch.empty(Sf * (din + 1) * dout, device=dev)

    def f32(on, which):
        def f():
            K.set_gemm256(on)
            if which == "fwd":
                K.f32_dense_fwd(xf, wf, yf, B, dout, din, dout, b, True)
            elif which == "dgrad":
                K.f32_dense_dgrad(dyf, wf, dxf, B, din, dout, None)
            else:
                K.f32_dense_wgrad(xf, dyf, slabf, B, din, dout, Sf if on else 3)
        return f
    for which in ("fwd", "dgrad", "wgrad"):
        cases[f"f32_{which}_gemm256"] = f32(True, which)
        cases[f"f32_{which}_f32_hip"] = f32(False, which)
    res = {k: [] for k in cases}
    for _ in range(2):
        for f in cases.values():
            f()
    for _ in range(7):
        for name, f in cases.items():
            f()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                f()
            e1.record()
            torch.cuda.synchronize()
            res[name].append(e0.elapsed_time(e1) / 10 * 1e3)
    K.set_gemm256(True)
    out = {"B": B}
    for k, v in res.items():
        m = statistics.median(v)
        out[k] = {"us": round(m, 1), "min_us": round(min(v), 1), "TF": round(flop / m / 1e6, 0)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
