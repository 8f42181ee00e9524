#!/usr/bin/env python3
"""Reference-CNN local3 GEMMs (B x 3136 -> 384) at B = 16384: this framework's
dense_fwd / dense_dgrad / dense_wgrad(+reduce) vs torch.matmul (hipBLASLt) on the
same bf16 operands, hipGraph-timed (device time only).
Usage: python bench/micro_local3.py [B] [Din] [Dout]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_tensorflow_ibm_mnist_amd.ops._ext import kernels  # noqa: E402
from distributed_tensorflow_ibm_mnist_amd.ops import functional as Fk  # noqa: E402


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(st):
        fn()
    torch.cuda.current_stream().wait_stream(st)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    Din = int(sys.argv[2]) if len(sys.argv) > 2 else 3136
    Dout = int(sys.argv[3]) if len(sys.argv) > 3 else 384
    K = kernels()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    x = (torch.randn(B, Din, device=dev) * 0.5).to(torch.bfloat16)
    w = (torch.randn(Din, Dout, device=dev) * 0.05).to(torch.bfloat16)
    bias = torch.randn(Dout, device=dev)
    dy = (torch.randn(B, Dout, device=dev) * 0.1).to(torch.bfloat16)
    y = torch.empty(B, Dout, dtype=torch.bfloat16, device=dev)
    dx = torch.empty(B, Din, dtype=torch.bfloat16, device=dev)
    flop = 2.0 * B * Din * Dout

    def rep(name, us, ref=None, out=None):
        err = ""
        if ref is not None:
            e = ((out.float() - ref.float()).abs().max() / ref.float().abs().max()).item()
            err = f" relerr {e:.2e}"
        print(f"{name:28s} {us:8.1f} us  {flop / us / 1e6:7.1f} TFLOP/s{err}", flush=True)

    wt = w.t().contiguous()
    # forward: y = relu(x w + b)
    us = timed(lambda: K.dense_fwd(x, w, y, B, Dout, Din, Din, Dout, Dout, bias, Dout, True, None, 0))
    ref = torch.relu(x.float() @ w.float() + bias)
    rep("fwd  mnistx", us, ref, y)
    us = timed(lambda: torch.matmul(x, w))
    rep("fwd  torch.matmul", us)
    us = timed(lambda: torch.nn.functional.linear(x, wt))
    rep("fwd  F.linear (W^T)", us)
    # dgrad: dx = dy w^T
    us = timed(lambda: K.dense_dgrad(dy, w, dx, B, Din, Dout, Dout, Dout, Din, None, 0))
    rep("dgrad mnistx", us, dy.float() @ w.float().t(), dx)
    us = timed(lambda: torch.matmul(dy, wt))
    rep("dgrad torch.matmul", us)
    # wgrad: dW = x^T dy (+ bias row), split-K + reduce
    M = Din + 1
    for S in (Fk.pick_splits(M, Dout, B, dense=True), 4, 8, 16, 32):
        slab = torch.empty(S * M * Dout + 64, device=dev)
        dw = torch.empty(Din * Dout, device=dev)
        db = torch.empty(Dout, device=dev)
        for code in (7, 4):
            def run():
                s = K.dense_wgrad(x, dy, slab, Din, Dout, B, Din, Dout, True, S, code)
                K.splitk_reduce_multi([slab], [dw], [db], torch.tensor([[s, M, Dout, 1, Din, Din, Dout, Din]]), [1.0])
            us = timed(run)
            rep(f"wgrad mnistx S={S} tile={code}", us, x.float().t() @ dy.float(), dw.view(Din, Dout))
    us = timed(lambda: torch.matmul(x.t(), dy))
    rep("wgrad torch.matmul", us)


if __name__ == "__main__":
    main()
