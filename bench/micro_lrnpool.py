#!/usr/bin/env python3
"""norm2 -> pool2 of the reference CNN at the benchmark batch: the generic lrn_pool kernels vs
the packed 14x14x64 ones (misc.hip lrn_pool14_*), CUDA-event timed, interleaved rounds, plus a
device copy of the same bytes as the bandwidth yardstick.

    python bench/micro_lrnpool.py [--batch 16384]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.environ.get("MICRO_PKG_ROOT") or os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributed_tensorflow_ibm_mnist_amd.ops._ext import kernels


def timed(fn, reps=10):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1000 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16384)
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    K = kernels()
    dev = torch.device("cuda")
    N = a.batch
    torch.manual_seed(0)
    x = (torch.randn(N, 14, 14, 64, device=dev) * 2).relu().to(torch.bfloat16)
    dP = torch.randn(N, 7, 7, 64, device=dev).to(torch.bfloat16)
    y = torch.empty(N, 7, 7, 64, dtype=torch.bfloat16, device=dev)
    arg = torch.empty(N, 7, 7, 64, dtype=torch.uint8, device=dev)
    dx = torch.empty_like(x)
    cp = torch.empty_like(x)
    lrn = (4, 1.0, 0.001 / 9.0, 0.75)

    def fwd():
        K.lrn_pool_fwd(x, y, arg, N, 14, 14, 64, *lrn, nonneg=True)

    def bwd():
        K.lrn_pool_bwd(x, dP, arg, dx, N, 14, 14, 64, *lrn, True)

    res = {k: [] for k in ("fwd_generic", "fwd_packed", "bwd_generic", "bwd_packed", "copy_x")}
    for _ in range(a.rounds):
        for packed in (0, 1):
            K.lrn_set_packed(bool(packed))
            tag = "packed" if packed else "generic"
            fwd(); bwd(); torch.cuda.synchronize()
            res["fwd_" + tag].append(timed(fwd))
            res["bwd_" + tag].append(timed(bwd))
        res["copy_x"].append(timed(lambda: cp.copy_(x)))
    K.lrn_set_packed(True)
    out = {k: round(min(v), 1) for k, v in res.items()}
    mb_f = (x.numel() * 2 + y.numel() * 3) / 1e6
    mb_b = (x.numel() * 4 + y.numel() * 3) / 1e6
    out.update({"fwd_MB": round(mb_f), "bwd_MB": round(mb_b), "copy_MB": round(x.numel() * 4 / 1e6),
                "fwd_packed_TBps": round(mb_f / out["fwd_packed"], 2), "bwd_packed_TBps": round(mb_b / out["bwd_packed"], 2),
                "copy_TBps": round(x.numel() * 4 / 1e6 / out["copy_x"], 2)})
    print(json.dumps(out))


if __name__ == "__main__":
    main()
