#!/usr/bin/env python3
"""The reference CNN's local3 GEMMs (B x 3136 -> 1024 at B = 16384) on the library path
(torch.mm / torch._addmm_activation -> hipBLASLt) next to this repo's gemm.hip launchers, to
decide which runs them (one JSON line; best of 3 x iters, us per call).

    python bench/micro_gemm_lib.py [--batch 16384] [--din 3136] [--dout 1024]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, iters=20):
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
    ap.add_argument("--din", type=int, default=3136)
    ap.add_argument("--dout", type=int, default=1024)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    B, I, O = a.batch, a.din, a.dout
    x = torch.randn(B, I, device=dev).to(torch.bfloat16)
    w = (torch.randn(I, O, device=dev) * 0.02).to(torch.bfloat16)
    bias = torch.randn(O, device=dev).to(torch.bfloat16)
    dy = torch.randn(B, O, device=dev).to(torch.bfloat16)
    fl = 2.0 * B * I * O
    res = {"B": B, "din": I, "dout": O}
    res["lib_fwd_bias_relu_us"] = timed(lambda: torch._addmm_activation(bias, x, w))
    res["lib_dgrad_us"] = timed(lambda: torch.mm(dy, w.t()))
    res["lib_wgrad_f32_us"] = timed(lambda: torch.mm(x.t(), dy, out_dtype=torch.float32))
    res["lib_wgrad_bf16_us"] = timed(lambda: torch.mm(x.t(), dy))
    for k in list(res):
        if k.endswith("_us") and k.startswith("lib"):
            res[k.replace("_us", "_TF")] = round(fl / res[k] * 1e-6, 1)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
