"""Microbenchmark: fused conv1 (LeNet-5) forward + weight gradient reading
(a) bf16 activations, (b) the uint8 dataset through a sequential index,
(c) the uint8 dataset through a random permutation (the training case)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_tensorflow_ibm_mnist_amd.ops._ext import kernels  # noqa: E402


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def main():
    K = kernels()
    dev = torch.device("cuda", 0)
    B, N = 65536, 60000
    geo = (1, 8, 5, 2, 28, 28)
    u8 = torch.randint(0, 256, (N, 784), dtype=torch.uint8, device=dev)
    x = (torch.rand(B, 28, 28, 1, device=dev) - 0.5).to(torch.bfloat16)
    w = (torch.randn(5, 5, 1, 8, device=dev) * 0.2).to(torch.bfloat16)
    b = torch.zeros(8, device=dev)
    pooled = torch.empty(B, 14, 14, 8, dtype=torch.bfloat16, device=dev)
    arg = torch.empty(B, 14, 14, 8, dtype=torch.uint8, device=dev)
    seq = (torch.arange(B, device=dev) % N).to(torch.int64)
    perm = (torch.randperm(4 * N, device=dev) % N)[:B].contiguous()
    res = {}
    res["fwd bf16"] = timeit(lambda: K.convpool_fwd(x, w, b, 6, pooled, arg, B, *geo))
    res["fwd u8 seq"] = timeit(lambda: K.convpool_fwd(x, w, b, 6, pooled, arg, B, *geo, u8=u8, idx=seq))
    res["fwd u8 perm"] = timeit(lambda: K.convpool_fwd(x, w, b, 6, pooled, arg, B, *geo, u8=u8, idx=perm))
    KM = K.convpool_rows(*geo)
    slab = torch.empty(1024 * KM * 8, device=dev)
    dP = torch.randn(B, 14, 14, 8, device=dev).to(torch.bfloat16)
    res["wgrad bf16"] = timeit(lambda: K.convpool_wgrad(x, dP, arg, slab, 1024, B, *geo))
    res["wgrad u8 seq"] = timeit(lambda: K.convpool_wgrad(x, dP, arg, slab, 1024, B, *geo, u8=u8, idx=seq))
    res["wgrad u8 perm"] = timeit(lambda: K.convpool_wgrad(x, dP, arg, slab, 1024, B, *geo, u8=u8, idx=perm))
    xi = torch.empty(B, 784, dtype=torch.bfloat16, device=dev)
    lab = torch.zeros(N, dtype=torch.int32, device=dev)
    lo = torch.empty(B, dtype=torch.int32, device=dev)
    res["prep_images perm"] = timeit(lambda: K.prep_images(u8, perm, lab, xi, lo, 784, 1, 1))
    for k, v in res.items():
        print(f"{k:20s} {v:8.1f} us")


if __name__ == "__main__":
    main()
