#!/usr/bin/env python3
"""Time the fused LeNet-5 conv-stack backward (lenet_bwd.hip) alone at the BASELINE batch,
against the three per-layer kernels it replaces, at smaller batches on the same grid (the
fixed vs per-tile cost), and print its per-phase clock split (s_memtime sums over all
waves; the prof build of the same launch).

    python bench/micro_lenet_bwd.py [B]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PHASES = ["stage_in", "dgrad", "c2_wgrad", "barrier1", "stage_dy2_p1", "c1_wgrad", "barrier2", "epilogue"]


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
    K.lenet_band_fwd(ds, w1, b1, 6, w2, b2, B, P2, A2, p1=P1, idx=idx)
    dP2 = (torch.randn(B, 400, device=dev) * 1e-3).to(torch.bfloat16)
    grid = K.lenet_bwd_blocks(B)
    s1 = torch.zeros(grid * 32 * 8, device=dev)
    s2 = torch.zeros(grid * 208 * 16, device=dev)

    def timeit(f, iters=30, reps=3):
        """best of `reps` means over `iters` back-to-back launches (us)"""
        for _ in range(5):
            f()
        torch.cuda.synchronize()
        best = float("inf")
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(iters):
                f()
            e1.record()
            torch.cuda.synchronize()
            best = min(best, e0.elapsed_time(e1) / iters * 1e3)
        return best

    timeit(lambda: K.lenet_bwd(ds, P1, dP2, A2, w2, B, s1, s2, grid, idx=idx), iters=200, reps=1)  # clocks up
    fused = timeit(lambda: K.lenet_bwd(ds, P1, dP2, A2, w2, B, s1, s2, grid, idx=idx))
    # cold caches: a 1 GiB write between launches evicts the inputs from L2 / MALL (the in-step
    # situation is in between: the band forward wrote pool1 / codes shortly before)
    junk = torch.empty(256 * 1024 * 1024, dtype=torch.float32, device=dev)
    cold = []
    for _ in range(12):
        junk.fill_(1.0)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        K.lenet_bwd(ds, P1, dP2, A2, w2, B, s1, s2, grid, idx=idx)
        e1.record()
        torch.cuda.synchronize()
        cold.append(e0.elapsed_time(e1) * 1e3)
    fused_cold = sorted(cold[2:])[len(cold[2:]) // 2]

    # the step's order: the band forward (writes pool1 / codes) right before, then ~150 MB of
    # other traffic (the head / its weight gradients) before the backward
    def seq_time(pre):
        ts = []
        for _ in range(12):
            pre()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            K.lenet_bwd(ds, P1, dP2, A2, w2, B, s1, s2, grid, idx=idx)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        return round(sorted(ts[2:])[len(ts[2:]) // 2], 1)
    band_call = lambda: K.lenet_band_fwd(ds, w1, b1, 6, w2, b2, B, P2, A2, p1=P1, idx=idx)
    traffic = junk[: 38 * 1024 * 1024]
    after_band = seq_time(band_call)
    after_band_traffic = seq_time(lambda: (band_call(), traffic.fill_(2.0)))
    after_traffic = seq_time(lambda: traffic.fill_(3.0))
    del junk, traffic
    # the band forward (conv1 + pool1 + conv2 + pool2, pool1 / codes copied out) on the same box
    band = timeit(lambda: K.lenet_band_fwd(ds, w1, b1, 6, w2, b2, B, P2, A2, p1=P1, idx=idx))
    # the input read as uint8 (half the bytes of the bf16 copy; normalised while staging)
    ds_u8 = torch.randint(0, 256, (n, 784), device=dev, dtype=torch.uint8)
    fused_u8 = timeit(lambda: K.lenet_bwd(ds_u8, P1, dP2, A2, w2, B, s1, s2, grid, idx=idx))
    # fixed vs per-tile cost: the same kernel over the first Bs images (grid stays 256 blocks
    # while Bs / 8 >= 256), 1 .. B/2048 tiles per block
    scaling = {}
    for Bs in (2048, 4096, 8192, 16384, 32768, B):
        if Bs <= B:
            gs = K.lenet_bwd_blocks(Bs)
            scaling[Bs] = round(timeit(lambda: K.lenet_bwd(ds, P1, dP2, A2, w2, Bs, s1, s2, gs, idx=idx)), 1)
    # the split path: conv2 dgrad -> dP1 in HBM, conv2 / conv1 weight gradients
    dP1 = torch.empty(B, 14, 14, 8, dtype=torch.bfloat16, device=dev)
    g2 = K.convpool_wgrad_grid(8, 16, 5, 0, 14, 14)
    g1 = K.convpool_wgrad_grid(1, 8, 5, 2, 28, 28)
    sl2 = torch.zeros(g2 * K.convpool_rows(8, 16, 5, 0, 14, 14) * 16, device=dev)
    sl1 = torch.zeros(g1 * K.convpool_rows(1, 8, 5, 2, 28, 28) * 8, device=dev)
    dgr = timeit(lambda: K.convpool_dgrad(dP2.view(B, 5, 5, 16), A2, w2, dP1, B, 8, 16, 5, 0, 14, 14))
    w2g = timeit(lambda: K.convpool_wgrad(P1, dP2.view(B, 5, 5, 16), A2, sl2, g2, B, 8, 16, 5, 0, 14, 14))
    w1g = timeit(lambda: K.convpool_wgrad(ds, dP1, A1, sl1, g1, B, 1, 8, 5, 2, 28, 28, idx=idx))
    # time attribution (prof launches, experiments): skip bits 1 dgrad, 2 conv2 wgrad, 4 conv1
    # wgrad, 8 staging, 16 loop barriers
    skip_us = {}
    pr_buf = torch.zeros(8, dtype=torch.int64, device=dev)
    for sk in [int(v) for v in os.environ.get("SKIPS", "0,1,2,4,8,16,7,15").split(",")]:
        os.environ["MNISTX_BWD_SKIP"] = str(sk)
        skip_us[sk] = round(timeit(lambda: K.lenet_bwd(ds, P1, dP2, A2, w2, B, s1, s2, grid, idx=idx,
                                                       prof=pr_buf)), 1)
    os.environ.pop("MNISTX_BWD_SKIP", None)
    os.environ["MNISTX_BWD_PROF_WAVES"] = "1"      # [8 phases] + [16 waves][8 phases]
    prof = torch.zeros(8 + 16 * 8, dtype=torch.int64, device=dev)
    K.lenet_bwd(ds, P1, dP2, A2, w2, B, s1, s2, grid, idx=idx, prof=prof)
    torch.cuda.synchronize()
    os.environ.pop("MNISTX_BWD_PROF_WAVES", None)
    allp = prof.tolist()
    pr = allp[:8]
    # per wave: phase-1 work (staging, dgrad, conv2 wgrad) and phase-2 work (next-tile issue,
    # conv1 wgrad + dY2 store) as shares of the wave's total, and the waits
    per_wave = []
    for w in range(16):
        v = allp[8 + 8 * w: 16 + 8 * w]
        t = max(1, sum(v))
        per_wave.append({"p1": round((v[0] + v[1] + v[2]) / t, 3), "bar1": round(v[3] / t, 3),
                         "p2": round((v[4] + v[5]) / t, 3), "bar2": round(v[6] / t, 3)})
    tot = max(1, sum(pr))
    print(json.dumps({"B": B, "grid": grid, "fused_us": round(fused, 1), "fused_cold_us": round(fused_cold, 1), "after_band_us": after_band,
                      "after_band_150MB_us": after_band_traffic, "after_150MB_us": after_traffic, "band_fwd_us": round(band, 1), "fused_u8_us": round(fused_u8, 1), "fused_us_by_batch": scaling, "prof_us_by_skip": skip_us,
                      "split_us": {"c2_dgrad": round(dgr, 1), "c2_wgrad": round(w2g, 1), "c1_wgrad": round(w1g, 1),
                                   "sum": round(dgr + w2g + w1g, 1)},
                      "phase_share": {k: round(v / tot, 3) for k, v in zip(PHASES, pr)},
                      "per_wave": per_wave}), flush=True)


if __name__ == "__main__":
    main()
