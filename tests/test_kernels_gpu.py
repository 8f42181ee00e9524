"""T3: every HIP kernel against a plain PyTorch fp32 reference of the same op.

Inputs are bf16-representable so the only differences are fp32 accumulation
order and the final bf16 rounding of the output.
"""
import math

import pytest
import torch
import torch.nn.functional as F

from distributed_tensorflow_ibm_mnist_amd.ops import functional as Fk
from distributed_tensorflow_ibm_mnist_amd.models.torch_ref import lrn_tf

pytestmark = pytest.mark.gpu


def rnd(*shape, dev, scale=1.0, dtype=torch.bfloat16):
    return (torch.randn(*shape, device=dev) * scale).to(dtype)


def close(out, ref, rel=2e-2):
    out = out.float()
    ref = ref.float()
    tol = rel * ref.abs().max().item() + 1e-6
    err = (out - ref).abs().max().item()
    assert err <= tol, f"max err {err:.3e} > tol {tol:.3e}"


# ---------------------------------------------------------------- dense
@pytest.mark.parametrize("M,N,Kd", [(128, 1024, 3136), (37, 120, 400), (5, 16, 88), (300, 192, 1024),
                                    (64, 64, 64), (1000, 88, 120), (3, 1024, 3136)])
@pytest.mark.parametrize("relu", [False, True])
def test_dense_forward(dev, K, M, N, Kd, relu):
    torch.manual_seed(0)
    x = rnd(M, Kd, dev=dev)
    w = rnd(Kd, N, dev=dev, scale=1 / math.sqrt(Kd))
    b = torch.randn(N, device=dev)
    out = Fk.dense(x, w, b, relu)
    ref = x.float() @ w.float() + b
    if relu:
        ref = ref.relu()
    close(out, ref)
    out32 = Fk.dense(x, w, b, relu, out_dtype=torch.float32)
    close(out32, ref, rel=1e-4)


def test_dense_bias_padding(dev, K):
    # bias only for the first 10 of 16 columns; padded columns must be exactly 0
    x = rnd(50, 84, dev=dev)
    w = torch.zeros(84, 16, device=dev)
    w[:, :10] = torch.randn(84, 10, device=dev) * 0.1
    w = w.to(torch.bfloat16)
    b = torch.randn(10, device=dev)
    out = Fk.dense(x, w, b, False, out_dtype=torch.float32, bias_n=10)
    ref = x.float() @ w.float()
    ref[:, :10] += b
    close(out, ref, rel=1e-4)
    assert out[:, 10:].abs().max().item() == 0.0


@pytest.mark.parametrize("M,Din,Dout", [(128, 3136, 1024), (37, 400, 120), (300, 1024, 192), (50, 88, 16)])
def test_dense_dgrad(dev, K, M, Din, Dout):
    torch.manual_seed(1)
    dy = rnd(M, Dout, dev=dev)
    w = rnd(Din, Dout, dev=dev, scale=0.05)
    mask = rnd(M, Din, dev=dev).relu().to(torch.bfloat16)
    out = Fk.dense_dgrad(dy, w)
    ref = dy.float() @ w.float().t()
    close(out, ref)
    outm = Fk.dense_dgrad(dy, w, mask=mask)
    close(outm, ref * (mask.float() > 0))


@pytest.mark.parametrize("B,Din,Dout,splits", [(128, 3136, 1024, None), (1000, 400, 120, None),
                                               (777, 120, 88, 3), (64, 88, 16, 1), (4096, 1024, 192, None),
                                               (96, 4096, 1024, None), (3000, 200, 32, None),
                                               (8192, 88, 16, 100), (20000, 120, 88, 300)])
def test_dense_wgrad(dev, K, B, Din, Dout, splits):
    torch.manual_seed(2)
    x = rnd(B, Din, dev=dev)
    dy = rnd(B, Dout, dev=dev)
    din, dout = Din - (Din % 8 == 0 and Din > 100) * 4, Dout - 6 * (Dout == 16)  # exercise unpadding
    dw, db = Fk.dense_wgrad(x, dy, din, dout, True, splits)
    ref = x.float().t() @ dy.float()
    close(dw, ref[:din, :dout], rel=1e-3)
    close(db, dy.float().sum(0)[:dout], rel=1e-3)


# every tile code of launch_any (large M reaches the 128/256-row tiles)
@pytest.mark.parametrize("M,N,Kd,tile", [(262144, 16, 88, (256, 16)), (262144, 32, 40, (256, 32)),
                                         (131072, 64, 64, (128, 64)), (131072, 128, 64, (128, 128)),
                                         (65536, 128, 400, (64, 128)), (4000, 64, 72, (64, 64)),
                                         (9000, 24, 48, (64, 32)), (1000, 10, 40, (64, 16)),
                                         (65536, 192, 72, (64, 192)), (2000, 184, 40, (32, 192))])
def test_gemm_tile_codes(dev, K, M, N, Kd, tile):
    assert tuple(K.gemm_tile(M, N, False)) == tile
    torch.manual_seed(5)
    x = rnd(M, Kd, dev=dev)
    w = rnd(Kd, N, dev=dev, scale=1 / math.sqrt(Kd))
    out = Fk.dense(x, w, None, False, out_dtype=torch.float32)
    close(out, x.float() @ w.float(), rel=1e-4)
    dx = Fk.dense_dgrad(out.to(torch.bfloat16)[:, :N], w)
    close(dx, out.to(torch.bfloat16).float() @ w.float().t())


@pytest.mark.parametrize("M,N", [(401, 120), (121, 88), (89, 16), (801, 64), (3137, 384), (4097, 1024),
                                 (201, 32), (26, 8), (49, 32)])
def test_wgrad_tile_mirror(K, M, N):
    assert tuple(K.gemm_tile(M, N, True)) == Fk.gemm_tile(M, N)


# ---------------------------------------------------------------- conv
def conv_ref(x, w, b, padding, relu):
    xn = x.float().permute(0, 3, 1, 2)
    wt = w.float().permute(3, 2, 0, 1)
    kh, kw = w.shape[:2]
    if padding == "SAME":
        xn = F.pad(xn, ((kw - 1) // 2, kw // 2, (kh - 1) // 2, kh // 2))
    y = F.conv2d(xn, wt)
    if b is not None:
        y = y + b.view(1, -1, 1, 1)
    if relu:
        y = y.relu()
    return y.permute(0, 2, 3, 1)


CONV_CASES = [
    # N, H, W, Cin, Cout, k, padding
    (4, 28, 28, 1, 8, 5, "SAME"),
    (3, 28, 28, 3, 32, 5, "SAME"),
    (2, 14, 14, 32, 64, 5, "SAME"),
    (5, 14, 14, 8, 16, 5, "VALID"),
    (1, 7, 9, 16, 32, 3, "SAME"),
]


@pytest.mark.parametrize("N,H,W,Ci,Co,k,pad", CONV_CASES)
def test_conv_fwd(dev, K, N, H, W, Ci, Co, k, pad):
    torch.manual_seed(3)
    x = rnd(N, H, W, Ci, dev=dev)
    w = rnd(k, k, Ci, Co, dev=dev, scale=1 / math.sqrt(k * k * Ci))
    b = torch.randn(Co, device=dev)
    y = Fk.conv2d(x, w, b, pad, relu=True)
    close(y, conv_ref(x, w, b, pad, True))


@pytest.mark.parametrize("cap", [0, 2])
@pytest.mark.parametrize("fv,dv", [(0, 0), (1, 1), (2, 2), (3, 3), (4, 4), (5, 5), (6, 6), (7, 7), (8, 8), (9, 9)])
def test_conv_halo_variants(dev, K, grid_cap, fv, dv, cap):
    """Every conv_halo.hip launch variant (reference conv2 geometry; odd batch leaves a
    partial image group) against the fp32 oracle: forward + bias + ReLU, masked dgrad.
    cap > 0: 2 persistent blocks over 25 images, so every block loops >= 3 times with the
    next image group prefetched (the path of the benchmark batch; the 4-image groups of
    the default forward: 7 groups, the last one partial)."""
    torch.manual_seed(7)
    N, H, W, Ci, Co, k, pad = 5, 14, 14, 32, 64, 5, "SAME"
    if cap:
        grid_cap(cap)
        N = 25
    x = rnd(N, H, W, Ci, dev=dev).float().requires_grad_(True)
    w = rnd(k, k, Ci, Co, dev=dev, scale=1 / math.sqrt(k * k * Ci))
    b = torch.randn(Co, device=dev)
    K.set_halo_variants(fv, dv)
    try:
        y = Fk.conv2d(x.detach().to(torch.bfloat16), w, b, pad, relu=True)
        close(y, conv_ref(x.detach().to(torch.bfloat16), w, b, pad, True))
        yr = conv_ref(x, w, None, pad, False)
        dy = rnd(*yr.shape, dev=dev)
        yr.backward(dy.float())
        mask = rnd(N, H, W, Ci, dev=dev).relu().to(torch.bfloat16)
        dxm = Fk.conv2d_dgrad(dy, w, (H, W), pad, mask=mask)
        close(dxm, x.grad * (mask.float() > 0))
    finally:
        K.set_halo_variants(-1, -1)


@pytest.mark.parametrize("N,H,W,Ci,Co,k,pad", [c for c in CONV_CASES if c[3] % 8 == 0])
def test_conv_dgrad(dev, K, N, H, W, Ci, Co, k, pad):
    torch.manual_seed(4)
    x = rnd(N, H, W, Ci, dev=dev).float().requires_grad_(True)
    w = rnd(k, k, Ci, Co, dev=dev, scale=1 / math.sqrt(k * k * Ci))
    y = conv_ref(x, w, None, pad, False)
    dy = rnd(*y.shape, dev=dev)
    y.backward(dy.float())
    dx = Fk.conv2d_dgrad(dy, w, (H, W), pad)
    close(dx, x.grad)
    mask = rnd(N, H, W, Ci, dev=dev).relu().to(torch.bfloat16)
    dxm = Fk.conv2d_dgrad(dy, w, (H, W), pad, mask=mask)
    close(dxm, x.grad * (mask.float() > 0))


@pytest.mark.parametrize("N,H,W,Ci,Co,k,pad", CONV_CASES)
@pytest.mark.parametrize("splits", [None, 1])
def test_conv_wgrad(dev, K, N, H, W, Ci, Co, k, pad, splits):
    torch.manual_seed(5)
    x = rnd(N, H, W, Ci, dev=dev)
    w = rnd(k, k, Ci, Co, dev=dev).float().requires_grad_(True)
    b = torch.zeros(Co, device=dev, requires_grad=True)
    y = conv_ref(x, w, b, pad, False)
    dy = rnd(*y.shape, dev=dev)
    y.backward(dy.float())
    ci_real = Ci - 2 if Ci == 8 else Ci   # padded-channel unpadding
    co_real = Co - 2 if Co == 8 else Co
    dw, db = Fk.conv2d_wgrad(x, dy, k, k, pad, ci_real, co_real, True, splits)
    close(dw, w.grad[:, :, :ci_real, :co_real], rel=1e-3)
    close(db, b.grad[:co_real], rel=1e-3)


# ---------------------------------------------------------------- pool / lrn / loss
@pytest.mark.parametrize("N,H,W,C", [(4, 28, 28, 8), (3, 14, 14, 64), (2, 7, 7, 16), (5, 10, 10, 16)])
def test_maxpool(dev, K, N, H, W, C):
    torch.manual_seed(6)
    x = rnd(N, H, W, C, dev=dev).relu().to(torch.bfloat16)
    y, arg = Fk.maxpool2x2(x)
    xn = x.float().permute(0, 3, 1, 2).requires_grad_(True)
    ref = F.max_pool2d(xn, 2, 2, ceil_mode=True)
    close(y, ref.permute(0, 2, 3, 1), rel=0)
    dy = rnd(*y.shape, dev=dev)
    ref.backward(dy.float().permute(0, 3, 1, 2))
    dx = Fk.maxpool2x2_bwd(dy, arg, y, (H, W), relu_mask=True)
    g = xn.grad.permute(0, 2, 3, 1) * (x.float() > 0)
    # ties (relu zeros) may route to a different window element; only nonzero inputs are defined
    close(dx.float() * (x.float() > 0), g, rel=0)


@pytest.mark.parametrize("C,r,alpha", [(32, 4, 0.001 / 9.0), (64, 4, 0.001 / 9.0), (64, 4, 0.05), (32, 2, 0.05),
                                       (64, 5, 0.05), (32, 5, 0.05), (16, 4, 0.05), (8, 4, 0.05)])
def test_lrn(dev, K, C, r, alpha):
    """Channel windows cross the 8-channel lane vectors (DPP neighbour exchange): a
    large alpha makes every neighbour term visible; 5x13x13 pixels leave a partial wave."""
    torch.manual_seed(7)
    bias, beta = 1.0, 0.75
    x = (rnd(5, 13, 13, C, dev=dev, scale=3.0)).relu().to(torch.bfloat16)
    y = Fk.lrn(x, r, bias, alpha, beta)
    xn = x.float().permute(0, 3, 1, 2).requires_grad_(True)
    ref = lrn_tf(xn, r, bias, alpha, beta)
    close(y, ref.permute(0, 2, 3, 1))
    dy = rnd(*y.shape, dev=dev)
    ref.backward(dy.float().permute(0, 3, 1, 2))
    dx = Fk.lrn_bwd(x, dy, r, bias, alpha, beta, relu_mask=False)
    close(dx, xn.grad.permute(0, 2, 3, 1))
    dxm = Fk.lrn_bwd(x, dy, r, bias, alpha, beta, relu_mask=True)
    close(dxm, xn.grad.permute(0, 2, 3, 1) * (x.float() > 0))


@pytest.mark.parametrize("B", [1, 3, 127, 128, 4099])
def test_softmax_ce(dev, K, B):
    torch.manual_seed(8)
    logits = torch.randn(B, 16, device=dev) * 3
    logits[:, 10:] = 0
    labels = torch.randint(0, 10, (B,), device=dev, dtype=torch.int32)
    dl, stats = Fk.softmax_ce(logits, labels, 10)
    l = logits[:, :10].clone().requires_grad_(True)
    loss = F.cross_entropy(l, labels.long())
    loss.backward()
    torch.cuda.synchronize()
    assert abs(stats[0].item() / B - loss.item()) < 1e-4 * max(1, loss.item())
    acc = (l.argmax(1) == labels.long()).float().sum().item()
    assert stats[1].item() == acc
    close(dl[:, :10], l.grad)
    assert dl[:, 10:].float().abs().max().item() == 0
    pr = Fk.softmax_probs(logits, 10)
    close(pr, torch.softmax(logits[:, :10], 1), rel=1e-5)


def test_softmax_nan_flag(dev, K):
    logits = torch.zeros(64, 16, device=dev)
    logits[5, 3] = float("nan")
    labels = torch.zeros(64, device=dev, dtype=torch.int32)
    _, stats = Fk.softmax_ce(logits, labels, 10)
    assert stats[2].item() == 1.0


def test_prep_images(dev, K):
    torch.manual_seed(9)
    src = torch.randint(0, 256, (100, 784), dtype=torch.uint8, device=dev)
    lab = torch.randint(0, 10, (100,), dtype=torch.int32, device=dev)
    idx = torch.randperm(100, device=dev)[:37]
    out = torch.empty(37, 28, 28, 1, dtype=torch.bfloat16, device=dev)
    lo = torch.empty(37, dtype=torch.int32, device=dev)
    K.prep_images(src, idx, lab, out, lo, 784, 1, 1)
    ref = src[idx].float() / 255.0 - 0.5
    close(out.view(37, 784), ref, rel=1e-2)
    assert torch.equal(lo, lab[idx])
    out3 = torch.empty(37, 28, 28, 3, dtype=torch.bfloat16, device=dev)
    K.prep_images(src, idx, lab, out3, lo, 784, 1, 3)
    close(out3, ref.view(37, 28, 28, 1).expand(37, 28, 28, 3), rel=1e-2)


def test_fused_optimizer(dev, K):
    from distributed_tensorflow_ibm_mnist_amd.runtime.params import FlatParams, OptConfig
    torch.manual_seed(10)
    shapes = [("a/weights", (5, 5, 3, 32), 0.0), ("a/biases", (32,), None), ("b/weights", (40, 10), 0.004),
              ("b/biases", (10,), None)]
    init = {n: torch.randn(*s) for n, s, _ in shapes}
    fp = FlatParams.build([(n, s, wd) for n, s, wd in shapes], init, dev, pads={"a/weights": (8 - 3 + 3, 32),
                                                                              "b/weights": (40, 16)})
    cfg = OptConfig(lr0=0.1, decay_rate=0.5, decay_steps=2, momentum=0.9, nesterov=True, use_momentum=True,
                    ema_max=0.9999)
    ref = {n: init[n].clone().to(dev) for n in init}
    mom = {n: torch.zeros_like(ref[n]) for n in ref}
    ema = {n: ref[n].clone() for n in ref}
    for step in range(5):
        g = {n: torch.randn_like(ref[n]) for n in ref}
        for n in ref:
            fp.grad_view(n).copy_(g[n])
        fp.apply(cfg, grad_scale=0.5)
        lr = 0.1 * 0.5 ** (step // 2)
        d = min(0.9999, (1 + step) / (10 + step))
        for n, s, wd in shapes:
            gg = g[n] * 0.5 + (wd or 0.0) * ref[n]
            mom[n] = mom[n] * 0.9 + gg
            ref[n] = ref[n] - lr * (gg + 0.9 * mom[n])
            ema[n] = ema[n] - (1 - d) * (ema[n] - ref[n])
        fp.step.add_(1)
    torch.cuda.synchronize()
    for n in ref:
        close(fp.param_view(n), ref[n], rel=1e-5)
        close(fp.ema_view(n), ema[n], rel=1e-5)
    wbf = fp.bf16_view("b/weights")
    assert wbf.shape == (40, 16)
    close(wbf[:, :10], ref["b/weights"], rel=1e-2)
    assert wbf[:, 10:].float().abs().max().item() == 0


# ---------------------------------------------------------------- fused conv + ReLU + max-pool blocks
CP_CASES = [
    # N, H, W, Cin(stride), cin_real, Cout(pad), cout_real, pad
    (7, 28, 28, 1, 1, 8, 6, 2),      # LeNet-5 conv1
    (6, 14, 14, 8, 6, 16, 16, 0),    # LeNet-5 conv2 (VALID)
    (5, 28, 28, 1, 1, 32, 32, 2),    # reference conv1, 1-channel input
    (5, 28, 28, 3, 3, 32, 32, 2),    # reference conv1, 3-channel (DLI) input
]


@pytest.mark.parametrize("cap", [0, 2])
@pytest.mark.parametrize("N,H,W,Ci,ci,Co,co,pad", CP_CASES)
def test_convpool(dev, K, grid_cap, N, H, W, Ci, ci, Co, co, pad, cap):
    """cap > 0: 3x the batch on a grid of `cap` persistent blocks (forward, dgrad and the
    weight gradient), so each block loops over several image groups with the next group
    prefetched -- the paths the benchmark batches run."""
    if cap:
        grid_cap(cap)
        N *= 3
    torch.manual_seed(11)
    padding = "SAME" if pad else "VALID"
    x = rnd(N, H, W, Ci, dev=dev)
    x[..., ci:] = 0
    w = torch.zeros(5, 5, Ci, Co, device=dev)
    w[:, :, :ci, :co] = torch.randn(5, 5, ci, co, device=dev) / math.sqrt(25 * ci)
    w = w.to(torch.bfloat16)
    b = torch.randn(co, device=dev) * 0.1
    OH, OW = (H, W) if pad else (H - 4, W - 4)
    PH, PW = OH // 2, OW // 2
    pooled = torch.empty(N, PH, PW, Co, dtype=torch.bfloat16, device=dev)
    ab = K.convpool_arg_bytes(Ci, Co, 5, pad, H, W)     # LeNet conv1: 8 codes packed 4 bits each
    arg = torch.empty(N, PH, PW, ab, dtype=torch.uint8, device=dev)
    K.convpool_fwd(x, w, b, co, pooled, arg, N, Ci, Co, 5, pad, H, W)
    # oracle: conv -> bias -> relu -> pool (fp32)
    xr = x.float().requires_grad_(True)
    wr = w.float().requires_grad_(True)
    br = torch.zeros(Co, device=dev)
    br[:co] = b
    br.requires_grad_(True)
    y = conv_ref(xr, wr, br, padding, True)                       # [N, OH, OW, Co]
    yp = F.max_pool2d(y.permute(0, 3, 1, 2), 2, 2).permute(0, 2, 3, 1)
    close(pooled, yp)
    if co < Co:
        assert pooled[..., co:].float().abs().max().item() == 0
    # backward: wgrad (+ bias via ones row) and, for LeNet conv2, dgrad
    dP = rnd(N, PH, PW, Co, dev=dev)
    yp.backward(dP.float())
    KM = K.convpool_rows(Ci, Co, 5, pad, H, W)
    grid = cap or 37
    slab = torch.empty(grid * KM * Co, dtype=torch.float32, device=dev)
    K.convpool_wgrad(x, dP, arg, slab, grid, N, Ci, Co, 5, pad, H, W)
    dw = torch.empty(5, 5, ci, co, device=dev)
    db = torch.empty(co, device=dev)
    G, Ip, I, brow = K.convpool_reduce_args(Ci, Co, 5, pad, H, W, ci)
    K.splitk_reduce(slab, grid, KM, Co, G, Ip, I, co, brow, dw, db, 1.0)
    close(dw, wr.grad[:, :, :ci, :co], rel=3e-2)
    close(db, br.grad[:co], rel=3e-2)
    # the ReLU mask lives in the argmax code: 4 exactly where the pooled output is 0
    codes = arg if ab == Co else torch.cat([arg & 15, arg >> 4], dim=-1)   # byte k = code k | code k+4 << 4
    assert torch.equal(codes == 4, pooled == 0)
    assert int(codes.max()) <= 4
    if K.convpool_has_dgrad(Ci, Co, 5, pad, H, W):
        dx = torch.empty(N, H, W, Ci, dtype=torch.bfloat16, device=dev)
        K.convpool_dgrad(dP, arg, w, dx, N, Ci, Co, 5, pad, H, W)
        close(dx[..., :ci], xr.grad[..., :ci])


# ---------------------------------------------------------------- split-K reduce
def test_splitk_reduce_multi_matches_single(dev, K):
    """One multi-tensor launch == per-slab reduces (bitwise) == fp64 sums, across the
    partial-pass (S > 64) and direct cases, with and without a bias row."""
    torch.manual_seed(0)
    cases = [  # (splits, M, N, G, Ipad, I, J, bias_row)
        (1024, 208, 16, 25, 8, 6, 16, 200),   # LeNet conv2 wgrad slab (partial pass)
        (48, 401, 120, 1, 400, 400, 120, 400),
        (7, 89, 16, 1, 88, 84, 10, 88),
        (300, 48, 8, 5, 8, 5, 6, 40),
    ]
    slabs, slabs2, w1, w2, b1, b2 = [], [], [], [], [], []
    for (S, M, N, G, Ip, I, J, br) in cases:
        s = torch.randn(S * M * N, device=dev)
        slabs.append(s)
        slabs2.append(s.clone())
        w1.append(torch.empty(G * I * J, device=dev))
        w2.append(torch.empty(G * I * J, device=dev))
        b1.append(torch.empty(J, device=dev))
        b2.append(torch.empty(J, device=dev))
    for i, c in enumerate(cases):
        K.splitk_reduce(slabs[i], *c, w1[i], b1[i], 0.5)
    geo = torch.tensor(cases, dtype=torch.int64)
    K.splitk_reduce_multi(slabs2, w2, b2, geo, [0.5] * len(cases))
    torch.cuda.synchronize()
    for i, (S, M, N, G, Ip, I, J, br) in enumerate(cases):
        assert torch.equal(w1[i], w2[i]) and torch.equal(b1[i], b2[i])
    # oracle on fresh data (the reduce pre-sums in place)
    S, M, N, G, Ip, I, J, br = cases[0]
    s = torch.randn(S * M * N, device=dev)
    ref = s.double().view(S, M, N).sum(0) * 0.5
    w = torch.empty(G * I * J, device=dev)
    b = torch.empty(J, device=dev)
    K.splitk_reduce_multi([s], [w], [b], torch.tensor([cases[0]]), [0.5])
    wr = ref[:G * Ip].view(G, Ip, N)[:, :I, :J].reshape(-1)
    assert torch.allclose(w.double(), wr, rtol=1e-5, atol=1e-4)
    assert torch.allclose(b.double(), ref[br, :J], rtol=1e-5, atol=1e-4)


def test_splitk_reduce_fused_matches_two_launch(dev, K):
    """The one-launch reduce (partial blocks finish their quads by ticket) == the partial +
    reduce launches: bitwise where the partial pass leaves <= 4 partials (the same summation
    order), to fp32 rounding otherwise; repeated launches (tickets reset) give the same bits."""
    torch.manual_seed(1)
    cases = [  # (splits, M, N, G, Ipad, I, J, bias_row)
        (256, 208, 16, 25, 8, 6, 16, 200),    # LeNet-5 conv2 slab: sb = 4
        (256, 32, 8, 25, 1, 1, 8, 25),        # LeNet-5 conv1 slab: one quad block
        (1024, 208, 16, 25, 8, 6, 16, 200),   # sb = 16
        (48, 401, 120, 1, 400, 400, 120, 400),   # no partial pass, same launch
        (300, 48, 8, 5, 8, 5, 6, 40),
    ]
    base = [torch.randn(S * M * N, device=dev) for (S, M, N, *_r) in cases]
    geo = torch.tensor(cases, dtype=torch.int64)

    def run(fused):
        K.set_reduce_fused(int(fused))
        ws = [torch.empty(G * I * J, device=dev) for (S, M, N, G, Ip, I, J, br) in cases]
        bs = [torch.empty(J, device=dev) for (S, M, N, G, Ip, I, J, br) in cases]
        K.splitk_reduce_multi([b.clone() for b in base], ws, bs, geo, [0.5] * len(cases))
        torch.cuda.synchronize()
        return ws, bs

    try:
        w0, b0 = run(False)
        w1, b1 = run(True)
        w2, b2 = run(True)
    finally:
        K.set_reduce_fused(1)
    assert K.reduce_fused_enabled()
    for i, c in enumerate(cases):
        assert torch.equal(w1[i], w2[i]) and torch.equal(b1[i], b2[i])
        if c[0] <= 256:
            assert torch.equal(w0[i], w1[i]) and torch.equal(b0[i], b1[i]), i
        else:
            assert torch.allclose(w0[i], w1[i], rtol=1e-5, atol=1e-5)
            assert torch.allclose(b0[i], b1[i], rtol=1e-5, atol=1e-5)


# odd (non multiple-of-8) dense shapes take the general scalar-tail loaders
@pytest.mark.parametrize("M,Din,Dout", [(77, 37, 13), (300, 101, 9), (5, 9, 3)])
def test_dense_general_loaders(dev, K, M, Din, Dout):
    torch.manual_seed(11)
    x = rnd(M, Din, dev=dev)
    w = rnd(Din, Dout, dev=dev, scale=1 / math.sqrt(Din))
    b = torch.randn(Dout, device=dev)
    out = Fk.dense(x, w, b, False, out_dtype=torch.float32)
    close(out, x.float() @ w.float() + b, rel=1e-4)
    dy = rnd(M, Dout, dev=dev)
    dx = Fk.dense_dgrad(dy, w)
    close(dx, dy.float() @ w.float().t())
    dw, db = Fk.dense_wgrad(x, dy, Din, Dout, True, None)
    close(dw, x.float().t() @ dy.float(), rel=1e-3)
    close(db, dy.float().sum(0), rel=1e-3)


@pytest.mark.parametrize("N,start,n,seed", [(60000, 0, 65536, 0), (60000, 524288 * 7 + 3, 65536, 9),
                                            (7, 0, 100, 1), (1, 5, 10, 2)])
def test_perm_positions_matches_torch(dev, K, N, start, n, seed):
    from distributed_tensorflow_ibm_mnist_amd.data.device_loader import perm_positions
    g = perm_positions(start, n, N, seed, device=dev)
    c = perm_positions(start, n, N, seed)
    assert torch.equal(g.cpu(), c)


def test_dense_wgrad_group_matches_single(dev, K):
    """Grouped split-K weight gradients (one launch) vs the fp32 reference, with the
    same effective split counts as the per-layer launches."""
    torch.manual_seed(21)
    B = 5000
    shapes = [(400, 120), (120, 88), (88, 16)]
    xs = [rnd(B, d, dev=dev) for d, _ in shapes]
    dys = [rnd(B, n, dev=dev) for _, n in shapes]
    splits = [37, 20, 9]
    slabs = [torch.zeros(s * (d + 1) * n, device=dev) for s, (d, n) in zip(splits, shapes)]
    S = K.dense_wgrad_group(xs, dys, slabs, [d for d, _ in shapes], [n for _, n in shapes], B, splits)
    for (d, n), x, dy, slab, s, sg in zip(shapes, xs, dys, slabs, splits, S):
        ref = torch.zeros_like(slab)
        s1 = K.dense_wgrad(x, dy, ref, d, n, B, d, n, True, s, 7)   # tile code 7 = 64x64
        assert s1 == sg
        tot = slab[: sg * (d + 1) * n].view(sg, d + 1, n).sum(0)
        exp = torch.cat([x.float().t() @ dy.float(), dy.float().sum(0, keepdim=True)])
        close(tot, exp, rel=1e-3)


def test_prep_images_perm_matches_two_step(dev, K):
    """Fused Feistel row + gather + normalise == perm_positions + prep_images."""
    from distributed_tensorflow_ibm_mnist_amd.data.device_loader import _half_bits, perm_positions
    torch.manual_seed(4)
    N, B = 1000, 300
    src = torch.randint(0, 256, (N, 784), dtype=torch.uint8, device=dev)
    lab = torch.randint(0, 10, (N,), dtype=torch.int32, device=dev)
    out = torch.empty(B, 28, 28, 1, dtype=torch.bfloat16, device=dev)
    lo = torch.empty(B, dtype=torch.int32, device=dev)
    K.prep_images_perm(src, lab, out, lo, B, 2500, 77, _half_bits(N))
    idx = perm_positions(2500, B, N, 77, device=dev)
    out2 = torch.empty_like(out)
    lo2 = torch.empty_like(lo)
    K.prep_images(src, idx, lab, out2, lo2, 784, 1, 1)
    assert torch.equal(out, out2) and torch.equal(lo, lo2)


@pytest.mark.parametrize("N,H,W,C,relu", [(7, 14, 14, 64, True), (3, 14, 14, 32, False), (5, 6, 10, 64, True)])
def test_lrn_pool_matches_two_step(dev, K, N, H, W, C, relu):
    """Fused LRN -> 2x2/2 max-pool (forward + backward) == lrn_fwd + maxpool_fwd and
    maxpool_bwd + lrn_bwd, bitwise (7x7x7 windows x 8 lanes leave a partial wave)."""
    torch.manual_seed(22)
    r, bias, alpha, beta = 4, 1.0, 0.05, 0.75
    x = rnd(N, H, W, C, dev=dev, scale=3.0)
    if relu:
        x = x.relu().to(torch.bfloat16)
    OH, OW = H // 2, W // 2
    y = torch.empty(N, OH, OW, C, dtype=torch.bfloat16, device=dev)
    arg = torch.empty(N, OH, OW, C, dtype=torch.uint8, device=dev)
    assert K.lrn_pool_supported(H, W, C, r)
    K.lrn_pool_fwd(x, y, arg, N, H, W, C, r, bias, alpha, beta, nonneg=relu)
    l = torch.empty_like(x)
    K.lrn_fwd(x, l, N * H * W, C, r, bias, alpha, beta)
    y2 = torch.empty_like(y)
    arg2 = torch.empty_like(arg)
    K.maxpool_fwd(l, y2, arg2, N, H, W, C, OH, OW)
    assert torch.equal(y, y2) and torch.equal(arg, arg2)
    dP = rnd(N, OH, OW, C, dev=dev)
    dx = torch.empty_like(x)
    K.lrn_pool_bwd(x, dP, arg, dx, N, H, W, C, r, bias, alpha, beta, relu)
    dl = torch.empty_like(x)
    K.maxpool_bwd(dP, arg2, y2, False, dl, N, H, W, C, OH, OW)
    dx2 = torch.empty_like(x)
    K.lrn_bwd(x, dl, dx2, N * H * W, C, r, bias, alpha, beta, relu)
    assert torch.equal(dx, dx2)


@pytest.mark.parametrize("N", [1, 77, 40000])
def test_lrn_pool_packed(dev, K, N):
    """The packed 14x14x64 norm2 -> pool2 kernels (misc.hip lrn_pool14_fwd_k / _bwd_k: v_pk math,
    integer-key argmax on the post-ReLU input) == the generic lrn_pool kernels, bitwise: pooled
    values, argmax codes (ties included: bf16-rounded inputs repeat) and the input gradient.
    N = 40000 runs two grid-stride iterations at the 16384-block cap."""
    torch.manual_seed(N)
    r, bias, alpha, beta = 4, 1.0, 0.001 / 9.0, 0.75
    x = (torch.randn(N, 14, 14, 64, device=dev) * 2).relu().to(torch.bfloat16)
    x[:, ::3, ::2, 5] = x[:, ::3, ::2, 7]      # repeated values: ties inside pool windows
    x[0, :2, :2, :] = 0                        # an all-zero window
    dP = (torch.randn(N, 7, 7, 64, device=dev)).to(torch.bfloat16)
    outs = []
    for packed in (False, True):
        K.lrn_set_packed(packed)
        try:
            y = torch.full((N, 7, 7, 64), 3.0, dtype=torch.bfloat16, device=dev)
            arg = torch.full((N, 7, 7, 64), 9, dtype=torch.uint8, device=dev)
            K.lrn_pool_fwd(x, y, arg, N, 14, 14, 64, r, bias, alpha, beta, nonneg=True)
            dx = torch.full_like(x, 5.0)
            K.lrn_pool_bwd(x, dP, arg, dx, N, 14, 14, 64, r, bias, alpha, beta, True)
            torch.cuda.synchronize()
            outs.append((y, arg, dx))
        finally:
            K.lrn_set_packed(True)
    for a, b, name in zip(outs[0], outs[1], ("pooled", "argmax", "dx")):
        assert torch.equal(a, b), name
    assert int(outs[1][1].max()) <= 3


@pytest.mark.parametrize("src", ["bf16_idx", "u8_idx"])
def test_lenet_conv1_wgrad_gathered_input(dev, K, src):
    """LeNet conv1 weight gradient (convpool_wgrad_pair_k, the split backward path) reading a resident
    dataset through the batch index (bf16, or uint8 normalised in the kernel) == the fp32
    oracle on the gathered, normalised batch; several grids (images per block 1..n)."""
    torch.manual_seed(5)
    n, N = 300, 97
    u8 = torch.randint(0, 256, (n, 784), dtype=torch.uint8, device=dev)
    norm = (u8.float() / 255.0 - 0.5).to(torch.bfloat16)
    idx = torch.randint(0, n, (N,), dtype=torch.int64, device=dev)
    xb = norm[idx].view(N, 28, 28, 1)
    w = torch.zeros(5, 5, 1, 8, device=dev)
    w[..., :6] = torch.randn(5, 5, 1, 6, device=dev) / 5
    w = w.to(torch.bfloat16)
    b = torch.randn(6, device=dev) * 0.1
    pooled = torch.empty(N, 14, 14, 8, dtype=torch.bfloat16, device=dev)
    arg = torch.empty(N, 14, 14, 4, dtype=torch.uint8, device=dev)
    K.convpool_fwd(xb, w, b, 6, pooled, arg, N, 1, 8, 5, 2, 28, 28)
    xr = xb.float()
    wr = w.float().requires_grad_(True)
    br = torch.zeros(8, device=dev)
    br[:6] = b
    br.requires_grad_(True)
    y = conv_ref(xr, wr, br, "SAME", True)
    yp = F.max_pool2d(y.permute(0, 3, 1, 2), 2, 2).permute(0, 2, 3, 1)
    dP = rnd(N, 14, 14, 8, dev=dev)
    dP[..., 6:] = 0
    yp.backward(dP.float())
    KM = K.convpool_rows(1, 8, 5, 2, 28, 28)
    G, Ip, I, brow = K.convpool_reduce_args(1, 8, 5, 2, 28, 28, 1)
    kw = {"idx": idx, "u8": u8} if src == "u8_idx" else {"idx": idx}
    xin = norm if src == "bf16_idx" else xb
    for grid in (1, 13, 96):
        slab = torch.full((grid * KM * 8,), float("nan"), dtype=torch.float32, device=dev)
        K.convpool_wgrad(xin, dP, arg, slab, grid, N, 1, 8, 5, 2, 28, 28, **kw)
        dw = torch.empty(5, 5, 1, 6, device=dev)
        db = torch.empty(6, device=dev)
        K.splitk_reduce(slab, grid, KM, 8, G, Ip, I, 6, brow, dw, db, 1.0)
        close(dw, wr.grad[:, :, :1, :6], rel=3e-2)
        close(db, br.grad[:6], rel=3e-2)
