"""LeNet-5 banded-MFMA conv stack (csrc/kernels/lenet_band.hip) against the fp32
PyTorch oracle and against the per-layer convpool kernels it replaces."""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _weights(dev, seed=3):
    g = torch.Generator(device="cpu").manual_seed(seed)
    w1 = torch.zeros(5, 5, 1, 8)
    w1[..., :6] = torch.randn(5, 5, 1, 6, generator=g) / 5.0
    b1 = torch.randn(6, generator=g) * 0.1
    w2 = torch.zeros(5, 5, 8, 16)
    w2[:, :, :6, :] = torch.randn(5, 5, 6, 16, generator=g) / math.sqrt(150)
    b2 = torch.randn(16, generator=g) * 0.1
    return (w1.to(dev, torch.bfloat16), b1.to(dev), w2.to(dev, torch.bfloat16), b2.to(dev))


def _conv_pool(x, w, b, pad):
    """fp32 oracle: NHWC conv (stride 1) + bias + ReLU + 2x2/2 max-pool."""
    y = F.conv2d(x.permute(0, 3, 1, 2).float(), w.float().permute(3, 2, 0, 1), b.float(), padding=pad)
    return F.max_pool2d(F.relu(y), 2, 2).permute(0, 2, 3, 1)


def _close(out, ref, rel=2e-2):
    err = (out.float() - ref.float()).abs().max().item()
    tol = rel * ref.float().abs().max().item() + 1e-6
    assert err <= tol, f"max err {err:.3e} > tol {tol:.3e}"


def _unpack1(arg1):   # byte k = code(c = k) | code(c = k + 4) << 4
    return torch.cat([arg1 & 15, arg1 >> 4], dim=-1)


def _combined(P1, A1):
    """The fused backward's pool1 records (lenet_band.hip P1OUT 2): per window channels 0-5
    of P1, then the window's 4-byte code word from A1 in the channel 6-7 slot."""
    B = P1.shape[0]
    c = P1.contiguous().clone()
    cb = c.view(torch.uint8).view(B * 196, 16)
    cb[:, 12:] = A1.contiguous().view(B * 196, 4)
    return c


def _band(K, x, w1, b1, w2, b2, B, idx=None, p1=True):
    dev = x.device
    P1 = torch.full((B, 14, 14, 8), 7.0, dtype=torch.bfloat16, device=dev)
    A1 = torch.full((B, 14, 14, 4), 0xEE, dtype=torch.uint8, device=dev)
    P2 = torch.full((B, 5, 5, 16), 7.0, dtype=torch.bfloat16, device=dev)
    A2 = torch.full((B, 5, 5, 16), 0xEE, dtype=torch.uint8, device=dev)
    if p1:
        K.lenet_band_fwd(x, w1, b1, 6, w2, b2, B, P2, A2, p1=P1, arg1=A1, idx=idx)
    else:
        K.lenet_band_fwd(x, w1, b1, 6, w2, b2, B, P2, A2, idx=idx)
    return P1, A1, P2, A2


@pytest.mark.parametrize("B,cap", [(1, 0), (3, 0), (16, 0), (17, 0), (100, 0), (1000, 0), (200, 4), (333, 3)])
def test_band_fwd_matches_oracle_and_convpool(dev, K, grid_cap, B, cap):
    """cap > 0: the grid is capped so every block runs several 8-image tiles (B=200, 4
    blocks: nk = 7; B=333, 3 blocks: a partial last tile) -- the double-buffered input /
    pool1 rings are reused, as at the benchmark batch (> 4096 images)."""
    grid_cap(cap)
    torch.manual_seed(B)
    w1, b1, w2, b2 = _weights(dev)
    x = (torch.rand(B, 28, 28, 1, device=dev) - 0.5).to(torch.bfloat16)
    P1, A1, P2, A2 = _band(K, x, w1, b1, w2, b2, B)
    # oracle, layer by layer (conv2 reads the kernel's own bf16 pool1)
    _close(P1, _conv_pool(x, w1, torch.cat([b1, torch.zeros(2, device=dev)]), 2))
    assert P1[..., 6:].abs().max().item() == 0
    _close(P2, _conv_pool(P1, w2, b2, 0))
    # the per-layer convpool kernels: same pooled values (bf16 rounding aside), same argmax
    # codes except at near-ties of the fp32 sums
    Q1 = torch.empty_like(P1)
    C1 = torch.empty_like(A1)
    K.convpool_fwd(x, w1, b1, 6, Q1, C1, B, 1, 8, 5, 2, 28, 28)
    Q2 = torch.empty_like(P2)
    C2 = torch.empty_like(A2)
    K.convpool_fwd(P1, w2, b2, 16, Q2, C2, B, 8, 16, 5, 0, 14, 14)
    _close(P1, Q1, rel=1e-2)
    _close(P2, Q2, rel=1e-2)
    c1, d1 = _unpack1(A1), _unpack1(C1)
    assert (c1 != d1).float().mean().item() < 2e-3
    assert (A2 != C2).float().mean().item() < 2e-3
    # ReLU mask folded into the codes: 4 exactly where the pooled output is 0
    assert torch.equal(c1 == 4, P1 == 0) and int(c1.max()) <= 4
    assert torch.equal(A2 == 4, P2 == 0) and int(A2.max()) <= 4


def test_band_fwd_dataset_gather(dev, K):
    """x = a resident dataset gathered through idx == the same rows passed as a batch;
    without p1 the pool2 outputs are unchanged."""
    torch.manual_seed(0)
    w1, b1, w2, b2 = _weights(dev, seed=5)
    n, B = 500, 77
    ds = (torch.rand(n, 784, device=dev) - 0.5).to(torch.bfloat16)
    idx = torch.randint(0, n, (B,), device=dev, dtype=torch.int64)
    P1, A1, P2, A2 = _band(K, ds, w1, b1, w2, b2, B, idx=idx)
    R1, S1, R2, S2 = _band(K, ds[idx].contiguous(), w1, b1, w2, b2, B)
    assert torch.equal(P1, R1) and torch.equal(A1, S1) and torch.equal(P2, R2) and torch.equal(A2, S2)
    # without p1 the pooling skips the argmax embedding (<= 3 ulp of fp32 apart)
    _, _, T2, U2 = _band(K, ds, w1, b1, w2, b2, B, idx=idx, p1=False)
    _close(T2, P2, rel=1e-2)
    assert (A2 != U2).float().mean().item() < 2e-3


def test_hipnet_band_step_matches_convpool(dev, K, monkeypatch):
    """A LeNet-5 training step with the banded forward == the same step on the
    per-layer convpool forward (loss to bf16 noise, parameters close)."""
    from distributed_tensorflow_ibm_mnist_amd.models import get_model, torch_ref
    from distributed_tensorflow_ibm_mnist_amd.runtime.executor import HipNet
    from distributed_tensorflow_ibm_mnist_amd.runtime.params import OptConfig

    spec = get_model("lenet5", 1)
    init = torch_ref.init_params(spec, seed=1)
    g = torch.Generator(device=dev).manual_seed(2)
    x = (torch.rand(256, 28, 28, 1, device=dev, generator=g) - 0.5).to(torch.bfloat16)
    y = torch.randint(0, 10, (256,), device=dev, generator=g, dtype=torch.int32)
    res = []
    for band in ("1", "0"):
        monkeypatch.setenv("MNISTX_BAND_FWD", band)
        net = HipNet(spec, 256, dev, init, OptConfig(lr0=0.05, use_momentum=True, momentum=0.9))
        assert net.band_fwd == (band == "1")
        losses = []
        for _ in range(3):
            net.x0.copy_(x)
            net.labels.copy_(y)
            net.train_step()
            losses.append(net.read_stats()["cross_entropy"])
        res.append((losses, net.fp.params.clone()))
    (l_a, p_a), (l_b, p_b) = res
    for a, b in zip(l_a, l_b):
        assert abs(a - b) < 2e-2 * max(1.0, abs(b)), (l_a, l_b)
    assert (p_a - p_b).abs().max().item() < 5e-3


@pytest.mark.parametrize("B,cap", [(1, 0), (100, 0), (1000, 0), (333, 3)])
def test_band_fwd_combined_records(dev, K, grid_cap, B, cap):
    """p1 without arg1: one 16-byte record per pool1 window (what lenet_bwd reads) ==
    the convpool-layout outputs recombined, bitwise; pool2 outputs unchanged."""
    grid_cap(cap)
    torch.manual_seed(B)
    w1, b1, w2, b2 = _weights(dev)
    x = (torch.rand(B, 28, 28, 1, device=dev) - 0.5).to(torch.bfloat16)
    P1, A1, P2, A2 = _band(K, x, w1, b1, w2, b2, B)
    R = torch.full((B, 14, 14, 8), 7.0, dtype=torch.bfloat16, device=dev)
    Q2 = torch.empty_like(P2)
    C2 = torch.empty_like(A2)
    K.lenet_band_fwd(x, w1, b1, 6, w2, b2, B, Q2, C2, p1=R)
    assert torch.equal(R.view(torch.uint8), _combined(P1, A1).view(torch.uint8))
    assert torch.equal(Q2, P2) and torch.equal(C2, A2)
