"""LeNet-5 conv-stack backward as one kernel (csrc/kernels/lenet_bwd.hip) against an fp32
PyTorch oracle of the same math (the forward's own argmax codes unpool the gradients, so
ties cannot differ) and against the three per-layer convpool kernels it replaces.

Reference: the backward of /root/reference/mnist_input.py:136-172 (conv blocks) produced
by compute_gradients (mnist_input.py:262), on the LeNet-5 geometry of the BASELINE config.
"""
import pytest
import torch
import torch.nn.functional as F

from test_lenet_band_gpu import _band, _combined, _weights

pytestmark = pytest.mark.gpu


def _unpool(dP, codes):
    """[B, H, W, C] pooled gradient + window-position codes (2a + b; 4 = ReLU off) ->
    [B, 2H, 2W, C] (fp32)."""
    B, H, W, C = dP.shape
    out = torch.zeros(B, 2 * H, 2 * W, C, device=dP.device)
    for d in range(4):
        out[:, d >> 1::2, d & 1::2, :] = torch.where(codes == d, dP.float(), torch.zeros((), device=dP.device))
    return out


def _oracle(x, P1, A1, A2, dP2, w2):
    """fp32: dY2 = unpool(dP2) -> dW2, db2, dP1 (conv2 VALID); dY1 = unpool(bf16(dP1)) ->
    dW1, db1 (conv1 SAME).  dP1 is rounded to bf16 as the kernels stage it."""
    B = x.shape[0]
    c1 = torch.cat([A1 & 15, A1 >> 4], dim=-1)                       # [B, 14, 14, 8]
    dY2 = _unpool(dP2.view(B, 5, 5, 16), A2.view(B, 5, 5, 16).long())  # [B, 10, 10, 16]
    g2 = dY2.permute(0, 3, 1, 2)
    p1 = P1.float().permute(0, 3, 1, 2)
    wt2 = w2.float().permute(3, 2, 0, 1)                              # [16, 8, 5, 5]
    dW2 = torch.nn.grad.conv2d_weight(p1, wt2.shape, g2).permute(2, 3, 1, 0)   # [5, 5, 8, 16]
    db2 = g2.sum((0, 2, 3))
    dP1 = torch.nn.grad.conv2d_input(p1.shape, wt2, g2).permute(0, 2, 3, 1)   # [B, 14, 14, 8]
    dY1 = _unpool(dP1.to(torch.bfloat16), c1.long())                   # [B, 28, 28, 8]
    g1 = dY1.permute(0, 3, 1, 2)
    dW1 = torch.nn.grad.conv2d_weight(x.float().permute(0, 3, 1, 2), (8, 1, 5, 5), g1, padding=2).permute(2, 3, 1, 0)
    db1 = _unpool(dP1, c1.long()).sum((0, 1, 2))                      # fp32 dP1 (the kernel's bias path)
    return dW1[:, :, 0, :6], db1[:6], dW2[:, :, :6, :], db2


def _fused(K, x, P1, A1, A2, dP2, w2, B, idx=None, xsrc=None):
    grid = K.lenet_bwd_blocks(B)
    s1 = torch.full((grid * 32 * 8,), float("nan"), device=x.device)
    s2 = torch.full((grid * 208 * 16,), float("nan"), device=x.device)
    K.lenet_bwd(x if xsrc is None else xsrc, _combined(P1, A1), dP2, A2, w2, B, s1, s2, grid, idx=idx)
    dW1 = torch.empty(5, 5, 1, 6, device=x.device)
    db1 = torch.empty(6, device=x.device)
    dW2 = torch.empty(5, 5, 6, 16, device=x.device)
    db2 = torch.empty(16, device=x.device)
    K.splitk_reduce(s2, grid, 208, 16, 25, 8, 6, 16, 200, dW2, db2, 1.0)
    K.splitk_reduce(s1, grid, 32, 8, 25, 1, 1, 6, 25, dW1, db1, 1.0)
    return dW1[:, :, 0, :], db1, dW2, db2, grid


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def _setup(dev, K, B, seed):
    torch.manual_seed(seed)
    w1, b1, w2, b2 = _weights(dev, seed=seed)
    x = (torch.rand(B, 28, 28, 1, device=dev) - 0.5).to(torch.bfloat16)
    P1, A1, P2, A2 = _band(K, x, w1, b1, w2, b2, B)
    dP2 = (torch.randn(B, 400, device=dev) * 0.1).to(torch.bfloat16)
    return x, w1, w2, P1, A1, A2, dP2


@pytest.mark.parametrize("B,cap", [(1, 0), (8, 0), (13, 0), (100, 0), (1000, 0), (200, 3), (1000, 5), (77, 2)])
def test_lenet_bwd_matches_oracle(dev, K, grid_cap, B, cap):
    """cap > 0: few persistent blocks, each over many 8-image tiles (the next tile's data
    prefetched during this one, accumulators carried across tiles) -- the benchmark path."""
    grid_cap(cap)
    x, w1, w2, P1, A1, A2, dP2 = _setup(dev, K, B, seed=B + cap)
    got = _fused(K, x, P1, A1, A2, dP2, w2, B)
    if cap:
        assert got[4] == min(cap, (B + 7) // 8)
    want = _oracle(x, P1, A1, A2, dP2, w2)
    for name, g, w in zip(("dW1", "db1", "dW2", "db2"), got[:4], want):
        assert g.shape == w.shape, (name, g.shape, w.shape)
        assert torch.isfinite(g).all(), name
        assert _rel(g, w) < 1e-2, f"{name}: rel err {_rel(g, w):.3e}"


def test_lenet_bwd_matches_convpool_kernels(dev, K):
    """Same gradients as the per-layer path (convpool dgrad -> dP1 in HBM, then the two
    weight-gradient kernels): the kernels it replaces."""
    B = 512
    x, w1, w2, P1, A1, A2, dP2 = _setup(dev, K, B, seed=5)
    dW1, db1, dW2, db2, _ = _fused(K, x, P1, A1, A2, dP2, w2, B)
    dP1 = torch.empty(B, 14, 14, 8, dtype=torch.bfloat16, device=dev)
    K.convpool_dgrad(dP2.view(B, 5, 5, 16), A2, w2, dP1, B, 8, 16, 5, 0, 14, 14)
    outs = []
    for xin, dP, arg, cin, cout, pad, hw, ci, co in ((P1, dP2.view(B, 5, 5, 16), A2, 8, 16, 0, 14, 6, 16),
                                                     (x, dP1, A1, 1, 8, 2, 28, 1, 6)):
        KM = K.convpool_rows(cin, cout, 5, pad, hw, hw)
        grid = 64
        slab = torch.empty(grid * KM * cout, device=dev)
        K.convpool_wgrad(xin, dP, arg, slab, grid, B, cin, cout, 5, pad, hw, hw)
        G, Ip, I, brow = K.convpool_reduce_args(cin, cout, 5, pad, hw, hw, ci)
        dw = torch.empty(5, 5, ci, co, device=dev)
        db = torch.empty(co, device=dev)
        K.splitk_reduce(slab, grid, KM, cout, G, Ip, I, co, brow, dw, db, 1.0)
        outs.append((dw, db))
    (rW2, rb2), (rW1, rb1) = outs
    assert _rel(dW2, rW2) < 1e-2 and _rel(db2, rb2) < 1e-2
    assert _rel(dW1, rW1[:, :, 0, :]) < 2e-2 and _rel(db1, rb1) < 2e-2


@pytest.mark.parametrize("src", ["bf16_idx", "u8_idx"])
def test_lenet_bwd_gathered_input(dev, K, src):
    """The input read through the batch index from a resident dataset (bf16 normalised once,
    or uint8 normalised in the kernel) == the same rows passed as a batch, bitwise."""
    torch.manual_seed(4)
    n, B = 700, 150
    w1, b1, w2, b2 = _weights(dev, seed=4)
    from distributed_tensorflow_ibm_mnist_amd.data.device_loader import DeviceDataset
    u8 = torch.randint(0, 256, (n, 784), device=dev, dtype=torch.uint8)
    # normalised by the K10 kernel: bitwise what the uint8 path computes while staging
    ds = DeviceDataset(u8, torch.zeros(n, dtype=torch.int32), dev, hw=784, channels=1).bf16_images()
    idx = torch.randint(0, n, (B,), device=dev, dtype=torch.int64)
    x = ds[idx].contiguous().view(B, 28, 28, 1)
    P1, A1, P2, A2 = _band(K, x, w1, b1, w2, b2, B)
    dP2 = (torch.randn(B, 400, device=dev) * 0.1).to(torch.bfloat16)
    ref = _fused(K, x, P1, A1, A2, dP2, w2, B)
    got = _fused(K, x, P1, A1, A2, dP2, w2, B, idx=idx, xsrc=ds if src == "bf16_idx" else u8)
    for a, b in zip(got[:4], ref[:4]):
        assert torch.equal(a, b)
