"""Reference-CNN conv1 weight gradient with the norm1 backward folded in
(csrc/kernels/refc1_wgrad.hip) against an fp32 PyTorch oracle (LRN backward by autograd,
rounded to bf16 as the kernel stages it, un-pooled through the forward's own codes) and
against the folded convpool_wgrad it replaces.

Reference: the backward of /root/reference/mnist_input.py:142-151 (conv1 -> ReLU -> pool1
-> norm1) produced by compute_gradients (mnist_input.py:262).
"""
import pytest
import torch

from test_lenet_bwd_gpu import _rel, _unpool

pytestmark = pytest.mark.gpu

LRN = dict(bias=1.0, alpha=0.001 / 9.0, beta=0.75)   # mnist_input.py:151


def _lrn_bwd_oracle(p, g, r=4):
    """dL/d(LRN input) of tf.nn.local_response_normalization over channels (fp32 autograd)."""
    x = p.float().requires_grad_(True)
    sq = torch.nn.functional.pad(x * x, (r, r))
    s = sum(sq[..., i:i + x.shape[-1]] for i in range(2 * r + 1))
    y = x * (LRN["bias"] + LRN["alpha"] * s) ** -LRN["beta"]
    y.backward(g.float())
    return x.grad


def _setup(dev, K, B, seed, cin=1):
    torch.manual_seed(seed)
    x = (torch.rand(B, 28, 28, cin, device=dev) - 0.5).to(torch.bfloat16)
    w = (torch.randn(5, 5, cin, 32, device=dev) * 0.2).to(torch.bfloat16)
    b = torch.randn(32, device=dev) * 0.05
    P1 = torch.empty(B, 14, 14, 32, dtype=torch.bfloat16, device=dev)
    A1 = torch.empty(B, 14, 14, 32, dtype=torch.uint8, device=dev)
    K.convpool_fwd(x, w, b, 32, P1, A1, B, cin, 32, 5, 2, 28, 28)
    dn = (torch.randn(B, 14, 14, 32, device=dev) * 0.1).to(torch.bfloat16)
    return x, P1, A1, dn


def _reduce(K, slab, grid, dev, cin=1):
    G, Ip, I, brow = K.convpool_reduce_args(cin, 32, 5, 2, 28, 28, cin)
    dw = torch.empty(5, 5, cin, 32, device=dev)
    db = torch.empty(32, device=dev)
    K.splitk_reduce(slab, grid, K.convpool_rows(cin, 32, 5, 2, 28, 28), 32, G, Ip, I, 32, brow, dw, db, 1.0)
    return dw, db


def _refc1(K, x, P1, A1, dn, B, cin=1, **src):
    grid = K.refc1_wgrad_blocks(B)
    slab = torch.full((grid * (48 if cin == 1 else 80) * 32,), float("nan"), device=P1.device)
    K.refc1_wgrad(x, dn, P1, A1, slab, grid, B, LRN["bias"], LRN["alpha"], LRN["beta"], **src, cin=cin)
    return (*_reduce(K, slab, grid, P1.device, cin), grid)


@pytest.mark.parametrize("B,cap,cin", [(1, 0, 1), (5, 0, 1), (100, 0, 1), (1000, 0, 1), (333, 3, 1), (77, 2, 1),
                                       (4096, 7, 1), (1, 0, 3), (100, 0, 3), (1000, 0, 3), (333, 3, 3),
                                       (4096, 7, 3)])
def test_refc1_wgrad_matches_oracle(dev, K, grid_cap, B, cap, cin):
    """cap > 0: few persistent blocks over many 4-image tiles (next tile prefetched, partial
    last tile, accumulators carried) -- the benchmark path.  cin 3: the reference's
    3-channel records (input planes de-interleaved while staging, the GEMM per plane)."""
    grid_cap(cap)
    x, P1, A1, dn = _setup(dev, K, B, seed=B + cap, cin=cin)
    dw, db, grid = _refc1(K, x, P1, A1, dn, B, cin=cin)
    if cap:
        assert grid == min(cap, (B + 3) // 4)
    dP1 = _lrn_bwd_oracle(P1, dn)
    dY = _unpool(dP1.to(torch.bfloat16), A1.long())                 # the kernel stages bf16 dP1
    g = dY.permute(0, 3, 1, 2)
    want_w = torch.nn.grad.conv2d_weight(x.float().permute(0, 3, 1, 2), (32, cin, 5, 5), g, padding=2)
    want_w = want_w.permute(2, 3, 1, 0)
    want_b = g.sum((0, 2, 3))
    assert torch.isfinite(dw).all() and torch.isfinite(db).all()
    assert _rel(dw, want_w) < 1e-2, _rel(dw, want_w)
    assert _rel(db, want_b) < 1e-2, _rel(db, want_b)


def test_refc1_wgrad_matches_convpool_fold(dev, K):
    """Same gradient as convpool_wgrad with the LRN fold (same lrn_bwd8 arithmetic and bf16
    rounding; fp32 sums in another order)."""
    B = 2000
    x, P1, A1, dn = _setup(dev, K, B, seed=11)
    dw, db, _ = _refc1(K, x, P1, A1, dn, B)
    again = _refc1(K, x, P1, A1, dn, B)
    assert torch.equal(dw, again[0]) and torch.equal(db, again[1]), "not deterministic"
    grid = 64
    slab = torch.empty(grid * K.convpool_rows(1, 32, 5, 2, 28, 28) * 32, device=dev)
    K.convpool_wgrad(x, dn, A1, slab, grid, B, 1, 32, 5, 2, 28, 28, lrn_p=P1, lrn_bias=LRN["bias"],
                     lrn_alpha=LRN["alpha"], lrn_beta=LRN["beta"], lrn_r=4)
    rw, rb = _reduce(K, slab, grid, dev)
    assert _rel(dw, rw) < 1e-4, _rel(dw, rw)
    assert _rel(db, rb) < 1e-4, _rel(db, rb)


@pytest.mark.parametrize("src", ["bf16_idx", "u8_idx"])
def test_refc1_wgrad_gathered_input(dev, K, src):
    """The input read through the batch index from a resident dataset (bf16 normalised once,
    or uint8 normalised in the kernel) == the same rows passed as a batch, bitwise."""
    torch.manual_seed(4)
    n, B = 700, 150
    from distributed_tensorflow_ibm_mnist_amd.data.device_loader import DeviceDataset
    u8 = torch.randint(0, 256, (n, 784), device=dev, dtype=torch.uint8)
    ds = DeviceDataset(u8, torch.zeros(n, dtype=torch.int32), dev, hw=784, channels=1).bf16_images()
    idx = torch.randint(0, n, (B,), device=dev, dtype=torch.int64)
    x = ds[idx].contiguous().view(B, 28, 28, 1)
    _, P1, A1, dn = _setup(dev, K, B, seed=4)
    ref = _refc1(K, x, P1, A1, dn, B)
    if src == "bf16_idx":
        got = _refc1(K, ds, P1, A1, dn, B, idx=idx)
    else:
        got = _refc1(K, x, P1, A1, dn, B, u8=u8, idx=idx)
    assert torch.equal(got[0], ref[0]) and torch.equal(got[1], ref[1])
