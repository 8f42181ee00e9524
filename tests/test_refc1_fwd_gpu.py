"""Reference-CNN conv1 forward with norm1 in the epilogue (csrc/kernels/lenet_band.hip
refc1n_fwd_k, refc1n3_fwd_k for 3 input channels): pool1 and its argmax codes bitwise the
round-5 kernel (refc1_band_fwd_k; 3 channels: the generic convpool kernel to bf16 rounding),
norm1 bitwise lrn_fwd_k over that pool1, both against an fp32 PyTorch oracle, and the whole
training step with the forward fold bitwise the step with the separate LRN launch.

Reference: /root/reference/mnist_input.py:136-153 (conv1 -> ReLU -> pool1 -> norm1:
tf.nn.lrn(pool1, 4, bias=1.0, alpha=0.001 / 9.0, beta=0.75)).
"""
import pytest
import torch

from distributed_tensorflow_ibm_mnist_amd.models import get_model, torch_ref
from distributed_tensorflow_ibm_mnist_amd.runtime.executor import HipNet
from distributed_tensorflow_ibm_mnist_amd.runtime.params import OptConfig

pytestmark = pytest.mark.gpu

LRN = dict(bias=1.0, alpha=0.001 / 9.0, beta=0.75)


def _inputs(dev, B, seed, src, cin=1):
    torch.manual_seed(seed)
    n = B + 37
    ds = (torch.rand(n, 784 * cin, device=dev) * 255).to(torch.uint8)
    xb = (ds.float() / 255.0 - 0.5).to(torch.bfloat16)
    idx = torch.randint(0, n, (B,), device=dev, dtype=torch.int64)
    w = (torch.randn(5, 5, cin, 32, device=dev) * 0.2).to(torch.bfloat16)
    b = torch.randn(32, device=dev) * 0.05
    if src == "batch":
        x, kw, xin = xb[idx].view(B, 28, 28, cin).contiguous(), {}, xb[idx]
    elif src == "bf16_ds":
        x, kw, xin = xb, {"idx": idx}, xb[idx]
    else:
        x, kw, xin = xb, {"u8": ds, "idx": idx}, xb[idx]
    return x, kw, xin.view(B, 28, 28, cin), w, b


def _fwd(K, x, kw, w, b, B, variant, norm=None, cin=1):
    K.refc1_set_fwd_variant(variant)
    try:
        P1 = torch.full((B, 14, 14, 32), 7.0, dtype=torch.bfloat16, device=x.device)
        A1 = torch.full((B, 14, 14, 32), 9, dtype=torch.uint8, device=x.device)
        lrn = {} if norm is None else dict(lrn_out=norm, lrn_bias=LRN["bias"], lrn_alpha=LRN["alpha"],
                                           lrn_beta=LRN["beta"], lrn_r=4)
        K.convpool_fwd(x, w, b, 32, P1, A1, B, cin, 32, 5, 2, 28, 28, **kw, **lrn)
        torch.cuda.synchronize()
        return P1, A1
    finally:
        K.refc1_set_fwd_variant(2)


@pytest.mark.parametrize("src", ["batch", "bf16_ds", "u8_ds"])
@pytest.mark.parametrize("B", [77, 4096])
def test_refc1n_pool1_bitwise_round5(dev, K, B, src, grid_cap):
    """pool1 + codes of the all-channels-per-wave kernel == the round-5 two-waves-per-unit
    kernel's (same MFMA sums, same pooling expressions), with and without norm1 written;
    B = 4096 at a capped grid runs several tiles per block."""
    grid_cap(64 if B > 1000 else 0)
    x, kw, _, w, b = _inputs(dev, B, 11, src)
    p_old, a_old = _fwd(K, x, kw, w, b, B, 1)
    p_new, a_new = _fwd(K, x, kw, w, b, B, 2)
    norm = torch.zeros(B, 14, 14, 32, dtype=torch.bfloat16, device=dev)
    p_lrn, a_lrn = _fwd(K, x, kw, w, b, B, 2, norm)
    assert torch.equal(p_new, p_old) and torch.equal(a_new, a_old)
    assert torch.equal(p_lrn, p_old) and torch.equal(a_lrn, a_old)


@pytest.mark.parametrize("src", ["batch", "bf16_ds"])
@pytest.mark.parametrize("B", [77, 4096])
def test_refc1n3_pool1_matches_convpool(dev, K, B, src, grid_cap):
    """3 input channels (refc1n3_fwd_k) vs the generic convpool kernel it replaces (MFMA sums in
    another order: pool1 to bf16 rounding, argmax codes equal except at near-ties), with and
    without norm1 written (pool1 / codes bitwise between those two)."""
    grid_cap(64 if B > 1000 else 0)
    x, kw, _, w, b = _inputs(dev, B, 13, src, cin=3)
    p_old, a_old = _fwd(K, x, kw, w, b, B, 1, cin=3)
    p_new, a_new = _fwd(K, x, kw, w, b, B, 2, cin=3)
    norm = torch.zeros(B, 14, 14, 32, dtype=torch.bfloat16, device=dev)
    p_lrn, a_lrn = _fwd(K, x, kw, w, b, B, 2, norm, cin=3)
    assert torch.equal(p_lrn, p_new) and torch.equal(a_lrn, a_new)
    d = (p_new.float() - p_old.float()).abs()
    assert d.max().item() <= 2 ** -7 * p_old.float().abs().max().item()
    assert (a_new != a_old).float().mean().item() < 2e-3


@pytest.mark.parametrize("cin", [1, 3])
@pytest.mark.parametrize("B", [77, 4096])
def test_refc1n_norm1_bitwise_lrn_fwd(dev, K, B, cin, grid_cap):
    """norm1 from the epilogue == lrn_fwd_k over the kernel's own pool1, bit for bit; pool1
    against an fp32 oracle (conv + bias + ReLU + 2x2 max-pool, bf16 rounding), norm1 against
    the fp32 TF-semantics LRN of that pool1."""
    grid_cap(64 if B > 1000 else 0)
    x, kw, xin, w, b = _inputs(dev, B, 12, "batch", cin)
    norm = torch.zeros(B, 14, 14, 32, dtype=torch.bfloat16, device=dev)
    P1, A1 = _fwd(K, x, kw, w, b, B, 2, norm, cin)
    ref = torch.empty_like(norm)
    K.lrn_fwd(P1, ref, B * 196, 32, 4, LRN["bias"], LRN["alpha"], LRN["beta"])
    torch.cuda.synchronize()
    assert torch.equal(norm, ref)
    # fp32 oracle of the forward
    y = torch.nn.functional.conv2d(xin.permute(0, 3, 1, 2).float(), w.float().permute(3, 2, 0, 1), padding=2)
    y = torch.relu(y + b.view(1, 32, 1, 1))
    pool = torch.nn.functional.max_pool2d(y, 2).permute(0, 2, 3, 1)
    assert (P1.float() - pool).abs().max().item() <= 0.01 * pool.abs().max().item() + 1e-3
    p = P1.float()
    sq = torch.nn.functional.pad(p * p, (4, 4))
    s = sum(sq[..., i:i + 32] for i in range(9))
    n32 = p * (LRN["bias"] + LRN["alpha"] * s) ** -LRN["beta"]
    assert (norm.float() - n32).abs().max().item() <= 2 ** -7 * n32.abs().max().item()
    assert int(A1.max()) <= 4


@pytest.mark.parametrize("cin", [1, 3])
def test_refcnn_norm1_forward_fold_step(dev, K, cin, monkeypatch):
    """A whole reference-CNN training step with norm1 written by conv1's launch
    (HipNet.fold_lrn_fwd1) == the step with the separate lrn_fwd launch: logits and every
    gradient bitwise; the LRN layer launches nothing in the folded net."""
    spec = get_model("reference_cnn", cin)
    init = torch_ref.init_params(spec, seed=6)
    B = 96
    x = (torch.rand(B, 28, 28, cin, device=dev) - 0.5).to(torch.bfloat16)
    y = torch.randint(0, 10, (B,), device=dev, dtype=torch.int32)

    def run(fold: str):
        monkeypatch.setenv("MNISTX_FOLD_LRN_FWD1", fold)
        net = HipNet(spec, B, dev, init, OptConfig(lr0=0.05))
        assert net.fold_lrn_fwd1 == (fold == "1")
        net.x0.copy_(x)
        net.labels.copy_(y)
        logits = net.forward(defer_head=True).clone()
        net.loss_and_grad()
        net.backward()
        torch.cuda.synchronize()
        return {"logits": logits, "norm1": net.activation("norm1").clone(),
                **{n: net.fp.grad_view(n).clone() for n in init}}

    ref, fold = run("0"), run("1")
    for k in ref:
        assert torch.equal(fold[k], ref[k]), k
