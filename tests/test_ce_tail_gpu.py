"""Reference-CNN softmax tail (csrc/kernels/mlp_head.hip ce_tail_k): softmax_linear (192 -> 10)
+ softmax cross-entropy + dL/d local4 (masked by local4 > 0) in one launch, checked against an
fp32 PyTorch oracle of the same op and, as a whole training step, against the layered plan
(dense GEMM + softmax_ce + dgrad GEMM, MNISTX_CE_TAIL=0); odd batch sizes cover partial waves
and blocks.

Reference: /root/reference/mnist_input.py:195-205 (softmax_linear), :226-234 (cross-entropy).
"""
import pytest
import torch

from distributed_tensorflow_ibm_mnist_amd.models import get_model, torch_ref
from distributed_tensorflow_ibm_mnist_amd.runtime.executor import HipNet
from distributed_tensorflow_ibm_mnist_amd.runtime.params import OptConfig

pytestmark = pytest.mark.gpu


def rel_err(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@pytest.mark.parametrize("nb", [1, 77, 1000, 4099])
def test_ce_tail_matches_oracle(dev, K, nb):
    torch.manual_seed(nb)
    x = torch.relu(torch.randn(nb, 192, device=dev)).to(torch.bfloat16)
    w = (torch.randn(192, 10, device=dev) * 0.2).to(torch.bfloat16)
    wt = torch.zeros(16, 192, dtype=torch.bfloat16, device=dev)
    wt[:10] = w.t()
    b = torch.randn(10, device=dev) * 0.1
    y = torch.randint(0, 10, (nb,), device=dev, dtype=torch.int32)
    logits = torch.full((nb, 16), 7.0, device=dev)
    dl = torch.full((nb, 16), 3.0, dtype=torch.bfloat16, device=dev)
    dx = torch.full((nb, 192), 5.0, dtype=torch.bfloat16, device=dev)
    stats = torch.zeros(8, device=dev)
    work = torch.zeros(4 * 1024 + 1, device=dev)
    nblk = K.ce_tail_blocks(nb)
    dbias = torch.full((nblk * 16,), 9.0, device=dev)
    scale = 1.0 / nb
    K.ce_tail(x, wt, b, 10, y, nb, scale, logits, dl=dl, dx=dx, stats=stats, work=work, dbias=dbias)
    torch.cuda.synchronize()
    ref = x.float() @ w.float() + b
    assert (logits[:, :10] - ref).abs().max().item() <= 1e-4 * ref.abs().max().item() + 1e-5
    assert not logits[:, 10:].any()
    g = (torch.softmax(ref, 1) - torch.nn.functional.one_hot(y.long(), 10).float()) * scale
    assert (dl[:, :10].float() - g).abs().max().item() <= 2 ** -8 * g.abs().max().item()
    assert not dl[:, 10:].any()
    # the data gradient from the kernel's own bf16 dlogits, masked by the ReLU output
    gx = (dl[:, :10].float() @ w.float().t()) * (x.float() > 0)
    assert (dx.float() - gx).abs().max().item() <= 2 ** -7 * gx.abs().max().item()
    assert not dx[x == 0].any()
    db = dbias.view(nblk, 16).sum(0)
    assert (db[:10] - g.sum(0)).abs().max().item() <= 1e-2 * g.abs().sum(0).max().item() + 1e-6
    ce = torch.nn.functional.cross_entropy(ref, y.long(), reduction="sum").item()
    assert abs(stats[0].item() - ce) <= 1e-4 * abs(ce) + 1e-4
    assert abs(stats[1].item() - (ref.argmax(1) == y.long()).sum().item()) <= 2
    # eval form: logits + statistics only
    logits2 = torch.zeros_like(logits)
    st2 = torch.zeros(8, device=dev)
    K.ce_tail(x, wt, b, 10, y, nb, 1.0, logits2, stats=st2, work=work)
    torch.cuda.synchronize()
    assert torch.equal(logits2, logits) and torch.equal(st2[:2], stats[:2])


def _net(dev, B, fused, monkeypatch, cin=1):
    monkeypatch.setenv("MNISTX_CE_TAIL", "1" if fused else "0")
    spec = get_model("reference_cnn", cin)
    init = torch_ref.init_params(spec, seed=B)
    net = HipNet(spec, B, dev, init, OptConfig(lr0=0.05))
    assert (net.head_kind == "tail") == fused
    return net, init


def _step(net, x, y):
    net.x0.copy_(x)
    net.labels.copy_(y)
    net.stats.zero_()
    net.forward(defer_head=True)
    net.loss_and_grad()
    net.backward()
    net.finalize(net.B, increment=False)
    torch.cuda.synchronize()


@pytest.mark.parametrize("B", [96, 301])
def test_ce_tail_step_matches_layered(dev, K, B, monkeypatch):
    """The whole training step with the fused tail == the layered one: logits, dlogits, the
    local4 data gradient and every weight gradient to bf16 rounding, loss / accuracy."""
    g = torch.Generator(device="cpu").manual_seed(B)
    x = (torch.rand(B, 28, 28, 1, generator=g) - 0.5).to(torch.bfloat16).to(dev)
    y = torch.randint(0, 10, (B,), generator=g, dtype=torch.int32).to(dev)
    fused, init = _net(dev, B, True, monkeypatch)
    layered, _ = _net(dev, B, False, monkeypatch)
    _step(fused, x, y)
    _step(layered, x, y)
    i = fused.head
    assert rel_err(fused.logits[:, :10], layered.logits[:, :10]) < 1e-3
    assert rel_err(fused.dlogits[:, :10], layered.dlogits[:, :10]) < 1e-2
    assert rel_err(fused.dbuf[i], layered.dbuf[i]) < 2e-2
    for name in init:
        e = rel_err(fused.fp.grad_view(name), layered.fp.grad_view(name))
        assert e < 2e-2, (name, e)
    sf, sl = fused.stats.cpu(), layered.stats.cpu()
    assert abs(sf[4] - sl[4]) <= 1e-3 * abs(sl[4]) + 1e-3 / B
    assert abs(sf[5] - sl[5]) * B <= 2
    # deterministic, and eval through the fused kernel == layered eval
    d0, g0 = fused.dbuf[i].clone(), fused.fp.grads.clone()
    _step(fused, x, y)
    assert torch.equal(fused.dbuf[i], d0) and torch.equal(fused.fp.grads, g0)
    fused.eval_stats.zero_()
    layered.eval_stats.zero_()
    fused.eval_batch(B)
    layered.eval_batch(B)
    a, b = fused.eval_stats.cpu(), layered.eval_stats.cpu()
    assert abs(a[0] - b[0]) <= 1e-3 * abs(b[0]) and abs(a[1] - b[1]) <= 2
