"""Fused LeNet-5 dense head (csrc/kernels/mlp_head.hip): fc3/fc4/fc5 + softmax-CE
+ data gradients in one kernel, checked against the layered kernels (dense GEMMs
+ softmax_ce, which the oracle tests pin to fp32 PyTorch) and against the fp32
oracle directly; odd batch sizes cover partial waves and blocks."""
import pytest
import torch
import torch.nn.functional as F

from distributed_tensorflow_ibm_mnist_amd.models import get_model, torch_ref
from distributed_tensorflow_ibm_mnist_amd.runtime.executor import HipNet
from distributed_tensorflow_ibm_mnist_amd.runtime.params import OptConfig

pytestmark = pytest.mark.gpu


def rel_err(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def _pair(dev, B, seed=0):
    spec = get_model("lenet5", 1)
    init = torch_ref.init_params(spec, seed=seed + 1)
    opt = OptConfig(lr0=0.05, decay_steps=0, use_momentum=False, ema_max=0.9999)
    fused = HipNet(spec, B, dev, init, opt)
    layered = HipNet(spec, B, dev, init, opt, fuse_head=False)
    g = torch.Generator(device="cpu").manual_seed(seed)
    x = (torch.rand(B, 28, 28, 1, generator=g) - 0.5).to(torch.bfloat16).to(dev)
    y = torch.randint(0, 10, (B,), generator=g, dtype=torch.int32).to(dev)
    for n in (fused, layered):
        n.x0.copy_(x)
        n.labels.copy_(y)
    return spec, init, fused, layered, x, y


def _step(net):
    net.forward(defer_head=True)
    net.loss_and_grad()
    net.backward()
    # the fused head leaves per-block CE partials that the step's finalize_k combines
    # (deferred statistics): read the finalized mean loss / accuracy (stats[4], [5])
    net.finalize(net.B, increment=False)
    torch.cuda.synchronize()


def test_head_selected(dev, K):
    _, _, fused, layered, _, _ = _pair(dev, 64)
    assert fused.head == len(fused.layers) - 3 and layered.head is None
    # other models keep the layered head
    assert HipNet(get_model("mlp", 1), 64, dev, torch_ref.init_params(get_model("mlp", 1), seed=0)).head is None


@pytest.mark.parametrize("B", [64, 300, 4099])
def test_fused_head_matches_layered(dev, K, B):
    spec, init, fused, layered, _, _ = _pair(dev, B, seed=B)
    _step(fused)
    _step(layered)
    i = fused.head
    assert rel_err(fused.logits[:B, :10], layered.logits[:B, :10]) < 1e-2
    assert torch.all(fused.logits[:B, 10:] == 0)
    for j in (i, i + 1):   # h3, h4 (bf16, padded columns zero)
        a, b = fused.layers[j].out[:B], layered.layers[j].out[:B]
        assert rel_err(a, b) < 1e-2, j
        assert torch.all(a[:, fused.layers[j].spec.dout:] == 0)
    assert rel_err(fused.dlogits[:B], layered.dlogits[:B]) < 1e-2
    for j in (i, i + 1, i + 2):   # dX, dh3, dh4
        e = rel_err(fused.dbuf[j][:B], layered.dbuf[j][:B])
        assert e < 2e-2, (j, e)
    for name in init:
        e = rel_err(fused.fp.grad_view(name), layered.fp.grad_view(name))
        assert e < 2e-2, (name, e)
    sf, sl = fused.stats.cpu(), layered.stats.cpu()
    assert abs(sf[4] - sl[4]) <= 1e-3 * abs(sl[4]) + 1e-3 / B
    assert abs(sf[5] - sl[5]) * B <= 2    # argmax ties can flip on rounding
    assert sf[2] == 0 and sf[0] == 0 and sf[1] == 0


def test_fused_head_matches_oracle(dev, K):
    B = 200
    spec, init, fused, _, x, y = _pair(dev, B, seed=7)
    _step(fused)
    p = {k: v.to(dev).to(torch.bfloat16).float().requires_grad_(True) for k, v in init.items()}
    ref_logits, _ = torch_ref.forward(spec, p, x.float())
    assert rel_err(fused.logits[:, :10], ref_logits) < 3e-2
    F.cross_entropy(ref_logits, y.long()).backward()
    p16 = {k: v.detach().clone().requires_grad_(True) for k, v in p.items()}
    with torch.autocast("cuda", dtype=torch.bfloat16):
        l16, _ = torch_ref.forward(spec, p16, x.float())
    F.cross_entropy(l16.float(), y.long()).backward()
    for name in init:
        e = rel_err(fused.fp.grad_view(name), p[name].grad)
        floor = rel_err(p16[name].grad, p[name].grad)
        assert e < max(3e-2, 3.0 * floor), f"{name}: rel err {e:.3e} (bf16 floor {floor:.3e})"
    ce = F.cross_entropy(ref_logits, y.long(), reduction="sum").item()
    assert abs(fused.stats[4].item() * B - ce) < 2e-2 * ce


def test_fused_head_deterministic_and_eval(dev, K):
    B = 1000
    _, _, fused, layered, _, _ = _pair(dev, B, seed=3)
    outs = []
    for _ in range(2):
        fused.stats.zero_()
        _step(fused)
        outs.append((fused.dbuf[fused.head].clone(), fused.fp.grads.clone(), fused.stats.clone()))
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    # eval (no gradients) through the fused kernel == layered eval
    fused.eval_stats.zero_()
    layered.eval_stats.zero_()
    fused.eval_batch(B)
    layered.eval_batch(B)
    a, b = fused.eval_stats.cpu(), layered.eval_stats.cpu()
    assert abs(a[0] - b[0]) <= 1e-3 * abs(b[0]) and abs(a[1] - b[1]) <= 2


def test_transposed_copies_track_optimizer(dev, K):
    """FlatParams.enable_transposed: the fused optimizer keeps W^T bf16 copies (zero
    padded) equal to the transposed padded bf16 weights after every update."""
    B = 128
    _, _, fused, _, _, _ = _pair(dev, B, seed=5)
    for _ in range(2):
        _step(fused)
        fused.update()
    torch.cuda.synchronize()
    fp = fused.fp
    assert len(fp.bft) == 3
    for name in fp.bft:
        e = fp.by_name[name]
        t = fp.bf16t_view(name)
        assert torch.equal(t[:e.J, :e.I], fp.bf16_view(name)[:e.I, :e.J].t())
        assert torch.equal(t[:e.J, :e.I], fp.param_view(name).to(torch.bfloat16).t())
        assert not t[e.J:].any() and not t[:, e.I:].any()
