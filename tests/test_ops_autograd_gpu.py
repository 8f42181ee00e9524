"""The autograd layer (ops/autograd.py, ops/nn.py): HIP kernels as ordinary
PyTorch modules, checked against the fp32 oracle (models/torch_ref.py) --
logits, CE loss and every parameter gradient -- and driven by a stock
torch.optim optimizer."""
import pytest
import torch
import torch.nn.functional as F

from distributed_tensorflow_ibm_mnist_amd.models import get_model, torch_ref
from distributed_tensorflow_ibm_mnist_amd.ops import autograd as A
from distributed_tensorflow_ibm_mnist_amd.ops.nn import HipModel, SoftmaxCrossEntropy

pytestmark = pytest.mark.gpu


def rel_err(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@pytest.mark.parametrize("model,cin,fuse", [("lenet5", 1, True), ("lenet5", 1, False), ("reference_cnn", 3, True),
                                            ("reference_cnn", 1, False), ("mlp", 1, True)])
def test_hip_model_matches_oracle(dev, K, model, cin, fuse):
    torch.manual_seed(0)
    spec = get_model(model, cin)
    init = torch_ref.init_params(spec, seed=2)
    net = HipModel(spec, fuse_convpool=fuse).to(dev)
    net.load_tf_params({k: v.to(torch.bfloat16).float() for k, v in init.items()})
    B = 77                                              # odd batch: partial tiles everywhere
    x = (torch.rand(B, 28, 28, cin, device=dev) - 0.5).to(torch.bfloat16)
    y = torch.randint(0, 10, (B,), device=dev, dtype=torch.int32)
    crit = SoftmaxCrossEntropy(10)
    logits = net(x)
    loss = crit(logits, y)
    loss.backward()
    assert logits.shape[1] == 16 and logits[:, 10:].abs().max().item() == 0.0
    p = {k: v.to(dev).to(torch.bfloat16).float().requires_grad_(True) for k, v in init.items()}
    ref_logits, _ = torch_ref.forward(spec, p, x.float())
    assert rel_err(logits[:, :10], ref_logits) < 3e-2
    ce = F.cross_entropy(ref_logits, y.long())
    assert abs(loss.item() - ce.item()) < 2e-2 * max(1.0, ce.item())
    assert int(crit.last_stats[1].item()) == int((logits[:, :10].argmax(1) == y.long()).sum().item())
    ce.backward()
    p16 = {k: v.detach().clone().requires_grad_(True) for k, v in p.items()}
    with torch.autocast("cuda", dtype=torch.bfloat16):
        l16, _ = torch_ref.forward(spec, p16, x.float())
    F.cross_entropy(l16.float(), y.long()).backward()
    for name, prm in net.named_tf_parameters():
        e = rel_err(prm.grad, p[name].grad)
        floor = rel_err(p16[name].grad, p[name].grad)
        assert e < max(3e-2, 3.0 * floor), f"{model} {name}: rel err {e:.3e} (bf16 floor {floor:.3e})"


def test_torch_optimizer_trains_hip_model(dev, K):
    from distributed_tensorflow_ibm_mnist_amd.data.synthetic import make_synthetic
    spec = get_model("lenet5", 1)
    net = HipModel(spec).to(dev)
    net.load_tf_params(torch_ref.init_params(spec, seed=0))
    opt = torch.optim.SGD(net.parameters(), lr=0.05, momentum=0.9)
    crit = SoftmaxCrossEntropy(10)
    imgs, labs = make_synthetic(4096, seed=0, device=dev)
    x = imgs.view(-1, 28, 28, 1).float() / 255.0 - 0.5
    losses = []
    for i in range(60):
        sl = slice((i * 256) % 4096, (i * 256) % 4096 + 256)
        opt.zero_grad(set_to_none=True)
        loss = crit(net(x[sl]), labs[sl])
        loss.backward()
        opt.step()
        losses.append(loss.item())
    assert losses[-1] < 0.5 * losses[0], losses


def test_conv_dgrad_requires_padded_channels(dev, K):
    w = torch.randn(5, 5, 3, 8, device=dev, requires_grad=True)
    x = torch.randn(2, 8, 8, 3, device=dev, dtype=torch.bfloat16, requires_grad=True)
    y = A.conv2d(x, w, torch.zeros(8, device=dev), "SAME", True)
    with pytest.raises(NotImplementedError):
        y.float().sum().backward()
