"""T3/T4: the whole HIP execution plan (fwd + explicit bwd + fused update) vs the
fp32 PyTorch oracle, per model; plus a short end-to-end training run."""
import pytest
import torch
import torch.nn.functional as F

from distributed_tensorflow_ibm_mnist_amd.models import get_model
from distributed_tensorflow_ibm_mnist_amd.models import torch_ref
from distributed_tensorflow_ibm_mnist_amd.runtime.executor import HipNet
from distributed_tensorflow_ibm_mnist_amd.runtime.params import OptConfig

pytestmark = pytest.mark.gpu


def rel_err(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


ORACLE_CHUNK = 96     # = test_step_matches_oracle's batch: its MIOpen kernels are already built


def _check_step(dev, model, cin, B, defer_head=False, seed=0, last_bias_tol=None):
    """One training step of the HIP plan vs the fp32 oracle: logits, every gradient (within
    3x the bf16 autocast noise floor), the fused update and the loss statistics.
    ``defer_head``: the bench / train_step path (fused head runs inside loss_and_grad)."""
    torch.manual_seed(seed)
    spec = get_model(model, cin)
    init = torch_ref.init_params(spec, seed=1)
    opt = OptConfig(lr0=0.05, decay_steps=0, use_momentum=False, ema_max=0.9999)
    net = HipNet(spec, B, dev, init, opt)
    x = (torch.rand(B, 28, 28, cin, device=dev) - 0.5).to(torch.bfloat16)
    y = torch.randint(0, 10, (B,), device=dev, dtype=torch.int32)
    net.x0.copy_(x)
    net.labels.copy_(y)
    if defer_head:
        net.forward(defer_head=True)
        net.loss_and_grad()
        logits = net.logits[:, :10].clone()
    else:
        logits = net.forward()[:, :10].clone()
        net.loss_and_grad()
    net.backward()
    # oracle on the same bf16-rounded weights, in chunks of ORACLE_CHUNK rows (the last one
    # padded with zero-weight rows): every MIOpen call has one shape, whatever B is
    p = {k: v.to(dev).to(torch.bfloat16).float().requires_grad_(True) for k, v in init.items()}
    # bf16 noise floor: the same oracle under bf16 autocast (bf16 activations and
    # gradients, fp32 accumulation) — gradient sums with heavy cancellation (first
    # layer at random init) are ill-conditioned, so compare against that floor.
    p16 = {k: v.detach().clone().requires_grad_(True) for k, v in p.items()}
    ref_logits = torch.empty(B, 10, device=dev)
    ce_sum = 0.0
    for c0 in range(0, B, ORACLE_CHUNK):
        n = min(ORACLE_CHUNK, B - c0)
        xs, ys = x[c0:c0 + n], y[c0:c0 + n].long()
        wts = torch.ones(ORACLE_CHUNK, device=dev)
        if n < ORACLE_CHUNK:
            xs = torch.cat([xs, xs[:1].expand(ORACLE_CHUNK - n, *xs.shape[1:])])
            ys = torch.cat([ys, ys[:1].expand(ORACLE_CHUNK - n)])
            wts[n:] = 0.0
        lg, _ = torch_ref.forward(spec, p, xs.float())
        ref_logits[c0:c0 + n] = lg[:n].detach()
        ce = (F.cross_entropy(lg, ys, reduction="none") * wts).sum() / B
        ce.backward()
        ce_sum += ce.item()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            l16, _ = torch_ref.forward(spec, p16, xs.float())
        ((F.cross_entropy(l16.float(), ys, reduction="none") * wts).sum() / B).backward()
    assert rel_err(logits, ref_logits) < 3e-2
    # one rule for every gradient; the last layer's bias gradient is a column sum of the
    # fp32 dlogits (the CE kernels' block partials), not of their bf16 copy
    last_b = f"{spec.weights()[-1].name}/biases"
    for name in init:
        e = rel_err(net.fp.grad_view(name), p[name].grad)
        floor = rel_err(p16[name].grad, p[name].grad)
        assert e < max(3e-2, 3.0 * floor), f"{model} B={B} {name}: rel err {e:.3e} (bf16 floor {floor:.3e})"
    if last_bias_tol is not None:
        e = rel_err(net.fp.grad_view(last_b), p[last_b].grad)
        assert e < last_bias_tol, f"{model} B={B} {last_b}: rel err {e:.3e}"
    # fused update = w - lr * (g + wd w)
    before = {n: net.fp.param_view(n).clone() for n in init}
    grads = {n: net.fp.grad_view(n).clone() for n in init}
    net.update()
    torch.cuda.synchronize()
    wd = {f"{L.name}/weights": (L.wd or 0.0) for L in spec.weights()}
    for n in init:
        exp = before[n] - 0.05 * (grads[n] + wd.get(n, 0.0) * before[n])
        assert torch.allclose(net.fp.param_view(n), exp, rtol=1e-5, atol=1e-6), n
    assert int(net.fp.step.item()) == 1
    st = net.read_stats()
    assert abs(st["cross_entropy"] - ce_sum) < 2e-2 * max(1.0, ce_sum)


@pytest.mark.parametrize("model,cin", [("lenet5", 1), ("reference_cnn", 3), ("reference_cnn", 1), ("mlp", 1)])
def test_step_matches_oracle(dev, K, model, cin):
    _check_step(dev, model, cin, 96)


@pytest.mark.parametrize("model,cin,B,cap", [("lenet5", 1, 600, 4), ("reference_cnn", 1, 120, 8),
                                             ("reference_cnn", 3, 64, 5)])
def test_step_matches_oracle_multi_iteration(dev, K, grid_cap, model, cin, B, cap):
    """The same check with every persistent kernel's grid capped, so each block loops over
    several tiles / images (ring reuse and next-tile prefetch: the paths the benchmark
    batches take), on the train_step path (deferred fused head)."""
    grid_cap(cap)
    _check_step(dev, model, cin, B, defer_head=True, seed=1)


@pytest.mark.parametrize("model,cin,B", [("lenet5", 1, 65536), ("reference_cnn", 1, 16384),
                                         ("reference_cnn", 3, 16384)])
def test_step_matches_oracle_bench_batch(dev, K, model, cin, B):
    """The benchmarked configs themselves (BASELINE stress batch for LeNet-5, the reference
    CNN's bench batch, and the reference's own 3-channel input: mnist_input.py:13-15,134 on
    the generic conv1 path), on the bench's train_step path, against the fp32 oracle; the
    last bias gradient (fp32 dlogits column sums) to 1e-2."""
    _check_step(dev, model, cin, B, defer_head=True, seed=2, last_bias_tol=1e-2)


@pytest.mark.parametrize("model", ["lenet5", "reference_cnn"])
def test_training_reduces_loss(dev, K, model):
    from distributed_tensorflow_ibm_mnist_amd.data.synthetic import make_synthetic
    from distributed_tensorflow_ibm_mnist_amd.data.device_loader import DeviceDataset, DeviceLoader
    spec = get_model(model, 1)
    init = torch_ref.init_params(spec, seed=0)
    # lr 0.05 + momentum 0.9 sits at the edge of divergence for LeNet-5 here (one of three
    # data orders diverged); 0.02 converges for every order tried
    net = HipNet(spec, 256, dev, init, OptConfig(lr0=0.02, use_momentum=True, momentum=0.9, ema_max=0.9999))
    imgs, labs = make_synthetic(8192, seed=0, device=dev)
    ds = DeviceDataset(imgs, labs, dev)
    loader = DeviceLoader(ds, net.x0, net.labels, seed=0)
    losses = []
    for i in range(120):
        loader.next()
        net.train_step()
        if i % 20 == 0 or i == 119:
            losses.append(net.read_stats()["cross_entropy"])
    assert losses[-1] < 0.5 * losses[0], losses
    assert net.read_stats()["nan"] == 0


def test_graph_replay_matches_eager(dev, K):
    from distributed_tensorflow_ibm_mnist_amd.runtime.graph import StepGraph
    spec = get_model("lenet5", 1)
    init = torch_ref.init_params(spec, seed=3)
    x = (torch.rand(128, 28, 28, 1, device=dev) - 0.5).to(torch.bfloat16)
    y = torch.randint(0, 10, (128,), device=dev, dtype=torch.int32)
    nets = []
    for use_graph in (False, True):
        net = HipNet(spec, 128, dev, init, OptConfig(lr0=0.05, use_momentum=True, momentum=0.9))
        net.x0.copy_(x)
        net.labels.copy_(y)
        if use_graph:
            g = StepGraph(net.train_step, warmup=2)   # 2 eager warmup steps; capture does not execute
            for _ in range(4):
                g.replay()
        else:
            for _ in range(6):
                net.train_step()
        nets.append(net)
    torch.cuda.synchronize()
    assert int(nets[0].fp.step.item()) == int(nets[1].fp.step.item()) == 6
    assert torch.equal(nets[0].fp.params, nets[1].fp.params)


@pytest.mark.parametrize("mode", ["u8", "bf16", "bf16_u8bwd"])
@pytest.mark.parametrize("model", ["lenet5", "reference_cnn", "reference_cnn3"])
def test_u8_input_path_bitwise_equal(dev, K, model, mode):
    """First fused conv gathering the resident dataset through the batch index (fused
    K10) -- uint8 normalised in the kernels, or bf16 normalised once (bf16_u8bwd: with
    the fused LeNet-5 conv backward reading the uint8 twin) -- must equal prep_images +
    bf16 x0, bitwise, through full train steps (forward, weight gradient, update) and the
    Feistel index+label launch must equal the prep's."""
    from distributed_tensorflow_ibm_mnist_amd.data.synthetic import make_synthetic
    from distributed_tensorflow_ibm_mnist_amd.data.device_loader import DeviceDataset, DeviceLoader
    # reference_cnn3: the reference's own 3-channel records (mnist_input.py:13-15), gathered by
    # conv1's forward (convpool) and weight gradient (refc1_wgrad) from the bf16 dataset
    cin = 3 if model == "reference_cnn3" else 1
    if cin == 3 and mode != "bf16":
        pytest.skip("3-channel records: the bf16 dataset only")
    spec = get_model(model.rstrip("3"), cin)
    init = torch_ref.init_params(spec, seed=3)
    opt = OptConfig(lr0=0.05, use_momentum=True, momentum=0.9, ema_max=0.9999)
    imgs, labs = make_synthetic(3000, seed=4, device=dev, channels=cin)
    ds = DeviceDataset(imgs, labs, dev, channels=cin)
    a = HipNet(spec, 200, dev, init, opt)
    b = HipNet(spec, 200, dev, init, opt)
    assert b.bind_u8_input(ds.images if mode == "u8" else ds.bf16_images(),
                           bwd_images=ds.images if mode == "bf16_u8bwd" else None)
    assert (b.bwd_u8 is not None) == (mode == "bf16_u8bwd" and b.fused_bwd)
    la = DeviceLoader(ds, a.x0, a.labels, seed=9)
    lb = DeviceLoader(ds, b.x0, b.labels, seed=9, idx_out=b.idx_buf)
    for _ in range(3):
        la.next()
        lb.next()
        if mode != "u8":         # the once-normalised rows are bitwise the per-step prep's
            assert torch.equal(ds.bf16_images()[b.idx_buf].view_as(a.x0), a.x0)
        a.train_step()
        b.train_step()
    torch.cuda.synchronize()
    assert torch.equal(a.labels, b.labels)
    assert torch.equal(a.fp.params, b.fp.params)
    # eval keeps reading x0
    b.x0.copy_(a.x0)
    assert torch.equal(a.eval_batch(200, torch.zeros(8, device=dev)), b.eval_batch(200, torch.zeros(8, device=dev)))


def test_weight_decay_total_loss(dev, K):
    """total_loss = cross-entropy + sum_i wd_i/2 ||W_i||^2 (pre-update weights): the
    fused optimizer's per-block sum(w^2) partials combined in block order by
    finalize_k; bitwise identical over two identical runs (no float atomics)."""
    spec = get_model("reference_cnn", 1)
    totals = []
    for _ in range(2):
        net = HipNet(spec, 64, dev, torch_ref.init_params(spec, seed=3), OptConfig(lr0=0.01))
        g = torch.Generator(device=dev).manual_seed(1)
        net.x0.copy_((torch.rand(net.x0.shape, device=dev, generator=g) - 0.5).to(torch.bfloat16))
        net.labels.copy_(torch.randint(0, 10, (64,), device=dev, generator=g, dtype=torch.int32))
        wd_term = sum(float(e.wd) * 0.5 * float((net.fp.param_view(e.name).double() ** 2).sum())
                      for e in net.fp.wd_entries)
        net.train_step()
        torch.cuda.synchronize()
        st = net.read_stats()
        assert wd_term > 0
        assert abs(st["total_loss"] - (st["cross_entropy"] + wd_term)) < 1e-4 * max(1.0, wd_term), (st, wd_term)
        totals.append(net.stats[6].item())
    assert totals[0] == totals[1]


def test_lrn_pool_fusion_bitwise(dev, K):
    """reference CNN: the fused norm2+pool2 layer gives the same logits and gradients
    as the separate LRN and pool layers."""
    torch.manual_seed(3)
    spec = get_model("reference_cnn", 1)
    init = torch_ref.init_params(spec, seed=2)
    B = 80
    x = (torch.rand(B, 28, 28, 1, device=dev) - 0.5).to(torch.bfloat16)
    y = torch.randint(0, 10, (B,), device=dev, dtype=torch.int32)
    out = []
    for fuse in (True, False):
        net = HipNet(spec, B, dev, init, OptConfig(lr0=0.05), fuse_lrnpool=fuse)
        assert any(type(l).__name__ == "LRNPoolLayer" for l in net.layers) == fuse
        net.x0.copy_(x)
        net.labels.copy_(y)
        net.forward(defer_head=True)
        net.loss_and_grad()
        net.backward()
        torch.cuda.synchronize()
        out.append((net.logits.clone(), net.fp.grads.clone()))
    assert torch.equal(out[0][0], out[1][0])
    assert torch.equal(out[0][1], out[1][1])


@pytest.mark.parametrize("B", [77, 1024])
def test_lenet_fused_conv_backward_step(dev, K, B):
    """The LeNet-5 conv stack's backward as one kernel (lenet_bwd.hip) vs the three
    per-layer kernels, whole training step: every gradient to bf16 noise, the head's
    bitwise (untouched), and the fused kernel bitwise reproducible run to run
    (deterministic split-K, no atomics)."""
    spec = get_model("lenet5", 1)
    init = torch_ref.init_params(spec, seed=3)
    x = (torch.rand(B, 28, 28, 1, device=dev) - 0.5).to(torch.bfloat16)
    y = torch.randint(0, 10, (B,), device=dev, dtype=torch.int32)

    def grads(fused: bool):
        net = HipNet(spec, B, dev, init, OptConfig(lr0=0.05), fused_lenet_bwd=fused)
        assert net.fused_bwd == fused
        net.x0.copy_(x)
        net.labels.copy_(y)
        net.forward(defer_head=True)
        net.loss_and_grad()
        net.backward()
        torch.cuda.synchronize()
        return {n: net.fp.grad_view(n).clone() for n in init}

    ref, fused, again = grads(False), grads(True), grads(True)
    for n in init:
        assert torch.equal(fused[n], again[n]), f"{n}: fused kernel not reproducible"
        if n.startswith("conv"):
            assert rel_err(fused[n], ref[n]) < 1e-2, (n, rel_err(fused[n], ref[n]))
        else:
            assert torch.equal(fused[n], ref[n]), n


@pytest.mark.parametrize("cin", [1, 3])
def test_refcnn_lrn1_backward_fold(dev, K, cin, monkeypatch):
    """norm1 folded away: its forward runs in conv2's halo staging (fwd + wgrad,
    HipNet.fold_lrn_fwd) and its backward in conv1's weight-gradient staging
    (HipNet.fold_lrn), vs lrn_fwd / lrn_bwd launches: logits and every other gradient
    bitwise (same LRN math, same bf16 rounding), conv1's to fp32 reassociation (the
    folded kernel stages one image per group)."""
    spec = get_model("reference_cnn", cin)
    init = torch_ref.init_params(spec, seed=5)
    B = 70
    x = (torch.rand(B, 28, 28, cin, device=dev) - 0.5).to(torch.bfloat16)
    y = torch.randint(0, 10, (B,), device=dev, dtype=torch.int32)

    def grads(fold: str):
        monkeypatch.setenv("MNISTX_FOLD_LRN", fold)
        # the opt-in forward fold, tested here too
        net = HipNet(spec, B, dev, init, OptConfig(lr0=0.05), fold_lrn_fwd=fold == "1")
        assert net.fold_lrn == (fold == "1") and net.fold_lrn_fwd == (fold == "1")
        net.x0.copy_(x)
        net.labels.copy_(y)
        logits = net.forward(defer_head=True).clone()
        net.loss_and_grad()
        net.backward()
        torch.cuda.synchronize()
        return {"logits": logits, **{n: net.fp.grad_view(n).clone() for n in init}}

    ref, fold = grads("0"), grads("1")
    assert torch.equal(fold.pop("logits"), ref.pop("logits"))
    for n in init:
        if n.startswith("conv1/"):
            assert rel_err(fold[n], ref[n]) < 1e-5, n
        else:
            assert torch.equal(fold[n], ref[n]), n

