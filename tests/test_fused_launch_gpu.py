"""Launch fusions of the step's tail (misc.hip):

* the optimizer launch runs the step's finalize in its last block (agent-scope ticket),
  instead of a separate finalize_k launch -- the same code on the same partials, so the step
  counter, the stats, the loss EMAs and the parameters are BITWISE those of the two-launch path;
* the split-K reduce's partial pass finishes its own quads by ticket (one launch instead of
  two) -- the same sums up to the fp32 order of > 4 partials.

Several steps, so the tickets' self-reset is exercised too.
"""
import pytest
import torch

from distributed_tensorflow_ibm_mnist_amd.models import get_model, torch_ref
from distributed_tensorflow_ibm_mnist_amd.runtime.params import OptConfig

pytestmark = pytest.mark.gpu


def _run(dev, K, model, B, fin_fused, red_fused, steps=3):
    from distributed_tensorflow_ibm_mnist_amd.runtime.executor import HipNet
    K.set_opt_fin_fused(int(fin_fused))
    K.set_reduce_fused(int(red_fused))
    try:
        spec = get_model(model, 1)
        net = HipNet(spec, B, dev, torch_ref.init_params(spec, seed=5),
                     OptConfig(lr0=0.05, momentum=0.9, use_momentum=True, ema_max=0.999))
        g = torch.Generator(device=dev).manual_seed(5)
        for _ in range(steps):
            net.x0.copy_((torch.rand(B, 28, 28, 1, device=dev, generator=g) - 0.5).to(torch.bfloat16))
            net.labels.copy_(torch.randint(0, 10, (B,), device=dev, generator=g, dtype=torch.int32))
            net.train_step()
        torch.cuda.synchronize()
        return {"params": net.fp.params.clone(), "stats": net.stats.clone(), "ema": net.loss_ema.clone(),
                "step": int(net.fp.step.item()), "grads": net.fp.grads.clone()}
    finally:
        K.set_opt_fin_fused(1)
        K.set_reduce_fused(1)


@pytest.mark.parametrize("model,B", [("lenet5", 4096), ("reference_cnn", 512)])
def test_optimizer_runs_finalize_bitwise(dev, K, model, B):
    a = _run(dev, K, model, B, fin_fused=False, red_fused=True)
    b = _run(dev, K, model, B, fin_fused=True, red_fused=True)
    assert a["step"] == b["step"] == 3
    for k in ("params", "stats", "ema"):
        assert torch.equal(a[k], b[k]), k
    assert K.opt_fin_fused_enabled() and K.reduce_fused_enabled()


@pytest.mark.parametrize("model,B", [("lenet5", 4096), ("reference_cnn", 512)])
def test_one_launch_reduce_matches_two(dev, K, model, B):
    a = _run(dev, K, model, B, fin_fused=True, red_fused=False)
    b = _run(dev, K, model, B, fin_fused=True, red_fused=True)
    assert a["step"] == b["step"] == 3
    err = ((a["params"].double() - b["params"].double()).norm() / a["params"].double().norm()).item()
    assert err < 1e-6, err
    gerr = ((a["grads"].double() - b["grads"].double()).norm() / a["grads"].double().norm()).item()
    assert gerr < 1e-5, gerr


def test_fused_reduce_on_two_streams_at_once(dev, K):
    """Tickets are per stream: one-launch reduces queued on two streams without any
    synchronisation between them (the executor's overlapped side-stream reduces) still sum
    every quad block exactly once."""
    torch.manual_seed(3)
    case = (256, 208, 16, 25, 8, 6, 16, 200)   # LeNet-5 conv2 slab: 13 quad blocks x 4 partials
    S, M, N, G, Ip, I, J, br = case
    geo = torch.tensor([case], dtype=torch.int64)
    n = 12
    slabs = [torch.randn(S * M * N, device=dev) for _ in range(n)]
    refs = [(s.double().view(S, M, N).sum(0) * 0.5) for s in slabs]
    outs = [(torch.empty(G * I * J, device=dev), torch.empty(J, device=dev)) for _ in range(n)]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    torch.cuda.synchronize()
    for i in range(n):
        with torch.cuda.stream(streams[i % 2]):
            K.splitk_reduce_multi([slabs[i]], [outs[i][0]], [outs[i][1]], geo, [0.5])
    torch.cuda.synchronize()
    for i in range(n):
        wr = refs[i][:G * Ip].view(G, Ip, N)[:, :I, :J].reshape(-1)
        assert torch.allclose(outs[i][0].double(), wr, rtol=1e-5, atol=1e-4), i
        assert torch.allclose(outs[i][1].double(), refs[i][br, :J], rtol=1e-5, atol=1e-4), i


@pytest.mark.parametrize("model", ["lenet5", "reference_cnn"])
def test_optimizer_launch_writes_next_batch_rows(dev, K, model):
    """DeviceLoader.lookahead_job: the optimizer launch of step k writes step k+1's shuffle
    rows + labels (extra blocks), the next ``next()`` launches nothing, and the rows are those
    of perm_positions at the right stream position, across epoch boundaries; the training is
    bitwise the same as with a perm launch per step."""
    from distributed_tensorflow_ibm_mnist_amd.data.device_loader import (DeviceDataset, DeviceLoader, _half_bits,
                                                                          perm_positions)
    from distributed_tensorflow_ibm_mnist_amd.data.synthetic import make_synthetic
    from distributed_tensorflow_ibm_mnist_amd.runtime.executor import HipNet
    B, N, steps = 256, 1000, 6   # epoch boundaries inside steps 3 and 7
    imgs, labs = make_synthetic(N, seed=2, channels=1, device=dev)
    ds = DeviceDataset(imgs, labs, dev, hw=784, channels=1)
    runs = []
    for ahead in (False, True):
        spec = get_model(model, 1)
        net = HipNet(spec, B, dev, torch_ref.init_params(spec, seed=9), OptConfig(lr0=0.05, momentum=0.9,
                                                                                   use_momentum=True))
        assert net.bind_u8_input(ds.images)
        loader = DeviceLoader(ds, net.x0, net.labels, seed=4, idx_out=net.idx_buf)
        if ahead:
            net.next_input_job = loader.lookahead_job
        for k in range(steps):
            loader.next()
            want = perm_positions(k * B, B, N, 4, device=dev)
            assert torch.equal(net.idx_buf[:B], want), (ahead, k)
            assert torch.equal(net.labels[:B], ds.labels[want]), (ahead, k)
            net.train_step()
        torch.cuda.synchronize()
        assert loader.pos == steps * B
        runs.append(net.fp.params.clone())
    assert torch.equal(runs[0], runs[1])
    assert _half_bits(N) == 5
