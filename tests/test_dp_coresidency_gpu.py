"""CU reservation for collectives (parallel/dp.py, kernels.set_reserve_cus) on one MI355X.

* with 8 CUs reserved, an RCCL-footprint probe (probe.hip: 256-thread blocks with 16 KB
  of LDS) launched on a second stream starts while the LeNet-5 fused conv backward and
  the reference CNN's conv2 dgrad run, instead of queueing behind them
  (bench/dp_coresidency.py has the full table, profiles/r5/dp_coresidency/);
* a reserved step computes the same gradients (the persistent grids shrink, so only the
  split-K partition and with it the fp32 summation order changes);
* the bucket plan of the fused LeNet-5 executor is ONE end-of-backward bucket.
"""
import pytest
import torch

from distributed_tensorflow_ibm_mnist_amd.models import get_model, torch_ref
from distributed_tensorflow_ibm_mnist_amd.runtime.params import OptConfig

pytestmark = pytest.mark.gpu


@pytest.fixture
def reserve(K):
    yield K.set_reserve_cus
    K.set_reserve_cus(0)


def _net(dev, model, B, seed=0):
    from distributed_tensorflow_ibm_mnist_amd.runtime.executor import HipNet
    spec = get_model(model, 1)
    net = HipNet(spec, B, dev, torch_ref.init_params(spec, seed=seed), OptConfig(lr0=0.01, use_momentum=False))
    g = torch.Generator(device=dev).manual_seed(seed)
    net.x0.copy_((torch.rand(B, 28, 28, 1, device=dev, generator=g) - 0.5).to(torch.bfloat16))
    net.labels.copy_(torch.randint(0, 10, (B,), device=dev, generator=g, dtype=torch.int32))
    return net


def _probe_frac(K, target, lds=16384):
    side = torch.cuda.Stream()
    stamps = torch.zeros(16, dtype=torch.int64, device="cuda")
    marks = torch.zeros(2, dtype=torch.int64, device="cuda")
    fr = []
    for _ in range(5):
        ev = torch.cuda.Event()
        K.clock_mark(marks, 0)
        ev.record()
        target()
        K.clock_mark(marks, 1)
        side.wait_event(ev)
        with torch.cuda.stream(side):
            K.coresidency_probe(stamps, 8, 256, lds, 200)
        torch.cuda.synchronize()
        m = marks.tolist()
        first = min(stamps.view(8, 2)[:, 0].tolist())
        fr.append((first - m[0]) / max(1, m[1] - m[0]))
    return sorted(fr)[len(fr) // 2]


def test_reserve_lets_a_collective_start_beside_lenet_bwd(dev, K, reserve):
    # B = 65536: a ~200 us kernel, so the host's enqueue of the probe (launched after the
    # target) is a small fraction of it; at 16384 (~50 us) that latency alone reached 0.57
    B = 65536
    net = _net(dev, "lenet5", B)
    net.train_step()
    assert net.fused_bwd
    target = lambda: net._fused_conv_backward(B, net.dbuf[2], [])   # noqa: E731
    reserve(8)
    assert K.reserve_cus() == 8
    assert K.lenet_bwd_blocks(B) < net.lb_grid
    f8 = _probe_frac(K, target)
    assert f8 < 0.5, f"probe started at {f8:.2f} of lenet_bwd_k even with 8 CUs reserved"


def test_reserve_lets_a_collective_start_beside_conv2_dgrad(dev, K, reserve):
    from distributed_tensorflow_ibm_mnist_amd.runtime.executor import ConvLayer
    B = 4096
    net = _net(dev, "reference_cnn", B)
    net.train_step()
    k = next(i for i, lay in enumerate(net.layers) if isinstance(lay, ConvLayer) and lay.name == "conv2")
    c2 = net.layers[k]
    reserve(8)
    f8 = _probe_frac(K, lambda: c2.bwd_data(B, net.dbuf[k + 1], net.dbuf[k]))
    assert f8 < 0.5, f"probe started at {f8:.2f} of the conv2 dgrad even with 8 CUs reserved"


@pytest.mark.parametrize("model,B", [("lenet5", 8192), ("reference_cnn", 2048)])
def test_reserved_step_matches_unreserved(dev, K, reserve, model, B):
    grads = []
    for r in (0, 8):
        reserve(r)
        net = _net(dev, model, B, seed=3)
        net.forward(defer_head=True)
        net.loss_and_grad()
        net.backward()
        torch.cuda.synchronize()
        grads.append(net.fp.grads.clone())
    a, b = grads
    err = ((a.double() - b.double()).norm() / b.double().norm()).item()
    assert err < 1e-5, err


def test_lenet_bucket_plan_is_one_bucket(dev, K):
    from distributed_tensorflow_ibm_mnist_amd.parallel.dp import DataParallel
    net = _net(dev, "lenet5", 1024)
    idx = {L.name: i for i, L in enumerate(net.spec.layers)}
    assert net.bucket_lockout == {idx["fc3"], idx["conv2"]}
    dp = DataParallel(net, bucket_cap_mb=0.125, world=2)
    assert len(dp.buckets) == 1 and dp.reserve_cus == 0
    assert K.reserve_cus() == 0
    net2 = _net(dev, "reference_cnn", 256)
    dp2 = DataParallel(net2, bucket_cap_mb=0.125, world=2)
    try:
        assert [[net2.spec.layers[i].name for i in b.layers] for b in dp2.buckets] == [
            ["softmax_linear", "local4"], ["local3"], ["conv2", "conv1"]]
        assert dp2.reserve_cus == 8 and K.reserve_cus() == 8
    finally:
        K.set_reserve_cus(0)
