"""bench.py ``--prewarm_steps`` leaves the timed steps bitwise unchanged (VERDICT r5 ask 5).

The prewarm runs N real steps on the real buffers and then restores, from a hand-kept list,
every piece of state a step changes (bench.prewarm_steps).  If that list ever misses a
buffer, the W + K steps the driver times would start from a different state.  Here the
bench configuration (fused gathered input, bf16 input + uint8 backward twin, the input
lookahead inside the optimizer launch, momentum + EMA) runs W + K steps once after a
prewarm and once without; parameters, momentum, EMA, bf16 copies, step counter, loss
statistics and loss EMAs must be identical to the bit.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
pytestmark = pytest.mark.gpu


def _run(dev, prewarm: int, B: int = 8192, steps: int = 12):
    import torch
    import bench
    from distributed_tensorflow_ibm_mnist_amd.data.device_loader import DeviceDataset, DeviceLoader
    from distributed_tensorflow_ibm_mnist_amd.data.synthetic import make_synthetic
    from distributed_tensorflow_ibm_mnist_amd.models import get_model
    from distributed_tensorflow_ibm_mnist_amd.models.torch_ref import init_params
    from distributed_tensorflow_ibm_mnist_amd.runtime.executor import HipNet
    from distributed_tensorflow_ibm_mnist_amd.runtime.params import OptConfig
    spec = get_model("lenet5", 1)
    net = HipNet(spec, B, dev, init_params(spec, seed=0),
                 OptConfig(lr0=0.01, decay_rate=0.1, decay_steps=0, momentum=0.9, use_momentum=True, ema_max=0.9999))
    imgs, labs = make_synthetic(20000, seed=0, channels=1, device=dev)
    ds = DeviceDataset(imgs, labs, dev, hw=784, channels=1)
    assert net.can_gather_input() and net.bind_u8_input(ds.bf16_images(), bwd_images=ds.images)
    loader = DeviceLoader(ds, net.x0, net.labels, idx_out=net.idx_buf)
    net.next_input_job = loader.lookahead_job

    def step():
        loader.next()
        net.train_step()

    assert bench.prewarm_steps(net, loader, step, prewarm) == prewarm
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    fp = net.fp
    out = {k: getattr(fp, k).clone() for k in ("params", "mom", "ema", "bf16", "step")}
    out["stats"] = net.stats.clone()
    out["loss_ema"] = net.loss_ema.clone()
    out["pos"] = loader.pos
    return out


@pytest.mark.timeout(240)
def test_prewarm_steps_leave_timed_steps_bitwise_unchanged(dev):
    import torch
    a = _run(dev, 0)
    b = _run(dev, 37)          # an odd count: the loader's epoch position moves too
    assert a["pos"] == b["pos"]
    for k in ("params", "mom", "ema", "bf16", "step", "stats", "loss_ema"):
        assert torch.equal(a[k], b[k]), f"{k} differs after the prewarm"
