import torch, sys
sys.path.insert(0, "/root/repo")
from distributed_tensorflow_ibm_mnist_amd.models import get_model
from distributed_tensorflow_ibm_mnist_amd.models.torch_ref import init_params
from distributed_tensorflow_ibm_mnist_amd.runtime.params import FlatParams, OptConfig
from distributed_tensorflow_ibm_mnist_amd.train.trainer import param_specs
from distributed_tensorflow_ibm_mnist_amd.ops._ext import kernels
from distributed_tensorflow_ibm_mnist_amd.parallel.ps import slot_len, stamp_view
dev = torch.device("cuda", 0)
spec = get_model("lenet5", 1)
fp = FlatParams.build(param_specs(spec), init_params(spec), dev, pads={})
n = fp.total
slot = torch.zeros(slot_len(n), device=dev)
stamp_view(slot).fill_(7)
err = torch.zeros(1, dtype=torch.int32, device=dev)
before = fp.params.clone()
o = OptConfig()
kernels().fused_optimizer(fp.params, slot[:n], fp.mom, fp.ema, fp.bf16, fp.segs, fp.step, o.lr0, o.decay_rate,
                          o.decay_steps, o.momentum, o.nesterov, o.use_momentum, 1.0, o.ema_max, None,
                          guard=stamp_view(slot), guard_want=8, guard_err=err, guard_id=3)
torch.cuda.synchronize()
print("err", err.item(), "unchanged", torch.equal(before, fp.params), "stamp", int(stamp_view(slot)))
