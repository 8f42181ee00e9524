#!/usr/bin/env python3
"""Times the fused LeNet-5 head kernel alone (HIP events) at batch B.
Usage: python bench/micro_mlp_head.py [B] [iters]"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from distributed_tensorflow_ibm_mnist_amd.models import get_model, torch_ref
from distributed_tensorflow_ibm_mnist_amd.runtime.executor import HipNet

B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 50
dev = torch.device("cuda:0")
spec = get_model("lenet5", 1)
net = HipNet(spec, B, dev, torch_ref.init_params(spec, seed=0))
net.layers[net.head - 1].out.copy_(torch.rand_like(net.layers[net.head - 1].out, dtype=torch.float32).to(torch.bfloat16))
net.labels.copy_(torch.randint(0, 10, (B,), device=dev, dtype=torch.int32))
for _ in range(5):
    net._run_head(B, 1.0 / B, True, net.stats)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(iters):
    net._run_head(B, 1.0 / B, True, net.stats)
e1.record()
torch.cuda.synchronize()
print(f"mlp_head B={B}: {e0.elapsed_time(e1) / iters * 1e3:.1f} us")
