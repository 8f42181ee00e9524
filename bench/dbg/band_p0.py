"""Debug: the band forward without pool1 output (P1OUT 0) vs with (P1OUT 1): where do the
pool2 outputs differ (pooled pixel, image slot, channel)?"""
import os, sys
sys.path.insert(0, os.getcwd())
import torch
sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
from test_lenet_band_gpu import _weights, _band
from distributed_tensorflow_ibm_mnist_amd.ops._ext import kernels
K = kernels()
dev = torch.device("cuda", 0)
torch.manual_seed(0)
w1, b1, w2, b2 = _weights(dev, seed=5)
n, B = 500, 77
ds = (torch.rand(n, 784, device=dev) - 0.5).to(torch.bfloat16)
idx = torch.randint(0, n, (B,), device=dev, dtype=torch.int64)
_, _, P2, _ = _band(K, ds, w1, b1, w2, b2, B, idx=idx)
_, _, T2, _ = _band(K, ds, w1, b1, w2, b2, B, idx=idx, p1=False)
d = (T2.float() - P2.float()).abs()
print("max err", d.max().item())
bad = (d > 1e-2 * P2.float().abs().max()).nonzero()
print("bad count", bad.shape[0], "of", d.numel())
if bad.shape[0]:
    img = bad[:, 0] % 8; pix = bad[:, 1] * 5 + bad[:, 2]; ch = bad[:, 3]
    print("images%8", torch.bincount(img, minlength=8).tolist())
    print("pixels", torch.bincount(pix, minlength=25).tolist())
    print("channels", torch.bincount(ch, minlength=16).tolist())
