"""Debug: pooled-K conv1 wgrad vs emulation, one image per block (grid >= N)."""
import torch, torch.nn.functional as F
import sys, os
sys.path.insert(0, os.getcwd())
from distributed_tensorflow_ibm_mnist_amd.ops._ext import kernels
K = kernels(); dev = torch.device("cuda", 0)
torch.manual_seed(0)
N = 2
x = (torch.randn(N, 28, 28, 1, device=dev)).to(torch.bfloat16)
w = torch.zeros(5, 5, 1, 8, device=dev); w[..., :6] = torch.randn(5, 5, 1, 6, device=dev) / 5
w = w.to(torch.bfloat16); b = torch.randn(6, device=dev) * 0.1
pooled = torch.empty(N, 14, 14, 8, dtype=torch.bfloat16, device=dev)
arg = torch.empty(N, 14, 14, 4, dtype=torch.uint8, device=dev)
K.convpool_fwd(x, w, b, 6, pooled, arg, N, 1, 8, 5, 2, 28, 28)
codes = torch.cat([arg & 15, arg >> 4], dim=-1).long()   # N,14,14,8
def run(dP, xx):
    slab = torch.full((N * 48 * 8,), float("nan"), device=dev)
    K.convpool_wgrad(xx, dP, arg, slab, N, N, 1, 8, 5, 2, 28, 28)
    torch.cuda.synchronize()
    return slab.view(N, 48, 8)[0].cpu()
def ref(dP, xx):
    xf = xx[0, :, :, 0].float().cpu(); dPf = dP[0].float().cpu(); cd = codes[0].cpu()
    dW = torch.zeros(5, 5, 8); db = torch.zeros(8)
    xp_ = F.pad(xf, (2, 2, 2, 2))
    for yp in range(14):
        for xq in range(14):
            for c in range(6):
                g = int(cd[yp, xq, c])
                if g >= 4: continue
                y, xx2 = 2 * yp + (g >> 1), 2 * xq + (g & 1)
                dW[:, :, c] += dPf[yp, xq, c] * xp_[y:y + 5, xx2:xx2 + 5]
                db[c] += dPf[yp, xq, c]
    out = torch.zeros(48, 8)
    for kh in range(5):
        out[kh * 8:kh * 8 + 5] = dW[kh]
    out[40] = db
    return out
tests = {}
dP = torch.zeros(N, 14, 14, 8, device=dev)
dP[..., :6] = torch.randn(N, 14, 14, 6, device=dev)
tests["random"] = (dP.to(torch.bfloat16), x)
ones = torch.ones_like(x)
tests["x=1"] = (dP.to(torch.bfloat16), ones)
d1 = torch.zeros(N, 14, 14, 8, device=dev); d1[:, 3, 4, 0] = 1
tests["one pixel c0"] = (d1.to(torch.bfloat16), x)
d2 = torch.zeros(N, 14, 14, 8, device=dev); d2[:, 3, 9, 2] = 1
tests["one pixel c2 xp9"] = (d2.to(torch.bfloat16), x)
torch.set_printoptions(precision=3, linewidth=200)
for name, (dp, xx) in tests.items():
    got, want = run(dp, xx), ref(dp, xx)
    err = (got - want).abs()
    print(f"== {name}: max err {err.max():.4f} (ref max {want.abs().max():.4f}); code at (3,4,0)={int(codes[0,3,4,0])} (3,9,2)={int(codes[0,3,9,2])}")
    if err.max() > 1e-2:
        for kh in range(5):
            print("got ", got[kh * 8:kh * 8 + 5, :6].flatten()[:12].tolist())
            print("want", want[kh * 8:kh * 8 + 5, :6].flatten()[:12].tolist())
        print("bias got", got[40, :6].tolist(), "want", want[40, :6].tolist())
