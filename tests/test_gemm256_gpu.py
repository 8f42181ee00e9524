"""256 x 256 LDS-DMA GEMM (csrc/kernels/gemm256.hip) against a PyTorch fp32 reference of the
same op, and against the gemm.hip engine it replaces for the GEMMs that fill the GPU
(dense_fwd / dense_dgrad route there when gemm256_ok; set_gemm256 flips the route)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def K():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from distributed_tensorflow_ibm_mnist_amd.ops._ext import kernels
    return kernels()


def _rel(a, b):
    return float((a.float() - b.float()).abs().max() / b.float().abs().max().clamp_min(1e-12))


@pytest.fixture(params=[0, 2, 4, 16], ids=["bk32_4stage", "bk64_2stage", "bk32_5stage", "bk32_4stage_rp"])
def ring(request, K):
    """gemm256's K-step ring: the default 4 x 32-deep stages, or 2 x 64 (set_gemm256_debug bit 1)."""
    K.set_gemm256_debug(request.param)
    yield request.param
    K.set_gemm256_debug(0)


def _both(K, f):
    """f() run on the gemm256 route and on gemm.hip; returns (new, old)."""
    K.set_gemm256(True)
    try:
        new = f()
        K.set_gemm256(False)
        old = f()
    finally:
        K.set_gemm256(True)
    torch.cuda.synchronize()
    return new, old


# (M, N, K): the reference CNN's local3 at B = 16384; a tail in every dimension (M, N not
# multiples of 256, K not a multiple of the 64-deep step); the smallest grid routed (256 tiles)
@pytest.mark.parametrize("M,N,Kd", [(16384, 1024, 3136), (8104, 2040, 520), (4096, 4096, 512)])
@pytest.mark.parametrize("out_dtype", [torch.bfloat16, torch.float32])
def test_gemm256_fwd_bias_relu(K, ring, M, N, Kd, out_dtype):
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(M + N + Kd)
    x = (torch.randn(M, Kd, device=dev, generator=g)).to(torch.bfloat16)
    w = (torch.randn(Kd, N, device=dev, generator=g) / Kd ** 0.5).to(torch.bfloat16)
    b = torch.randn(N, device=dev, generator=g) * 0.1
    ref = torch.relu(x.float() @ w.float() + b)

    def run():
        out = torch.full((M, N), float("nan"), device=dev, dtype=out_dtype)
        K.dense_fwd(x, w, out, M, N, Kd, Kd, N, N, b, N, True, None, 0)
        return out
    new, old = _both(K, run)
    tol = 1e-2 if out_dtype == torch.bfloat16 else 1e-4
    assert not torch.isnan(new.float()).any(), "unwritten outputs"
    assert _rel(new, ref) < tol, _rel(new, ref)
    assert _rel(old, ref) < tol
    if out_dtype == torch.float32:   # same products, fp32 sums: the two engines agree closely
        assert _rel(new, old) < 1e-5


@pytest.mark.parametrize("M,N,Kd", [(16384, 3136, 1024), (8104, 2040, 520)])
@pytest.mark.parametrize("with_mask", [False, True])
def test_gemm256_dgrad(K, ring, M, N, Kd, with_mask):
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(7 * M + N)
    dy = torch.randn(M, Kd, device=dev, generator=g).to(torch.bfloat16)
    w = (torch.randn(N, Kd, device=dev, generator=g) / Kd ** 0.5).to(torch.bfloat16)   # W[Din][Dout]
    mask = torch.randn(M, N, device=dev, generator=g).to(torch.bfloat16) if with_mask else None
    ref = dy.float() @ w.float().t()
    if with_mask:
        ref = torch.where(mask.float() > 0, ref, torch.zeros_like(ref))

    def run():
        out = torch.full((M, N), float("nan"), device=dev, dtype=torch.bfloat16)
        K.dense_dgrad(dy, w, out, M, N, Kd, Kd, Kd, N, mask, N if with_mask else 0)
        return out
    new, old = _both(K, run)
    assert not torch.isnan(new.float()).any()
    assert _rel(new, ref) < 1e-2, _rel(new, ref)
    assert _rel(old, ref) < 1e-2


def test_gemm256_route_is_on_by_default(K):
    assert K.gemm256_enabled()


@pytest.mark.parametrize("B,Din,Dout", [(16384, 3136, 1024), (5000, 3000, 1000)])
def test_gemm256_wgrad_bias_row(K, ring, B, Din, Dout):
    """Split-K weight gradient with the bias row (the ones column of X^T patched into the LDS
    image): the partials the call reports having written sum to X^T dY and dY's column sums."""
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(B + Din)
    x = torch.randn(B, Din, device=dev, generator=g).to(torch.bfloat16)
    dy = torch.randn(B, Dout, device=dev, generator=g).to(torch.bfloat16)
    M, cap = Din + 1, 8
    ref = torch.cat([x.float().t() @ dy.float(), dy.float().sum(0, keepdim=True)], 0)

    def run():
        slab = torch.full((cap * M * Dout,), float("nan"), device=dev)
        S = K.dense_wgrad(x, dy, slab, Din, Dout, B, Din, Dout, True, cap)
        return slab.view(cap, M, Dout)[:S].sum(0), S
    K.set_gemm256(True)
    (new, s_new) = run()
    K.set_gemm256(False)
    try:
        (old, s_old) = run()
    finally:
        K.set_gemm256(True)
    torch.cuda.synchronize()
    assert 1 <= s_new < cap, s_new          # the 256 x 256 path took it, with its own split count
    assert s_old == cap
    assert not torch.isnan(new).any()
    assert _rel(new, ref) < 1e-4, _rel(new, ref)
    assert _rel(new[Din], ref[Din]) < 1e-4, _rel(new[Din], ref[Din])   # bias row
    assert _rel(old, ref) < 1e-4


def _rel64(a, ref):
    return float((a.double() - ref).norm() / ref.norm().clamp_min(1e-30))


# fp32 (--precision fp32): the same tiles on v_mfma_f32_16x16x4_f32, against float64 (the
# fp32 route also needs its last round of tiles >= 90 % full: the forwards of the first two
# shapes and the dgrad of the third (4096 x 4096 out) are routed; local3's dgrad (3.25
# rounds) stays on f32.hip -- either way the result must match)
@pytest.mark.parametrize("M,N,Kd", [(16384, 1024, 3136), (8104, 2040, 520), (4096, 512, 4096)])
def test_gemm256_f32_fwd_dgrad(K, M, N, Kd):
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(3 * M + Kd)
    x = torch.randn(M, Kd, device=dev, generator=g)
    w = torch.randn(Kd, N, device=dev, generator=g) / Kd ** 0.5
    b = torch.randn(N, device=dev, generator=g) * 0.1
    y = torch.full((M, N), float("nan"), device=dev)
    K.set_gemm256(True)
    K.f32_dense_fwd(x, w, y, M, N, Kd, N, b, True)
    ref = torch.relu(x.double() @ w.double() + b.double())
    assert not torch.isnan(y).any()
    assert _rel64(y, ref) < 1e-5, _rel64(y, ref)   # fp32 sums over K (f32.hip tests: 1e-5)
    # dgrad: dx[M, Kd] = dy[M, N] . w[Kd, N]^T, masked (w here plays W[Din = Kd][Dout = N])
    dy = torch.randn(M, N, device=dev, generator=g)
    mask = torch.randn(M, Kd, device=dev, generator=g)
    dx = torch.full((M, Kd), float("nan"), device=dev)
    K.f32_dense_dgrad(dy, w, dx, M, Kd, N, mask)
    refd = (dy.double() @ w.double().t()) * (mask > 0)
    assert not torch.isnan(dx).any()
    assert _rel64(dx, refd) < 1e-5, _rel64(dx, refd)


@pytest.mark.parametrize("B,Din,Dout", [(16384, 3136, 1024), (5000, 3000, 1000)])
def test_gemm256_f32_wgrad_bias_row(K, B, Din, Dout):
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(B + Dout)
    x = torch.randn(B, Din, device=dev, generator=g)
    dy = torch.randn(B, Dout, device=dev, generator=g)
    cap = 8
    assert 1 <= K.f32_wgrad_splits_cap(Din, Dout, B) < cap
    slab = torch.full((cap * (Din + 1) * Dout,), float("nan"), device=dev)
    S = K.f32_dense_wgrad(x, dy, slab, B, Din, Dout, cap)
    torch.cuda.synchronize()
    assert S == K.f32_wgrad_splits_cap(Din, Dout, B)
    tot = slab.view(cap, Din + 1, Dout)[:S].sum(0)
    assert not torch.isnan(tot).any()
    # fp32 sums over K = B rows (1.1e-6 measured at B = 16384; f32.hip's tests use 1e-5)
    assert _rel64(tot[:Din], x.double().t() @ dy.double()) < 1e-5
    assert _rel64(tot[Din], dy.double().sum(0)) < 1e-5


def test_gemm256_respects_reserved_cus(K):
    """With CUs reserved for a collective (data-parallel, world > 1), gemm256 sizes its split
    counts for the CUs left (local3's weight gradient: 248 // 48 full tiles = 5 splits) and
    routes no one-round grid that would spill into a second round; results unchanged."""
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(11)
    B, Din, Dout = 16384, 3136, 1024
    x = torch.randn(B, Din, device=dev, generator=g).to(torch.bfloat16)
    dy = torch.randn(B, Dout, device=dev, generator=g).to(torch.bfloat16)
    w = (torch.randn(Din, Dout, device=dev, generator=g) / Din ** 0.5).to(torch.bfloat16)
    slab = torch.full((8 * (Din + 1) * Dout,), float("nan"), device=dev)
    y = torch.empty(B, Dout, device=dev, dtype=torch.bfloat16)
    K.set_reserve_cus(8)
    try:
        S = K.dense_wgrad(x, dy, slab, Din, Dout, B, Din, Dout, True, 8)
        K.dense_fwd(x, w, y, B, Dout, Din, Din, Dout, Dout, None, 0, False, None, 0)
        torch.cuda.synchronize()
    finally:
        K.set_reserve_cus(0)
    assert S == 5
    tot = slab.view(8, Din + 1, Dout)[:S].sum(0)
    ref = torch.cat([x.float().t() @ dy.float(), dy.float().sum(0, keepdim=True)], 0)
    assert _rel(tot, ref) < 1e-4
    assert _rel(y, x.float() @ w.float()) < 1e-2
