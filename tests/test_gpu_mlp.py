"""The fused MLP kernels (vs_mlp_fwd / vs_mlp_bwd_da, csrc/mlp.hip) against fp64 references of
VideoMAEIntermediate + VideoMAEOutput (modeling_videomae.py:370-399) on the same bf16 inputs.

Tolerances (max-abs error / max |reference|): the kernels round the GELU output to bf16 before the
second product (2^-9 relative per element, as every bf16 GEMM chain) -> 8e-3 on the MLP output; the
backward's bf16 outputs da and a -> 8e-3.  Reruns are bitwise identical (fixed MFMA order).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from vspike import _lib
    _lib.lib()


def _gelu64(x):
    return 0.5 * x * (1.0 + torch.erf(x / 2 ** 0.5))


def _gelu64_grad(x):
    return 0.5 * (1.0 + torch.erf(x / 2 ** 0.5)) + x * torch.exp(-0.5 * x * x) / (2 * torch.pi) ** 0.5


def _maxrel(a, b):
    return float((a.double() - b).abs().max() / b.abs().max().clamp_min(1e-30))


def _operands(M, D, F, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    h2 = torch.randn(M, D, device=DEV, generator=g).to(torch.bfloat16)
    w1 = (torch.randn(F, D, device=DEV, generator=g) * 0.08).to(torch.bfloat16)
    b1 = torch.randn(F, device=DEV, generator=g) * 0.3
    w2 = (torch.randn(D, F, device=DEV, generator=g) * 0.04).to(torch.bfloat16)
    b2 = torch.randn(D, device=DEV, generator=g) * 0.3
    y = torch.randn(M, D, device=DEV, generator=g)
    return h2, w1, b1, w2, b2, y


# 200,704 = the bench's 128 clips (784 rounds of 256 tokens over the CUs: several rounds per
# workgroup); 25,088 = 16 clips; ragged counts and a single partial round
@pytest.mark.parametrize("M,F", [(200704, 768), (25088, 768), (12345, 768), (100, 768), (4096, 64), (3000, 3072)])
def test_mlp_fwd_matches_fp64(M, F):
    from vspike import ops, _lib as L
    D = 192
    h2, w1, b1, w2, b2, y = _operands(M, D, F, seed=M + F)
    out = torch.full((M, D), 7.0, device=DEV)
    L.dispatch_reset()
    ops.mlp_fwd(h2, w1, b1, w2, b2, y, out)
    torch.cuda.synchronize()
    assert L.dispatch_counts()["mlp_fwd"] == 1
    pre = h2.double() @ w1.double().t() + b1.double()
    mlp = _gelu64(pre) @ w2.double().t() + b2.double()
    err = _maxrel(out - y, mlp)
    print(f"\n[mlp fwd M={M} F={F}] max rel err {err:.2e}")
    assert err < 8e-3
    out2 = torch.empty_like(out)
    ops.mlp_fwd(h2, w1, b1, w2, b2, y, out2)
    torch.cuda.synchronize()
    assert torch.equal(out, out2)


@pytest.mark.parametrize("M,F", [(200704, 768), (25088, 768), (12345, 768), (100, 768), (4096, 64), (3000, 3072)])
def test_mlp_bwd_da_matches_fp64(M, F):
    from vspike import ops, _lib as L
    D = 192
    h2, w1, b1, w2, _, _ = _operands(M, D, F, seed=M + F + 1)
    g = torch.Generator(device=DEV).manual_seed(F)
    dy = torch.randn(M, D, device=DEV, generator=g).to(torch.bfloat16)
    da = torch.full((M, F), 3.0, dtype=torch.bfloat16, device=DEV)
    a = torch.full((M, F), 3.0, dtype=torch.bfloat16, device=DEV)
    L.dispatch_reset()
    ops.mlp_bwd_da(h2, w1, b1, w2, dy, da, a)
    torch.cuda.synchronize()
    assert L.dispatch_counts()["mlp_bwd"] == 1
    pre = h2.double() @ w1.double().t() + b1.double()
    ea = _maxrel(a, _gelu64(pre))
    eda = _maxrel(da, (dy.double() @ w2.double()) * _gelu64_grad(pre))
    print(f"\n[mlp bwd M={M} F={F}] a {ea:.2e} da {eda:.2e}")
    assert ea < 8e-3 and eda < 8e-3
    da2, a2 = torch.empty_like(da), torch.empty_like(a)
    ops.mlp_bwd_da(h2, w1, b1, w2, dy, da2, a2)
    torch.cuda.synchronize()
    assert torch.equal(da, da2) and torch.equal(a, a2)


def test_mlp_bwd_gelu_is_the_forward_gelu():
    """The backward recomputes pre with the forward's MFMA chain: its a = gelu(pre) (bf16) fed to a
    plain GEMM reproduces the fused forward's output to within that GEMM's own rounding (same bf16
    operands, f32 sums in another order): 1e-5 of the output."""
    from vspike import ops
    M, D, F = 25088, 192, 768
    h2, w1, b1, w2, b2, y = _operands(M, D, F, seed=5)
    out = torch.empty(M, D, device=DEV)
    ops.mlp_fwd(h2, w1, b1, w2, b2, y, out)
    da = torch.empty(M, F, dtype=torch.bfloat16, device=DEV)
    a = torch.empty(M, F, dtype=torch.bfloat16, device=DEV)
    ops.mlp_bwd_da(h2, w1, b1, w2, torch.zeros(M, D, dtype=torch.bfloat16, device=DEV), da, a)
    torch.cuda.synchronize()
    ref = a.double() @ w2.double().t() + b2.double()
    assert _maxrel(out - y, ref) < 1e-5
    assert int(torch.count_nonzero(da)) == 0


def test_mlp_fused_ok_shapes():
    from vspike import ops
    assert ops.mlp_fused_ok(200704, 192, 768)
    assert not ops.mlp_fused_ok(25088, 768, 3072)     # ViT-Base: the two-GEMM path
    assert not ops.mlp_fused_ok(100, 192, 100)


@pytest.mark.parametrize("M", [200704, 12345, 100])
def test_mlp_fwd_ln_next_layernorm(M):
    """vs_mlp_fwd_ln: the fused MLP plus the NEXT block's LayerNorm1 on its output rows (eps 1e-12):
    x' as vs_mlp_fwd writes it (bitwise), h within bf16 rounding of the fp64 LayerNorm of x', row
    mean / rstd within 1e-5 relative."""
    import ctypes
    from vspike import ops, _lib as L
    D, F = 192, 768
    h2, w1, b1, w2, b2, y = _operands(M, D, F, seed=M + 3)
    g = torch.Generator(device=DEV).manual_seed(M)
    gam = torch.randn(D, device=DEV, generator=g) * 0.3 + 1
    bet = torch.randn(D, device=DEV, generator=g) * 0.1
    out, out_ref = torch.empty(M, D, device=DEV), torch.empty(M, D, device=DEV)
    hn = torch.empty(M, D, dtype=torch.bfloat16, device=DEV)
    mean, rstd = torch.empty(M, device=DEV), torch.empty(M, device=DEV)
    ops.mlp_fwd(h2, w1, b1, w2, b2, y, out_ref)
    L.check(L.lib().vs_mlp_fwd_ln(M, D, F, h2.data_ptr(), D, w1.data_ptr(), b1.data_ptr(), w2.data_ptr(),
                                  b2.data_ptr(), y.data_ptr(), D, out.data_ptr(), D, gam.data_ptr(), bet.data_ptr(),
                                  ctypes.c_float(1e-12), hn.data_ptr(), D, mean.data_ptr(), rstd.data_ptr(),
                                  L.stream()), "vs_mlp_fwd_ln")
    torch.cuda.synchronize()
    assert torch.equal(out, out_ref)
    x = out.double()
    mu = x.mean(1)
    var = ((x - mu[:, None]) ** 2).mean(1)
    rs = 1.0 / torch.sqrt(var + 1e-12)
    href = (x - mu[:, None]) * rs[:, None] * gam.double() + bet.double()
    assert _maxrel(hn, href) < 8e-3
    assert float(((mean.double() - mu).abs() / x.abs().max()).max()) < 1e-5
    assert float(((rstd.double() - rs).abs() / rs).max()) < 1e-5
