"""Op-level parity of the HIP kernels (through the C-ABI) against torch-CPU references.

f32 ops: within 1e-5 relative (exact-f32 MFMA / f32 VALU).  bf16 ops: inputs are rounded to bf16
first and the CPU reference runs in f32/f64 on those same values; outputs are checked against a
tolerance stated per test (f32 accumulation; bf16 rounding of outputs ~4e-3 relative).
"""
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _lib():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from vspike import _lib
    _lib.lib()


def rel(a, b):
    a = a.double().cpu()
    b = b.double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


def _rand(*shape, dtype=torch.float32, seed=0, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(dtype)


# ------------------------------------------------------------------------------------------ GEMM
GEMM_SHAPES = [(64, 64, 64), (200, 136, 72), (25, 40, 16), (1568, 192, 192), (7, 576, 192), (256, 64, 2048),
               (296, 200, 128), (136, 72, 192), (264, 64, 64)]   # whole-K-in-LDS path, ragged M/N


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("akc,bkc", [(True, True), (True, False), (False, True), (False, False)])
@pytest.mark.parametrize("shape", GEMM_SHAPES)
def test_gemm_layouts(dtype, akc, bkc, shape):
    from vspike import ops
    M, N, K = shape
    vec = 8 if dtype == torch.bfloat16 else 4
    if (not akc and M % vec) or (not bkc and N % vec) or (K % vec and (akc or bkc)):
        pytest.skip("contiguous extent must be a multiple of 16 bytes")
    A = _rand(M, K, seed=1).to(dtype).float()
    B = _rand(K, N, seed=2).to(dtype).float()
    ref = A.double() @ B.double()
    a_dev = (A if akc else A.t().contiguous()).to(dtype).to(DEV)
    b_dev = (B.t().contiguous() if bkc else B).to(dtype).to(DEV)
    c = torch.empty(M, N, dtype=torch.float32, device=DEV)
    ops.gemm(a_dev, b_dev, c, M=M, N=N, K=K, a_kcontig=akc, b_kcontig=bkc, lda=a_dev.stride(0),
             ldb=b_dev.stride(0), ldc=N)
    torch.cuda.synchronize()
    # error bound of an f32-accumulated dot product over K terms
    bound = 1e-5 * math.sqrt(K) / 8 + 1e-6
    err = ((c.double().cpu() - ref).abs() / (A.abs().double() @ B.abs().double()).clamp_min(1e-30)).max().item()
    assert err < bound, (err, bound)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_gemm_epilogues(dtype):
    from vspike import ops, _lib as L
    M, N, K = 300, 192, 128
    x = _rand(M, K, seed=3).to(dtype)
    w = _rand(N, K, seed=4, scale=0.1).to(dtype)
    bias = _rand(N, seed=5)
    res = _rand(M, N, seed=6)
    pos = _rand(100, N, seed=7)
    pre_ref = x.double() @ w.double().t() + bias.double()
    dev = lambda t: t.to(DEV)  # noqa: E731
    # bias + pos
    c = torch.empty(M, N, device=DEV)
    ops.linear(dev(x), dev(w), c, bias=dev(bias), epilogue=L.EPI_POS, pos=dev(pos), pos_rows=100)
    ref = pre_ref + pos.double()[torch.arange(M) % 100]
    assert rel(c, ref) < 1e-5
    # bias + gelu (aux_out = pre-activation in operand dtype) + residual
    a = torch.empty(M, N, dtype=dtype, device=DEV)
    pre = torch.empty(M, N, dtype=dtype, device=DEV)
    ops.linear(dev(x), dev(w), a, bias=dev(bias), epilogue=L.EPI_GELU, aux_out=pre, ld_aux_out=N)
    tol = 1e-5 if dtype == torch.float32 else 8e-3
    assert rel(pre.float(), pre_ref) < tol
    assert rel(a.float(), torch.nn.functional.gelu(pre_ref)) < tol
    r = torch.empty(M, N, device=DEV)
    ops.linear(dev(x), dev(w), r, bias=dev(bias), epilogue=L.EPI_RESIDUAL, residual=dev(res), ld_residual=N)
    assert rel(r, pre_ref + res.double()) < 1e-5
    # relu and relu-bwd / gelu-bwd masks
    rl = torch.empty(M, N, device=DEV)
    ops.linear(dev(x), dev(w), rl, bias=dev(bias), epilogue=L.EPI_RELU)
    assert rel(rl, pre_ref.clamp_min(0)) < 1e-5
    g = torch.empty(M, N, device=DEV)
    ops.linear(dev(x), dev(w), g, epilogue=L.EPI_GELU_BWD, aux_in=pre, ld_aux_in=N)
    xp = pre.double().cpu().requires_grad_()
    gg = torch.autograd.grad(torch.nn.functional.gelu(xp).sum(), xp)[0]
    assert rel(g, (x.double() @ w.double().t()) * gg) < 1e-5
    rb = torch.empty(M, N, device=DEV)
    ops.linear(dev(x), dev(w), rb, epilogue=L.EPI_RELU_BWD, aux_in=res.to(dtype).to(DEV), ld_aux_in=N)
    assert rel(rb, (x.double() @ w.double().t()) * (res.to(dtype).double() > 0)) < 1e-5


@pytest.mark.parametrize("bkc", [True, False])
@pytest.mark.parametrize("shape", [(20000, 576, 192), (25088, 768, 192), (3001, 192, 128)])
def test_gemm_panel_path_many_items(bkc, shape):
    """Large K <= 192 products: the GELU forward (per-tile path) and the GELU' dX product, which runs
    on the persistent row-panel kernel (K <= 192, N % 64 == 0) at sizes where each workgroup
    walks several (panel, chunk) items and crosses panels; GELU and GELU' epilogues, ragged M."""
    from vspike import ops, _lib as L
    M, N, K = shape
    x = _rand(M, K, seed=11).to(torch.bfloat16).to(DEV)
    w = _rand(N, K, seed=12, scale=0.1).to(torch.bfloat16).to(DEV)
    bias = _rand(N, seed=13).to(DEV)
    ref = x.float() @ w.float().t() + bias
    a = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    pre = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    if bkc:
        ops.linear(x, w, a, bias=bias, epilogue=L.EPI_GELU, aux_out=pre, ld_aux_out=N)
        assert rel(pre.float(), ref) < 8e-3
        assert rel(a.float(), torch.nn.functional.gelu(ref)) < 8e-3
    else:  # dX form: B(k, n) = wt[k, n] (n-contiguous), GELU' epilogue against the saved pre
        wt = w.t().contiguous()
        pre.copy_(ref.to(torch.bfloat16))
        g = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
        ops.gemm(x, wt, g, M=M, N=N, K=K, a_kcontig=True, b_kcontig=False, lda=K, ldb=N, ldc=N,
                 epilogue=L.EPI_GELU_BWD, aux_in=pre, ld_aux_in=N)
        xp = pre.float().requires_grad_()
        gg = torch.autograd.grad(torch.nn.functional.gelu(xp).sum(), xp)[0]
        assert rel(g.float(), (x.float() @ w.float().t()) * gg) < 1.5e-2


@pytest.mark.parametrize("bkc", [True, False])
@pytest.mark.parametrize("shape", [(25088, 192, 768), (25088, 192, 192), (25088, 192, 576), (8200, 64, 128),
                                   (12345, 128, 64), (40000, 192, 128)])
@pytest.mark.parametrize("epi", ["none", "bias", "bias_res"])
@pytest.mark.parametrize("wv", [0, 8])
def test_gemm_row_slab_path(knobs, bkc, shape, epi, wv):
    """N <= 192 bf16 products at M >= 8192 run on the row-slab kernel (one balanced row range per
    workgroup, all N columns): the ViT block's proj / fc2 (+ bias + f32 residual) and the dX
    products (plain, f32 or bf16 out).  Ragged M (slabs of 16..17 rows), M > 32,768 (two 64-row
    tiles per workgroup), both W layouts; wv = 8 forces the 8-wave / 128-row-tile variant (the
    default from 256 rows per workgroup) on the same shapes (slabs shorter than a tile, 128-row tiles
    with partial halves).  Reference: fp64 on the same bf16 inputs; tolerance 1e-5 of max|ref| for f32
    outputs (f32 accumulation), 8e-3 for bf16 outputs (one rounding)."""
    from vspike import ops, _lib as L
    knobs("slab_wv", wv)
    M, N, K = shape
    x = _rand(M, K, seed=21).to(torch.bfloat16).to(DEV)
    w = _rand(N, K, seed=22, scale=0.1).to(torch.bfloat16).to(DEV)
    bias = _rand(N, seed=23).to(DEV)
    res = _rand(M, N, seed=24).to(DEV)
    ref = x.double() @ w.double().t()
    out_bf16 = epi == "none" and K == 192
    c = torch.empty(M, N, dtype=torch.bfloat16 if out_bf16 else torch.float32, device=DEV)
    flags, kw = 0, {}
    if epi != "none":
        flags |= L.EPI_BIAS
        kw["bias"] = bias
        ref = ref + bias.double()
    if epi == "bias_res":
        flags |= L.EPI_RESIDUAL
        kw.update(residual=res, ld_residual=N)
        ref = ref + res.double()
    if bkc:
        ops.gemm(x, w, c, M=M, N=N, K=K, a_kcontig=True, b_kcontig=True, lda=K, ldb=K, ldc=N, epilogue=flags, **kw)
    else:
        wt = w.t().contiguous()
        ops.gemm(x, wt, c, M=M, N=N, K=K, a_kcontig=True, b_kcontig=False, lda=K, ldb=N, ldc=N, epilogue=flags, **kw)
    torch.cuda.synchronize()
    assert rel(c.float(), ref) < (8e-3 if out_bf16 else 1e-5)


@pytest.mark.parametrize("bkc", [True, False])
@pytest.mark.parametrize("shape", [(25088, 576, 192), (25088, 768, 192), (12345, 256, 128), (40000, 768, 64),
                                   (8192, 320, 192)])
@pytest.mark.parametrize("epi", ["bias", "gelu", "gelu_bwd", "none"])
def test_gemm_wide_row_slab_path(bkc, shape, epi):
    """K <= 192, N > 192 bf16 products at M >= 8192 run on the wide row-slab kernel (balanced row
    ranges, 64-column chunks, prefetched W chunk and GELU' operand): qkv (+ bias), fc1 (+ bias +
    GELU, pre-activation written too) and the GELU' dX product; ragged M, two tiles per workgroup
    (M > 32,768), N not a multiple of 128.  Reference fp64 on the same bf16 inputs; bf16 outputs
    within 8e-3 of max|ref| (one rounding; GELU' 1.5e-2: the saved pre-activation is bf16)."""
    from vspike import ops, _lib as L
    M, N, K = shape
    x = _rand(M, K, seed=31).to(torch.bfloat16).to(DEV)
    w = _rand(N, K, seed=32, scale=0.1).to(torch.bfloat16).to(DEV)
    bias = _rand(N, seed=33).to(DEV)
    b_dev, ldb = (w, K) if bkc else (w.t().contiguous(), N)
    ref = x.double() @ w.double().t()
    out = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    kw = dict(M=M, N=N, K=K, a_kcontig=True, b_kcontig=bkc, lda=K, ldb=ldb, ldc=N)
    if epi == "bias":
        ops.gemm(x, b_dev, out, epilogue=L.EPI_BIAS, bias=bias, **kw)
        ref = ref + bias.double()
        tol = 8e-3
    elif epi == "none":
        ops.gemm(x, b_dev, out, **kw)
        tol = 8e-3
    elif epi == "gelu":
        pre = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
        ops.gemm(x, b_dev, out, epilogue=L.EPI_BIAS | L.EPI_GELU, bias=bias, aux_out=pre, ld_aux_out=N, **kw)
        ref = ref + bias.double()
        assert rel(pre.float(), ref) < 8e-3
        ref = torch.nn.functional.gelu(ref)
        tol = 8e-3
    else:
        pre = _rand(M, N, seed=34).to(torch.bfloat16).to(DEV)
        ops.gemm(x, b_dev, out, epilogue=L.EPI_GELU_BWD, aux_in=pre, ld_aux_in=N, **kw)
        xp = pre.double().requires_grad_()
        gg = torch.autograd.grad(torch.nn.functional.gelu(xp).sum(), xp)[0]
        ref = ref * gg
        tol = 1.5e-2
    torch.cuda.synchronize()
    assert rel(out.float(), ref) < tol


@pytest.mark.parametrize("bkc", [True, False])
@pytest.mark.parametrize("shape", [(8269, 384, 192), (25093, 576, 192), (25088, 768, 192)])
@pytest.mark.parametrize("epi", ["bias", "gelu", "gelu_bwd", "none", "gelu_grad", "mul_aux"])
@pytest.mark.parametrize("wv", [0, 8])
def test_gemm_w_resident_path(knobs, bkc, shape, epi, wv):
    """K = 192, N a multiple of 192 (qkv, fc1 + GELU, the GELU' product) run on the W-resident kernel
    (W part in LDS once per workgroup, permuted rows so a lane stores 8 consecutive columns, ragged
    row ranges / token blocks): fp64 reference on the same bf16 inputs (tolerances as the wide
    row-slab test), and the same values as the tile kernels (knob no_wres) to bf16 rounding; both
    workgroup sizes (4 and 8 waves sharing one W part)."""
    from vspike import ops, _lib as L
    knobs("wres_gbwd", 1)   # the GELU' product too (off by default)
    knobs("wres_wv", wv)    # 4 waves per workgroup at these row counts, or the 8-wave variant
    M, N, K = shape
    x = _rand(M, K, seed=41).to(torch.bfloat16).to(DEV)
    w = _rand(N, K, seed=42, scale=0.1).to(torch.bfloat16).to(DEV)
    bias = _rand(N, seed=43).to(DEV)
    pre_in = _rand(M, N, seed=44).to(torch.bfloat16).to(DEV)
    b_dev, ldb = (w, K) if bkc else (w.t().contiguous(), N)
    kw = dict(M=M, N=N, K=K, a_kcontig=True, b_kcontig=bkc, lda=K, ldb=ldb, ldc=N)

    def run():
        out = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
        pre = torch.zeros(M, N, dtype=torch.bfloat16, device=DEV)
        if epi == "bias":
            ops.gemm(x, b_dev, out, epilogue=L.EPI_BIAS, bias=bias, **kw)
        elif epi == "none":
            ops.gemm(x, b_dev, out, **kw)
        elif epi == "gelu":
            ops.gemm(x, b_dev, out, epilogue=L.EPI_BIAS | L.EPI_GELU, bias=bias, aux_out=pre, ld_aux_out=N, **kw)
        elif epi == "gelu_grad":   # the bf16 ViT fc1: aux_out = gelu'(pre), the backward's factor
            ops.gemm(x, b_dev, out, epilogue=L.EPI_BIAS | L.EPI_GELU | L.EPI_GELU_GRAD, bias=bias, aux_out=pre,
                     ld_aux_out=N, **kw)
        elif epi == "mul_aux":     # the bf16 ViT GELU' product: v *= stored gelu'
            ops.gemm(x, b_dev, out, epilogue=L.EPI_MUL_AUX, aux_in=pre_in, ld_aux_in=N, **kw)
        else:
            ops.gemm(x, b_dev, out, epilogue=L.EPI_GELU_BWD, aux_in=pre_in, ld_aux_in=N, **kw)
        torch.cuda.synchronize()
        return out, pre

    out, pre = run()
    ref = x.double() @ w.double().t()
    tol = 8e-3
    if epi in ("bias", "gelu", "gelu_grad"):
        ref = ref + bias.double()
    if epi == "gelu":
        assert rel(pre.float(), ref) < 8e-3
        ref = torch.nn.functional.gelu(ref)
    if epi == "gelu_grad":
        xp = ref.clone().requires_grad_()
        gref = torch.autograd.grad(torch.nn.functional.gelu(xp).sum(), xp)[0]
        assert rel(pre.float(), gref) < 8e-3
        ref = torch.nn.functional.gelu(ref)
    if epi == "mul_aux":
        ref = ref * pre_in.double()
    if epi == "gelu_bwd":
        xp = pre_in.double().requires_grad_()
        ref = ref * torch.autograd.grad(torch.nn.functional.gelu(xp).sum(), xp)[0]
        tol = 1.5e-2
    assert rel(out.float(), ref) < tol
    knobs("no_wres", 1)
    out2, pre2 = run()
    assert (out.float() - out2.float()).abs().max() <= 1e-2 * out2.float().abs().max()
    if epi in ("gelu", "gelu_grad"):
        assert (pre.float() - pre2.float()).abs().max() <= 1e-2 * pre2.float().abs().max()


@pytest.mark.parametrize("kernel", ["big", "g256", "g256a3"])
@pytest.mark.parametrize("bkc", [True, False])
@pytest.mark.parametrize("shape,epi", [((25088, 3072, 768), "gelu"), ((25088, 768, 3072), "bias_res"),
                                       ((4100, 512, 512), "bias"), ((8192, 2304, 768), "none"),
                                       ((6000, 768, 1536), "gelu_bwd"),
                                       # ragged long-M tiles (M % 256 != 0) for the 256 x 256 kernel
                                       ((17000, 3072, 768), "gelu"), ((16500, 768, 3072), "bias_res"),
                                       ((20000, 2304, 768), "bias"), ((18000, 768, 2304), "none"),
                                       ((17777, 3072, 768), "gelu_bwd"), ((16411, 512, 256), "gelu_grad")])
def test_gemm_big_tile_path(bkc, shape, epi, kernel, knobs):
    """K >= 512, N >= 512 bf16 products (ViT-Base's D = 768 / F = 3072 block) on the 256 x 128 8-wave
    big-tile kernel and (M >= 16,384, N % 256 == 0) on the 256 x 256 persistent one, each forced by knob
    g256: every epilogue the block uses, both W layouts, ragged M (M % 256 != 0; the 256 x 256 kernel's
    last tile clamps its row DMA and masks its stores).  Reference fp64 on the same bf16 inputs: f32
    outputs 1e-5 of max|ref|, bf16 outputs 8e-3 (GELU' 1.5e-2, against a bf16 pre-activation)."""
    from vspike import ops, _lib as L
    M, N, K = shape
    if kernel != "big" and (M < 16384 or N % 256 or K % 64 or K < 256):
        pytest.skip("the 256 x 256 kernel takes M >= 16,384, N % 256 == 0, K % 64 == 0")
    if kernel == "big" and (K < 512 or N % 128):
        pytest.skip("the big-tile kernel takes K >= 512, N % 128 == 0")
    knobs("g256", 2 if kernel == "big" else 1)
    knobs("g256_a3", 1 if kernel == "g256a3" else 2)    # g256a3: A in three LDS slots (VS_KNOB_G256_A3)
    L.dispatch_reset()
    x = _rand(M, K, seed=51).to(torch.bfloat16).to(DEV)
    w = _rand(N, K, seed=52, scale=K ** -0.5).to(torch.bfloat16).to(DEV)
    bias = _rand(N, seed=53).to(DEV)
    b_dev, ldb = (w, K) if bkc else (w.t().contiguous(), N)
    kw = dict(M=M, N=N, K=K, a_kcontig=True, b_kcontig=bkc, lda=K, ldb=ldb, ldc=N)
    ref = x.double() @ w.double().t()
    if epi == "bias_res":
        res = _rand(M, N, seed=54).to(DEV)
        out = torch.empty(M, N, device=DEV)
        ops.gemm(x, b_dev, out, epilogue=L.EPI_BIAS | L.EPI_RESIDUAL, bias=bias, residual=res, ld_residual=N, **kw)
        ref, tol = ref + bias.double() + res.double(), 1e-5
    elif epi == "bias":
        out = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
        ops.gemm(x, b_dev, out, epilogue=L.EPI_BIAS, bias=bias, **kw)
        ref, tol = ref + bias.double(), 8e-3
    elif epi == "none":
        out = torch.empty(M, N, device=DEV)
        ops.gemm(x, b_dev, out, **kw)
        tol = 1e-5
    elif epi == "gelu":
        out = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
        pre = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
        ops.gemm(x, b_dev, out, epilogue=L.EPI_BIAS | L.EPI_GELU, bias=bias, aux_out=pre, ld_aux_out=N, **kw)
        ref = ref + bias.double()
        torch.cuda.synchronize()
        assert rel(pre.float(), ref) < 8e-3
        ref, tol = torch.nn.functional.gelu(ref), 8e-3
    elif epi == "gelu_grad":      # gelu(pre) out, gelu'(pre) into aux (bf16 forward)
        out = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
        gp = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
        ops.gemm(x, b_dev, out, epilogue=L.EPI_BIAS | L.EPI_GELU | L.EPI_GELU_GRAD, bias=bias, aux_out=gp,
                 ld_aux_out=N, **kw)
        pre = ref + bias.double()
        torch.cuda.synchronize()
        xp = pre.to(torch.bfloat16).double().requires_grad_()
        gg = torch.autograd.grad(torch.nn.functional.gelu(xp).sum(), xp)[0]
        assert rel(gp.float(), gg) < 1.5e-2
        ref, tol = torch.nn.functional.gelu(pre), 8e-3
    else:
        out = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
        pre = _rand(M, N, seed=55).to(torch.bfloat16).to(DEV)
        ops.gemm(x, b_dev, out, epilogue=L.EPI_GELU_BWD, aux_in=pre, ld_aux_in=N, **kw)
        xp = pre.double().requires_grad_()
        gg = torch.autograd.grad(torch.nn.functional.gelu(xp).sum(), xp)[0]
        ref, tol = ref * gg, 1.5e-2
    torch.cuda.synchronize()
    assert L.dispatch_counts()["gemm_big" if kernel == "big" else "gemm_g256"] == 1, L.dispatch_counts()
    assert rel(out.float(), ref) < tol


# the C3 block's products at the bench's 128 clips (M = 200,704 token rows, D = 768, F = 3072), with the
# operand layouts and epilogues vit_exec.hip launches: forward (W [N, K], K-contiguous) and dX (W read
# transposed: [K, N] storage)
C3_PRODUCTS = {
    "fwd_qkv": ((2304, 768), True, "bias"), "fwd_proj": ((768, 768), True, "bias_res"),
    "fwd_fc1": ((3072, 768), True, "gelu_grad"), "fwd_fc2": ((768, 3072), True, "bias_res"),
    "dx_fc2": ((3072, 768), False, "mul_aux"), "dx_fc1": ((768, 3072), False, "none_f32"),
    "dx_proj": ((768, 768), False, "none_bf16"), "dx_qkv": ((768, 2304), False, "none_f32"),
    "patch": ((768, 1536), True, "bias_pos"),
}


@pytest.mark.parametrize("kernel", ["big", "g256", "g256a3"])
@pytest.mark.parametrize("prod", sorted(C3_PRODUCTS))
def test_gemm_big_tile_c3_bench128(prod, kernel, knobs):
    """Every C3 block product at its benched size (200,704 rows: VERDICT r4 item 1) on the big-tile
    path (the 256 x 128 kernel and the 256 x 256 persistent one, each forced by knob g256), against fp64 on
    the device from the same bf16 operands; the dispatch counter shows the big-tile kernel ran.  f32
    outputs 1e-5 of max|ref|, bf16 outputs 8e-3 (one bf16 rounding)."""
    from vspike import ops, _lib as L
    (N, K), bkc, epi = C3_PRODUCTS[prod]
    if kernel != "big" and epi == "bias_pos":
        pytest.skip("the 256 x 256 kernel has no position-table epilogue (the patch embedding stays on the big tile)")
    knobs("g256", 2 if kernel == "big" else 1)
    knobs("g256_a3", 1 if kernel == "g256a3" else 2)
    M = 200704
    g = torch.Generator(device=DEV).manual_seed(N + 7 * K)
    x = torch.randn(M, K, device=DEV, generator=g).to(torch.bfloat16)
    w = (torch.randn(N, K, device=DEV, generator=g) * K ** -0.5).to(torch.bfloat16)
    bias = torch.randn(N, device=DEV, generator=g)
    b_dev, ldb = (w, K) if bkc else (w.t().contiguous(), N)
    kw = dict(M=M, N=N, K=K, a_kcontig=True, b_kcontig=bkc, lda=K, ldb=ldb, ldc=N)
    ref = x.double() @ w.double().t()
    L.dispatch_reset()
    if epi == "bias_res":
        res = torch.randn(M, N, device=DEV, generator=g)
        out = torch.empty(M, N, device=DEV)
        ops.gemm(x, b_dev, out, epilogue=L.EPI_BIAS | L.EPI_RESIDUAL, bias=bias, residual=res, ld_residual=N, **kw)
        ref, tol = ref.add_(bias.double()).add_(res.double()), 1e-5
        del res
    elif epi == "bias":
        out = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
        ops.gemm(x, b_dev, out, epilogue=L.EPI_BIAS, bias=bias, **kw)
        ref, tol = ref.add_(bias.double()), 8e-3
    elif epi == "bias_pos":   # the patch embedding: + bias + sinusoid[token % 1568]
        pos = ops.sinusoid_table(1568, N, DEV)
        out = torch.empty(M, N, device=DEV)
        ops.gemm(x, b_dev, out, epilogue=L.EPI_BIAS | L.EPI_POS, bias=bias, pos=pos, pos_rows=1568, **kw)
        ref = ref.add_(bias.double()).view(-1, 1568, N).add_(pos.double()).view(M, N)
        tol = 1e-5
    elif epi == "none_f32":
        out = torch.empty(M, N, device=DEV)
        ops.gemm(x, b_dev, out, **kw)
        tol = 1e-5
    elif epi == "none_bf16":
        out = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
        ops.gemm(x, b_dev, out, **kw)
        tol = 8e-3
    elif epi == "gelu_grad":   # bf16 forward: gelu(pre) out, gelu'(pre) into aux
        out = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
        gp = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
        ops.gemm(x, b_dev, out, epilogue=L.EPI_BIAS | L.EPI_GELU | L.EPI_GELU_GRAD, bias=bias, aux_out=gp,
                 ld_aux_out=N, **kw)
        pre = ref.add_(bias.double())
        torch.cuda.synchronize()
        xp = pre.to(torch.bfloat16).double().requires_grad_()
        gg = torch.autograd.grad(torch.nn.functional.gelu(xp).sum(), xp)[0]
        assert rel(gp.float(), gg) < 1.5e-2
        del xp, gg, gp
        ref, tol = torch.nn.functional.gelu(pre), 8e-3
    else:                      # mul_aux: da = (dx' W2) * gelu'(pre), the stored factor
        aux = (torch.rand(M, N, device=DEV, generator=g) * 1.2 - 0.1).to(torch.bfloat16)
        out = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
        ops.gemm(x, b_dev, out, epilogue=L.EPI_MUL_AUX, aux_in=aux, ld_aux_in=N, **kw)
        ref, tol = ref.mul_(aux.double()), 8e-3
    torch.cuda.synchronize()
    assert L.dispatch_counts()["gemm_big" if kernel == "big" else "gemm_g256"] == 1, L.dispatch_counts()
    err = ((out.double() - ref).abs().max() / ref.abs().max()).item()
    print(f"\n[{prod}] M={M} N={N} K={K} max err / max|ref| = {err:.3e}")
    assert err < tol


def test_g256_early_dma_instances_have_no_scratch():
    """The 256 x 256 kernel's early-DMA wait is vmcnt(<the epilogue's store count>): exact only while
    the epilogue issues no other vector-memory op (a register spill adds scratch loads / stores).  The
    launcher falls back to vmcnt(0) per instance on its own; this pins that the benched instances keep
    the fast path."""
    from vspike import _lib as L
    assert L.lib().vs_g256_scratch_free() == 1


@pytest.mark.parametrize("M", [25088, 9000])
def test_patch_embed_gemm_pos_on_row_slab(M):
    """The patch embedding x0 = cols W^T + b + sinusoid[token] (K = 1536, N = 192, pos rows = 1568)
    on the row-slab kernel: fp64 reference, and the row -> table-row mapping m % pos_rows."""
    from vspike import ops, _lib as L
    N, K, P = 192, 1536, 1568
    x = _rand(M, K, seed=61).to(torch.bfloat16).to(DEV)
    w = _rand(N, K, seed=62, scale=0.05).to(torch.bfloat16).to(DEV)
    b = _rand(N, seed=63).to(DEV)
    pos = _rand(P, N, seed=64).to(DEV)
    out = torch.empty(M, N, device=DEV)
    ops.linear(x, w, out, bias=b, epilogue=L.EPI_POS, pos=pos, pos_rows=P)
    torch.cuda.synchronize()
    rows = torch.arange(M, device=DEV) % P
    ref = x.double() @ w.double().t() + b.double() + pos.double()[rows]
    assert rel(out, ref) < 1e-5


@pytest.mark.parametrize("shape", [(25088, 192, 192), (9409, 192, 192), (25088, 192, 768)])
@pytest.mark.parametrize("bias", [True, False])
@pytest.mark.parametrize("wv", [0, 8])
def test_gemm_ln_fwd_fused(knobs, shape, bias, wv):
    """vs_gemm_ln_fwd: y = x W^T (+ b) + residual and h = LayerNorm(y) in one row-slab launch (the
    ViT block's proj product + layernorm_after) — bitwise the two-launch result (same epilogue order,
    same 16-lane row layout and reduction order as ln_fwd_vec_kernel), and close to fp64; wv = 8: the
    8-wave / 128-row-tile slab kernel."""
    knobs("slab_wv", wv)
    from vspike import ops, _lib as L
    M, N, K = shape
    x = _rand(M, K, seed=51).to(torch.bfloat16).to(DEV)
    w = _rand(N, K, seed=52, scale=0.1).to(torch.bfloat16).to(DEV)
    b = _rand(N, seed=53).to(DEV) if bias else None
    res = _rand(M, N, seed=54).to(DEV)
    g = (1 + 0.1 * _rand(N, seed=55)).to(DEV)
    be = (0.1 * _rand(N, seed=56)).to(DEV)
    y = torch.empty(M, N, device=DEV)
    h = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    mean, rstd = torch.empty(M, device=DEV), torch.empty(M, device=DEV)
    ops.linear_ln_fwd(x, w, y, res, g, be, 1e-12, h, mean, rstd, bias=b)
    y2 = torch.empty_like(y)
    epi = L.EPI_RESIDUAL | (L.EPI_BIAS if bias else 0)
    ops.gemm(x, w, y2, M=M, N=N, K=K, a_kcontig=True, b_kcontig=True, lda=K, ldb=K, ldc=N, epilogue=epi, bias=b,
             residual=res, ld_residual=N)
    h2 = torch.empty_like(h)
    m2, r2 = torch.empty_like(mean), torch.empty_like(rstd)
    ops.layernorm_fwd(y2, g, be, 1e-12, h2, m2, r2)
    torch.cuda.synchronize()
    assert torch.equal(y, y2) and torch.equal(h, h2) and torch.equal(mean, m2) and torch.equal(rstd, r2)
    ref = x.double() @ w.double().t() + res.double() + (b.double() if bias else 0)
    assert rel(y, ref) < 1e-5
    href = torch.nn.functional.layer_norm(ref, (N,), g.double(), be.double(), 1e-12)
    assert rel(h.float(), href) < 8e-3


@pytest.mark.parametrize("shape", [(25088, 192, 768), (25088, 192, 576), (12345, 128, 64), (40000, 64, 128),
                                   (300, 192, 256)])
@pytest.mark.parametrize("dres,lp", [(True, True), (False, False)])
@pytest.mark.parametrize("wv", [0, 8])
def test_gemm_ln_bwd_fused(knobs, shape, dres, lp, wv):
    """vs_gemm_ln_bwd: the block's dh = dY W product with the LayerNorm backward in its epilogue
    (fused for bf16, N <= 192, M >= 8192: ragged slabs, two tiles per workgroup at M > 32,768; the
    small case runs the unfused GEMM + vs_layernorm_bwd).  Reference: fp64 autograd of
    LayerNorm(eps 1e-12) on dh = dY W computed from the same bf16 inputs.  dx within 1e-4 of
    max|ref| (f32 arithmetic), dgamma/dbeta 1e-4 of their max (the 16-lane row sums reorder), the
    bf16 copy within 8e-3; the fused call is bitwise reproducible.  wv = 8: the 8-wave / 128-row-tile
    slab kernel (its dgamma/dbeta partial rows sum 8 waves)."""
    from vspike import ops
    knobs("slab_wv", wv)
    M, D, Nout = shape
    dy = _rand(M, Nout, seed=41).to(torch.bfloat16).to(DEV)
    w = _rand(Nout, D, seed=42, scale=0.05).to(torch.bfloat16).to(DEV)
    x = (_rand(M, D, seed=43) * 2 + 0.5).to(DEV)
    gamma = (_rand(D, seed=44) * 0.3 + 1).to(DEV)
    r = _rand(M, D, seed=45).to(DEV) if dres else None
    mean = x.mean(1)
    rstd = torch.rsqrt(x.var(1, unbiased=False) + 1e-12)
    dx = torch.empty(M, D, device=DEV)
    dx_lp = torch.empty(M, D, dtype=torch.bfloat16, device=DEV) if lp else None
    dg0, db0 = _rand(D, seed=46).to(DEV), _rand(D, seed=47).to(DEV)
    dg, db = dg0.clone(), db0.clone()
    ops.linear_dx_ln_bwd(dy, w, x, mean, rstd, gamma, dx, dg, db, dres=r, dx_lp=dx_lp)
    torch.cuda.synchronize()
    xd = x.double().cpu().requires_grad_()
    gd = gamma.double().cpu().requires_grad_()
    bd = torch.zeros(D, dtype=torch.float64, requires_grad=True)
    y = torch.nn.functional.layer_norm(xd, (D,), gd, bd, eps=1e-12)
    dh = dy.double().cpu() @ w.double().cpu()
    gx, gg, gb = torch.autograd.grad(y, (xd, gd, bd), dh)
    if dres:
        gx = gx + r.double().cpu()
    assert rel(dx, gx) < 1e-4
    assert rel(dg - dg0, gg) < 1e-4 and rel(db - db0, gb) < 1e-4
    if lp:
        assert rel(dx_lp.float(), gx) < 8e-3
    dx2 = torch.empty_like(dx)
    dg2, db2 = dg0.clone(), db0.clone()
    ops.linear_dx_ln_bwd(dy, w, x, mean, rstd, gamma, dx2, dg2, db2, dres=r, dx_lp=dx_lp)
    torch.cuda.synchronize()
    assert torch.equal(dx, dx2) and torch.equal(dg, dg2) and torch.equal(db, db2)


@pytest.mark.parametrize("K", [768, 576])
@pytest.mark.parametrize("wv", [0, 8])
def test_gemm_ln_bwd_fused_bench_rows(knobs, K, wv):
    """vs_gemm_ln_bwd at the benched 128-clip row count (M = 200,704 = 128 x 1568; grid 512 -> 392
    rows per slab: multi-tile ragged slabs), both slab widths, with the bench's operands (dres, bf16
    copy).  Reference: fp64 on the device (the CPU would take minutes).  K = 768: dh2 = da W1 (the
    MLP's dX + LN2'); K = 576: dh1 = dqkv Wqkv (+ LN1')."""
    from vspike import ops, _lib as L
    knobs("slab_wv", wv)
    M, D = 200704, 192
    g = torch.Generator(device=DEV).manual_seed(K + wv)
    dy = torch.randn(M, K, device=DEV, generator=g).to(torch.bfloat16)
    w = (torch.randn(K, D, device=DEV, generator=g) * 0.05).to(torch.bfloat16)
    x = torch.randn(M, D, device=DEV, generator=g) * 2 + 0.5
    gamma = torch.randn(D, device=DEV, generator=g) * 0.3 + 1
    r = torch.randn(M, D, device=DEV, generator=g)
    mean = x.mean(1)
    rstd = torch.rsqrt(x.var(1, unbiased=False) + 1e-12)
    dx = torch.empty(M, D, device=DEV)
    dx_lp = torch.empty(M, D, dtype=torch.bfloat16, device=DEV)
    dg, db = torch.zeros(D, device=DEV), torch.zeros(D, device=DEV)
    L.dispatch_reset()
    ops.linear_dx_ln_bwd(dy, w, x, mean, rstd, gamma, dx, dg, db, dres=r, dx_lp=dx_lp)
    torch.cuda.synchronize()
    assert L.dispatch_counts()["gemm_ln_bwd"] == 1
    # fp64 reference of LayerNorm' (eps 1e-12) on dh = dY W
    dh = dy.double() @ w.double()
    xh = (x.double() - mean.double()[:, None]) * rstd.double()[:, None]
    gdh = dh * gamma.double()
    gx = rstd.double()[:, None] * (gdh - gdh.mean(1, keepdim=True) - xh * (gdh * xh).mean(1, keepdim=True)) + r.double()
    assert rel(dx, gx) < 1e-4
    assert rel(dg, (dh * xh).sum(0)) < 1e-4 and rel(db, dh.sum(0)) < 1e-4
    assert rel(dx_lp.float(), gx) < 8e-3
    dx2, dg2, db2 = torch.empty_like(dx), torch.zeros_like(dg), torch.zeros_like(db)
    ops.linear_dx_ln_bwd(dy, w, x, mean, rstd, gamma, dx2, dg2, db2, dres=r, dx_lp=dx_lp)
    torch.cuda.synchronize()
    assert torch.equal(dx, dx2) and torch.equal(dg, dg2) and torch.equal(db, db2)


@pytest.mark.parametrize("shape", [(192, 768, 200704), (768, 192, 200704), (192, 192, 200704), (576, 192, 200704),
                                   (192, 1536, 200704),
                                   # C3 (videomae-base): dW2, dW1, dWqkv, dWproj and the patch dW from cols
                                   (768, 3072, 200704), (3072, 768, 200704), (2304, 768, 200704),
                                   (768, 768, 200704), (768, 1536, 200704),
                                   # the 256 x 256 kernel at other token counts (C3 at 16 clips, C5, odd splits)
                                   (768, 1536, 25088), (2304, 768, 50176), (3072, 768, 64 * 1001)])
@pytest.mark.parametrize("kernel", ["dw", "dw256"])
def test_dw_bench128_split_plan(shape, kernel, knobs):
    """The weight gradients at the benched 128 clips (K = 200,704 tokens): the dW-tile kernel with the
    split plan the timed step uses and its fixed-order reduce, and (256-multiple widths) the 256 x 256
    persistent dW kernel with its split-ordered reduce, against fp64 on the device; bitwise
    reproducible; the dispatch counter shows which kernel ran."""
    from vspike import ops, _lib as L
    M, N, K = shape
    if kernel == "dw256" and (M % 256 or N % 256 or M * N <= 768 * 768):
        pytest.skip("the 256 x 256 dW kernel takes 256-multiple widths above 768 x 768")
    if kernel == "dw" and K != 200704:
        pytest.skip("split-K dW kernel: the benched token count only")
    knobs("no_dw256", int(kernel == "dw"))
    g = torch.Generator(device=DEV).manual_seed(M + N)
    dy = torch.randn(K, M, device=DEV, generator=g).to(torch.bfloat16)
    x = torch.randn(K, N, device=DEV, generator=g).to(torch.bfloat16)
    nb = ops.splitk_workspace_bytes(torch.bfloat16, M, N, K)
    ws = torch.empty(nb // 4 + 64, device=DEV)
    outs = []
    L.dispatch_reset()
    for _ in range(2):
        c = torch.full((M, N), 0.25, device=DEV)
        db = torch.full((M,), 1.5, device=DEV)
        ops.linear_dw(dy, x, c, db=db, workspace=ws)
        outs.append((c, db))
    torch.cuda.synchronize()
    assert L.dispatch_counts()["gemm_" + kernel] == 2, L.dispatch_counts()
    ref = dy.double().t() @ x.double() + 0.25
    assert rel(outs[0][0], ref) < 2e-5
    assert rel(outs[0][1], dy.double().sum(0) + 1.5) < 2e-5
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("ws", [None, False])       # split-K partials + reduce launch, or f32 atomics
@pytest.mark.parametrize("shape", [(64, 192, 25088), (192, 768, 25088), (104, 40, 5000), (768, 192, 25088),
                                   (576, 192, 3136), (192, 192, 1568), (192, 1536, 25088), (8, 16, 70)])
def test_gemm_splitk_atomic_accumulates(dtype, ws, shape):
    from vspike import ops
    M, N, K = shape                    # the dW shapes: reduction over B*N tokens (+ a ragged one)
    dy = _rand(K, M, seed=8).to(dtype)
    x = _rand(K, N, seed=9).to(dtype)
    c = torch.ones(M, N, device=DEV)   # accumulates on top of existing values
    db = torch.full((M,), 3.0, device=DEV)
    ops.linear_dw(dy.to(DEV), x.to(DEV), c, db=db, workspace=ws)   # bias gradient fused (row sums of A)
    ref = dy.double().t() @ x.double() + 1.0
    assert rel(c, ref) < 2e-5
    assert rel(db, dy.double().sum(0) + 3.0) < 2e-5
    if ws is None:                     # the partial-sum path is deterministic: bit-identical reruns
        c2 = torch.ones(M, N, device=DEV)
        ops.linear_dw(dy.to(DEV), x.to(DEV), c2, workspace=ws)
        assert torch.equal(c, c2)


@pytest.mark.parametrize("shape", [(192, 768, 25088), (768, 192, 25088), (192, 192, 25088), (576, 192, 25088),
                                   (192, 1536, 25088)])
def test_dw_bench_split_plan(shape):
    """The weight gradients of the ViT-Tiny block (dW2, dW1, dWproj, dWqkv) and of the patch
    embedding at the bench's 25,088 tokens (B=16): the dW-tile kernel with the PLANNED split (the
    timed step's plan) and its fixed-order reduce, against fp64 with the fused bias row sums;
    reruns are bit-identical and the dispatch counter shows the dW kernel ran."""
    from vspike import ops, _lib as L
    M, N, K = shape
    dy = _rand(K, M, seed=58).to(torch.bfloat16).to(DEV)
    x = _rand(K, N, seed=59).to(torch.bfloat16).to(DEV)
    nb = ops.splitk_workspace_bytes(torch.bfloat16, M, N, K)
    ws = torch.empty(nb // 4 + 64, device=DEV)
    outs = []
    L.dispatch_reset()
    for _ in range(2):
        c = torch.full((M, N), 0.25, device=DEV)
        db = torch.full((M,), 1.5, device=DEV)
        ops.linear_dw(dy, x, c, db=db, workspace=ws)
        outs.append((c, db))
    torch.cuda.synchronize()
    assert L.dispatch_counts()["gemm_dw"] == 2
    ref = dy.double().t() @ x.double() + 0.25
    assert rel(outs[0][0], ref) < 2e-5
    assert rel(outs[0][1], dy.double().sum(0) + 1.5) < 2e-5
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("bn", [64, 128])
@pytest.mark.parametrize("bm", [64, 128, 192])
@pytest.mark.parametrize("shape", [(192, 768, 3136 + 40), (576, 192, 1568), (200, 72, 999)])
def test_dw_kernel_every_tile_height(knobs, bm, bn, shape):
    """The token-reduction dW kernel (gemm_dw.hip) at every tile shape, with ragged tiles, a
    partial last token step, swapped operands (M > N: C stored transposed, bias = column sums of
    the swapped B) and the fixed-order split reduce: bit-identical reruns."""
    from vspike import ops
    knobs("dw_bm", bm)
    knobs("dw_bn", bn)
    M, N, K = shape
    dy = _rand(K, M, seed=18).to(torch.bfloat16).to(DEV)
    x = _rand(K, N, seed=19).to(torch.bfloat16).to(DEV)
    outs = []
    for _ in range(2):
        c = torch.full((M, N), 0.5, device=DEV)
        db = torch.full((M,), -1.0, device=DEV)
        ops.linear_dw(dy, x, c, db=db)
        outs.append((c, db))
    ref = dy.double().t() @ x.double() + 0.5
    assert rel(outs[0][0], ref) < 2e-5
    assert rel(outs[0][1], dy.double().sum(0) - 1.0) < 2e-5
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("shape", [(16, 64, 301056), (5, 48, 3200), (40, 16, 2048 + 96), (64, 64, 4096)])
def test_skinny_splitk_kcontig(shape):
    """The head's Linear(N*D -> 64) forward shape (M = clips, K = N*D): the skinny split-K kernel
    loading MFMA fragments straight from HBM, partials summed in split order (bias once, C +=)."""
    from vspike import ops, _lib as L
    M, N, K = shape
    x = _rand(M, K, seed=31).to(torch.bfloat16).to(DEV)
    w = _rand(N, K, seed=32, scale=K ** -0.5).to(torch.bfloat16).to(DEV)
    bias = _rand(N, seed=33).to(DEV)
    nb = ops.splitk_workspace_bytes(torch.bfloat16, M, N, K)
    ws = torch.empty(nb // 4 + 4, device=DEV)
    outs = []
    for _ in range(2):
        c = torch.full((M, N), 0.25, device=DEV)
        ops.gemm(x, w, c, M=M, N=N, K=K, a_kcontig=True, b_kcontig=True, lda=K, ldb=K, ldc=N,
                 epilogue=L.EPI_ATOMIC | L.EPI_BIAS, bias=bias, workspace=ws)
        outs.append(c)
    ref = x.double() @ w.double().t() + bias.double() + 0.25
    assert rel(outs[0], ref) < 2e-5
    assert torch.equal(outs[0], outs[1])


def test_gemm_splitk_workspace_bias_once():
    from vspike import ops, _lib as L
    M, N, K = 96, 128, 20000
    a = _rand(K, M, seed=21).to(torch.bfloat16).to(DEV)
    b = _rand(K, N, seed=22).to(torch.bfloat16).to(DEV)
    bias = _rand(N, seed=23).to(DEV)
    c = torch.zeros(M, N, device=DEV)
    nb = ops.splitk_workspace_bytes(torch.bfloat16, M, N, K)
    assert nb > 0
    ws = torch.empty(nb // 4, device=DEV)
    ops.gemm(a, b, c, M=M, N=N, K=K, a_kcontig=False, b_kcontig=False, lda=M, ldb=N, ldc=N,
             epilogue=L.EPI_ATOMIC | L.EPI_BIAS, bias=bias, workspace=ws)
    ref = a.double().t() @ b.double() + bias.double()
    assert rel(c, ref) < 2e-5


# ----------------------------------------------------------------------------------- LayerNorm
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("cols", [128, 192, 768])
@pytest.mark.parametrize("ws", [None, False])       # two-stage dgamma/dbeta reduction, or per-block atomics
def test_layernorm_fwd_bwd(dtype, cols, ws):
    from vspike import ops
    rows = 333
    x = _rand(rows, cols, seed=10) * 3 + 1
    g = 1 + 0.1 * _rand(cols, seed=11)
    b = 0.1 * _rand(cols, seed=12)
    dy = _rand(rows, cols, seed=13)
    dres = _rand(rows, cols, seed=14)
    y = torch.empty(rows, cols, dtype=dtype, device=DEV)
    mean = torch.empty(rows, device=DEV)
    rstd = torch.empty(rows, device=DEV)
    ops.layernorm_fwd(x.to(DEV), g.to(DEV), b.to(DEV), 1e-12, y, mean, rstd)
    xr = x.double().requires_grad_()
    gr, br = g.double().requires_grad_(), b.double().requires_grad_()
    yr = torch.nn.functional.layer_norm(xr, (cols,), gr, br, 1e-12)
    assert rel(y.float(), yr.detach()) < (1e-5 if dtype == torch.float32 else 5e-3)
    dx = torch.empty(rows, cols, device=DEV)
    dx_lp = torch.empty(rows, cols, dtype=torch.bfloat16, device=DEV)
    dg = torch.zeros(cols, device=DEV)
    db = torch.zeros(cols, device=DEV)
    ops.layernorm_bwd(dy.to(DEV), x.to(DEV), mean, rstd, g.to(DEV), dx, dg, db, dres=dres.to(DEV), dx_lp=dx_lp,
                      workspace=ws)
    gx, gg, gb = torch.autograd.grad(yr, (xr, gr, br), dy.double())
    assert rel(dx, gx + dres.double()) < 1e-5
    assert torch.equal(dx_lp, dx.to(torch.bfloat16))          # the bf16 copy is the rounded f32 result
    assert rel(dg, gg) < 1e-5 and rel(db, gb) < 1e-5
    # no residual gradient
    dx2 = torch.empty(rows, cols, device=DEV)
    dg.zero_()
    db.zero_()
    ops.layernorm_bwd(dy.to(DEV), x.to(DEV), mean, rstd, g.to(DEV), dx2, dg, db, workspace=ws)
    assert rel(dg, gg) < 1e-5 and rel(db, gb) < 1e-5
    assert rel(dx2, gx) < 1e-5
    # bf16 incoming gradient (the bf16 ViT block's dh1 / dh2): exact vs fp64 on the same rounded dy
    dyb = dy.to(torch.bfloat16)
    yr2 = torch.nn.functional.layer_norm(xr, (cols,), gr, br, 1e-12)
    gxb, ggb, gbb = torch.autograd.grad(yr2, (xr, gr, br), dyb.double())
    dx3 = torch.empty(rows, cols, device=DEV)
    dg.zero_()
    db.zero_()
    ops.layernorm_bwd(dyb.to(DEV), x.to(DEV), mean, rstd, g.to(DEV), dx3, dg, db, dres=dres.to(DEV), workspace=ws)
    assert rel(dx3, gxb + dres.double()) < 1e-5
    assert rel(dg, ggb) < 1e-5 and rel(db, gbb) < 1e-5


# ----------------------------------------------------------------------------------- attention
def _attn_ref(qkv, B, N, H, scale=0.125):
    D = H * 64
    q, k, v = qkv.view(B, N, 3, H, 64).permute(2, 0, 3, 1, 4)
    p = torch.softmax((q @ k.transpose(-1, -2)) * scale, dim=-1)
    o = (p @ v).permute(0, 2, 1, 3).reshape(B * N, D)
    lse = torch.logsumexp((q @ k.transpose(-1, -2)) * scale, dim=-1)
    return o, lse


ATTN_SHAPES = [(1, 100, 1), (2, 196, 2), (1, 1568, 3), (2, 130, 1)]


@pytest.mark.parametrize("variant", [0, 6, 8])
@pytest.mark.parametrize("shape", ATTN_SHAPES + [(2, 3136, 1), (1, 1600, 2), (3, 33, 1), (1, 1, 1)])
def test_attention_fwd_variants(knobs, variant, shape):
    """The bf16 forward kernels (VS_KNOB_ATTN_VARIANT low nibble: 0 = 3 waves/SIMD x 32 rows with
    QK(b) issued ahead of PV(a); 6 = the same body in the round-2 order; 8 = the same tile on
    16x16x32 MFMAs) against fp64 on the same bf16 inputs, at tails of
    every kind: N = 1 / 33 / 100 / 130 / 196 (partial 32-key block), 1568 (= 4 x 384 + 32: a
    workgroup with one live q-block), 1600 (partial 64-key tile), 3136 (C5: 98 blocks)."""
    from vspike import ops
    knobs("attn_variant", variant)
    B, N, H = shape
    D = H * 64
    qkv = _rand(B * N, 3 * D, seed=24, scale=1.5).to(torch.bfloat16)
    o = torch.full((B * N, D), 7.0, dtype=torch.bfloat16, device=DEV)
    lse = torch.full((B, H, N), 7.0, device=DEV)
    ops.attn_fwd(qkv.to(DEV), o, lse, B, N, H)
    torch.cuda.synchronize()
    o_ref, lse_ref = _attn_ref(qkv.double(), B, N, H)
    assert rel(o.float(), o_ref) < 1.5e-2
    assert rel(lse, lse_ref) < 3e-3
    per = ((o.float().cpu().double() - o_ref).view(B, N, H, 64).norm(dim=(1, 3)) /
           o_ref.view(B, N, H, 64).norm(dim=(1, 3)))
    assert float(per.max()) < 3e-2


@pytest.mark.parametrize("variant", [0, 0x60, 0x90])
@pytest.mark.parametrize("shape", ATTN_SHAPES + [(2, 3136, 1), (1, 1600, 2), (3, 33, 1), (1, 1, 1), (1, 400, 1)])
def test_attention_bwd_variants(knobs, variant, shape):
    """The bf16 backward kernels (VS_KNOB_ATTN_VARIANT bits 4-7: 0 = picked by grid size; 6 = software-
    pipelined pairs of 32-row units, 2 waves/SIMD; 9 = 3 waves/SIMD x 32 rows) against the fp64 gradient of
    the fp64 attention on the same bf16 inputs, O and LSE from the forward kernel (as in training),
    at the tails of test_attention_fwd_variants."""
    from vspike import ops
    knobs("attn_variant", variant)
    B, N, H = shape
    D = H * 64
    qkv = _rand(B * N, 3 * D, seed=25, scale=1.5).to(torch.bfloat16)
    do = _rand(B * N, D, seed=26).to(torch.bfloat16)
    qd = qkv.to(DEV)
    o = torch.empty(B * N, D, dtype=torch.bfloat16, device=DEV)
    lse = torch.empty(B, H, N, device=DEV)
    ops.attn_fwd(qd, o, lse, B, N, H)
    dqkv = torch.full((B * N, 3 * D), 7.0, dtype=torch.bfloat16, device=DEV)
    ws = torch.empty(ops.attn_bwd_workspace_bytes(B, N, H) // 4 + 64, device=DEV)
    ops.attn_bwd(qd, o, do.to(DEV), lse, dqkv, ws, B, N, H)
    torch.cuda.synchronize()
    ref_in = qkv.double().requires_grad_()
    o_ref, _ = _attn_ref(ref_in, B, N, H)
    (g_ref,) = torch.autograd.grad(o_ref, ref_in, do.double())
    for part in range(3):
        sl = slice(part * D, (part + 1) * D)
        e = rel(dqkv[:, sl].float(), g_ref[:, sl])
        assert e < 3e-2, ("qkv"[part], e)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape", ATTN_SHAPES)
def test_attention_fwd_bwd(dtype, shape):
    from vspike import ops
    B, N, H = shape
    D = H * 64
    qkv = _rand(B * N, 3 * D, seed=20, scale=1.5).to(dtype)
    do = _rand(B * N, D, seed=21).to(dtype)
    qd = qkv.to(DEV)
    o = torch.empty(B * N, D, dtype=dtype, device=DEV)
    lse = torch.empty(B, H, N, device=DEV)
    ops.attn_fwd(qd, o, lse, B, N, H)
    ref_in = qkv.double().requires_grad_()
    o_ref, lse_ref = _attn_ref(ref_in, B, N, H)
    ftol = 1e-5 if dtype == torch.float32 else 1.5e-2
    assert rel(o.float(), o_ref.detach()) < ftol
    assert rel(lse, lse_ref.detach()) < (1e-5 if dtype == torch.float32 else 3e-3)
    dqkv = torch.empty(B * N, 3 * D, dtype=dtype, device=DEV)
    ws = torch.empty(ops.attn_bwd_workspace_bytes(B, N, H) // 4 + 64, device=DEV)
    # the backward consumes the forward's own O (as in training)
    ops.attn_bwd(qd, o, do.to(DEV), lse, dqkv, ws, B, N, H)
    (g_ref,) = torch.autograd.grad(o_ref, ref_in, do.double())
    btol = 2e-5 if dtype == torch.float32 else 3e-2
    for part in range(3):
        sl = slice(part * D, (part + 1) * D)
        assert rel(dqkv[:, sl].float(), g_ref[:, sl]) < btol, ("qkv"[part], rel(dqkv[:, sl].float(), g_ref[:, sl]))


def test_attention_bf16_matches_f32_kernel_on_same_inputs():
    """bf16 MFMA path vs the exact f32 kernel on identical (bf16-representable) inputs."""
    from vspike import ops
    B, N, H = 2, 1568, 3
    D = H * 64
    qkv = _rand(B * N, 3 * D, seed=30, scale=2.0).to(torch.bfloat16)
    o16 = torch.empty(B * N, D, dtype=torch.bfloat16, device=DEV)
    o32 = torch.empty(B * N, D, device=DEV)
    l16 = torch.empty(B, H, N, device=DEV)
    l32 = torch.empty(B, H, N, device=DEV)
    ops.attn_fwd(qkv.to(DEV), o16, l16, B, N, H)
    ops.attn_fwd(qkv.float().to(DEV), o32, l32, B, N, H)
    assert rel(o16.float(), o32) < 1e-2
    # the bf16 kernel pre-scales Q by log2(e)/8 in bf16 (one extra rounding of each q element,
    # 2^-9 relative): LSE agrees to ~1.3e-3 relative at |scores| ~ 50
    assert rel(l16, l32) < 3e-3


@pytest.mark.parametrize("variant", [0, 6, 8])
def test_attention_rescale_branch_forced(knobs, variant):
    """A huge score late in the sequence forces the online-softmax rescale (guide rule 26)."""
    from vspike import ops
    knobs("attn_variant", variant)
    B, N, H = 1, 700, 1
    qkv = _rand(N, 192, seed=40, scale=0.5)
    qkv[600, 64:128] = qkv[5, 0:64] * 40.0            # key 600 dominates query 5
    for dtype, tol in ((torch.float32, 1e-5), (torch.bfloat16, 2e-2)):
        x = qkv.to(dtype)
        o = torch.empty(N, 64, dtype=dtype, device=DEV)
        lse = torch.empty(1, 1, N, device=DEV)
        ops.attn_fwd(x.to(DEV), o, lse, B, N, H)
        o_ref, _ = _attn_ref(x.double(), B, N, H)
        assert rel(o.float(), o_ref) < tol


@pytest.mark.gpu
@pytest.mark.parametrize("variant", [0, 6, 8])
def test_attention_extreme_logits_move_reference(knobs, variant):
    """Queries whose scores all lie far below / above 0 force the forward's softmax reference off
    its default 0 on the first block (m < -32 or > 32 in log2 units), then a late larger score
    moves it again; the rest of the wave stays on the unshifted fast path."""
    from vspike import ops
    knobs("attn_variant", variant)
    B, N, H = 1, 900, 1
    qkv = _rand(N, 192, seed=41, scale=0.3)
    u = torch.ones(64) / 8.0
    qkv[:, 64:128] += u * 6.0                           # every key ~ u
    qkv[3, 0:64] = -u * 400.0                           # query 3: all scores ~ -37..-40 (log2 ~ -55)
    qkv[40, 0:64] = u * 400.0                           # query 40: all scores ~ +37 (log2 ~ +55)
    qkv[70, 0:64] = qkv[800, 64:128] * 30.0             # query 70: key 800 dominates late
    for dtype, tol in ((torch.float32, 1e-5), (torch.bfloat16, 2e-2)):
        x = qkv.to(dtype)
        o = torch.empty(N, 64, dtype=dtype, device=DEV)
        lse = torch.empty(1, 1, N, device=DEV)
        ops.attn_fwd(x.to(DEV), o, lse, B, N, H)
        o_ref, lse_ref = _attn_ref(x.double(), B, N, H)
        assert torch.isfinite(o.float()).all() and torch.isfinite(lse).all()
        assert rel(o.float(), o_ref) < tol
        assert rel(lse, lse_ref) < (1e-5 if dtype == torch.float32 else 3e-3)
        for r in (3, 40, 70):
            assert rel(o[r].float(), o_ref[r]) < 3 * tol, r


# ---------------------------------------------------------------------------- im2col / misc ops
def test_im2col_matches_oracle():
    from oracle import cpu_ref
    from vspike import ops
    cfg = cpu_ref.VIT_SMALL_FIXTURE
    px = torch.from_numpy(cpu_ref.make_pixels(cfg, 2))
    ref = cpu_ref.im2col(px, cfg)
    for dtype in (torch.float32, torch.bfloat16):
        out = torch.empty(ref.shape, dtype=dtype, device=DEV)
        ops.patch_im2col(px.to(DEV), out, cfg.tubelet_size, cfg.patch_size)
        assert torch.equal(out.cpu(), ref.to(dtype))


@pytest.mark.parametrize("D", [64, 128, 192])
@pytest.mark.parametrize("geo", [(6, 16, 3, 224, 224), (3, 8, 3, 112, 112), (1, 4, 1, 32, 48)])
def test_patch_embed_fused_matches_im2col_gemm(knobs, D, geo):
    """vs_patch_embed_fwd (tubelet gather in the GEMM's A-load, bias + position table in the epilogue)
    against the im2col + row-slab GEMM path on the same inputs: the same bf16 operands, MFMA tiles,
    k order and epilogue, so the outputs agree to the last bit; the optional bf16 cols side output
    equals im2col's.  Also against fp64 (Conv3d on the bf16-rounded pixels).  Geometries: the bench
    clips (B=6 of 16 x 224^2: M = 9,408 rows, the row-slab GEMM's range), a ragged token count (3 clips x 4 x 7 x 7), 1 channel / non-square."""
    from oracle import cpu_ref
    from vspike import ops, _lib as L
    B, F, C, H, W = geo
    t, p = 2, 16
    n_tok = (F // t) * (H // p) * (W // p)
    M, K = B * n_tok, C * t * p * p
    px = _rand(B, F, C, H, W, seed=90)
    w = _rand(D, K, seed=91, scale=K ** -0.5).to(torch.bfloat16).to(DEV)
    bias = _rand(D, seed=92).to(DEV)
    pos = cpu_ref.sinusoid_table(n_tok, D).to(DEV)
    out = torch.full((M, D), 3.0, device=DEV)
    cols = torch.zeros(M, K, dtype=torch.bfloat16, device=DEV)
    L.dispatch_reset()
    ops.patch_embed_fwd(px.to(DEV), w, bias, pos, out, t, p, cols=cols)
    out2 = torch.full((M, D), 5.0, device=DEV)
    ops.patch_embed_fwd(px.to(DEV), w, bias, pos, out2, t, p)          # no side output
    assert L.dispatch_counts()["patch_fused"] == 2
    ref_cols = torch.empty(M, K, dtype=torch.bfloat16, device=DEV)
    ops.patch_im2col(px.to(DEV), ref_cols, t, p)
    knobs("no_slab", 0)
    ref = torch.empty(M, D, device=DEV)
    ops.linear(ref_cols, w, ref, bias=bias, epilogue=L.EPI_POS, pos=pos, pos_rows=n_tok)
    torch.cuda.synchronize()
    assert torch.equal(cols, ref_cols)
    assert torch.equal(out, out2)
    r64 = ref_cols.double() @ w.double().t() + bias.double() + pos.double().repeat(B, 1)
    assert rel(out, r64) < 1e-5
    if M >= 8192:      # the row-slab kernel (the im2col path's GEMM at M >= 8192): the same bits
        assert torch.equal(out, ref)
    else:
        assert rel(out, ref.double()) < 1e-5


@pytest.mark.parametrize("D", [64, 128, 192, 768])
@pytest.mark.parametrize("geo", [(2, 16, 3, 224, 224), (3, 8, 3, 112, 112), (1, 4, 1, 32, 48), (128, 16, 3, 224, 224)])
def test_patch_embed_dw_matches_im2col_dw(D, geo, knobs):
    """vs_patch_embed_dw (the tubelet gather in the dW kernel's B-operand load, no cols) against
    vs_patch_im2col + the dW product of vs_gemm on the same inputs: the same bf16 operand rounding,
    split plan, MFMA order and fixed-order split reduce, so dW and db agree to the last bit (both
    accumulate into non-zero gradients); and against fp64.  Geometries: 2 bench clips, a ragged token
    count (3 x 4 x 7 x 7 = 1,176: a partial last 64-token step), 12 tokens (one partial step), and the
    bench's 128 clips (200,704 tokens) at D = 192 (C2) and D = 768 (C3's width)."""
    from vspike import ops, _lib as L
    B, F, C, H, W = geo
    if B == 128 and D not in (192, 768):
        pytest.skip("bench batch at the ViT-Tiny / ViT-Base widths only")
    t, p = 2, 16
    if D > C * t * p * p:
        pytest.skip("the gather dW keeps D on the tile's narrow side: D <= C * 512 (ops.patch_dw_ok)")
    n_tok = (F // t) * (H // p) * (W // p)
    M, K = B * n_tok, C * t * p * p
    g = torch.Generator(device=DEV).manual_seed(93)
    px = torch.randn(B, F, C, H, W, device=DEV, generator=g)
    dx = torch.randn(M, D, device=DEV, generator=g).to(torch.bfloat16)
    dw0 = torch.randn(D, K, device=DEV, generator=g)
    db0 = torch.randn(D, device=DEV, generator=g)
    dw, db = dw0.clone(), db0.clone()
    L.dispatch_reset()
    ops.patch_embed_dw(px, dx, dw, db, t, p)
    assert L.dispatch_counts()["patch_dw"] == 1
    cols = torch.empty(M, K, dtype=torch.bfloat16, device=DEV)
    ops.patch_im2col(px, cols, t, p)
    dw2, db2 = dw0.clone(), db0.clone()
    knobs("no_dw256", 1)          # the same split-K dW kernel as the gather path (bitwise comparison)
    ops.linear_dw(dx, cols, dw2, db=db2)
    torch.cuda.synchronize()
    assert torch.equal(dw, dw2) and torch.equal(db, db2)
    if M <= 4096:
        r64 = dw0.double() + dx.double().t() @ cols.double()
        assert rel(dw, r64) < 1e-5
        assert rel(db, db0.double() + dx.double().sum(0)) < 1e-5


def test_sinusoid_table_matches_oracle():
    from oracle import cpu_ref
    from vspike import ops
    t = ops.sinusoid_table(1568, 192, DEV)
    assert (t.cpu() - cpu_ref.sinusoid_table(1568, 192)).abs().max().item() < 1e-6


@pytest.mark.parametrize("rows,cols,dtype", [(1000, 300, torch.float32), (25088, 192, torch.bfloat16),
                                             (777, 576, torch.float32), (64, 8, torch.bfloat16)])
def test_colsum(rows, cols, dtype):
    from vspike import ops
    x = _rand(rows, cols, seed=50).to(dtype)
    out = torch.full((cols,), 2.0, device=DEV)
    ops.colsum(x.to(DEV), out)
    assert rel(out, x.double().sum(0) + 2.0) < 1e-5


def test_cast():
    from vspike import ops
    x = _rand(1000, 300, seed=50)
    xb = torch.empty(1000, 300, dtype=torch.bfloat16, device=DEV)
    ops.cast(x.to(DEV), xb)
    assert torch.equal(xb.cpu(), x.to(torch.bfloat16))


def test_poisson_nll_and_grad():
    from oracle import prng
    from vspike import ops
    x = _rand(4, 100, 128, seed=60, scale=0.5)
    y = torch.from_numpy(prng.spike_targets(1, (4, 100, 128)))
    loss = torch.empty((), device=DEV)
    dx = torch.empty_like(x, device=DEV)
    ops.poisson_nll(x.to(DEV), y.to(DEV), loss, dx=dx)
    xr = x.double().requires_grad_()
    lr = torch.nn.PoissonNLLLoss(log_input=True, reduction="none")(xr, y.double()).mean()
    (gr,) = torch.autograd.grad(lr, xr)
    assert abs(loss.item() - lr.item()) < 1e-6 * abs(lr.item())
    assert rel(dx, gr) < 1e-6


def test_mse_loss_and_grad():
    """The MSE head option (vs_mse_loss) against torch.nn.MSELoss() in fp64: loss, gradient, the
    upstream-scaled backward entry point, and a ragged size (n not a multiple of the block)."""
    from vspike import ops, mse_mean
    for shape in ((4, 100, 128), (3, 7, 11)):
        x = _rand(*shape, seed=61, scale=0.7)
        y = _rand(*shape, seed=62).abs() * 3.0
        loss = torch.empty((), device=DEV)
        dx = torch.empty_like(x, device=DEV)
        ops.mse_loss(x.to(DEV), y.to(DEV), loss, dx=dx)
        xr = x.double().requires_grad_()
        lr = torch.nn.MSELoss()(xr, y.double())
        (gr,) = torch.autograd.grad(lr, xr)
        assert abs(loss.item() - lr.item()) < 1e-6 * abs(lr.item())
        assert rel(dx, gr) < 1e-6
        g = torch.tensor([0.5], device=DEV)
        dx2 = torch.empty_like(dx)
        ops.mse_loss_bwd(x.to(DEV), y.to(DEV), g, dx2)
        assert rel(dx2, 0.5 * gr) < 1e-6
        xa = x.to(DEV).requires_grad_()
        la = mse_mean(xa, y.to(DEV))
        (la * 3.0).backward()
        assert rel(xa.grad, 3.0 * gr) < 1e-6


def test_fused_adamw_matches_torch():
    from vspike import FusedAdamW
    p0 = _rand(5000, seed=70)
    grads = [_rand(5000, seed=71 + i) for i in range(4)]
    ref = p0.clone().requires_grad_()
    opt_r = torch.optim.AdamW([ref], lr=3e-3, weight_decay=0.01, eps=1e-8)
    mine = torch.nn.Parameter(p0.clone().to(DEV))
    opt_m = FusedAdamW([mine], lr=3e-3, weight_decay=0.01, eps=1e-8)
    for g in grads:
        ref.grad = g.clone()
        opt_r.step()
        mine.grad = g.to(DEV)
        opt_m.step()
    assert rel(mine.detach(), ref.detach()) < 1e-6
