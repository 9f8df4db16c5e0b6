"""MX-FP8 (BASELINE C5's fp8 MFMA): the quantiser (vs_quant_mxfp8) against a torch restatement of
the OCP MX recipe (E8M0 scale per 32 consecutive elements, e = ceil(log2(amax / 448)), elements
rounded to nearest-even e4m3 with torch.float8_e4m3fn), byte for byte; the block-scaled GEMM
(vs_gemm_mxfp8, v_mfma_scale_f32_32x32x64_f8f6f4) against the fp64 product of the DEQUANTISED
operands (exact products, so only the f32 accumulation differs: 1e-5 of max |ref|), with every
epilogue the ViT block uses.  Parity of the quantisation itself to the fp32 reference is a
property of the format (3 mantissa bits: <= 2^-4 relative per element), checked per element here
and, end to end, by the C5 model test in test_gpu_parity_bench.py.
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


def mx_ref(x):
    """(codes uint8 [M, K], exps uint8 [M, K/32]) of the MX-FP8 recipe, on the device in torch."""
    M, K = x.shape
    xb = x.float().view(M, K // 32, 32)
    amax = xb.abs().amax(-1)
    r = amax * torch.tensor(1.0 / 448.0, dtype=torch.float32, device=x.device)
    bits = r.view(torch.int32)
    e = ((bits >> 23) & 0xFF) - 127
    e = e + ((bits & 0x7FFFFF) != 0).int()
    e = torch.where(((bits >> 23) & 0xFF) == 0, torch.full_like(e, -126), e).clamp(-126, 127)
    e = torch.where(amax > 0, e, torch.zeros_like(e))
    inv = torch.ldexp(torch.ones_like(amax), -e)
    q = (xb * inv[..., None]).to(torch.float8_e4m3fn).view(torch.uint8).view(M, K)
    return q, (e + 127).to(torch.uint8)


def dequant(q, s):
    M, K = q.shape
    v = q.view(torch.float8_e4m3fn).double().view(M, K // 32, 32)
    return (v * torch.ldexp(torch.ones_like(s, dtype=torch.float64), s.long() - 127)[..., None]).view(M, K)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("M,K", [(3136, 768), (257, 3072), (5, 32)])
def test_quant_mxfp8_matches_recipe(dtype, M, K):
    from vspike import ops
    g = torch.Generator(device=DEV).manual_seed(M + K)
    x = torch.randn(M, K, device=DEV, generator=g) * torch.exp(torch.randn(M, 1, device=DEV, generator=g) * 3)
    x[0, :32] = 0.0                        # an all-zero block: scale 1 (e = 127), codes 0
    if M > 1:
        x[1, 5] = 448.0 * 4                # amax exactly 448 * 2^k
    x = x.to(dtype)
    q = torch.empty(M, K, dtype=torch.uint8, device=DEV)
    s = torch.empty(M, K // 32, dtype=torch.uint8, device=DEV)
    ops.quant_mxfp8(x, q, s)
    torch.cuda.synchronize()
    qr, sr = mx_ref(x)
    assert torch.equal(s, sr)
    bad = (q != qr).nonzero()
    if len(bad):
        scaled = (x.float().view(M, K // 32, 32) * torch.ldexp(torch.ones(M, K // 32, device=DEV),
                                                               127 - s.int())[..., None]).view(M, K)
        for r, c in bad[:12].tolist():
            print(f"  mismatch ({r},{c}): x*2^-e = {scaled[r, c].item()!r} ours {q[r, c].item():#04x} "
                  f"({q[r, c:c + 1].view(torch.float8_e4m3fn).float().item()!r}) torch {qr[r, c].item():#04x} "
                  f"({qr[r, c:c + 1].view(torch.float8_e4m3fn).float().item()!r})")
    print(f"\n[quant {M}x{K} {dtype}] code mismatches vs torch.float8_e4m3fn: {len(bad)} of {M * K}")
    assert torch.equal(q, qr), len(bad)
    # the format's own error bound: |deq - x| <= 2^-4 |x| (+ the smallest subnormal step of the block)
    d = dequant(q, s)
    xd = x.double()
    step = torch.ldexp(torch.ones_like(s, dtype=torch.float64), s.long() - 127 - 9).repeat_interleave(32, 1)
    assert bool(((d - xd).abs() <= xd.abs() * 2.0 ** -4 + step).all())


@pytest.mark.parametrize("M,N,K,epi", [(6272, 2304, 768, "bias"), (3136, 768, 768, "bias_res"),
                                       (3000, 3072, 768, "gelu"), (1000, 768, 3072, "bias_res"), (77, 128, 128, "none")])
def test_gemm_mxfp8_matches_dequantised_fp64(M, N, K, epi):
    from vspike import ops, _lib as L
    g = torch.Generator(device=DEV).manual_seed(M + N + K)
    x = torch.randn(M, K, device=DEV, generator=g).to(torch.bfloat16)
    w = (torch.randn(N, K, device=DEV, generator=g) * 0.05).to(torch.bfloat16)
    b = torch.randn(N, device=DEV, generator=g)
    res = torch.randn(M, N, device=DEV, generator=g)
    xq = torch.empty(M, K, dtype=torch.uint8, device=DEV)
    xs = torch.empty(M, K // 32, dtype=torch.uint8, device=DEV)
    wq = torch.empty(N, K, dtype=torch.uint8, device=DEV)
    ws = torch.empty(N, K // 32, dtype=torch.uint8, device=DEV)
    ops.quant_mxfp8(x, xq, xs)
    ops.quant_mxfp8(w, wq, ws)
    out_bf16 = epi in ("bias", "gelu")
    c = torch.full((M, N), 5.0, dtype=torch.bfloat16 if out_bf16 else torch.float32, device=DEV)
    aux = torch.empty(M, N, dtype=torch.bfloat16, device=DEV) if epi == "gelu" else None
    flags = {"none": 0, "bias": L.EPI_BIAS, "bias_res": L.EPI_BIAS | L.EPI_RESIDUAL,
             "gelu": L.EPI_BIAS | L.EPI_GELU | L.EPI_GELU_GRAD}[epi]
    L.dispatch_reset()
    ops.gemm_mxfp8(xq, xs, wq, ws, c, epilogue=flags, bias=b if epi != "none" else None,
                   residual=res if epi == "bias_res" else None, aux_out=aux)
    torch.cuda.synchronize()
    assert L.dispatch_counts()["gemm_fp8"] == 1
    ref = dequant(xq, xs) @ dequant(wq, ws).t()
    if epi != "none":
        ref = ref + b.double()
    if epi == "gelu":
        pre = ref.float().to(torch.bfloat16).double()
        ref = 0.5 * pre * (1 + torch.erf(pre / 2 ** 0.5))
    if epi == "bias_res":
        ref = ref + res.double()
    tol = 1e-5 if not out_bf16 else 8e-3
    err = float((c.double() - ref).abs().max() / ref.abs().max())
    print(f"\n[mxfp8 {M}x{N}x{K} {epi}] max rel err {err:.2e}")
    assert err < tol
    # and the fp8 product stays within the format's error of the bf16 product
    exact = x.double() @ w.double().t()
    pe = float(((dequant(xq, xs) @ dequant(wq, ws).t()) - exact).abs().max() / exact.abs().max())
    assert pe < 0.1
