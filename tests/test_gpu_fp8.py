"""MX-FP8 (BASELINE C5's fp8 MFMA): the quantiser (vs_quant_mxfp8) against a torch restatement of
the OCP MX recipe (E8M0 scale per 32 consecutive elements, e = ceil(log2(amax / 448)), elements
rounded to nearest-even e4m3 with torch.float8_e4m3fn), byte for byte; the block-scaled GEMM
(vs_gemm_mxfp8, v_mfma_scale_f32_32x32x64_f8f6f4) against the fp64 product of the DEQUANTISED
operands (exact products, so only the f32 accumulation differs: 1e-4 of max |ref|, measured 2.3e-5), with every
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
    inv = ((127 - e) << 23).view(torch.float32)       # 2^-e exactly (torch.ldexp is not exact)
    q = (xb * inv[..., None]).to(torch.float8_e4m3fn).view(torch.uint8).view(M, K)
    return q, (e + 127).to(torch.uint8)


def _pow2(e):
    """2^e exactly (f64), e an integer tensor in [-126, 127]."""
    return ((e.long() + 1023) << 52).view(torch.float64)


def dequant(q, s):
    M, K = q.shape
    v = q.view(torch.float8_e4m3fn).double().view(M, K // 32, 32)
    return (v * _pow2(s.long() - 127)[..., None]).view(M, K)


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
        scaled = (x.double().view(M, K // 32, 32) * _pow2(127 - s.long())[..., None]).view(M, K)
        for r, c in bad[:12].tolist():
            print(f"  mismatch ({r},{c}): x*2^-e = {scaled[r, c].item()!r} ours {q[r, c].item():#04x} "
                  f"({q[r, c:c + 1].view(torch.float8_e4m3fn).float().item()!r}) torch {qr[r, c].item():#04x} "
                  f"({qr[r, c:c + 1].view(torch.float8_e4m3fn).float().item()!r})")
    print(f"\n[quant {M}x{K} {dtype}] code mismatches vs torch.float8_e4m3fn: {len(bad)} of {M * K}")
    assert torch.equal(q, qr), len(bad)
    # the format's own error bound: |deq - x| <= 2^-4 |x| (+ the smallest subnormal step of the block)
    d = dequant(q, s)
    xd = x.double()
    step = _pow2(s.long() - 127 - 9).repeat_interleave(32, 1)
    assert bool(((d - xd).abs() <= xd.abs() * 2.0 ** -4 + step).all())


def test_gemm_mxfp8_operand_and_scale_map():
    """Structured inputs that expose the 32x32x64 f8 MFMA's operand / scale map: (a) random e4m3
    codes with unit scales (data pairing only); (b) all-ones data with a distinct scale per
    (row, k-block) (which scale meets which k-block)."""
    from vspike import ops
    g = torch.Generator(device=DEV).manual_seed(7)
    M, N, K = 64, 128, 256
    # (a) codes of values in [-4, 4] (exact in e4m3), unit scales
    av = (torch.randint(-8, 9, (M, K), device=DEV, generator=g).float() / 2).to(torch.float8_e4m3fn)
    bv = (torch.randint(-8, 9, (N, K), device=DEV, generator=g).float() / 2).to(torch.float8_e4m3fn)
    one_a = torch.full((M, K // 32), 127, dtype=torch.uint8, device=DEV)
    one_b = torch.full((N, K // 32), 127, dtype=torch.uint8, device=DEV)
    c = torch.empty(M, N, device=DEV)
    ops.gemm_mxfp8(av.view(torch.uint8), one_a, bv.view(torch.uint8), one_b, c)
    torch.cuda.synchronize()
    ref = av.double() @ bv.double().t()
    ea = float((c.double() - ref).abs().max())
    print(f"\n[mxfp8 map] (a) unit scales: max abs err {ea}")
    # (b) all ones, scale of A (row m, block kb) = 2^(kb % 4) * 2^(4 (m % 2)) ... distinct per block
    ones = torch.ones(M, K, device=DEV).to(torch.float8_e4m3fn).view(torch.uint8)
    onesb = torch.ones(N, K, device=DEV).to(torch.float8_e4m3fn).view(torch.uint8)
    kb = torch.arange(K // 32, device=DEV)
    sa = (127 + kb[None, :] + 8 * (torch.arange(M, device=DEV)[:, None] % 2)).to(torch.uint8)
    c2 = torch.empty(M, N, device=DEV)
    ops.gemm_mxfp8(ones, sa, onesb, one_b, c2)
    torch.cuda.synchronize()
    want = 32.0 * _pow2(sa.long() - 127).sum(1)
    print(f"[mxfp8 map] (b) A-scale per block: got rows 0,1 = {c2[0, 0].item()}, {c2[1, 0].item()}; "
          f"want {want[0].item()}, {want[1].item()}")
    # (c) B scales per block
    sb = (127 + kb[None, :] + 8 * (torch.arange(N, device=DEV)[:, None] % 2)).to(torch.uint8)
    c3 = torch.empty(M, N, device=DEV)
    ops.gemm_mxfp8(ones, one_a, onesb, sb, c3)
    torch.cuda.synchronize()
    wantb = 32.0 * _pow2(sb.long() - 127).sum(1)
    print(f"[mxfp8 map] (c) B-scale per block: got cols 0,1 = {c3[0, 0].item()}, {c3[0, 1].item()}; "
          f"want {wantb[0].item()}, {wantb[1].item()}")
    # (d) one k-block of A nonzero at a time (unit scales): which k positions pair
    for blk in range(K // 32):
        a1 = torch.zeros(M, K, device=DEV)
        a1[:, blk * 32:(blk + 1) * 32] = 1.0
        c4 = torch.empty(M, N, device=DEV)
        ops.gemm_mxfp8(a1.to(torch.float8_e4m3fn).view(torch.uint8), one_a, bv.view(torch.uint8), one_b, c4)
        torch.cuda.synchronize()
        r4 = a1.double() @ bv.double().t()
        print(f"[mxfp8 map] (d) only k-block {blk}: max abs err {float((c4.double() - r4).abs().max())}")
    # (e) subnormal e4m3 codes (exponent field 0), unit scales
    sub = torch.randint(1, 8, (M, K), device=DEV, generator=g).to(torch.uint8) | \
        (torch.randint(0, 2, (M, K), device=DEV, generator=g).to(torch.uint8) << 7)
    c5 = torch.empty(M, N, device=DEV)
    ops.gemm_mxfp8(sub, one_a, bv.view(torch.uint8), one_b, c5)
    torch.cuda.synchronize()
    r5 = sub.view(torch.float8_e4m3fn).double() @ bv.double().t()
    print(f"[mxfp8 map] (e) subnormal A codes: max abs err {float((c5.double() - r5).abs().max())} "
          f"(ref max {float(r5.abs().max())})")
    # (f) scales below 1 (E8M0 110..126), all-ones data
    sa_lo = (110 + kb[None, :] + 8 * (torch.arange(M, device=DEV)[:, None] % 2)).to(torch.uint8)
    c6 = torch.empty(M, N, device=DEV)
    ops.gemm_mxfp8(ones, sa_lo, onesb, one_b, c6)
    torch.cuda.synchronize()
    want6 = 32.0 * _pow2(sa_lo.long() - 127).sum(1)
    print(f"[mxfp8 map] (f) scales < 1: got rows 0,1 = {c6[0, 0].item()}, {c6[1, 0].item()}; "
          f"want {want6[0].item()}, {want6[1].item()}")
    # (g) quantised random data, unit scales substituted (data path of real codes)
    x = torch.randn(M, K, device=DEV, generator=g)
    xq = torch.empty(M, K, dtype=torch.uint8, device=DEV)
    xs = torch.empty(M, K // 32, dtype=torch.uint8, device=DEV)
    ops.quant_mxfp8(x, xq, xs)
    c7 = torch.empty(M, N, device=DEV)
    ops.gemm_mxfp8(xq, one_a, bv.view(torch.uint8), one_b, c7)
    torch.cuda.synchronize()
    r7 = xq.view(torch.float8_e4m3fn).double() @ bv.double().t()
    print(f"[mxfp8 map] (g) real codes, unit scales: max abs err {float((c7.double() - r7).abs().max())} "
          f"(ref max {float(r7.abs().max())}); codes {xq[0, :8].tolist()} scales {xs[0].tolist()}")
    c8 = torch.empty(M, N, device=DEV)
    ops.gemm_mxfp8(xq, xs, bv.view(torch.uint8), one_b, c8)
    torch.cuda.synchronize()
    r8 = dequant(xq, xs) @ bv.double().t()
    print(f"[mxfp8 map] (h) real codes + scales: max abs err {float((c8.double() - r8).abs().max())} "
          f"(ref max {float(r8.abs().max())}); c {c8[0, :4].tolist()} ref {r8[0, :4].tolist()}")
    # (i) several tiles and k-steps: exact small codes, unit scales, M = 600 (3 row tiles, ragged),
    # N = 256 (2 column tiles), K = 768 (6 k-steps): per tile / per k-step errors
    M2, N2, K2 = 600, 256, 768
    a2 = (torch.randint(-8, 9, (M2, K2), device=DEV, generator=g).float() / 2).to(torch.float8_e4m3fn)
    b2 = (torch.randint(-8, 9, (N2, K2), device=DEV, generator=g).float() / 2).to(torch.float8_e4m3fn)
    sa2 = torch.full((M2, K2 // 32), 127, dtype=torch.uint8, device=DEV)
    sb2 = torch.full((N2, K2 // 32), 127, dtype=torch.uint8, device=DEV)
    c9 = torch.empty(M2, N2, device=DEV)
    ops.gemm_mxfp8(a2.view(torch.uint8), sa2, b2.view(torch.uint8), sb2, c9)
    torch.cuda.synchronize()
    r9 = a2.double() @ b2.double().t()
    e9 = (c9.double() - r9).abs()
    tiles = [[float(e9[i * 256:(i + 1) * 256, j * 128:(j + 1) * 128].max()) for j in range(2)] for i in range(3)]
    print(f"[mxfp8 map] (i) 3x2 tiles, 6 k-steps, unit scales: max abs err per tile {tiles}")
    for ks in range(K2 // 128):
        a3 = torch.zeros(M2, K2, device=DEV)
        a3[:, ks * 128:(ks + 1) * 128] = a2[:, ks * 128:(ks + 1) * 128].float()
        c10 = torch.empty(M2, N2, device=DEV)
        ops.gemm_mxfp8(a3.to(torch.float8_e4m3fn).view(torch.uint8), sa2, b2.view(torch.uint8), sb2, c10)
        torch.cuda.synchronize()
        r10 = a3.double() @ b2.double().t()
        print(f"[mxfp8 map] (i) only k-step {ks}: max abs err {float((c10.double() - r10).abs().max())}")
    # (j) which row's scale meets row m: data = ones in ONE k-block kb only, scale of row m = 2^(m - 40)
    # (distinct per row): C[m, n] = 32 * 2^(src - 40) names the row src whose scale was applied
    import math
    for kbj in (0, 1, 2, 5):
        a4 = torch.zeros(M, K, device=DEV)
        a4[:, kbj * 32:(kbj + 1) * 32] = 1.0
        sa4 = (87 + torch.arange(M, device=DEV)[:, None] + 0 * kb[None, :]).to(torch.uint8)
        c11 = torch.empty(M, N, device=DEV)
        ops.gemm_mxfp8(a4.to(torch.float8_e4m3fn).view(torch.uint8), sa4, onesb, one_b, c11)
        torch.cuda.synchronize()
        src = [round(math.log2(max(v, 1e-30) / 32.0)) + 40 for v in c11[:, 0].tolist()]
        print(f"[mxfp8 map] (j) A k-block {kbj}: scale source row per row m: {src}")
        sb4 = (87 + torch.arange(N, device=DEV)[:, None] + 0 * kb[None, :]).to(torch.uint8)
        c12 = torch.empty(M, N, device=DEV)
        ops.gemm_mxfp8(a4.to(torch.float8_e4m3fn).view(torch.uint8), one_a, onesb, sb4, c12)
        torch.cuda.synchronize()
        srcb = [round(math.log2(max(v, 1e-30) / 32.0)) + 40 for v in c12[0, :64].tolist()]
        print(f"[mxfp8 map] (j) B k-block {kbj}: scale source col per col n < 64: {srcb}")
    # (k) which k-block scale meets k position p: A = 1 at k = p only, scale of block kb = 2^kb
    sak = (127 + kb[None, :] + 0 * torch.arange(M, device=DEV)[:, None]).to(torch.uint8)
    blocks = []
    for p in range(0, K, 4):
        a5 = torch.zeros(M, K, device=DEV)
        a5[:, p] = 1.0
        c13 = torch.empty(M, N, device=DEV)
        ops.gemm_mxfp8(a5.to(torch.float8_e4m3fn).view(torch.uint8), sak, onesb, one_b, c13)
        torch.cuda.synchronize()
        blocks.append(round(math.log2(max(float(c13[0, 0]), 1e-30))))
    print(f"[mxfp8 map] (k) A scale block applied at k = 0, 4, 8, ...: {blocks}")
    assert ea == 0.0
    assert blocks == [p // 32 for p in range(0, K, 4)]          # each 32-k block meets its own scale
    assert float((c8.double() - r8).abs().max()) < 1e-4 * float(r8.abs().max())


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
    # f32 output: the block-scaled MFMA's own accumulation order (measured up to 2.3e-5 of max |ref| at
    # K = 768..3072); bf16 output: its rounding
    tol = 1e-4 if not out_bf16 else 8e-3
    err = float((c.double() - ref).abs().max() / ref.abs().max())
    print(f"\n[mxfp8 {M}x{N}x{K} {epi}] max rel err {err:.2e}")
    assert err < tol
    # and the fp8 product stays within the format's error of the bf16 product
    exact = x.double() @ w.double().t()
    pe = float(((dequant(xq, xs) @ dequant(wq, ws).t()) - exact).abs().max() / exact.abs().max())
    assert pe < 0.1
