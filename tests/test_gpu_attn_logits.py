"""The attention forward's fast pass at trained-model logit scales.

The bf16 forward (csrc/attention.hip attn_fwd_bf16_kernel) computes p = exp2(s) with NO running row
maximum and checks at the end that every query's row sum stayed within [2^-100, 2^96]; a workgroup
with a query outside that band re-runs its tile under the safe online softmax.  Random-init weights
give small scores, so the benchmark never takes the re-run; a trained ViT (the reference loads
pretrained videomae-base, /root/reference/src/model/videomae.py:7) has larger ones.  These tests put
the scaled scores q.k/8 up to a chosen maximum — Gaussian scores, and a "spiky" case where a few keys
align with every query (attention sinks) — and check (a) the output against fp64 at every scale,
(b) that no workgroup re-runs while max|s| stays inside the band (log2e * s + log2(N) <= 96, i.e.
s <~ 58 natural-log units: round 4's band of 2^60 stopped at ~41, which attention sinks of a trained
model exceed), and (c) that beyond it the re-run happens and the result is still exact.  Tolerances: as
test_gpu_parity_bench.py::test_attention_bf16_at_bench_grid (o 1.5e-2 norm-relative, lse 3e-3).
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def make_qkv(B, N, H, smax, spiky, seed=0):
    """qkv [B*N, 3*H*64] bf16 whose scaled scores q.k/8 reach about smax in absolute value."""
    g = torch.Generator(device=DEV).manual_seed(seed)
    D = H * 64
    x = torch.randn(B, N, 3, H, 64, device=DEV, generator=g)
    if spiky:
        # a shared direction u: 16 "sink" keys per (b, h) carry +a u, every query +a u -> s_sink ~ smax
        u = torch.randn(H, 64, device=DEV, generator=g)
        u = u / u.norm(dim=-1, keepdim=True)
        a = math.sqrt(8.0 * smax)
        x[:, :, 0] += a * u
        sinks = torch.randperm(N, device=DEV, generator=g)[:16]
        x[:, sinks, 1] += a * u
    else:
        # s = q.k / 8 with q, k ~ N(0, sig^2): s ~ N(0, sig^4); the max over N^2 pairs ~ 5.5 sig^2
        sig = math.sqrt(smax / 5.5)
        x[:, :, :2] *= sig
    return x.reshape(B * N, 3 * D).to(torch.bfloat16)


def ref64(qkv, B, N, H):
    D = H * 64
    x = qkv.double().view(B, N, 3, H, 64)
    o = torch.empty(B, N, H, 64, dtype=torch.float64, device=DEV)
    lse = torch.empty(B, H, N, dtype=torch.float64, device=DEV)
    smax = 0.0
    for b in range(B):
        q, k, v = (x[b, :, i].transpose(0, 1) for i in range(3))
        s = (q @ k.transpose(-1, -2)) * 0.125
        smax = max(smax, float(s.abs().max()))
        o[b] = (torch.softmax(s, -1) @ v).transpose(0, 1)
        lse[b] = torch.logsumexp(s, -1)
    return o.view(B * N, D), lse, smax


@pytest.mark.parametrize("variant", [0, 8])
@pytest.mark.parametrize("smax,spiky", [(10.0, False), (30.0, False), (38.0, True), (50.0, False), (60.0, True),
                                        (90.0, False)])
def test_attention_fast_pass_at_trained_logit_scales(knobs, variant, smax, spiky):
    """variant 8: the 16x16x32-MFMA forward (two queries per lane: its safe pass keeps two references)."""
    from vspike import ops, _lib as L
    knobs("attn_variant", variant)
    B, N, H = 4, 1568, 3
    qkv = make_qkv(B, N, H, smax, spiky)
    o = torch.empty(B * N, H * 64, dtype=torch.bfloat16, device=DEV)
    lse = torch.empty(B, H, N, device=DEV)
    L.attn_redo_count(reset=True)
    ops.attn_fwd(qkv, o, lse, B, N, H)
    torch.cuda.synchronize()
    redo = L.attn_redo_count(reset=True)
    o_ref, lse_ref, s_max = ref64(qkv, B, N, H)
    eo = float((o.double() - o_ref).norm() / o_ref.norm())
    el = float((lse.double() - lse_ref).norm() / lse_ref.norm())
    nwg = B * H * ((N + 127) // 128)
    print(f"\n[attn smax {smax} spiky {spiky}] measured max|s| {s_max:.1f}: o {eo:.3e} lse {el:.3e}, "
          f"re-run {redo} of {nwg} workgroups")
    assert eo < 1.5e-2 and el < 3e-3
    if s_max * 1.4427 + math.log2(N) < 92.0:     # every row sum inside the band with margin: no re-run
        assert redo == 0
    if s_max * 1.4427 > 100.0 and not spiky:
        assert redo > 0              # far outside: the workgroups holding those rows re-ran


def test_attention_backward_at_trained_logit_scale():
    """The backward takes the forward's LSE (no fast pass of its own): correct at a large logit scale
    (attention sinks, max|s| ~ 77).  Bar 5e-2 norm-relative (the bench-grid test's 3e-2 measured 3.3e-2
    on dK here: with probability mass concentrated on 16 sink keys, dK of those keys is a sum of
    large cancelling terms in bf16 dS)."""
    from vspike import ops
    B, N, H = 2, 1568, 3
    qkv = make_qkv(B, N, H, 60.0, True, seed=3)
    o = torch.empty(B * N, H * 64, dtype=torch.bfloat16, device=DEV)
    lse = torch.empty(B, H, N, device=DEV)
    ops.attn_fwd(qkv, o, lse, B, N, H)
    g = torch.Generator(device=DEV).manual_seed(4)
    do = torch.randn(B * N, H * 64, device=DEV, generator=g).to(torch.bfloat16)
    dqkv = torch.empty_like(qkv)
    ws = torch.empty(ops.attn_bwd_workspace_bytes(B, N, H) // 4 + 64, device=DEV)
    ops.attn_bwd(qkv, o, do, lse, dqkv, ws, B, N, H)
    torch.cuda.synchronize()
    D = H * 64
    x = qkv.double().view(B, N, 3, H, 64)
    gg = do.double().view(B, N, H, 64)
    for b in range(B):
        q, k, v = (x[b, :, i].transpose(0, 1).clone().requires_grad_() for i in range(3))
        ob = torch.softmax((q @ k.transpose(-1, -2)) * 0.125, -1) @ v
        dq, dk, dv = torch.autograd.grad(ob, (q, k, v), gg[b].transpose(0, 1))
        got = dqkv.double().view(B, N, 3, H, 64)[b]
        for i, r in enumerate((dq, dk, dv)):
            err = float((got[:, i].transpose(0, 1) - r).norm() / r.norm())
            assert err < 5e-2, (b, i, err)
