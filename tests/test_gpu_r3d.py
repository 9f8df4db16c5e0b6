"""BASELINE C4: the R3D-18 encoder (csrc/conv3d.hip, vspike/r3d.py) against the CPU oracle's torch
restatement (oracle/cpu_ref.py r3d18_forward: F.conv3d / F.batch_norm / F.relu on NCDHW tensors).

PARITY UNPINNED: the reference has no CNN encoder, so no reference output
exists for this path; the oracle restates torchvision's published r3d_18 (not installed here).

Tolerances (fp32 path, exact-f32 MFMA with a different summation order than the CPU):
  * ops: conv outputs / dX / dW within 1e-5 of max|ref| (an f32 sum over K = 27 * Ci <= 13,824 terms),
    BatchNorm within 1e-5;
  * the model at C4's full geometry (32 x 112 x 112, B = 2) against the oracle run in f64: log-rates
    1e-4 of max|ref| (the north star's fp32 bar), loss 1e-5 relative, every conv / head gradient 1e-3
    of its norm and every BatchNorm affine gradient 3e-3 (they are sums of ~10^4-10^5 terms that
    cancel to ~1e-3 of their absolute sums: an f32 CPU reference carries up to 2e-3 itself, and a
    ReLU mask flipping within rounding of zero moves them by one whole element), or 3x torch-f32's
    own distance from f64 where that is larger; running statistics 1e-5; a 3-step AdamW + OneCycleLR
    curve within 1e-4 of the f32 oracle's; eval mode (running statistics) 1e-4.
"""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import cpu_ref, prng

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _maxrel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def _cl(x):           # NCDHW -> channels-last NDHWC
    return x.permute(0, 2, 3, 4, 1).contiguous()


def _tile_partials(yr):
    """The BatchNorm statistics partials vs_conv3d_fwd writes, in f64: per 128-row tile the column sum
    and the column sum of squared deviations from the tile mean."""
    S, M2 = [], []
    for i in range(0, yr.shape[0], 128):
        t = yr[i:i + 128].double()
        S.append(t.sum(0))
        M2.append(((t - t.mean(0)) ** 2).sum(0))
    return torch.stack(S), torch.stack(M2)


def _spec(ci, co, k, s, p):
    from vspike.r3d import ConvSpec
    return ConvSpec("t.0", ci, co, k, s, p, ci)


# (N, D, H, W, Ci, Co, k, s, p): the stem, the stride-1 3x3x3 body conv, the stride-2 first convs of
# stages 2-4, the 1x1x1 stride-2 shortcut, odd extents (tails of the 128-row tiles, parity classes of
# unequal size)
CONV_CASES = [
    (2, 8, 20, 20, 4, 64, (3, 7, 7), (1, 2, 2), (1, 3, 3)),
    (2, 6, 14, 14, 64, 64, (3, 3, 3), (1, 1, 1), (1, 1, 1)),
    (2, 6, 14, 14, 64, 128, (3, 3, 3), (2, 2, 2), (1, 1, 1)),
    (1, 5, 9, 7, 128, 256, (3, 3, 3), (2, 2, 2), (1, 1, 1)),
    (2, 6, 14, 14, 64, 128, (1, 1, 1), (2, 2, 2), (0, 0, 0)),
    (1, 3, 5, 5, 256, 64, (3, 3, 3), (1, 1, 1), (1, 1, 1)),
]


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv3d_fwd_dx_dw_match_torch(case):
    """vs_conv3d_fwd / _dx / _dw against torch's conv3d and its autograd (fp64 on the CPU) on the same
    f32 inputs; dX both overwriting and accumulating; the fused BatchNorm statistics partials."""
    from vspike import r3d, _lib as L
    N, D, H, W, Ci, Co, k, s, p = case
    g = torch.Generator().manual_seed(sum(case[:6]))
    x = torch.randn(N, Ci, D, H, W, generator=g)
    w = torch.randn(Co, Ci, *k, generator=g) / math.sqrt(Ci * k[0] * k[1] * k[2])
    xd = x.double().requires_grad_()
    wd = w.double().requires_grad_()
    ref = F.conv3d(xd, wd, None, s, p)
    gy = torch.randn(ref.shape, generator=g).double()
    rdx, rdw = torch.autograd.grad(ref, (xd, wd), gy)
    d = r3d._desc(_spec(Ci, Co, k, s, p), N, D, H, W)
    assert (d.Do, d.Ho, d.Wo) == tuple(ref.shape[2:])
    x_dev, w_dev = _cl(x).to(DEV), w.permute(0, 2, 3, 4, 1).contiguous().to(DEV)
    y = torch.empty(N, d.Do, d.Ho, d.Wo, Co, device=DEV)
    rows = r3d.conv3d_stats_rows(d)
    stats = torch.empty(rows, 2, Co, device=DEV)
    L.dispatch_reset()
    r3d.conv3d_fwd(d, x_dev, w_dev, y, stats)
    gy_dev = _cl(gy.float()).to(DEV)
    dw = torch.empty_like(w_dev)
    r3d.conv3d_dw(d, x_dev, gy_dev, dw)
    torch.cuda.synchronize()
    assert L.dispatch_counts()["conv_igemm"] >= 1 and L.dispatch_counts()["conv_dw"] == 1
    assert _maxrel(y, _cl(ref.detach())) < 1e-5
    yr = _cl(ref.detach()).reshape(-1, Co)
    s_ref, m2_ref = _tile_partials(yr)
    st = stats.double().cpu()
    # per 128-row tile: the column sum (rounding relative to the sum of |y|: the sums can cancel to ~0)
    # and the sum of squared deviations from the tile's own mean
    tabs = torch.stack([yr[i:i + 128].abs().sum(0) for i in range(0, yr.shape[0], 128)])
    assert float(((st[:, 0] - s_ref).abs() / tabs).max()) < 1e-5
    assert _maxrel(st[:, 1], m2_ref) < 1e-5
    assert _maxrel(dw, rdw.permute(0, 2, 3, 4, 1)) < 1e-5
    if Ci % 64 == 0:
        dx = torch.full((N, D, H, W, Ci), float("nan"), device=DEV)      # every element must be written
        r3d.conv3d_dx(d, gy_dev, w_dev, dx)
        base = torch.randn(N, D, H, W, Ci, generator=g).to(DEV)
        dx2 = base.clone()
        r3d.conv3d_dx(d, gy_dev, w_dev, dx2, accumulate=True)
        torch.cuda.synchronize()
        assert torch.isfinite(dx).all()
        assert _maxrel(dx, _cl(rdx)) < 1e-5
        assert _maxrel(dx2, _cl(rdx) + base.double().cpu()) < 1e-5
    # bitwise reproducible (fixed-order partial sums, no atomics)
    dw2 = torch.empty_like(w_dev)
    r3d.conv3d_dw(d, x_dev, gy_dev, dw2)
    y2 = torch.empty_like(y)
    r3d.conv3d_fwd(d, x_dev, w_dev, y2)
    torch.cuda.synchronize()
    assert torch.equal(dw, dw2) and torch.equal(y, y2)


@pytest.mark.parametrize("C,relu,res", [(64, True, False), (128, True, True), (512, False, False)])
def test_bn3d_train_forward_backward_match_torch(C, relu, res):
    """vs_bn3d_stats / _apply / _bwd (training-mode BatchNorm3d + residual + ReLU) vs torch autograd."""
    from vspike import r3d
    g = torch.Generator().manual_seed(C)
    N, D, H, W = 2, 4, 7, 9
    y = torch.randn(N, C, D, H, W, generator=g) * 1.7 + 0.3
    gamma = torch.randn(C, generator=g) * 0.1 + 1.0
    beta = torch.randn(C, generator=g) * 0.1
    resid = torch.randn(N, C, D, H, W, generator=g)
    rm, rv = torch.randn(C, generator=g) * 0.1, torch.rand(C, generator=g) + 0.5
    yd, gd, bd = y.double().requires_grad_(), gamma.double().requires_grad_(), beta.double().requires_grad_()
    rd = resid.double().requires_grad_()
    rmd, rvd = rm.double().clone(), rv.double().clone()
    o = F.batch_norm(yd, rmd, rvd, gd, bd, training=True, momentum=0.1, eps=1e-5)
    if res:
        o = o + rd
    if relu:
        o = F.relu(o)
    go = torch.randn(o.shape, generator=g).double()
    dy_r, dg_r, db_r, dres_r = torch.autograd.grad(o, (yd, gd, bd, rd), go, allow_unused=True)
    M = N * D * H * W
    y_cl = _cl(y).to(DEV)
    ts, tm2 = _tile_partials(y_cl.view(M, C).cpu())
    stats = torch.stack([ts, tm2], 1).float()
    mean, rstd, scale, shift = (torch.empty(C, device=DEV) for _ in range(4))
    rm_d, rv_d = rm.clone().to(DEV), rv.clone().to(DEV)
    g_d, b_d = gamma.to(DEV), beta.to(DEV)
    r3d.bn3d_stats(stats.to(DEV), stats.shape[0], M, g_d, b_d, 1e-5, 0.1, mean, rstd, scale, shift, rm_d, rv_d)
    out = torch.empty_like(y_cl)
    res_cl = _cl(resid).to(DEV) if res else None
    r3d.bn3d_apply(y_cl, scale, shift, out, residual=res_cl, relu=relu)
    dy = torch.empty_like(y_cl)
    dres = torch.empty_like(y_cl) if res else None
    dgam, dbet = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
    r3d.bn3d_bwd(_cl(go.float()).to(DEV), out, relu, y_cl, mean, rstd, g_d, dy, dres, dgam, dbet)
    torch.cuda.synchronize()
    assert _maxrel(out, _cl(o.detach())) < 1e-5
    assert _maxrel(rm_d, rmd) < 1e-5 and _maxrel(rv_d, rvd) < 1e-5
    assert _maxrel(dy, _cl(dy_r)) < 1e-5
    assert _maxrel(dgam, dg_r) < 1e-5 and _maxrel(dbet, db_r) < 1e-5
    if res:
        assert _maxrel(dres, _cl(dres_r)) < 1e-6


def test_bn3d_stats_large_channel_offset():
    """Batch statistics when |mean| >> std (mean ~1e3, std ~1: trained weights can reach this), through
    the conv epilogue's partials and vs_bn3d_stats, vs f64: a one-pass sum of y^2 in f32 loses the
    variance to cancellation (E[y^2] - mean^2 with E[y^2] ~ 1e6); the tile-mean-centred partials merged
    with Chan's formula keep it."""
    from vspike import r3d
    C, N, D, H, W = 64, 2, 4, 10, 13
    g = torch.Generator().manual_seed(11)
    x = torch.randn(N, C, D, H, W, generator=g) + 1000.0 + torch.arange(C).view(1, C, 1, 1, 1) * 3.0
    w = torch.eye(C).view(C, C, 1, 1, 1)                       # 1x1x1 identity conv: y = x
    d = r3d._desc(_spec(C, C, (1, 1, 1), (1, 1, 1), (0, 0, 0)), N, D, H, W)
    y = torch.empty(N, D, H, W, C, device=DEV)
    rows = r3d.conv3d_stats_rows(d)
    stats = torch.empty(rows, 2, C, device=DEV)
    r3d.conv3d_fwd(d, _cl(x).to(DEV), w.permute(0, 2, 3, 4, 1).contiguous().to(DEV), y, stats)
    mean, rstd, scale, shift = (torch.empty(C, device=DEV) for _ in range(4))
    M = N * D * H * W
    r3d.bn3d_stats(stats, rows, M, torch.ones(C, device=DEV), torch.zeros(C, device=DEV), 1e-5, 0.1, mean, rstd,
                   scale, shift)
    torch.cuda.synchronize()
    yd = _cl(x).reshape(M, C).double()
    var = yd.var(0, unbiased=False)
    assert _maxrel(mean, yd.mean(0)) < 1e-6
    got_var = 1.0 / rstd.double().cpu() ** 2 - 1e-5
    err = float(((got_var - var).abs() / var).max())
    print(f"\n[bn stats, mean ~1e3, std ~1] variance rel err {err:.2e}")
    assert err < 1e-4


@pytest.mark.parametrize("relu,res", [(True, True), (False, False)])
def test_bn3d_eval_backward_matches_torch(relu, res):
    """vs_bn3d_bwd_eval: the backward of an eval-mode (running-statistics) BatchNorm3d + residual + ReLU
    vs torch autograd through F.batch_norm(training=False): dy = gamma rstd g."""
    from vspike import r3d
    C = 128
    g = torch.Generator().manual_seed(3)
    N, D, H, W = 2, 3, 5, 6
    y = torch.randn(N, C, D, H, W, generator=g) * 1.3 + 0.2
    gamma = torch.randn(C, generator=g) * 0.1 + 1.0
    beta = torch.randn(C, generator=g) * 0.1
    resid = torch.randn(N, C, D, H, W, generator=g)
    rm, rv = torch.randn(C, generator=g) * 0.3, torch.rand(C, generator=g) + 0.5
    yd, gd, bd = y.double().requires_grad_(), gamma.double().requires_grad_(), beta.double().requires_grad_()
    o = F.batch_norm(yd, rm.double(), rv.double(), gd, bd, training=False, eps=1e-5)
    if res:
        o = o + resid.double()
    if relu:
        o = F.relu(o)
    go = torch.randn(o.shape, generator=g).double()
    dy_r, dg_r, db_r = torch.autograd.grad(o, (yd, gd, bd), go)
    y_cl = _cl(y).to(DEV)
    rstd = torch.rsqrt(rv + 1e-5).to(DEV)
    mean = rm.to(DEV)
    g_d = gamma.to(DEV)
    scale, shift = g_d * rstd, beta.to(DEV) - mean * g_d * rstd
    out = torch.empty_like(y_cl)
    r3d.bn3d_apply(y_cl, scale, shift, out, residual=_cl(resid).to(DEV) if res else None, relu=relu)
    dy = torch.empty_like(y_cl)
    dgam, dbet = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
    r3d.bn3d_bwd(_cl(go.float()).to(DEV), out, relu, y_cl, mean, rstd, g_d, dy, None, dgam, dbet,
                 batch_stats=False)
    torch.cuda.synchronize()
    assert _maxrel(out, _cl(o.detach())) < 1e-5
    assert _maxrel(dy, _cl(dy_r)) < 1e-5
    assert _maxrel(dgam, dg_r) < 1e-5 and _maxrel(dbet, db_r) < 1e-5


def _r3d_model(cfg, n, enc_out=64):
    from vspike import R3D
    conf = {"model_class": "R3D", "compute_dtype": "fp32", "freeze_encoder": False,
            "backbone": {"num_frames": cfg.num_frames, "image_size": cfg.image_size, "num_channels": cfg.num_channels},
            "encoder": {"output_dim": enc_out}, "decoder": {"output_dim": 100 * n}}
    m = R3D(conf).to(DEV)
    m.load_reference_state_dict({k: torch.from_numpy(v) for k, v in cpu_ref.make_r3d_params(cfg, enc_out, n).items()},
                                strict=False)
    return m


@pytest.mark.parametrize("geo", [(8, 56, 2), (32, 112, 2)])
def test_r3d_plugin_forward_backward_matches_oracle(geo):
    """The whole R3D plugin (C4: 32 x 112 x 112 at B = 2, and a small geometry) vs the oracle:
    log-rates, loss, every gradient, the BatchNorm running statistics."""
    from vspike import poisson_nll_mean, _lib as L
    T, S, B = geo
    cfg, n = cpu_ref.R3DCfg(num_frames=T, image_size=S), 256
    params = cpu_ref.make_r3d_params(cfg, 64, n)
    # the oracle in f64: the BatchNorm bias gradients are sums of ~10^4 terms that cancel to ~1e-3 of
    # their absolute sum, so an f32 CPU reference carries as much rounding as the kernel under test
    P = {k: torch.from_numpy(v).double().requires_grad_() for k, v in params.items()}
    running = {}
    for name, ci, co, *_ in cpu_ref.r3d_conv_specs(cfg):
        bn = name[:-2] + ".1"
        running[bn + ".running_mean"] = torch.zeros(co, dtype=torch.float64)
        running[bn + ".running_var"] = torch.ones(co, dtype=torch.float64)
    px = torch.from_numpy(cpu_ref.make_r3d_pixels(cfg, B, seed=5))
    y = torch.from_numpy(prng.spike_targets(5, (B, 100, n)))
    m = _r3d_model(cfg, n)
    m.keep_relu_masks = True
    L.dispatch_reset()
    out = m(px.to(DEV))
    # the oracle conditioned on the plugin's ReLU decisions (r3d18_forward relu_masks): a pre-activation
    # within rounding of zero lands on either side in two correct computations, and one flipped element
    # moves a cancelling gradient sum by a whole element (r06: 1-2e-3 on layer4 at this geometry from
    # ties alone); the flips themselves are checked to be rounding-level ties below
    masks = {k: v.cpu() for k, v in m.relu_masks.items()}
    m.keep_relu_masks = False
    flips = {}
    ref = cpu_ref.r3d18_forward(px.double(), P, cfg, running=running, relu_masks=masks, mask_log=flips)
    rloss = cpu_ref.poisson_nll_mean(ref, y.double())
    rloss.backward()
    # the same oracle in f32 (torch's own CPU kernels, same decisions): f32 arithmetic's own distance
    P32 = cpu_ref.to_torch(params)
    cpu_ref.poisson_nll_mean(cpu_ref.r3d18_forward(px, P32, cfg, relu_masks=masks), y).backward()
    e32 = {k: float((P32[k].grad.double() - P[k].grad).norm() / P[k].grad.norm()) for k in P}
    nflip = sum(f[0] for f in flips.values())
    tie = max((f[1] / f[2] for f in flips.values() if f[0]), default=0.0)
    print(f"\n[r3d {geo}] ReLU decisions differing from f64: {nflip} of {sum(v.numel() for v in masks.values())}, "
          f"largest |pre-activation| among them {tie:.2e} of its unit's max")
    assert tie < 1e-5
    loss = poisson_nll_mean(out, y.to(DEV))
    loss.backward()
    torch.cuda.synchronize()
    counts = L.dispatch_counts()
    assert counts["conv_igemm"] > 0 and counts["conv_dw"] == len(m.layout.convs), counts
    out_err = _maxrel(out.detach(), ref.detach())
    loss_err = abs(loss.item() - rloss.item()) / abs(rloss.item())
    lay = m.layout
    errs = {}
    for c in lay.convs:
        gw = lay.enc.view(m.enc_flat.grad, c.name + ".weight")[..., :c.ci_ref].permute(0, 4, 1, 2, 3)
        errs[c.name + ".weight"] = float((gw.double().cpu() - P[c.name + ".weight"].grad.double()).norm() /
                                         P[c.name + ".weight"].grad.double().norm())
        bn = c.name[:-2] + ".1"
        for suf in (".weight", ".bias"):
            gb = lay.enc.view(m.enc_flat.grad, bn + suf)
            errs[bn + suf] = float((gb.double().cpu() - P[bn + suf].grad.double()).norm() /
                                   P[bn + suf].grad.double().norm())
    for ref_name, slot in (("encoder.weight", "enc_w"), ("encoder.bias", "enc_b"), ("decoder.weight", "dec_w"),
                           ("decoder.bias", "dec_b")):
        gh = lay.head.view(m.head_flat.grad, slot)
        errs[ref_name] = float((gh.double().cpu() - P[ref_name].grad.double()).norm() / P[ref_name].grad.double().norm())
    # bar per gradient (ReLU decisions shared with the oracle): 1e-3 of its norm, or 3x torch-f32's own
    # distance from f64 where that is larger (BatchNorm-affine gradients are sums of ~10^4-10^5 terms that
    # cancel to ~1e-3 of their absolute sums)
    bars = {k: max(1e-3, 3.0 * e32[k]) for k in errs}
    worst = max(errs, key=lambda k: errs[k] / bars[k])
    sd = m.reference_state_dict()
    run_err = max(_maxrel(sd[k], v) for k, v in running.items())
    print(f"\n[r3d {geo}] log-rates {out_err:.3e} loss {loss_err:.3e} worst grad {worst} {errs[worst]:.3e} "
          f"(torch f32 {e32[worst]:.3e}, bar {bars[worst]:.3e}) running {run_err:.3e}; "
          f"{sum(e32[k] > 1e-3 / 3 for k in errs)} of {len(errs)} gradients above 3.3e-4 in torch f32")
    assert out_err < 1e-4 and loss_err < 1e-5
    bad = {k: (errs[k], bars[k]) for k in errs if errs[k] > bars[k]}
    assert not bad, bad
    assert run_err < 1e-5


def test_r3d_plugin_loss_curve_and_eval_match_oracle():
    """3 steps of the reference loop (AdamW + OneCycleLR, src/train.py:44-57, base.py:144-159) on the
    R3D plugin vs the oracle's curve, then an eval-mode forward (running statistics) vs the oracle."""
    from vspike import FusedAdamW, poisson_nll_mean
    cfg, B, n = cpu_ref.R3DCfg(num_frames=8, image_size=56), 2, 32
    params = cpu_ref.make_r3d_params(cfg, 64, n)
    P = cpu_ref.to_torch(params)
    running = {}
    for name, ci, co, *_ in cpu_ref.r3d_conv_specs(cfg):
        bn = name[:-2] + ".1"
        running[bn + ".running_mean"] = torch.zeros(co)
        running[bn + ".running_var"] = torch.ones(co)
    batches = [(torch.from_numpy(cpu_ref.make_r3d_pixels(cfg, B, seed=40 + s)),
                torch.from_numpy(prng.spike_targets(50 + s, (B, 100, n)))) for s in range(3)]
    curve = cpu_ref.train_curve(lambda x, PP: cpu_ref.r3d18_forward(x, PP, cfg, running=running), P, batches,
                                lr=1e-4)
    m = _r3d_model(cfg, n)
    opt = FusedAdamW([p for p in m.parameters() if p.requires_grad], lr=1e-4, weight_decay=0.01, eps=1e-8)
    sched = torch.optim.lr_scheduler.OneCycleLR(opt, total_steps=3, max_lr=1e-4, pct_start=0.15, div_factor=10)
    losses = []
    for x, yy in batches:
        loss = poisson_nll_mean(m(x.to(DEV)), yy.to(DEV))
        loss.backward()
        opt.step()
        sched.step()
        opt.zero_grad()
        losses.append(loss.item())
    rel = np.abs(np.array(losses) - np.array(curve)) / np.abs(np.array(curve))
    print(f"\n[r3d curve] {losses} ref {curve} max rel {rel.max():.3e}")
    assert rel.max() < 1e-4
    # eval mode (nn.BatchNorm3d.eval(): the running statistics), on freshly loaded weights with given
    # running buffers (after training, Adam turns the sign noise of near-zero gradients into lr-sized
    # weight differences, which the eval outputs would compare instead of the eval path)
    g = torch.Generator().manual_seed(9)
    sd = {k: torch.from_numpy(v) for k, v in params.items()}
    for k in running:
        running[k] = (torch.rand(running[k].shape, generator=g) + 0.5 if k.endswith("var")
                      else torch.randn(running[k].shape, generator=g) * 0.1)
        sd[k] = running[k]
    m2 = _r3d_model(cfg, n)
    m2.load_reference_state_dict(sd, strict=True)
    m2.eval()
    with torch.no_grad():
        xe = batches[0][0]
        ev = m2(xe.to(DEV))
        ref = cpu_ref.r3d18_forward(xe, cpu_ref.to_torch(params, requires_grad=False), cfg, running=running,
                                    training=False)
    print(f"[r3d eval] {_maxrel(ev, ref):.3e}")
    assert _maxrel(ev, ref) < 1e-4
    # backward through the eval-mode forward (frozen-BN fine-tuning): the running
    # statistics are constants, so BN' is gamma rstd g with no batch-statistics terms; vs the f64 oracle
    yy = batches[0][1]
    m2.keep_relu_masks = True
    loss = poisson_nll_mean(m2(xe.to(DEV)), yy.to(DEV))
    loss.backward()
    torch.cuda.synchronize()
    masks = {k: v.cpu() for k, v in m2.relu_masks.items()}
    Pd = {k: torch.from_numpy(v).double().requires_grad_() for k, v in params.items()}
    rund = {k: v.double() for k, v in running.items()}
    flips = {}
    rl = cpu_ref.poisson_nll_mean(cpu_ref.r3d18_forward(xe.double(), Pd, cfg, running=rund, training=False,
                                                        relu_masks=masks, mask_log=flips), yy.double())
    rl.backward()
    assert max((f[1] / f[2] for f in flips.values() if f[0]), default=0.0) < 1e-5
    lay = m2.layout
    worst = 0.0
    for c in lay.convs:
        gw = lay.enc.view(m2.enc_flat.grad, c.name + ".weight")[..., :c.ci_ref].permute(0, 4, 1, 2, 3)
        rg = Pd[c.name + ".weight"].grad
        worst = max(worst, float((gw.double().cpu() - rg).norm() / rg.norm()))
        bn = c.name[:-2] + ".1"
        for suf in (".weight", ".bias"):
            gb, rb = lay.enc.view(m2.enc_flat.grad, bn + suf), Pd[bn + suf].grad
            worst = max(worst, float((gb.double().cpu() - rb).norm() / rb.norm()))
    print(f"[r3d eval backward] loss {abs(loss.item() - rl.item()) / abs(rl.item()):.3e} worst grad {worst:.3e}")
    assert abs(loss.item() - rl.item()) / abs(rl.item()) < 1e-5
    assert worst < 1e-3


def test_r3d_raw_video_input_and_registry():
    """NAME2MODEL['R3D'] from the r3d18 YAML; the raw gray video the reference loader yields
    (B, 120, 1, 128, 128) runs through the on-device preprocessing to 32 x 112 x 112 clips."""
    import os
    from vspike import NAME2MODEL, load_run_config
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cfgd = os.path.join(root, "video-spike_amd", "config")
    conf = load_run_config(os.path.join(cfgd, "model", "r3d18.yaml"), os.path.join(cfgd, "train", "vmae_video.yaml"))
    conf["model"]["decoder"]["output_dim"] = 100 * 8
    m = NAME2MODEL[conf["model"]["model_class"]](conf["model"]).to(DEV)
    video = torch.from_numpy(prng.video_frames(3, (1, 120, 1, 128, 128))).to(DEV)
    out = m(video)
    assert out.shape == (1, 100, 8) and torch.isfinite(out).all()
    pv = m.preprocess(video)
    assert pv.shape == (1, 32, 3, 112, 112)
