"""hipGraph replay of the train step (vspike.graph.GraphedStep) against the eager Trainer.step.

The replay re-issues the captured launches — same kernels, operands and stream order, with the
weight-gradient side stream forked/joined by captured event edges — so, with every reduction of
the bf16 step in a fixed order at hidden 192 (test_bf16_backward_bitwise_reproducible), the loss
curve and the final weights of K replayed steps must be BIT-identical to K eager steps from the
same state, including the scheduler's lr and the bias-correction step counts it stages per replay.
"""
import numpy as np
import pytest
import torch

from oracle import cpu_ref, prng

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _setup(cfg, B, n, dtype, freeze, seed=7):
    from vspike import FusedAdamW, VideoMAE
    from vspike.trainer import Trainer
    conf = {"model_class": "VideoMAE", "freeze_encoder": freeze, "compute_dtype": dtype,
            "backbone": {k: getattr(cfg, k) for k in ("image_size", "patch_size", "num_channels", "num_frames",
                                                       "tubelet_size", "hidden_size", "num_hidden_layers",
                                                       "num_attention_heads", "intermediate_size",
                                                       "layer_norm_eps")},
            "encoder": {"output_dim": 64}, "decoder": {"output_dim": 100 * n}}
    m = VideoMAE(conf).to(DEV)
    m.load_reference_state_dict({k: torch.from_numpy(v) for k, v in cpu_ref.make_vit_params(cfg, 64, n).items()})
    opt = FusedAdamW([p for p in m.parameters() if p.requires_grad], lr=1e-4, weight_decay=0.01, eps=1e-8)
    sched = torch.optim.lr_scheduler.OneCycleLR(opt, total_steps=12, max_lr=1e-4, pct_start=0.3, div_factor=10)
    tr = Trainer(m, opt, sched, config={"training": {"loss": "poisson"}})
    px = torch.from_numpy(cpu_ref.make_pixels(cfg, B, seed=seed)).to(DEV)
    y = torch.from_numpy(prng.spike_targets(seed + 1, (B, 100, n))).to(DEV)
    return m, tr, px, y


@pytest.mark.parametrize("dtype,freeze", [("bf16", False), ("fp32", False), ("bf16", True)])
def test_graphed_step_bitwise_equals_eager(dtype, freeze):
    from vspike.graph import GraphedStep
    cfg = cpu_ref.ViTCfg(image_size=112, num_frames=8, hidden_size=192, num_hidden_layers=2,
                         num_attention_heads=3, intermediate_size=768)
    B, n, K = 2, 16, 5
    runs = {}
    for mode in ("eager", "graph"):
        m, tr, px, y = _setup(cfg, B, n, dtype, freeze)
        losses = [float(tr.step(px, y))]            # one eager step in both runs (graph: before capture)
        if mode == "graph":
            gs = GraphedStep(tr, px, y)
            losses += [gs.step() for _ in range(K)]
        else:
            losses += [tr.step(px, y) for _ in range(K)]
        torch.cuda.synchronize()
        runs[mode] = ([float(x) for x in losses], m.enc_flat.detach().cpu().clone(), m.head_flat.detach().cpu().clone(),
                      tr.optimizer.param_groups[0]["lr"])
    (le, ee, he, lre), (lg, eg, hg, lrg) = runs["eager"], runs["graph"]
    assert le == lg, (le, lg)
    assert lre == lrg
    assert torch.equal(he, hg)
    assert torch.equal(ee, eg)
    assert len(set(le)) > 1          # the weights moved between steps


def test_graphed_step_copies_new_inputs_and_rejects_exchange():
    """A different input tensor is copied into the captured one (a data loader's batches), and a
    Trainer with a data-parallel exchange is refused (the collective is not captured)."""
    from vspike.graph import GraphedStep
    cfg = cpu_ref.ViTCfg(image_size=112, num_frames=8, hidden_size=192, num_hidden_layers=1,
                         num_attention_heads=3, intermediate_size=768)
    B, n = 2, 16
    m, tr, px, y = _setup(cfg, B, n, "bf16", False)
    m2, tr2, _, _ = _setup(cfg, B, n, "bf16", False)
    tr.step(px, y)
    tr2.step(px, y)
    gs = GraphedStep(tr, px.clone(), y.clone())
    px2 = torch.from_numpy(cpu_ref.make_pixels(cfg, B, seed=99)).to(DEV)
    y2 = torch.from_numpy(prng.spike_targets(98, (B, 100, n))).to(DEV)
    a = [float(gs.step(px2, y2)), float(gs.step(px, y))]
    b = [float(tr2.step(px2, y2)), float(tr2.step(px, y))]
    assert a == b
    tr.exchange = object()
    with pytest.raises(ValueError):
        GraphedStep(tr, px, y)
    np.testing.assert_array_equal(m.enc_flat.detach().cpu().numpy(), m2.enc_flat.detach().cpu().numpy())
