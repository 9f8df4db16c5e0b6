"""Generate the golden fixtures under tests/golden/ FROM THE REFERENCE ITSELF.

TEST INFRASTRUCTURE ONLY.  Run once, in the build container where `/root/reference` exists:

    python -m oracle.gen_fixtures

What runs the reference here (nothing is copied out of it, only outputs are saved):
  * `Linear` plugin: imported from `/root/reference/src/model/linear.py` and built from a
    model YAML with the reference's own loader `src/utils/config_utils.py:59-75`.
  * `VideoMAE` plugin: `src/model/videomae.py:4-32` cannot be constructed offline
    (`from_pretrained("MCG-NJU/videomae-base")` at :7-8 needs the Hub, and :24 hard-codes
    `.cuda()`), so its forward from `pixel_values` on is composed from the third-party encoder the
    reference executes — the installed HF `transformers.VideoMAEModel` (5.15.0; reference pins
    4.38.2, env.yaml:30) with eager attention and k-bias zeroed (4.38 uses a fixed zero k-bias,
    modeling_videomae.py:233) — plus two `nn.Linear` layers exactly as `videomae.py:13-14,28-31`.
  * Train loop: the body of `src/trainer/base.py:144-159` with the optimiser/scheduler of
    `src/train.py:44-57` driving those modules.
  * Config loader: the reference's `update_config`/`config_from_kwargs` over this repo's YAMLs.

Inputs and weights come from `oracle.prng` (seeded by name), so only outputs are committed.
"""
from __future__ import annotations

import json
import math
import os
import sys

import numpy as np
import torch

sys.dont_write_bytecode = True          # never write into /root/reference

from oracle import cpu_ref, prng  # noqa: E402

REF_SRC = "/root/reference/src"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "tests", "golden")
CFG = os.path.join(ROOT, "video-spike_amd", "config")


def _ref_imports():
    if REF_SRC not in sys.path:
        sys.path.insert(0, REF_SRC)
    from model.linear import Linear                      # noqa: E402
    from utils.config_utils import update_config, config_from_kwargs   # noqa: E402
    return Linear, update_config, config_from_kwargs


def _grads_summary(named_grads):
    out = {}
    for name, g in named_grads.items():
        out.update(cpu_ref.summarize(name, g.detach().numpy()))
    return out


def _ref_train_loop(module, batches, trainable, lr, wd=0.01, eps=1e-8, warmup_pct=0.15, div_factor=10):
    """Body of src/trainer/base.py:144-159 with src/train.py:44-59's optimiser/scheduler/criterion."""
    for p in module.parameters():                         # start from a clean slate (no stale .grad)
        p.grad = None
    optimizer = torch.optim.AdamW(trainable, lr=lr, weight_decay=wd, eps=eps)
    sched = torch.optim.lr_scheduler.OneCycleLR(optimizer=optimizer, total_steps=len(batches), max_lr=lr,
                                                pct_start=warmup_pct, div_factor=div_factor)
    criterion = torch.nn.PoissonNLLLoss(reduction="none", log_input=True)
    losses = []
    module.train()
    for x, y in batches:
        outputs = module(x)
        loss = criterion(outputs, y).mean()
        loss.backward()
        optimizer.step()
        sched.step()
        optimizer.zero_grad()
        losses.append(loss.item())
    return np.array(losses, dtype=np.float64)


# ----------------------------------------------------------------------------------------------
def gen_linear():
    Linear, update_config, config_from_kwargs = _ref_imports()
    B, T, HW, n = 4, 8, 64, 16
    config = config_from_kwargs({"model": "include:" + os.path.join(CFG, "model", "linear_video.yaml")})
    config = update_config(os.path.join(CFG, "train", "linear_video.yaml"), config)
    config["model"]["encoder"]["input_dim"] = T * HW * HW
    config["model"]["decoder"]["output_dim"] = 100 * n
    module = Linear(config.model)
    shapes = {k: tuple(v.shape) for k, v in module.state_dict().items()}
    params = cpu_ref.make_linear_params(shapes)
    module.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()})

    video = np.floor(prng.uniform(0, B * T * HW * HW, "video") * 256.0).astype(np.float32).reshape(B, T, 1, HW, HW)
    ap = prng.spike_targets(1, (B, 100, n))
    x, y = torch.from_numpy(video), torch.from_numpy(ap)
    inp = x.flatten(1)                                   # base.py:64-67 (Linear: cat of flattened modalities)
    out = module(inp)
    loss = torch.nn.PoissonNLLLoss(reduction="none", log_input=True)(out, y).mean()
    loss.backward()
    fx = {"log_rates": out.detach().numpy(), "loss": np.array([loss.item()])}
    fx.update(_grads_summary({k: p.grad for k, p in module.named_parameters()}))

    # 5-step loss curve (fresh weights); lr small because the raw 0..255 inputs make the first layer stiff
    module.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()})
    batches = []
    for s in range(5):
        v = np.floor(prng.uniform(100 + s, B * T * HW * HW, "video") * 256.0).astype(np.float32)
        batches.append((torch.from_numpy(v.reshape(B, T, 1, HW, HW)).flatten(1),
                        torch.from_numpy(prng.spike_targets(200 + s, (B, 100, n)))))
    fx["curve"] = _ref_train_loop(module, batches, list(module.parameters()), lr=1e-6)
    np.savez(os.path.join(OUT, "linear_f.npz"), **fx)
    print("linear_f", fx["loss"], fx["curve"])


def _hf_encoder(cfg: cpu_ref.ViTCfg):
    from transformers import VideoMAEConfig, VideoMAEModel
    hc = VideoMAEConfig(image_size=cfg.image_size, patch_size=cfg.patch_size, num_channels=cfg.num_channels,
                        num_frames=cfg.num_frames, tubelet_size=cfg.tubelet_size, hidden_size=cfg.hidden_size,
                        num_hidden_layers=cfg.num_hidden_layers, num_attention_heads=cfg.num_attention_heads,
                        intermediate_size=cfg.intermediate_size, hidden_act="gelu", hidden_dropout_prob=0.0,
                        attention_probs_dropout_prob=0.0, layer_norm_eps=cfg.layer_norm_eps, qkv_bias=True,
                        use_mean_pooling=True)
    hc._attn_implementation = "eager"
    return VideoMAEModel(hc)


class _RefVideoMAEHead(torch.nn.Module):
    """`src/model/videomae.py:13-14,26-31` from pixel_values on (encoder = HF VideoMAEModel)."""

    def __init__(self, cfg, enc_out, n_out):
        super().__init__()
        self.video_mae = _hf_encoder(cfg)
        self.encoder = torch.nn.Linear(cfg.num_tokens * cfg.hidden_size, enc_out)
        self.decoder = torch.nn.Linear(enc_out, 100 * n_out)
        self.freeze = True

    def forward(self, pixel_values):
        B = pixel_values.shape[0]
        if self.freeze:
            with torch.no_grad():
                outputs = self.video_mae(pixel_values=pixel_values).last_hidden_state.flatten(1)
        else:
            outputs = self.video_mae(pixel_values=pixel_values).last_hidden_state.flatten(1)
        outputs = self.encoder(outputs)
        outputs = self.decoder(outputs)
        return outputs.reshape(B, 100, -1)


def _load_vit(module, cfg, enc_out, n_out):
    params = cpu_ref.make_vit_params(cfg, enc_out, n_out)
    sd = {k: torch.from_numpy(v) for k, v in params.items()}
    for i in range(cfg.num_hidden_layers):                # installed HF has a learnable k bias: pin to 0
        sd[f"video_mae.encoder.layer.{i}.attention.attention.key.bias"] = torch.zeros(cfg.hidden_size)
    missing, unexpected = module.load_state_dict(sd, strict=False)
    assert not unexpected and not missing, (missing, unexpected)
    return params


def gen_vit_small():
    cfg, B, enc_out, n = cpu_ref.VIT_SMALL_FIXTURE, 2, 64, 16
    torch.manual_seed(0)
    m = _RefVideoMAEHead(cfg, enc_out, n)
    _load_vit(m, cfg, enc_out, n)
    px = torch.from_numpy(cpu_ref.make_pixels(cfg, B))
    y = torch.from_numpy(prng.spike_targets(1, (B, 100, n)))
    m.freeze = False                                      # north-star: encoder fwd+bwd
    hid = m.video_mae(pixel_values=px).last_hidden_state
    out = m(px)
    loss = torch.nn.PoissonNLLLoss(reduction="none", log_input=True)(out, y).mean()
    loss.backward()
    fx = {"last_hidden": hid.detach().numpy(), "log_rates": out.detach().numpy(), "loss": np.array([loss.item()])}
    grads = {k: p.grad for k, p in m.named_parameters() if ".key.bias" not in k}
    fx.update(_grads_summary(grads))

    def batches(base):
        return [(torch.from_numpy(cpu_ref.make_pixels(cfg, B, seed=base + s)),
                 torch.from_numpy(prng.spike_targets(base + 50 + s, (B, 100, n)))) for s in range(4)]
    # frozen (reference default): AdamW over model.parameters(); frozen ones have grad None
    _load_vit(m, cfg, enc_out, n)
    m.freeze = True
    for p in m.video_mae.parameters():
        p.requires_grad = False
    fx["curve_frozen"] = _ref_train_loop(m, batches(300), list(m.parameters()), lr=1e-5)
    # trainable encoder (north-star flag); k bias excluded (4.38 has none)
    _load_vit(m, cfg, enc_out, n)
    m.freeze = False
    for k, p in m.named_parameters():
        p.requires_grad = ".key.bias" not in k
    fx["curve_train"] = _ref_train_loop(m, batches(300), [p for p in m.parameters() if p.requires_grad], lr=1e-5)
    np.savez(os.path.join(OUT, "vit_small.npz"), **fx)
    print("vit_small", fx["loss"], fx["curve_frozen"], fx["curve_train"])


def gen_vit_tiny1l():
    cfg = cpu_ref.ViTCfg(hidden_size=192, num_attention_heads=3, intermediate_size=768, num_hidden_layers=1)
    B, enc_out, n = 1, 64, 8
    m = _RefVideoMAEHead(cfg, enc_out, n)
    _load_vit(m, cfg, enc_out, n)
    px = torch.from_numpy(cpu_ref.make_pixels(cfg, B))
    y = torch.from_numpy(prng.spike_targets(1, (B, 100, n)))
    with torch.no_grad():
        hid = m.video_mae(pixel_values=px).last_hidden_state
        out = m(px)
        loss = torch.nn.PoissonNLLLoss(reduction="none", log_input=True)(out, y).mean()
    fx = {"log_rates": out.numpy(), "loss": np.array([loss.item()])}
    fx.update(cpu_ref.summarize("last_hidden", hid.numpy()))
    np.savez(os.path.join(OUT, "vit_tiny1l.npz"), **fx)
    print("vit_tiny1l", fx["loss"])


def _grads_summary_small(named_grads, full_limit=4096):
    out = {}
    for name, g in named_grads.items():
        out.update(cpu_ref.summarize(name, g.detach().numpy(), full_limit=full_limit))
    return out


def gen_vit_tiny12():
    """The bench geometry (BASELINE C2: ViT-Tiny/16, 12 layers, 16x224x224 -> 1568 tokens, n=128),
    trainable encoder, B=2: forward, every gradient (summarised), and a 4-step train curve with
    the reference's optimiser (AdamW wd 0.01 + OneCycleLR) at lr 1e-6: the YAML's 5e-5 moves the
    301,056-wide head input by ~12 logits per step with these seeded weights and the curve diverges."""
    cfg = cpu_ref.VIT_TINY
    B, enc_out, n = 2, 64, 128
    torch.manual_seed(0)
    m = _RefVideoMAEHead(cfg, enc_out, n)
    _load_vit(m, cfg, enc_out, n)
    m.freeze = False
    px = torch.from_numpy(cpu_ref.make_pixels(cfg, B))
    y = torch.from_numpy(prng.spike_targets(1, (B, 100, n)))
    hid = m.video_mae(pixel_values=px).last_hidden_state
    out = m(px)
    loss = torch.nn.PoissonNLLLoss(reduction="none", log_input=True)(out, y).mean()
    loss.backward()
    fx = {"log_rates": out.detach().numpy(), "loss": np.array([loss.item()])}
    fx.update(cpu_ref.summarize("last_hidden", hid.detach().numpy(), full_limit=0))
    fx.update(_grads_summary_small({k: p.grad for k, p in m.named_parameters() if ".key.bias" not in k}))
    _load_vit(m, cfg, enc_out, n)
    for k, p in m.named_parameters():
        p.requires_grad = ".key.bias" not in k
    batches = [(torch.from_numpy(cpu_ref.make_pixels(cfg, B, seed=400 + s)),
                torch.from_numpy(prng.spike_targets(450 + s, (B, 100, n)))) for s in range(4)]
    fx["curve_train"] = _ref_train_loop(m, batches, [p for p in m.parameters() if p.requires_grad], lr=1e-6)
    np.savez_compressed(os.path.join(OUT, "vit_tiny12.npz"), **fx)
    print("vit_tiny12", fx["loss"], fx["curve_train"])


def gen_vit_tiny12_b16():
    """The bench's EXACT dispatch (BASELINE C2 at the bench batch: ViT-Tiny/16, 12 layers, B=16 ->
    M = 25,088 token rows, n=128, trainable encoder): forward, every gradient (summarised) and a
    3-step train curve (AdamW wd 0.01 + OneCycleLR, lr 1e-6 as gen_vit_tiny12).  At M >= 8192 the
    HIP path runs its row-slab, W-resident, fused GEMM+LayerNorm and dW-tile kernels, which the
    B=2 fixture (M = 3,136) never reaches."""
    cfg = cpu_ref.VIT_TINY
    B, enc_out, n = 16, 64, 128
    torch.manual_seed(0)
    m = _RefVideoMAEHead(cfg, enc_out, n)
    _load_vit(m, cfg, enc_out, n)
    m.freeze = False
    px = torch.from_numpy(cpu_ref.make_pixels(cfg, B, seed=16))
    y = torch.from_numpy(prng.spike_targets(16, (B, 100, n)))
    out = m(px)
    loss = torch.nn.PoissonNLLLoss(reduction="none", log_input=True)(out, y).mean()
    loss.backward()
    fx = {"log_rates": out.detach().numpy(), "loss": np.array([loss.item()])}
    fx.update(_grads_summary_small({k: p.grad for k, p in m.named_parameters() if ".key.bias" not in k}))
    del out, loss
    _load_vit(m, cfg, enc_out, n)
    for k, p in m.named_parameters():
        p.grad = None
        p.requires_grad = ".key.bias" not in k
    batches = [(torch.from_numpy(cpu_ref.make_pixels(cfg, B, seed=600 + s)),
                torch.from_numpy(prng.spike_targets(650 + s, (B, 100, n)))) for s in range(3)]
    fx["curve_train"] = _ref_train_loop(m, batches, [p for p in m.parameters() if p.requires_grad], lr=1e-6)
    np.savez_compressed(os.path.join(OUT, "vit_tiny12_b16.npz"), **fx)
    print("vit_tiny12_b16", fx["loss"], fx["curve_train"])


def gen_vit_tiny12_b16_enc(lr=None):
    """Encoder-sensitive curve at the bench batch: the fresh-batch lr 1e-6 curves
    move the loss by < 0.1 %, and the trainable- and frozen-encoder curves differ by <= 4e-4, so a
    wrong encoder update could pass them.  Here the HEAD is frozen (requires_grad False, so AdamW
    skips it, as the reference's optimiser skips any parameter without a gradient) and only the
    encoder trains, on ONE batch repeated for 4 steps at a large lr: every change of the loss comes
    from the encoder's backward + AdamW update.  B = 16 (M = 25,088 token rows: the benched kernels)."""
    cfg = cpu_ref.VIT_TINY
    B, enc_out, n = 16, 64, 128
    lr = lr if lr is not None else 1e-4
    torch.manual_seed(0)
    m = _RefVideoMAEHead(cfg, enc_out, n)
    _load_vit(m, cfg, enc_out, n)
    m.freeze = False
    for k, p in m.named_parameters():
        p.grad = None
        p.requires_grad = k.startswith("video_mae.") and ".key.bias" not in k
    px = torch.from_numpy(cpu_ref.make_pixels(cfg, B, seed=700))
    y = torch.from_numpy(prng.spike_targets(750, (B, 100, n)))
    batches = [(px, y)] * 4
    curve = _ref_train_loop(m, batches, [p for p in m.parameters() if p.requires_grad], lr=lr)
    fx = {"curve_enc": curve, "lr": np.array([lr])}
    np.savez_compressed(os.path.join(OUT, "vit_tiny12_b16_enc.npz"), **fx)
    print("vit_tiny12_b16_enc", lr, curve, "moved", abs(curve[-1] - curve[0]) / abs(curve[0]))


def gen_vit_base32f():
    """BASELINE C5's encoder geometry (videomae-base width, 32 frames -> 3,136 tokens = 24 * 128 + 64,
    n = 1024) with one layer, B=1, trainable: forward and every gradient.  C5's temporal transformer
    and fp8 have no reference code; the encoder is the reference plugin's at
    num_frames=32."""
    cfg = cpu_ref.ViTCfg(num_frames=32, num_hidden_layers=1)
    B, enc_out, n = 1, 64, 1024
    torch.manual_seed(0)
    m = _RefVideoMAEHead(cfg, enc_out, n)
    _load_vit(m, cfg, enc_out, n)
    m.freeze = False
    px = torch.from_numpy(cpu_ref.make_pixels(cfg, B, seed=32))
    y = torch.from_numpy(prng.spike_targets(32, (B, 100, n)))
    out = m(px)
    loss = torch.nn.PoissonNLLLoss(reduction="none", log_input=True)(out, y).mean()
    loss.backward()
    fx = {"log_rates": out.detach().numpy(), "loss": np.array([loss.item()])}
    fx.update(_grads_summary_small({k: p.grad for k, p in m.named_parameters() if ".key.bias" not in k}))
    np.savez_compressed(os.path.join(OUT, "vit_base32f.npz"), **fx)
    print("vit_base32f", fx["loss"])


def gen_vit_base2l_b16():
    """C3 at its benched dispatch: the reference plugin's width (videomae-base:
    d768, 12 heads, videomae.py:7-8; C3's n = 512) with two layers at B = 16 -> M = 25,088 token rows,
    trainable: forward and every gradient (summarised).  The HIP test forces the 128-clip choices
    (f32 dh + LayerNorm' launches, the big-tile products, the dW split plan of 256 slots) at this
    batch; two layers exercise the block-to-block gradient hand-off."""
    cfg = cpu_ref.ViTCfg(num_hidden_layers=2)
    B, enc_out, n = 16, 64, 512
    torch.manual_seed(0)
    m = _RefVideoMAEHead(cfg, enc_out, n)
    _load_vit(m, cfg, enc_out, n)
    m.freeze = False
    px = torch.from_numpy(cpu_ref.make_pixels(cfg, B, seed=768))
    y = torch.from_numpy(prng.spike_targets(768, (B, 100, n)))
    out = m(px)
    loss = torch.nn.PoissonNLLLoss(reduction="none", log_input=True)(out, y).mean()
    loss.backward()
    fx = {"log_rates": out.detach().numpy(), "loss": np.array([loss.item()])}
    fx.update(_grads_summary_small({k: p.grad for k, p in m.named_parameters() if ".key.bias" not in k}))
    np.savez_compressed(os.path.join(OUT, "vit_base2l_b16.npz"), **fx)
    print("vit_base2l_b16", fx["loss"])


def gen_vit_base1l():
    """The reference plugin's real width (videomae-base: d768, 12 heads, videomae.py:7-8; C3's
    n=512) with one layer, full 1568 tokens, B=1: trainable forward+backward, and a 3-step curve in
    the reference's default frozen-encoder mode (videomae.py:12,17,34-36)."""
    cfg = cpu_ref.ViTCfg(num_hidden_layers=1)
    B, enc_out, n = 1, 64, 512
    torch.manual_seed(0)
    m = _RefVideoMAEHead(cfg, enc_out, n)
    _load_vit(m, cfg, enc_out, n)
    m.freeze = False
    px = torch.from_numpy(cpu_ref.make_pixels(cfg, B))
    y = torch.from_numpy(prng.spike_targets(1, (B, 100, n)))
    out = m(px)
    loss = torch.nn.PoissonNLLLoss(reduction="none", log_input=True)(out, y).mean()
    loss.backward()
    fx = {"log_rates": out.detach().numpy(), "loss": np.array([loss.item()])}
    fx.update(_grads_summary_small({k: p.grad for k, p in m.named_parameters() if ".key.bias" not in k}))
    _load_vit(m, cfg, enc_out, n)
    m.freeze = True
    for p in m.video_mae.parameters():
        p.requires_grad = False
    batches = [(torch.from_numpy(cpu_ref.make_pixels(cfg, B, seed=500 + s)),
                torch.from_numpy(prng.spike_targets(550 + s, (B, 100, n)))) for s in range(3)]
    fx["curve_frozen"] = _ref_train_loop(m, batches, list(m.parameters()), lr=2e-7)
    np.savez_compressed(os.path.join(OUT, "vit_base1l.npz"), **fx)
    print("vit_base1l", fx["loss"], fx["curve_frozen"])


def gen_k0():
    """K0 (src/model/videomae.py:10-11, 18-25): the reference's preprocessing call pattern on a
    seeded video, run through the HF image processor itself (VideoMAEImageProcessor, whose
    videomae-base settings are the class defaults apart from mean/std; the Hub's
    preprocessor_config cannot be fetched here, so mean/std are ImageNet's, the values the
    videomae-base pretraining head un-normalises with, modeling_videomae.py:890-891)."""
    from transformers import VideoMAEImageProcessor
    proc = VideoMAEImageProcessor(image_mean=list(cpu_ref.IMAGENET_DEFAULT_MEAN),
                                  image_std=list(cpu_ref.IMAGENET_DEFAULT_STD))
    B, T, H = 2, 120, 128
    video = prng.video_frames(11, (B, T, 1, H, H))
    indicies = (torch.linspace(0, 1, 16) * 119).long()                 # videomae.py:10-11
    inputs = torch.from_numpy(video)[:, indicies]                       # videomae.py:18-22
    inputs = inputs.squeeze(2).unsqueeze(-1)
    inputs = inputs.repeat(1, 1, 1, 1, 3)
    inputs = inputs.reshape(B * len(indicies), inputs.shape[2], inputs.shape[3], inputs.shape[4])
    pv = proc(list(inputs), return_tensors="pt")["pixel_values"].squeeze(0)   # :23-24 (minus .cuda())
    pv = pv.reshape(B, len(indicies), pv.shape[1], pv.shape[2], pv.shape[3]).numpy()
    # the f32 output is a function of the uint8 resize: recover it exactly from channel 0
    m0, s0 = np.float32(cpu_ref.IMAGENET_DEFAULT_MEAN[0]), np.float32(cpu_ref.IMAGENET_DEFAULT_STD[0])
    lut = ((np.arange(256).astype(np.float64) * (1 / 255)).astype(np.float32) - m0) / s0
    u8 = np.searchsorted(lut, pv[:, :, 0])
    assert np.array_equal(lut[u8], pv[:, :, 0])
    fx = {"seed": np.int64(11), "shape": np.array([B, T, 1, H, H]), "idx": indicies.numpy().astype(np.int32),
          "mean": np.array(cpu_ref.IMAGENET_DEFAULT_MEAN, np.float32), "std": np.array(cpu_ref.IMAGENET_DEFAULT_STD, np.float32),
          "u8_frames": np.array([0, 5, 10, 15]), "u8": u8[0, [0, 5, 10, 15]].astype(np.uint8)}
    fx.update(cpu_ref.summarize("pixel_values", pv))
    np.savez_compressed(os.path.join(OUT, "k0_preprocess.npz"), **fx)
    print("k0", pv.shape, float(np.linalg.norm(pv)))


def gen_configs():
    _, update_config, config_from_kwargs = _ref_imports()
    res = {}
    for m in ("linear_video", "vmae_video", "vmae_tiny"):
        t = "vmae_video" if m.startswith("vmae") else m
        config = config_from_kwargs({"model": "include:" + os.path.join(CFG, "model", m + ".yaml")})
        config = update_config(os.path.join(CFG, "train", t + ".yaml"), config)
        res[f"{m}+{t}"] = json.loads(json.dumps(config))
    with open(os.path.join(OUT, "configs.json"), "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    print("configs", list(res))


def _ref_metric_functions():
    """The reference's own eval-metric functions, taken from its source files by name
    (metric_utils.py imports `torcheval` at module level and utils.py imports plugins whose
    dependencies are absent, so the modules cannot be imported whole).  `logger` is undefined in
    the reference module (metric_utils.py:70); a stand-in logger is supplied."""
    import ast
    import logging
    from scipy.special import gammaln
    from sklearn.metrics import accuracy_score, r2_score as r2_score_sklearn
    ns = {"np": np, "torch": torch, "gammaln": gammaln, "r2_score_sklearn": r2_score_sklearn,
          "accuracy_score": accuracy_score, "logger": logging.getLogger("reference")}
    for path, names in ((os.path.join(REF_SRC, "utils", "metric_utils.py"), ("neg_log_likelihood", "bits_per_spike")),
                        (os.path.join(REF_SRC, "utils", "utils.py"), ("metrics_list",))):
        tree = ast.parse(open(path).read(), filename=path)
        defs = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name in names]
        assert len(defs) == len(names), (path, names)
        exec(compile(ast.Module(body=defs, type_ignores=[]), path, "exec"), ns)
    return ns


def gen_metrics():
    from oracle import metrics_ref
    ns = _ref_metric_functions()
    fx = {}
    for name, (R, T, N, seed, metrics, log_input) in metrics_ref.METRIC_CASES.items():
        gt, pred = metrics_ref.metric_case(name)
        g = torch.from_numpy(gt)
        p = torch.exp(torch.from_numpy(pred)) if log_input else torch.from_numpy(pred)   # base.py:186
        res = ns["metrics_list"](gt=g.transpose(-1, 0), pred=p.transpose(-1, 0), metrics=list(metrics),
                                 device="cpu")                                         # base.py:190-195
        for k, v in res.items():
            fx[f"{name}.{k}"] = np.float64(v)
        if "bps" in metrics:
            _g, _p = g.numpy(), p.numpy()
            fx[f"{name}.bps_per_neuron"] = np.array(
                [ns["bits_per_spike"](_p[:, :, [i]], _g[:, :, [i]]) for i in range(min(R, N))], dtype=np.float64)
        print("metrics", name, {k: float(v) for k, v in res.items()})
    # the reference's IndexError when trials > N (utils.py:128-129)
    gt, pred = metrics_ref.metric_case("m_wide")
    try:
        ns["metrics_list"](gt=torch.from_numpy(gt).transpose(-1, 0),
                           pred=torch.exp(torch.from_numpy(pred)).transpose(-1, 0), metrics=["bps"], device="cpu")
        fx["m_wide.bps_error"] = np.array("none")
    except IndexError as e:
        fx["m_wide.bps_error"] = np.array("IndexError: " + str(e))
    np.savez_compressed(os.path.join(OUT, "metrics.npz"), **fx)


if __name__ == "__main__":
    os.makedirs(OUT, exist_ok=True)
    torch.set_num_threads(8)
    which = sys.argv[1:] or ["configs", "linear", "vit_small", "vit_tiny1l", "vit_tiny12", "vit_tiny12_b16",
                             "vit_base1l", "vit_base32f", "k0", "metrics"]
    for w in which:
        globals()["gen_" + w]()
