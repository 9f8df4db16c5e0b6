"""CPU fp32 restatement of the reference's video->spike training hot path.

TEST INFRASTRUCTURE ONLY.  This module is the parity *checker*: only `tests/`,
`__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may import it.  The product
path (`video-spike_amd/vspike`) never imports it and has no CPU fallback.

Every function restates one piece of the reference with plain torch CPU fp32 ops (autograd
supplies the backward for the checker).  Parity of this restatement is PINNED by golden
fixtures generated from the reference itself (`oracle/gen_fixtures.py` imports
`/root/reference/src/model/linear.py` and the installed HF `transformers.VideoMAEModel`, the
third-party encoder the reference runs) — see `tests/test_oracle_golden.py`.

Reference citations (paths relative to the reference repo root):
  * `src/model/linear.py:3-56`                       Linear plugin (flatten -> MLP enc -> MLP dec -> reshape)
  * `src/model/videomae.py:16-32`                    VideoMAE plugin forward (encoder -> flatten -> Linear -> Linear)
  * `src/model/videomae/modeling_videomae.py:101-112` fixed sinusoid position table
  * `src/model/videomae/modeling_videomae.py:183-196` tubelet Conv3d patch embedding
  * `src/model/videomae/modeling_videomae.py:230-266` self-attention (q/v bias, k bias == 0, softmax(QK^T/sqrt(dh))V)
  * `src/model/videomae/modeling_videomae.py:419-445` pre-LN block
  * `src/train.py:59` + `src/trainer/base.py:141-143` PoissonNLLLoss(log_input=True).mean()
  * `src/train.py:44-57` + `src/trainer/base.py:144-159` AdamW + OneCycleLR train step
  * `src/model/videomae.py:10-11,18-25`             K0 preprocessing: frame gather, gray->RGB, HF image processor
    (third-party: transformers VideoMAEImageProcessor -> PIL Image.resize BILINEAR on uint8 frames,
    Pillow `src/libImaging/Resample.c`; rescale in float64 `image_transforms.rescale`; f32 normalise)
"""
from __future__ import annotations

import dataclasses
import math
from typing import Dict, List, Tuple

import numpy as np
import torch

from . import prng


# ----------------------------------------------------------------------------------------------
# configuration
# ----------------------------------------------------------------------------------------------
@dataclasses.dataclass(frozen=True)
class ViTCfg:
    """Encoder geometry (keys mirror `config/model/videomae/videomae.yaml` of the reference)."""
    image_size: int = 224
    patch_size: int = 16
    num_channels: int = 3
    num_frames: int = 16
    tubelet_size: int = 2
    hidden_size: int = 768
    num_hidden_layers: int = 12
    num_attention_heads: int = 12
    intermediate_size: int = 3072
    layer_norm_eps: float = 1e-12

    @property
    def num_tokens(self) -> int:
        g = self.image_size // self.patch_size
        return (self.num_frames // self.tubelet_size) * g * g

    @property
    def patch_dim(self) -> int:
        return self.num_channels * self.tubelet_size * self.patch_size * self.patch_size


VIT_BASE = ViTCfg()
VIT_TINY = ViTCfg(hidden_size=192, num_attention_heads=3, intermediate_size=768)
VIT_SMALL_FIXTURE = ViTCfg(image_size=112, num_frames=8, hidden_size=128, num_hidden_layers=2,
                           num_attention_heads=2, intermediate_size=512)


# ----------------------------------------------------------------------------------------------
# deterministic parameters / inputs (names follow the reference plugin's state_dict)
# ----------------------------------------------------------------------------------------------
def vit_param_shapes(cfg: ViTCfg, enc_out: int, n_out: int) -> Dict[str, Tuple[int, ...]]:
    D, F = cfg.hidden_size, cfg.intermediate_size
    s: Dict[str, Tuple[int, ...]] = {
        "video_mae.embeddings.patch_embeddings.projection.weight":
            (D, cfg.num_channels, cfg.tubelet_size, cfg.patch_size, cfg.patch_size),
        "video_mae.embeddings.patch_embeddings.projection.bias": (D,),
    }
    for i in range(cfg.num_hidden_layers):
        p = f"video_mae.encoder.layer.{i}."
        s.update({
            p + "attention.attention.query.weight": (D, D), p + "attention.attention.query.bias": (D,),
            p + "attention.attention.key.weight": (D, D),
            p + "attention.attention.value.weight": (D, D), p + "attention.attention.value.bias": (D,),
            p + "attention.output.dense.weight": (D, D), p + "attention.output.dense.bias": (D,),
            p + "intermediate.dense.weight": (F, D), p + "intermediate.dense.bias": (F,),
            p + "output.dense.weight": (D, F), p + "output.dense.bias": (D,),
            p + "layernorm_before.weight": (D,), p + "layernorm_before.bias": (D,),
            p + "layernorm_after.weight": (D,), p + "layernorm_after.bias": (D,),
        })
    s["encoder.weight"] = (enc_out, cfg.num_tokens * D)
    s["encoder.bias"] = (enc_out,)
    s["decoder.weight"] = (n_out * 100, enc_out)
    s["decoder.bias"] = (n_out * 100,)
    return s


def make_vit_params(cfg: ViTCfg, enc_out: int, n_out: int, seed: int = 2) -> Dict[str, np.ndarray]:
    """Seeded weights.  Matrices ~ N(0, 0.02) like HF `_init_weights` (modeling_videomae.py:512-522);
    biases and LayerNorm affine terms are perturbed away from 0/1 so that every term is exercised."""
    out = {}
    for name, shape in vit_param_shapes(cfg, enc_out, n_out).items():
        if name.endswith("layernorm_before.weight") or name.endswith("layernorm_after.weight"):
            out[name] = prng.normal(seed, shape, name, std=0.1, mean=1.0)
        elif name in ("encoder.weight",):
            out[name] = prng.normal(seed, shape, name, std=1.0 / math.sqrt(shape[1]))
        elif name in ("decoder.weight",):
            out[name] = prng.normal(seed, shape, name, std=0.5 / math.sqrt(shape[1]))
        elif len(shape) == 1:
            out[name] = prng.normal(seed, shape, name, std=0.02)
        else:
            out[name] = prng.normal(seed, shape, name, std=0.02)
    return out


def linear_param_shapes(input_dim: int, enc_hidden: List[int], enc_out: int,
                        dec_hidden: List[int], output_dim: int) -> Dict[str, Tuple[int, ...]]:
    """Names of `src/model/linear.py:17-56` (nn.Sequential indices 0,2,4 hold the Linear layers)."""
    s = {}
    dims = [input_dim] + list(enc_hidden) + [enc_out]
    for j in range(len(dims) - 1):
        s[f"encoder.layers.{2 * j}.weight"] = (dims[j + 1], dims[j])
        s[f"encoder.layers.{2 * j}.bias"] = (dims[j + 1],)
    dims = [enc_out] + list(dec_hidden) + [output_dim]
    for j in range(len(dims) - 1):
        s[f"decoder.layers.{2 * j}.weight"] = (dims[j + 1], dims[j])
        s[f"decoder.layers.{2 * j}.bias"] = (dims[j + 1],)
    return s


def make_linear_params(shapes: Dict[str, Tuple[int, ...]], seed: int = 2,
                       input_scale: float = 1.0 / 128.0) -> Dict[str, np.ndarray]:
    """std 0.5/sqrt(fan_in); the first layer also absorbs `input_scale` because the plugin's raw
    inputs are 0..255 pixel values (base.py:64-67 feeds them unnormalised)."""
    out = {}
    for name, shape in shapes.items():
        fan_in = shape[1] if len(shape) == 2 else shapes[name.replace(".bias", ".weight")][1]
        std = 0.5 / math.sqrt(fan_in) * (input_scale if name == "encoder.layers.0.weight" else 1.0)
        out[name] = prng.normal(seed, shape, name, std=std)
    return out


def make_pixels(cfg: ViTCfg, batch: int, seed: int = 0) -> np.ndarray:
    return prng.normal(seed, (batch, cfg.num_frames, cfg.num_channels, cfg.image_size, cfg.image_size),
                       "pixel_values")


# ----------------------------------------------------------------------------------------------
# encoder restatement
# ----------------------------------------------------------------------------------------------
def sinusoid_table(n_position: int, d_hid: int) -> torch.Tensor:
    """Fixed position table, `modeling_videomae.py:101-112` (float64 angles, cast to float32)."""
    pos = np.arange(n_position, dtype=np.float64)[:, None]
    j = np.arange(d_hid)[None, :]
    angle = pos / np.power(10000.0, 2 * (j // 2) / d_hid)
    table = np.empty_like(angle)
    table[:, 0::2] = np.sin(angle[:, 0::2])
    table[:, 1::2] = np.cos(angle[:, 1::2])
    return torch.from_numpy(table.astype(np.float32))


def im2col(pixels: torch.Tensor, cfg: ViTCfg) -> torch.Tensor:
    """(B, F, C, H, W) -> (B*N, C*t*p*p).  Token n = (f', hp, wp) row-major (the Conv3d output's
    `flatten(2).transpose(1, 2)` order, `modeling_videomae.py:194-195`); column = (c, t, i, j),
    the Conv3d weight's flatten order."""
    B, F, C, H, W = pixels.shape
    t, p = cfg.tubelet_size, cfg.patch_size
    x = pixels.reshape(B, F // t, t, C, H // p, p, W // p, p)
    x = x.permute(0, 1, 4, 6, 3, 2, 5, 7)          # B, f', hp, wp, C, t, i, j
    return x.reshape(B * (F // t) * (H // p) * (W // p), C * t * p * p)


def layer_norm(x, g, b, eps):
    return torch.nn.functional.layer_norm(x, (x.shape[-1],), g, b, eps)


def _plain_mm(a: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    return a @ w.T


def vit_layer(x: torch.Tensor, P: Dict[str, torch.Tensor], prefix: str, cfg: ViTCfg, mm=None) -> torch.Tensor:
    """One pre-LN block, `modeling_videomae.py:419-445` with `VideoMAESelfAttention` :230-266.
    `mm(a, W)` is the block's four Linear products (qkv, proj, fc1, fc2: a @ W^T by default;
    `mx_matmul` for the MX-FP8 products of BASELINE C5)."""
    mm = mm or _plain_mm
    B, N, D = x.shape
    H = cfg.num_attention_heads
    dh = D // H
    h = layer_norm(x, P[prefix + "layernorm_before.weight"], P[prefix + "layernorm_before.bias"],
                   cfg.layer_norm_eps)
    q = mm(h, P[prefix + "attention.attention.query.weight"]) + P[prefix + "attention.attention.query.bias"]
    k = mm(h, P[prefix + "attention.attention.key.weight"])           # k bias is identically zero
    v = mm(h, P[prefix + "attention.attention.value.weight"]) + P[prefix + "attention.attention.value.bias"]
    q, k, v = (t.reshape(B, N, H, dh).permute(0, 2, 1, 3) for t in (q, k, v))
    s = (q @ k.transpose(-1, -2)) / math.sqrt(dh)
    pr = torch.softmax(s, dim=-1)
    o = (pr @ v).permute(0, 2, 1, 3).reshape(B, N, D)
    y = x + mm(o, P[prefix + "attention.output.dense.weight"]) + P[prefix + "attention.output.dense.bias"]
    h2 = layer_norm(y, P[prefix + "layernorm_after.weight"], P[prefix + "layernorm_after.bias"],
                    cfg.layer_norm_eps)
    a = torch.nn.functional.gelu(mm(h2, P[prefix + "intermediate.dense.weight"]) + P[prefix + "intermediate.dense.bias"])
    return y + mm(a, P[prefix + "output.dense.weight"]) + P[prefix + "output.dense.bias"]


def mx_dequant(x: torch.Tensor) -> torch.Tensor:
    """MX-FP8 round trip of an operand as BASELINE C5's products see it (csrc/fp8.hip:7-10 recipe, the
    OCP MX format): the value rounded to bf16 (the activations / weights the kernels quantise are
    bf16), then per 32 consecutive elements of the last axis an E8M0 scale 2^e with e = ceil(log2(
    amax / 448)) (amax * f32(1/448), clamped to [-126, 127], 0 for an all-zero block) and elements
    rounded to nearest-even e4m3 (torch.float8_e4m3fn); returned dequantised in f32."""
    shp = x.shape
    xb = x.detach().to(torch.bfloat16).float().reshape(*shp[:-1], shp[-1] // 32, 32)
    amax = xb.abs().amax(-1)
    bits = (amax * torch.tensor(1.0 / 448.0, dtype=torch.float32)).view(torch.int32)
    e = ((bits >> 23) & 0xFF) - 127 + ((bits & 0x7FFFFF) != 0).int()
    e = torch.where(((bits >> 23) & 0xFF) == 0, torch.full_like(e, -126), e).clamp(-126, 127)
    e = torch.where(amax > 0, e, torch.zeros_like(e))
    inv = ((127 - e) << 23).view(torch.float32)[..., None]       # 2^-e exactly
    scale = ((127 + e) << 23).view(torch.float32)[..., None]     # 2^e exactly
    return ((xb * inv).to(torch.float8_e4m3fn).float() * scale).reshape(shp)


class _MXLinear(torch.autograd.Function):
    """a @ W^T on the MX-FP8 round trips of both operands; the backward is the straight-through one the
    HIP path runs (bf16 products on the unquantised activations and weights: dA = g W, dW = g^T a)."""

    @staticmethod
    def forward(ctx, a, w):
        ctx.save_for_backward(a, w)
        return mx_dequant(a) @ mx_dequant(w).T

    @staticmethod
    def backward(ctx, g):
        a, w = ctx.saved_tensors
        return g @ w, g.reshape(-1, g.shape[-1]).T @ a.reshape(-1, a.shape[-1])


def mx_matmul(a: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """`mm` for vit_layer: the block products of BASELINE C5's fp8 encoder (compute_dtype "fp8")."""
    return _MXLinear.apply(a, w)


def videomae_encoder(pixels: torch.Tensor, P: Dict[str, torch.Tensor], cfg: ViTCfg, mm=None) -> torch.Tensor:
    """`VideoMAEModel.forward` (modeling_videomae.py:592-715): patch-embed + sinusoid, 12 blocks,
    no final LayerNorm because `use_mean_pooling=True` (:571-574)."""
    B = pixels.shape[0]
    N, D = cfg.num_tokens, cfg.hidden_size
    cols = im2col(pixels, cfg)
    w = P["video_mae.embeddings.patch_embeddings.projection.weight"].reshape(D, -1)
    x = cols @ w.T + P["video_mae.embeddings.patch_embeddings.projection.bias"]
    x = x.reshape(B, N, D) + sinusoid_table(N, D)
    for i in range(cfg.num_hidden_layers):
        x = vit_layer(x, P, f"video_mae.encoder.layer.{i}.", cfg, mm)
    return x


def videomae_plugin_forward(pixels: torch.Tensor, P: Dict[str, torch.Tensor], cfg: ViTCfg,
                            freeze_encoder: bool = True, mm=None) -> torch.Tensor:
    """`src/model/videomae.py:16-32` from `pixel_values` on (the CPU preprocessing K0 is outside)."""
    B = pixels.shape[0]
    if freeze_encoder:
        with torch.no_grad():
            hid = videomae_encoder(pixels, P, cfg, mm)
    else:
        hid = videomae_encoder(pixels, P, cfg, mm)
    z = hid.flatten(1) @ P["encoder.weight"].T + P["encoder.bias"]
    r = z @ P["decoder.weight"].T + P["decoder.bias"]
    return r.reshape(B, 100, -1)


def linear_plugin_forward(x: torch.Tensor, P: Dict[str, torch.Tensor]) -> torch.Tensor:
    """`src/model/linear.py:10-15`: ReLU after every hidden Linear, none after the encoder's
    output layer nor the decoder's output layer."""
    def mlp(h, prefix):
        idx = sorted(int(k.split(".")[2]) for k in P if k.startswith(prefix) and k.endswith(".weight"))
        for j, i in enumerate(idx):
            h = h @ P[f"{prefix}{i}.weight"].T + P[f"{prefix}{i}.bias"]
            if j < len(idx) - 1:
                h = torch.relu(h)
        return h
    B = x.shape[0]
    h = mlp(x.flatten(1), "encoder.layers.")
    r = mlp(h, "decoder.layers.")
    return r.reshape(B, 100, -1)


def poisson_nll_mean(log_rate: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
    """`PoissonNLLLoss(reduction='none', log_input=True)(...).mean()`: mean(exp(x) - y*x)."""
    return (torch.exp(log_rate) - target * log_rate).mean()


# ----------------------------------------------------------------------------------------------
# train-step restatement (loss curve oracle)
# ----------------------------------------------------------------------------------------------
def to_torch(params: Dict[str, np.ndarray], requires_grad=True) -> Dict[str, torch.Tensor]:
    return {k: torch.tensor(v, dtype=torch.float32, requires_grad=requires_grad) for k, v in params.items()}


def mse_mean(pred: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
    """`torch.nn.MSELoss()` (mean reduction): the north_star's MSE head option.  The reference
    itself trains with PoissonNLL only (src/train.py:59) and computes mse as an eval metric
    (src/utils/utils.py:169-171)."""
    return ((pred - target) ** 2).mean()


def train_curve(forward, params: Dict[str, torch.Tensor], batches, lr=5e-5, wd=0.01, eps=1e-8,
                warmup_pct=0.15, div_factor=10.0, trainable=None, criterion=None) -> List[float]:
    """`src/train.py:44-57` (AdamW + OneCycleLR, total_steps = len(batches)) and the loop body of
    `src/trainer/base.py:144-159`.  Returns the per-step training loss.  criterion: default the
    reference's PoissonNLL mean (src/train.py:59)."""
    criterion = criterion or poisson_nll_mean
    names = list(params) if trainable is None else [n for n in params if trainable(n)]
    opt = torch.optim.AdamW([params[n] for n in names], lr=lr, weight_decay=wd, eps=eps)
    sched = torch.optim.lr_scheduler.OneCycleLR(opt, total_steps=len(batches), max_lr=lr,
                                                pct_start=warmup_pct, div_factor=div_factor)
    losses = []
    for x, y in batches:
        loss = criterion(forward(x, params), y)
        loss.backward()
        opt.step()
        sched.step()
        opt.zero_grad()
        losses.append(float(loss.item()))
    return losses


# ----------------------------------------------------------------------------------------------
# fixture comparison helpers
# ----------------------------------------------------------------------------------------------
FULL_GRAD_LIMIT = 65536


def summarize(name: str, t: np.ndarray, seed: int = 7, full_limit: int = FULL_GRAD_LIMIT) -> Dict[str, np.ndarray]:
    """Full tensor when small (<= full_limit elements), else (norm, 3 seeded projections, first
    512 values)."""
    t = np.array(t, dtype=np.float32, copy=True)       # never keep a view of a live .grad
    if t.size <= full_limit:
        return {"full/" + name: t}
    flat = t.reshape(-1).astype(np.float64)
    projs = np.array([float(flat @ prng.normal(seed, (flat.size,), f"{name}#proj{i}").astype(np.float64))
                      for i in range(3)])
    return {"norm/" + name: np.array([np.linalg.norm(flat)]), "proj/" + name: projs,
            "head/" + name: t.reshape(-1)[:512].copy()}


def compare_summary(name: str, t: np.ndarray, fx: Dict[str, np.ndarray], rtol: float, atol: float,
                    seed: int = 7) -> Tuple[bool, str]:
    t = np.asarray(t, dtype=np.float32)
    if "full/" + name in fx:
        ref = fx["full/" + name]
        err = np.abs(t - ref)
        ok = bool(np.all(err <= atol + rtol * np.abs(ref)))
        return ok, f"{name}: max|d|={err.max():.3e} max|ref|={np.abs(ref).max():.3e}"
    mine = summarize(name, t, seed, full_limit=0)
    msgs, ok = [], True
    for key in ("norm/", "proj/", "head/"):
        ref, got = fx[key + name], mine[key + name]
        # a random projection of an error vector e has magnitude ~||e||, so projections (and the
        # norm itself) are judged against the tensor norm; leading values against their own max.
        scale = float(fx["norm/" + name][0]) if key != "head/" else float(np.abs(ref).max())
        err = np.abs(got - ref).max()
        good = err <= atol + rtol * max(scale, 1e-30)
        ok &= bool(good)
        msgs.append(f"{key}{name} max|d|={err:.3e} scale={scale:.3e}")
    return ok, "; ".join(msgs)


def summary_rel_error(name: str, t: np.ndarray, fx: Dict[str, np.ndarray], seed: int = 7) -> float:
    """One norm-relative error figure of `t` against its fixture entry (the bar for reduced
    precision, where element-wise relative tolerances are meaningless near zero): for a full tensor
    ||t - ref|| / ||ref||; for a summarised one the largest of |norm - ref| and |proj_i - ref_i|
    over the reference norm, and of the leading values' max|diff| over their max|ref|."""
    t = np.asarray(t, dtype=np.float64)
    if "full/" + name in fx:
        ref = fx["full/" + name].astype(np.float64)
        return float(np.linalg.norm((t - ref).ravel()) / max(np.linalg.norm(ref.ravel()), 1e-30))
    mine = summarize(name, t, seed, full_limit=0)
    nrm = max(float(fx["norm/" + name][0]), 1e-30)
    e = max(abs(float(mine["norm/" + name][0]) - nrm), float(np.abs(mine["proj/" + name] - fx["proj/" + name]).max()))
    head = fx["head/" + name].astype(np.float64)
    eh = float(np.abs(mine["head/" + name] - head).max() / max(np.abs(head).max(), 1e-30))
    return max(e / nrm, eh)


# ------------------------------------------------------------------------------------------------
# K0: the VideoMAE plugin's preprocessing (src/model/videomae.py:10-11, 18-25), restated.
# ------------------------------------------------------------------------------------------------
IMAGENET_DEFAULT_MEAN = (0.485, 0.456, 0.406)   # the un-normalisation videomae-base's pretraining head uses
IMAGENET_DEFAULT_STD = (0.229, 0.224, 0.225)    # (src/model/videomae/modeling_videomae.py:890-891)


def frame_indices(n_frames: int = 16, n_source: int = 120) -> np.ndarray:
    """`videomae.py:10-11`: (torch.linspace(0, 1, 16) * 119).long()."""
    return (torch.linspace(0, 1, n_frames) * (n_source - 1)).long().numpy().astype(np.int32)


_PIL_BITS = 22  # Pillow PRECISION_BITS for 8-bit images: 32 - 8 - 2


def pil_bilinear_coeffs(in_size: int, out_size: int):
    """Pillow Resample.c `precompute_coeffs` (bilinear, support 1) + `normalize_coeffs_8bpc`:
    per output index: (xmin, fixed-point weights).  Python floats are IEEE doubles evaluated in
    the C expression order, so the weights are Pillow's exactly."""
    scale = in_size / out_size
    filterscale = max(scale, 1.0)
    support = 1.0 * filterscale
    ss = 1.0 / filterscale
    out = []
    for xx in range(out_size):
        center = (xx + 0.5) * scale
        xmin = max(int(center - support + 0.5), 0)
        xmax = min(int(center + support + 0.5), in_size) - xmin
        w = []
        for x in range(xmax):
            t = abs((x + xmin - center + 0.5) * ss)
            w.append(1.0 - t if t < 1.0 else 0.0)
        ww = 0.0
        for v in w:
            ww += v
        w = [v / ww if ww != 0.0 else v for v in w]
        k = [int(-0.5 + v * (1 << _PIL_BITS)) if v < 0 else int(0.5 + v * (1 << _PIL_BITS)) for v in w]
        out.append((xmin, np.array(k, dtype=np.int64)))
    return out


def _clip8(v: np.ndarray) -> np.ndarray:
    return np.where(v >= (1 << _PIL_BITS << 8), 255, np.where(v <= 0, 0, v >> _PIL_BITS)).astype(np.int64)


def pil_resize_u8(img: np.ndarray, out_h: int, out_w: int) -> np.ndarray:
    """PIL `Image.resize((out_w, out_h), BILINEAR)` of a uint8 (H, W) image: horizontal pass into a
    uint8 intermediate, then vertical (Resample.c ImagingResampleHorizontal/Vertical_8bpc)."""
    h, w = img.shape
    src = img.astype(np.int64)
    tmp = np.zeros((h, out_w), dtype=np.int64)
    for xx, (xmin, k) in enumerate(pil_bilinear_coeffs(w, out_w)):
        acc = np.full(h, 1 << (_PIL_BITS - 1), dtype=np.int64)
        for i, kk in enumerate(k):
            acc += src[:, xmin + i] * kk
        tmp[:, xx] = _clip8(acc)
    out = np.zeros((out_h, out_w), dtype=np.int64)
    for yy, (ymin, k) in enumerate(pil_bilinear_coeffs(h, out_h)):
        acc = np.full(out_w, 1 << (_PIL_BITS - 1), dtype=np.int64)
        for j, kk in enumerate(k):
            acc += tmp[ymin + j, :] * kk
        out[yy, :] = _clip8(acc)
    return out.astype(np.uint8)


def video_preprocess(video: np.ndarray, idx: np.ndarray, size: int = 224, mean=IMAGENET_DEFAULT_MEAN,
                     std=IMAGENET_DEFAULT_STD) -> np.ndarray:
    """`videomae.py:18-25` for square frames: video (B, T, 1, H, W) integer-valued 0..255 ->
    pixel_values (B, F, 3, size, size) f32.  Gray is repeated to RGB (so the three channels differ
    only by mean/std); HF casts the float frame to uint8 (`astype`), resizes the shortest edge to
    `size` with PIL, centre-crops `size` (a no-op here), rescales in float64
    (`image.astype(np.float64) * (1/255)` -> f32) and normalises in f32."""
    b, t, c, h, w = video.shape
    assert c == 1 and h == w
    m = np.asarray(mean, dtype=np.float32)
    sd = np.asarray(std, dtype=np.float32)
    out = np.empty((b, len(idx), 3, size, size), dtype=np.float32)
    for bi in range(b):
        for fi, src in enumerate(idx):
            u8 = video[bi, src, 0].astype(np.uint8)
            r = pil_resize_u8(u8, size, size)
            x = (r.astype(np.float64) * (1 / 255)).astype(np.float32)
            for ch in range(3):
                out[bi, fi, ch] = (x - m[ch]) / sd[ch]
    return out


# ----------------------------------------------------------------------------------------------
# R3D-18 (BASELINE C4).  NOT in the reference (no CNN encoder, registry
# src/utils/utils.py:28-34): this restates torchvision's published video ResNet r3d_18
# (VideoResNet(BasicBlock, [Conv3DSimple] * 4, [2, 2, 2, 2], BasicStem); torchvision is not installed
# here) with torch CPU ops, under the reference head (src/model/videomae.py:13-14,28-31).  The HIP
# path is checked against it; parity is UNPINNED by any reference output.
# ----------------------------------------------------------------------------------------------
@dataclasses.dataclass(frozen=True)
class R3DCfg:
    num_frames: int = 32
    image_size: int = 112
    num_channels: int = 3
    layers: Tuple[int, ...] = (2, 2, 2, 2)
    widths: Tuple[int, ...] = (64, 128, 256, 512)
    bn_eps: float = 1e-5
    bn_momentum: float = 0.1


def r3d_conv_specs(cfg: R3DCfg):
    """(name, ci, co, kernel, stride, padding) in forward order; names as torchvision's r3d_18."""
    specs = [("stem.0", cfg.num_channels, 64, (3, 7, 7), (1, 2, 2), (1, 3, 3))]
    cin = 64
    for li, (nb, w) in enumerate(zip(cfg.layers, cfg.widths)):
        for b in range(nb):
            s = 2 if (b == 0 and li > 0) else 1
            pre = f"layer{li + 1}.{b}."
            specs.append((pre + "conv1.0", cin, w, (3, 3, 3), (s, s, s), (1, 1, 1)))
            specs.append((pre + "conv2.0", w, w, (3, 3, 3), (1, 1, 1), (1, 1, 1)))
            if s != 1 or cin != w:
                specs.append((pre + "downsample.0", cin, w, (1, 1, 1), (s, s, s), (0, 0, 0)))
            cin = w
    return specs


def make_r3d_params(cfg: R3DCfg, enc_out: int, n_out: int, seed: int = 3) -> Dict[str, np.ndarray]:
    """Seeded weights in torch layouts: convs ~ N(0, sqrt(2 / fan_out)) (torchvision's kaiming fan_out
    init), BN affine perturbed around (1, 0) so every term is exercised, the reference head ~ its
    nn.Linear scale."""
    out = {}
    for name, ci, co, k, _, _ in r3d_conv_specs(cfg):
        fan_out = co * k[0] * k[1] * k[2]
        out[name + ".weight"] = prng.normal(seed, (co, ci) + tuple(k), name, std=math.sqrt(2.0 / fan_out))
        bn = name[:-2] + ".1"
        out[bn + ".weight"] = prng.normal(seed, (co,), bn + ".weight", std=0.1, mean=1.0)
        out[bn + ".bias"] = prng.normal(seed, (co,), bn + ".bias", std=0.1)
    feat = cfg.widths[-1]
    out["encoder.weight"] = prng.normal(seed, (enc_out, feat), "encoder.weight", std=1.0 / math.sqrt(feat))
    out["encoder.bias"] = prng.normal(seed, (enc_out,), "encoder.bias", std=0.02)
    out["decoder.weight"] = prng.normal(seed, (100 * n_out, enc_out), "decoder.weight", std=0.5 / math.sqrt(enc_out))
    out["decoder.bias"] = prng.normal(seed, (100 * n_out,), "decoder.bias", std=0.02)
    return out


def make_r3d_pixels(cfg: R3DCfg, batch: int, seed: int = 0) -> np.ndarray:
    """Clips in the plugin's pixel layout (B, T, C, H, W) (the VideoMAE pixel_values order)."""
    return prng.normal(seed, (batch, cfg.num_frames, cfg.num_channels, cfg.image_size, cfg.image_size), "r3d_pixels")


def r3d18_forward(pixels: torch.Tensor, P: Dict[str, torch.Tensor], cfg: R3DCfg, running=None,
                  training: bool = True, relu_masks=None, mask_log=None) -> torch.Tensor:
    """log-rates (B, 100, N): the R3D-18 encoder (training-mode BatchNorm: batch statistics; `running`
    = dict of running_mean / running_var tensors updated in place when given) -> AdaptiveAvgPool3d(1)
    -> the reference head.

    relu_masks (checker option): {conv name: bool tensor (N, D, H, W, C), channels-last} -- the ReLU
    decisions the implementation under test took.  A pre-activation within rounding of zero can land
    on either side of the ReLU in two correct f32 / f64 computations, and one flipped element moves a
    gradient that sums ~10^5 cancelling terms by a whole element; conditioning the oracle on the same
    discrete decisions (out = pre * mask) leaves only arithmetic differences to compare.  mask_log
    (a dict) receives per unit the count of flipped decisions and the largest |pre-activation| among
    them, so a caller can check the flips are only rounding-level ties."""
    import torch.nn.functional as F
    B = pixels.shape[0]
    x = pixels.permute(0, 2, 1, 3, 4)                       # (B, C, T, H, W): torch's NCDHW

    def unit(name, x, stride, pad, relu, residual=None):
        y = F.conv3d(x, P[name + ".weight"], None, stride, pad)
        bn = name[:-2] + ".1"
        rm = running.get(bn + ".running_mean") if running is not None else None
        rv = running.get(bn + ".running_var") if running is not None else None
        y = F.batch_norm(y, rm, rv, P[bn + ".weight"], P[bn + ".bias"], training=training,
                         momentum=cfg.bn_momentum, eps=cfg.bn_eps)
        if residual is not None:
            y = y + residual
        if relu and relu_masks is not None and name in relu_masks:
            m = relu_masks[name].permute(0, 4, 1, 2, 3).to(y.dtype)
            if mask_log is not None:
                with torch.no_grad():
                    flip = (y.detach() > 0) != (m > 0)
                    mask_log[name] = (int(flip.sum()), float(y.detach().abs()[flip].max()) if flip.any() else 0.0,
                                      float(y.detach().abs().max()))
            return y * m
        return F.relu(y) if relu else y

    specs = {s[0]: s for s in r3d_conv_specs(cfg)}
    x = unit("stem.0", x, (1, 2, 2), (1, 3, 3), True)
    for li, nb in enumerate(cfg.layers):
        for b in range(nb):
            pre = f"layer{li + 1}.{b}."
            s1 = specs[pre + "conv1.0"]
            h = unit(pre + "conv1.0", x, s1[4], s1[5], True)
            if pre + "downsample.0" in specs:
                sd = specs[pre + "downsample.0"]
                sc = unit(pre + "downsample.0", x, sd[4], sd[5], False)
            else:
                sc = x
            x = unit(pre + "conv2.0", h, (1, 1, 1), (1, 1, 1), True, residual=sc)
    feat = x.mean(dim=(2, 3, 4))                             # AdaptiveAvgPool3d(1) + flatten
    z = F.linear(feat, P["encoder.weight"], P["encoder.bias"])    # videomae.py:29
    r = F.linear(z, P["decoder.weight"], P["decoder.bias"])        # videomae.py:30
    return r.reshape(B, 100, -1)                                   # videomae.py:31
