"""R3D plugin: an R3D-18 video encoder (BASELINE C4: "ResNet-18 3D-conv encoder, 32x112x112 clips ->
256 neurons, fp32") under the reference's head and plugin surface.

The reference has NO CNN encoder (its registry src/utils/utils.py:28-34 holds
Linear / VideoMAE / SSL classes only), so there is nothing of the reference's to pin the encoder to:
parity is against the CPU oracle's torch restatement (oracle/cpu_ref.py r3d18_*), "parity unpinned"
in DESIGN.md's sense.  The architecture is torchvision's video ResNet r3d_18 (torchvision is not
installed here; restated from its published definition): stem Conv3d(3, 64, (3, 7, 7), stride
(1, 2, 2), pad (1, 3, 3)) + BatchNorm3d + ReLU; four stages of two BasicBlocks (3x3x3 convs, widths
64 / 128 / 256 / 512, stride 2 at the first block of stages 2-4 with a 1x1x1 stride-2 conv + BN
shortcut); AdaptiveAvgPool3d(1).  The 512-d pooled feature feeds the reference head exactly as
src/model/videomae.py:13-14,28-31 feeds the flattened token grid: Linear(512 -> encoder.output_dim),
Linear(-> decoder.output_dim = 100 * neurons), reshape (B, 100, N) log-rates.

Constructor / forward / module obligations as VideoMAE (vspike/vit.py): `R3D(config.model)`,
`forward(x) -> (B, 100, N)`, x = pixel clips (B, T, 3, H, W) (the layout VideoMAE's pixel_values use)
or raw gray video (B, T0, 1, H0, W0) preprocessed on the device (vs_video_preprocess, 112 x 112).
MI355X design: every op is a libvspike launch (csrc/conv3d.hip: implicit-GEMM Conv3d forward / dX /
dW on the exact-f32 MFMA, BatchNorm3d statistics in the conv epilogue, fused BN + residual + ReLU,
fixed-order reductions); activations channels-last f32; parameters in two flat f32 buffers (one fused
AdamW launch each); the backward hand-sequenced (one autograd node).  Training-mode BatchNorm (batch
statistics, running buffers updated with momentum 0.1) in `train()`, the running statistics in
`eval()`.
"""
from __future__ import annotations

import ctypes
import dataclasses
import math
from typing import List, Optional, Tuple

import torch
from torch import nn

from . import _lib as L
from . import ops
from .layout import FlatLayout
from ._lib import check, lib, require_device, stream


@dataclasses.dataclass(frozen=True)
class R3DCfg:
    num_frames: int = 32
    image_size: int = 112
    num_channels: int = 3
    layers: Tuple[int, ...] = (2, 2, 2, 2)
    widths: Tuple[int, ...] = (64, 128, 256, 512)
    bn_eps: float = 1e-5
    bn_momentum: float = 0.1

    @classmethod
    def from_config(cls, d) -> "R3DCfg":
        if not d:
            return cls()
        d = dict(d)
        kw = {}
        for f in dataclasses.fields(cls):
            if f.name in d:
                v = d[f.name]
                kw[f.name] = tuple(int(x) for x in v) if f.name in ("layers", "widths") else \
                    (float(v) if f.name.startswith("bn_") else int(v))
        return cls(**kw)


@dataclasses.dataclass
class ConvSpec:
    name: str          # torchvision-style module prefix of the conv (its BN is the sibling ".1")
    ci: int            # input channels as stored (the 3-channel stem input padded to 4)
    co: int
    k: Tuple[int, int, int]
    s: Tuple[int, int, int]
    p: Tuple[int, int, int]
    ci_ref: int = 0    # the reference (torch) input channel count


def r3d_convs(cfg: R3DCfg) -> List[ConvSpec]:
    """Every conv of the network in forward order (stem, then per block conv1, conv2, downsample)."""
    convs = [ConvSpec("stem.0", 4, 64, (3, 7, 7), (1, 2, 2), (1, 3, 3), cfg.num_channels)]
    cin = 64
    for li, (nb, w) in enumerate(zip(cfg.layers, cfg.widths)):
        for b in range(nb):
            s = 2 if (b == 0 and li > 0) else 1
            pre = f"layer{li + 1}.{b}."
            convs.append(ConvSpec(pre + "conv1.0", cin, w, (3, 3, 3), (s, s, s), (1, 1, 1), cin))
            convs.append(ConvSpec(pre + "conv2.0", w, w, (3, 3, 3), (1, 1, 1), (1, 1, 1), w))
            if s != 1 or cin != w:
                convs.append(ConvSpec(pre + "downsample.0", cin, w, (1, 1, 1), (s, s, s), (0, 0, 0), cin))
            cin = w
    return convs


def _bn_name(conv_name: str) -> str:
    return conv_name[:-2] + ".1"


class R3DLayout:
    """enc flat: per conv its weight [Co][kd][kh][kw][Ci] (channels-last), then its BN gamma, beta;
    head flat: enc_w [enc_out, 512], enc_b, dec_w [out_dim, enc_out], dec_b (the reference head)."""

    def __init__(self, cfg: R3DCfg, enc_out: int, out_dim: int):
        self.cfg, self.enc_out, self.out_dim = cfg, enc_out, out_dim
        self.convs = r3d_convs(cfg)
        e = FlatLayout()
        for c in self.convs:
            e.add(c.name + ".weight", (c.co,) + c.k + (c.ci,))
            bn = _bn_name(c.name)
            e.add(bn + ".weight", (c.co,))
            e.add(bn + ".bias", (c.co,))
        self.enc = e
        h = FlatLayout()
        feat = cfg.widths[-1]
        h.add("enc_w", (enc_out, feat))
        h.add("enc_b", (enc_out,))
        h.add("dec_w", (out_dim, enc_out))
        h.add("dec_b", (out_dim,))
        self.head = h
        # each conv unit's span of enc_flat (its weight, BN gamma and beta, padding included, up to the
        # next unit's first slot): the range the data-parallel exchange may reduce once that unit's
        # backward has run (the spans tile the buffer, so adjacent finished units coalesce)
        starts = [e.slots[c.name + ".weight"].offset for c in self.convs] + [e.numel]
        self.unit_span = {c.name: (starts[i], starts[i + 1]) for i, c in enumerate(self.convs)}
        # running statistics (buffers): [mean | var] per BN
        self.bn_off = {}
        off = 0
        for c in self.convs:
            self.bn_off[_bn_name(c.name)] = off
            off += 2 * c.co
        self.bn_numel = off


# ------------------------------------------------------------------------------------------------
# thin bindings of csrc/conv3d.hip (include/vspike.h "R3D-18 video encoder")
# ------------------------------------------------------------------------------------------------
def _desc(c: ConvSpec, N: int, D: int, H: int, W: int) -> L.Conv3dDesc:
    d = L.Conv3dDesc()
    d.N, d.Di, d.Hi, d.Wi, d.Ci = N, D, H, W, c.ci
    d.Do = (D + 2 * c.p[0] - c.k[0]) // c.s[0] + 1
    d.Ho = (H + 2 * c.p[1] - c.k[1]) // c.s[1] + 1
    d.Wo = (W + 2 * c.p[2] - c.k[2]) // c.s[2] + 1
    d.Co = c.co
    d.kd, d.kh, d.kw = c.k
    d.sd, d.sh, d.sw = c.s
    d.pd, d.ph, d.pw = c.p
    return d


def conv3d_fwd(d, x, w, y, stats=None):
    require_device(x, w, y)
    check(lib().vs_conv3d_fwd(ctypes.byref(d), x.data_ptr(), w.data_ptr(), y.data_ptr(),
                              None if stats is None else stats.data_ptr(), stream()), "vs_conv3d_fwd")


def conv3d_stats_rows(d) -> int:
    return int(lib().vs_conv3d_stats_rows(ctypes.byref(d)))


def conv3d_dx(d, dy, w, dx, accumulate=False):
    require_device(dy, w, dx)
    nb = int(lib().vs_conv3d_dx_workspace_bytes(ctypes.byref(d)))
    ws = torch.empty(nb // 4 + 64, dtype=torch.float32, device=dy.device)
    check(lib().vs_conv3d_dx(ctypes.byref(d), dy.data_ptr(), w.data_ptr(), dx.data_ptr(), int(accumulate),
                             ws.data_ptr(), ws.numel() * 4, stream()), "vs_conv3d_dx")


def conv3d_dw(d, x, dy, dw, accumulate=False):
    require_device(x, dy, dw)
    nb = int(lib().vs_conv3d_dw_workspace_bytes(ctypes.byref(d)))
    ws = torch.empty(nb // 4 + 64, dtype=torch.float32, device=dy.device)
    check(lib().vs_conv3d_dw(ctypes.byref(d), x.data_ptr(), dy.data_ptr(), dw.data_ptr(), int(accumulate),
                             ws.data_ptr(), ws.numel() * 4, stream()), "vs_conv3d_dw")


def bn3d_stats(part, rows, count, gamma, beta, eps, momentum, mean, rstd, scale, shift, rmean=None, rvar=None):
    C = gamma.numel()
    nb = int(lib().vs_bn3d_stats_workspace_bytes(rows, C))
    ws = torch.empty(nb // 4 + 64, dtype=torch.float32, device=part.device)
    check(lib().vs_bn3d_stats(rows, C, part.data_ptr(), count, gamma.data_ptr(), beta.data_ptr(), eps, momentum,
                              mean.data_ptr(), rstd.data_ptr(), scale.data_ptr(), shift.data_ptr(),
                              L.ptr(rmean), L.ptr(rvar), ws.data_ptr(), stream()), "vs_bn3d_stats")


def bn3d_apply(y, scale, shift, out, residual=None, relu=True):
    C = y.shape[-1]
    check(lib().vs_bn3d_apply(y.numel() // C, C, y.data_ptr(), scale.data_ptr(), shift.data_ptr(),
                              L.ptr(residual), int(relu), out.data_ptr(), stream()), "vs_bn3d_apply")


def bn3d_bwd(dout, out, relu, y, mean, rstd, gamma, dy, dres, dgamma, dbeta, batch_stats=True):
    """batch_stats: the forward normalised by the batch statistics (training mode); False: by the
    running statistics (eval mode), whose backward has no mean / variance terms."""
    C = y.shape[-1]
    M = y.numel() // C
    nb = int(lib().vs_bn3d_bwd_workspace_bytes(M, C))
    ws = torch.empty(nb // 4 + 64, dtype=torch.float32, device=y.device)
    fn = lib().vs_bn3d_bwd if batch_stats else lib().vs_bn3d_bwd_eval
    check(fn(M, C, dout.data_ptr(), L.ptr(out), int(relu), y.data_ptr(), mean.data_ptr(),
             rstd.data_ptr(), gamma.data_ptr(), dy.data_ptr(), L.ptr(dres), L.ptr(dgamma),
             L.ptr(dbeta), ws.data_ptr(), stream()), "vs_bn3d_bwd")


def to_channels_last(x, cp=4):
    """(B, T, C, H, W) -> channels-last (B, T, H, W, cp), channels C..cp-1 zero."""
    B, T, C, H, W = x.shape
    out = torch.empty(B, T, H, W, cp, dtype=torch.float32, device=x.device)
    check(lib().vs_to_channels_last(B, T, C, H, W, cp, x.data_ptr(), out.data_ptr(), stream()),
          "vs_to_channels_last")
    return out


def avgpool3d(x):
    N, C = x.shape[0], x.shape[-1]
    S = x.numel() // (N * C)
    out = torch.empty(N, C, dtype=torch.float32, device=x.device)
    check(lib().vs_avgpool3d(N, S, C, x.data_ptr(), out.data_ptr(), stream()), "vs_avgpool3d")
    return out


def avgpool3d_bwd(dpool, like):
    N, C = like.shape[0], like.shape[-1]
    S = like.numel() // (N * C)
    dx = torch.empty_like(like)
    check(lib().vs_avgpool3d_bwd(N, S, C, dpool.data_ptr(), dx.data_ptr(), stream()), "vs_avgpool3d_bwd")
    return dx


# ------------------------------------------------------------------------------------------------
# the plugin
# ------------------------------------------------------------------------------------------------
def _cfg_get(config, key, default=None):
    try:
        return config[key] if key in config else default
    except TypeError:
        return getattr(config, key, default)


class R3D(nn.Module):
    def __init__(self, config):
        super().__init__()
        self.backbone = R3DCfg.from_config(_cfg_get(config, "backbone"))
        cdt = str(_cfg_get(config, "compute_dtype", "fp32")).lower()
        if cdt not in ("fp32", "float32", "f32"):
            raise ValueError("R3D runs in fp32 (BASELINE C4's precision): compute_dtype must be fp32")
        self.freeze_encoder = bool(_cfg_get(config, "freeze_encoder", False))
        enc_out = int(config["encoder"]["output_dim"])
        out_dim = int(config["decoder"]["output_dim"])
        if out_dim % 100:
            raise ValueError("decoder.output_dim must be 100 * neurons (src/train.py:41)")
        if self.backbone.num_channels > 4:
            raise ValueError("R3D: at most 4 input channels (the stem input is padded to 4)")
        self.layout = R3DLayout(self.backbone, enc_out, out_dim)
        self.enc_flat = nn.Parameter(torch.zeros(self.layout.enc.numel), requires_grad=not self.freeze_encoder)
        self.head_flat = nn.Parameter(torch.zeros(self.layout.head.numel))
        self.register_buffer("bn_running", torch.zeros(self.layout.bn_numel))
        self.register_buffer("num_batches_tracked", torch.zeros((), dtype=torch.long))
        self.register_buffer("frame_indices", (torch.linspace(0, 1, self.backbone.num_frames) * 119).long(),
                             persistent=False)
        self.grad_sink = None
        # checker support: when True, every forward leaves its ReLU decisions in `relu_masks`
        # ({conv name: bool (N, D, H, W, C)}), so a parity check can condition its oracle on them
        # (oracle/cpu_ref.r3d18_forward relu_masks); off in training
        self.keep_relu_masks = False
        self.relu_masks = None
        self.reset_parameters()

    @torch.no_grad()
    def reset_parameters(self, generator: Optional[torch.Generator] = None):
        """torchvision VideoResNet init: kaiming_normal_(fan_out, relu) convs, BN (1, 0), running
        (0, 1); the head as nn.Linear's default (the reference head, src/model/videomae.py:13-14)."""
        lay = self.layout
        self.enc_flat.zero_()
        for c in lay.convs:
            w = lay.enc.view(self.enc_flat, c.name + ".weight")
            fan_out = c.co * c.k[0] * c.k[1] * c.k[2]
            w.normal_(0.0, math.sqrt(2.0 / fan_out), generator=generator)
            if c.ci != c.ci_ref:
                w[..., c.ci_ref:] = 0.0                   # the padded input channels
            lay.enc.view(self.enc_flat, _bn_name(c.name) + ".weight").fill_(1.0)
            off = lay.bn_off[_bn_name(c.name)]
            self.bn_running[off:off + c.co] = 0.0
            self.bn_running[off + c.co:off + 2 * c.co] = 1.0
        self.head_flat.zero_()
        for wname, bname in (("enc_w", "enc_b"), ("dec_w", "dec_b")):
            w = lay.head.view(self.head_flat, wname)
            bound = 1.0 / math.sqrt(w.shape[1])
            w.uniform_(-bound, bound, generator=generator)
            lay.head.view(self.head_flat, bname).uniform_(-bound, bound, generator=generator)

    # ---- reference-style state dict (torch layouts) -------------------------------------------
    def reference_state_dict(self):
        """torchvision r3d_18 names and layouts (conv weights [Co][Ci][kd][kh][kw]) + the head as
        `encoder.*` / `decoder.*`, and the BN running buffers."""
        lay, out = self.layout, {}
        enc = self.enc_flat.detach()
        for c in lay.convs:
            w = lay.enc.view(enc, c.name + ".weight")[..., :c.ci_ref]
            out[c.name + ".weight"] = w.permute(0, 4, 1, 2, 3).contiguous().clone()
            bn = _bn_name(c.name)
            out[bn + ".weight"] = lay.enc.view(enc, bn + ".weight").clone()
            out[bn + ".bias"] = lay.enc.view(enc, bn + ".bias").clone()
            off = lay.bn_off[bn]
            out[bn + ".running_mean"] = self.bn_running[off:off + c.co].clone()
            out[bn + ".running_var"] = self.bn_running[off + c.co:off + 2 * c.co].clone()
        head = self.head_flat.detach()
        for ref, slot in (("encoder.weight", "enc_w"), ("encoder.bias", "enc_b"), ("decoder.weight", "dec_w"),
                          ("decoder.bias", "dec_b")):
            out[ref] = lay.head.view(head, slot).clone()
        return out

    @torch.no_grad()
    def load_reference_state_dict(self, sd, strict: bool = True):
        lay = self.layout
        for c in lay.convs:
            key = c.name + ".weight"
            if key not in sd:
                if strict:
                    raise KeyError(f"missing {key}")
                continue
            w = torch.as_tensor(sd[key]).to(self.enc_flat.device, torch.float32)      # [Co][Ci][kd][kh][kw]
            dst = lay.enc.view(self.enc_flat, key)
            dst.zero_()
            dst[..., :c.ci_ref].copy_(w.permute(0, 2, 3, 4, 1))
            bn = _bn_name(c.name)
            for suf in (".weight", ".bias"):
                if bn + suf in sd:
                    lay.enc.view(self.enc_flat, bn + suf).copy_(torch.as_tensor(sd[bn + suf]))
                elif strict:
                    raise KeyError(f"missing {bn + suf}")
            off = lay.bn_off[bn]
            if bn + ".running_mean" in sd:
                self.bn_running[off:off + c.co].copy_(torch.as_tensor(sd[bn + ".running_mean"]))
                self.bn_running[off + c.co:off + 2 * c.co].copy_(torch.as_tensor(sd[bn + ".running_var"]))
        for ref, slot in (("encoder.weight", "enc_w"), ("encoder.bias", "enc_b"), ("decoder.weight", "dec_w"),
                          ("decoder.bias", "dec_b")):
            if ref in sd:
                lay.head.view(self.head_flat, slot).copy_(torch.as_tensor(sd[ref]))
            elif strict:
                raise KeyError(f"missing {ref}")

    # ---- forward ---------------------------------------------------------------------------------
    def preprocess(self, video: torch.Tensor) -> torch.Tensor:
        """Raw gray video (B, T, 1, H, W) -> pixel clips (B, num_frames, 3, S, S) on the device
        (the reference's VideoMAE preprocessing, src/model/videomae.py:18-25, at this encoder's size)."""
        cfg = self.backbone
        idx = (torch.linspace(0, 1, cfg.num_frames) * (video.shape[1] - 1)).long().tolist()
        return ops.video_preprocess(video, idx, cfg.image_size, (0.485, 0.456, 0.406), (0.229, 0.224, 0.225))

    def forward(self, inputs: torch.Tensor) -> torch.Tensor:
        cfg = self.backbone
        if inputs.dim() != 5:
            raise ValueError("R3D expects a 5-D tensor")
        L.require_device(inputs)
        shape = (cfg.num_frames, cfg.num_channels, cfg.image_size, cfg.image_size)
        if tuple(inputs.shape[1:]) != shape:
            if inputs.shape[2] != 1 or inputs.shape[3] != inputs.shape[4]:
                raise ValueError(f"expected pixel clips (B, {', '.join(map(str, shape))}) or raw gray video "
                                 "(B, T, 1, H, H)")
            with torch.no_grad():
                inputs = self.preprocess(inputs.detach())
        pixels = inputs.detach().to(torch.float32).contiguous()
        return _R3DFn.apply(pixels, self.enc_flat, self.head_flat, self)

    def _bn(self, c: ConvSpec, which: str):
        return self.layout.enc.view(self.enc_flat.detach(), _bn_name(c.name) + which)

    def _unit_fwd(self, c: ConvSpec, x, shape, residual, relu, save):
        """y = conv(x); out = [relu](bn(y) [+ residual]).  Returns (out, out_shape)."""
        N, D, H, W = shape
        d = _desc(c, N, D, H, W)
        dev = x.device
        y = torch.empty(N, d.Do, d.Ho, d.Wo, c.co, dtype=torch.float32, device=dev)
        w = self.layout.enc.view(self.enc_flat.detach(), c.name + ".weight")
        mean = torch.empty(c.co, dtype=torch.float32, device=dev)
        rstd, scale, shift = torch.empty_like(mean), torch.empty_like(mean), torch.empty_like(mean)
        gamma, beta = self._bn(c, ".weight"), self._bn(c, ".bias")
        off = self.layout.bn_off[_bn_name(c.name)]
        rm, rv = self.bn_running[off:off + c.co], self.bn_running[off + c.co:off + 2 * c.co]
        if self.training:
            rows = conv3d_stats_rows(d)
            stats = torch.empty(rows, 2, c.co, dtype=torch.float32, device=dev)
            conv3d_fwd(d, x, w, y, stats)
            bn3d_stats(stats, rows, N * d.Do * d.Ho * d.Wo, gamma, beta, self.backbone.bn_eps,
                       self.backbone.bn_momentum, mean, rstd, scale, shift, rm, rv)
        else:   # running statistics (nn.BatchNorm3d.eval())
            conv3d_fwd(d, x, w, y)
            torch.rsqrt(rv + self.backbone.bn_eps, out=rstd)
            mean.copy_(rm)
            torch.mul(gamma, rstd, out=scale)
            torch.sub(beta, mean * scale, out=shift)
        out = torch.empty_like(y)
        bn3d_apply(y, scale, shift, out, residual=residual, relu=relu)
        if relu and self.keep_relu_masks:
            self.relu_masks[c.name] = out > 0
        if save is not None:
            save[c.name] = {"x": x, "y": y, "out": out, "mean": mean, "rstd": rstd, "shape": shape, "d": d,
                            "relu": relu, "batch_stats": bool(self.training)}
        return out, (N, d.Do, d.Ho, d.Wo)

    def _run_forward(self, pixels, save_encoder: bool):
        cfg = self.backbone
        B = pixels.shape[0]
        lay = self.layout
        save = {} if save_encoder else None
        if self.keep_relu_masks:
            self.relu_masks = {}
        x = to_channels_last(pixels.view(B, cfg.num_frames, cfg.num_channels, cfg.image_size, cfg.image_size), 4)
        shape = (B, cfg.num_frames, cfg.image_size, cfg.image_size)
        convs = {c.name: c for c in lay.convs}
        x, shape = self._unit_fwd(convs["stem.0"], x, shape, None, True, save)
        for li, nb in enumerate(cfg.layers):
            for b in range(nb):
                pre = f"layer{li + 1}.{b}."
                h, hshape = self._unit_fwd(convs[pre + "conv1.0"], x, shape, None, True, save)
                if pre + "downsample.0" in convs:
                    sc, _ = self._unit_fwd(convs[pre + "downsample.0"], x, shape, None, False, save)
                else:
                    sc = x
                x, shape = self._unit_fwd(convs[pre + "conv2.0"], h, hshape, sc, True, save)
        if self.training:
            self.num_batches_tracked += 1
        feat = avgpool3d(x)                                   # (B, 512)
        head32 = self.head_flat.detach()
        z = torch.empty(B, lay.enc_out, dtype=torch.float32, device=pixels.device)
        ops.linear(feat, lay.head.view(head32, "enc_w"), z, bias=lay.head.view(head32, "enc_b"))
        r = torch.empty(B, lay.out_dim, dtype=torch.float32, device=pixels.device)
        ops.linear(z, lay.head.view(head32, "dec_w"), r, bias=lay.head.view(head32, "dec_b"))
        st = {"save": save, "feat": feat, "z": z, "x_last": x, "B": B}
        return r.view(B, 100, -1), st

    # ---- backward --------------------------------------------------------------------------------
    def _grad_buffer(self, p):
        if self.grad_sink is not None:
            return self.grad_sink.grad_buffer(p)
        return torch.zeros_like(p)

    def _unit_bwd(self, c: ConvSpec, s, dout, g_enc, dres=None, want_dx=True, dx=None, dx_accumulate=False):
        """Backward of out = [relu](bn(conv(x)) [+ res]): BN' (dgamma, dbeta), conv dW, conv dX.
        dres: buffer for the residual's gradient (g, the masked dout).  Returns dx."""
        lay = self.layout
        G = lambda n: lay.enc.view(g_enc, n)  # noqa: E731
        bn = _bn_name(c.name)
        dy = torch.empty_like(s["y"])
        bn3d_bwd(dout, s["out"], s["relu"], s["y"], s["mean"], s["rstd"], self._bn(c, ".weight"), dy, dres,
                 G(bn + ".weight"), G(bn + ".bias"), batch_stats=s["batch_stats"])
        conv3d_dw(s["d"], s["x"], dy, G(c.name + ".weight"), accumulate=False)
        if self.grad_sink is not None:      # this unit's weight / gamma / beta gradients are final
            self.grad_sink.mark_ready(self.enc_flat, *lay.unit_span[c.name])
        if not want_dx:
            return None
        if dx is None:
            dx = torch.empty_like(s["x"])
        w = lay.enc.view(self.enc_flat.detach(), c.name + ".weight")
        conv3d_dx(s["d"], dy, w, dx, accumulate=dx_accumulate)
        return dx

    def _run_backward(self, st, d_logrates, want_enc: bool, want_head: bool):
        lay = self.layout
        B = st["B"]
        head32 = self.head_flat.detach()
        dr = d_logrates.reshape(B, lay.out_dim).to(torch.float32).contiguous()
        # dZ = dr dec_w reduces over K = 100 * neurons (25,600 at C4) for 16 x 64 outputs: split-K with the
        # partials summed in a fixed order (as the ViT head); one 128 x 64 tile walking K alone was
        # 869 us per step (profiles/r05_r3d_kernel_stats_bn.txt, gemm_f32_kernel<true, false>)
        dz = torch.zeros(B, lay.enc_out, dtype=torch.float32, device=dr.device)
        dz_ws = torch.empty(max(ops.splitk_workspace_bytes(torch.float32, B, lay.enc_out, lay.out_dim), 16) // 4 + 64,
                            dtype=torch.float32, device=dr.device)
        ops.linear_dx(dr, lay.head.view(head32, "dec_w"), dz, accumulate=True, workspace=dz_ws)
        g_head = None
        if want_head:
            g_head = self._grad_buffer(self.head_flat)
            Gh = lambda n: lay.head.view(g_head, n)  # noqa: E731
            ops.linear_dw(dr, st["z"], Gh("dec_w"), db=Gh("dec_b"), accumulate=False)
            ops.linear_dw(dz, st["feat"], Gh("enc_w"), db=Gh("enc_b"), accumulate=False)
            if self.grad_sink is not None:
                self.grad_sink.mark_ready(self.head_flat, 0, self.head_flat.numel())
        if not want_enc:
            return None, g_head
        dfeat = torch.empty(B, lay.cfg.widths[-1], dtype=torch.float32, device=dr.device)
        ops.linear_dx(dz, lay.head.view(head32, "enc_w"), dfeat)
        g_enc = self._grad_buffer(self.enc_flat)
        save = st["save"]
        convs = {c.name: c for c in lay.convs}
        d = avgpool3d_bwd(dfeat, st["x_last"])                # gradient of the last block's output
        cfg = self.backbone
        for li in reversed(range(len(cfg.layers))):
            for b in reversed(range(cfg.layers[li])):
                pre = f"layer{li + 1}.{b}."
                c2, c1 = convs[pre + "conv2.0"], convs[pre + "conv1.0"]
                ds = convs.get(pre + "downsample.0")
                s2, s1 = save[c2.name], save[c1.name]
                dres = torch.empty_like(d)                   # the shortcut's gradient g
                dh = self._unit_bwd(c2, s2, d, g_enc, dres=dres)
                if ds is not None:
                    dx = self._unit_bwd(ds, save[ds.name], dres, g_enc)          # overwrites every element
                else:
                    dx = dres                                                     # identity shortcut
                d = self._unit_bwd(c1, s1, dh, g_enc, dx=dx, dx_accumulate=True)
        self._unit_bwd(convs["stem.0"], save["stem.0"], d, g_enc, want_dx=False)
        # (every unit marked its span ready as its backward finished, in reverse order: the exchange
        # all-reduces each >= bucket-sized run of finished spans while the earlier units' backward runs,
        # as DDP's reducer does for src/trainer/base.py:150's accelerator.backward)
        return g_enc, g_head


class _R3DFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pixels, enc_flat, head_flat, mod):
        want_enc = bool(ctx.needs_input_grad[1])
        out, st = mod._run_forward(pixels, save_encoder=want_enc)
        ctx.want = (want_enc, bool(ctx.needs_input_grad[2]))
        ctx.mod, ctx.st = mod, (st if any(ctx.want) else None)
        return out

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, grad):
        mod = ctx.mod
        g_enc, g_head = mod._run_backward(ctx.st, grad, *ctx.want)
        ctx.st = None
        sink = mod.grad_sink
        if sink is not None and hasattr(sink, "end_backward"):
            sink.end_backward()
        if sink is not None and not getattr(sink, "return_grads", False):
            return None, None, None, None
        return None, g_enc, g_head, None
