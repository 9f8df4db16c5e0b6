"""VideoMAE plugin — drop-in for the reference's `src/model/videomae.py:4-36` (NAME2MODEL['VideoMAE']).

Reference behaviour kept:
  * constructor `VideoMAE(config.model)` with `encoder.output_dim` / `decoder.output_dim`
    (videomae.py:13-14; decoder.output_dim = 100 * neurons injected by src/train.py:41);
  * `forward(x) -> log-rates (B, 100, N)` (videomae.py:31); consumed by
    PoissonNLLLoss(log_input=True) (src/train.py:59);
  * the encoder is frozen by default (videomae.py:12,17,34-36) — `freeze_encoder: false`
    trains it (north-star mode); ViT geometry from an optional `backbone:` section, default
    videomae-base (ViT-B/16, tubelet 2, 1568 tokens).
MI355X design: parameters live in two flat f32 buffers (layout.py); every op runs in libvspike
(im2col + patch GEMM with the sinusoid table fused in its epilogue, 12 native block executors,
split-K head GEMM) and the whole backward is hand-sequenced here (no autograd graph inside).
`compute_dtype: bf16` runs activations/weights in bf16 with f32 accumulation, f32 residual stream,
f32 master weights and f32 weight gradients.
"""
from __future__ import annotations

import math
import os
import weakref
from typing import Optional

import torch
from torch import nn

from . import _lib as L
from . import ops
from .layout import BackboneCfg, VitLayout, modern_name
from .memory import Arena
from .optim import lp_key, register_lp_shadow

# Side-stream joins of the block backward.  A join at every block end costs a ~24 us cross-queue
# stall per block (the main stream waits on the dWqkv product, which the side stream finishes last).
# Deferring every product (VS_BWD_DEFER_JOIN, VSPIKE_DEFER=1) removes the stall but lets the dW
# products spill into the next block's kernels (6.61 ms/step); deferring only dWqkv
# (VS_BWD_DEFER_LAST, the default) keeps the other three joined: 6.33 vs 6.41 ms/step for
# join-every-block (VSPIKE_DEFER=0), same box, 3 round-robin runs of 30 steps (scripts/ab_env.sh).
_DEFER = {"0": 0, "1": 1, "last": 2}.get(os.environ.get("VSPIKE_DEFER", "last"), 2)
# VSPIKE_SIDE=0: no side stream (every dW product in order on the main stream), for A/B runs
_SIDE = os.environ.get("VSPIKE_SIDE", "1") != "0"
# VS_BWD_FUSE_LN (the dX products fused with the LayerNorm backwards, see vspike.h): on by default from
# _LN_FUSE_ROWS token rows (128 clips: 33.97 -> 33.70 ms/step, profiles/r03_v5_ab_b128_knobs.txt), off
# below (16 clips: 90 us/step slower beside the side-stream dW products);
# VSPIKE_LN_FUSE=1 / 0 forces it either way
_LN_FUSE = {"1": True, "0": False}.get(os.environ.get("VSPIKE_LN_FUSE", ""), None)
_LN_FUSE_ROWS = 65536
# The fused MLP (vs_mlp_fwd / vs_mlp_bwd_da: the 4x-wide intermediate never stored, the backward
# recomputes the pre-activation) wherever the shape allows it (bf16, D = 192); VSPIKE_MLP_FUSE=0 keeps
# the two-GEMM MLP with the stored gelu / gelu' pair (A/B)
_MLP_FUSE = os.environ.get("VSPIKE_MLP_FUSE", "1") != "0"
# ... with block i+1's LayerNorm1 computed in block i's fused MLP epilogue (VSPIKE_LN_CHAIN=0: off, A/B)
_LN_CHAIN = os.environ.get("VSPIKE_LN_CHAIN", "1") != "0"

_DTYPES = {"fp32": torch.float32, "float32": torch.float32, "f32": torch.float32,
           "bf16": torch.bfloat16, "bfloat16": torch.bfloat16,
           # BASELINE C5: the bf16 block with its four Linear forwards on MX-FP8 (vs_gemm_mxfp8)
           "fp8": torch.bfloat16, "mxfp8": torch.bfloat16}


class _FwdState(dict):
    """What one forward saves for its backward; the cached buffers it names stay reserved while
    an instance is alive (VideoMAE._fwd_buffers holds a weak reference)."""


def _dev_key(dev) -> str:
    """Canonical per-device cache key ('cuda' and 'cuda:0' are the same device)."""
    d = torch.device(dev)
    if d.type == "cuda" and d.index is None:
        d = torch.device("cuda", torch.cuda.current_device())
    return str(d)


def _cfg_get(config, key, default=None):
    try:
        return config[key] if key in config else default
    except TypeError:
        return getattr(config, key, default)


class VideoMAE(nn.Module):
    def __init__(self, config):
        super().__init__()
        self.backbone = BackboneCfg.from_config(_cfg_get(config, "backbone"))
        self.freeze_encoder = bool(_cfg_get(config, "freeze_encoder", True))
        cdt = str(_cfg_get(config, "compute_dtype", "fp32")).lower()
        self.compute_dtype = _DTYPES[cdt]
        self.fp8 = cdt in ("fp8", "mxfp8")
        enc_out = int(config["encoder"]["output_dim"])
        out_dim = int(config["decoder"]["output_dim"])
        if out_dim % 100:
            raise ValueError("decoder.output_dim must be 100 * neurons (src/train.py:41)")
        cfg = self.backbone
        if cfg.hidden_size != 64 * cfg.num_attention_heads:
            raise ValueError("this build supports head dim 64 (hidden_size = 64 * num_attention_heads)")
        if self.fp8 and (cfg.hidden_size % 128 or cfg.intermediate_size % 128):
            raise ValueError("compute_dtype fp8 (MX-FP8 block products) needs hidden_size and intermediate_size "
                             "multiples of 128 (e.g. videomae-base)")
        self.layout = VitLayout(cfg, enc_out, out_dim)
        self.enc_flat = nn.Parameter(torch.zeros(self.layout.enc.numel), requires_grad=not self.freeze_encoder)
        self.head_flat = nn.Parameter(torch.zeros(self.layout.head.numel))
        # raw-video path (videomae.py:10-11, 18-25): uniform num_frames-of-T frame selection, then
        # the HF image processor's resize/normalise as one device kernel (vs_video_preprocess).
        # mean/std: the Hub preprocessor_config of videomae-base cannot be fetched here; default =
        # ImageNet's, the values its pretraining head un-normalises with (modeling_videomae.py:890-891)
        self.register_buffer("frame_indices", (torch.linspace(0, 1, cfg.num_frames) * 119).long(), persistent=False)
        pp = _cfg_get(config, "preprocess", None) or {}
        self.pp_mean = tuple(float(v) for v in (pp.get("mean") if hasattr(pp, "get") and pp.get("mean") else
                                                (0.485, 0.456, 0.406)))
        self.pp_std = tuple(float(v) for v in (pp.get("std") if hasattr(pp, "get") and pp.get("std") else
                                               (0.229, 0.224, 0.225)))
        self.grad_sink = None          # set by vspike.dp.GradExchange for overlapped all-reduce
        self._pos_cache = {}
        self.reset_parameters()

    # ---------------------------------------------------------------------------------------
    # parameters
    # ---------------------------------------------------------------------------------------
    @torch.no_grad()
    def reset_parameters(self, generator: Optional[torch.Generator] = None):
        """HF VideoMAE `_init_weights` for the encoder (modeling_videomae.py:512-522): N(0, 0.02)
        weights, zero biases, LayerNorm (1, 0); nn.Linear default init for the head."""
        enc, head, lay = self.enc_flat, self.head_flat, self.layout
        enc.zero_()
        for name, slot in lay.enc.slots.items():
            v = lay.enc.view(enc, name)
            if name.endswith(("ln1_g", "ln2_g")):
                v.fill_(1.0)
            elif len(slot.shape) == 2:
                v.normal_(0.0, 0.02, generator=generator)
        head.zero_()
        for wname, bname in (("enc_w", "enc_b"), ("dec_w", "dec_b")):
            w = lay.head.view(head, wname)
            bound = 1.0 / math.sqrt(w.shape[1])
            w.uniform_(-bound, bound, generator=generator)
            lay.head.view(head, bname).uniform_(-bound, bound, generator=generator)

    def _flat(self, which):
        return self.enc_flat if which == "enc" else self.head_flat

    def _flat_layout(self, which):
        return self.layout.enc if which == "enc" else self.layout.head

    def reference_state_dict(self, modern_names: bool = False):
        """Parameters under the reference plugin's names (HF VideoMAEModel + two Linears): the
        transformers 4.38 spelling the reference pins (`...attention.attention.q_bias` / `v_bias`),
        or with `modern_names` the newer `query.bias` / `value.bias`."""
        out = {}
        for name, which, slot, rows in self.layout.hf_items():
            t = self._flat_layout(which).view(self._flat(which).detach(), slot)
            if slot == "patch_w":
                t = t.view(self.backbone.hidden_size, self.backbone.num_channels, self.backbone.tubelet_size,
                           self.backbone.patch_size, self.backbone.patch_size)
            out[modern_name(name) if modern_names else name] = (t if rows is None else t[rows]).clone()
        return out

    @torch.no_grad()
    def load_reference_state_dict(self, sd, strict: bool = True):
        """Load reference-named weights (e.g. a videomae-base checkpoint + head, or a reference
        `model_best.pt` state_dict).  Q/V biases are accepted under the 4.38 names the reference
        pins (`q_bias` / `v_bias`, modeling_videomae.py:216-218) or the newer `query.bias` /
        `value.bias`; a newer version's `key.bias` must be zero (4.38 has none: :233)."""
        seen = set()
        for name, which, slot, rows in self.layout.hf_items():
            key = name if name in sd else modern_name(name)
            if key not in sd:
                if strict:
                    raise KeyError(f"missing {name}")
                continue
            dst = self._flat_layout(which).view(self._flat(which), slot)
            src = torch.as_tensor(sd[key]).to(dst.device, torch.float32).reshape(
                dst[rows].shape if rows is not None else dst.shape)
            (dst[rows] if rows is not None else dst).copy_(src)
            seen.add(key)
        for k, v in sd.items():
            if k.endswith("attention.attention.key.bias"):
                if torch.as_tensor(v).abs().max() != 0:
                    raise ValueError(f"{k} is non-zero; the reference encoder has no key bias")
                seen.add(k)
        if strict:
            extra = set(sd) - seen
            if extra:
                raise KeyError(f"unexpected keys: {sorted(extra)[:5]}")

    # ---------------------------------------------------------------------------------------
    # forward
    # ---------------------------------------------------------------------------------------
    def raw_frame_indices(self, n_source: int):
        """videomae.py:10-11 (written for 120 source frames: linspace(0, 1, 16) * 119)."""
        return (torch.linspace(0, 1, self.backbone.num_frames) * (n_source - 1)).long().tolist()

    def preprocess(self, video: torch.Tensor) -> torch.Tensor:
        """Raw gray video (B, T, 1, H, W) (float 0..255 or uint8) -> pixel_values on the device."""
        cfg = self.backbone
        return ops.video_preprocess(video, self.raw_frame_indices(video.shape[1]), cfg.image_size, self.pp_mean,
                                    self.pp_std)

    def forward(self, inputs: torch.Tensor) -> torch.Tensor:
        cfg = self.backbone
        if inputs.dim() != 5:
            raise ValueError("VideoMAE expects a 5-D tensor")
        L.require_device(inputs)
        pixel_shape = (cfg.num_frames, cfg.num_channels, cfg.image_size, cfg.image_size)
        if tuple(inputs.shape[1:]) != pixel_shape:
            if inputs.shape[2] != 1 or inputs.shape[3] != inputs.shape[4]:
                raise ValueError(f"expected pixel_values (B, {', '.join(map(str, pixel_shape))}) or raw gray video "
                                 "(B, T, 1, H, H) as the reference's loader yields (videomae.py:18-25)")
            with torch.no_grad():
                inputs = self.preprocess(inputs.detach())
        pixels = inputs.detach().to(torch.float32).contiguous()
        return _VideoMAEFn.apply(pixels, self.enc_flat, self.head_flat, self)

    def _pos_table(self, device):
        key = _dev_key(device)
        if key not in self._pos_cache:
            self._pos_cache[key] = ops.sinusoid_table(self.backbone.num_tokens, self.backbone.hidden_size, device)
        return self._pos_cache[key]

    def __getstate__(self):
        st = super().__getstate__() if hasattr(super(), "__getstate__") else self.__dict__.copy()
        st = dict(st)
        st["_pos_cache"] = {}
        for k in ("_fwd_cache", "_bwd_cache", "_gs_cache", "_chains", "_lp"):
            st.pop(k, None)
        st["grad_sink"] = None
        return st

    def _mlp_fused(self, B: int) -> bool:
        cfg = self.backbone
        return (_MLP_FUSE and self.compute_dtype == torch.bfloat16 and not self.fp8 and
                ops.mlp_fused_ok(B * cfg.num_tokens, cfg.hidden_size, cfg.intermediate_size))

    # activation buffers of one block (names match VitLayer fields)
    def _plan_layer(self, ar: Arena, pfx: str, B: int):
        cfg, dt = self.backbone, self.compute_dtype
        N, D, F, H = cfg.num_tokens, cfg.hidden_size, cfg.intermediate_size, cfg.num_attention_heads
        M = B * N
        mlp = () if self._mlp_fused(B) else (("a_pre", (M, F), dt), ("a_act", (M, F), dt))
        for name, shape, d in (("h1", (M, D), dt), ("mean1", (M,), torch.float32), ("rstd1", (M,), torch.float32),
                               ("qkv", (M, 3 * D), dt), ("attn_o", (M, D), dt), ("lse", (B, H, N), torch.float32),
                               ("y", (M, D), torch.float32), ("h2", (M, D), dt), ("mean2", (M,), torch.float32),
                               ("rstd2", (M,), torch.float32)) + mlp:
            ar.add(pfx + name, shape, d)

    def _layer_struct(self, i, B, x_in, x_out, act, pfx, w_lp, w32):
        cfg = self.backbone
        lay = self.layout.enc
        s = L.VitLayer()
        s.dtype = L.VS_FP8 if self.fp8 else L.dtype_code(self.compute_dtype)
        s.heads = cfg.num_attention_heads
        s.batch, s.tokens, s.hidden, s.mlp = B, cfg.num_tokens, cfg.hidden_size, cfg.intermediate_size
        s.ln_eps = cfg.layer_norm_eps
        s.attn_scale = 1.0 / math.sqrt(64.0)
        for k in ("ln1_g", "ln1_b", "ln2_g", "ln2_b", "b_qkv", "b_proj", "b_fc1", "b_fc2"):
            setattr(s, k, lay.view(w32, f"{i}.{k}").data_ptr())
        for k in ("w_qkv", "w_proj", "w_fc1", "w_fc2"):
            setattr(s, k, lay.view(w_lp, f"{i}.{k}").data_ptr())
        s.x_in, s.x_out = x_in.data_ptr(), x_out.data_ptr()
        for k in ("h1", "mean1", "rstd1", "qkv", "attn_o", "lse", "y", "h2", "mean2", "rstd2"):
            setattr(s, k, act[pfx + k].data_ptr())
        if self._mlp_fused(B):   # fused MLP: a_pre NULL, a_act = the backward's shared gelu(pre) scratch
            s.a_pre, s.a_act = None, act["mlp_a"].data_ptr()
        else:
            s.a_pre, s.a_act = act[pfx + "a_pre"].data_ptr(), act[pfx + "a_act"].data_ptr()
        if self.fp8:
            s.fp8_ws, s.fp8_ws_bytes = act["fp8_ws"].data_ptr(), act["fp8_ws"].numel()
        return s

    def set_side_stream(self, enabled: bool) -> None:
        """Run the weight-gradient products on the side stream (default, overlapped with the next
        products of the backward) or in order on the main stream (VSPIKE_SIDE=0 for the whole
        process).  bench.py's instrumented pass uses the latter so every launch is timed alone."""
        self.__dict__["_side"] = bool(enabled)
        self._caches()[2].clear()

    def _caches(self):
        d = self.__dict__
        for k in ("_fwd_cache", "_bwd_cache", "_gs_cache", "_chains", "_lp"):
            if k not in d:
                d[k] = {}
        return d["_fwd_cache"], d["_bwd_cache"], d["_gs_cache"]

    def _lp_shadows(self, dev):
        """Persistent bf16 shadows of the two flat parameter buffers on `dev` (one per device, shared
        by every cached forward arena), registered with FusedAdamW so the optimizer step rewrites
        them.  NB: an optimizer step between a forward and ITS backward would change the weights the
        backward uses (the reference's loop never does that: base.py:144-159)."""
        self._caches()
        sh = self.__dict__["_lp"]
        key = _dev_key(dev)
        if key not in sh:
            dt = self.compute_dtype
            ent = {}
            for name, p in (("enc", self.enc_flat), ("head", self.head_flat)):
                t = torch.empty(p.numel(), dtype=dt, device=dev)
                stamp = {}
                register_lp_shadow(p, t, stamp)
                ent[name] = (t, stamp)
            sh[key] = ent
        return sh[key]

    def invalidate_lp(self):
        """Force the next forward to re-cast the bf16 shadows (after writing parameters through
        `.data`, which torch does not version)."""
        for ent in self.__dict__.get("_lp", {}).values():
            for _, stamp in ent.values():
                stamp.clear()

    def _chain(self, dev):
        """This model's vs_bwd_chain on `dev`: the side stream and deferred-join state of its
        block backwards (one backward sequence of a model runs at a time, as its scratch is
        shared too)."""
        self._caches()
        chains = self.__dict__["_chains"]
        key = _dev_key(dev)
        if key not in chains:
            with torch.cuda.device(dev):
                chains[key] = L.BwdChain()
        return chains[key]

    def _fwd_buffers(self, B: int, dev, save_encoder: bool):
        """Activation arena, low-precision weight shadows and the 12 executor structs of one
        (batch, device, save_encoder) shape: planned once, then reused every step while no live
        autograd state holds them (a second forward before the first one's backward builds a
        private set).  Rebuilding per step cost ~1.2 ms of host time with the GPU idle."""
        fwd_cache, _, _ = self._caches()
        enc32, head32 = self.enc_flat.detach(), self.head_flat.detach()
        sig = (enc32.data_ptr(), head32.data_ptr())
        key = (B, _dev_key(dev), save_encoder, self.compute_dtype)
        ent = fwd_cache.get(key)
        if ent is not None and ent["sig"] == sig and (ent["owner"] is None or ent["owner"]() is None):
            return ent
        cfg, dt = self.backbone, self.compute_dtype
        N, D, Lyr = cfg.num_tokens, cfg.hidden_size, cfg.num_hidden_layers
        M = B * N
        lp = dt != torch.float32
        ar = Arena()
        # patch embedding: the fused gather GEMM (49.9 us vs 61.8 us for im2col + GEMM at C2,
        # profiles/r03_v2_microbench_patch.txt); when the encoder trains, its weight gradient gathers
        # the pixels again in its own operand load (vs_patch_embed_dw), so no cols tensor exists in
        # bf16 at all.  fp32 (and shapes outside the fused kernels) keep im2col + GEMM.
        fused = ops.patch_embed_fused_ok(cfg, dt) and (not save_encoder or ops.patch_dw_ok(cfg, dt))
        if not fused:
            ar.add("cols", (M, cfg.patch_dim), dt)
        ar.add("x0", (M, D), torch.float32)
        for j in range(Lyr if save_encoder else 1):
            self._plan_layer(ar, f"L{j}.", B)
        if self._mlp_fused(B):   # gelu(pre) of the layer being back-propagated (written by its backward)
            ar.add("mlp_a", (M, cfg.intermediate_size), dt)
        if self.fp8:             # MX-FP8 operands + scales of the product being run (shared by the layers)
            ar.add("fp8_ws", (int(L.lib().vs_vit_fp8_workspace_bytes(M, D, cfg.intermediate_size)),), torch.uint8)
        for j in range(Lyr if save_encoder else 2):
            ar.add(f"X{j}", (M, D), torch.float32)
        if lp:
            ar.add("x_lp", (B, N * D), dt)
        ar.add("z", (B, self.layout.enc_out), torch.float32)
        # split-K over the N*D = 301,056-long reduction; partials summed in order (deterministic)
        hws = ops.splitk_workspace_bytes(dt, B, self.layout.enc_out, N * D)
        if hws:
            ar.add("head_ws", (hws // 4 + 4,), torch.float32)
        act = ar.allocate(dev)
        if lp:
            enc_lp, head_lp = self._lp_shadows(dev)["enc"][0], self._lp_shadows(dev)["head"][0]
        else:
            enc_lp, head_lp = enc32, head32
        x = act["x0"]
        structs = []
        for i in range(Lyr):
            j = i if save_encoder else 0
            x_out = act[f"X{i}"] if save_encoder else act[f"X{i % 2}"]
            structs.append(self._layer_struct(i, B, x, x_out, act, f"L{j}.", enc_lp, enc32))
            x = x_out
        if self._mlp_fused(B) and _LN_CHAIN:
            # block i's fused MLP epilogue runs block i+1's LayerNorm1 (its h1 / mean1 / rstd1)
            lay = self.layout.enc
            for i in range(Lyr - 1):
                s, t = structs[i], structs[i + 1]
                s.next_ln_g, s.next_ln_b = lay.view(enc32, f"{i + 1}.ln1_g").data_ptr(), lay.view(enc32, f"{i + 1}.ln1_b").data_ptr()
                s.next_h1, s.next_mean1, s.next_rstd1 = t.h1, t.mean1, t.rstd1
                t.ln1_ready = 1
        new = {"act": act, "structs": structs, "enc_lp": enc_lp, "head_lp": head_lp, "x_final": x, "fused": fused,
               "x_flat_lp": act["x_lp"] if lp else x.view(B, N * D), "head_ws": act.get("head_ws"),
               "sig": sig, "owner": None}
        if ent is None or ent["sig"] != sig:
            fwd_cache[key] = new
        return new

    def _run_forward(self, pixels, save_encoder: bool):
        cfg, dt = self.backbone, self.compute_dtype
        B = pixels.shape[0]
        N, D = cfg.num_tokens, cfg.hidden_size
        dev = pixels.device
        enc32, head32 = self.enc_flat.detach(), self.head_flat.detach()
        le, lh = self.layout.enc, self.layout.head
        ent = self._fwd_buffers(B, dev, save_encoder)
        act, enc_lp, head_lp = ent["act"], ent["enc_lp"], ent["head_lp"]
        if dt != torch.float32:
            # bf16 shadows: FusedAdamW rewrites them with each update (vs_adamw param_lp); cast only
            # when the master weights changed some other way (load, init, a user's in-place write)
            sh = self._lp_shadows(dev)
            for p, (shadow, stamp) in ((self.enc_flat, sh["enc"]), (self.head_flat, sh["head"])):
                if stamp.get("key") != lp_key(p):
                    ops.cast(p.detach(), shadow)
                    stamp["key"] = lp_key(p)

        if ent["fused"]:   # tubelet gather inside the GEMM's operand load (no im2col pass)
            ops.patch_embed_fwd(pixels, le.view(enc_lp, "patch_w"), le.view(enc32, "patch_b"), self._pos_table(dev),
                                act["x0"], cfg.tubelet_size, cfg.patch_size, cols=act.get("cols"))
        else:
            ops.patch_im2col(pixels, act["cols"], cfg.tubelet_size, cfg.patch_size)
            ops.linear(act["cols"], le.view(enc_lp, "patch_w"), act["x0"], bias=le.view(enc32, "patch_b"),
                       epilogue=L.EPI_POS, pos=self._pos_table(dev), pos_rows=N)
        for s in ent["structs"]:
            ops.vit_layer_fwd(s)
        x_flat_lp = ent["x_flat_lp"]
        if dt != torch.float32:
            ops.cast(ent["x_final"].view(B, N * D), x_flat_lp)
        z = act["z"]
        r = torch.empty(B, self.layout.out_dim, dtype=torch.float32, device=dev)   # handed to the caller
        z.zero_()
        ops.gemm(x_flat_lp, lh.view(head_lp, "enc_w"), z, M=B, N=self.layout.enc_out, K=N * D, a_kcontig=True,
                 b_kcontig=True, lda=N * D, ldb=N * D, ldc=self.layout.enc_out, epilogue=L.EPI_ATOMIC | L.EPI_BIAS,
                 bias=lh.view(head32, "enc_b"), workspace=ent["head_ws"])
        ops.linear(z, lh.view(head32, "dec_w"), r, bias=lh.view(head32, "dec_b"))
        state = _FwdState(act=act, structs=ent["structs"], enc_lp=enc_lp, head_lp=head_lp, x_flat_lp=x_flat_lp,
                          x_final=ent["x_final"], B=B, pixels=pixels if "cols" not in act else None,
                          pixels_version=pixels._version)
        ent["owner"] = weakref.ref(state)
        return r.view(B, 100, -1), state

    # ---------------------------------------------------------------------------------------
    # backward
    # ---------------------------------------------------------------------------------------
    def _grad_buffer(self, p):
        if self.grad_sink is not None:
            return self.grad_sink.grad_buffer(p)
        return torch.zeros_like(p)

    def _ready(self, p, lo, hi):
        if self.grad_sink is not None:
            self.grad_sink.mark_ready(p, lo, hi)

    def _run_backward(self, st, d_logrates, want_enc: bool, want_head: bool):
        cfg, dt = self.backbone, self.compute_dtype
        B = st["B"]
        N, D, F, Lyr = cfg.num_tokens, cfg.hidden_size, cfg.intermediate_size, cfg.num_hidden_layers
        H = cfg.num_attention_heads
        M = B * N
        lay, le, lh = self.layout, self.layout.enc, self.layout.head
        act = st["act"]
        dev = d_logrates.device
        head32 = self.head_flat.detach()
        dr = d_logrates.reshape(B, lay.out_dim).to(torch.float32).contiguous()

        lp = dt != torch.float32
        _, bwd_cache, gs_cache = self._caches()
        bkey = (B, _dev_key(dev), dt)
        g = bwd_cache.get(bkey)
        if g is None:
            # backward scratch: only used inside this call, in stream order, so one set per shape
            ar = Arena()
            for k, shape, d in (("d_a", (M, F), dt), ("d_h", (M, D), torch.float32), ("dy", (M, D), torch.float32),
                                ("d_o", (M, D), dt), ("d_qkv", (M, 3 * D), dt), ("dxA", (M, D), torch.float32),
                                ("dxB", (M, D), torch.float32), ("dz", (B, lay.enc_out), torch.float32)):
                ar.add(k, shape, d)
            if lp:
                for k in ("dy_lp", "dxA_lp", "dxB_lp"):
                    ar.add(k, (M, D), dt)
                ar.add("dz_lp", (B, lay.enc_out), dt)
            ar.add("attn_ws", (ops.attn_bwd_workspace_bytes(B, N, H) // 4 + 64,), torch.float32)
            # head dZ = dr dec_w over K = 100 * neurons: split-K partials summed in a fixed order
            ar.add("dz_ws", (max(ops.splitk_workspace_bytes(torch.float32, B, lay.enc_out, lay.out_dim), 16) // 4 + 64,),
                   torch.float32)
            pws = max(ops.splitk_workspace_bytes(dt, D, cfg.patch_dim, M),
                      ops.patch_embed_dw_workspace_bytes(M, D, cfg.patch_dim) if lp and D % 64 == 0 else 0)
            if pws:
                ar.add("patch_ws", (pws // 4 + 64,), torch.float32)
            ar.add("ln_ws", (ops.layernorm_bwd_workspace_bytes(B * N, D) // 4 + 64,), torch.float32)
            gws = max(ops.splitk_workspace_bytes(dt, m, n, M) for m, n in ((D, F), (F, D), (D, D), (3 * D, D)))
            ar.add("gemm_ws", (gws // 4 + 64,), torch.float32)
            g = ar.allocate(dev)
            bwd_cache[bkey] = g

        g_head = self._grad_buffer(self.head_flat) if want_head else None
        Gh = lambda n: lh.view(g_head, n)  # noqa: E731
        z = act["z"]
        dz = g["dz"]
        dz.zero_()
        ops.linear_dx(dr, lh.view(head32, "dec_w"), dz, accumulate=True,     # K = 100*neurons: split-K,
                      workspace=g["dz_ws"])                                  # fixed-order partial sums
        if lp:
            dz_lp = g["dz_lp"]
            ops.cast(dz, dz_lp)
        else:
            dz_lp = dz
        if want_head:
            ops.linear_dw(dr, z, Gh("dec_w"), db=Gh("dec_b"))
            ops.colsum(dz, Gh("enc_b"))                      # dz is B x 64: the lp copy may be rounded
            # reduction over the batch only (K = B): plain stores into the freshly zeroed buffer —
            # f32 atomics on its 19 M elements cost 64 us
            ops.linear_dw(dz_lp, st["x_flat_lp"], Gh("enc_w"), accumulate=False)
            self._ready(self.head_flat, 0, self.head_flat.numel())
        if not want_enc:
            return None, g_head

        g_enc = self._grad_buffer(self.enc_flat)
        Ge = lambda n: le.view(g_enc, n)  # noqa: E731

        dx, dx_lp = g["dxA"], (g["dxA_lp"] if lp else None)
        ops.linear_dx(dz_lp, lh.view(st["head_lp"], "enc_w"), dx.view(B, N * D))
        if lp:
            ops.cast(dx, dx_lp)
        gkey = (bkey, g_enc.data_ptr())
        grads = gs_cache.get(gkey)
        if grads is None:
            if len(gs_cache) > 8:
                gs_cache.clear()
            grads = {}
            cur = "dxA"
            for i in reversed(range(Lyr)):
                gs = L.VitLayerGrad()
                for k in ("ln1_g", "ln1_b", "ln2_g", "ln2_b", "w_qkv", "b_qkv", "w_proj", "b_proj", "w_fc1",
                          "b_fc1", "w_fc2", "b_fc2"):
                    setattr(gs, k, Ge(f"{i}.{k}").data_ptr())
                nxt = "dxB" if cur == "dxA" else "dxA"
                gs.dx_out, gs.dx_out_lp = g[cur].data_ptr(), (g[cur + "_lp"].data_ptr() if lp else None)
                gs.dx_in, gs.dx_in_lp = g[nxt].data_ptr(), (g[nxt + "_lp"].data_ptr() if lp else None)
                gs.d_a, gs.d_h, gs.dy = g["d_a"].data_ptr(), g["d_h"].data_ptr(), g["dy"].data_ptr()
                gs.dy_lp = g["dy_lp"].data_ptr() if lp else None
                gs.d_o, gs.d_qkv, gs.attn_ws = g["d_o"].data_ptr(), g["d_qkv"].data_ptr(), g["attn_ws"].data_ptr()
                gs.ln_ws = g["ln_ws"].data_ptr()
                side = self.__dict__.get("_side", _SIDE)
                gs.chain = self._chain(dev).handle if side else None
                gs.gemm_ws, gs.gemm_ws_bytes = g["gemm_ws"].data_ptr(), g["gemm_ws"].numel() * 4
                # opt-in: every block but the last one defers its side-stream join to the next
                gs.flags = ({1: L.BWD_DEFER_JOIN, 2: L.BWD_DEFER_LAST}[_DEFER] if i > 0 and _DEFER and side else 0)
                fuse_ln = _LN_FUSE if _LN_FUSE is not None else B * N >= _LN_FUSE_ROWS
                gs.flags |= L.BWD_FUSE_LN if fuse_ln else 0
                grads[i] = (gs, nxt)
                cur = nxt
            gs_cache[gkey] = grads
        prev = None
        for i in reversed(range(Lyr)):
            gs, nxt = grads[i]
            ops.vit_layer_bwd(st["structs"][i], gs)
            dx, dx_lp = g[nxt], (g[nxt + "_lp"] if lp else None)
            # joined block: its weight gradients are complete in stream order now; deferred block:
            # once block i-1 (which waits on them) is enqueued.  The last block always joins.
            if not gs.flags:
                if prev is not None:
                    self._ready(self.enc_flat, *lay.layer_ranges[prev])
                self._ready(self.enc_flat, *lay.layer_ranges[i])
                prev = None
                continue
            if prev is not None:
                self._ready(self.enc_flat, *lay.layer_ranges[prev])
            prev = i
        if prev is not None:
            self._ready(self.enc_flat, *lay.layer_ranges[prev])
        # patch embedding: dW = dx0^T cols, db = colsum(dx0); the position table is fixed
        if "cols" not in act:   # cols = the tubelet gather of the pixels, done in the dW's operand load
            ops.patch_embed_dw(st["pixels"], dx_lp, Ge("patch_w"), Ge("patch_b"), cfg.tubelet_size, cfg.patch_size,
                               workspace=g["patch_ws"])
        elif lp:   # bias gradient fused as row sums of dx^T (fixed-order, like every block's dW)
            ops.linear_dw(dx_lp, act["cols"], Ge("patch_w"), db=Ge("patch_b"), workspace=g.get("patch_ws"))
        else:
            ops.linear_dw(dx, act["cols"], Ge("patch_w"), db=Ge("patch_b"))
        self._ready(self.enc_flat, 0, lay.layer_ranges[0][0] if lay.layer_ranges else self.enc_flat.numel())
        return g_enc, g_head


class _VideoMAEFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pixels, enc_flat, head_flat, mod):
        want_enc = bool(ctx.needs_input_grad[1])
        out, st = mod._run_forward(pixels, save_encoder=want_enc)
        ctx.want = (want_enc, bool(ctx.needs_input_grad[2]))
        # keep the saved state (and with it the reservation of the cached buffers) only when a
        # backward can follow
        ctx.mod, ctx.st = mod, (st if any(ctx.want) else None)
        return out

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, grad):
        mod = ctx.mod
        st = ctx.st
        if st is not None and st.get("pixels") is not None and st["pixels"]._version != st["pixels_version"]:
            # the cols-free patch dW gathers the caller's pixels again here: an in-place
            # write between forward and backward (a loader refilling its buffer) would silently give
            # the next batch's gradient — refuse it the way autograd refuses a modified saved tensor
            raise RuntimeError("VideoMAE backward: the input pixels were modified in place after the forward "
                               "(the patch-embedding weight gradient reads them again); pass a tensor that "
                               "stays unchanged until backward, or a copy")
        g_enc, g_head = mod._run_backward(st, grad, *ctx.want)
        ctx.st = None
        sink = mod.grad_sink
        if sink is not None and hasattr(sink, "end_backward"):
            sink.end_backward()
        if sink is not None and not getattr(sink, "return_grads", False):
            return None, None, None, None      # the sink owns .grad (all-reduced in place)
        return None, g_enc, g_head, None
