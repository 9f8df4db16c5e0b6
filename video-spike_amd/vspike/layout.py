"""Flat parameter layout of the VideoMAE plugin.

All encoder parameters live in ONE f32 buffer and all head parameters in another, so that the
optimizer step is one fused kernel per buffer and the data-parallel gradient exchange is a few
large contiguous all-reduces (no per-tensor bucketing on the host).  Every tensor starts on a
64-element (256 B) boundary.  `hf_name` maps each slice to the reference plugin's state_dict
name (`video_mae.*` = HF VideoMAEModel, `encoder.*`/`decoder.*` = src/model/videomae.py:13-14).
"""
from __future__ import annotations

import dataclasses
from typing import Dict, List, Optional, Tuple

ALIGN = 64


@dataclasses.dataclass(frozen=True)
class BackboneCfg:
    """Encoder geometry; defaults = videomae-base (the checkpoint src/model/videomae.py:7 loads)."""
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

    @classmethod
    def from_config(cls, d: Optional[dict]) -> "BackboneCfg":
        if not d:
            return cls()
        names = {f.name for f in dataclasses.fields(cls)}
        kw = {k: (float(v) if k == "layer_norm_eps" else int(v)) for k, v in dict(d).items() if k in names}
        return cls(**kw)


@dataclasses.dataclass
class Slot:
    name: str
    shape: Tuple[int, ...]
    offset: int

    @property
    def numel(self) -> int:
        n = 1
        for s in self.shape:
            n *= s
        return n


class FlatLayout:
    def __init__(self):
        self.slots: Dict[str, Slot] = {}
        self.numel = 0

    def add(self, name: str, shape: Tuple[int, ...]) -> Slot:
        s = Slot(name, tuple(shape), self.numel)
        self.slots[name] = s
        self.numel += (s.numel + ALIGN - 1) // ALIGN * ALIGN
        return s

    def view(self, flat, name: str):
        s = self.slots[name]
        return flat[s.offset:s.offset + s.numel].view(s.shape)


# transformers 4.38 (reference pin) -> newer transformers names of the Q/V biases
LEGACY_BIAS_ALIASES = {"attention.attention.q_bias": "attention.attention.query.bias",
                       "attention.attention.v_bias": "attention.attention.value.bias"}


def modern_name(name: str) -> str:
    """The newer-transformers spelling of a reference (4.38) state_dict name."""
    for old, new in LEGACY_BIAS_ALIASES.items():
        if name.endswith(old):
            return name[: -len(old)] + new
    return name


LAYER_KEYS = ("ln1_g", "ln1_b", "w_qkv", "b_qkv", "w_proj", "b_proj", "ln2_g", "ln2_b", "w_fc1", "b_fc1",
              "w_fc2", "b_fc2")


class VitLayout:
    """encoder flat: patch_w, patch_b, then per layer LAYER_KEYS; head flat: enc_w, enc_b, dec_w, dec_b."""

    def __init__(self, cfg: BackboneCfg, enc_out: int, out_dim: int):
        self.cfg, self.enc_out, self.out_dim = cfg, enc_out, out_dim
        D, F = cfg.hidden_size, cfg.intermediate_size
        e = FlatLayout()
        e.add("patch_w", (D, cfg.patch_dim))
        e.add("patch_b", (D,))
        self.layer_ranges: List[Tuple[int, int]] = []
        for i in range(cfg.num_hidden_layers):
            lo = e.numel
            for k, shape in (("ln1_g", (D,)), ("ln1_b", (D,)), ("w_qkv", (3 * D, D)), ("b_qkv", (3 * D,)),
                             ("w_proj", (D, D)), ("b_proj", (D,)), ("ln2_g", (D,)), ("ln2_b", (D,)),
                             ("w_fc1", (F, D)), ("b_fc1", (F,)), ("w_fc2", (D, F)), ("b_fc2", (D,))):
                e.add(f"{i}.{k}", shape)
            self.layer_ranges.append((lo, e.numel))
        self.enc = e
        h = FlatLayout()
        h.add("enc_w", (enc_out, cfg.num_tokens * D))
        h.add("enc_b", (enc_out,))
        h.add("dec_w", (out_dim, enc_out))
        h.add("dec_b", (out_dim,))
        self.head = h

    # ---- reference state_dict names -----------------------------------------------------------
    def hf_items(self):
        """Yield (hf_name, which_flat, slot_name, row_slice) for every reference parameter.

        Names are those of the transformers version the reference pins (4.38.2, env.yaml:30):
        the Q/V biases are separate parameters `attention.attention.q_bias` / `v_bias` and there is
        no key bias (vendored modeling_videomae.py:216-218, 233).  Newer transformers store them as
        `query.bias` / `value.bias` (+ a `key.bias`): see `modern_name` / `LEGACY_BIAS_ALIASES`."""
        D = self.cfg.hidden_size
        yield "video_mae.embeddings.patch_embeddings.projection.weight", "enc", "patch_w", None
        yield "video_mae.embeddings.patch_embeddings.projection.bias", "enc", "patch_b", None
        for i in range(self.cfg.num_hidden_layers):
            p = f"video_mae.encoder.layer.{i}."
            yield p + "attention.attention.query.weight", "enc", f"{i}.w_qkv", slice(0, D)
            yield p + "attention.attention.key.weight", "enc", f"{i}.w_qkv", slice(D, 2 * D)
            yield p + "attention.attention.value.weight", "enc", f"{i}.w_qkv", slice(2 * D, 3 * D)
            yield p + "attention.attention.q_bias", "enc", f"{i}.b_qkv", slice(0, D)
            yield p + "attention.attention.v_bias", "enc", f"{i}.b_qkv", slice(2 * D, 3 * D)
            yield p + "attention.output.dense.weight", "enc", f"{i}.w_proj", None
            yield p + "attention.output.dense.bias", "enc", f"{i}.b_proj", None
            yield p + "intermediate.dense.weight", "enc", f"{i}.w_fc1", None
            yield p + "intermediate.dense.bias", "enc", f"{i}.b_fc1", None
            yield p + "output.dense.weight", "enc", f"{i}.w_fc2", None
            yield p + "output.dense.bias", "enc", f"{i}.b_fc2", None
            yield p + "layernorm_before.weight", "enc", f"{i}.ln1_g", None
            yield p + "layernorm_before.bias", "enc", f"{i}.ln1_b", None
            yield p + "layernorm_after.weight", "enc", f"{i}.ln2_g", None
            yield p + "layernorm_after.bias", "enc", f"{i}.ln2_b", None
        yield "encoder.weight", "head", "enc_w", None
        yield "encoder.bias", "head", "enc_b", None
        yield "decoder.weight", "head", "dec_w", None
        yield "decoder.bias", "head", "dec_b", None
