"""Fused AdamW — torch.optim.AdamW semantics (src/train.py:44-49) in one HIP pass per parameter.

A drop-in `torch.optim.Optimizer`.  Parameters with a registered bf16 shadow (LP_SHADOWS) get it
rewritten in the same pass (2 more bytes per parameter instead of a separate 6-byte cast pass).
 `param_groups[i]['lr']` is honoured, so torch's OneCycleLR
(src/train.py:50-57) drives it unchanged.  Hyper-parameters travel in a small device tensor
(lr, beta1, beta2, eps, wd, step, grad_scale) so the update never syncs the host; `grad_scale`
folds the data-parallel 1/world average into the same pass.  All parameters' rows are staged in
one pinned host block and sent with one asynchronous copy per device per step (a pageable
`torch.tensor(...).to(device)` per parameter was a synchronous ~100 us copy each).
"""
from __future__ import annotations

import weakref

import torch

from . import ops

# Low-precision shadows of parameters (registered by the plugins, vspike.vit): FusedAdamW writes the
# bf16 copy of each updated parameter in the same pass (vs_adamw `param_lp`), so the next forward
# does not re-cast the f32 master weights.  id(param) -> (weakref(param), shadow tensor, stamp dict);
# stamp["key"] is (data_ptr, _version) of the parameter the shadow was last made from — any
# autograd-visible in-place write to the parameter bumps _version and makes the forward cast again.
# (Keyed by id: a WeakKeyDictionary compares tensor keys with ==, which is elementwise.)
LP_SHADOWS: dict = {}


def register_lp_shadow(param: torch.Tensor, shadow: torch.Tensor, stamp: dict) -> None:
    pid = id(param)
    LP_SHADOWS[pid] = (weakref.ref(param, lambda _r, pid=pid: LP_SHADOWS.pop(pid, None)), shadow, stamp)


def lp_shadow(param: torch.Tensor):
    ent = LP_SHADOWS.get(id(param))
    if ent is None or ent[0]() is not param:
        return None
    return ent[1], ent[2]


def lp_key(param: torch.Tensor):
    return (param.data_ptr(), param._version)


class FusedAdamW(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2, grad_scale=1.0):
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, grad_scale=grad_scale)
        super().__init__(params, defaults)

    def _work(self, advance: bool):
        """device -> [(param, state, hyper row)] of the parameters that have a gradient; `advance`
        counts this update in each parameter's step (the row carries the new count)."""
        work = {}
        for group in self.param_groups:
            b1, b2 = group["betas"]
            for p in group["params"]:
                if p.grad is None:
                    continue
                st = self.state[p]
                if not st:
                    st["step"] = 0
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                step = st["step"] + 1
                if advance:
                    st["step"] = step
                row = [group["lr"], b1, b2, group["eps"], group["weight_decay"], float(step), group["grad_scale"], 0.0]
                work.setdefault(p.device, []).append((p, st, row))
        return work

    @staticmethod
    def _upload(items, dev, out=None):
        host = torch.tensor([r for _, _, r in items], dtype=torch.float32)
        if dev.type != "cpu":
            # the caching host allocator keeps the pinned block alive until the copy has run
            host = host.pin_memory()
        if out is None:
            return host.to(dev, non_blocking=True)
        out[:len(items)].copy_(host, non_blocking=True)
        return out

    @staticmethod
    def _launch(items, hyper):
        for k, (p, st, _) in enumerate(items):
            g = p.grad
            if g.dtype != torch.float32 or not g.is_contiguous():
                g = g.float().contiguous()
            ent = lp_shadow(p)
            lp = ent[0] if ent is not None and ent[0].device == p.device and ent[0].numel() == p.numel() else None
            ops.adamw(p.data, g, st["exp_avg"], st["exp_avg_sq"], hyper[k], param_lp=lp)
            if lp is not None:
                ent[1]["key"] = lp_key(p)

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for dev, items in self._work(advance=True).items():
            self._launch(items, self._upload(items, dev))
        return loss

    # ---- hipGraph capture (vspike.graph.GraphedStep) -------------------------------------------
    @torch.no_grad()
    def static_hyper(self):
        """device -> hyper-parameter block with a row for every parameter of the groups (those with
        a gradient use the first rows, in `_work` order), to be captured: the launches of
        `launch_static` read it, `stage` rewrites it before every replay."""
        rows = {}
        for group in self.param_groups:
            for p in group["params"]:
                rows[p.device] = rows.get(p.device, 0) + 1
        return {dev: torch.zeros(n, 8, dtype=torch.float32, device=dev) for dev, n in rows.items()}

    @torch.no_grad()
    def launch_static(self, hyper):
        """The update launches of `step` reading `hyper` (inside a capture; no host-side state moves)."""
        for dev, items in self._work(advance=False).items():
            self._launch(items, hyper[dev])

    @torch.no_grad()
    def stage(self, hyper):
        """Host half of one captured update: count the step and send this step's rows (lr from the
        scheduler, bias-correction step) into `hyper` on the current stream, ahead of the replay."""
        for dev, items in self._work(advance=True).items():
            self._upload(items, dev, out=hyper[dev])
