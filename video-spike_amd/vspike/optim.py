"""Fused AdamW — torch.optim.AdamW semantics (src/train.py:44-49) in one HIP pass per parameter.

A drop-in `torch.optim.Optimizer`: `param_groups[i]['lr']` is honoured, so torch's OneCycleLR
(src/train.py:50-57) drives it unchanged.  Hyper-parameters travel in a small device tensor
(lr, beta1, beta2, eps, wd, step, grad_scale) so the update never syncs the host; `grad_scale`
folds the data-parallel 1/world average into the same pass.  All parameters' rows are staged in
one pinned host block and sent with one asynchronous copy per device per step (a pageable
`torch.tensor(...).to(device)` per parameter was a synchronous ~100 us copy each).
"""
from __future__ import annotations

import torch

from . import ops


class FusedAdamW(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2, grad_scale=1.0):
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, grad_scale=grad_scale)
        super().__init__(params, defaults)

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
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
                st["step"] += 1
                row = [group["lr"], b1, b2, group["eps"], group["weight_decay"], float(st["step"]),
                       group["grad_scale"], 0.0]
                work.setdefault(p.device, []).append((p, st, row))
        for dev, items in work.items():
            host = torch.tensor([r for _, _, r in items], dtype=torch.float32)
            if dev.type != "cpu":
                # the caching host allocator keeps the pinned block alive until the copy has run
                host = host.pin_memory()
            hyper = host.to(dev, non_blocking=True)
            for k, (p, st, _) in enumerate(items):
                g = p.grad
                if g.dtype != torch.float32 or not g.is_contiguous():
                    g = g.float().contiguous()
                ops.adamw(p.data, g, st["exp_avg"], st["exp_avg_sq"], hyper[k])
        return loss
