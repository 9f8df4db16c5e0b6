"""Spike-count loss: PoissonNLLLoss(log_input=True) + mean, fused with its gradient.

Replaces `torch.nn.PoissonNLLLoss(reduction="none", log_input=True)` (src/train.py:59) followed by
`.mean()` (src/trainer/base.py:142): one pass computes exp(x) - y*x, a deterministic two-stage
mean, and stashes d/dx = (exp(x) - y)/n for the backward (no second pass over x in the common
upstream-gradient-is-1 case).
"""
from __future__ import annotations

import torch
from torch import nn

from . import _lib as L
from . import ops


class _PoissonMean(torch.autograd.Function):
    @staticmethod
    def forward(ctx, log_rate, target):
        x = log_rate.detach().to(torch.float32).contiguous()
        y = target.detach().to(torch.float32).contiguous()
        loss = torch.empty((), dtype=torch.float32, device=x.device)
        dx = torch.empty_like(x) if ctx.needs_input_grad[0] else None
        ops.poisson_nll(x, y, loss, dx=dx, grad_scale=1.0)
        ctx.save_for_backward(dx)
        return loss

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, g):
        (dx,) = ctx.saved_tensors
        # scale by the upstream gradient on device (no host sync)
        return dx * g.to(dx.dtype), None


def poisson_nll_mean(log_rate: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
    """mean(exp(log_rate) - target * log_rate) on the GPU (HIP), differentiable in log_rate."""
    L.require_device(log_rate, target)
    if log_rate.shape != target.shape:
        raise ValueError(f"shape mismatch {tuple(log_rate.shape)} vs {tuple(target.shape)}")
    return _PoissonMean.apply(log_rate, target)


class PoissonNLLMeanLoss(nn.Module):
    """criterion(outputs, ap) -> scalar; equals PoissonNLLLoss(log_input=True)(...).mean()."""

    def forward(self, log_rate, target):
        return poisson_nll_mean(log_rate, target)
