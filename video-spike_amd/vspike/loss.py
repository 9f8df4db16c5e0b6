"""Spike-count regression losses, each fused with its gradient.

* Poisson (the reference's only training loss): `torch.nn.PoissonNLLLoss(reduction="none",
  log_input=True)` (src/train.py:59) followed by `.mean()` (src/trainer/base.py:142).  One pass
  computes exp(x) - y*x, a deterministic two-stage mean, and stashes d/dx = (exp(x) - y)/n for the
  backward (no second pass over x in the common upstream-gradient-is-1 case).
* MSE (BASELINE north_star: "Poisson/MSE spike-count regression head"): `torch.nn.MSELoss()`
  semantics, mean((x - y)^2), d/dx = 2 (x - y)/n.  The reference has no MSE training loss; it
  computes mse only as an eval metric (src/utils/utils.py:169-171).  Selected by the train config
  key `training.loss: mse` (default `poisson`), see `make_criterion`.
"""
from __future__ import annotations

import torch
from torch import nn

from . import _lib as L
from . import ops


class _FusedMeanLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pred, target, kind):
        x = pred.detach().to(torch.float32).contiguous()
        y = target.detach().to(torch.float32).contiguous()
        loss = torch.empty((), dtype=torch.float32, device=x.device)
        dx = torch.empty_like(x) if ctx.needs_input_grad[0] else None
        (ops.poisson_nll if kind == "poisson" else ops.mse_loss)(x, y, loss, dx=dx, grad_scale=1.0)
        ctx.save_for_backward(dx)
        return loss

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, g):
        (dx,) = ctx.saved_tensors
        # scale by the upstream gradient on device (no host sync)
        return dx * g.to(dx.dtype), None, None


def _check(pred, target):
    L.require_device(pred, target)
    if pred.shape != target.shape:
        raise ValueError(f"shape mismatch {tuple(pred.shape)} vs {tuple(target.shape)}")


def poisson_nll_mean(log_rate: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
    """mean(exp(log_rate) - target * log_rate) on the GPU (HIP), differentiable in log_rate."""
    _check(log_rate, target)
    return _FusedMeanLoss.apply(log_rate, target, "poisson")


def mse_mean(pred: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
    """mean((pred - target)^2) on the GPU (HIP), differentiable in pred (torch.nn.MSELoss())."""
    _check(pred, target)
    return _FusedMeanLoss.apply(pred, target, "mse")


class PoissonNLLMeanLoss(nn.Module):
    """criterion(outputs, ap) -> scalar; equals PoissonNLLLoss(log_input=True)(...).mean()."""

    def forward(self, log_rate, target):
        return poisson_nll_mean(log_rate, target)


class MSEMeanLoss(nn.Module):
    """criterion(outputs, ap) -> scalar; equals torch.nn.MSELoss()(outputs, ap)."""

    def forward(self, pred, target):
        return mse_mean(pred, target)


LOSSES = {"poisson": poisson_nll_mean, "mse": mse_mean}


def make_criterion(config=None):
    """The training criterion named by `config.training.loss` (default "poisson", the reference's
    src/train.py:59).  With "mse" the model's outputs are regressed on the counts directly."""
    name = "poisson"
    if config is not None:
        try:
            name = str((config["training"] or {}).get("loss", "poisson") or "poisson").lower()
        except (KeyError, TypeError, AttributeError):
            name = "poisson"
    if name not in LOSSES:
        raise ValueError(f"training.loss must be one of {sorted(LOSSES)}, got {name!r}")
    return LOSSES[name]
