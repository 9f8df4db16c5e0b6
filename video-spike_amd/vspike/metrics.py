"""Evaluation metrics of the reference's eval loop, computed on the device (vs_spike_metrics).

Mirrors `metrics_list(gt, pred, metrics, device)` (src/utils/utils.py:122-181) for the metrics the
trainer asks for (`['bps', 'rsquared']`, src/trainer/base.py:40) plus 'mse' / 'mae':
  * same arguments: `gt` and `pred` arrive transposed exactly as base.py:190-195 passes them
    (`tensor.transpose(-1, 0)` of the session's (trials, T, N) concatenation; pred already
    exponentiated, base.py:186) — `eval_session()` takes the untransposed log-rates instead and
    fuses the exp;
  * same quirks: bps loops `for i in range(gt.shape[-1])` (= trials) and indexes the NEURON axis
    with i (utils.py:128-129), so only the first `trials` neurons are scored and trials > N
    raises IndexError; +-inf per-neuron bps count as NaN; means ignore NaN;
  * same errors: NaN / negative rates -> AssertionError (metric_utils.py:65-67), NaN / inf
    inputs to rsquared -> ValueError (sklearn's input check).
Numerics: f64 accumulation (the reference runs numpy in f32); agreement is to ~1e-5 relative.
'r2' (torcheval), 'behave_r2' and 'acc' are not on the trainer's path and raise
NotImplementedError.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib as L
from ._lib import check, lib, require_device, stream

_SUPPORTED = ("bps", "rsquared", "mse", "mae")


def _run(x_gt: torch.Tensor, x_pred: torch.Tensor, log_input: bool, n_eval: int, want_r2: bool, per_neuron=False):
    """x_gt, x_pred: (trials, T, N) f32 device tensors (untransposed)."""
    require_device(x_gt, x_pred)
    if x_gt.shape != x_pred.shape or x_gt.dim() != 3:
        raise AssertionError(f"neg_log_likelihood: Rates and spikes should be of the same shape. "
                             f"spikes: {tuple(x_gt.shape)}, rates: {tuple(x_pred.shape)}")
    R, T, N = (int(s) for s in x_gt.shape)
    gt = x_gt.detach().to(torch.float32).contiguous()
    pr = x_pred.detach().to(torch.float32).contiguous()
    dev = gt.device
    ws = torch.empty(int(lib().vs_spike_metrics_workspace_bytes(R, T, N)) // 8 + 2, dtype=torch.float64, device=dev)
    out = torch.empty(8, dtype=torch.float64, device=dev)
    bps_n = torch.empty(max(n_eval, 1), dtype=torch.float64, device=dev) if per_neuron else None
    r2_t = torch.empty(R, dtype=torch.float64, device=dev) if per_neuron else None
    check(lib().vs_spike_metrics(R, T, N, gt.data_ptr(), pr.data_ptr(), int(log_input), int(n_eval), int(want_r2),
                                 out.data_ptr(), L.ptr(bps_n), L.ptr(r2_t), ws.data_ptr(), stream()),
          "vs_spike_metrics")
    return out, bps_n, r2_t


def _check_rates(o):
    if o[2] > 0:
        raise AssertionError("neg_log_likelihood: NaN rate predictions found")
    if o[3] > 0:
        raise AssertionError("neg_log_likelihood: Negative rate predictions found")


def _metrics(x_gt, x_pred, metrics, log_input):
    for m in metrics:
        if m not in _SUPPORTED:
            raise NotImplementedError(f"metric {m!r} is not on the trainer's eval path (supported: {_SUPPORTED})")
    R, N = int(x_gt.shape[0]), int(x_gt.shape[-1])
    want_bps = "bps" in metrics
    if want_bps and R > N:
        # utils.py:128-129 indexes axis 2 (neurons) with the trial loop variable
        raise IndexError(f"index {N} is out of bounds for axis 2 with size {N}")
    want_r2 = any(m in metrics for m in ("rsquared", "mse", "mae"))
    out, _, _ = _run(x_gt, x_pred, log_input, R if want_bps else 0, want_r2)
    o = out.cpu().tolist()
    results = {}
    if want_bps:
        _check_rates(o)
        results["bps"] = o[0]
    if want_r2 and o[4] > 0:
        raise ValueError("Input contains NaN or infinity.")
    if "rsquared" in metrics:
        results["rsquared"] = o[1]
    if "mse" in metrics:
        results["mse"] = torch.tensor(o[5], dtype=torch.float32)
    if "mae" in metrics:
        results["mae"] = torch.tensor(o[6], dtype=torch.float32)
    return {m: results[m] for m in metrics}


def metrics_list(gt: torch.Tensor, pred: torch.Tensor, metrics=("bps", "rsquared"), device="cpu"):
    """utils.py:122-181 with the arguments base.py:190-195 passes: gt, pred = (N, T, trials)
    transposed views of the session tensors; pred are rates.  `device` is accepted for signature
    compatibility (the computation runs where the tensors live)."""
    del device
    return _metrics(gt.transpose(-1, 0), pred.transpose(-1, 0), list(metrics), log_input=False)


def eval_session(gt: torch.Tensor, log_rates: torch.Tensor, metrics=("bps", "rsquared")):
    """base.py:184-195 for one session: gt (trials, 100, N) spike counts and the model's
    log-rate outputs (trials, 100, N) -> {metric: value}; the exp is fused into the kernel."""
    return _metrics(gt, log_rates, list(metrics), log_input=True)


def per_neuron_bps(gt: torch.Tensor, rates: torch.Tensor):
    """bits_per_spike (metric_utils.py:78-102) of each neuron c < trials, as a device f64 tensor
    (NaN where the reference yields NaN or +-inf) — the list utils.py:127-132 averages."""
    R, N = int(gt.shape[0]), int(gt.shape[-1])
    n = min(R, N)
    out, bps_n, _ = _run(gt, rates, False, n, False, per_neuron=True)
    _check_rates(out.cpu().tolist())
    return bps_n[:n]
