"""Eval metrics on the device (vs_spike_metrics) against the CPU
restatement (oracle/metrics_ref.py, pinned to the reference's own metrics_list / bits_per_spike
by tests/golden/metrics.npz).

Tolerances: the kernel accumulates in f64; against the f64 restatement on the same f32 inputs the
bar is 1e-9 relative (rates given) / 1e-6 (log-rates: the device expf and numpy's exp may differ
by one f32 ulp).  Against the reference's own f32 numpy arithmetic (the fixture) it is 1e-6
absolute — measured restatement f32-vs-f64 gaps are <= 1.4e-7."""
import warnings

import numpy as np
import pytest
import torch

from oracle import metrics_ref as M

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    warnings.simplefilter("ignore", RuntimeWarning)


@pytest.mark.parametrize("name", list(M.METRIC_CASES))
def test_metrics_match_reference_fixture(golden, name):
    from vspike import metrics
    fx = golden("metrics.npz")
    R, T, N, seed, mets, log_input = M.METRIC_CASES[name]
    gt, pred = M.metric_case(name)
    g, p = torch.from_numpy(gt).to(DEV), torch.from_numpy(pred).to(DEV)
    if log_input:
        got = metrics.eval_session(g, p, mets)
        want64 = M.eval_session(gt, pred, mets, dtype=np.float64)
    else:
        got = metrics.metrics_list(g.transpose(-1, 0), p.transpose(-1, 0), mets)
        want64 = M.metrics_list(np.swapaxes(gt, -1, 0), np.swapaxes(pred, -1, 0), mets, dtype=np.float64)
    for k in mets:
        assert abs(got[k] - float(fx[f"{name}.{k}"])) <= 1e-6, (k, got[k], fx[f"{name}.{k}"])
        assert abs(got[k] - want64[k]) <= (1e-6 if log_input else 1e-9) * max(1.0, abs(want64[k])), (k, got[k], want64[k])


def test_metrics_list_takes_the_reference_call_shape():
    """base.py:190-195 passes gt.transpose(-1, 0) and exp(preds).transpose(-1, 0)."""
    from vspike import metrics
    gt, lr = M.metric_case("m_basic")
    g = torch.from_numpy(gt).to(DEV)
    rates = torch.exp(torch.from_numpy(lr).to(DEV))
    a = metrics.metrics_list(gt=g.transpose(-1, 0), pred=rates.transpose(-1, 0), metrics=["bps", "rsquared"],
                             device=DEV)
    b = metrics.eval_session(g, torch.from_numpy(lr).to(DEV))
    assert list(a) == ["bps", "rsquared"]
    assert abs(a["bps"] - b["bps"]) < 1e-9 and abs(a["rsquared"] - b["rsquared"]) < 1e-9


def test_per_neuron_bps_and_nan_rules(golden):
    from vspike import metrics
    fx = golden("metrics.npz")
    for name in ("m_basic", "m_square"):
        gt, lr = M.metric_case(name)
        rates = np.exp(lr).astype(np.float32)
        got = metrics.per_neuron_bps(torch.from_numpy(gt).to(DEV), torch.from_numpy(rates).to(DEV)).cpu().numpy()
        want = fx[f"{name}.bps_per_neuron"].copy()
        want[np.isinf(want)] = np.nan
        assert np.array_equal(np.isnan(got), np.isnan(want))       # silent neuron -> NaN
        np.testing.assert_allclose(got[~np.isnan(got)], want[~np.isnan(want)], rtol=1e-5, atol=2e-6)
        ref64 = M.per_neuron_bps(gt, rates)
        np.testing.assert_allclose(got[~np.isnan(got)], ref64[~np.isnan(ref64)], rtol=1e-9, atol=1e-12)


def test_metrics_error_behaviour():
    from vspike import metrics
    gt, lr = M.metric_case("m_wide")                 # trials 40 > neurons 32
    g, p = torch.from_numpy(gt).to(DEV), torch.from_numpy(lr).to(DEV)
    with pytest.raises(IndexError):
        metrics.eval_session(g, p, ["bps"])
    r = metrics.eval_session(g, p, ["rsquared"])
    assert np.isfinite(r["rsquared"])
    gt, lr = M.metric_case("m_basic")
    rates = torch.exp(torch.from_numpy(lr)).to(DEV)
    g = torch.from_numpy(gt).to(DEV)
    bad = rates.clone()
    bad[1, 2, 3] = float("nan")
    with pytest.raises(AssertionError, match="NaN rate"):
        metrics.metrics_list(g.transpose(-1, 0), bad.transpose(-1, 0), ["bps"])
    bad = rates.clone()
    bad[0, 0, 0] = -1.0
    with pytest.raises(AssertionError, match="Negative rate"):
        metrics.metrics_list(g.transpose(-1, 0), bad.transpose(-1, 0), ["bps"])
    gnan = g.clone()
    gnan[0, 0, 0] = float("nan")
    with pytest.raises(ValueError):
        metrics.metrics_list(gnan.transpose(-1, 0), rates.transpose(-1, 0), ["rsquared"])
    with pytest.raises(NotImplementedError):
        metrics.metrics_list(g.transpose(-1, 0), rates.transpose(-1, 0), ["acc"])


def test_metrics_zero_rates_and_mse_mae():
    """zero rates -> 1e-9 (metric_utils.py:68-73); mse / mae (utils.py:169-175)."""
    from vspike import metrics
    gt, lr = M.metric_case("m_basic")
    rates = np.exp(lr).astype(np.float32)
    rates[0, :5, 1] = 0.0
    g, p = torch.from_numpy(gt).to(DEV), torch.from_numpy(rates).to(DEV)
    got = metrics.metrics_list(g.transpose(-1, 0), p.transpose(-1, 0), ["bps", "mse", "mae"])
    want = M.metrics_list(np.swapaxes(gt, -1, 0), np.swapaxes(rates, -1, 0), ["bps"], dtype=np.float64)
    assert abs(got["bps"] - want["bps"]) <= 1e-9 * max(1, abs(want["bps"]))
    d = gt.astype(np.float64) - rates.astype(np.float64)
    assert abs(float(got["mse"]) - np.mean(d * d)) <= 1e-6 * np.mean(d * d)
    assert abs(float(got["mae"]) - np.mean(np.abs(d))) <= 1e-6 * np.mean(np.abs(d))


def test_metrics_large_session_properties():
    """A session at eval scale (500 trials x 100 bins x 512 neurons): deterministic (bit-identical
    repeat) and equal to the f64 restatement on a neuron subset."""
    from vspike import metrics
    from oracle import prng
    R, T, N = 500, 100, 512
    gt = prng.spike_targets(31, (R, T, N)).astype(np.float32)
    lr = prng.normal(31, (R, T, N), name="lr", std=0.5, mean=-1.5)
    g, p = torch.from_numpy(gt).to(DEV), torch.from_numpy(lr).to(DEV)
    a = metrics.eval_session(g, p)
    b = metrics.eval_session(g, p)
    assert a == b
    rates = np.exp(lr)
    sub = M.per_neuron_bps(gt[:, :, :8], rates[:, :, :8])
    got = metrics.per_neuron_bps(g, torch.from_numpy(rates).to(DEV)).cpu().numpy()[:8]
    np.testing.assert_allclose(got, sub, rtol=1e-6, atol=1e-9)
