"""The oracle's MX-FP8 round trip (oracle/cpu_ref.py mx_dequant, the reference side of the C5 fp8
check) against a second restatement of the OCP MX recipe written without torch's float8 dtype:
E8M0 scale 2^e per 32 elements, e = ceil(log2(amax / 448)), elements rounded to the nearest e4m3
value (ties to the even code) found by search over the format's 253 finite magnitudes.  CPU only."""
import math

import numpy as np
import torch

from oracle import cpu_ref


def _e4m3_values():
    """every finite non-negative OCP e4m3 (fn) value with its code, ascending"""
    vals = []
    for code in range(0x7F):                # 0x7F is NaN
        e, mnt = code >> 3, code & 7
        v = (mnt / 8.0) * 2.0 ** -6 if e == 0 else (1 + mnt / 8.0) * 2.0 ** (e - 7)
        vals.append((v, code))
    return vals


E4M3 = _e4m3_values()


def _round_e4m3(x: float) -> float:
    a = abs(x)
    best = min(E4M3, key=lambda vc: (abs(vc[0] - a), vc[1] & 1))   # nearest, ties to the even code
    return math.copysign(best[0], x)


def _mx_block(blk: np.ndarray) -> np.ndarray:
    blk = blk.astype(np.float32)
    amax = float(np.abs(blk).max())
    if amax == 0.0:
        e = 0
    else:
        r = float(np.float32(amax) * np.float32(1.0 / 448.0))
        m, ex = math.frexp(r)                 # r = m 2^ex, m in [0.5, 1)
        e = ex - 1 if m == 0.5 else ex        # ceil(log2 r)
        e = max(-126, min(127, e))
    return np.array([_round_e4m3(float(v) * 2.0 ** -e) * 2.0 ** e for v in blk], dtype=np.float64), e


def test_mx_dequant_matches_an_independent_restatement():
    rng = np.random.default_rng(5)
    x = rng.standard_normal((6, 96)).astype(np.float32) * np.exp(rng.standard_normal((6, 1)) * 4).astype(np.float32)
    x[0, :32] = 0.0                     # all-zero block
    x[1, 40] = 448.0 * 8                # amax exactly 448 * 2^3
    x[2, 70] = 1e-30                    # tiny values in a block with a normal amax
    x[3, 64:96] = 3e-39                 # subnormal f32 block
    xb = torch.from_numpy(x).to(torch.bfloat16).float().numpy()   # the recipe quantises the bf16 value
    got = cpu_ref.mx_dequant(torch.from_numpy(x)).double().numpy()
    blocks = [[_mx_block(xb[r, k:k + 32]) for k in range(0, 96, 32)] for r in range(6)]
    want = np.stack([np.concatenate([v for v, _ in row]) for row in blocks])
    assert np.array_equal(got, want), np.argwhere(got != want)[:5]
    # the format's bound: 2^-4 relative, or half the block's subnormal step 2^(e - 9)
    step = np.stack([np.repeat([2.0 ** (e - 10) for _, e in row], 32) for row in blocks])
    assert np.all(np.abs(got - xb) <= np.abs(xb) * 2.0 ** -4 + step)


def test_mx_matmul_forward_and_straight_through_backward():
    g = torch.Generator().manual_seed(3)
    a = torch.randn(2, 5, 64, generator=g, requires_grad=True)
    w = torch.randn(7, 64, generator=g, requires_grad=True)
    y = cpu_ref.mx_matmul(a, w)
    assert torch.allclose(y, cpu_ref.mx_dequant(a) @ cpu_ref.mx_dequant(w).T)
    gy = torch.randn(2, 5, 7, generator=g)
    y.backward(gy)
    assert torch.allclose(a.grad, gy @ w.detach())
    assert torch.allclose(w.grad, gy.reshape(-1, 7).T @ a.detach().reshape(-1, 64))
