"""Counter-based deterministic generator shared by the fixture generator and the tests.

TEST INFRASTRUCTURE ONLY — never imported by the product path (`video-spike_amd/vspike`).

The golden fixtures under `tests/golden/` commit only OUTPUTS.  Inputs and weights are
re-derived bit-for-bit from (seed, name) with this generator, so the fixture generator
(run once, here, with the reference importable) and the tests (run anywhere, without the
reference) see the same tensors.  Recipe follows SURVEY.md §8(c) "Fixture recipe":
splitmix64 → 53-bit uniform → Box–Muller.
"""
from __future__ import annotations

import zlib

import numpy as np

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def stream_key(seed: int, name: str = "") -> int:
    """64-bit stream key from an integer seed and a tensor name."""
    return (int(seed) * 0x100000001B3 + zlib.crc32(name.encode())) & 0xFFFFFFFFFFFFFFFF


def uniform(seed: int, n: int, name: str = "") -> np.ndarray:
    """n float64 samples in [0, 1)."""
    key = np.uint64(stream_key(seed, name))
    with np.errstate(over="ignore"):
        ctr = np.arange(n, dtype=np.uint64) * np.uint64(0xD1B54A32D192ED03) + key
    bits = _splitmix64(ctr) >> np.uint64(11)
    return bits.astype(np.float64) * (1.0 / 9007199254740992.0)


def video_frames(seed: int, shape, name: str = "video") -> np.ndarray:
    """Integer-valued float32 frames in 0..255 (decoded-mp4 pixel values), `shape` e.g. (B, 120, 1, H, W)."""
    n = int(np.prod(shape))
    return np.floor(uniform(seed, n, name) * 256.0).astype(np.float32).reshape(shape)


def normal(seed: int, shape, name: str = "", std: float = 1.0, mean: float = 0.0) -> np.ndarray:
    """float32 N(mean, std) samples by Box–Muller over two uniform streams."""
    n = int(np.prod(shape)) if len(tuple(np.atleast_1d(shape))) else 1
    u1 = uniform(seed, n, name + "#bm1")
    u2 = uniform(seed, n, name + "#bm2")
    r = np.sqrt(-2.0 * np.log1p(-u1))          # 1-u1 in (0,1]
    z = r * np.cos(2.0 * np.pi * u2)
    return (mean + std * z).astype(np.float32).reshape(shape)


def poisson(seed: int, lam: np.ndarray, name: str = "") -> np.ndarray:
    """Poisson(lam) counts (as float32) by inversion of one uniform per element (lam <= ~20)."""
    lam = np.asarray(lam, dtype=np.float64)
    u = uniform(seed, lam.size, name).reshape(lam.shape)
    k = np.zeros(lam.shape, dtype=np.float64)
    p = np.exp(-lam)
    cdf = p.copy()
    for i in range(1, 64):
        more = u > cdf
        if not more.any():
            break
        k += more
        p = p * lam / i
        cdf = cdf + p
    return k.astype(np.float32)


def spike_targets(seed: int, shape, name: str = "ap") -> np.ndarray:
    """Synthetic binned spike counts per BASELINE.md: lam = exp(N(-2,1)) clipped to [0.01, 5]."""
    lam = np.clip(np.exp(normal(seed, shape, name + "#lam", std=1.0, mean=-2.0).astype(np.float64)), 0.01, 5.0)
    return poisson(seed, lam, name + "#cnt")
