"""Host-side check of the token decomposition vs_patch_embed_dw's gather uses (gemm_dw.hip, tok_base):
m -> (b, f', hp, wp) by an f32 reciprocal product truncated to int and corrected by one step either
way.  The same IEEE f32 arithmetic in numpy, over every token index of the geometries the kernel
serves (and the 2^24 cap it enforces), must equal exact integer division."""
import numpy as np
import pytest


def _div(n, d):
    """q = (int)((float)n * (1.0f / d)), then q -= q*d > n, q += (q+1)*d <= n  (as tok_base)."""
    inv = np.float32(1.0) / np.float32(d)
    q = (n.astype(np.float32) * inv).astype(np.int64)   # f32 product (RNE), truncation toward 0
    q -= (q * d > n).astype(np.int64)
    q += ((q + 1) * d <= n).astype(np.int64)
    return q


@pytest.mark.parametrize("geo", [(16, 224, 224), (8, 112, 112), (4, 32, 48), (32, 224, 224), (120, 128, 128),
                                 (2, 16, 16), (16, 240, 320)])
def test_token_decomposition_exact(geo):
    F, H, W = geo
    Wp, HpWp = W // 16, (H // 16) * (W // 16)
    n_tok = (F // 2) * HpWp
    top = (1 << 24) - 1                       # the kernel's cap: < 2^24 tokens per launch
    m = np.concatenate([np.arange(0, min(top, 4 << 20), dtype=np.int64),
                        np.arange(top - (1 << 20), top + 1, dtype=np.int64)])
    b = _div(m, n_tok)
    n = m - b * n_tok
    fp = _div(n, HpWp)
    r = n - fp * HpWp
    hp = _div(r, Wp)
    wp = r - hp * Wp
    assert np.array_equal(b, m // n_tok)
    assert np.array_equal(fp, n // HpWp) and np.array_equal(hp, r // Wp)
    assert (wp >= 0).all() and (wp < Wp).all()
