"""The dropout-mask restatement (oracle/dropout_ref.py) on its own: the 16-bit threshold, and the
mask's statistics -- a Bernoulli(1 - p) keep per element, the two halves of one hash (even / odd
columns) and neighbouring row keys uncorrelated.  The GPU kernels are pinned to it bit for bit in
tests/test_gpu_dropout_mask.py."""
import numpy as np
import pytest

from oracle.dropout_ref import keep_mask, lowbias32, threshold


def test_threshold():
    assert threshold(0.0) == 0
    assert threshold(0.1) == 6554  # round(0.1f * 65536)
    assert threshold(0.5) == 32768
    assert threshold(1e-9) == 1    # the smallest nonzero rate
    assert threshold(0.999999) == 65535


def test_lowbias32_is_a_bijection_sample():
    x = np.arange(1 << 16, dtype=np.uint32) * np.uint32(65537)
    h = lowbias32(x)
    assert len(np.unique(h)) == len(x)
    assert int(lowbias32(np.array([0], dtype=np.uint32))[0]) == 0


@pytest.mark.parametrize("p", [0.1, 0.5])
def test_mask_statistics(p):
    M, N = 2000, 1024
    keep = keep_mask(0xDEADBEEF12345, np.arange(M) + 77, N, p)
    q = threshold(p) / 65536
    n = keep.size
    assert abs((1 - keep.mean()) - q) < 5 * (q * (1 - q) / n) ** 0.5
    ev, od = keep[:, 0::2].astype(np.float64), keep[:, 1::2].astype(np.float64)
    for a, b in ((ev, od), (keep[:-1].astype(np.float64), keep[1:].astype(np.float64))):
        c = np.corrcoef(a.ravel(), b.ravel())[0, 1]
        assert abs(c) < 5 / a.size ** 0.5, c
    # a different seed gives a different mask; the same seed the same one
    assert not np.array_equal(keep, keep_mask(0xDEADBEEF12346, np.arange(M) + 77, N, p))
    assert np.array_equal(keep, keep_mask(0xDEADBEEF12345, np.arange(M) + 77, N, p))


@pytest.mark.parametrize("p", [0.1, 0.2, 0.5, 0.9, 1e-3, 2.0 ** -16, 0.99999])
def test_product_scale_is_the_kept_rate_reciprocal(p):
    """lpgnn.fc.dropout_scale (what the backward passes use) equals the oracle's restatement of
    dropout_params' scale: 2^16 / (2^16 - threshold), so E[kept * scale] = 1 exactly."""
    from lpgnn.fc import dropout_scale
    from oracle.dropout_ref import scale

    s = dropout_scale(p)
    assert s == scale(p)
    q = threshold(p) / 65536.0
    assert abs(s * (1 - q) - 1.0) < 2e-7


@pytest.mark.parametrize("p", [1e-6, 2.0 ** -18, 1.0, 1.5])
def test_product_scale_refuses_undrawable_rates(p):
    from lpgnn.fc import dropout_scale

    with pytest.raises(ValueError):
        dropout_scale(p)
