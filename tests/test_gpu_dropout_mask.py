"""The fused dropout mask of every FC kernel family against its restatement (oracle/dropout_ref.py):
the kept set of ``fc(..., relu=True, dropout_p=p, seed=s)`` is exactly ``keep_mask(s, keys, N, p)``,
bit for bit, and kept values are the no-dropout output times 1 / (1 - q), q the drawn rate (the reference's
F.dropout after the ReLU, arch.py:186-188).  Every output of these cases is positive before the
dropout (bias +4, small operands), so "kept" is "stored output > 0"."""
import numpy as np
import pytest
import torch

from oracle.dropout_ref import keep_mask, scale as keep_scale, threshold

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _ops(M, N, K1, K2, dtype=torch.float32, seed=0):
    g = torch.Generator(device=DEV).manual_seed(seed + M + N)
    r = lambda *s: (torch.rand(*s, device=DEV, generator=g) * 0.05).to(dtype)  # noqa: E731
    A1, W1 = r(M, K1), r(N, K1)
    A2, W2 = (r(M, K2), r(N, K2)) if K2 else (None, None)
    b = torch.full((N,), 4.0, device=DEV)
    return A1, W1, A2, W2, b


def _check(y, base, seed, keys, p):
    assert bool((base > 0).all())
    want = keep_mask(seed, keys, y.shape[1], p)
    got = (y != 0).cpu().numpy()
    assert np.array_equal(got, want), f"{int((got != want).sum())} of {got.size} mask bits differ"
    kept = torch.from_numpy(want).to(DEV)
    scale = torch.tensor(keep_scale(p), dtype=torch.float32)
    if y.dtype == torch.float32:
        assert torch.equal(y[kept], base[kept] * scale.to(DEV))
    else:  # one RNE of the fp32 value: kept = 16-bit(fp32 result * scale)
        ref = (y.float()[kept] - base.float()[kept] * float(scale)).abs()
        assert float(ref.max()) <= 2 ** -7 * float(base.float().abs().max() * scale) + 1e-3


@pytest.mark.parametrize("arith", ["x3", "fp32"])
@pytest.mark.parametrize("M,N,K1,K2,row_off", [
    (3000, 256, 64, 64, 0),       # tiled kernels
    (777, 1024, 1024, 0, 12345),  # ragged rows, a slice of a larger node set
    (2500, 128, 8, 8, 7),         # the narrow-input (conv1) kernel
    (300, 36, 64, 0, 0),          # N not a multiple of 16 (per-element epilogue columns)
])
@pytest.mark.parametrize("p", [0.1, 0.5])
def test_fp32_kernels_mask_equals_oracle(arith, M, N, K1, K2, row_off, p):
    from lpgnn.fc import fc_forward

    A1, W1, A2, W2, b = _ops(M, N, K1, K2)
    seed = 0x1234_5678_9ABC + M
    base = fc_forward(A1, W1, A2, W2, b, True, arith=arith, row_offset=row_off)
    y = fc_forward(A1, W1, A2, W2, b, True, p, seed=seed, arith=arith, row_offset=row_off)
    _check(y, base, seed, np.arange(M) + row_off, p)


def test_x3_fused_heads_mask_equals_oracle():
    from lpgnn.fc import fc_forward

    M, N, K = 3000, 1024, 512
    A1, W1, _, _, b = _ops(M, N, K, 0, seed=3)
    Wh = torch.randn(3, N, device=DEV) * 0.01
    seed = 99
    base, _ = fc_forward(A1, W1, None, None, b, True, heads=(Wh, None), arith="x3")
    y, lg = fc_forward(A1, W1, None, None, b, True, 0.1, seed=seed, heads=(Wh, None), arith="x3")
    _check(y, base, seed, np.arange(M), 0.1)


@pytest.mark.parametrize("kernel", [0, 1, 2, 3, 4, 5])
@pytest.mark.parametrize("M,N,K1,K2", [(5000, 512, 128, 128), (700, 256, 64, 0), (3000, 256, 8, 8)])
def test_bf16_kernels_mask_equals_oracle(kernel, M, N, K1, K2):
    from lpgnn.fc import fc_forward_bf16

    A1, W1, A2, W2, b = _ops(M, N, K1, K2, torch.bfloat16, seed=kernel)
    seed, p = 4242 + kernel, 0.2
    idx = torch.arange(M, device=DEV) * 3 + 11  # explicit per-row keys (a general partition's ids)
    base = fc_forward_bf16(A1, W1, A2, W2, b, True, kernel=kernel)
    y = fc_forward_bf16(A1, W1, A2, W2, b, True, p, seed, kernel=kernel, row_keys=idx)
    _check(y, base, seed, idx.cpu().numpy(), p)


def test_fp16_kernels_mask_equals_oracle():
    from lpgnn.fc import fc_forward_bf16

    M, N, K = 4096, 512, 256
    A1, W1, _, _, b = _ops(M, N, K, 0, torch.float16, seed=5)
    base = fc_forward_bf16(A1, W1, None, None, b, True)
    y = fc_forward_bf16(A1, W1, None, None, b, True, 0.1, 77)
    _check(y, base, 77, np.arange(M), 0.1)


@pytest.mark.parametrize("p", [0.1, 0.3, 0.9])
def test_mask_rate_and_independence(p):
    """The drawn mask over a c2-size block of rows: drop rate within 5 sigma of the 16-bit
    threshold's p (itself within 2^-17 of p), even and odd columns (the two halves of one hash)
    each at that rate and uncorrelated, rows of consecutive keys uncorrelated."""
    from lpgnn.fc import fc_forward_bf16

    M, N, K = 20000, 1024, 64
    A1, W1, _, _, b = _ops(M, N, K, 0, torch.bfloat16, seed=9)
    y = fc_forward_bf16(A1, W1, None, None, b, True, p, 2024)
    kept = (y != 0).float()
    q = threshold(p) / 65536.0
    assert abs(q - p) <= 2 ** -17
    n = kept.numel()
    sd = (q * (1 - q) / n) ** 0.5
    assert abs((1 - kept.mean().item()) - q) < 5 * sd
    ev, od = kept[:, 0::2], kept[:, 1::2]
    sd_h = (q * (1 - q) / ev.numel()) ** 0.5
    assert abs((1 - ev.mean().item()) - q) < 5 * sd_h and abs((1 - od.mean().item()) - q) < 5 * sd_h
    for a, c in ((ev, od), (kept[:-1], kept[1:])):
        corr = torch.corrcoef(torch.stack((a.flatten(), c.flatten())))[0, 1].item()
        assert abs(corr) < 5 / a.numel() ** 0.5, corr
