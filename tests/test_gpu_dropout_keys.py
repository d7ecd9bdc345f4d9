"""Per-row dropout keys (``row_keys``, include/lpgnn.h lpg_fc_*): an FC call over an arbitrary
subset of a node set's rows -- a general partition's owned variables, which need not be one
contiguous range -- draws for every row the mask the whole-set call draws for that node.

For every FC kernel family (exact fp32, x3, x3 with the heads fused, bf16 on each kernel choice,
the narrow-input conv1 kernels), ``fc(A[idx], ..., row_keys=idx)`` equals ``fc(A, ...)[idx]``
bit for bit: the outputs of a row depend only on that row's operands and its key."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _idx(M, seed=0):
    """A sorted, non-contiguous subset of [0, M) (gaps of 1-3 rows) and its complement's size."""
    rng = np.random.default_rng(seed)
    keep = np.sort(rng.choice(M, size=M // 2, replace=False))
    assert (np.diff(keep) > 1).any()
    return torch.from_numpy(keep.astype(np.int64)).to(DEV)


@pytest.mark.parametrize("arith", ["x3", "fp32"])
@pytest.mark.parametrize("M,N,K1,K2", [(3000, 256, 64, 64), (1000, 1024, 1024, 0), (2500, 128, 8, 8)])
def test_fp32_fc_row_keys(arith, M, N, K1, K2):
    from lpgnn.fc import fc_forward

    g = torch.Generator(device=DEV).manual_seed(M + N)
    A1 = torch.randn(M, K1, device=DEV, generator=g)
    A2 = torch.randn(M, K2, device=DEV, generator=g) if K2 else None
    W1 = torch.randn(N, K1, device=DEV, generator=g) * 0.1
    W2 = torch.randn(N, K2, device=DEV, generator=g) * 0.1 if K2 else None
    b = torch.randn(N, device=DEV, generator=g) * 0.1
    idx = _idx(M)
    full = fc_forward(A1, W1, A2, W2, b, True, 0.25, seed=77, arith=arith)
    sub = fc_forward(A1[idx], W1, None if A2 is None else A2[idx], W2, b, True, 0.25, seed=77, arith=arith,
                     row_keys=idx)
    assert torch.equal(sub, full[idx])
    # the keys matter: without them the subset draws rows 0.. of the mask
    plain = fc_forward(A1[idx], W1, None if A2 is None else A2[idx], W2, b, True, 0.25, seed=77, arith=arith)
    assert not torch.equal(plain, full[idx])


def test_x3_fused_heads_row_keys():
    """The last layer with the heads in its epilogue (lpg_fc_x3_heads_f32), accumulate flag on."""
    from lpgnn.fc import fc_forward

    g = torch.Generator(device=DEV).manual_seed(5)
    M, N, K = 3000, 1024, 1024
    A = torch.randn(M, K, device=DEV, generator=g)
    W = torch.randn(N, K, device=DEV, generator=g) * 0.03
    b = torch.randn(N, device=DEV, generator=g) * 0.1
    P = torch.randn(M, N, device=DEV, generator=g)
    Wh = torch.randn(3, N, device=DEV, generator=g) * 0.03
    bh = torch.randn(3, device=DEV, generator=g)
    idx = _idx(M, 1)
    full, lg = fc_forward(A, W, None, None, b, True, 0.1, seed=9, out=P.clone(), accumulate=True, heads=(Wh, bh))
    sub, lgs = fc_forward(A[idx], W, None, None, b, True, 0.1, seed=9, out=P[idx].clone(), accumulate=True,
                          heads=(Wh, bh), row_keys=idx)
    assert torch.equal(sub, full[idx]) and torch.equal(lgs, lg[idx])


@pytest.mark.parametrize("kernel", [0, 1, 2, 3, 4, 5])
@pytest.mark.parametrize("M,N,K1,K2", [(5000, 512, 128, 128), (700, 256, 64, 0), (3000, 256, 8, 8)])
def test_bf16_fc_row_keys(kernel, M, N, K1, K2):
    from lpgnn.fc import fc_forward_bf16

    g = torch.Generator(device=DEV).manual_seed(M + K1)
    bf = lambda *s: (torch.randn(*s, device=DEV, generator=g) * 0.2).to(torch.bfloat16)  # noqa: E731
    A1, W1 = bf(M, K1), bf(N, K1)
    A2, W2 = (bf(M, K2), bf(N, K2)) if K2 else (None, None)
    b = torch.randn(N, device=DEV, generator=g) * 0.1
    idx = _idx(M, 2)
    full = fc_forward_bf16(A1, W1, A2, W2, b, True, 0.2, 31, kernel=kernel)
    sub = fc_forward_bf16(A1[idx], W1, None if A2 is None else A2[idx], W2, b, True, 0.2, 31, kernel=kernel,
                          row_keys=idx)
    assert torch.equal(sub, full[idx])


def test_row_keys_rejected_when_malformed():
    from lpgnn.fc import fc_forward

    A = torch.randn(10, 64, device=DEV)
    W = torch.randn(64, 64, device=DEV)
    with pytest.raises(RuntimeError, match="row_keys"):
        fc_forward(A, W, None, None, None, True, 0.1, 3, row_keys=torch.arange(9, device=DEV))
    with pytest.raises(RuntimeError, match="row_keys"):
        fc_forward(A, W, None, None, None, True, 0.1, 3, row_keys=torch.arange(10, device=DEV, dtype=torch.int32))
