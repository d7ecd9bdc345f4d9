"""torch.ops.lpgnn.spmm_sum (torch_sparse's spmm_sum schema) on the HIP
kernel: forward and mat-gradient bitwise vs the oracle's spmm_cpu order."""
import numpy as np
import pytest
import torch

from oracle import model_ref as O

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _torch_sparse_args(rng, m, n, nnz):
    """(row, rowptr, col, value, colptr, csr2csc) as SparseTensor stores them."""
    keys = np.sort(rng.choice(m * n, size=nnz, replace=False))  # row-major sorted = CSR order
    row, col = keys // n, keys % n
    val = rng.uniform(-1, 1, nnz).astype(np.float32)
    rowptr = np.zeros(m + 1, np.int64)
    np.add.at(rowptr, row + 1, 1)
    rowptr = np.cumsum(rowptr)
    csr2csc = np.argsort(col * m + row, kind="stable")
    colptr = np.zeros(n + 1, np.int64)
    np.add.at(colptr, col + 1, 1)
    colptr = np.cumsum(colptr)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(DEV)
    return t(row), t(rowptr), t(col), t(val), t(colptr), t(csr2csc), (rowptr, col, val)


@pytest.mark.parametrize("m,n,nnz,F", [(300, 500, 4000, 64), (1, 7, 7, 8), (50, 40, 0, 16), (2000, 100, 30000, 1024)])
def test_spmm_sum_forward_backward_bitwise(m, n, nnz, F):
    import lpgnn  # noqa: F401

    rng = np.random.default_rng(m + nnz)
    row, rowptr, col, val, colptr, csr2csc, (rp, c, v) = _torch_sparse_args(rng, m, n, nnz)
    X = rng.standard_normal((n, F)).astype(np.float32)
    mat = torch.from_numpy(X).to(DEV).requires_grad_(True)
    out = torch.ops.lpgnn.spmm_sum(row, rowptr, col, val, colptr, csr2csc, mat)
    assert np.array_equal(out.detach().cpu().numpy(), O.spmm_f32(rp, c, v, X))
    G = rng.standard_normal((m, F)).astype(np.float32)
    out.backward(torch.from_numpy(G).to(DEV))
    AT = O.csr_transpose(rp, c.astype(np.int32), v, m, n)
    assert np.array_equal(mat.grad.cpu().numpy(), O.spmm_f32(*AT, G))
    # row=None (derived from rowptr) and value=None (ones) as upstream allows
    mat2 = torch.from_numpy(X).to(DEV).requires_grad_(True)
    out2 = torch.ops.lpgnn.spmm_sum(None, rowptr, col, None, colptr, csr2csc, mat2)
    assert np.array_equal(out2.detach().cpu().numpy(), O.spmm_f32(rp, c, np.ones_like(v), X))
    out2.sum().backward()
    assert np.array_equal(mat2.grad.cpu().numpy(),
                          O.spmm_f32(*O.csr_transpose(rp, c.astype(np.int32), np.ones_like(v), m, n),
                                     np.ones((m, F), np.float32)))


def test_spmm_sum_errors_like_upstream():
    import lpgnn  # noqa: F401

    rng = np.random.default_rng(0)
    row, rowptr, col, val, colptr, csr2csc, _ = _torch_sparse_args(rng, 20, 30, 100)
    mat = torch.randn(30, 8, device=DEV, requires_grad=True)
    out = torch.ops.lpgnn.spmm_sum(row, rowptr, col, val, None, None, mat)
    with pytest.raises(RuntimeError, match="colptr and csr2csc"):
        out.sum().backward()
    v = val.clone().requires_grad_(True)
    out = torch.ops.lpgnn.spmm_sum(row, rowptr, col, v, colptr, csr2csc, mat)
    with pytest.raises(RuntimeError, match="edge values"):
        out.sum().backward()
    with pytest.raises(RuntimeError, match="2-D"):
        torch.ops.lpgnn.spmm_sum(row, rowptr, col, val, colptr, csr2csc, torch.randn(2, 30, 8, device=DEV))


def test_spmm_sum_opcheck():
    import lpgnn  # noqa: F401

    rng = np.random.default_rng(1)
    row, rowptr, col, val, colptr, csr2csc, _ = _torch_sparse_args(rng, 40, 60, 300)
    mat = torch.randn(60, 16, device=DEV, requires_grad=True)
    torch.library.opcheck(torch.ops.lpgnn.spmm_sum.default, (row, rowptr, col, val, colptr, csr2csc, mat),
                          test_utils=("test_schema", "test_autograd_registration", "test_faketensor"))


@pytest.mark.parametrize("M,C,weighted,ignore", [(100_000, 3, True, False), (777, 3, False, True), (5, 2, True, True),
                                                 (1, 4, True, False)])
def test_weighted_ce_matches_torch(M, C, weighted, ignore):
    """lpg_weighted_ce_{fwd,bwd}_f32 == coef * nn.CrossEntropyLoss(weight=w) (value and gradient)."""
    from lpgnn.train import weighted_ce

    g = torch.Generator().manual_seed(M)
    x = (torch.randn(M, C, generator=g) * 5).to(DEV)
    y = torch.randint(0, C, (M,), generator=g)
    if ignore:
        y[::3] = -100
    y = y.to(DEV)
    w = (torch.rand(C, generator=g) + 0.5).to(DEV) if weighted else None
    coef = 1.7
    xa = x.clone().requires_grad_(True)
    got = weighted_ce(xa, y, w, coef)
    (got * 0.3).backward()
    xr = x.clone().requires_grad_(True)
    ref = coef * torch.nn.CrossEntropyLoss(weight=w)(xr, y)
    (ref * 0.3).backward()
    torch.testing.assert_close(got, ref, rtol=2e-5, atol=1e-6)
    torch.testing.assert_close(xa.grad, xr.grad, rtol=1e-4, atol=1e-9)


def test_weighted_ce_bad_label_is_nan():
    from lpgnn.train import weighted_ce

    x = torch.randn(10, 3, device=DEV)
    y = torch.tensor([0, 1, 2, 3, 0, 1, 2, 0, 1, 2], device=DEV)
    assert torch.isnan(weighted_ce(x, y, None, 1.0)).item()
