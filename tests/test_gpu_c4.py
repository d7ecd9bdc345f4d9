"""c4 at full size on ONE GPU (BASELINE.json configs[3]: 2M cons x 4M vars, nnz 40M, hid 1024,
depth 3 -- the regime the reference sends to NeighborLoader, train.py:103-116, utils.py:808).

The whole graph trains on one MI355X (116 GB of HBM).  At this size the oracle cannot evaluate
the network in test time, so the checks are size-independent properties plus sampled exact ones:

* the F = 1024 SpMM in both directions: 2000 sampled rows per direction BITWISE equal to the
  oracle's torch_sparse spmm_cpu loop (the rows' own edges, gathered from the same X), plus
  linearity (A(x + y) vs Ax + Ay within one fp32 rounding per edge) on the whole output;
* one training step (fwd + balanced loss + bwd + Adam): a finite positive loss, every gradient
  finite and nonzero, the step changes every parameter, and the
  same step run twice from the same state gives the same bits (fixed-order reductions)."""
import numpy as np
import pytest
import torch

from oracle import model_ref as O

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(900)]
DEV = "cuda:0"
_CACHE = {}


def _graph():
    if "g" not in _CACHE:
        from lpgnn import synth

        _CACHE["g"] = synth.c4_spec().full()
    return _CACHE["g"]


def _sub_csr(rowptr, col, val, rows):
    """The sampled rows' CSR with columns renumbered over the distinct sources they touch."""
    lens = rowptr[rows + 1] - rowptr[rows]
    idx = np.concatenate([np.arange(rowptr[r], rowptr[r + 1]) for r in rows]).astype(np.int64)
    srcs, local = np.unique(col[idx], return_inverse=True)
    sub_rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    return sub_rp, local.astype(np.int32), val[idx].astype(np.float32), srcs


@pytest.mark.parametrize("direction", ["cons<-vars", "vars<-cons"])
def test_c4_spmm_sampled_rows_bitwise(direction):
    from lpgnn import BipartiteCSR
    from lpgnn.sparse import spmm_forward

    g = _graph()
    adj = BipartiteCSR.from_coo(g.row, g.col, g.val, g.m, g.n, device=DEV)
    csr, n_src = (adj.fwd, g.n) if direction == "cons<-vars" else (adj.bwd, g.m)
    gen = torch.Generator(device=DEV).manual_seed(11)
    X = torch.randn(n_src, 1024, device=DEV, generator=gen)
    Y = spmm_forward(csr, X)
    rp, col, val = csr.rowptr.cpu().numpy(), csr.col.cpu().numpy(), csr.val.cpu().numpy()
    rows = np.sort(np.random.default_rng(5).choice(csr.n_rows, 2000, replace=False))
    sub_rp, sub_col, sub_val, srcs = _sub_csr(rp, col, val, rows)
    Xs = X[torch.from_numpy(srcs).to(DEV)].cpu().numpy()
    want = O.spmm_f32(sub_rp, sub_col, sub_val, Xs)
    got = Y[torch.from_numpy(rows).to(DEV)].cpu().numpy()
    assert np.array_equal(got, want)
    # linearity over the whole output: A(X + Z) = AX + AZ to one rounding per edge
    Z = torch.randn(n_src, 1024, device=DEV, generator=gen)
    lhs = spmm_forward(csr, X + Z)
    rhs = Y + spmm_forward(csr, Z)
    absA = BipartiteCSR.from_coo(g.row, g.col, np.abs(g.val), g.m, g.n, device=DEV)
    acsr = absA.fwd if direction == "cons<-vars" else absA.bwd
    bound = spmm_forward(acsr, X.abs() + Z.abs())
    deg = (csr.rowptr[1:] - csr.rowptr[:-1]).to(torch.float32)[:, None]
    assert bool(((lhs - rhs).abs() <= (deg + 2) * 2.0 ** -23 * bound + 1e-30).all())


def test_c4_training_step_properties():
    from lpgnn import BipartiteBatch, BipartiteCSR, GCN_FC
    from lpgnn.train import make_optimizer, train_step

    g = _graph()
    adj = BipartiteCSR.from_coo(g.row, g.col, g.val, g.m, g.n, device=DEV)
    batch = BipartiteBatch(x_s=torch.from_numpy(g.x_s).to(DEV), x_t=torch.from_numpy(g.x_t).to(DEV),
                           y_s=torch.from_numpy(g.y_s).to(DEV), y_t=torch.from_numpy(g.y_t).to(DEV),
                           edge_index=adj, s_bs=g.m, t_bs=g.n)
    torch.manual_seed(0)
    model = GCN_FC(8, 8, hids=1024, depth=3).to(DEV)
    opt, _ = make_optimizer(model)
    before = {k: v.detach().clone() for k, v in model.state_dict().items()}

    def one_step(o):
        torch.manual_seed(1)  # the dropout seeds
        return train_step(model, batch, o).item()

    loss = one_step(opt)
    # the balanced loss (train.py:39-46) of a fresh network on add_knowledge logits in [-20, 10]
    assert np.isfinite(loss) and 0 < loss < 100, loss
    for k, p in model.named_parameters():
        assert p.grad is not None and bool(torch.isfinite(p.grad).all()) and p.grad.abs().sum().item() > 0, k
        assert not torch.equal(p.detach(), before[k]), f"{k} unchanged by the Adam step"
    grads1 = {k: p.grad.detach().clone() for k, p in model.named_parameters()}
    after1 = {k: v.detach().clone() for k, v in model.state_dict().items()}
    # the same step again from the same state (fresh Adam): the same bits (no atomics on float
    # data, fixed-order folds)
    model.load_state_dict(before)
    opt2, _ = make_optimizer(model)
    assert one_step(opt2) == loss
    for k, p in model.named_parameters():
        assert torch.equal(p.grad, grads1[k]), k
    for k, v in model.state_dict().items():
        assert torch.equal(v, after1[k]), k
