"""GCN_FC forward + backward on degenerate LP graphs against the oracle (the reference's PyG path
restated in fp32, oracle/model_ref.py): one constraint and one variable, no edges at all, constraint
rows touching every variable, every edge on one variable, isolated nodes on both sides, and node
counts that are not multiples of any tile (arch.py:167-193; SpMM edge cases of torch_sparse's
spmm_cpu loop: empty rows give zeros)."""
import numpy as np
import pytest
import torch

from oracle import model_ref as O

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
LOGIT_ATOL = 1e-4


def _graph(kind, seed=0):
    from lpgnn import synth

    rs = np.random.default_rng(seed)
    if kind == "one_one":
        m, n, row, col = 1, 1, np.array([0]), np.array([0])
    elif kind == "no_edges":
        m, n, row, col = 5, 7, np.zeros(0, np.int64), np.zeros(0, np.int64)
    elif kind == "dense_rows":  # 3 constraints over all 1500 variables
        m, n = 3, 1500
        row, col = np.repeat(np.arange(m), n), np.tile(np.arange(n), m)
    elif kind == "star":  # every constraint touches variable 0 only (a 1000-edge variable row)
        m, n = 1000, 37
        row, col = np.arange(m), np.zeros(m, np.int64)
    elif kind == "isolated":  # a third of each side has no edge
        m, n = 301, 517
        row = rs.integers(0, 200, 2000)
        col = rs.integers(0, 340, 2000)
        key = np.unique(row * n + col)
        row, col = key // n, key % n
    else:
        raise ValueError(kind)
    row, col = np.asarray(row, np.int64), np.asarray(col, np.int64)
    val = rs.uniform(-1, 1, row.shape[0]).astype(np.float32)
    val[val == 0] = 0.5
    base = synth.uniform_lp(m, n, m, seed=seed)  # LP-layout features and labels only (its edges unused)
    return m, n, row, col, val, base.x_s, base.x_t, base.y_s, base.y_t


@pytest.mark.parametrize("kind", ["one_one", "no_edges", "dense_rows", "star", "isolated"])
@pytest.mark.parametrize("depth,hids", [(3, 64), (4, 256)])
def test_degenerate_graph_vs_oracle(kind, depth, hids):
    from lpgnn import BipartiteBatch, BipartiteCSR, GCN_FC
    from lpgnn.train import balanced

    m, n, row, col, val, x_s, x_t, y_s, y_t = _graph(kind)
    torch.manual_seed(0)
    model = GCN_FC(8, 8, hids=hids, depth=depth, dp=0.0).to(DEV)
    sd = {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}
    adj = BipartiteCSR.from_coo(row, col, val, m, n, device=DEV)
    batch = BipartiteBatch(x_s=torch.from_numpy(x_s).to(DEV), x_t=torch.from_numpy(x_t).to(DEV),
                           y_s=torch.from_numpy(y_s).to(DEV), y_t=torch.from_numpy(y_t).to(DEV),
                           edge_index=adj, s_bs=m, t_bs=n)
    model.train()
    lc, lv = model(batch)
    loss = balanced(lc, lv, batch.y_s, batch.y_t)
    loss.backward()
    A = O.csr_from_coo(row, col, val, m, n)
    AT = O.csr_transpose(*A, m, n)
    params = {k: v.clone().requires_grad_(True) for k, v in sd.items()}
    rc, rv = O.gcn_fc_forward(params, torch.from_numpy(x_s), torch.from_numpy(x_t), A, AT, depth)
    np.testing.assert_allclose(lc.detach().cpu().numpy(), rc.detach().numpy(), rtol=0, atol=LOGIT_ATOL)
    np.testing.assert_allclose(lv.detach().cpu().numpy(), rv.detach().numpy(), rtol=0, atol=LOGIT_ATOL)
    rloss = O.balanced(rc, rv, torch.from_numpy(y_s), torch.from_numpy(y_t))
    rloss.backward()
    assert abs(loss.item() - rloss.item()) <= 1e-4 * max(1.0, abs(rloss.item()))  # the balanced loss weights m+n over m
    for k, p in model.named_parameters():  # atol relative to the tensor's scale (a 1000-edge hub row)
        ref = params[k].grad.numpy()
        np.testing.assert_allclose(p.grad.cpu().numpy(), ref, rtol=2e-3, atol=2e-5 * max(1.0, float(np.abs(ref).max())),
                                   err_msg=k)
    # eval (the no-grad heads-only forward) and the device basis labels with their invariants
    from lpgnn.val import inference_gnn

    model.eval()
    with torch.no_grad():
        ec, ev = model(batch)
    with torch.no_grad():
        rc, rv = O.gcn_fc_forward({k: v.detach() for k, v in params.items()}, torch.from_numpy(x_s),
                                  torch.from_numpy(x_t), A, AT, depth)
    np.testing.assert_allclose(ec.cpu().numpy(), rc.numpy(), rtol=0, atol=LOGIT_ATOL)
    np.testing.assert_allclose(ev.cpu().numpy(), rv.numpy(), rtol=0, atol=LOGIT_ATOL)
    lab = inference_gnn(torch.cat((ec, ev)), m)  # asserts val.py:119-122's invariants
    assert lab.shape == (m + n,) and int((lab == 1).sum()) == m
