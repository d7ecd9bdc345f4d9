"""Generate the committed golden fixtures under tests/golden/.

Run HERE (the CPU container, where /root/reference exists):

    python tests/golden/make_golden.py

What is pinned by the REFERENCE's own code: the script parses the reference
sources with ``ast`` and executes only the named top-level function / class
bodies (never the modules: utils.py's import-time ``pip install`` and the
absent torch_geometric / torch_sparse imports are never executed):

  arch.py   add_knowledge (129-141), GraphConvTwoDirection (51-81),
            GCNBase (108-114), GCN_FC (167-193)
  val.py    inference_gnn (106-124)
  train.py  balanced (39-46)
  utils.py  labels_to_balanced_weights (286-299)
  dataset.py MyToBipartite.__call__ (275-332), scaling (23-76), cvt_to_features (79-96)
  utils.py  sparse_mat_div_by_vec, count_nonzero_sparse_mat, cos_sim_*, expand_inf,
            concatenate_on_lst_dim (323-384)

The names those bodies reference but the reference does not define are
supplied from oracle/model_ref.py (the restatement of the un-vendored
upstream: PyG 2.1 GraphConv with torch_sparse 0.6.12 spmm_sum) or are small
recorders (a SparseTensor stand-in whose ``from_edge_index`` only records its
arguments, and an edge_index object whose ``.t()`` swaps orientation).  So
these fixtures pin the reference's orchestration, direction convention,
masking, top-m rule, loss weighting and relabelling; the upstream arithmetic
itself stays "parity unpinned" (DESIGN.md).

No reference source text is stored: only inputs and outputs (npz).
"""
from __future__ import annotations

import ast
import os
import sys
import types

import numpy as np
import torch
import torch.nn.functional as F
from torch import nn

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
from oracle import model_ref as O  # noqa: E402


def extract(path: str, names: list[str], ns: dict) -> dict:
    """Exec only the listed top-level defs of `path` inside namespace `ns`."""
    src = open(path).read()
    tree = ast.parse(src)
    keep = [n for n in tree.body if isinstance(n, (ast.FunctionDef, ast.ClassDef)) and n.name in names]
    found = {n.name for n in keep}
    missing = set(names) - found
    assert not missing, f"{path}: missing {missing}"
    mod = ast.Module(body=keep, type_ignores=[])
    exec(compile(mod, path, "exec"), ns)
    return ns


# ----------------------------------------------------------------- stand-ins
class OracleGraphConv(nn.Module):
    """PyG 2.1 GraphConv((in_src, in_dst), out) restated (aggr='add')."""

    def __init__(self, in_channels, out_channels, **kw):
        super().__init__()
        s, d = in_channels
        self.lin_rel = nn.Linear(s, out_channels, bias=True)
        self.lin_root = nn.Linear(d, out_channels, bias=False)

    def forward(self, x, adj_t, edge_weight=None):
        agg = O.spmm_t(adj_t.csr, adj_t.t().csr, x[0])
        out = self.lin_rel(agg)
        out = out + self.lin_root(x[1])
        return out


class EdgeIndex:
    """Stand-in for the SparseTensor(m x n) edge_index: .t() swaps."""

    def __init__(self, csr, csr_t):
        self.csr, self._t = csr, csr_t

    def t(self):
        return EdgeIndex(self._t, self.csr)


class RecordingSparseTensor:
    calls = []

    @classmethod
    def from_edge_index(cls, edge_index, edge_attr=None, sparse_sizes=None):
        cls.calls.append((edge_index.clone(), edge_attr.clone(), tuple(sparse_sizes)))
        return ("SparseTensor", len(cls.calls) - 1)


def ref_namespace():
    ns = {"torch": torch, "F": F, "nn": nn, "np": np, "GraphConv": OracleGraphConv,
          "BaseTransform": object, "SparseTensor": RecordingSparseTensor}
    extract(f"{REF}/utils.py", ["labels_to_balanced_weights"], ns)
    extract(f"{REF}/arch.py", ["GraphConvTwoDirection", "GCNBase", "add_knowledge", "GCN_FC"], ns)
    extract(f"{REF}/val.py", ["inference_gnn"], ns)
    extract(f"{REF}/train.py", ["balanced"], ns)
    extract(f"{REF}/dataset.py", ["MyToBipartite", "scaling", "cvt_to_features"], ns)
    extract(f"{REF}/utils.py", ["sparse_mat_div_by_vec", "count_nonzero_sparse_mat", "cos_sim_vec_and_sparse_mat",
                                "cos_sim_sparse_mat_and_vec", "expand_inf", "concatenate_on_lst_dim"], ns)
    return ns


# ------------------------------------------------------------------ inputs
def lp_features(rng, k, p_lo, p_hi):
    """[k, 8] features, layout of dataset.py:79-96 + utils.py:368-374."""
    x = np.zeros((k, 8), np.float32)
    x[:, :4] = rng.uniform(-1, 1, (k, 4))
    x[:, 5] = -(rng.random(k) < p_lo).astype(np.float32)
    x[:, 4] = np.where(x[:, 5] != 0, 0, rng.uniform(-1, 1, k))
    x[:, 7] = (rng.random(k) < p_hi).astype(np.float32)
    x[:, 6] = np.where(x[:, 7] != 0, 0, rng.uniform(-1, 1, k))
    return x


def make_graph_fixture(rng, m, n, nnz):
    keys = np.sort(rng.choice(m * n, size=nnz, replace=False))
    row, col = keys // n, keys % n
    # edge cases: an empty constraint row, an empty variable column, a dense row
    sel = (row != 1) & (col != 2) & (row != 0)
    row, col = row[sel], col[sel]
    row = np.concatenate([row, np.zeros(n - 1, np.int64)])
    col = np.concatenate([col, np.delete(np.arange(n), 2)])
    val = rng.uniform(-1, 1, size=len(row)).astype(np.float32)
    val[val == 0] = 0.25
    perm = rng.permutation(len(row))  # arbitrary COO order in, CSR order out
    return row[perm].astype(np.int64), col[perm].astype(np.int64), val[perm]


def main():
    torch.set_num_threads(4)
    rng = np.random.default_rng(1234)
    ns = ref_namespace()


    # ---- SpMM: tiny graph, several widths (oracle C loop; drift detector) ----
    m, n = 64, 128
    row, col, val = make_graph_fixture(rng, m, n, 512)
    A = O.csr_from_coo(row, col, val, m, n)
    AT = O.csr_transpose(*A, m, n)
    sp = dict(coo_row=row, coo_col=col, coo_val=val, m=m, n=n,
              a_rowptr=A[0], a_col=A[1], a_val=A[2], at_rowptr=AT[0], at_col=AT[1], at_val=AT[2])
    for Fd in (1, 8, 40, 256, 1024):
        Xv = rng.standard_normal((n, Fd)).astype(np.float32)
        Xc = rng.standard_normal((m, Fd)).astype(np.float32)
        sp[f"Xv_{Fd}"], sp[f"Xc_{Fd}"] = Xv, Xc
        sp[f"Yc_{Fd}"] = O.spmm_f32(*A, Xv)      # cons <- vars
        sp[f"Yv_{Fd}"] = O.spmm_f32(*AT, Xc)     # vars <- cons
    np.savez_compressed(os.path.join(HERE, "spmm_small.npz"), **sp)

    # ---- GCN_FC via the reference's own class bodies ----
    for depth, hids in ((3, 32), (4, 16)):
        m, n = 48, 96
        row, col, val = make_graph_fixture(rng, m, n, 400)
        A = O.csr_from_coo(row, col, val, m, n)
        AT = O.csr_transpose(*A, m, n)
        x_s = torch.from_numpy(lp_features(rng, m, 0.5, 0.5))
        x_t = torch.from_numpy(lp_features(rng, n, 0.1, 0.7))
        y_s = torch.from_numpy(rng.integers(0, 3, m))
        y_t = torch.from_numpy(rng.integers(0, 3, n))
        torch.manual_seed(0)
        model = ns["GCN_FC"](8, 8, hids=hids, depth=depth, dp=0.0)
        batch = types.SimpleNamespace(x_s=x_s, x_t=x_t, edge_index=EdgeIndex(A, AT))
        model.eval()
        with torch.no_grad():
            lc, lv = model(batch)
        labels = ns["inference_gnn"](torch.cat((lc, lv), 0), m)
        model.train()
        lc2, lv2 = model(batch)
        loss = ns["balanced"](lc2, lv2, y_s, y_t)
        model.zero_grad()
        loss.backward()
        fx = dict(m=m, n=n, depth=depth, hids=hids, coo_row=row, coo_col=col, coo_val=val,
                  x_s=x_s.numpy(), x_t=x_t.numpy(), y_s=y_s.numpy(), y_t=y_t.numpy(),
                  logit_cons=lc.numpy(), logit_vars=lv.numpy(), labels=labels.numpy(),
                  loss=np.float32(loss.item()))
        for k, v in model.state_dict().items():
            fx["sd." + k] = v.numpy()
        for k, p in model.named_parameters():
            fx["grad." + k] = p.grad.numpy()
        np.savez_compressed(os.path.join(HERE, f"gcn_fc_d{depth}_h{hids}.npz"), **fx)

    # ---- post-processing and loss (reference bodies) ----
    post = {}
    for i, (m, n) in enumerate(((30, 50), (7, 13), (100, 40))):
        logits = torch.randn(m + n, 3) * 5
        if i == 1:
            logits[3] = float("nan")  # half-model NaN path, val.py:111
        feas_l = torch.from_numpy(lp_features(rng, m, 0.5, 0.5))
        feas_r = torch.from_numpy(lp_features(rng, n, 0.1, 0.7))
        kl, kr = ns["add_knowledge"](logits[:m].clone(), logits[m:].clone(), feas_l, feas_r)
        post[f"logits_{i}"], post[f"m_{i}"] = logits.numpy(), m
        post[f"feas_l_{i}"], post[f"feas_r_{i}"] = feas_l.numpy(), feas_r.numpy()
        post[f"know_l_{i}"], post[f"know_r_{i}"] = kl.numpy(), kr.numpy()
        post[f"pred_{i}"] = ns["inference_gnn"](torch.cat((kl, kr), 0), m).numpy()
    for i, labels in enumerate((np.array([0, 1, 2, 1, 1, 0, 2, 2, 1]), np.array([0, 1, 1, 0, 1]),
                                np.array([1, 1, 1]), np.array([2, 1, 2, 2]))):
        post[f"bw_in_{i}"] = labels
        post[f"bw_out_{i}"] = ns["labels_to_balanced_weights"](torch.from_numpy(labels)).numpy()
    lc, lv = torch.randn(20, 3), torch.randn(35, 3)
    ys, yt = torch.from_numpy(rng.integers(0, 3, 20)), torch.from_numpy(rng.integers(0, 3, 35))
    post.update(bal_lc=lc.numpy(), bal_lv=lv.numpy(), bal_ys=ys.numpy(), bal_yt=yt.numpy(),
                bal_loss=np.float32(ns["balanced"](lc, lv, ys, yt).item()))
    np.savez_compressed(os.path.join(HERE, "post_small.npz"), **post)

    # ---- MyToBipartite (dataset.py:275-332) on an LPDataset.get-style graph ----
    m, n = 20, 31
    keys = np.sort(rng.choice(m * n, size=90, replace=False))
    r, c = keys // n, keys % n
    a = rng.uniform(-1, 1, 90).astype(np.float32)
    nn_ = m + n
    ei, ea = O.to_undirected(np.stack([r, c + m]), a, nn_)  # dataset.py:250-252
    perm_nodes = rng.permutation(nn_)  # NeighborLoader-style interleaved node order
    inv = np.empty_like(perm_nodes)
    inv[perm_nodes] = np.arange(nn_)
    x = rng.standard_normal((nn_, 8)).astype(np.float32)[perm_nodes]
    y = rng.integers(0, 3, nn_)[perm_nodes]
    is_vars = (perm_nodes >= m).astype(np.int64)
    ei_p = inv[ei]
    batch = types.SimpleNamespace(x=torch.from_numpy(x), y=torch.from_numpy(y),
                                  is_vars=torch.from_numpy(is_vars), edge_index=torch.from_numpy(ei_p.copy()),
                                  edge_attr=torch.from_numpy(ea), num_nodes=nn_, batch=None)
    RecordingSparseTensor.calls.clear()
    res = ns["MyToBipartite"].__call__(types.SimpleNamespace(thresh_num=np.inf, phase="val"), batch)
    (l2r, l2r_attr, sizes), = RecordingSparseTensor.calls
    np.savez_compressed(os.path.join(HERE, "bipartite_small.npz"),
                        x=x, y=y, is_vars=is_vars, edge_index=ei_p, edge_attr=ea, num_nodes=nn_,
                        x_s=res.x_s.numpy(), x_t=res.x_t.numpy(), y_s=res.y_s.numpy(), y_t=res.y_t.numpy(),
                        l2r=l2r.numpy(), l2r_attr=l2r_attr.numpy(), sizes=np.array(sizes),
                        s_bs=res.s_bs, t_bs=res.t_bs)
    # ---- LP scaling + node features (dataset.py:23-96 with utils.py helpers) ----
    import scipy.sparse as sp

    feats = {}
    for i, (m, n, nnz) in enumerate(((12, 20, 60), (40, 25, 200))):
        keys = np.sort(rng.choice(m * n, size=nnz, replace=False))
        r, c = keys // n, keys % n
        r = r[r != m - 1]  # an empty constraint row
        c = c[:len(r)]
        data = rng.normal(0, 50, len(r))
        cvec = rng.normal(0, 10, n)
        b_l = rng.normal(-5, 20, m)
        b_u = b_l + rng.uniform(0, 30, m)
        b_l[rng.random(m) < 0.4] = -np.inf
        b_u[rng.random(m) < 0.4] = np.inf
        b_l[0] = -1e309  # < -1e308 -> -inf (dataset.py:25)
        l_ = np.where(rng.random(n) < 0.7, 0.0, -np.inf)
        u_ = np.where(rng.random(n) < 0.5, np.inf, rng.uniform(1, 100, n))
        A = sp.coo_matrix((data, (r, c)), shape=(m, n)).tocsr()
        args = [x.copy() for x in (cvec, b_l)] + [A.copy()] + [x.copy() for x in (b_u, l_, u_)]
        cs, bls, As, bus, ls, us = ns["scaling"](*args)
        v_f, c_f = ns["cvt_to_features"](cs, bls, As, bus, ls, us)
        Ac = As.tocoo()
        feats.update({f"in_row_{i}": r, f"in_col_{i}": c, f"in_data_{i}": data, f"in_c_{i}": cvec,
                      f"in_bl_{i}": b_l, f"in_bu_{i}": b_u, f"in_l_{i}": l_, f"in_u_{i}": u_,
                      f"m_{i}": m, f"n_{i}": n, f"out_row_{i}": Ac.row, f"out_col_{i}": Ac.col,
                      f"out_data_{i}": Ac.data, f"out_c_{i}": cs, f"v_feas_{i}": v_f, f"c_feas_{i}": c_f})
    np.savez_compressed(os.path.join(HERE, "features_small.npz"), **feats)
    print("wrote", sorted(f for f in os.listdir(HERE) if f.endswith(".npz")))


if __name__ == "__main__":
    main()
