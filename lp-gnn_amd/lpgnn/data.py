"""Batch boundary: LPDataset.get -> MyToBipartite -> HIP dual-CSR pack.

The reference loads one LP per step as a homogeneous graph
(``UnipartiteData``, dataset.py:16-20, 229-264), and ``MyToBipartite``
(dataset.py:268-332) relabels it into a bipartite batch with
``x_s, x_t, y_s, y_t, edge_index: SparseTensor(m x n), bs, s_bs, t_bs``.
This module keeps that contract attribute for attribute; the only change is
the type of ``edge_index``: a :class:`~lpgnn.sparse.BipartiteCSR` packed
once (CSR(A) and CSR(A^T)) instead of a torch_sparse SparseTensor that is
transposed again in every layer.
"""
from __future__ import annotations

import numpy as np
import torch

from .sparse import BipartiteCSR


class UnipartiteData:
    """dataset.py:16-20 / 255-262: x, y, is_vars, edge_index (2,E), edge_attr."""

    def __init__(self, x, y, edge_index, edge_attr=None, is_vars=None, num_nodes=None, **aux):
        self.x, self.y, self.edge_index, self.edge_attr = x, y, edge_index, edge_attr
        self.is_vars = is_vars
        self.num_nodes = int(num_nodes if num_nodes is not None else x.shape[0])
        for k, v in aux.items():
            setattr(self, k, v)


class BipartiteBatch:
    """What MyToBipartite returns (dataset.py:307-326)."""

    _TENSORS = ("x_s", "x_t", "y_s", "y_t")

    def __init__(self, **kw):
        for k, v in kw.items():
            setattr(self, k, v)

    def __getitem__(self, k):  # batch_to (utils.py:909-915) indexes by name
        return getattr(self, k)

    def __setitem__(self, k, v):
        setattr(self, k, v)

    def to(self, device, non_blocking: bool = False) -> "BipartiteBatch":
        for k in self._TENSORS:
            if getattr(self, k, None) is not None:
                setattr(self, k, getattr(self, k).to(device, non_blocking=non_blocking))
        self.edge_index = self.edge_index.to(device, non_blocking=non_blocking)
        return self

    @property
    def num_nodes(self) -> int:
        return int(self.x_s.shape[0] + self.x_t.shape[0])


def to_undirected(edge_index: torch.Tensor, edge_attr: torch.Tensor, num_nodes: int):
    """PyG 2.1 ``to_undirected(edge_index, edge_attr)`` (dataset.py:252):
    both directions, coalesced (sorted by row*N + col, duplicates added)."""
    row = torch.cat([edge_index[0], edge_index[1]])
    col = torch.cat([edge_index[1], edge_index[0]])
    attr = torch.cat([edge_attr, edge_attr])
    key = row * num_nodes + col
    key, perm = torch.sort(key, stable=True)
    attr = attr[perm]
    uniq, inv = torch.unique_consecutive(key, return_inverse=True)
    summed = torch.zeros(uniq.numel(), dtype=attr.dtype).index_add_(0, inv, attr)
    return torch.stack([uniq // num_nodes, uniq % num_nodes]), summed


def lp_to_unipartite(row, col, A_data, c_feas, v_feas, y_s, y_t, **aux) -> UnipartiteData:
    """LPDataset.get after the msgpack load (dataset.py:234-264)."""
    A_data = np.asarray(A_data)
    c_feas = np.asarray(c_feas)
    assert A_data.max() <= 1 and A_data.min() >= -1  # dataset.py:235-236
    assert c_feas.max() <= 1 and c_feas.min() >= -1  # dataset.py:237-238
    ncons = c_feas.shape[0]
    nnodes = ncons + np.asarray(v_feas).shape[0]
    c_feas, v_feas, y_s, y_t = (torch.as_tensor(np.asarray(a)) for a in (c_feas, v_feas, y_s, y_t))
    edge_attr = torch.as_tensor(A_data).float()
    edge_index = torch.as_tensor(np.asarray([row, np.asarray(col) + ncons], dtype=np.int64))
    edge_index, edge_attr = to_undirected(edge_index, edge_attr, nnodes)
    is_vars = torch.zeros(nnodes, dtype=torch.long)
    is_vars[ncons:] = 1
    return UnipartiteData(x=torch.cat((c_feas, v_feas), 0), y=torch.cat((y_s, y_t), 0), is_vars=is_vars,
                          edge_index=edge_index, edge_attr=edge_attr, num_nodes=nnodes, **aux)


class MyToBipartite:
    """dataset.py:268-332, with the SparseTensor build replaced by the dual-CSR
    pack on ``dev`` ('cpu' = host pack in the loader worker, a HIP device =
    lpg_csr_pack_f32)."""

    def __init__(self, dev="cpu", phase="train", thresh_num=np.inf):
        self.dev = dev
        self.phase = phase
        self.thresh_num = thresh_num

    def __call__(self, batch):
        if hasattr(batch, "x_s"):  # already bipartite
            return batch
        if batch.edge_index.shape[-1] // 2 > self.thresh_num:
            return batch
        is_vars = batch.is_vars.bool()
        is_cons = ~is_vars
        nnodes = batch.num_nodes
        nvars = int(is_vars.sum().item())
        ncons = nnodes - nvars

        where = batch.edge_index.device
        mapping_vec = torch.empty(ncons + nvars, dtype=torch.long, device=where)
        mapping_vec[is_cons] = torch.arange(ncons, device=where)
        mapping_vec[is_vars] = torch.arange(nvars, device=where) + ncons
        edge_index = mapping_vec[batch.edge_index]

        edge_mask = edge_index[0, :] < ncons
        assert edge_mask.sum().item() * 2 == edge_mask.shape[0]  # dataset.py:297
        edge_index_l2r = edge_index[:, edge_mask].clone()
        edge_index_l2r[1, :] -= ncons
        # a batch already in HBM (the device NeighborLoader) is packed where it is
        pack_dev = where if where.type == "cuda" else self.dev
        adj = BipartiteCSR.from_edge_index(edge_index_l2r, batch.edge_attr[edge_mask], (ncons, nvars),
                                           device=pack_dev)
        bs = getattr(batch, "batch_size", None) or batch.num_nodes
        t_bs = int(batch.is_vars[:bs].sum().item())
        extra = {k: v for k, v in vars(batch).items()
                 if k not in ("x", "y", "edge_index", "edge_attr", "is_vars", "num_nodes", "batch", "batch_size")}
        return BipartiteBatch(x_s=batch.x[is_cons, :], x_t=batch.x[is_vars, :], y_s=batch.y[is_cons],
                              y_t=batch.y[is_vars], edge_index=adj, bs=bs, s_bs=bs - t_bs, t_bs=t_bs, **extra)


def bipartite_from_lp(row, col, A_data, c_feas, v_feas, y_s, y_t, device, **aux) -> BipartiteBatch:
    """LPDataset.get + MyToBipartite without the detour.

    The reference symmetrises the LP's edge list (to_undirected, dataset.py:252),
    relabels it and keeps only the cons->var half again (dataset.py:296-304).
    For a coalesced LP matrix -- one entry per (row, col), which scipy's CSR
    and the msgpack records hold -- that round trip returns the original
    entries, so the dual CSR is packed straight from (row, col, value) on
    `device` (one device sort, no host coalesce over 2·nnz edges).  The result
    equals the reference chain attribute for attribute (tests/test_lpio.py);
    an LP with duplicate entries takes the reference chain, which sums them.
    """
    A_data = np.asarray(A_data)
    c_feas, v_feas = np.asarray(c_feas), np.asarray(v_feas)
    assert A_data.max() <= 1 and A_data.min() >= -1  # dataset.py:235-236
    assert c_feas.max() <= 1 and c_feas.min() >= -1  # dataset.py:237-238
    m, n = c_feas.shape[0], v_feas.shape[0]
    try:
        adj = BipartiteCSR.from_coo(np.asarray(row, np.int64), np.asarray(col, np.int64),
                                    A_data.astype(np.float32), m, n, device=device)
    except RuntimeError as e:
        if "duplicate" not in str(e):
            raise
        return MyToBipartite(dev=device)(lp_to_unipartite(row, col, A_data, c_feas, v_feas, y_s, y_t, **aux))
    t = lambda a: torch.as_tensor(np.asarray(a))
    return BipartiteBatch(x_s=t(c_feas), x_t=t(v_feas), y_s=t(y_s), y_t=t(y_t), edge_index=adj, bs=m + n,
                          s_bs=m, t_bs=n, **aux)


def batch_to(batch, dev, half: bool = False):
    """utils.py:909-915.  ``half``: the features and the adjacency's values to fp16 (SparseTensor.half());
    the labels stay int64 (the reference casts them to half too, which only its accuracy reads)."""
    for nm in ("x_s", "x_t", "y_s", "y_t"):
        t = batch[nm]
        if half and t.is_floating_point():
            t = t.half()
        batch[nm] = t.to(dev)
    adj = batch["edge_index"].to(dev)
    batch["edge_index"] = adj.half() if half and hasattr(adj, "half") else adj
    return batch
