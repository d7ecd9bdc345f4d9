"""k-hop NeighborLoader on the device (train.py:103-116, val.py:12-27).

The reference hands graphs above MyToBipartite's threshold to PyG 2.1's
``NeighborLoader(data, num_neighbors, input_nodes=None, directed=False,
shuffle, transform=MyToBipartite(thresh_num=inf), batch_size, ...)``, which
samples on the host in C++ (torch_sparse 0.6.12 ``neighbor_sample``) inside
DataLoader workers.  Here the graph's CSC lives in HBM and every hop is a
handful of HIP kernels (csrc/sample.hip, ``lpg_sample_*``); the only host
round trips are the per-hop sizes.

Semantics kept (oracle/model_ref.py:neighbor_sample restates them):
  * node list = seeds, then each hop's new nodes in first-appearance order
    (frontier order, neighbours in CSC = ascending-source order);
  * fanout -1 takes every neighbour; k samples min(k, deg) distinct
    neighbours (Floyd's algorithm; our counter-based RNG, so the particular
    draws differ from torch_sparse's -- the distribution is the same);
  * directed=False returns the subgraph induced on the sampled nodes (both
    call sites use it); directed=True the sampled edges only;
  * the batch is a UnipartiteData with x/y/is_vars/edge_attr sliced,
    ``batch_size`` = number of seeds (MyToBipartite turns it into s_bs/t_bs).
``num_workers`` / ``pin_memory`` / ``prefetch_factor`` are accepted and
ignored: there is no worker pool to feed.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from . import _lib
from .data import UnipartiteData


def to_csc(edge_index: torch.Tensor, num_nodes: int):
    """PyG 2.1 ``to_csc``: in-edges of each node sorted by source.
    Returns (colptr [N+1], row [E], perm [E]) with row = edge_index[0][perm]."""
    row, col = edge_index[0].long(), edge_index[1].long()
    perm = torch.argsort(col * num_nodes + row, stable=True)
    colptr = torch.searchsorted(col[perm], torch.arange(num_nodes + 1, device=col.device))
    return colptr.contiguous(), row[perm].contiguous(), perm


class NeighborSampler:
    """Device k-hop sampler over one graph (CSC + per-graph scratch in HBM)."""

    def __init__(self, edge_index: torch.Tensor, num_nodes: int, num_neighbors, directed: bool = True,
                 device=None, seed: int | None = None):
        self.device = torch.device(device) if device is not None else edge_index.device
        if self.device.type != "cuda":
            raise RuntimeError("NeighborSampler runs on a HIP device; there is no CPU sampler in lpgnn")
        self.num_nodes = int(num_nodes)
        self.num_neighbors = [int(k) for k in num_neighbors]
        if any(k > 256 for k in self.num_neighbors):
            raise ValueError("fanouts above 256 are not supported (use -1 for all neighbours)")
        self.directed = bool(directed)
        self.colptr, self.row, self.perm = to_csc(edge_index.to(self.device), self.num_nodes)
        self.local = torch.full((self.num_nodes,), -1, dtype=torch.int64, device=self.device)
        self.first = torch.full((self.num_nodes,), -1, dtype=torch.int64, device=self.device)  # = UINT64_MAX
        self._rng = np.random.default_rng(seed)

    # -- helpers -----------------------------------------------------------
    def _stream(self):
        return torch.cuda.current_stream(self.device).cuda_stream

    def _scan(self, x: torch.Tensor) -> torch.Tensor:
        L = _lib.lib()
        n = x.numel()
        out = torch.empty(n + 1, dtype=torch.int64, device=self.device)
        nb = int(L.lpg_scan_i64_workspace_bytes(n))
        ws = torch.empty(max(nb, 1), dtype=torch.uint8, device=self.device)
        _lib.check(L.lpg_scan_i64(_lib.ptr(x) if n else None, n, out.data_ptr(), ws.data_ptr(), nb, self._stream()),
                   "lpg_scan_i64")
        return out

    def _empty(self, n: int) -> torch.Tensor:
        return torch.empty(max(int(n), 0), dtype=torch.int64, device=self.device)

    @staticmethod
    def _p(t: torch.Tensor):
        return t.data_ptr() if t.numel() else None

    def _add_new(self, cand: torch.Tensor, base: int) -> torch.Tensor:
        """Dedupe candidates against the sampled set; append the new ones."""
        L, p, st = _lib.lib(), self._p, self._stream()
        nc = cand.numel()
        flag = self._empty(nc)
        _lib.check(L.lpg_sample_dedupe(p(cand), nc, self.local.data_ptr(), self.first.data_ptr(), p(flag), st),
                   "lpg_sample_dedupe")
        rank = self._scan(flag)
        n_new = int(rank[-1].item())
        chunk = self._empty(max(n_new, 1))  # never written when nothing is new
        _lib.check(L.lpg_sample_assign(p(cand), nc, base, p(flag), rank.data_ptr(), p(chunk), self.local.data_ptr(),
                                       self.first.data_ptr(), st), "lpg_sample_assign")
        return chunk[:n_new]

    # -- torch_sparse.neighbor_sample(colptr, row, input_node, num_neighbors, replace=False, directed) ------
    @torch.no_grad()
    def sample(self, index: torch.Tensor):
        """-> (node, row, col, edge): sampled global node ids, local edge
        endpoints (row = source, col = destination) and CSC edge positions."""
        L, p, st = _lib.lib(), self._p, self._stream()
        index = index.to(self.device, torch.int64).contiguous()
        chunks = [self._add_new(index, 0)]
        if chunks[0].numel() != index.numel():
            raise ValueError("input nodes of a batch must be distinct")
        begin, total = 0, index.numel()
        rows, cols, edges = [], [], []
        for k in self.num_neighbors:
            frontier = chunks[-1]
            nf = frontier.numel()
            if nf == 0:
                break
            counts = self._empty(nf)
            _lib.check(L.lpg_sample_count(p(frontier), nf, self.colptr.data_ptr(), k, p(counts), st),
                       "lpg_sample_count")
            offs = self._scan(counts)
            nc = int(offs[-1].item())
            if nc == 0:  # the frontier has no in-edges: nothing further to reach
                break
            cand, cand_edge, cand_dst = self._empty(nc), self._empty(nc), self._empty(nc)
            hop_seed = int(self._rng.integers(0, 2 ** 63))
            _lib.check(L.lpg_sample_fill(p(frontier), nf, begin, self.colptr.data_ptr(), self.row.data_ptr(), k,
                                         hop_seed, offs.data_ptr(), p(cand), p(cand_edge), p(cand_dst), st),
                       "lpg_sample_fill")
            chunks.append(self._add_new(cand, total))
            if self.directed:
                lr = self._empty(nc)
                _lib.check(L.lpg_sample_local_ids(p(cand), nc, self.local.data_ptr(), p(lr), st),
                           "lpg_sample_local_ids")
                rows.append(lr), cols.append(cand_dst), edges.append(cand_edge)
            begin, total = total, total + chunks[-1].numel()
        node = torch.cat(chunks)
        ns = node.numel()
        if self.directed:
            row = torch.cat(rows) if rows else self._empty(0)
            col = torch.cat(cols) if cols else self._empty(0)
            edge = torch.cat(edges) if edges else self._empty(0)
        else:
            counts = self._empty(ns)
            _lib.check(L.lpg_induced_count(p(node), ns, self.colptr.data_ptr(), self.row.data_ptr(),
                                           self.local.data_ptr(), p(counts), st), "lpg_induced_count")
            offs = self._scan(counts)
            ne = int(offs[-1].item())
            row, col, edge = self._empty(ne), self._empty(ne), self._empty(ne)
            if ne:
                _lib.check(L.lpg_induced_fill(p(node), ns, self.colptr.data_ptr(), self.row.data_ptr(),
                                              self.local.data_ptr(), offs.data_ptr(), p(row), p(col), p(edge), st),
                           "lpg_induced_fill")
        _lib.check(L.lpg_sample_reset(p(node), ns, self.local.data_ptr(), st), "lpg_sample_reset")
        return node, row, col, edge


class NeighborLoader:
    """PyG 2.1 ``NeighborLoader`` over one homogeneous LP graph, sampled on the GPU."""

    def __init__(self, data: UnipartiteData, num_neighbors, input_nodes=None, directed: bool = True,
                 shuffle: bool = False, transform=None, batch_size: int = 1, drop_last: bool = False,
                 device=None, seed: int | None = None, replace: bool = False, **_loader_kwargs):
        if replace:
            raise NotImplementedError("sampling with replacement is not used by the reference (replace=False)")
        self.device = torch.device(device) if device is not None else (
            data.x.device if data.x.is_cuda else torch.device("cuda", torch.cuda.current_device()))
        self.data = data
        N = int(data.num_nodes)
        self.sampler = NeighborSampler(data.edge_index, N, num_neighbors, directed, self.device, seed)
        dev = self.device
        self._x, self._y = data.x.to(dev), data.y.to(dev)
        self._is_vars = data.is_vars.to(dev) if getattr(data, "is_vars", None) is not None else None
        self._edge_attr = data.edge_attr.to(dev) if getattr(data, "edge_attr", None) is not None else None
        if input_nodes is None:
            inp = torch.arange(N, device=dev)
        else:
            inp = torch.as_tensor(input_nodes, device=dev)
            inp = inp.nonzero().view(-1) if inp.dtype == torch.bool else inp.long()
        self.input_nodes = inp
        self.batch_size, self.shuffle, self.drop_last = int(batch_size), bool(shuffle), bool(drop_last)
        self.transform = transform
        self._gen = torch.Generator(device="cpu")
        self._gen.manual_seed(int(np.random.default_rng(seed).integers(0, 2 ** 62)))

    def __len__(self) -> int:
        n = self.input_nodes.numel()
        return n // self.batch_size if self.drop_last else math.ceil(n / self.batch_size)

    def filter(self, index, node, row, col, edge) -> UnipartiteData:
        """PyG ``filter_data``: slice node and edge attributes."""
        edge_attr = None if self._edge_attr is None else self._edge_attr[self.sampler.perm[edge]]
        return UnipartiteData(x=self._x[node], y=self._y[node], edge_index=torch.stack([row, col]),
                              edge_attr=edge_attr,
                              is_vars=None if self._is_vars is None else self._is_vars[node],
                              num_nodes=node.numel(), batch_size=index.numel(), n_id=node, input_id=index)

    def __iter__(self):
        n = self.input_nodes.numel()
        order = torch.randperm(n, generator=self._gen).to(self.device) if self.shuffle else None
        for s in range(0, len(self) * self.batch_size, self.batch_size):
            sl = slice(s, min(s + self.batch_size, n))
            index = self.input_nodes[order[sl]] if order is not None else self.input_nodes[sl]
            sub = self.filter(index, *self.sampler.sample(index))
            yield self.transform(sub) if self.transform is not None else sub
