"""Bipartite adjacency (dual CSR) and the differentiable HIP SpMM.

Replaces, for the GCN_FC hot path:

* ``torch_sparse.SparseTensor`` as the batch's ``edge_index``
  (dataset.py:301-304) and its per-layer ``.t()`` (arch.py:71):
  :class:`BipartiteCSR` holds CSR(A) and CSR(A^T) on the device, packed once
  (``lpg_csr_pack_f32``), and ``.t()`` just swaps the two views;
* ``torch_sparse.matmul(adj_t, x, reduce='add')`` -> ``spmm_sum`` and its
  autograd ``SPMMSum`` (PyG GraphConv.message_and_aggregate, arch.py:75-80):
  :func:`spmm` -- forward ``lpg_spmm_f32(adj)``, backward
  ``lpg_spmm_f32(adj.t())`` (no gradient w.r.t. edge values, which the
  reference never trains: dataset.py:250).

All compute runs in liblpgnn_hip.so on the tensor's current HIP stream.
There is no CPU path: a CPU tensor raises.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np
import torch

from . import _lib
from .timing import TIMER


@dataclass
class CSR:
    """One orientation: rows = destination nodes, cols = source nodes."""

    rowptr: torch.Tensor  # int64 [n_rows+1]
    col: torch.Tensor     # int32 [nnz]
    val: torch.Tensor     # f32 [nnz]
    n_rows: int
    n_cols: int

    def __post_init__(self):
        self._c = None

    @property
    def nnz(self) -> int:
        return int(self.col.numel())

    @property
    def device(self) -> torch.device:
        return self.rowptr.device

    def cstruct(self) -> _lib.LpgCsr:
        if self._c is None:
            self._c = _lib.LpgCsr(self.n_rows, self.n_cols, self.nnz, self.rowptr.data_ptr(),
                                  self.col.data_ptr() if self.nnz else None,
                                  self.val.data_ptr() if self.nnz else None)
        return self._c

    def to(self, device) -> "CSR":
        return CSR(self.rowptr.to(device), self.col.to(device), self.val.to(device), self.n_rows, self.n_cols)

    def degrees(self) -> torch.Tensor:
        return self.rowptr[1:] - self.rowptr[:-1]

    def heavy_rows(self, thresh: int):
        """(int32 device tensor of the rows with more than `thresh` edges,
        their count) -- computed once per CSR and threshold (one host sync at
        the graph's first SpMM, none per layer)."""
        cache = self.__dict__.setdefault("_heavy", {})
        if thresh not in cache:
            deg = self.degrees()
            idx = torch.nonzero(deg > thresh).view(-1)
            # longest rows first: their chains start at the head of the launch (lpg_spmm_f32_heavy)
            idx = idx[torch.argsort(deg[idx], descending=True, stable=True)].to(torch.int32)
            cache[thresh] = (idx, int(idx.numel()))
        return cache[thresh]

    def hot_source_fraction(self, rows: int) -> float:
        """The fraction of the edges whose source (column) is among the `rows` most-referenced sources --
        how much of an SpMM's gather traffic a cache holding that many source rows serves.  Once per CSR
        and row budget (one host sync at the graph's first SpMM)."""
        cache = self.__dict__.setdefault("_hot", {})
        if rows not in cache:
            if self.nnz == 0 or rows <= 0:
                cache[rows] = 0.0
            else:
                cnt = torch.bincount(self.col.long(), minlength=self.n_cols)
                top = torch.topk(cnt, min(rows, self.n_cols)).values
                cache[rows] = float(top.sum().item()) / self.nnz
        return cache[rows]


# Gather locality (the skewed workload): when most of an F-wide SpMM's edge gathers hit a
# small set of hot source rows (a skewed LP's dense constraints, gathered by every variable that touches
# them), those rows stay in L2 / MALL whatever the slice width, and full-width rows (one wave per
# (row, 1024 columns), the edge list read once instead of once per 128-column slice) win: the skewed
# vars<-cons launch 0.95 -> 0.57 ms (profiles/r06_spmm_skewed_sweep.log).  On a graph without such a hot
# set the 128-column slices keep the gathered table slice MALL-resident (uniform c2: 1.11 vs 1.15+ ms).
HOT_CACHE_BYTES = 64 << 20   # the source rows a launch may count on finding in cache
HOT_FRACTION = 0.6           # ... serving at least this fraction of its edges -> full-width rows
WIDE_SLICE = 1024


class BipartiteCSR:
    """Drop-in for the reference batch's ``edge_index`` SparseTensor(m x n).

    ``sparse_sizes()`` is (rows, cols) of the current orientation; ``t()``
    returns the transposed view without moving data (the reference re-derives
    it with a csr2csc gather every layer, arch.py:71).
    """

    def __init__(self, fwd: CSR, bwd: CSR):
        self.fwd, self.bwd = fwd, bwd

    # -- SparseTensor-like surface used by the reference call sites --
    def t(self) -> "BipartiteCSR":
        return BipartiteCSR(self.bwd, self.fwd)

    def sparse_sizes(self):
        return (self.fwd.n_rows, self.fwd.n_cols)

    def sparse_size(self, dim: int) -> int:
        return self.sparse_sizes()[dim]

    def nnz(self) -> int:
        return self.fwd.nnz

    @property
    def device(self) -> torch.device:
        return self.fwd.device

    def to(self, device, non_blocking: bool = False) -> "BipartiteCSR":
        return BipartiteCSR(self.fwd.to(device), self.bwd.to(device))

    def half(self) -> "BipartiteCSR":
        """SparseTensor.half() (batch_to(half=True), utils.py:909-915): the edge values rounded to fp16
        (kept in fp32 storage -- exact -- which the SpMM kernels read; the products are those of the
        fp16 values)."""
        r = lambda c: CSR(c.rowptr, c.col, c.val.half().float(), c.n_rows, c.n_cols)  # noqa: E731
        return BipartiteCSR(r(self.fwd), r(self.bwd))

    def __repr__(self) -> str:
        r, c = self.sparse_sizes()
        return f"BipartiteCSR(sparse_sizes=({r}, {c}), nnz={self.nnz()}, device={self.device})"

    # -- construction --
    @classmethod
    def from_edge_index(cls, edge_index: torch.Tensor, edge_attr: torch.Tensor, sparse_sizes,
                        device=None) -> "BipartiteCSR":
        """SparseTensor.from_edge_index(edge_index, edge_attr, (m, n)) (dataset.py:301-304).

        On a HIP device the pack runs on the GPU (lpg_csr_pack_f32); for host
        tensors with ``device`` None/'cpu' it runs in the library's host pack
        (lpg_csr_pack_host) -- the data-loader worker analogue; the result
        must be moved to the GPU before any spmm.
        """
        m, n = int(sparse_sizes[0]), int(sparse_sizes[1])
        device = torch.device(device) if device is not None else edge_index.device
        row = edge_index[0].to(torch.int64).contiguous()
        col = edge_index[1].to(torch.int64).contiguous()
        val = edge_attr.to(torch.float32).contiguous().view(-1)
        nnz = int(row.numel())
        if val.numel() != nnz:
            raise ValueError(f"edge_attr has {val.numel()} values for {nnz} edges")
        if device.type == "cpu":
            return cls._pack_host(row.cpu(), col.cpu(), val.cpu(), nnz, m, n)
        return cls._pack_device(row.to(device), col.to(device), val.to(device), nnz, m, n)

    @classmethod
    def from_coo(cls, row, col, val, m: int, n: int, device) -> "BipartiteCSR":
        ei = torch.stack([torch.as_tensor(np.asarray(row)), torch.as_tensor(np.asarray(col))])
        return cls.from_edge_index(ei, torch.as_tensor(np.asarray(val, dtype=np.float32)), (m, n), device)

    @classmethod
    def _pack_host(cls, row, col, val, nnz, m, n) -> "BipartiteCSR":
        L = _lib.lib()
        a_rp = torch.empty(m + 1, dtype=torch.int64)
        at_rp = torch.empty(n + 1, dtype=torch.int64)
        a_c, at_c = torch.empty(nnz, dtype=torch.int32), torch.empty(nnz, dtype=torch.int32)
        a_v, at_v = torch.empty(nnz, dtype=torch.float32), torch.empty(nnz, dtype=torch.float32)
        p = lambda t: t.data_ptr() if t.numel() else None
        _lib.check(L.lpg_csr_pack_host(p(row), p(col), p(val), nnz, m, n, a_rp.data_ptr(), p(a_c), p(a_v),
                                       at_rp.data_ptr(), p(at_c), p(at_v)), "lpg_csr_pack_host")
        return cls(CSR(a_rp, a_c, a_v, m, n), CSR(at_rp, at_c, at_v, n, m))

    @classmethod
    def _pack_device(cls, row, col, val, nnz, m, n) -> "BipartiteCSR":
        L = _lib.lib()
        dev = row.device
        ws_bytes = L.lpg_csr_pack_workspace_bytes(nnz, m, n)
        ws = torch.empty(max(ws_bytes, 16), dtype=torch.uint8, device=dev)
        kw = dict(device=dev)
        a_rp, at_rp = torch.empty(m + 1, dtype=torch.int64, **kw), torch.empty(n + 1, dtype=torch.int64, **kw)
        a_c, at_c = torch.empty(nnz, dtype=torch.int32, **kw), torch.empty(nnz, dtype=torch.int32, **kw)
        a_v, at_v = torch.empty(nnz, dtype=torch.float32, **kw), torch.empty(nnz, dtype=torch.float32, **kw)
        p = lambda t: t.data_ptr() if t.numel() else None
        with torch.cuda.device(dev):
            _lib.check(L.lpg_csr_pack_f32(p(row), p(col), p(val), nnz, m, n, a_rp.data_ptr(), p(a_c), p(a_v),
                                          at_rp.data_ptr(), p(at_c), p(at_v), ws.data_ptr(), _lib.stream_of(row)),
                       "lpg_csr_pack_f32")
            bad, dup = ws[:16].view(torch.int64).tolist()  # one sync per graph load, not per layer
        if bad or dup:
            raise RuntimeError(f"lpg_csr_pack_f32: invalid argument: {bad} edge(s) with an out-of-range index, "
                               f"{dup} duplicate (row, col) pair(s); coalesce first (dataset.py:252)")
        return cls(CSR(a_rp, a_c, a_v, m, n), CSR(at_rp, at_c, at_v, n, m))


DEFAULT_HEAVY = 1024  # PathOptions.spmm_heavy's default (rows above it: heavy wave units)
# F <= 64 (conv1's input): rows above this many edges (or above spmm_heavy, if lower) run as one
# 256-lane LDS-staged block each instead of one FW-lane chain of dependent loads (spmm.hip
# narrow_heavy_row): a 6 000-edge Zipf row took the whole 1 ms launch in the FW-lane form
NARROW_HEAVY = 64


def spmm_forward(adj: CSR, x: torch.Tensor, slice_cols: int = 0, depth: int = 0, heavy: int | None = None) -> torch.Tensor:
    """Y = adj @ x on the GPU (no autograd).  fp32, bf16 or fp16 storage.  ``slice_cols`` / ``depth``: the
    per-call tuning of lpg_spmm_*_tuned (0 = auto; every choice gives the same bits).  ``heavy``: rows with
    more edges than this run as (heavy row, slice) wave units, 0 = off (PathOptions.spmm_heavy; None = the
    default options')."""
    from .options import DEFAULT

    heavy_thresh = DEFAULT.spmm_heavy if heavy is None else int(heavy)
    if x.device.type != "cuda" or adj.device != x.device:
        raise RuntimeError(f"lpgnn.spmm: x ({x.device}) and adj ({adj.device}) must be on the same HIP device; "
                           "there is no CPU path")
    if x.dim() != 2 or x.shape[0] != adj.n_cols:
        raise RuntimeError(f"lpgnn.spmm: x must be [{adj.n_cols}, F], got {tuple(x.shape)}")
    if x.stride(1) != 1:
        x = x.contiguous()
    Fd = x.shape[1]
    y = torch.empty((adj.n_rows, Fd), dtype=x.dtype, device=x.device)
    L = _lib.lib()
    if x.dtype == torch.float32:
        name = "lpg_spmm_f32_tuned"
    elif x.dtype == torch.bfloat16:
        name = "lpg_spmm_bf16_tuned"
    elif x.dtype == torch.float16:
        name = "lpg_spmm_f16_tuned"
    else:
        raise RuntimeError(f"lpgnn.spmm: unsupported dtype {x.dtype}")
    heavy = None
    if Fd <= 64 and heavy_thresh > 0:  # narrow F: rows above NARROW_HEAVY on one block each (LDS-staged)
        heavy_thresh = min(heavy_thresh, NARROW_HEAVY)
    if (Fd >= 256 or Fd <= 64) and heavy_thresh > 0:  # degree-aware: rows above the threshold on their own units
        heavy = adj.heavy_rows(heavy_thresh)
        if heavy[1] == 0:
            heavy = None
    if (slice_cols == 0 and x.dtype == torch.float32 and Fd >= WIDE_SLICE and heavy_thresh > 0
            and adj.hot_source_fraction(HOT_CACHE_BYTES // (Fd * 4)) >= HOT_FRACTION):
        slice_cols = WIDE_SLICE  # a hot, cache-resident source set: full-width rows (degree-aware, as heavy rows)
    with torch.cuda.device(x.device):
        stream = _lib.stream_of(x)
        tok = TIMER.start(("spmm", adj.n_rows, adj.n_cols, Fd, str(x.dtype)))
        st = getattr(L, name)(ctypes.byref(adj.cstruct()), x.data_ptr(), x.stride(0), y.data_ptr(), y.stride(0), Fd,
                              None if heavy is None else heavy[0].data_ptr(), 0 if heavy is None else heavy[1],
                              heavy_thresh if heavy is not None else 0, int(slice_cols), int(depth), stream)
        TIMER.stop(tok)
    _lib.check(st, name)
    return y


class _SpMM(torch.autograd.Function):
    """torch_sparse SPMMSum: fwd spmm(A, X), bwd dX = spmm(A^T, dY)."""

    @staticmethod
    def forward(ctx, x, adj):
        ctx.adj = adj
        return spmm_forward(adj.fwd, x)

    @staticmethod
    def backward(ctx, gy):
        if not ctx.needs_input_grad[0]:
            return None, None
        return spmm_forward(ctx.adj.bwd, gy), None


def spmm(adj: BipartiteCSR, x: torch.Tensor) -> torch.Tensor:
    """``torch_sparse.matmul(adj_t, x, reduce='add')`` on the HIP kernels.

    A partitioned adjacency (lpgnn.partition.PartitionedCSR) runs its local
    SpMM plus the boundary exchange."""
    f = getattr(adj, "partitioned_spmm", None)
    if f is not None:
        return f(x)
    return _SpMM.apply(x, adj)
