"""Constraint-row partitioning of one large LP graph across GPUs.

The reference has no distributed code (train.py:81-82: DataParallel
commented out); graphs above 12M edges fall back to NeighborLoader
mini-batches (train.py:103-116).  Here a large LP is split instead:

* constraint rows -> P contiguous, nnz-balanced blocks, one per rank;
* a variable touched by one block only is *interior* to it (untouched
  variables go to the rank of their id block); a variable touched by >= 2
  blocks is a *boundary* variable, replicated on every rank;
* each rank packs CSR(A_p) / CSR(A_p^T) over its cons rows and its local
  variables, numbered in ascending global id -- so every row keeps the
  reference's per-row edge order and interior results are bitwise those of
  the single-GPU run;
* per layer: cons<-vars is purely local (boundary rows are replicated);
  vars<-cons gives full sums for interior variables and partial sums for
  boundary ones -> ONE all-reduce(sum) of the boundary aggregate rows over
  RCCL.  Its autograd backward is the same all-reduce on the gradient.
  Everything after (FC, ReLU) runs redundantly and identically on every
  rank for the boundary rows.
* loss: each node is owned by exactly one rank (boundary variables by the
  lowest rank touching them); the balanced loss (train.py:39-46) uses
  all-reduced class counts and weight sums, so the per-rank losses add up
  to the single-graph loss; weight gradients are summed with one bucketed
  all-reduce before the optimizer step (identical on every rank).

The local SpMM and the FC are the product HIP kernels; tests swap them for
the oracle to exercise this module with gloo on CPU.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch
import torch.distributed as dist
import torch.nn.functional as F

from . import sparse as _sparse
from .sparse import BipartiteCSR


# ----------------------------------------------------------------------- plan
@dataclass
class PartitionPlan:
    rank: int
    world: int
    m: int                 # global cons
    n: int                 # global vars
    row_lo: int            # this rank's cons block [row_lo, row_hi)
    row_hi: int
    local_vars: np.ndarray  # int64 [n_p] global var ids, ascending
    boundary: np.ndarray   # int64 [n_b] local indices of the (replicated) boundary vars
    var_owned: np.ndarray  # bool [n_p] this rank owns the var's output/loss
    e_row: np.ndarray      # local edges (local cons id, local var id, value)
    e_col: np.ndarray
    e_val: np.ndarray
    n_boundary_global: int

    @property
    def m_local(self) -> int:
        return self.row_hi - self.row_lo

    @property
    def n_local(self) -> int:
        return int(self.local_vars.shape[0])

    @property
    def nnz_local(self) -> int:
        return int(self.e_row.shape[0])


def row_blocks(row: np.ndarray, m: int, world: int) -> np.ndarray:
    """nnz-balanced contiguous split points [0 = b_0 <= ... <= b_P = m]."""
    deg = np.bincount(row, minlength=m)
    cum = np.cumsum(deg)
    nnz = int(cum[-1]) if m else 0
    b = [0]
    for k in range(1, world):
        b.append(int(np.searchsorted(cum, k * nnz / world, side="left")) + 1)
    b.append(m)
    b = np.maximum.accumulate(np.minimum(np.array(b, dtype=np.int64), m))
    return b


def plan_partition(row, col, val, m: int, n: int, world: int, rank: int) -> PartitionPlan:
    row = np.asarray(row, np.int64)
    col = np.asarray(col, np.int64)
    val = np.asarray(val, np.float32)
    bounds = row_blocks(row, m, world)
    blk = np.searchsorted(bounds, row, side="right") - 1
    vmin = np.full(n, world, np.int64)
    vmax = np.full(n, -1, np.int64)
    np.minimum.at(vmin, col, blk)
    np.maximum.at(vmax, col, blk)
    untouched = vmax < 0
    owner = np.where(untouched, (np.arange(n, dtype=np.int64) * world) // max(n, 1), vmin)
    is_boundary = (~untouched) & (vmin != vmax)
    local_mask = is_boundary | (owner == rank)
    local_vars = np.nonzero(local_mask)[0].astype(np.int64)
    g2l = np.full(n, -1, np.int64)
    g2l[local_vars] = np.arange(local_vars.shape[0])
    lo, hi = int(bounds[rank]), int(bounds[rank + 1])
    sel = (row >= lo) & (row < hi)
    e_row, e_col = row[sel] - lo, g2l[col[sel]]
    assert (e_col >= 0).all()
    boundary = g2l[np.nonzero(is_boundary)[0]]
    var_owned = owner[local_vars] == rank
    return PartitionPlan(rank, world, m, n, lo, hi, local_vars, boundary.astype(np.int64), var_owned,
                         e_row, e_col, val[sel], int(is_boundary.sum()))


# ------------------------------------------------------------ communication
def _all_reduce_(t: torch.Tensor, group=None) -> torch.Tensor:
    """Sum-all-reduce in place.  RCCL on HIP tensors; with the gloo backend
    (CPU tests, or several ranks sharing one GPU) HIP tensors are staged
    through host memory."""
    if dist.get_backend(group) == "gloo" and t.is_cuda:
        h = t.cpu()
        dist.all_reduce(h, group=group)
        t.copy_(h)
    else:
        dist.all_reduce(t, group=group)
    return t


class _BoundaryAllReduce(torch.autograd.Function):
    """y = x with rows `bidx` replaced by their sum over ranks.  Backward:
    the same all-reduce on the gradient rows (sum of every rank's share)."""

    @staticmethod
    def forward(ctx, x, bidx, group):
        ctx.bidx, ctx.group = bidx, group
        if bidx.numel():
            buf = x.index_select(0, bidx)
            _all_reduce_(buf, group)
            x.index_copy_(0, bidx, buf)
        ctx.mark_dirty(x)  # x is a fresh SpMM output that nothing else saved
        return x

    @staticmethod
    def backward(ctx, g):
        g = g.clone()
        if ctx.bidx.numel():
            buf = g.index_select(0, ctx.bidx)
            _all_reduce_(buf, ctx.group)
            g.index_copy_(0, ctx.bidx, buf)
        return g, None, None


# local compute hooks (the product HIP kernels; tests swap in the oracle)
def _local_spmm(adj: BipartiteCSR, x: torch.Tensor) -> torch.Tensor:
    return _sparse.spmm(adj, x)


class PartitionedCSR:
    """The edge_index of a rank's batch: local dual CSR + boundary exchange.

    Orientation "cons" = A_p (rows = local cons) -- cons<-vars, local only;
    orientation "vars" = A_p^T (rows = local vars) -- vars<-cons, partial
    sums on boundary rows completed by the all-reduce.
    """

    def __init__(self, local: BipartiteCSR, bidx: torch.Tensor, group, orient: str = "cons"):
        self.local, self.bidx, self.group, self.orient = local, bidx, group, orient

    def t(self) -> "PartitionedCSR":
        return PartitionedCSR(self.local.t(), self.bidx, self.group, "vars" if self.orient == "cons" else "cons")

    def sparse_sizes(self):
        return self.local.sparse_sizes()

    def nnz(self) -> int:
        return self.local.nnz()

    @property
    def device(self):
        return self.local.device

    def to(self, device, non_blocking=False):
        return PartitionedCSR(self.local.to(device), self.bidx.to(device), self.group, self.orient)

    def partitioned_spmm(self, x: torch.Tensor) -> torch.Tensor:
        y = _local_spmm(self.local, x)
        if self.orient == "vars":
            y = _BoundaryAllReduce.apply(y, self.bidx, self.group)
        return y


def make_local_batch(plan: PartitionPlan, x_s, x_t, y_s, y_t, device, group=None, pack_device=None):
    """Rank-local BipartiteBatch with a PartitionedCSR edge_index."""
    from .data import BipartiteBatch

    pd = device if pack_device is None else pack_device
    local = BipartiteCSR.from_coo(plan.e_row, plan.e_col, plan.e_val, plan.m_local, plan.n_local, device=pd)
    if str(pd) != str(device):
        local = local.to(device)
    lv = torch.from_numpy(plan.local_vars)
    adj = PartitionedCSR(local, torch.from_numpy(plan.boundary).to(device), group)
    b = BipartiteBatch(
        x_s=torch.as_tensor(x_s[plan.row_lo:plan.row_hi]).to(device),
        x_t=torch.as_tensor(np.asarray(x_t)[plan.local_vars]).to(device),
        y_s=None if y_s is None else torch.as_tensor(y_s[plan.row_lo:plan.row_hi]).to(device),
        y_t=None if y_t is None else torch.as_tensor(np.asarray(y_t)[plan.local_vars]).to(device),
        edge_index=adj, s_bs=plan.m_local, t_bs=plan.n_local, bs=plan.m_local + plan.n_local)
    b.var_owned = torch.from_numpy(plan.var_owned).to(device)
    b.local_vars = lv
    b.plan = plan
    return b


# ----------------------------------------------------------------------- loss
def _balanced_weights_from_counts(cnt: torch.Tensor) -> torch.Tensor:
    """labels_to_balanced_weights (utils.py:286-299) from global counts."""
    present = cnt > 0
    res = torch.zeros(3, dtype=torch.float32, device=cnt.device)
    tot = cnt.sum().to(torch.float32)
    res[present] = tot / cnt[present].to(torch.float32)
    if int(present.sum()) != 2:
        res[0] = res[2] = (res[0] + res[2]) / 2.
    return res


def balanced_distributed(lc, lv, y_s, y_t, var_owned, group=None):
    """Per-rank share of train.py:39-46 so that sum over ranks == the
    single-graph balanced loss (class weights and the weighted-mean
    denominators are global)."""
    ys, yt = y_s, y_t[var_owned]
    lv = lv[var_owned]
    cnt = torch.cat([torch.bincount(ys, minlength=3), torch.bincount(yt, minlength=3)]).to(torch.float64)
    _all_reduce_(cnt, group)
    cs, ct = cnt[:3], cnt[3:]
    m, n = cs.sum().item(), ct.sum().item()
    ws, wt = _balanced_weights_from_counts(cs), _balanced_weights_from_counts(ct)
    ce_s = F.cross_entropy(lc, ys, reduction="none")
    ce_t = F.cross_entropy(lv, yt, reduction="none")
    den = torch.stack([ws[ys].sum(), wt[yt].sum()]).to(torch.float64)
    _all_reduce_(den, group)
    return (m + n) / m * (ws[ys] * ce_s).sum() / den[0].float() + (m + n) / n * (wt[yt] * ce_t).sum() / den[1].float()


def all_reduce_grads(model, group=None):
    """One bucketed sum-all-reduce of every parameter gradient."""
    grads = [p.grad for p in model.parameters() if p.grad is not None]
    if not grads:
        return
    flat = torch.cat([g.reshape(-1) for g in grads])
    _all_reduce_(flat, group)
    off = 0
    for g in grads:
        k = g.numel()
        g.copy_(flat[off:off + k].view_as(g))
        off += k


def train_step_distributed(model, batch, opt, group=None):
    lc, lv = model(batch)
    loss = balanced_distributed(lc, lv, batch.y_s, batch.y_t, batch.var_owned, group)
    opt.zero_grad()
    loss.backward()
    all_reduce_grads(model, group)
    opt.step()
    return loss


# ---------------------------------------------------------------- bench job
@dataclass
class BenchJob:
    step: object
    local_nnz: int
    workload: str
    plan: PartitionPlan


def build_bench_job(args, rank: int, world: int, device) -> BenchJob:
    """Weak scaling: the global graph is `world` c2-sized row blocks
    (world*m cons x world*n vars, world*nnz edges), a fraction rho of each
    block's edges landing on other blocks' variables."""
    from . import synth
    from .arch import GCN_FC
    from .train import make_optimizer

    g = synth.block_lp(args.m * world, args.n * world, args.nnz * world, parts=world, rho=args.rho, seed=0)
    plan = plan_partition(g.row, g.col, g.val, g.m, g.n, world, rank)
    batch = make_local_batch(plan, g.x_s, g.x_t, g.y_s, g.y_t, device)
    torch.manual_seed(0)
    model = GCN_FC(8, 8, hids=args.hids, depth=args.depth).to(device)
    opt, _ = make_optimizer(model)
    step = lambda: train_step_distributed(model, batch, opt)
    wl = (f"row-partitioned synthetic LP {g.m}x{g.n} nnz={g.nnz} over {world} GPUs (c2-sized block per GPU, "
          f"rho={args.rho}, {plan.n_boundary_global} boundary vars), GCN_FC(8,8,hids={args.hids},"
          f"depth={args.depth}) fwd+bwd+Adam")
    return BenchJob(step, plan.nnz_local, wl, plan)
