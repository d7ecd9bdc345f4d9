"""Constraint-row partitioning of one large LP graph across GPUs.

The reference has no distributed code (train.py:81-82: DataParallel
commented out); graphs above 12M edges fall back to NeighborLoader
mini-batches (train.py:103-116).  Here one large LP is split instead, one
process per GPU:

* constraint rows -> P contiguous, nnz-balanced blocks, one per rank;
* every variable has ONE owner: the rank holding most of its edges (ties:
  lowest rank; untouched variables: the rank of their id block).  A rank
  keeps its owned variables plus a *halo* of the remote-owned variables its
  constraints touch (boundary variables), local ids = [owned | halo], each
  part ascending in global id;
* CSR(A_p) keeps every constraint row's edges in GLOBAL variable order (the
  reference's per-row summation order), CSR(A_p^T) has one row per local
  variable;
* per layer, cons<-vars is purely local (halo rows hold the owners' current
  embeddings); vars<-cons gives partial aggregates on halo rows, which are
  REDUCED to their owners (RCCL all_to_all, summed in ascending source-rank
  order after the owner's own partial -- deterministic), the owner runs the
  FC (+ReLU, +dropout) for its variables only -- no replicated compute --
  and the result is BROADCAST back to the touching ranks' halo rows (second
  all_to_all).  The autograd backward of reduce is broadcast and vice versa.
  Together the pair is the sparse all-reduce of boundary-variable
  embeddings: every rank ends with the full value of exactly the boundary
  rows it uses, and only those rows cross xGMI;
* loss: owned nodes only; the balanced loss (train.py:39-46) uses
  all-reduced class counts and weight sums so the per-rank losses add up to
  the single-graph loss; parameter gradients are summed with one bucketed
  all-reduce (every FC row is computed once, so nothing is double counted).

Local compute is the product HIP path; tests swap `_local_spmm` and the FC
for the oracle to exercise this module with gloo on CPU.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch
import torch.distributed as dist
import torch.nn.functional as F

from . import sparse as _sparse
from .sparse import CSR, BipartiteCSR
from .timing import TIMER


# ----------------------------------------------------------------------- plan
@dataclass
class PartitionPlan:
    rank: int
    world: int
    m: int                  # global cons
    n: int                  # global vars
    row_lo: int             # this rank's cons block [row_lo, row_hi)
    row_hi: int
    owned: np.ndarray       # int64 global ids of owned vars (ascending)
    halo: np.ndarray        # int64 global ids of remote-owned vars touched here (ascending)
    e_row: np.ndarray       # local edges: local cons id, GLOBAL var id, local var id, value
    e_gcol: np.ndarray
    e_col: np.ndarray
    e_val: np.ndarray
    send_idx: np.ndarray    # reduce phase: local halo rows, grouped by owner rank (ascending var in group)
    send_counts: list
    recv_idx: np.ndarray    # reduce phase: local owned rows, grouped by source rank
    recv_counts: list
    n_boundary_global: int  # variables touched by >= 2 ranks

    @property
    def m_local(self) -> int:
        return self.row_hi - self.row_lo

    @property
    def n_own(self) -> int:
        return int(self.owned.shape[0])

    @property
    def n_local(self) -> int:
        return int(self.owned.shape[0] + self.halo.shape[0])

    @property
    def local_vars(self) -> np.ndarray:
        return np.concatenate([self.owned, self.halo])

    @property
    def var_owned(self) -> np.ndarray:
        v = np.zeros(self.n_local, dtype=bool)
        v[:self.n_own] = True
        return v

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
    return np.maximum.accumulate(np.minimum(np.array(b, dtype=np.int64), m))


def plan_partition(row, col, val, m: int, n: int, world: int, rank: int, bounds=None,
                   owner=None) -> PartitionPlan:
    """The plan of `rank` from the global edge list (tests, small graphs).
    bounds: cons block split points (default nnz-balanced); owner: int64 [n]
    owner rank per variable (default: the rank holding most of its edges)."""
    row = np.asarray(row, np.int64)
    col = np.asarray(col, np.int64)
    val = np.asarray(val, np.float32)
    bounds = row_blocks(row, m, world) if bounds is None else np.asarray(bounds, np.int64)
    blk = np.searchsorted(bounds, row, side="right") - 1
    # touches (var, rank) with edge counts, sorted by var then rank
    ukey, cnt = np.unique(col * world + blk, return_counts=True)
    tv, tr = ukey // world, ukey % world
    if owner is None:
        owner = (np.arange(n, dtype=np.int64) * world) // max(n, 1)
        order = np.lexsort((tr, -cnt, tv))  # per var: most edges first, then lowest rank
        first = order[np.r_[True, tv[order][1:] != tv[order][:-1]]] if len(order) else order
        owner[tv[first]] = tr[first]
    else:
        owner = np.asarray(owner, np.int64)
    ntouch = np.bincount(tv, minlength=n)
    is_halo = tr != owner[tv]
    hv, hr = tv[is_halo], tr[is_halo]  # var hv is touched by rank hr and owned elsewhere (sorted by var)

    owned = np.nonzero(owner == rank)[0].astype(np.int64)
    halo = hv[hr == rank]
    local_vars = np.concatenate([owned, halo])
    g2l = np.full(n, -1, np.int64)
    g2l[local_vars] = np.arange(local_vars.shape[0])

    o = owner[halo]
    srt = np.argsort(o, kind="stable")
    send_idx = g2l[halo[srt]]
    send_counts = np.bincount(o, minlength=world).tolist()
    mine = owner[hv] == rank
    rv, rq = hv[mine], hr[mine]
    srt = np.argsort(rq, kind="stable")
    recv_idx = g2l[rv[srt]]
    recv_counts = np.bincount(rq, minlength=world).tolist()

    lo, hi = int(bounds[rank]), int(bounds[rank + 1])
    sel = (row >= lo) & (row < hi)
    e_gcol = col[sel]
    e_col = g2l[e_gcol]
    assert (e_col >= 0).all()
    return PartitionPlan(rank, world, m, n, lo, hi, owned, halo, row[sel] - lo, e_gcol, e_col, val[sel],
                         send_idx.astype(np.int64), send_counts, recv_idx.astype(np.int64), recv_counts,
                         int((ntouch >= 2).sum()))


def plan_partition_local(row, col, val, m: int, n: int, world: int, rank: int, group=None, bounds=None,
                         local: bool = False) -> PartitionPlan:
    """plan_partition's plan of `rank`, built from the rank's OWN constraint rows (the general planner of
    a loaded LP: lpgnn.run --partition).  Equal to plan_partition field for field
    (tests/test_partition.py), without any rank holding the partition's global structures:

    * row blocks: nnz-balanced split points from the global row degrees (``bounds``, or row_blocks of
      the global host `row`);
    * owners: each rank counts its edges per variable; one MAX all-reduce of (count, lowest rank)
      keys picks, per variable, the rank holding most of its edges (ties: lowest rank), untouched
      variables going to the rank of their id block -- plan_partition's rule;
    * receive lists: the owners learn who touches their variables from one all_to_all of the halo id
      lists (plan_partition_blocks' exchange); the boundary count from one SUM all-reduce.

    ``local``: (row, col, val) already hold only this rank's rows [bounds[rank], bounds[rank+1]) (global
    row ids) -- then ``bounds`` is required.  Host numpy throughout; nothing goes to the device here."""
    row = np.asarray(row, np.int64)
    col = np.asarray(col, np.int64)
    val = np.asarray(val, np.float32)
    if bounds is None:
        if local:
            raise ValueError("plan_partition_local(local=True) needs the row block bounds")
        bounds = row_blocks(row, m, world)
    bounds = np.asarray(bounds, np.int64)
    lo, hi = int(bounds[rank]), int(bounds[rank + 1])
    if not local:
        sel = (row >= lo) & (row < hi)
        row, col, val = row[sel], col[sel], val[sel]
    cnt = np.bincount(col, minlength=n).astype(np.int64)  # this rank's edges per variable
    touch = (cnt > 0).astype(np.int64)
    if world > 1:
        # key: count * world + (world - 1 - rank) -- the MAX is the most edges, then the lowest rank
        key = torch.from_numpy(np.where(cnt > 0, cnt * world + (world - 1 - rank), -1))
        ntouch = torch.from_numpy(touch)
        gpu = dist.get_backend(group) != "gloo"
        if gpu:
            key, ntouch = key.cuda(), ntouch.cuda()
        dist.all_reduce(key, op=dist.ReduceOp.MAX, group=group)
        dist.all_reduce(ntouch, group=group)
        key, ntouch = key.cpu().numpy(), ntouch.cpu().numpy()
    else:
        key, ntouch = np.where(cnt > 0, cnt * world + (world - 1 - rank), -1), touch
    owner = (np.arange(n, dtype=np.int64) * world) // max(n, 1)
    hit = key >= 0
    owner[hit] = world - 1 - key[hit] % world
    owned = np.nonzero(owner == rank)[0].astype(np.int64)
    touched = np.nonzero(cnt)[0].astype(np.int64)
    halo = touched[owner[touched] != rank]  # ascending
    o = owner[halo]
    srt = np.argsort(o, kind="stable")       # grouped by owner rank, ascending variable within a group
    send_counts = np.bincount(o, minlength=world).tolist()
    send_idx = owned.shape[0] + srt.astype(np.int64)
    if world > 1:
        got, recv_counts = _a2a_ids(halo[srt], send_counts, group)
        recv_idx = np.searchsorted(owned, got).astype(np.int64)
    else:
        recv_idx, recv_counts = np.empty(0, np.int64), [0]
    is_own = owner[col] == rank
    e_col = np.where(is_own, np.searchsorted(owned, col), owned.shape[0] + np.searchsorted(halo, col))
    return PartitionPlan(rank, world, m, n, lo, hi, owned, halo, row - lo, col, e_col.astype(np.int64), val,
                         send_idx, send_counts, recv_idx, recv_counts, int((ntouch >= 2).sum()))


def _block_owner_ranges(blocks: int, world: int):
    if blocks % world:
        raise ValueError(f"{blocks} row blocks do not split evenly over {world} ranks")
    return blocks // world


def block_owner(spec, world: int) -> np.ndarray:
    """Variable owners of plan_partition_blocks (int64 [n]): the rank whose
    row blocks share the variable's block (tests compare against it)."""
    per = _block_owner_ranges(spec.blocks, world)
    return (np.arange(spec.n, dtype=np.int64) // spec.nb) // per


def _a2a_ids(send: np.ndarray, send_counts: list, group) -> tuple:
    """all_to_all of int64 id lists (the plan's setup exchange, once per
    graph).  Returns (received ids grouped by source rank, recv counts)."""
    world = dist.get_world_size(group)
    dev = torch.device("cpu") if dist.get_backend(group) == "gloo" else torch.device("cuda",
                                                                                      torch.cuda.current_device())
    sc = torch.tensor(send_counts, dtype=torch.int64, device=dev)
    rc = torch.empty(world, dtype=torch.int64, device=dev)
    dist.all_to_all_single(rc, sc, group=group)
    recv_counts = rc.cpu().tolist()
    out = torch.empty(sum(recv_counts), dtype=torch.int64, device=dev)
    dist.all_to_all_single(out, torch.from_numpy(np.ascontiguousarray(send)).to(dev), recv_counts, send_counts,
                           group=group)
    return out.cpu().numpy(), recv_counts


def plan_partition_blocks(spec, world: int, rank: int, group=None, edges=None, exchange: bool = True) -> PartitionPlan:
    """The plan of `rank` for a synth.BlockLP, built from the rank's OWN rows
    only (no global edge list): rank r holds row blocks [r*B/P, (r+1)*B/P)
    and owns the variables of the same blocks' variable ranges; its halo is
    the remote variables its rows touch.  The owners learn who touches their
    variables with one all_to_all of id lists (the only O(halo) setup
    traffic).  Equal to plan_partition(global graph, bounds, block_owner)
    field for field (tests/test_partition.py).  `edges`: the rank's
    (row, col, val) if already generated.  ``exchange=False``: no process group -- the local
    CSR fields only (the receive lists stay empty, n_boundary_global = -1; tools/pmc_rank_share.py)."""
    per = _block_owner_ranges(spec.blocks, world)
    b0, b1 = rank * per, (rank + 1) * per
    row, col, val = edges if edges is not None else spec.rows(b0, b1)[:3]
    row, col, val = np.asarray(row, np.int64), np.asarray(col, np.int64), np.asarray(val, np.float32)
    lo, hi = b0 * spec.mb, b1 * spec.mb
    v_lo, v_hi = b0 * spec.nb, b1 * spec.nb
    owned = np.arange(v_lo, v_hi, dtype=np.int64)
    far = col[(col < v_lo) | (col >= v_hi)]
    halo = np.unique(far)  # ascending, hence grouped by owner rank
    local_vars = np.concatenate([owned, halo])
    h_owner = (halo // spec.nb) // per
    send_counts = np.bincount(h_owner, minlength=world).tolist()
    send_idx = np.arange(owned.shape[0], local_vars.shape[0], dtype=np.int64)
    if world > 1 and not exchange:
        recv_idx, recv_counts, n_boundary = np.empty(0, np.int64), [0] * world, -1
    elif world > 1:
        got, recv_counts = _a2a_ids(halo, send_counts, group)
        recv_idx = got - v_lo
        # boundary = touched by >= 2 ranks (plan_partition's rule): an owned variable a remote rank
        # touches counts if this rank's rows touch it too or a second remote rank does
        rv, rc = np.unique(got, return_counts=True)
        mine = np.unique(col[(col >= v_lo) & (col < v_hi)])
        nb_loc = int(((rc >= 2) | np.isin(rv, mine, assume_unique=True)).sum())
        nb_glob = torch.tensor([nb_loc], dtype=torch.int64)
        if dist.get_backend(group) != "gloo":
            nb_glob = nb_glob.cuda()
        dist.all_reduce(nb_glob, group=group)
        n_boundary = int(nb_glob.item())
    else:
        recv_idx, recv_counts, n_boundary = np.empty(0, np.int64), [0], 0
    # local column ids: owned = v - v_lo, halo = n_own + position in halo
    e_col = np.where((col >= v_lo) & (col < v_hi), col - v_lo,
                     owned.shape[0] + np.searchsorted(halo, col))
    return PartitionPlan(rank, world, spec.m, spec.n, lo, hi, owned, halo, row - lo, col, e_col, val,
                         send_idx, send_counts, recv_idx.astype(np.int64), recv_counts, n_boundary)


def local_dual_csr(plan: PartitionPlan, device) -> BipartiteCSR:
    """CSR(A_p) with each row's edges in global variable order (columns then
    remapped to local ids), CSR(A_p^T) over the local variables."""
    fwd = BipartiteCSR.from_coo(plan.e_row, plan.e_gcol, plan.e_val, plan.m_local, plan.n, device=device).fwd
    g2l = torch.full((plan.n,), -1, dtype=torch.int32)
    g2l[torch.from_numpy(plan.local_vars)] = torch.arange(plan.n_local, dtype=torch.int32)
    fwd_col = g2l.to(fwd.col.device)[fwd.col.long()] if fwd.nnz else fwd.col
    fwd = CSR(fwd.rowptr, fwd_col.contiguous(), fwd.val, plan.m_local, plan.n_local)
    bwd = BipartiteCSR.from_coo(plan.e_row, plan.e_col, plan.e_val, plan.m_local, plan.n_local, device=device).bwd
    return BipartiteCSR(fwd, bwd)


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


def _a2a(send: torch.Tensor, in_counts: list, out_counts: list, group) -> torch.Tensor:
    recv = send.new_empty((sum(out_counts),) + tuple(send.shape[1:]))
    if sum(in_counts) == 0 and sum(out_counts) == 0:
        return recv
    if dist.get_backend(group) == "gloo" and send.is_cuda:
        h = torch.empty(recv.shape, dtype=recv.dtype)
        dist.all_to_all_single(h, send.cpu(), out_counts, in_counts, group=group)
        recv.copy_(h)
    else:
        dist.all_to_all_single(recv, send.contiguous(), out_counts, in_counts, group=group)
    return recv


class _Pending:
    """An all_to_all in flight (RCCL runs it on its own stream; `finish`
    makes the current stream wait, then applies `then` to the received rows).
    gloo with HIP tensors stages through the host synchronously.

    With bench.py's timer on (lpgnn.timing), an RCCL exchange records two HIP-event spans on the
    compute stream: "span" from the issue to the point where the rows are consumed, and "exposed"
    across the wait itself -- the time the compute stream sat idle for the collective, i.e. the part
    of the exchange NOT hidden under independent compute."""

    def __init__(self, recv, work=None, host=None, then=None, tok=None):
        self.recv, self.work, self.host, self.then, self.tok = recv, work, host, then, tok

    def finish(self):
        if self.work is not None:
            key = None if self.tok is None else self.tok[0]
            tok = TIMER.start(key[:4] + ("exposed",)) if key is not None else None
            self.work.wait()
            TIMER.stop(tok)
            TIMER.stop(self.tok)
        if self.host is not None:
            self.recv.copy_(self.host)
        return self.then(self.recv) if self.then is not None else self.recv


def _a2a_start(send: torch.Tensor, in_counts: list, out_counts: list, group) -> _Pending:
    recv = send.new_empty((sum(out_counts),) + tuple(send.shape[1:]))
    if dist.get_backend(group) == "gloo" and send.is_cuda:
        h = torch.empty(recv.shape, dtype=recv.dtype)
        dist.all_to_all_single(h, send.cpu(), out_counts, in_counts, group=group)
        return _Pending(recv, host=h)
    tok = TIMER.start(("exchange", sum(in_counts), sum(out_counts), int(np.prod(send.shape[1:])), "span"))
    work = dist.all_to_all_single(recv, send.contiguous(), out_counts, in_counts, group=group, async_op=True)
    return _Pending(recv, work=work, tok=tok)


class Exchange:
    """The static boundary exchange of one rank (see module docstring)."""

    def __init__(self, plan: PartitionPlan, device, group=None):
        self.n_own, self.n_local = plan.n_own, plan.n_local
        self.m, self.n = plan.m, plan.n  # global sizes: rank-independent layout decisions
        # dropout keys: every node is keyed by its GLOBAL id, so each node draws the mask a single-GPU
        # run draws.  The constraint rows are the block [row_lo, row_hi) (the FC's row_offset); the
        # owned variables are one contiguous range in every block plan (row_offset = owned[0]) and
        # any set in a general plan (the owner with most edges): then the FC takes one key per row
        # (row_keys = the owned global ids, int64 on the device).
        self.cons_key0 = int(plan.row_lo)
        own = plan.owned
        self.var_key0 = int(own[0]) if own.shape[0] else 0
        contiguous = own.shape[0] == 0 or int(own[-1]) - int(own[0]) + 1 == own.shape[0]
        self.var_keys = None if contiguous else torch.from_numpy(np.ascontiguousarray(own, np.int64)).to(device)
        self.send_idx = torch.from_numpy(plan.send_idx).to(device)
        self.recv_idx = torch.from_numpy(plan.recv_idx).to(device)
        self.send_counts, self.recv_counts = list(plan.send_counts), list(plan.recv_counts)
        self.group = group
        # per-source slices of recv_idx (ascending source rank)
        off = np.concatenate([[0], np.cumsum(self.recv_counts)]).astype(np.int64)
        self.recv_slices = [(int(off[q]), int(off[q + 1])) for q in range(len(self.recv_counts))
                            if off[q + 1] > off[q]]
        # all_to_all is a collective: every rank calls it, or (no boundary
        # rows anywhere in the partition) none does -- decided once, globally
        tot = torch.tensor([float(sum(self.send_counts) + sum(self.recv_counts))])
        if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
            if dist.get_backend(group) != "gloo":
                tot = tot.to(device)
            dist.all_reduce(tot, group=group)
        self.active = bool(tot.item() > 0)
        self._deferred = []  # (data_ptr, pending broadcast) of layer outputs whose halo rows are in flight

    def defer(self, full: torch.Tensor, pending: _Pending) -> None:
        """Leave a broadcast of `full`'s halo rows in flight: the consumer settles it (settle) right
        before it first reads those rows, so the exchange runs under the compute in between."""
        self._deferred.append((full.data_ptr(), pending))

    def settle(self, full: torch.Tensor) -> torch.Tensor:
        """Finish the deferred broadcast into `full`, if any (its halo rows are then current)."""
        if self._deferred:
            ptr = full.data_ptr()
            keep = []
            for q, p in self._deferred:
                if q == ptr:
                    p.finish()
                else:
                    keep.append((q, p))
            self._deferred = keep
        return full

    def settle_all(self) -> None:
        for _, p in self._deferred:
            p.finish()
        self._deferred = []

    @property
    def var_key_args(self) -> dict:
        """The FC keyword arguments that key the owned variables' dropout rows by their global ids."""
        return {"row_offset": self.var_key0, "row_keys": self.var_keys}

    @property
    def cons_key_args(self) -> dict:
        return {"row_offset": self.cons_key0, "row_keys": None}

    def _a2a(self, send, in_counts, out_counts):
        if not self.active:
            return send.new_empty((0,) + tuple(send.shape[1:]))
        return _a2a(send, in_counts, out_counts, self.group)

    def start_reduce(self, full: torch.Tensor, inplace: bool) -> _Pending:
        """Asynchronous reduce_rows: finish() returns the [n_own, F] owner sums."""
        def then(recv):
            owned = full[:self.n_own]
            if self.recv_slices:
                if not inplace:
                    owned = owned.clone()
                self.add_partials(owned, recv)
            return owned
        if not self.active:
            return _Pending(None, then=lambda _: full[:self.n_own])
        p = _a2a_start(full.index_select(0, self.send_idx), self.send_counts, self.recv_counts, self.group)
        p.then = then
        return p

    def start_broadcast_(self, full: torch.Tensor, quiet: bool = False) -> _Pending:
        """Asynchronous broadcast_rows_: finish() fills the halo rows and returns `full`.  quiet: the
        rows are written through a storage alias that leaves `full`'s autograd version alone -- for a
        layer output whose halo rows land after the node that made it returned (Exchange.defer; that
        node's backward reads only its owned rows)."""
        dst = full.data if quiet else full

        def then(recv):
            if self.send_idx.numel():
                dst.index_copy_(0, self.send_idx, recv)
                if quiet:  # (no version bump: drop the f16x2 scales cached on full's storage)
                    from .fc import _SCALES
                    _SCALES.forget(full)
            return full
        if not self.active:
            return _Pending(None, then=lambda _: full)
        p = _a2a_start(full[:self.n_own].index_select(0, self.recv_idx), self.recv_counts, self.send_counts,
                       self.group)
        p.then = then
        return p

    def reduce_rows(self, full: torch.Tensor, inplace: bool) -> torch.Tensor:
        """[n_local, F] partials -> [n_own, F] owner sums.  With inplace the
        owners' rows of `full` are updated and a view is returned; otherwise
        they are copied only if something is received."""
        recv = self._a2a(full.index_select(0, self.send_idx), self.send_counts, self.recv_counts)
        owned = full[:self.n_own]
        if self.recv_slices:
            if not inplace:
                owned = owned.clone()
            self.add_partials(owned, recv)
        return owned

    def broadcast_rows_(self, full: torch.Tensor) -> torch.Tensor:
        """Fill the halo rows of [n_local, F] `full` from their owners, in place."""
        recv = self._a2a(full[:self.n_own].index_select(0, self.recv_idx), self.recv_counts, self.send_counts)
        if self.send_idx.numel():
            full.index_copy_(0, self.send_idx, recv)
        return full

    def add_partials(self, owned: torch.Tensor, recv: torch.Tensor) -> None:
        for a, b in self.recv_slices:  # deterministic: one index_add_ per source rank, unique rows each
            owned.index_add_(0, self.recv_idx[a:b], recv[a:b])

    def reduce(self, full: torch.Tensor) -> torch.Tensor:
        """[n_local, F] partials -> [n_own, F] sums (own partial + sources in rank order)."""
        recv = self._a2a(full.index_select(0, self.send_idx), self.send_counts, self.recv_counts)
        owned = full[:self.n_own].clone()
        self.add_partials(owned, recv)
        return owned

    def broadcast(self, owned: torch.Tensor) -> torch.Tensor:
        """[n_own, F] owner values -> [n_local, F] with the halo rows filled."""
        recv = self._a2a(owned.index_select(0, self.recv_idx), self.recv_counts, self.send_counts)
        out = owned.new_empty((self.n_local,) + tuple(owned.shape[1:]))
        out[:self.n_own] = owned
        if self.send_idx.numel():
            out.index_copy_(0, self.send_idx, recv)
        return out

    def broadcast_grad(self, g_owned: torch.Tensor) -> torch.Tensor:
        """Backward of reduce: every holder of a row gets the owner's gradient."""
        return self.broadcast(g_owned)

    def reduce_grad(self, g_local: torch.Tensor) -> torch.Tensor:
        """Backward of broadcast: halo-row gradients are summed into the owner."""
        return self.reduce(g_local)


class _Reduce(torch.autograd.Function):
    @staticmethod
    def forward(ctx, full, ex):
        ctx.ex = ex
        return ex.reduce(full)

    @staticmethod
    def backward(ctx, g):
        return ctx.ex.broadcast_grad(g.contiguous()), None


class _Broadcast(torch.autograd.Function):
    @staticmethod
    def forward(ctx, owned, ex):
        ctx.ex = ex
        return ex.broadcast(owned)

    @staticmethod
    def backward(ctx, g):
        return ctx.ex.reduce_grad(g.contiguous()), None


# local compute hook (the product HIP kernel; tests swap in the oracle)
def _local_spmm(adj: BipartiteCSR, x: torch.Tensor) -> torch.Tensor:
    return _sparse.spmm(adj, x)


_product_spmm = _local_spmm


class _PartTwoDirection(torch.autograd.Function):
    """One GraphConvTwoDirection layer on a rank's partition, one autograd node
    (the partitioned twin of lpgnn.conv._TwoDirection).

    right = local variables [owned | halo], left = local constraints.
    left2right: partial aggregates for every local variable, REDUCED to the
    owners in place; the owners' FC writes straight into the first n_own rows
    of the [n_local, F] output, whose halo rows are then BROADCAST from the
    owners.  right2left is local (the halo rows are current).  Backward
    mirrors it: the halo-row gradients of right' are reduced to their owners,
    the aggregate gradient of the owned rows is broadcast back before the
    transposed SpMM.  Gradient sums accumulate inside the GEMMs (x3 accumulate flag / addmm_) as in the
    one-GPU node.
    left2right follows conv.py's association rule (on the global node counts):
    re-associated, the reduced partials are those of A^T (left W_rel^T) and the
    owners' lin_root + bias + ReLU is accumulated onto them in place.
    """

    @staticmethod
    def forward(ctx, left, right, padj, w_rel_l2r, b_l2r, w_root_l2r, w_rel_r2l, b_r2l, w_root_r2l, relu, dropout,
                opts=None, prev=None, defer=False):
        left_new, right_new, saved, _ = _part_forward_core(ctx, left, right, padj, w_rel_l2r, b_l2r, w_root_l2r,
                                                           w_rel_r2l, b_r2l, w_root_r2l, relu, dropout, opts=opts,
                                                           defer=defer)
        _link_prev(ctx, prev)
        ctx.save_for_backward(*saved)
        return left_new, right_new

    @staticmethod
    def backward(ctx, g_left, g_right):
        return _part_backward_core(ctx, ctx.saved_tensors, ctx.needs_input_grad, g_left, g_right) + (None, None,
                                                                                                      None)


def _link_prev(ctx, prev):
    """prev: conv1's node whose weight gradients this layer's input-gradient GEMMs compute (the
    partitioned conv1 fold, _part_backward_core)."""
    ctx.wgk_prev = prev
    if prev is not None:
        prev.wgk_folded = True


def _fc_x3like():
    from .fc import X3LIKE

    return X3LIKE


def foldable_producer(left, right, opts):
    """conv1's partitioned node (fp32, ReLU, no dropout, narrow LP-feature inputs that need no
    gradient) when it produced (left, right) and the options fold its weight gradients into the next
    layer's x3 input-gradient GEMMs (options.fold_conv1_wgrad, lpg_fc_x3_relu_wgrad_f32); else None."""
    g = left.grad_fn
    if (g is None or g is not right.grad_fn or not isinstance(g, _PartTwoDirection._backward_cls)
            or not torch.is_grad_enabled() or not getattr(g, "small_relu", False)):
        return None
    if not (opts.fold_conv1_wgrad and opts.arith in _fc_x3like() and g.opts.arith in _fc_x3like()) or \
            any(g.needs_input_grad[:2]):
        return None
    # the fold hands conv1's outputs zero-stride gradients: not when something observes them (a hook or
    # retain_grad on left / right) -- then the two-pass route, as conv.foldable_producer
    if any(x.retains_grad or x._backward_hooks for x in (left, right)):
        return None
    return g


def _part_forward_core(ctx, left, right, padj, w_rel_l2r, b_l2r, w_root_l2r, w_rel_r2l, b_r2l, w_root_r2l, relu,
                       dropout, heads=None, opts=None, defer=False):
    """_PartTwoDirection's forward; returns (left_new, right_new, tensors to save, logits).
    heads = ((Wh_l, bh_l), (Wh_r, bh_r)): the heads in the FC epilogues (conv._forward_core's
    rule) for the rows the FCs compute, a separate Linear for the halo rows; logits None without --
    and then right_new's halo rows are never read (the halo logits are the owners', broadcast), so
    they are not broadcast.  defer: the broadcast of right_new's halo rows stays in flight for the
    next partitioned layer to settle (Exchange.defer) -- it runs under that layer's first GEMM and
    SpMM, which read no halo row of it."""
    import functools

    from . import fc as _fc
    from .conv import reassociate
    from .options import DEFAULT
    from .sparse import spmm_forward as _spmm_forward

    opts = DEFAULT if opts is None else opts
    fcf = functools.partial(_fc.fc_forward, arith=opts.arith)
    spmm_forward = functools.partial(_spmm_forward, heavy=opts.spmm_heavy)

    if dropout > 0 and not relu:
        raise RuntimeError("lpgnn FC: fused dropout requires the ReLU epilogue")
    if left.dtype != torch.float32:
        raise RuntimeError("the row-partitioned path runs fp32 (the c2/c4 configurations)")
    ex = padj.ex
    A, AT = padj.local.fwd, padj.local.bwd  # A: local cons x local vars
    n_own = ex.n_own
    seed_r = _fc._new_seed() if dropout > 0 else 0
    seed_l = _fc._new_seed() if dropout > 0 else 0
    # conv.py's association rule on the GLOBAL node counts (every rank decides alike, so the
    # reduced rows have the same width everywhere)
    ra = reassociate(ex.m, ex.n, left.shape[1], w_rel_l2r.shape[0], opts.reassociate)
    if ra:  # partials of A^T (left W_rel^T) for [owned | halo]
        agg_r = spmm_forward(AT, fcf(left, w_rel_l2r, None, None, None, False))
    else:
        agg_r = spmm_forward(AT, left)          # partials for [owned | halo]
    red = ex.start_reduce(agg_r, inplace=True)  # halo partials -> owners, in flight ...
    ex.settle(right)                            # (the previous layer's deferred halo rows)
    agg_l = spmm_forward(A, right)              # ... under the purely local constraint side
    hl, hr = heads if heads is not None else (None, None)
    left_new = fcf(agg_l, w_rel_r2l, left, w_root_r2l, b_r2l, relu, dropout, seed_l, heads=hl,
                              row_offset=ex.cons_key0)
    if hl is not None:
        left_new, logit_l = left_new
    red.finish()                                # owners' rows of agg_r now hold the full sums
    if ra:  # lin_root + bias + ReLU accumulated onto the owners' sums, in place
        right_new, agg_r = agg_r, None
        own = fcf(right[:n_own], w_root_l2r, None, None, b_l2r, relu, dropout, seed_r,
                             out=right_new[:n_own], accumulate=True, heads=hr, **ex.var_key_args)
    else:
        right_new = torch.empty((right.shape[0], w_rel_l2r.shape[0]), dtype=torch.float32, device=left.device)
        own = fcf(agg_r[:n_own], w_rel_l2r, right[:n_own], w_root_l2r, b_l2r, relu, dropout, seed_r,
                             out=right_new[:n_own], heads=hr, **ex.var_key_args)
    if heads is None:
        bc = ex.start_broadcast_(right_new, quiet=defer)
        if defer:
            ex.defer(right_new, bc)
        else:
            bc.finish()
    logits = None
    if heads is not None:
        # halo rows are copies of other ranks' variables: their logits are the OWNERS' logits, broadcast
        # (3 floats a row) rather than recomputed -- bitwise the owner's values, and no GEMM over the halo
        logit_r = torch.empty((right_new.shape[0], hr[0].shape[0]), dtype=torch.float32, device=left.device)
        logit_r[:n_own] = own[1]
        ex.start_broadcast_(logit_r).finish()
        logits = (logit_l, logit_r)
    ctx.padj, ctx.relu, ctx.opts = padj, relu, opts
    ctx.scale = _fc.dropout_scale(dropout)
    # conv1's shape (narrow LP features, aggregates kept, ReLU without dropout): its weight gradients
    # can come out of the next layer's input-gradient GEMMs (foldable_producer)
    ctx.small_relu = (relu and dropout == 0 and agg_l is not None and agg_r is not None
                      and agg_l.shape[1] + left.shape[1] <= 16 and agg_r.shape[1] + right.shape[1] <= 16)
    ctx.has_b = (b_l2r is not None, b_r2l is not None)
    return left_new, right_new, (left, right, agg_l, agg_r, left_new, right_new, w_rel_l2r, w_root_l2r,
                                 w_rel_r2l, w_root_r2l), logits


def _part_forward_f16(left, right, padj, l2r, r2l, relu, opts, defer):
    """One GraphConvTwoDirection layer of the reference's --fp16 evaluation (val.py:269 model.half(),
    utils.py:909-915 batch_to(half=True)) on a row partition: fp16 storage, the one-GPU path's fp16
    kernels and association rule (lpgnn.conv._forward_core), forward only (the reference trains in fp32).
    The vars<-cons aggregate's partial sums are formed and reduced to the owners in fp32 and rounded to
    fp16 once -- as the one-GPU fp16 SpMM sums a row in fp32 and rounds once -- so the partition changes
    only the order of that fp32 sum.  The constraint side is local (bitwise the one-GPU rows).  Returns
    (left_new, right_new) with right_new's halo rows broadcast (deferred with ``defer``, as the fp32 node)."""
    import functools

    from . import fc as _fc
    from .conv import reassociate
    from .sparse import spmm_forward as _spmm_forward

    if torch.is_grad_enabled() and any(p.requires_grad for p in (left, right)):
        raise RuntimeError("the fp16 row-partitioned path is the reference's inference mode: no gradients")
    spmm = functools.partial(_spmm_forward, heavy=opts.spmm_heavy)
    f16 = torch.float16
    w16 = lambda t: t.detach().to(f16)  # noqa: E731 (model.half(): already fp16)
    b32 = lambda t: None if t is None else t.detach()  # noqa: E731 (fc_forward_bf16 adds the bias in fp32)
    w_rel_l2r, b_l2r, w_root_l2r = w16(l2r.lin_rel.weight), b32(l2r.lin_rel.bias), w16(l2r.lin_root.weight)
    w_rel_r2l, b_r2l, w_root_r2l = w16(r2l.lin_rel.weight), b32(r2l.lin_rel.bias), w16(r2l.lin_root.weight)
    fc16 = _fc.fc_forward_bf16  # dispatches the fp16 kernels on fp16 operands (lpg_fc_f16)
    ex = padj.ex
    A, AT = padj.local.fwd, padj.local.bwd
    n_own = ex.n_own
    f_out = w_rel_l2r.shape[0]
    with torch.no_grad():
        ra = reassociate(ex.m, ex.n, left.shape[1], f_out, opts.reassociate)
        src = fc16(left, w_rel_l2r, None, None, None, False) if ra else left
        red = ex.start_reduce(spmm(AT, src.float()), inplace=True)  # fp32 partials -> owners, in flight ...
        ex.settle(right)
        agg_l = spmm(A, right)  # ... under the purely local constraint side (fp16 storage)
        left_new = fc16(agg_l, w_rel_r2l, left, w_root_r2l, b_r2l, relu)
        agg_own = red.finish().to(f16)  # the owners' fp32 sums, rounded once
        right_new = torch.empty((right.shape[0], f_out), dtype=f16, device=left.device)
        if ra:  # lin_root + bias + ReLU accumulated onto the aggregated product
            right_new[:n_own] = agg_own
            fc16(right[:n_own], w_root_l2r, None, None, b_l2r, relu, out=right_new[:n_own], accumulate=True)
        else:
            fc16(agg_own, w_rel_l2r, right[:n_own], w_root_l2r, b_l2r, relu, out=right_new[:n_own])
        bc = ex.start_broadcast_(right_new, quiet=defer)
        if defer:
            ex.defer(right_new, bc)
        else:
            bc.finish()
    return left_new, right_new


def _relu_bwd(ctx, g, y, want_db):
    """(dZ, bias gradient) of a layer output gradient through the layer's ReLU/dropout."""
    from . import fc as _fc

    if not ctx.relu:
        g = g.contiguous()
        return g, (g.sum(0) if want_db else None)
    return _fc.relu_bwd_colsum(g.contiguous(), y, ctx.scale, want_db)


def _part_backward_core(ctx, saved, need, g_left, g_right, dz=None):
    """_PartTwoDirection's backward from the output gradients, or -- dz =
    (dz_l, db_r2l, dz_r_own, db_l2r) -- from gradients that already went
    through the layer's ReLU/dropout, owners' rows reduced (fused heads)."""
    import functools

    from . import fc as _fc
    from .conv import _src_first
    from .sparse import spmm_forward as _spmm_forward

    igf = functools.partial(_fc.input_grad, arith=ctx.opts.arith)
    wgf = functools.partial(_fc.wgrad, arith=ctx.opts.arith)
    spmm_forward = functools.partial(_spmm_forward, heavy=ctx.opts.spmm_heavy)

    left, right, agg_l, agg_r, left_new, right_new, w_rel_l2r, w_root_l2r, w_rel_r2l, w_root_r2l = saved
    ex = ctx.padj.ex
    A, AT = ctx.padj.local.fwd, ctx.padj.local.bwd
    n_own = ex.n_own
    pre = getattr(ctx, "folded_wgk", None)
    if getattr(ctx, "wgk_folded", False) and pre is not None:
        # conv1 whose weight gradients the next layer computed in its input-gradient GEMMs: no pass over
        # its output gradients and no exchange (every rank takes this path alike)
        ctx.folded_wgk = None
        (dw_rel_l2r, dw_root_l2r, db_l2r), (dw_rel_r2l, dw_root_r2l, db_r2l) = pre
        keep = lambda t, i, has=True: t if (need[i] and has) else None  # noqa: E731
        return (None, None, None, keep(dw_rel_l2r, 3), keep(db_l2r, 4, ctx.has_b[0]), keep(dw_root_l2r, 5),
                keep(dw_rel_r2l, 6), keep(db_r2l, 7, ctx.has_b[1]), keep(dw_root_r2l, 8), None, None)
    prev = getattr(ctx, "wgk_prev", None)
    ctx.wgk_prev = None
    if prev is not None and need[0] and need[1]:
        if dz is None:  # through this layer's ReLU/dropout first (halo gradients reduced to the owners)
            g_right = torch.zeros_like(right_new) if g_right is None else g_right
            g_left = torch.zeros_like(left_new) if g_left is None else g_left
            red = ex.start_reduce(g_right.contiguous(), inplace=False)
            dz_l, db_r2l = _relu_bwd(ctx, g_left, left_new, ctx.has_b[1] and need[7])
            dz_r, db_l2r = _relu_bwd(ctx, red.finish(), right_new[:n_own], ctx.has_b[0] and need[4])
            dz = (dz_l, db_r2l, dz_r, db_l2r)
        return _part_backward_folded(ctx, saved, need, dz, prev, igf, wgf, spmm_forward)
    if dz is None:
        if g_right is None:
            g_right = torch.zeros_like(right_new)
        if g_left is None:
            g_left = torch.zeros_like(left_new)
        red = ex.start_reduce(g_right.contiguous(), inplace=False)  # halo grads -> owners, in flight ...

    def mask(g, y, want_db):
        return _relu_bwd(ctx, g, y, want_db)

    def wgrads(dz, agg, x_dst, need_rel, need_root):
        if not (need_rel or need_root):
            return None, None
        if agg is not None and agg.shape[1] + x_dst.shape[1] <= 16 and dz.shape[1] % 4 == 0:
            d_rel, d_root = _fc.wgrad_smallk(dz, agg.contiguous(), x_dst.contiguous())
        else:
            d_rel = wgf(dz, agg) if need_rel else None
            d_root = wgf(dz, x_dst) if need_root else None
        return (d_rel if need_rel else None), (d_root if need_root else None)

    def narrow(agg, x_dst):  # conv1: the inputs are features -- weight gradients straight from (g, y)
        return (dz is None and ctx.relu and not (need[0] or need[1]) and agg is not None
                and agg.shape[1] + x_dst.shape[1] <= 16 and left_new.shape[1] % 4 == 0)

    # ... under everything that only needs the constraint side's gradient
    if dz is not None:
        dz_l, db_r2l = dz[0], dz[1]
        dw_rel_r2l, dw_root_r2l = wgrads(dz_l, agg_l, left, need[6], need[8])
    elif narrow(agg_l, left):
        dz_l = None
        dw_rel_r2l, dw_root_r2l, db_r2l = _fc.relu_wgrad_smallk(g_left, left_new, ctx.scale, agg_l, left,
                                                                ctx.has_b[1] and need[7])
    else:
        dz_l, db_r2l = mask(g_left, left_new, ctx.has_b[1] and need[7])
        dw_rel_r2l, dw_root_r2l = wgrads(dz_l, agg_l, left, need[6], need[8])
    g_r = None
    if need[1]:  # right [owned | halo] as the source of right2left: every local row
        if _src_first(A, dz_l.shape[1], w_rel_r2l.shape[1], 4):
            g_r = igf(spmm_forward(AT, dz_l), w_rel_r2l)
        else:
            g_r = spmm_forward(AT, igf(dz_l, w_rel_r2l))
    g_right_own = red.finish() if dz is None else None
    if narrow(agg_r, right):
        dw_rel_l2r, dw_root_l2r, db_l2r = _fc.relu_wgrad_smallk(g_right_own, right_new[:n_own], ctx.scale,
                                                                agg_r[:n_own], right[:n_own],
                                                                ctx.has_b[0] and need[4])
        return (None, None, None, dw_rel_l2r if need[3] else None, db_l2r, dw_root_l2r if need[5] else None,
                dw_rel_r2l if need[6] else None, db_r2l, dw_root_r2l if need[8] else None, None, None)
    if dz is None:
        dz_r, db_l2r = mask(g_right_own, right_new[:n_own], ctx.has_b[0] and need[4])
    else:
        dz_r, db_l2r = dz[2], dz[3]
    # with T = A bcast(dZ_r) (computed for left's gradient below), lin_rel's weight gradient
    # dZ_r^T reduce(A^T left) = T^T left runs over the local constraints instead of the variables
    # (and is the only route when the forward was re-associated: agg_r was not kept)
    first = need[0] and _src_first(AT, dz_r.shape[1], w_rel_l2r.shape[1], 4)
    rel_from_t = need[3] and (agg_r is None or (first and A.n_rows < ex.n_own))
    use_t = first or rel_from_t
    bc = full = None
    if need[0] or use_t:  # left: source of left2right through reduce(AT @ left)[:n_own]
        f_out, f_in = dz_r.shape[1], w_rel_l2r.shape[1]
        if use_t and right.shape[0] == n_own and dz_r.is_contiguous():
            full = dz_r  # no halo rows (one rank): dZ_r is the whole source table, no copy
        else:
            full = torch.empty((right.shape[0], f_out if use_t else f_in), dtype=torch.float32, device=left.device)
            if use_t:
                full[:n_own] = dz_r
            else:
                igf(dz_r, w_rel_l2r, out=full[:n_own])
        bc = ex.start_broadcast_(full)           # owners' aggregate gradient -> halo rows, in flight ...
    # ... under the weight gradients and the variables' root-path and the constraints' root-path gradients
    dw_rel_l2r, dw_root_l2r = wgrads(dz_r, None if agg_r is None else agg_r[:n_own], right[:n_own],
                                     need[3] and not rel_from_t, need[5])
    if need[1]:  # ... and as the destination of left2right (owned rows)
        igf(dz_r, w_root_l2r, out=g_r[:n_own], accumulate=True)

    g_l = None
    if bc is not None:
        root = igf(dz_l, w_root_r2l) if need[0] else None
        bc.finish()
        if use_t:
            t = spmm_forward(A, full)
            if rel_from_t:
                dw_rel_l2r = wgf(t, left)
            if need[0]:
                g_l = igf(t, w_rel_l2r, out=root, accumulate=True)
        else:
            g_l = spmm_forward(A, full).add_(root)
    return (g_l, g_r, None, dw_rel_l2r, db_l2r, dw_root_l2r, dw_rel_r2l, db_r2l, dw_root_r2l, None, None)


def _part_backward_folded(ctx, saved, need, dz, prev, igf, wgf, spmm_forward):
    """_part_backward_core of the layer after conv1 (gradients through its ReLU/dropout given, dz) with
    conv1's weight gradients folded into this layer's input-gradient GEMMs (lpg_fc_x3_relu_wgrad_f32:
    the masked tile times conv1's 8 + 8 inputs, never storing conv1's output gradient).

    Variables: conv1's output gradient on an owned variable is the source-side term of right2left summed
    over every rank that touches it, plus the root term of left2right.  The source-side term's halo
    rows are REDUCED to their owners before the fused GEMM (the exchange conv1's own backward would
    have done on the product): T = A^T dZ_l (then (T W_rel + dZ_r W_root) in one two-part GEMM) or
    P = A^T (dZ_l W_rel) (then dZ_r W_root + P), whichever association the one-GPU path takes.
    Constraints are local: conv.py's fold as is.
    conv1's node receives zero-stride gradients and returns the handed weight gradients."""
    from . import fc as _fc

    left, right, agg_l, agg_r, left_new, right_new, w_rel_l2r, w_root_l2r, w_rel_r2l, w_root_r2l = saved
    ex = ctx.padj.ex
    A, AT = ctx.padj.local.fwd, ctx.padj.local.bwd
    n_own = ex.n_own
    dz_l, db_r2l, dz_r, db_l2r = dz
    p_left, p_right, p_agg_l, p_agg_r, p_left_new, p_right_new = prev.saved_tensors[:6]
    from .conv import _src_first

    # Both exchanges are issued first and finished where their rows are consumed, so they run under the
    # four weight-gradient GEMMs (which need neither): the source-side term of conv1's left2right
    # (below) to the owners, and the owners' aggregate gradient to the halo rows.
    src_first = _src_first(A, dz_l.shape[1], w_rel_r2l.shape[1], 4)
    red = ex.start_reduce(spmm_forward(AT, dz_l if src_first else igf(dz_l, w_rel_r2l)), inplace=True)
    f_out, f_in = dz_r.shape[1], w_rel_l2r.shape[1]
    use_t = _src_first(AT, f_out, f_in, 4) or agg_r is None
    rel_from_t = need[3] and (agg_r is None or (use_t and A.n_rows < n_own))
    if use_t and right.shape[0] == n_own and dz_r.is_contiguous():
        full = dz_r  # no halo rows (one rank): dZ_r is the whole source table, no copy
    else:
        full = torch.empty((right.shape[0], f_out if use_t else f_in), dtype=torch.float32, device=left.device)
        if use_t:
            full[:n_own] = dz_r
        else:
            igf(dz_r, w_rel_l2r, out=full[:n_own])
    bc = ex.start_broadcast_(full)
    # ... under: this layer's weight gradients, both directions
    dw_rel_r2l, dw_root_r2l = (wgf(dz_l, agg_l) if need[6] else None), (wgf(dz_l, left) if need[8] else None)
    dw_rel_l2r = wgf(dz_r, agg_r[:n_own]) if need[3] and not rel_from_t else None
    dw_root_l2r = wgf(dz_r, right[:n_own]) if need[5] else None

    def fused(G1, W1, G2, W2, addend, y, x1, x2, two_pass):
        r = _fc.input_grad_relu_wgrad(G1, W1, G2, W2, addend, y, x1, x2, arith=ctx.opts.arith)
        if r is None:  # operands the fused kernel does not take: the stored gradient, then conv1's pass
            r = _fc.relu_wgrad_smallk(two_pass(), y, 1.0, x1, x2, True)
        return r

    # conv1's left2right (owned variables): the source-side term's halo partials reduced to the owners,
    # then the fused GEMM -- in the association the one-GPU path picks (conv._src_first): (A^T dZ_l) W_rel
    # over the variables, or A^T (dZ_l W_rel) with the GEMM over the constraints and the reduced SpMM
    # output as the fused kernel's addend
    if src_first:
        T_own = red.finish()

        def g_right_own():
            g = igf(T_own, w_rel_r2l)
            return igf(dz_r, w_root_l2r, out=g, accumulate=True)
        wk_r = fused(T_own, w_rel_r2l, dz_r, w_root_l2r, None, p_right_new[:n_own], p_agg_r[:n_own],
                     p_right[:n_own], g_right_own)
    else:
        P_own = red.finish()

        def g_right_own():
            return igf(dz_r, w_root_l2r, out=P_own.clone(), accumulate=True)
        wk_r = fused(dz_r, w_root_l2r, None, None, P_own, p_right_new[:n_own], p_agg_r[:n_own], p_right[:n_own],
                     g_right_own)

    # conv1's right2left (constraints, local) from the broadcast aggregate gradient
    bc.finish()
    t = spmm_forward(A, full)
    if use_t:
        if rel_from_t:
            dw_rel_l2r = wgf(t, left)

        def g_left():
            g = igf(dz_l, w_root_r2l)
            return igf(t, w_rel_l2r, out=g, accumulate=True)
        wk_l = fused(t, w_rel_l2r, dz_l, w_root_r2l, None, p_left_new, p_agg_l, p_left, g_left)
    else:
        def g_left():
            return igf(dz_l, w_root_r2l, out=t.clone(), accumulate=True)
        wk_l = fused(dz_l, w_root_r2l, None, None, t, p_left_new, p_agg_l, p_left, g_left)
    prev.folded_wgk = (wk_r, wk_l)
    g_l = torch.zeros((), dtype=left.dtype, device=left.device).expand(left.shape)
    g_r = torch.zeros((), dtype=right.dtype, device=right.device).expand(right.shape)
    return (g_l, g_r, None, dw_rel_l2r, db_l2r, dw_root_l2r, dw_rel_r2l, db_r2l, dw_root_r2l, None, None)


class _PartTwoDirectionHeads(torch.autograd.Function):
    """The last hidden layer + heads on a partition (conv._TwoDirectionHeads'
    twin).  Backward: the halo rows' LOGIT gradients (3 wide) are reduced to
    their owners -- a halo row is a copy of its owner's output, so the owner's
    layer-output gradient is (its own + its halo copies' logit gradients) W --
    then one pass over the owned rows gives dZ, the head and bias gradients
    (lpg_heads_relu_bwd_f32)."""

    @staticmethod
    def forward(ctx, left, right, padj, w_rel_l2r, b_l2r, w_root_l2r, w_rel_r2l, b_r2l, w_root_r2l, relu, dropout,
                wh_l, bh_l, wh_r, bh_r, opts=None, prev=None):
        import functools

        from . import fc as _fc
        from .options import DEFAULT

        opts = DEFAULT if opts is None else opts
        _link_prev(ctx, prev)
        fcf = functools.partial(_fc.fc_forward, arith=opts.arith)
        left_new, right_new, saved, logits = _part_forward_core(
            ctx, left, right, padj, w_rel_l2r, b_l2r, w_root_l2r, w_rel_r2l, b_r2l, w_root_r2l, relu, dropout,
            heads=((wh_l, bh_l), (wh_r, bh_r)) if opts.fuse_head_fwd else None, opts=opts)
        if logits is None:
            logits = (fcf(left_new, wh_l, None, None, bh_l, False),
                      fcf(right_new, wh_r, None, None, bh_r, False))
        logit_l, logit_r = logits
        ctx.heads_b = (bh_l is not None, bh_r is not None)
        ctx.save_for_backward(*saved, wh_l, wh_r)
        return logit_l, logit_r

    @staticmethod
    def backward(ctx, g_ll, g_lr):
        from . import fc as _fc

        *saved, wh_l, wh_r = ctx.saved_tensors
        need = ctx.needs_input_grad
        left_new, right_new = saved[4], saved[5]
        ex = ctx.padj.ex
        g_ll = torch.zeros(left_new.shape[0], wh_l.shape[0], device=left_new.device) if g_ll is None else g_ll
        g_lr = torch.zeros(right_new.shape[0], wh_r.shape[0], device=right_new.device) if g_lr is None else g_lr
        red = ex.start_reduce(g_lr.contiguous(), inplace=False)  # halo logit grads -> owners, in flight ...
        # dZ is only read below (copied into a [owned | halo] buffer where halo rows exist): its f16x2 scales
        # come out of the same pass (heads_relu_bwd with the model's arithmetic)
        ar = ctx.opts.arith
        dz_l, dwh_l, dbh_l, db_r2l = _fc.heads_relu_bwd(g_ll, wh_l, left_new, ctx.scale, ctx.has_b[1] and need[7],
                                                        arith=ar)
        g_own = red.finish()
        dz_r, dwh_r, dbh_r, db_l2r = _fc.heads_relu_bwd(g_own, wh_r, right_new[:ex.n_own], ctx.scale,
                                                        ctx.has_b[0] and need[4], arith=ar)
        core = _part_backward_core(ctx, saved, need, None, None, dz=(dz_l, db_r2l, dz_r, db_l2r))
        keep = lambda t, i, has=True: t if (need[i] and has) else None
        return (*core, keep(dwh_l, 11), keep(dbh_l, 12, ctx.heads_b[0]), keep(dwh_r, 13),
                keep(dbh_r, 14, ctx.heads_b[1]), None, None)


class PartitionedCSR:
    """The edge_index of a rank's batch: local dual CSR + boundary exchange.

    orient "cons": A_p, rows = local cons (cons<-vars, local only);
    orient "vars": A_p^T, rows = local vars (vars<-cons, reduce/broadcast).
    """

    def __init__(self, local: BipartiteCSR, ex: Exchange, orient: str = "cons"):
        self.local, self.ex, self.orient = local, ex, orient

    def t(self) -> "PartitionedCSR":
        return PartitionedCSR(self.local.t(), self.ex, "vars" if self.orient == "cons" else "cons")

    def to(self, device, non_blocking: bool = False) -> "PartitionedCSR":
        """batch_to (utils.py:909-915): a partition lives on its rank's device already."""
        if torch.device(device) != self.device and not (torch.device(device).index is None
                                                         and torch.device(device).type == self.device.type):
            raise RuntimeError(f"a row partition stays on its rank's device {self.device}, not {device}")
        return self

    def half(self) -> "PartitionedCSR":
        """SparseTensor.half() (batch_to(half=True), the reference's --fp16 mode): the local edge values
        rounded to fp16 (kept in fp32 storage), as BipartiteCSR.half()."""
        return PartitionedCSR(self.local.half(), self.ex, self.orient)

    def sparse_sizes(self):
        return self.local.sparse_sizes()

    def nnz(self) -> int:
        return self.local.nnz()

    @property
    def device(self):
        return self.local.device

    def two_direction_conv(self, left, right, left2right, right2left, relu=False, dropout=0.0, opts=None,
                           fold_in=False, feeds_conv=False):
        """GraphConvTwoDirection.forward on this partition (one autograd node).  ``fold_in``: (left,
        right) feed nothing but this layer (GCN_FC's chain): if conv1 produced them, its weight
        gradients come out of this layer's input-gradient GEMMs.  ``feeds_conv``: the outputs go only
        to another partitioned layer (GCN_FC's chain), which settles the broadcast of their halo rows
        itself -- it stays in flight under that layer's first GEMM and SpMM (Exchange.defer)."""
        if self.orient == "cons" and left.dtype == torch.float16 and _local_spmm is _product_spmm:
            from .options import DEFAULT

            return _part_forward_f16(left, right, self, left2right, right2left, bool(relu), opts or DEFAULT,
                                     bool(feeds_conv))
        if self.orient != "cons" or left.dtype != torch.float32 or _local_spmm is not _product_spmm:
            return None  # generic per-direction path (oracle tests, bf16)
        from .options import DEFAULT

        prev = foldable_producer(left, right, opts or DEFAULT) if fold_in else None
        return _PartTwoDirection.apply(left, right, self, left2right.lin_rel.weight, left2right.lin_rel.bias,
                                       left2right.lin_root.weight, right2left.lin_rel.weight,
                                       right2left.lin_rel.bias, right2left.lin_root.weight, bool(relu),
                                       float(dropout), opts, prev, bool(feeds_conv))

    def two_direction_heads(self, left, right, left2right, right2left, lin_left, lin_right, dropout=0.0, opts=None,
                            fold_in=False):
        """The last layer + heads (arch.py:184-190) on this partition, one autograd node (None: not applicable)."""
        if self.orient != "cons" or left.dtype != torch.float32 or _local_spmm is not _product_spmm:
            return None
        from .options import DEFAULT

        prev = foldable_producer(left, right, opts or DEFAULT) if fold_in else None
        return _PartTwoDirectionHeads.apply(left, right, self, left2right.lin_rel.weight, left2right.lin_rel.bias,
                                            left2right.lin_root.weight, right2left.lin_rel.weight,
                                            right2left.lin_rel.bias, right2left.lin_root.weight, True,
                                            float(dropout), lin_left.weight, lin_left.bias, lin_right.weight,
                                            lin_right.bias, opts, prev)

    def partitioned_conv(self, x, fc):
        """One GraphConv direction: fc(agg, x_dst) is lin_rel + lin_root (+ReLU, +dropout)."""
        agg = _local_spmm(self.local, x[0])
        ex = self.ex
        if self.orient == "cons":
            return fc(agg, x[1], **ex.cons_key_args)
        agg_own = _Reduce.apply(agg, ex)
        out_own = fc(agg_own, x[1][:ex.n_own], **ex.var_key_args)
        return _Broadcast.apply(out_own, ex)


def make_local_batch(plan: PartitionPlan, x_s, x_t, y_s, y_t, device, group=None):
    """Rank-local BipartiteBatch whose edge_index is a PartitionedCSR, from
    GLOBAL node arrays (sliced here)."""
    lv = plan.local_vars
    sl = lambda a, idx: None if a is None else np.asarray(a)[idx]
    rows = slice(plan.row_lo, plan.row_hi)
    return local_batch(plan, sl(x_s, rows), sl(x_t, lv), sl(y_s, rows), sl(y_t, lv), device, group)


def make_block_batch(spec, plan: PartitionPlan, device, group=None, cons=None):
    """Rank-local batch of a synth.BlockLP partition: only this rank's
    constraint blocks and its [owned | halo] variables are generated.
    cons: the rank's (x_s, y_s) if already generated."""
    per = spec.blocks // plan.world
    b0 = plan.rank * per
    if cons is None:
        cons = [spec.cons_block(b) for b in range(b0, b0 + per)]
        cons = (np.concatenate([c[0] for c in cons]), np.concatenate([c[1] for c in cons]))
    x_t, y_t = spec.var_rows(plan.local_vars)
    return local_batch(plan, cons[0], x_t, cons[1], y_t, device, group)


def lp_partition_batch(record, world: int, rank: int, device, group=None):
    """This rank's batch of a processed LP record ([row, col, A_data, c_feas, v_feas, y_s, y_t,
    nnodes], dataset.py:213-217 -- what lpio.msgpack_load returns for a .pk file): the rank-local plan
    (plan_partition_local over the host edge list), its constraint block and [owned | halo] variable
    rows, the local dual CSR and boundary exchange on `device`.  The checks of LPDataset.get
    (dataset.py:235-238) apply to the whole record, as there."""
    row, col, A_data, c_feas, v_feas, y_s, y_t, nnodes = record
    A_data = np.asarray(A_data)
    c_feas, v_feas = np.asarray(c_feas, np.float32), np.asarray(v_feas, np.float32)
    assert A_data.max() <= 1 and A_data.min() >= -1  # dataset.py:235-236
    assert c_feas.max() <= 1 and c_feas.min() >= -1  # dataset.py:237-238
    m, n = c_feas.shape[0], v_feas.shape[0]
    assert int(nnodes) == m + n
    plan = plan_partition_local(row, col, A_data.astype(np.float32), m, n, world, rank, group)
    lv = plan.local_vars
    y_s, y_t = np.asarray(y_s, np.int64), np.asarray(y_t, np.int64)
    rows = slice(plan.row_lo, plan.row_hi)
    return local_batch(plan, c_feas[rows], v_feas[lv], y_s[rows], y_t[lv], device, group)


def gather_logits(lc: torch.Tensor, lv: torch.Tensor, batch, group=None):
    """The whole graph's (cons [m, C], vars [n, C]) logits on every rank from the ranks' partitioned
    outputs: each rank contributes its constraint block and its OWNED variables (a halo row is a copy
    of its owner's); one padded all_gather.  For the metrics of lpgnn.run (accuracy, validation)."""
    plan = batch.plan
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    own = torch.cat((lc.detach().float(), lv.detach().float()[:plan.n_own]))
    if world == 1:
        return own[:plan.m_local].clone(), own[plan.m_local:].clone()
    gloo = dist.get_backend(group) == "gloo"
    cnt = torch.tensor([own.shape[0]], dtype=torch.int64, device="cpu" if gloo else own.device)
    cnts = [torch.empty_like(cnt) for _ in range(world)]
    dist.all_gather(cnts, cnt, group=group)
    cnts = [int(c.item()) for c in cnts]
    big = max(cnts)
    pad = own.new_zeros((big, own.shape[1]))
    pad[:own.shape[0]] = own
    if gloo:
        pad = pad.cpu()
    parts = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(parts, pad, group=group)
    # every rank's block bounds and owned ids (host metadata, once per call)
    meta = [None] * world
    dist.all_gather_object(meta, (plan.row_lo, plan.row_hi, plan.owned), group=group)
    C = own.shape[1]
    cons = own.new_empty((plan.m, C))
    var = own.new_empty((plan.n, C))
    for q, (lo, hi, owned) in enumerate(meta):
        p = parts[q].to(own.device)
        cons[lo:hi] = p[:hi - lo]
        var[torch.from_numpy(np.asarray(owned)).to(own.device)] = p[hi - lo:cnts[q]]
    return cons, var


def local_batch(plan: PartitionPlan, x_s, x_t, y_s, y_t, device, group=None):
    """Rank-local BipartiteBatch from rank-LOCAL node arrays: x_s/y_s of the
    rows [row_lo, row_hi), x_t/y_t of local_vars ([owned | halo])."""
    from .data import BipartiteBatch

    local = local_dual_csr(plan, device)
    lv = plan.local_vars
    adj = PartitionedCSR(local, Exchange(plan, device, group))
    dev = lambda a: None if a is None else torch.as_tensor(np.ascontiguousarray(a)).to(device)
    b = BipartiteBatch(x_s=dev(x_s), x_t=dev(x_t), y_s=dev(y_s), y_t=dev(y_t),
                       edge_index=adj, s_bs=plan.m_local, t_bs=plan.n_local, bs=plan.m_local + plan.n_local)
    b.var_owned = torch.from_numpy(plan.var_owned).to(device)
    b.n_own = plan.n_own
    b.local_vars = torch.from_numpy(lv)
    b.plan = plan
    return b


# ----------------------------------------------------------------------- loss
def _balanced_weights_from_counts(cnt: torch.Tensor) -> torch.Tensor:
    """labels_to_balanced_weights (utils.py:286-299) from global counts,
    without host syncs (the same formula as lpgnn.train's)."""
    present = cnt > 0
    tot = cnt.sum().to(torch.float32)
    res = torch.where(present, tot / cnt.to(torch.float32), torch.zeros((), device=cnt.device))
    merged = (res[0] + res[2]) / 2.
    two = present.sum() == 2
    return torch.stack([torch.where(two, res[0], merged), res[1], torch.where(two, res[2], merged)])


def balanced_distributed(lc, lv, y_s, y_t, var_owned, group=None):
    """Per-rank share of train.py:39-46 so that sum over ranks == the
    single-graph balanced loss (class weights and the weighted-mean
    denominators are global).  `var_owned`: the number of owned variables
    (they are the first local rows) or the legacy boolean mask.  No host sync."""
    if isinstance(var_owned, int):
        yt, lv = y_t[:var_owned], lv[:var_owned]
    else:
        yt, lv = y_t[var_owned], lv[var_owned]
    ys = y_s
    cnt = torch.zeros(6, dtype=torch.int64, device=ys.device)  # integer atomics: fp64 ones serialise on 3 bins
    cnt[:3].scatter_add_(0, ys, torch.ones_like(ys))
    cnt[3:].scatter_add_(0, yt, torch.ones_like(yt))
    cnt = cnt.to(torch.float64)
    _all_reduce_(cnt, group)
    cs, ct = cnt[:3], cnt[3:]
    m, n = cs.sum(), ct.sum()
    ws, wt = _balanced_weights_from_counts(cs), _balanced_weights_from_counts(ct)
    ce_s = F.cross_entropy(lc, ys, reduction="none")
    ce_t = F.cross_entropy(lv, yt, reduction="none")
    den = torch.stack([ws[ys].sum(), wt[yt].sum()]).to(torch.float64)
    _all_reduce_(den, group)
    return ((m + n) / m).float() * (ws[ys] * ce_s).sum() / den[0].float() + \
        ((m + n) / n).float() * (wt[yt] * ce_t).sum() / den[1].float()


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
    loss = balanced_distributed(lc, lv, batch.y_s, batch.y_t, batch.n_own, group)
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
    batch: object
    spec: object


def bench_spec(args, world: int):
    """c4 (BASELINE.json configs[3]): the fixed 2M x 4M, nnz 40M, 8-block
    graph split over `world` ranks -- strong scaling.  Otherwise weak
    scaling: `world` blocks of args.m x args.n, args.nnz each."""
    from . import synth

    if args.config == "c4":
        return synth.BlockLP(args.m, args.n, args.nnz, blocks=8, rho=args.rho, seed=0)
    return synth.BlockLP(args.m * world, args.n * world, args.nnz * world, blocks=world, rho=args.rho, seed=0)


def build_bench_job(args, rank: int, world: int, device) -> BenchJob:
    """One rank's share of the bench graph: the rank generates and plans only
    its own row blocks and [owned | halo] variables (plan_partition_blocks)."""
    from .arch import GCN_FC
    from .train import make_optimizer

    spec = bench_spec(args, world)
    per = spec.blocks // world
    row, col, val, x_s, y_s = spec.rows(rank * per, (rank + 1) * per)
    plan = plan_partition_blocks(spec, world, rank, edges=(row, col, val))
    del row, col, val
    batch = make_block_batch(spec, plan, device, cons=(x_s, y_s))
    torch.manual_seed(0)
    model = GCN_FC(8, 8, hids=args.hids, depth=args.depth).to(device)
    opt, _ = make_optimizer(model)
    step = lambda: train_step_distributed(model, batch, opt)
    kind = ("c4: synthetic block LP" if args.config == "c4" else
            f"{args.config} weak scaling: {world} x ({args.m}x{args.n}, nnz {args.nnz}) blocks,")
    wl = (f"{kind} {spec.m}x{spec.n} nnz={spec.nnz} ({spec.blocks} row blocks, rho={spec.rho}) row-partitioned "
          f"over {world} GPU(s), GCN_FC(8,8,hids={args.hids},depth={args.depth}) fwd+bwd+Adam")
    return BenchJob(step, plan.nnz_local, wl, plan, batch, spec)


def rho_sweep(args, rank: int, world: int, rhos, F: int) -> list:
    """SURVEY.md §8d/§8e's locality sweep for the bench graph: for each rho (the fraction of a
    block's edges on other blocks' variables) this rank generates and plans its own blocks again
    and the ranks pool their boundary counts.  Per rho: boundary variables (touched by >= 2
    ranks), halo rows per rank, rows each rank sends + receives in one exchange, and the MiB that
    moves per exchange at width F (fp32) on the busiest rank -- the plan, not a timing."""
    import copy

    out = []
    for rho in rhos:
        a = copy.copy(args)
        a.rho = float(rho)
        spec = bench_spec(a, world)
        plan = plan_partition_blocks(spec, world, rank)
        mine = [int(plan.halo.shape[0]), int(plan.n_own), int(sum(plan.send_counts)), int(sum(plan.recv_counts)),
                len({r for r, c in enumerate(plan.send_counts) if c and r != rank} |
                    {r for r, c in enumerate(plan.recv_counts) if c and r != rank})]  # distinct peer ranks
        every = [None] * world
        dist.all_gather_object(every, mine)
        rows = [h[2] + h[3] for h in every]
        out.append({"rho": float(rho), "boundary_vars_global": plan.n_boundary_global,
                    "halo_rows_per_rank": [h[0] for h in every], "owned_vars_per_rank": [h[1] for h in every],
                    "exchange_rows_per_rank": rows, "peers_max": max(h[4] for h in every),
                    "mib_per_exchange_max": max(rows) * F * 4 / 2 ** 20})
        del plan
    return out


def time_exchange(ex: Exchange, F: int, device, reps: int = 5) -> dict:
    """Standalone cost of one boundary exchange at width F (outside the timed
    steps): an owner reduce and a halo broadcast of [n_local, F] fp32 rows,
    barrier + device sync around each; median ms.  Inside the training step
    the same exchanges run asynchronously under independent compute."""
    import time

    full = torch.zeros((ex.n_local, F), dtype=torch.float32, device=device)
    out = {"reduce_ms": [], "broadcast_ms": []}
    for _ in range(reps + 1):
        for name, fn in (("reduce_ms", lambda: ex.reduce_rows(full, inplace=True)),
                         ("broadcast_ms", lambda: ex.broadcast_rows_(full))):
            torch.cuda.synchronize(device)
            dist.barrier()
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize(device)
            out[name].append((time.perf_counter() - t0) * 1e3)
    res = {k: float(np.median(v[1:])) for k, v in out.items()}
    res["rows_out"] = int(sum(ex.send_counts))
    res["rows_in"] = int(sum(ex.recv_counts))
    res["bytes_per_exchange"] = (res["rows_out"] + res["rows_in"]) * F * 4
    return res
