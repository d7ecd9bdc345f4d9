"""The dense boundary all-reduce of the row partition, in native code (include/lpgnn.h "multi-GPU":
lpg_spmm_partitioned_f32, lpg_boundary_*_f32, lpg_comm_*; SURVEY.md §8b "Multi-GPU", §8e).

SURVEY.md §8e's exchange: after the local vars<-cons SpMM a boundary variable (touched by >= 2
ranks' constraint blocks) holds only this rank's partial sum; one RCCL all-reduce (sum) of the dense
``[n_boundary, F]`` buffer ``Bbuf`` -- boundary variables in ascending GLOBAL id, zero rows for the
ones a rank does not touch -- gives every touching rank the full sums.  ``lpgnn.partition``'s
training path uses the sparse owner form of the same sum (all_to_all of only the rows that cross,
through torch.distributed); this module is the library-level form a non-Python host binds
(INTEGRATION.md), with the collective issued by the library on the caller's stream over a
communicator of its own (``LibComm``).

The reference has no distributed code (train.py:81-82).
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch
import torch.distributed as dist

from . import _lib
from .sparse import CSR

COMM_ID_BYTES = 128  # LPG_COMM_ID_BYTES


class LibComm:
    """The library's RCCL communicator over the ranks of ``group`` (torch.distributed, any backend; a
    single rank when torch.distributed is not initialised): rank 0 draws the unique id
    (lpg_comm_unique_id), ``group`` broadcasts it, every rank joins (lpg_comm_init, collective) on
    ``device``.  ``close()`` (or the context manager) destroys it."""

    def __init__(self, device, group=None):
        L = _lib.lib()
        device = torch.device(device)
        if device.type != "cuda":
            raise RuntimeError("lpgnn LibComm: RCCL needs a HIP device (there is no CPU path)")
        on = dist.is_available() and dist.is_initialized()
        self.rank = dist.get_rank(group) if on else 0
        self.world = dist.get_world_size(group) if on else 1
        uid = (ctypes.c_char * COMM_ID_BYTES)()
        if self.rank == 0:
            _lib.check(L.lpg_comm_unique_id(uid), "lpg_comm_unique_id")
        if self.world > 1:
            t = torch.frombuffer(bytearray(uid.raw), dtype=torch.uint8).clone()
            if dist.get_backend(group) == "nccl":
                t = t.to(device)
            src = dist.get_global_rank(group, 0) if group is not None else 0
            dist.broadcast(t, src=src, group=group)
            uid = (ctypes.c_char * COMM_ID_BYTES).from_buffer_copy(t.cpu().numpy().tobytes())
        self.handle = ctypes.c_void_p()
        self.device = device
        with torch.cuda.device(device):
            _lib.check(L.lpg_comm_init(ctypes.byref(self.handle), self.world, uid, self.rank), "lpg_comm_init")

    def info(self) -> tuple:
        """(nranks, rank) as RCCL reports them (lpg_comm_info)."""
        n, r = ctypes.c_int32(), ctypes.c_int32()
        _lib.check(_lib.lib().lpg_comm_info(self.handle, ctypes.byref(n), ctypes.byref(r)), "lpg_comm_info")
        return n.value, r.value

    def close(self) -> None:
        if self.handle:
            _lib.check(_lib.lib().lpg_comm_destroy(self.handle), "lpg_comm_destroy")
            self.handle = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def boundary_vars(halos: list) -> np.ndarray:
    """The global boundary variables (ascending) from every rank's halo: a variable in some rank's
    halo is touched by that rank and by its owner (the rank with most of its edges), and every
    variable touched by >= 2 ranks is in the halo of each non-owner -- so the union is exactly the
    variables touched by >= 2 ranks."""
    hs = [np.asarray(h, dtype=np.int64) for h in halos]
    return np.unique(np.concatenate(hs)) if hs else np.zeros(0, np.int64)


def boundary_map(local_vars: np.ndarray, gb: np.ndarray) -> np.ndarray:
    """int32 [len(gb)]: the local row of global boundary variable gb[b] on a rank whose local rows
    hold the global variables ``local_vars`` (PartitionPlan.local_vars: [owned | halo]), or -1."""
    lv = np.asarray(local_vars, dtype=np.int64)
    if gb.shape[0] == 0:
        return np.zeros(0, np.int32)
    order = np.argsort(lv, kind="stable")
    pos = np.searchsorted(lv[order], gb)
    pos_c = np.minimum(pos, max(lv.shape[0] - 1, 0))
    hit = (pos < lv.shape[0]) & (lv[order][pos_c] == gb) if lv.shape[0] else np.zeros(gb.shape[0], bool)
    out = np.full(gb.shape[0], -1, np.int32)
    out[hit] = order[pos_c[hit]].astype(np.int32)
    return out


def plan_boundary(plan, group=None) -> tuple:
    """(global boundary ids, this rank's int32 map) of a PartitionPlan; collective over ``group``
    (the halos are gathered) when torch.distributed is initialised with more than one rank."""
    on = dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1
    if on:
        halos = [None] * dist.get_world_size(group)
        dist.all_gather_object(halos, np.asarray(plan.halo, np.int64), group=group)
    else:
        halos = [plan.halo]
    gb = boundary_vars(halos)
    return gb, boundary_map(plan.local_vars, gb)


def _check_rows(y: torch.Tensor, bmap: torch.Tensor, buf: torch.Tensor) -> tuple:
    if y.dtype != torch.float32 or buf.dtype != torch.float32 or bmap.dtype != torch.int32:
        raise RuntimeError("lpgnn boundary: fp32 rows / buffer and an int32 map expected")
    if y.dim() != 2 or y.stride(1) != 1 or not buf.is_contiguous() or not bmap.is_contiguous():
        raise RuntimeError("lpgnn boundary: row-major rows, contiguous buffer and map expected")
    nb, F = bmap.shape[0], y.shape[1]
    if buf.shape != (nb, F):
        raise RuntimeError(f"lpgnn boundary: buffer must be [{nb}, {F}], got {tuple(buf.shape)}")
    if not (y.device == buf.device == bmap.device) or y.device.type != "cuda":
        raise RuntimeError("lpgnn boundary: rows, map and buffer on one HIP device (there is no CPU path)")
    return nb, F


def boundary_pack(y: torch.Tensor, bmap: torch.Tensor, buf: torch.Tensor | None = None) -> torch.Tensor:
    """buf[b] = y[bmap[b]] (zero rows where bmap[b] is -1): lpg_boundary_pack_f32."""
    if buf is None:
        buf = torch.empty((bmap.shape[0], y.shape[1]), dtype=torch.float32, device=y.device)
    nb, F = _check_rows(y, bmap, buf)
    with torch.cuda.device(y.device):
        st = _lib.lib().lpg_boundary_pack_f32(y.data_ptr(), y.stride(0), y.shape[0], F, nb, bmap.data_ptr(),
                                              buf.data_ptr(), _lib.stream_of(y))
    _lib.check(st, "lpg_boundary_pack_f32")
    return buf


def _forget_scales(y: torch.Tensor) -> None:
    """y was rewritten through its pointer (a write autograd's version counter does not see): drop any f16x2
    row / column scales cached on its storage (lpgnn.fc._ScaleCache), as the FC's ``out=`` paths do."""
    from .fc import _SCALES

    _SCALES.forget(y)


def boundary_unpack_(y: torch.Tensor, bmap: torch.Tensor, buf: torch.Tensor) -> torch.Tensor:
    """y[bmap[b]] = buf[b] where bmap[b] >= 0, in place: lpg_boundary_unpack_f32."""
    nb, F = _check_rows(y, bmap, buf)
    with torch.cuda.device(y.device):
        st = _lib.lib().lpg_boundary_unpack_f32(y.data_ptr(), y.stride(0), y.shape[0], F, nb, bmap.data_ptr(),
                                                buf.data_ptr(), _lib.stream_of(y))
    _lib.check(st, "lpg_boundary_unpack_f32")
    _forget_scales(y)
    return y


def boundary_allreduce_(y: torch.Tensor, bmap: torch.Tensor, comm: LibComm,
                        buf: torch.Tensor | None = None) -> torch.Tensor:
    """The mapped rows of y summed over comm's ranks, in place (lpg_boundary_allreduce_f32; collective)."""
    if buf is None:
        buf = torch.empty((bmap.shape[0], y.shape[1]), dtype=torch.float32, device=y.device)
    nb, F = _check_rows(y, bmap, buf)
    with torch.cuda.device(y.device):
        st = _lib.lib().lpg_boundary_allreduce_f32(y.data_ptr(), y.stride(0), y.shape[0], F, nb, bmap.data_ptr(),
                                                   buf.data_ptr(), comm.handle, _lib.stream_of(y))
    _lib.check(st, "lpg_boundary_allreduce_f32")
    _forget_scales(y)
    return y


def spmm_partitioned(adj: CSR, x: torch.Tensor, bmap: torch.Tensor, comm: LibComm,
                     buf: torch.Tensor | None = None) -> torch.Tensor:
    """Y = adj @ x on this rank's local CSR, then the boundary rows summed over the ranks
    (lpg_spmm_partitioned_f32; collective).  fp32."""
    if x.dtype != torch.float32 or x.dim() != 2 or x.shape[0] != adj.n_cols or x.device != adj.device:
        raise RuntimeError(f"lpgnn spmm_partitioned: x must be fp32 [{adj.n_cols}, F] on {adj.device}")
    if x.stride(1) != 1:
        x = x.contiguous()
    y = torch.empty((adj.n_rows, x.shape[1]), dtype=torch.float32, device=x.device)
    if buf is None:
        buf = torch.empty((bmap.shape[0], x.shape[1]), dtype=torch.float32, device=x.device)
    nb, F = _check_rows(y, bmap, buf)
    with torch.cuda.device(x.device):
        st = _lib.lib().lpg_spmm_partitioned_f32(ctypes.byref(adj.cstruct()), x.data_ptr(), x.stride(0), y.data_ptr(),
                                                 y.stride(0), F, nb, bmap.data_ptr(), buf.data_ptr(), comm.handle,
                                                 _lib.stream_of(x))
    _lib.check(st, "lpg_spmm_partitioned_f32")
    return y
