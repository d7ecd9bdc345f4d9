"""``torch.ops.lpgnn.spmm_sum``: the torch_sparse native op, on the HIP kernel.

The reference reaches its SpMM through ``torch_sparse.matmul(adj_t, x,
reduce='add')`` (PyG 2.1 GraphConv.message_and_aggregate, arch.py:75-80),
which calls the TorchScript op registered by torch_sparse 0.6.12
(csrc/spmm.cpp, python/torch_sparse/matmul.py ``spmm_sum``)::

    torch.ops.torch_sparse.spmm_sum(row, rowptr, col, value, colptr, csr2csc, mat)

This module registers the same schema as ``torch.ops.lpgnn.spmm_sum``
(``torch.library.custom_op`` + ``register_autograd``), so code written
against the torch_sparse op switches by changing the namespace:

* row (optional, int64 [nnz]), rowptr (int64 [m+1]), col (int64 or int32
  [nnz], sorted within each row), value (optional fp32 [nnz]; None = ones),
  colptr / csr2csc (optional int64, the CSC pointer and the CSR->CSC
  permutation: needed, as upstream, only for the gradient w.r.t. mat),
  mat (fp32 or bf16 [n, F]) -> out [m, F];
* out[i] = sum over the row's edges, in CSR order, of value[e] * mat[col[e]]
  (lpg_spmm_f32 / lpg_spmm_bf16: bitwise torch_sparse's CPU loop order);
* backward: grad_mat = spmm over (colptr, row[csr2csc], value[csr2csc]) --
  upstream's SPMMSum.backward -- on the same kernel.  A gradient w.r.t.
  ``value`` (upstream: (grad_out[row] * mat[col]).sum(-1)) is not provided:
  the reference never trains edge values (dataset.py:250), and asking for
  it raises rather than silently returning zeros.

Errors mirror upstream's TORCH_CHECKs as RuntimeError.  There is no CPU
path: CPU tensors raise.
"""
from __future__ import annotations

from typing import Optional

import torch
from torch import Tensor

from .sparse import CSR, spmm_forward


def _csr(rowptr: Tensor, col: Tensor, value: Optional[Tensor], n_cols: int) -> CSR:
    if rowptr.dim() != 1 or rowptr.dtype != torch.int64:
        raise RuntimeError("lpgnn::spmm_sum: rowptr must be a 1-D int64 tensor")
    if col.dim() != 1 or col.dtype not in (torch.int64, torch.int32):
        raise RuntimeError("lpgnn::spmm_sum: col must be a 1-D int64/int32 tensor")
    nnz = col.numel()
    if value is None:
        value = torch.ones(nnz, dtype=torch.float32, device=col.device)
    elif value.dim() != 1 or value.numel() != nnz:
        raise RuntimeError("lpgnn::spmm_sum: value must be 1-D with one entry per edge (no multi-dim values)")
    if n_cols >= 2 ** 31:
        raise RuntimeError("lpgnn::spmm_sum: column ids must fit int32")
    return CSR(rowptr.contiguous(), col.to(torch.int32).contiguous(), value.to(torch.float32).contiguous(),
               rowptr.numel() - 1, n_cols)


@torch.library.custom_op("lpgnn::spmm_sum", mutates_args=())
def spmm_sum(row: Optional[Tensor], rowptr: Tensor, col: Tensor, value: Optional[Tensor], colptr: Optional[Tensor],
             csr2csc: Optional[Tensor], mat: Tensor) -> Tensor:
    if mat.dim() != 2:
        raise RuntimeError("lpgnn::spmm_sum: mat must be 2-D [n, F] (batched mats are not supported)")
    return spmm_forward(_csr(rowptr, col, value, mat.shape[0]), mat)


@spmm_sum.register_fake
def _(row, rowptr, col, value, colptr, csr2csc, mat):
    return mat.new_empty((rowptr.shape[0] - 1, mat.shape[1]))


def _setup(ctx, inputs, output):
    row, rowptr, col, value, colptr, csr2csc, mat = inputs
    ctx.n_rows = rowptr.numel() - 1
    ctx.save_for_backward(row, rowptr, value, colptr, csr2csc)


def _backward(ctx, grad_out):
    row, rowptr, value, colptr, csr2csc = ctx.saved_tensors
    if ctx.needs_input_grad[3]:
        raise RuntimeError("lpgnn::spmm_sum: no gradient w.r.t. edge values (the reference never trains them)")
    grad_mat = None
    if ctx.needs_input_grad[6]:
        if colptr is None or csr2csc is None:
            raise RuntimeError("lpgnn::spmm_sum: the gradient w.r.t. mat needs colptr and csr2csc (as upstream)")
        if row is None:  # upstream derives row from rowptr the same way
            deg = rowptr[1:] - rowptr[:-1]
            row = torch.repeat_interleave(torch.arange(ctx.n_rows, device=rowptr.device), deg)
        val_t = None if value is None else value[csr2csc]
        grad_mat = spmm_forward(_csr(colptr, row[csr2csc], val_t, ctx.n_rows), grad_out)
    return None, None, None, None, None, None, grad_mat


spmm_sum.register_autograd(_backward, setup_context=_setup)
