"""ctypes binding of liblpgnn_hip.so (C ABI: include/lpgnn.h).

This is the same binding a maintainer would add on the reference side
(INTEGRATION.md): plain pointers and sizes, the HIP stream as a void*, the
status code turned into a RuntimeError carrying lpg_last_error() -- the
behaviour of torch_sparse's TORCH_CHECK failures.

There is no fallback: if the library is missing or fails to load, every
entry point raises.  ``torch`` is imported first on purpose: its bundled
libamdhip64.so (soname libamdhip64.so.7) is then the HIP runtime that the
library's NEEDED entry resolves to, so there is one runtime per process.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (see module docstring)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("LPGNN_LIB") or os.path.join(_HERE, "liblpgnn_hip.so")  # override: tools/ experiments
HEADER_SYMBOLS = (
    "lpg_last_error",
    "lpg_build_info",
    "lpg_csr_pack_host",
    "lpg_csr_pack_workspace_bytes",
    "lpg_csr_pack_f32",
    "lpg_spmm_f32",
    "lpg_spmm_f32_heavy",
    "lpg_spmm_bf16",
    "lpg_spmm_bf16_heavy",
    "lpg_spmm_f32_tuned",
    "lpg_spmm_bf16_tuned",
    "lpg_spmm_f16",
    "lpg_spmm_f16_tuned",
    "lpg_fc_f32",
    "lpg_fc_bf16",
    "lpg_fc_f16",
    "lpg_fc_bf16_relu_bwd",
    "lpg_fc_bf16_mask",
    "lpg_fc_bf16_relu_bwd_bits",
    "lpg_fc_bf16_relu_bwd_db",
    "lpg_fc_bf16_relu_bwd_bits_db",
    "lpg_fc16_workspace_bytes",
    "lpg_fc16",
    "lpg_colsum_bf16",
    "lpg_transpose_bf16",
    "lpg_wgrad_bf16_workspace_bytes",
    "lpg_wgrad_bf16",
    "lpg_split3_f32",
    "lpg_fc_x3_f32",
    "lpg_fc_x3_heads_workspace_bytes",
    "lpg_fc_x3_heads_f32",
    "lpg_fc_x3_relu_wgrad_workspace_bytes",
    "lpg_fc_x3_relu_wgrad_f32",
    "lpg_wgrad_x3_workspace_bytes",
    "lpg_wgrad_x3_f32",
    "lpg_weighted_ce_workspace_bytes",
    "lpg_class_counts_workspace_bytes",
    "lpg_class_counts3",
    "lpg_balanced_weights3",
    "lpg_basis_labels_workspace_bytes",
    "lpg_basis_labels_f32",
    "lpg_basis_labels_f16",
    "lpg_weighted_ce_fwd_f32",
    "lpg_weighted_ce_bwd_f32",
    "lpg_relu_dropout_bwd_f32",
    "lpg_relu_bwd_colsum_workspace_bytes",
    "lpg_relu_bwd_colsum_f32",
    "lpg_relu_bwd_colsum_bf16",
    "lpg_wgrad_smallk_workspace_bytes",
    "lpg_wgrad_smallk_f32",
    "lpg_relu_wgrad_smallk_f32",
    "lpg_linear_small_bwd_workspace_bytes",
    "lpg_linear_small_bwd_f32",
    "lpg_heads_relu_bwd_f32",
    "lpg_heads_scales_workspace_bytes",
    "lpg_fc_smallk_scales_workspace_bytes",
    "lpg_fc_smallk_scales_f32",
    "lpg_heads_relu_bwd_scales_f32",
    "lpg_relu_wgrad_smallk_bf16",
    "lpg_linear_small_fwd_bf16",
    "lpg_linear_small_fwd_f16",
    "lpg_heads_bwd_bf16_workspace_bytes",
    "lpg_heads_bwd_bf16",
    "lpg_knowledge_f32",
    "lpg_knowledge_f16",
    "lpg_knowledge_bwd_f32",
    "lpg_scan_i64_workspace_bytes",
    "lpg_scan_i64",
    "lpg_sample_count",
    "lpg_sample_fill",
    "lpg_sample_dedupe",
    "lpg_sample_assign",
    "lpg_sample_local_ids",
    "lpg_induced_count",
    "lpg_induced_fill",
    "lpg_sample_reset",
    "lpg_comm_unique_id",
    "lpg_comm_init",
    "lpg_comm_destroy",
    "lpg_comm_info",
    "lpg_boundary_pack_f32",
    "lpg_boundary_unpack_f32",
    "lpg_boundary_allreduce_f32",
    "lpg_spmm_partitioned_f32",
    "lpg_rowscale_f32",
    "lpg_split_f16x2",
    "lpg_fc_f16x2_f32",
    "lpg_fc_f16x2_heads_f32",
    "lpg_fc_f16x2_relu_wgrad_f32",
    "lpg_wgrad_f16x2_f32",
    "lpg_colscale_workspace_bytes",
    "lpg_colscale_f32",
    "lpg_rowcolscale_workspace_bytes",
    "lpg_rowcolscale_f32",
)

c_i64, c_i32, c_p = ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p


class LpgCsr(ctypes.Structure):
    _fields_ = [("n_rows", c_i64), ("n_cols", c_i64), ("nnz", c_i64),
                ("rowptr", c_p), ("col", c_p), ("val", c_p)]


class LpgFc16Call(ctypes.Structure):
    """include/lpgnn.h lpg_fc16_call: every 16-bit FC form in one call (lpg_fc16)."""
    _fields_ = [("dtype", c_i32), ("flags", c_i32), ("M", c_i64), ("N", c_i64), ("K1", c_i64), ("K2", c_i64),
                ("A1", c_p), ("W1", c_p), ("A2", c_p), ("W2", c_p), ("lda1", c_i64), ("ldw1", c_i64),
                ("lda2", c_i64), ("ldw2", c_i64), ("bias", c_p), ("C", c_p), ("ldc", c_i64),
                ("dropout_p", ctypes.c_float), ("seed", ctypes.c_uint64), ("row_offset", c_i64), ("row_keys", c_p),
                ("mask_out", c_p), ("ldmo", c_i64), ("Y", c_p), ("ldy", c_i64), ("mask_in", c_p), ("ldmi", c_i64),
                ("scale", ctypes.c_float), ("db", c_p), ("db_workspace", c_p)]


_lib = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} is not built; run `make -C lp-gnn_amd` or __graft_entry__.build(). "
                           "There is no CPU fallback for the lpgnn hot path.")
    L = ctypes.CDLL(LIB_PATH)
    L.lpg_last_error.restype = ctypes.c_char_p
    L.lpg_build_info.restype = ctypes.c_char_p
    L.lpg_csr_pack_host.argtypes = [c_p, c_p, c_p, c_i64, c_i64, c_i64, c_p, c_p, c_p, c_p, c_p, c_p]
    L.lpg_csr_pack_host.restype = c_i32
    L.lpg_csr_pack_workspace_bytes.argtypes = [c_i64, c_i64, c_i64]
    L.lpg_csr_pack_workspace_bytes.restype = c_i64
    L.lpg_csr_pack_f32.argtypes = [c_p, c_p, c_p, c_i64, c_i64, c_i64, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p]
    L.lpg_csr_pack_f32.restype = c_i32
    L.lpg_spmm_f32.argtypes = [ctypes.POINTER(LpgCsr), c_p, c_i64, c_p, c_i64, c_i64, c_p]
    L.lpg_spmm_f32.restype = c_i32
    L.lpg_comm_unique_id.argtypes = [c_p]
    L.lpg_comm_init.argtypes = [ctypes.POINTER(c_p), c_i32, c_p, c_i32]
    L.lpg_comm_destroy.argtypes = [c_p]
    L.lpg_comm_info.argtypes = [c_p, ctypes.POINTER(c_i32), ctypes.POINTER(c_i32)]
    L.lpg_boundary_pack_f32.argtypes = [c_p, c_i64, c_i64, c_i64, c_i64, c_p, c_p, c_p]
    L.lpg_boundary_unpack_f32.argtypes = L.lpg_boundary_pack_f32.argtypes
    L.lpg_boundary_allreduce_f32.argtypes = [c_p, c_i64, c_i64, c_i64, c_i64, c_p, c_p, c_p, c_p]
    L.lpg_spmm_partitioned_f32.argtypes = [ctypes.POINTER(LpgCsr), c_p, c_i64, c_p, c_i64, c_i64, c_i64, c_p, c_p, c_p,
                                           c_p]
    for _n in ("lpg_comm_unique_id", "lpg_comm_init", "lpg_comm_destroy", "lpg_comm_info", "lpg_boundary_pack_f32",
               "lpg_boundary_unpack_f32", "lpg_boundary_allreduce_f32", "lpg_spmm_partitioned_f32"):
        getattr(L, _n).restype = c_i32
    L.lpg_spmm_f32_heavy.argtypes = [ctypes.POINTER(LpgCsr), c_p, c_i64, c_p, c_i64, c_i64, c_p, c_i64, c_i64, c_p]
    L.lpg_spmm_f32_heavy.restype = c_i32
    L.lpg_spmm_bf16.argtypes = [ctypes.POINTER(LpgCsr), c_p, c_i64, c_p, c_i64, c_i64, c_p]
    L.lpg_spmm_bf16.restype = c_i32
    L.lpg_spmm_bf16_heavy.argtypes = L.lpg_spmm_f32_heavy.argtypes
    L.lpg_spmm_bf16_heavy.restype = c_i32
    L.lpg_spmm_f32_tuned.argtypes = [ctypes.POINTER(LpgCsr), c_p, c_i64, c_p, c_i64, c_i64, c_p, c_i64, c_i64, c_i64,
                                     c_i32, c_p]
    L.lpg_spmm_f32_tuned.restype = c_i32
    L.lpg_spmm_bf16_tuned.argtypes = L.lpg_spmm_f32_tuned.argtypes
    L.lpg_spmm_bf16_tuned.restype = c_i32
    L.lpg_spmm_f16.argtypes = L.lpg_spmm_bf16.argtypes
    L.lpg_spmm_f16.restype = c_i32
    L.lpg_spmm_f16_tuned.argtypes = L.lpg_spmm_f32_tuned.argtypes
    L.lpg_spmm_f16_tuned.restype = c_i32
    L.lpg_fc_f32.argtypes = [c_i64, c_i64, c_i64, c_p, c_i64, c_p, c_i64, c_i64, c_p, c_i64, c_p, c_i64,
                             c_p, c_p, c_i64, c_i32, ctypes.c_float, ctypes.c_uint64, c_i64, c_p, c_p]
    L.lpg_fc_f32.restype = c_i32
    L.lpg_fc_bf16.argtypes = L.lpg_fc_f32.argtypes
    L.lpg_fc_f16.argtypes = L.lpg_fc_f32.argtypes
    L.lpg_fc_f16.restype = c_i32
    L.lpg_fc16_workspace_bytes.argtypes = []
    L.lpg_fc16_workspace_bytes.restype = c_i64
    L.lpg_fc16.argtypes = [ctypes.POINTER(LpgFc16Call), c_p, c_i64, c_p]
    L.lpg_fc16.restype = c_i32
    L.lpg_fc_bf16_relu_bwd.argtypes = [c_i64, c_i64, c_i64, c_p, c_i64, c_p, c_i64, c_i64, c_p, c_i64, c_p, c_i64,
                                       c_p, c_i64, c_i32, c_p, c_i64, ctypes.c_float, c_p]
    L.lpg_fc_bf16_relu_bwd.restype = c_i32
    L.lpg_fc_bf16_mask.argtypes = L.lpg_fc_f32.argtypes[:-1] + [c_p, c_i64, c_p]
    L.lpg_fc_bf16_mask.restype = c_i32
    L.lpg_fc_bf16_relu_bwd_bits.argtypes = L.lpg_fc_bf16_relu_bwd.argtypes
    L.lpg_fc_bf16_relu_bwd_bits.restype = c_i32
    L.lpg_fc_bf16_relu_bwd_db.argtypes = L.lpg_fc_bf16_relu_bwd.argtypes[:-1] + [c_p, c_p, c_p]
    L.lpg_fc_bf16_relu_bwd_db.restype = c_i32
    L.lpg_fc_bf16_relu_bwd_bits_db.argtypes = L.lpg_fc_bf16_relu_bwd_db.argtypes
    L.lpg_fc_bf16_relu_bwd_bits_db.restype = c_i32
    L.lpg_colsum_bf16.argtypes = [c_i64, c_i64, c_p, c_i64, c_p, c_p, c_p]
    L.lpg_colsum_bf16.restype = c_i32
    L.lpg_class_counts_workspace_bytes.argtypes = [c_i64]
    L.lpg_class_counts_workspace_bytes.restype = c_i64
    L.lpg_class_counts3.argtypes = [c_i64, c_p, c_p, c_p, c_p]
    L.lpg_class_counts3.restype = c_i32
    L.lpg_balanced_weights3.argtypes = [c_i64, c_p, c_i32, c_p, c_p, c_p]
    L.lpg_balanced_weights3.restype = c_i32
    L.lpg_basis_labels_workspace_bytes.argtypes = [c_i64]
    L.lpg_basis_labels_workspace_bytes.restype = c_i64
    L.lpg_basis_labels_f32.argtypes = [c_i64, c_i64, c_p, c_i64, c_p, c_p, c_p]
    L.lpg_basis_labels_f32.restype = c_i32
    L.lpg_basis_labels_f16.argtypes = L.lpg_basis_labels_f32.argtypes
    L.lpg_basis_labels_f16.restype = c_i32
    L.lpg_transpose_bf16.argtypes = [c_i64, c_i64, c_p, c_i64, c_p, c_i64, c_p]
    L.lpg_transpose_bf16.restype = c_i32
    L.lpg_split3_f32.argtypes = [c_i64, c_i64, c_p, c_i64, c_i32, c_p, c_i64, c_i64, c_p]
    L.lpg_split3_f32.restype = c_i32
    L.lpg_fc_x3_f32.argtypes = [c_i64, c_i64, c_i64, c_p, c_i64, c_p, c_i64, c_i64, c_i64, c_p, c_i64, c_p, c_i64,
                                c_i64, c_p, c_p, c_i64, c_i32, ctypes.c_float, ctypes.c_uint64, c_i64, c_p, c_p]
    L.lpg_fc_x3_f32.restype = c_i32
    L.lpg_fc_x3_heads_workspace_bytes.argtypes = [c_i64, c_i64]
    L.lpg_fc_x3_heads_workspace_bytes.restype = c_i64
    L.lpg_fc_x3_heads_f32.argtypes = L.lpg_fc_x3_f32.argtypes[:-1] + [c_i32, c_p, c_i64, c_p, c_p, c_i64, c_p, c_p]
    L.lpg_fc_x3_heads_f32.restype = c_i32
    L.lpg_fc_x3_relu_wgrad_workspace_bytes.argtypes = [c_i64, c_i64, c_i64]
    L.lpg_fc_x3_relu_wgrad_workspace_bytes.restype = c_i64
    L.lpg_fc_x3_relu_wgrad_f32.argtypes = [c_i64, c_i64, c_i64, c_p, c_i64, c_p, c_i64, c_i64, c_i64, c_p, c_i64, c_p,
                                           c_i64, c_i64, c_p, c_i64, c_i32, c_p, c_i64, c_i64, c_p, c_i64, c_i64, c_p,
                                           c_i64, c_p, c_p, c_p, c_p, c_p]
    L.lpg_fc_x3_relu_wgrad_f32.restype = c_i32
    # the f16x2 entries: the x3 signatures with the row scales (sa, sw) after ps2
    for _x3, _f16 in (("lpg_fc_x3_f32", "lpg_fc_f16x2_f32"), ("lpg_fc_x3_heads_f32", "lpg_fc_f16x2_heads_f32"),
                      ("lpg_fc_x3_relu_wgrad_f32", "lpg_fc_f16x2_relu_wgrad_f32")):
        _t = getattr(L, _x3).argtypes
        getattr(L, _f16).argtypes = _t[:14] + [c_p, c_p] + _t[14:]
        getattr(L, _f16).restype = c_i32
    L.lpg_wgrad_f16x2_f32.argtypes = [c_i64, c_i64, c_i64, c_p, c_i64, c_p, c_i64, c_p, c_p, c_p, c_i64, c_p, c_p]
    L.lpg_wgrad_f16x2_f32.restype = c_i32
    L.lpg_colscale_workspace_bytes.argtypes = [c_i64, c_i64]
    L.lpg_colscale_workspace_bytes.restype = c_i64
    L.lpg_colscale_f32.argtypes = [c_i64, c_i64, c_p, c_i64, c_p, c_p, c_p]
    L.lpg_colscale_f32.restype = c_i32
    L.lpg_rowcolscale_workspace_bytes.argtypes = [c_i64, c_i64]
    L.lpg_rowcolscale_workspace_bytes.restype = c_i64
    L.lpg_rowcolscale_f32.argtypes = [c_i64, c_i64, c_p, c_i64, c_p, c_p, c_p, c_p]
    L.lpg_rowcolscale_f32.restype = c_i32
    L.lpg_rowscale_f32.argtypes = [c_i64, c_i64, c_p, c_i64, c_i64, c_p, c_i64, c_p, c_p]
    L.lpg_rowscale_f32.restype = c_i32
    L.lpg_split_f16x2.argtypes = [c_i64, c_i64, c_p, c_i64, c_i64, c_p, c_i64, c_i32, c_p, c_i64, c_p, c_i64, c_i64,
                                  c_p, c_p]
    L.lpg_split_f16x2.restype = c_i32
    L.lpg_wgrad_x3_workspace_bytes.argtypes = [c_i64, c_i64, c_i64]
    L.lpg_wgrad_x3_workspace_bytes.restype = c_i64
    L.lpg_wgrad_x3_f32.argtypes = [c_i64, c_i64, c_i64, c_p, c_i64, c_p, c_i64, c_p, c_i64, c_p, c_p]
    L.lpg_wgrad_x3_f32.restype = c_i32
    L.lpg_weighted_ce_workspace_bytes.argtypes = [c_i64]
    L.lpg_weighted_ce_workspace_bytes.restype = c_i64
    L.lpg_weighted_ce_fwd_f32.argtypes = [c_i64, c_i64, c_p, c_i64, c_p, c_p, ctypes.c_float, c_p, c_p, c_p, c_p]
    L.lpg_weighted_ce_fwd_f32.restype = c_i32
    L.lpg_weighted_ce_bwd_f32.argtypes = [c_i64, c_i64, c_p, c_i64, c_p, c_p, c_p, c_p, ctypes.c_float, c_p, c_i64,
                                          c_p]
    L.lpg_weighted_ce_bwd_f32.restype = c_i32
    L.lpg_fc_bf16.restype = c_i32
    L.lpg_wgrad_bf16_workspace_bytes.argtypes = [c_i64, c_i64, c_i64]
    L.lpg_wgrad_bf16_workspace_bytes.restype = c_i64
    L.lpg_wgrad_bf16.argtypes = [c_i64, c_i64, c_i64, c_p, c_i64, c_p, c_i64, c_p, c_i64, c_p, c_p]
    L.lpg_wgrad_bf16.restype = c_i32
    L.lpg_relu_dropout_bwd_f32.argtypes = [c_i64, c_p, c_p, ctypes.c_float, c_p, c_p]
    L.lpg_relu_dropout_bwd_f32.restype = c_i32
    L.lpg_relu_bwd_colsum_workspace_bytes.argtypes = [c_i64, c_i64]
    L.lpg_relu_bwd_colsum_workspace_bytes.restype = c_i64
    L.lpg_relu_bwd_colsum_f32.argtypes = [c_i64, c_i64, c_p, c_i64, c_p, c_i64, ctypes.c_float, c_p, c_i64, c_p, c_p,
                                          c_p]
    L.lpg_relu_bwd_colsum_f32.restype = c_i32
    L.lpg_relu_bwd_colsum_bf16.argtypes = L.lpg_relu_bwd_colsum_f32.argtypes
    L.lpg_relu_bwd_colsum_bf16.restype = c_i32
    L.lpg_wgrad_smallk_workspace_bytes.argtypes = [c_i64, c_i64, c_i64]
    L.lpg_wgrad_smallk_workspace_bytes.restype = c_i64
    L.lpg_wgrad_smallk_f32.argtypes = [c_i64, c_i64, c_p, c_i64, c_i64, c_p, c_i64, c_i64, c_p, c_i64, c_p, c_p, c_p,
                                       c_p]
    L.lpg_wgrad_smallk_f32.restype = c_i32
    L.lpg_relu_wgrad_smallk_f32.argtypes = [c_i64, c_i64, c_p, c_i64, c_p, c_i64, ctypes.c_float, c_i64, c_p, c_i64,
                                            c_i64, c_p, c_i64, c_p, c_p, c_p, c_p, c_p]
    L.lpg_relu_wgrad_smallk_f32.restype = c_i32
    L.lpg_linear_small_bwd_workspace_bytes.argtypes = [c_i64, c_i64, c_i64]
    L.lpg_linear_small_bwd_workspace_bytes.restype = c_i64
    L.lpg_linear_small_bwd_f32.argtypes = [c_i64, c_i64, c_i64, c_p, c_i64, c_p, c_p, c_i64, c_p, c_i64, c_p, c_p,
                                           c_p, c_p]
    L.lpg_linear_small_bwd_f32.restype = c_i32
    L.lpg_heads_relu_bwd_f32.argtypes = [c_i64, c_i64, c_i64, c_p, c_i64, c_p, c_p, c_i64, ctypes.c_float, c_p, c_i64,
                                         c_p, c_p, c_p, c_p, c_p]
    L.lpg_heads_relu_bwd_f32.restype = c_i32
    L.lpg_fc_smallk_scales_workspace_bytes.argtypes = [c_i64, c_i64]
    L.lpg_fc_smallk_scales_workspace_bytes.restype = c_i64
    L.lpg_fc_smallk_scales_f32.argtypes = [c_i64, c_i64, c_i64, c_p, c_i64, c_p, c_i64, c_i64, c_p, c_i64, c_p, c_i64,
                                           c_p, c_p, c_i64, c_i32, c_p, c_p, c_p, c_p]
    L.lpg_fc_smallk_scales_f32.restype = c_i32
    L.lpg_heads_scales_workspace_bytes.argtypes = [c_i64, c_i64]
    L.lpg_heads_scales_workspace_bytes.restype = c_i64
    L.lpg_heads_relu_bwd_scales_f32.argtypes = [c_i64, c_i64, c_i64, c_p, c_i64, c_p, c_p, c_i64, ctypes.c_float, c_p,
                                                c_i64, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p]
    L.lpg_heads_relu_bwd_scales_f32.restype = c_i32
    L.lpg_relu_wgrad_smallk_bf16.argtypes = L.lpg_relu_wgrad_smallk_f32.argtypes
    L.lpg_relu_wgrad_smallk_bf16.restype = c_i32
    L.lpg_linear_small_fwd_bf16.argtypes = [c_i64, c_i64, c_i64, c_p, c_i64, c_p, c_p, c_p, c_i64, c_p]
    L.lpg_linear_small_fwd_bf16.restype = c_i32
    L.lpg_linear_small_fwd_f16.argtypes = L.lpg_linear_small_fwd_bf16.argtypes
    L.lpg_linear_small_fwd_f16.restype = c_i32
    L.lpg_heads_bwd_bf16_workspace_bytes.argtypes = [c_i64, c_i64, c_i64]
    L.lpg_heads_bwd_bf16_workspace_bytes.restype = c_i64
    L.lpg_heads_bwd_bf16.argtypes = [c_i64, c_i64, c_i64, c_p, c_i64, c_p, c_p, c_i64, c_i32, ctypes.c_float, c_p,
                                     c_i64, c_p, c_p, c_p, c_p, c_p]
    L.lpg_heads_bwd_bf16.restype = c_i32
    L.lpg_knowledge_f32.argtypes = [c_i64, c_p, c_i64, c_p, c_i64, c_i64, ctypes.c_float, c_p, c_i64, c_p]
    L.lpg_knowledge_f32.restype = c_i32
    L.lpg_knowledge_f16.argtypes = L.lpg_knowledge_f32.argtypes
    L.lpg_knowledge_f16.restype = c_i32
    L.lpg_knowledge_bwd_f32.argtypes = [c_i64, c_p, c_i64, c_p, c_i64, c_p, c_i64, c_p]
    L.lpg_knowledge_bwd_f32.restype = c_i32
    L.lpg_scan_i64_workspace_bytes.argtypes = [c_i64]
    L.lpg_scan_i64_workspace_bytes.restype = c_i64
    L.lpg_scan_i64.argtypes = [c_p, c_i64, c_p, c_p, c_i64, c_p]
    L.lpg_sample_count.argtypes = [c_p, c_i64, c_p, c_i64, c_p, c_p]
    L.lpg_sample_fill.argtypes = [c_p, c_i64, c_i64, c_p, c_p, c_i64, ctypes.c_uint64, c_p, c_p, c_p, c_p, c_p]
    L.lpg_sample_dedupe.argtypes = [c_p, c_i64, c_p, c_p, c_p, c_p]
    L.lpg_sample_assign.argtypes = [c_p, c_i64, c_i64, c_p, c_p, c_p, c_p, c_p, c_p]
    L.lpg_sample_local_ids.argtypes = [c_p, c_i64, c_p, c_p, c_p]
    L.lpg_induced_count.argtypes = [c_p, c_i64, c_p, c_p, c_p, c_p, c_p]
    L.lpg_induced_fill.argtypes = [c_p, c_i64, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p]
    L.lpg_sample_reset.argtypes = [c_p, c_i64, c_p, c_p]
    for nm in ("lpg_scan_i64", "lpg_sample_count", "lpg_sample_fill", "lpg_sample_dedupe", "lpg_sample_assign",
               "lpg_sample_local_ids", "lpg_induced_count", "lpg_induced_fill", "lpg_sample_reset"):
        getattr(L, nm).restype = c_i32
    _lib = L
    return L


FC_RELU, FC_ACCUMULATE = 1, 2


def fc_kernel(k: int) -> int:
    """LPG_FC_KERNEL(k): the per-call kernel choice in an FC entry's flags (include/lpgnn.h)."""
    return int(k) << 8


def check(status: int, what: str) -> None:
    if status != 0:
        msg = lib().lpg_last_error().decode(errors="replace")
        kind = {1: "invalid argument", 2: "HIP error", 3: "unsupported"}.get(status, f"status {status}")
        raise RuntimeError(f"{what}: {kind}: {msg}")


def ptr(t: "torch.Tensor | None") -> int | None:
    return None if t is None else t.data_ptr()


def stream_of(t: torch.Tensor) -> int:
    """The torch current stream of t's device, as a raw hipStream_t."""
    return torch.cuda.current_stream(t.device).cuda_stream
