"""Per-model choices of the hot path's kernels and fusions (no module state that callers mutate).

Every choice here computes the same function (the tests compare them); they exist for A/B
measurements and for the bitwise contract of the exact-fp32 FC.  A model carries its own
``PathOptions`` (``GCN_FC(..., options=...)``); the defaults come from the environment once, at
import, so a whole run can be switched from the shell:

  LPGNN_FC_ARITH=x3          every fp32 GEMM (FC, input and weight gradients) on the exact three-way
                             bf16 split (six products) instead of the default f16x2 (two row- or
                             column-scaled fp16 terms per operand, three products)
  LPGNN_FC_ARITH=fp32        the exact-fp32 MFMA FC (bitwise oracle/fc_ref.c) + hipBLASLt backward
  LPGNN_REASSOC=0            lin_rel(S x) never re-associated as S (x W_rel^T)
  LPGNN_FUSE_HEADS=0         the heads as their own autograd node
  LPGNN_FUSE_HEAD_FWD=0      the heads' forward as their own kernels (not in the last FC's epilogue)
  LPGNN_FOLD_RELU_BWD=0      bf16: a layer's ReLU/dropout backward as its own pass
  LPGNN_FOLD_CONV1_WGRAD=0   fp32: conv1's weight gradient as its own pass (not in the next layer's
                             input-gradient GEMM)
  LPGNN_OVERLAP=1            independent SpMMs on a second stream beside the FC
  LPGNN_RELU_BITS=0          bf16: the folded ReLU backward re-reads the layer output instead of the
                             1-bit mask its forward wrote beside it
  LPGNN_FOLD_BIAS_SUMS=0     bf16: a hidden layer's bias gradient as its own column-sum pass over dZ (not
                             summed in the next layer's folded input-gradient store)
  LPGNN_SPMM_HEAVY=<deg>     SpMM rows with more edges than this run as (heavy row, slice) wave units
                             (lpg_spmm_*_tuned's heavy list); 0 = off (default 1024)
"""
from __future__ import annotations

import dataclasses
import os


def _env(name: str, default: str) -> str:
    return os.environ.get(name, default)


@dataclasses.dataclass(frozen=True)
class PathOptions:
    arith: str = "f16x2"
    reassociate: bool = True
    fuse_heads: bool = True
    fuse_head_fwd: bool = True
    fold_relu_bwd: bool = True
    fold_conv1_wgrad: bool = True
    overlap: bool = False
    relu_bits: bool = True
    fold_bias_sums: bool = True
    spmm_heavy: int = 1024  # sparse.DEFAULT_HEAVY

    def __post_init__(self):
        if self.arith not in ("x3", "fp32", "f16x2"):
            raise ValueError(f"PathOptions.arith must be 'x3', 'f16x2' or 'fp32', got {self.arith!r}")
        if int(self.spmm_heavy) < 0:
            raise ValueError(f"PathOptions.spmm_heavy must be >= 0, got {self.spmm_heavy}")

    @classmethod
    def from_env(cls) -> "PathOptions":
        return cls(arith=_env("LPGNN_FC_ARITH", "f16x2"),
                   reassociate=_env("LPGNN_REASSOC", "1") == "1",
                   fuse_heads=_env("LPGNN_FUSE_HEADS", "1") == "1",
                   fuse_head_fwd=_env("LPGNN_FUSE_HEAD_FWD", "1") == "1",
                   fold_relu_bwd=_env("LPGNN_FOLD_RELU_BWD", "1") == "1",
                   fold_conv1_wgrad=_env("LPGNN_FOLD_CONV1_WGRAD", "1") == "1",
                   overlap=_env("LPGNN_OVERLAP", "0") == "1",
                   relu_bits=_env("LPGNN_RELU_BITS", "1") == "1",
                   fold_bias_sums=_env("LPGNN_FOLD_BIAS_SUMS", "1") == "1",
                   spmm_heavy=int(_env("LPGNN_SPMM_HEAVY", "1024")))

    def replace(self, **kw) -> "PathOptions":
        return dataclasses.replace(self, **kw)


DEFAULT = PathOptions.from_env()
