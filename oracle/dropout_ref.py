"""ORACLE -- test infrastructure only.

numpy restatement of the fused dropout mask every FC kernel of the HIP library draws
(``lp-gnn_amd/csrc/fc_common.h``: lowbias32, drop_row_key, drop_col_key, drop_bits; the
threshold of ``dropout_params``).  The reference applies ``F.dropout(x, p, training)`` after
each hidden layer's ReLU (arch.py:186-188 in vbdai/lp-gnn); torch draws that mask from its own
Philox stream, which no other implementation reproduces, so what parity means here is (1) every
kernel draws exactly this function's mask (checked bit for bit by tests/test_gpu_dropout_mask.py)
and (2) the mask is a Bernoulli(1 - q) keep, q = round(p * 2^16) / 2^16 (within 2^-17 of p), with
kept values scaled by 1 / (1 - q) -- F.dropout's 1 / (1 - p) at the rate actually drawn, so the
expectation is exact (statistical checks in the same test).
Nothing in ``lp-gnn_amd/`` imports this module.
"""
from __future__ import annotations

import numpy as np

_M32 = np.uint64(0xFFFFFFFF)


def _mul32(x: np.ndarray, c: int) -> np.ndarray:
    return ((x.astype(np.uint64) * np.uint64(c)) & _M32).astype(np.uint32)


def lowbias32(x: np.ndarray) -> np.ndarray:
    """fc_common.h lowbias32 (uint32 -> uint32, elementwise)."""
    x = np.asarray(x, dtype=np.uint32)
    x = x ^ (x >> np.uint32(16))
    x = _mul32(x, 0x7FEB352D)
    x = x ^ (x >> np.uint32(15))
    x = _mul32(x, 0x846CA68B)
    return x ^ (x >> np.uint32(16))


def threshold(p: float) -> int:
    """dropout_params: the 16-bit threshold of drop probability p (float32 p, as the C-ABI takes it)."""
    if p <= 0:
        return 0
    th = float(np.float32(p)) * 65536.0 + 0.5
    return 65535 if th >= 65535.0 else int(max(th, 1.0))


def scale(p: float) -> float:
    """dropout_params: the kept values' scale 2^16 / (2^16 - threshold(p)) as float32 (1 at p = 0)."""
    th = threshold(p)
    return float(np.float32(65536.0) / np.float32(65536 - th)) if th else 1.0


def keep_mask(seed: int, row_keys: np.ndarray, n_cols: int, p: float) -> np.ndarray:
    """bool [len(row_keys), n_cols]: True where the FC kernels keep output (row, col) under
    dropout p with this seed; row_keys = the rows' dropout keys (row_offset + m, or the caller's
    row_keys[m])."""
    th = threshold(p)
    keys = np.asarray(row_keys, dtype=np.int64)
    if th == 0:
        return np.ones((keys.shape[0], n_cols), dtype=bool)
    seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    lo, hi = np.uint32(seed & 0xFFFFFFFF), np.uint32(seed >> 32)
    rk = lowbias32(keys.astype(np.uint64).astype(np.uint32) ^ lo) ^ hi  # drop_row_key
    cols = np.arange(n_cols, dtype=np.int64)
    ck = _mul32((cols >> 1).astype(np.uint32), 0x9E3779B9)  # drop_col_key
    h = lowbias32(rk[:, None] ^ ck[None, :])
    bits = np.where((cols & 1)[None, :] == 1, h >> np.uint32(16), h & np.uint32(0xFFFF))
    return bits >= np.uint32(th)
