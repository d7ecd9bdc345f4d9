"""Synthetic bipartite LP graphs of stated (n_cons, n_vars, nnz).

There is no network for the mirp LPs (readme.md:193), so bench and tests use
graphs with the reference's feature layout (dataset.py:79-96 +
utils.py:368-374: cols 0-3 dense features, 4/5 = value/tag of the lower
bound, 6/7 = value/tag of the upper bound; tag -1 for -inf, +1 for +inf,
value := 0 where tagged) and scaled coefficients A_ij in [-1, 1] \\ {0}.

Seeds: structure seed 0, features seed 1 (numpy PCG64), weights
torch.manual_seed(0).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np


@dataclass
class LPGraph:
    m: int
    n: int
    row: np.ndarray  # int64 [nnz], sorted by (row, col)
    col: np.ndarray  # int64 [nnz]
    val: np.ndarray  # f32 [nnz]
    x_s: np.ndarray  # f32 [m, 8]
    x_t: np.ndarray  # f32 [n, 8]
    y_s: np.ndarray  # int64 [m]
    y_t: np.ndarray  # int64 [n]

    @property
    def nnz(self) -> int:
        return int(self.row.shape[0])


def _distinct_cols_per_row(rng, m: int, n: int, deg: int) -> np.ndarray:
    """[m, deg] column ids, distinct within each row, sorted (rejection
    sampling: meant for deg^2 << n, where a row is duplicate-free with
    probability ~exp(-deg^2 / 2n))."""
    cols = np.sort(rng.integers(0, n, size=(m, deg), dtype=np.int64), axis=1)
    while True:
        dup = (np.diff(cols, axis=1) == 0).any(axis=1)
        if not dup.any():
            return cols
        k = int(dup.sum())
        cols[dup] = np.sort(rng.integers(0, n, size=(k, deg), dtype=np.int64), axis=1)


def _features(rng, k: int, p_lo: float, p_hi: float) -> np.ndarray:
    x = np.zeros((k, 8), np.float32)
    x[:, :4] = rng.uniform(-1, 1, (k, 4))
    x[:, 5] = -(rng.random(k) < p_lo).astype(np.float32)
    x[:, 4] = np.where(x[:, 5] != 0, 0, rng.uniform(-1, 1, k))
    x[:, 7] = (rng.random(k) < p_hi).astype(np.float32)
    x[:, 6] = np.where(x[:, 7] != 0, 0, rng.uniform(-1, 1, k))
    return x


def _labels(rng, x: np.ndarray) -> np.ndarray:
    """Basis-status labels consistent with the bound tags (dataset.py:201-207):
    never 0 at an infinite lower bound, never 2 at an infinite upper bound."""
    y = rng.integers(0, 3, x.shape[0])
    y[(x[:, 5] != 0) & (y == 0)] = 1
    y[(x[:, 7] != 0) & (y == 2)] = 1
    return y.astype(np.int64)


def _values(rng, nnz: int) -> np.ndarray:
    v = rng.uniform(-1, 1, nnz).astype(np.float32)
    v[v == 0] = 0.5
    return v


def uniform_lp(m: int, n: int, nnz: int, seed: int = 0) -> LPGraph:
    """c2-style graph: every constraint row has exactly nnz/m distinct
    variables drawn uniformly (variable degree ~ Binomial, mean nnz/n)."""
    if nnz % m:
        raise ValueError("uniform_lp needs nnz divisible by m")
    deg = nnz // m
    rs = np.random.default_rng(np.random.PCG64(seed))
    cols = _distinct_cols_per_row(rs, m, n, deg)
    row = np.repeat(np.arange(m, dtype=np.int64), deg)
    col = cols.reshape(-1)
    val = _values(rs, nnz)
    rf = np.random.default_rng(np.random.PCG64(seed + 1))
    x_s = _features(rf, m, 0.5, 0.5)
    x_t = _features(rf, n, 0.1, 0.7)
    return LPGraph(m, n, row, col, val, x_s, x_t, _labels(rf, x_s), _labels(rf, x_t))


def skewed_lp(m: int, n: int, nnz: int, a: float = 1.5, seed: int = 0) -> LPGraph:
    """Zipf(a) constraint-row degrees (capped at n), rescaled to ~nnz edges:
    exercises load balance on skewed LP degrees."""
    rs = np.random.default_rng(np.random.PCG64(seed))
    d = np.minimum(rs.zipf(a, m).astype(np.float64), n)
    d = np.maximum(1, np.round(d * (nnz / d.sum()))).astype(np.int64)
    d = np.minimum(d, n)
    rows, cols = [], []
    order = np.argsort(d)
    for deg in np.unique(d):
        ids = order[d[order] == deg]
        if deg * deg < 2 * n:  # rejection sampling only where a row is likely duplicate-free (birthday bound)
            c = _distinct_cols_per_row(rs, len(ids), n, int(deg))
        else:
            c = np.stack([np.sort(rs.choice(n, int(deg), replace=False)) for _ in ids])
        rows.append(np.repeat(ids, deg))
        cols.append(c.reshape(-1))
    row, col = np.concatenate(rows), np.concatenate(cols)
    key = np.argsort(row * n + col, kind="stable")
    row, col = row[key], col[key]
    val = _values(rs, row.shape[0])
    rf = np.random.default_rng(np.random.PCG64(seed + 1))
    x_s = _features(rf, m, 0.5, 0.5)
    x_t = _features(rf, n, 0.1, 0.7)
    return LPGraph(m, n, row.astype(np.int64), col.astype(np.int64), val, x_s, x_t, _labels(rf, x_s),
                   _labels(rf, x_t))


def block_lp(m: int, n: int, nnz: int, parts: int, rho: float = 0.02, seed: int = 0) -> LPGraph:
    """c4-style graph for constraint-row partitioning:
    `parts` row blocks; each edge of block p stays inside p's variable range
    with probability 1 - rho, otherwise lands on a uniform variable."""
    if nnz % m or m % parts or n % parts:
        raise ValueError("block_lp needs nnz % m == 0 and m, n divisible by parts")
    deg = nnz // m
    rs = np.random.default_rng(np.random.PCG64(seed))
    mb, nb = m // parts, n // parts
    cols = np.empty((m, deg), np.int64)
    for p in range(parts):
        local = _distinct_cols_per_row(rs, mb, nb, deg) + p * nb
        glob = rs.integers(0, n, size=(mb, deg), dtype=np.int64)
        c = np.where(rs.random((mb, deg)) < rho, glob, local)
        c = np.sort(c, axis=1)
        # re-draw rows that collided (local and global picks can coincide)
        bad = (np.diff(c, axis=1) == 0).any(axis=1)
        while bad.any():
            k = int(bad.sum())
            c[bad] = np.sort(_distinct_cols_per_row(rs, k, nb, deg) + p * nb, axis=1)
            bad = (np.diff(c, axis=1) == 0).any(axis=1)
        cols[p * mb:(p + 1) * mb] = c
    row = np.repeat(np.arange(m, dtype=np.int64), deg)
    val = _values(rs, nnz)
    rf = np.random.default_rng(np.random.PCG64(seed + 1))
    x_s = _features(rf, m, 0.5, 0.5)
    x_t = _features(rf, n, 0.1, 0.7)
    return LPGraph(m, n, row, cols.reshape(-1), val, x_s, x_t, _labels(rf, x_s), _labels(rf, x_t))


CONFIGS = {
    # BASELINE.json configs[1]: 100K cons x 200K vars, nnz 2M, hid 1024, depth 3
    "c2": dict(m=100_000, n=200_000, nnz=2_000_000, hids=1024, depth=3),
    # configs[3] per GPU share: 2M x 4M, nnz 40M over 8 GPUs
    "c4": dict(m=2_000_000, n=4_000_000, nnz=40_000_000, hids=1024, depth=3),
    # configs[4]: c2 graph, hid 2048, depth 6, bf16
    "c5": dict(m=100_000, n=200_000, nnz=2_000_000, hids=2048, depth=6),
}
