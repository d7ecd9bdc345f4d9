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


@dataclass
class BlockLP:
    """A block-structured LP defined block by block, so a
    rank generates only the rows it owns (and the variable features it
    needs) -- no rank ever materialises the global edge list.

    `blocks` row blocks of m/blocks constraints; block b's edges stay in
    variable block b's range with probability 1 - rho, else land on a uniform
    variable.  Every constraint row has exactly nnz/m distinct columns.  Each
    block is seeded on its own (numpy SeedSequence([seed, tag, b])), so the
    graph is the same whatever the number of ranks it is split over: a
    strong-scaling workload."""
    m: int
    n: int
    nnz: int
    blocks: int
    rho: float = 0.02
    seed: int = 0

    def __post_init__(self):
        if self.nnz % self.m or self.m % self.blocks or self.n % self.blocks:
            raise ValueError("BlockLP needs nnz % m == 0 and m, n divisible by blocks")

    @property
    def mb(self) -> int:
        return self.m // self.blocks

    @property
    def nb(self) -> int:
        return self.n // self.blocks

    def _rng(self, tag: int, b: int):
        return np.random.default_rng(np.random.SeedSequence([self.seed, tag, b]))

    def block_edges(self, b: int):
        """(row, col, val) of row block b, global ids, sorted by (row, col)."""
        deg, mb, nb = self.nnz // self.m, self.mb, self.nb
        rs = self._rng(0, b)
        c = _distinct_cols_per_row(rs, mb, nb, deg) + b * nb
        far = rs.random((mb, deg)) < self.rho
        c = np.where(far, rs.integers(0, self.n, size=(mb, deg), dtype=np.int64), c)
        c = np.sort(c, axis=1)
        bad = (np.diff(c, axis=1) == 0).any(axis=1)  # a far pick may hit a local one: re-draw those rows local
        while bad.any():
            c[bad] = _distinct_cols_per_row(rs, int(bad.sum()), nb, deg) + b * nb
            bad = (np.diff(c, axis=1) == 0).any(axis=1)
        row = np.repeat(np.arange(b * mb, (b + 1) * mb, dtype=np.int64), deg)
        return row, c.reshape(-1), _values(rs, mb * deg)

    def cons_block(self, b: int):
        """(x_s, y_s) of the constraints of row block b."""
        rf = self._rng(1, b)
        x = _features(rf, self.mb, 0.5, 0.5)
        return x, _labels(rf, x)

    def var_block(self, b: int):
        """(x_t, y_t) of the variables of variable block b."""
        rf = self._rng(2, b)
        x = _features(rf, self.nb, 0.1, 0.7)
        return x, _labels(rf, x)

    def var_rows(self, ids: np.ndarray):
        """(x_t, y_t) of arbitrary global variable ids (generates only the
        variable blocks they fall in)."""
        ids = np.asarray(ids, np.int64)
        x = np.empty((ids.shape[0], 8), np.float32)
        y = np.empty(ids.shape[0], np.int64)
        blk = ids // self.nb
        for b in np.unique(blk):
            sel = blk == b
            xb, yb = self.var_block(int(b))
            x[sel], y[sel] = xb[ids[sel] - b * self.nb], yb[ids[sel] - b * self.nb]
        return x, y

    def rows(self, b0: int, b1: int):
        """Edges and constraint features of row blocks [b0, b1)."""
        parts = [self.block_edges(b) for b in range(b0, b1)]
        cons = [self.cons_block(b) for b in range(b0, b1)]
        cat = lambda xs: np.concatenate(xs) if xs else np.empty(0)
        return (cat([p[0] for p in parts]), cat([p[1] for p in parts]), cat([p[2] for p in parts]).astype(np.float32),
                cat([c[0] for c in cons]).reshape(-1, 8).astype(np.float32), cat([c[1] for c in cons]).astype(np.int64))

    def full(self) -> LPGraph:
        """The whole graph (single-GPU runs and tests)."""
        row, col, val, x_s, y_s = self.rows(0, self.blocks)
        x_t, y_t = self.var_rows(np.arange(self.n, dtype=np.int64))
        return LPGraph(self.m, self.n, row, col, val, x_s, x_t, y_s, y_t)


def c4_spec(scale: int = 1, seed: int = 0) -> BlockLP:
    """BASELINE.json configs[3]: 2M cons x 4M vars, nnz 40M, 8 row blocks,
    rho = 0.02 (1/scale of it per dimension for reduced-size tests)."""
    return BlockLP(2_000_000 // scale, 4_000_000 // scale, 40_000_000 // scale, blocks=8, rho=0.02, seed=seed)


CONFIGS = {
    # BASELINE.json configs[1]: 100K cons x 200K vars, nnz 2M, hid 1024, depth 3
    "c2": dict(m=100_000, n=200_000, nnz=2_000_000, hids=1024, depth=3),
    # configs[3] per GPU share: 2M x 4M, nnz 40M over 8 GPUs
    "c4": dict(m=2_000_000, n=4_000_000, nnz=40_000_000, hids=1024, depth=3),
    # configs[4]: c2 graph, hid 2048, depth 6, bf16
    "c5": dict(m=100_000, n=200_000, nnz=2_000_000, hids=2048, depth=6),
    # SURVEY.md 8d skewed-degree workload: Zipf(1.5) row degrees (skewed_lp) at the c2 sizes and model
    "skewed": dict(m=100_000, n=200_000, nnz=2_000_000, hids=1024, depth=3),
}
