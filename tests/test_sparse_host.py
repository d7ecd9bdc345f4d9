"""Host-side scheduling decisions of lpgnn.sparse (no kernel runs): the degree-aware heavy-row list and the
gather-locality rule that picks full-width SpMM rows (round 6), on CSRs packed by the library's host pack."""
import numpy as np

from lpgnn import BipartiteCSR, synth
from lpgnn import sparse as S


def _adj(g):
    return BipartiteCSR.from_coo(g.row, g.col, g.val, g.m, g.n, device="cpu")


def test_hot_source_fraction_separates_skewed_from_uniform():
    """The c2-sized uniform LP: the 16 K most-referenced sources (64 MB of F = 1024 fp32 rows) serve 13-17 %
    of the edges in both directions -> 128-column slices stay; the Zipf(1.5) LP's vars<-cons direction
    (gathering 408 dense constraint rows) serves >= 90 % -> full-width rows."""
    rows = S.HOT_CACHE_BYTES // (1024 * 4)
    uni = _adj(synth.uniform_lp(100_000, 200_000, 2_000_000, seed=0))
    sk = _adj(synth.skewed_lp(100_000, 200_000, 2_000_000, a=1.5, seed=0))
    for csr in (uni.fwd, uni.bwd, sk.fwd):
        assert csr.hot_source_fraction(rows) < S.HOT_FRACTION
    assert sk.bwd.hot_source_fraction(rows) >= 0.9


def test_hot_source_fraction_exact_and_cached():
    """The fraction is exactly (edges on the top-k sources) / nnz; a graph whose sources all fit is 1.0,
    an empty one 0.0; the value is computed once per (CSR, budget)."""
    rng = np.random.default_rng(3)
    m, n = 50, 40
    deg_src = rng.integers(0, 6, n)  # edges per source column
    col = np.repeat(np.arange(n), deg_src)
    row = np.concatenate([rng.choice(m, d, replace=False) for d in deg_src]).astype(np.int64)
    g = BipartiteCSR.from_coo(row, col, np.ones(len(col), np.float32), m, n, device="cpu")
    top = np.sort(deg_src)[::-1]
    for k in (1, 5, 17):
        assert abs(g.fwd.hot_source_fraction(k) - top[:k].sum() / len(col)) < 1e-12
    assert g.fwd.hot_source_fraction(n) == 1.0
    assert g.fwd._hot[5] == g.fwd.hot_source_fraction(5)
    e = BipartiteCSR.from_coo(np.zeros(0, np.int64), np.zeros(0, np.int64), np.zeros(0, np.float32), 3, 4,
                              device="cpu")
    assert e.fwd.hot_source_fraction(10) == 0.0


def test_heavy_rows_list_longest_first():
    """heavy_rows(thresh): exactly the rows above the threshold, longest first (their units start first)."""
    g = _adj(synth.skewed_lp(3000, 5000, 60000, seed=11))
    deg = (g.fwd.rowptr[1:] - g.fwd.rowptr[:-1]).numpy()
    for t in (0, 64, 1024):
        idx, cnt = g.fwd.heavy_rows(t)
        idx = idx.numpy()
        assert cnt == int((deg > t).sum()) and set(idx.tolist()) == set(np.nonzero(deg > t)[0].tolist())
        assert np.all(np.diff(deg[idx]) <= 0)
