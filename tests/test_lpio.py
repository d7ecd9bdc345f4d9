"""On-disk format + LP features (lpgnn.lpio), host side, vs golden vectors
made from the reference's own scaling / cvt_to_features bodies."""
import numpy as np
import scipy.sparse as sp
import torch

from oracle import model_ref as O


def test_scaling_and_features_match_reference_bodies(golden_dir):
    from lpgnn import lpio

    g = dict(np.load(f"{golden_dir}/features_small.npz"))
    for i in range(2):
        m, n = int(g[f"m_{i}"]), int(g[f"n_{i}"])
        A = sp.coo_matrix((g[f"in_data_{i}"], (g[f"in_row_{i}"], g[f"in_col_{i}"])), shape=(m, n)).tocsr()
        args = [g[f"in_{k}_{i}"].copy() for k in ("c", "bl")] + [A] + [g[f"in_{k}_{i}"].copy() for k in ("bu", "l", "u")]
        c, bl, As, bu, l, u = lpio.scaling(*args)
        v_f, c_f = lpio.cvt_to_features(c, bl, As, bu, l, u)
        Ac = As.tocoo()
        assert np.array_equal(Ac.row, g[f"out_row_{i}"]) and np.array_equal(Ac.col, g[f"out_col_{i}"])
        assert np.array_equal(Ac.data, g[f"out_data_{i}"])
        assert np.array_equal(c, g[f"out_c_{i}"])
        assert np.array_equal(v_f, g[f"v_feas_{i}"])
        assert np.array_equal(c_f, g[f"c_feas_{i}"])
        # scaled coefficients and cons features lie in [-1, 1] (dataset.py:235-238)
        assert np.abs(Ac.data).max() <= 1 and np.abs(c_f).max() <= 1


def test_msgpack_numpy_roundtrip(tmp_path):
    from lpgnn import lpio

    rec = [np.arange(5, dtype=np.float64), np.array([-np.inf, 1.5]),
           (np.array([0, 1], np.int32), np.array([2, 0], np.int64), np.array([0.5, -1.0])),
           np.float64(3.25), np.array([[1, 2], [3, 4]], np.int16), np.array(["c0", "c1"]), 7, "name"]
    p = tmp_path / "x.pk"
    lpio.msgpack_dump(rec, p)
    back = lpio.msgpack_load(p)
    assert np.array_equal(back[0], rec[0]) and back[0].dtype == np.float64
    assert np.array_equal(back[1], rec[1])
    assert all(np.array_equal(a, b) and a.dtype == b.dtype for a, b in zip(back[2], rec[2]))
    assert back[3] == 3.25  # np.float64 is a float subclass: msgpack packs it natively
    assert np.array_equal(back[4], rec[4]) and back[4].shape == (2, 2)
    assert list(back[5]) == ["c0", "c1"] and back[6] == 7 and back[7] == "name"


def test_raw_to_processed_to_bipartite(tmp_path, golden_dir):
    """cvt_to_pkl raw record -> LPDataset.process -> .pk -> LPDataset.get +
    MyToBipartite (host pack) == the oracle restatement of the same chain."""
    from lpgnn import lpio

    g = dict(np.load(f"{golden_dir}/features_small.npz"))
    i = 1
    m, n = int(g[f"m_{i}"]), int(g[f"n_{i}"])
    # labels consistent with the bound tags (dataset.py:203-207)
    rng = np.random.default_rng(0)
    y_s = np.where(np.isinf(g[f"in_bl_{i}"]), 1, rng.integers(0, 3, m))
    y_s[np.isinf(g[f"in_bu_{i}"]) & (y_s == 2)] = 1
    y_t = np.where(np.isinf(g[f"in_u_{i}"]), rng.integers(0, 2, n), rng.integers(0, 3, n))
    raw = [g[f"in_c_{i}"], g[f"in_bl_{i}"], (g[f"in_row_{i}"], g[f"in_col_{i}"], g[f"in_data_{i}"]),
           g[f"in_bu_{i}"], g[f"in_l_{i}"], g[f"in_u_{i}"], y_s, y_t,
           np.array([f"c{k}" for k in range(m)]), np.array([f"v{k}" for k in range(n)])]
    raw_p, proc_p = tmp_path / "raw.pk", tmp_path / "proc.pk"
    lpio.msgpack_dump(raw, raw_p)
    proc = lpio.process_raw(lpio.msgpack_load(raw_p))
    assert np.array_equal(proc[3], g[f"c_feas_{i}"].astype(np.float32))
    lpio.msgpack_dump(proc, proc_p)
    batch = lpio.load_processed(proc_p, device="cpu")
    row, col, A_data, c_feas, v_feas, ys, yt, nnodes = proc
    ei, ea = O.to_undirected(np.stack([row, col + m]), A_data.astype(np.float32), m + n)
    r = O.my_to_bipartite(np.concatenate([c_feas, v_feas]), np.concatenate([ys, yt]),
                          np.r_[np.zeros(m, int), np.ones(n, int)], ei, ea, m + n)
    assert torch.equal(batch.x_s, torch.from_numpy(r["x_s"])) and torch.equal(batch.x_t, torch.from_numpy(r["x_t"]))
    assert torch.equal(batch.y_s, torch.from_numpy(r["y_s"])) and (batch.s_bs, batch.t_bs) == (r["s_bs"], r["t_bs"])
    for a, b in zip((batch.edge_index.fwd.rowptr, batch.edge_index.fwd.col, batch.edge_index.fwd.val), r["A"]):
        assert np.array_equal(a.numpy(), b)


def test_direct_bipartite_equals_reference_chain(tmp_path, golden_dir):
    """load_bipartite (no to_undirected round trip) == load_processed (the
    reference chain) attribute for attribute, host pack."""
    from lpgnn import lpio

    g = dict(np.load(f"{golden_dir}/features_small.npz"))
    i = 1
    m, n = int(g[f"m_{i}"]), int(g[f"n_{i}"])
    rng = np.random.default_rng(1)
    rec = [g[f"out_row_{i}"], g[f"out_col_{i}"], g[f"out_data_{i}"].astype(np.float32),
           g[f"c_feas_{i}"].astype(np.float32), g[f"v_feas_{i}"].astype(np.float32),
           rng.integers(0, 3, m), rng.integers(0, 3, n), m + n]
    p = tmp_path / "p.pk"
    lpio.msgpack_dump(rec, p)
    a, b = lpio.load_processed(p), lpio.load_bipartite(p)
    for k in ("x_s", "x_t", "y_s", "y_t"):
        assert torch.equal(getattr(a, k), getattr(b, k)), k
    assert (a.s_bs, a.t_bs, a.bs) == (b.s_bs, b.t_bs, b.bs)
    for o in ("fwd", "bwd"):
        ca, cb = getattr(a.edge_index, o), getattr(b.edge_index, o)
        for f in ("rowptr", "col", "val"):
            assert torch.equal(getattr(ca, f), getattr(cb, f)), (o, f)
    # duplicate entries take the reference chain (summed by to_undirected)
    rec2 = list(rec)
    rec2[0] = np.r_[rec[0], rec[0][:1]]
    rec2[1] = np.r_[rec[1], rec[1][:1]]
    rec2[2] = np.r_[rec[2], rec[2][:1]]
    lpio.msgpack_dump(rec2, p)
    c = lpio.load_bipartite(p)
    assert c.edge_index.nnz() == a.edge_index.nnz()
