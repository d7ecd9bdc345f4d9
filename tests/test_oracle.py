"""The oracle (oracle/) pinned against the golden vectors made from the
reference's own function bodies (tests/golden/make_golden.py)."""
import numpy as np
import pytest
import torch

from oracle import model_ref as O


def _load(golden_dir, name):
    return dict(np.load(f"{golden_dir}/{name}", allow_pickle=False))


def test_spmm_loop_bitwise(golden_dir):
    g = _load(golden_dir, "spmm_small.npz")
    A = (g["a_rowptr"], g["a_col"], g["a_val"])
    AT = (g["at_rowptr"], g["at_col"], g["at_val"])
    for Fd in (1, 8, 40, 256, 1024):
        for nt in (1, 3):
            assert np.array_equal(O.spmm_f32(*A, g[f"Xv_{Fd}"], nthreads=nt), g[f"Yc_{Fd}"])
            assert np.array_equal(O.spmm_f32(*AT, g[f"Xc_{Fd}"], nthreads=nt), g[f"Yv_{Fd}"])


def test_spmm_loop_matches_fp64_sum(golden_dir):
    g = _load(golden_dir, "spmm_small.npz")
    import scipy.sparse as sp

    A = sp.csr_matrix((g["a_val"].astype(np.float64), g["a_col"], g["a_rowptr"]), shape=(int(g["m"]), int(g["n"])))
    ref = A @ g["Xv_256"].astype(np.float64)
    np.testing.assert_allclose(g["Yc_256"], ref, rtol=1e-5, atol=1e-5)


def test_csr_pack_orders(golden_dir):
    g = _load(golden_dir, "spmm_small.npz")
    m, n = int(g["m"]), int(g["n"])
    A = O.csr_from_coo(g["coo_row"], g["coo_col"], g["coo_val"], m, n)
    for a, b in zip(A, (g["a_rowptr"], g["a_col"], g["a_val"])):
        assert np.array_equal(a, b)
    # rows sorted by column, transpose sorted by row (torch_sparse order)
    for rp, c in ((g["a_rowptr"], g["a_col"]), (g["at_rowptr"], g["at_col"])):
        for i in range(len(rp) - 1):
            seg = c[rp[i]:rp[i + 1]]
            assert np.all(np.diff(seg) > 0)
    # dense row 0, empty row 1, empty column 2 (edge cases of the fixture)
    assert g["a_rowptr"][1] - g["a_rowptr"][0] == n - 1
    assert g["a_rowptr"][2] == g["a_rowptr"][1]
    assert g["at_rowptr"][3] == g["at_rowptr"][2]


def test_bf16_loop_rounds_once():
    rng = np.random.default_rng(0)
    rowptr = np.array([0, 3, 3, 5], np.int64)
    col = np.array([0, 1, 2, 0, 2], np.int32)
    val = rng.uniform(-1, 1, 5).astype(np.float32)
    X = rng.standard_normal((3, 16)).astype(np.float32)
    Xb = (X.view(np.uint32) >> 16).astype(np.uint16)
    Y = O.spmm_bf16(rowptr, col, val, Xb)
    Xf = (Xb.astype(np.uint32) << 16).view(np.float32)
    Yf = O.spmm_f32(rowptr, col, val, Xf)
    u = Yf.view(np.uint32).astype(np.uint64)
    rne = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)
    assert np.array_equal(Y, rne)


@pytest.mark.parametrize("name", ["gcn_fc_d3_h32.npz", "gcn_fc_d4_h16.npz"])
def test_model_restatement_matches_reference_bodies(golden_dir, name):
    g = _load(golden_dir, name)
    m, n, depth = int(g["m"]), int(g["n"]), int(g["depth"])
    A = O.csr_from_coo(g["coo_row"], g["coo_col"], g["coo_val"], m, n)
    AT = O.csr_transpose(*A, m, n)
    sd = {k[3:]: torch.from_numpy(v) for k, v in g.items() if k.startswith("sd.")}
    x_s, x_t = torch.from_numpy(g["x_s"]), torch.from_numpy(g["x_t"])
    with torch.no_grad():
        lc, lv = O.gcn_fc_forward(sd, x_s, x_t, A, AT, depth)
    np.testing.assert_allclose(lc.numpy(), g["logit_cons"], rtol=0, atol=1e-6)
    np.testing.assert_allclose(lv.numpy(), g["logit_vars"], rtol=0, atol=1e-6)
    labels = O.inference_gnn(torch.cat((lc, lv)), m)
    assert np.array_equal(labels.numpy(), g["labels"])
    # training step gradients (dropout p = 0)
    params = {k: v.clone().requires_grad_(True) for k, v in sd.items()}
    lc, lv = O.gcn_fc_forward(params, x_s, x_t, A, AT, depth)
    loss = O.balanced(lc, lv, torch.from_numpy(g["y_s"]), torch.from_numpy(g["y_t"]))
    loss.backward()
    assert abs(loss.item() - float(g["loss"])) < 1e-5
    for k, p in params.items():
        np.testing.assert_allclose(p.grad.numpy(), g["grad." + k], rtol=1e-4, atol=1e-6)


def test_model_fp64_agrees(golden_dir):
    g = _load(golden_dir, "gcn_fc_d3_h32.npz")
    m, n = int(g["m"]), int(g["n"])
    A = O.csr_from_coo(g["coo_row"], g["coo_col"], g["coo_val"], m, n)
    AT = O.csr_transpose(*A, m, n)
    sd = {k[3:]: torch.from_numpy(v) for k, v in g.items() if k.startswith("sd.")}
    sd64 = {k: v.double() for k, v in sd.items()}
    lc, lv = O.gcn_fc_forward(sd64, torch.from_numpy(g["x_s"]).double(), torch.from_numpy(g["x_t"]).double(),
                              A, AT, 3)
    np.testing.assert_allclose(lc.numpy(), g["logit_cons"], atol=1e-4)
    np.testing.assert_allclose(lv.numpy(), g["logit_vars"], atol=1e-4)


def test_postprocessing_matches_reference_bodies(golden_dir):
    g = _load(golden_dir, "post_small.npz")
    for i in range(3):
        m = int(g[f"m_{i}"])
        lg = torch.from_numpy(g[f"logits_{i}"])
        kl, kr = O.add_knowledge(lg[:m].clone(), lg[m:].clone(), torch.from_numpy(g[f"feas_l_{i}"]),
                                 torch.from_numpy(g[f"feas_r_{i}"]))
        np.testing.assert_array_equal(kl.numpy(), g[f"know_l_{i}"])
        np.testing.assert_array_equal(kr.numpy(), g[f"know_r_{i}"])
        assert np.array_equal(O.inference_gnn(torch.cat((kl, kr)), m).numpy(), g[f"pred_{i}"])
    for i in range(4):
        w = O.labels_to_balanced_weights(torch.from_numpy(g[f"bw_in_{i}"]))
        np.testing.assert_array_equal(w.numpy(), g[f"bw_out_{i}"])
    loss = O.balanced(*(torch.from_numpy(g[k]) for k in ("bal_lc", "bal_lv", "bal_ys", "bal_yt")))
    assert loss.item() == pytest.approx(float(g["bal_loss"]), abs=1e-6)


def test_to_bipartite_matches_reference_body(golden_dir):
    g = _load(golden_dir, "bipartite_small.npz")
    r = O.my_to_bipartite(g["x"], g["y"], g["is_vars"], g["edge_index"], g["edge_attr"], int(g["num_nodes"]))
    for k in ("x_s", "x_t", "y_s", "y_t"):
        assert np.array_equal(r[k], g[k])
    assert (r["m"], r["n"]) == tuple(g["sizes"])
    assert (r["s_bs"], r["t_bs"]) == (int(g["s_bs"]), int(g["t_bs"]))
    ref = O.csr_from_coo(g["l2r"][0], g["l2r"][1], g["l2r_attr"], *g["sizes"])
    for a, b in zip(r["A"], ref):
        assert np.array_equal(a, b)
