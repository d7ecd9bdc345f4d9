"""HIP SpMM / pack parity vs the oracle (bitwise: the kernel reproduces the
torch_sparse spmm_cpu summation order exactly).  All through the C ABI."""
import numpy as np
import pytest
import torch

from oracle import model_ref as O

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _graph(rng, m, n, nnz, dense_row=False):
    keys = rng.choice(m * n, size=nnz, replace=False)
    row, col = keys // n, keys % n
    if dense_row:
        row = np.concatenate([row[row != 0], np.zeros(n, np.int64)])
        col = np.concatenate([col[(keys // n) != 0], np.arange(n)])
    val = rng.uniform(-1, 1, len(row)).astype(np.float32)
    return row.astype(np.int64), col.astype(np.int64), val


def _adj(row, col, val, m, n):
    from lpgnn import BipartiteCSR

    return BipartiteCSR.from_coo(row, col, val, m, n, device=DEV)


def _oracle_pair(row, col, val, m, n):
    A = O.csr_from_coo(row, col, val, m, n)
    return A, O.csr_transpose(*A, m, n)


def test_golden_fixture_bitwise(golden_dir):
    from lpgnn.sparse import spmm_forward

    g = dict(np.load(f"{golden_dir}/spmm_small.npz"))
    m, n = int(g["m"]), int(g["n"])
    adj = _adj(g["coo_row"], g["coo_col"], g["coo_val"], m, n)
    assert np.array_equal(adj.fwd.col.cpu().numpy(), g["a_col"])
    assert np.array_equal(adj.bwd.rowptr.cpu().numpy(), g["at_rowptr"])
    for Fd in (1, 8, 40, 256, 1024):
        yc = spmm_forward(adj.fwd, torch.from_numpy(g[f"Xv_{Fd}"]).to(DEV)).cpu().numpy()
        yv = spmm_forward(adj.bwd, torch.from_numpy(g[f"Xc_{Fd}"]).to(DEV)).cpu().numpy()
        assert np.array_equal(yc, g[f"Yc_{Fd}"]), f"cons<-vars F={Fd}"
        assert np.array_equal(yv, g[f"Yv_{Fd}"]), f"vars<-cons F={Fd}"


@pytest.mark.parametrize("Fd", [1, 2, 3, 5, 8, 16, 33, 64, 65, 100, 128, 256, 260, 512, 768, 1000, 1024, 1028, 2048])
def test_widths_bitwise(Fd):
    from lpgnn.sparse import spmm_forward

    rng = np.random.default_rng(Fd)
    m, n = 300, 517
    row, col, val = _graph(rng, m, n, 4000, dense_row=True)
    adj = _adj(row, col, val, m, n)
    A, AT = _oracle_pair(row, col, val, m, n)
    Xv = rng.standard_normal((n, Fd)).astype(np.float32)
    Xc = rng.standard_normal((m, Fd)).astype(np.float32)
    assert np.array_equal(spmm_forward(adj.fwd, torch.from_numpy(Xv).to(DEV)).cpu().numpy(), O.spmm_f32(*A, Xv))
    assert np.array_equal(spmm_forward(adj.bwd, torch.from_numpy(Xc).to(DEV)).cpu().numpy(), O.spmm_f32(*AT, Xc))


@pytest.mark.parametrize("slice_cols", [64, 128, 256, 512, 1024])
def test_slice_widths_bitwise(slice_cols):
    from lpgnn import _lib
    from lpgnn.sparse import spmm_forward

    rng = np.random.default_rng(7)
    m, n, Fd = 200, 300, 1024
    row, col, val = _graph(rng, m, n, 3000)
    adj = _adj(row, col, val, m, n)
    A, _ = _oracle_pair(row, col, val, m, n)
    Xv = rng.standard_normal((n, Fd)).astype(np.float32)
    y = spmm_forward(adj.fwd, torch.from_numpy(Xv).to(DEV), slice_cols=slice_cols).cpu().numpy()
    assert np.array_equal(y, O.spmm_f32(*A, Xv))


def test_strided_and_misaligned_inputs():
    from lpgnn.sparse import spmm_forward

    rng = np.random.default_rng(3)
    m, n, Fd = 50, 80, 300
    row, col, val = _graph(rng, m, n, 600)
    adj = _adj(row, col, val, m, n)
    A, _ = _oracle_pair(row, col, val, m, n)
    big = torch.from_numpy(rng.standard_normal((n, Fd + 5)).astype(np.float32)).to(DEV)
    X = big[:, 1:Fd + 1]  # row stride Fd+5, base misaligned -> generic kernel
    y = spmm_forward(adj.fwd, X).cpu().numpy()
    assert np.array_equal(y, O.spmm_f32(*A, X.cpu().numpy()))


def test_edge_cases_empty():
    from lpgnn.sparse import spmm_forward

    # no edges at all: output is zeros
    adj = _adj(np.zeros(0, np.int64), np.zeros(0, np.int64), np.zeros(0, np.float32), 4, 6)
    y = spmm_forward(adj.fwd, torch.randn(6, 1024, device=DEV))
    assert y.shape == (4, 1024) and bool((y == 0).all())
    y = spmm_forward(adj.bwd, torch.randn(4, 8, device=DEV))
    assert y.shape == (6, 8) and bool((y == 0).all())
    # zero destination rows
    adj = _adj(np.zeros(0, np.int64), np.zeros(0, np.int64), np.zeros(0, np.float32), 0, 3)
    assert spmm_forward(adj.fwd, torch.randn(3, 16, device=DEV)).shape == (0, 16)


def test_long_rows_cross_chunk_boundaries():
    """Rows with 63, 64, 65, 130 and n edges exercise the 64-edge (col,val)
    chunking and the U-unrolled tail."""
    from lpgnn.sparse import spmm_forward

    rng = np.random.default_rng(11)
    n, Fd = 1500, 1024
    degs = [0, 1, 3, 4, 5, 63, 64, 65, 127, 128, 130, 1500]
    row = np.concatenate([np.full(d, i) for i, d in enumerate(degs)]).astype(np.int64)
    col = np.concatenate([np.sort(rng.choice(n, d, replace=False)) for d in degs]).astype(np.int64)
    val = rng.uniform(-1, 1, len(row)).astype(np.float32)
    m = len(degs)
    adj = _adj(row, col, val, m, n)
    A, AT = _oracle_pair(row, col, val, m, n)
    Xv = rng.standard_normal((n, Fd)).astype(np.float32)
    assert np.array_equal(spmm_forward(adj.fwd, torch.from_numpy(Xv).to(DEV)).cpu().numpy(), O.spmm_f32(*A, Xv))
    Xc = rng.standard_normal((m, 8)).astype(np.float32)
    assert np.array_equal(spmm_forward(adj.bwd, torch.from_numpy(Xc).to(DEV)).cpu().numpy(), O.spmm_f32(*AT, Xc))


@pytest.mark.parametrize("Fd", [3, 8, 17, 40, 64, 100, 512, 1024, 2048, 2056])
def test_bf16_bitwise(Fd):
    """bf16 SpMM bitwise vs the oracle: narrow (F <= 64), generic, slice and wide-row paths."""
    from lpgnn.sparse import spmm_forward

    rng = np.random.default_rng(100 + Fd)
    m, n = 120, 260
    row, col, val = _graph(rng, m, n, 2000)
    adj = _adj(row, col, val, m, n)
    A, _ = _oracle_pair(row, col, val, m, n)
    X = torch.randn(n, Fd).to(torch.bfloat16)
    Xbits = X.view(torch.int16).numpy().view(np.uint16)
    y = spmm_forward(adj.fwd, X.to(DEV)).cpu().view(torch.int16).numpy().view(np.uint16)
    assert np.array_equal(y, O.spmm_bf16(*A, Xbits))


def test_device_pack_equals_host_pack():
    from lpgnn import BipartiteCSR

    rng = np.random.default_rng(5)
    for m, n, nnz in ((1, 1, 1), (100, 37, 900), (2000, 3000, 40000)):
        row, col, val = _graph(rng, m, n, nnz)
        perm = rng.permutation(len(row))
        h = BipartiteCSR.from_coo(row[perm], col[perm], val[perm], m, n, device="cpu")
        d = BipartiteCSR.from_coo(row[perm], col[perm], val[perm], m, n, device=DEV)
        for a, b in ((h.fwd, d.fwd), (h.bwd, d.bwd)):
            assert torch.equal(a.rowptr, b.rowptr.cpu())
            assert torch.equal(a.col, b.col.cpu())
            assert torch.equal(a.val, b.val.cpu())


def test_device_pack_rejects_bad_input():
    from lpgnn import BipartiteCSR

    with pytest.raises(RuntimeError, match="duplicate"):
        BipartiteCSR.from_coo([0, 0, 1], [1, 1, 0], [0.5, 0.5, 1.0], 2, 2, device=DEV)
    with pytest.raises(RuntimeError, match="out-of-range"):
        BipartiteCSR.from_coo([0, 5], [1, 1], [0.5, 0.5], 2, 2, device=DEV)


def test_autograd_backward_is_transpose_spmm():
    from lpgnn import spmm

    rng = np.random.default_rng(9)
    m, n, Fd = 150, 260, 1024
    row, col, val = _graph(rng, m, n, 2500)
    adj = _adj(row, col, val, m, n)
    A, AT = _oracle_pair(row, col, val, m, n)
    X = torch.from_numpy(rng.standard_normal((n, Fd)).astype(np.float32)).to(DEV).requires_grad_(True)
    G = rng.standard_normal((m, Fd)).astype(np.float32)
    Y = spmm(adj, X)
    Y.backward(torch.from_numpy(G).to(DEV))
    assert np.array_equal(X.grad.cpu().numpy(), O.spmm_f32(*AT, G))


def test_deterministic_run_to_run():
    from lpgnn.sparse import spmm_forward

    rng = np.random.default_rng(1)
    m, n = 5000, 9000
    row, col, val = _graph(rng, m, n, 100000)
    adj = _adj(row, col, val, m, n)
    X = torch.randn(n, 1024, device=DEV)
    y0 = spmm_forward(adj.fwd, X)
    for _ in range(3):
        assert torch.equal(spmm_forward(adj.fwd, X), y0)


def test_full_size_c2_sampled_rows_and_linearity():
    """BASELINE config c2 at full size (100K x 200K, nnz 2M, F 1024): a
    sample of 3000 output rows per direction is compared bitwise with the
    oracle loop on exactly those rows; linearity and the all-ones row-sum
    identity cover the whole output (size-independent properties)."""
    from lpgnn import synth
    from lpgnn.sparse import spmm_forward

    g = synth.uniform_lp(100_000, 200_000, 2_000_000, seed=0)
    adj = _adj(g.row, g.col, g.val, g.m, g.n)
    A, AT = _oracle_pair(g.row, g.col, g.val, g.m, g.n)
    rng = np.random.default_rng(0)
    for csr, oc, K in ((adj.fwd, A, g.n), (adj.bwd, AT, g.m)):
        X = torch.randn(K, 1024, device=DEV)
        Y = spmm_forward(csr, X)
        rows = np.sort(rng.choice(csr.n_rows, 3000, replace=False))
        rp, c, v = oc
        sub_rp = np.concatenate([[0], np.cumsum(rp[rows + 1] - rp[rows])])
        idx = np.concatenate([np.arange(rp[r], rp[r + 1]) for r in rows])
        ref = O.spmm_f32(sub_rp, c[idx], v[idx], X.cpu().numpy())
        assert np.array_equal(Y[torch.from_numpy(rows).to(DEV)].cpu().numpy(), ref)
        # linearity: spmm(2X) == 2 spmm(X) exactly (power-of-two scaling is exact)
        assert torch.equal(spmm_forward(csr, 2 * X), 2 * Y)
        # ones: row sums of |A| structure
        ones = torch.ones(K, 256, device=DEV)
        rs = spmm_forward(csr, ones)[:, 0].double().cpu().numpy()
        exact = np.add.reduceat(np.concatenate([v.astype(np.float64), [0]]), rp[:-1]) * (np.diff(rp) > 0)
        np.testing.assert_allclose(rs, exact, atol=1e-4)


def test_direct_bipartite_device_pack_equals_reference_chain():
    """bipartite_from_lp on the GPU == MyToBipartite(lp_to_unipartite(...)) (the reference chain)."""
    from lpgnn import synth
    from lpgnn.data import MyToBipartite, bipartite_from_lp, lp_to_unipartite

    g = synth.skewed_lp(3000, 5000, 40000, seed=3)
    args = (g.row, g.col, g.val, g.x_s, g.x_t, g.y_s, g.y_t)
    a = MyToBipartite(dev=DEV)(lp_to_unipartite(*args))
    b = bipartite_from_lp(*args, device=DEV)
    for k in ("x_s", "x_t", "y_s", "y_t"):
        assert torch.equal(getattr(a, k), getattr(b, k)), k
    for o in ("fwd", "bwd"):
        ca, cb = getattr(a.edge_index, o), getattr(b.edge_index, o)
        for f in ("rowptr", "col", "val"):
            assert torch.equal(getattr(ca, f), getattr(cb, f)), (o, f)


@pytest.mark.parametrize("thresh", [0, 3, 64, 1024])
@pytest.mark.parametrize("Fd,slice_cols", [(1024, 0), (1000, 0), (512, 512), (2048, 1024), (300, 0)])
def test_degree_aware_heavy_rows_bitwise(thresh, Fd, slice_cols, monkeypatch):
    """lpg_spmm_f32_heavy on a Zipf(1.5) skewed LP (rows up to thousands of
    edges, many of degree 1, empty rows): rows above the threshold run as
    64-column wave units, the rest as usual -- both directions bitwise the
    torch_sparse spmm_cpu loop, for every threshold (0 = every non-empty row
    heavy), ragged F and every slice width."""
    from lpgnn import _lib, sparse, synth
    from lpgnn.sparse import spmm_forward

    g = synth.skewed_lp(3000, 5000, 60000, seed=11)
    row = np.concatenate([g.row, np.full(4000, 7, np.int64)])  # row 7: a dense constraint (4000 extra edges)
    col = np.concatenate([g.col, np.arange(1000, 5000, dtype=np.int64)])
    key = np.unique(row * g.n + col)
    row, col = key // g.n, key % g.n
    val = np.random.default_rng(2).uniform(-1, 1, len(row)).astype(np.float32)
    adj = _adj(row, col, val, g.m, g.n)
    A, AT = _oracle_pair(row, col, val, g.m, g.n)
    assert adj.fwd.degrees().max().item() > 4000
    rng = np.random.default_rng(Fd)
    for csr, ref, n_src in ((adj.fwd, A, g.n), (adj.bwd, AT, g.m)):
        X = rng.standard_normal((n_src, Fd)).astype(np.float32)
        got = spmm_forward(csr, torch.from_numpy(X).to(DEV), slice_cols=slice_cols, heavy=thresh).cpu().numpy()
        assert np.array_equal(got, O.spmm_f32(*ref, X))
        if thresh < csr.degrees().max().item():  # the heavy path actually ran in this direction
            assert csr.heavy_rows(thresh)[1] > 0


@pytest.mark.parametrize("depth", [8, 16, 32])
@pytest.mark.parametrize("Fd,dt", [(1024, torch.float32), (300, torch.float32), (2048, torch.float32)])
def test_gather_depth_bitwise(depth, Fd, dt):
    """Every gather depth (edges in flight per wave; a chunk's remainder gathered together,
    predicated per edge) gives the oracle loop's bits, for 128- and 256-column slices; degrees
    0..150 so every remainder length 0 .. depth-1 occurs, and rows cross the 64-edge chunks."""
    from lpgnn.sparse import spmm_forward

    rng = np.random.default_rng(depth + Fd)
    m, n = 700, 900
    deg = rng.integers(0, 151, m)
    row = np.repeat(np.arange(m), deg)
    col = np.concatenate([rng.choice(n, d, replace=False) for d in deg]).astype(np.int64)
    val = rng.uniform(-1, 1, len(row)).astype(np.float32)
    adj = _adj(row, col, val, m, n)
    X = torch.from_numpy(rng.standard_normal((n, Fd)).astype(np.float32)).to(dt)
    outs = [spmm_forward(adj.fwd, X.to(DEV), slice_cols=sl, depth=depth).cpu() for sl in (0, 256)]
    assert torch.equal(outs[0], outs[1])
    A, _ = _oracle_pair(row, col, val, m, n)
    assert np.array_equal(outs[0].numpy(), O.spmm_f32(*A, X.numpy()))


@pytest.mark.parametrize("slice_cols", [0, 256, 512, 1024])
@pytest.mark.parametrize("Fd", [256, 1000, 2048])
def test_bf16_slice_widths_bitwise(slice_cols, Fd):
    """bf16 SpMM: the 256-column slice kernel (the default) and the 16-B-per-lane row
    kernels give the oracle's bits for every slice width, degrees 0..150."""
    from lpgnn import _lib
    from lpgnn.sparse import spmm_forward

    rng = np.random.default_rng(Fd + slice_cols)
    m, n = 300, 500
    deg = rng.integers(0, 151, m)
    row = np.repeat(np.arange(m), deg)
    col = np.concatenate([rng.choice(n, d, replace=False) for d in deg]).astype(np.int64)
    val = rng.uniform(-1, 1, len(row)).astype(np.float32)
    adj = _adj(row, col, val, m, n)
    A, _ = _oracle_pair(row, col, val, m, n)
    X = torch.randn(n, Fd).to(torch.bfloat16)
    Xbits = X.view(torch.int16).numpy().view(np.uint16)
    y = spmm_forward(adj.fwd, X.to(DEV), slice_cols=slice_cols).cpu().view(torch.int16).numpy().view(np.uint16)
    assert np.array_equal(y, O.spmm_bf16(*A, Xbits))


@pytest.mark.parametrize("thresh", [0, 3, 64])
@pytest.mark.parametrize("Fd", [512, 1000, 2048])
def test_bf16_heavy_rows_bitwise(thresh, Fd, monkeypatch):
    """bf16 degree-aware split (lpg_spmm_bf16_heavy): rows above the threshold on
    (row, 128-column) wave units give the oracle's bits; a 2000-edge row crosses many
    64-edge chunks and the 32-gather batches."""
    from lpgnn import sparse as S
    from lpgnn.sparse import spmm_forward

    rng = np.random.default_rng(Fd + thresh)
    m, n = 200, 2500
    deg = rng.integers(0, 40, m)
    deg[[3, 77, 150]] = [2000, 130, 65]
    row = np.repeat(np.arange(m), deg)
    col = np.concatenate([rng.choice(n, d, replace=False) for d in deg]).astype(np.int64)
    val = rng.uniform(-1, 1, len(row)).astype(np.float32)
    adj = _adj(row, col, val, m, n)
    A, _ = _oracle_pair(row, col, val, m, n)
    X = torch.randn(n, Fd).to(torch.bfloat16)
    Xbits = X.view(torch.int16).numpy().view(np.uint16)
    y = spmm_forward(adj.fwd, X.to(DEV), heavy=thresh).cpu().view(torch.int16).numpy().view(np.uint16)
    assert np.array_equal(y, O.spmm_bf16(*A, Xbits))


def _long_row_graph(rng, m, n, long_deg):
    """Rows of degree 0..70 (so the 64-edge narrow threshold falls inside the range) plus a row of
    `long_deg` edges (crosses many LDS chunks) and one of exactly 64 and 65 edges."""
    deg = rng.integers(0, 71, m)
    deg[[1, 5, 9]] = [long_deg, 64, 65]
    row = np.repeat(np.arange(m), deg)
    col = np.concatenate([np.sort(rng.choice(n, d, replace=False)) for d in deg]).astype(np.int64)
    val = rng.uniform(-1, 1, len(row)).astype(np.float32)
    return row, col, val


@pytest.mark.parametrize("thresh", [0, 3, 64, 1024])
@pytest.mark.parametrize("Fd", [1, 3, 8, 16, 33, 64])
def test_narrow_heavy_rows_bitwise(thresh, Fd):
    """F <= 64 with the heavy-row unit (spmm.hip narrow_heavy_row: one 256-lane block per row above
    min(thresh, NARROW_HEAVY) edges, products staged in LDS, each column's chain summed in CSR order):
    bitwise the oracle's spmm_cpu loop, in fp32 and in bf16 / fp16 storage, on a graph with a
    50 000-edge row (12+ LDS chunks at F = 8) and rows on both sides of the threshold."""
    from lpgnn import sparse as S
    from lpgnn.sparse import spmm_forward

    rng = np.random.default_rng(Fd * 7 + thresh)
    m, n = 400, 60000
    row, col, val = _long_row_graph(rng, m, n, 50000)
    adj = _adj(row, col, val, m, n)
    A, _ = _oracle_pair(row, col, val, m, n)
    eff = min(thresh, S.NARROW_HEAVY) if thresh > 0 else 0
    if eff > 0:
        assert adj.fwd.heavy_rows(eff)[1] > 0  # the heavy units really run
    X = rng.standard_normal((n, Fd)).astype(np.float32)
    got = spmm_forward(adj.fwd, torch.from_numpy(X).to(DEV), heavy=thresh).cpu().numpy()
    assert np.array_equal(got, O.spmm_f32(*A, X))
    Xb = torch.from_numpy(X).to(torch.bfloat16)
    yb = spmm_forward(adj.fwd, Xb.to(DEV), heavy=thresh).cpu().view(torch.int16).numpy().view(np.uint16)
    assert np.array_equal(yb, O.spmm_bf16(*A, Xb.view(torch.int16).numpy().view(np.uint16)))
    Xh = torch.from_numpy(X).half()  # fp16 mode: the edge values rounded to fp16 too (batch_to(half=True))
    yh = spmm_forward(adj.half().fwd, Xh.to(DEV), heavy=thresh).cpu()
    assert torch.equal(yh.float(), O.spmm_f16(*A, Xh))


def test_narrow_heavy_strided_output_and_empty():
    """The heavy unit honours ldx / ldy (an F = 8 slice of wider buffers) and leaves other columns alone;
    a graph whose only edges are in one heavy row, and a heavy list on a graph with no edges."""
    from lpgnn.sparse import spmm_forward
    from lpgnn import _lib
    import ctypes

    rng = np.random.default_rng(5)
    m, n = 3, 5000
    row = np.full(5000, 1, np.int64)
    col = np.arange(5000, dtype=np.int64)
    val = rng.uniform(-1, 1, 5000).astype(np.float32)
    adj = _adj(row, col, val, m, n)
    A, _ = _oracle_pair(row, col, val, m, n)
    X = rng.standard_normal((n, 8)).astype(np.float32)
    y = spmm_forward(adj.fwd, torch.from_numpy(X).to(DEV), heavy=64).cpu().numpy()
    assert np.array_equal(y, O.spmm_f32(*A, X))
    # strided: X is [n, 8] inside [n, 12], Y is [m, 8] inside [m, 20] (sentinel elsewhere)
    Xbig = torch.zeros(n, 12, device=DEV)
    Xbig[:, 2:10] = torch.from_numpy(X).to(DEV)
    Ybig = torch.full((m, 20), 7.0, device=DEV)
    idx, cnt = adj.fwd.heavy_rows(64)
    L = _lib.lib()
    with torch.cuda.device(DEV):
        st = L.lpg_spmm_f32_heavy(ctypes.byref(adj.fwd.cstruct()), Xbig[:, 2:].data_ptr(), 12, Ybig[:, 4:].data_ptr(),
                                  20, 8, idx.data_ptr(), cnt, 64, _lib.stream_of(Xbig))
    _lib.check(st, "lpg_spmm_f32_heavy")
    Yb = Ybig.cpu().numpy()
    assert np.array_equal(Yb[:, 4:12], O.spmm_f32(*A, X))
    assert (Yb[:, :4] == 7).all() and (Yb[:, 12:] == 7).all()


def test_narrow_heavy_skewed_lp_full_size():
    """The skewed sub-record's conv1 input SpMM (synth.skewed_lp at the c2 sizes, Zipf(1.5) rows up to
    6 025 edges, F = 8) bitwise the oracle loop in both directions, with the default options."""
    from lpgnn import synth
    from lpgnn.sparse import spmm_forward

    g = synth.skewed_lp(100_000, 200_000, 2_000_000, a=1.5, seed=0)
    adj = _adj(g.row, g.col, g.val, g.m, g.n)
    A, AT = _oracle_pair(g.row, g.col, g.val, g.m, g.n)
    rng = np.random.default_rng(0)
    Xv = rng.standard_normal((g.n, 8)).astype(np.float32)
    Xc = rng.standard_normal((g.m, 8)).astype(np.float32)
    assert np.array_equal(spmm_forward(adj.fwd, torch.from_numpy(Xv).to(DEV)).cpu().numpy(), O.spmm_f32(*A, Xv))
    assert np.array_equal(spmm_forward(adj.bwd, torch.from_numpy(Xc).to(DEV)).cpu().numpy(), O.spmm_f32(*AT, Xc))
