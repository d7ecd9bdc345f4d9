"""The f16x2 arithmetic of the fp32 FC kernels (LPGNN_FC_ARITH=f16x2; csrc/fc_x3.hip fc_x3_wide<..., F16>,
lpg_rowscale_f32, lpg_split_f16x2, lpg_fc_f16x2_*): every operand as two fp16 terms after a power-of-2
row scale, three matrix-core products.  Checked against float64 with the error bound the scheme states
(|err| <= 2^-20 sum |a b|, below an fp32 SGEMM's own), against the x3 kernels (same dropout mask, same
epilogues), on the fused heads and conv1-fold forms, and on rows whose scales spread over 2^+-20 (the
case a per-tensor scale breaks)."""
import pytest
import torch

from lpgnn import fc as F

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
BOUND = 2.0 ** -20  # of sum |a b| (tools/experiments/split_error.py measures ~2^-25)


def _err(C, A1, W1, A2=None, W2=None, bias=None, addend=None, relu=False):
    """(max |C - ref| / (sum |a b| + tiny), ref) with ref in float64 (pre-dropout)."""
    A1d, W1d = A1.double(), W1.double()
    ref = A1d @ W1d.T
    den = A1d.abs() @ W1d.abs().T
    if A2 is not None:
        ref = ref + A2.double() @ W2.double().T
        den = den + A2.double().abs() @ W2.double().abs().T
    if addend is not None:
        ref = ref + addend.double()
        den = den + addend.double().abs()
    if bias is not None:
        ref = ref + bias.double()
        den = den + bias.double().abs()
    if relu:
        ref = ref.clamp_min(0)
    return float(((C.double() - ref).abs() / (den + 1e-30)).max()), ref


def test_rowscale_and_split():
    torch.manual_seed(0)
    A = torch.randn(1000, 256, device=DEV) * torch.exp(4 * torch.randn(1000, 1, device=DEV))
    A[7] = 0.0
    s = F.rowscale(A)
    mx = A.abs().amax(1) * s
    nz = A.abs().amax(1) > 0
    assert bool(((mx[nz] >= 2 ** 14) & (mx[nz] < 2 ** 15)).all())
    assert float(s[7]) == 2.0 ** 115  # an all-zero row: the largest scale (combines by min)
    s2 = F.rowscale(A, A * 4)
    assert torch.equal(s2, F.rowscale(A * 4))  # side by side: the smaller scale
    assert F.rowscale(A) is s  # cached for the live, unchanged operand
    A.mul_(2)
    assert F.rowscale(A) is not s and torch.equal((F.rowscale(A) * 2)[nz], s[nz])  # an in-place change re-sweeps
    assert bool((torch.frexp(s).mantissa == 0.5).all())  # powers of two
    W = torch.randn(384, 512, device=DEV) * torch.exp(2 * torch.randn(384, 1, device=DEV))
    for transpose in (False, True):
        P, _, sw = F.split_f16x2(W, None, transpose)
        Wt = W.t() if transpose else W
        h = P[0].view(torch.float16).float()[:, :Wt.shape[1]].double()
        lo = P[1].view(torch.float16).float()[:, :Wt.shape[1]].double()
        x = Wt.double() * sw.double()[:, None]
        assert float(((h + lo - x).abs() - (2 ** -22 * x.abs() + 2 ** -25)).max()) <= 0
        assert bool((P[:, :, Wt.shape[1]:] == 0).all())  # zero padding


@pytest.mark.parametrize("R,N", [(1000, 256), (100_000, 1024), (3001, 2048), (257, 1028), (5, 4), (0, 64), (64, 0)])
def test_rowcolscale_equals_separate_sweeps(R, N):
    """lpg_rowcolscale_f32 (one read, both scales) gives exactly the row sweep's and the column sweep's scales
    (ragged rows and columns, N above one column block, zero rows, empty operands)."""
    from lpgnn import _lib
    torch.manual_seed(R + N)
    G = torch.randn(R, N, device=DEV) * torch.exp(3 * torch.randn(R, 1, device=DEV)) \
        * torch.exp(3 * torch.randn(1, N, device=DEV))
    if R > 10:
        G[3] = 0.0
    L = _lib.lib()
    rs = torch.full((R,), -1.0, device=DEV)
    cs = torch.full((N,), -1.0, device=DEV)
    ws = torch.empty(max(16, L.lpg_rowcolscale_workspace_bytes(R, N)), dtype=torch.uint8, device=DEV)
    _lib.check(L.lpg_rowcolscale_f32(R, N, G.data_ptr(), max(N, 4), rs.data_ptr(), cs.data_ptr(), ws.data_ptr(),
                                     _lib.stream_of(G)), "lpg_rowcolscale_f32")
    zero = 2.0 ** 115
    ref_r = F._rowscale1(G) if N else torch.full((R,), zero, device=DEV)
    ref_c = F._colscale1(G) if R else torch.full((N,), zero, device=DEV)
    assert torch.equal(rs, ref_r)
    assert torch.equal(cs, ref_c)


def test_scale_cache_one_sweep_for_both():
    """A row-scale request fills the column entry too (and the other way round)."""
    G = torch.randn(5000, 512, device=DEV)
    r = F.rowscale(G)
    c = F._SCALES.lookup("col", G)
    assert c is not None and torch.equal(c, F._colscale1(G)) and F.colscale(G) is c
    H = torch.randn(700, 96, device=DEV)
    c = F.colscale(H)
    assert torch.equal(F._SCALES.lookup("row", H), F._rowscale1(H)) and torch.equal(c, F._colscale1(H))
    del r


@pytest.mark.parametrize("M,N,K1,K2,relu,acc,bias", [
    (5000, 1024, 1024, 0, False, False, False),
    (5000, 1024, 1024, 0, True, False, True),
    (3001, 384, 512, 512, True, False, True),   # two operands, ragged M
    (4096, 1024, 1024, 0, True, True, True),    # addend (the re-associated var side)
    (777, 256, 64, 0, False, False, False),
])
def test_fc_f16x2_against_fp64(M, N, K1, K2, relu, acc, bias):
    torch.manual_seed(M + N)
    A1 = torch.randn(M, K1, device=DEV) * torch.exp(torch.randn(M, 1, device=DEV))
    W1 = torch.randn(N, K1, device=DEV) * 0.03
    A2 = torch.randn(M, K2, device=DEV) if K2 else None
    W2 = torch.randn(N, K2, device=DEV) * 0.03 if K2 else None
    b = torch.randn(N, device=DEV) * 0.1 if bias else None
    addend = torch.randn(M, N, device=DEV) if acc else None
    out = addend.clone() if acc else None
    C = F.fc_forward(A1, W1, A2, W2, b, relu, out=out, accumulate=acc, arith="f16x2")
    e, _ = _err(C, A1, W1, A2, W2, b, addend, relu)
    x3 = F.fc_forward(A1, W1, A2, W2, b, relu, out=None if not acc else addend.clone(), accumulate=acc, arith="x3")
    e3, _ = _err(x3, A1, W1, A2, W2, b, addend, relu)
    print(f"f16x2 {e:.2e}  x3 {e3:.2e}")
    assert e <= BOUND


def test_dropout_mask_equals_x3():
    torch.manual_seed(3)
    A = torch.randn(6000, 1024, device=DEV)
    W = torch.randn(1024, 1024, device=DEV) * 0.03
    b = torch.randn(1024, device=DEV) * 0.1
    y16 = F.fc_forward(A, W, None, None, b, True, 0.1, 77, arith="f16x2", row_offset=123)
    y3 = F.fc_forward(A, W, None, None, b, True, 0.1, 77, arith="x3", row_offset=123)
    # the same keep mask wherever the pre-dropout value is clearly positive
    clear = y3.abs() > 1e-3
    assert torch.equal((y16 != 0) & clear, (y3 != 0) & clear)
    assert float(((y16 - y3).abs() / (y3.abs() + 1)).max()) < 1e-5


def test_heads_and_input_grad_f16x2():
    torch.manual_seed(5)
    M, N = 5000, 1024
    A = torch.randn(M, N, device=DEV)
    W = torch.randn(N, N, device=DEV) * 0.03
    b = torch.randn(N, device=DEV) * 0.1
    Wh = torch.randn(3, N, device=DEV) * 0.05
    bh = torch.randn(3, device=DEV)
    C16, L16 = F.fc_forward(A, W, None, None, b, True, heads=(Wh, bh), arith="f16x2")
    C3, L3 = F.fc_forward(A, W, None, None, b, True, heads=(Wh, bh), arith="x3")
    assert float((C16 - C3).abs().max()) <= 1e-5 * float(C3.abs().max())
    assert float((L16 - L3).abs().max()) <= 1e-5 * float(L3.abs().max())
    # input gradient G W (+ G2 W2), gradient-like rows spread over e^(4 N(0,1))
    G = torch.randn(M, N, device=DEV) * torch.exp(4 * torch.randn(M, 1, device=DEV))
    g16 = F.input_grad(G, W, arith="f16x2")
    ref = G.double() @ W.double()
    den = G.double().abs() @ W.double().abs()
    assert float(((g16.double() - ref).abs() / (den + 1e-30)).max()) <= BOUND
    # every row relative to itself (a per-tensor scale would lose the small rows entirely)
    rel_row = ((g16.double() - ref).norm(dim=1) / ref.norm(dim=1)).max()
    assert float(rel_row) <= 1e-6


def test_conv1_fold_f16x2_equals_x3():
    torch.manual_seed(9)
    M, N, k = 6000, 1024, 8
    G = torch.randn(M, N, device=DEV) * 1e-3
    W = torch.randn(N, N, device=DEV) * 0.03
    Y = torch.relu(torch.randn(M, N, device=DEV))
    X1 = torch.randn(M, k, device=DEV)
    X2 = torch.randn(M, k, device=DEV)
    r16 = F.input_grad_relu_wgrad(G, W, None, None, None, Y, X1, X2, arith="f16x2")
    r3 = F.input_grad_relu_wgrad(G, W, None, None, None, Y, X1, X2, arith="x3")
    assert r16 is not None and r3 is not None
    for a, b in zip(r16, r3):
        assert float((a - b).abs().max()) <= 1e-5 * float(b.abs().max())


def test_model_step_f16x2_close_to_x3():
    from lpgnn import GCN_FC, BipartiteBatch, BipartiteCSR, synth
    from lpgnn.options import DEFAULT
    from lpgnn.train import balanced

    g = synth.uniform_lp(3000, 6000, 60000, seed=2)
    t = lambda a: torch.from_numpy(a).to(DEV)  # noqa: E731
    batch = BipartiteBatch(x_s=t(g.x_s), x_t=t(g.x_t), y_s=t(g.y_s), y_t=t(g.y_t),
                           edge_index=BipartiteCSR.from_coo(g.row, g.col, g.val, g.m, g.n, device=DEV),
                           s_bs=g.m, t_bs=g.n, bs=g.m + g.n)
    out = {}
    for arith in ("x3", "f16x2"):
        torch.manual_seed(0)
        model = GCN_FC(8, 8, hids=256, depth=3, dp=0.0, options=DEFAULT.replace(arith=arith)).to(DEV)
        lc, lv = model(batch)
        loss = balanced(lc, lv, batch.y_s, batch.y_t)
        loss.backward()
        out[arith] = (float(loss.detach()), [p.grad.clone() for p in model.parameters()], lc.detach(), lv.detach())
    assert abs(out["x3"][0] - out["f16x2"][0]) <= 1e-5 * abs(out["x3"][0])
    for a, b in zip(out["x3"][1], out["f16x2"][1]):
        assert float((a - b).norm()) <= 1e-4 * float(b.norm()) + 1e-12
    # the normalised logits (add_knowledge's 10 / |h| amplifies the heads' difference): the north star's 1e-4
    for a, b in zip(out["x3"][2:], out["f16x2"][2:]):
        d = float((a - b).abs().max())
        print(f"max |logit_x3 - logit_f16x2| = {d:.2e}")
        assert d <= 1e-4


def test_forward_under_inference_mode_equals_no_grad():
    """A GCN_FC forward under torch.inference_mode() with the f16x2 default: its tensors carry no autograd
    version counter, so the scale cache computes their scales per use instead of keying on the version
     -- the same logits, bit for bit, as under torch.no_grad(), in eval and in train mode
    (dropout keyed the same way)."""
    from lpgnn import GCN_FC, BipartiteBatch, BipartiteCSR, synth
    from lpgnn.options import DEFAULT

    g = synth.uniform_lp(3000, 6000, 60000, seed=4)
    t = lambda a: torch.from_numpy(a).to(DEV)  # noqa: E731
    batch = BipartiteBatch(x_s=t(g.x_s), x_t=t(g.x_t), y_s=t(g.y_s), y_t=t(g.y_t),
                           edge_index=BipartiteCSR.from_coo(g.row, g.col, g.val, g.m, g.n, device=DEV),
                           s_bs=g.m, t_bs=g.n, bs=g.m + g.n)
    torch.manual_seed(0)
    model = GCN_FC(8, 8, hids=256, depth=3, options=DEFAULT.replace(arith="f16x2")).to(DEV)
    for train in (False, True):
        model.train(train)
        with torch.no_grad():
            torch.manual_seed(1)
            ref = model(batch)
        with torch.inference_mode():
            torch.manual_seed(1)
            got = model(batch)
            assert got[0].is_inference()
            got2 = model(batch) if not train else got  # twice: nothing stale was cached
        for a, b in zip(ref, got):
            assert torch.equal(a, b)
        for a, b in zip(ref, got2):
            assert torch.equal(a, b)


@pytest.mark.parametrize("R,N,K", [(100_000, 1024, 1024), (20_000, 256, 384), (1000, 64, 16 * 8)])
def test_wgrad_f16x2_against_fp64(R, N, K):
    torch.manual_seed(R)
    G = torch.randn(R, N, device=DEV) * torch.exp(4 * torch.randn(1, N, device=DEV))  # column scales spread
    X = torch.relu(torch.randn(R, K, device=DEV)) * torch.exp(torch.randn(1, K, device=DEV))
    sG = F.colscale(G)
    mx = G.abs().amax(0) * sG
    assert bool(((mx >= 2 ** 14) & (mx < 2 ** 15)).all())
    dW = F.wgrad(G, X, arith="f16x2")
    ref = G.double().t() @ X.double()
    den = G.double().abs().t() @ X.double().abs()
    e = float(((dW.double() - ref).abs() / (den + 1e-30)).max())
    e3 = float(((F.wgrad(G, X, arith="x3").double() - ref).abs() / (den + 1e-30)).max())
    # every output row (a column of G) relative to itself, beside an fp32 GEMM's (hipBLASLt through torch.mm)
    rowrel = lambda d: float(((d.double() - ref).norm(dim=1) / ref.norm(dim=1)).max())  # noqa: E731
    rel, rel32 = rowrel(dW), rowrel(G.t() @ X)
    print(f"wgrad f16x2 {e:.2e}  x3 {e3:.2e}; worst row relative: f16x2 {rel:.2e}  fp32 GEMM {rel32:.2e}")
    assert e <= BOUND
    # one R range per CU (wgrad_splits) makes each fp32 accumulation chain R / (S * 32) chunks long: measured
    # 1.3e-6 at R = 100 K, a third of the fp32 GEMM's 4.1e-6 (profiles/r06_wgrad_split_ab.log)
    assert rel <= 2e-6 and rel <= rel32


@pytest.mark.parametrize("M,N,relu,bias", [(100_000, 1024, True, True), (777, 256, True, False), (5, 1000, False, True),
                                           (3001, 1024, False, False)])
def test_smallk_scales_from_the_stores(M, N, relu, bias):
    """conv1's narrow FC with arith f16x2 (lpg_fc_smallk_scales_f32): C bitwise the plain small-K kernel's,
    and the row / column scales it caches for C exactly the sweep's."""
    torch.manual_seed(M + N)
    A1 = torch.randn(M, 8, device=DEV) * torch.exp(2 * torch.randn(M, 1, device=DEV))
    A2 = torch.randn(M, 8, device=DEV)
    W1 = torch.randn(N, 8, device=DEV)
    W2 = torch.randn(N, 8, device=DEV)
    b = torch.randn(N, device=DEV) if bias else None
    C = F.fc_forward(A1, W1, A2, W2, b, relu, arith="f16x2")
    C0 = F.fc_forward(A1, W1, A2, W2, b, relu, arith="fp32")
    assert torch.equal(C, C0)
    rs, cs = F._SCALES.lookup("row", C), F._SCALES.lookup("col", C)
    assert rs is not None and cs is not None
    assert torch.equal(rs, F._rowscale1(C))
    assert torch.equal(cs, F._colscale1(C))


@pytest.mark.parametrize("M,K", [(100_000, 1024), (5000, 2048), (130, 64), (1, 1024)])
def test_heads_scales_from_the_stores(M, K):
    """The heads' backward with arith f16x2 (lpg_heads_relu_bwd_scales_f32): dZ, dW, db, dbY bitwise the
    plain entry's, and dZ's cached row / column scales exactly the sweep's."""
    torch.manual_seed(M + K)
    Y = torch.relu(torch.randn(M, K, device=DEV))
    G = torch.randn(M, 3, device=DEV) * torch.exp(3 * torch.randn(M, 1, device=DEV))
    W = torch.randn(3, K, device=DEV)
    r16 = F.heads_relu_bwd(G, W, Y, 1.25, True, arith="f16x2")
    r0 = F.heads_relu_bwd(G, W, Y, 1.25, True)
    for a, b in zip(r16, r0):
        assert torch.equal(a, b)
    dZ = r16[0]
    rs, cs = F._SCALES.lookup("row", dZ), F._SCALES.lookup("col", dZ)
    assert rs is not None and cs is not None
    assert torch.equal(rs, F._rowscale1(dZ))
    assert torch.equal(cs, F._colscale1(dZ))
