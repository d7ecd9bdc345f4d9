"""The c5 (bf16) model's narrow kernels, through the C ABI:

* conv1's forward on the streaming small-K kernel (lpg_fc_bf16 with 4 <= K1, K1 + K2 <= 16, no
  padding) against the MFMA kernel on the zero-padded operands and against fp64;
* conv1's weight / bias gradients (lpg_relu_wgrad_smallk_bf16) against fp64, the on-the-fly ReLU /
  dropout backward bitwise the separate relu_bwd_colsum_bf16 pass;
* the heads' forward (lpg_linear_small_fwd_bf16) and backward (lpg_heads_bwd_bf16) against fp64,
  the folded dZ bitwise the separate pass over the plain dH, dbY bitwise lpg_colsum_bf16.

No CPU restatement of these sums exists bit for bit (the MFMA kernels they replace sum in the
hardware's order): bf16 outputs within one bf16 rounding of the fp64 value of the same bf16
operands, fp32 sums within the recursive-summation bound."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
BF = torch.bfloat16


def _gen(seed):
    return torch.Generator().manual_seed(seed)


def _mk(g, *s, sc=1.0):
    return (torch.randn(*s, generator=g) * sc).to(BF).to(DEV)


def _within_bf16_ulp(got, ref64, what):
    err = (got.double() - ref64).abs()
    bound = ref64.abs() * 2.0 ** -8 + 1e-6  # one RNE rounding (half an ulp) + fp32 summation slack
    bad = (err > bound).nonzero()
    assert bad.shape[0] == 0, f"{what}: {bad.shape[0]} outputs off, first {bad[:5].tolist()}, max {err.max().item():.3g}"


def _sum_bound(terms_abs_sum, n):
    return n * 2.0 ** -24 * terms_abs_sum + 1e-30


@pytest.mark.parametrize("M,N,K1,K2", [(1, 4, 8, 8), (200, 2048, 8, 8), (1001, 1028, 4, 0), (4097, 256, 12, 4),
                                       (65, 8, 16, 0), (300, 2052, 4, 12)])
@pytest.mark.parametrize("relu,bias,drop,acc", [(True, True, 0.0, False), (False, False, 0.0, False),
                                                (True, True, 0.1, False), (True, True, 0.0, True)])
def test_fc_smallk_bf16(M, N, K1, K2, relu, bias, drop, acc):
    from lpgnn.fc import fc_forward_bf16

    g = _gen(M * 7 + N + K1)
    A1, W1 = _mk(g, M, K1), _mk(g, N, K1, sc=0.3)
    A2, W2 = (_mk(g, M, K2), _mk(g, N, K2, sc=0.3)) if K2 else (None, None)
    b = (torch.randn(N, generator=g) * 0.1).to(DEV) if bias else None
    P = _mk(g, M, N) if acc else None
    seed = 1234567
    out = P.clone() if acc else None
    got = fc_forward_bf16(A1, W1, A2, W2, b, relu, drop, seed, out=out, accumulate=acc)
    # the MFMA kernel on the same operands zero-padded to 64 (the pre-round-3 conv1 path)
    pad = lambda t: None if t is None else torch.nn.functional.pad(t, (0, 64 - t.shape[1]))
    outp = P.clone() if acc else None
    want = fc_forward_bf16(pad(A1), pad(W1), pad(A2), pad(W2), b, relu, drop, seed, out=outp, accumulate=acc)
    assert ((got == 0) == (want == 0)).float().mean().item() > 0.999  # ReLU / dropout masks agree
    diff = (got.float() - want.float()).abs()
    assert bool((diff <= want.float().abs() * 2.0 ** -7 + 1e-6).all())  # at most one bf16 ulp apart
    ref = A1.double() @ W1.double().t()
    if K2:
        ref = ref + A2.double() @ W2.double().t()
    if acc:
        ref = ref + P.double()
    if bias:
        ref = ref + b.double()
    if relu:
        ref = ref.clamp_min(0)
    if drop:
        keep = want != 0  # the MFMA kernel's mask (same hash) where it kept a nonzero value
        ref = torch.where(keep, ref / (1 - drop), torch.zeros((), dtype=ref.dtype, device=DEV))
        got = torch.where(keep, got, torch.zeros((), dtype=got.dtype, device=DEV))
    _within_bf16_ulp(got.float(), ref, "fc_smallk_bf16")


def test_fc_smallk_bf16_row_offset_mask():
    """The dropout mask is keyed on (row_offset + row, col), as in every FC kernel."""
    from lpgnn.fc import fc_forward_bf16

    g = _gen(3)
    A1, W1, A2, W2 = _mk(g, 300, 8), _mk(g, 256, 8), _mk(g, 300, 8), _mk(g, 256, 8)
    full = fc_forward_bf16(A1, W1, A2, W2, None, True, 0.3, 99)
    part = fc_forward_bf16(A1[100:], W1, A2[100:], W2, None, True, 0.3, 99, row_offset=100)
    assert torch.equal(full[100:], part)


@pytest.mark.parametrize("M,N,K1,K2", [(1, 4, 8, 8), (1000, 2048, 8, 8), (257, 1028, 4, 0), (513, 64, 12, 4)])
@pytest.mark.parametrize("scale", [1.0, 1.0 / 0.9])
def test_relu_wgrad_smallk_bf16(M, N, K1, K2, scale):
    from lpgnn.fc import relu_bwd_colsum_bf16, relu_wgrad_smallk_bf16

    g = _gen(M + N)
    G = _mk(g, M, N)
    Y = torch.relu(_mk(g, M, N))
    A1 = _mk(g, M, K1)
    A2 = _mk(g, M, K2) if K2 else None
    dW1, dW2, db = relu_wgrad_smallk_bf16(G, Y, scale, A1, A2, True)
    dz, db_sep = relu_bwd_colsum_bf16(G, Y, scale, True)
    # from dZ directly (the folded form): the same dZ bits, so the same sums
    e1, e2, edb = relu_wgrad_smallk_bf16(dz, None, 1.0, A1, A2, True)
    assert torch.equal(dW1, e1) and torch.equal(db, edb) and (K2 == 0 or torch.equal(dW2, e2))
    Z = dz.double()
    for got, X in ((dW1, A1), (dW2, A2)):
        if X is None:
            continue
        ref = Z.t() @ X.double()
        bound = _sum_bound(Z.abs().t() @ X.double().abs(), 256 + 64)
        assert bool(((got.double() - ref).abs() <= bound).all())
    ref_db = Z.sum(0)
    assert bool(((db.double() - ref_db).abs() <= _sum_bound(Z.abs().sum(0), 256 + 64)).all())
    assert bool(((db_sep.double() - ref_db).abs() <= _sum_bound(Z.abs().sum(0), 256 + 64)).all())


@pytest.mark.parametrize("M,K,N", [(1, 8, 3), (5, 2048, 3), (1001, 2048, 3), (333, 264, 4), (4096, 1000, 1),
                                   (70000, 2048, 3)])
def test_linear_small_fwd_bf16(M, K, N):
    from lpgnn.fc import fc_forward_bf16, linear_small_fwd_bf16

    g = _gen(M + K + N)
    H = torch.relu(_mk(g, M, K))
    W = torch.randn(N, K, generator=g).to(DEV) * 0.05
    b = torch.randn(N, generator=g).to(DEV)
    got = linear_small_fwd_bf16(H, W, b)
    Wb = W.to(BF)
    ref = H.double() @ Wb.double().t() + b.double()
    _within_bf16_ulp(got.float(), ref, "linear_small_fwd_bf16")
    # against the MFMA kernel it replaced (the same bf16 operands; N padded inside lpg_fc_bf16): both
    # are RNE_bf16 of an fp32 sum of the same exact products in different orders, so
    #   |got - want| <= |s1 - s2| + 2^-8 max(|s1|, |s2|),  |s1 - s2| <= 2 (K + 1) 2^-24 (|H| |Wb|^T + |b|)
    # (the recursive-summation bound of each order against the exact sum)
    want = fc_forward_bf16(H, Wb, None, None, b, False).float()
    terms = H.double().abs() @ Wb.double().abs().t() + b.double().abs()
    s_gap = 2 * (K + 1) * 2.0 ** -24 * terms
    bound = s_gap + 2.0 ** -8 * (want.double().abs() + s_gap)
    assert bool(((got.double() - want.double()).abs() <= bound).all())
    assert torch.equal(linear_small_fwd_bf16(H, W, b), got)  # run to run
    # strided rows (a view inside a wider tensor)
    wide = torch.zeros(M, K + 16, dtype=BF, device=DEV)
    wide[:, 8:8 + K] = H
    assert torch.equal(linear_small_fwd_bf16(wide[:, 8:8 + K], W, b), got)


@pytest.mark.parametrize("M,K,N", [(1, 8, 3), (63, 2048, 3), (1000, 2048, 3), (129, 264, 4), (5000, 1000, 2)])
@pytest.mark.parametrize("scale", [1.0, 1.0 / 0.9])
def test_heads_bwd_bf16(M, K, N, scale):
    from lpgnn.fc import colsum_bf16, heads_bwd_bf16, relu_bwd_colsum_bf16

    g = _gen(M * 3 + K)
    G = _mk(g, M, N)  # the bf16 logits' gradient
    W = torch.randn(N, K, generator=g).to(DEV) * 0.05
    Y = torch.relu(_mk(g, M, K))
    dH, dW, db, _ = heads_bwd_bf16(G, W, Y, None, False)
    dZ, dW2, db2, dbY = heads_bwd_bf16(G, W, Y, scale, True)
    # the folded form: bitwise the separate ReLU/dropout pass over the plain dH, and its column sums
    sep, sep_db = relu_bwd_colsum_bf16(dH, Y, scale, True)
    assert torch.equal(dZ, sep) and torch.equal(dbY, sep_db) and torch.equal(dbY, colsum_bf16(dZ))
    assert torch.equal(dW, dW2) and torch.equal(db, db2)
    Wb = W.to(BF).double()
    Gd = G.double()
    _within_bf16_ulp(dH.float(), Gd @ Wb, "heads dH")
    ref_dw = Gd.t() @ Y.double()
    assert bool(((dW.double() - ref_dw).abs() <= _sum_bound(Gd.abs().t() @ Y.double().abs(), 128 + 64)).all())
    assert bool(((db.double() - Gd.sum(0)).abs() <= _sum_bound(Gd.abs().sum(0), 128 + 64)).all())
    # run to run
    again = heads_bwd_bf16(G, W, Y, scale, True)
    assert all(torch.equal(a, b) for a, b in zip(again, (dZ, dW2, db2, dbY)))


def test_bf16_model_uses_narrow_kernels():
    """The c5 model's conv1 and heads run the streaming kernels (TIMER keys), and one training step
    is finite."""
    from lpgnn import BipartiteBatch, BipartiteCSR, GCN_FC, synth
    from lpgnn.timing import TIMER
    from lpgnn.train import balanced

    gr = synth.uniform_lp(700, 1500, 7000, seed=2)
    adj = BipartiteCSR.from_coo(gr.row, gr.col, gr.val, gr.m, gr.n, device=DEV)
    batch = BipartiteBatch(x_s=torch.from_numpy(gr.x_s).to(DEV), x_t=torch.from_numpy(gr.x_t).to(DEV),
                           y_s=torch.from_numpy(gr.y_s).to(DEV), y_t=torch.from_numpy(gr.y_t).to(DEV),
                           edge_index=adj, s_bs=gr.m, t_bs=gr.n)
    torch.manual_seed(0)
    model = GCN_FC(8, 8, hids=256, depth=3, compute_dtype="bf16").to(DEV).train()
    TIMER.reset()
    TIMER.enabled = True
    try:
        lc, lv = model(batch)
        loss = balanced(lc, lv, batch.y_s, batch.y_t)
        loss.backward()
        torch.cuda.synchronize()
        keys = {k[0] for k in TIMER.summary()}
    finally:
        TIMER.enabled = False
    assert {"heads_fwd", "heads_bwd", "wgrad_smallk"} <= keys, keys
    assert torch.isfinite(loss).item()
    for k, p in model.named_parameters():
        assert p.grad is not None and bool(torch.isfinite(p.grad).all()), k


def test_bf16_heads_colsum_handoff_is_used():
    """The bf16 heads' backward hands the last hidden layer its bias column sums (computed in the
    same pass); the layer takes them only for the very gradient tensor the heads returned (identity
    check, conv.py) -- in a plain model step that is always the case, so no separate colsum pass
    runs for it (a replaced gradient would fall back to lpg_colsum_bf16, the same bits)."""
    from lpgnn import BipartiteBatch, BipartiteCSR, GCN_FC, fc, synth
    from lpgnn.train import balanced

    gr = synth.uniform_lp(700, 1500, 7000, seed=4)
    adj = BipartiteCSR.from_coo(gr.row, gr.col, gr.val, gr.m, gr.n, device=DEV)
    batch = BipartiteBatch(x_s=torch.from_numpy(gr.x_s).to(DEV), x_t=torch.from_numpy(gr.x_t).to(DEV),
                           y_s=torch.from_numpy(gr.y_s).to(DEV), y_t=torch.from_numpy(gr.y_t).to(DEV),
                           edge_index=adj, s_bs=gr.m, t_bs=gr.n)
    torch.manual_seed(0)
    model = GCN_FC(8, 8, hids=256, depth=3, compute_dtype="bf16").to(DEV).train()
    calls = []
    orig = fc.colsum_bf16
    fc.colsum_bf16 = lambda g: calls.append(g.shape) or orig(g)
    try:
        lc, lv = model(batch)
        balanced(lc, lv, batch.y_s, batch.y_t).backward()
        torch.cuda.synchronize()
    finally:
        fc.colsum_bf16 = orig
    assert calls == [], calls
