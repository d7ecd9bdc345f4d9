"""fp32 FC on the bf16 matrix cores (lpg_fc_x3_f32, lpg_split3_f32): exact
split, fp32-GEMM accuracy against fp64 beside the exact-fp32 kernel, and the
epilogue (bias, ReLU, accumulate, fused dropout) semantics."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"

# Error bound of the three-way split (csrc/fc_x3.hip): every dropped term is
# <= 2^-23 |a b| and the fp32 accumulation of K products rounds like an fp32
# GEMM; we require |y - y64| <= 16 * 2^-24 * sum_k |a_k b_k| + 2^-24 |y64|
# (observed maxima are ~3x below this at K = 2048; an exact-fp32 sequential
# chain is bounded by K * 2^-24 * sum|ab|, 128x looser).
U = 2.0 ** -24


def _bf16_bits_to_f64(t):
    return (t.to(torch.int32) & 0xFFFF).bitwise_left_shift(16).view(torch.float32).double()


@pytest.mark.parametrize("transpose", [False, True])
def test_split3_is_exact(transpose):
    from lpgnn.fc import split3

    g = torch.Generator().manual_seed(0)
    x = torch.randn(67, 45, generator=g) * torch.logspace(-20, 20, 45)
    x[0, :5] = torch.tensor([0.0, -0.0, 1.0, -3.0e38, 1.1754944e-38])
    x[1, :3] = torch.tensor([float(np.float32(1 + 2 ** -23)), 2 ** -126, float(np.nextafter(np.float32(1), 2))])
    s = split3(x.to(DEV), transpose=transpose).cpu()
    want = (x.t() if transpose else x).double()
    R, C = want.shape
    assert s.shape[0] == 3 and s.shape[1] == R and s.shape[2] >= C
    parts = [_bf16_bits_to_f64(s[p, :, :C]) for p in range(3)]
    assert torch.equal(parts[0] + parts[1] + parts[2], want)
    # term sizes: |t1| <= 2^-8 |x|, |t2| <= 2^-16 |x|
    assert (parts[1].abs() <= want.abs() * 2 ** -8).all()
    assert (parts[2].abs() <= want.abs() * 2 ** -16).all()
    # padded columns are zero terms
    if s.shape[2] > C:
        assert (s[:, :, C:] == 0).all()


def _ref64(A1, W1, A2, W2, b, relu):
    y = A1.double() @ W1.double().t()
    s = A1.double().abs() @ W1.double().abs().t()
    if A2 is not None:
        y += A2.double() @ W2.double().t()
        s += A2.double().abs() @ W2.double().abs().t()
    if b is not None:
        y += b.double()
    if relu:
        y = y.relu()
    return y, s


@pytest.mark.parametrize("M,N,K1,K2,relu,bias", [
    (1000, 1024, 1024, 1024, True, True),  # hidden layer
    (4096, 1024, 1024, 0, False, False),   # re-associated lin_rel GEMM / input gradient
    (129, 130, 64, 32, False, True),       # ragged tiles
    (257, 96, 2048, 0, True, True),
    (1, 33, 32, 32, True, True),
    (300, 200, 96, 0, False, True),
])
def test_x3_accuracy_vs_fp64(M, N, K1, K2, relu, bias):
    from lpgnn.fc import fc_forward

    g = torch.Generator().manual_seed(M + 3 * N)
    A1 = torch.randn(M, K1, generator=g)
    W1 = torch.randn(N, K1, generator=g) * 0.05
    A2 = torch.randn(M, K2, generator=g) if K2 else None
    W2 = torch.randn(N, K2, generator=g) * 0.05 if K2 else None
    b = torch.randn(N, generator=g) if bias else None
    t = lambda x: None if x is None else x.to(DEV)
    y = fc_forward(t(A1), t(W1), t(A2), t(W2), t(b), relu, arith="x3").cpu().double()
    y32 = fc_forward(t(A1), t(W1), t(A2), t(W2), t(b), relu, arith="fp32").cpu().double()
    ref, s = _ref64(A1, W1, A2, W2, b, relu)
    bound = 16 * U * s + U * ref.abs() + 1e-30
    err = (y - ref).abs()
    assert (err <= bound).all(), f"max err/bound {(err / bound).max().item():.3f}"
    # and in the same error class as the exact-fp32 kernel (blocked fma chains)
    e32 = (y32 - ref).abs()
    assert err.mean().item() <= 4 * e32.mean().item() + 1e-12


def test_x3_kernels_identical_when_strides_differ():
    """lda1 != lda2: the default falls back to fc_fwd_x3_16 (the wide kernel needs one offset set
    for both k phases) -- the same bits as choosing it explicitly (LPG_FC_KERNEL(1))."""
    from lpgnn.fc import fc_forward

    g = torch.Generator().manual_seed(5)
    A1, A2 = torch.randn(700, 256, generator=g).to(DEV), torch.randn(700, 128, generator=g).to(DEV)
    W1, W2 = torch.randn(300, 256, generator=g).to(DEV), torch.randn(300, 128, generator=g).to(DEV)
    b = torch.randn(300, generator=g).to(DEV)
    outs = [fc_forward(A1, W1, A2, W2, b, True, arith="x3", kernel=k) for k in (0, 1)]
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("M,N,K1,K2,accum,drop", [
    (700, 300, 128, 128, False, 0.0),   # ragged M and N tiles, both k phases
    (37, 1024, 256, 0, True, 0.0),      # fewer rows than one tile, accumulate
    (5000, 1024, 1024, 1024, False, 0.1),
    (1000, 1024, 256, 0, True, 0.1),    # interior tiles (the unchecked epilogue), accumulate + dropout
    (1, 130, 64, 64, False, 0.0),
])
def test_x3_wide_variants_bitwise(M, N, K1, K2, accum, drop):
    """fc_x3_wide (the default): buffer_load ... lds staging and wide wave strips, the same MFMA
    shape, k order and product sequence per output as fc_fwd_x3_16 (LPG_FC_KERNEL(1)) and as itself in
    round 3's tile order (LPG_FC_KERNEL(2)) -- bitwise the same C, incl. ragged edges (clamped rows/columns), dropout and the accumulate flag's addend."""
    from lpgnn.fc import fc_forward

    g = torch.Generator().manual_seed(M + N + K1)
    A1 = torch.randn(M, K1, generator=g).to(DEV)
    A2 = torch.randn(M, K2, generator=g).to(DEV) if K2 else None
    W1 = (torch.randn(N, K1, generator=g) * 0.05).to(DEV)
    W2 = (torch.randn(N, K2, generator=g) * 0.05).to(DEV) if K2 else None
    b = torch.randn(N, generator=g).to(DEV)
    P = torch.randn(M, N, generator=g).to(DEV) if accum else None
    outs = [fc_forward(A1, W1, A2, W2, b, True, drop, 5, out=None if P is None else P.clone(), accumulate=accum,
                       arith="x3", kernel=k) for k in (1, 0, 2, 3)]
    assert torch.equal(outs[0], outs[1])
    assert torch.equal(outs[0], outs[2])  # choice 2: the default kernel in round 3's tile order
    assert torch.equal(outs[0], outs[3])  # choice 3: the n-quarter order


@pytest.mark.parametrize("M,N,K,hn,accum,drop", [
    (1000, 1024, 1024, 3, False, 0.0),  # the last hidden layer + lin_left / lin_right
    (333, 200, 96, 3, True, 0.0),       # ragged 128-column tiles, accumulate (re-associated direction)
    (37, 130, 64, 1, False, 0.2),       # one head, dropout
    (1000, 1024, 256, 3, True, 0.1),    # interior tiles: accumulate + dropout + heads (the c2 root FC)
    (5000, 1024, 2048, 4, False, 0.0),
])
def test_x3_fused_heads_match_separate_linear(M, N, K, hn, accum, drop):
    """lpg_fc_x3_heads_f32: C is bitwise the unfused kernel's; the logits are the Linear on C to fp32
    rounding (bound: 32 * 2^-24 * sum|y w| + 2^-24 |logit|)."""
    from lpgnn.fc import fc_forward

    g = torch.Generator().manual_seed(M + N)
    A = torch.randn(M, K, generator=g).to(DEV)
    W = (torch.randn(N, K, generator=g) * 0.05).to(DEV)
    b = torch.randn(N, generator=g).to(DEV)
    Wh = (torch.randn(hn, N, generator=g) * 0.1).to(DEV)
    bh = torch.randn(hn, generator=g).to(DEV)
    P = torch.randn(M, N, generator=g).to(DEV) if accum else None
    y0 = fc_forward(A, W, None, None, b, True, drop, 77, out=None if P is None else P.clone(), accumulate=accum,
                    arith="x3")
    y, lg = fc_forward(A, W, None, None, b, True, drop, 77, out=None if P is None else P.clone(), accumulate=accum,
                       arith="x3", heads=(Wh, bh))
    assert torch.equal(y, y0)
    assert lg.shape == (M, hn)
    ref = y0.double() @ Wh.double().t() + bh.double()
    s = y0.double().abs() @ Wh.double().abs().t()
    err = (lg.double() - ref).abs()
    bound = 32 * U * s + U * ref.abs() + 1e-30
    assert (err <= bound).all(), f"max err/bound {(err / bound).max().item():.3f}"
    torch.testing.assert_close(lg, fc_forward(y0, Wh, None, None, bh, False), rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("kernel", [0, 1])
@pytest.mark.parametrize("M", [1000, 997])
def test_x3_fused_heads_under_every_kernel(kernel, M):
    """The fused-heads C equals lpg_fc_x3_f32's C under either kernel (one MFMA shape, one k
    order: bitwise), and the two kernels' logits agree bitwise too (the wide kernel reads its
    outputs back from an LDS image in the order the other accumulates them in registers)."""
    from lpgnn.fc import fc_forward

    g = torch.Generator().manual_seed(M)
    N, K = 1024, 256
    A = torch.relu(torch.randn(M, K, generator=g)).to(DEV)
    W = (torch.randn(N, K, generator=g) * 0.05).to(DEV)
    b = torch.randn(N, generator=g).to(DEV)
    Wh = (torch.randn(3, N, generator=g) * 0.1).to(DEV)
    bh = torch.randn(3, generator=g).to(DEV)
    y0 = fc_forward(A, W, None, None, b, True, arith="x3", kernel=kernel)
    y, lg = fc_forward(A, W, None, None, b, True, arith="x3", heads=(Wh, bh), kernel=kernel)
    assert torch.equal(y, y0)
    torch.testing.assert_close(lg, fc_forward(y0, Wh, None, None, bh, False), rtol=1e-5, atol=1e-5)
    _, lg_other = fc_forward(A, W, None, None, b, True, arith="x3", heads=(Wh, bh), kernel=1 - kernel)
    assert torch.equal(lg, lg_other)


@pytest.mark.parametrize("relu", [False, True])
def test_x3_accumulate(relu):
    """flags bit 1: C = act(A W^T + C + b), the addend read before the store."""
    from lpgnn.fc import fc_forward

    g = torch.Generator().manual_seed(9)
    M, N, K = 333, 160, 96
    A = torch.randn(M, K, generator=g).to(DEV)
    W = torch.randn(N, K, generator=g).to(DEV) * 0.1
    P = torch.randn(M, N, generator=g).to(DEV)
    b = torch.randn(N, generator=g).to(DEV)
    plain = fc_forward(A, W, None, None, None, False, arith="x3")
    C = P.clone()
    got = fc_forward(A, W, None, None, b, relu, out=C, accumulate=True, arith="x3")
    assert got.data_ptr() == C.data_ptr()
    want = plain + P + b
    if relu:
        want = want.relu()
    assert torch.equal(got, want)


def test_x3_dropout_mask_matches_fp32_kernel():
    """Same counter-based mask as the exact kernel (the backward relies on
    kept <=> output > 0 for every FC variant)."""
    from lpgnn.fc import fc_forward

    g = torch.Generator().manual_seed(11)
    M, N, K = 513, 256, 64
    A = torch.randn(M, K, generator=g).to(DEV)
    W = torch.randn(N, K, generator=g).to(DEV) * 0.2
    b = torch.full((N,), 5.0, device=DEV)  # every pre-dropout value > 0
    y3 = fc_forward(A, W, None, None, b, True, 0.3, 1234, arith="x3")
    y32 = fc_forward(A, W, None, None, b, True, 0.3, 1234, arith="fp32")
    assert torch.equal(y3 == 0, y32 == 0)
    kept = (y3 != 0).float().mean().item()
    assert 0.66 < kept < 0.74
    torch.testing.assert_close(y3, y32, rtol=1e-5, atol=1e-5)


def test_x3_rejects_bad_shapes():
    from lpgnn import _lib

    L = _lib.lib()
    a = torch.zeros(4, 40, device=DEV)
    w = torch.zeros(3, 4, 40, dtype=torch.int16, device=DEV)
    c = torch.zeros(4, 4, device=DEV)
    st = L.lpg_fc_x3_f32(4, 4, 40, a.data_ptr(), 40, w.data_ptr(), 40, 160, 0, None, 0, None, 0, 0, None,
                         c.data_ptr(), 4, 0, 0.0, 0, 0, None, None)
    assert st != 0 and b"multiples of 32" in L.lpg_last_error()


@pytest.mark.parametrize("R,N,K", [
    (4096, 1024, 1024),   # hidden-layer weight gradient shape (fewer rows)
    (1000, 256, 128),     # R not a multiple of the 32-row chunk
    (37, 132, 260),       # ragged output tiles, a single partial chunk
    (0, 64, 64),          # no rows: zeros
    (70000, 128, 64),     # many R splits
    (20, 64, 64),         # one partial chunk per split (T = 1)
    (3000, 128, 128),     # T = 9 (odd: the last chunk in the first plane buffer), shorter last split
    (1000, 300, 200),     # N, K not multiples of the 256 x 128 tile
])
def test_wgrad_x3_accuracy_vs_fp64(R, N, K):
    from lpgnn.fc import wgrad

    g = torch.Generator().manual_seed(R + N)
    G = torch.randn(R, N, generator=g)
    X = torch.randn(R, K, generator=g).relu()
    got = wgrad(G.to(DEV), X.to(DEV), arith="x3").cpu().double()
    ref = G.double().t() @ X.double()
    s = G.double().abs().t() @ X.double().abs()
    bound = 16 * U * s + U * ref.abs() + 1e-30
    err = (got - ref).abs()
    assert (err <= bound).all(), f"max err/bound {(err / bound).max().item():.3f}"
    again = wgrad(G.to(DEV), X.to(DEV), arith="x3").cpu().double()
    assert torch.equal(got, again)  # fixed-order split reduction: run-to-run identical


def test_wgrad_x3_strided_inputs():
    from lpgnn.fc import wgrad

    g = torch.Generator().manual_seed(3)
    big = torch.randn(900, 300, generator=g).to(DEV)
    G, X = big[:, :64], big[:, 100:228]  # row stride 300 (a multiple of 4)
    got = wgrad(G, X, arith="x3")
    torch.testing.assert_close(got, G.t() @ X, rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("two", [False, True])
@pytest.mark.parametrize("accumulate", [False, True])
def test_input_grad_x3(two, accumulate):
    """dZ1 W1 [+ dZ2 W2] [+ out] with Linear weights [out, in] split transposed."""
    from lpgnn.fc import input_grad

    g = torch.Generator().manual_seed(17)
    M, F, H = 777, 256, 160
    G1, W1 = torch.randn(M, F, generator=g), torch.randn(F, H, generator=g) * 0.1
    G2, W2 = torch.randn(M, F, generator=g), torch.randn(F, H, generator=g) * 0.1
    P = torch.randn(M, H, generator=g)
    ref = G1.double() @ W1.double()
    s = G1.double().abs() @ W1.double().abs()
    if two:
        ref += G2.double() @ W2.double()
        s += G2.double().abs() @ W2.double().abs()
    if accumulate:
        ref += P.double()
        s += P.double().abs()
    out = P.to(DEV).clone() if accumulate else None
    got = input_grad(G1.to(DEV), W1.to(DEV), G2.to(DEV) if two else None, W2.to(DEV) if two else None,
                     out=out, accumulate=accumulate, arith="x3").cpu().double()
    bound = 16 * U * s + U * ref.abs() + 1e-30
    assert ((got - ref).abs() <= bound).all()


@pytest.mark.parametrize("M,N,K,k1,k2,two,addend", [
    (3000, 1024, 1024, 8, 8, True, False),   # c2 layer 2: T W_rel + dZ_root W_root, conv1 p = q = 8
    (2999, 1024, 1024, 8, 8, False, True),   # the other association: dZ_root W_root + S^T(dZ W_rel)
    (517, 256, 256, 8, 8, True, True),       # ragged rows, narrower layer
    (1000, 128, 64, 12, 0, False, False),    # no root input, k = 12
])
def test_input_grad_relu_wgrad_vs_fp64(M, N, K, k1, k2, two, addend):
    """lpg_fc_x3_relu_wgrad_f32: conv1's (dW_rel, dW_root, db) from the next layer's input-gradient
    GEMM without storing g = G1 W1 [+ G2 W2] [+ addend] -- against fp64 of the same formula and at
    most as far from it as the two-pass route (input_grad + relu_wgrad_smallk) plus a floor at fp32
    resolution of the tensor (the fold sums the R = M rows in a different order)."""
    from lpgnn.fc import input_grad, input_grad_relu_wgrad, relu_wgrad_smallk

    gen = torch.Generator(device=DEV).manual_seed(M + N)
    r = lambda *s: torch.randn(*s, device=DEV, generator=gen)
    G1, W1 = r(M, K) * 1e-3, r(K, N) / K ** 0.5
    G2, W2 = (r(M, K) * 1e-3, r(K, N) / K ** 0.5) if two else (None, None)
    add = r(M, N) * 1e-3 if addend else None
    Y = torch.relu(r(M, N))  # conv1's ReLU output: about half the entries are zero
    X1 = r(M, k1)
    X2 = r(M, k2) if k2 else None
    got = input_grad_relu_wgrad(G1, W1, G2, W2, add, Y, X1, X2)
    assert got is not None
    g64 = G1.double() @ W1.double()
    if two:
        g64 += G2.double() @ W2.double()
    if addend:
        g64 += add.double()
    dz = torch.where(Y > 0, g64, torch.zeros_like(g64))
    want = (dz.t() @ X1.double(), None if X2 is None else dz.t() @ X2.double(), dz.sum(0))
    g = input_grad(G1, W1, G2, W2) if two else input_grad(G1, W1)
    if addend:
        g = g + add
    two_pass = relu_wgrad_smallk(g, Y, 1.0, X1, X2, True)
    for name, a, b, w in zip(("dW_rel", "dW_root", "db"), got, two_pass, want):
        if w is None:
            assert a is None
            continue
        e_fold, e_two = (a.double() - w).abs().max().item(), (b.double() - w).abs().max().item()
        floor = 64 * U * w.abs().max().item()
        print(f"{name}: max|fold - fp64| = {e_fold:.3e}, max|two-pass - fp64| = {e_two:.3e}")
        assert e_fold <= 2 * e_two + floor, name


@pytest.mark.parametrize("hids,depth", [(1024, 3), (256, 4)])
def test_conv1_wgrad_fold_equals_separate_pass(hids, depth):
    """options.fold_conv1_wgrad: conv1's weight gradients out of layer 2's input-gradient GEMMs give
    the same loss and, within fp32 summation-order differences, the same gradients as the separate
    input-gradient + relu_wgrad_smallk passes (training dropout, same dropout seeds); the other
    parameters' gradients are bitwise unchanged."""
    from lpgnn import BipartiteBatch, BipartiteCSR, GCN_FC, synth
    from lpgnn.train import balanced

    g = synth.uniform_lp(1300, 2600, 26000, seed=11)
    adj = BipartiteCSR.from_coo(g.row, g.col, g.val, g.m, g.n, device=DEV)
    batch = BipartiteBatch(x_s=torch.from_numpy(g.x_s).to(DEV), x_t=torch.from_numpy(g.x_t).to(DEV),
                           y_s=torch.from_numpy(g.y_s).to(DEV), y_t=torch.from_numpy(g.y_t).to(DEV),
                           edge_index=adj, s_bs=g.m, t_bs=g.n)
    torch.manual_seed(0)
    model = GCN_FC(8, 8, hids=hids, depth=depth, dp=0.1).to(DEV).train()
    base = model.options.replace(arith="x3")
    out = {}
    for fold in (True, False):
        model.options = base.replace(fold_conv1_wgrad=fold)
        model.zero_grad()
        torch.manual_seed(77)
        lc, lv = model(batch)
        loss = balanced(lc, lv, batch.y_s, batch.y_t)
        loss.backward()
        out[fold] = (loss.item(), {k: p.grad.clone() for k, p in model.named_parameters()})
    assert out[True][0] == out[False][0]
    for k, v in out[True][1].items():
        w = out[False][1][k]
        if k.startswith("conv1."):
            torch.testing.assert_close(v, w, rtol=1e-4, atol=1e-4 * w.abs().max().item(), msg=k)
        else:
            assert torch.equal(v, w), k


def test_conv1_wgrad_fold_keeps_feature_gradients():
    """with x_s / x_t requiring grad (saliency use) the fold must not apply -- conv1's
    folded backward returns no input gradients.  The feature gradients and every parameter gradient
    equal the run with options.fold_conv1_wgrad off, bitwise."""
    from lpgnn import BipartiteBatch, BipartiteCSR, GCN_FC, synth
    from lpgnn.train import balanced

    g = synth.uniform_lp(700, 1400, 9100, seed=5)
    adj = BipartiteCSR.from_coo(g.row, g.col, g.val, g.m, g.n, device=DEV)
    torch.manual_seed(0)
    model = GCN_FC(8, 8, hids=256, depth=3, dp=0.0).to(DEV).train()
    base = model.options.replace(arith="x3")
    out = {}
    for fold in (True, False):
        model.options = base.replace(fold_conv1_wgrad=fold)
        model.zero_grad()
        x_s = torch.from_numpy(g.x_s).to(DEV).requires_grad_(True)
        x_t = torch.from_numpy(g.x_t).to(DEV).requires_grad_(True)
        batch = BipartiteBatch(x_s=x_s, x_t=x_t, y_s=torch.from_numpy(g.y_s).to(DEV),
                               y_t=torch.from_numpy(g.y_t).to(DEV), edge_index=adj, s_bs=g.m, t_bs=g.n)
        lc, lv = model(batch)
        balanced(lc, lv, batch.y_s, batch.y_t).backward()
        assert x_s.grad is not None and x_t.grad is not None and x_s.grad.abs().sum() > 0
        out[fold] = (x_s.grad.clone(), x_t.grad.clone(), {k: p.grad.clone() for k, p in model.named_parameters()})
    assert torch.equal(out[True][0], out[False][0]) and torch.equal(out[True][1], out[False][1])
    for k, v in out[True][2].items():
        assert torch.equal(v, out[False][2][k]), k
