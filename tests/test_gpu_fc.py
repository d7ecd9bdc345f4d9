"""fp32 MFMA FC kernel and add_knowledge kernel: bitwise vs the oracle."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import model_ref as O

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(autouse=True)
def _exact_fp32(monkeypatch):
    """These tests pin the exact-fp32 kernel's bitwise contract (fc_ref.c);
    the default x3 arithmetic is tested in test_gpu_x3.py."""
    from lpgnn import fc

    monkeypatch.setattr(fc, "ARITH", "fp32")


@pytest.mark.parametrize("M,N,K1,K2,relu,bias", [
    (1, 1, 4, 0, False, True),
    (37, 3, 1024, 0, False, True),        # heads
    (300, 1024, 8, 8, True, True),        # conv1 (p = q = 8)
    (1000, 1024, 1024, 1024, True, True), # hidden layer
    (129, 130, 36, 20, False, False),     # ragged tiles, no bias
    (257, 64, 1024, 12, True, True),
    (64, 33, 0, 40, True, True),          # only the root part
    (1, 4, 4, 0, True, False),            # narrow-input (small-K) kernel ...
    (5001, 1028, 8, 8, True, True),       # ... ragged column chunk
    (333, 1024, 12, 4, False, True),
    (77, 64, 16, 0, True, True),
    (100, 30, 8, 8, True, True),          # N % 4 != 0: tiled MFMA path
])
def test_fc_bitwise(M, N, K1, K2, relu, bias):
    from lpgnn.fc import fc_forward

    rng = np.random.default_rng(M * 7 + N)
    A1 = rng.standard_normal((M, K1)).astype(np.float32)
    W1 = (rng.standard_normal((N, K1)) * 0.05).astype(np.float32)
    A2 = rng.standard_normal((M, K2)).astype(np.float32) if K2 else None
    W2 = (rng.standard_normal((N, K2)) * 0.05).astype(np.float32) if K2 else None
    b = rng.standard_normal(N).astype(np.float32) if bias else None
    t = lambda x: None if x is None else torch.from_numpy(x).to(DEV)
    if K1 == 0:  # only a root part: pass it as the first operand
        got = fc_forward(t(A2), t(W2), None, None, t(b), relu).cpu().numpy()
        ref = O.fc_kchain(A2, W2, bias=b, relu=relu)
    else:
        got = fc_forward(t(A1), t(W1), t(A2), t(W2), t(b), relu).cpu().numpy()
        ref = O.fc_kchain(A1, W1, A2, W2, b, relu=relu)
    assert np.array_equal(got, ref)
    # and the math is the expected one (catches a transposed C/D map)
    want = A1.astype(np.float64) @ W1.T.astype(np.float64) if K1 else 0
    if K2:
        want = want + A2.astype(np.float64) @ W2.T.astype(np.float64)
    if bias:
        want = want + b
    if relu:
        want = np.maximum(want, 0)
    np.testing.assert_allclose(got, want, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("M,N,K,relu,bias", [
    (1000, 1024, 1024, True, True),   # re-associated left2right root part
    (129, 130, 36, False, True),      # ragged tiles (clamped addend loads)
    (77, 64, 8, True, False),         # narrow-input kernel
    (37, 3, 64, False, True),         # head-shaped tile
])
def test_fc_accumulate_bitwise(M, N, K, relu, bias):
    """Accumulate flag: C = act(A W^T + C + b) in place, bitwise the oracle
    chain + P + bias, and equal to the non-accumulating product + P + b."""
    from lpgnn.fc import fc_forward

    rng = np.random.default_rng(M + N + K)
    A = rng.standard_normal((M, K)).astype(np.float32)
    W = (rng.standard_normal((N, K)) * 0.05).astype(np.float32)
    P = rng.standard_normal((M, N)).astype(np.float32)
    b = rng.standard_normal(N).astype(np.float32) if bias else None
    t = lambda x: None if x is None else torch.from_numpy(x).to(DEV)
    out = t(P).clone()
    got = fc_forward(t(A), t(W), None, None, t(b), relu, out=out, accumulate=True, arith="fp32")
    plain = fc_forward(t(A), t(W), None, None, None, False, arith="fp32")
    assert got.data_ptr() == out.data_ptr()
    got = got.cpu().numpy()
    assert np.array_equal(got, O.fc_kchain(A, W, bias=b, relu=relu, add=P))
    want = plain.cpu() + torch.from_numpy(P)
    if bias:
        want = want + torch.from_numpy(b)
    if relu:
        want = torch.relu(want)
    assert np.array_equal(got, want.numpy())


@pytest.mark.parametrize("p,bias,acc", [(0.0, True, False), (0.25, True, False), (0.0, False, False),
                                        (0.25, False, True), (0.0, True, True)])
def test_fc_smallk_equals_tiled_path(p, bias, acc):
    """The narrow-input kernel (K1 + K2 <= 16) and the MFMA tile kernel give
    the same bits, dropout mask included: zero-padding K1 to 20 moves the
    same chain onto the tiled path (fma(0, 0, p) = p).  Every epilogue form
    (bias or not, dropout or not, accumulate or not)."""
    from lpgnn.fc import fc_forward

    torch.manual_seed(5)
    M, N = 2050, 1024
    A1, A2 = torch.randn(M, 8, device=DEV), torch.randn(M, 8, device=DEV)
    W1, W2 = torch.randn(N, 8, device=DEV) * 0.3, torch.randn(N, 8, device=DEV) * 0.3
    b = torch.randn(N, device=DEV) * 0.1 if bias else None
    P = torch.randn(M, N, device=DEV)
    pad = lambda x: torch.cat([x, torch.zeros(x.shape[0], 12, device=DEV)], 1).contiguous()
    kw = dict(out=P.clone(), accumulate=True) if acc else {}
    small = fc_forward(A1, W1, A2, W2, b, True, p, seed=77, **kw)
    kw = dict(out=P.clone(), accumulate=True) if acc else {}
    tiled = fc_forward(pad(A1), pad(W1), A2, W2, b, True, p, seed=77, arith="fp32", **kw)
    assert torch.equal(small, tiled)


def test_fc_odd_k_is_padded_exactly():
    from lpgnn.fc import fc_forward

    rng = np.random.default_rng(0)
    A = rng.standard_normal((50, 7)).astype(np.float32)
    W = rng.standard_normal((20, 7)).astype(np.float32)
    got = fc_forward(torch.from_numpy(A).to(DEV), torch.from_numpy(W).to(DEV), None, None, None, False)
    assert np.array_equal(got.cpu().numpy(), O.fc_kchain(A, W))


def test_fc_identity_asymmetric():
    """A = I with an asymmetric W catches a row/col swap in the epilogue."""
    from lpgnn.fc import fc_forward

    K = 64
    A = torch.eye(K, device=DEV)
    W = torch.arange(K * 96, dtype=torch.float32, device=DEV).view(96, K) / 100.0
    got = fc_forward(A, W, None, None, None, False)
    assert torch.equal(got, W.t().contiguous())


def test_fc_autograd_matches_torch():
    from lpgnn.fc import graph_conv_fc

    torch.manual_seed(0)
    A1 = torch.randn(300, 64, device=DEV, requires_grad=True)
    A2 = torch.randn(300, 32, device=DEV, requires_grad=True)
    W1 = torch.randn(48, 64, device=DEV, requires_grad=True)
    W2 = torch.randn(48, 32, device=DEV, requires_grad=True)
    b = torch.randn(48, device=DEV, requires_grad=True)
    g = torch.randn(300, 48, device=DEV)
    y = graph_conv_fc(A1, A2, W1, b, W2, True)
    y.backward(g)
    got = [t.grad.clone() for t in (A1, A2, W1, W2, b)]
    for t in (A1, A2, W1, W2, b):
        t.grad = None
    y2 = torch.relu(F.linear(A1, W1, b) + F.linear(A2, W2))
    y2.backward(g)
    for a, t in zip(got, (A1, A2, W1, W2, b)):
        torch.testing.assert_close(a, t.grad, rtol=1e-4, atol=1e-4)


def test_knowledge_bitwise_vs_torch_cpu():
    from lpgnn.fc import knowledge

    rng = np.random.default_rng(3)
    M = 20000
    logit = (rng.standard_normal((M, 3)) * rng.uniform(0, 10, (M, 1))).astype(np.float32)
    logit[:5] = 0.0  # eps clamp path
    logit[5] = [1e-20, -1e-20, 3e-21]
    feas = np.zeros((M, 8), np.float32)
    feas[:, 5] = -(rng.random(M) < 0.5).astype(np.float32)
    feas[:, 7] = rng.random(M) < 0.5
    got = knowledge(torch.from_numpy(logit).to(DEV), torch.from_numpy(feas).to(DEV)).cpu()
    ref, _ = O.add_knowledge(torch.from_numpy(logit), torch.from_numpy(logit[:1]), torch.from_numpy(feas),
                             torch.from_numpy(feas[:1]))
    assert torch.equal(got, ref)


def test_knowledge_backward_matches_torch():
    from lpgnn.fc import knowledge

    torch.manual_seed(1)
    x = torch.randn(500, 3, device=DEV) * 3
    x[0] = 0
    x.requires_grad_(True)
    feas = torch.zeros(500, 8, device=DEV)
    g = torch.randn(500, 3, device=DEV)
    knowledge(x, feas).backward(g)
    got = x.grad.clone()
    x.grad = None
    (F.normalize(x) * 10).backward(g)
    torch.testing.assert_close(got, x.grad, rtol=1e-5, atol=1e-5)


def test_fc_tiles_bitwise():
    """Ragged tiles, both k phases, padded K: the exact-fp32 kernel gives the oracle's bits."""
    from lpgnn.fc import fc_forward

    rng = np.random.default_rng(0)
    t = lambda x: torch.from_numpy(x).to(DEV)
    for M, N, K1, K2 in ((777, 300, 96, 40), (777, 300, 96, 64), (1000, 1024, 256, 256)):
        A1, A2 = rng.standard_normal((M, K1)).astype(np.float32), rng.standard_normal((M, K2)).astype(np.float32)
        W1, W2 = rng.standard_normal((N, K1)).astype(np.float32), rng.standard_normal((N, K2)).astype(np.float32)
        b = rng.standard_normal(N).astype(np.float32)
        got = fc_forward(t(A1), t(W1), t(A2), t(W2), t(b), True, arith="fp32").cpu().numpy()
        assert np.array_equal(got, O.fc_kchain(A1, W1, A2, W2, b, relu=True)), (M, N, K1, K2)


def test_fused_dropout_epilogue_and_backward():
    """Dropout fused after the ReLU: kept values are exactly relu(v)/(1-p),
    the drop rate is p, the mask is reproducible from the seed, and the
    backward equals torch autograd through the realised mask."""
    from lpgnn.fc import fc_forward, graph_conv_fc
    from oracle.dropout_ref import scale as keep_scale

    torch.manual_seed(3)
    M, N, K = 4000, 256, 64
    A1 = torch.randn(M, K, device=DEV)
    A2 = torch.randn(M, K, device=DEV)
    W1 = torch.randn(N, K, device=DEV) * 0.1
    W2 = torch.randn(N, K, device=DEV) * 0.1
    b = torch.randn(N, device=DEV) * 0.1
    p = 0.1
    base = fc_forward(A1, W1, A2, W2, b, True)
    y = fc_forward(A1, W1, A2, W2, b, True, p, seed=1234)
    assert torch.equal(y, fc_forward(A1, W1, A2, W2, b, True, p, seed=1234))
    assert not torch.equal(y, fc_forward(A1, W1, A2, W2, b, True, p, seed=99))
    pos = base > 0
    kept = (y > 0)
    assert bool((kept <= pos).all())
    rate = 1.0 - kept[pos].float().mean().item()
    assert abs(rate - p) < 0.01, rate
    scale = torch.tensor(keep_scale(p), dtype=torch.float32)
    assert torch.equal(y[kept], base[kept] * scale.to(DEV))
    # backward through the fused op == torch through the realised mask
    A1r, A2r = A1.clone().requires_grad_(True), A2.clone().requires_grad_(True)
    W1r, W2r, br = (t.clone().requires_grad_(True) for t in (W1, W2, b))
    torch.manual_seed(7)
    out = graph_conv_fc(A1r, A2r, W1r, br, W2r, True, dropout=p)
    g = torch.randn_like(out)
    out.backward(g)
    mask = (out > 0).float() * keep_scale(p)
    A1t, A2t = A1.clone().requires_grad_(True), A2.clone().requires_grad_(True)
    W1t, W2t, bt = (t.clone().requires_grad_(True) for t in (W1, W2, b))
    ref = torch.relu(torch.nn.functional.linear(A1t, W1t, bt) + torch.nn.functional.linear(A2t, W2t)) * mask
    ref.backward(g)
    for a, t in ((A1r, A1t), (A2r, A2t), (W1r, W1t), (W2r, W2t), (br, bt)):
        torch.testing.assert_close(a.grad, t.grad, rtol=1e-4, atol=1e-4)


def test_relu_dropout_bwd_kernel():
    from lpgnn.fc import relu_dropout_bwd

    g = torch.randn(1000, 36, device=DEV)
    y = torch.relu(torch.randn(1000, 36, device=DEV))
    out = relu_dropout_bwd(g, y, 1.25)
    assert torch.equal(out, torch.where(y > 0, g * 1.25, torch.zeros((), device=DEV)))


@pytest.mark.parametrize("M,K,N", [(1, 4, 3), (1000, 1024, 3), (1537, 260, 2), (70000, 1024, 3)])
def test_linear_small_bwd_matches_torch(M, K, N):
    from lpgnn.fc import linear

    torch.manual_seed(M)
    x = torch.randn(M, K, device=DEV, requires_grad=True)
    W = torch.randn(N, K, device=DEV, requires_grad=True)
    b = torch.randn(N, device=DEV, requires_grad=True)
    g = torch.randn(M, N, device=DEV)
    linear(x, W, b).backward(g)
    got = [t.grad.clone() for t in (x, W, b)]
    for t in (x, W, b):
        t.grad = None
    torch.nn.functional.linear(x, W, b).backward(g)
    # fp32 sums over M rows in a different order than torch's: check both against
    # fp64 with the recursive-summation bound |err| <= L * 2^-24 * sum|terms|,
    # L = the longest add chain (rows per block + number of blocks)
    xd, Wd, gd = x.detach().double(), W.detach().double(), g.double()
    ref = (gd @ Wd, gd.t() @ xd, gd.sum(0))
    mag = (gd.abs() @ Wd.abs(), gd.abs().t() @ xd.abs(), gd.abs().sum(0))
    chain = 128 + (M + 127) // 128 + N
    for a, t, r, s in zip(got, (x.grad, W.grad, b.grad), ref, mag):
        err = (a.double() - r).abs()
        assert bool((err <= chain * 2.0 ** -24 * s + 1e-30).all()), (err.max().item(), (t.double() - r).abs().max().item())


@pytest.mark.parametrize("M,N", [(1, 4), (63, 8), (1000, 1024), (4099, 1028), (70000, 256)])
def test_relu_bwd_colsum(M, N):
    from lpgnn.fc import relu_bwd_colsum

    torch.manual_seed(M + N)
    g = torch.randn(M, N, device=DEV)
    y = torch.relu(torch.randn(M, N, device=DEV))
    out, db = relu_bwd_colsum(g, y, 1.25, True)
    want = torch.where(y > 0, g * 1.25, torch.zeros((), device=DEV))
    assert torch.equal(out, want)
    # block-ordered deterministic sum: matches fp64 within the recursive-summation bound
    chain = 64 + (M + 63) // 64
    err = (db.double() - want.double().sum(0)).abs()
    assert bool((err <= chain * 2.0 ** -24 * want.double().abs().sum(0) + 1e-30).all())
    out2, db2 = relu_bwd_colsum(g, y, 1.25, True)
    assert torch.equal(db, db2)  # run-to-run deterministic
    out3, none = relu_bwd_colsum(g, y, 1.25, False)
    assert none is None and torch.equal(out3, want)


@pytest.mark.parametrize("M,N,K1,K2", [(1, 4, 8, 8), (1000, 1024, 8, 8), (5000, 260, 3, 0), (70001, 1024, 8, 8),
                                       (300, 64, 1, 15)])
def test_wgrad_smallk(M, N, K1, K2):
    from lpgnn.fc import wgrad_smallk

    torch.manual_seed(M)
    dz = torch.randn(M, N, device=DEV)
    A1 = torch.randn(M, K1, device=DEV)
    A2 = torch.randn(M, K2, device=DEV) if K2 else None
    dW1, dW2 = wgrad_smallk(dz, A1, A2)
    chain = 256 + (M + 255) // 256
    for dW, A in ((dW1, A1), (dW2, A2)):
        if A is None:
            assert dW is None
            continue
        r = dz.double().t() @ A.double()
        s = dz.double().abs().t() @ A.double().abs()
        err = (dW.double() - r).abs()
        assert dW.shape == (N, A.shape[1]) and bool((err <= chain * 2.0 ** -24 * s + 1e-30).all())


@pytest.mark.parametrize("M,N,K1,K2,scale", [(1, 4, 8, 8, 1.0), (1000, 1024, 8, 8, 1.0), (70001, 1024, 8, 8, 1.25),
                                             (300, 64, 3, 0, 1.0)])
def test_relu_wgrad_smallk_equals_unfused(M, N, K1, K2, scale):
    """conv1's fused backward == mask -> wgrad_smallk / colsum (same products, same bound vs fp64)."""
    from lpgnn.fc import relu_wgrad_smallk

    torch.manual_seed(M + N)
    g = torch.randn(M, N, device=DEV)
    y = torch.relu(torch.randn(M, N, device=DEV))
    A1 = torch.randn(M, K1, device=DEV)
    A2 = torch.randn(M, K2, device=DEV) if K2 else None
    dW1, dW2, db = relu_wgrad_smallk(g, y, scale, A1, A2, True)
    dz = torch.where(y > 0, g * scale, torch.zeros((), device=DEV)).double()
    chain = 256 + (M + 255) // 256
    for dW, A in ((dW1, A1), (dW2, A2)):
        if A is None:
            assert dW is None
            continue
        r = dz.t() @ A.double()
        bound = chain * 2.0 ** -24 * (dz.abs().t() @ A.double().abs())
        assert bool(((dW.double() - r).abs() <= bound + 1e-30).all())
    assert bool(((db.double() - dz.sum(0)).abs() <= chain * 2.0 ** -24 * dz.abs().sum(0) + 1e-30).all())


@pytest.mark.parametrize("M,K,N,scale", [(1000, 1024, 3, 1.0), (777, 256, 3, 1.0 / 0.9), (5, 64, 2, 2.0)])
def test_heads_relu_bwd_matches_unfused(M, K, N, scale):
    """lpg_heads_relu_bwd_f32 == linear backward then ReLU/dropout backward + bias column sums."""
    from lpgnn.fc import heads_relu_bwd

    g = torch.Generator().manual_seed(M)
    Y = torch.randn(M, K, generator=g).relu_().to(DEV)  # a ReLU output (zeros = dropped or inactive)
    G = torch.randn(M, N, generator=g).to(DEV)
    W = torch.randn(N, K, generator=g).to(DEV)
    dZ, dW, db, dbY = heads_relu_bwd(G, W, Y, scale, True)
    dH = G.double() @ W.double()
    want_dz = torch.where(Y > 0, dH * scale, torch.zeros_like(dH))
    torch.testing.assert_close(dZ.double(), want_dz, rtol=1e-5, atol=1e-5)
    assert torch.equal(dZ == 0, Y == 0) or bool(((dZ == 0) | (Y > 0)).all())
    torch.testing.assert_close(dW.double(), G.double().t() @ Y.double(), rtol=1e-5, atol=1e-3)
    torch.testing.assert_close(db.double(), G.double().sum(0), rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(dbY.double(), want_dz.sum(0), rtol=1e-5, atol=1e-3)
