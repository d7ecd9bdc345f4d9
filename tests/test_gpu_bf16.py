"""bf16 path (c5, BASELINE.json configs[4]): lpg_fc_bf16 against an fp32
GEMM of the same bf16-rounded operands, and the bf16 GCN_FC against the
fp32 model.  No bitwise contract: bf16 outputs are compared within one
bf16 rounding of the fp32-accumulated reference (rtol 2^-7)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
BF = torch.bfloat16


def _ref(A1, W1, A2, W2, b, relu):
    r = A1.float() @ W1.float().t()
    if A2 is not None:
        r = r + A2.float() @ W2.float().t()
    if b is not None:
        r = r + b
    return torch.relu(r) if relu else r


@pytest.mark.parametrize("M,N,K1,K2,relu,bias", [
    (1, 1, 64, 0, False, True),
    (300, 1024, 64, 64, True, True),
    (129, 130, 128, 0, False, False),     # ragged tiles
    (37, 3, 2048, 0, False, True),        # heads
    (200, 256, 8, 8, True, True),         # conv1: K padded to 64
    (1000, 2048, 2048, 2048, True, True), # c5 hidden layer shape
    (4099, 512, 192, 320, True, True),    # 256 x 256 tiles from here (M >= 4096)
    (9000, 1000, 1024, 64, False, True),
])
def test_fc_bf16_matches_fp32_gemm(M, N, K1, K2, relu, bias):
    from lpgnn.fc import fc_forward_bf16

    g = torch.Generator().manual_seed(M * 31 + N)
    mk = lambda *s, sc=1.0: (torch.randn(*s, generator=g) * sc).to(BF).to(DEV)
    A1, W1 = mk(M, K1), mk(N, K1, sc=0.05)
    A2, W2 = (mk(M, K2), mk(N, K2, sc=0.05)) if K2 else (None, None)
    b = (torch.randn(N, generator=g) * 0.1).to(DEV) if bias else None
    got = fc_forward_bf16(A1, W1, A2, W2, b, relu).float()
    ref = _ref(A1, W1, A2, W2, b, relu)
    torch.testing.assert_close(got, ref.to(BF).float(), rtol=2 ** -7, atol=2e-3)


# per-call kernel choices of lpg_fc_bf16 (LPG_FC_KERNEL, include/lpgnn.h): 1 = 128 x 128,
# 2 = 256 x 256, 3 = the pipelined transposed-fragment kernel (the default from 4096 rows)
KERNELS = (1, 2, 3, 4, 5, 6, 7)


def _f64_ulp_check(out, A, W, P, b, relu, A2=None, W2=None):
    """Every output within one bf16 ulp of the fp64 value of the same bf16 operands (one RNE
    rounding of an fp32-accumulated sum; a wrong register or a stale load is off by far more)."""
    ref = A.double() @ W.double().t()
    if A2 is not None:
        ref = ref + A2.double() @ W2.double().t()
    if P is not None:
        ref = ref + P.double()
    if b is not None:
        ref = ref + b.double()
    if relu:
        ref = ref.clamp_min(0)
    err = (out.double() - ref).abs()
    bound = ref.abs() * 2.0 ** -7 + 1e-5
    bad = (err > bound).nonzero()
    assert bad.shape[0] == 0, (f"{bad.shape[0]} outputs off by more than one bf16 ulp, first (row, col) "
                               f"{bad[:6].tolist()}, max err {err.max().item():.3g}")


@pytest.mark.parametrize("kernel", KERNELS)
@pytest.mark.parametrize("M,N,K,relu,bias", [
    (5000, 1024, 1024, True, True),  # re-associated left2right root part
    (129, 130, 64, False, True),     # N % 8 != 0: per-element epilogue, one k-tile
    (129, 136, 64, False, True),     # one k-tile, LDS-image epilogue
    (300, 130, 128, False, True),    # two k-tiles, several row tiles
    (4099, 264, 128, True, False),   # ragged 256 x 256 tiles
])
def test_fc_bf16_accumulate(M, N, K, relu, bias, kernel):
    """Accumulate flag: C = bf16(act(A W^T + C + b)) in place; every kernel gives the bits of the
    default choice AND each output is within one bf16 ulp of the fp64 result of the same bf16
    operands.  The second check is the one that caught a miscompiled spilling kernel (a 4-wave,
    256-accumulator tile whose spill code dropped the last dword of an accumulator tuple: rows
    4i + 3 of one 16-column fragment were off by O(1)); comparing kernels with each other alone
    cannot tell which one is wrong."""
    from lpgnn.fc import fc_forward_bf16

    g = torch.Generator().manual_seed(M + N + K)
    A = torch.randn(M, K, generator=g).to(BF).to(DEV)
    W = (torch.randn(N, K, generator=g) * 0.05).to(BF).to(DEV)
    P = torch.randn(M, N, generator=g).to(BF).to(DEV)
    b = (torch.randn(N, generator=g) * 0.1).to(DEV) if bias else None
    outs = []
    for k in (kernel, 0):
        out = P.clone()
        got = fc_forward_bf16(A, W, None, None, b, relu, out=out, accumulate=True, kernel=k)
        assert got.data_ptr() == out.data_ptr()
        outs.append(got)
    assert torch.equal(outs[0], outs[1])
    _f64_ulp_check(outs[0].cpu(), A.cpu(), W.cpu(), P.cpu(), None if b is None else b.cpu(), relu)


def test_fc_bf16_kernels_identical():
    """Every kernel runs the same per-output MFMA chain order: identical bits (ReLU + dropout,
    two k phases), each within one bf16 ulp of fp64."""
    from lpgnn.fc import fc_forward_bf16

    torch.manual_seed(1)
    A1, A2 = (torch.randn(5000, 256, device=DEV).to(BF) for _ in range(2))
    W1, W2 = ((torch.randn(384, 256, device=DEV) * 0.05).to(BF) for _ in range(2))
    b = torch.randn(384, device=DEV)
    outs = [fc_forward_bf16(A1, W1, A2, W2, b, True, 0.2, seed=9, kernel=k) for k in KERNELS]
    for o in outs:
        assert torch.equal(o, outs[0])
    outs = [fc_forward_bf16(A1, W1, A2, W2, b, True, kernel=k) for k in KERNELS]
    _f64_ulp_check(outs[0].cpu(), A1.cpu(), W1.cpu(), None, b.cpu(), True, A2.cpu(), W2.cpu())


def test_fc_bf16_tail_split_identical():
    """The default choice runs the partial last round of 256 x 256 tiles as a second launch on
    128 x 128 tiles (rows offset, dropout keys offset); with enough rows for a full round plus a small
    tail that path runs, and it gives the bits of the single pipelined launch (kernel 3): ReLU +
    dropout, accumulate, and the folded ReLU backward."""
    from lpgnn.fc import fc_forward_bf16

    cus = torch.cuda.get_device_properties(0).multi_processor_count
    N = 2048
    per_round = (cus // (N // 256)) * 256
    M = per_round + per_round // 3 + 77  # a full round + a third of one, ragged
    torch.manual_seed(4)
    A1 = torch.randn(M, 128, device=DEV).to(BF)
    W1 = (torch.randn(N, 128, device=DEV) * 0.05).to(BF)
    b = torch.randn(N, device=DEV)
    got = fc_forward_bf16(A1, W1, None, None, b, True, 0.2, seed=3, row_offset=11, kernel=0)
    want = fc_forward_bf16(A1, W1, None, None, b, True, 0.2, seed=3, row_offset=11, kernel=3)
    assert torch.equal(got, want)
    P = torch.randn(M, N, device=DEV).to(BF)
    got = fc_forward_bf16(A1, W1, None, None, b, True, 0.1, seed=5, out=P.clone(), accumulate=True, kernel=0)
    want = fc_forward_bf16(A1, W1, None, None, b, True, 0.1, seed=5, out=P.clone(), accumulate=True, kernel=3)
    assert torch.equal(got, want)
    Y = torch.relu(torch.randn(M, N, device=DEV)).to(BF)
    got = fc_forward_bf16(A1, W1, None, None, None, False, mask=(Y, 1.25), kernel=0)
    want = fc_forward_bf16(A1, W1, None, None, None, False, mask=(Y, 1.25), kernel=3)
    assert torch.equal(got, want)


@pytest.mark.parametrize("M,N,relu,drop,bias", [
    (5000, 1024, True, 0.1, True),    # interior tiles
    (4099, 1000, True, 0.3, False),   # ragged rows and columns
    (3000, 512, False, 0.0, True),    # linear (the lin_rel GEMM of the re-associated direction)
])
def test_fc_bf16_transposed_fragments_identical(M, N, relu, drop, bias):
    """The pipelined kernel issues the MFMA as W x A^T (transposed fragments, 8-byte accesses to
    the LDS image): the same bits as the untransposed 256 x 256 kernel, with accumulate and dropout."""
    from lpgnn.fc import fc_forward_bf16

    g = torch.Generator().manual_seed(M + N)
    A = torch.randn(M, 256, generator=g).to(BF).to(DEV)
    W = (torch.randn(N, 256, generator=g) * 0.05).to(BF).to(DEV)
    P = torch.randn(M, N, generator=g).to(BF).to(DEV)
    b = (torch.randn(N, generator=g) * 0.1).to(DEV) if bias else None
    outs = []
    for k in (2, 3):
        for acc in (False, True):
            outs.append(fc_forward_bf16(A, W, None, None, b, relu, drop, seed=3, out=P.clone() if acc else None,
                                        accumulate=acc, kernel=k))
    assert torch.equal(outs[0], outs[2]) and torch.equal(outs[1], outs[3])


def test_fc_bf16_asymmetric_identity():
    """A = I with an asymmetric W catches a transposed C/D or operand map."""
    from lpgnn.fc import fc_forward_bf16

    K = 128
    A = torch.eye(K, dtype=BF, device=DEV)
    W = (torch.arange(96 * K, dtype=torch.float32).view(96, K) % 61 - 30).to(BF).to(DEV)
    got = fc_forward_bf16(A, W, None, None, None, False)
    assert torch.equal(got, W.t().contiguous())


def test_fc_bf16_dropout_same_mask_as_fp32():
    """The bf16 and fp32 kernels share the mask function: identical kept sets."""
    from lpgnn.fc import fc_forward, fc_forward_bf16

    torch.manual_seed(0)
    M, N, K = 3000, 256, 64
    A = torch.rand(M, K, device=DEV).to(BF)
    W = torch.rand(N, K, device=DEV).to(BF)  # all outputs > 0 before dropout
    p = 0.25
    y16 = fc_forward_bf16(A, W, None, None, None, True, p, seed=4321)
    y32 = fc_forward(A.float(), W.float(), None, None, None, True, p, seed=4321)
    assert torch.equal(y16 > 0, y32 > 0)
    rate = 1.0 - (y16 > 0).float().mean().item()
    assert abs(rate - p) < 0.01


def test_gcn_fc_bf16_close_to_fp32_and_trains():
    from lpgnn import BipartiteBatch, BipartiteCSR, GCN_FC, synth
    from lpgnn.train import balanced

    g = synth.uniform_lp(3000, 5000, 30000, seed=2)
    adj = BipartiteCSR.from_coo(g.row, g.col, g.val, g.m, g.n, device=DEV)
    batch = BipartiteBatch(x_s=torch.from_numpy(g.x_s).to(DEV), x_t=torch.from_numpy(g.x_t).to(DEV),
                           y_s=torch.from_numpy(g.y_s).to(DEV), y_t=torch.from_numpy(g.y_t).to(DEV),
                           edge_index=adj, s_bs=g.m, t_bs=g.n)
    torch.manual_seed(0)
    m32 = GCN_FC(8, 8, hids=256, depth=4).to(DEV).eval()
    m16 = GCN_FC(8, 8, hids=256, depth=4, compute_dtype="bf16").to(DEV).eval()
    m16.load_state_dict(m32.state_dict())
    with torch.no_grad():
        l32, r32 = m32(batch)
        l16, r16 = m16(batch)
    assert l16.dtype == torch.float32 and torch.isfinite(l16).all() and torch.isfinite(r16).all()
    # knowledge-normalised logits live in [-20, 10]; bf16 activations move them by ~1e-2 typically
    # (more where a node's raw logit vector is near zero: normalize() amplifies it)
    d = torch.cat([l16 - l32, r16 - r32]).abs().flatten()
    assert d.mean().item() < 0.05 and torch.quantile(d, 0.99).item() < 0.25, (d.mean().item(), d.max().item())
    agree = (torch.cat([l16, r16]).argmax(1) == torch.cat([l32, r32]).argmax(1)).float().mean().item()
    assert agree > 0.97
    # one training step: finite fp32 grads close in direction to the fp32 model's
    m16.train(), m32.train()
    m16.dp = m32.dp = 0.0
    for m in (m16, m32):
        m.zero_grad()
        lc, lv = m(batch)
        balanced(lc, lv, batch.y_s, batch.y_t).backward()
    for (k, p16), (_, p32) in zip(m16.named_parameters(), m32.named_parameters()):
        assert p16.grad is not None and p16.grad.dtype == torch.float32 and torch.isfinite(p16.grad).all(), k
        cos = torch.nn.functional.cosine_similarity(p16.grad.flatten(), p32.grad.flatten(), dim=0).item()
        assert cos > 0.95, (k, cos)


@pytest.mark.parametrize("M,N", [(1, 8), (63, 16), (1000, 2048), (4099, 1032), (70000, 256)])
def test_relu_bwd_colsum_bf16(M, N):
    from lpgnn.fc import relu_bwd_colsum_bf16

    torch.manual_seed(M + N)
    g = torch.randn(M, N, device=DEV).to(BF)
    y = torch.relu(torch.randn(M, N, device=DEV)).to(BF)
    for scale in (1.0, 1.0 / 0.9):
        out, db = relu_bwd_colsum_bf16(g, y, scale, True)
        want = torch.where(y > 0, g * scale, torch.zeros((), dtype=BF, device=DEV))
        assert out.dtype == BF and torch.equal(out, want)
        ref = want.double().sum(0)
        chain = 64 + (M + 63) // 64
        assert bool(((db.double() - ref).abs() <= chain * 2.0 ** -24 * want.double().abs().sum(0) + 1e-30).all())


def _wgrad_bound(G, X):
    """fp32-accumulation bound for G^T X over R rows: the MFMA sums 32 products per
    instruction and the chain adds one instruction result per 32 rows, the fold one
    range partial per range -- (R / 32 + 64) * 2^-24 * sum |g x| covers every order."""
    R = G.shape[0]
    return (R / 32 + 128) * 2.0 ** -24 * (G.double().abs().t() @ X.double().abs())


@pytest.mark.parametrize("R,N,K", [
    (0, 64, 64),            # no rows: zeros
    (1, 8, 8),              # one row, narrow
    (100, 264, 136),        # ragged tiles, one R-range
    (4097, 256, 512),       # ragged last R-tile
    (70001, 1024, 1024),    # several R-ranges + fold
    (20000, 2048, 2048),    # c5 weight shape
])
def test_wgrad_bf16_vs_fp64(R, N, K):
    """lpg_wgrad_bf16 (fp32 accumulation of exact bf16 x bf16 products) against
    fp64 G^T X of the same bf16 operands; run-to-run identical."""
    from lpgnn.fc import wgrad_bf16

    g = torch.Generator().manual_seed(R + N + K)
    G = torch.randn(R, N, generator=g).to(BF)
    X = torch.relu(torch.randn(R, K, generator=g)).to(BF)
    Gd, Xd = G.to(DEV), X.to(DEV)
    outs = [wgrad_bf16(Gd, Xd) for _ in range(2)]
    assert outs[0].dtype == torch.float32 and outs[0].shape == (N, K)
    for o in outs[1:]:
        assert torch.equal(outs[0], o)
    ref = G.double().t() @ X.double()
    err = (outs[0].cpu().double() - ref).abs()
    assert bool((err <= _wgrad_bound(G, X) + 1e-30).all()), err.max().item()


def test_wgrad_bf16_asymmetric():
    """G = I (R = N) with an asymmetric X catches a transposed operand or D map:
    dW = X exactly (each output is one product)."""
    from lpgnn.fc import wgrad_bf16

    R = 272
    G = torch.eye(R, dtype=BF, device=DEV)
    X = (torch.arange(R * 264, dtype=torch.float32, device=DEV).view(R, 264) % 61 - 30).to(BF)
    assert torch.equal(wgrad_bf16(G, X), X.float())


def test_wgrad_bf16_strided_operands():
    """Column slices of wider tensors (leading dimension > N, K), as the layer's
    [agg | x_dst] halves would be."""
    from lpgnn.fc import wgrad_bf16

    torch.manual_seed(3)
    Gw = torch.randn(5000, 640, device=DEV).to(BF)
    Xw = torch.randn(5000, 776, device=DEV).to(BF)
    G, X = Gw[:, 128:512], Xw[:, 8:520]
    got = wgrad_bf16(G, X)
    ref = G.double().t() @ X.double()
    assert bool(((got.double() - ref).abs() <= _wgrad_bound(G, X) + 1e-30).all())


@pytest.mark.parametrize("M,N,Nout,two,acc", [
    (1000, 2048, 2048, False, False),
    (4099, 1024, 2048, True, False),   # the two-part form (T W_rel + dZ_root W_root)
    (5000, 1024, 1024, False, True),   # accumulated onto an SpMM result
    (300, 264, 136, True, True),
])
def test_input_grad_bf16(M, N, Nout, two, acc):
    """G1 W1 [+ G2 W2] [+ P] on lpg_fc_bf16 with the transposed weights, within one
    bf16 rounding of the fp32 product of the same bf16 operands."""
    from lpgnn.fc import input_grad_bf16

    g = torch.Generator().manual_seed(M + N)
    G1 = torch.randn(M, Nout, generator=g).to(BF).to(DEV)
    W1 = (torch.randn(Nout, N, generator=g) * 0.05).to(DEV)  # fp32 master weights
    G2 = torch.randn(M, Nout, generator=g).to(BF).to(DEV) if two else None
    W2 = (torch.randn(Nout, N, generator=g) * 0.05).to(DEV) if two else None
    P = torch.randn(M, N, generator=g).to(BF).to(DEV) if acc else None
    ref = G1.float() @ W1.to(BF).float()
    if two:
        ref = ref + G2.float() @ W2.to(BF).float()
    if acc:
        ref = ref + P.float()
    got = input_grad_bf16(G1, W1, G2, W2, out=P, accumulate=acc)
    assert got.dtype == BF and got.shape == (M, N)
    torch.testing.assert_close(got.float(), ref.to(BF).float(), rtol=2 ** -7, atol=2e-3)


@pytest.mark.parametrize("M,N,Nin,two,acc,kernel", [
    (1000, 2048, 2048, False, True, 0),    # 128 x 128 kernel (M < 4096), accumulate form
    (1000, 256, 512, True, False, 0),      # two-part form
    (5003, 2048, 2048, True, False, 0),    # pipelined kernel (transposed fragments, LDS image)
    (5003, 1024, 2048, False, True, 0),    # accumulate on the pipelined kernel, ragged last tile
    (5003, 1032, 512, False, True, 2),     # untransposed image epilogue, ragged columns
    (5003, 512, 512, True, False, 1),      # 128 x 128 kernel above 4096 rows
])
def test_fc_bf16_relu_bwd_folded_bitwise(M, N, Nin, two, acc, kernel):
    """lpg_fc_bf16_relu_bwd = input_grad_bf16 then relu_bwd_colsum_bf16 (the separate pass), bit
    for bit, for the accumulate and two-part forms the c5 backward uses; lpg_colsum_bf16 on the
    folded dZ = the separate pass's bias gradient, bit for bit."""
    from lpgnn import _lib
    from lpgnn.fc import colsum_bf16, input_grad_bf16, relu_bwd_colsum_bf16

    torch.manual_seed(M + N + kernel)
    G1 = torch.randn(M, N, device=DEV).to(BF)
    W1 = torch.randn(N, Nin, device=DEV) * 0.03  # Linear [out = N, in = Nin]: dX = G W
    G2 = torch.randn(M, N, device=DEV).to(BF) if two else None
    W2 = torch.randn(N, Nin, device=DEV) * 0.03 if two else None
    Y = torch.relu(torch.randn(M, Nin, device=DEV)).to(BF)
    add = torch.randn(M, Nin, device=DEV).to(BF) if acc else None
    for scale in (1.0, 1.0 / 0.9):
        ref = input_grad_bf16(G1, W1, G2, W2, out=None if add is None else add.clone(), accumulate=acc,
                              kernel=kernel)
        want, db_want = relu_bwd_colsum_bf16(ref, Y, scale, True)
        got = input_grad_bf16(G1, W1, G2, W2, out=None if add is None else add.clone(), accumulate=acc,
                              mask=(Y, scale), kernel=kernel)
        assert torch.equal(got, want)
        assert torch.equal(colsum_bf16(got), db_want)


def test_fc_bf16_relu_bwd_rejects_bias_and_bad_layouts():
    from lpgnn import _lib
    from lpgnn.fc import fc_forward_bf16, relu_bwd_colsum_bf16

    A = torch.randn(64, 128, device=DEV).to(BF)
    W = (torch.randn(24, 128, device=DEV) * 0.05).to(BF)
    Y = torch.relu(torch.randn(64, 24, device=DEV)).to(BF)
    with pytest.raises(RuntimeError):
        fc_forward_bf16(A, W, None, None, torch.zeros(24, device=DEV), False, mask=(Y, 1.0))
    # a column count the folded store does not take (N % 8 != 0 after the output view): two passes, same bits
    W20 = W[:20].contiguous()
    Y20 = Y[:, :20]
    got = fc_forward_bf16(A, W20, None, None, None, False, mask=(Y20, 1.25))
    want = relu_bwd_colsum_bf16(fc_forward_bf16(A, W20, None, None, None, False), Y20, 1.25, False)[0]
    assert torch.equal(got, want)
    L = _lib.lib()
    C = torch.empty(64, 24, dtype=BF, device=DEV)
    st = L.lpg_fc_bf16_relu_bwd(64, 24, 128, A.data_ptr(), 128, W.data_ptr(), 128, 0, None, 0, None, 0,
                                C.data_ptr(), 24, 1, Y.data_ptr(), 24, 1.0, None)  # ReLU flag: refused
    assert st != 0


def test_gcn_fc_bf16_folded_relu_bwd_identical(monkeypatch):
    """The c5 model's backward with each layer's ReLU/dropout backward folded into the next layer's
    input-gradient stores gives the same loss and the same gradient bits as the separate passes
    (training dropout, same dropout seeds)."""
    from lpgnn import BipartiteBatch, BipartiteCSR, GCN_FC, synth
    from lpgnn.train import balanced

    g = synth.uniform_lp(1500, 5200, 30000, seed=5)
    adj = BipartiteCSR.from_coo(g.row, g.col, g.val, g.m, g.n, device=DEV)
    batch = BipartiteBatch(x_s=torch.from_numpy(g.x_s).to(DEV), x_t=torch.from_numpy(g.x_t).to(DEV),
                           y_s=torch.from_numpy(g.y_s).to(DEV), y_t=torch.from_numpy(g.y_t).to(DEV),
                           edge_index=adj, s_bs=g.m, t_bs=g.n)
    torch.manual_seed(0)
    model = GCN_FC(8, 8, hids=256, depth=5, dp=0.1, compute_dtype="bf16").to(DEV).train()
    out = {}
    base = model.options
    for fold in (True, False, "bias"):
        # "bias": the folded ReLU backward with the bias gradients as their own column-sum passes
        model.options = base.replace(fold_relu_bwd=bool(fold), fold_bias_sums=fold is True)
        model.zero_grad()
        torch.manual_seed(321)  # same dropout seeds
        lc, lv = model(batch)
        loss = balanced(lc, lv, batch.y_s, batch.y_t)
        loss.backward()
        out[fold] = (loss.item(), {k: p.grad.clone() for k, p in model.named_parameters()})
    for alt in (False, "bias"):
        assert out[True][0] == out[alt][0]
        for k, v in out[True][1].items():
            assert torch.equal(v, out[alt][1][k]), (alt, k)


@pytest.mark.parametrize("R,C", [(8, 8), (2048, 2048), (72, 136), (1000, 8), (2048, 24)])
def test_transpose_bf16(R, C):
    from lpgnn.fc import transpose_bf16

    W = torch.randn(R, C, device=DEV).to(BF)
    assert torch.equal(transpose_bf16(W), W.t().contiguous())
    big = torch.randn(R, C + 16, device=DEV).to(BF)[:, 8:8 + C]  # strided source rows
    assert torch.equal(transpose_bf16(big), big.t().contiguous())


@pytest.mark.parametrize("M,N", [(1, 8), (7, 16), (63, 16), (65, 256), (1000, 2048), (4099, 1032), (70001, 256)])
def test_colsum_bf16_bitwise_masked_pass(M, N):
    """lpg_colsum_bf16 (read-only column sums, double-buffered rows) == the bias gradient of
    relu_bwd_colsum_bf16 with every element kept and scale 1 (the same blocks, row order and fold),
    incl. ragged last blocks."""
    from lpgnn.fc import colsum_bf16, relu_bwd_colsum_bf16

    torch.manual_seed(M * 7 + N)
    g = torch.randn(M, N, device=DEV).to(BF)
    y = torch.ones(M, N, device=DEV, dtype=BF)
    out, db = relu_bwd_colsum_bf16(g, y, 1.0, True)
    assert torch.equal(out, g)
    assert torch.equal(colsum_bf16(g), db)


def _packbits(y):
    """uint8 [M, N / 8]: bit e of byte t of row m = (y[m, 8 t + e] > 0) -- the lpg_fc_bf16_mask layout."""
    pos = (y.float() > 0).to(torch.uint8).reshape(y.shape[0], -1, 8)
    w = (2 ** torch.arange(8, device=y.device, dtype=torch.int32)).to(torch.uint8)
    return (pos * w).sum(-1, dtype=torch.int32).to(torch.uint8)


@pytest.mark.parametrize("kernel", [0, 1, 2, 3, 4, 5])
@pytest.mark.parametrize("M,N,K1,K2,acc,p", [
    (5000, 512, 128, 128, False, 0.2),   # two k phases, dropout
    (700, 256, 64, 0, True, 0.0),        # small M (128 x 128 kernel), accumulate
    (3000, 256, 8, 8, False, 0.1),       # conv1: the narrow-input kernel (nibbles paired across lanes)
    (19384, 2048, 64, 0, True, 0.1),     # two full rounds + 3000 rows (the tail launch of choice 0)
    (3000, 200, 64, 0, False, 0.1),      # N % 64 != 0: 25 mask bytes a row (byte stores at the edge, unaligned rows)
])
def test_fc_bf16_mask_out_is_the_relu_mask(kernel, M, N, K1, K2, acc, p):
    """lpg_fc_bf16_mask: C bit for bit lpg_fc_bf16's, and the mask is exactly (C > 0) packed 8 per byte."""
    from lpgnn.fc import fc_forward_bf16

    g = torch.Generator(device=DEV).manual_seed(M + N + kernel)
    r = lambda *s: (torch.randn(*s, device=DEV, generator=g) * 0.2).to(BF)  # noqa: E731
    A1, W1 = r(M, K1), r(N, K1)
    A2, W2 = (r(M, K2), r(N, K2)) if K2 else (None, None)
    b = torch.randn(N, device=DEV, generator=g) * 0.1
    P = r(M, N) if acc else None
    ref = fc_forward_bf16(A1, W1, A2, W2, b, True, p, 11, out=None if P is None else P.clone(), accumulate=acc,
                          kernel=kernel)
    bits = torch.full((M, N // 8), 0xA5, dtype=torch.uint8, device=DEV)
    got = fc_forward_bf16(A1, W1, A2, W2, b, True, p, 11, out=None if P is None else P.clone(), accumulate=acc,
                          kernel=kernel, mask_out=bits)
    assert torch.equal(got, ref)
    assert torch.equal(bits, _packbits(ref))


@pytest.mark.parametrize("two,acc", [(True, False), (False, True)])
def test_relu_bwd_bits_equal_relu_bwd_from_y(two, acc):
    """lpg_fc_bf16_relu_bwd_bits: the folded ReLU backward from the 1-bit mask gives the bits of the
    Y form (same product, same rounding per pair)."""
    from lpgnn.fc import input_grad_bf16

    M, N, K = 6000, 1024, 512
    g = torch.Generator(device=DEV).manual_seed(3)
    r = lambda *s: (torch.randn(*s, device=DEV, generator=g) * 0.2).to(BF)  # noqa: E731
    G1, W1 = r(M, K), r(K, N)
    G2, W2 = (r(M, K), r(K, N)) if two else (None, None)
    Y = torch.relu(r(M, N))
    Y[::7, ::5] = 0
    P = r(M, N) if acc else None
    want = input_grad_bf16(G1, W1, G2, W2, out=None if P is None else P.clone(), accumulate=acc, mask=(Y, 1.25))
    got = input_grad_bf16(G1, W1, G2, W2, out=None if P is None else P.clone(), accumulate=acc,
                          mask=(_packbits(Y), 1.25))
    assert torch.equal(got, want)


@pytest.mark.parametrize("kernel", [0, 1, 2, 3, 4, 5])
@pytest.mark.parametrize("M,N,bits,acc", [(19384, 2048, True, True),   # c5's two-part launch (tail: colsum pass)
                                          (4099, 1032, False, False),  # ragged last 64-row chunk, N tail tile
                                          (5000, 200, True, False),    # one partial n-tile
                                          (64, 256, False, True)])     # one chunk (the small-tile kernel)
def test_relu_bwd_db_equals_colsum(kernel, M, N, bits, acc):
    """lpg_fc_bf16_relu_bwd*_db: the bias column sums the pipelined kernel takes in its store loop (the
    colsum pass for rows and kernels it does not cover) are bitwise colsum_bf16 of the dZ it stores, and
    dZ is the plain folded call's."""
    from lpgnn.fc import colsum_bf16, input_grad_bf16

    K = 256
    g = torch.Generator(device=DEV).manual_seed(M + N + kernel)
    r = lambda *s: (torch.randn(*s, device=DEV, generator=g) * 0.2).to(BF)  # noqa: E731
    G1, W1 = r(M, K), r(K, N)
    Y = torch.relu(r(M, N))
    P = r(M, N) if acc else None
    mask = (_packbits(Y) if bits else Y, 1.25)
    want = input_grad_bf16(G1, W1, out=None if P is None else P.clone(), accumulate=acc, mask=mask, kernel=kernel)
    db = torch.full((N,), float("nan"), device=DEV)
    got = input_grad_bf16(G1, W1, out=None if P is None else P.clone(), accumulate=acc, mask=mask, kernel=kernel,
                          db_out=db)
    assert torch.equal(got, want)
    assert torch.equal(db, colsum_bf16(want))


def test_relu_bwd_db_empty_rows():
    from lpgnn.fc import input_grad_bf16

    G1, W1 = torch.zeros(0, 64, device=DEV, dtype=BF), torch.ones(64, 16, device=DEV, dtype=BF)
    db = torch.full((16,), 7.0, device=DEV)
    out = input_grad_bf16(G1, W1, mask=(torch.zeros(0, 16, device=DEV, dtype=BF), 1.0), db_out=db)
    assert out.shape == (0, 16) and bool((db == 0).all())


def test_gcn_fc_bf16_relu_bits_identical():
    """options.relu_bits: every bf16 ReLU layer writes its 1-bit mask and the next layer's folded ReLU
    backward reads it instead of the layer output -- the same loss and the same gradient bits."""
    from lpgnn import BipartiteBatch, BipartiteCSR, GCN_FC, synth
    from lpgnn.train import balanced

    g = synth.uniform_lp(1500, 5200, 30000, seed=5)
    adj = BipartiteCSR.from_coo(g.row, g.col, g.val, g.m, g.n, device=DEV)
    batch = BipartiteBatch(x_s=torch.from_numpy(g.x_s).to(DEV), x_t=torch.from_numpy(g.x_t).to(DEV),
                           y_s=torch.from_numpy(g.y_s).to(DEV), y_t=torch.from_numpy(g.y_t).to(DEV),
                           edge_index=adj, s_bs=g.m, t_bs=g.n)
    torch.manual_seed(0)
    model = GCN_FC(8, 8, hids=256, depth=5, dp=0.1, compute_dtype="bf16").to(DEV).train()
    base = model.options
    out = {}
    for bits in (True, False):
        model.options = base.replace(relu_bits=bits)
        model.zero_grad()
        torch.manual_seed(321)
        lc, lv = model(batch)
        loss = balanced(lc, lv, batch.y_s, batch.y_t)
        loss.backward()
        out[bits] = (loss.item(), {k: p.grad.clone() for k, p in model.named_parameters()})
    assert out[True][0] == out[False][0]
    for k, v in out[True][1].items():
        assert torch.equal(v, out[False][1][k]), k


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("M,N,K1,K2,relu,drop,acc", [
    (16384 + 77, 1024, 1024, 0, False, 0.0, False),   # fp16-inference shape family, ragged rows
    (20000, 1024, 512, 512, True, 0.2, False),         # two k phases, ReLU + dropout
    (30011, 2048, 256, 0, True, 0.0, True),            # accumulate addend, many boundaries
    (8192, 2048, 64, 64, False, 0.0, False),           # nk = 2: ranges of a few k-tiles, most tiles split
])
def test_fc16_stream_k_identical(dt, M, N, K1, K2, relu, drop, acc):
    """lpg_fc16's persistent stream-K form (fc_bf16_sk: the (tile, k-tile) iterations split into one
    range per CU, a tile cut by a range boundary carrying its fp32 accumulators from block to block
    through the workspace) gives exactly the bits of the one-tile-per-block pipelined kernel (choice 3)
    -- the same MFMA chain per output -- with dropout keyed the same, an addend, two k phases, ragged
    rows; and within one 16-bit ulp of fp64 of the same operands."""
    from lpgnn.fc import fc_forward_bf16

    cus = torch.cuda.get_device_properties(0).multi_processor_count
    assert ((M + 255) // 256) * ((N + 255) // 256) >= cus // 8 * 8  # the stream-K form applies
    g = torch.Generator(device=DEV).manual_seed(M + N)
    r = lambda *s: torch.randn(*s, device=DEV, generator=g)  # noqa: E731
    A1, W1 = r(M, K1).to(dt), (r(N, K1) * 0.05).to(dt)
    A2, W2 = (r(M, K2).to(dt), (r(N, K2) * 0.05).to(dt)) if K2 else (None, None)
    b = r(N) * 0.1
    P = r(M, N).to(dt) if acc else None
    outs = []
    for k in (6, 3, 0):  # (6 = the stream-K form, 3 = the one-tile pipelined kernel, 0 = default)
        out = P.clone() if acc else None
        outs.append(fc_forward_bf16(A1, W1, A2, W2, b, relu, drop, seed=77, out=out, accumulate=acc, kernel=k))
    assert torch.equal(outs[0], outs[1]), int((outs[0] != outs[1]).sum())
    assert torch.equal(outs[2], outs[1])
    if dt == torch.bfloat16 and drop == 0.0:
        _f64_ulp_check(outs[0].cpu(), A1.cpu(), W1.cpu(), None if P is None else P.cpu(), b.cpu(), relu,
                       None if A2 is None else A2.cpu(), None if W2 is None else W2.cpu())
