"""The reference's --fp16 inference mode (val.py:269 ``model.half()``, utils.py:909-915
``batch_to(half=True)``, scripts/pred_basis.py:146, 170) on the fp16 kernels, through the C ABI:

* SpMM with fp16 storage (lpg_spmm_f16): BITWISE the oracle's sequential fp32 loop over the fp16
  values, rounded once to fp16 (oracle.model_ref.spmm_f16), every kernel form;
* the FC on v_mfma_f32_16x16x32_f16 (lpg_fc_f16): within one fp16 rounding of the fp64 value of
  the same fp16 operands; every kernel choice bitwise equal; the narrow conv1 kernel likewise;
* the heads (lpg_linear_small_fwd_f16), add_knowledge in half precision (lpg_knowledge_f16) and
  the basis labels on fp16 logits (lpg_basis_labels_f16) against the oracle's restatements;
* the whole model after model.half() against the oracle's fp16-storage evaluation
  (gcn_fc_forward_fp16) on a mid-size graph.  The full c2 size is in test_gpu_c2_parity.py."""
import numpy as np
import pytest
import torch

from oracle import model_ref as O

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
H = torch.float16
ULP16 = 2.0 ** -11  # fp16 unit roundoff (RNE: half an ulp relative)


def _gen(seed):
    return torch.Generator().manual_seed(seed)


@pytest.mark.parametrize("F", [1, 8, 16, 40, 64, 256, 1000, 1024, 2048])
def test_spmm_f16_bitwise_vs_oracle(F):
    from lpgnn import BipartiteCSR, synth
    from lpgnn.sparse import spmm_forward

    g = synth.uniform_lp(2000, 3000, 20000, seed=F)
    adj = BipartiteCSR.from_coo(g.row, g.col, g.val, g.m, g.n, device=DEV).half()
    A = O.csr_from_coo(g.row, g.col, g.val, g.m, g.n)
    AT = O.csr_transpose(*A, g.m, g.n)
    for csr, rows_src in ((A, g.n), (AT, g.m)):
        X = (torch.randn(rows_src, F, generator=_gen(F)) * 3).half()
        orient = adj.fwd if csr is A else adj.bwd
        got = spmm_forward(orient, X.to(DEV)).cpu()
        assert got.dtype == H
        ref = O.spmm_f16(*csr, X)
        assert torch.equal(got.float(), ref), (F, (got.float() - ref).abs().max())


def test_spmm_f16_skewed_heavy_rows_bitwise():
    """Skewed rows with three above the heavy-row threshold (1024 edges: the split path), the rest
    Zipf-like short rows: the fp16-storage oracle's bits."""
    from lpgnn import BipartiteCSR
    from lpgnn import sparse as S
    from lpgnn.sparse import spmm_forward

    rng = np.random.default_rng(3)
    m, n = 3000, 4000
    deg = np.minimum(rng.zipf(1.5, m), 200)
    deg[[5, 1500, 2999]] = [3000, 1500, 1100]
    assert int(deg.max()) > S.DEFAULT_HEAVY  # heavy rows take the split path
    row = np.repeat(np.arange(m), deg)
    col = np.concatenate([rng.choice(n, d, replace=False) for d in deg]).astype(np.int64)
    val = rng.uniform(-1, 1, len(row)).astype(np.float32)
    adj = BipartiteCSR.from_coo(row, col, val, m, n, device=DEV).half()
    A = O.csr_from_coo(row, col, val, m, n)
    X = torch.randn(n, 1024, generator=_gen(5)).half()
    got = spmm_forward(adj.fwd, X.to(DEV)).cpu().float()
    assert torch.equal(got, O.spmm_f16(*A, X))


def _fp64(A1, W1, A2, W2, b, relu, add=None):
    y = A1.double() @ W1.double().t()
    if A2 is not None:
        y = y + A2.double() @ W2.double().t()
    if add is not None:
        y = y + add.double()
    if b is not None:
        y = y + b.double()
    return torch.relu(y) if relu else y


@pytest.mark.parametrize("M,N,K1,K2", [(5000, 512, 256, 256), (777, 300, 64, 0), (9000, 1024, 1024, 0),
                                       (3000, 256, 8, 8), (200, 1028, 4, 0)])
@pytest.mark.parametrize("relu,acc", [(True, False), (False, False), (True, True)])
def test_fc_f16_within_one_rounding_and_kernels_identical(M, N, K1, K2, relu, acc):
    from lpgnn.fc import fc_forward_bf16

    g = _gen(M + N + K1)
    A1 = (torch.randn(M, K1, generator=g)).half()
    W1 = (torch.randn(N, K1, generator=g) / K1 ** 0.5).half()
    A2 = (torch.randn(M, K2, generator=g)).half() if K2 else None
    W2 = (torch.randn(N, K2, generator=g) / K2 ** 0.5).half() if K2 else None
    b = torch.randn(N, generator=g) * 0.1
    P = (torch.randn(M, N, generator=g)).half() if acc else None
    d = lambda t: None if t is None else t.to(DEV)  # noqa: E731
    outs = []
    for kernel in ([0, 1, 2, 3] if K1 >= 64 else [0]):
        out = None if P is None else P.clone().to(DEV)
        y = fc_forward_bf16(d(A1), d(W1), d(A2), d(W2), d(b), relu, out=out, accumulate=acc, kernel=kernel)
        assert y.dtype == H
        outs.append(y.cpu())
    for o in outs[1:]:
        assert torch.equal(o, outs[0])
    ref = _fp64(A1, W1, A2, W2, b, relu, P)
    terms = A1.double().abs() @ W1.double().abs().t()
    if A2 is not None:
        terms = terms + A2.double().abs() @ W2.double().abs().t()
    # one RNE rounding to fp16 (half an ulp, 2^-11 relative) + the fp32 accumulation's error on sum |a w|
    bound = ref.abs() * ULP16 + (K1 + K2 + 2) * 2.0 ** -24 * terms + 6e-8  # (6e-8: fp16 subnormal half-ulp)
    err = (outs[0].double() - ref).abs()
    assert bool((err <= bound).all()), (err - bound).max()


@pytest.mark.parametrize("M,K,N", [(1, 8, 3), (1001, 1024, 3), (4096, 2048, 3), (333, 264, 4)])
def test_heads_f16(M, K, N):
    from lpgnn.fc import linear_small_fwd_bf16

    g = _gen(M + K)
    Hm = torch.relu(torch.randn(M, K, generator=g)).half()
    W = (torch.randn(N, K, generator=g) * 0.05).half()
    b = (torch.randn(N, generator=g)).half()
    got = linear_small_fwd_bf16(Hm.to(DEV), W.to(DEV), b.to(DEV)).cpu()
    assert got.dtype == H
    ref = Hm.double() @ W.double().t() + b.double()
    bound = ref.abs() * ULP16 + (K + 2) * 2.0 ** -24 * (Hm.double().abs() @ W.double().abs().t() + b.double().abs())
    assert bool(((got.double() - ref).abs() <= bound + 6e-8).all())


def test_knowledge_f16_bitwise_vs_oracle():
    from lpgnn.fc import knowledge

    g = _gen(11)
    x = torch.cat([torch.randn(20000, 3, generator=g) * s for s in (1e-3, 0.1, 1.0, 30.0)]).half()
    x[5] = 0  # a zero row: 0 / 0 = NaN, as torch's half path gives
    feas = torch.zeros(x.shape[0], 8)
    feas[::3, 5] = -1
    feas[::5, 7] = 1
    got = knowledge(x.to(DEV), feas.to(DEV)).cpu()
    assert got.dtype == H
    ref = O.add_knowledge_fp16(x, feas)
    same = (got.float() == ref) | (torch.isnan(got.float()) & torch.isnan(ref))
    bad = (~same).any(1).nonzero().flatten()[:5]
    assert bool(same.all()), [(int(i), x[i].tolist(), got[i].tolist(), ref[i].tolist()) for i in bad]
    assert torch.isnan(got[5]).all()


def test_basis_labels_f16_vs_oracle():
    """inference_gnn on fp16 logits: the kernel's fp16 probabilities (its fp32 softmax, rounded) against
    the oracle's fp16 rounding of the exact (fp64) softmax.  The two fp32 evaluations of exp differ by an
    ulp or two, which can move a probability across an fp16 rounding midpoint: such values ("ambiguous")
    are counted, and every label difference must be attributable to one (a node whose own P is
    ambiguous, or one displaced at the top-m boundary by such a node: at most one per ambiguous value)."""
    from lpgnn.val import inference_gnn

    g = _gen(3)
    logits = (torch.randn(300000, 3, generator=g) * 4).half()
    logits[::97] = logits[0]  # exact ties of P[:, 1] (and of P0 / P2 on the same rows)
    p64 = torch.softmax(logits.double(), -1)
    r = lambda t: t.half().double()  # noqa: E731
    amb = ((r(p64 * (1 - 2.0 ** -21)) != r(p64 * (1 + 2.0 ** -21))).any(-1))
    for m in (0, 1, 100000, 300000):
        got = inference_gnn(logits.to(DEV), m).cpu()
        assert int((got == 1).sum()) == m
        ref = O.inference_gnn_fp16(logits, m)
        diff = got != ref
        print(f"m={m}: {int(diff.sum())} label differences, {int(amb.sum())} ambiguous fp16 roundings")
        assert int(diff.sum()) <= 2 * int(amb.sum())
        assert bool((amb | (got == 1) | (ref == 1))[diff].all())  # a non-boundary difference is ambiguous
    # the host path (CPU logits) applies the same fp16 rounding of P
    host = inference_gnn(logits[:5000], 1500)
    ref = O.inference_gnn_fp16(logits[:5000], 1500)
    p1 = O.r16(torch.softmax(logits[:5000].float(), -1))[:, 1]
    thr = p1.topk(1500).values[-1]
    ok = (host == ref) | (p1 == thr)  # torch.topk's choice among the ties at the m-th value is open
    assert bool(ok.all())


def _mid_graph():
    from lpgnn import BipartiteBatch, BipartiteCSR, batch_to, synth

    g = synth.uniform_lp(6000, 12000, 120000, seed=7)
    adj = BipartiteCSR.from_coo(g.row, g.col, g.val, g.m, g.n, device=DEV)
    b = BipartiteBatch(x_s=torch.from_numpy(g.x_s), x_t=torch.from_numpy(g.x_t), y_s=torch.from_numpy(g.y_s),
                       y_t=torch.from_numpy(g.y_t), edge_index=adj, s_bs=g.m, t_bs=g.n)
    return g, batch_to(b, DEV, half=True)


def test_half_model_vs_fp16_oracle():
    """model.half() + batch_to(half=True) (the reference's --fp16 evaluation) against the oracle's
    fp16-storage evaluation: heads within a few fp16 roundings, logits likewise where the heads are
    not small (add_knowledge's 10 h / |h| amplifies a head difference by 20 / |h|), basis labels equal
    up to the nodes such a difference can move; the fp16 logits are in the fp32 model's error class."""
    from lpgnn import GCN_FC
    from lpgnn.val import inference_gnn

    g, batch = _mid_graph()
    assert batch.x_s.dtype == H and batch.edge_index.fwd.val.dtype == torch.float32
    torch.manual_seed(0)
    model = GCN_FC(8, 8, hids=256, depth=4).to(DEV)
    sd = {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}
    model.half().eval()
    with torch.no_grad():
        lc, lv = model(batch)
        labels = inference_gnn(torch.cat((lc, lv)), g.m).cpu()
    assert lc.dtype == H and lv.dtype == H
    A = O.csr_from_coo(g.row, g.col, g.val, g.m, g.n)
    AT = O.csr_transpose(*A, g.m, g.n)
    keep = {}
    rc, rv = O.gcn_fc_forward_fp16(sd, torch.from_numpy(g.x_s), torch.from_numpy(g.x_t), A, AT, 4, keep=keep)
    got, ref = torch.cat((lc, lv)).cpu().double(), torch.cat((rc, rv)).double()
    d = (got - ref).abs()
    rel = d.max(-1).values / ref.abs().max(-1).values.clamp_min(1e-3)
    print(f"fp16 model vs fp16 oracle: mean |d| {d.mean():.2e}, max {d.max():.3e}, "
          f"nodes off by more than 4 fp16 ulps: {int((rel > 8 * ULP16).sum())}")
    assert d.mean().item() <= 2e-3
    assert float(torch.quantile(rel.float(), 0.99)) <= 8 * ULP16
    f32c, f32v = O.gcn_fc_forward(sd, torch.from_numpy(g.x_s), torch.from_numpy(g.x_t), A, AT, 4)
    f32 = torch.cat((f32c, f32v)).double()
    assert (got - f32).abs().mean().item() <= 3 * (ref - f32).abs().mean().item() + 1e-3
    rl = O.inference_gnn_fp16(torch.cat((rc, rv)), g.m)
    assert (labels != rl).float().mean().item() <= 2e-3


def test_run_validation_fp16_mode(tmp_path):
    """The CLI's --fp16 on the evaluation model: model.half() after the load, every batch through
    batch_to(half=True); fp16 logits in the fp32 model's error class (val.py:269, utils.py:909-915)."""
    from lpgnn import GCN_FC

    g, batch = _mid_graph()
    torch.manual_seed(0)
    m32 = GCN_FC(8, 8, hids=64, depth=3).to(DEV).eval()
    m16 = GCN_FC(8, 8, hids=64, depth=3).to(DEV)
    m16.load_state_dict(m32.state_dict())
    m16.half().eval()
    from lpgnn import BipartiteBatch, BipartiteCSR

    adj = BipartiteCSR.from_coo(g.row, g.col, g.val, g.m, g.n, device=DEV)
    b32 = BipartiteBatch(x_s=torch.from_numpy(g.x_s).to(DEV), x_t=torch.from_numpy(g.x_t).to(DEV),
                         y_s=torch.from_numpy(g.y_s).to(DEV), y_t=torch.from_numpy(g.y_t).to(DEV),
                         edge_index=adj, s_bs=g.m, t_bs=g.n)
    from lpgnn.val import model_inference_with_batch

    with torch.no_grad():
        a = torch.cat(m32(b32))
        lc, lv = model_inference_with_batch(m16, b32, "GCN_FC(8,8,hids=64,depth=3)", dev=DEV, fp16=True)
    assert lc.dtype == H and b32.x_s.dtype == torch.float32  # the caller's batch keeps its dtypes
    assert (torch.cat((lc, lv)).float() - a.cpu()).abs().mean().item() < 0.02
    with pytest.raises(RuntimeError, match="inference mode"):
        m16.train()(batch)
