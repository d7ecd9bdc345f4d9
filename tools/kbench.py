"""Kernel microbenchmarks on one GPU (HIP events, interleaved rounds, median).

  python tools/kbench.py [fc] [spmm] [bwd]

fc   : lpg_fc_f32 at the c2 shapes vs torch (hipBLASLt) linear+linear+add+relu
fcpmc: only the two hidden-layer FC kernels (fp32 c2 and bf16 c5 shapes), for PMC passes
bf16 : lpg_fc_bf16 at the c5 shape vs torch bf16 (hipBLASLt)
bf16bwd: the c5 backward GEMMs (lpg_wgrad_bf16, lpg_fc_bf16 on transposed weights) vs torch
load : graph load at c2 -- reference chain (to_undirected + MyToBipartite + device pack) vs direct pack
spmm : lpg_spmm_f32 at c2, both directions, slice widths 256/512/1024
bwd  : the FC backward GEMMs at c2 shapes through torch (hipBLASLt)
wgk  : lpg_wgrad_bf16 vs R (per-launch fixed cost)
x3epi: lpg_fc_x3 at the c2 shapes, one line per epilogue (plain / ReLU+dropout / +accumulate / +heads)
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lp-gnn_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def timeit(fns, rounds=7, iters=5):
    """fns: {name: callable}; returns {name: median ms per call}."""
    res = {k: [] for k in fns}
    for fn in fns.values():
        fn()
    torch.cuda.synchronize()
    for _ in range(rounds):
        for k, fn in fns.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(iters):
                fn()
            e1.record()
            torch.cuda.synchronize()
            res[k].append(e0.elapsed_time(e1) / iters)
    return {k: float(np.median(v)) for k, v in res.items()}


def bench_fc(out):
    """The exact-fp32 FC (LPGNN_FC_ARITH=fp32's kernel) and the default x3 FC at the c2 shapes vs torch."""
    from lpgnn.fc import fc_forward

    dev = "cuda"
    for M, K in ((200_000, 1024), (100_000, 1024)):
        A1 = torch.randn(M, K, device=dev)
        A2 = torch.randn(M, K, device=dev)
        W1 = torch.randn(1024, K, device=dev) * 0.03
        W2 = torch.randn(1024, K, device=dev) * 0.03
        b = torch.randn(1024, device=dev)
        flops = 2.0 * M * 1024 * 2 * K
        t = timeit({
            "lpg_fc_f32": lambda: fc_forward(A1, W1, A2, W2, b, True, arith="fp32"),
            "lpg_fc_x3_f32": lambda: fc_forward(A1, W1, A2, W2, b, True, arith="x3"),
            "torch_2gemm_add_relu": lambda: torch.relu(F.linear(A1, W1, b) + F.linear(A2, W2)),
        })
        for k, v in t.items():
            out[f"fc M={M} K={2*K} {k}"] = dict(ms=v, tflops=flops / v / 1e9)
        H = torch.randn(M, 1024, device=dev)
        Wh = torch.randn(3, 1024, device=dev)
        bh = torch.randn(3, device=dev)
        X8 = torch.randn(M, 8, device=dev)
        W8 = torch.randn(1024, 8, device=dev)
        t = timeit({"heads": lambda: fc_forward(H, Wh, None, None, bh, False),
                    "conv1": lambda: fc_forward(X8, W8, X8, W8, b, True)})
        out[f"fc heads M={M}"] = dict(ms=t["heads"], gbs=M * 1024 * 4 / t["heads"] / 1e6)
        out[f"fc conv1 M={M}"] = dict(ms=t["conv1"], gbs=M * 1024 * 4 / t["conv1"] / 1e6)


def bench_bwd(out):
    dev = "cuda"
    for M in (200_000, 100_000):
        g = torch.randn(M, 1024, device=dev)
        W = torch.randn(1024, 1024, device=dev)
        A = torch.randn(M, 1024, device=dev)
        fl = 2.0 * M * 1024 * 1024
        t = timeit({"dA=g@W": lambda: g @ W, "dW=g.t()@A": lambda: g.t() @ A,
                    "mask": lambda: g.masked_fill(A <= 0, 0.0), "colsum": lambda: g.sum(0)})
        for k, v in t.items():
            out[f"bwd M={M} {k}"] = dict(ms=v, tflops=fl / v / 1e9 if "@" in k else None)


def bench_spmm(out):
    from lpgnn import BipartiteCSR, _lib, synth
    from lpgnn.sparse import spmm_forward

    L = _lib.lib()
    for gname, g in (("uniform", synth.uniform_lp(100_000, 200_000, 2_000_000, seed=0)),
                     ("skewed", synth.skewed_lp(100_000, 200_000, 2_000_000, seed=0))):
        _spmm_graph(out, L, gname, g, spmm_forward, BipartiteCSR)


def _spmm_graph(out, L, gname, g, spmm_forward, BipartiteCSR):
    """c2-sized graph (uniform rows, or Zipf(1.5) row degrees -- SURVEY.md 8d's load-balance variant)."""
    adj = BipartiteCSR.from_coo(g.row, g.col, g.val, g.m, g.n, device="cuda")
    for name, csr, K in (("cons<-vars", adj.fwd, g.n), ("vars<-cons", adj.bwd, g.m)):
        X = torch.randn(K, 1024, device="cuda")
        fns = {}
        ref = spmm_forward(csr, X)
        from lpgnn import sparse as S
        h0 = S.DEFAULT_HEAVY
        for sl, u, h in ((0, 0, h0), (128, 8, h0), (128, 16, h0), (256, 8, h0), (256, 16, h0), (256, 32, h0),
                         (512, 8, h0), (256, 8, 0), (256, 8, 256)):
            def f(sl=sl, u=u, h=h):  # degree-aware split: rows above h on (row, slice) waves; 0 = off
                return spmm_forward(csr, X, slice_cols=sl, depth=u, heavy=h)
            assert torch.equal(f(), ref)
            fns[f"slice{sl} depth{u} heavy>{h}"] = f
        t = timeit(fns)
        B = g.nnz * 1024 * 4 + g.nnz * 8 + (csr.n_rows + 1) * 8 + csr.n_rows * 1024 * 4
        for k, v in t.items():
            out[f"spmm {gname} {name} {k}"] = dict(ms=v, gbs=B / v / 1e6, frac=B / v / 1e6 / 8000,
                                                   max_deg=int(csr.degrees().max().item()))


def bench_spmmbig(out):
    """fp32 SpMM slice widths on graphs whose gathered table is far above the Infinity Cache: a c4
    rank's share at N = 8 (250K x 500K, nnz 5M) and the whole c4 graph (2M x 4M, nnz 40M); c2 beside."""
    from lpgnn import BipartiteCSR, _lib, synth
    from lpgnn.sparse import spmm_forward

    L = _lib.lib()
    for gname, (m, n, nnz) in (("c2", (100_000, 200_000, 2_000_000)), ("c4/8", (250_000, 500_000, 5_000_000)),
                               ("c4", (2_000_000, 4_000_000, 40_000_000))):
        g = synth.uniform_lp(m, n, nnz, seed=0)
        adj = BipartiteCSR.from_coo(g.row, g.col, g.val, g.m, g.n, device="cuda")
        del g
        for name, csr, K in (("cons<-vars", adj.fwd, n), ("vars<-cons", adj.bwd, m)):
            X = torch.randn(K, 1024, device="cuda")
            ref = spmm_forward(csr, X)
            fns = {}
            for sl in (256, 128, 64):
                def f(sl=sl):
                    return spmm_forward(csr, X, slice_cols=sl)
                assert torch.equal(f(), ref)
                fns[f"slice{sl}"] = f
            t = timeit(fns, rounds=5, iters=3)
            rows = csr.n_rows
            B = nnz * 1024 * 4 + nnz * 8 + (rows + 1) * 8 + rows * 1024 * 4
            for k, v in t.items():
                out[f"spmm {gname} {name} {k}"] = dict(ms=v, gbs=B / v / 1e6, frac=B / v / 1e6 / 8000)
            del X, ref
        del adj
        torch.cuda.empty_cache()


def bench_spmm16(out):
    """bf16 SpMM at the c5 width (F = 2048), both directions, slice widths (256 = rowslim)."""
    from lpgnn import BipartiteCSR, _lib, synth
    from lpgnn.sparse import spmm_forward

    L = _lib.lib()
    for gname, g in (("uniform", synth.uniform_lp(100_000, 200_000, 2_000_000, seed=0)),
                     ("skewed", synth.skewed_lp(100_000, 200_000, 2_000_000, seed=0))):
        adj = BipartiteCSR.from_coo(g.row, g.col, g.val, g.m, g.n, device="cuda")
        for name, csr, K in (("cons<-vars", adj.fwd, g.n), ("vars<-cons", adj.bwd, g.m)):
            X = torch.randn(K, 2048, device="cuda").to(torch.bfloat16)
            ref = spmm_forward(csr, X, slice_cols=1024, heavy=0)  # the whole-row (round-1) form as the reference
            fns = {}
            from lpgnn import sparse as S
            h0 = S.DEFAULT_HEAVY
            for sl, h in ((256, h0), (256, 0), (512, 0), (1024, 0)):
                def f(sl=sl, h=h):
                    return spmm_forward(csr, X, slice_cols=sl, heavy=h)
                assert torch.equal(f(), ref)
                fns[f"slice{sl} heavy>{h}"] = f
            t = timeit(fns)
            B = g.nnz * 2048 * 2 + g.nnz * 8 + (csr.n_rows + 1) * 8 + csr.n_rows * 2048 * 2
            for k, v in t.items():
                out[f"spmm bf16 {gname} {name} {k}"] = dict(ms=v, gbs=B / v / 1e6, frac=B / v / 1e6 / 8000)


def bench_fcpmc(out):
    from lpgnn.fc import fc_forward, fc_forward_bf16

    M = 200_000
    A1, A2 = torch.randn(M, 1024, device="cuda"), torch.randn(M, 1024, device="cuda")
    W1, W2 = torch.randn(1024, 1024, device="cuda") * 0.03, torch.randn(1024, 1024, device="cuda") * 0.03
    b = torch.randn(1024, device="cuda")
    t = timeit({"f32": lambda: fc_forward(A1, W1, A2, W2, b, True)}, rounds=3, iters=3)
    out["fcpmc f32 M=200000 K=2048"] = dict(ms=t["f32"], tflops=2.0 * M * 1024 * 2048 / t["f32"] / 1e9)
    del A1, A2
    B1, B2 = (torch.randn(M, 2048, device="cuda").to(torch.bfloat16) for _ in range(2))
    V1, V2 = ((torch.randn(2048, 2048, device="cuda") * 0.02).to(torch.bfloat16) for _ in range(2))
    b2 = torch.randn(2048, device="cuda")
    t = timeit({"bf16": lambda: fc_forward_bf16(B1, V1, B2, V2, b2, True)}, rounds=3, iters=3)
    out["fcpmc bf16 M=200000 K=4096"] = dict(ms=t["bf16"], tflops=2.0 * M * 2048 * 4096 / t["bf16"] / 1e9)


def bench_bf16(out):
    from lpgnn.fc import fc_forward_bf16

    M = 200_000
    B1, B2 = (torch.randn(M, 2048, device="cuda").to(torch.bfloat16) for _ in range(2))
    V1, V2 = ((torch.randn(2048, 2048, device="cuda") * 0.02).to(torch.bfloat16) for _ in range(2))
    b2 = torch.randn(2048, device="cuda")
    Bc = torch.cat([B1, B2], 1)
    Vc = torch.cat([V1, V2], 1)

    def ker(k):
        return lambda: fc_forward_bf16(B1, V1, B2, V2, b2, True, kernel=k)
    y0 = ker(0)()
    for k in (1, 2, 3):
        assert torch.equal(ker(k)(), y0), f"bf16 kernel {k} differs"
    t = timeit({"lpg_fc_bf16 k2 256x256 2buf": ker(2), "lpg_fc_bf16 k3 pipelined (default)": ker(3),
                "torch_bf16_1gemm_relu": lambda: torch.relu(F.linear(Bc, Vc, b2.to(torch.bfloat16)))})
    for k, v in t.items():
        out[f"bf16 M={M} K=4096 {k}"] = dict(ms=v, tflops=2.0 * M * 2048 * 4096 / v / 1e9)


def bench_fck(out):
    """lpg_fc_bf16 (default kernel) at M = 200K / 100K, N = 2048 for K = 1024 .. 8192 (one phase, no
    epilogue options, and with ReLU + dropout + accumulate in place): per-block fixed cost vs the k loop."""
    from lpgnn.fc import fc_forward_bf16

    BF = torch.bfloat16
    for M in (200_000, 100_000):
        for K in (1024, 2048, 4096, 8192):
            A = torch.randn(M, K, device="cuda").to(BF)
            W = (torch.randn(2048, K, device="cuda") * 0.02).to(BF)
            b = torch.randn(2048, device="cuda")
            P = torch.randn(M, 2048, device="cuda").to(BF)

            def run(acc, A=A, W=W, b=b, P=P):
                def f():
                    if acc:
                        return fc_forward_bf16(A, W, None, None, b, True, 0.1, 7, out=P, accumulate=True)
                    return fc_forward_bf16(A, W, None, None, None, False)
                return f
            t = timeit({("relu+drop+acc" if acc else "plain"): run(acc) for acc in (False, True)}, rounds=5, iters=3)
            for k, v in t.items():
                out[f"fcK M={M} K={K} {k}"] = dict(ms=v, tflops=2.0 * M * 2048 * K / v / 1e9)
            del A, W, P


def bench_fckern(out):
    """lpg_fc_bf16's per-call kernel choices (LPG_FC_KERNEL: 1 = 128 x 128 tiles, 4 waves, 2 blocks
    per CU; 2 = 256 x 256; 3 = the pipelined 256 x 256 default) at the c5 shapes, ReLU + dropout."""
    from lpgnn.fc import fc_forward_bf16

    BF = torch.bfloat16
    for M, K in ((200_000, 2048), (100_000, 4096), (200_000, 4096)):
        A = torch.randn(M, K, device="cuda").to(BF)
        W = (torch.randn(2048, K, device="cuda") * 0.02).to(BF)
        b = torch.randn(2048, device="cuda")
        fns = {f"kernel={k}": (lambda k=k: fc_forward_bf16(A, W, None, None, b, True, 0.1, 7, kernel=k)) for k in (0, 1, 2, 3)}
        t = timeit(fns, rounds=5, iters=3)
        for k, v in t.items():
            out[f"fckern M={M} K={K} {k}"] = dict(ms=v, tflops=2.0 * M * 2048 * K / v / 1e9)
        del A, W


def bench_epidrop(out):
    """What each epilogue option costs in the hidden-layer GEMMs: the c5 bf16 FC (M = 200K, N = 2048,
    K = 2048) and the c2 x3 FC (M = 200K, N = 1024, K = 1024) with plain / bias+ReLU / +dropout /
    +accumulate epilogues."""
    from lpgnn.fc import fc_forward, fc_forward_bf16

    BF = torch.bfloat16
    M = 200_000
    for name, N, K, dt in (("bf16", 2048, 2048, BF), ("x3", 1024, 1024, torch.float32)):
        A = torch.randn(M, K, device="cuda").to(dt)
        W = (torch.randn(N, K, device="cuda") * 0.02).to(dt)
        b = torch.randn(N, device="cuda")
        P = torch.randn(M, N, device="cuda").to(dt)
        fwd = fc_forward_bf16 if name == "bf16" else (lambda *a, **k: fc_forward(*a, arith="x3", **k))
        fns = {"plain": lambda: fwd(A, W, None, None, None, False),
               "bias+relu": lambda: fwd(A, W, None, None, b, True),
               "bias+relu+drop": lambda: fwd(A, W, None, None, b, True, 0.1, 7),
               "bias+relu+acc": lambda: fwd(A, W, None, None, b, True, out=P, accumulate=True),
               "bias+relu+drop+acc": lambda: fwd(A, W, None, None, b, True, 0.1, 7, out=P, accumulate=True)}
        t = timeit(fns, rounds=5, iters=3)
        for k, v in t.items():
            out[f"epidrop {name} M={M} N={N} K={K} {k}"] = dict(ms=v, tflops=2.0 * M * N * K / v / 1e9)
        del A, W, P


def bench_spmmdepth(out):
    """The c2 / c5 SpMMs (uniform 100K x 200K, nnz 2M) at gather depth 8 / 16 and each slice width."""
    from lpgnn import BipartiteCSR, synth
    from lpgnn.sparse import spmm_forward

    g = synth.uniform_lp(100_000, 200_000, 2_000_000, seed=0)
    adj = BipartiteCSR.from_coo(g.row, g.col, g.val, g.m, g.n, device="cuda")
    for dt, F in ((torch.float32, 1024), (torch.bfloat16, 2048)):
        for name, csr, K in (("cons<-vars", adj.fwd, g.n), ("vars<-cons", adj.bwd, g.m)):
            X = torch.randn(K, F, device="cuda").to(dt)
            ref = spmm_forward(csr, X)
            fns = {}
            slices = (64, 128, 256) if dt == torch.float32 else (256, 512)
            for d in (8, 16):
                for sl in slices:
                    f = (lambda d=d, sl=sl: spmm_forward(csr, X, slice_cols=sl, depth=d))
                    assert torch.equal(f(), ref)
                    fns[f"depth{d} slice{sl}"] = f
            t = timeit(fns)
            esz = 2 if dt == torch.bfloat16 else 4
            B = g.nnz * F * esz + g.nnz * 8 + (csr.n_rows + 1) * 8 + csr.n_rows * F * esz
            for k, v in t.items():
                out[f"spmm {dt} {name} {k}"] = dict(ms=v, frac=B / v / 1e6 / 8000)


def bench_x3kern(out):
    """lpg_fc_x3_f32's per-call kernel choice (0 = the wide 128 x 128 kernel, 1 = the 16-row strip
    kernel) at the c2 FC shapes, plain and ReLU + dropout + accumulate."""
    from lpgnn.fc import fc_forward

    for M, K1, K2 in ((200_000, 1024, 0), (100_000, 1024, 1024), (100_000, 1024, 0)):
        A1 = torch.randn(M, K1, device="cuda")
        A2 = torch.randn(M, K2, device="cuda") if K2 else None
        W1 = torch.randn(1024, K1, device="cuda") * 0.03
        W2 = torch.randn(1024, K2, device="cuda") * 0.03 if K2 else None
        b = torch.randn(1024, device="cuda")
        P = torch.randn(M, 1024, device="cuda")
        fns = {}
        for k in (0, 1):
            fns[f"kernel={k} plain"] = (lambda k=k: fc_forward(A1, W1, A2, W2, None, False, arith="x3", kernel=k))
            fns[f"kernel={k} relu+drop+acc"] = (lambda k=k: fc_forward(A1, W1, A2, W2, b, True, 0.1, 7, out=P,
                                                                       accumulate=True, arith="x3", kernel=k))
        t = timeit(fns, rounds=5, iters=3)
        for name, v in t.items():
            out[f"x3kern M={M} K={K1}+{K2} {name}"] = dict(ms=v, tflops=2.0 * M * 1024 * (K1 + K2) / v / 1e9)
        del A1, A2, P


def bench_wgk(out):
    """lpg_wgrad_bf16 at N = K = 2048 for R = 25K .. 400K: the per-launch fixed cost (prologue,
    partial-tile epilogue, fold) against the per-row slope."""
    from lpgnn.fc import wgrad_bf16

    BF = torch.bfloat16
    for R in (25_000, 50_000, 100_000, 200_000, 400_000):
        G = torch.randn(R, 2048, device="cuda").to(BF)
        X = torch.relu(torch.randn(R, 2048, device="cuda")).to(BF)
        t = timeit({"wgrad_bf16": lambda G=G, X=X: wgrad_bf16(G, X)}, rounds=5, iters=4)
        for k, v in t.items():
            out[f"wgk R={R} {k}"] = dict(ms=v, tflops=2.0 * R * 2048 * 2048 / v / 1e9)
        del G, X


def bench_rbwd(out):
    """lpg_relu_bwd_colsum_bf16 at the c5 shapes (200K / 100K x 2048) and lpg_relu_bwd_colsum_f32
    at c2 (200K x 1024): GB/s of g + y read and dZ written."""
    from lpgnn.fc import relu_bwd_colsum, relu_bwd_colsum_bf16

    for M in (200_000, 100_000):
        g = torch.randn(M, 2048, device="cuda").to(torch.bfloat16)
        y = torch.randn(M, 2048, device="cuda").to(torch.bfloat16)
        t = timeit({"bf16": lambda: relu_bwd_colsum_bf16(g, y, 1.1, True)}, rounds=7, iters=5)
        out[f"rbwd bf16 M={M}"] = dict(ms=t["bf16"], gbs=3 * M * 2048 * 2 / t["bf16"] / 1e6)
        del g, y
    g = torch.randn(200_000, 1024, device="cuda")
    y = torch.randn(200_000, 1024, device="cuda")
    t = timeit({"f32": lambda: relu_bwd_colsum(g, y, 1.1, True)}, rounds=7, iters=5)
    out["rbwd f32 M=200000"] = dict(ms=t["f32"], gbs=3 * 200_000 * 1024 * 4 / t["f32"] / 1e6)


def bench_x3epi(out):
    """lpg_fc_x3 at the c2 FC shapes with each epilogue: plain, ReLU + dropout (two phases) and
    ReLU + dropout + accumulate (in place, no clone in the timed region), heads fused."""
    from lpgnn.fc import fc_forward

    for M, K1, K2, mode in ((200_000, 1024, 0, "lin"), (200_000, 1024, 0, "relu+drop+acc"),
                            (200_000, 1024, 0, "relu+drop+acc+heads"),
                            (100_000, 1024, 1024, "relu+drop"), (100_000, 1024, 0, "lin")):
        A1 = torch.randn(M, K1, device="cuda")
        A2 = torch.randn(M, K2, device="cuda") if K2 else None
        W1 = torch.randn(1024, K1, device="cuda") * 0.03
        W2 = torch.randn(1024, K2, device="cuda") * 0.03 if K2 else None
        b = torch.randn(1024, device="cuda")
        P = torch.randn(M, 1024, device="cuda")
        hd = (torch.randn(3, 1024, device="cuda") * 0.03, torch.randn(3, device="cuda"))

        def f(A1=A1, A2=A2, W1=W1, W2=W2, b=b, P=P, mode=mode):
            if mode == "lin":
                return fc_forward(A1, W1, A2, W2, None, False, arith="x3")
            return fc_forward(A1, W1, A2, W2, b, True, 0.1, 7, out=P if "acc" in mode else None,
                              accumulate="acc" in mode, arith="x3", heads=hd if "heads" in mode else None)
        t = timeit({mode: f}, rounds=7, iters=4)
        for k, v in t.items():
            out[f"x3epi M={M} K={K1}+{K2} {k}"] = dict(ms=v, tflops=2.0 * M * 1024 * (K1 + K2) / v / 1e9)
        del A1, A2, P


def bench_bf16bwd(out):
    """c5 backward GEMMs: lpg_wgrad_bf16 vs torch (G^T X).float(); the input gradient on
    lpg_fc_bf16 (transposed weights) vs torch G @ W."""
    from lpgnn.fc import input_grad_bf16, wgrad_bf16

    BF = torch.bfloat16
    for R in (100_000, 200_000):
        G = torch.randn(R, 2048, device="cuda").to(BF)
        X = torch.relu(torch.randn(R, 2048, device="cuda")).to(BF)
        W = torch.randn(2048, 2048, device="cuda") * 0.02
        Wb = W.to(BF)
        a = wgrad_bf16(G, X)
        ref = (G.float().t() @ X.float())
        print(f"R={R} wgrad max|ours - fp32 torch| = {(a - ref).abs().max().item():.3e}  "
              f"max|torch bf16 - fp32| = {((G.t() @ X).float() - ref).abs().max().item():.3e}", flush=True)
        del ref
        t = timeit({"wgrad": lambda: wgrad_bf16(G, X),
                    "wgrad torch (G^T X).float()": lambda: (G.t() @ X).float(),
                    "igrad": lambda: input_grad_bf16(G, W), "igrad torch G @ W": lambda: G @ Wb,
                    "igrad2": lambda: input_grad_bf16(G, W, G, W),
                    "igrad2 torch": lambda: torch.addmm(G @ Wb, G, Wb)}, rounds=5, iters=3)
        for k, v in t.items():
            fl = 2.0 * R * 2048 * 2048 * (2 if k.startswith("igrad2") else 1)
            out[f"bf16bwd R={R} {k}"] = dict(ms=v, tflops=fl / v / 1e9)
        del G, X


def bench_tail(out):
    """Wave-quantisation tail of the FC launches: time vs M around the c2 / c5 row counts
    (x3: 128x128 tiles, 8 n-tiles, 512 block slots -> one round = 8192 rows; bf16: 256x256 tiles,
    8 n-tiles, 256 slots -> one round = 8192 rows)."""
    from lpgnn.fc import fc_forward, fc_forward_bf16

    for arith, N, K, dt in (("x3", 1024, 1024, torch.float32), ("bf16", 2048, 2048, torch.bfloat16)):
        Mmax = 114_688
        A1 = torch.randn(Mmax, K, device="cuda").to(dt)
        W1 = (torch.randn(N, K, device="cuda") * 0.03)
        b = torch.randn(N, device="cuda")
        if dt == torch.bfloat16:
            W1 = W1.to(dt)
        for M in (90_112, 98_304, 100_000, 102_400, 106_496, 114_688):
            A = A1[:M]

            def f(A=A):
                if arith == "bf16":
                    return fc_forward_bf16(A, W1, None, None, b, True)
                return fc_forward(A, W1, None, None, b, True, arith="x3")
            t = timeit({"f": f}, rounds=7, iters=4)["f"]
            out[f"tail {arith} M={M} N={N} K={K}"] = dict(ms=t, us_per_krow=t * 1e6 / M,
                                                          tflops=2.0 * M * N * K / t / 1e9)
        del A1
    from lpgnn.fc import wgrad
    for R in (100_000, 200_000, 400_000):
        G = torch.randn(R, 1024, device="cuda")
        X = torch.randn(R, 1024, device="cuda")
        t = timeit({"f": lambda G=G, X=X: wgrad(G, X, arith="x3")}, rounds=7, iters=4)["f"]
        out[f"tail wgrad_x3 R={R} splits={os.environ.get('LPGNN_WGRAD_SPLITS', 'auto')}"] = dict(
            ms=t, tflops=2.0 * R * 1024 * 1024 / t / 1e9)
        del G, X


def bench_load(out):
    import time

    from lpgnn import synth
    from lpgnn.data import MyToBipartite, bipartite_from_lp, lp_to_unipartite

    g = synth.uniform_lp(100_000, 200_000, 2_000_000, seed=0)
    args = (g.row, g.col, g.val, g.x_s, g.x_t, g.y_s, g.y_t)

    def ref():
        return MyToBipartite(dev="cuda")(lp_to_unipartite(*args))

    def direct():
        return bipartite_from_lp(*args, device="cuda")

    for name, fn in (("reference chain (host to_undirected + relabel, device pack)", ref),
                     ("direct (device pack of the LP entries)", direct)):
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(3):
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        out[f"load c2 {name}"] = dict(ms=float(np.median(ts)) * 1e3)


def bench_fcpi(out):
    """The x3 FC kernels (default wide, LPG_FC_KERNEL(1)) and the exact-fp32 kernel at the c2
    hidden-layer shapes vs hipBLASLt (torch)."""
    from lpgnn.fc import fc_forward

    dev = "cuda"
    for M, K1, K2 in ((200_000, 1024, 1024), (200_000, 1024, 0), (100_000, 1024, 0)):
        A1 = torch.randn(M, K1, device=dev).relu_()
        A2 = torch.randn(M, K2, device=dev).relu_() if K2 else None
        W1 = torch.randn(1024, K1, device=dev) * 0.03
        W2 = torch.randn(1024, K2, device=dev) * 0.03 if K2 else None
        b = torch.randn(1024, device=dev)
        flops = 2.0 * M * 1024 * (K1 + K2)
        fns = {"x3 wide": lambda: fc_forward(A1, W1, A2, W2, b, True, arith="x3"),
               "x3 k1": lambda: fc_forward(A1, W1, A2, W2, b, True, arith="x3", kernel=1),
               "fp32": lambda: fc_forward(A1, W1, A2, W2, b, True, arith="fp32")}
        assert torch.equal(fns["x3 wide"](), fns["x3 k1"]())
        if K2:
            fns["torch"] = lambda: torch.relu(torch.addmm(b, A1, W1.t()).addmm_(A2, W2.t()))
        else:
            fns["torch"] = lambda: torch.relu(torch.addmm(b, A1, W1.t()))
        t = timeit(fns)
        for k, v in t.items():
            out[f"fcpi M={M} K={K1}+{K2} {k}"] = dict(ms=v, tflops=flops / v / 1e9)
        del A1, A2


def bench_stream(out):
    """The c2 / c5 steps' streaming kernels at 100K / 200K rows (GB/s of the bytes each must move):
    heads + ReLU backward (read Y, write dZ), conv1 weight gradients from (g, y) or from dZ (read
    both / one), conv1 forward with ReLU + dropout (write C), the bf16 heads' forward (read Y);
    fp32 at F = 1024 (c2), bf16 at F = 2048 (c5); torch copy_ / fill_ as the box's streaming rates."""
    from lpgnn.fc import (fc_forward, fc_forward_bf16, heads_bwd_bf16, heads_relu_bwd, linear_small_fwd_bf16,
                          relu_wgrad_smallk, relu_wgrad_smallk_bf16)

    dev = "cuda"
    BF = torch.bfloat16
    for M in (100_000, 200_000):
        g = torch.randn(M, 1024, device=dev)
        y = torch.relu(torch.randn(M, 1024, device=dev))
        G3 = torch.randn(M, 3, device=dev)
        W3 = torch.randn(3, 1024, device=dev)
        X8, X8b = torch.randn(M, 8, device=dev), torch.randn(M, 8, device=dev)
        W8, W8b = torch.randn(1024, 8, device=dev), torch.randn(1024, 8, device=dev)
        b = torch.randn(1024, device=dev)
        dst = torch.empty_like(g)
        nb = M * 1024 * 4
        t = timeit({"heads_relu_bwd": lambda: heads_relu_bwd(G3, W3, y, 1.1, True),
                    "relu_wgrad_smallk": lambda: relu_wgrad_smallk(g, y, 1.1, X8, X8b, True),
                    "conv1_fwd": lambda: fc_forward(X8, W8, X8b, W8b, b, True, 0.1, 7),
                    "torch_copy": lambda: dst.copy_(g), "torch_fill": lambda: dst.fill_(1.0)})
        for k, v in t.items():
            nbytes = nb * (1 if k in ("conv1_fwd", "torch_fill") else 2)
            out[f"stream M={M} {k}"] = dict(ms=v, gbs=nbytes / v / 1e6)
        del g, y, dst
        # c5 (bf16, F = 2048): the same bytes per row
        gb = torch.randn(M, 2048, device=dev).to(BF)
        yb = torch.relu(torch.randn(M, 2048, device=dev)).to(BF)
        Gb = torch.randn(M, 3, device=dev).to(BF)
        W3b = torch.randn(3, 2048, device=dev)
        X8h, X8bh = X8.to(BF), X8b.to(BF)
        W8h, W8bh = torch.randn(2048, 8, device=dev).to(BF), torch.randn(2048, 8, device=dev).to(BF)
        b2 = torch.randn(2048, device=dev)
        nb = M * 2048 * 2
        t = timeit({"bf16 heads_bwd(mask)": lambda: heads_bwd_bf16(Gb, W3b, yb, 1.1, True),
                    "bf16 relu_wgrad_smallk(g,y)": lambda: relu_wgrad_smallk_bf16(gb, yb, 1.1, X8h, X8bh, True),
                    "bf16 wgrad_smallk(dZ)": lambda: relu_wgrad_smallk_bf16(gb, None, 1.0, X8h, X8bh, True),
                    "bf16 conv1_fwd": lambda: fc_forward_bf16(X8h, W8h, X8bh, W8bh, b2, True, 0.1, 7),
                    "bf16 heads_fwd": lambda: linear_small_fwd_bf16(yb, W3b, b2[:3])})
        for k, v in t.items():
            nbytes = nb * (2 if ("heads_bwd" in k or "(g,y)" in k) else 1)
            out[f"stream M={M} {k}"] = dict(ms=v, gbs=nbytes / v / 1e6)
        del gb, yb


if __name__ == "__main__":
    which = sys.argv[1:] or ["fc", "spmm", "bwd"]
    out = {}
    for w in which:
        {"fc": bench_fc, "spmm": bench_spmm, "bwd": bench_bwd, "fcpmc": bench_fcpmc, "bf16": bench_bf16,
         "bf16bwd": bench_bf16bwd, "spmm16": bench_spmm16,
         "spmmbig": bench_spmmbig, "fck": bench_fck, "x3epi": bench_x3epi, "wgk": bench_wgk, "rbwd": bench_rbwd,
         "load": bench_load, "fcpi": bench_fcpi, "stream": bench_stream, "tail": bench_tail, "fckern": bench_fckern,
         "epidrop": bench_epidrop, "spmmdepth": bench_spmmdepth, "x3kern": bench_x3kern}[w](out)
        torch.cuda.empty_cache()
    for k, v in out.items():
        print(f"{k:45s} " + " ".join(f"{a}={b:.4g}" for a, b in v.items() if b is not None))
    json.dump(out, open(os.path.join(ROOT, "gpurun_out", "kbench.json"), "w"), indent=1)
