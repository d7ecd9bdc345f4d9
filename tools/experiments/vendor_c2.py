"""Vendor libraries on the c2 hot-path shapes, beside our kernels: the SpMM (rocSPARSE through
torch.sparse.mm on a CSR tensor) for both directions at F = 1024 fp32, and the FC forward (hipBLASLt
through torch.nn.functional.linear, fp32) at the hidden-layer shapes, against lpg_spmm_f32 and the x3
FC (lpg_fc_x3_f32).  Same operands, median of 15 launches."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "lp-gnn_amd"))
from lpgnn import BipartiteCSR, synth  # noqa: E402
from lpgnn import fc as FC  # noqa: E402
from lpgnn.sparse import spmm_forward  # noqa: E402

DEV = "cuda:0"


def bench(fn, reps=15):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    g = synth.uniform_lp(100_000, 200_000, 2_000_000, seed=0)
    adj = BipartiteCSR.from_coo(g.row, g.col, g.val, g.m, g.n, device=DEV)
    F = 1024
    for name, csr in (("cons<-vars", adj.fwd), ("vars<-cons", adj.bwd)):
        X = torch.randn(csr.n_cols, F, device=DEV)
        S = torch.sparse_csr_tensor(csr.rowptr, csr.col.long(), csr.val, (csr.n_rows, csr.n_cols), device=DEV)
        ours = spmm_forward(csr, X)
        ref = torch.sparse.mm(S, X)
        err = float((ours - ref).abs().max())
        t_o = bench(lambda: spmm_forward(csr, X))
        t_v = bench(lambda: torch.sparse.mm(S, X))
        print(f"spmm {name:10s} ours {t_o:7.3f} ms {g.nnz / t_o / 1e6:7.3f} G edges/s | vendor {t_v:7.3f} ms "
              f"{g.nnz / t_v / 1e6:7.3f} G edges/s | max |diff| {err:.2e}", flush=True)
        del X, S, ours, ref
    torch.manual_seed(0)
    for M, K in ((100_000, 1024), (200_000, 1024), (100_000, 2048)):
        N = 1024
        A = torch.randn(M, K, device=DEV)
        W = torch.randn(N, K, device=DEV) * 0.03
        b = torch.randn(N, device=DEV)
        flops = 2.0 * M * N * K
        t_o = bench(lambda: FC.fc_forward(A, W, None, None, b, True))
        t_v = bench(lambda: torch.relu(torch.nn.functional.linear(A, W, b)))
        print(f"fc fp32 [{M}x{K}]x[{K}x{N}]+relu ours(x3) {t_o:7.3f} ms {flops / t_o / 1e9:6.1f} TF/s | vendor fp32 "
              f"{t_v:7.3f} ms {flops / t_v / 1e9:6.1f} TF/s", flush=True)
        del A, W
    torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
