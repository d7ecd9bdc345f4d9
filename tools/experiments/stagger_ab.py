"""First-round stagger A/B of the one-tile GEMM grids (common.h stagger_params): the odd-XCD blocks of the
first round sleep S x 127 x 64 clocks, so half the chip's epilogues (HBM-bound when every CU stores at once)
run beside the other half's k loops.  c5 bf16 shapes (fc_bf16_p) and c2 f16x2 shapes (fc_x3_wide), with the
epilogues the steps use (addend, ReLU, dropout).  Interleaved rounds, median ms per launch.

  python tools/experiments/stagger_ab.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lp-gnn_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from lpgnn import fc as F  # noqa: E402

dev = "cuda:0"
torch.manual_seed(0)
bf, f32 = torch.bfloat16, torch.float32
STAG = [0, 2, 4, 8, 12]


def shapes():
    out = {}
    # c5: vars side (200K rows, K 2048, addend = the SpMM output, ReLU + dropout 0.1)
    A = torch.randn(200_000, 2048, device=dev).to(bf)
    W = (torch.randn(2048, 2048, device=dev) * 0.02).to(bf)
    b = torch.randn(2048, device=dev)
    C = torch.randn(200_000, 2048, device=dev).to(bf)
    out["bf16 200Kx2048 K2048 relu+add+drop"] = (
        "LPGNN_FC16_STAGGER",
        lambda: F.fc_forward_bf16(A, W, None, None, b, True, 0.1, 7, out=C, accumulate=True), 2 * 200e3 * 2048 * 2048)
    out["bf16 200Kx2048 K2048 plain"] = (
        "LPGNN_FC16_STAGGER", lambda: F.fc_forward_bf16(A, W, None, None, None, False), 2 * 200e3 * 2048 * 2048)
    A1 = torch.randn(100_000, 2048, device=dev).to(bf)
    A2 = torch.randn(100_000, 2048, device=dev).to(bf)
    out["bf16 100Kx2048 K4096 relu+drop"] = (
        "LPGNN_FC16_STAGGER", lambda: F.fc_forward_bf16(A1, W, A2, W, b, True, 0.1, 7), 2 * 100e3 * 2048 * 4096)
    # c2 f16x2: vars side (200K rows, K 1024, addend, ReLU + dropout), cons side (100K, K 2048)
    X = torch.randn(200_000, 1024, device=dev)
    Wf = torch.randn(1024, 1024, device=dev) * 0.03
    bf_ = torch.randn(1024, device=dev)
    Cf = torch.randn(200_000, 1024, device=dev)
    out["f16x2 200Kx1024 K1024 relu+add+drop"] = (
        "LPGNN_FCX3_STAGGER",
        lambda: F.fc_forward(X, Wf, None, None, bf_, True, 0.1, 7, out=Cf, accumulate=True, arith="f16x2"),
        3 * 2 * 200e3 * 1024 * 1024)
    X1 = torch.randn(100_000, 1024, device=dev)
    X2 = torch.randn(100_000, 1024, device=dev)
    out["f16x2 100Kx1024 K2048 relu+drop"] = (
        "LPGNN_FCX3_STAGGER", lambda: F.fc_forward(X1, Wf, X2, Wf, bf_, True, 0.1, 7, arith="f16x2"),
        3 * 2 * 100e3 * 1024 * 2048)
    return out


def main():
    sh = shapes()
    res = {(k, s): [] for k in sh for s in STAG}
    for k, (env, fn, _) in sh.items():
        fn()
    torch.cuda.synchronize()
    for rnd in range(5):
        for k, (env, fn, _) in sh.items():
            for s in STAG:
                os.environ[env] = str(s)
                fn()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(4):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                res[(k, s)].append(e0.elapsed_time(e1) / 4)
        os.environ.pop("LPGNN_FC16_STAGGER", None)
        os.environ.pop("LPGNN_FCX3_STAGGER", None)
    for k, (env, fn, flops) in sh.items():
        line = []
        for s in STAG:
            t = float(np.median(res[(k, s)]))
            line.append(f"S={s:2d}: {t:.4f} ms ({flops / t / 1e9 / 2500:.3f})")
        print(f"{k:38s} " + "  ".join(line), flush=True)


if __name__ == "__main__":
    main()
