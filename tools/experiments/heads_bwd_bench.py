"""The fused heads + ReLU backward (lpg_heads_relu_bwd_f32 / _scales_f32, csrc/bwd.hip heads_bwd_p1) at the
c2 shapes: M = 100 K / 200 K rows, K = 1024, N = 3 heads; with and without the f16x2 scales (the SC form the
c2 step runs).  Median ms per call and the HBM rate of its compulsory bytes (read Y, write dZ).

  python tools/experiments/heads_bwd_bench.py
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
for M in (100_000, 200_000):
    Y = torch.relu(torch.randn(M, 1024, device=dev))
    G = torch.randn(M, 3, device=dev)
    W = torch.randn(3, 1024, device=dev)
    for arith in (None, "f16x2"):
        f = lambda: F.heads_relu_bwd(G, W, Y, 1.1, True, arith=arith)  # noqa: E731
        f()
        torch.cuda.synchronize()
        ts = []
        for _ in range(7):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                f()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / 5)
        t = float(np.median(ts))
        print(f"M={M} {'scales' if arith else 'plain '}: {t:.4f} ms  {2 * M * 1024 * 4 / t / 1e9:.2f} TB/s", flush=True)
    # the same bytes through torch's elementwise kernel (read Y, write Z): what a plain stream reaches here
    Z = torch.empty_like(Y)
    torch.mul(Y, 1.1, out=Z)
    torch.cuda.synchronize()
    ts = []
    for _ in range(7):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            torch.mul(Y, 1.1, out=Z)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / 5)
    t = float(np.median(ts))
    print(f"M={M} torch mul (read + write): {t:.4f} ms  {2 * M * 1024 * 4 / t / 1e9:.2f} TB/s", flush=True)
