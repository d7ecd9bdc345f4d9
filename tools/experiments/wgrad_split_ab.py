"""The f16x2 / x3 weight gradient's R-split at the c2 shapes (N = K = 1024, R = 100 K / 200 K).  The round-6
A/B (profiles/r06_wgrad_split_ab.log) ran it once per block target with a temporary LPGNN_WGRAD_TARGET read in
csrc/fc_x3.hip wgrad_splits; that hook is gone (the split is a function of the shape and the CU count only),
so the script now times the shipped rule.
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
res = []
for R in (100_000, 200_000):
    G = torch.randn(R, 1024, device=dev)
    X = torch.randn(R, 1024, device=dev)
    F.wgrad(G, X, arith="f16x2")
    torch.cuda.synchronize()
    ts = []
    for _ in range(7):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(4):
            F.wgrad(G, X, arith="f16x2")
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / 4)
    t = float(np.median(ts))
    res.append(f"R={R}: {t:.4f} ms ({3 * 2 * R * 1024 * 1024 / t / 1e9 / 2500:.3f} of 2.5 PF)")
print("  ".join(res), flush=True)
