"""The f16x2 / x3 weight gradient's R-split (wgrad_splits' block target, LPGNN_WGRAD_TARGET, read once per
process) at the c2 shapes: run once per target value, e.g.

  for t in 1024 2048 4096; do LPGNN_WGRAD_TARGET=$t python tools/experiments/wgrad_split_ab.py; done
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
print(f"target {os.environ.get('LPGNN_WGRAD_TARGET', '2048')}: " + "  ".join(res), flush=True)
