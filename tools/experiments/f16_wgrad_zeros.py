"""The f16x2 weight gradient at the c2 shapes on random and on zero operands (power probe)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "lp-gnn_amd"))
from lpgnn import fc as F  # noqa: E402

DEV = "cuda:0"


def timed(fn, reps=20):
    for _ in range(5):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


for R in (100_000, 200_000):
    for zeros in (False, True):
        G = torch.randn(R, 1024, device=DEV)
        X = torch.relu(torch.randn(R, 1024, device=DEV))
        if zeros:
            G.zero_()
            X.zero_()
        F.colscale(G), F.colscale(X)  # (cached: the timed launches are the GEMM)
        t = timed(lambda: F.wgrad(G, X, arith="f16x2"))
        print(f"R={R} {'zeros ' if zeros else 'random'}: {t:7.1f} us  {2 * R * 1024 * 1024 * 3 / t / 1e9:6.1f} PF/s "
              "(f16 MFMA work)", flush=True)
