"""Per-call time of the heads' fused ReLU backward (lpg_heads_relu_bwd_f32 and its f16x2-scales form) at the
c2 shapes, with whatever library LPGNN_LIB names (rows-per-block A/B builds: -DLPG_HEADS_RB=64)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "lp-gnn_amd"))
from lpgnn import fc as F  # noqa: E402

DEV = "cuda:0"


def timed(fn, reps=30):
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


def main():
    torch.manual_seed(0)
    for M in (100_000, 200_000):
        Y = torch.relu(torch.randn(M, 1024, device=DEV))
        G = torch.randn(M, 3, device=DEV)
        W = torch.randn(3, 1024, device=DEV)
        t0 = timed(lambda: F.heads_relu_bwd(G, W, Y, 1.0, True))
        t1 = timed(lambda: F.heads_relu_bwd(G, W, Y, 1.0, True, arith="f16x2"))
        gb = 2 * M * 1024 * 4 / 1e9
        print(f"M={M}: plain {t0:7.1f} us ({gb / t0 * 1e3:.2f} TB/s)   with scales {t1:7.1f} us ({gb / t1 * 1e3:.2f} TB/s)",
              flush=True)


if __name__ == "__main__":
    main()
