"""The vendor GEMM (hipBLASLt through torch.mm) on the weight-gradient shapes dZ^T X of the c2 step
(R = 100 K / 200 K rows, N = K = 1024) in bf16 and fp32, beside our kernels (lpg_wgrad_bf16,
lpg_wgrad_x3_f32): what rate the chip gives a tuned library on the long-R reduction shape."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "lp-gnn_amd"))
from lpgnn import fc as F  # noqa: E402

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
    torch.manual_seed(0)
    for R in (100_000, 200_000):
        N = K = 1024
        flops = 2.0 * R * N * K
        G32 = torch.randn(R, N, device=DEV)
        X32 = torch.randn(R, K, device=DEV)
        Gb, Xb = G32.to(torch.bfloat16), X32.to(torch.bfloat16)
        rows = [("vendor bf16 torch.mm(G^T, X)", lambda: torch.mm(Gb.t(), Xb)),
                ("ours wgrad_bf16", lambda: F.wgrad_bf16(Gb, Xb)),
                ("vendor fp32 torch.mm(G^T, X)", lambda: torch.mm(G32.t(), X32)),
                ("ours wgrad_x3 (fp32)", lambda: F.wgrad(G32, X32))]
        for name, fn in rows:
            ms = bench(fn)
            print(f"R={R:7d} {name:32s} {ms:8.3f} ms {flops / ms / 1e9:8.1f} TF/s", flush=True)
        del G32, X32, Gb, Xb
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
