"""What bounds the x3 weight gradient: the x3 GEMM issues 6 bf16 MFMA products per
fp32 product, so a pre-split form (operands as three bf16 planes, no split VALU in the loop) can at best
run its MFMA work at the rate the plain bf16 weight gradient (wgrad_bf16: staged bf16 operands, no VALU
beside the MFMAs) reaches on the same shapes.  Times, at the c2 shapes (R = 100 K / 200 K, N = K = 1024):
  x3 wgrad (lpg_wgrad_x3_f32) on random and on all-zero operands (the clock the chip holds: DVFS),
  bf16 wgrad (lpg_wgrad_bf16) on random and zero operands,
and prints TF/s fp32-equivalent (x3) and bf16 TF/s (x3 x 6 = its bf16 MFMA work)."""
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
        for fill in ("random", "zeros"):
            if fill == "random":
                G, X = torch.randn(R, N, device=DEV) * 1e-3, torch.randn(R, K, device=DEV)
            else:
                G, X = torch.zeros(R, N, device=DEV), torch.zeros(R, K, device=DEV)
            ms = bench(lambda: F.wgrad(G, X, arith="x3"))
            print(f"x3   wgrad R={R} {fill:6s} {ms:7.3f} ms  {flops / ms / 1e9:6.1f} TF/s fp32-equiv  "
                  f"{6 * flops / ms / 1e9:7.1f} TF/s bf16 MFMA work", flush=True)
            Gb, Xb = G.to(torch.bfloat16), X.to(torch.bfloat16)
            ms = bench(lambda: F.wgrad_bf16(Gb, Xb))
            print(f"bf16 wgrad R={R} {fill:6s} {ms:7.3f} ms  {flops / ms / 1e9:7.1f} TF/s bf16 "
                  f"(x3 bound if pre-split: {flops / ms / 1e9 / 6:6.1f} TF/s fp32-equiv)", flush=True)
            del G, X, Gb, Xb
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
