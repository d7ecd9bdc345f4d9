"""Per-call time of the plain f16x2 FC at the c2 shapes with whatever library LPGNN_LIB names (block-shape
A/B builds), and its error against fp64 on 2000 sampled rows.  Round 5: an 8-wave 256 x 128 block (one
per CU) measured 7-8 % slower than the default 4-wave 128 x 128 (two per CU) -- profiles/r05_f16_fc_ab.log"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "lp-gnn_amd"))
from lpgnn import fc as F  # noqa: E402

DEV = "cuda:0"
KERNELS = [int(k) for k in os.environ.get("F16_FC_KERNELS", "").split(",") if k]  # LPG_FC_KERNEL choices (tile order)


def timed(fn, reps=20):
    for _ in range(3):
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
    for M, K1, K2 in [(100_000, 1024, 0), (200_000, 1024, 0), (100_000, 1024, 1024)]:
        A1 = torch.randn(M, K1, device=DEV)
        A2 = torch.randn(M, K2, device=DEV) if K2 else None
        if os.environ.get("F16_FC_ZEROS"):  # power probe: zero activations (the same instructions, no toggling)
            A1.zero_()
            if A2 is not None:
                A2.zero_()
        W1 = torch.randn(1024, K1, device=DEV) * 0.03
        W2 = torch.randn(1024, K2, device=DEV) * 0.03 if K2 else None
        C = torch.empty(M, 1024, device=DEV)
        for kern in KERNELS:
            run = lambda: F.fc_forward(A1, W1, A2, W2, None, False, out=C, arith="f16x2", kernel=kern)  # noqa: E731
            t = timed(run)
            print(f"M={M} K={K1 + K2} kernel {kern}: {t:8.1f} us", flush=True)
        run = lambda: F.fc_forward(A1, W1, A2, W2, None, False, out=C, arith="f16x2")  # noqa: E731
        t = timed(run)
        run()
        idx = torch.randint(0, M, (2000,), device=DEV)
        ref = A1[idx].double() @ W1.double().T
        den = A1[idx].double().abs() @ W1.double().abs().T
        if K2:
            ref += A2[idx].double() @ W2.double().T
            den += A2[idx].double().abs() @ W2.double().abs().T
        err = float(((C[idx].double() - ref).abs() / den).max())
        fl = 2 * M * 1024 * (K1 + K2) * 3
        print(f"M={M} K={K1 + K2}: {t:8.1f} us  {fl / t / 1e9:7.1f} PF/s (f16 MFMA work)  err {err:.2e}", flush=True)


if __name__ == "__main__":
    main()
