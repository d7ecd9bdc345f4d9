"""What each epilogue component costs on the 200K-row GEMMs of the c2 (f16x2, fc_x3_wide) and c5 (bf16,
fc_bf16_p) steps: plain / + bias / + addend / + ReLU / + dropout, one at a time (interleaved rounds, median
ms per launch; the fraction of 2.5 PF counts the matrix-core products).

  python tools/experiments/epi_cost.py
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


def cases():
    out = {}
    X = torch.randn(200_000, 1024, device=dev)
    W = torch.randn(1024, 1024, device=dev) * 0.03
    b = torch.randn(1024, device=dev)
    C = torch.randn(200_000, 1024, device=dev)
    fl = 3 * 2 * 200e3 * 1024 * 1024

    def f(**k):
        return F.fc_forward(X, W, None, None, k.get("b"), k.get("relu", False), k.get("p", 0.0), 7, out=C,
                            accumulate=k.get("acc", False), arith="f16x2")
    out["f16x2 plain"] = (lambda: f(), fl)
    out["f16x2 +bias"] = (lambda: f(b=b), fl)
    out["f16x2 +bias+relu"] = (lambda: f(b=b, relu=True), fl)
    out["f16x2 +bias+relu+drop"] = (lambda: f(b=b, relu=True, p=0.1), fl)
    out["f16x2 +bias+add"] = (lambda: f(b=b, acc=True), fl)
    out["f16x2 +bias+add+relu+drop"] = (lambda: f(b=b, relu=True, p=0.1, acc=True), fl)
    A = torch.randn(200_000, 2048, device=dev).to(torch.bfloat16)
    Wb = (torch.randn(2048, 2048, device=dev) * 0.02).to(torch.bfloat16)
    bb = torch.randn(2048, device=dev)
    Cb = torch.randn(200_000, 2048, device=dev).to(torch.bfloat16)
    flb = 2 * 200e3 * 2048 * 2048

    def g(**k):
        return F.fc_forward_bf16(A, Wb, None, None, k.get("b"), k.get("relu", False), k.get("p", 0.0), 7, out=Cb,
                                 accumulate=k.get("acc", False))
    out["bf16 plain"] = (lambda: g(), flb)
    out["bf16 +bias"] = (lambda: g(b=bb), flb)
    out["bf16 +bias+relu"] = (lambda: g(b=bb, relu=True), flb)
    out["bf16 +bias+relu+drop"] = (lambda: g(b=bb, relu=True, p=0.1), flb)
    out["bf16 +bias+add"] = (lambda: g(b=bb, acc=True), flb)
    out["bf16 +bias+add+relu+drop"] = (lambda: g(b=bb, relu=True, p=0.1, acc=True), flb)
    return out


def main():
    cs = cases()
    res = {k: [] for k in cs}
    for fn, _ in cs.values():
        fn()
    torch.cuda.synchronize()
    for _ in range(5):
        for k, (fn, _) in cs.items():
            fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(4):
                fn()
            e1.record()
            torch.cuda.synchronize()
            res[k].append(e0.elapsed_time(e1) / 4)
    for k, (fn, fl) in cs.items():
        t = float(np.median(res[k]))
        print(f"{k:28s} {t:.4f} ms  {fl / t / 1e9 / 2500:.3f} of 2.5 PF", flush=True)


if __name__ == "__main__":
    main()
