"""conv1's streaming small-K FC at the c5 / fp16-inference shapes (csrc/fc_bf16.hip fc_smallk_bf16):
M = 100 K / 200 K rows, K = 8 + 8 LP features, N = 2048 (c5, bf16, with and without the 1-bit ReLU mask
output) and N = 1024 (fp16).  Median ms per call and the output write rate.

  python tools/experiments/smallk_bf16_bench.py
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


def timed(f):
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
    return float(np.median(ts))


for dt, N in ((torch.bfloat16, 2048), (torch.float16, 1024)):
    for M in (100_000, 200_000):
        A1 = torch.randn(M, 8, device=dev).to(dt)
        A2 = torch.randn(M, 8, device=dev).to(dt)
        W1 = (torch.randn(N, 8, device=dev) * 0.3).to(dt)
        W2 = (torch.randn(N, 8, device=dev) * 0.3).to(dt)
        b = torch.randn(N, device=dev)
        out = torch.empty(M, N, device=dev, dtype=dt)
        mo = torch.empty(M, N // 8, device=dev, dtype=torch.uint8)
        t = timed(lambda: F.fc_forward_bf16(A1, W1, A2, W2, b, True, out=out))
        line = f"{str(dt)[6:]:9s} M={M} N={N}: {t:.4f} ms ({M * N * out.element_size() / t / 1e9:.2f} TB/s)"
        if dt == torch.bfloat16:
            tm = timed(lambda: F.fc_forward_bf16(A1, W1, A2, W2, b, True, out=out, mask_out=mo))
            line += f"  +mask {tm:.4f} ms ({M * N * (out.element_size() + 1 / 8) / tm / 1e9:.2f} TB/s)"
        print(line, flush=True)
