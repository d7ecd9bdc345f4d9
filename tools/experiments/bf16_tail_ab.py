"""The bf16 FC's partial last round (c5 shapes): per-call kernel choices 0 (the default: 256 x 256 rounds,
the partial last round on 128 x 128 tiles), 8 (the same with the last round on the 4-wave 128 x 256
pipelined form) and 9 (that form for the whole call).  Interleaved rounds, median ms per call, the
fraction of 2.5 PF, and whether every choice wrote the same bits.

  python tools/experiments/bf16_tail_ab.py

Choices 8 and 9 existed only in the A/B build (profiles/r06_bf16_tail_ab.log); the library rejects them now.
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
CHOICES = (0, 8, 9)
for M, K, acc, p in ((200_000, 2048, True, 0.1), (200_000, 2048, False, 0.0), (100_000, 4096, False, 0.1),
                     (100_000, 2048, False, 0.0)):
    N = 2048
    A = torch.randn(M, K, device=dev).to(torch.bfloat16)
    W = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
    b = torch.randn(N, device=dev)
    C0 = torch.randn(M, N, device=dev).to(torch.bfloat16)
    outs, ts = {}, {c: [] for c in CHOICES}
    for c in CHOICES:
        o = C0.clone()
        F.fc_forward_bf16(A, W, None, None, b, True, p, 7, out=o, accumulate=acc, kernel=c)
        outs[c] = o
    same = all(torch.equal(outs[0], outs[c]) for c in CHOICES)
    o = C0.clone()
    torch.cuda.synchronize()
    for _ in range(5):
        for c in CHOICES:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(4):
                F.fc_forward_bf16(A, W, None, None, b, True, p, 7, out=o, accumulate=acc, kernel=c)
            e1.record()
            torch.cuda.synchronize()
            ts[c].append(e0.elapsed_time(e1) / 4)
    fl = 2 * M * N * K
    row = "  ".join(f"k{c}: {np.median(ts[c]):.4f} ms ({fl / np.median(ts[c]) / 1e9 / 2500:.3f})" for c in CHOICES)
    print(f"M={M} K={K} {'add ' if acc else ''}{'drop' if p else ''}: {row}  same bits: {same}", flush=True)
