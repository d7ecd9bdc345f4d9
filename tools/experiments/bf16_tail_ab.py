"""The bf16 FC's partial last round at the c5 shapes: per-call kernel choice 0 (the whole 256 x 256 rounds,
then the partial last round as a second launch on 128 x 128 tiles) against 8 (fc_bf16_pt: the last round's
rows as 128 x 256 tiles on the first block ids of the same launch).  Forward forms (ReLU, addend, dropout)
and the folded ReLU backward (mask bits in, bias column sums out).  Interleaved rounds, median ms per call,
the fraction of 2.5 PF, and whether both wrote the same bits.

  python tools/experiments/bf16_tail_ab.py

Choice 8 existed only in the A/B builds (profiles/r06_bf16_tail_ab.log); the shipped library rejects it.
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
CHOICES = (0, 8)


def run(name, call, fl, outs_of):
    outs = {}
    for c in CHOICES:
        outs[c] = outs_of(call(c))
    same = all(all(torch.equal(x, y) for x, y in zip(outs[0], outs[c])) for c in CHOICES)
    ts = {c: [] for c in CHOICES}
    torch.cuda.synchronize()
    for _ in range(5):
        for c in CHOICES:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(4):
                call(c)
            e1.record()
            torch.cuda.synchronize()
            ts[c].append(e0.elapsed_time(e1) / 4)
    row = "  ".join(f"k{c}: {np.median(ts[c]):.4f} ms ({fl / np.median(ts[c]) / 1e9 / 2500:.3f})" for c in CHOICES)
    print(f"{name}: {row}  same bits: {same}", flush=True)


N = 2048
for M, K, acc, p in ((200_000, 2048, True, 0.1), (200_000, 2048, False, 0.0), (100_000, 4096, False, 0.1),
                     (100_000, 2048, False, 0.0)):
    A = torch.randn(M, K, device=dev).to(torch.bfloat16)
    W = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
    b = torch.randn(N, device=dev)
    C0 = torch.randn(M, N, device=dev).to(torch.bfloat16)
    mo = torch.empty(M, N // 8, device=dev, dtype=torch.uint8)

    def fwd(c, A=A, W=W, b=b, C0=C0, acc=acc, p=p, mo=mo):
        o = C0.clone() if acc else torch.empty_like(C0)
        F.fc_forward_bf16(A, W, None, None, b, True, p, 7, out=o, accumulate=acc, kernel=c, mask_out=mo)
        return o, mo.clone()
    run(f"fwd M={M} K={K} {'add ' if acc else ''}{'drop' if p else ''}", fwd, 2 * M * N * K, lambda r: r)
# the folded ReLU backward: dZ = (bits) ? bf16(G W * scale) : 0 with the bias column sums
for M in (200_000, 100_000):
    G = torch.randn(M, N, device=dev).to(torch.bfloat16)
    W = (torch.randn(N, N, device=dev) * 0.02).to(torch.bfloat16)
    bits = torch.randint(0, 256, (M, N // 8), device=dev, dtype=torch.uint8)

    def bwd(c, G=G, W=W, bits=bits):
        db = torch.empty(N, device=dev)
        o = F.fc_forward_bf16(G, W, None, None, None, False, kernel=c, mask=(bits, 1.25), db_out=db)
        return o, db
    run(f"relu-bwd M={M} K={N}", bwd, 2 * M * N * N, lambda r: r)
