"""Diagnostic for VERDICT r02 item 1: which bf16 FC tile variant differs, where, and which one
matches an fp64 evaluation of the same bf16 operands.  Run once per library build
(LPGNN_LIB=... selects it); prints one line per (shape, variant) with the mismatch count against
variant 0 and against the fp64-rounded reference, run-to-run stability, and the first few
differing (row, col) elements."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "lp-gnn_amd"))
from lpgnn import _lib  # noqa: E402
from lpgnn.fc import fc_forward_bf16  # noqa: E402

BF = torch.bfloat16
DEV = "cuda:0"
print("lib:", _lib.LIB_PATH, flush=True)
L = _lib.lib()
shapes = [(129, 130, 64, False, True), (5000, 1024, 1024, True, True), (4099, 264, 128, True, False),
          (129, 136, 64, False, True), (300, 130, 128, False, True)]
for (M, N, K, relu, bias) in shapes:
    g = torch.Generator().manual_seed(M + N + K)
    A = torch.randn(M, K, generator=g).to(BF).to(DEV)
    W = (torch.randn(N, K, generator=g) * 0.05).to(BF).to(DEV)
    P = torch.randn(M, N, generator=g).to(BF).to(DEV)
    b = (torch.randn(N, generator=g) * 0.1).to(DEV) if bias else None
    ref = A.double() @ W.double().t() + P.double() + (b.double() if bias else 0.0)
    if relu:
        ref = ref.clamp_min(0)
    ref16 = ref.float().to(BF)  # one rounding from (near-)exact; double rounding possible but rare
    outs = {}
    for v in (0, 1, 2, 4, 5, 6, 7, 8, 9, 10):
        reps = []
        for rep in range(3):
            L.lpg_fc_bf16_set_variant(v)
            out = P.clone()
            fc_forward_bf16(A, W, None, None, b, relu, out=out, accumulate=True)
            torch.cuda.synchronize()
            reps.append(out.clone())
        L.lpg_fc_bf16_set_variant(0)
        outs[v] = reps[0]
        stable = all(torch.equal(reps[0], r) for r in reps[1:])
        d0 = (reps[0] != outs[0]).nonzero()
        dr = (reps[0] != ref16).nonzero()
        line = f"M={M} N={N} K={K} v={v}: stable={stable} diff_v0={d0.shape[0]} diff_ref={dr.shape[0]}"
        if d0.shape[0]:
            pts = []
            for (r, c) in d0[:6].tolist():
                pts.append(f"({r},{c}) v{v}={reps[0][r, c].item():.6g} v0={outs[0][r, c].item():.6g} "
                           f"f64={ref[r, c].item():.8g}")
            line += " | " + "; ".join(pts)
            rows = d0[:, 0].unique().tolist()
            cols = d0[:, 1].unique().tolist()
            line += f" | rows {rows[:12]}{'...' if len(rows) > 12 else ''} cols {cols[:12]}{'...' if len(cols) > 12 else ''}"
        if not stable:
            for k, r in enumerate(reps[1:]):
                dd = (reps[0] != r).nonzero()
                line += f" | rep{k + 1} differs at {dd.shape[0]} elems, first {dd[:4].tolist()}"
        print(line, flush=True)
