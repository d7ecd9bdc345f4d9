"""Time the F = 8 (conv1 input) SpMM on the skewed LP (synth.skewed_lp, the bench's skewed sub-record graph)
and on the uniform c2 graph, with and without the narrow heavy-row units (median of HIP-event timings).

  python tools/experiments/narrow_skewed.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lp-gnn_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from lpgnn import BipartiteCSR, synth  # noqa: E402
from lpgnn.sparse import spmm_forward  # noqa: E402


def med(fn, reps=20):
    fn()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return float(np.median(ts))


dev = "cuda:0"
for name, g in (("skewed", synth.skewed_lp(100_000, 200_000, 2_000_000, a=1.5, seed=0)),
                ("c2", synth.uniform_lp(100_000, 200_000, 2_000_000, seed=0))):
    adj = BipartiteCSR.from_coo(g.row, g.col, g.val, g.m, g.n, device=dev)
    for d, csr in (("cons<-vars", adj.fwd), ("vars<-cons", adj.bwd)):
        for dt in (torch.float32, torch.bfloat16):
            x = torch.randn(csr.n_cols, 8, device=dev).to(dt)
            row = []
            for heavy in (1024, 0):
                row.append(med(lambda: spmm_forward(csr, x, heavy=heavy)))
            same = torch.equal(spmm_forward(csr, x, heavy=1024), spmm_forward(csr, x, heavy=0))
            print(f"{name:7s} {d:11s} {str(dt):15s} F=8  heavy units {row[0]:.4f} ms   FW-lane only {row[1]:.4f} ms"
                  f"   same bits {same}", flush=True)
