"""F = 1024 fp32 SpMM per direction on the skewed (Zipf 1.5) and uniform c2 graphs over the per-call tunings
(slice width x gather depth, lpg_spmm_f32_tuned; every choice the same bits): what bounds the skewed
vars<-cons direction, whose gathers hit a few hundred hot constraint rows in cache (PMC: 1.87 GB per launch
against 8.8 GB on the uniform graph).

  python tools/experiments/spmm_skewed_sweep.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lp-gnn_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from lpgnn import BipartiteCSR, synth  # noqa: E402
from lpgnn.sparse import spmm_forward  # noqa: E402


def med(fn, reps=15):
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
        x = torch.randn(csr.n_cols, 1024, device=dev)
        ref = spmm_forward(csr, x)
        res = []
        for sl in (0, 128, 256, 512, 1024):
            for dp in (8, 16, 32):
                if sl in (128,) and dp == 32:
                    continue
                for heavy in ((1024, 0) if sl in (0, 256, 512) else (0,)):
                    try:
                        t = med(lambda: spmm_forward(csr, x, slice_cols=sl, depth=dp, heavy=heavy))
                    except RuntimeError as e:
                        continue
                    same = torch.equal(spmm_forward(csr, x, slice_cols=sl, depth=dp, heavy=heavy), ref)
                    res.append((t, sl, dp, heavy, same))
        res.sort()
        t0 = med(lambda: spmm_forward(csr, x))
        print(f"{name:7s} {d:11s} default {t0:.4f} ms; best:", flush=True)
        for t, sl, dp, hv, same in res[:6]:
            print(f"    slice {sl:4d} depth {dp:2d} heavy {hv:4d}: {t:.4f} ms  same bits {same}", flush=True)
