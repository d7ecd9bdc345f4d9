"""A/B of the x3 FC kernels at the c2 shapes: fc_fwd_x3_16 (variant 0) vs the
wide-strip kernels (variants 12-15).  Every variant's C must equal variant 0's
bit for bit (same MFMA shape, k order and product sequence); prints ms and TF/s
(fp32-equivalent: 2 M N K).

  LPG_X3V=0,12,13,14,15 python tools/experiments/exp_wide.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lp-gnn_amd")]
import torch  # noqa: E402

from tools.kbench import timeit  # noqa: E402

from lpgnn import _lib  # noqa: E402
from lpgnn.fc import fc_forward  # noqa: E402

L = _lib.lib()
torch.manual_seed(0)
variants = [int(v) for v in os.environ.get("LPG_X3V", "0,12,13,14,15").split(",")]
shapes = [(200_000, 1024, 1024, True), (200_000, 1024, 0, False), (100_000, 1024, 1024, True),
          (100_000, 1024, 0, False)]
for M, K1, K2, relu in shapes:
    A1 = torch.randn(M, K1, device="cuda").relu_()
    A2 = torch.randn(M, K2, device="cuda").relu_() if K2 else None
    W1 = torch.randn(1024, K1, device="cuda") * 0.03
    W2 = torch.randn(1024, K2, device="cuda") * 0.03 if K2 else None
    b = torch.randn(1024, device="cuda") * 0.1
    flops = 2.0 * M * 1024 * (K1 + K2)

    def run(v):
        def f():
            L.lpg_fc_x3_set_variant(v)
            return fc_forward(A1, W1, A2, W2, b, relu, arith="x3")
        return f
    fns = {f"v{v}": run(v) for v in variants}
    ref = fns[f"v{variants[0]}"]()
    for k, f in fns.items():
        y = f()
        print(f"M={M} K={K1}+{K2} {k:5s} bitwise_equal_to_{variants[0]}={torch.equal(y, ref)} "
              f"maxdiff={(y - ref).abs().max().item():.3e}", flush=True)
    t = timeit(fns)
    for k, ms in t.items():
        print(f"M={M} K={K1}+{K2} {k:5s} {ms:.3f} ms {flops / ms / 1e9:.1f} TF/s", flush=True)
    L.lpg_fc_x3_set_variant(0)
    del A1, A2, ref
    torch.cuda.empty_cache()
