"""Timing of the c2 backward GEMMs: x3 weight gradient / input gradient vs
hipBLASLt (torch), HIP events."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lp-gnn_amd")]
import torch  # noqa: E402

from tools.kbench import timeit  # noqa: E402

from lpgnn import _lib  # noqa: E402
from lpgnn.fc import input_grad, wgrad  # noqa: E402

L = _lib.lib()


def wg(v):
    def f():
        L.lpg_fc_x3_set_variant(v)
        return wgrad(G, X, arith="x3")
    return f

for R in (100_000, 200_000):
    G = torch.randn(R, 1024, device="cuda")
    X = torch.randn(R, 1024, device="cuda").relu_()
    W = torch.randn(1024, 1024, device="cuda") * 0.03
    fl = 2.0 * R * 1024 * 1024
    d = (wgrad(G, X, arith="x3") - G.t() @ X).abs().max().item()
    d16 = (wg(101)() - wg(100)()).abs().max().item()
    dc = (wg(102)() - wg(101)()).abs().max().item()
    print(f"R={R} max|coop - m16| = {dc:.3e}  pc == coop bitwise: {torch.equal(wg(103)(), wg(102)())}  "
          f"wide == coop: {torch.equal(wg(104)(), wg(102)())}  wide/sched == coop: {torch.equal(wg(105)(), wg(102)())}")
    t = timeit({"wgrad_x3_coop": wg(102), "wgrad_x3_wide": wg(104), "wgrad_x3_wsched": wg(105),
                "wgrad_torch": lambda: G.t() @ X,
                "igrad_x3": lambda: input_grad(G, W, arith="x3"), "igrad_torch": lambda: G @ W})
    for k, ms in t.items():
        print(f"R={R} {k:12s} {ms:.3f} ms {fl / ms / 1e9:.1f} TF/s", flush=True)
    print(f"R={R} wgrad max|x3 - torch| = {d:.3e}  max|m16 - m32| = {d16:.3e}")
    L.lpg_fc_x3_set_variant(102)
