"""A/B of lpg_fc_f32 arithmetic: exact fp32 MFMA vs the three-way bf16 split
(flag 4), at the c2 hidden-layer shapes: time (HIP events) and error vs an
fp64 GEMM of the same operands."""
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
variants = [int(v) for v in os.environ.get("LPG_X3V", "0,1,2").split(",")]
for M, K1, K2 in ((200_000, 1024, 1024), (200_000, 1024, 0), (100_000, 1024, 0)):
    A1 = torch.randn(M, K1, device="cuda").relu_()
    A2 = torch.randn(M, K2, device="cuda").relu_() if K2 else None
    W1 = torch.randn(1024, K1, device="cuda") * 0.03
    W2 = torch.randn(1024, K2, device="cuda") * 0.03 if K2 else None
    b = torch.randn(1024, device="cuda") * 0.1
    flops = 2.0 * M * 1024 * (K1 + K2)
    rows = slice(0, 4096)
    ref = A1[rows].double() @ W1.double().t() + b.double()
    if K2:
        ref += A2[rows].double() @ W2.double().t()
    ref = ref.relu()
    absref = (A1[rows].double().abs() @ W1.double().abs().t())
    if K2:
        absref += A2[rows].double().abs() @ W2.double().abs().t()

    def run(arith, v):
        def f():
            L.lpg_fc_x3_set_variant(v)
            return fc_forward(A1, W1, A2, W2, b, True, arith=arith)
        return f
    fns = {"fp32": run("fp32", 0)}
    for v in variants:
        fns[f"x3v{v}"] = run("x3", v)
    for k, f in fns.items():
        y = f()[rows].double()
        e = (y - ref).abs()
        print(f"M={M} K={K1}+{K2} {k:8s} maxerr={e.max().item():.3e} meanerr={e.mean().item():.3e} "
              f"max_rel_to_abs={(e / absref.clamp_min(1e-30)).max().item():.3e}", flush=True)
    tl = {}
    if K2:
        fns["torch"] = lambda: torch.relu(torch.addmm(b, A1, W1.t()).addmm_(A2, W2.t()))
    else:
        fns["torch"] = lambda: torch.relu(torch.addmm(b, A1, W1.t()))
    t = timeit(fns)
    L.lpg_fc_x3_set_variant(0)
    for k, ms in t.items():
        print(f"M={M} K={K1}+{K2} {k:8s} {ms:.3f} ms {flops / ms / 1e9:.1f} TF/s", flush=True)
    del A1, A2
    torch.cuda.empty_cache()
