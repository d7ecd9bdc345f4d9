"""The f16x2 GEMMs at their c2 in-step shapes, a few launches each, for rocprofv3 --pmc passes
(tools/experiments/f16x2_pmc.sh): plain FC 100K x 1024 x 1024, ReLU + accumulate FC 200K x 1024 x 1024,
weight gradient R = 100K, 1024 x 1024.  Operand scales are computed before the timed launches (cached)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lp-gnn_amd")]

import torch  # noqa: E402

from lpgnn.fc import fc_forward, wgrad  # noqa: E402

torch.manual_seed(0)
A = torch.randn(100_000, 1024, device="cuda")
W = torch.randn(1024, 1024, device="cuda") * 0.03
b = torch.randn(1024, device="cuda")
A2 = torch.randn(200_000, 1024, device="cuda")
P = torch.randn(200_000, 1024, device="cuda")
G = torch.randn(100_000, 1024, device="cuda")
for _ in range(3):
    fc_forward(A, W, None, None, None, False, arith="f16x2")
    fc_forward(A2, W, None, None, b, True, 0.1, 7, out=P, accumulate=True, arith="f16x2")
    wgrad(G, A, arith="f16x2")
torch.cuda.synchronize()
print("done")
