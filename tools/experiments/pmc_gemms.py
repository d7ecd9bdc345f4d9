"""The hidden-width GEMMs at their in-step shapes, a few launches each, for rocprofv3 --pmc passes
(tools/pmc_round.sh): x3 FC (200K x 1024 x 1024, and the ReLU + dropout + accumulate epilogue),
x3 weight gradient (R = 100K, 1024 x 1024), bf16 FC (200K x 2048 x 2048, ReLU + dropout),
bf16 weight gradient (R = 100K, 2048 x 2048)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lp-gnn_amd")]

import torch  # noqa: E402

from lpgnn.fc import fc_forward, fc_forward_bf16, wgrad, wgrad_bf16  # noqa: E402

torch.manual_seed(0)
BF = torch.bfloat16
A = torch.randn(200_000, 1024, device="cuda")
W = torch.randn(1024, 1024, device="cuda") * 0.03
b = torch.randn(1024, device="cuda")
P = torch.randn(200_000, 1024, device="cuda")
G = torch.randn(100_000, 1024, device="cuda")
X = torch.randn(100_000, 1024, device="cuda")
for _ in range(3):
    fc_forward(A, W, None, None, None, False, arith="x3")
    fc_forward(A, W, None, None, b, True, 0.1, 7, out=P, accumulate=True, arith="x3")
    wgrad(G, X, arith="x3")
torch.cuda.synchronize()
del A, W, P, G, X
Ab = torch.randn(200_000, 2048, device="cuda").to(BF)
Wb = (torch.randn(2048, 2048, device="cuda") * 0.02).to(BF)
b2 = torch.randn(2048, device="cuda")
Gb = torch.randn(100_000, 2048, device="cuda").to(BF)
Xb = torch.randn(100_000, 2048, device="cuda").to(BF)
for _ in range(3):
    fc_forward_bf16(Ab, Wb, None, None, b2, True, 0.1, 7)
    wgrad_bf16(Gb, Xb)
torch.cuda.synchronize()
print("done")
