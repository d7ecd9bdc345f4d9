"""Run only the c5 bf16 GEMM kernels a few times -- a short program for rocprofv3 PMC passes:
'fc' = lpg_fc_bf16 (default variant) at M = 200K, N = 2048, K = 2048 + 2048 with ReLU,
'wg' = lpg_wgrad_bf16 at R = 200K, N = K = 2048."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lp-gnn_amd")]
import torch  # noqa: E402

from lpgnn.fc import fc_forward_bf16, wgrad_bf16  # noqa: E402

what = sys.argv[1] if len(sys.argv) > 1 else "fc"
BF = torch.bfloat16
M = 200_000
if what == "fc":
    A1 = torch.randn(M, 2048, device="cuda").relu_().to(BF)
    A2 = torch.randn(M, 2048, device="cuda").relu_().to(BF)
    W1 = (torch.randn(2048, 2048, device="cuda") * 0.02).to(BF)
    W2 = (torch.randn(2048, 2048, device="cuda") * 0.02).to(BF)
    b = torch.randn(2048, device="cuda")
    for _ in range(3):
        fc_forward_bf16(A1, W1, A2, W2, b, True)
else:
    G = torch.randn(M, 2048, device="cuda").to(BF)
    X = torch.randn(M, 2048, device="cuda").relu_().to(BF)
    for _ in range(3):
        wgrad_bf16(G, X)
torch.cuda.synchronize()
print("done")
