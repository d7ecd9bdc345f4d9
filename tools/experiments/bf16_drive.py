"""Run only the c5 bf16 GEMM kernels a few times -- a short program for rocprofv3 PMC passes:
'fc' = lpg_fc_bf16 (default variant) at M = 200K, N = 2048, K = 2048 + 2048 with ReLU,
'wg' = lpg_wgrad_bf16 at R = 200K, N = K = 2048,
'ig' / 'igm' = the two-part input gradient G1 W1 + G2 W2 at M = 200K, 2048 -> 2048, without / with the
folded ReLU backward of the producing layer (lpg_fc_bf16_relu_bwd)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lp-gnn_amd")]
import torch  # noqa: E402

from lpgnn.fc import fc_forward_bf16, input_grad_bf16, wgrad_bf16  # noqa: E402

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
elif what in ("ig", "igm"):
    G1 = torch.randn(M, 2048, device="cuda").to(BF)
    G2 = torch.randn(M, 2048, device="cuda").to(BF)
    W1 = torch.randn(2048, 2048, device="cuda") * 0.02
    W2 = torch.randn(2048, 2048, device="cuda") * 0.02
    Y = torch.randn(M, 2048, device="cuda").relu_().to(BF)
    mask = (Y, 1.0 / 0.9) if what == "igm" else None
    for _ in range(3):
        input_grad_bf16(G1, W1, G2, W2, mask=mask)
else:
    G = torch.randn(M, 2048, device="cuda").to(BF)
    X = torch.randn(M, 2048, device="cuda").relu_().to(BF)
    for _ in range(3):
        wgrad_bf16(G, X)
torch.cuda.synchronize()
print("done")
