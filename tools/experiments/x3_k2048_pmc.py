"""x3 FC at the verdict's K = 2048 shape (M = 200 K, K = 1024 + 1024, N = 1024, ReLU), a few
launches, for rocprofv3 --pmc passes (past-L2 bytes, MFMA busy, clock).  X3_KERNEL = the per-call
kernel choice (LPG_FC_KERNEL: 0 default, 2 = round 3's m-major tile order); X3_M = the rows (default
200 000; 128 = one m-tile, the calibration of FETCH_SIZE for the W planes' 64-byte row segments)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lp-gnn_amd")]
import torch  # noqa: E402

from lpgnn.fc import fc_forward  # noqa: E402

torch.manual_seed(0)
M = int(os.environ.get("X3_M", "200000"))  # X3_M=128: one m-tile, every W plane byte read by one block
A1 = torch.randn(M, 1024, device="cuda")
A2 = torch.randn(M, 1024, device="cuda")
W1 = torch.randn(1024, 1024, device="cuda") * 0.03
W2 = torch.randn(1024, 1024, device="cuda") * 0.03
b = torch.randn(1024, device="cuda")
kern = int(os.environ.get("X3_KERNEL", "0"))
for _ in range(4):
    fc_forward(A1, W1, A2, W2, b, True, arith="x3", kernel=kern)
torch.cuda.synchronize()
print("done")
