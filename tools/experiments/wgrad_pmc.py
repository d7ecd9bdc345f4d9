"""x3 weight gradient at R = 100K, 1024 x 1024, a few launches, for rocprofv3 --pmc passes of the
kernel LPGNN_WGRAD_KERNEL selects (tools/experiments/gpu_r03q3.sh)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lp-gnn_amd")]
import torch  # noqa: E402

from lpgnn.fc import wgrad  # noqa: E402

torch.manual_seed(0)
G = torch.randn(100_000, 1024, device="cuda")
X = torch.randn(100_000, 1024, device="cuda").relu_()
for _ in range(4):
    wgrad(G, X, arith="x3")
torch.cuda.synchronize()
print("done")
