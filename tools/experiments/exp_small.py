"""Timing of the streaming backward kernels at c2 shapes (heads backward fused with the
ReLU mask, conv1 weight gradient, heads forward) -- A/B of builds via LPGNN_LIB."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lp-gnn_amd")]
import torch  # noqa: E402

from tools.kbench import timeit  # noqa: E402

from lpgnn import fc as _fc  # noqa: E402

M, K = 200_000, 1024
Y = torch.randn(M, K, device="cuda").relu_()
G = torch.randn(M, 3, device="cuda")
W = torch.randn(3, K, device="cuda")
g = torch.randn(M, K, device="cuda")
A1 = torch.randn(M, 8, device="cuda")
A2 = torch.randn(M, 8, device="cuda")
b = torch.randn(3, device="cuda")
t = timeit({
    "heads_relu_bwd": lambda: _fc.heads_relu_bwd(G, W, Y, 1.1, True),
    "relu_wgrad_smallk": lambda: _fc.relu_wgrad_smallk(g, Y, 1.1, A1, A2, True),
    "heads_fwd": lambda: _fc.fc_forward(Y, W, None, None, b, False),
    "conv1_fwd": lambda: _fc.fc_forward(A1, torch.ones(1024, 8, device="cuda"), A2, torch.ones(1024, 8, device="cuda"),
                                        None, True),
})
bytes_ = {"heads_relu_bwd": 2 * M * K * 4, "relu_wgrad_smallk": 2 * M * K * 4, "heads_fwd": M * K * 4,
          "conv1_fwd": M * K * 4}
lib = os.environ.get("LPGNN_LIB", "default")
for k, ms in t.items():
    print(f"{os.path.basename(lib):28s} {k:18s} {ms:.3f} ms  {bytes_[k] / ms / 1e9:.0f} GB/s", flush=True)
