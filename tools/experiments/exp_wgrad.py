"""Ad-hoc timing of lpg_relu_wgrad_smallk_f32 at the conv1 c2 shapes (A/B of builds via LPGNN_LIB)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lp-gnn_amd")]
import torch  # noqa: E402

from tools.kbench import timeit  # noqa: E402

from lpgnn.fc import relu_wgrad_smallk  # noqa: E402

res = {}
for M in (200_000, 100_000):
    g = torch.randn(M, 1024, device="cuda")
    y = torch.relu(torch.randn(M, 1024, device="cuda"))
    A1, A2 = torch.randn(M, 8, device="cuda"), torch.randn(M, 8, device="cuda")
    res[M] = timeit({"x": lambda: relu_wgrad_smallk(g, y, 1.0, A1, A2, True)})["x"]
print(os.environ.get("LPGNN_LIB", "default"), {M: (ms, 2 * M * 1024 * 4 / ms / 1e9) for M, ms in res.items()})
