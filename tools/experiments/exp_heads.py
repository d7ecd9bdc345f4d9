"""Ad-hoc timing of lpg_linear_small_bwd_f32 at the heads' c2 shapes (A/B of builds via LPGNN_LIB)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lp-gnn_amd")]
import torch  # noqa: E402

from tools.kbench import timeit  # noqa: E402

from lpgnn.fc import linear_small_bwd  # noqa: E402

res = {}
for M in (200_000, 100_000):
    G = torch.randn(M, 3, device="cuda")
    W = torch.randn(3, 1024, device="cuda")
    H = torch.randn(M, 1024, device="cuda")
    res[M] = timeit({"x": lambda: linear_small_bwd(G, W, H, True)})["x"]
print(os.environ.get("LPGNN_LIB", "default"), {M: (ms, 2 * M * 1024 * 4 / ms / 1e9) for M, ms in res.items()})
