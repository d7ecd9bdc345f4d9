"""Ad-hoc timing of lpg_fc_f32 variant 7 at the c2 200K-row shape (for A/B of
experimental builds loaded through LPGNN_LIB)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lp-gnn_amd")]
import torch  # noqa: E402

from tools.kbench import timeit  # noqa: E402

from lpgnn import _lib  # noqa: E402
from lpgnn.fc import fc_forward  # noqa: E402

M = 200_000
A1, A2 = torch.randn(M, 1024, device="cuda"), torch.randn(M, 1024, device="cuda")
W1, W2 = torch.randn(1024, 1024, device="cuda") * 0.03, torch.randn(1024, 1024, device="cuda") * 0.03
b = torch.randn(1024, device="cuda")
L = _lib.lib()
res = {}
for v in (0, 7):
    L.lpg_fc_set_variant(v)
    res[v] = timeit({"x": lambda: fc_forward(A1, W1, A2, W2, b, True)})["x"]
print(os.environ.get("LPGNN_LIB", "default"), {v: (ms, 2.0 * M * 1024 * 2048 / ms / 1e9) for v, ms in res.items()})
