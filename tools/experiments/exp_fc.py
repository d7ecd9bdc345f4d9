"""Ad-hoc timing of lpg_fc_f32 variant 7 at the c2 200K-row shape (for A/B of
experimental builds loaded through LPGNN_LIB)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
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
ref = fc_forward(A1, W1, A2, W2, b, True)
for v in (0, 7):
    for ng in (0,):
        L.lpg_fc_set_variant(v)
        assert torch.equal(fc_forward(A1, W1, A2, W2, b, True), ref)
        res[(v, ng)] = timeit({"x": lambda: fc_forward(A1, W1, A2, W2, b, True)})["x"]
L.lpg_fc_set_variant(0)
for k, ms in res.items():
    print(f"variant {k[0]}: {ms:.3f} ms {2.0 * M * 1024 * 2048 / ms / 1e9:.1f} TF/s")
