"""Run only lpg_fc_x3_f32 (or the exact fp32 kernel with arg 'fp32') at the c2
hidden-layer shape a few times -- a short program for rocprofv3 PMC passes."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lp-gnn_amd")]
import torch  # noqa: E402

from lpgnn import _lib  # noqa: E402
from lpgnn.fc import fc_forward  # noqa: E402

_lib.check(_lib.lib().lpg_fc_x3_set_variant(int(os.environ.get("LPG_X3V", "0"))), "set_variant")

arith = sys.argv[1] if len(sys.argv) > 1 else "x3"
M = 200_000
A1 = torch.randn(M, 1024, device="cuda").relu_()
A2 = torch.randn(M, 1024, device="cuda").relu_()
W1 = torch.randn(1024, 1024, device="cuda") * 0.03
W2 = torch.randn(1024, 1024, device="cuda") * 0.03
b = torch.randn(1024, device="cuda")
for _ in range(3):
    fc_forward(A1, W1, A2, W2, b, True, arith=arith)
torch.cuda.synchronize()
print("done")
