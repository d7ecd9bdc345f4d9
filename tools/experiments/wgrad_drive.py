"""Run only lpg_wgrad_x3_f32 at the c2 shape (R=200K, 1024 x 1024) a few times -- for PMC passes."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lp-gnn_amd")]
import torch  # noqa: E402

from lpgnn import _lib  # noqa: E402
from lpgnn.fc import wgrad  # noqa: E402

if os.environ.get("LPG_WGV"):  # weight-gradient kernel variant (lpg_fc_x3_set_variant 100..105)
    _lib.check(_lib.lib().lpg_fc_x3_set_variant(int(os.environ["LPG_WGV"])), "set_variant")

G = torch.randn(200_000, 1024, device="cuda")
X = torch.randn(200_000, 1024, device="cuda").relu_()
for _ in range(3):
    wgrad(G, X, arith="x3")
torch.cuda.synchronize()
print("done")
