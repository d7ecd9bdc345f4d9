import sys, torch
sys.path.insert(0, "lp-gnn_amd")
from lpgnn import fc as F
DEV = "cuda:0"
torch.manual_seed(0)
for M in (900, 5000):
    A = torch.randn(M, 256, device=DEV); A2 = torch.randn(M, 256, device=DEV)
    W = torch.randn(256, 256, device=DEV) * 0.05; W2 = torch.randn(256, 256, device=DEV) * 0.05
    b = torch.randn(256, device=DEV) * 0.1
    Wh = torch.randn(3, 256, device=DEV) * 0.05; bh = torch.randn(3, device=DEV)
    for arith in ("x3", "f16x2"):
        C1, L1 = F.fc_forward(A, W, A2, W2, b, True, 0.1, 5, heads=(Wh, bh), arith=arith)
        C2 = F.fc_forward(A, W, A2, W2, b, True, 0.1, 5, arith=arith)
        print(M, arith, "C equal:", torch.equal(C1, C2), float((C1 - C2).abs().max()))
