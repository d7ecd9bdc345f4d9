"""A/B of the bf16 FC's tile orders at the c5 shapes, alternating in one process, outputs checked bitwise
equal.  Round 4 ran it with LPG_FC_KERNEL(0) = the pipelined 256 x 256 kernel in the m-major order (each
XCD walking contiguous m-tiles with all their n-tiles) + the tail launch, and (4) = the same in the
n-split order (profiles/r04_bf16_order_ab.log); the n-split order has been choice 0 since, choice 4 the
m-major one.

  python tools/experiments/bf16_order_ab.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lp-gnn_amd")]
import torch  # noqa: E402

from lpgnn.fc import fc_forward_bf16  # noqa: E402

BF = torch.bfloat16
SHAPES = [  # (M, K1, K2, N, accumulate + dropout) -- the c5 step's hidden-width FC launches
    (200_000, 2048, 0, 2048, True),
    (100_000, 2048, 2048, 2048, False),
    (200_000, 2048, 0, 2048, False),
    (100_000, 2048, 0, 2048, False),
]


def run(kern, A1, A2, W1, W2, b, P, acc, n=10):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        out = fc_forward_bf16(A1, W1, A2, W2, b, True, 0.1 if acc else 0.0, 7, out=P if acc else None,
                              accumulate=acc, kernel=kern)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n, out


def main():
    torch.manual_seed(0)
    for M, K1, K2, N, acc in SHAPES:
        A1 = torch.randn(M, K1, device="cuda").to(BF)
        A2 = torch.randn(M, K2, device="cuda").to(BF) if K2 else None
        W1 = (torch.randn(N, K1, device="cuda") * 0.02).to(BF)
        W2 = (torch.randn(N, K2, device="cuda") * 0.02).to(BF) if K2 else None
        b = torch.randn(N, device="cuda")
        P = torch.zeros(M, N, device="cuda").to(BF) if acc else None
        flops = 2.0 * M * N * (K1 + K2)
        t = {0: [], 4: [], 5: []}
        run(0, A1, A2, W1, W2, b, P, acc, 3)
        for rnd in range(4):
            for k in (0, 4, 5) if rnd % 2 == 0 else (5, 4, 0):
                t[k].append(run(k, A1, A2, W1, W2, b, P, acc, 10)[0])
        outs = {}
        for k in (0, 4, 5):
            if acc:
                P.zero_()
            outs[k] = run(k, A1, A2, W1, W2, b, P, acc, 1)[1].clone()
        line = f"M={M} K={K1}+{K2} N={N} acc+drop={acc}: "
        for k in (0, 4, 5):
            ms = sorted(t[k])[len(t[k]) // 2]
            line += f"kernel {k}: {ms:.3f} ms ({flops / ms / 1e9:.0f} TF/s)  "
        print(line + f"bitwise equal: {torch.equal(outs[0], outs[4]) and torch.equal(outs[0], outs[5])}", flush=True)
        del A1, A2, P


if __name__ == "__main__":
    main()
