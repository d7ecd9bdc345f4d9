"""A/B of the x3 FC's tile orders at the c2 shapes, alternating in one process, outputs checked
bitwise equal.  Round 4 ran it with LPG_FC_KERNEL(0) = the m-major order (each XCD walks contiguous
m-tiles with all their n-tiles) and (2) = the n-split order (half the XCDs take the first half of the
n-tiles), profiles/r04_x3_order_ab.log; the n-split order has been kernel 0 (the default) since, and
kernel 2 the m-major order.

  python tools/experiments/x3_order_ab.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lp-gnn_amd")]
import torch  # noqa: E402

from lpgnn.fc import fc_forward  # noqa: E402

SHAPES = [  # (M, K1, K2, N, accumulate + dropout) -- the c2 step's hidden-width FC launches
    (200_000, 1024, 1024, 1024, False),
    (200_000, 1024, 0, 1024, True),
    (100_000, 1024, 1024, 1024, False),
    (100_000, 1024, 0, 1024, False),
]


def run(M, K1, K2, N, acc, kern, A1, A2, W1, W2, b, P, n=10):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        out = fc_forward(A1, W1, A2, W2, b, True, 0.1 if acc else 0.0, 7, out=P if acc else None,
                         accumulate=acc, arith="x3", kernel=kern)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n, out


def main():
    torch.manual_seed(0)
    for M, K1, K2, N, acc in SHAPES:
        A1 = torch.randn(M, K1, device="cuda")
        A2 = torch.randn(M, K2, device="cuda") if K2 else None
        W1 = torch.randn(N, K1, device="cuda") * 0.03
        W2 = torch.randn(N, K2, device="cuda") * 0.03 if K2 else None
        b = torch.randn(N, device="cuda")
        P = torch.zeros(M, N, device="cuda") if acc else None
        flops = 2.0 * M * N * (K1 + K2)
        t = {0: [], 2: [], 3: []}
        for _ in range(2):
            run(M, K1, K2, N, acc, 0, A1, A2, W1, W2, b, P, 3)
        for rnd in range(4):
            for k in (0, 2, 3) if rnd % 2 == 0 else (3, 2, 0):
                t[k].append(run(M, K1, K2, N, acc, k, A1, A2, W1, W2, b, P, 10)[0])
        outs = {}
        for k in (0, 2, 3):
            if acc:
                P.zero_()
            outs[k] = run(M, K1, K2, N, acc, k, A1, A2, W1, W2, b, P, 1)[1].clone()
        same = torch.equal(outs[0], outs[2]) and torch.equal(outs[0], outs[3])
        line = f"M={M} K={K1}+{K2} N={N} acc+drop={acc}: "
        for k in (0, 2, 3):
            ms = sorted(t[k])[len(t[k]) // 2]
            line += f"kernel {k}: {ms:.3f} ms ({flops / ms / 1e9:.0f} TF/s)  "
        print(line + f"bitwise equal: {same}", flush=True)
        del A1, A2, P


if __name__ == "__main__":
    main()
