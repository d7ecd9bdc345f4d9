"""What bounds the 16-bit FC: the default pipelined kernel (lpg_fc_bf16 /
lpg_fc_f16, choice 0) at the c5 and fp16-inference shapes on random operands and on all-zero operands
(the same instruction stream and memory traffic, no bit toggling in the MFMA datapath: the clock the
power limit then allows).  A large zero-operand gain means the k loop is power-bound, so a structural
change (tile shape, epilogue overlap) cannot buy much; no gain means the structure is the limit."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "lp-gnn_amd"))
from lpgnn import fc as F  # noqa: E402

DEV = "cuda:0"
SHAPES = [  # (name, dtype, M, N, K1, K2, relu, dropout, accumulate)
    ("c5 lin 100K K2048", torch.bfloat16, 100_000, 2048, 2048, 0, False, 0.0, False),
    ("c5 relu 100K K4096", torch.bfloat16, 100_000, 2048, 2048, 2048, True, 0.1, False),
    ("c5 relu+acc 200K K2048", torch.bfloat16, 200_000, 2048, 2048, 0, True, 0.1, True),
    ("f16 lin 100K K1024", torch.float16, 100_000, 1024, 1024, 0, False, 0.0, False),
    ("f16 relu+acc 200K K1024", torch.float16, 200_000, 1024, 1024, 0, True, 0.0, True),
]


def bench(fn, reps=15):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    torch.manual_seed(0)
    for name, dt, M, N, K1, K2, relu, drop, acc in SHAPES:
        flops = 2.0 * M * N * (K1 + K2)
        for fill in ("random", "zeros", "random"):
            mk = (lambda *s: torch.zeros(*s, device=DEV)) if fill == "zeros" else \
                (lambda *s: torch.randn(*s, device=DEV))
            A1 = mk(M, K1).to(dt)
            W1 = (mk(N, K1) * 0.03).to(dt)
            A2 = mk(M, K2).to(dt) if K2 else None
            W2 = (mk(N, K2) * 0.03).to(dt) if K2 else None
            b = torch.randn(N, device=DEV) * 0.1
            out = torch.empty(M, N, device=DEV, dtype=dt)
            if acc:
                out.copy_(mk(M, N).to(dt))

            def run():
                return F.fc_forward_bf16(A1, W1, A2, W2, b, relu, drop, 5, out=out, accumulate=acc)
            ms = bench(run)
            print(f"{name:26s} {fill:7s} {ms:8.3f} ms  {flops / ms / 1e9:7.1f} TF/s", flush=True)
            if fill == "random" and not acc:
                # the vendor GEMM (hipBLASLt through torch) on the same operands: A [M, K] @ W^T, bias, no
                # ReLU / dropout epilogue, the two K parts as one concatenated operand
                Ac = A1 if A2 is None else torch.cat([A1, A2], 1)
                Wc = W1 if W2 is None else torch.cat([W1, W2], 1)
                bb = b.to(dt)
                ms_v = bench(lambda: torch.nn.functional.linear(Ac, Wc, bb))
                print(f"{name:26s} {'vendor':7s} {ms_v:8.3f} ms  {flops / ms_v / 1e9:7.1f} TF/s  (torch linear)",
                      flush=True)
                del Ac, Wc
            del A1, W1, A2, W2, out
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
