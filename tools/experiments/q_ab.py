"""A/B of the 16-bit FC's two-blocks-per-CU form (kernel choice 7, fc_bf16_q: 4-wave 128 x 256
tiles, one LDS stage) against the one-block-per-CU pipelined kernel with its 128 x 128 tail launch
(choice 0 through the per-call entries) and without it (choice 3), at the c5 and fp16-inference
shapes.  Prints ms and TF/s per shape and choice; checks the bits agree."""
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
    ("f16 relu 100K K2048", torch.float16, 100_000, 1024, 1024, 1024, True, 0.0, False),
    ("f16 relu+acc 200K K1024", torch.float16, 200_000, 1024, 1024, 0, True, 0.0, True),
]


def legacy(dt, M, N, K1, K2, relu, drop, acc, A1, W1, A2, W2, b, out):
    """lpg_fc_bf16 / lpg_fc_f16 with choice 0 and no workspace: the pipelined kernel + 128 x 128 tail."""
    from lpgnn import _lib

    L = _lib.lib()
    flags = (1 if relu else 0) | (2 if acc else 0)
    entry = L.lpg_fc_f16 if dt == torch.float16 else L.lpg_fc_bf16
    st = entry(M, N, K1, A1.data_ptr(), A1.stride(0), W1.data_ptr(), W1.stride(0), K2,
               None if A2 is None else A2.data_ptr(), A2.stride(0) if K2 else 0,
               None if W2 is None else W2.data_ptr(), W2.stride(0) if K2 else 0, b.data_ptr(), out.data_ptr(),
               out.stride(0), flags, float(drop), 5, 0, None, _lib.stream_of(A1))
    _lib.check(st, "legacy")
    return out


def run(dt, M, N, K1, K2, relu, drop, acc, kernel, A1, W1, A2, W2, b, P, out):
    if acc:
        out.copy_(P)
    if kernel is None:
        return legacy(dt, M, N, K1, K2, relu, drop, acc, A1, W1, A2, W2, b, out)
    return F.fc_forward_bf16(A1, W1, A2, W2, b, relu, drop, 5, out=out, accumulate=acc, kernel=kernel)


def main():
    torch.manual_seed(0)
    for name, dt, M, N, K1, K2, relu, drop, acc in SHAPES:
        A1 = torch.randn(M, K1, device=DEV).to(dt)
        W1 = (torch.randn(N, K1, device=DEV) * 0.03).to(dt)
        A2 = torch.randn(M, K2, device=DEV).to(dt) if K2 else None
        W2 = (torch.randn(N, K2, device=DEV) * 0.03).to(dt) if K2 else None
        b = torch.randn(N, device=DEV) * 0.1
        P = torch.randn(M, N, device=DEV).to(dt) if acc else None
        out = torch.empty(M, N, device=DEV, dtype=dt)
        flops = 2.0 * M * N * (K1 + K2)
        res = {}
        for label, kernel in (("q(7)", 7), ("p+tail(0)", None), ("p(3)", 3)):
            for _ in range(3):
                y = run(dt, M, N, K1, K2, relu, drop, acc, kernel, A1, W1, A2, W2, b, P, out)
            res[label] = y.clone()
            ts = []
            for _ in range(15):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                run(dt, M, N, K1, K2, relu, drop, acc, kernel, A1, W1, A2, W2, b, P, out)
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            ts.sort()
            ms = ts[len(ts) // 2]
            print(f"{name:26s} {label:10s} {ms:8.3f} ms  {flops / ms / 1e9:7.1f} TF/s  (min {ts[0]:.3f})", flush=True)
        same = torch.equal(res["q(7)"], res["p(3)"]) and torch.equal(res["p+tail(0)"], res["p(3)"])
        print(f"{name:26s} bits identical: {same}", flush=True)
        del A1, W1, A2, W2, P, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
