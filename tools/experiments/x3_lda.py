"""x3 FC (200K x 1024 -> 1024, plain) with the activations' row stride padded: does the power-of-two
row stride (4 KiB) of A and C cost L2 hits?  `python x3_lda.py time` times lda = ldc in {1024, 1040,
1056, 1088}; `python x3_lda.py one LDA` runs a few launches of one stride (for rocprofv3 --pmc)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lp-gnn_amd")]
import torch  # noqa: E402

M, K, N = 200_000, 1024, 1024


def operands(ld):
    g = torch.Generator(device="cuda").manual_seed(0)
    Ab = torch.randn(M, ld, device="cuda", generator=g)
    A = Ab[:, :K]
    W = torch.randn(N, K, device="cuda", generator=g) * 0.03
    Cb = torch.empty(M, ld, device="cuda")
    return A, W, Cb[:, :N]


def run(ld, reps):
    from lpgnn.fc import fc_forward
    A, W, C = operands(ld)
    for _ in range(reps):
        fc_forward(A, W, None, None, None, False, out=C, arith="x3")
    torch.cuda.synchronize()
    return A, W, C


if __name__ == "__main__":
    if sys.argv[1] == "one":
        run(int(sys.argv[2]), 4)
        print("done")
    else:
        from tools.kbench import timeit
        from lpgnn.fc import fc_forward
        ref = None
        for ld in (1024, 1040, 1056, 1088, 1024):
            A, W, C = run(ld, 2)
            out = C.clone()
            ref = out if ref is None else ref
            t = timeit({"fc": lambda: fc_forward(A, W, None, None, None, False, out=C, arith="x3")}, rounds=7,
                       iters=4)["fc"]
            print(f"x3 fc lda=ldc={ld} {t:.3f} ms {2.0 * M * N * K / t / 1e9:.1f} TF/s same={torch.equal(out, ref)}",
                  flush=True)
            del A, W, C
