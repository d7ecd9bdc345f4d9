"""x3 weight gradient at the c2 shapes for the kernel LPGNN_WGRAD_KERNEL selects (read once per
process: run once per kernel): time, TF/s, and the error against an fp64 GEMM in units of
tests/test_gpu_x3.py's bound (16 u sum|ab| + u |ref|).

  LPGNN_WGRAD_KERNEL=1 python tools/experiments/wgrad_q.py q
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lp-gnn_amd")]
import torch  # noqa: E402


def main(tag):
    from tools.kbench import timeit
    from lpgnn.fc import wgrad

    u = 2.0 ** -24
    g = torch.Generator(device="cuda").manual_seed(5)
    for R in (100_000, 200_000):
        G = torch.randn(R, 1024, device="cuda", generator=g)
        X = torch.randn(R, 1024, device="cuda", generator=g).relu_()
        got = wgrad(G, X, arith="x3").double()
        ref = G.double().t() @ X.double()
        s = G.double().abs().t() @ X.double().abs()
        r = ((got - ref).abs() / (16 * u * s + u * ref.abs() + 1e-30)).max().item()
        e = ((got - ref).abs() / (u * s)).mean().item()
        del ref, s, got
        t = timeit({"w": lambda: wgrad(G, X, arith="x3")}, rounds=7, iters=4)["w"]
        print(f"{tag} R={R} wgrad_x3 {t:.3f} ms {2.0 * R * 1024 * 1024 / t / 1e9:.1f} TF/s "
              f"max err/bound {r:.4f} mean err/(u sum|ab|) {e:.4f}", flush=True)
        del G, X


if __name__ == "__main__":
    main(sys.argv[1])
