"""Is a per-launch fixed cost worth batching the weight gradients?  Three back-to-back launches at
R = 100K against one launch at R = 300K (the same FLOPs), bf16 (c5: N = K = 2048) and x3 (c2:
N = K = 1024); HIP events, median of rounds."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lp-gnn_amd")]
import torch  # noqa: E402


def main():
    from tools.kbench import timeit
    from lpgnn.fc import wgrad, wgrad_bf16

    BF = torch.bfloat16
    for name, F, fn, dt in (("bf16", 2048, wgrad_bf16, BF), ("x3", 1024, lambda g, x: wgrad(g, x, arith="x3"),
                                                               torch.float32)):
        G = torch.randn(300_000, F, device="cuda").to(dt)
        X = torch.randn(300_000, F, device="cuda").relu_().to(dt)
        parts = [(G[i * 100_000:(i + 1) * 100_000], X[i * 100_000:(i + 1) * 100_000]) for i in range(3)]
        t = timeit({"3 x R=100K": lambda: [fn(g, x) for g, x in parts], "1 x R=300K": lambda: fn(G, X),
                    "1 x R=100K": lambda: fn(*parts[0])}, rounds=7, iters=4)
        for k, v in t.items():
            r = 300_000 if "3 x" in k or "300K" in k else 100_000
            print(f"{name} {k:12s} {v:.3f} ms {2.0 * r * F * F / v / 1e9:.1f} TF/s", flush=True)
        del G, X, parts


if __name__ == "__main__":
    main()
