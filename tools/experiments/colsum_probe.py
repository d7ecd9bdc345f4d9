"""Rate of the bf16 column sum (lpg_colsum_bf16, the folded layers' bias gradient) at the c5 shapes."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lp-gnn_amd")]
import torch  # noqa: E402


def main():
    from tools.kbench import timeit
    from lpgnn.fc import colsum_bf16

    for M in (200_000, 100_000):
        g = torch.randn(M, 2048, device="cuda").to(torch.bfloat16)
        t = timeit({"colsum": lambda: colsum_bf16(g), "copy": lambda: g.clone()}, rounds=7, iters=5)
        print(f"M={M} colsum {t['colsum']:.4f} ms {M * 2048 * 2 / t['colsum'] / 1e9:.0f} GB/s; "
              f"torch copy {t['copy']:.4f} ms {2 * M * 2048 * 2 / t['copy'] / 1e9:.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
