"""x3 weight gradient (lpg_wgrad_x3_f32) at the c2 shapes: time, TF/s and a checksum of the result,
for A/B runs of two builds of the library (LPGNN_LIB selects the build):

  LPGNN_LIB=tools/experiments/var_dup/liblpgnn_hip.so python tools/experiments/wgrad_bal.py dup
  python tools/experiments/wgrad_bal.py head

Each run saves its dW to gpurun_out/wgrad_bal_<tag>.pt; `--compare a b` checks them bitwise.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lp-gnn_amd")]
import torch  # noqa: E402

OUT = os.path.join(ROOT, "gpurun_out")


def main(tag):
    from tools.kbench import timeit
    from lpgnn.fc import wgrad

    os.makedirs(OUT, exist_ok=True)
    g = torch.Generator(device="cuda").manual_seed(5)
    res = {}
    for R in (100_000, 200_000):
        G = torch.randn(R, 1024, device="cuda", generator=g)
        X = torch.randn(R, 1024, device="cuda", generator=g).relu_()
        res[R] = wgrad(G, X, arith="x3").cpu()
        t = timeit({"wgrad_x3": lambda: wgrad(G, X, arith="x3")}, rounds=7, iters=4)
        ms = t["wgrad_x3"]
        print(f"{tag} R={R} wgrad_x3 {ms:.3f} ms {2.0 * R * 1024 * 1024 / ms / 1e9:.1f} TF/s", flush=True)
        del G, X
    torch.save(res, os.path.join(OUT, f"wgrad_bal_{tag}.pt"))


def compare(a, b):
    ra = torch.load(os.path.join(OUT, f"wgrad_bal_{a}.pt"), weights_only=True)
    rb = torch.load(os.path.join(OUT, f"wgrad_bal_{b}.pt"), weights_only=True)
    for R in ra:
        print(f"R={R} {a} == {b} bitwise: {torch.equal(ra[R], rb[R])}")
        assert torch.equal(ra[R], rb[R])


if __name__ == "__main__":
    if sys.argv[1] == "--compare":
        compare(sys.argv[2], sys.argv[3])
    else:
        main(sys.argv[1])
