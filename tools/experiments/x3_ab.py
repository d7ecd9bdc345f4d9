"""x3 FC forward (lpg_fc_x3_f32) at the c2 shapes: time, TF/s and the outputs, for A/B runs of two
builds of the library (LPGNN_LIB selects the build):

  LPGNN_LIB=tools/experiments/var_w16/liblpgnn_hip.so python tools/experiments/x3_ab.py w16
  python tools/experiments/x3_ab.py head
  python tools/experiments/x3_ab.py --compare head w16
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lp-gnn_amd")]
import torch  # noqa: E402

OUT = os.path.join(ROOT, "gpurun_out")
SHAPES = ((200_000, 1024, 0), (100_000, 1024, 1024), (100_000, 1024, 0))


def main(tag):
    from tools.kbench import timeit
    from lpgnn.fc import fc_forward

    os.makedirs(OUT, exist_ok=True)
    g = torch.Generator(device="cuda").manual_seed(11)
    res = {}
    for M, K1, K2 in SHAPES:
        A1 = torch.randn(M, K1, device="cuda", generator=g)
        A2 = torch.randn(M, K2, device="cuda", generator=g) if K2 else None
        W1 = torch.randn(1024, K1, device="cuda", generator=g) * 0.03
        W2 = torch.randn(1024, K2, device="cuda", generator=g) * 0.03 if K2 else None
        b = torch.randn(1024, device="cuda", generator=g)
        P0 = torch.randn(M, 1024, device="cuda", generator=g)
        P = P0.clone()
        fns = {"plain": lambda: fc_forward(A1, W1, A2, W2, None, False, arith="x3"),
               "relu+drop+acc": lambda: fc_forward(A1, W1, A2, W2, b, True, 0.1, 7, out=P, accumulate=True,
                                                   arith="x3")}
        res[(M, K1, K2, "plain")] = fns["plain"]().cpu()
        P.copy_(P0)
        res[(M, K1, K2, "acc")] = fns["relu+drop+acc"]().cpu()
        t = timeit(fns, rounds=7, iters=3)
        for name, ms in t.items():
            print(f"{tag} M={M} K={K1}+{K2} {name:14s} {ms:.3f} ms "
                  f"{2.0 * M * 1024 * (K1 + K2) / ms / 1e9:.1f} TF/s", flush=True)
        del A1, A2, P, P0
    torch.save({str(k): v for k, v in res.items()}, os.path.join(OUT, f"x3_ab_{tag}.pt"))


def compare(a, b):
    ra = torch.load(os.path.join(OUT, f"x3_ab_{a}.pt"), weights_only=True)
    rb = torch.load(os.path.join(OUT, f"x3_ab_{b}.pt"), weights_only=True)
    ok = True
    for k in ra:
        eq = torch.equal(ra[k], rb[k])
        ok &= eq
        print(f"{k} {a} == {b} bitwise: {eq}")
    assert ok


if __name__ == "__main__":
    if sys.argv[1] == "--compare":
        compare(sys.argv[2], sys.argv[3])
    else:
        main(sys.argv[1])
