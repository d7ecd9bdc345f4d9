"""What the fused dropout costs in a training step: c2 / c5 steps with the model's dp = 0.1 (the
reference default) against dp = 0, alternating in one process (the mask hash runs in the FC
epilogues; the backward reads the kept set from the stored output)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lp-gnn_amd")]
import torch  # noqa: E402


def main():
    from lpgnn import BipartiteBatch, BipartiteCSR, GCN_FC, synth
    from lpgnn.train import make_optimizer, train_step

    dev = "cuda:0"
    g = synth.uniform_lp(100_000, 200_000, 2_000_000, seed=0)
    adj = BipartiteCSR.from_coo(g.row, g.col, g.val, g.m, g.n, device=dev)
    batch = BipartiteBatch(x_s=torch.from_numpy(g.x_s).to(dev), x_t=torch.from_numpy(g.x_t).to(dev),
                           y_s=torch.from_numpy(g.y_s).to(dev), y_t=torch.from_numpy(g.y_t).to(dev),
                           edge_index=adj, s_bs=g.m, t_bs=g.n)
    for name, hids, depth, dt in (("c2", 1024, 3, torch.float32), ("c5", 2048, 6, torch.bfloat16)):
        torch.manual_seed(0)
        model = GCN_FC(8, 8, hids=hids, depth=depth, compute_dtype=dt).to(dev)
        opt, _ = make_optimizer(model)
        res = {0.1: [], 0.0: []}
        for rep in range(3):
            for dp in (0.1, 0.0):
                model.dp = dp
                for _ in range(2):
                    train_step(model, batch, opt)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(10):
                    train_step(model, batch, opt)
                torch.cuda.synchronize()
                res[dp].append((time.perf_counter() - t0) / 10 * 1e3)
        print(f"{name}: dp=0.1 {min(res[0.1]):.2f} ms/step, dp=0 {min(res[0.0]):.2f} ms/step "
              f"(all: {[round(x, 2) for x in res[0.1]]} / {[round(x, 2) for x in res[0.0]]})", flush=True)
        del model, opt


if __name__ == "__main__":
    main()
