"""The F=hid SpMM of ONE rank's share of a row-partitioned bench workload, on one GPU, for the
rocprofv3 PMC passes that give bench.py's ``roofline.traffic`` at N > 1 (its key:
bench.rank_share_key).  The rank's blocks are generated and planned exactly as bench.py's
partitioned job does (lpgnn.partition.plan_partition_blocks, no process group needed for the
local CSR); the kernel launches are those of the training step: both orientations, F = 1024,
`reps` times each.

  python tools/pmc_rank_share.py --family c2 --world 8 [--rank 0] [--reps 3]
  python tools/pmc_rank_share.py --family c2 --world 8 --print-key
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "lp-gnn_amd"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--family", choices=("c2", "c4"), required=True)
    ap.add_argument("--world", type=int, required=True)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--print-key", action="store_true")
    a = ap.parse_args()
    import bench

    args = bench.parse(["--config", a.family, "--gpus", str(a.world)])
    fam = f"c2 weak scaling (rho={args.rho})" if a.family == "c2" else f"c4 (rho={args.rho})"
    key = bench.rank_share_key(fam, a.world, a.rank)
    if a.print_key:
        print(key)
        return
    import torch

    from lpgnn import partition
    from lpgnn.sparse import spmm_forward

    spec = partition.bench_spec(args, a.world)
    plan = partition.plan_partition_blocks(spec, a.world, a.rank, exchange=False)
    dev = torch.device("cuda", 0)
    adj = partition.local_dual_csr(plan, dev)
    F = args.hids
    g = torch.Generator(device=dev).manual_seed(0)
    xv = torch.randn((plan.n_local, F), device=dev, generator=g)
    xc = torch.randn((plan.m_local, F), device=dev, generator=g)
    for _ in range(a.reps):
        spmm_forward(adj.fwd, xv)  # cons <- [owned | halo] vars
        spmm_forward(adj.bwd, xc)  # [owned | halo] vars <- cons
    torch.cuda.synchronize()
    print(f"{key}: m_local={plan.m_local} n_local={plan.n_local} (owned {plan.n_own}, halo {plan.halo.shape[0]}) "
          f"nnz_local={plan.nnz_local}", flush=True)


if __name__ == "__main__":
    main()
