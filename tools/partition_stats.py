"""Boundary-exchange volume of the row partition vs rho (report
scaling versus rho).  For the bench's weak-scaling graphs (N c2-sized row
blocks, synth.block_lp) it prints, for rank 0: owned / halo variables,
global boundary variables, rows sent + received per exchange, and the bytes
one exchange moves at F = 1024 fp32 (a depth-3 step runs 5 such exchanges:
forward reduce + broadcast of the hidden layer and conv1's broadcast, backward
reduce + broadcast of the hidden layer's gradients; conv1's input reduce is at F = 8).

  python tools/partition_stats.py [--ranks 2 4 8] [--rho 0 0.02 0.1 1.0]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lp-gnn_amd")]

from lpgnn import synth  # noqa: E402
from lpgnn.partition import plan_partition  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, nargs="+", default=[2, 4, 8])
    ap.add_argument("--rho", type=float, nargs="+", default=[0.0, 0.02, 0.1, 1.0])
    ap.add_argument("--m", type=int, default=100_000)
    ap.add_argument("--n", type=int, default=200_000)
    ap.add_argument("--nnz", type=int, default=2_000_000)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    rows = []
    for world in a.ranks:
        for rho in a.rho:
            t0 = time.time()
            g = synth.block_lp(a.m * world, a.n * world, a.nnz * world, parts=world, rho=rho, seed=0)
            p = plan_partition(g.row, g.col, g.val, g.m, g.n, world, 0)
            sent, recv = int(sum(p.send_counts)), int(sum(p.recv_counts))
            r = dict(world=world, rho=rho, owned=p.n_own, halo=int(p.halo.shape[0]),
                     boundary_global=p.n_boundary_global, rows_sent=sent, rows_recv=recv,
                     mib_per_exchange_f1024=(sent + recv) * 1024 * 4 / 2**20,
                     peers=int(sum(1 for c in p.send_counts if c)), secs=round(time.time() - t0, 1))
            rows.append(r)
            print(json.dumps(r), flush=True)
    if a.out:
        json.dump(rows, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
