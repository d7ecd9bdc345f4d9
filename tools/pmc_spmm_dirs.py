"""Per-direction HBM traffic of the F = hid SpMM (SURVEY.md 8d's counter-bytes model beside the edge-gather
and compulsory ones), for the c2 graph and the skewed (Zipf 1.5) graph of bench.py's sub-record.

  GPU program (under rocprofv3 --pmc FETCH_SIZE, then WRITE_SIZE, separate passes):
    python tools/pmc_spmm_dirs.py run
  summary (in this container or on the box):
    python tools/pmc_spmm_dirs.py summarize <fetch_dir> <write_dir> <out_prefix>
      -> <out_prefix>_c2.json, <out_prefix>_skewed.json  ({"workload", "directions": {dir: bytes}, ...})

The program launches, per graph and direction, REPS + 1 SpMMs (the first a warm-up) with bench.py's default
options, in a fixed order; the summary assigns the SpMM dispatches (sorted by dispatch id) to (graph,
direction) by that order and averages all but each group's first.  HBM bytes = 2 * FETCH_SIZE + WRITE_SIZE
KiB (the gfx950 FETCH halving, MI355X_MICROARCH.md), as tools/pmc_summary.py.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lp-gnn_amd")]

REPS = 3
GRAPHS = ("c2", "skewed")
DIRS = ("cons<-vars", "vars<-cons")
SPMM_NAMES = ("spmm_f32_rowwave", "spmm_f32_rowslim")


def workload(config):
    import bench

    return bench.workload_name(bench.sub_args(bench.parse([]), config))


def run():
    import torch

    from lpgnn import BipartiteCSR, synth
    from lpgnn.sparse import spmm_forward

    dev = "cuda:0"
    for name in GRAPHS:
        g = (synth.uniform_lp(100_000, 200_000, 2_000_000, seed=0) if name == "c2" else
             synth.skewed_lp(100_000, 200_000, 2_000_000, a=1.5, seed=0))
        adj = BipartiteCSR.from_coo(g.row, g.col, g.val, g.m, g.n, device=dev)
        for d, csr in zip(DIRS, (adj.fwd, adj.bwd)):
            x = torch.randn(csr.n_cols, 1024, device=dev)
            for _ in range(REPS + 1):
                spmm_forward(csr, x)
            torch.cuda.synchronize()
            print(name, d, "done", flush=True)
        del adj


def _read(d, counter):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") == counter and any(s in r["Kernel_Name"] for s in SPMM_NAMES):
                rows.append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
    per = defaultdict(float)  # a dispatch may report one row per XCD / instance: sum them
    for did, v in rows:
        per[did] += v
    return [per[k] for k in sorted(per)]


def summarize(fetch_dir, write_dir, prefix):
    fetch, write = _read(fetch_dir, "FETCH_SIZE"), _read(write_dir, "WRITE_SIZE")
    n = len(GRAPHS) * len(DIRS) * (REPS + 1)
    if len(fetch) != n or len(write) != n:
        raise SystemExit(f"expected {n} SpMM dispatches per pass, got {len(fetch)} / {len(write)}")
    k = 0
    for name in GRAPHS:
        out = {"workload": workload(name), "correction": "hbm = (2*FETCH_SIZE + WRITE_SIZE) KiB (gfx950 FETCH halving)",
               "source": "tools/pmc_spmm_dirs.py (F=1024 fp32 SpMM alone, default options, mean of %d launches "
                         "after one warm-up)" % REPS, "directions": {}, "fetch_kib_raw": {}, "write_kib": {}}
        for d in DIRS:
            f = fetch[k + 1:k + REPS + 1]
            w = write[k + 1:k + REPS + 1]
            k += REPS + 1
            fk, wk = sum(f) / len(f), sum(w) / len(w)
            out["directions"][d] = (2 * fk + wk) * 1024.0
            out["fetch_kib_raw"][d], out["write_kib"][d] = fk, wk
        path = f"{prefix}_{name}.json"
        json.dump(out, open(path, "w"), indent=1)
        print(path, {d: round(v / 1e9, 3) for d, v in out["directions"].items()}, "GB per launch")


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run()
    else:
        summarize(*sys.argv[2:5])
