"""Headline benchmark: edges/s of the bipartite SpMM in GCN_FC (hid=1024,
depth=3) training steps on MI355X, with the HBM-roofline fraction of the
SpMM kernel and the oracle CPU path timed beside it.

  python bench.py [--gpus N] [--steps K] [--warmup W]

With --gpus N > 1 and no RANK / WORLD_SIZE in the environment, bench.py launches the N ranks
itself (one child process per GPU, started before this process touches the GPU; rank 0 prints
the JSON line) -- the same line as under ``torch.distributed.run --nproc-per-node N``.
``--share-gpu`` makes the N ranks share the visible GPU(s) over gloo (a rehearsal on a 1-GPU
box; the measured runs use RCCL, one rank per GPU).

A step = one GCN_FC(8, 8, hids=1024, depth=3) training iteration of
train.py:117-129 on the synthetic c2 graph (100K cons x 200K vars, nnz 2M,
BASELINE.json configs[1]): forward (2 SpMM at F=8 + 2 at F=1024, FC stacks,
heads, add_knowledge), balanced loss, backward (2 SpMM at F=1024 + FC
grads), Adam step.  value = (hid-width SpMM edge traversals in the step) /
step time, whole job.

N>1 defaults to ``--config c4`` (BASELINE.json configs[3]): the fixed
2M cons x 4M vars, nnz 40M block LP, constraint-row partitioned over the N
ranks (one process per GPU, torchrun) -- STRONG scaling; each rank generates
and plans only its own row blocks (lpgnn.partition.plan_partition_blocks),
boundary-variable rows are reduced to their owners and broadcast back over
RCCL.  ``--config c2`` with N>1 is the weak-scaling variant (N c2-sized
blocks).  ``--config c4`` at N=1 runs the whole c4 graph on one GPU.

``--config c5`` runs BASELINE.json configs[4] instead (same graph,
GCN_FC hids=2048 depth=6, bf16 activations / SpMM storage / MFMA FC, fp32
master weights) -- the MFMA-utilisation stress line, not the headline.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "lp-gnn_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP32_MFMA_PEAK_TFLOPS = 157.3
BF16_MFMA_PEAK_TFLOPS = 2500.0  # dense (MI355X_MICROARCH.md; the 5 PF figure is 2:1 sparse)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--config", choices=("c2", "c4", "c5"), default=None,
                    help="c2 = headline fp32 hid 1024 depth 3 (default at N=1); c4 = 2M x 4M nnz 40M "
                         "row-partitioned, strong scaling (default at N>1); c5 = bf16 hid 2048 depth 6")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--m", type=int, default=None)
    ap.add_argument("--n", type=int, default=None)
    ap.add_argument("--nnz", type=int, default=None)
    ap.add_argument("--hids", type=int, default=None)
    ap.add_argument("--depth", type=int, default=None)
    ap.add_argument("--rho", type=float, default=0.02, help="boundary edge fraction for N>1 partitions")
    ap.add_argument("--cpu-steps", type=int, default=1, help="oracle CPU steps for cpu_baseline (0 = skip)")
    ap.add_argument("--profile-only", action="store_true", help="no CPU baseline, no JSON extras (rocprof runs)")
    ap.add_argument("--print-workload", action="store_true", help="print the N=1 workload string and exit")
    ap.add_argument("--partitioned", action="store_true",
                    help="use the row-partitioned RCCL path even at N=1 (the N>1 code path)")
    ap.add_argument("--share-gpu", action="store_true",
                    help="self-launched N>1: ranks share the visible GPU(s) over gloo (rehearsal, not a measurement)")
    ap.add_argument("--rho-sweep", default="0,0.02,0.1,1.0",
                    help="c4 at N>1: rho values whose partition boundary counts go into the JSON ('' = off)")
    ap.add_argument("--inference", action="store_true",
                    help="time eval-mode forward + inference_gnn (the reference's timed path) instead of training")
    args = ap.parse_args()
    if args.config is None:
        args.config = "c2" if args.gpus == 1 else "c4"
    from lpgnn.synth import CONFIGS

    for k, v in CONFIGS[args.config].items():
        if getattr(args, k) is None:
            setattr(args, k, v)
    args.bf16 = args.config == "c5"
    return args


def spmm_bytes(n_rows: int, nnz: int, F: int, s: int = 4) -> int:
    """Edge-gather algorithmic bytes of one SpMM launch:
    every edge gathers one F-wide source row, col (int32) + val (f32) read
    once, rowptr (int64) once, output row written once."""
    return nnz * F * s + nnz * 8 + (n_rows + 1) * 8 + n_rows * F * s


def load_pmc_traffic(workload: str):
    """Per-launch HBM bytes of the dominant kernel from the committed rocprofv3
    PMC summary (profiles/*pmc*.json, produced by tools/pmc_summary.py)."""
    import glob

    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*.json")), reverse=True):
        try:
            d = json.load(open(path))
        except Exception:
            continue
        if d.get("workload") == workload and d.get("hbm_bytes_per_launch"):
            return d["hbm_bytes_per_launch"], os.path.basename(path)
    return None, None


def cpu_baseline(g, hids, depth, steps):
    """The oracle (C restatement of torch_sparse spmm_cpu + torch CPU GEMMs)
    timed on this host for `steps` full fwd+bwd steps of the same workload."""
    from oracle import model_ref as O

    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
    threads = min(threads, len(os.sched_getaffinity(0)))
    torch.set_num_threads(threads)
    os.environ.setdefault("OMP_NUM_THREADS", str(threads))
    A = O.csr_from_coo(g.row, g.col, g.val, g.m, g.n)
    AT = O.csr_transpose(*A, g.m, g.n)
    sd = {k: v.clone().requires_grad_(True) for k, v in O.init_state_dict(8, 8, hids, depth).items()}
    x_s, x_t = torch.from_numpy(g.x_s), torch.from_numpy(g.x_t)
    y_s, y_t = torch.from_numpy(g.y_s), torch.from_numpy(g.y_t)
    opt = torch.optim.Adam(list(sd.values()), lr=1e-3, weight_decay=5e-4)

    def step():
        lc, lv = O.gcn_fc_forward(sd, x_s, x_t, A, AT, depth)
        loss = O.balanced(lc, lv, y_s, y_t)
        opt.zero_grad()
        loss.backward()
        opt.step()

    step()  # untimed warm-up: first-touch allocations, MKL / OpenMP thread start-up
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    dt = (time.perf_counter() - t0) / steps
    return dt, threads


def cpu_inference(g, hids, depth, steps, bf16=False):
    """The oracle's eval-mode forward (C spmm_cpu loop + torch CPU GEMMs, fp32: the reference's
    CPU arithmetic) + inference_gnn (val.py:106-124) on this host, `steps` graphs after one
    untimed warm-up -- the reference's timed inference path (scripts/pred_basis.py:113-118)."""
    from oracle import model_ref as O

    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
    threads = min(threads, len(os.sched_getaffinity(0)))
    torch.set_num_threads(threads)
    A = O.csr_from_coo(g.row, g.col, g.val, g.m, g.n)
    AT = O.csr_transpose(*A, g.m, g.n)
    sd = O.init_state_dict(8, 8, hids, depth)
    x_s, x_t = torch.from_numpy(g.x_s), torch.from_numpy(g.x_t)

    def infer():
        with torch.no_grad():
            lc, lv = O.gcn_fc_forward(sd, x_s, x_t, A, AT, depth)
            return O.inference_gnn(torch.cat((lc, lv)), g.m)

    infer()
    t0 = time.perf_counter()
    for _ in range(steps):
        infer()
    return (time.perf_counter() - t0) / steps, threads


def cpu_spmm(g, F, reps=3):
    """SURVEY.md §8d's two CPU SpMM numbers at F = hid, per direction (median of
    `reps`): (1) the oracle's C restatement of torch_sparse spmm_cpu (OpenMP,
    the reference's loop order), (2) torch.sparse CSR mm (MKL)."""
    from oracle import model_ref as O

    rs = np.random.default_rng(5)
    A = O.csr_from_coo(g.row, g.col, g.val, g.m, g.n)
    AT = O.csr_transpose(*A, g.m, g.n)
    X = {"cons<-vars": rs.standard_normal((g.n, F), dtype=np.float32),
         "vars<-cons": rs.standard_normal((g.m, F), dtype=np.float32)}
    mats = {"cons<-vars": A, "vars<-cons": AT}
    out = {}
    for d, (rp, col, val) in mats.items():
        x = X[d]
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            O.spmm_f32(rp, col, val, x)
            ts.append(time.perf_counter() - t0)
        sp = torch.sparse_csr_tensor(torch.from_numpy(rp), torch.from_numpy(col.astype(np.int64)),
                                     torch.from_numpy(val), size=(len(rp) - 1, x.shape[0]))
        xt = torch.from_numpy(x)
        tm = []
        for _ in range(reps):
            t0 = time.perf_counter()
            torch.sparse.mm(sp, xt)
            tm.append(time.perf_counter() - t0)
        nnz = len(col)
        out[d] = {"oracle_c_ms": float(np.median(ts)) * 1e3, "oracle_c_edges_per_s": nnz / float(np.median(ts)),
                  "torch_sparse_mm_ms": float(np.median(tm)) * 1e3,
                  "torch_sparse_mm_edges_per_s": nnz / float(np.median(tm))}
    return out


def workload_name(args) -> str:
    dt = ", bf16" if args.bf16 else ""
    kind = "synthetic block LP (8 row blocks, rho=%g)" % args.rho if args.config == "c4" else "synthetic LP"
    what = "eval forward + inference_gnn" if getattr(args, "inference", False) else "fwd+bwd+Adam"
    return (f"{args.config}: {kind} {args.m}x{args.n} nnz={args.nnz}, "
            f"GCN_FC(8,8,hids={args.hids},depth={args.depth}{dt}) {what}")


def _free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def self_launch(args) -> int:
    """--gpus N > 1 without a launcher: start N ranks as child processes (this process never
    initialises the GPU and never execs), forward their output, return the first failing exit
    status (0 if all ranks succeed).  If one rank fails the others are stopped."""
    import signal
    import subprocess

    port = _free_port()
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        if args.share_gpu:
            env["LPGNN_DIST_BACKEND"] = "gloo"
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      start_new_session=True))
    rc = 0
    try:
        while procs:
            for p in list(procs):
                code = p.poll()
                if code is None:
                    continue
                procs.remove(p)
                if code != 0 and rc == 0:
                    rc = code
                    for q in procs:  # a failed rank: stop the others (they would wait in a collective)
                        os.killpg(q.pid, signal.SIGTERM)
            time.sleep(0.2)
    except KeyboardInterrupt:
        for q in procs:
            os.killpg(q.pid, signal.SIGTERM)
        raise
    return rc


def main():
    args = parse()
    if args.print_workload:
        print(workload_name(args))
        return
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(self_launch(args))
    if args.inference and (args.gpus > 1 or args.partitioned):
        raise SystemExit("--inference times the one-GPU eval path (the reference's scripts/pred_basis.py)")
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    # LPGNN_DIST_BACKEND=gloo: a rehearsal of the N-rank path with several ranks sharing the visible
    # GPU(s) (host-staged exchanges); the measured runs use RCCL ("nccl"), one rank per GPU
    backend = os.environ.get("LPGNN_DIST_BACKEND", "nccl")
    if backend not in ("nccl", "gloo"):
        raise SystemExit(f"LPGNN_DIST_BACKEND={backend}: nccl or gloo")
    if backend == "gloo":
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    distributed = world > 1 or args.partitioned
    if distributed:
        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29531")
        if backend == "gloo":
            dist.init_process_group("gloo", rank=rank, world_size=world)
        else:
            dist.init_process_group("nccl", device_id=dev, rank=rank, world_size=world)

    import lpgnn
    from lpgnn import BipartiteBatch, BipartiteCSR, GCN_FC, synth
    from lpgnn.timing import TIMER
    from lpgnn.train import make_optimizer, train_step

    exch = None
    if not distributed:
        if args.config == "c4":  # the whole c4 graph on one GPU
            from lpgnn.partition import bench_spec

            g = bench_spec(args, 1).full()
        else:
            g = synth.uniform_lp(args.m, args.n, args.nnz, seed=0)
        adj = BipartiteCSR.from_coo(g.row, g.col, g.val, g.m, g.n, device=dev)
        batch = BipartiteBatch(x_s=torch.from_numpy(g.x_s).to(dev), x_t=torch.from_numpy(g.x_t).to(dev),
                               y_s=torch.from_numpy(g.y_s).to(dev), y_t=torch.from_numpy(g.y_t).to(dev),
                               edge_index=adj, s_bs=g.m, t_bs=g.n)
        torch.manual_seed(0)
        model = GCN_FC(8, 8, hids=args.hids, depth=args.depth,
                       compute_dtype=torch.bfloat16 if args.bf16 else torch.float32).to(dev)
        if args.inference:
            # the reference's timed path (scripts/pred_basis.py:113-118, 169-173): eval-mode
            # model(batch) + inference_gnn on the concatenated logits (val.py:106-124, with its
            # invariant checks), one graph per step
            from lpgnn.val import inference_gnn

            model.eval()

            def step():
                with torch.no_grad():
                    lc, lv = model(batch)
                    return inference_gnn(torch.cat((lc, lv), 0), g.m)
        else:
            opt, _ = make_optimizer(model)
            step = lambda: train_step(model, batch, opt)
        local_nnz = g.nnz
        workload = workload_name(args)
        parallelism = "single"
    else:
        from lpgnn import partition

        job = partition.build_bench_job(args, rank, world, dev)
        step, local_nnz, g = job.step, job.local_nnz, None
        workload = job.workload
        parallelism = f"rowpart{world}"
        spec = job.spec

    def sync():
        torch.cuda.synchronize()
        if distributed:
            torch.distributed.barrier()
            torch.cuda.synchronize()

    for _ in range(args.warmup):
        step()
    sync()
    TIMER.reset()
    TIMER.enabled = True
    tw0 = time.clock_gettime_ns(time.CLOCK_BOOTTIME)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    sync()
    dt = time.perf_counter() - t0
    if os.environ.get("LPGNN_TRACE_WINDOW"):  # the timed region on the profiler's clock (tools/trace_timeline.py)
        print(f"TRACE_WINDOW rank={rank} boottime_ns={tw0} {time.clock_gettime_ns(time.CLOCK_BOOTTIME)}",
              file=sys.stderr, flush=True)
    TIMER.enabled = False
    kern = TIMER.summary()
    per_launch = TIMER.launches()
    if distributed:  # the boundary exchange on its own, after the timed steps
        exch = partition.time_exchange(job.batch.edge_index.ex, args.hids, dev)
        exch.update(halo_rows=int(job.plan.halo.shape[0]), owned_vars=job.plan.n_own,
                    boundary_vars_global=job.plan.n_boundary_global)
        gathered = [None] * world
        torch.distributed.all_gather_object(gathered, exch)
        exch = {"per_rank": gathered,
                "note": "standalone F=hid owner-reduce / halo-broadcast of [n_local, F] fp32 rows (median ms, "
                        "barrier + sync around each); in the step they run async under independent compute"}
        if args.config == "c4" and world > 1 and args.rho_sweep:  # after the timed region
            exch["rho_sweep"] = partition.rho_sweep(args, rank, world,
                                                    [float(r) for r in args.rho_sweep.split(",")], args.hids)

    # hid-width SpMM launches (the metric's kernel) measured on their stream
    hid_keys = [k for k in kern if k[0] == "spmm" and k[3] == args.hids]
    launches = sum(kern[k][0] for k in hid_keys)
    spmm_ms = sum(kern[k][1] for k in hid_keys)
    nnz_of = lambda k: local_nnz  # every launch traverses the local graph's edges once
    esz = 2 if args.bf16 else 4
    bytes_total = sum(kern[k][0] * spmm_bytes(k[1], nnz_of(k), k[3], esz) for k in hid_keys)
    # dense GEMMs of hidden width on the hand-written kernels (FC forward + x3 input and weight
    # gradients; K >= hid): MFMA utilisation.  x3 = fp32 through the exact three-way bf16 split,
    # 6 bf16 MFMA products per fp32 product, so its MFMA-bound peak is the dense bf16 peak / 6.
    fc_keys = [k for k in kern if k[0] in ("fc", "wgrad") and k[3] >= args.hids and k[2] >= 64]
    x3 = any(str(k[4]).endswith("x3") for k in fc_keys)
    fc_flops = sum(kern[k][0] * 2.0 * k[1] * k[2] * k[3] for k in fc_keys)
    fc_ms = sum(kern[k][1] for k in fc_keys)
    fc_peak = BF16_MFMA_PEAK_TFLOPS if args.bf16 else (BF16_MFMA_PEAK_TFLOPS / 6 if x3 else FP32_MFMA_PEAK_TFLOPS)
    fc_tf = fc_flops / (fc_ms / 1e3) / 1e12 if fc_ms > 0 else 0.0
    edges_local = launches * local_nnz / args.steps  # per step
    t = torch.tensor([dt], device=dev)
    e = torch.tensor([edges_local], device=dev, dtype=torch.float64)
    if distributed:
        import torch.distributed as dist

        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(e, op=dist.ReduceOp.SUM)
    dt_max = t.item()
    value = e.item() * args.steps / dt_max

    achieved = bytes_total / (spmm_ms / 1e3) / 1e9 if spmm_ms > 0 else 0.0
    per_launch_bytes = bytes_total / max(launches, 1)
    traffic, traffic_src = load_pmc_traffic(workload)
    if distributed and backend != "nccl":
        workload += f" [rehearsal: {world} ranks over {backend} sharing {torch.cuda.device_count()} GPU(s)]"
    out = {
        "metric": "edges/sec bipartite SpMM (hid=1024, depth=3) at 1/2/4/8 MI355X; % HBM roofline",
        "value": value,
        "unit": "edges/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt_max / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong" if args.config == "c4" else "weak",
        "vs_baseline": None,
        "dtype": "bf16" if args.bf16 else "fp32",
        "data": "synthetic (seeded uniform LP graph, LP feature layout; random-init GCN_FC weights)",
        "config": {"workload": workload, "n_cons": spec.m if distributed else args.m,
                   "n_vars": spec.n if distributed else args.n, "nnz": spec.nnz if distributed else args.nnz,
                   "hid": args.hids, "depth": args.depth, "parallelism": parallelism},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": ("lpg spmm_bf16_rowslim / rowwave" if args.bf16 else "lpg spmm_f32_rowslim / rowwave")
                               + " (F=hid, both directions, fwd+bwd)",
                     "bytes_per_launch": per_launch_bytes,
                     "avg_launch_ms": spmm_ms / max(launches, 1), "launches": launches,
                     "traffic_source": traffic_src},
        "fc_roofline": {"bound": "mfma", "achieved": fc_tf, "peak": fc_peak, "unit": "TFLOP/s",
                        "frac": fc_tf / fc_peak, "launches": sum(kern[k][0] for k in fc_keys),
                        "kernel": ("lpg fc_bf16 + wgrad_bf16 (hidden-width GEMMs, fwd + bwd: FC forward, input "
                                   "gradients on the FC kernel, weight gradients)" if args.bf16 else
                                   "lpg fc_fwd_x3 + wgrad_x3 (hidden-width GEMMs, fwd + bwd; fp32 via exact "
                                   "3-way bf16 split, peak = dense bf16 / 6)" if x3 else
                                   "lpg fc_fwd_f32 (hidden GraphConv FC, fwd)"),
                        "fp32_mfma_peak_frac": None if args.bf16 else fc_tf / FP32_MFMA_PEAK_TFLOPS,
                        # the bf16 MFMA work these launches issue (x3: 6 bf16 products per fp32 product),
                        # comparable with a plain bf16 GEMM's rate on this chip
                        "bf16_mfma_equiv_tflops": fc_tf * (6 if x3 and not args.bf16 else 1)},
        "spmm_directions": {
            ("cons<-vars" if (k[1], k[2]) == (args.m, args.n) and not distributed else
             "vars<-cons" if (k[1], k[2]) == (args.n, args.m) and not distributed else f"{k[1]}x{k[2]}"):
            {"median_ms": float(np.median(v)), "launches": len(v),
             "edges_per_s": local_nnz / (float(np.median(v)) / 1e3),
             "roofline_frac": spmm_bytes(k[1], local_nnz, k[3], esz) / (float(np.median(v)) / 1e3) / 1e9
             / HBM_PEAK_GBS}
            for k, v in per_launch.items() if k[0] == "spmm" and k[3] == args.hids},
        "spmm_edges_per_s_kernel": launches * local_nnz / (spmm_ms / 1e3) if spmm_ms > 0 else None,
        "spmm_ms_per_step": spmm_ms / args.steps,
        "kernels": {f"{k[0]}[{k[1]}x{k[2]},F={k[3]},{k[4]}]": {"launches": v[0], "ms": v[1]}
                    for k, v in sorted(kern.items())},
        "library": lpgnn.library_path(),
        "max_hbm_allocated_gb": torch.cuda.max_memory_allocated(dev) / 1e9,
    }
    if exch is not None:
        out["exchange"] = exch
    if args.inference:
        out["mode"] = "inference: eval-mode model(batch) + inference_gnn (scripts/pred_basis.py:113-118)"
        out["ms_per_graph"] = out["ms_per_step"]
    if (rank == 0 and world == 1 and args.cpu_steps > 0 and not args.profile_only and g is not None
            and args.inference):
        cdt, threads = cpu_inference(g, args.hids, args.depth, args.cpu_steps)
        out["cpu_baseline"] = {"value": edges_local / cdt, "unit": "edges/s", "cores": threads, "kind": "port",
                               "sample": f"{args.cpu_steps} eval forward(s) + inference_gnn of the same "
                                         f"{args.config} graph after one untimed warm-up: oracle C spmm_cpu loop "
                                         f"(OpenMP) + torch CPU GEMMs in fp32, {cdt:.2f} s/graph",
                               "s_per_step": cdt}
    elif rank == 0 and world == 1 and args.cpu_steps > 0 and not args.profile_only and g is not None and args.config == "c2":
        cdt, threads = cpu_baseline(g, args.hids, args.depth, args.cpu_steps)
        out["cpu_baseline"] = {"value": edges_local / cdt, "unit": "edges/s", "cores": threads, "kind": "port",
                               "sample": f"{args.cpu_steps} full fwd+bwd+Adam step(s) of the same c2 workload after one "
                                         f"untimed warm-up step: "
                                         f"oracle C spmm_cpu loop (OpenMP) + torch CPU GEMMs, "
                                         f"{cdt:.2f} s/step",
                               "s_per_step": cdt}
        out["cpu_spmm"] = dict(cpu_spmm(g, args.hids), threads=threads,
                               note="F=hid SpMM alone on the host, median of 3 (SURVEY.md 8d CPU numbers)")
    if rank == 0:
        print(json.dumps(out), flush=True)
    if distributed:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
