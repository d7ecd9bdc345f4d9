"""Headline benchmark: edges/s of the bipartite SpMM in GCN_FC (hid=1024,
depth=3) training steps on MI355X, with the HBM-roofline fraction of the
SpMM kernel and the oracle CPU path timed beside it.

  python bench.py [--gpus N] [--steps K] [--warmup W]

One workload family at every N (the line the driver turns into a scaling curve):

* headline ``value`` -- c2 WEAK scaling (BASELINE.json configs[1] per GPU).  A step = one
  GCN_FC(8, 8, hids=1024, depth=3) training iteration of train.py:117-129: forward (2 SpMM at F=8
  + 2 at F=1024, FC stacks, heads, add_knowledge), balanced loss, backward (2 SpMM at F=1024 + FC
  grads), Adam.  N=1: the synthetic c2 graph (100K cons x 200K vars, nnz 2M) on one GPU.  N>1: N
  c2-sized row blocks of one block LP (each block's edges leave its variable range with
  probability rho = 0.02), constraint-row partitioned, one block per rank (lpgnn.partition:
  owner reduce / halo broadcast of boundary-variable rows over RCCL).  value = (hid-width SpMM
  edge traversals of all ranks in the timed steps) / (max-over-ranks time).
* sub-record ``c4`` -- BASELINE.json configs[3] (2M x 4M, nnz 40M, fixed) at the same N: the whole
  graph on one GPU at N=1, row-partitioned over the N ranks at N>1 (STRONG scaling), with the
  locality (rho) sweep of the partition at N>1.
* sub-record ``inference`` (N=1) -- the reference's own timed path (scripts/pred_basis.py:157-176):
  eval-mode model(batch) + inference_gnn on c2, ms/graph, with the oracle's CPU inference beside it;
  ``inference_fp16`` the same after model.half() + batch_to(half=True) (its --fp16 mode, val.py:269).
* sub-record ``c5`` (N=1) -- BASELINE.json configs[4]: the c2 graph, GCN_FC(8,8,hids=2048,depth=6)
  in bf16, training steps, with its SpMM and MFMA rooflines and one oracle CPU training step (fp32,
  the reference's arithmetic) beside it.
* sub-record ``skewed`` (N=1) -- SURVEY.md §8d's skewed-degree workload: Zipf(1.5) constraint-row
  degrees (synth.skewed_lp, 100K x 200K, ~2M edges), the c2 model's training step, per-direction
  SpMM rooflines (the heavy-row units live).

With --gpus N > 1 and no RANK / WORLD_SIZE in the environment, bench.py launches the N ranks
itself (one child process per GPU, started before this process touches the GPU; rank 0 prints
the JSON line) -- the same line as under ``torch.distributed.run --nproc-per-node N``.
``--share-gpu`` makes the N ranks share the visible GPU(s) over gloo (a rehearsal on a 1-GPU
box; the measured runs use RCCL, one rank per GPU).

``--config c4`` times c4 as the headline instead, ``--config c5`` BASELINE.json configs[4]
(same graph, GCN_FC hids=2048 depth=6, bf16 activations / SpMM storage / MFMA FC, fp32 master
weights; one GPU) -- the MFMA-utilisation stress line, not the headline.  ``--inference`` times
the eval path as the headline (``--fp16``: the reference's model.half() mode, val.py:269).
"""
from __future__ import annotations

import argparse
import copy
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "lp-gnn_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

METRIC = "edges/sec bipartite SpMM (hid=1024, depth=3) at 1/2/4/8 MI355X; % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP32_MFMA_PEAK_TFLOPS = 157.3
BF16_MFMA_PEAK_TFLOPS = 2500.0  # dense (MI355X_MICROARCH.md; the 5 PF figure is 2:1 sparse); fp16 the same


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--config", choices=("c2", "c4", "c5", "skewed"), default="c2",
                    help="c2 = headline fp32 hid 1024 depth 3, weak scaling over N (default); c4 = 2M x 4M nnz 40M "
                         "(whole graph at N=1, row-partitioned at N>1: strong scaling); c5 = bf16 hid 2048 depth 6")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--m", type=int, default=None)
    ap.add_argument("--n", type=int, default=None)
    ap.add_argument("--nnz", type=int, default=None)
    ap.add_argument("--hids", type=int, default=None)
    ap.add_argument("--depth", type=int, default=None)
    ap.add_argument("--rho", type=float, default=0.02, help="boundary edge fraction for N>1 partitions")
    ap.add_argument("--cpu-steps", type=int, default=1, help="oracle CPU steps for cpu_baseline (0 = skip)")
    ap.add_argument("--profile-only", action="store_true", help="no CPU baseline, no sub-records (rocprof runs)")
    ap.add_argument("--print-workload", action="store_true", help="print the workload string and exit")
    ap.add_argument("--vendor", type=int, default=1,
                    help="1: time rocSPARSE's SpMM (torch.sparse.mm) beside ours on the c2 graph at N=1 (vendor_spmm)")
    ap.add_argument("--partitioned", action="store_true",
                    help="use the row-partitioned RCCL path even at N=1 (the N>1 code path)")
    ap.add_argument("--share-gpu", action="store_true",
                    help="self-launched N>1: ranks share the visible GPU(s) over gloo (rehearsal, not a measurement)")
    ap.add_argument("--rho-sweep", default="0,0.02,0.1,1.0",
                    help="c4 at N>1: rho values whose partition boundary counts go into the JSON ('' = off)")
    ap.add_argument("--inference", action="store_true",
                    help="time eval-mode forward + inference_gnn (the reference's timed path) instead of training")
    ap.add_argument("--fp16", action="store_true",
                    help="with --inference: the reference's --fp16 mode (model.half(), batch_to(half=True))")
    ap.add_argument("--sub", default="c4,inference,inference_fp16,c5,skewed",
                    help="sub-records after the headline ('' = none): c4 (configs[3] at the same N), "
                         "inference (N=1: the reference's timed eval path on c2), inference_fp16 (the same in "
                         "the reference's --fp16 mode), c5 (N=1: configs[4], bf16 hid 2048 depth 6), skewed "
                         "(N=1: Zipf(1.5) row degrees, the c2 model)")
    ap.add_argument("--c5-steps", type=int, default=10)
    ap.add_argument("--c5-warmup", type=int, default=3)
    ap.add_argument("--c5-cpu-steps", type=int, default=1, help="oracle CPU training steps of c5 (0 = skip)")
    ap.add_argument("--c4-steps", type=int, default=5)
    ap.add_argument("--c4-warmup", type=int, default=2)
    ap.add_argument("--c4-scale", type=int, default=1, help="c4 sub-record at 1/scale size (rehearsals)")
    ap.add_argument("--inf-steps", type=int, default=20)
    args = ap.parse_args(argv)
    fill(args)
    return args


def fill(args):
    from lpgnn.synth import CONFIGS

    for k, v in CONFIGS[args.config].items():
        if getattr(args, k) is None:
            setattr(args, k, v)
    args.bf16 = args.config == "c5"
    if args.fp16 and not args.inference:
        raise SystemExit("--fp16 is the reference's inference mode (val.py:269, pred_basis.py:146): use --inference")
    return args


def spmm_bytes(n_rows: int, nnz: int, F: int, s: int = 4) -> int:
    """Edge-gather algorithmic bytes of one SpMM launch:
    every edge gathers one F-wide source row, col (int32) + val (f32) read
    once, rowptr (int64) once, output row written once."""
    return nnz * F * s + nnz * 8 + (n_rows + 1) * 8 + n_rows * F * s


def load_pmc_traffic(key: str):
    """Per-launch HBM bytes of the dominant kernel from the committed rocprofv3
    PMC summary (profiles/*pmc*.json, produced by tools/pmc_summary.py), matched
    on its ``workload`` key (the N=1 workload string, or a rank-share key)."""
    import glob

    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*.json")), reverse=True):
        try:
            d = json.load(open(path))
        except Exception:
            continue
        if d.get("workload") == key and d.get("hbm_bytes_per_launch"):
            return d["hbm_bytes_per_launch"], os.path.basename(path)
    return None, None


def load_pmc_dir_traffic(key: str):
    """Per-direction HBM bytes per launch of the F=hid SpMM ({"cons<-vars": B, "vars<-cons": B}) from the
    committed per-direction PMC summary (profiles/*pmc_dirs*.json, tools/pmc_spmm_dirs.py), or None."""
    import glob

    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc_dirs*.json")), reverse=True):
        try:
            d = json.load(open(path))
        except Exception:
            continue
        if d.get("workload") == key and d.get("directions"):
            return d["directions"]
    return None


def rank_share_key(family: str, world: int, rank: int = 0) -> str:
    """The PMC key of one rank's share of a partitioned workload (tools/pmc_rank_share.py)."""
    return f"{family} rank share: rank {rank} of {world}, F=1024 SpMM both directions"


def _arith() -> str:
    from lpgnn.options import DEFAULT

    return DEFAULT.arith


def _threads():
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
    return min(threads, len(os.sched_getaffinity(0)))


def cpu_baseline(g, hids, depth, steps, warmup=True):
    """The oracle (C restatement of torch_sparse spmm_cpu + torch CPU GEMMs)
    timed on this host for `steps` full fwd+bwd steps of the same workload (after one untimed
    warm-up step unless ``warmup`` is False -- c5, whose CPU step is long, runs after the c2 leg
    has already started the MKL / OpenMP threads)."""
    from oracle import model_ref as O

    threads = _threads()
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

    if warmup:
        step()  # untimed warm-up: first-touch allocations, MKL / OpenMP thread start-up
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    dt = (time.perf_counter() - t0) / steps
    return dt, threads


def cpu_inference(g, hids, depth, steps, fp16=False):
    """The oracle's eval-mode forward (C spmm_cpu loop + torch CPU GEMMs, fp32: the reference's
    CPU arithmetic; ``fp16``: the same with every stored tensor rounded to fp16, the oracle of the
    --fp16 mode) + inference_gnn (val.py:106-124) on this host, `steps` graphs after one untimed
    warm-up -- the reference's timed inference path (scripts/pred_basis.py:113-118)."""
    from oracle import model_ref as O

    threads = _threads()
    torch.set_num_threads(threads)
    A = O.csr_from_coo(g.row, g.col, g.val, g.m, g.n)
    AT = O.csr_transpose(*A, g.m, g.n)
    sd = O.init_state_dict(8, 8, hids, depth)
    x_s, x_t = torch.from_numpy(g.x_s), torch.from_numpy(g.x_t)

    def infer():
        with torch.no_grad():
            if fp16:
                lc, lv = O.gcn_fc_forward_fp16(sd, x_s, x_t, A, AT, depth)
            else:
                lc, lv = O.gcn_fc_forward(sd, x_s, x_t, A, AT, depth)
            return O.inference_gnn(torch.cat((lc.float(), lv.float())), g.m)

    infer()
    t0 = time.perf_counter()
    for _ in range(steps):
        infer()
    return (time.perf_counter() - t0) / steps, threads


def vendor_spmm(g, F, dev, reps=5):
    """The vendor sparse library on the headline SpMM, on the GPU beside ours: rocSPARSE through
    torch.sparse.mm on a CSR tensor (fp32, F = hid) against lpg_spmm_f32, per direction, median of
    `reps` after one warm-up (HIP events on the current stream).  Not a baseline the metric uses."""
    import lpgnn
    from lpgnn.sparse import spmm_forward

    adj = lpgnn.BipartiteCSR.from_coo(g.row, g.col, g.val, g.m, g.n, device=dev)
    gen = torch.Generator(device=dev).manual_seed(5)
    out = {}
    for d, csr in (("cons<-vars", adj.fwd), ("vars<-cons", adj.bwd)):
        x = torch.randn(csr.n_cols, F, device=dev, generator=gen)
        sp = torch.sparse_csr_tensor(csr.rowptr, csr.col.long(), csr.val, size=(csr.n_rows, csr.n_cols))

        def med(fn):
            fn()
            ts = []
            for _ in range(reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                fn()
                e1.record()
                torch.cuda.synchronize(dev)
                ts.append(e0.elapsed_time(e1))
            return float(np.median(ts))
        t_v = med(lambda: torch.sparse.mm(sp, x))
        t_o = med(lambda: spmm_forward(csr, x))
        diff = float((torch.sparse.mm(sp, x) - spmm_forward(csr, x)).abs().max())
        out[d] = {"rocsparse_ms": t_v, "rocsparse_edges_per_s": csr.nnz / (t_v / 1e3), "ours_ms": t_o,
                  "ours_edges_per_s": csr.nnz / (t_o / 1e3), "speedup": t_v / t_o, "max_abs_diff": diff}
        del x, sp
    return out


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
        import warnings

        with warnings.catch_warnings():
            warnings.simplefilter("ignore")  # torch's "sparse CSR support is in beta" notice (keeps stderr short)
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
    """The one-GPU workload string (also the PMC key of the N=1 line)."""
    dt = ", bf16" if args.bf16 else (", fp16" if getattr(args, "fp16", False) else "")
    kind = ("synthetic block LP (8 row blocks, rho=%g)" % args.rho if args.config == "c4" else
            "synthetic Zipf(1.5) row-degree LP" if args.config == "skewed" else "synthetic LP")
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


# ------------------------------------------------------------------- measurement
class Ctx:
    """Per-process run context: rank, world, device, backend, whether a process group is up."""

    def __init__(self, rank, world, dev, backend, distributed):
        self.rank, self.world, self.dev, self.backend, self.distributed = rank, world, dev, backend, distributed

    def sync(self):
        torch.cuda.synchronize()
        if self.distributed:
            torch.distributed.barrier()
            torch.cuda.synchronize()

    def gather(self, obj):
        if not self.distributed:
            return [obj]
        out = [None] * self.world
        torch.distributed.all_gather_object(out, obj)
        return out


def timed(ctx, step, steps, warmup):
    """W untimed warm-up steps, then exactly K steps bracketed by a barrier + device sync on both
    sides; the hot-path kernels' HIP events recorded on their launch stream (lpgnn.timing).
    Returns (this rank's seconds, {key: (launches, ms)}, {key: [ms per launch]})."""
    from lpgnn.timing import TIMER

    for _ in range(warmup):
        step()
    ctx.sync()
    TIMER.reset()
    TIMER.enabled = True
    tw0 = time.clock_gettime_ns(time.CLOCK_BOOTTIME)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    ctx.sync()
    dt = time.perf_counter() - t0
    if os.environ.get("LPGNN_TRACE_WINDOW"):  # the timed region on the profiler's clock (tools/trace_timeline.py)
        print(f"TRACE_WINDOW rank={ctx.rank} boottime_ns={tw0} {time.clock_gettime_ns(time.CLOCK_BOOTTIME)}",
              file=sys.stderr, flush=True)
    TIMER.enabled = False
    kern, per_launch = TIMER.summary(), TIMER.launches()
    TIMER.reset()
    return dt, kern, per_launch


def report(ctx, dt, kern, per_launch, *, steps, hids, local_nnz, esz, traffic_key, single_dirs=None, fp16=False,
           training=True, touched=None):
    """value, ms_per_step, the SpMM roofline and the hidden-width GEMM roofline of one timed run,
    aggregated over the ranks (collective: every rank calls it).

    value = sum over ranks of the hid-width SpMM edge traversals / the max-over-ranks wall time.
    roofline.achieved = per-GPU GB/s = (sum over ranks of the algorithmic bytes of the F=hid SpMM
    launches) / (N x the slowest rank's summed SpMM kernel time); at N=1 bytes / time of the one GPU.
    roofline.per_rank keeps every rank's own fraction."""
    hid_keys = [k for k in kern if k[0] == "spmm" and k[3] == hids]
    launches = sum(kern[k][0] for k in hid_keys)
    spmm_ms = sum(kern[k][1] for k in hid_keys)
    bytes_total = sum(kern[k][0] * spmm_bytes(k[1], local_nnz, k[3], esz) for k in hid_keys)
    # dense GEMMs of hidden width on the hand-written kernels (FC forward + x3 input and weight
    # gradients; K >= hid): MFMA utilisation.  x3 = fp32 through the exact three-way bf16 split,
    # 6 bf16 MFMA products per fp32 product, so its MFMA-bound peak is the dense bf16 peak / 6.
    fc_keys = [k for k in kern if k[0] in ("fc", "wgrad") and k[3] >= hids and k[2] >= 64]
    # matrix-core products per fp32 product: x3 six bf16, f16x2 three fp16 (LPGNN_FC_ARITH=f16x2)
    prods = lambda k: 6 if str(k[4]).endswith("x3") else 3 if str(k[4]).endswith("f16x2") else 1  # noqa: E731
    x3 = any(prods(k) > 1 for k in fc_keys)
    f16x2 = any(prods(k) == 3 for k in fc_keys)
    half = esz == 2
    fc_flops = sum(kern[k][0] * 2.0 * k[1] * k[2] * k[3] for k in fc_keys)
    fc_work = sum(kern[k][0] * 2.0 * k[1] * k[2] * k[3] * prods(k) for k in fc_keys)
    fc_ms = sum(kern[k][1] for k in fc_keys)
    fc_launches = sum(kern[k][0] for k in fc_keys)
    # RCCL exchanges (lpgnn.partition._Pending): issue -> consumption span and the compute stream's
    # exposed wait, both HIP-event spans on the compute stream
    ex_span = sum(v[1] for k, v in kern.items() if k[0] == "exchange" and k[4] == "span")
    ex_exposed = sum(v[1] for k, v in kern.items() if k[0] == "exchange" and k[4] == "exposed")
    ex_n = sum(v[0] for k, v in kern.items() if k[0] == "exchange" and k[4] == "span")
    mine = dict(dt=dt, edges=launches * local_nnz, bytes=bytes_total, spmm_ms=spmm_ms, launches=launches,
                fc_flops=fc_flops, fc_work=fc_work, fc_ms=fc_ms, ex_span=ex_span, ex_exposed=ex_exposed, ex_n=ex_n)
    every = ctx.gather(mine)
    dt_max = max(r["dt"] for r in every)
    world = len(every)
    value = sum(r["edges"] for r in every) / dt_max
    t_max = max(r["spmm_ms"] for r in every)
    b_sum = sum(r["bytes"] for r in every)
    achieved = b_sum / (world * t_max / 1e3) / 1e9 if t_max > 0 else 0.0
    traffic, traffic_src = load_pmc_traffic(traffic_key)
    roof = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
            "kernel": ("lpg spmm_%s_rowslim / rowwave" % ("f16" if fp16 else "bf16" if half else "f32"))
                      + " (F=hid, both directions%s)" % (", fwd+bwd" if training else ", eval forward"),
            "bytes_per_launch": b_sum / max(1, sum(r["launches"] for r in every)),
            "avg_launch_ms": sum(r["spmm_ms"] for r in every) / max(1, sum(r["launches"] for r in every)),
            "launches": sum(r["launches"] for r in every), "traffic_source": traffic_src, "traffic_key": traffic_key}
    if world > 1:
        roof["aggregation"] = ("per-GPU: sum of all ranks' algorithmic bytes / (N x the slowest rank's SpMM "
                               "kernel time); traffic = the PMC of rank 0's share on one GPU")
        roof["achieved_all_gpus"] = b_sum / (t_max / 1e3) / 1e9 if t_max > 0 else 0.0
        roof["peak_all_gpus"] = HBM_PEAK_GBS * world
        roof["per_rank"] = [{"frac": (r["bytes"] / (r["spmm_ms"] / 1e3) / 1e9 / HBM_PEAK_GBS) if r["spmm_ms"] else 0.0,
                             "avg_launch_ms": r["spmm_ms"] / max(1, r["launches"]), "launches": r["launches"],
                             "bytes_per_launch": r["bytes"] / max(1, r["launches"])} for r in every]
    fc_tf_all = sum(r["fc_flops"] for r in every) / (max(r["fc_ms"] for r in every) * world / 1e3) / 1e12 \
        if any(r["fc_ms"] for r in every) else 0.0
    fc_peak = BF16_MFMA_PEAK_TFLOPS if half else (BF16_MFMA_PEAK_TFLOPS / 6 if x3 else FP32_MFMA_PEAK_TFLOPS)
    work_tf = sum(r["fc_work"] for r in every) / (max(r["fc_ms"] for r in every) * world / 1e3) / 1e12 \
        if any(r["fc_ms"] for r in every) else 0.0
    if f16x2 and not half:  # mixed products per fp32 product: the peak the launches' matrix-core work implies
        fc_peak = fc_tf_all * BF16_MFMA_PEAK_TFLOPS / work_tf if work_tf > 0 else BF16_MFMA_PEAK_TFLOPS / 6
    fc = {"bound": "mfma", "achieved": fc_tf_all, "peak": fc_peak, "unit": "TFLOP/s", "frac": fc_tf_all / fc_peak,
          "launches": fc_launches,
          "kernel": ("lpg fc_f16 (hidden-width FC forward on v_mfma_f32_16x16x32_f16)" if fp16 else
                     "lpg fc_bf16 + wgrad_bf16 (hidden-width GEMMs, fwd + bwd: FC forward, input "
                     "gradients on the FC kernel, weight gradients)" if half else
                     "lpg fc_x3_wide f16x2 + wgrad_x3w f16x2 (hidden-width GEMMs, fwd + bwd; fp32 via two "
                     "row-scaled fp16 terms (3 products) and the exact 3-way bf16 split (6); peak = dense "
                     "bf16 over the launches' products)" if f16x2 and not half else
                     "lpg fc_fwd_x3 + wgrad_x3 (hidden-width GEMMs, fwd + bwd; fp32 via exact "
                     "3-way bf16 split, peak = dense bf16 / 6)" if x3 else
                     "lpg fc_fwd_f32 (hidden GraphConv FC, fwd)"),
          "fp32_mfma_peak_frac": None if half else fc_tf_all / FP32_MFMA_PEAK_TFLOPS,
          # the bf16 MFMA work these launches issue (x3: 6 bf16 products per fp32 product),
          # comparable with a plain bf16 GEMM's rate on this chip
          "bf16_mfma_equiv_tflops": work_tf if not half else fc_tf_all}
    dirs, narrow = {}, {}
    dir_traffic = load_pmc_dir_traffic(traffic_key)
    for k, v in per_launch.items():
        if k[0] != "spmm":
            continue
        name = (single_dirs or {}).get((k[1], k[2]), f"{k[1]}x{k[2]}")
        med = float(np.median(v))
        if k[3] <= 64:  # conv1's input (F = 8): the narrow kernel, latency-bound, its time per launch
            narrow[name] = med
            continue
        if k[3] != hids:
            continue
        d = {"median_ms": med, "launches": len(v), "edges_per_s": local_nnz / (med / 1e3),
             "roofline_frac": spmm_bytes(k[1], local_nnz, k[3], esz) / (med / 1e3) / 1e9 / HBM_PEAK_GBS}
        if touched and (k[1], k[2]) in touched:  # SURVEY 8d compulsory model: each touched source row once
            d["compulsory_frac"] = (spmm_bytes(k[1], local_nnz, k[3], esz) - (local_nnz - touched[(k[1], k[2])])
                                    * k[3] * esz) / (med / 1e3) / 1e9 / HBM_PEAK_GBS
        if dir_traffic and name in dir_traffic:  # counter bytes (PMC) over the measured launch time
            d["traffic_bytes"] = dir_traffic[name]
            d["traffic_frac"] = dir_traffic[name] / (med / 1e3) / 1e9 / HBM_PEAK_GBS
        # what bounds the direction, from the three models: HBM when the counter bytes run near the peak;
        # the cache hierarchy when the edge gathers exceed what HBM could deliver (hot source rows re-read
        # from L2 / MALL: the compulsory bytes are the HBM floor, the gathers the cache's work)
        tf = d.get("traffic_frac")
        d["bound"] = ("hbm" if (tf if tf is not None else d["roofline_frac"]) >= 0.75 else
                      "cache (gathers of hot sources from L2/MALL)" if d["roofline_frac"] > 1.0 else "latency")
        dirs[name] = d
    out = {"value": value, "ms_per_step": dt_max / max(1, steps) * 1e3, "roofline": roof, "fc_roofline": fc}
    if any(r["ex_n"] for r in every):
        st = max(1, steps)
        out["exchange_overlap"] = {
            "what": "RCCL all_to_all boundary exchanges of the timed steps: span = issue -> rows consumed, "
                    "exposed = the compute stream's wait for the collective (HIP events on the compute stream); "
                    "hidden = 1 - exposed / span",
            "per_rank": [{"exchanges_per_step": r["ex_n"] / st, "span_ms_per_step": r["ex_span"] / st,
                          "exposed_ms_per_step": r["ex_exposed"] / st,
                          "hidden_frac": (1.0 - r["ex_exposed"] / r["ex_span"]) if r["ex_span"] > 0 else None}
                         for r in every],
            "max_exposed_ms_per_step": max(r["ex_exposed"] for r in every) / st}
    if narrow:
        out["narrow_ms"] = narrow
    out.update({"spmm_directions": dirs,
            "spmm_edges_per_s_kernel": launches * local_nnz / (spmm_ms / 1e3) if spmm_ms > 0 else None,
            "spmm_ms_per_step": spmm_ms / max(1, steps),
            "kernels": {f"{k[0]}[{k[1]}x{k[2]},F={k[3]},{k[4]}]": {"launches": v[0], "ms": v[1]}
                        for k, v in sorted(kern.items(), key=lambda kv: tuple(map(str, kv[0])))
                        if k[0] != "exchange"}})
    return out


# --------------------------------------------------------------------- output
HEADLINE_MAX_BYTES = 6144  # the driver keeps the last ~8 KB of stdout+stderr; the line must fit whole
SUB_NAMES = ("c4", "inference", "inference_fp16", "c5", "skewed")
BULKY = ("kernels", "cpu_spmm", "vendor_spmm", "exchange", "library") + SUB_NAMES


def _r(x, nd=4):
    """x to nd significant digits; anything that is not a real number (None, a label) as it is."""
    if isinstance(x, bool) or not isinstance(x, (int, float)):
        return x
    return float(f"{x:.{nd}g}")


def _compact_roof(roof):
    keep = ("bound", "achieved", "peak", "unit", "frac", "traffic", "bytes_per_launch", "avg_launch_ms", "launches",
            "kernel", "traffic_source")
    out = {k: (_r(roof[k], 6) if isinstance(roof[k], float) else roof[k]) for k in keep if k in roof}
    if roof.get("traffic") and roof.get("avg_launch_ms"):  # PMC bytes over the measured launch time
        out["traffic_frac"] = _r(roof["traffic"] / (roof["avg_launch_ms"] / 1e3) / 1e9 / roof["peak"])
    if "per_rank" in roof:
        out["per_rank_frac"] = [_r(r["frac"]) for r in roof["per_rank"]]
    return out


def sub_summary(name, rec):
    """One sub-record's figures for the headline: step time, value and both rooflines (the full record with
    its kernel table goes to the detail file)."""
    s = {"value": _r(rec.get("value"), 6), "ms_per_step": _r(rec.get("ms_per_step"), 5),
         "spmm_frac": _r(rec.get("roofline", {}).get("frac")), "fc_frac": _r(rec.get("fc_roofline", {}).get("frac"))}
    if rec.get("roofline", {}).get("traffic_frac") is not None:
        s["spmm_traffic_frac"] = rec["roofline"]["traffic_frac"]
    cb = rec.get("cpu_baseline")
    if cb:
        s["cpu_s"] = _r(cb.get("s_per_step", cb.get("s_per_graph")))
    if name == "skewed":  # the edge-gather, compulsory and counter-bytes fractions per direction
        s["dirs"] = {d: {k: _r(v.get(k)) for k in ("median_ms", "roofline_frac", "compulsory_frac", "traffic_frac",
                                                      "bound") if v.get(k) is not None}
                     for d, v in rec.get("spmm_directions", {}).items()}
        s["narrow_F8_ms"] = {d: _r(v) for d, v in rec.get("narrow_ms", {}).items()}
    if "exchange_overlap" in rec:
        s["max_exposed_ms"] = _r(rec["exchange_overlap"]["max_exposed_ms_per_step"])
    return s


def compact_headline(out, detail_path=None):
    """The one JSON line the driver parses: the contract's keys, both rooflines, the CPU baseline, the rank
    devices and one short summary per sub-record -- never the per-kernel tables (those stay in the detail
    file).  Asserted below HEADLINE_MAX_BYTES by tests/test_bench_report.py."""
    head = {k: v for k, v in out.items() if k not in BULKY}
    head["roofline"] = _compact_roof(out["roofline"])
    fc = out.get("fc_roofline")
    if fc:
        head["fc_roofline"] = {k: (_r(fc[k], 6) if isinstance(fc[k], float) else fc[k])
                               for k in ("bound", "achieved", "peak", "unit", "frac", "launches",
                                         "bf16_mfma_equiv_tflops") if k in fc}
        head["fc_roofline"]["kernel"] = fc.get("kernel", "")[:90]
    if "spmm_directions" in out:
        head["spmm_directions"] = {d: {"median_ms": _r(v["median_ms"]), "frac": _r(v["roofline_frac"])}
                                   for d, v in out["spmm_directions"].items()}
    d = out.get("dist", {})
    head["dist"] = {"backend": d.get("backend"), "world_size": d.get("world_size"),
                    "pci": [r.get("pci") for r in d.get("ranks", [])], "launcher": d.get("launcher")}
    if "exchange_overlap" in out:
        head["exchange_overlap"] = {"max_exposed_ms_per_step": _r(out["exchange_overlap"]["max_exposed_ms_per_step"]),
                                    "hidden_frac": [_r(r["hidden_frac"]) for r in
                                                    out["exchange_overlap"]["per_rank"]]}
    subs = {n: sub_summary(n, out[n]) for n in SUB_NAMES if n in out}
    if subs:
        head["subs"] = subs
    if detail_path:
        head["detail"] = detail_path
    for k in ("value", "ms_per_step", "ms_per_graph", "max_hbm_allocated_gb"):
        if isinstance(head.get(k), float):
            head[k] = _r(head[k], 7)
    return head


def emit(out, args):
    """Write the full record (every sub-record with its kernel table) to the detail file, then print the
    compact headline as the LAST line of stdout."""
    path = os.environ.get("LPGNN_BENCH_DETAIL", os.path.join("gpurun_out", "bench_detail.json"))
    try:
        os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
        with open(path, "w") as f:
            json.dump(out, f, indent=1)
    except OSError as e:  # a read-only tree: the headline still prints
        print(f"bench: detail file {path} not written ({e})", file=sys.stderr)
        path = None
    try:
        line = json.dumps(compact_headline(out, path))
    except Exception as e:  # never lose the headline to a summary bug: the contract's keys, as measured
        print(f"bench: compact headline failed ({type(e).__name__}: {e}); minimal line", file=sys.stderr)
        line = json.dumps({k: out.get(k) for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup",
                                                   "ms_per_step", "higher_is_better", "scaling", "vs_baseline",
                                                   "dtype", "arith", "data", "config", "roofline", "fc_roofline",
                                                   "cpu_baseline")} | {"detail": path}, default=str)
    if len(line) > HEADLINE_MAX_BYTES:
        print(f"bench: headline {len(line)} bytes > {HEADLINE_MAX_BYTES}", file=sys.stderr)
    sys.stderr.flush()
    print(line, flush=True)


# ------------------------------------------------------------------------ jobs
def one_gpu_job(args, dev, inference=False, fp16=False):
    """The one-GPU workload of args.config: (step, graph, local nnz).  c2/c5: the uniform c2 graph;
    c4: the whole block LP (lpgnn.partition.bench_spec at one rank)."""
    from lpgnn import BipartiteBatch, BipartiteCSR, GCN_FC, synth
    from lpgnn.train import make_optimizer, train_step

    if args.config == "c4":
        from lpgnn.partition import bench_spec

        g = bench_spec(args, 1).full()
    elif args.config == "skewed":
        g = synth.skewed_lp(args.m, args.n, args.nnz, a=1.5, seed=0)
    else:
        g = synth.uniform_lp(args.m, args.n, args.nnz, seed=0)
    adj = BipartiteCSR.from_coo(g.row, g.col, g.val, g.m, g.n, device=dev)
    batch = BipartiteBatch(x_s=torch.from_numpy(g.x_s).to(dev), x_t=torch.from_numpy(g.x_t).to(dev),
                           y_s=torch.from_numpy(g.y_s).to(dev), y_t=torch.from_numpy(g.y_t).to(dev),
                           edge_index=adj, s_bs=g.m, t_bs=g.n)
    torch.manual_seed(0)
    model = GCN_FC(8, 8, hids=args.hids, depth=args.depth,
                   compute_dtype=torch.bfloat16 if args.bf16 else torch.float32).to(dev)
    if inference:
        # the reference's timed path (scripts/pred_basis.py:113-118, 169-173): eval-mode
        # model(batch) + inference_gnn on the concatenated logits (val.py:106-124, with its
        # invariant checks), one graph per step; --fp16: model.half() + batch_to(half=True)
        from lpgnn.data import batch_to
        from lpgnn.val import inference_gnn

        if fp16:
            model.half()
            batch = batch_to(batch, dev, half=True)
        model.eval()

        def step():
            with torch.no_grad():
                lc, lv = model(batch)
                return inference_gnn(torch.cat((lc, lv), 0), g.m)
    else:
        opt, _ = make_optimizer(model)
        step = lambda: train_step(model, batch, opt)  # noqa: E731
    return step, g, g.nnz


def c4_args(args):
    a = copy.copy(args)
    a.config, a.m, a.n, a.nnz, a.hids, a.depth = "c4", None, None, None, None, None
    a.inference, a.fp16 = False, False
    fill(a)
    if args.c4_scale > 1:
        a.m, a.n, a.nnz = a.m // args.c4_scale, a.n // args.c4_scale, a.nnz // args.c4_scale
    return a


def sub_args(args, config):
    """args for a one-GPU sub-record of BASELINE config `config` (c5, skewed) at its own sizes."""
    a = copy.copy(args)
    a.config, a.m, a.n, a.nnz, a.hids, a.depth = config, None, None, None, None, None
    a.inference, a.fp16 = False, False
    return fill(a)


def run_config(ctx, a, steps, warmup, family):
    """Time args `a`'s training workload at the current N: one GPU (N=1, not --partitioned) or this
    rank's share of the row partition.  Returns (record, graph or None)."""
    from lpgnn import partition

    part = ctx.distributed
    if not part:
        step, g, local_nnz = one_gpu_job(a, ctx.dev)
        workload = workload_name(a)
        dirs = {(a.m, a.n): "cons<-vars", (a.n, a.m): "vars<-cons"}
        touched = {(g.m, g.n): int(np.count_nonzero(np.bincount(g.col, minlength=g.n))),
                   (g.n, g.m): int(np.count_nonzero(np.bincount(g.row, minlength=g.m)))}
        key = workload
    else:
        job = partition.build_bench_job(a, ctx.rank, ctx.world, ctx.dev)
        step, g, local_nnz, workload = job.step, None, job.local_nnz, job.workload
        dirs, touched = None, None
        key = rank_share_key(family, ctx.world) if ctx.world > 1 else workload
    dt, kern, per_launch = timed(ctx, step, steps, warmup)
    rec = report(ctx, dt, kern, per_launch, steps=steps, hids=a.hids, local_nnz=local_nnz,
                 esz=2 if a.bf16 else 4, traffic_key=key, single_dirs=dirs, touched=touched)
    rec["workload"] = workload
    rec["config"] = {"workload": workload, "n_cons": a.m * (ctx.world if part and a.config != "c4" else 1),
                     "n_vars": a.n * (ctx.world if part and a.config != "c4" else 1),
                     "nnz": a.nnz * (ctx.world if part and a.config != "c4" else 1),
                     "hid": a.hids, "depth": a.depth,
                     "parallelism": f"rowpart{ctx.world}" if part else "single"}
    if part:
        if a.config == "c4":
            rec["config"]["n_cons"], rec["config"]["n_vars"], rec["config"]["nnz"] = \
                job.spec.m, job.spec.n, job.spec.nnz
        exch = partition.time_exchange(job.batch.edge_index.ex, a.hids, ctx.dev)
        exch.update(halo_rows=int(job.plan.halo.shape[0]), owned_vars=job.plan.n_own,
                    boundary_vars_global=job.plan.n_boundary_global)
        rec["exchange"] = {"per_rank": ctx.gather(exch),
                           "note": "standalone F=hid owner-reduce / halo-broadcast of [n_local, F] fp32 rows "
                                   "(median ms, barrier + sync around each); in the step they run async under "
                                   "independent compute"}
        if a.config == "c4" and ctx.world > 1 and a.rho_sweep:  # after the timed region
            rec["exchange"]["rho_sweep"] = partition.rho_sweep(a, ctx.rank, ctx.world,
                                                               [float(r) for r in a.rho_sweep.split(",")], a.hids)
        del job
    del step
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return rec, g


def run_inference(ctx, a, steps, warmup, fp16, with_cpu):
    """The reference's timed eval path on one GPU (N=1): eval forward + inference_gnn per graph."""
    step, g, nnz = one_gpu_job(a, ctx.dev, inference=True, fp16=fp16)
    dt, kern, per_launch = timed(ctx, step, steps, warmup)
    wl = workload_name(a)
    rec = report(ctx, dt, kern, per_launch, steps=steps, hids=a.hids, local_nnz=nnz,
                 esz=2 if (a.bf16 or fp16) else 4, traffic_key=wl,
                 single_dirs={(a.m, a.n): "cons<-vars", (a.n, a.m): "vars<-cons"}, fp16=fp16, training=False)
    rec["ms_per_graph"] = dt / steps * 1e3
    rec["ms_per_step"] = rec["ms_per_graph"]
    rec["workload"] = wl
    rec["mode"] = ("inference: eval-mode model(batch) + inference_gnn (scripts/pred_basis.py:113-118)"
                   + ("; --fp16: model.half() + batch_to(half=True) (val.py:269, utils.py:909-915)" if fp16 else ""))
    if with_cpu and a.cpu_steps > 0:
        cdt, threads = cpu_inference(g, a.hids, a.depth, a.cpu_steps, fp16=fp16)
        rec["cpu_baseline"] = {"value": rec["value"] * dt / steps / cdt, "unit": "edges/s", "cores": threads,
                               "kind": "port", "s_per_graph": cdt,
                               "sample": f"{a.cpu_steps} eval forward(s) + inference_gnn of the same "
                                         f"{a.config} graph after one untimed warm-up: oracle C spmm_cpu loop "
                                         f"(OpenMP) + torch CPU GEMMs in fp32"
                                         + (" with fp16-rounded storage" if fp16 else "")
                                         + f", {cdt:.2f} s/graph"}
    del step
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return rec, g


def main():
    args = parse()
    if args.print_workload:
        print(workload_name(args))
        return
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(self_launch(args))
    if args.inference and (args.gpus > 1 or args.partitioned):
        raise SystemExit("--inference times the one-GPU eval path (the reference's scripts/pred_basis.py)")
    if args.config == "c5" and (args.gpus > 1 or args.partitioned):
        raise SystemExit("c5 (bf16, configs[4]) is a one-GPU configuration")
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
    ctx = Ctx(rank, world, dev, backend if distributed else "none", distributed)

    import lpgnn

    subs = [s for s in args.sub.split(",") if s] if not args.profile_only else []
    g = None
    if args.inference:
        head, g = run_inference(ctx, args, args.steps, args.warmup, args.fp16, with_cpu=False)
        family = args.config
    else:
        family = f"{args.config} weak scaling (rho={args.rho})" if args.config != "c4" else f"c4 (rho={args.rho})"
        head, g = run_config(ctx, args, args.steps, args.warmup, family)
    workload = head.pop("workload")
    props = torch.cuda.get_device_properties(dev)
    me = {"rank": rank, "local_rank": local, "device": str(dev), "name": props.name,
          "pci": "%04x:%02x:%02x" % (getattr(props, "pci_domain_id", 0), getattr(props, "pci_bus_id", 0),
                                     getattr(props, "pci_device_id", 0)),
          "uuid": str(getattr(props, "uuid", ""))}
    ranks = ctx.gather(me)
    if distributed and backend != "nccl":
        workload += f" [rehearsal: {world} ranks over {backend} sharing {torch.cuda.device_count()} GPU(s)]"
    cfg = head.pop("config", None) or {"workload": workload, "n_cons": args.m, "n_vars": args.n, "nnz": args.nnz,
                                       "hid": args.hids, "depth": args.depth, "parallelism": "single"}
    cfg["workload"] = workload
    out = {
        "metric": METRIC,
        "value": head.pop("value"),
        "unit": "edges/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": head.pop("ms_per_step"),
        "higher_is_better": True,
        "scaling": "strong" if args.config == "c4" else "weak",
        "vs_baseline": None,
        "dtype": "bf16" if args.bf16 else ("fp16" if args.fp16 else "fp32"),
        # the matrix-core arithmetic of the fp32 GEMMs: f16x2 = two row/column-scaled fp16 terms per operand,
        # three products (22-bit scaled operands, fp32-class by a tested error bound)
        "arith": "bf16" if args.bf16 else ("fp16" if args.fp16 else _arith()),
        "data": "synthetic (seeded uniform / block LP graphs, LP feature layout; random-init GCN_FC weights)",
        "config": cfg,
        "dist": {"backend": ctx.backend, "world_size": world, "ranks": ranks,
                 "launcher": "torchrun / self-launched children" if distributed else "single process"},
    }
    out.update(head)
    out["library"] = lpgnn.library_path()
    out["max_hbm_allocated_gb"] = torch.cuda.max_memory_allocated(dev) / 1e9
    main_cpu = rank == 0 and world == 1 and args.cpu_steps > 0 and not args.profile_only and g is not None
    if main_cpu and args.inference:
        cdt, threads = cpu_inference(g, args.hids, args.depth, args.cpu_steps, fp16=args.fp16)
        out["cpu_baseline"] = {"value": out["value"] * out["ms_per_step"] / 1e3 / cdt, "unit": "edges/s",
                               "cores": threads, "kind": "port", "s_per_step": cdt,
                               "sample": f"{args.cpu_steps} eval forward(s) + inference_gnn of the same "
                                         f"{args.config} graph after one untimed warm-up: oracle C spmm_cpu loop "
                                         f"(OpenMP) + torch CPU GEMMs in fp32"
                                         + (" with fp16-rounded storage" if args.fp16 else "")
                                         + f", {cdt:.2f} s/graph"}
    elif main_cpu and args.config == "c2":
        cdt, threads = cpu_baseline(g, args.hids, args.depth, args.cpu_steps)
        edges_step = out["value"] * out["ms_per_step"] / 1e3
        out["cpu_baseline"] = {"value": edges_step / cdt, "unit": "edges/s", "cores": threads, "kind": "port",
                               "sample": f"{args.cpu_steps} full fwd+bwd+Adam step(s) of the same c2 workload after one "
                                         f"untimed warm-up step: "
                                         f"oracle C spmm_cpu loop (OpenMP) + torch CPU GEMMs, "
                                         f"{cdt:.2f} s/step",
                               "s_per_step": cdt}
        out["cpu_spmm"] = dict(cpu_spmm(g, args.hids), threads=threads,
                               note="F=hid SpMM alone on the host, median of 3 (SURVEY.md 8d CPU numbers)")
    if rank == 0 and world == 1 and not args.inference and not args.partitioned and args.config == "c2" and \
            g is not None and not args.profile_only and args.vendor:
        import warnings

        with warnings.catch_warnings():
            warnings.simplefilter("ignore")  # torch's "sparse CSR support is in beta" notice
            out["vendor_spmm"] = dict(vendor_spmm(g, args.hids, dev),
                                      note="rocSPARSE (torch.sparse.mm, CSR, fp32) on the same graph and GPU, "
                                           "beside lpg_spmm_f32; not part of value")
    del g
    if args.inference:
        out["mode"] = head.get("mode")
        out["ms_per_graph"] = out["ms_per_step"]
    # ---- sub-records: the same N, after the headline (its memory released) ----
    if "c4" in subs and not args.inference and args.config != "c4":
        a4 = c4_args(args)
        rec, _ = run_config(ctx, a4, args.c4_steps, args.c4_warmup, f"c4 (rho={a4.rho})")
        rec["scaling"] = "strong"
        rec["steps"], rec["warmup"] = args.c4_steps, args.c4_warmup
        rec["note"] = ("BASELINE.json configs[3] at this N: the whole graph on one GPU at N=1, constraint-row "
                       "partitioned over the N ranks at N>1 (fixed total work); value = all ranks' F=hid SpMM "
                       "edges / max-over-ranks time")
        if distributed and backend != "nccl":
            rec["workload"] += " [rehearsal over gloo]"
        out["c4"] = rec
    if "inference" in subs and not args.inference and world == 1 and not args.partitioned and args.config == "c2":
        a_inf = copy.copy(args)
        a_inf.inference = True
        rec, _ = run_inference(ctx, a_inf, args.inf_steps, 3, False, with_cpu=rank == 0)
        out["inference"] = rec
    if "inference_fp16" in subs and not args.inference and world == 1 and not args.partitioned and args.config == "c2":
        a_inf = copy.copy(args)
        a_inf.inference, a_inf.fp16 = True, True
        rec, _ = run_inference(ctx, a_inf, args.inf_steps, 3, True, with_cpu=rank == 0)
        out["inference_fp16"] = rec
    if "c5" in subs and not args.inference and world == 1 and not args.partitioned and args.config == "c2":
        a5 = sub_args(args, "c5")
        rec, g5 = run_config(ctx, a5, args.c5_steps, args.c5_warmup, "c5")
        rec["steps"], rec["warmup"] = args.c5_steps, args.c5_warmup
        rec["dtype"] = "bf16"
        rec["note"] = ("BASELINE.json configs[4]: the c2 graph, GCN_FC(8,8,hids=2048,depth=6), bf16 activations / "
                       "SpMM storage / MFMA FC (fp32 accumulation, fp32 master weights), fwd+bwd+Adam on one GPU")
        if rank == 0 and args.c5_cpu_steps > 0:
            cdt, threads = cpu_baseline(g5, a5.hids, a5.depth, args.c5_cpu_steps, warmup=False)
            edges_step = rec["value"] * rec["ms_per_step"] / 1e3
            rec["cpu_baseline"] = {"value": edges_step / cdt, "unit": "edges/s", "cores": threads, "kind": "port",
                                   "sample": f"{args.c5_cpu_steps} full fwd+bwd+Adam step(s) of the same c5 workload "
                                             f"in fp32 (the reference's CPU arithmetic), no separate warm-up step "
                                             f"(the c2 leg started the MKL / OpenMP threads): oracle C spmm_cpu loop "
                                             f"(OpenMP) + torch CPU GEMMs, {cdt:.2f} s/step",
                                   "s_per_step": cdt}
        del g5
        out["c5"] = rec
    if "skewed" in subs and not args.inference and world == 1 and not args.partitioned and args.config == "c2":
        ask = sub_args(args, "skewed")
        rec, _ = run_config(ctx, ask, args.steps, args.warmup, "skewed")
        rec["steps"], rec["warmup"] = args.steps, args.warmup
        rec["note"] = ("SURVEY.md 8d skewed-degree workload: Zipf(1.5) constraint-row degrees (synth.skewed_lp, "
                       "capped at n, rescaled to ~2M edges), uniform variables, GCN_FC(8,8,hids=1024,depth=3) "
                       "fwd+bwd+Adam; spmm_directions = per-direction roofline (cons<-vars carries the heavy rows)")
        out["skewed"] = rec
    if rank == 0:
        emit(out, args)
    if distributed:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
