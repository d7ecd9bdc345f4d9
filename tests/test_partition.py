"""Constraint-row partitioning (lpgnn.partition) with gloo, world size 2, on
CPU.  The product's local compute (HIP SpMM / FC / knowledge kernels) is
swapped for the oracle so the distributed logic -- plan, boundary
all-reduce and its backward, distributed balanced loss, gradient
all-reduce -- is checked against the single-graph oracle."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn.functional as F

from oracle import model_ref as O


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _graph():
    from lpgnn import synth

    return synth.block_lp(240, 480, 2400, parts=2, rho=0.15, seed=2)


def test_plan_invariants():
    from lpgnn.partition import local_dual_csr, plan_partition

    g = _graph()
    for world in (1, 2, 3, 4):
        plans = [plan_partition(g.row, g.col, g.val, g.m, g.n, world, r) for r in range(world)]
        # cons blocks tile [0, m); every edge lands on exactly one rank
        assert plans[0].row_lo == 0 and plans[-1].row_hi == g.m
        for a, b in zip(plans, plans[1:]):
            assert a.row_hi == b.row_lo
        assert sum(p.nnz_local for p in plans) == g.nnz
        # every variable owned exactly once; owned/halo ascending and disjoint
        owned = np.concatenate([p.owned for p in plans])
        assert np.array_equal(np.sort(owned), np.arange(g.n))
        for p in plans:
            assert np.all(np.diff(p.owned) > 0) and np.all(np.diff(p.halo) > 0)
            assert not np.intersect1d(p.owned, p.halo).size
            # the halo is exactly the remote-owned vars this block touches
            sel = (g.row >= p.row_lo) & (g.row < p.row_hi)
            touched = np.unique(g.col[sel])
            assert np.array_equal(np.sort(np.union1d(np.intersect1d(touched, p.owned), p.halo)),
                                  np.union1d(np.intersect1d(touched, p.owned), p.halo))
            assert np.array_equal(p.halo, np.setdiff1d(touched, p.owned))
            # local edges reproduce the global block
            gr, gc = p.e_row + p.row_lo, p.local_vars[p.e_col]
            assert np.array_equal(np.sort(gr * g.n + gc), np.sort(g.row[sel] * g.n + g.col[sel]))
            assert np.array_equal(gc, p.e_gcol)
        # reduce-phase sends and receives pair up (same vars, same order)
        for p in plans:
            off = np.concatenate([[0], np.cumsum(p.send_counts)])
            for o in range(world):
                sent = p.local_vars[p.send_idx[off[o]:off[o + 1]]]
                q = plans[o]
                roff = np.concatenate([[0], np.cumsum(q.recv_counts)])
                got = q.local_vars[q.recv_idx[roff[p.rank]:roff[p.rank + 1]]]
                assert np.array_equal(sent, got)
                assert o != p.rank or len(sent) == 0
    # local CSR(A_p) keeps each row's edges in global variable order
    p = plan_partition(g.row, g.col, g.val, g.m, g.n, 3, 1)
    adj = local_dual_csr(p, "cpu")
    rp, c = adj.fwd.rowptr.numpy(), adj.fwd.col.numpy()
    gl = p.local_vars[c]
    for i in range(p.m_local):
        assert np.all(np.diff(gl[rp[i]:rp[i + 1]]) > 0)
    assert adj.bwd.n_rows == p.n_local and adj.fwd.n_cols == p.n_local


# ------------------------------------------------------- oracle-backed doubles
def _cpu_local_spmm(adj, x):
    fwd = (adj.fwd.rowptr.numpy(), adj.fwd.col.numpy(), adj.fwd.val.numpy())
    bwd = (adj.bwd.rowptr.numpy(), adj.bwd.col.numpy(), adj.bwd.val.numpy())
    return O.spmm_t(fwd, bwd, x)


def _cpu_graph_conv_fc(agg, x_dst, w_rel, b_rel, w_root, relu, dropout=0.0, row_offset=0, row_keys=None,
                       arith=None):
    out = F.linear(agg, w_rel, b_rel) + F.linear(x_dst, w_root)
    out = torch.relu(out) if relu else out
    return F.dropout(out, p=dropout, training=True) if dropout > 0 else out


def _cpu_knowledge(logit, feas, bound=10):
    l, _ = O.add_knowledge(logit, logit[:1], feas, feas[:1], bound)
    return l


def _c4_small(scale=50):
    from lpgnn import synth

    return synth.c4_spec(scale=scale, seed=3)  # 1/50: 40K x 80K, nnz 800K -- the c4 generator reduced


def _worker(rank, world, port, out_dir, mode="global", scale=50, hids=16):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    try:
        import lpgnn.fc as fc
        import lpgnn.partition as part
        from lpgnn import GCN_FC

        part._local_spmm = _cpu_local_spmm
        fc.graph_conv_fc = _cpu_graph_conv_fc
        fc.linear = lambda x, w, b, fold_in=False, opts=None: F.linear(x, w, b)
        fc.knowledge = _cpu_knowledge

        if mode == "c4":  # each rank generates and plans only its own blocks
            spec = _c4_small(scale)
            plan = part.plan_partition_blocks(spec, world, rank)
            batch = part.make_block_batch(spec, plan, device="cpu")
            g = spec.full()  # the single-graph reference below
            _check_block_plan(plan, g, spec, world, rank)
        else:
            g = _graph()
            plan = part.plan_partition(g.row, g.col, g.val, g.m, g.n, world, rank)
            batch = part.make_local_batch(plan, g.x_s, g.x_t, g.y_s, g.y_t, device="cpu")
        torch.manual_seed(0)
        model = GCN_FC(8, 8, hids=hids, depth=4, dp=0.0)
        sd0 = {k: v.detach().clone() for k, v in model.state_dict().items()}
        model.train()
        lc, lv = model(batch)
        loss = part.balanced_distributed(lc, lv, batch.y_s, batch.y_t, batch.var_owned)
        loss_n = part.balanced_distributed(lc, lv, batch.y_s, batch.y_t, batch.n_own)  # owned rows come first
        assert torch.allclose(loss, loss_n, rtol=1e-6, atol=1e-7)
        model.zero_grad()
        loss.backward()
        part.all_reduce_grads(model)
        tot = loss.detach().clone()
        dist.all_reduce(tot)

        # single-graph oracle
        A = O.csr_from_coo(g.row, g.col, g.val, g.m, g.n)
        AT = O.csr_transpose(*A, g.m, g.n)
        params = {k: v.clone().requires_grad_(True) for k, v in sd0.items()}
        rc, rv = O.gcn_fc_forward(params, torch.from_numpy(g.x_s), torch.from_numpy(g.x_t), A, AT, 4)
        rloss = O.balanced(rc, rv, torch.from_numpy(g.y_s), torch.from_numpy(g.y_t))
        rloss.backward()

        # the owner reduce adds the halo partials in source-rank order (a re-association of each boundary
        # variable's edge sum): fp32 rounding -- the north star's 1e-4 per logit (|logit| <= 20)
        np.testing.assert_allclose(lc.detach().numpy(), rc.detach().numpy()[plan.row_lo:plan.row_hi], rtol=2e-5,
                                   atol=1e-4)
        # owned AND halo rows agree with the full graph (halo = owners' values)
        np.testing.assert_allclose(lv.detach().numpy(), rv.detach().numpy()[plan.local_vars], rtol=2e-5, atol=1e-4)
        assert abs(tot.item() - rloss.item()) < 1e-4, (tot.item(), rloss.item())
        for k, p in model.named_parameters():
            np.testing.assert_allclose(p.grad.numpy(), params[k].grad.numpy(), rtol=1e-3, atol=1e-5, err_msg=k)
        open(os.path.join(out_dir, f"ok{rank}"), "w").write(f"{tot.item()} {plan.n_boundary_global} {len(plan.halo)}")
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_partitioned_training_step_matches_single_graph(tmp_path, world):
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    for r in range(world):
        assert (tmp_path / f"ok{r}").exists()


def _check_block_plan(plan, g, spec, world, rank):
    """The rank-local plan equals the global planner's with the same cons
    blocks and the block owner rule, field for field."""
    from lpgnn import partition as part

    per = spec.blocks // world
    bounds = np.arange(world + 1, dtype=np.int64) * per * spec.mb
    ref = part.plan_partition(g.row, g.col, g.val, g.m, g.n, world, rank, bounds=bounds,
                              owner=part.block_owner(spec, world))
    for f in ("row_lo", "row_hi", "send_counts", "recv_counts", "n_boundary_global"):
        assert getattr(plan, f) == getattr(ref, f), f
    for f in ("owned", "halo", "e_row", "e_gcol", "e_col", "e_val", "send_idx", "recv_idx"):
        assert np.array_equal(getattr(plan, f), getattr(ref, f)), f


def test_block_lp_generator_is_rank_independent():
    """BlockLP is defined block by block: any split of the blocks generates
    the same graph (strong scaling keeps the workload fixed)."""
    spec = _c4_small()
    g = spec.full()
    assert g.nnz == spec.nnz and g.m == spec.m and g.n == spec.n
    row, col, val, xs, ys = spec.rows(2, 4)
    sel = (g.row >= 2 * spec.mb) & (g.row < 4 * spec.mb)
    assert np.array_equal(row, g.row[sel]) and np.array_equal(col, g.col[sel]) and np.array_equal(val, g.val[sel])
    assert np.array_equal(xs, g.x_s[2 * spec.mb:4 * spec.mb]) and np.array_equal(ys, g.y_s[2 * spec.mb:4 * spec.mb])
    ids = np.array([5, spec.n - 1, spec.nb, 3 * spec.nb + 7])
    x, y = spec.var_rows(ids)
    assert np.array_equal(x, g.x_t[ids]) and np.array_equal(y, g.y_t[ids])
    # rows have exactly nnz/m distinct, sorted columns; about rho of the edges leave their block
    deg = np.diff(np.searchsorted(g.row, np.arange(g.m + 1)))
    assert (deg == spec.nnz // spec.m).all()
    key = g.row * g.n + g.col
    assert (np.diff(key) > 0).all()
    far = (g.col // spec.nb) != (g.row // spec.mb)
    assert abs(far.mean() - spec.rho * (1 - 1 / spec.blocks)) < 0.005


def test_c4_reduced_two_ranks_match_single_graph(tmp_path):
    """The c4 generator at 1/50 size on 2 gloo ranks: rank-local planning ==
    the global planner, and the partitioned training step (logits of owned
    and halo rows, loss, gradients) == the single-graph oracle."""
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), "c4"), nprocs=world, join=True)
    for r in range(world):
        assert (tmp_path / f"ok{r}").exists()


@pytest.mark.parametrize("world", [4, 8])
def test_c4_reduced_world_4_8_match_single_graph(tmp_path, world):
    """The N = 4 and N = 8 topologies of the c4 block planner (3 and 7 exchange peers per rank at
    N = 8) at 1/200 size, hid 32, oracle local compute: rank-local plans == the global planner,
    owned AND halo logits, the summed loss and every gradient == the single-graph oracle."""
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), "c4", 200, 32), nprocs=world, join=True)
    for r in range(world):
        assert (tmp_path / f"ok{r}").exists()
    # every rank exchanged with at least one other rank (the block LP has boundary variables)
    assert all(int((tmp_path / f"ok{r}").read_text().split()[2]) > 0 for r in range(world))


def _worker_rho(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from types import SimpleNamespace

        import lpgnn.partition as part

        args = SimpleNamespace(config="c4", m=40_000, n=80_000, nnz=800_000, rho=0.02)
        sw = part.rho_sweep(args, rank, world, [0.0, 0.02, 0.1, 1.0], 1024)
        assert [s["rho"] for s in sw] == [0.0, 0.02, 0.1, 1.0]
        assert sw[0]["boundary_vars_global"] == 0 and sw[0]["halo_rows_per_rank"] == [0] * world
        assert sw[0]["exchange_rows_per_rank"] == [0] * world
        b = [s["boundary_vars_global"] for s in sw]
        assert b[0] < b[1] < b[2] < b[3], b
        for s in sw:  # every rank reports the same pooled numbers; owned variables tile [0, n)
            assert sum(s["owned_vars_per_rank"]) == args.n
        # the sweep's plan at the bench rho is the bench's own plan
        spec = part.bench_spec(args, world)
        plan = part.plan_partition_blocks(spec, world, rank)
        assert sw[1]["halo_rows_per_rank"][rank] == plan.halo.shape[0]
        assert sw[1]["boundary_vars_global"] == plan.n_boundary_global
        open(os.path.join(out_dir, f"ok{rank}"), "w").write("ok")
    finally:
        dist.destroy_process_group()


def test_rho_sweep_boundary_counts(tmp_path):
    """bench.py's c4 rho sweep: no boundary at rho = 0, growing with rho, pooled
    identically on every rank, equal to the bench's own plan at the bench rho."""
    mp.spawn(_worker_rho, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    assert (tmp_path / "ok0").exists() and (tmp_path / "ok1").exists()


def test_exchange_dropout_keys_are_global_ids():
    """Every owned variable's dropout row is keyed by its global id: one row_offset when the owned
    set is one contiguous range (block plans), the owned id list (row_keys) when it is not (the
    general owner rule on a weakly blocked graph); constraint rows by row_lo + i."""
    from lpgnn import synth
    from lpgnn.partition import Exchange, plan_partition

    g = synth.block_lp(400, 800, 8000, parts=2, rho=0.6, seed=1)
    scattered = 0
    for r in range(2):
        p = plan_partition(g.row, g.col, g.val, g.m, g.n, 2, r)
        ex = Exchange(p, "cpu")
        assert ex.cons_key_args == {"row_offset": p.row_lo, "row_keys": None}
        if p.owned[-1] - p.owned[0] + 1 == p.n_own:
            assert ex.var_keys is None and ex.var_key_args["row_offset"] == p.owned[0]
        else:
            scattered += 1
            assert np.array_equal(ex.var_key_args["row_keys"].numpy(), p.owned)
    assert scattered >= 1
    g = _graph()
    p = plan_partition(g.row, g.col, g.val, g.m, g.n, 2, 1, bounds=[0, 120, 240],
                       owner=(np.arange(g.n) * 2) // g.n)
    assert Exchange(p, "cpu").var_keys is None


# ------------------------------------------- the rank-local general planner (lpgnn.run --partition)
def _plan_fields_equal(a, b):
    for f in ("rank", "world", "m", "n", "row_lo", "row_hi", "send_counts", "recv_counts", "n_boundary_global"):
        assert getattr(a, f) == getattr(b, f), f
    for f in ("owned", "halo", "e_row", "e_gcol", "e_col", "e_val", "send_idx", "recv_idx"):
        assert np.array_equal(getattr(a, f), getattr(b, f)), f


def _local_plan_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from lpgnn import partition as part, synth

        for g in (_graph(), synth.skewed_lp(300, 700, 3000, a=1.5, seed=4), synth.uniform_lp(200, 900, 1000, seed=1)):
            want = part.plan_partition(g.row, g.col, g.val, g.m, g.n, world, rank)
            _plan_fields_equal(part.plan_partition_local(g.row, g.col, g.val, g.m, g.n, world, rank), want)
            # from the rank's own rows only
            b = part.row_blocks(np.asarray(g.row, np.int64), g.m, world)
            sel = (g.row >= b[rank]) & (g.row < b[rank + 1])
            _plan_fields_equal(part.plan_partition_local(g.row[sel], g.col[sel], g.val[sel], g.m, g.n, world, rank,
                                                         bounds=b, local=True), want)
        open(os.path.join(out_dir, f"ok{rank}"), "w").write("ok")
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_plan_partition_local_equals_global_planner(tmp_path, world):
    """The rank-local planner (one MAX all-reduce of owner keys, one all_to_all of halo ids) builds
    exactly plan_partition's plan from the global edge list, field for field -- including the
    skewed-degree graph whose dense rows tie owners, and a graph with untouched variables."""
    mp.spawn(_local_plan_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    for r in range(world):
        assert (tmp_path / f"ok{r}").exists()


def test_plan_partition_local_world_one():
    from lpgnn import partition as part

    g = _graph()
    _plan_fields_equal(part.plan_partition_local(g.row, g.col, g.val, g.m, g.n, 1, 0),
                       part.plan_partition(g.row, g.col, g.val, g.m, g.n, 1, 0))


def _defer_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from lpgnn import partition as part

        g = _graph()
        plan = part.plan_partition(g.row, g.col, g.val, g.m, g.n, world, rank)
        ex = part.Exchange(plan, "cpu")
        assert ex.active and plan.halo.shape[0] > 0
        # every local row holds its global id: after the broadcast the halo rows hold their owners' ids
        full = torch.full((plan.n_local, 3), -1.0)
        full[:plan.n_own] = torch.from_numpy(plan.owned.astype(np.float32))[:, None]
        other = torch.zeros(plan.n_local, 3)
        ex.defer(full, ex.start_broadcast_(full, quiet=True))
        ex.defer(other, ex.start_broadcast_(other))
        v0 = full._version
        # in flight: the halo rows are not written until the consumer settles them
        assert bool((full[plan.n_own:] == -1).all())
        ex.settle(other)
        assert len(ex._deferred) == 1 and bool((full[plan.n_own:] == -1).all())
        ex.settle(full)
        assert ex._deferred == []
        assert torch.equal(full[:, 0], torch.from_numpy(plan.local_vars.astype(np.float32)))
        assert full._version == v0  # quiet: written past autograd's version counter
        ex.settle(full)  # nothing pending: a no-op
        # a later exchange on the same group still pairs up after deferred ones (issue order)
        ex.defer(full, ex.start_broadcast_(full))
        red = ex.reduce_rows(torch.ones(plan.n_local, 2), inplace=False)
        ex.settle_all()
        assert ex._deferred == [] and red.shape == (plan.n_own, 2)
        open(os.path.join(out_dir, f"ok{rank}"), "w").write("ok")
    finally:
        dist.destroy_process_group()


def test_deferred_broadcast_settles_on_demand(tmp_path):
    """Exchange.defer / settle (the partitioned forward leaves a layer output's halo broadcast in
    flight for the next layer): the halo rows stay untouched until settled, settling one target leaves
    the others pending, and every deferred broadcast lands its owners' rows exactly."""
    mp.spawn(_defer_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    for r in range(2):
        assert (tmp_path / f"ok{r}").exists()


def _gather16_worker(rank, world, port, out_dir):
    """--fp16 evaluation of a row-partitioned graph (run.validation with --partition): batch_to(half=True)
    on a partitioned batch (fp16 features, fp16-rounded local edge values, the same exchange), then the
    ranks' fp16 logits gathered into global order by gather_logits."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import lpgnn.partition as part
        from lpgnn.data import batch_to

        g = _graph()
        plan = part.plan_partition(g.row, g.col, g.val, g.m, g.n, world, rank)
        batch = part.make_local_batch(plan, g.x_s, g.x_t, g.y_s, g.y_t, device="cpu")
        ex0 = batch.edge_index.ex
        val0 = batch.edge_index.local.fwd.val.clone()
        b16 = batch_to(batch, "cpu", half=True)
        assert b16.x_s.dtype == torch.float16 and b16.x_t.dtype == torch.float16 and b16.y_s.dtype == torch.int64
        adj = b16.edge_index
        assert isinstance(adj, part.PartitionedCSR) and adj.ex is ex0 and adj.orient == "cons"
        assert torch.equal(adj.local.fwd.val, val0.half().float())
        # logits = the global node id (exact in fp16 below 2048) in column 0, its negation in column 1
        gid_c = torch.arange(plan.row_lo, plan.row_hi, dtype=torch.float32) % 2048
        gid_v = torch.from_numpy(plan.local_vars).float() % 2048
        lc = torch.stack((gid_c, -gid_c), 1).half()
        lv = torch.stack((gid_v, -gid_v), 1).half()
        cons, var = part.gather_logits(lc, lv, b16)
        want_c = torch.arange(g.m, dtype=torch.float32) % 2048
        want_v = torch.arange(g.n, dtype=torch.float32) % 2048
        assert cons.dtype == torch.float32 and torch.equal(cons[:, 0], want_c) and torch.equal(cons[:, 1], -want_c)
        assert torch.equal(var[:, 0], want_v) and torch.equal(var[:, 1], -want_v)
        open(os.path.join(out_dir, f"ok{rank}"), "w").write("ok")
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_fp16_partitioned_batch_and_gather_order(tmp_path, world):
    mp.spawn(_gather16_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    for r in range(world):
        assert (tmp_path / f"ok{r}").exists()
