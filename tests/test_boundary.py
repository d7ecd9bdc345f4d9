"""The dense boundary all-reduce of the row partition (lpgnn.boundary; include/lpgnn.h
lpg_spmm_partitioned_f32 / lpg_boundary_*): its host logic on CPU -- the global boundary set, the
per-rank maps, and the exchange's arithmetic emulated in numpy over every rank's local partials
against the whole graph's A^T x (the oracle's spmm) -- plus the plan collective over gloo."""
import os
import socket

import numpy as np
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import model_ref as O


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _graph():
    from lpgnn import synth

    return synth.block_lp(240, 480, 2400, parts=3, rho=0.15, seed=5)


def _plans(g, world):
    from lpgnn.partition import plan_partition

    return [plan_partition(g.row, g.col, g.val, g.m, g.n, world, r) for r in range(world)]


def test_boundary_vars_are_the_vars_touched_by_two_blocks():
    from lpgnn.boundary import boundary_vars

    g = _graph()
    for world in (1, 2, 3, 5):
        plans = _plans(g, world)
        gb = boundary_vars([p.halo for p in plans])
        touched_by = np.zeros(g.n, np.int64)
        for p in plans:
            sel = (g.row >= p.row_lo) & (g.row < p.row_hi)
            touched_by[np.unique(g.col[sel])] += 1
        assert np.array_equal(gb, np.nonzero(touched_by >= 2)[0])
        assert gb.shape[0] == plans[0].n_boundary_global
        if world == 1:
            assert gb.shape[0] == 0


def test_boundary_map_rows():
    from lpgnn.boundary import boundary_map

    lv = np.array([4, 9, 12, 2, 7], np.int64)  # [owned | halo], each part ascending
    gb = np.array([1, 2, 7, 8, 12, 30], np.int64)
    assert boundary_map(lv, gb).tolist() == [-1, 3, 4, -1, 2, -1]
    assert boundary_map(np.zeros(0, np.int64), gb).tolist() == [-1] * 6
    assert boundary_map(lv, np.zeros(0, np.int64)).dtype == np.int32


def _emulate(g, plans, x, F):
    """Every rank's vars<-cons partials over its local edges (the oracle's CSR loop), packed by its map,
    summed over the ranks, unpacked: the local rows after lpg_spmm_partitioned_f32's semantics."""
    from lpgnn.boundary import boundary_map, boundary_vars

    gb = boundary_vars([p.halo for p in plans])
    ys, maps = [], []
    for p in plans:
        # A_p^T over the local variables: rows = local vars, cols = the block's constraints (global x rows)
        AT = O.csr_transpose(*O.csr_from_coo(p.e_row, p.e_col, p.e_val, p.m_local, p.n_local), p.m_local, p.n_local)
        ys.append(O.spmm_f32(*AT, x[p.row_lo:p.row_hi]))
        maps.append(boundary_map(p.local_vars, gb))
    buf = np.zeros((gb.shape[0], F), np.float64)
    for y, bm in zip(ys, maps):
        buf[bm >= 0] += y[bm[bm >= 0]]
    for y, bm in zip(ys, maps):
        y[bm[bm >= 0]] = buf[bm >= 0]
    return ys


def test_exchange_arithmetic_gives_every_rank_the_full_sums():
    g = _graph()
    F = 6
    x = np.random.default_rng(0).standard_normal((g.m, F)).astype(np.float32)
    A = O.csr_from_coo(g.row, g.col, g.val, g.m, g.n)
    full = O.spmm_f32(*O.csr_transpose(*A, g.m, g.n), x)  # [n, F], the whole graph's vars<-cons
    for world in (1, 2, 3, 4):
        plans = _plans(g, world)
        for p, y in zip(plans, _emulate(g, plans, x, F)):
            # every local row (owned and halo) holds the whole graph's sum, to fp32 reassociation
            np.testing.assert_allclose(y, full[p.local_vars], rtol=1e-5, atol=1e-5)


def _plan_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from lpgnn.boundary import plan_boundary

        g = _graph()
        p = _plans(g, world)[rank]
        gb, bm = plan_boundary(p)
        np.savez(os.path.join(out_dir, f"r{rank}.npz"), gb=gb, bm=bm, lv=p.local_vars)
    finally:
        dist.destroy_process_group()


def test_plan_boundary_collective_two_ranks(tmp_path):
    world = 2
    mp.spawn(_plan_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    from lpgnn.boundary import boundary_map, boundary_vars

    g = _graph()
    plans = _plans(g, world)
    gb = boundary_vars([p.halo for p in plans])
    for r in range(world):
        d = np.load(os.path.join(tmp_path, f"r{r}.npz"))
        assert np.array_equal(d["gb"], gb)
        assert np.array_equal(d["bm"], boundary_map(plans[r].local_vars, gb))
        # each mapped row is the boundary variable it names
        ok = d["bm"] >= 0
        assert np.array_equal(d["lv"][d["bm"][ok]], gb[ok])


def test_no_cpu_path():
    import pytest
    import torch

    from lpgnn.boundary import LibComm, boundary_pack

    with pytest.raises(RuntimeError, match="no CPU path"):
        boundary_pack(torch.zeros(4, 3), torch.zeros(2, dtype=torch.int32))
    with pytest.raises(RuntimeError, match="no CPU path"):
        LibComm("cpu")
