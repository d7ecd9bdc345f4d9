"""The native boundary exchange on the GPU (include/lpgnn.h lpg_boundary_pack_f32 / _unpack_f32 /
_allreduce_f32, lpg_spmm_partitioned_f32, lpg_comm_*): pack / unpack bitwise against torch indexing
(maps with absent and out-of-range rows, strided rows, every vector path); a 3-rank exchange emulated
on one GPU through the HIP pack / unpack over each rank's HIP local SpMM, against the whole graph's
sums (the oracle); and the RCCL path end to end on a one-rank communicator of the library's own.
(The box has one GPU: RCCL cannot place two ranks on it, so more ranks are covered by the emulation
and, for the plan, by tests/test_boundary.py over gloo.)"""
import numpy as np
import pytest
import torch

from oracle import model_ref as O

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _ref_pack(y, bm):
    rows = y.shape[0]
    out = torch.zeros((bm.shape[0], y.shape[1]), dtype=y.dtype, device=y.device)
    ok = (bm >= 0) & (bm < rows)
    out[ok] = y[bm[ok].long()]
    return out


@pytest.mark.parametrize("F,pad", [(1, 0), (3, 2), (8, 0), (8, 3), (1024, 0), (1024, 4)])
def test_pack_unpack_bitwise(F, pad):
    from lpgnn.boundary import boundary_pack, boundary_unpack_

    torch.manual_seed(F + pad)
    rows, nb = 700, 1500
    wide = torch.randn(rows, F + pad, device=DEV)
    y = wide[:, :F]  # row stride F + pad
    g = torch.Generator().manual_seed(3)
    perm = torch.randperm(rows, generator=g)[: rows // 2].to(torch.int32)
    bm = torch.full((nb,), -1, dtype=torch.int32)
    slots = torch.randperm(nb, generator=g)[: perm.shape[0]]
    bm[slots] = perm
    bm[slots[:5]] = rows + 7  # out of range: treated as absent
    bm = bm.to(DEV)
    buf = boundary_pack(y, bm)
    torch.cuda.synchronize()
    assert torch.equal(buf, _ref_pack(y, bm))
    # unpack writes the buffer's rows back into the mapped rows only
    new = torch.randn(nb, F, device=DEV)
    before = wide.clone()
    boundary_unpack_(y, bm, new)
    ref = before.clone()
    ok = (bm >= 0) & (bm < rows)
    ref[bm[ok].long(), :F] = new[ok]
    assert torch.equal(wide, ref)  # the pad columns and unmapped rows untouched


def test_emulated_three_rank_exchange_matches_whole_graph():
    from lpgnn import synth
    from lpgnn.boundary import boundary_map, boundary_pack, boundary_unpack_, boundary_vars
    from lpgnn.partition import local_dual_csr, plan_partition
    from lpgnn.sparse import spmm_forward

    g = synth.block_lp(3000, 6000, 60000, parts=3, rho=0.1, seed=11)
    F, world = 64, 3
    x = torch.randn(g.m, F, generator=torch.Generator().manual_seed(1))
    A = O.csr_from_coo(g.row, g.col, g.val, g.m, g.n)
    full = O.spmm_f32(*O.csr_transpose(*A, g.m, g.n), x.numpy())
    plans = [plan_partition(g.row, g.col, g.val, g.m, g.n, world, r) for r in range(world)]
    gb = boundary_vars([p.halo for p in plans])
    assert gb.shape[0] > 100
    ys, maps = [], []
    for p in plans:
        adj = local_dual_csr(p, DEV)
        ys.append(spmm_forward(adj.bwd, x[p.row_lo:p.row_hi].to(DEV)))
        maps.append(torch.from_numpy(boundary_map(p.local_vars, gb)).to(DEV))
    total = sum(boundary_pack(y, bm) for y, bm in zip(ys, maps))  # the all-reduce, in rank order
    for p, y, bm in zip(plans, ys, maps):
        boundary_unpack_(y, bm, total)
        np.testing.assert_allclose(y.cpu().numpy(), full[p.local_vars], rtol=1e-5, atol=1e-5)
    # every rank holds the same bits for a boundary variable it touches
    for b in range(0, gb.shape[0], 37):
        vals = [y[int(bm[b])].cpu() for y, bm in zip(ys, maps) if int(bm[b]) >= 0]
        assert len(vals) >= 2 and all(torch.equal(v, vals[0]) for v in vals)


def test_rccl_one_rank_partitioned_spmm():
    from lpgnn import BipartiteCSR
    from lpgnn.boundary import LibComm, boundary_allreduce_, spmm_partitioned
    from lpgnn.sparse import spmm_forward

    rng = np.random.default_rng(4)
    m, n, nnz, F = 500, 900, 6000, 256
    keys = rng.choice(m * n, size=nnz, replace=False)
    adj = BipartiteCSR.from_coo(keys // n, keys % n, rng.uniform(-1, 1, nnz).astype(np.float32), m, n, device=DEV)
    x = torch.randn(m, F, device=DEV)
    bm = torch.full((300,), -1, dtype=torch.int32)
    bm[::2] = torch.randperm(n, generator=torch.Generator().manual_seed(0))[:150].to(torch.int32)
    bm = bm.to(DEV)
    with LibComm(DEV) as comm:
        assert comm.info() == (1, 0)
        y = spmm_partitioned(adj.bwd, x, bm, comm)  # one rank: the all-reduce returns its own rows
        ref = spmm_forward(adj.bwd, x)
        torch.cuda.synchronize()
        assert torch.equal(y, ref)
        z = ref.clone()
        boundary_allreduce_(z, bm, comm)
        torch.cuda.synchronize()
        assert torch.equal(z, ref)
        # no boundary: no collective, plain SpMM
        assert torch.equal(spmm_partitioned(adj.bwd, x, bm[:0], comm), ref)
