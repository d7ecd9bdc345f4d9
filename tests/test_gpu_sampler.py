"""Device k-hop sampler + NeighborLoader vs the oracle restatement of
torch_sparse 0.6.12 neighbor_sample (element for element at fanout -1),
sampling properties at fanout k, and the reference's own mini-batch ==
full-graph logits check (val.py:37-41) through GCN_FC."""
import numpy as np
import pytest
import torch

from oracle import model_ref as O

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _graph(N=3000, E=20000, seed=0):
    rng = np.random.default_rng(seed)
    a, b = rng.integers(0, N, E), rng.integers(0, N, E)
    ei = np.unique(np.stack([np.r_[a, b], np.r_[b, a]]), axis=1)
    return ei[:, ei[0] != ei[1]], N


@pytest.mark.parametrize("directed", [True, False])
@pytest.mark.parametrize("seeds,hops", [([5], [-1, -1]), (list(range(0, 3000, 97)), [-1, -1]),
                                        ([7, 3, 2999, 0], [-1, -1, -1]), ([11], [-1])])
def test_full_neighbourhood_matches_oracle(directed, seeds, hops):
    from lpgnn.loader import NeighborSampler

    ei, N = _graph()
    colptr, row, perm = O.to_csc(ei, N)
    s = NeighborSampler(torch.from_numpy(ei), N, hops, directed=directed, device=DEV)
    assert np.array_equal(s.colptr.cpu().numpy(), colptr) and np.array_equal(s.row.cpu().numpy(), row)
    got = [t.cpu().numpy() for t in s.sample(torch.tensor(seeds))]
    want = O.neighbor_sample(colptr, row, seeds, hops, directed)
    for g, w in zip(got, want):
        assert np.array_equal(g, w)
    assert bool((s.local == -1).all()) and bool((s.first == -1).all())  # scratch restored


def test_isolated_and_empty_frontier():
    from lpgnn.loader import NeighborSampler

    ei = np.array([[0, 1], [1, 0]])
    s = NeighborSampler(torch.from_numpy(ei), 4, [-1, -1], directed=False, device=DEV)
    node, r, c, e = s.sample(torch.tensor([3, 2]))
    assert node.tolist() == [3, 2] and r.numel() == 0
    node, r, c, e = s.sample(torch.tensor([1]))
    assert node.tolist() == [1, 0] and sorted(zip(r.tolist(), c.tolist())) == [(0, 1), (1, 0)]


@pytest.mark.parametrize("k", [1, 2, 6, 64])
def test_fanout_sampling_properties(k):
    from lpgnn.loader import NeighborSampler

    ei, N = _graph(seed=3)
    colptr, row, _ = O.to_csc(ei, N)
    s = NeighborSampler(torch.from_numpy(ei), N, [k, k], directed=True, device=DEV, seed=1)
    seeds = list(range(0, N, 13))
    node, r, c, e = (t.cpu().numpy() for t in s.sample(torch.tensor(seeds)))
    assert node[:len(seeds)].tolist() == seeds and len(np.unique(node)) == len(node)
    assert np.array_equal(row[e], node[r])  # each edge's source is the sampled node
    for ci in np.unique(c):
        sel = c == ci
        deg = colptr[node[ci] + 1] - colptr[node[ci]]
        assert sel.sum() == min(k, deg)  # min(k, deg) distinct in-edges of the destination
        assert len(np.unique(e[sel])) == sel.sum()
        assert bool(((colptr[node[ci]] <= e[sel]) & (e[sel] < colptr[node[ci] + 1])).all())
    # uniform without replacement: over many draws each neighbour of a hub is hit ~k/deg of the time
    hub = int(np.argmax(np.diff(colptr)))
    deg = int(colptr[hub + 1] - colptr[hub])
    s1 = NeighborSampler(torch.from_numpy(ei), N, [k], directed=True, device=DEV, seed=2)
    hits = np.zeros(deg)
    for _ in range(400):
        _, _, _, e1 = s1.sample(torch.tensor([hub]))
        hits[e1.cpu().numpy() - colptr[hub]] += 1
    freq = hits / 400
    assert abs(freq.mean() - min(k, deg) / deg) < 1e-9
    assert freq.std() < 0.15


def test_loader_batches_cover_all_nodes_once():
    from lpgnn.data import UnipartiteData
    from lpgnn.loader import NeighborLoader

    ei, N = _graph()
    x = torch.randn(N, 8)
    data = UnipartiteData(x=x, y=torch.arange(N), edge_index=torch.from_numpy(ei),
                          edge_attr=torch.randn(ei.shape[1]), is_vars=(torch.arange(N) % 3 == 0).long())
    seen = []
    for b in NeighborLoader(data, [-1], shuffle=True, batch_size=700, directed=False, device=DEV, seed=0):
        assert b.batch_size == b.input_id.numel() and torch.equal(b.n_id[:b.batch_size], b.input_id)
        assert torch.equal(b.y[:b.batch_size].cpu(), b.input_id.cpu())
        assert torch.equal(b.x.cpu(), x[b.n_id.cpu()])
        seen.append(b.input_id.cpu())
    assert torch.equal(torch.cat(seen).sort().values, torch.arange(N))
    assert len(NeighborLoader(data, [-1], batch_size=700, drop_last=True, device=DEV)) == N // 700


def test_minibatch_logits_equal_full_graph():
    """val.py:12-36 through the device NeighborLoader (all neighbours, depth-1
    hops) == the full-graph forward on the same LP (val.py:37-41's check),
    and the basis labels are identical."""
    from lpgnn import synth
    from lpgnn.arch import GCN_FC
    from lpgnn.data import MyToBipartite, lp_to_unipartite
    from lpgnn.val import inference_gnn, model_inference_with_batch

    lp = synth.uniform_lp(600, 1100, 6000, seed=4)
    uni = lambda: lp_to_unipartite(lp.row, lp.col, lp.val, lp.x_s, lp.x_t, lp.y_s, lp.y_t)
    g = uni()
    torch.manual_seed(0)
    model = GCN_FC(8, 8, hids=64, depth=3).to(DEV)
    full = MyToBipartite()(uni())
    lc_f, lv_f = model_inference_with_batch(model, full, "GCN_FC(8,8,hids=64,depth=3)", DEV)
    lc, lv = model_inference_with_batch(model, g, "GCN_FC(8,8,hids=64,depth=3)", DEV, batch_size=250)
    assert lc.shape == lc_f.shape and lv.shape == lv_f.shape
    torch.testing.assert_close(lc, lc_f, rtol=0, atol=1e-4)
    torch.testing.assert_close(lv, lv_f, rtol=0, atol=1e-4)
    m = lc.shape[0]
    assert torch.equal(inference_gnn(torch.cat([lc, lv]), m), inference_gnn(torch.cat([lc_f, lv_f]), m))


def test_epoch_batches_train_step_on_sampled_subgraphs():
    """train.py:103-129 on a homogeneous graph: NeighborLoader(fanout 6,
    shuffled, drop_last) batches -> GCN_FC step on each seed slice."""
    from lpgnn import synth
    from lpgnn.arch import GCN_FC
    from lpgnn.data import lp_to_unipartite
    from lpgnn.train import epoch_batches, make_optimizer, train_step

    lp = synth.uniform_lp(500, 900, 5000, seed=7)
    g = lp_to_unipartite(lp.row, lp.col, lp.val, lp.x_s, lp.x_t, lp.y_s, lp.y_t)
    torch.manual_seed(0)
    model = GCN_FC(8, 8, hids=32, depth=3).to(DEV)
    opt, _ = make_optimizer(model, lr=1e-2)
    batches = epoch_batches(g, "GCN_FC(8,8,hids=32,depth=3)", batch_size=300, dev=DEV, seed=0)
    assert len(batches) == (500 + 900) // 300
    seen = 0
    for b in batches:
        assert b.s_bs + b.t_bs == 300 and b.x_s.is_cuda
        loss = train_step(model, b, opt)
        assert torch.isfinite(loss)
        seen += 1
    assert seen == len(batches)
