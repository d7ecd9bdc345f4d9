"""k-hop NeighborLoader: the oracle restatement of torch_sparse 0.6.12
neighbor_sample on hand-checked graphs (CPU), and the device sampler
(csrc/sample.hip) against it (GPU).  Parity unpinned at the sampler layer:
torch_sparse is absent here and the reference holds no sampler fixtures;
the end-to-end anchor is the reference's own mini-batch == full-graph check
(val.py:37-41), tested in test_gpu_sampler.py."""
import numpy as np

from oracle import model_ref as O


def _path_graph():
    # undirected path 0-1-2-3-4 plus chord 1-3, both directions
    und = [(0, 1), (1, 2), (2, 3), (3, 4), (1, 3)]
    ei = np.array([[a for a, b in und] + [b for a, b in und], [b for a, b in und] + [a for a, b in und]])
    return ei, 5


def test_to_csc_sorts_sources_per_destination():
    ei, N = _path_graph()
    colptr, row, perm = O.to_csc(ei, N)
    assert colptr.tolist() == [0, 1, 4, 6, 9, 10]
    assert row.tolist() == [1, 0, 2, 3, 1, 3, 1, 2, 4, 3]
    assert np.array_equal(ei[0][perm], row)


def test_neighbor_sample_full_hand_checked():
    ei, N = _path_graph()
    colptr, row, _ = O.to_csc(ei, N)
    # seeds [4]: hop 1 -> 3; hop 2 -> neighbours of 3 in CSC order: 1, 2, 4 -> new 1, 2
    node, r, c, e = O.neighbor_sample(colptr, row, [4], [-1, -1], directed=True)
    assert node.tolist() == [4, 3, 1, 2]
    assert list(zip(r.tolist(), c.tolist())) == [(1, 0), (2, 1), (3, 1), (0, 1)]
    assert np.array_equal(row[e], node[r]) and all(colptr[node[ci]] <= ei_ < colptr[node[ci] + 1]
                                                   for ci, ei_ in zip(c, e))
    node, r, c, e = O.neighbor_sample(colptr, row, [4], [-1, -1], directed=False)
    assert node.tolist() == [4, 3, 1, 2]
    # induced: every edge among {1,2,3,4}, by destination local id then CSC order
    got = sorted(zip(node[r].tolist(), node[c].tolist()))
    want = sorted((a, b) for a, b in zip(ei[0].tolist(), ei[1].tolist()) if a in (1, 2, 3, 4) and b in (1, 2, 3, 4))
    assert got == want
    assert c.tolist() == sorted(c.tolist())


def test_neighbor_sample_fanout_properties():
    rng = np.random.default_rng(0)
    N = 200
    a, b = rng.integers(0, N, 1500), rng.integers(0, N, 1500)
    ei = np.unique(np.stack([np.r_[a, b], np.r_[b, a]]), axis=1)
    ei = ei[:, ei[0] != ei[1]]
    colptr, row, _ = O.to_csc(ei, N)
    node, r, c, e = O.neighbor_sample(colptr, row, [0, 5, 7], [3, 2], directed=True)
    assert len(set(node.tolist())) == len(node) and node[:3].tolist() == [0, 5, 7]
    for ci in np.unique(c):
        sel = c == ci
        deg = colptr[node[ci] + 1] - colptr[node[ci]]
        assert sel.sum() <= min(3, deg) and len(set(e[sel].tolist())) == sel.sum()
