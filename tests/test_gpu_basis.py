"""lpg_basis_labels_f32 (the device inference_gnn, val.py:106-124) against the reference's torch
chain run on the host: softmax, NaN -> 0, topk(m) of P[:, 1], argmax over {0, 2}.

The two paths compute the softmax with different exp implementations, so labels may differ only
where the rule itself is a near-tie: a node whose P[:, 1] is within EPS of the m-th largest value,
or whose P[:, 0] and P[:, 2] are within EPS.  Exact ties at the threshold are resolved by index on
the device (torch.topk leaves the choice open): checked by the invariants instead."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
EPS = 1e-6


def _host_labels(logits, m):
    from lpgnn.val import inference_gnn

    return inference_gnn(logits.cpu(), m)


def _probs64(logits):
    p = torch.softmax(logits.double().cpu(), dim=-1)
    p[torch.isnan(p)] = 0
    return p


def _device_labels(logits, m, check=True):
    from lpgnn.val import inference_gnn

    return inference_gnn(logits.to(DEV), m, check=check).cpu()


@pytest.mark.parametrize("total,m,scale", [
    (300_000, 100_000, 4.0),   # the c2 shape: 100 K constraints of 300 K nodes
    (300_000, 100_000, 30.0),  # saturated softmax (add_knowledge's range is [-20, 10])
    (1000, 1, 1.0),
    (1000, 999, 1.0),
    (1000, 1000, 1.0),
    (7, 3, 1.0),
    (1, 1, 1.0),
    (257, 0, 1.0),             # no constraint rows: nothing basic
])
def test_basis_labels_match_host_chain(total, m, scale):
    g = torch.Generator().manual_seed(total + m)
    logits = torch.randn(total, 3, generator=g) * scale
    dev = _device_labels(logits, m)
    host = _host_labels(logits, m)
    assert dev.dtype == torch.int64 and dev.shape == (total,)
    assert int((dev == 1).sum()) == m
    p = _probs64(logits)
    diff = dev != host
    if m > 0:
        thr = p[:, 1].topk(m).values[-1]
        near = (p[:, 1] - thr).abs() <= EPS
    else:
        near = torch.zeros(total, dtype=torch.bool)
    near |= (p[:, 0] - p[:, 2]).abs() <= EPS
    assert bool((~diff | near).all()), f"{int((diff & ~near).sum())} labels differ outside a near-tie"
    print(f"total={total} m={m} scale={scale}: {int(diff.sum())} labels differ, all at near-ties")


def test_basis_labels_ties_lowest_index_and_invariants():
    """Heavy exact ties (rows drawn from 40 distinct logit triples): the basic set is every node
    above the m-th largest P[:, 1] plus the lowest-index nodes equal to it."""
    g = torch.Generator().manual_seed(3)
    pool = torch.randn(40, 3, generator=g) * 2
    idx = torch.randint(0, 40, (400_000,), generator=g)  # 1563 blocks: the tie scan runs >1 block per thread
    logits = pool[idx]
    m = 137_321
    dev = _device_labels(logits, m)
    p1 = torch.softmax(logits.to(DEV), dim=-1)[:, 1].cpu()
    # the device's own P[:, 1] order: recompute the keys the kernel selected on
    basic = dev == 1
    assert int(basic.sum()) == m
    thr = p1[basic].min()
    assert bool((p1[~basic] <= thr).all()) and bool((p1[basic] >= thr).all())
    # of the rows equal to the threshold row's triple, the basic ones are the lowest indices
    tied = idx == idx[basic & (p1 == thr)][0]
    tied_basic = torch.nonzero(tied & basic).flatten()
    tied_all = torch.nonzero(tied).flatten()
    assert torch.equal(tied_basic, tied_all[:tied_basic.numel()])
    # outside the basic set: argmax(P0, P2) with the first maximum on a tie
    p = torch.softmax(logits.double(), dim=-1)
    side = torch.where(p[:, 0] >= p[:, 2], 0, 2)
    assert torch.equal(dev[~basic], side[~basic])


def test_basis_labels_nan_rows_and_determinism():
    g = torch.Generator().manual_seed(9)
    logits = torch.randn(5000, 3, generator=g)
    logits[::7, 1] = float("nan")  # NaN rows: P = 0 everywhere, never preferred, side label 0
    m = 1200
    a = _device_labels(logits, m)
    b = _device_labels(logits, m)
    assert torch.equal(a, b)
    nan_rows = torch.zeros(5000, dtype=torch.bool)
    nan_rows[::7] = True
    assert bool((a[nan_rows] == 0).all())
    host = _host_labels(logits, m)
    p = _probs64(logits)
    thr = p[:, 1].topk(m).values[-1]
    near = ((p[:, 1] - thr).abs() <= EPS) | ((p[:, 0] - p[:, 2]).abs() <= EPS)
    assert bool(((a == host) | near).all())


def test_basis_labels_strided_logits_and_errors():
    from lpgnn import _lib

    g = torch.Generator().manual_seed(4)
    big = torch.randn(3000, 8, generator=g)
    view = big[:, 2:5]  # row stride 8
    assert torch.equal(_device_labels(view, 900), _device_labels(view.contiguous(), 900))
    with pytest.raises(RuntimeError):
        _device_labels(view, 3001)
    L = _lib.lib()
    st = L.lpg_basis_labels_f32(10, 11, None, 3, None, None, None)
    assert st != 0 and b"m <= total" in L.lpg_last_error()
