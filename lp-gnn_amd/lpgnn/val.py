"""Inference callers of the hot path (val.py:12-36, 106-124, 199-237).

``inference_gnn`` turns per-node logits into basis labels (0 = at lower
bound, 1 = basic, 2 = at upper bound): the m nodes with the largest P(basic)
are basic, every other node takes argmax over {0, 2}.  It runs on whatever
device the logits live on; the reference runs it on host copies.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

from .arch import arch_depth


@torch.no_grad()
def inference_gnn(logits, m, check: bool = True, **kwargs):
    """val.py:106-124.  ``check=False`` skips the two invariant asserts
    (val.py:119-122), the only host syncs, for per-step use on the device."""
    n = logits.shape[0] - m
    pr = F.softmax(logits.float(), dim=-1)
    pr = pr.clone()
    pr[torch.isnan(pr)] = 0
    _, topk_idx = pr[:, 1].topk(m)
    pr[:, 1] = pr.min() - 1
    pr[topk_idx, 1] = pr.max() + 1
    pred = pr.argmax(-1)
    if check:
        assert (pred == 1).sum().item() == m
        assert (pred[m:m + n] == 1).sum().item() == ((pred[:m] == 0) | (pred[:m] == 2)).sum().item()
    return pred


@torch.no_grad()
def accuracy_device(logits, gt, num_cons):
    """accuracy(..., return_pr=True) (val.py:199-237) computed on the device
    with no host sync: per-side accuracy averaged, and sklearn's
    precision/recall for labels=[1], zero_division=0, averaged over sides.
    Returns three 0-dim tensors."""
    pred = inference_gnn(logits, num_cons, check=False)

    def side(p, g):
        acc = (p == g).float().mean()
        tp = ((p == 1) & (g == 1)).sum().float()
        pp, gp = (p == 1).sum().float(), (g == 1).sum().float()
        prec = torch.where(pp > 0, tp / pp.clamp(min=1), torch.zeros_like(tp))
        rec = torch.where(gp > 0, tp / gp.clamp(min=1), torch.zeros_like(tp))
        return acc, prec, rec

    a1, p1, r1 = side(pred[:num_cons], gt[:num_cons])
    a2, p2, r2 = side(pred[num_cons:], gt[num_cons:])
    return (a1 + a2) / 2., (p1 + p2) / 2., (r1 + r2) / 2.


@torch.no_grad()
def accuracy(logits, gt, num_cons, return_pr=False, dataset_name=""):
    """val.py:199-237 (per-side accuracy, precision/recall of class 1)."""
    from sklearn import metrics

    pred = inference_gnn(logits, num_cons)
    pred_np, gt_np = pred.cpu().numpy(), gt.cpu().numpy()
    acc1 = (gt_np[:num_cons] == pred_np[:num_cons]).mean()
    acc2 = (gt_np[num_cons:] == pred_np[num_cons:]).mean()
    if dataset_name and "stoch" in dataset_name:
        acc1 = acc2
    acc = (acc1 + acc2) / 2.
    kw = dict(labels=[1], average="macro", zero_division=0)
    p1 = metrics.precision_score(gt_np[:num_cons], pred_np[:num_cons], **kw)
    p2 = metrics.precision_score(gt_np[num_cons:], pred_np[num_cons:], **kw)
    r1 = metrics.recall_score(gt_np[:num_cons], pred_np[:num_cons], **kw)
    r2 = metrics.recall_score(gt_np[num_cons:], pred_np[num_cons:], **kw)
    if dataset_name and "stoch" in dataset_name:
        p1, r1 = p2, r2
    prec, recl = (p1 + p2) / 2., (r1 + r2) / 2.
    return (acc, prec, recl) if return_pr else acc


@torch.no_grad()
def model_inference_with_batch(model, batched_graphs, arch: str = "GCN_FC(8,8)", dev="cuda",
                               batch_size: int = 10240 * 8 * 4):
    """val.py:12-36.  A bipartite batch runs full-graph; a homogeneous graph
    (above MyToBipartite's threshold) goes through the device k-hop
    NeighborLoader with every neighbour (num_neighbors=[-1]*(depth-1),
    directed=False, val.py:22-27) in seed order, and the seed logits are
    concatenated -- equal to the full-graph logits up to summation order
    (the reference's own check, val.py:37-41)."""
    from .data import MyToBipartite
    from .loader import NeighborLoader

    depth = arch_depth(arch)
    model.eval()
    if hasattr(batched_graphs, "x_s"):
        loader = [batched_graphs]
    else:
        bs = min(int(batch_size), int(batched_graphs.num_nodes))
        loader = NeighborLoader(batched_graphs, num_neighbors=[-1] * depth, input_nodes=None, directed=False,
                                shuffle=False, transform=MyToBipartite(thresh_num=np.inf), batch_size=bs,
                                drop_last=False, device=dev)
    lc, lv = [], []
    for batch in loader:
        batch = batch.to(dev)
        logit_cons, logit_vars = model(batch)
        lc.append(logit_cons[:batch.s_bs].cpu()), lv.append(logit_vars[:batch.t_bs].cpu())
    return torch.cat(lc, 0), torch.cat(lv, 0)
