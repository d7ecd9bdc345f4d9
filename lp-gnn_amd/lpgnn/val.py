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
def inference_gnn(logits, m, **kwargs):
    """val.py:106-124."""
    n = logits.shape[0] - m
    pr = F.softmax(logits.float(), dim=-1)
    pr = pr.clone()
    pr[torch.isnan(pr)] = 0
    _, topk_idx = pr[:, 1].topk(m)
    pr[:, 1] = pr.min() - 1
    pr[topk_idx, 1] = pr.max() + 1
    pred = pr.argmax(-1)
    assert (pred == 1).sum().item() == m
    assert (pred[m:m + n] == 1).sum().item() == ((pred[:m] == 0) | (pred[:m] == 2)).sum().item()
    return pred


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
def model_inference_with_batch(model, batch, arch: str = "GCN_FC(8,8)", dev="cuda"):
    """val.py:12-36 for a bipartite batch (full-graph forward).

    Graphs above the NeighborLoader threshold (nnz > 12e6, utils.py:808) are
    run full-graph too: one MI355X holds the whole graph (288 GB HBM) and
    the partitioned path (lpgnn.partition) covers multi-GPU; the k-hop
    sampler is §8f rank 4 ("next").
    """
    _ = arch_depth(arch)
    model.eval()
    batch = batch.to(dev)
    lc, lv = model(batch)
    return lc[:batch.s_bs].cpu(), lv[:batch.t_bs].cpu()
