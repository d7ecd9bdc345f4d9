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
    (val.py:119-122), the only host sync, for per-step use on the device.
    On a HIP device the whole chain (softmax, NaN -> 0, top-m of P[:, 1],
    argmax over {0, 2}) is one lpg_basis_labels_f32 call (exact radix select;
    of the nodes tied at the m-th largest P[:, 1] the lowest indices are
    basic, a choice torch.topk leaves open); on the host, the reference's
    torch ops."""
    n = logits.shape[0] - m
    if logits.is_cuda and logits.dim() == 2 and logits.shape[1] == 3:
        # fp16 logits (the --fp16 mode): the half softmax's fp16 probabilities decide (lpg_basis_labels_f16)
        pred = _basis_labels_device(logits if logits.dtype == torch.float16 else logits.float(), m)
    else:
        pr = F.softmax(logits.float(), dim=-1)
        if logits.dtype == torch.float16:  # a half softmax stores fp16 probabilities (the device kernel's rule)
            pr = pr.half().float()
        pr = pr.clone()
        pr[torch.isnan(pr)] = 0
        _, topk_idx = pr[:, 1].topk(m)
        pr[:, 1] = pr.min() - 1
        pr[topk_idx, 1] = pr.max() + 1
        pred = pr.argmax(-1)
    if check:
        basic = pred == 1
        outer = (pred[:m] == 0) | (pred[:m] == 2)
        got = torch.stack((basic.sum(), basic[m:m + n].sum(), outer.sum())).tolist()  # one host sync
        assert got[0] == m
        assert got[1] == got[2]
    return pred


def _basis_labels_device(logits, m):
    from . import _lib

    total = logits.shape[0]
    if logits.stride(1) != 1:
        logits = logits.contiguous()
    if not 0 <= m <= total:
        raise RuntimeError(f"inference_gnn: m = {m} outside [0, {total}] (topk)")
    L = _lib.lib()
    f16 = logits.dtype == torch.float16
    entry = "lpg_basis_labels_f16" if f16 else "lpg_basis_labels_f32"
    pred = torch.empty(total, dtype=torch.int64, device=logits.device)
    ws = torch.empty((max(16, L.lpg_basis_labels_workspace_bytes(total)) + 15) // 16 * 4, dtype=torch.float32,
                     device=logits.device)
    from .timing import TIMER

    with torch.cuda.device(logits.device):
        tok = TIMER.start(("basis_labels", total, 3, m, "f16" if f16 else "f32"))
        st = getattr(L, entry)(total, m, logits.data_ptr(), logits.stride(0), pred.data_ptr(), ws.data_ptr(),
                               _lib.stream_of(logits))
        TIMER.stop(tok)
    _lib.check(st, entry)
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
                               batch_size: int = 10240 * 8 * 4, fp16: bool = False):
    """val.py:12-36.  A bipartite batch runs full-graph; a homogeneous graph
    (above MyToBipartite's threshold) goes through the device k-hop
    NeighborLoader with every neighbour (num_neighbors=[-1]*(depth-1),
    directed=False, val.py:22-27) in seed order, and the seed logits are
    concatenated -- equal to the full-graph logits up to summation order
    (the reference's own check, val.py:37-41).  ``fp16``: batch_to(batch, dev, half=True) on every
    batch (val.py:31, args.fp16) -- a copy, the caller's graph keeps its dtypes."""
    import copy

    from .data import batch_to
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
        batch = batch_to(copy.copy(batch), dev, half=True) if fp16 else batch.to(dev)
        logit_cons, logit_vars = model(batch)
        lc.append(logit_cons[:batch.s_bs].cpu()), lv.append(logit_vars[:batch.t_bs].cpu())
    return torch.cat(lc, 0), torch.cat(lv, 0)
