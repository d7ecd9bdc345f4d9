"""Training caller of the hot path (train.py:18-53, 85-129; utils.py:286-299)."""
from __future__ import annotations

import torch
import torch.nn.functional as F
from torch import nn
from torch.optim.lr_scheduler import StepLR


@torch.no_grad()
def labels_to_balanced_weights(labels, merge_lu=True):
    """utils.py:286-299: w[c] = N / count_c for present classes; unless
    exactly two classes are present, w0 = w2 = mean(w0, w2).

    Restated without torch.unique / len(lbl) (which force a device->host
    sync every step).  On a HIP device one call,
    lpg_balanced_weights3: the class counts (a scatter-add onto three bins
    serialises its atomics: 41 us per call at 200 K labels) and the formula
    in the counts' fold (instead of ~13 elementwise launches); on the host
    the tensor form below.  Both bitwise the reference's result
    (tests/test_gpu_model.py)."""
    labels = labels.view(-1)
    if labels.device.type == "cuda" and labels.dtype == torch.int64:
        # counts and the formula below in one device pass (lpg_balanced_weights3), the same bits
        from . import _lib

        labels = labels.contiguous()
        L = _lib.lib()
        res = torch.empty(3, dtype=torch.float32, device=labels.device)
        ws = torch.empty(L.lpg_class_counts_workspace_bytes(labels.numel()) // 8, dtype=torch.int64,
                         device=labels.device)
        with torch.cuda.device(labels.device):
            st = L.lpg_balanced_weights3(labels.numel(), labels.data_ptr(), 1 if merge_lu else 0, res.data_ptr(),
                                         ws.data_ptr(), _lib.stream_of(labels))
        _lib.check(st, "lpg_balanced_weights3")
        return res
    # host-side callers (data preparation, CPU tests of the formula)
    cnt = torch.zeros(3, dtype=torch.int64, device=labels.device)
    cnt.scatter_add_(0, labels, torch.ones_like(labels))
    present = cnt > 0
    wei = cnt.sum() / cnt
    res = torch.where(present, wei, torch.zeros((), dtype=wei.dtype, device=labels.device))
    if merge_lu:
        merged = (res[0] + res[2]) / 2.
        two = present.sum() == 2
        res = torch.stack([torch.where(two, res[0], merged), res[1], torch.where(two, res[2], merged)])
    return res


class _WeightedCE(torch.autograd.Function):
    """coef * nn.CrossEntropyLoss(weight=w)(x, y) on lpg_weighted_ce_{fwd,bwd}_f32:
    one pass per direction, deterministic reduction, no host sync (torch's
    weighted nll_loss reduces in a single workgroup: 75-165 us per call)."""

    @staticmethod
    def forward(ctx, x, y, w, coef):
        from . import _lib

        x = x if (x.stride(-1) == 1 and x.dtype == torch.float32) else x.float().contiguous()
        y = y.contiguous()
        w = None if w is None else w.float().contiguous()
        M, C = x.shape
        L = _lib.lib()
        out = torch.empty(2, dtype=torch.float32, device=x.device)  # loss, sum of weights
        ws = torch.empty(max(2, L.lpg_weighted_ce_workspace_bytes(M) // 4), dtype=torch.float32, device=x.device)
        with torch.cuda.device(x.device):
            st = L.lpg_weighted_ce_fwd_f32(M, C, x.data_ptr(), x.stride(0), y.data_ptr(),
                                           None if w is None else w.data_ptr(), float(coef), out.data_ptr(),
                                           out.data_ptr() + 4, ws.data_ptr(), _lib.stream_of(x))
        _lib.check(st, "lpg_weighted_ce_fwd_f32")
        ctx.save_for_backward(x, y, w, out)
        ctx.coef = float(coef)
        return out[0]

    @staticmethod
    def backward(ctx, g):
        from . import _lib

        x, y, w, out = ctx.saved_tensors
        g = g.float().contiguous()
        dx = torch.empty_like(x)
        with torch.cuda.device(x.device):
            st = _lib.lib().lpg_weighted_ce_bwd_f32(x.shape[0], x.shape[1], x.data_ptr(), x.stride(0), y.data_ptr(),
                                                    None if w is None else w.data_ptr(), out.data_ptr() + 4,
                                                    g.data_ptr(), ctx.coef, dx.data_ptr(), dx.stride(0),
                                                    _lib.stream_of(x))
        _lib.check(st, "lpg_weighted_ce_bwd_f32")
        return dx, None, None, None


def weighted_ce(x, y, w, coef=1.0):
    """coef * nn.CrossEntropyLoss(weight=w)(x, y): the HIP kernels for device
    tensors (the training hot path), torch's own criterion for host tensors
    (host-side tests of the loss logic)."""
    if x.device.type == "cuda" and x.shape[1] <= 4:
        return _WeightedCE.apply(x, y, w, coef)
    return coef * nn.CrossEntropyLoss(weight=w)(x, y)


def balanced(logpr_cons, logpr_vars, y_s, y_t):
    """train.py:39-46 (the loss of the published experiment)."""
    m, n = len(y_s), len(y_t)
    loss = weighted_ce(logpr_cons, y_s, labels_to_balanced_weights(y_s), (m + n) / m)
    return loss + weighted_ce(logpr_vars, y_t, labels_to_balanced_weights(y_t), (m + n) / n)


def unbalanced(logpr_cons, logpr_vars, y_s, y_t):
    """train.py:32-37."""
    return nn.CrossEntropyLoss()(torch.cat((logpr_cons, logpr_vars), 0), torch.cat((y_s, y_t), 0))


class FocalLoss(nn.modules.loss._WeightedLoss):
    """train.py:18-28."""

    def __init__(self, weight=None, gamma=2, reduction="mean"):
        super().__init__(weight, reduction=reduction)
        self.gamma = gamma
        self.weight = weight

    def forward(self, input, target):
        ce_loss = F.cross_entropy(input, target, reduction=self.reduction, weight=self.weight)
        pt = torch.exp(-ce_loss)
        return ((1 - pt) ** self.gamma * ce_loss).mean()


def focal(logpr_cons, logpr_vars, y_s, y_t):
    """train.py:49-53."""
    return FocalLoss()(torch.cat((logpr_cons, logpr_vars), 0), torch.cat((y_s, y_t), 0))


LOSSES = {"balanced": balanced, "unbalanced": unbalanced, "focal": focal}


def make_optimizer(model, opt="adam", lr=1e-3, epochs=800):
    """train.py:85-89: Adam/SGD(weight_decay=5e-4) + StepLR(epochs//4, 0.1).
    With every parameter on the GPU, Adam runs as torch's fused kernel (one
    launch per step instead of the foreach path's eight multi-tensor passes:
    0.15 -> ~0.03 ms of the c2 step); the same update rule."""
    if opt == "adam":
        params = list(model.parameters())
        fused = bool(params) and all(p.is_cuda for p in params)
        o = torch.optim.Adam(params, lr=lr, weight_decay=5e-4, fused=fused or None)
    else:
        o = torch.optim.SGD(model.parameters(), lr=lr, weight_decay=5e-4)
    return o, StepLR(o, step_size=max(epochs // 4, 1), gamma=0.1)


def epoch_batches(graph, arch: str = "GCN_FC(8,8)", batch_size: int = 10240 * 8 * 4, dev="cuda", seed=None):
    """train.py:103-116: a bipartite graph is one batch; a homogeneous one
    (above the MyToBipartite threshold) is cut into seed batches by the
    device k-hop NeighborLoader (6 sampled neighbours per hop, depth-1 hops,
    shuffled, drop_last, induced subgraphs)."""
    import numpy as np

    from .arch import arch_depth
    from .data import MyToBipartite
    from .loader import NeighborLoader

    if hasattr(graph, "x_s"):
        return [graph]
    if graph.edge_index.shape[-1] == 0:
        return []
    bs = min(int(batch_size), int(graph.num_nodes))
    return NeighborLoader(graph, num_neighbors=[6] * arch_depth(arch), input_nodes=None, directed=False,
                          shuffle=True, transform=MyToBipartite(thresh_num=np.inf), batch_size=bs,
                          drop_last=True, device=dev, seed=seed)


def train_step(model, batch, opt, loss="balanced", check_nan=True):
    """One inner iteration of train.py:117-129: forward on the batch, slice
    the seed nodes, loss, backward, optimizer step.  Returns the loss tensor
    (no host sync unless check_nan)."""
    logit_cons, logit_vars = model(batch)
    # the seed-node slices (train.py:122-123); a slice that covers the whole tensor is skipped: its
    # autograd node would allocate a zero gradient and copy into it every step for the same values
    seed = lambda t, k: t if k == t.shape[0] else t[:k]
    logit_cons, logit_vars = seed(logit_cons, batch.s_bs), seed(logit_vars, batch.t_bs)
    y_s, y_t = batch.y_s[:batch.s_bs], batch.y_t[:batch.t_bs]
    L = LOSSES[loss](logit_cons, logit_vars, y_s, y_t)
    if check_nan:
        assert not torch.isnan(L).item()  # train.py:126
    opt.zero_grad()
    L.backward()
    opt.step()
    return L
