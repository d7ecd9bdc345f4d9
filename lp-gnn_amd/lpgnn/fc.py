"""Dense per-node FC stack of GraphConv and the add_knowledge epilogue.

``graph_conv_fc`` computes, for one GraphConv direction (PyG 2.1
GraphConv.forward after propagate):

    out = lin_rel(agg) + lin_root(x_dst)        [+ ReLU, arch.py:182/188]
        = agg @ W_rel^T + b_rel + x_dst @ W_root^T

``knowledge`` is arch.py:129-141 for one side.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F
from torch import Tensor


def graph_conv_fc(agg: Tensor, x_dst: Tensor, w_rel: Tensor, b_rel, w_root: Tensor, relu: bool) -> Tensor:
    if agg.device.type != "cuda":
        raise RuntimeError("lpgnn: the GCN_FC hot path runs on a HIP device only")
    out = F.linear(agg, w_rel, b_rel)
    out = out + F.linear(x_dst, w_root)
    return out.relu_() if relu else out


def knowledge(logit: Tensor, feas: Tensor, bound=10) -> Tensor:
    """One side of add_knowledge: normalize(logit) * 10, then -bound on
    column 0 where feas[:, -3] != 0 (lower bound = -inf) and on column 2
    where feas[:, -1] != 0 (upper bound = +inf)."""
    l_mask, u_mask = feas[:, -3].abs().bool(), feas[:, -1].abs().bool()
    logit = F.normalize(logit) * 10
    logit[l_mask, 0] = logit[l_mask, 0] - bound
    logit[u_mask, 2] = logit[u_mask, 2] - bound
    return logit
