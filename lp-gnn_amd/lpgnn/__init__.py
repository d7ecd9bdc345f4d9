"""lpgnn -- MI355X-native hot path of vbdai/lp-gnn's GCN_FC.

Public surface (mirrors the reference's names):
  arch:  GCN_FC, GraphConvTwoDirection, GraphConv, add_knowledge, build_model
  data:  MyToBipartite, lp_to_unipartite, batch_to, BipartiteBatch
  loader: NeighborLoader, NeighborSampler (device k-hop sampling)
  sparse: BipartiteCSR (the batch's edge_index), spmm
  ops:   torch.ops.lpgnn.spmm_sum (torch_sparse's spmm_sum schema + autograd)
  val:   inference_gnn, accuracy, model_inference_with_batch
  train: balanced, labels_to_balanced_weights, train_step, make_optimizer
"""
from . import _lib
from .sparse import BipartiteCSR, CSR, spmm
from .arch import GCN_FC, GraphConv, GraphConvTwoDirection, Linear, add_knowledge, build_model
from .data import BipartiteBatch, MyToBipartite, UnipartiteData, batch_to, lp_to_unipartite
from .loader import NeighborLoader, NeighborSampler
from . import ops  # registers torch.ops.lpgnn.spmm_sum

__all__ = [
    "BipartiteCSR", "CSR", "spmm", "GCN_FC", "GraphConv", "GraphConvTwoDirection", "Linear",
    "add_knowledge", "build_model", "BipartiteBatch", "MyToBipartite", "UnipartiteData", "batch_to",
    "lp_to_unipartite", "NeighborLoader", "NeighborSampler",
]


def library_path() -> str:
    return _lib.LIB_PATH
