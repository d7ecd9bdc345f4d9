"""GCN_FC on MI355X: the reference's model API with the HIP hot path.

Mirrors arch.py of vbdai/lp-gnn (and the PyG 2.1 ``GraphConv`` it builds on)
name for name, so that ``GCN_FC(8, 8, hids=1024, depth=3)`` has the same
constructor, ``forward(batch) -> (logit_cons [m,3], logit_vars [n,3])`` and
state_dict keys/shapes -- a reference ``mdl.pth`` loads unchanged
(``GCNBase.load``, arch.py:112-114).

What runs where:
  aggregation  sum_j A_ij x_j     -> lpgnn.sparse.spmm  (HIP CSR SpMM, both
                                     directions, fwd and bwd)
  dense FC     lin_rel + lin_root -> lpgnn.fc (hand-written fp32 MFMA kernel,
               + bias + ReLU         one fma chain per output, fused epilogue)
  heads        lin_left/lin_right -> the same kernel (N = 3 tile)
  add_knowledge                   -> lpg_knowledge_f32 (bitwise torch-CPU
                                     F.normalize semantics)
"""
from __future__ import annotations

import ast
import math
import re

import torch
import torch.nn.functional as F
from torch import Tensor, nn

from .sparse import BipartiteCSR, spmm
from . import conv as _conv
from . import fc as _fc
from .options import DEFAULT as _DEFAULT_OPTIONS, PathOptions


class Linear(nn.Module):
    """torch_geometric.nn.dense.linear.Linear (PyG 2.1), default initialisers:
    weight kaiming_uniform(fan=in, a=sqrt(5)), bias uniform(1/sqrt(in)).
    Parameter names ``weight``/``bias`` as in PyG (state_dict compatible)."""

    def __init__(self, in_channels: int, out_channels: int, bias: bool = True):
        super().__init__()
        self.in_channels, self.out_channels = in_channels, out_channels
        self.weight = nn.Parameter(torch.empty(out_channels, in_channels))
        if bias:
            self.bias = nn.Parameter(torch.empty(out_channels))
        else:
            self.register_parameter("bias", None)
        self.reset_parameters()

    @torch.no_grad()
    def reset_parameters(self):
        bound = math.sqrt(6.0 / ((1 + 5.0) * self.in_channels))
        self.weight.uniform_(-bound, bound)
        if self.bias is not None:
            b = 1.0 / math.sqrt(self.in_channels)
            self.bias.uniform_(-b, b)

    def forward(self, x: Tensor) -> Tensor:
        return F.linear(x, self.weight, self.bias)


class GraphConv(nn.Module):
    """PyG 2.1 ``GraphConv((in_src, in_dst), out, aggr='add')`` with a sparse adj_t:

        out = lin_rel(sum_{j} adj_t[i, j] * x_src[j]) + lin_root(x_dst[i])

    lin_rel has a bias, lin_root has none; aggregation precedes lin_rel.
    ``forward`` may also apply the following ReLU in the same fused kernel
    (``relu=True``); the reference applies it right after (arch.py:182, 188).
    """

    def __init__(self, in_channels, out_channels: int, aggr: str = "add", bias: bool = True):
        super().__init__()
        if aggr != "add":
            raise NotImplementedError("GCN_FC uses aggr='add' only (arch.py:57-62)")
        if isinstance(in_channels, int):
            in_channels = (in_channels, in_channels)
        self.in_channels, self.out_channels = in_channels, out_channels
        self.lin_rel = Linear(in_channels[0], out_channels, bias=bias)
        self.lin_root = Linear(in_channels[1], out_channels, bias=False)
        self.reset_parameters()

    def reset_parameters(self):
        self.lin_rel.reset_parameters()
        self.lin_root.reset_parameters()

    def forward(self, x, edge_index: BipartiteCSR, edge_weight=None, size=None, relu: bool = False,
                dropout: float = 0.0, opts: PathOptions | None = None) -> Tensor:
        if isinstance(x, Tensor):
            x = (x, x)
        if edge_weight is not None:
            raise NotImplementedError("edge weights come from the adjacency values (arch.py:77)")
        arith = (opts or _DEFAULT_OPTIONS).arith

        def fc(agg, x_dst, **keys):  # lin_rel + lin_root, ReLU and (training) dropout fused in one kernel
            # keys: the dropout row keys of a partition's rows (row_offset / row_keys, lpgnn.partition)
            return _fc.graph_conv_fc(agg, x_dst, self.lin_rel.weight, self.lin_rel.bias, self.lin_root.weight, relu,
                                     dropout, arith=arith, **keys)

        pc = getattr(edge_index, "partitioned_conv", None)  # row-partitioned multi-GPU adjacency
        if pc is not None:
            return pc(x, fc)
        return fc(spmm(edge_index, x[0]), x[1])  # message_and_aggregate: matmul(adj_t, x[0], 'add')


class GraphConvTwoDirection(nn.Module):
    """arch.py:51-81.  left = constraints, right = variables."""

    def __init__(self, left_dim, right_dim, out_dim):
        super().__init__()
        self.left2right = GraphConv((left_dim, right_dim), out_dim)
        self.right2left = GraphConv((right_dim, left_dim), out_dim)

    def forward(self, left_feas, right_feas, edge_index: BipartiteCSR, edge_weight=None, relu: bool = False,
                dropout: float = 0.0, fold_in: bool = False, opts: PathOptions | None = None,
                feeds_conv: bool = False):
        # edge_index is A (m x n, rows = cons).  arch.py:71-74: l2r = A^T, r2l = A.
        opts = opts or _DEFAULT_OPTIONS
        if edge_weight is None and isinstance(edge_index, BipartiteCSR) and \
                getattr(edge_index, "partitioned_conv", None) is None:
            # one autograd node for both directions (lpgnn.conv): same forward,
            # fused gradient sums and the cheaper association in backward
            return _conv.two_direction(left_feas, right_feas, edge_index, self.left2right, self.right2left,
                                       relu, dropout, fold_in, opts, feeds_conv)
        tdc = getattr(edge_index, "two_direction_conv", None)  # row-partitioned multi-GPU adjacency
        if tdc is not None and edge_weight is None:
            out = tdc(left_feas, right_feas, self.left2right, self.right2left, relu, dropout, opts, fold_in, feeds_conv)
            if out is not None:
                return out
        l2r, r2l = edge_index.t(), edge_index
        right_updated = self.left2right((left_feas, right_feas), l2r, edge_weight, relu=relu, dropout=dropout,
                                        opts=opts)
        left_updated = self.right2left((right_feas, left_feas), r2l, edge_weight, relu=relu, dropout=dropout,
                                       opts=opts)
        return left_updated, right_updated


def add_knowledge(left_logit, right_logit, left_feas, right_feas, bound=10):
    """arch.py:129-141: L2-normalise x10, -bound on impossible statuses."""
    return _fc.knowledge(left_logit, left_feas, bound), _fc.knowledge(right_logit, right_feas, bound)


class GCNBase(nn.Module):
    """arch.py:108-114 (state_dict-only checkpoints)."""

    def save(self, pn):
        torch.save(self.state_dict(), pn)

    def load(self, pn):
        st = torch.load(pn, map_location=torch.device("cpu"), weights_only=True)
        self.load_state_dict(st)


class GCN_FC(GCNBase):
    """arch.py:167-193."""

    def __init__(self, p, q, hids=128, depth=3, dp=.1, *args, compute_dtype=torch.float32,
                 options: PathOptions | None = None, **kwargs):
        super().__init__()
        # the kernel / fusion choices of this model's hot path (lpgnn.options; defaults from the environment)
        self.options = options or _DEFAULT_OPTIONS
        # bf16 = the c5 configuration (BASELINE.json configs[4]): activations,
        # SpMM storage and FC operands in bf16 (fp32 accumulation, fp32 master
        # weights); logits return to fp32 before add_knowledge.
        if compute_dtype in ("bf16", "bfloat16"):
            compute_dtype = torch.bfloat16
        if compute_dtype not in (torch.float32, torch.bfloat16):
            raise ValueError(f"compute_dtype must be float32 or bfloat16, got {compute_dtype}")
        self.compute_dtype = compute_dtype
        self.conv1 = GraphConvTwoDirection(p, q, hids)
        self.layers = nn.ModuleList()
        for _ in range(depth - 2):
            self.layers.append(GraphConvTwoDirection(hids, hids, hids))
        self.lin_left = nn.Linear(hids, 3)
        self.lin_right = nn.Linear(hids, 3)
        self.dp = dp

    def set_compute_dtype(self, dtype) -> "GCN_FC":
        """fp32 (default) or bf16 activations / SpMM / MFMA FC (fp32 master
        weights either way) -- the 16-bit path the CLI's --fp16 selects."""
        if dtype in ("bf16", "bfloat16"):
            dtype = torch.bfloat16
        if dtype not in (torch.float32, torch.bfloat16):
            raise ValueError(f"compute_dtype must be float32 or bfloat16, got {dtype}")
        self.compute_dtype = dtype
        return self

    def forward(self, batch):
        x_left, x_right, edge_index = batch.x_s, batch.x_t, batch.edge_index
        cd = self.compute_dtype
        half = (x_left.dtype == torch.float16 or x_right.dtype == torch.float16
                or self.lin_left.weight.dtype == torch.float16)
        if half:
            # val.py:269 model.half() + batch_to(half=True) (utils.py:909-915): the reference's --fp16
            # inference mode -- fp16 storage of features, activations, weights and logits on the fp16
            # kernels (v_mfma_f32_16x16x32_f16 FC, fp16 SpMM, heads, add_knowledge in half precision);
            # fp32 accumulation inside every kernel, one rounding per stored tensor.  Forward only, as
            # in the reference (train.py trains in fp32).
            if self.training:
                raise RuntimeError("GCN_FC: fp16 is the reference's inference mode (val.py:269 model.half() "
                                   "+ model.eval()); train in fp32 or bf16")
            cd = torch.float16
        # conv -> ReLU (arch.py:181-182): the ReLU is the FC kernel's epilogue.
        opts = self.options
        dp = self.dp if self.training else 0.0
        layers = list(self.layers)
        single = isinstance(edge_index, BipartiteCSR) and getattr(edge_index, "partitioned_conv", None) is None
        part_heads = getattr(edge_index, "two_direction_heads", None)  # row-partitioned multi-GPU adjacency
        fuse_heads = opts.fuse_heads and len(layers) > 0 and cd == torch.float32 and (single or part_heads is not None)
        ex = getattr(edge_index, "ex", None)  # a partition's boundary exchange (lpgnn.partition.Exchange)
        if ex is not None:  # no halo broadcast of an earlier (e.g. aborted) forward may still be in flight
            ex.settle_all()
        # feeds_conv: the layer's outputs go to another GraphConvTwoDirection (not to the heads)
        left, right = self.conv1(x_left.to(cd), x_right.to(cd), edge_index, relu=True, opts=opts,
                                 feeds_conv=len(layers) > 0)
        chain = layers[:-1] if fuse_heads else layers
        for i, conv in enumerate(chain):
            # conv -> dropout -> ReLU (arch.py:185-188).  ReLU commutes with
            # dropout (x * mask / (1-p), a non-negative scale), so the ReLU is
            # fused into the FC and dropout follows it (inside the conv, so a
            # partitioned run drops each variable once, at its owner).
            # fold_in: the previous layer's outputs feed only this layer (bf16: its ReLU/dropout
            # backward runs in this layer's input-gradient stores)
            left, right = conv(left, right, edge_index, relu=True, dropout=dp, fold_in=True, opts=opts,
                               feeds_conv=fuse_heads or i < len(chain) - 1)
        out = None
        if fuse_heads:  # last layer + heads (arch.py:184-190) as one node: one backward pass over its output
            last = layers[-1]
            if single:
                out = _conv.two_direction_heads(left, right, edge_index, last.left2right, last.right2left,
                                                self.lin_left, self.lin_right, dp, fold_in=True, opts=opts)
            else:
                out = part_heads(left, right, last.left2right, last.right2left, self.lin_left, self.lin_right, dp,
                                 opts, fold_in=True)
                if out is None:  # not applicable on this adjacency: the separate path
                    left, right = last(left, right, edge_index, relu=True, dropout=dp, opts=opts)
        if ex is not None:  # every deferred broadcast was settled by its consumer; make sure of it
            ex.settle_all()
        if out is not None:
            left, right = out
        else:
            # both heads fold the last layer's ReLU/dropout backward (bf16) or neither does
            left = _fc.linear(left, self.lin_left.weight, self.lin_left.bias, fold_in=True, opts=opts)
            right = _fc.linear(right, self.lin_right.weight, self.lin_right.bias, fold_in=True, opts=opts)
        if half:  # arch.py:191 on the fp16 logits, in half precision (fp16 out, as the reference's)
            return add_knowledge(left, right, x_left, x_right)
        return add_knowledge(left.float(), right.float(), x_left, x_right)


_ARCH_RE = re.compile(r"^\s*([A-Za-z_]\w*)\s*\((.*)\)\s*$", re.S)


def build_model(arch: str) -> nn.Module:
    """Safe replacement for ``eval(args.arch)`` (train.py:79, val.py:266,
    pred_basis.py:128): parses e.g. ``GCN_FC(8,8,hids=1024,depth=3)``
    with literal arguments only."""
    mt = _ARCH_RE.match(arch)
    if not mt:
        raise ValueError(f"cannot parse arch string {arch!r}")
    name, argstr = mt.group(1), mt.group(2)
    classes = {"GCN_FC": GCN_FC}
    if name not in classes:
        raise ValueError(f"arch {name!r} is outside this build's scope (GCN_FC only; SURVEY.md §2)")
    call = ast.parse(f"f({argstr})", mode="eval").body
    args = [ast.literal_eval(a) for a in call.args]
    kwargs = {k.arg: ast.literal_eval(k.value) for k in call.keywords}
    return classes[name](*args, **kwargs)


def arch_depth(arch: str) -> int:
    """train.py:108-110 / val.py:14-16: hops = depth - 1 (2 if absent)."""
    d = re.findall(r"depth=(\d+)", arch)
    return 2 if len(d) == 0 else int(d[0]) - 1
