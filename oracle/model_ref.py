"""ORACLE -- test infrastructure only.

CPU restatement of the reference's GCN_FC hot path, used by tests/,
``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline leg as the
checker / the timed CPU baseline.  Nothing in ``lp-gnn_amd/`` imports this
module; the product path fails loudly without its HIP library.

Every function cites what it restates:

* reference files (vbdai/lp-gnn @ /root/reference): arch.py, dataset.py,
  val.py, train.py, utils.py;
* upstream, NOT vendored in /root/reference, restated from the versions the
  reference pins (readme.md:51-52): torch_geometric 2.1 (``GraphConv``,
  ``Linear`` init, ``to_undirected``) and torch_sparse 0.6.12
  (``SparseTensor.from_edge_index``, ``.t()``/``csr2csc``, ``spmm_sum``,
  ``neighbor_sample`` behind PyG's ``NeighborLoader``).

Parity pinning (see DESIGN.md "Parity"): the pure-torch reference functions
(add_knowledge arch.py:129-141, inference_gnn val.py:106-124, balanced
train.py:39-46, labels_to_balanced_weights utils.py:286-299) and the GCN_FC /
GraphConvTwoDirection orchestration (arch.py:51-81, 167-193) are pinned by
golden vectors produced by running the reference's own function bodies
(tests/golden/make_golden.py).  The upstream torch_sparse/PyG arithmetic has
no vectors anywhere ("parity unpinned" for that layer): it is restated here.
"""
from __future__ import annotations

import ctypes
import math
import os

import numpy as np
import torch
import torch.nn.functional as F

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


# --------------------------------------------------------------------------
# C restatement of torch_sparse spmm_cpu (spmm_ref.c)
# --------------------------------------------------------------------------
def lib():
    """Load (building if needed) oracle/liboracle_spmm.so."""
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle_spmm.so")
        if not os.path.exists(path):
            import subprocess

            subprocess.run(["make", "-s", "-C", _HERE], check=True)
        L = ctypes.CDLL(path)
        i64, p = ctypes.c_int64, ctypes.c_void_p
        L.oracle_spmm_f32.argtypes = [i64, p, p, p, p, i64, i64, p, i64, ctypes.c_int]
        L.oracle_spmm_f32.restype = None
        L.oracle_spmm_bf16.argtypes = [i64, p, p, p, p, i64, i64, p, i64, ctypes.c_int]
        L.oracle_spmm_bf16.restype = None
        L.oracle_max_threads.restype = ctypes.c_int
        L.oracle_fc_f32.argtypes = [i64, i64, i64, p, i64, p, i64, i64, p, i64, p, i64, p, p, i64, p, i64,
                                    ctypes.c_int, ctypes.c_int]
        L.oracle_fc_f32.restype = None
        _LIB = L
    return _LIB


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def spmm_f32(rowptr, col, val, X, nthreads: int = 0) -> np.ndarray:
    """Y = CSR(rowptr, col, val) @ X in torch_sparse spmm_cpu order (fp32)."""
    rowptr = np.ascontiguousarray(rowptr, dtype=np.int64)
    col = np.ascontiguousarray(col, dtype=np.int32)
    val = np.ascontiguousarray(val, dtype=np.float32)
    X = np.ascontiguousarray(X, dtype=np.float32)
    M = rowptr.shape[0] - 1
    Fd = X.shape[1]
    Y = np.empty((M, Fd), dtype=np.float32)
    if M > 0 and Fd > 0:
        lib().oracle_spmm_f32(M, _ptr(rowptr), _ptr(col), _ptr(val), _ptr(X), Fd, Fd, _ptr(Y), Fd, nthreads)
    return Y


def spmm_bf16(rowptr, col, val, Xbits, nthreads: int = 0) -> np.ndarray:
    """bf16-storage variant (uint16 bit patterns in/out, fp32 accumulate)."""
    rowptr = np.ascontiguousarray(rowptr, dtype=np.int64)
    col = np.ascontiguousarray(col, dtype=np.int32)
    val = np.ascontiguousarray(val, dtype=np.float32)
    Xbits = np.ascontiguousarray(Xbits, dtype=np.uint16)
    M = rowptr.shape[0] - 1
    Fd = Xbits.shape[1]
    Y = np.empty((M, Fd), dtype=np.uint16)
    if M > 0 and Fd > 0:
        lib().oracle_spmm_bf16(M, _ptr(rowptr), _ptr(col), _ptr(val), _ptr(Xbits), Fd, Fd, _ptr(Y), Fd, nthreads)
    return Y


def fc_kchain(A1, W1, A2=None, W2=None, bias=None, relu=False, nthreads: int = 0, add=None) -> np.ndarray:
    """lin_rel(A1) + lin_root(A2) [+ ReLU] as lpg_fc_f32 evaluates it: one
    fp32 fma chain per output in k order (A1 part then A2 part) from +0, then
    + add (the accumulate flag's addend, [M, N]), then + bias (fc_ref.c).
    Arrays are numpy/torch fp32; weights [out, in]."""
    f = lambda t: None if t is None else np.ascontiguousarray(
        t.detach().numpy() if isinstance(t, torch.Tensor) else t, dtype=np.float32)
    A1, W1, A2, W2, bias, add = f(A1), f(W1), f(A2), f(W2), f(bias), f(add)
    M, K1 = A1.shape
    N = W1.shape[0]
    K2 = 0 if A2 is None else A2.shape[1]
    C = np.empty((M, N), np.float32)
    if M and N:
        z = np.zeros(1, np.float32)
        lib().oracle_fc_f32(M, N, K1, _ptr(A1), K1, _ptr(W1), K1, K2, _ptr(A2 if K2 else z), max(K2, 1),
                            _ptr(W2 if K2 else z), max(K2, 1), None if bias is None else _ptr(bias), _ptr(C), N,
                            None if add is None else _ptr(add), N, int(relu), nthreads)
    return C


# --------------------------------------------------------------------------
# Sparse layout restatement (torch_sparse 0.6.12 SparseTensor)
# --------------------------------------------------------------------------
def csr_from_coo(row, col, val, m: int, n: int):
    """SparseTensor.from_edge_index(edge_index, edge_attr, (m, n)) -> CSR.

    Upstream: ``idx = row * n + col; perm = idx.argsort()`` (stable for unique
    keys), ``rowptr = ind2ptr(row[perm], m)``.  Called at dataset.py:301-304.
    Returns (rowptr int64[m+1], col int32[nnz], val f32[nnz]).
    """
    row = np.asarray(row, dtype=np.int64)
    col = np.asarray(col, dtype=np.int64)
    key = row * n + col
    perm = np.argsort(key, kind="stable")
    r = row[perm]
    rowptr = np.zeros(m + 1, dtype=np.int64)
    np.add.at(rowptr, r + 1, 1)
    rowptr = np.cumsum(rowptr)
    return rowptr, col[perm].astype(np.int32), np.asarray(val, dtype=np.float32)[perm]


def csr_transpose(rowptr, col, val, m: int, n: int):
    """SparseTensor.t() (arch.py:71): csr2csc = argsort(col * m + row)."""
    rowptr = np.asarray(rowptr, dtype=np.int64)
    row = np.repeat(np.arange(m, dtype=np.int64), np.diff(rowptr))
    return csr_from_coo(col.astype(np.int64), row, val, n, m)


# --------------------------------------------------------------------------
# Model restatement
# --------------------------------------------------------------------------
class _OracleSpMM(torch.autograd.Function):
    """torch_sparse SPMMSum (csrc/spmm.cpp): fwd spmm(A, X); bwd spmm(A^T, dY)."""

    @staticmethod
    def forward(ctx, X, fwd, bwd):
        ctx.bwd = bwd
        return torch.from_numpy(spmm_f32(*fwd, X.detach().numpy()))

    @staticmethod
    def backward(ctx, gY):
        return torch.from_numpy(spmm_f32(*ctx.bwd, gY.contiguous().numpy())), None, None


def _scipy64(csr, n_cols: int):
    import scipy.sparse as sp

    rowptr, col, val = csr
    return sp.csr_matrix((np.asarray(val, np.float64), col, rowptr), shape=(rowptr.shape[0] - 1, n_cols))


class _OracleSpMM64(torch.autograd.Function):
    """fp64 spmm (scipy, order-free: the 'truth' side of the fp32 comparisons);
    bwd = A^T dY, as SPMMSum's."""

    @staticmethod
    def forward(ctx, X, fwd, bwd):
        ctx.bwd, ctx.n_src = bwd, X.shape[0]
        return torch.from_numpy(_scipy64(fwd, X.shape[0]) @ X.detach().numpy())

    @staticmethod
    def backward(ctx, gY):
        A_t = _scipy64(ctx.bwd, gY.shape[0])
        return torch.from_numpy(A_t @ gY.detach().contiguous().numpy()), None, None


def spmm_t(csr, csr_t, X: torch.Tensor) -> torch.Tensor:
    """Differentiable spmm: fp32 in torch_sparse spmm_cpu order; fp64 through
    scipy (the order-free fp64 truth)."""
    if X.dtype == torch.float64:
        return _OracleSpMM64.apply(X, csr, csr_t)
    return _OracleSpMM.apply(X, csr, csr_t)


def reassociate(n_src: int, n_dst: int, f_src: int, f_out: int) -> bool:
    """The association rule of lpgnn/conv.py restated: lin_rel(S x) is
    evaluated as S (x W_rel^T) iff the source side has fewer rows than the
    destination side and f_out <= f_src."""
    return n_src < n_dst and f_out <= f_src


def graph_conv(x_src, x_dst, adj, adj_t, W_rel, b_rel, W_root, fc="mkl", relu=False, reassoc=False):
    """PyG 2.1 GraphConv.forward with a SparseTensor adj_t (aggr='add'):

    out = propagate(...)      -> message_and_aggregate = matmul(adj_t, x[0], 'add')
    out = self.lin_rel(out)   -> F.linear(out, W_rel, b_rel)
    out += self.lin_root(x[1])-> F.linear(x_dst, W_root)   (lin_root: bias=False)

    fc="mkl": torch CPU F.linear (the reference's own evaluation, autograd);
    fc="kchain": the bitwise order of lpg_fc_f32 (forward only).
    relu: the following ReLU (arch.py:182/188) applied here.
    reassoc (kchain only): apply the association rule -- when it holds, the
    HIP path's order: h = kchain(x_src W_rel^T), P = S h (spmm), then
    kchain(x_dst W_root^T) + P + b_rel (returns agg = None).
    """
    if fc == "kchain" and reassoc and reassociate(x_src.shape[0], x_dst.shape[0], x_src.shape[1], W_rel.shape[0]):
        P = spmm_f32(*adj, fc_kchain(x_src, W_rel))
        return torch.from_numpy(fc_kchain(x_dst, W_root, bias=b_rel, relu=relu, add=P)), None
    agg = spmm_t(adj, adj_t, x_src)
    if fc == "kchain":
        out = torch.from_numpy(fc_kchain(agg, W_rel, x_dst, W_root, b_rel, relu=relu))
        return out, agg
    out = F.linear(agg, W_rel, b_rel)
    out = out + F.linear(x_dst, W_root)
    return (torch.relu(out) if relu else out), agg


def conv_two_direction(sd, prefix, left, right, A, AT, fc="mkl", relu=False, reassoc=False):
    """GraphConvTwoDirection.forward, arch.py:65-81.

    l2r, r2l = edge_index, edge_index.t(); l2r, r2l = r2l, l2r  (arch.py:71-74)
    => left2right aggregates with A^T (rows = vars), right2left with A.
    Both directions read the same-layer inputs.
    """
    g = lambda d, k: sd[f"{prefix}.{d}.{k}"]
    right_new, agg_r = graph_conv(left, right, AT, A, g("left2right", "lin_rel.weight"),
                                  g("left2right", "lin_rel.bias"), g("left2right", "lin_root.weight"), fc, relu,
                                  reassoc)
    left_new, agg_l = graph_conv(right, left, A, AT, g("right2left", "lin_rel.weight"),
                                 g("right2left", "lin_rel.bias"), g("right2left", "lin_root.weight"), fc, relu,
                                 reassoc)
    return left_new, right_new, agg_l, agg_r


def add_knowledge(left_logit, right_logit, left_feas, right_feas, bound=10):
    """arch.py:129-141."""
    cons_l_mask, cons_u_mask = left_feas[:, -3].abs().bool(), left_feas[:, -1].abs().bool()
    vars_l_mask, vars_u_mask = right_feas[:, -3].abs().bool(), right_feas[:, -1].abs().bool()
    left_logit = F.normalize(left_logit) * 10
    right_logit = F.normalize(right_logit) * 10
    left_logit[cons_l_mask, 0] = left_logit[cons_l_mask, 0] - bound
    left_logit[cons_u_mask, 2] = left_logit[cons_u_mask, 2] - bound
    right_logit[vars_l_mask, 0] = right_logit[vars_l_mask, 0] - bound
    right_logit[vars_u_mask, 2] = right_logit[vars_u_mask, 2] - bound
    return left_logit, right_logit


def gcn_fc_forward(sd, x_s, x_t, A, AT, depth: int, keep=None, fc="mkl", reassoc=False):
    """GCN_FC.forward, arch.py:179-193, eval mode (dropout is identity).

    sd: state_dict (tensors), A/AT: (rowptr, col, val) CSR of A and A^T.
    keep: optional dict that receives per-layer intermediates.
    fc: "mkl" (torch CPU F.linear, differentiable) or "kchain" (bitwise order
    of the HIP FC kernel, forward only); reassoc: with "kchain", the HIP
    path's association rule (graph_conv).
    """
    left, right, agg_l, agg_r = conv_two_direction(sd, "conv1", x_s, x_t, A, AT, fc, relu=True, reassoc=reassoc)
    if keep is not None:
        keep["agg_l0"], keep["agg_r0"], keep["left0"], keep["right0"] = agg_l, agg_r, left, right
    for i in range(depth - 2):
        left, right, agg_l, agg_r = conv_two_direction(sd, f"layers.{i}", left, right, A, AT, fc, relu=True,
                                                       reassoc=reassoc)
        if keep is not None:
            keep[f"agg_l{i+1}"], keep[f"agg_r{i+1}"] = agg_l, agg_r
            keep[f"left{i+1}"], keep[f"right{i+1}"] = left, right
    if fc == "kchain":
        left = torch.from_numpy(fc_kchain(left, sd["lin_left.weight"], bias=sd["lin_left.bias"]))
        right = torch.from_numpy(fc_kchain(right, sd["lin_right.weight"], bias=sd["lin_right.bias"]))
    else:
        left = F.linear(left, sd["lin_left.weight"], sd["lin_left.bias"])
        right = F.linear(right, sd["lin_right.weight"], sd["lin_right.bias"])
    if keep is not None:
        keep["head_l"], keep["head_r"] = left, right
    return add_knowledge(left, right, x_s, x_t)


# --------------------------------------------------------------------------
# The --fp16 inference mode (val.py:269 model.half(), utils.py:909-915 batch_to(half=True))
# --------------------------------------------------------------------------
def r16(t: torch.Tensor) -> torch.Tensor:
    """The fp16 storage of a tensor computed in fp32 (torch's half ops compute in fp32 and round
    each stored result to nearest even): fp16 values, held as fp32."""
    return t.half().float()


def spmm_f16(rowptr, col, val, X16) -> torch.Tensor:
    """torch_sparse spmm_sum on fp16 storage as this build defines it: the fp16 values (X16 and the
    edge values, exact in fp32) summed in spmm_cpu's sequential order in fp32, one rounding to fp16 per
    output.  (torch_sparse 0.6.12's CUDA kernel accumulates in the storage type -- absent here, not
    reproduced; the fp32 sum is the more accurate one.)"""
    val16 = r16(torch.from_numpy(np.asarray(val, np.float32))).numpy()
    X = np.ascontiguousarray(X16.detach().float().numpy() if isinstance(X16, torch.Tensor) else X16, np.float32)
    return r16(torch.from_numpy(spmm_f32(rowptr, col, val16, X)))


def _linear16(x, W, b=None):
    """F.linear of fp16 operands with fp32 accumulation (MKL), the bias added in fp32: NOT rounded."""
    y = x.float() @ r16(W.float()).t()
    return y if b is None else y + r16(b.float())


def graph_conv_fp16(x_src, x_dst, adj, W_rel, b_rel, W_root, relu=False, reassoc=True):
    """GraphConv (PyG 2.1, arch.py:57-62) with fp16 storage, one rounding per stored tensor:
    out = r16(act(agg W_rel^T + x_dst W_root^T + b_rel)), agg = spmm_f16(adj, x_src); with the
    association rule (lpgnn/conv.py), P = spmm_f16(r16(x_src W_rel^T)) and out = r16(act(x_dst W_root^T
    + P + b_rel)) -- the HIP path's fused FC epilogue."""
    if reassoc and reassociate(x_src.shape[0], x_dst.shape[0], x_src.shape[1], W_rel.shape[0]):
        P = spmm_f16(*adj, r16(_linear16(x_src, W_rel)))
        out = _linear16(x_dst, W_root) + P + r16(b_rel.float())
    else:
        agg = spmm_f16(*adj, x_src)
        out = _linear16(agg, W_rel, b_rel) + _linear16(x_dst, W_root)
    return r16(torch.relu(out) if relu else out)


def _fma_f32_exact(a64: np.ndarray, b64: np.ndarray, c32: np.ndarray) -> np.ndarray:
    """fma(a, b, c) correctly rounded to fp32 for a * b exact in fp64 (fp16 operands) and fp32 c:
    TwoSum of the product and c, then a round-to-nearest-even of hi + lo that resolves fp64 ties."""
    p = a64 * b64
    c = c32.astype(np.float64)
    hi = p + c
    bb = hi - p
    lo = (p - (hi - bb)) + (c - bb)
    r = hi.astype(np.float32)
    r64 = r.astype(np.float64)
    diff = hi - r64
    other = np.nextafter(r, np.where(diff > 0, np.float32(np.inf), np.float32(-np.inf)).astype(np.float32))
    tie = (diff != 0) & (np.abs(diff) * 2 == np.abs(other.astype(np.float64) - r64))
    return np.where(tie & (np.sign(lo) == np.sign(diff)), other, r)


def add_knowledge_fp16(logit16, feas, bound=10):
    """arch.py:129-141 on fp16 logits as torch's half ops define it on the device the reference's
    --fp16 mode runs on (lpg_knowledge_f16): each op computes in fp32 with IEEE-correct rounding and
    stores fp16 -- n = fp16(sqrt(fma(x2, x2, fma(x1, x1, x0 x0)))), clamp_min(1e-12) of a half tensor
    = max(n, 0), y = fp16(fp16(x / n) * 10), y0 / y2 = fp16(y - bound) where the masks say so.  Restated
    with numpy's IEEE float32 sqrt / divide and an exact fma (torch's vectorised CPU sqrt is not
    correctly rounded on every host: one box's oracle differed in 3 of 720 000 values)."""
    x16 = logit16.numpy().astype(np.float16)
    x = x16.astype(np.float64)
    ss = (x[:, 0] * x[:, 0]).astype(np.float32)  # exact: 22-bit product
    ss = _fma_f32_exact(x[:, 1], x[:, 1], ss)
    ss = _fma_f32_exact(x[:, 2], x[:, 2], ss)
    with np.errstate(divide="ignore", invalid="ignore"):
        n = np.sqrt(ss).astype(np.float16).astype(np.float32)
        d = np.maximum(n, np.float32(0.0))
        q = (x16.astype(np.float32) / d[:, None]).astype(np.float16).astype(np.float32)
        y = (q * np.float32(10.0)).astype(np.float16).astype(np.float32)
    m0 = feas[:, -3].numpy() != 0
    m2 = feas[:, -1].numpy() != 0
    y[m0, 0] = (y[m0, 0] - np.float32(bound)).astype(np.float16).astype(np.float32)
    y[m2, 2] = (y[m2, 2] - np.float32(bound)).astype(np.float16).astype(np.float32)
    return torch.from_numpy(y)


def gcn_fc_forward_fp16(sd, x_s, x_t, A, AT, depth: int, keep=None):
    """GCN_FC.forward (arch.py:179-193) after model.half() and batch_to(half=True): the oracle of the
    --fp16 mode.  Features, edge values, weights rounded to fp16; every layer's stored output
    rounded to fp16 (fp32 accumulation inside each op); heads r16(h W^T + b); add_knowledge in half
    precision.  Returns the fp16 logits (held as fp32)."""
    w = {k: (None if v is None else r16(v.float())) for k, v in sd.items()}
    left, right = r16(x_s.float()), r16(x_t.float())
    for i, prefix in enumerate(["conv1"] + [f"layers.{j}" for j in range(depth - 2)]):
        g = lambda d, k: w[f"{prefix}.{d}.{k}"]  # noqa: E731
        right_new = graph_conv_fp16(left, right, AT, g("left2right", "lin_rel.weight"), g("left2right", "lin_rel.bias"),
                                    g("left2right", "lin_root.weight"), relu=True)
        left_new = graph_conv_fp16(right, left, A, g("right2left", "lin_rel.weight"), g("right2left", "lin_rel.bias"),
                                   g("right2left", "lin_root.weight"), relu=True)
        left, right = left_new, right_new
        if keep is not None:
            keep[f"left{i}"], keep[f"right{i}"] = left, right
    hl = r16(_linear16(left, w["lin_left.weight"], w["lin_left.bias"]))
    hr = r16(_linear16(right, w["lin_right.weight"], w["lin_right.bias"]))
    if keep is not None:
        keep["head_l"], keep["head_r"] = hl, hr
    return add_knowledge_fp16(hl, x_s), add_knowledge_fp16(hr, x_t)


@torch.no_grad()
def inference_gnn_fp16(logits16, m):
    """val.py:106-124 on fp16 logits: the half softmax's fp16 probabilities (NaN -> 0); of the nodes tied
    at the m-th largest P[:, 1] the lowest indices are basic (torch.topk leaves that open; the HIP kernel's
    rule); argmax over {0, 2} with ties to 0."""
    pr = r16(F.softmax(logits16.float(), dim=-1))
    pr[torch.isnan(pr)] = 0
    order = np.lexsort((np.arange(pr.shape[0]), -pr[:, 1].double().numpy()))
    top = torch.from_numpy(order[:m])
    pred = torch.where(pr[:, 0] >= pr[:, 2], 0, 2).to(torch.int64)
    pred[top] = 1
    return pred


def init_state_dict(p: int, q: int, hids: int, depth: int, seed: int = 0):
    """GCN_FC(p, q, hids, depth) parameters with the reference's RNG stream.

    PyG 2.1 GraphConv.__init__ builds lin_rel = Linear(in_src, out, bias) and
    lin_root = Linear(in_dst, out, bias=False) -- each Linear.__init__ calls
    reset_parameters() -- and then GraphConv.reset_parameters() initialises
    both again.  PyG Linear init: kaiming_uniform(fan=in, a=sqrt(5)) on the
    weight, uniform(1/sqrt(in)) on the bias: the same bounds and draw order
    as torch.nn.Linear.  Heads are torch.nn.Linear (arch.py:175-176).
    """
    g = torch.Generator().manual_seed(seed)
    sd = {}

    def lin(out_f, in_f, bias):
        w = torch.empty(out_f, in_f)
        bound = math.sqrt(6.0 / ((1 + 5.0) * in_f))
        w.uniform_(-bound, bound, generator=g)
        b = None
        if bias:
            b = torch.empty(out_f)
            bb = 1.0 / math.sqrt(in_f)
            b.uniform_(-bb, bb, generator=g)
        return w, b

    def conv(prefix, l_dim, r_dim, out):
        for d, (src, dst) in (("left2right", (l_dim, r_dim)), ("right2left", (r_dim, l_dim))):
            lin(out, src, True)  # Linear ctor draws (discarded by the re-init below)
            lin(out, dst, False)
            w_rel, b_rel = lin(out, src, True)
            w_root, _ = lin(out, dst, False)
            sd[f"{prefix}.{d}.lin_rel.weight"] = w_rel
            sd[f"{prefix}.{d}.lin_rel.bias"] = b_rel
            sd[f"{prefix}.{d}.lin_root.weight"] = w_root

    conv("conv1", p, q, hids)
    for i in range(depth - 2):
        conv(f"layers.{i}", hids, hids, hids)
    for side in ("lin_left", "lin_right"):
        w, b = lin(3, hids, True)
        sd[f"{side}.weight"], sd[f"{side}.bias"] = w, b
    return sd


# --------------------------------------------------------------------------
# Post-processing / loss restatements
# --------------------------------------------------------------------------
@torch.no_grad()
def inference_gnn(logits, m):
    """val.py:106-124 (top-m basic, argmax over {0,2} for the rest)."""
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
def labels_to_balanced_weights(labels, merge_lu=True):
    """utils.py:286-299."""
    res = torch.zeros(3).to(labels.device)
    lbl, cnt = torch.unique(labels, return_counts=True)
    wei = cnt.sum() / cnt
    if len(lbl) == 2:
        res[lbl] = wei
    else:
        res[lbl] = wei
        if merge_lu:
            res[0] = res[2] = (res[0] + res[2]) / 2.
    return res


def balanced(logpr_cons, logpr_vars, y_s, y_t):
    """train.py:39-46."""
    loss = 0.
    m, n = len(y_s), len(y_t)
    criterion = torch.nn.CrossEntropyLoss(weight=labels_to_balanced_weights(y_s).to(logpr_cons.dtype))
    loss += (m + n) / m * criterion(logpr_cons, y_s)
    criterion = torch.nn.CrossEntropyLoss(weight=labels_to_balanced_weights(y_t).to(logpr_vars.dtype))
    loss += (m + n) / n * criterion(logpr_vars, y_t)
    return loss


# --------------------------------------------------------------------------
# Batch boundary restatement (dataset.py)
# --------------------------------------------------------------------------
def to_undirected(edge_index: np.ndarray, edge_attr: np.ndarray, num_nodes: int):
    """PyG 2.1 utils.to_undirected(edge_index, edge_attr) as called at
    dataset.py:252: cat both directions, coalesce (sort by row*N+col, add
    duplicate attrs)."""
    row = np.concatenate([edge_index[0], edge_index[1]])
    col = np.concatenate([edge_index[1], edge_index[0]])
    attr = np.concatenate([edge_attr, edge_attr])
    key = row * num_nodes + col
    perm = np.argsort(key, kind="stable")
    key, attr = key[perm], attr[perm]
    uniq, start = np.unique(key, return_index=True)
    summed = np.add.reduceat(attr, start) if len(attr) else attr
    return np.stack([uniq // num_nodes, uniq % num_nodes]), summed.astype(np.float32)


def to_csc(edge_index: np.ndarray, num_nodes: int):
    """PyG 2.1 ``loader.utils.to_csc`` (what NeighborSampler builds at
    construction): perm = argsort(col * N + row); colptr from the sorted
    destinations; row = sources in that order."""
    row, col = np.asarray(edge_index[0], np.int64), np.asarray(edge_index[1], np.int64)
    perm = np.argsort(col * num_nodes + row, kind="stable")
    colptr = np.searchsorted(col[perm], np.arange(num_nodes + 1))
    return colptr.astype(np.int64), row[perm], perm


def neighbor_sample(colptr, row, input_node, num_neighbors, directed: bool):
    """torch_sparse 0.6.12 ``neighbor_sample`` (csrc/cpu/neighbor_sample_cpu.cpp,
    replace=False), the sampler of PyG 2.1 NeighborLoader (train.py:111-116,
    val.py:22-27).  Only fanout -1 (all neighbours, val.py:23) is
    deterministic; a positive fanout is restated with Floyd's algorithm and
    Python's RNG, so only its properties are comparable.

    samples = input nodes; per hop, for every frontier node in order, every
    (or each sampled) in-neighbour v in CSC order is inserted into
    to_local_node if new (appended to samples); directed=True records the
    edge (local(v) -> frontier index).  directed=False instead returns, for
    every sample i in order, each in-edge whose source is sampled."""
    import random

    samples = [int(v) for v in input_node]
    to_local = {}
    for i, v in enumerate(samples):
        to_local.setdefault(v, i)
    rows, cols, edges = [], [], []
    begin, end = 0, len(samples)
    for k in num_neighbors:
        for i in range(begin, end):
            w = samples[i]
            c0, c1 = int(colptr[w]), int(colptr[w + 1])
            deg = c1 - c0
            if deg == 0:
                continue
            if k < 0 or k >= deg:
                picks = range(deg)
            else:
                chosen, picks = set(), []
                for j in range(deg - k, deg):
                    t = random.randint(0, j)
                    if t in chosen:
                        t = j
                    chosen.add(t)
                    picks.append(t)
            for t in picks:
                v = int(row[c0 + t])
                if v not in to_local:
                    to_local[v] = len(samples)
                    samples.append(v)
                if directed:
                    rows.append(to_local[v]), cols.append(i), edges.append(c0 + t)
        begin, end = end, len(samples)
    if not directed:
        for i, w in enumerate(samples):
            for e in range(int(colptr[w]), int(colptr[w + 1])):
                v = int(row[e])
                if v in to_local:
                    rows.append(to_local[v]), cols.append(i), edges.append(e)
    a = lambda x: np.asarray(x, dtype=np.int64)
    return a(samples), a(rows), a(cols), a(edges)


def my_to_bipartite(x, y, is_vars, edge_index, edge_attr, num_nodes, bs=None):
    """MyToBipartite.__call__, dataset.py:275-332 (batch_size = num_nodes).

    Returns dict(x_s, x_t, y_s, y_t, A=(rowptr,col,val), m, n, s_bs, t_bs).
    """
    is_vars = np.asarray(is_vars).astype(bool)
    is_cons = ~is_vars
    nvars = int(is_vars.sum())
    ncons = num_nodes - nvars
    mapping = np.empty(num_nodes, dtype=np.int64)
    mapping[is_cons] = np.arange(ncons)
    mapping[is_vars] = np.arange(nvars) + ncons
    ei = mapping[edge_index]
    mask = ei[0] < ncons
    assert mask.sum() * 2 == mask.shape[0]
    l2r = ei[:, mask].copy()
    l2r[1] -= ncons
    A = csr_from_coo(l2r[0], l2r[1], np.asarray(edge_attr)[mask], ncons, nvars)
    bs = num_nodes if bs is None else bs
    t_bs = int(is_vars[:bs].sum())
    return dict(x_s=x[is_cons], x_t=x[is_vars], y_s=y[is_cons], y_t=y[is_vars], A=A, m=ncons, n=nvars,
                s_bs=bs - t_bs, t_bs=t_bs)
