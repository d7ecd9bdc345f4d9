"""One GraphConvTwoDirection layer (arch.py:65-81) as a single autograd node.

Forward is exactly the per-direction path of ``GraphConv`` (PyG 2.1,
arch.py:57-62): for each direction the HIP SpMM aggregates the source side
(aggregation before ``lin_rel``, the reference's order) and one fused FC
kernel adds ``lin_rel``, its bias, ``lin_root`` and the ReLU (+ training
dropout).  Both directions read the same-layer inputs (arch.py:74-80).

Owning both directions in one backward lets the layer do what two separate
autograd nodes cannot:

* each input receives two gradients -- as the destination (root) of one
  direction and as the source (aggregated) side of the other -- and they are
  summed inside the second GEMM (``addmm_``, hipBLASLt beta = 1) instead of by
  a separate autograd accumulation pass over [rows, F];
* the source-side gradient Sᵀ(dZ·W_rel) is evaluated as (Sᵀ dZ)·W_rel
  whenever that puts the GEMM on the smaller node set (c2: the 100 K
  constraints instead of the 200 K variables for left2right): the same
  product, one GEMM over half the rows.

* a direction whose source side has fewer rows than its destination side
  (c2 left2right: 100 K constraints -> 200 K variables) and does not widen
  (f_out <= f_src) is evaluated re-associated, lin_rel(S x) = S (x W_rel^T):
  the lin_rel GEMM runs over the source rows, the SpMM aggregates the product,
  and the FC kernel adds lin_root + bias + ReLU onto it in place (lpg_fc_f32
  accumulate flag).  Same product, one GEMM over half the rows; its
  backward is the one the source-side gradient already uses (T = S^T dZ gives
  lin_rel's weight gradient as T^T x_src).  ``REASSOCIATE = False``
  (LPGNN_REASSOC=0) keeps the reference's association everywhere.

Forward numerics are bitwise the oracle's kchain order with the same
association rule (oracle/model_ref.py); logits stay within the north-star
1e-4 of the reference's MKL evaluation either way.  Gradients are
tolerance-level (the reference's own backward is autograd through MKL).
"""
from __future__ import annotations

import functools

import torch
from torch import Tensor

from . import fc as _fc
from .options import DEFAULT, PathOptions
from .sparse import BipartiteCSR, CSR, spmm_forward as _spmm_forward

_GEMM_FLOPS = 160e12  # in-step rates used only to pick the cheaper association
_SPMM_BYTES = 7e12
# options.overlap (LPGNN_OVERLAP=1): run the HBM-bound SpMMs that are independent of the current FC /
# GEMM on a second stream beside it.  Measured on c2: ~1 ms (2.6 %) more whole-step throughput in
# round 1; at the round-3 kernels 20.88-21.09 against 21.05-21.08 ms (noise), while the overlapped
# SpMM launches share CUs and HBM with the FC and read 0.85 of the roofline instead of 0.98 -- off by
# default.
_SIDE = {}


def _side_stream(device):
    if device not in _SIDE:
        _SIDE[device] = torch.cuda.Stream(device)
    return _SIDE[device]


def reassociate(n_src: int, n_dst: int, f_src: int, f_out: int, enabled: bool = True) -> bool:
    """The association rule: lin_rel(S x) evaluated as S (x W_rel^T) iff the
    source side is the smaller node set and the SpMM does not get wider
    (never worse on either the GEMM or the SpMM); ``enabled`` = options.reassociate."""
    return enabled and n_src < n_dst and f_out <= f_src


def _src_first(S: CSR, f_out: int, f_in: int, esz: int) -> bool:
    """True if grad_src = (Sᵀ dZ) W is cheaper than Sᵀ (dZ W) (S: dst x src)."""
    gemm = lambda rows: 2.0 * rows * f_out * f_in / _GEMM_FLOPS
    spmm = lambda f: (S.nnz * f + S.n_cols * f) * esz / _SPMM_BYTES
    return spmm(f_out) + gemm(S.n_cols) < gemm(S.n_rows) + spmm(f_in)


def _forward_core(ctx, left, right, adj, w_rel_l2r, b_l2r, w_root_l2r, w_rel_r2l, b_r2l, w_root_r2l, relu, dropout,
                  heads=None, heads_only=False, opts: PathOptions = DEFAULT, bits_out: bool = False):
    """The layer's forward (both directions); records on ctx what the backward
    needs and returns (left_new, right_new, tensors to save, logits).  With
    heads = ((Wh_l, bh_l), (Wh_r, bh_r)) the heads run in the FC epilogues
    (fp32) and logits = (logit_l, logit_r), else None."""
    if dropout > 0 and not relu:
        raise RuntimeError("lpgnn FC: fused dropout requires the ReLU epilogue")
    # bf16 (c5) or fp16 (the --fp16 inference mode: forward only) storage: the 16-bit kernels
    bf16 = left.dtype in _fc.HALF16
    ws = (w_rel_l2r, w_root_l2r, w_rel_r2l, w_root_r2l)
    if bf16:
        ws = tuple(w.to(left.dtype) for w in ws)
    A, AT = adj.fwd, adj.bwd  # A: cons x vars (right2left), AT: vars x cons (left2right)
    seed_r = _fc._new_seed() if dropout > 0 else 0
    seed_l = _fc._new_seed() if dropout > 0 else 0
    f_out = ws[0].shape[0]
    ra_r = reassociate(AT.n_cols, AT.n_rows, left.shape[1], f_out, opts.reassociate)
    ra_l = reassociate(A.n_cols, A.n_rows, right.shape[1], f_out, opts.reassociate)
    fwd32 = functools.partial(_fc.fc_forward, arith=opts.arith)
    spmm_forward = functools.partial(_spmm_forward, heavy=opts.spmm_heavy)  # noqa: F811 (the model's options)

    hd = heads if heads is not None and not bf16 else (None, None)
    # no-grad (eval) forward of the heads layer: its output feeds only the heads, so the fused kernels
    # skip storing it (LPG_FC_HEADS_ONLY); the returned layer outputs then hold no values.  (Decided by
    # the caller: inside an autograd.Function's forward grad mode is always off.)
    ho = heads is not None and heads_only

    # bf16 ReLU layers also write their output's 1-bit ReLU mask (options.relu_bits): the next layer's
    # folded ReLU backward reads it instead of the output (lpg_fc_bf16_relu_bwd_bits, 1/16 of the bytes).
    # bits_out (decided by the caller, outside the autograd.Function): a GraphConvTwoDirection layer
    # consumes this output and a backward will run -- the heads read Y, an eval forward reads nothing
    want_bits = bits_out and bf16 and relu and opts.relu_bits and f_out % 8 == 0 and left.dtype == torch.bfloat16

    def direction(S, x_src, x_dst, w_rel, b, w_root, seed, ra, agg=None, head=None):
        """(output, aggregate kept for the backward, logits of `head` or None, ReLU mask bits or None)."""
        fc = _fc.fc_forward_bf16 if bf16 else fwd32
        bits = (torch.empty((x_dst.shape[0], f_out // 8), dtype=torch.uint8, device=x_dst.device) if want_bits
                else None)
        mo = {} if bits is None else {"mask_out": bits}
        if ra:  # S (x_src W_rel^T), then lin_root + bias + ReLU accumulated onto it in place
            y = spmm_forward(S, fc(x_src, w_rel, None, None, None, False))
            if head is not None:
                y, lg = fwd32(x_dst, w_root, None, None, b, relu, dropout, seed, out=y, accumulate=True, heads=head,
                              heads_only=ho)
                return y, None, lg, None
            return fc(x_dst, w_root, None, None, b, relu, dropout, seed, out=y, accumulate=True, **mo), None, None, bits
        agg = spmm_forward(S, x_src) if agg is None else agg
        if head is not None:
            y, lg = fwd32(agg, w_rel, x_dst, w_root, b, relu, dropout, seed, heads=head, heads_only=ho)
            return y, agg, lg, None
        return fc(agg, w_rel, x_dst, w_root, b, relu, dropout, seed, **mo), agg, None, bits

    side = _side_stream(left.device) if opts.overlap and not ra_l else None
    agg_l = None
    if side is not None:  # right2left's HBM-bound SpMM beside left2right's MFMA-bound FC
        side.wait_stream(torch.cuda.current_stream(left.device))
        with torch.cuda.stream(side):
            agg_l = spmm_forward(A, right)
    # arch.py:75-77: right' = left2right((left, right), A^T)
    right_new, agg_r, logit_r, bits_r = direction(AT, left, right, ws[0], b_l2r, ws[1], seed_r, ra_r, head=hd[1])
    if side is not None:
        torch.cuda.current_stream(left.device).wait_stream(side)
        agg_l.record_stream(torch.cuda.current_stream(left.device))
    # arch.py:78-80: left' = right2left((right, left), A)
    left_new, agg_l, logit_l, bits_l = direction(A, right, left, ws[2], b_r2l, ws[3], seed_l, ra_l, agg_l,
                                                 head=hd[0])
    ctx.adj, ctx.relu, ctx.bf16, ctx.opts = adj, relu, bf16, opts
    ctx.out_bits = (bits_l, bits_r) if want_bits else None
    ctx.f16 = left.dtype == torch.float16
    ctx.scale = _fc.dropout_scale(dropout)
    ctx.has_b = (b_l2r is not None, b_r2l is not None)
    # conv1's shape (narrow LP-feature inputs, kept aggregates, ReLU without dropout, fp32): its weight
    # gradients can be folded into the next layer's input-gradient GEMM (lpg_fc_x3_relu_wgrad_f32)
    ctx.narrow = (agg_l is not None and agg_r is not None and agg_l.shape[1] + left.shape[1] <= 16
                  and agg_r.shape[1] + right.shape[1] <= 16)
    ctx.small_relu = not bf16 and relu and dropout == 0 and ctx.narrow
    logits = None if heads is None or bf16 else (logit_l, logit_r)
    return left_new, right_new, (left, right, agg_l, agg_r, left_new, right_new, *ws), logits


class _TwoDirection(torch.autograd.Function):
    @staticmethod
    def forward(ctx, left, right, adj, w_rel_l2r, b_l2r, w_root_l2r, w_rel_r2l, b_r2l, w_root_r2l, relu, dropout,
                prev=None, opts=DEFAULT, bits_out=False):
        """``prev``: the backward node of the layer that produced (left, right) and feeds only this
        layer (foldable_producer): bf16 -- its ReLU/dropout backward is folded into this layer's
        input-gradient stores (lpg_fc_bf16_relu_bwd) and it takes dZ as given (column sums only);
        fp32 conv1 -- its weight gradients are folded into this layer's input-gradient GEMMs
        (lpg_fc_x3_relu_wgrad_f32) and handed to it (``folded_wgk``)."""
        left_new, right_new, saved, _ = _forward_core(ctx, left, right, adj, w_rel_l2r, b_l2r, w_root_l2r,
                                                      w_rel_r2l, b_r2l, w_root_r2l, relu, dropout, opts=opts,
                                                      bits_out=bits_out)
        _link_prev(ctx, prev)
        ctx.save_for_backward(*saved)
        return left_new, right_new

    @staticmethod
    def backward(ctx, g_left, g_right):
        if ctx.f16:
            raise RuntimeError("lpgnn: fp16 is the reference's inference mode (val.py:269); train in fp32 or bf16")
        return _backward_core(ctx, ctx.saved_tensors, ctx.needs_input_grad, g_left, g_right) + (None, None, None)


def _link_prev(ctx, prev):
    ctx.in_scale, ctx.wgk_prev, ctx.in_bits, ctx.db_prev = None, None, None, None
    if prev is None:
        return
    if prev.bf16:
        ctx.in_scale = prev.scale
        ctx.in_bits = getattr(prev, "out_bits", None)  # (bits of left, bits of right) or None
        prev.out_folded = True
        # a hidden layer (not conv1, whose backward sums dZ with its small-K weight gradients): its bias
        # gradients come out of this layer's folded input-gradient stores (lpg_fc_bf16_relu_bwd*_db)
        ctx.db_prev = None if getattr(prev, "narrow", True) or not ctx.opts.fold_bias_sums else prev
    else:
        ctx.wgk_prev = prev
        prev.wgk_folded = True


def _backward_core(ctx, saved, need, g_left, g_right, dz=None):
    """The layer's backward from its output gradients (g_left, g_right), or --
    dz = (dz_l, db_r2l, dz_r, db_l2r) -- from gradients that already went
    through its ReLU/dropout (the fused heads' backward)."""
    left, right, agg_l, agg_r, left_new, right_new, w_rel_l2r, w_root_l2r, w_rel_r2l, w_root_r2l = saved
    A, AT = ctx.adj.fwd, ctx.adj.bwd
    bf16 = ctx.bf16
    dt = torch.bfloat16 if bf16 else torch.float32
    opts = ctx.opts
    spmm_forward = functools.partial(_spmm_forward, heavy=opts.spmm_heavy)  # noqa: F811 (the model's options)
    pre = getattr(ctx, "folded_wgk", None)
    if getattr(ctx, "wgk_folded", False) and pre is not None:
        # conv1 whose weight gradients the next layer computed in its input-gradient GEMMs
        ctx.folded_wgk = None
        (dw_rel_l2r, dw_root_l2r, db_l2r), (dw_rel_r2l, dw_root_r2l, db_r2l) = pre
        keep = lambda t, i, has=True: t if (need[i] and has) else None  # noqa: E731
        return (None, None, None, keep(dw_rel_l2r, 3), keep(db_l2r, 4, ctx.has_b[0]), keep(dw_root_l2r, 5),
                keep(dw_rel_r2l, 6), keep(db_r2l, 7, ctx.has_b[1]), keep(dw_root_r2l, 8), None, None)

    def mask(g, y, want_db):
        if g is None:
            g = torch.zeros_like(y)
        if getattr(ctx, "out_folded", False):  # the next layer's input-gradient store applied our ReLU backward
            g = g.to(dt).contiguous()
            if not want_db:
                return g, None
            # the bf16 heads' backward (fc.heads_bwd_bf16) or the next layer's folded input-gradient store
            # (lpg_fc_bf16_relu_bwd*_db) already summed these columns: the bits of colsum_bf16
            pre = (getattr(ctx, "folded_colsum", None) or {}).pop(y.data_ptr(), None)
            return g, (pre[1] if pre is not None and pre[0] is g else _fc.colsum_bf16(g))
        if not ctx.relu:
            g = g.to(dt).contiguous()
            return g, (g.float().sum(0) if want_db else None)
        if bf16:
            return _fc.relu_bwd_colsum_bf16(g, y, ctx.scale, want_db)
        return _fc.relu_bwd_colsum(g.contiguous(), y, ctx.scale, want_db)

    small = (dz is None and ctx.relu and agg_r is not None and agg_l is not None
             and agg_r.shape[1] + right.shape[1] <= 16 and agg_l.shape[1] + left.shape[1] <= 16
             and right_new.shape[1] % 4 == 0 and left_new.shape[1] % 4 == 0)
    if small and not (need[0] or need[1]):
        # conv1: the inputs are features -- weight and bias gradients straight from (g, y); bf16: from
        # dZ itself when the next layer's input-gradient store already applied the ReLU backward
        g_r0 = torch.zeros_like(right_new) if g_right is None else g_right
        g_l0 = torch.zeros_like(left_new) if g_left is None else g_left
        if bf16:
            folded = getattr(ctx, "out_folded", False)
            wk = lambda g, y, a, x, wb: _fc.relu_wgrad_smallk_bf16(g, None if folded else y, ctx.scale, a, x, wb)
        else:
            wk = lambda g, y, a, x, wb: _fc.relu_wgrad_smallk(g, y, ctx.scale, a, x, wb)
        dw_rel_l2r, dw_root_l2r, db_l2r = wk(g_r0, right_new, agg_r, right, ctx.has_b[0] and need[4])
        dw_rel_r2l, dw_root_r2l, db_r2l = wk(g_l0, left_new, agg_l, left, ctx.has_b[1] and need[7])
        keep = lambda t, i: t if need[i] else None
        return (None, None, None, keep(dw_rel_l2r, 3), db_l2r, keep(dw_root_l2r, 5), keep(dw_rel_r2l, 6), db_r2l,
                keep(dw_root_r2l, 8), None, None)

    if dz is None:
        dz_r, db_l2r = mask(g_right, right_new, ctx.has_b[0] and need[4])
        dz_l, db_r2l = mask(g_left, left_new, ctx.has_b[1] and need[7])
    else:
        dz_l, db_r2l, dz_r, db_l2r = dz
    main = torch.cuda.current_stream(dz_r.device)
    side = _side_stream(dz_r.device) if opts.overlap else None
    esz = 2 if bf16 else 4

    # Per direction (S = dst x src): T = S^T dZ serves the source-side gradient T W_rel when
    # that association is cheaper, and lin_rel's weight gradient T^T x_src when the source
    # side is the smaller node set (or the forward was re-associated and kept no S x_src).
    # T only needs dZ -- on the side stream it streams HBM under the weight-gradient GEMMs.
    def plan(S, St, dz, x_src, w_rel, agg, need_src, need_rel):
        t_src = need_src and _src_first(S, dz.shape[1], w_rel.shape[1], esz)
        rel_t = need_rel and (agg is None or (t_src and S.n_cols < S.n_rows))
        T = None
        if t_src or rel_t:
            if side is not None:
                side.wait_stream(main)
                with torch.cuda.stream(side):
                    T = spmm_forward(St, dz)
            else:
                T = spmm_forward(St, dz)
        return T, t_src, rel_t

    t_r, tsrc_r, relt_r = plan(AT, A, dz_r, left, w_rel_l2r, agg_r, need[0], need[3])
    t_l, tsrc_l, relt_l = plan(A, AT, dz_l, right, w_rel_r2l, agg_l, need[1], need[6])

    # fp32: the x3 kernels (weight gradient G^T X, input gradient G W) unless LPGNN_FC_ARITH=fp32;
    # bf16: lpg_wgrad_bf16 (fp32 weight gradients) and lpg_fc_bf16 on the transposed weights
    wg = _fc.wgrad_bf16 if bf16 else functools.partial(_fc.wgrad, arith=opts.arith)
    ig = _fc.input_grad_bf16 if bf16 else functools.partial(_fc.input_grad, arith=opts.arith)

    def wgrads(dz, agg, x_dst, need_rel, need_root):
        if not (need_rel or need_root):
            return None, None
        k = x_dst.shape[1] + (agg.shape[1] if agg is not None else 0)
        if not bf16 and agg is not None and k <= 16 and dz.shape[1] % 4 == 0:  # conv1: dZ read once
            d_rel, d_root = _fc.wgrad_smallk(dz, agg, x_dst)
        else:
            d_rel = wg(dz, agg) if need_rel else None
            d_root = wg(dz, x_dst) if need_root else None
        return (d_rel if need_rel else None), (d_root if need_root else None)

    dw_rel_l2r, dw_root_l2r = wgrads(dz_r, agg_r, right, need[3] and not relt_r, need[5])
    dw_rel_r2l, dw_root_r2l = wgrads(dz_l, agg_l, left, need[6] and not relt_l, need[8])
    if side is not None and (t_r is not None or t_l is not None):
        main.wait_stream(side)
        for t in (t_r, t_l):
            if t is not None:
                t.record_stream(main)
    if relt_r:
        dw_rel_l2r = wg(t_r, left)
    if relt_l:
        dw_rel_r2l = wg(t_l, right)

    in_scale = getattr(ctx, "in_scale", None) if bf16 else None
    in_bits = getattr(ctx, "in_bits", None) if bf16 else None
    db_prev = getattr(ctx, "db_prev", None) if bf16 else None
    ctx.in_bits = ctx.db_prev = None
    # fp32: conv1 produced (left, right) and feeds only this layer -- its weight gradients come out of
    # this layer's input-gradient GEMMs (prev = conv1's node; its saved inputs, aggregates and outputs)
    prev = getattr(ctx, "wgk_prev", None)
    ctx.wgk_prev = None
    p_saved = prev.saved_tensors if prev is not None and (need[0] or need[1]) else None

    def src_root_grad(St, dz, w_rel, T, t_src, dz_root, w_root, x_in, conv1=None, bits=None, has_b=False):
        """S^T (dZ W_rel) in the cheaper association + dZ_root W_root (the input's two gradients);
        with a folded previous layer, through its ReLU/dropout backward (x_in = its output) -- and,
        has_b, that layer's bias gradient from the same stores, handed to its node (folded_colsum).
        conv1 = (Y, X1, X2) of the conv1 direction whose output x_in is: returns that direction's
        weight gradients (dW_rel, dW_root, db) instead, the gradient itself never stored."""
        if conv1 is not None:
            y, x1, x2 = conv1
            if t_src:
                r = _fc.input_grad_relu_wgrad(T, w_rel, dz_root, w_root, None, y, x1, x2, arith=opts.arith)
            else:
                r = _fc.input_grad_relu_wgrad(dz_root, w_root, None, None, spmm_forward(St, ig(dz, w_rel)), y, x1,
                                              x2, arith=opts.arith)
            if r is not None:
                return r
            g = src_root_grad(St, dz, w_rel, T, t_src, dz_root, w_root, x_in)  # the two-pass route
            return _fc.relu_wgrad_smallk(g, y, 1.0, x1, x2, True)
        kw = {} if in_scale is None else {"mask": (x_in if bits is None else bits, in_scale)}
        db = None
        if kw and db_prev is not None and has_b:
            db = kw["db_out"] = torch.empty(x_in.shape[1], dtype=torch.float32, device=x_in.device)
        if t_src:  # both terms over the same rows: one two-part GEMM
            g = ig(T, w_rel, dz_root, w_root, **kw)
        else:
            g = ig(dz_root, w_root, out=spmm_forward(St, ig(dz, w_rel)), accumulate=True, **kw)
        if db is not None:  # keyed by the layer output's storage, checked by identity (`pre[0] is g`)
            if getattr(db_prev, "folded_colsum", None) is None:
                db_prev.folded_colsum = {}
            db_prev.folded_colsum[x_in.data_ptr()] = (g, db)
        return g

    g_l = g_r = None
    if p_saved is not None:
        p_left, p_right, p_agg_l, p_agg_r, p_left_new, p_right_new = p_saved[:6]
        # right = conv1's left2right output (Y, from A^T x_s and x_t); left = its right2left output
        wk_r = src_root_grad(AT, dz_l, w_rel_r2l, t_l, tsrc_l, dz_r, w_root_l2r, right,
                             conv1=(p_right_new, p_agg_r, p_right))
        wk_l = src_root_grad(A, dz_r, w_rel_l2r, t_r, tsrc_r, dz_l, w_root_r2l, left,
                             conv1=(p_left_new, p_agg_l, p_left))
        prev.folded_wgk = (wk_r, wk_l)
        # conv1's node still runs (it returns the gradients handed to it): its incoming gradients carry
        # no values -- zero-stride views, no memory
        g_r = torch.zeros((), dtype=right.dtype, device=right.device).expand(right.shape)
        g_l = torch.zeros((), dtype=left.dtype, device=left.device).expand(left.shape)
    else:
        if need[1]:  # right = src of right2left (S = A), dst of left2right
            g_r = src_root_grad(AT, dz_l, w_rel_r2l, t_l, tsrc_l, dz_r, w_root_l2r, right,
                                bits=None if in_bits is None else in_bits[1],
                                has_b=db_prev is not None and db_prev.has_b[0])
        if need[0]:  # left = src of left2right (S = A^T), dst of right2left
            g_l = src_root_grad(A, dz_r, w_rel_l2r, t_r, tsrc_r, dz_l, w_root_r2l, left,
                                bits=None if in_bits is None else in_bits[0],
                                has_b=db_prev is not None and db_prev.has_b[1])
    return (g_l, g_r, None, dw_rel_l2r, db_l2r, dw_root_l2r, dw_rel_r2l, db_r2l, dw_root_r2l, None, None)


class _TwoDirectionHeads(torch.autograd.Function):
    """The last hidden layer and the heads (arch.py:184-190) as one node: the
    hidden outputs feed only lin_left / lin_right, so the heads' backward and
    the layer's ReLU/dropout backward (+ its bias column sums) are one pass
    over the layer output (lpg_heads_relu_bwd_f32) instead of two (the heads'
    dH, then relu_bwd_colsum re-reading dH and Y).  fp32, ReLU layers only."""

    @staticmethod
    def forward(ctx, left, right, adj, w_rel_l2r, b_l2r, w_root_l2r, w_rel_r2l, b_r2l, w_root_r2l, relu, dropout,
                wh_l, bh_l, wh_r, bh_r, heads_only=False, prev=None, opts=DEFAULT):
        # the heads fused into the layer's FC epilogues (x3 arithmetic), else their own Linear kernels
        left_new, right_new, saved, logits = _forward_core(
            ctx, left, right, adj, w_rel_l2r, b_l2r, w_root_l2r, w_rel_r2l, b_r2l, w_root_r2l, relu, dropout,
            heads=((wh_l, bh_l), (wh_r, bh_r)) if opts.fuse_head_fwd else None, heads_only=heads_only, opts=opts)
        if logits is None:
            logits = (_fc.fc_forward(left_new, wh_l, None, None, bh_l, False, arith=opts.arith),
                      _fc.fc_forward(right_new, wh_r, None, None, bh_r, False, arith=opts.arith))
        logit_l, logit_r = logits
        ctx.heads_b = (bh_l is not None, bh_r is not None)
        _link_prev(ctx, prev)
        ctx.save_for_backward(*saved, wh_l, wh_r)
        return logit_l, logit_r

    @staticmethod
    def backward(ctx, g_ll, g_lr):
        *saved, wh_l, wh_r = ctx.saved_tensors
        need = ctx.needs_input_grad
        left_new, right_new = saved[4], saved[5]
        g_ll = torch.zeros(left_new.shape[0], wh_l.shape[0], device=left_new.device) if g_ll is None else g_ll
        g_lr = torch.zeros(right_new.shape[0], wh_r.shape[0], device=right_new.device) if g_lr is None else g_lr
        ar = ctx.opts.arith  # dZ is only read below: its f16x2 scales come out of the same pass
        dz_l, dwh_l, dbh_l, db_r2l = _fc.heads_relu_bwd(g_ll, wh_l, left_new, ctx.scale, ctx.has_b[1] and need[7],
                                                        arith=ar)
        dz_r, dwh_r, dbh_r, db_l2r = _fc.heads_relu_bwd(g_lr, wh_r, right_new, ctx.scale, ctx.has_b[0] and need[4],
                                                        arith=ar)
        core = _backward_core(ctx, saved, need, None, None, dz=(dz_l, db_r2l, dz_r, db_l2r))
        keep = lambda t, i, has=True: t if (need[i] and has) else None
        return (*core, keep(dwh_l, 11), keep(dbh_l, 12, ctx.heads_b[0]), keep(dwh_r, 13),
                keep(dbh_r, 14, ctx.heads_b[1]), None, None, None)


def two_direction_heads(left: Tensor, right: Tensor, adj: BipartiteCSR, left2right, right2left, lin_left, lin_right,
                        dropout: float = 0.0, fold_in: bool = False, opts: PathOptions = DEFAULT):
    """GraphConvTwoDirection (ReLU, dropout) followed by the heads lin_left /
    lin_right (arch.py:184-190) through one autograd node: (logit_l, logit_r).  ``fold_in`` as
    two_direction's."""
    ts = (left, right, left2right.lin_rel.weight, left2right.lin_rel.bias, left2right.lin_root.weight,
          right2left.lin_rel.weight, right2left.lin_rel.bias, right2left.lin_root.weight, lin_left.weight,
          lin_left.bias, lin_right.weight, lin_right.bias)
    # nothing will differentiate through this call: the layer output (which feeds only the heads) is not needed
    heads_only = not (torch.is_grad_enabled() and any(t is not None and t.requires_grad for t in ts))
    prev = _fold_prev(left, right, fold_in, opts)
    return _TwoDirectionHeads.apply(left, right, adj, left2right.lin_rel.weight, left2right.lin_rel.bias,
                                    left2right.lin_root.weight, right2left.lin_rel.weight, right2left.lin_rel.bias,
                                    right2left.lin_root.weight, True, float(dropout), lin_left.weight,
                                    lin_left.bias, lin_right.weight, lin_right.bias, heads_only, prev, opts)


def foldable_producer(x: Tensor, opts: PathOptions = DEFAULT):
    """The backward node of the layer (_TwoDirection) that produced x, if a consumer may fold part of
    its backward into its own: a bf16 ReLU layer (its ReLU/dropout backward into the consumer's
    input-gradient stores, options.fold_relu_bwd) or fp32 conv1 (its weight gradients into the
    consumer's x3 input-gradient GEMMs, options.fold_conv1_wgrad); else None."""
    g = x.grad_fn
    if g is None or not isinstance(g, _TwoDirection._backward_cls) or not getattr(g, "relu", False):
        return None
    if getattr(g, "bf16", False):
        return g if opts.fold_relu_bwd and x.dtype == torch.bfloat16 else None
    # conv1's folded backward returns no input gradients and hands its outputs zero-stride gradients:
    # only when nothing differentiates through its inputs (features without requires_grad) or
    # observes its outputs' gradients (a hook / retain_grad on them) -- else the two-pass route
    if opts.fold_conv1_wgrad and opts.arith in _fc.X3LIKE and getattr(g, "small_relu", False) and \
            x.dtype == torch.float32 and g.opts.arith in _fc.X3LIKE and not any(g.needs_input_grad[:2]) and \
            not x.retains_grad and not x._backward_hooks:
        return g
    return None


def _fold_prev(left: Tensor, right: Tensor, fold_in: bool, opts: PathOptions):
    if not (fold_in and torch.is_grad_enabled()):
        return None
    prev = foldable_producer(left, opts)
    return prev if prev is not None and prev is right.grad_fn else None


def two_direction(left: Tensor, right: Tensor, adj: BipartiteCSR, left2right, right2left, relu: bool = False,
                  dropout: float = 0.0, fold_in: bool = False, opts: PathOptions = DEFAULT, feeds_conv: bool = False):
    """GraphConvTwoDirection.forward (arch.py:65-81) through one autograd node.  ``fold_in``: the
    caller guarantees (left, right) feed nothing but this layer (GCN_FC's layer chain) -- if they
    are a bf16 ReLU layer's outputs, that layer's ReLU/dropout backward is folded into this one's
    input-gradient stores; if they are fp32 conv1's, conv1's weight gradients come out of this
    layer's input-gradient GEMMs.  ``feeds_conv``: the outputs feed the next GraphConvTwoDirection
    layer (so a bf16 ReLU layer writes the 1-bit masks that layer's folded backward reads)."""
    prev = _fold_prev(left, right, fold_in, opts)
    return _TwoDirection.apply(left, right, adj, left2right.lin_rel.weight, left2right.lin_rel.bias,
                               left2right.lin_root.weight, right2left.lin_rel.weight, right2left.lin_rel.bias,
                               right2left.lin_root.weight, bool(relu), float(dropout), prev, opts,
                               bool(feeds_conv and torch.is_grad_enabled()))
