"""Dense per-node FC of GraphConv and the add_knowledge epilogue, on the
hand-written fp32 MFMA kernels of liblpgnn_hip.so.

``graph_conv_fc`` computes, for one GraphConv direction (PyG 2.1
GraphConv.forward after propagate, arch.py:57-62 / 75-80):

    out = lin_rel(agg) + lin_root(x_dst)  [+ ReLU, arch.py:182/188]
        = agg @ W_rel^T + b_rel + x_dst @ W_root^T

in ONE kernel (lpg_fc_f32: no concat, no separate add / ReLU pass), and
``linear`` the heads lin_left / lin_right (arch.py:190).  ``knowledge`` is
arch.py:129-141 for one side (lpg_knowledge_f32).

Forward numerics are bitwise reproducible (oracle/fc_ref.c).  Training-mode
dropout (arch.py:186-187) is fused into the FC epilogue with a counter-based
RNG seeded from torch's generator.  Backward: dZ = (Y > 0) ? dY/(1-p) : 0 in
one pass (lpg_relu_dropout_bwd_f32); dA = dZ W and dW = dZ^T A on the x3
kernels (fp32) or lpg_fc_bf16 / lpg_wgrad_bf16 (bf16, c5), the library GEMMs
only with LPGNN_FC_ARITH=fp32; db = sum(dZ); the heads' backward (N = 3)
runs in lpg_linear_small_bwd_f32.  Tolerance-level parity for gradients.
"""
from __future__ import annotations

import ctypes
import weakref


import torch
import torch.nn.functional as F
from torch import Tensor

from . import _lib
from .options import DEFAULT as _DEFAULT_OPTIONS
from .timing import TIMER


def _prep(t: Tensor | None) -> Tensor | None:
    if t is None:
        return None
    if t.dtype != torch.float32:
        raise RuntimeError(f"lpgnn FC: fp32 only, got {t.dtype}")
    if t.stride(-1) != 1 or t.stride(0) % 4 or t.data_ptr() % 16:
        t = t.contiguous()
    return t


def _pad_k(t: Tensor, mult: int = 4) -> Tensor:
    """Zero-pad the reduction dim to a multiple of `mult` (zeros are exact
    no-ops in the fma chain: the accumulator is never -0)."""
    k = t.shape[1]
    return t if k % mult == 0 else F.pad(t, (0, mult - k % mult))


# fp32 FC arithmetic: "fp32" = the exact fp32 MFMA kernel (bitwise contract of oracle/fc_ref.c),
# "x3" = fp32 on the bf16 matrix cores through the exact three-way bf16 split (lpg_fc_x3_f32, lpg_wgrad_x3_f32).
# The default of calls that pass no ``arith``; a model passes its own (GCN_FC(options=...), lpgnn.options).
ARITH = _DEFAULT_OPTIONS.arith
# "f16x2" (the default) = the same kernels' fp16 form: two fp16 terms per operand after a power-of-2 row
# (weight gradient: column) scale, three products (lpg_fc_f16x2_*, lpg_wgrad_f16x2_f32: half the
# matrix-core work, representation error a quarter of an fp32 SGEMM's); where it does not apply (operands
# the wide kernel does not take) the call runs x3
X3LIKE = ("x3", "f16x2")

_FC_BK = 32  # lpg_fc_f32's tiled k-tile: K1, K2 are zero-padded to it unless the narrow-input kernel applies


def fc_forward(A1: Tensor, W1: Tensor, A2: Tensor | None, W2: Tensor | None, bias: Tensor | None,
               relu: bool, dropout_p: float = 0.0, seed: int = 0, out: Tensor | None = None,
               accumulate: bool = False, arith: str | None = None, heads=None, kernel: int = 0,
               row_offset: int = 0, heads_only: bool = False, row_keys: Tensor | None = None):
    """act(A1 W1^T + A2 W2^T [+ out] + bias) through lpg_fc_f32; with
    ``accumulate`` the caller's ``out`` holds the addend and is overwritten.
    ``arith`` ("fp32" | "x3", default ``ARITH``) picks the tiled kernel's arithmetic.
    ``heads`` = (Wh [<= 4, N], bh or None): also return the logits C Wh^T + bh
    -- fused into the x3 kernel's epilogue (lpg_fc_x3_heads_f32), else the
    separate Linear on C (the fp32 contract's own kernel).  ``kernel``: the x3 entries' per-call
    kernel choice (LPG_FC_KERNEL, include/lpgnn.h; 0 = by shape; every choice gives the same bits).
    ``row_offset``: the dropout mask keys row m as row_offset + m (the global node id of the first
    row when this call computes a slice of a node set: the row partition); ``row_keys`` (int64 [M] on
    the device) keys row m as row_keys[m] instead -- the global ids of rows that are not one
    contiguous range (a general partition's owned variables)).
    ``heads_only`` (with ``heads``): C is not needed -- the fused x3 kernel then does not write it
    (LPG_FC_HEADS_ONLY) and the returned C holds no values (the no-grad forward of the last layer)."""
    if heads is not None:
        M, N = A1.shape[0], W1.shape[0]
        k4 = lambda k: -(-k // 4) * 4
        small = 4 <= k4(A1.shape[1]) and k4(A1.shape[1]) + (0 if A2 is None else k4(A2.shape[1])) <= 16
        if (arith or ARITH) in X3LIKE and not small and N > 32 and heads[0].shape[0] <= 4:
            return _fc_forward(A1, W1, A2, W2, bias, relu, dropout_p, seed, out, accumulate, arith, heads, kernel,
                               row_offset, heads_only, row_keys)
        C = _fc_forward(A1, W1, A2, W2, bias, relu, dropout_p, seed, out, accumulate, arith, kernel=kernel,
                        row_offset=row_offset, row_keys=row_keys)
        return C, _fc_forward(C, heads[0], None, None, heads[1], False, arith=arith)
    return _fc_forward(A1, W1, A2, W2, bias, relu, dropout_p, seed, out, accumulate, arith, kernel=kernel,
                       row_offset=row_offset, row_keys=row_keys)


def _keys(row_keys: Tensor | None, M: int, dev) -> Tensor | None:
    """The per-row dropout keys as the kernels take them (int64 [M], contiguous, on the device)."""
    if row_keys is None:
        return None
    if row_keys.dtype != torch.int64 or row_keys.shape != (M,) or row_keys.device != dev:
        raise RuntimeError(f"lpgnn FC: row_keys must be int64 [{M}] on {dev}")
    return row_keys.contiguous()


def _fc_forward(A1, W1, A2, W2, bias, relu, dropout_p=0.0, seed=0, out=None, accumulate=False, arith=None,
                heads=None, kernel=0, row_offset=0, heads_only=False, row_keys=None):
    if A1.device.type != "cuda":
        raise RuntimeError("lpgnn: the GCN_FC hot path runs on a HIP device only (no CPU path)")
    M, N = A1.shape[0], W1.shape[0]
    row_keys = _keys(row_keys, M, A1.device)
    k4 = lambda k: -(-k // 4) * 4
    K1_4, K2_4 = k4(A1.shape[1]), (0 if A2 is None else k4(A2.shape[1]))
    small = 4 <= K1_4 and K1_4 + K2_4 <= 16 and N % 4 == 0 and (out is None or (
        out.stride(0) % 4 == 0 and out.data_ptr() % 16 == 0))
    mult = 4 if small else _FC_BK
    if A1.shape[1] % mult:
        A1, W1 = _pad_k(A1, mult), _pad_k(W1, mult)
    if A2 is not None and A2.shape[1] % mult:
        A2, W2 = _pad_k(A2, mult), _pad_k(W2, mult)
    A1, W1, A2, W2 = _prep(A1), _prep(W1), _prep(A2), _prep(W2)
    bias = None if bias is None else bias.contiguous()
    if out is not None:  # caller-provided rows (e.g. the owned rows of a partition's [owned | halo] buffer)
        if out.shape != (M, N) or out.dtype != torch.float32 or out.stride(1) != 1 or out.device != A1.device:
            raise RuntimeError("lpgnn FC: `out` must be a float32 [M, N] row-major view on the same device")
        C = out
        _SCALES.forget(out)  # (rewritten through its pointer below: no version bump)
    elif accumulate:
        raise RuntimeError("lpgnn FC: accumulate needs the addend in `out`")
    else:
        C = torch.empty((M, N), dtype=torch.float32, device=A1.device)
    K2 = 0 if A2 is None else A2.shape[1]
    L = _lib.lib()
    flags = (1 if relu else 0) | (2 if accumulate else 0)
    if (arith or ARITH) in X3LIKE and not small and N > 32:
        if heads is not None and heads_only:
            flags |= 4  # LPG_FC_HEADS_ONLY
        return _fc_x3(M, N, A1, W1, A2, W2, K2, bias, C, flags | _lib.fc_kernel(kernel), dropout_p, seed, relu,
                      heads=heads, row_offset=row_offset, row_keys=row_keys, f16=(arith or ARITH) == "f16x2")
    if (small and (arith or ARITH) == "f16x2" and out is None and not accumulate and dropout_p == 0
            and row_keys is None and 0 < N <= 1024 and M > 0):
        # conv1 (narrow LP features) feeding f16x2 GEMMs: C's row / column scales from its own stores
        # (lpg_fc_smallk_scales_f32), cached for it -- C is fresh, so nothing rewrites it behind autograd
        rs = torch.empty(M, dtype=torch.float32, device=A1.device)
        cs = torch.empty(N, dtype=torch.float32, device=A1.device)
        sws = torch.empty(max(16, L.lpg_fc_smallk_scales_workspace_bytes(M, N)) // 4, dtype=torch.float32,
                          device=A1.device)
        with torch.cuda.device(A1.device):
            tok = TIMER.start(("fc", M, N, A1.shape[1] + K2, "relu" if relu else "lin"))
            st = L.lpg_fc_smallk_scales_f32(M, N, A1.shape[1], A1.data_ptr(), A1.stride(0), W1.data_ptr(),
                                            W1.stride(0), K2, None if A2 is None else A2.data_ptr(),
                                            A2.stride(0) if K2 else 0, None if W2 is None else W2.data_ptr(),
                                            W2.stride(0) if K2 else 0, None if bias is None else bias.data_ptr(),
                                            C.data_ptr(), C.stride(0), 1 if relu else 0, rs.data_ptr(),
                                            cs.data_ptr(), sws.data_ptr(), _lib.stream_of(A1))
            TIMER.stop(tok)
        if st != 3:  # (LPG_ERR_UNSUPPORTED: the plain entry below)
            _lib.check(st, "lpg_fc_smallk_scales_f32")
            _SCALES.put("row", C, rs)
            _SCALES.put("col", C, cs)
            return C
    with torch.cuda.device(A1.device):
        tok = TIMER.start(("fc", M, N, A1.shape[1] + K2, "relu" if relu else "lin"))
        st = L.lpg_fc_f32(M, N, A1.shape[1], A1.data_ptr(), A1.stride(0), W1.data_ptr(), W1.stride(0),
                          K2, None if A2 is None else A2.data_ptr(), A2.stride(0) if K2 else 0,
                          None if W2 is None else W2.data_ptr(), W2.stride(0) if K2 else 0,
                          None if bias is None else bias.data_ptr(), C.data_ptr(), C.stride(0), flags,
                          float(dropout_p), int(seed) & (2**64 - 1), int(row_offset), _lib.ptr(row_keys),
                          _lib.stream_of(A1))
        TIMER.stop(tok)
    _lib.check(st, "lpg_fc_f32")
    return C


def split3(W: Tensor, transpose: bool = False) -> Tensor:
    """The exact three-way bf16 split of an fp32 matrix (lpg_split3_f32):
    int16 [3, R, C] holding the bf16 terms t0 + t1 + t2 = S exactly, S = W or
    W^T; C padded to a multiple of 8 (zero terms)."""
    W = W.detach()
    if W.dtype != torch.float32:
        raise RuntimeError(f"lpgnn split3: fp32 only, got {W.dtype}")
    if W.stride(-1) != 1:
        W = W.contiguous()
    R, Cc = (W.shape[1], W.shape[0]) if transpose else W.shape
    ld = -(-Cc // 8) * 8
    out = torch.zeros((3, R, ld), dtype=torch.int16, device=W.device) if ld != Cc else \
        torch.empty((3, R, ld), dtype=torch.int16, device=W.device)
    with torch.cuda.device(W.device):
        st = _lib.lib().lpg_split3_f32(R, Cc, W.data_ptr(), W.stride(0), 1 if transpose else 0, out.data_ptr(),
                                       ld, R * ld, _lib.stream_of(W))
    _lib.check(st, "lpg_split3_f32")
    return out


class _ScaleCache:
    """The f16x2 row / column scales of live operands, by storage region and autograd version: the key
    is the tensor's base (a view's ``_base``, held only by a weak reference) with the view's offset,
    shape and strides, so an operand several GEMMs of one step use -- a layer input in the forward lin
    and the constraint-side FC, dZ or a layer input in two weight gradients, a partition's owned rows
    sliced afresh at each use -- is swept once.  A freed base drops its entries, and an in-place change
    bumps the version (shared by a base and its views), so an entry never outlives the values it
    describes."""

    def __init__(self):
        self._d = {}

    @staticmethod
    def _key(kind: str, t: Tensor):
        base = t._base if t._base is not None else t
        return base, (kind, id(base), t.storage_offset(), tuple(t.shape), tuple(t.stride()))

    def lookup(self, kind: str, t: Tensor):
        if t.is_inference():  # an inference-mode tensor has no version counter: never cached
            return None
        base, key = self._key(kind, t)
        e = self._d.get(key)
        if e is not None and e[0]() is base and e[1] == t._version and e[2] == base.data_ptr():
            return e[3]
        return None

    def put(self, kind: str, t: Tensor, v):
        if t.is_inference():  # no version counter to key on (torch.inference_mode): computed per use
            return
        if len(self._d) > 64:
            self._d = {k: x for k, x in self._d.items() if x[0]() is not None}
        base, key = self._key(kind, t)
        self._d[key] = (weakref.ref(base), t._version, base.data_ptr(), v)

    def get(self, kind: str, t: Tensor, make):
        v = self.lookup(kind, t)
        if v is None:
            v = make(t)
            self.put(kind, t, v)
        return v

    def forget(self, t: Tensor) -> None:
        """Drop every entry on t's base: its storage was written by a path the autograd version does not
        see (our kernels writing a caller's ``out`` through its pointer, a quiet halo broadcast)."""
        base = t._base if t._base is not None else t
        b = id(base)
        self._d = {k: x for k, x in self._d.items() if k[1] != b}


_SCALES = _ScaleCache()


def _both_ok(t: Tensor) -> bool:
    return (t.dtype == torch.float32 and t.dim() == 2 and t.stride(1) == 1 and t.shape[1] % 4 == 0
            and t.stride(0) % 4 == 0 and t.data_ptr() % 16 == 0 and t.shape[1] > 0)


def _scale(kind: str, t: Tensor) -> Tensor:
    """The cached ``kind`` ("row" / "col") scales of t; a miss on an operand lpg_rowcolscale_f32 accepts
    sweeps it once for both (every f16x2 operand of a training step -- layer inputs, dZ, S^T dZ -- is a
    row-scaled GEMM operand and a column-scaled weight-gradient operand)."""
    v = _SCALES.lookup(kind, t)
    if v is not None:
        return v
    if not _both_ok(t):
        v = (_rowscale1 if kind == "row" else _colscale1)(t)
        _SCALES.put(kind, t, v)
        return v
    R, N = t.shape
    L = _lib.lib()
    rs = torch.empty(R, dtype=torch.float32, device=t.device)
    cs = torch.empty(N, dtype=torch.float32, device=t.device)
    ws = torch.empty(max(4, L.lpg_rowcolscale_workspace_bytes(R, N)) // 4, dtype=torch.float32, device=t.device)
    with torch.cuda.device(t.device):
        st = L.lpg_rowcolscale_f32(R, N, t.data_ptr(), t.stride(0), rs.data_ptr(), cs.data_ptr(), ws.data_ptr(),
                                   _lib.stream_of(t))
    _lib.check(st, "lpg_rowcolscale_f32")
    _SCALES.put("row", t, rs)
    _SCALES.put("col", t, cs)
    return rs if kind == "row" else cs


def _rowscale1(A: Tensor) -> Tensor:
    M = A.shape[0]
    out = torch.empty(M, dtype=torch.float32, device=A.device)
    with torch.cuda.device(A.device):
        st = _lib.lib().lpg_rowscale_f32(M, A.shape[1], A.data_ptr(), A.stride(0), 0, None, 0, out.data_ptr(),
                                         _lib.stream_of(A))
    _lib.check(st, "lpg_rowscale_f32")
    return out


def rowscale(A1: Tensor, A2: Tensor | None = None) -> Tensor:
    """The f16x2 power-of-2 scale of every row of [A1 | A2] (fp32 [M]; lpg_rowscale_f32): the row's largest
    |x| times it lies in [2^14, 2^15) (an all-zero row: 2^115).  Per operand, cached (_ScaleCache, both
    scales of an operand from one sweep: _scale); the scale of the two side by side is the smaller of
    theirs (a power of 2 decreasing in the maximum)."""
    s1 = _scale("row", A1)
    if A2 is None or A2.shape[1] == 0:
        return s1
    return torch.minimum(s1, _scale("row", A2))


def split_f16x2(W1: Tensor, W2: Tensor | None = None, transpose: bool = False):
    """(P1, P2, sw): rows of [W1 | W2] (columns with ``transpose``) times their shared power-of-2 scale sw,
    as two fp16 planes each (int16 [2, R, ld], ld the columns rounded up to 8, zero padded; P2 None without
    W2) -- the weights of the f16x2 kernels (lpg_split_f16x2)."""
    W1 = W1.detach().float()
    W2 = None if W2 is None else W2.detach().float()
    W1 = W1 if W1.stride(-1) == 1 else W1.contiguous()
    W2 = None if W2 is None else (W2 if W2.stride(-1) == 1 else W2.contiguous())
    R = W1.shape[1] if transpose else W1.shape[0]
    c1 = W1.shape[0] if transpose else W1.shape[1]
    c2 = 0 if W2 is None else (W2.shape[0] if transpose else W2.shape[1])
    ld = -(-max(c1, c2) // 8) * 8
    mk = (lambda: torch.zeros((2, R, ld), dtype=torch.int16, device=W1.device)) if (ld != c1 or (c2 and ld != c2)) \
        else (lambda: torch.empty((2, R, ld), dtype=torch.int16, device=W1.device))
    P1 = mk()
    P2 = mk() if W2 is not None else None
    sw = torch.empty(R, dtype=torch.float32, device=W1.device)
    with torch.cuda.device(W1.device):
        st = _lib.lib().lpg_split_f16x2(R, c1, W1.data_ptr(), W1.stride(0), c2, None if W2 is None else W2.data_ptr(),
                                        W2.stride(0) if c2 else 0, 1 if transpose else 0, P1.data_ptr(), ld,
                                        None if P2 is None else P2.data_ptr(), ld, R * ld, sw.data_ptr(),
                                        _lib.stream_of(W1))
    _lib.check(st, "lpg_split_f16x2")
    return P1, P2, sw


def _fc_x3(M, N, A1, W1, A2, W2, K2, bias, C, flags, dropout_p, seed, relu, W1s=None, W2s=None, heads=None,
           row_offset=0, row_keys=None, f16=False, transpose=False):
    """lpg_fc_x3_f32 on fp32 A and pre-split W (split here unless given); with
    ``heads`` = (Wh, bh) lpg_fc_x3_heads_f32, returning (C, logits).  ``f16``: the f16x2 form
    (lpg_fc_f16x2_f32 / _heads_f32) from the fp32 weights W1, W2 (``transpose``: the input-gradient GEMM's
    W^T), falling back to x3 where it does not apply."""
    L = _lib.lib()
    if f16:
        sa = rowscale(A1, A2 if K2 else None)
        P1, P2, sw = split_f16x2(W1, W2 if K2 else None, transpose)
        args = (M, N, A1.shape[1], A1.data_ptr(), A1.stride(0), P1.data_ptr(), P1.stride(1), P1.stride(0), K2,
                None if A2 is None else A2.data_ptr(), A2.stride(0) if K2 else 0,
                None if P2 is None else P2.data_ptr(), P2.stride(1) if K2 else 0, P2.stride(0) if K2 else 0,
                sa.data_ptr(), sw.data_ptr(),
                None if bias is None else bias.data_ptr(), C.data_ptr(), C.stride(0), flags, float(dropout_p),
                int(seed) & (2**64 - 1), int(row_offset), _lib.ptr(row_keys))
        key = ("fc", M, N, A1.shape[1] + K2, ("relu" if relu else "lin") + "-f16x2")
        with torch.cuda.device(A1.device):
            if heads is None:
                tok = TIMER.start(key)
                st = L.lpg_fc_f16x2_f32(*args, _lib.stream_of(A1))
                TIMER.stop(tok)
                if st != 3:  # LPG_ERR_UNSUPPORTED: the x3 form below
                    _lib.check(st, "lpg_fc_f16x2_f32")
                    return C
            else:
                Wh = heads[0].detach().contiguous()
                bh = None if heads[1] is None else heads[1].detach().contiguous()
                if Wh.dtype != torch.float32 or Wh.shape[1] != N:
                    raise RuntimeError("lpgnn fused heads: fp32 head weight [hn, N] expected")
                logits = torch.empty((M, Wh.shape[0]), dtype=torch.float32, device=A1.device)
                ws = torch.empty(max(16, L.lpg_fc_x3_heads_workspace_bytes(M, N)), dtype=torch.uint8,
                                 device=A1.device)
                tok = TIMER.start(key)
                st = L.lpg_fc_f16x2_heads_f32(*args, Wh.shape[0], Wh.data_ptr(), Wh.stride(0),
                                              None if bh is None else bh.data_ptr(), logits.data_ptr(),
                                              logits.stride(0), ws.data_ptr(), _lib.stream_of(A1))
                TIMER.stop(tok)
                if st != 3:
                    _lib.check(st, "lpg_fc_f16x2_heads_f32")
                    return C, logits
    if W1s is None:
        W1s = split3(W1, transpose=transpose)
    if K2 and W2s is None:
        W2s = split3(W2, transpose=transpose)
    W2s = W2s if K2 else None
    args = (M, N, A1.shape[1], A1.data_ptr(), A1.stride(0), W1s.data_ptr(), W1s.stride(1), W1s.stride(0), K2,
            None if A2 is None else A2.data_ptr(), A2.stride(0) if K2 else 0,
            None if W2s is None else W2s.data_ptr(), W2s.stride(1) if K2 else 0, W2s.stride(0) if K2 else 0,
            None if bias is None else bias.data_ptr(), C.data_ptr(), C.stride(0), flags, float(dropout_p),
            int(seed) & (2**64 - 1), int(row_offset), _lib.ptr(row_keys))
    key = ("fc", M, N, A1.shape[1] + K2, ("relu" if relu else "lin") + "-x3")
    with torch.cuda.device(A1.device):
        if heads is None:
            tok = TIMER.start(key)
            st = L.lpg_fc_x3_f32(*args, _lib.stream_of(A1))
            TIMER.stop(tok)
            _lib.check(st, "lpg_fc_x3_f32")
            return C
        Wh = heads[0].detach().contiguous()
        bh = None if heads[1] is None else heads[1].detach().contiguous()
        if Wh.dtype != torch.float32 or Wh.shape[1] != N:
            raise RuntimeError("lpgnn fused heads: fp32 head weight [hn, N] expected")
        logits = torch.empty((M, Wh.shape[0]), dtype=torch.float32, device=A1.device)
        ws = torch.empty(max(16, L.lpg_fc_x3_heads_workspace_bytes(M, N)), dtype=torch.uint8, device=A1.device)
        tok = TIMER.start(key)
        st = L.lpg_fc_x3_heads_f32(*args, Wh.shape[0], Wh.data_ptr(), Wh.stride(0),
                                   None if bh is None else bh.data_ptr(), logits.data_ptr(), logits.stride(0),
                                   ws.data_ptr(), _lib.stream_of(A1))
        TIMER.stop(tok)
    _lib.check(st, "lpg_fc_x3_heads_f32")
    return C, logits


def wgrad(G: Tensor, X: Tensor, arith: str | None = None) -> Tensor:
    """G^T X (the weight gradient dZ^T x of a Linear, [N, K]) in fp32:
    lpg_wgrad_x3_f32 (deterministic split-R reduction) or, with arith
    "fp32", the library GEMM (hipBLASLt)."""
    if (arith or ARITH) not in X3LIKE or G.shape[1] % 4 or X.shape[1] % 4 or G.dtype != torch.float32:
        return G.t() @ X
    if G.device.type != "cuda":
        raise RuntimeError("lpgnn: the GCN_FC hot path runs on a HIP device only (no CPU path)")
    G, X = _prep(G), _prep(X)
    R, N, K = G.shape[0], G.shape[1], X.shape[1]
    L = _lib.lib()
    dW = torch.empty((N, K), dtype=torch.float32, device=G.device)
    ws = torch.empty(max(1, L.lpg_wgrad_x3_workspace_bytes(R, N, K)), dtype=torch.uint8, device=G.device)
    f16 = (arith or ARITH) == "f16x2"
    with torch.cuda.device(G.device):
        if f16:
            sG, sX = colscale(G), colscale(X)
            tok = TIMER.start(("wgrad", R, N, K, "f16x2"))
            st = L.lpg_wgrad_f16x2_f32(R, N, K, G.data_ptr(), G.stride(0), X.data_ptr(), X.stride(0), sG.data_ptr(),
                                       sX.data_ptr(), dW.data_ptr(), dW.stride(0), ws.data_ptr(), _lib.stream_of(G))
        else:
            tok = TIMER.start(("wgrad", R, N, K, "x3"))
            st = L.lpg_wgrad_x3_f32(R, N, K, G.data_ptr(), G.stride(0), X.data_ptr(), X.stride(0), dW.data_ptr(),
                                    dW.stride(0), ws.data_ptr(), _lib.stream_of(G))
        TIMER.stop(tok)
    _lib.check(st, "lpg_wgrad_f16x2_f32" if f16 else "lpg_wgrad_x3_f32")
    return dW


def colscale(G: Tensor) -> Tensor:
    """The f16x2 power-of-2 scale of every column of G [R, N] (fp32 [N]; lpg_colscale_f32): the column's
    largest |x| over the rows times it lies in [2^14, 2^15) (cached per operand with its row scales, _scale)."""
    return _scale("col", G)


def _colscale1(G: Tensor) -> Tensor:
    R, N = G.shape
    L = _lib.lib()
    out = torch.empty(N, dtype=torch.float32, device=G.device)
    ws = torch.empty(max(4, L.lpg_colscale_workspace_bytes(R, N)) // 4, dtype=torch.float32, device=G.device)
    with torch.cuda.device(G.device):
        st = L.lpg_colscale_f32(R, N, G.data_ptr(), G.stride(0), out.data_ptr(), ws.data_ptr(), _lib.stream_of(G))
    _lib.check(st, "lpg_colscale_f32")
    return out


def input_grad(G1: Tensor, W1: Tensor, G2: Tensor | None = None, W2: Tensor | None = None,
               out: Tensor | None = None, accumulate: bool = False, arith: str | None = None) -> Tensor:
    """G1 W1 [+ G2 W2] [+ out] for Linear weights W [out, in] (the input
    gradient of lin_rel / lin_root): the x3 FC kernel with the weights split
    transposed, or the library GEMMs with arith "fp32"."""
    if (arith or ARITH) not in X3LIKE or G1.shape[1] % 32 or (G2 is not None and G2.shape[1] % 32) \
            or W1.shape[1] <= 32 or G1.dtype != torch.float32:
        r = out if accumulate else None
        if r is None:
            r = G1 @ W1
        else:
            r.addmm_(G1, W1)
        if G2 is not None:
            r.addmm_(G2, W2)
        if out is not None and r is not out:
            out.copy_(r)
            r = out
        return r
    if G1.device.type != "cuda":
        raise RuntimeError("lpgnn: the GCN_FC hot path runs on a HIP device only (no CPU path)")
    G1, G2 = _prep(G1), _prep(G2)
    M, N = G1.shape[0], W1.shape[1]
    if out is None:
        if accumulate:
            raise RuntimeError("lpgnn input_grad: accumulate needs the addend in `out`")
        out = torch.empty((M, N), dtype=torch.float32, device=G1.device)
    else:
        _SCALES.forget(out)  # (rewritten through its pointer: no version bump)
    K2 = 0 if G2 is None else G2.shape[1]
    return _fc_x3(M, N, G1, W1, G2, W2, K2, None, out, 2 if accumulate else 0, 0.0, 0, False,
                  f16=(arith or ARITH) == "f16x2", transpose=True)


def input_grad_relu_wgrad(G1: Tensor, W1: Tensor, G2: Tensor | None, W2: Tensor | None, addend: Tensor | None,
                          Y: Tensor, X1: Tensor, X2: Tensor | None, arith: str | None = None):
    """conv1's weight gradients folded into the input-gradient GEMM of the layer it feeds
    (lpg_fc_x3_relu_wgrad_f32): g = G1 W1 [+ G2 W2] [+ addend] is the gradient of conv1's ReLU output
    Y, and instead of g the call returns (dW1 [N, k1] = dZ^T X1, dW2 [N, k2] = dZ^T X2 or None,
    db [N] = sum dZ), dZ = (Y > 0) ? g : 0 (conv1 has no dropout; arch.py:181-182) -- what
    relu_wgrad_smallk computes from the stored g, without storing it.  None when the operands do not
    fit the fused kernel (the caller then takes input_grad + relu_wgrad_smallk).  ``arith`` "f16x2": the
    GEMM in the f16x2 form (lpg_fc_f16x2_relu_wgrad_f32)."""
    k1, k2 = X1.shape[1], (0 if X2 is None else X2.shape[1])
    if (G1.dtype != torch.float32 or G1.shape[1] % 32 or (G2 is not None and G2.shape[1] % 32)
            or W1.shape[1] <= 32 or W1.shape[1] % 2 or not 1 <= k1 + k2 <= 16 or Y.dtype != torch.float32):
        return None
    G1, G2 = _prep(G1), _prep(G2)
    if G2 is not None and G2.stride(0) != G1.stride(0):
        return None
    M, N = G1.shape[0], W1.shape[1]
    f16 = (arith or ARITH) == "f16x2"
    if f16:
        W1s, W2s, sw = split_f16x2(W1, W2 if G2 is not None else None, transpose=True)
        sa = rowscale(G1, G2)
    else:
        W1s = split3(W1, transpose=True)
        W2s = split3(W2, transpose=True) if G2 is not None else None
    if W2s is not None and W2s.shape != W1s.shape:
        return None
    Y = Y if (Y.stride(1) == 1 and Y.stride(0) % 2 == 0 and Y.data_ptr() % 8 == 0) else Y.contiguous()
    X1 = X1.contiguous()
    X2 = None if X2 is None else X2.contiguous()
    if addend is not None and (addend.shape != (M, N) or addend.stride(1) != 1 or addend.dtype != torch.float32
                               or addend.stride(0) % 2 or addend.data_ptr() % 8):
        return None
    L = _lib.lib()
    dW1 = torch.empty((N, k1), dtype=torch.float32, device=G1.device)
    dW2 = torch.empty((N, k2), dtype=torch.float32, device=G1.device) if k2 else None
    db = torch.empty(N, dtype=torch.float32, device=G1.device)
    ws = torch.empty(max(16, L.lpg_fc_x3_relu_wgrad_workspace_bytes(M, N, k1 + k2)) // 4 + 4, dtype=torch.float32,
                     device=G1.device)
    K2 = 0 if G2 is None else G2.shape[1]
    head = (M, N, G1.shape[1], G1.data_ptr(), G1.stride(0), W1s.data_ptr(), W1s.stride(1), W1s.stride(0), K2,
            None if G2 is None else G2.data_ptr(), G2.stride(0) if K2 else 0,
            None if W2s is None else W2s.data_ptr(), W2s.stride(1) if K2 else 0, W2s.stride(0) if K2 else 0)
    tail = (None if addend is None else addend.data_ptr(), N if addend is None else addend.stride(0),
            2 if addend is not None else 0, Y.data_ptr(), Y.stride(0), k1, X1.data_ptr(), X1.stride(0), k2,
            None if X2 is None else X2.data_ptr(), X2.stride(0) if k2 else 0, dW1.data_ptr(),
            None if dW2 is None else dW2.data_ptr(), db.data_ptr(), ws.data_ptr(), _lib.stream_of(G1))
    name = "lpg_fc_f16x2_relu_wgrad_f32" if f16 else "lpg_fc_x3_relu_wgrad_f32"
    with torch.cuda.device(G1.device):
        tok = TIMER.start(("fc", M, N, G1.shape[1] + K2, "wgk-f16x2" if f16 else "wgk-x3"))
        if f16:
            st = L.lpg_fc_f16x2_relu_wgrad_f32(*head, sa.data_ptr(), sw.data_ptr(), *tail)
        else:
            st = L.lpg_fc_x3_relu_wgrad_f32(*head, *tail)
        TIMER.stop(tok)
    _lib.check(st, name)
    return dW1, dW2, db


_BF16_BK = 64  # lpg_fc_bf16's k-tile: K1, K2 are zero-padded to a multiple of it


HALF16 = (torch.bfloat16, torch.float16)  # the 16-bit storage types: bf16 (c5), fp16 (--fp16 inference)


def _prep_bf16(t: Tensor | None, dt=torch.bfloat16) -> Tensor | None:
    if t is None:
        return None
    if t.dtype != dt:
        raise RuntimeError(f"lpgnn 16-bit FC: {dt} operands expected, got {t.dtype}")
    if t.shape[1] % _BF16_BK:
        t = F.pad(t, (0, _BF16_BK - t.shape[1] % _BF16_BK))
    if t.stride(-1) != 1 or t.stride(0) % 8 or t.data_ptr() % 16:
        t = t.contiguous()
    return t


def fc_forward_bf16(A1: Tensor, W1: Tensor, A2: Tensor | None, W2: Tensor | None, bias: Tensor | None,
                    relu: bool, dropout_p: float = 0.0, seed: int = 0, out: Tensor | None = None,
                    accumulate: bool = False, key: str | None = None, mask=None, kernel: int = 0,
                    row_offset: int = 0, row_keys: Tensor | None = None, mask_out: Tensor | None = None,
                    db_out: Tensor | None = None) -> Tensor:
    """The c5 bf16 path: bf16 A/W, fp32 accumulate + fp32 bias, bf16 out (lpg_fc_bf16); with fp16
    operands (the --fp16 inference mode, val.py:269) the same kernels on the fp16 MFMA (lpg_fc_f16);
    ``accumulate`` adds the bf16 addend held in ``out`` (overwritten).
    ``mask`` = (Y, scale): an input gradient with the previous layer's ReLU/dropout backward
    folded into the store, C = (Y > 0) ? bf16(C * scale) : 0 (lpg_fc_bf16_relu_bwd; no bias /
    ReLU / dropout of its own) -- the bits of this call without ``mask`` followed by
    relu_bwd_colsum_bf16(C, Y, scale).  ``kernel``: the per-call kernel choice (LPG_FC_KERNEL,
    include/lpgnn.h; 0 = by shape, 1 = 128 x 128, 2 = 256 x 256, 3 = pipelined; the same bits).
    ``row_offset`` / ``row_keys``: the dropout row keys, as fc_forward.  ``mask_out`` (uint8 [M, N / 8],
    bf16 ReLU calls): filled with the output's 1-bit ReLU mask (bit e of byte t of row m: C[m, 8 t + e] > 0,
    lpg_fc_bf16_mask), which a later ``mask`` = (bits, scale) takes in place of Y (1/16 of its bytes).
    ``db_out`` (fp32 [N], with ``mask``): filled with the column sums of the returned dZ, the bias
    gradient of the layer whose ReLU is folded -- bitwise colsum_bf16(dZ), taken in the FC's store loop
    (lpg_fc_bf16_relu_bwd*_db) instead of a second pass over dZ."""
    if A1.device.type != "cuda":
        raise RuntimeError("lpgnn: the GCN_FC hot path runs on a HIP device only (no CPU path)")
    M, N = A1.shape[0], W1.shape[0]
    row_keys = _keys(row_keys, M, A1.device)
    dt = A1.dtype
    if dt not in HALF16:
        raise RuntimeError(f"lpgnn 16-bit FC: bf16 or fp16 operands expected, got {dt}")
    f16 = dt == torch.float16
    if f16 and mask is not None:
        raise RuntimeError("lpgnn fp16 FC: the folded ReLU backward is a bf16 training path")
    if db_out is not None and (mask is None or db_out.dtype != torch.float32 or db_out.shape != (N,)
                               or not db_out.is_contiguous() or db_out.device != A1.device):
        raise RuntimeError("lpgnn bf16 FC: db_out needs `mask` and an fp32 [N] contiguous tensor on the same device")
    k1, k2 = A1.shape[1], (0 if A2 is None else A2.shape[1])
    # conv1 (narrow LP features): the streaming small-K kernel takes the operands unpadded
    small = (mask is None and 4 <= k1 and k1 + k2 <= 16 and k1 % 4 == 0 and k2 % 4 == 0 and N % 4 == 0
             and (out is None or (out.stride(0) % 4 == 0 and out.data_ptr() % 8 == 0)))
    if small:
        A1, W1 = A1.contiguous(), W1.contiguous()
        A2 = None if A2 is None else A2.contiguous()
        W2 = None if W2 is None else W2.contiguous()
        if any(t is not None and t.dtype != dt for t in (A1, W1, A2, W2)):
            raise RuntimeError(f"lpgnn 16-bit FC: {dt} operands expected")
    else:
        A1, W1, A2, W2 = _prep_bf16(A1, dt), _prep_bf16(W1, dt), _prep_bf16(A2, dt), _prep_bf16(W2, dt)
    bias = None if bias is None else bias.float().contiguous()
    if out is not None:
        if out.shape != (M, N) or out.dtype != dt or out.stride(1) != 1 or out.device != A1.device:
            raise RuntimeError(f"lpgnn 16-bit FC: `out` must be a {dt} [M, N] row-major view on the same device")
        C = out
    elif accumulate:
        raise RuntimeError("lpgnn bf16 FC: accumulate needs the addend in `out`")
    else:
        C = torch.empty((M, N), dtype=dt, device=A1.device)
    K2 = 0 if A2 is None else A2.shape[1]
    L = _lib.lib()
    flags = (1 if relu else 0) | (2 if accumulate else 0) | _lib.fc_kernel(kernel)
    if mask is not None and mask[0].dtype == torch.uint8:  # the previous layer's ReLU as bits
        bits, scale = mask
        if relu or bias is not None or dropout_p > 0:
            raise RuntimeError("lpgnn bf16 FC: the folded ReLU backward takes no bias / ReLU / dropout")
        if (bits.shape != (M, N // 8) or bits.device != A1.device or bits.stride(1) != 1 or N % 8
                or C.stride(0) % 8 or C.data_ptr() % 16):  # the same bits through the Y form
            y = ((bits[:, :, None] >> torch.arange(8, device=bits.device, dtype=torch.uint8)) & 1).reshape(M, -1)
            return fc_forward_bf16(A1, W1, A2, W2, None, False, out=out, accumulate=accumulate, key=key,
                                   mask=(y[:, :N].to(torch.bfloat16), scale), kernel=kernel, db_out=db_out)
        entry = "lpg_fc_bf16_relu_bwd_bits" + ("_db" if db_out is not None else "")
        dargs = _db_args(L, M, N, db_out, A1.device)
        with torch.cuda.device(A1.device):
            tok = TIMER.start(("fc", M, N, A1.shape[1] + K2, key or "lin-bf16-relubwd"))
            st = getattr(L, entry)(M, N, A1.shape[1], A1.data_ptr(), A1.stride(0), W1.data_ptr(),
                                   W1.stride(0), K2, None if A2 is None else A2.data_ptr(),
                                   A2.stride(0) if K2 else 0, None if W2 is None else W2.data_ptr(),
                                   W2.stride(0) if K2 else 0, C.data_ptr(), C.stride(0), flags,
                                   bits.data_ptr(), bits.stride(0), float(scale), *dargs, _lib.stream_of(A1))
            TIMER.stop(tok)
        _lib.check(st, entry)
        return C
    if mask is not None:
        Y, scale = mask
        if relu or bias is not None or dropout_p > 0:
            raise RuntimeError("lpgnn bf16 FC: the folded ReLU backward takes no bias / ReLU / dropout")
        if (Y.shape != (M, N) or Y.dtype != torch.bfloat16 or Y.device != A1.device or Y.stride(1) != 1
                or Y.stride(0) % 8 or Y.data_ptr() % 16 or N % 8 or C.stride(0) % 8 or C.data_ptr() % 16):
            # layouts the folded store does not take: the same bits in two passes
            C = fc_forward_bf16(A1, W1, A2, W2, None, False, out=out, accumulate=accumulate, key=key, kernel=kernel)
            dz = relu_bwd_colsum_bf16(C, Y, scale, False)[0]
            if db_out is not None:
                db_out.copy_(colsum_bf16(dz))
            return dz
        entry = "lpg_fc_bf16_relu_bwd" + ("_db" if db_out is not None else "")
        dargs = _db_args(L, M, N, db_out, A1.device)
        with torch.cuda.device(A1.device):
            tok = TIMER.start(("fc", M, N, A1.shape[1] + K2, key or "lin-bf16-relubwd"))
            st = getattr(L, entry)(M, N, A1.shape[1], A1.data_ptr(), A1.stride(0), W1.data_ptr(), W1.stride(0),
                                   K2, None if A2 is None else A2.data_ptr(), A2.stride(0) if K2 else 0,
                                   None if W2 is None else W2.data_ptr(), W2.stride(0) if K2 else 0,
                                   C.data_ptr(), C.stride(0), flags, Y.data_ptr(), Y.stride(0), float(scale),
                                   *dargs, _lib.stream_of(A1))
            TIMER.stop(tok)
        _lib.check(st, entry)
        return C
    entry = "lpg_fc_f16" if f16 else "lpg_fc_bf16"
    if mask_out is None and not small and kernel == 6:
        # the persistent stream-K form with its workspace (lpg_fc16, choice 6): the same bits, no partial
        # last round -- measured slower than the default (profiles/r05_sk_ab.log), kept as a choice
        call = _lib.LpgFc16Call(
            dtype=1 if f16 else 0, flags=flags, M=M, N=N, K1=A1.shape[1], K2=K2, A1=A1.data_ptr(), W1=W1.data_ptr(),
            A2=None if A2 is None else A2.data_ptr(), W2=None if W2 is None else W2.data_ptr(), lda1=A1.stride(0),
            ldw1=W1.stride(0), lda2=A2.stride(0) if K2 else 0, ldw2=W2.stride(0) if K2 else 0,
            bias=None if bias is None else bias.data_ptr(), C=C.data_ptr(), ldc=C.stride(0),
            dropout_p=float(dropout_p), seed=int(seed) & (2**64 - 1), row_offset=int(row_offset),
            row_keys=_lib.ptr(row_keys), scale=1.0)
        ws = _workspace(L.lpg_fc16_workspace_bytes(), A1.device)
        with torch.cuda.device(A1.device):
            tok = TIMER.start(("fc", M, N, A1.shape[1] + K2,
                               key or (("relu-" if relu else "lin-") + ("f16" if f16 else "bf16"))))
            st = L.lpg_fc16(ctypes.byref(call), ws.data_ptr(), ws.numel() * 4, _lib.stream_of(A1))
            TIMER.stop(tok)
        _lib.check(st, "lpg_fc16")
        return C
    margs = ()
    if mask_out is not None:
        if (f16 or not relu or N % 8 or C.stride(0) % 8 or C.data_ptr() % 16 or mask_out.dtype != torch.uint8
                or mask_out.shape != (M, N // 8) or mask_out.stride(1) != 1 or mask_out.device != A1.device):
            raise RuntimeError("lpgnn bf16 FC: mask_out needs a bf16 ReLU call, N and ldc multiples of 8, an aligned "
                               "C and a uint8 [M, N / 8] row-major mask on the same device")
        entry = "lpg_fc_bf16_mask"
        margs = (mask_out.data_ptr(), mask_out.stride(0))
    with torch.cuda.device(A1.device):
        tok = TIMER.start(("fc", M, N, A1.shape[1] + K2,
                           key or (("relu-" if relu else "lin-") + ("f16" if f16 else "bf16"))))
        st = getattr(L, entry)(M, N, A1.shape[1], A1.data_ptr(), A1.stride(0), W1.data_ptr(), W1.stride(0),
                           K2, None if A2 is None else A2.data_ptr(), A2.stride(0) if K2 else 0,
                           None if W2 is None else W2.data_ptr(), W2.stride(0) if K2 else 0,
                           None if bias is None else bias.data_ptr(), C.data_ptr(), C.stride(0), flags,
                           float(dropout_p), int(seed) & (2**64 - 1), int(row_offset), _lib.ptr(row_keys),
                           *margs, _lib.stream_of(A1))
        TIMER.stop(tok)
    _lib.check(st, entry)
    return C


def _db_args(L, M: int, N: int, db_out: Tensor | None, device) -> tuple:
    """(db, workspace) pointers of the lpg_fc_bf16_relu_bwd*_db entries, () without db_out."""
    if db_out is None:
        return ()
    ws = _workspace(L.lpg_relu_bwd_colsum_workspace_bytes(M, N), device)
    return db_out.data_ptr(), ws.data_ptr()


def wgrad_bf16(G: Tensor, X: Tensor) -> Tensor:
    """G^T X for bf16 G [R, N], X [R, K]: the fp32 weight gradient [N, K] of a
    Linear in the c5 bf16 model (lpg_wgrad_bf16: fp32 accumulation, fp32 out,
    deterministic split-R reduction)."""
    if G.device.type != "cuda":
        raise RuntimeError("lpgnn: the GCN_FC hot path runs on a HIP device only (no CPU path)")
    G, X = G.to(torch.bfloat16), X.to(torch.bfloat16)
    R, N, K = G.shape[0], G.shape[1], X.shape[1]
    pad = lambda t, c: t if c % 8 == 0 else F.pad(t, (0, 8 - c % 8))
    Gp, Xp = pad(G, N), pad(X, K)
    if Gp.stride(1) != 1 or Gp.stride(0) % 8 or Gp.data_ptr() % 16:
        Gp = Gp.contiguous()
    if Xp.stride(1) != 1 or Xp.stride(0) % 8 or Xp.data_ptr() % 16:
        Xp = Xp.contiguous()
    Np, Kp = Gp.shape[1], Xp.shape[1]
    L = _lib.lib()
    dW = torch.empty((Np, Kp), dtype=torch.float32, device=G.device)
    ws = torch.empty(max(16, L.lpg_wgrad_bf16_workspace_bytes(R, Np, Kp)), dtype=torch.uint8, device=G.device)
    with torch.cuda.device(G.device):
        tok = TIMER.start(("wgrad", R, N, K, "bf16"))
        st = L.lpg_wgrad_bf16(R, Np, Kp, Gp.data_ptr(), Gp.stride(0), Xp.data_ptr(), Xp.stride(0), dW.data_ptr(),
                              dW.stride(0), ws.data_ptr(), _lib.stream_of(G))
        TIMER.stop(tok)
    _lib.check(st, "lpg_wgrad_bf16")
    return dW if (Np, Kp) == (N, K) else dW[:N, :K]


def input_grad_bf16(G1: Tensor, W1: Tensor, G2: Tensor | None = None, W2: Tensor | None = None,
                    out: Tensor | None = None, accumulate: bool = False, mask=None, kernel: int = 0,
                    db_out: Tensor | None = None) -> Tensor:
    """G1 W1 [+ G2 W2] [+ out] in bf16 for Linear weights W [out, in]: the
    c5 input gradient of lin_rel / lin_root on the bf16 FC kernel (lpg_fc_bf16
    with the weights transposed; fp32 accumulation, one bf16 rounding).
    ``mask`` = (Y, scale): the previous layer's ReLU/dropout backward folded into the store
    (fc_forward_bf16); ``db_out``: that layer's bias gradient, the column sums of the result."""
    t = lambda W: None if W is None else transpose_bf16(W.detach().to(torch.bfloat16))
    G1 = G1.to(torch.bfloat16)
    G2 = None if G2 is None else G2.to(torch.bfloat16)
    return fc_forward_bf16(G1, t(W1), G2, t(W2), None, False, out=out, accumulate=accumulate, key="igrad-bf16",
                           mask=mask, kernel=kernel, db_out=db_out)


def relu_dropout_bwd(g: Tensor, y: Tensor, scale: float) -> Tensor:
    """(y > 0) ? g * scale : 0 in one pass (ReLU + dropout backward)."""
    g = g.contiguous()
    out = torch.empty_like(g)
    n = g.numel()
    if n % 4 or g.data_ptr() % 16 or y.data_ptr() % 16 or not y.is_contiguous():
        return torch.where(y > 0, g * scale, torch.zeros((), device=g.device))
    with torch.cuda.device(g.device):
        st = _lib.lib().lpg_relu_dropout_bwd_f32(n, g.data_ptr(), y.data_ptr(), float(scale), out.data_ptr(),
                                                 _lib.stream_of(g))
    _lib.check(st, "lpg_relu_dropout_bwd_f32")
    return out


def _workspace(nbytes: int, device) -> Tensor:
    return torch.empty(max(int(nbytes), 16) // 4 + 4, dtype=torch.float32, device=device)


def relu_bwd_colsum(g: Tensor, y: Tensor, scale: float, want_db: bool):
    """(dZ, db): dZ = (y > 0) ? g * scale : 0 and db = dZ.sum(0) in one pass."""
    M, N = g.shape
    g = g if (g.stride(1) == 1 and g.stride(0) % 4 == 0 and g.data_ptr() % 16 == 0) else g.contiguous()
    if N % 4 or y.stride(1) != 1 or y.stride(0) % 4 or y.data_ptr() % 16:
        dz = relu_dropout_bwd(g, y, scale)
        return dz, (dz.sum(0) if want_db else None)
    out = torch.empty((M, N), dtype=torch.float32, device=g.device)
    L = _lib.lib()
    db = torch.empty(N, dtype=torch.float32, device=g.device) if want_db else None
    ws = _workspace(L.lpg_relu_bwd_colsum_workspace_bytes(M, N), g.device) if want_db else None
    with torch.cuda.device(g.device):
        st = L.lpg_relu_bwd_colsum_f32(M, N, g.data_ptr(), g.stride(0), y.data_ptr(), y.stride(0), float(scale),
                                       out.data_ptr(), N, None if db is None else db.data_ptr(),
                                       None if ws is None else ws.data_ptr(), _lib.stream_of(g))
    _lib.check(st, "lpg_relu_bwd_colsum_f32")
    return out, db


def relu_bwd_colsum_bf16(g: Tensor, y: Tensor, scale: float, want_db: bool):
    """bf16 twin of relu_bwd_colsum: (dZ bf16, db fp32) in one pass."""
    M, N = g.shape
    g = g.to(torch.bfloat16)
    if g.stride(1) != 1 or g.stride(0) % 8 or g.data_ptr() % 16:
        g = g.contiguous()
    if N % 8 or y.stride(1) != 1 or y.stride(0) % 8 or y.data_ptr() % 16:
        dz = torch.where(y > 0, g * scale, torch.zeros((), dtype=g.dtype, device=g.device))
        return dz, (dz.float().sum(0) if want_db else None)
    out = torch.empty((M, N), dtype=torch.bfloat16, device=g.device)
    L = _lib.lib()
    db = torch.empty(N, dtype=torch.float32, device=g.device) if want_db else None
    ws = _workspace(L.lpg_relu_bwd_colsum_workspace_bytes(M, N), g.device) if want_db else None
    with torch.cuda.device(g.device):
        st = L.lpg_relu_bwd_colsum_bf16(M, N, g.data_ptr(), g.stride(0), y.data_ptr(), y.stride(0), float(scale),
                                        out.data_ptr(), N, None if db is None else db.data_ptr(),
                                        None if ws is None else ws.data_ptr(), _lib.stream_of(g))
    _lib.check(st, "lpg_relu_bwd_colsum_bf16")
    return out, db


def transpose_bf16(W: Tensor) -> Tensor:
    """W^T as a contiguous bf16 tensor (lpg_transpose_bf16; shapes it does not take: torch)."""
    R, C = W.shape
    if W.dtype != torch.bfloat16 or R % 8 or C % 8 or W.stride(1) != 1 or W.stride(0) % 8 or W.data_ptr() % 16:
        return W.t().to(torch.bfloat16).contiguous()
    out = torch.empty((C, R), dtype=torch.bfloat16, device=W.device)
    with torch.cuda.device(W.device):
        st = _lib.lib().lpg_transpose_bf16(R, C, W.data_ptr(), W.stride(0), out.data_ptr(), R, _lib.stream_of(W))
    _lib.check(st, "lpg_transpose_bf16")
    return out


def colsum_bf16(g: Tensor) -> Tensor:
    """db = g.sum(0) in fp32 for a bf16 dZ that already went through its ReLU/dropout backward
    (lpg_colsum_bf16: the blocks and fold of relu_bwd_colsum_bf16, so the same bits)."""
    M, N = g.shape
    if g.dtype != torch.bfloat16 or N % 8 or g.stride(1) != 1 or g.stride(0) % 8 or g.data_ptr() % 16:
        g = g.to(torch.bfloat16).contiguous()
        if N % 8:
            return g.float().sum(0)
    L = _lib.lib()
    db = torch.empty(N, dtype=torch.float32, device=g.device)
    ws = _workspace(L.lpg_relu_bwd_colsum_workspace_bytes(M, N), g.device)
    with torch.cuda.device(g.device):
        st = L.lpg_colsum_bf16(M, N, g.data_ptr(), g.stride(0), db.data_ptr(), ws.data_ptr(), _lib.stream_of(g))
    _lib.check(st, "lpg_colsum_bf16")
    return db


def wgrad_smallk(dz: Tensor, A1: Tensor, A2: Tensor | None):
    """(dW1, dW2) = (dZ^T A1, dZ^T A2) for narrow inputs (K1 + K2 <= 16)."""
    M, N = dz.shape
    A1 = A1.contiguous()
    A2 = None if A2 is None else A2.contiguous()
    K1, K2 = A1.shape[1], (0 if A2 is None else A2.shape[1])
    L = _lib.lib()
    ws = _workspace(L.lpg_wgrad_smallk_workspace_bytes(M, N, K1 + K2), dz.device)
    dW1 = torch.empty((N, K1), dtype=torch.float32, device=dz.device)
    dW2 = torch.empty((N, K2), dtype=torch.float32, device=dz.device) if K2 else None
    with torch.cuda.device(dz.device):
        st = L.lpg_wgrad_smallk_f32(M, N, dz.data_ptr(), dz.stride(0), K1, A1.data_ptr(), max(K1, 1), K2,
                                    None if A2 is None else A2.data_ptr(), max(K2, 1), dW1.data_ptr(),
                                    None if dW2 is None else dW2.data_ptr(), ws.data_ptr(), _lib.stream_of(dz))
    _lib.check(st, "lpg_wgrad_smallk_f32")
    return dW1, dW2


def relu_wgrad_smallk(g: Tensor, y: Tensor, scale: float, A1: Tensor, A2: Tensor | None, want_db: bool):
    """(dW1, dW2, db) of a narrow-input FC straight from (g, y): the ReLU /
    dropout backward is applied on the fly and dZ is never stored."""
    M, N = g.shape
    g, y = g.contiguous(), y.contiguous()
    A1 = A1.contiguous()
    A2 = None if A2 is None else A2.contiguous()
    K1, K2 = A1.shape[1], (0 if A2 is None else A2.shape[1])
    L = _lib.lib()
    ws = _workspace(L.lpg_wgrad_smallk_workspace_bytes(M, N, K1 + K2), g.device)
    dW1 = torch.empty((N, K1), dtype=torch.float32, device=g.device)
    dW2 = torch.empty((N, K2), dtype=torch.float32, device=g.device) if K2 else None
    db = torch.empty(N, dtype=torch.float32, device=g.device) if want_db else None
    with torch.cuda.device(g.device):
        st = L.lpg_relu_wgrad_smallk_f32(M, N, g.data_ptr(), g.stride(0), y.data_ptr(), y.stride(0), float(scale),
                                         K1, A1.data_ptr(), max(K1, 1), K2, None if A2 is None else A2.data_ptr(),
                                         max(K2, 1), dW1.data_ptr(), None if dW2 is None else dW2.data_ptr(),
                                         None if db is None else db.data_ptr(), ws.data_ptr(), _lib.stream_of(g))
    _lib.check(st, "lpg_relu_wgrad_smallk_f32")
    return dW1, dW2, db


def relu_wgrad_smallk_bf16(g: Tensor, y: Tensor | None, scale: float, A1: Tensor, A2: Tensor | None, want_db: bool):
    """bf16 twin of relu_wgrad_smallk (c5 conv1, lpg_relu_wgrad_smallk_bf16): (dW1, dW2, db) fp32 from one
    read of the gradient.  ``y`` None: g already is dZ (the next layer folded this layer's ReLU /
    dropout backward into its input-gradient store); else dZ = (y > 0) ? bf16(g * scale) : 0 on the fly."""
    M, N = g.shape
    g = g.to(torch.bfloat16).contiguous()
    y = None if y is None else y.contiguous()
    A1 = A1.to(torch.bfloat16).contiguous()
    A2 = None if A2 is None else A2.to(torch.bfloat16).contiguous()
    K1, K2 = A1.shape[1], (0 if A2 is None else A2.shape[1])
    L = _lib.lib()
    ws = _workspace(L.lpg_wgrad_smallk_workspace_bytes(M, N, K1 + K2), g.device)
    dW1 = torch.empty((N, K1), dtype=torch.float32, device=g.device)
    dW2 = torch.empty((N, K2), dtype=torch.float32, device=g.device) if K2 else None
    db = torch.empty(N, dtype=torch.float32, device=g.device) if want_db else None
    with torch.cuda.device(g.device):
        tok = TIMER.start(("wgrad_smallk", M, N, K1 + K2, "bf16"))
        st = L.lpg_relu_wgrad_smallk_bf16(M, N, g.data_ptr(), g.stride(0), None if y is None else y.data_ptr(),
                                          0 if y is None else y.stride(0), float(scale), K1, A1.data_ptr(), max(K1, 1),
                                          K2, None if A2 is None else A2.data_ptr(), max(K2, 1), dW1.data_ptr(),
                                          None if dW2 is None else dW2.data_ptr(), None if db is None else db.data_ptr(),
                                          ws.data_ptr(), _lib.stream_of(g))
        TIMER.stop(tok)
    _lib.check(st, "lpg_relu_wgrad_smallk_bf16")
    return dW1, dW2, db


def _small_heads_bf16(x: Tensor, W: Tensor) -> bool:
    """The bf16 heads' streaming kernels take this Linear (N <= 4 outputs, K <= 2048)."""
    K = x.shape[1]
    return (x.dtype in HALF16 and W.shape[0] <= 4 and 8 <= K <= 2048 and K % 8 == 0 and x.stride(1) == 1
            and x.stride(0) % 8 == 0 and x.data_ptr() % 16 == 0)


def linear_small_fwd_bf16(x: Tensor, W: Tensor, b: Tensor | None) -> Tensor:
    """The 16-bit heads' forward (lpg_linear_small_fwd_bf16 / _f16 by x's dtype): [M, N] = RNE(x W^T + b),
    W rounded to the storage type first (the c5 / --fp16 model's weights), fp32 sums."""
    M, K = x.shape
    N = W.shape[0]
    dt = x.dtype
    Wf = W.detach().to(dt).float().contiguous()
    b = None if b is None else b.detach().float().contiguous()
    out = torch.empty((M, N), dtype=dt, device=x.device)
    entry = "lpg_linear_small_fwd_f16" if dt == torch.float16 else "lpg_linear_small_fwd_bf16"
    with torch.cuda.device(x.device):
        tok = TIMER.start(("heads_fwd", M, N, K, "f16" if dt == torch.float16 else "bf16"))
        st = getattr(_lib.lib(), entry)(M, K, N, x.data_ptr(), x.stride(0), Wf.data_ptr(),
                                        None if b is None else b.data_ptr(), out.data_ptr(), N, _lib.stream_of(x))
        TIMER.stop(tok)
    _lib.check(st, entry)
    return out


def heads_bwd_bf16(G: Tensor, W: Tensor, Y: Tensor, scale: float | None, want_dby: bool):
    """(dH, dW, db, dbY) of the bf16 heads in one pass over their input Y (lpg_heads_bwd_bf16).
    ``scale`` not None: dH goes through the producing layer's ReLU/dropout backward (the layer's dZ,
    the bits of the separate relu_bwd_colsum_bf16 pass), and dbY = its column sums (the bits of
    colsum_bf16 on dH)."""
    M, K = Y.shape
    N = W.shape[0]
    Gf = G.float().contiguous()
    Wf = W.detach().to(torch.bfloat16).float().contiguous()
    L = _lib.lib()
    ws = _workspace(L.lpg_heads_bwd_bf16_workspace_bytes(M, K, N), Y.device)
    dH = torch.empty((M, K), dtype=torch.bfloat16, device=Y.device)
    dW = torch.empty((N, K), dtype=torch.float32, device=Y.device)
    db = torch.empty(N, dtype=torch.float32, device=Y.device)
    dbY = torch.empty(K, dtype=torch.float32, device=Y.device) if want_dby else None
    with torch.cuda.device(Y.device):
        tok = TIMER.start(("heads_bwd", M, N, K, "bf16"))
        st = L.lpg_heads_bwd_bf16(M, K, N, Gf.data_ptr(), Gf.stride(0), Wf.data_ptr(), Y.data_ptr(), Y.stride(0),
                                  0 if scale is None else 1, 1.0 if scale is None else float(scale), dH.data_ptr(), K,
                                  dW.data_ptr(), db.data_ptr(), None if dbY is None else dbY.data_ptr(), ws.data_ptr(),
                                  _lib.stream_of(Y))
        TIMER.stop(tok)
    _lib.check(st, "lpg_heads_bwd_bf16")
    return dH, dW, db, dbY


def dropout_scale(p: float) -> float:
    """The scale the FC kernels give kept values under dropout p (fc_common.h dropout_params):
    2^16 / (2^16 - round(p * 2^16)) as float32, the reciprocal of the rate actually kept -- F.dropout's
    1 / (1 - p) for the 16-bit threshold.  The backward passes use the same value.  p below 2^-17
    (which the 16-bit threshold cannot draw) is refused rather than silently drawn at 2^-16."""
    if p <= 0:
        return 1.0
    if p >= 1.0 or p * 65536.0 < 0.5:
        raise ValueError(f"lpgnn dropout: p = {p} outside [2^-17, 1) (16-bit keep threshold)")
    th = int(min(max(float(torch.tensor(p, dtype=torch.float32)) * 65536.0 + 0.5, 1.0), 65535.0))
    return float(torch.tensor(65536.0, dtype=torch.float32) / torch.tensor(65536 - th, dtype=torch.float32))


def _new_seed() -> int:
    """A dropout seed from torch's default generator (torch.manual_seed reproducible)."""
    return int(torch.randint(0, 2**62, (1,), dtype=torch.int64).item())


class _FC(torch.autograd.Function):
    @staticmethod
    def forward(ctx, A1, A2, W1, W2, b, relu, dropout_p, row_offset=0, row_keys=None, arith=None):
        if dropout_p > 0 and not relu:
            raise RuntimeError("lpgnn FC: fused dropout requires the ReLU epilogue")
        seed = _new_seed() if dropout_p > 0 else 0
        ctx.bf16 = A1.dtype == torch.bfloat16
        kw = dict(row_offset=row_offset, row_keys=row_keys)
        if ctx.bf16:  # c5 path: bf16 activations, fp32 master weights cast per call
            W1 = W1.to(torch.bfloat16)
            W2 = None if W2 is None else W2.to(torch.bfloat16)
            C = fc_forward_bf16(A1, W1, A2, W2, b, relu, dropout_p, seed, **kw)
        else:
            C = fc_forward(A1, W1, A2, W2, b, relu, dropout_p, seed, arith=arith, **kw)
        ctx.relu, ctx.has_a2, ctx.has_b = relu, A2 is not None, b is not None
        ctx.scale = dropout_scale(dropout_p)
        ctx.save_for_backward(A1, A2 if A2 is not None else A1, W1, W2 if W2 is not None else W1,
                              C if relu else A1)
        return C

    @staticmethod
    def backward(ctx, gC):
        A1, A2, W1, W2, C = ctx.saved_tensors
        need = ctx.needs_input_grad
        want_db = ctx.has_b and need[4]
        if ctx.bf16:  # bf16 input grads on lpg_fc_bf16, fp32 weight grads on lpg_wgrad_bf16, fp32 bias grad
            if ctx.relu:
                g, db = relu_bwd_colsum_bf16(gC, C, ctx.scale, want_db)
            else:
                g, db = gC.to(torch.bfloat16), (gC.float().sum(0) if want_db else None)
            dA1 = input_grad_bf16(g, W1) if need[0] else None
            dA2 = input_grad_bf16(g, W2) if ctx.has_a2 and need[1] else None
            dW1 = wgrad_bf16(g, A1) if need[2] else None
            dW2 = wgrad_bf16(g, A2) if ctx.has_a2 and need[3] else None
            return dA1, dA2, dW1, dW2, db, None, None, None, None, None
        if ctx.relu:
            g, db = relu_bwd_colsum(gC, C, ctx.scale, want_db)  # ReLU + dropout bwd, bias grad fused
        else:
            g, db = gC, (gC.sum(0) if want_db else None)
        dA1 = g @ W1 if need[0] else None
        dA2 = g @ W2 if ctx.has_a2 and need[1] else None
        K = A1.shape[1] + (A2.shape[1] if ctx.has_a2 else 0)
        if (need[2] or need[3]) and K <= 16 and g.shape[1] % 4 == 0:
            dW1, dW2 = wgrad_smallk(g, A1, A2 if ctx.has_a2 else None)  # conv1: dZ read once
            dW1 = dW1 if need[2] else None
            dW2 = dW2 if need[3] else None
        else:
            dW1 = g.t() @ A1 if need[2] else None
            dW2 = g.t() @ A2 if ctx.has_a2 and need[3] else None
        return dA1, dA2, dW1, dW2, db, None, None, None, None, None


def graph_conv_fc(agg: Tensor, x_dst: Tensor, w_rel: Tensor, b_rel, w_root: Tensor, relu: bool,
                  dropout: float = 0.0, row_offset: int = 0, row_keys: Tensor | None = None,
                  arith: str | None = None) -> Tensor:
    """GraphConv's lin_rel(agg) + lin_root(x_dst) (+ ReLU, dropout) as one autograd node; the dropout
    mask keys rows by row_keys[m] or row_offset + m (a partition's global node ids)."""
    return _FC.apply(agg, x_dst, w_rel, w_root, b_rel, relu, float(dropout), int(row_offset), row_keys, arith)


def linear_small_bwd(G: Tensor, W: Tensor, H: Tensor, need_dh: bool):
    """(dH, dW, db) of a Linear with N <= 4 outputs (lpg_linear_small_bwd_f32)."""
    M, K = H.shape
    N = W.shape[0]
    G, W, H = G.contiguous(), W.contiguous(), H.contiguous()
    L = _lib.lib()
    ws = torch.empty(max(L.lpg_linear_small_bwd_workspace_bytes(M, K, N), 16) // 4 + 4, dtype=torch.float32,
                     device=H.device)
    dH = torch.empty_like(H) if need_dh else None
    dW = torch.empty_like(W)
    db = torch.empty(N, dtype=torch.float32, device=H.device)
    with torch.cuda.device(H.device):
        st = L.lpg_linear_small_bwd_f32(M, K, N, G.data_ptr(), G.stride(0), W.data_ptr(), H.data_ptr(), H.stride(0),
                                        None if dH is None else dH.data_ptr(), K, dW.data_ptr(), db.data_ptr(),
                                        ws.data_ptr(), _lib.stream_of(H))
    _lib.check(st, "lpg_linear_small_bwd_f32")
    return dH, dW, db


def heads_relu_bwd(G: Tensor, W: Tensor, Y: Tensor, scale: float, want_dby: bool, arith: str | None = None):
    """(dZ, dW, db, dbY): the heads' backward through the producing layer's
    ReLU/dropout in one pass over Y (lpg_heads_relu_bwd_f32).  ``arith`` "f16x2" (explicit, not the
    process default: the caller vouches that dZ is only read afterwards): dZ feeds f16x2 GEMMs, so the same
    pass also returns its row / column scales (lpg_heads_relu_bwd_scales_f32), cached for it."""
    M, K = Y.shape
    N = W.shape[0]
    G, W = G.contiguous(), W.contiguous()
    Y = Y if (Y.stride(1) == 1 and Y.stride(0) % 4 == 0 and Y.data_ptr() % 16 == 0) else Y.contiguous()
    L = _lib.lib()
    ws = torch.empty(max(L.lpg_linear_small_bwd_workspace_bytes(M, K, N), 16) // 4 + 4, dtype=torch.float32,
                     device=Y.device)
    dZ = torch.empty((M, K), dtype=torch.float32, device=Y.device)
    dW = torch.empty_like(W)
    db = torch.empty(N, dtype=torch.float32, device=Y.device)
    dbY = torch.empty(K, dtype=torch.float32, device=Y.device) if want_dby else None
    sc = arith == "f16x2" and K % 4 == 0 and M > 0  # (opt-in: the caller knows dZ is not rewritten later)
    with torch.cuda.device(Y.device):
        tok = TIMER.start(("heads_relu_bwd", M, N, K, "f32"))
        if sc:
            rs = torch.empty(M, dtype=torch.float32, device=Y.device)
            cs = torch.empty(K, dtype=torch.float32, device=Y.device)
            sws = torch.empty(max(16, L.lpg_heads_scales_workspace_bytes(M, K)) // 4, dtype=torch.float32,
                              device=Y.device)
            st = L.lpg_heads_relu_bwd_scales_f32(M, K, N, G.data_ptr(), G.stride(0), W.data_ptr(), Y.data_ptr(),
                                                 Y.stride(0), float(scale), dZ.data_ptr(), K, dW.data_ptr(),
                                                 db.data_ptr(), None if dbY is None else dbY.data_ptr(), rs.data_ptr(),
                                                 cs.data_ptr(), sws.data_ptr(), ws.data_ptr(), _lib.stream_of(Y))
        else:
            st = L.lpg_heads_relu_bwd_f32(M, K, N, G.data_ptr(), G.stride(0), W.data_ptr(), Y.data_ptr(),
                                          Y.stride(0), float(scale), dZ.data_ptr(), K, dW.data_ptr(), db.data_ptr(),
                                          None if dbY is None else dbY.data_ptr(), ws.data_ptr(), _lib.stream_of(Y))
        TIMER.stop(tok)
    _lib.check(st, "lpg_heads_relu_bwd_scales_f32" if sc else "lpg_heads_relu_bwd_f32")
    if sc:
        _SCALES.put("row", dZ, rs)
        _SCALES.put("col", dZ, cs)
    return dZ, dW, db, dbY


class _Linear(torch.autograd.Function):
    """torch.nn.Linear on lpg_fc_f32; few-output backward on the HIP kernel."""

    @staticmethod
    def forward(ctx, x, W, b, prev=None, arith=None):
        ctx.has_b = b is not None
        ctx.bf16 = x.dtype in HALF16  # (fp16: the --fp16 inference mode, forward only)
        ctx.f16 = x.dtype == torch.float16
        ctx.in_scale = None
        ctx.small, ctx.prev = False, None
        if prev is not None:  # x = a bf16 ReLU layer's output feeding only this Linear: fold its backward
            ctx.in_scale = prev.scale
            prev.out_folded = True
        if ctx.bf16:
            W = W.to(x.dtype)
            ctx.save_for_backward(x, W)
            ctx.small = _small_heads_bf16(x, W)
            ctx.prev = prev
            if ctx.small:  # the heads (N = 3): one streaming pass over x
                return linear_small_fwd_bf16(x, W, b)
            return fc_forward_bf16(x, W, None, None, b, False)
        ctx.save_for_backward(x, W)
        return fc_forward(x, W, None, None, b, False, arith=arith)

    @staticmethod
    def backward(ctx, g):
        if ctx.f16:
            raise RuntimeError("lpgnn: fp16 is the reference's inference mode (val.py:269); train in fp32 or bf16")
        x, W = ctx.saved_tensors
        need = ctx.needs_input_grad
        if ctx.bf16 and ctx.small:
            # one pass over x: dx (through the producing layer's ReLU/dropout backward when folded),
            # dW, db, and that layer's bias column sums, handed to its backward node (conv.py)
            dx, dW, db, dby = heads_bwd_bf16(g.to(torch.bfloat16), W, x, ctx.in_scale, ctx.in_scale is not None)
            if ctx.prev is not None and dby is not None:
                if getattr(ctx.prev, "folded_colsum", None) is None:
                    ctx.prev.folded_colsum = {}
                # keyed by the layer output's storage; the gradient handed over is checked by identity
                # (`g is dx` in conv.py), and dx is held here, so its memory cannot be reused for another
                # tensor while the entry exists (a hook that replaces the gradient falls back to colsum)
                ctx.prev.folded_colsum[x.data_ptr()] = (dx, dby)
            ctx.prev = None
            return (dx if need[0] else None), (dW if need[1] else None), (db if ctx.has_b and need[2] else None), \
                None, None
        if ctx.bf16:
            g = g.to(torch.bfloat16)
            mask = None if ctx.in_scale is None else (x, ctx.in_scale)
            dx = input_grad_bf16(g, W, mask=mask) if need[0] else None
            dW = wgrad_bf16(g, x) if need[1] else None
            db = g.float().sum(0) if ctx.has_b and need[2] else None
            return dx, dW, db, None, None
        if W.shape[0] <= 4 and x.shape[1] % 4 == 0:
            dx, dW, db = linear_small_bwd(g, W, x, need[0])
            return dx, dW if need[1] else None, db if (ctx.has_b and need[2]) else None, None, None
        dx = g @ W if need[0] else None
        dW = g.t() @ x if need[1] else None
        db = g.sum(0) if ctx.has_b and need[2] else None
        return dx, dW, db, None, None


def linear(x: Tensor, weight: Tensor, bias, fold_in: bool = False, opts=None) -> Tensor:
    """torch.nn.Linear.forward on lpg_fc_f32 (heads, arch.py:190).  ``fold_in`` (GCN_FC's heads,
    bf16): the caller guarantees both outputs of the producing layer feed only its heads, so that
    layer's ReLU/dropout backward is folded into the heads' input-gradient stores."""
    opts = opts or _DEFAULT_OPTIONS
    prev = None
    if fold_in and x.dtype == torch.bfloat16 and torch.is_grad_enabled():
        from . import conv as _conv

        prev = _conv.foldable_producer(x, opts)
    return _Linear.apply(x, weight, bias, prev, opts.arith)


class _Knowledge(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logit, feas, bound):
        if logit.device.type != "cuda":
            raise RuntimeError("lpgnn: add_knowledge runs on a HIP device only (no CPU path)")
        logit = logit.contiguous()
        feas = feas.contiguous().float()
        out = torch.empty_like(logit)
        L = _lib.lib()
        with torch.cuda.device(logit.device):
            st = L.lpg_knowledge_f32(logit.shape[0], logit.data_ptr(), logit.stride(0), feas.data_ptr(),
                                     feas.stride(0), feas.shape[1], float(bound), out.data_ptr(), out.stride(0),
                                     _lib.stream_of(logit))
        _lib.check(st, "lpg_knowledge_f32")
        ctx.save_for_backward(logit)
        return out

    @staticmethod
    def backward(ctx, g):
        """autograd of F.normalize(x) * 10 in one pass (lpg_knowledge_bwd_f32)."""
        (x,) = ctx.saved_tensors
        g = g.contiguous().float()
        dx = torch.empty_like(x)
        with torch.cuda.device(x.device):
            st = _lib.lib().lpg_knowledge_bwd_f32(x.shape[0], x.data_ptr(), x.stride(0), g.data_ptr(), g.stride(0),
                                                  dx.data_ptr(), dx.stride(0), _lib.stream_of(x))
        _lib.check(st, "lpg_knowledge_bwd_f32")
        return dx, None, None


def knowledge(logit: Tensor, feas: Tensor, bound=10) -> Tensor:
    """One side of add_knowledge: normalize(logit) * 10, then -bound on
    column 0 where feas[:, -3] != 0 (lower bound = -inf) and on column 2
    where feas[:, -1] != 0 (upper bound = +inf).  fp16 logits (the --fp16
    inference mode): lpg_knowledge_f16, half-precision semantics, fp16 out, no backward."""
    if logit.dtype == torch.float16:
        return knowledge_f16(logit, feas, bound)
    return _Knowledge.apply(logit, feas, bound)


def knowledge_f16(logit: Tensor, feas: Tensor, bound=10) -> Tensor:
    """arch.py:129-141 on fp16 logits as torch's half ops evaluate it (lpg_knowledge_f16)."""
    if logit.device.type != "cuda":
        raise RuntimeError("lpgnn: add_knowledge runs on a HIP device only (no CPU path)")
    if torch.is_grad_enabled() and logit.requires_grad:
        raise RuntimeError("lpgnn: fp16 is the reference's inference mode (val.py:269); no backward")
    logit = logit.contiguous()
    feas = feas.contiguous().float()
    out = torch.empty_like(logit)
    with torch.cuda.device(logit.device):
        st = _lib.lib().lpg_knowledge_f16(logit.shape[0], logit.data_ptr(), logit.stride(0), feas.data_ptr(),
                                          feas.stride(0), feas.shape[1], float(bound), out.data_ptr(), out.stride(0),
                                          _lib.stream_of(logit))
    _lib.check(st, "lpg_knowledge_f16")
    return out
