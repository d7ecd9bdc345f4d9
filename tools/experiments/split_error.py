"""Representation error of fp32 GEMMs emulated on 16-bit matrix-core operands (CPU, fp64 accumulation so
only the operand splits are measured), against the fp32 SGEMM's own total error (fp32 products and
accumulation), at K = 1024 on ReLU-like activations with per-row scales (and a gradient-like case whose row
scales spread over e^(4 N(0,1))):
  x3       -- the default fp32 path: three bf16 planes per operand, six products (fc_x3.hip);
  f16x2 3p -- two fp16 planes per operand after a power-of-2 scale (per tensor, or per row), three
              products hh + hl + lh (half the MFMA work of x3);
  f16x2 4p -- the same with the ll product.
The question it answers: how many matrix-core products an fp32-class GEMM needs here."""
import torch

torch.manual_seed(0)
M, N, K = 2000, 512, 1024


def bf(x):
    return x.float().bfloat16().double()


def hf(x):
    return x.float().half().double()


def x3(A, W):
    def s3(x):
        h = bf(x)
        m = bf(x - h)
        return h, m, bf(x - h - m)
    ah, am, al = s3(A)
    wh, wm, wl = s3(W)
    return ah @ wh.T + ah @ wm.T + am @ wh.T + ah @ wl.T + am @ wm.T + al @ wh.T


def scale(x, per_row):
    mx = x.abs().amax(dim=1, keepdim=True) if per_row else x.abs().max()
    return 2.0 ** (15 - torch.ceil(torch.log2(mx.clamp_min(1e-300))))


def f16x2(A, W, four=False, per_row=False):
    sa, sw = scale(A, per_row), scale(W, per_row)
    a, w = A * sa, W * sw
    ah, wh = hf(a), hf(w)
    al, wl = hf(a - ah), hf(w - wh)
    c = ah @ wh.T + ah @ wl.T + al @ wh.T + ((al @ wl.T) if four else 0)
    return c / (sa * (sw.T if per_row else sw))


for label, spread in (("activations (row scales e^N(0,1))", 1.0), ("gradient-like (row scales e^(4 N(0,1)))", 4.0)):
    A = torch.relu(torch.randn(M, K, dtype=torch.float64)) * torch.exp(spread * torch.randn(M, 1, dtype=torch.float64))
    A = A.float().double()
    W = (torch.randn(N, K, dtype=torch.float64) * 0.03).float().double()
    ref = A @ W.T
    den = A.abs() @ W.abs().T
    print(label)
    rows = [("fp32 SGEMM (total error)", (A.float() @ W.float().T).double()),
            ("x3 bf16 6 products", x3(A, W)),
            ("f16x2 3 products, tensor scale", f16x2(A, W)),
            ("f16x2 3 products, row scale", f16x2(A, W, per_row=True)),
            ("f16x2 4 products, row scale", f16x2(A, W, four=True, per_row=True))]
    for name, C in rows:
        e = (C - ref).abs()
        rel_row = (e.norm(dim=1) / ref.norm(dim=1).clamp_min(1e-300)).max()
        print(f"  {name:34s} max |err|/sum|ab| {float((e / den).max()):.2e}   worst row rel {float(rel_row):.2e}")
