"""Where the bf16 FC's time goes per block: run fc_bf16_p from the probe build
(make -C lp-gnn_amd OUT=../tools/experiments/var_probe/liblpgnn_hip.so
 OBJDIR=../tools/experiments/var_probe/build EXTRA=-DLPG_PHASE_PROBE)
and read each block's timestamps: start, first tile landed, k loop done, epilogue stores done.

  LPGNN_LIB=tools/experiments/var_probe/liblpgnn_hip.so python tools/experiments/phase_probe.py
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lp-gnn_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from lpgnn import _lib  # noqa: E402
from lpgnn.fc import fc_forward_bf16  # noqa: E402


def run(M, N, K, relu, drop, label):
    BF = torch.bfloat16
    A = torch.randn(M, K, device="cuda").to(BF)
    W = (torch.randn(N, K, device="cuda") * 0.02).to(BF)
    b = torch.randn(N, device="cuda")
    nblk = ((M + 255) // 256) * ((N + 255) // 256)
    buf = torch.zeros(nblk * 8, dtype=torch.int64, device="cuda")
    L = _lib.lib()
    L.lpg_debug_set_probe.argtypes = [ctypes.c_void_p]
    f = lambda: fc_forward_bf16(A, W, None, None, b if relu else None, relu, drop, 7, kernel=3)
    L.lpg_debug_set_probe(None)
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    L.lpg_debug_set_probe(buf.data_ptr())
    f()
    torch.cuda.synchronize()
    L.lpg_debug_set_probe(None)
    t = buf.cpu().numpy().reshape(nblk, 8).astype(np.float64)
    rt = (t[:, :4] - t[:, 0].min()) / 100.0  # 100 MHz -> us
    cyc = t[:, 4:]
    pro, main, epi = rt[:, 1] - rt[:, 0], rt[:, 2] - rt[:, 1], rt[:, 3] - rt[:, 2]
    clk = (cyc[:, 3] - cyc[:, 0]) / (rt[:, 3] - rt[:, 0]) / 1e3  # GHz
    span = rt[:, 3].max()
    busy = (rt[:, 3] - rt[:, 0]).sum()
    cus = 256
    print(f"{label}: M={M} N={N} K={K} blocks={nblk} launch span {span:.1f} us; per block: prologue "
          f"{np.median(pro):.2f} us (p90 {np.percentile(pro, 90):.2f}), k loop {np.median(main):.2f} "
          f"(p10 {np.percentile(main, 10):.2f}, p90 {np.percentile(main, 90):.2f}), epilogue {np.median(epi):.2f} "
          f"(p90 {np.percentile(epi, 90):.2f}); clock {np.median(clk):.2f} GHz; block-time / (span x {cus} CUs) "
          f"= {busy / (span * cus):.3f}; share of block time: prologue {pro.sum() / busy:.3f} k-loop "
          f"{main.sum() / busy:.3f} epilogue {epi.sum() / busy:.3f}")
    # rounds: start-time histogram
    starts = np.sort(rt[:, 0])
    gaps = np.diff(starts)
    print(f"   start times: first {starts[0]:.1f}, 256th {starts[min(255, nblk - 1)]:.1f}, last {starts[-1]:.1f} us;"
          f" end of first finisher {rt[:, 3].min():.1f} us; largest start gap {gaps.max() if len(gaps) else 0:.2f} us")


if __name__ == "__main__":
    torch.manual_seed(0)
    run(200_000, 2048, 2048, False, 0.0, "plain")
    run(200_000, 2048, 2048, True, 0.1, "relu+drop")
    run(200_000, 2048, 4096, True, 0.1, "relu+drop")
    run(100_000, 2048, 4096, True, 0.1, "relu+drop")
