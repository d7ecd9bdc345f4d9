"""Per-call time of the f16x2 operand sweeps: lpg_rowscale_f32 + lpg_colscale_f32 (two reads) against
lpg_rowcolscale_f32 (one read, both scales) at the c2 operand shapes.  Usage: python sweep_ab.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "lp-gnn_amd"))
from lpgnn import _lib  # noqa: E402
from lpgnn import fc as F  # noqa: E402

DEV = "cuda:0"


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    L = _lib.lib()
    for R, N in [(100_000, 1024), (200_000, 1024), (200_000, 2048)]:
        G = torch.randn(R, N, device=DEV)
        rs, cs = torch.empty(R, device=DEV), torch.empty(N, device=DEV)
        ws = torch.empty(max(16, L.lpg_rowcolscale_workspace_bytes(R, N)), dtype=torch.uint8, device=DEV)
        st = _lib.stream_of(G)
        t_r = timed(lambda: F._rowscale1(G))
        t_c = timed(lambda: F._colscale1(G))
        t_b = timed(lambda: L.lpg_rowcolscale_f32(R, N, G.data_ptr(), N, rs.data_ptr(), cs.data_ptr(), ws.data_ptr(),
                                                  st))
        gb = R * N * 4 / 1e9
        print(f"[{R}x{N}] row {t_r:7.1f} us  col {t_c:7.1f} us  (sum {t_r + t_c:7.1f})  both {t_b:7.1f} us "
              f"= {gb / t_b * 1e6 / 1e3:.2f} TB/s", flush=True)


if __name__ == "__main__":
    main()
