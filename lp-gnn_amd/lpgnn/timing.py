"""Per-kernel HIP-event timing for bench.py's roofline measurement.

When enabled, every hot-path launch is bracketed by a pair of
``torch.cuda.Event`` records on the stream the kernel is launched on (the
library launches on torch's current stream, so the events order against the
kernel exactly).  Disabled (the default) it costs one attribute check.
"""
from __future__ import annotations

from collections import defaultdict

import torch


class KernelTimer:
    def __init__(self):
        self.enabled = False
        self._pending = []

    def reset(self):
        self._pending.clear()

    def start(self, key):
        if not self.enabled:
            return None
        ev0 = torch.cuda.Event(enable_timing=True)
        ev0.record()
        return (key, ev0)

    def stop(self, tok):
        if tok is None:
            return
        ev1 = torch.cuda.Event(enable_timing=True)
        ev1.record()
        self._pending.append((tok[0], tok[1], ev1))

    def summary(self):
        """{key: (launches, total_ms)} -- synchronises."""
        torch.cuda.synchronize()
        out = defaultdict(lambda: [0, 0.0])
        for key, e0, e1 in self._pending:
            out[key][0] += 1
            out[key][1] += e0.elapsed_time(e1)
        return {k: tuple(v) for k, v in out.items()}


    def launches(self):
        """{key: [ms of each launch]} -- synchronises."""
        torch.cuda.synchronize()
        out = defaultdict(list)
        for key, e0, e1 in self._pending:
            out[key].append(e0.elapsed_time(e1))
        return dict(out)


TIMER = KernelTimer()
