"""Condense per-rank rocprofv3 kernel + memory-copy traces into a step timeline (markdown).

Usage: python tools/trace_timeline.py [--steps S] OUT.md RANKDIR0 [RANKDIR1 ...]
Each RANKDIR holds that rank's rocprofv3 CSVs (``*kernel_trace.csv``, ``*memory_copy_trace.csv``)
and ``rank.log`` with bench.py's ``TRACE_WINDOW rank=R boottime_ns=T0 T1`` line
(LPGNN_TRACE_WINDOW=1); only records inside that window (the timed steps) are kept.

The timeline groups the records into phases and reports the gaps in which the rank had nothing
on the GPU (host work: with gloo, the boundary exchange's TCP
all_to_all between its D2H and H2D copies).  The segment table lists the first of the S timed
steps (the window split evenly); the category totals cover the whole window."""
import csv
import glob
import os
import re
import sys


def category(name: str) -> str:
    n = name.lower()
    if "copybuffer" in n:  # ROCclr blit kernels: the host<->device staging of the gloo exchange
        return "copy"
    if "spmm" in n:
        return "spmm"
    if "wgrad" in n:
        return "wgrad"
    if "x3" in n or "fc_" in n or "linear" in n:
        return "fc"
    if "split" in n or "fold" in n:
        return "fold"
    return "other"


def load(rankdir: str):
    win = None
    for line in open(os.path.join(rankdir, "rank.log"), errors="replace"):
        m = re.search(r"TRACE_WINDOW rank=(\d+) boottime_ns=(\d+) (\d+)", line)
        if m:
            win = (int(m.group(1)), int(m.group(2)), int(m.group(3)))
    if win is None:
        raise SystemExit(f"{rankdir}/rank.log: no TRACE_WINDOW line")
    rank, t0, t1 = win
    ev = []
    for path in glob.glob(os.path.join(rankdir, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            if t0 <= s and e <= t1:
                ev.append((s, e, category(r["Kernel_Name"]), r["Kernel_Name"], 0))
    for path in glob.glob(os.path.join(rankdir, "**", "*memory_copy_trace.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            if t0 <= s and e <= t1:
                d = r.get("Direction", "copy")
                kind = "D2H" if "DEVICE_TO_HOST" in d else "H2D" if "HOST_TO_DEVICE" in d else "D2D"
                size = int(r.get("Size", 0) or 0)
                ev.append((s, e, kind, d, size))
    ev.sort()
    return rank, t0, t1, ev


def segments(ev, t0, gap_ns=1_000_000):
    """Phases: records separated by less than gap_ns of GPU idle time are one phase; each phase
    carries its per-category busy time.  Idle gaps >= gap_ns are phases of their own."""
    out, cur, busy_to = [], None, t0
    for s, e, cat, _name, size in ev:
        if s - busy_to >= gap_ns:
            if cur:
                out.append(cur)
                cur = None
            out.append(["idle", busy_to, s, {}, 0])
        if cur is None:
            cur = ["busy", s, e, {}, 0]
        cur[2] = max(cur[2], e)
        cur[3][cat] = cur[3].get(cat, 0.0) + (e - s) / 1e6
        cur[4] += 1
        busy_to = max(busy_to, e)
    if cur:
        out.append(cur)
    return out


def main():
    argv = sys.argv[1:]
    steps = 1
    if argv and argv[0] == "--steps":
        steps, argv = int(argv[1]), argv[2:]
    out_md, dirs = argv[0], argv[1:]
    lines = ["# Timed-step timeline per rank (rocprofv3 kernel + memory-copy trace)", ""]
    for d in dirs:
        rank, t0, t1, ev = load(d)
        span = (t1 - t0) / 1e6
        tot = {}
        for s, e, cat, _n, _sz in ev:
            tot[cat] = tot.get(cat, 0.0) + (e - s) / 1e6
        segs = segments(ev, t0)
        idle = sum((g[2] - g[1]) / 1e6 for g in segs if g[0] == "idle")
        lines += [f"## rank {rank}: window {span:.2f} ms, {len(ev)} records", "",
                  "| category | ms (sum of record durations) |", "|---|---|"]
        lines += [f"| {k} | {v:.3f} |" for k, v in sorted(tot.items(), key=lambda kv: -kv[1])]
        lines += [f"| GPU idle >= 1 ms (host: gloo TCP all_to_all, Python) | {idle:.3f} |", "",
                  f"Phases of the first of {steps} timed steps (busy = records less than 1 ms apart):", "",
                  "| t (ms) | phase | ms | records | GPU time by category (ms) |", "|---|---|---|---|---|"]
        for kind, s, e, cats, n in segs:
            if s - t0 > (t1 - t0) / steps:
                break
            desc = ", ".join(f"{k} {v:.2f}" for k, v in sorted(cats.items(), key=lambda kv: -kv[1]))
            lines.append(f"| {(s - t0) / 1e6:.2f} | {kind} | {(e - s) / 1e6:.2f} | {n or ''} | {desc} |")
        lines.append("")
    open(out_md, "w").write("\n".join(lines) + "\n")
    print("\n".join(lines[:40]))


if __name__ == "__main__":
    main()
