"""Summarise a rocprofv3 --kernel-trace --stats run into profiles/<tag>_kernels.md
(+ .json), grouping the hot-path kernels by name.

  python tools/prof_summary.py gpurun_out/prof/run_kernel_stats.csv profiles/r01_c2_kernels
"""
import csv
import json
import sys


def short(name: str) -> str:
    for key in ("spmm_f32_rowwave", "spmm_f32_narrow", "spmm_bf16", "fc_fwd_f32", "knowledge_f32",
                "fc_bwd", "fc_dw", "Cijk_", "elementwise", "reduce_kernel", "dropout", "nll_loss"):
        if key in name:
            return name[:160]
    return name[:160]


def main(src, dst):
    rows = list(csv.DictReader(open(src)))
    rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
    total = sum(float(r["TotalDurationNs"]) for r in rows)
    out = []
    for r in rows:
        out.append(dict(name=short(r["Name"]), calls=int(r["Calls"]), total_ms=float(r["TotalDurationNs"]) / 1e6,
                        avg_us=float(r["AverageNs"]) / 1e3, min_us=float(r["MinNs"]) / 1e3,
                        max_us=float(r["MaxNs"]) / 1e3, pct=float(r["Percentage"])))
    json.dump(dict(source=src, total_ms=total / 1e6, kernels=out), open(dst + ".json", "w"), indent=1)
    with open(dst + ".md", "w") as f:
        f.write(f"# rocprofv3 --kernel-trace --stats summary\n\nsource: `{src}`; total GPU kernel time "
                f"{total / 1e6:.2f} ms\n\n| % | calls | total ms | avg us | min us | max us | kernel |\n"
                "|---:|---:|---:|---:|---:|---:|---|\n")
        for k in out[:40]:
            f.write(f"| {k['pct']:.1f} | {k['calls']} | {k['total_ms']:.2f} | {k['avg_us']:.1f} | "
                    f"{k['min_us']:.1f} | {k['max_us']:.1f} | `{k['name'][:110]}` |\n")
    print(open(dst + ".md").read()[:3000])


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
