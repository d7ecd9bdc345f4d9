"""Summary of tools/experiments/x3_traffic_probe.sh: per variant, the mean past-L2 bytes per fc_x3_wide
launch (FETCH_SIZE doubled -- gfx950 counts half of a 16-B-per-lane read, MI355X_MICROARCH.md -- and
WRITE_SIZE, KiB), and for the default the clock / MFMA busy from the SQ pass
(tools/pmc_kernel_summary.py's formulas).

  python tools/experiments/x3_traffic_summary.py gpurun_out/x3traffic default x3p1 x3p2
"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from pmc_summary import read_counter  # noqa: E402

KERNEL = "fc_x3_wide"


def mean_of(d, counter):
    per = read_counter(d, counter)
    vals = [v for k, vs in per.items() if KERNEL in k for v in vs]
    return sum(vals) / len(vals) if vals else None, len(vals)


def main(out, *variants):
    res = {"kernel": KERNEL, "shape": "M = 200000, K = 1024 + 1024, N = 1024, ReLU (x3 FC at K = 2048)",
           "correction": "past-L2 read bytes = 2 x FETCH_SIZE KiB x 1024; write bytes = WRITE_SIZE KiB x 1024",
           "algorithmic_gb": {"A": 200000 * 2048 * 4 / 1e9, "W_planes": 3 * 1024 * 2048 * 2 / 1e9,
                              "C": 200000 * 1024 * 4 / 1e9}}
    for v in variants:
        f, nf = mean_of(os.path.join(out, f"{v}_FETCH_SIZE"), "FETCH_SIZE")
        w, nw = mean_of(os.path.join(out, f"{v}_WRITE_SIZE"), "WRITE_SIZE")
        res[v] = {"read_gb": None if f is None else 2 * f * 1024 / 1e9,
                  "write_gb": None if w is None else w * 1024 / 1e9, "launches": [nf, nw]}
    sq = os.path.join(out, "default_sq")
    if os.path.isdir(sq):
        import subprocess

        subprocess.run([sys.executable, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                                     "pmc_kernel_summary.py"), sq,
                        os.path.join(out, "default_FETCH_SIZE"), os.path.join(out, "default_WRITE_SIZE"), KERNEL,
                        os.path.join(out, "default_kernel.json"), res["shape"]], check=False)
        try:
            res["default_kernel"] = json.load(open(os.path.join(out, "default_kernel.json")))
        except Exception as e:  # noqa: BLE001
            res["default_kernel"] = f"unavailable: {e}"
    json.dump(res, open(os.path.join(out, "summary.json"), "w"), indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "default_kernel"}, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
