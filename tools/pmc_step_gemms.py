"""Issue-mix counters of the GEMM kernels inside the c2 training step (one rocprofv3 --pmc pass over
`bench.py --profile-only`, tools/pmc_step_gemms.sh), per kernel instantiation: MFMA busy fraction,
VALU instructions per MFMA, clock, wave-cycle split.  Units and corrections as tools/pmc_kernel_summary.py
(MI355X_MICROARCH.md): SQ_VALU_MFMA_BUSY_CYCLES summed over the 1024 SIMDs, GRBM_GUI_ACTIVE over the 8 XCDs,
SQ_INSTS_VALU counting the MFMAs too.

  python tools/pmc_step_gemms.py gpurun_out/stepq/sq profiles/r06_pmc_step_gemms.json
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

SIMDS = 256 * 4
WANT = ("fc_x3_wide", "wgrad_x3w", "fc_bf16_p", "wgrad_bf16<")


def main(d, out):
    per = defaultdict(lambda: defaultdict(dict))  # kernel -> dispatch -> counter -> value
    ns = defaultdict(dict)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if not any(w in k for w in WANT):
                continue
            did = r.get("Dispatch_Id")
            per[k][did][r["Counter_Name"]] = float(r["Counter_Value"])
            if r.get("Start_Timestamp") and r.get("End_Timestamp"):
                ns[k][did] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    res = {"source": f"rocprofv3 --pmc over bench.py --profile-only (c2 training step), {d}", "kernels": {}}
    for k, disp in sorted(per.items()):
        names = set().union(*[set(v) for v in disp.values()])
        c = {n: sum(v.get(n, 0.0) for v in disp.values()) / len(disp) for n in names}
        t = sum(ns[k].values()) / len(ns[k]) if ns[k] else None
        der = {"launches": len(disp), "kernel_us": t / 1e3 if t else None}
        if t and c.get("GRBM_GUI_ACTIVE"):
            cyc = c["GRBM_GUI_ACTIVE"] / 8
            der["clock_GHz"] = cyc / t
            if "SQ_VALU_MFMA_BUSY_CYCLES" in c:
                der["mfma_util"] = c["SQ_VALU_MFMA_BUSY_CYCLES"] / SIMDS / cyc
        if c.get("SQ_INSTS_MFMA"):
            der["valu_insts_per_mfma"] = (c["SQ_INSTS_VALU"] - c["SQ_INSTS_MFMA"]) / c["SQ_INSTS_MFMA"]
        if c.get("SQ_WAVE_CYCLES"):
            wc = c["SQ_WAVE_CYCLES"]
            der["wave_cycles"] = {"active": c.get("SQ_ACTIVE_INST_ANY", 0) / wc,
                                  "wait_inst": c.get("SQ_WAIT_INST_ANY", 0) / wc,
                                  "wait_any": c.get("SQ_WAIT_ANY", 0) / wc}
        res["kernels"][k[:160]] = {"counters": c, "derived": der}
        print(f"{k[:110]:110s} n={len(disp):3d} us={der['kernel_us'] or 0:8.1f} "
              f"mfma={der.get('mfma_util', 0):.3f} valu/mfma={der.get('valu_insts_per_mfma', 0):.2f} "
              f"GHz={der.get('clock_GHz', 0):.2f}")
    json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main(*sys.argv[1:3])
