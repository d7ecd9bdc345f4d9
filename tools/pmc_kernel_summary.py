"""Derived issue / clock / HBM metrics of one kernel from three rocprofv3 --pmc
passes (SQ + GRBM counters, FETCH_SIZE, WRITE_SIZE; tools/pmc_wgrad.sh).

  python tools/pmc_kernel_summary.py gpurun_out/pmcw1 gpurun_out/pmcw2 gpurun_out/pmcw3 \
      wgrad_x3c profiles/r01_pmc_wgrad_x3.json "<description>"

Counter units and corrections: MI355X_MICROARCH.md (SQ_* wave counters in
quad-cycles, SQ_VALU_MFMA_BUSY_CYCLES in cycles summed over the 1024 SIMDs,
GRBM_GUI_ACTIVE summed over the 8 XCDs, FETCH_SIZE halved on gfx950 for wide
coalesced reads, KiB units).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

SIMDS = 256 * 4


def read(d, want):
    vals, ns = defaultdict(list), []
    seen = set()
    for f in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if want not in r["Kernel_Name"]:
                continue
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
            did = r.get("Dispatch_Id")
            if did not in seen and r.get("Start_Timestamp") and r.get("End_Timestamp"):
                seen.add(did)
                ns.append(float(r["End_Timestamp"]) - float(r["Start_Timestamp"]))
    mean = {k: sum(v) / len(v) for k, v in vals.items()}
    return mean, (sum(ns) / len(ns) if ns else None)


def main(d1, d2, d3, want, out, desc):
    c, t1 = read(d1, want)
    f, t2 = read(d2, want)
    w, t3 = read(d3, want)
    res = {"kernel": desc, "source": "rocprofv3 --pmc passes (tools/pmc_wgrad.sh), averages over the launches"}
    res.update(c)
    res.update(f)
    res.update(w)
    res.update(pmc1_kernel_ns=t1, pmc2_kernel_ns=t2, pmc3_kernel_ns=t3)
    der = {}
    if t1 and "GRBM_GUI_ACTIVE" in c:
        cyc = c["GRBM_GUI_ACTIVE"] / 8
        der["clock_GHz (GRBM_GUI_ACTIVE/8/t)"] = cyc / t1
        if "SQ_VALU_MFMA_BUSY_CYCLES" in c:
            der["mfma_util (MFMA busy cycles per SIMD / kernel cycles)"] = c["SQ_VALU_MFMA_BUSY_CYCLES"] / SIMDS / cyc
    if c.get("SQ_INSTS_MFMA"):
        der["valu_insts_per_mfma"] = (c["SQ_INSTS_VALU"] - c["SQ_INSTS_MFMA"]) / c["SQ_INSTS_MFMA"]
    if c.get("SQ_WAVE_CYCLES"):
        wc = c["SQ_WAVE_CYCLES"]
        der["wave_cycle_split"] = {"active": c.get("SQ_ACTIVE_INST_ANY", 0) / wc,
                                   "wait_inst (pipe busy / dependency)": c.get("SQ_WAIT_INST_ANY", 0) / wc,
                                   "wait_any (waitcnt / barrier)": c.get("SQ_WAIT_ANY", 0) / wc}
    if "FETCH_SIZE" in f and "WRITE_SIZE" in w:
        der["hbm_side_bytes (2*FETCH_SIZE+WRITE_SIZE KiB, gfx950 correction)"] = \
            (2 * f["FETCH_SIZE"] + w["WRITE_SIZE"]) * 1024.0
    res["derived"] = der
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(der, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:7])
