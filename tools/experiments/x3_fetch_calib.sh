#!/bin/bash
# FETCH_SIZE calibration for the x3 FC's W-plane reads: at M = 128 (one m-tile) every byte of the three
# 1024 x 2048 bf16 W planes (12.58 MB) is read by exactly one block and the A panel is 1 MB, so the raw
# FETCH_SIZE per launch says whether the W planes' 64-byte row segments are counted at half their bytes
# (like 16-B-per-lane 128-B lines, MI355X_MICROARCH.md) or in full.  Summary on stdout.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/x3calib; mkdir -p "$OUT"; export TMPDIR=/tmp
X3_M=128 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/m128" -o run -- \
  python3 tools/experiments/x3_k2048_pmc.py > "$OUT/m128.log" 2>&1
rc=$?; echo "m128 FETCH_SIZE rc=$rc"; [ $rc -eq 0 ] || exit 3
python3 - "$OUT/m128" <<'PY'
import os, sys
sys.path.insert(0, "tools")
from pmc_summary import read_counter
per = read_counter(sys.argv[1], "FETCH_SIZE")
vals = [v for k, vs in per.items() if "fc_x3_wide" in k for v in vs]
raw = sum(vals) / len(vals) * 1024
print(f"fc_x3_wide M=128: raw FETCH_SIZE {raw / 1e6:.2f} MB per launch over {len(vals)} launches; "
      f"W planes 12.58 MB + A panel 1.05 MB = 13.63 MB read once")
PY
