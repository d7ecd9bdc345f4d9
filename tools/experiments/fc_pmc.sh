#!/bin/bash
# PMC passes over the two hidden-layer FC kernels (tools/kbench.py fcpmc):
# MFMA busy, clocks, LDS bank conflicts, L2 hit rate.  One counter group per pass.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/fcpmc"
mkdir -p "$OUT"
export TMPDIR=/tmp
rocprofv3 --list-avail > "$OUT/avail.txt" 2>&1 || true
i=0
for grp in "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES" \
           "SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS" \
           "TCC_HIT_sum TCC_MISS_sum" \
           "SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o run -- \
    python "$ROOT/tools/kbench.py" fcpmc > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "pass $i ($grp) rc=$rc"
  if [ $rc -ge 2 ] && [ $rc -ne 2 ]; then exit $rc; fi
done
