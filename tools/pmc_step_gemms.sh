#!/bin/bash
# One SQ/GRBM --pmc pass over the c2 training step (bench.py --profile-only), summarized per GEMM kernel
# instantiation by tools/pmc_step_gemms.py.  Arguments: a name for the outputs, then extra bench.py
# arguments (quoted), e.g.  bash tools/pmc_step_gemms.sh c5 "--config c5"
set -u
NAME=${1:-c2}
OUT=gpurun_out/stepq_$NAME
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES \
  SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE --output-format csv -d "$OUT/sq" -o run \
  -- python3 bench.py --steps 2 --warmup 1 --profile-only ${2:-} > "$OUT/sq.log" 2>&1
rc=$?
echo "sq rc=$rc"
[ $rc -eq 0 ] || exit 3
python3 tools/pmc_step_gemms.py "$OUT/sq" "$OUT/r06_pmc_step_gemms_$NAME.json"
