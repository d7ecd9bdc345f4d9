#!/bin/bash
# PMC passes over the f16x2 GEMMs (f16x2_pmc.py): issue mix, MFMA busy, LDS, L2.  One group per run.
set -u
OUT=gpurun_out/f16pmc
mkdir -p "$OUT"
export TMPDIR=/tmp
pass() {  # pass <name> <counters...>
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- python3 tools/experiments/f16x2_pmc.py > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  [ $rc -eq 0 ] || exit 3
}
pass sq SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE
pass lds SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
pass l2 TCC_HIT_sum TCC_MISS_sum
pass fetch FETCH_SIZE
echo pmc done
