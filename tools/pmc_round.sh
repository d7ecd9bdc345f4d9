#!/bin/bash
# PMC passes at HEAD, one counter group per run (MI355X_MICROARCH.md HBM / rocprofv3 recipe):
# the hidden-width GEMMs (tools/experiments/pmc_gemms.py: SQ issue / MFMA busy / clock, FETCH_SIZE,
# WRITE_SIZE) and the SpMM traffic of the c2 training and inference steps.  Stops at the first
# pass that fails or times out.
set -u
OUT=gpurun_out/pmc
mkdir -p "$OUT"
export TMPDIR=/tmp
SQ="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE"
pass() {  # pass <name> <counters> -- <program...>
  local name=$1 counters=$2; shift 3
  timeout -s KILL 240 rocprofv3 --pmc $counters --output-format csv -d "$OUT/$name" -o run -- "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  [ $rc -eq 0 ] || exit 3
}
pass g_sq "$SQ" -- python3 tools/experiments/pmc_gemms.py
pass g_fetch FETCH_SIZE -- python3 tools/experiments/pmc_gemms.py
pass g_write WRITE_SIZE -- python3 tools/experiments/pmc_gemms.py
pass c2_fetch FETCH_SIZE -- python3 bench.py --steps 2 --warmup 1 --profile-only
pass c2_write WRITE_SIZE -- python3 bench.py --steps 2 --warmup 1 --profile-only
pass c2i_fetch FETCH_SIZE -- python3 bench.py --inference --steps 2 --warmup 1 --profile-only
pass c2i_write WRITE_SIZE -- python3 bench.py --inference --steps 2 --warmup 1 --profile-only
echo pmc done
