#!/bin/bash
# PMC passes over the x3 weight-gradient kernel at the c2 shape (tools/experiments/wgrad_drive.py, variant
# $LPG_WGV, kernel name filter $LPG_WGK): SQ issue/wait counters + GRBM_GUI_ACTIVE (clock), then
# FETCH_SIZE, then WRITE_SIZE (separate passes), summarised into gpurun_out/pmc_wgrad_$LPG_WGV.json.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
V=${LPG_WGV:-102}; K=${LPG_WGK:-wgrad_x3}
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmcw1_$V -o run -- python tools/experiments/wgrad_drive.py > gpurun_out/pmcw1_$V.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcw2_$V -o run -- python tools/experiments/wgrad_drive.py > gpurun_out/pmcw2_$V.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcw3_$V -o run -- python tools/experiments/wgrad_drive.py > gpurun_out/pmcw3_$V.log 2>&1
rc=$?
echo rc=$rc
[ $rc -eq 0 ] && python tools/pmc_kernel_summary.py gpurun_out/pmcw1_$V gpurun_out/pmcw2_$V gpurun_out/pmcw3_$V $K gpurun_out/pmc_wgrad_$V.json "x3 weight gradient variant $V, R=200000 N=K=1024 (tools/experiments/wgrad_drive.py)"
exit $rc
