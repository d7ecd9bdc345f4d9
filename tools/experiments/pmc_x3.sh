#!/bin/bash
# PMC passes over the x3 FC kernel at the c2 hidden-layer shape (tools/experiments/x3_drive.py, variant
# $LPG_X3V): SQ issue/wait counters + GRBM_GUI_ACTIVE (clock), then FETCH_SIZE, then WRITE_SIZE
# (separate passes), summarised by tools/pmc_kernel_summary.py into gpurun_out/pmc_x3_v$LPG_X3V.json.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
V=${LPG_X3V:-0}; K=${LPG_X3K:-fc_x3_wide}
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc1_v$V -o run -- python tools/experiments/x3_drive.py x3 > gpurun_out/pmc1_v$V.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc2_v$V -o run -- python tools/experiments/x3_drive.py x3 > gpurun_out/pmc2_v$V.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc3_v$V -o run -- python tools/experiments/x3_drive.py x3 > gpurun_out/pmc3_v$V.log 2>&1
rc=$?
echo rc=$rc
[ $rc -eq 0 ] && python tools/pmc_kernel_summary.py gpurun_out/pmc1_v$V gpurun_out/pmc2_v$V gpurun_out/pmc3_v$V $K gpurun_out/pmc_x3_v$V.json "x3 FC variant $V, M=200000 N=1024 K=1024+1024, ReLU (tools/experiments/x3_drive.py)"
exit $rc
