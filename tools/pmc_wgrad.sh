#!/bin/bash
# PMC passes over the x3 weight-gradient kernel at the c2 shape (tools/wgrad_drive.py):
# SQ issue/wait counters + GRBM_GUI_ACTIVE (clock), then FETCH_SIZE, then WRITE_SIZE (separate passes).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmcw1 -o run -- python tools/wgrad_drive.py > gpurun_out/pmcw1.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcw2 -o run -- python tools/wgrad_drive.py > gpurun_out/pmcw2.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcw3 -o run -- python tools/wgrad_drive.py > gpurun_out/pmcw3.log 2>&1
echo rc=$?
