#!/bin/bash
# PMC passes over one c5 bf16 GEMM kernel (tools/experiments/bf16_drive.py fc | wg): SQ issue/wait counters +
# GRBM_GUI_ACTIVE (clock), then FETCH_SIZE, then WRITE_SIZE (separate passes), summarised by
# tools/pmc_kernel_summary.py into gpurun_out/pmc_bf16_$W.json.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
W=${1:-fc}; K=${2:-fc_bf16_p}; DESC=${3:-bf16 GEMM}
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmcb1_$W -o run -- python tools/experiments/bf16_drive.py $W > gpurun_out/pmcb1_$W.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcb2_$W -o run -- python tools/experiments/bf16_drive.py $W > gpurun_out/pmcb2_$W.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcb3_$W -o run -- python tools/experiments/bf16_drive.py $W > gpurun_out/pmcb3_$W.log 2>&1
rc=$?
echo rc=$rc
[ $rc -eq 0 ] && python tools/pmc_kernel_summary.py gpurun_out/pmcb1_$W gpurun_out/pmcb2_$W gpurun_out/pmcb3_$W $K gpurun_out/pmc_bf16_$W.json "$DESC"
exit $rc
