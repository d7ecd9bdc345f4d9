set -u
mkdir -p gpurun_out; export TMPDIR=/tmp
SQ="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE"
for c in "$SQ" FETCH_SIZE WRITE_SIZE; do
  n=$(echo $c | cut -c1-5)
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d gpurun_out/k2048/$n -o run -- python3 tools/experiments/x3_k2048_pmc.py > gpurun_out/k2048_$n.log 2>&1 || exit 3
done
python3 tools/pmc_kernel_summary.py gpurun_out/k2048/SQ_IN gpurun_out/k2048/FETCH gpurun_out/k2048/WRITE fc_x3_wide gpurun_out/k2048.json "x3 FC 200K x (1024+1024) -> 1024, ReLU (the VERDICT r02 item-5 shape)"
