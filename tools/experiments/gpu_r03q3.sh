# PMC (SQ issue / MFMA busy / clock, FETCH_SIZE, WRITE_SIZE) of the two x3 weight-gradient kernels
set -u
mkdir -p gpurun_out; export TMPDIR=/tmp
SQ="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE"
for k in 0 1; do
  export LPGNN_WGRAD_KERNEL=$k
  for c in "$SQ" FETCH_SIZE WRITE_SIZE; do
    n=$(echo $c | cut -c1-5)
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d gpurun_out/wq_pmc$k/$n -o run -- python3 tools/experiments/wgrad_pmc.py > gpurun_out/wq_pmc${k}_$n.log 2>&1 || exit 3
  done
done
python3 tools/pmc_kernel_summary.py gpurun_out/wq_pmc0/SQ_IN gpurun_out/wq_pmc0/FETCH gpurun_out/wq_pmc0/WRITE wgrad_x3w gpurun_out/wq_pmc0.json "wgrad_x3w R=100K 1024x1024"
python3 tools/pmc_kernel_summary.py gpurun_out/wq_pmc1/SQ_IN gpurun_out/wq_pmc1/FETCH gpurun_out/wq_pmc1/WRITE wgrad_x3q gpurun_out/wq_pmc1.json "wgrad_x3q R=100K 1024x1024"
