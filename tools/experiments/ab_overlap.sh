set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --sub "" --cpu-steps 0 --steps 40 > gpurun_out/ab_ov0_$i.log 2>&1
  LPGNN_OVERLAP=1 timeout -k 10 200 python bench.py --sub "" --cpu-steps 0 --steps 40 > gpurun_out/ab_ov1_$i.log 2>&1
done
grep -o "ms_per_step.: [0-9.]*" gpurun_out/ab_ov*_*.log | grep -v "4\.[0-9]*$"
