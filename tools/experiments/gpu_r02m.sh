#!/bin/bash
# packed relu_bwd8: bf16 tests, PMC of the folded input gradient, c5 A/B
set -u
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_bf16.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_bf16.log 2>&1 || { tail -30 gpurun_out/pytest_bf16.log; exit 1; }
tail -2 gpurun_out/pytest_bf16.log
bash tools/experiments/pmc_bf16.sh igm fc_bf16_p "bf16 input gradient + folded ReLU backward (packed mask), M=200K, 2x2048 -> 2048" > gpurun_out/pmc_igm.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 300 python bench.py --config c5 --steps 10 --warmup 3 > gpurun_out/bench_c5_p$i.log 2>&1 || exit $?
  LPGNN_FOLD_RELU_BWD=0 timeout -k 10 300 python bench.py --config c5 --steps 10 --warmup 3 > gpurun_out/bench_c5_nofold$i.log 2>&1 || exit $?
done
for f in gpurun_out/bench_c5_p*.log gpurun_out/bench_c5_nofold*.log; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $f)"; done
echo done
