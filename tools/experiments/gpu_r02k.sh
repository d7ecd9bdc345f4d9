#!/bin/bash
# folded ReLU backward, mask loads interleaved with the image writes: bf16 tests, c5 A/B x2
set -u
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_bf16.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_bf16.log 2>&1 || { tail -30 gpurun_out/pytest_bf16.log; exit 1; }
tail -2 gpurun_out/pytest_bf16.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --config c5 --steps 10 --warmup 3 > gpurun_out/bench_c5_k$i.log 2>&1 || exit $?
  LPGNN_FOLD_RELU_BWD=0 timeout -k 10 300 python bench.py --config c5 --steps 10 --warmup 3 > gpurun_out/bench_c5_nofold$i.log 2>&1 || exit $?
done
for f in gpurun_out/bench_c5_k*.log gpurun_out/bench_c5_nofold*.log; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $f)"; done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5 -o run -- python bench.py --config c5 --steps 3 --warmup 2 --profile-only > gpurun_out/prof_c5.log 2>&1 || exit $?
echo done
