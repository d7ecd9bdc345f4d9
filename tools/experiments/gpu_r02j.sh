#!/bin/bash
# conv1 narrow FC with per-launch epilogue choices: FC tests, stream kbench, c2 bench x2
set -u
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_fc.py tests/test_gpu_model.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_fc.log 2>&1 || { tail -30 gpurun_out/pytest_fc.log; exit 1; }
tail -2 gpurun_out/pytest_fc.log
timeout -k 10 300 python -u tools/kbench.py stream > gpurun_out/kbench_stream.log 2>&1 || exit $?
grep stream gpurun_out/kbench_stream.log
for i in 1 2; do
  timeout -k 10 300 python bench.py > gpurun_out/bench_c2_$i.log 2>&1 || exit $?
  grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_c2_$i.log
done
echo done
