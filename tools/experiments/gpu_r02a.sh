#!/bin/bash
# round-2 GPU session: c5 parity, partition tests, c4 at N=1 (whole graph, and through the partitioned path)
mkdir -p gpurun_out && export TMPDIR=/tmp
run() {  # run <name> <timeout> <cmd...>: stops the session on a crash/abort/timeout (exit >= 2)
  local name=$1 tmo=$2; shift 2
  timeout -k 10 "$tmo" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ge 2 ]; then tail -20 "gpurun_out/$name.log"; exit $rc; fi
}
run c5parity 900 python -u -m pytest tests/test_gpu_c2_parity.py -k c5 -v -s -p no:cacheprovider --timeout 900 --timeout-method thread
run gpart 300 python -u -m pytest tests/test_gpu_partition.py -v -p no:cacheprovider --timeout 200 --timeout-method thread
run c4_n1 400 python -u bench.py --config c4 --steps 5 --warmup 2
run c4_part1 400 python -u bench.py --config c4 --partitioned --steps 5 --warmup 2
