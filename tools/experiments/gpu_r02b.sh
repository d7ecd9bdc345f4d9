#!/bin/bash
# round-2 GPU session b: the hand-written bf16 backward (wgrad_bf16, input grad on lpg_fc_bf16) and the
# pipelined bf16 FC variants -- tests, then kernel timings at the c5 shapes
mkdir -p gpurun_out && export TMPDIR=/tmp
run() {  # run <name> <timeout> <cmd...>: stops the session on a crash/abort/timeout (exit >= 2)
  local name=$1 tmo=$2; shift 2
  timeout -k 10 "$tmo" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ge 2 ]; then tail -30 "gpurun_out/$name.log"; exit $rc; fi
}
for s in ${*:-tests kb}; do
  case $s in
    tests) run bf16tests 400 python -u -m pytest tests/test_gpu_bf16.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread ;;
    kb) run kbench_bf16 400 python -u tools/kbench.py bf16 bf16bwd ;;
    c5) run bench_c5 600 python -u bench.py --config c5 --steps 10 --warmup 3 ;;
    profc5) run prof_c5 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5 -o run -- \
              python bench.py --config c5 --steps 3 --warmup 2 --profile-only ;;
    c5parity) run c5parity 900 python -u -m pytest tests/test_gpu_c2_parity.py -k c5 -v -s -p no:cacheprovider --timeout 900 --timeout-method thread ;;
    *) echo "unknown stage $s"; exit 2 ;;
  esac
done
