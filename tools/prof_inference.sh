#!/bin/bash
# Kernel-trace summaries of the reference's timed path on c2 (eval forward + inference_gnn), fp32 and the
# fp16 mode: bench.py --inference [--fp16] --profile-only under rocprofv3 --kernel-trace --stats.
set -u
OUT=gpurun_out/infprof
mkdir -p "$OUT"
export TMPDIR=/tmp
for mode in fp32 fp16; do
  extra=""; [ $mode = fp16 ] && extra="--fp16"
  timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$mode" -o run \
    -- python3 bench.py --inference $extra --steps 20 --warmup 3 --profile-only > "$OUT/$mode.log" 2>&1
  rc=$?
  echo "$mode rc=$rc"
  [ $rc -eq 0 ] || exit 3
  python3 tools/prof_summary.py "$OUT/$mode/run_kernel_stats.csv" "$OUT/r06_inference_${mode}_kernels"
done
