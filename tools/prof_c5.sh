#!/bin/bash
# Kernel-trace summary of the c5 training step (bench.py --config c5 --profile-only).
set -u
OUT=gpurun_out/c5prof
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -s KILL 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run \
  -- python3 bench.py --config c5 --steps 5 --warmup 2 --profile-only > "$OUT/c5.log" 2>&1
rc=$?
echo "c5 rc=$rc"
[ $rc -eq 0 ] || exit 3
python3 tools/prof_summary.py "$OUT/trace/run_kernel_stats.csv" "$OUT/r06_c5_step_kernels"
