#!/bin/bash
# Kernel-trace summary of the c2 training step at HEAD (bench.py --profile-only); argument: output name.
set -u
NAME=${1:-r06_c2_step_kernels_final}
OUT=gpurun_out/c2prof
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run \
  -- python3 bench.py --steps 10 --warmup 3 --profile-only > "$OUT/c2.log" 2>&1
rc=$?
echo "c2 rc=$rc"
[ $rc -eq 0 ] || exit 3
python3 tools/prof_summary.py "$OUT/trace/run_kernel_stats.csv" "$OUT/$NAME"
