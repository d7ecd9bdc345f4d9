#!/bin/bash
# One gloo rehearsal of the row-partitioned step (2 ranks sharing the GPU, c4 at 1/5 size), each
# rank under its own rocprofv3 kernel + memory-copy trace; then the per-rank step timeline.
# Ranks are started here with their env (no launcher re-exec under the profiler).
mkdir -p gpurun_out/trace && export TMPDIR=/tmp
ARGS="--gpus 2 --config c4 --m 400000 --n 800000 --nnz 8000000 --steps 2 --warmup 2 --profile-only --rho-sweep="
pids=()
for r in 0 1; do
  mkdir -p gpurun_out/trace/r$r
  RANK=$r LOCAL_RANK=$r WORLD_SIZE=2 LOCAL_WORLD_SIZE=2 MASTER_ADDR=127.0.0.1 MASTER_PORT=29571 \
  LPGNN_DIST_BACKEND=gloo LPGNN_TRACE_WINDOW=1 \
    timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv \
      -d gpurun_out/trace/r$r -o run -- python3 bench.py $ARGS > gpurun_out/trace/r$r/rank.log 2>&1 &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=$?; done
tail -3 gpurun_out/trace/r0/rank.log gpurun_out/trace/r1/rank.log
[ $rc -eq 0 ] || exit $rc
python3 tools/trace_timeline.py --steps 2 gpurun_out/trace/timeline.md gpurun_out/trace/r0 gpurun_out/trace/r1
