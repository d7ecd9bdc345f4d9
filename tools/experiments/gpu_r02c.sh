#!/bin/bash
# round-2 GPU session c: full GPU tests, then the c2 and c5 benches
mkdir -p gpurun_out && export TMPDIR=/tmp
run() {  # run <name> <timeout> <cmd...>: stops the session on a crash/abort/timeout (exit >= 2)
  local name=$1 tmo=$2; shift 2
  timeout -k 10 "$tmo" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  tail -3 "gpurun_out/$name.log"
  if [ $rc -ge 2 ]; then tail -30 "gpurun_out/$name.log"; exit $rc; fi
}
for s in ${*:-tests c2 c5}; do
  case $s in
    tests) run pytest_gpu 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread ;;
    c2) run bench_c2 600 python -u bench.py ;;
    c5) run bench_c5 600 python -u bench.py --config c5 --steps 10 --warmup 3 ;;
    kbf16) run kbench_bf16 400 python -u tools/kbench.py bf16 bf16bwd ;;
    mtests) run pytest_model 400 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_x3.py tests/test_gpu_partition.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread ;;
    c4n1) run bench_c4_n1 900 python -u bench.py --config c4 --steps 5 --warmup 2 ;;
    rehearse2)  # the N = 2 c4 bench path end to end, 2 ranks sharing this box's GPU over gloo
      LPGNN_DIST_BACKEND=gloo run rehearse_c4_n2 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
        --master-addr 127.0.0.1 --master-port 29600 bench.py --gpus 2 --steps 3 --warmup 1 ;;
    rehearse4)  # N = 4: four ranks sharing this box's GPU over gloo (three exchange peers per rank)
      LPGNN_DIST_BACKEND=gloo run rehearse_c4_n4 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
        --master-addr 127.0.0.1 --master-port 29601 bench.py --gpus 4 --steps 2 --warmup 1 ;;
    *) echo "unknown stage $s"; exit 2 ;;
  esac
done
