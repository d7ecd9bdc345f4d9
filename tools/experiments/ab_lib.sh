#!/bin/bash
# Same-box A/B of library builds on a training step: each named build (LPGNN_LIB; "tree" = the in-tree
# build) alternating, N rounds, printing ms/step and fc_roofline.frac.
#   bash tools/experiments/ab_lib.sh 3 "tree ab/variant.so" [bench args...]
set -u
N=$1; LIBS=$2; shift 2
mkdir -p gpurun_out
for i in $(seq 1 "$N"); do
  for v in $LIBS; do
    if [ "$v" = tree ]; then unset LPGNN_LIB; else export LPGNN_LIB=$v; fi
    timeout -k 10 300 python bench.py --cpu-steps 0 --sub "" --vendor 0 "$@" > gpurun_out/ab_run.log 2>&1 || exit 1
    tail -1 gpurun_out/ab_run.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$v', d['ms_per_step'], d['fc_roofline']['frac'])"
  done
done
