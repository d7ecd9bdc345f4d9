#!/bin/bash
# Same-box A/B of two builds of the library on the c2 training step: the in-tree build against a
# baseline build (LPGNN_LIB), alternating, N rounds each.
#   bash tools/experiments/ab_lib.sh ab/base.so 3 [bench args...]
set -u
BASE=$1; N=$2; shift 2
mkdir -p gpurun_out
for i in $(seq 1 "$N"); do
  for v in base new; do
    if [ $v = base ]; then export LPGNN_LIB=$BASE; else unset LPGNN_LIB; fi
    timeout -k 10 200 python bench.py --cpu-steps 0 --sub "" --vendor 0 "$@" > gpurun_out/ab_$v.log 2>&1 || exit 1
    tail -1 gpurun_out/ab_$v.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$v', d['ms_per_step'], d['fc_roofline']['frac'])"
  done
done
