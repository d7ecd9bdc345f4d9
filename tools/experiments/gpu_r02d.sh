#!/bin/bash
# FC launch time vs M around one block round (tail quantisation) and the x3 weight gradient vs R / split count
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u tools/kbench.py tail > gpurun_out/kbench_tail.log 2>&1 || exit $?
for S in 16 64 128; do
  LPGNN_WGRAD_SPLITS=$S timeout -k 10 200 python -u -c "
import sys; sys.path[:0]=['tools']
import kbench, json
out={}
from lpgnn.fc import wgrad
import torch
for R in (100_000, 200_000):
    G=torch.randn(R,1024,device='cuda'); X=torch.randn(R,1024,device='cuda')
    t=kbench.timeit({'f': lambda: wgrad(G,X,arith='x3')}, rounds=7, iters=4)['f']
    print(json.dumps({'R':R,'splits':$S,'ms':t,'tflops':2.0*R*1024*1024/t/1e9}))
" >> gpurun_out/kbench_tail.log 2>&1 || exit $?
done
cat gpurun_out/kbench_tail.log | grep -v Warning
