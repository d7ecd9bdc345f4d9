#!/bin/bash
# PMC of the c5 input gradient with and without the folded ReLU backward
set -u
bash tools/experiments/pmc_bf16.sh ig fc_bf16_p "bf16 input gradient, M=200K, 2x2048 -> 2048" || exit $?
bash tools/experiments/pmc_bf16.sh igm fc_bf16_p "bf16 input gradient + folded ReLU backward, M=200K, 2x2048 -> 2048" || exit $?
cat gpurun_out/pmc_bf16_ig.json gpurun_out/pmc_bf16_igm.json
