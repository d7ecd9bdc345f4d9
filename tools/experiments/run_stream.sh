#!/bin/bash
# kbench stream on the default library and each variant of build_stream_variants.sh
set -eo pipefail
mkdir -p gpurun_out
for v in default u8 r64 r256; do
  if [ $v = default ]; then lib=""; else lib=$PWD/tools/experiments/var_$v/liblpgnn_hip.so; fi
  echo "== $v" | tee -a gpurun_out/stream.log
  LPGNN_LIB=$lib timeout -k 10 180 python -u tools/kbench.py stream 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/stream.log
done
