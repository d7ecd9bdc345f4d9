#!/bin/bash
# Builds liblpgnn_hip.so variants of the streaming kernels' row-block sizes / unrolls
# (bwd.hip, fc.hip re-compiled with -D knobs, every other object from the default build)
# into tools/experiments/var_<name>/ for `LPGNN_LIB=... python tools/kbench.py stream`.
set -euo pipefail
cd "$(dirname "$0")/../../lp-gnn_amd"
make -s >/dev/null
FLAGS="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -Wall -I../include -Icsrc"
build() {
  local name=$1; shift
  local d=../tools/experiments/var_$name; mkdir -p $d
  /opt/rocm/bin/hipcc $FLAGS "$@" -c -o $d/bwd.o csrc/bwd.hip &
  /opt/rocm/bin/hipcc $FLAGS -mllvm -amdgpu-mfma-vgpr-form "$@" -c -o $d/fc.o csrc/fc.hip &
  wait
  objs=$(ls build/*.o | grep -v -e '/bwd.hip.o' -e '/fc.hip.o')
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $d/liblpgnn_hip.so $objs $d/bwd.o $d/fc.o
  rm -f $d/*.o
  echo "built $d"
}
build u8 -DLPG_LINEAR_UNROLL=8 -DLPG_WGRAD_UNROLL=16 -DLPG_SMALLK_ROWS=128
build r64 -DLPG_LINEAR_ROWS=64 -DLPG_WGRAD_ROWS=128 -DLPG_SMALLK_ROWS=32
build r256 -DLPG_LINEAR_ROWS=256 -DLPG_LINEAR_UNROLL=8 -DLPG_WGRAD_ROWS=512 -DLPG_SMALLK_ROWS=16
