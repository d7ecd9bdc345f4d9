#!/bin/bash
# Attribution of the x3 FC's past-L2 bytes at K = 2048: FETCH_SIZE / WRITE_SIZE of
# fc_x3_wide (tools/experiments/x3_k2048_pmc.py) on the default build and on two probe builds
#   var_x3p1: every block reads one W slice  -> the A panels' traffic (+ one 1.5 MB W slice)
#   var_x3p2: every block reads one A panel  -> the W slices' traffic (+ one 1 MB A panel)
# built on the CPU side with
#   make -C lp-gnn_amd OUT=../tools/experiments/var_x3p1/liblpgnn_hip.so OBJDIR=build_x3p1 EXTRA=-DLPG_X3_TRAFFIC_PROBE=1
#   make -C lp-gnn_amd OUT=../tools/experiments/var_x3p2/liblpgnn_hip.so OBJDIR=build_x3p2 EXTRA=-DLPG_X3_TRAFFIC_PROBE=2
#   order0: the library with LPG_FC_KERNEL(2), round 3's m-major tile order (the default is the n-split
#           order since round 4; the probe builds keep the m-major order)
# plus an SQ/GRBM pass (MFMA busy, clock) of the default.  Summary: gpurun_out/x3traffic/summary.json.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/x3traffic; mkdir -p "$OUT"; export TMPDIR=/tmp
VARIANTS=${VARIANTS:-"default x3p1 x3p2 order0"}
DRIVER=${DRIVER:-tools/experiments/x3_k2048_pmc.py}
for v in $VARIANTS; do
  unset X3_KERNEL
  if [ "$v" = default ]; then unset LPGNN_LIB
  elif [ "$v" = order0 ]; then unset LPGNN_LIB; export X3_KERNEL=2   # round 3's m-major tile order
  else export LPGNN_LIB="$PWD/tools/experiments/var_$v/liblpgnn_hip.so"; fi
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d "$OUT/${v}_$c" -o run -- python3 $DRIVER > "$OUT/${v}_$c.log" 2>&1
    rc=$?; echo "$v $c rc=$rc"; [ $rc -eq 0 ] || exit 3
  done
done
unset LPGNN_LIB X3_KERNEL
if [ -z "${NO_SQ:-}" ]; then
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA GRBM_GUI_ACTIVE --output-format csv -d "$OUT/default_sq" -o run \
    -- python3 $DRIVER > "$OUT/default_sq.log" 2>&1
  rc=$?; echo "default SQ rc=$rc"; [ $rc -eq 0 ] || exit 3
fi
python3 tools/experiments/x3_traffic_summary.py "$OUT" $VARIANTS
