#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes (separate runs, MI355X_MICROARCH.md HBM recipe) for the bench
# sub-records' SpMM traffic: the skewed workload and c5.  One counter per run; stops at the first
# failure.  Summarise with tools/pmc_summary.py (gfx950 FETCH_SIZE x 2 correction).
set -u
OUT=gpurun_out/pmc_sub
mkdir -p "$OUT"
export TMPDIR=/tmp
pass() {  # pass <name> <counter> -- <program...>
  local name=$1 counters=$2; shift 3
  timeout -s KILL 240 rocprofv3 --pmc $counters --output-format csv -d "$OUT/$name" -o run -- "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  [ $rc -eq 0 ] || exit 3
}
pass sk_fetch FETCH_SIZE -- python3 bench.py --config skewed --steps 2 --warmup 1 --profile-only
pass sk_write WRITE_SIZE -- python3 bench.py --config skewed --steps 2 --warmup 1 --profile-only
pass c5_fetch FETCH_SIZE -- python3 bench.py --config c5 --steps 2 --warmup 1 --profile-only
pass c5_write WRITE_SIZE -- python3 bench.py --config c5 --steps 2 --warmup 1 --profile-only
echo pmc done
