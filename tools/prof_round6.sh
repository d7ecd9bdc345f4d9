#!/bin/bash
# Round-6 profiles at HEAD (one GPU): per-direction SpMM traffic (c2 + skewed), the c2 step's SpMM traffic
# (roofline.traffic), and the kernel-trace summary of the c2 and skewed training steps.  Each rocprofv3
# pass is its own run with its own time limit (MI355X_MICROARCH.md: FETCH_SIZE and WRITE_SIZE in separate
# --pmc passes); stops at the first failure.
set -u
OUT=gpurun_out/r6prof
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # run <name> <seconds> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -s KILL "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  [ $rc -eq 0 ] || exit 3
}
WL_C2=$(python3 bench.py --print-workload)
run dirs_f 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/dirs_f" -o run -- python3 tools/pmc_spmm_dirs.py run
run dirs_w 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/dirs_w" -o run -- python3 tools/pmc_spmm_dirs.py run
python3 tools/pmc_spmm_dirs.py summarize "$OUT/dirs_f" "$OUT/dirs_w" "$OUT/r06_pmc_dirs"
run c2_f 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/c2_f" -o run -- python3 bench.py --steps 2 --warmup 1 --profile-only
run c2_w 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/c2_w" -o run -- python3 bench.py --steps 2 --warmup 1 --profile-only
python3 tools/pmc_summary.py "$OUT/c2_f" "$OUT/c2_w" "$OUT/r06_pmc_spmm_c2.json" "$WL_C2" > "$OUT/pmc_c2_summary.log"
run trace_c2 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_c2" -o run -- python3 bench.py --steps 10 --warmup 3 --profile-only
python3 tools/prof_summary.py "$OUT/trace_c2/run_kernel_stats.csv" "$OUT/r06_c2_step_kernels"
run trace_sk 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_sk" -o run -- python3 bench.py --config skewed --steps 10 --warmup 3 --profile-only
python3 tools/prof_summary.py "$OUT/trace_sk/run_kernel_stats.csv" "$OUT/r06_skewed_step_kernels"
echo prof done
