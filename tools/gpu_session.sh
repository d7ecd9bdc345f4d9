#!/bin/bash
# One GPU-box session: parity tests -> smoke -> bench -> rocprofv3 kernel stats.
# Usage (from the repo root, via gpurun):  bash tools/gpu_session.sh [stages...]
# stages: tests tests_files smoke bench prof pmc bench_c5 prof_c5 kbench kbfc mfma x3traffic rehearse2/8 pmc_rs   (default: tests smoke bench prof)
# Every GPU step has its own time limit; the script stops at the first step
# that crashes, aborts or times out (exit >= 2 or signal), and continues past
# a plain test failure (exit 1) so the bench still runs.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
export TMPDIR=/tmp
export HSA_ENABLE_IPC_MODE_LEGACY=0
STAGES="${*:-tests smoke bench prof}"

step() {  # step <name> <timeout> <cmd...>
  local name=$1 tmo=$2; shift 2
  echo "=== $name: $*" | tee -a "$OUT/session.log"
  local t0=$(date +%s)
  timeout -k 10 "$tmo" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name exit=$rc ($(( $(date +%s) - t0 ))s)" | tee -a "$OUT/session.log"
  tail -n 25 "$OUT/$name.log"
  if [ $rc -ge 2 ]; then
    echo "stopping after $name (exit $rc)" | tee -a "$OUT/session.log"
    exit $rc
  fi
  return 0
}

rocminfo 2>/dev/null | grep -m2 -E "gfx950|Marketing" > "$OUT/device.txt" || true
for s in $STAGES; do
  case $s in
    tests) step pytest_gpu 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread ;;
    tests_files)  # PYTEST_FILES (space-separated), every failure reported (maxfail PYTEST_MAXFAIL, default 30)
      step pytest_files 700 python -u -m pytest ${PYTEST_FILES} -m gpu --maxfail ${PYTEST_MAXFAIL:-30} -v \
        -p no:cacheprovider -rf --timeout 120 --timeout-method thread ;;
    tests_s)  # the whole -m gpu suite with -s (the parity tests print their measured counts), every failure reported
      step pytest_s 900 python -u -m pytest tests -m gpu -s --maxfail ${PYTEST_MAXFAIL:-30} -v -p no:cacheprovider -rf \
        --timeout 300 --timeout-method thread ;;
    tests_all)  # the whole -m gpu suite, every failure reported
      step pytest_all 800 python -u -m pytest tests -m gpu --maxfail ${PYTEST_MAXFAIL:-30} -v -p no:cacheprovider -rf \
        --timeout 300 --timeout-method thread ;;
    x3traffic) step x3traffic 420 bash tools/experiments/x3_traffic_probe.sh ;;
    x3calib) step x3calib 180 bash tools/experiments/x3_fetch_calib.sh ;;
    x3ab) step x3ab 300 python tools/experiments/x3_order_ab.py ;;
    bf16ab) step bf16ab 300 python tools/experiments/bf16_order_ab.py ;;
    smoke) step smoke 600 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 900 python bench.py ;;
    prof)
      step prof 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
        python "$ROOT/bench.py" --steps 5 --warmup 2 --profile-only
      ;;
    bench_part) step bench_part 600 python bench.py --partitioned --sub "" --cpu-steps 0 ;;  # N = 1 through the N > 1 path
    bench_c5_nobits) LPGNN_RELU_BITS=0 step bench_c5_nobits 900 python bench.py --config c5 --steps 10 --warmup 3 ;;
    bench_c5_nodb) LPGNN_FOLD_BIAS_SUMS=0 step bench_c5_nodb 900 python bench.py --config c5 --steps 10 --warmup 3 ;;
    bench_c5) step bench_c5 900 python bench.py --config c5 --steps 10 --warmup 3 ;;
    bench_inf) step bench_inf 600 python bench.py --inference ;;
    bench_c4) step bench_c4 900 python bench.py --config c4 --steps 5 --warmup 2 --cpu-steps 0 ;;
    prof_c5)
      step prof_c5 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c5" -o run -- \
        python "$ROOT/bench.py" --config c5 --steps 3 --warmup 2 --profile-only
      ;;
    kbench) step kbench 600 python tools/kbench.py ;;
    rehearse8)  # the N = 8 topology: 8 self-launched ranks sharing the GPU over gloo, 1/10 sizes
      step rehearse8 900 python bench.py --gpus 8 --share-gpu --steps 2 --warmup 1 --m 10000 --n 20000 \
        --nnz 200000 --c4-scale 10 --c4-steps 2 --c4-warmup 1 ;;
    rehearse2)
      step rehearse2 900 python bench.py --gpus 2 --share-gpu --steps 3 --warmup 1 --c4-scale 10 ;;
    pmc_rs) step pmc_rs 1200 bash tools/pmc_rank_shares.sh ;;
    tests_part) step pytest_part 900 python -u -m pytest tests/test_gpu_partition.py -m gpu -x -v -p no:cacheprovider \
        --timeout 900 --timeout-method thread ;;
    mfma) step mfma_peak 120 tools/experiments/mfma_peak 3 ;;  # sustained bf16 MFMA rate (build: see the source)
    kbfc) step kbench_fc 600 python tools/kbench.py fc ;;
    pmc)
      step pmc_fetch 900 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- \
        python "$ROOT/bench.py" --steps 3 --warmup 1 --profile-only
      step pmc_write 900 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- \
        python "$ROOT/bench.py" --steps 3 --warmup 1 --profile-only
      python tools/pmc_summary.py "$OUT/pmc_fetch" "$OUT/pmc_write" "$OUT/pmc_spmm.json" \
        "$(python bench.py --print-workload)" || true
      ;;
    pmc_inf16)  # the fp16 inference sub-record's SpMM traffic
      step pmc_fetch_inf16 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch_inf16" -o run -- \
        python "$ROOT/bench.py" --inference --fp16 --steps 3 --warmup 1 --profile-only
      step pmc_write_inf16 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write_inf16" -o run -- \
        python "$ROOT/bench.py" --inference --fp16 --steps 3 --warmup 1 --profile-only
      python tools/pmc_summary.py "$OUT/pmc_fetch_inf16" "$OUT/pmc_write_inf16" "$OUT/r04_pmc_spmm_inference_fp16.json" \
        "$(python bench.py --inference --fp16 --print-workload)" || true
      ;;
    pmc_c5)
      step pmc_fetch_c5 900 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch_c5" -o run -- \
        python "$ROOT/bench.py" --config c5 --steps 2 --warmup 1 --profile-only
      step pmc_write_c5 900 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write_c5" -o run -- \
        python "$ROOT/bench.py" --config c5 --steps 2 --warmup 1 --profile-only
      python tools/pmc_summary.py "$OUT/pmc_fetch_c5" "$OUT/pmc_write_c5" "$OUT/pmc_spmm_c5.json" \
        "$(python bench.py --config c5 --print-workload)" || true
      ;;
    *) echo "unknown stage $s"; exit 2 ;;
  esac
done
echo "session done"
