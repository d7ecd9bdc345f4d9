set -u
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 240 python -u tools/experiments/x3_lda.py time > gpurun_out/lda_time.log 2>&1 || exit $?
for ld in 1024 1056; do
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/lda_f$ld -o run -- python3 tools/experiments/x3_lda.py one $ld > gpurun_out/lda_f$ld.log 2>&1 || exit 3
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/lda_w$ld -o run -- python3 tools/experiments/x3_lda.py one $ld > gpurun_out/lda_w$ld.log 2>&1 || exit 3
done
cat gpurun_out/lda_time.log | grep x3
