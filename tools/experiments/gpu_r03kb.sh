set -u
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_fc.py tests/test_gpu_model.py tests/test_gpu_model_degenerate.py tests/test_gpu_c2_parity.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/kb_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/kb_pytest.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do timeout -k 10 300 python -u bench.py --cpu-steps 0 > gpurun_out/kb_bench.log 2>&1 || exit $?; tail -1 gpurun_out/kb_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2', round(d['ms_per_step'],2))"; done
