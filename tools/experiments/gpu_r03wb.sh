set -u
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_x3.py tests/test_gpu_bf16.py tests/test_gpu_model.py tests/test_gpu_model_degenerate.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/wb_pytest.log 2>&1; rc=$?; tail -4 gpurun_out/wb_pytest.log; [ $rc -ne 0 ] && exit $rc
for c in c2 c5; do
  timeout -k 10 300 python -u bench.py --config $c --cpu-steps 0 > gpurun_out/wb_bench_$c.log 2>&1 || exit $?
  tail -1 gpurun_out/wb_bench_$c.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', d['ms_per_step'], d['fc_roofline']['frac'], {k:round(v['ms']/d['steps'],3) for k,v in d['kernels'].items() if 'wgrad' in k})"
done
