set -u
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_x3.py tests/test_gpu_basis.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/ho_pytest.log 2>&1; rc=$?; tail -4 gpurun_out/ho_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --inference --cpu-steps 0 > gpurun_out/ho_bench_inf.log 2>&1 || exit $?
tail -1 gpurun_out/ho_bench_inf.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], {k:round(v['ms']/d['steps'],3) for k,v in d['kernels'].items()})"
