set -u
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_model_degenerate.py tests/test_gpu_basis.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/deg_pytest.log 2>&1; rc=$?; tail -15 gpurun_out/deg_pytest.log; exit $rc
