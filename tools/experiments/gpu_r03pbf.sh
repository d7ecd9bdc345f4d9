set -u
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_partition.py -k bf16 -x -v -s -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pbf_pytest.log 2>&1; rc=$?; tail -25 gpurun_out/pbf_pytest.log; exit $rc
