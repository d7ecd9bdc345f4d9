set -u
mkdir -p gpurun_out; export TMPDIR=/tmp
LPGNN_WGRAD_KERNEL=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_x3.py -k wgrad -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/q_pytest.log 2>&1; rc=$?; tail -5 gpurun_out/q_pytest.log; [ $rc -ge 2 ] && exit $rc
timeout -k 10 240 python -u tools/experiments/wgrad_q.py w > gpurun_out/q_time0.log 2>&1 || exit $?
LPGNN_WGRAD_KERNEL=1 timeout -k 10 240 python -u tools/experiments/wgrad_q.py q > gpurun_out/q_time1.log 2>&1 || exit $?
grep wgrad_x3 gpurun_out/q_time*.log
