set -u
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_x3.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pers_pytest.log 2>&1; rc=$?; tail -4 gpurun_out/pers_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u tools/kbench.py x3kern > gpurun_out/pers_kbench.log 2>&1 || exit $?
grep x3kern gpurun_out/pers_kbench.log
