#!/bin/bash
# the whole -m gpu suite on one box (one pytest process), log under gpurun_out/
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -rf ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -30 gpurun_out/pytest_gpu.log
exit $rc
