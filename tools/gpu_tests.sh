#!/bin/bash
# the whole -m gpu suite on one box (one pytest process), log under gpurun_out/
# PYTEST_K: a -k expression; PYTEST_FILES: test files (default: tests); PYTEST_MAXFAIL (default 1)
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest ${PYTEST_FILES:-tests} -m gpu --maxfail ${PYTEST_MAXFAIL:-1} -v -p no:cacheprovider \
  --timeout 300 --timeout-method thread -rf ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -30 gpurun_out/pytest_gpu.log
exit $rc
