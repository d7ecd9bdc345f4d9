set -u
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 240 python -u tools/experiments/wgrad_q.py w > gpurun_out/q_time0.log 2>&1 || exit $?
LPGNN_WGRAD_KERNEL=1 timeout -k 10 240 python -u tools/experiments/wgrad_q.py q > gpurun_out/q_time1.log 2>&1 || exit $?
grep wgrad_x3 gpurun_out/q_time*.log
