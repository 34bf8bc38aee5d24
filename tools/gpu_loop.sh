set -u
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 700 python -m pytest tests -m gpu -q -x -k "${PYTEST_K:-gpu or not gpu}" > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
CFGS=${CFGS:-c3 c5} bash tools/gpu_loop_trace.sh
