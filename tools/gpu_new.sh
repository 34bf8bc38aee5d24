#!/bin/bash
# The tests added this round, then the default bench line (with its in-run PMC traffic).
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_validation.py tests/test_gpu_fullsize.py} -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_new.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_new.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
[ -n "${NOBENCH:-}" ] && exit $rc
timeout -k 10 600 python bench.py --steps 200 --warmup 20 --cpu-seconds 5 > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
echo ok
