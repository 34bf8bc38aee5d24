#!/bin/bash
# One GPU session: parity tests, smoke, short bench.  Stops after any crash,
# abort or timeout (exit codes other than 0/1 from pytest).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 ${PYTEST_TIMEOUT:-700} python -m pytest tests -m gpu -q --maxfail=${MAXFAIL:-10} ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?
echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py ${BENCH_ARGS:---steps 200 --warmup 20 --cpu-seconds 5} > gpurun_out/bench.log 2>&1
rc=$?
echo "bench rc=$rc"; tail -3 gpurun_out/bench.log
exit $rc
