#!/bin/bash
# FETCH_SIZE calibration per access width (tools/fetch_calib.hip), then the
# validation tests and a default bench line with its in-run PMC traffic.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/calib
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/calib/fetch -o run --output-format csv -- ./tools/fetch_calib.bin > gpurun_out/calib/fetch.log 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/calib/trace -o run --output-format csv -- ./tools/fetch_calib.bin > gpurun_out/calib/trace.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest tests/test_gpu_validation.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_validation.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --steps 200 --warmup 20 --cpu-seconds 5 > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
echo ok
