#!/bin/bash
# GPU parity tests then interleaved A/B of kernel variants (tools/ab.py).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 ${PYTEST_TIMEOUT:-700} python -m pytest tests -m gpu -q --maxfail=${MAXFAIL:-5} ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
for c in ${AB_CONFIGS:-c3 c4 c5}; do
  timeout -k 10 300 python tools/ab.py --config $c --rounds ${AB_ROUNDS:-5} --steps ${AB_STEPS:-100} ${AB_VARIANTS:+--variants $AB_VARIANTS} >> gpurun_out/ab.log 2>&1 || exit $?
done
cat gpurun_out/ab.log
