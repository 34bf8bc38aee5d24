#!/bin/bash
# GPU: full parity suite on the default build, the parity core on a variant
# build (VARLIB), then interleave-free A/B of variants (tools/gpu_var.sh).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q --maxfail=5 > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
if [ -n "${VARLIB:-}" ]; then
  DRL_LIB=$VARLIB timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q --maxfail=5 \
    -k "trajectory or rollout_matches or full_size or ragged or streaming" > gpurun_out/pytest_var.log 2>&1
  rc=$?; echo "variant pytest ($VARLIB) rc=$rc"; tail -3 gpurun_out/pytest_var.log
  [ $rc -le 1 ] || exit $rc
fi
bash tools/gpu_var.sh
