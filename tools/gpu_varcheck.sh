#!/bin/bash
# GPU: the parity core on one variant build (VARLIB), then the interleave-free
# A/B of variants (tools/gpu_var.sh: VARS, AB_VARIANTS).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
DRL_LIB=$VARLIB timeout -k 10 500 python -m pytest tests/test_gpu_parity.py -q --maxfail=3 \
  -k "trajectory or rollout or full_size or ragged or streaming or kat or compat or obs_variants or shard" \
  > gpurun_out/pytest_var.log 2>&1
rc=$?; echo "variant pytest ($VARLIB) rc=$rc"; tail -2 gpurun_out/pytest_var.log
[ $rc -le 1 ] || exit $rc
bash tools/gpu_var.sh
