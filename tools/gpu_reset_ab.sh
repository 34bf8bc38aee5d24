#!/bin/bash
# GPU: reset parity tests on a variant build (VARLIB), then resets/s of the
# wave kernel for each build in VARS (tools/var_<v>.so), alternating, two rounds.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
DRL_LIB=$VARLIB timeout -k 10 400 python -m pytest tests/test_gpu_parity.py -q --maxfail=3 -k "reset or trajectory or full_size" > gpurun_out/pytest_var.log 2>&1
rc=$?; echo "variant reset tests ($VARLIB) rc=$rc"; tail -1 gpurun_out/pytest_var.log
[ $rc -le 1 ] || exit $rc
for r in 1 2; do
  for v in $VARS; do
    echo "== $v"
    DRL_LIB=tools/var_$v.so timeout -k 10 300 python tools/reset_rate.py --configs ${RR_CFGS:-c3,c4,c5} --variants wave --rounds 2 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
