#!/bin/bash
# The parity core on the in-tree library, then an interleave-free A/B of
# variant builds (VARS="name:cfg ...", tools/var_<name>.so), results appended
# to gpurun_out/var.log as they come.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -q -x --timeout 300 --timeout-method thread \
  ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_core.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_core.log
[ $rc -le 1 ] || exit $rc
: > gpurun_out/var.log
for vc in $VARS; do
  v=${vc%%:*}; c=${vc##*:}
  timeout -k 10 200 python tools/ab.py --lib tools/var_$v.so --config $c --rounds ${AB_ROUNDS:-5} --steps 100 \
    --variants ${AB_VARIANTS:-spec1_nt1,spec1,spec1_noobs} >> gpurun_out/var.log 2>&1 || exit $?
done
grep -v amdgpu.ids gpurun_out/var.log
