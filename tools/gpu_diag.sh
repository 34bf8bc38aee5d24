#!/bin/bash
# Timing-only diagnostic builds (wrong results; never the product): where does
# a C3 drl_step launch spend its time?  base / no twist / no respawn rounds,
# each with streaming and cached observation stores and without observation.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
: > gpurun_out/var.log
for v in ${DIAG_VARS:-base notwist noresp}; do
  for c in ${DIAG_CFGS:-c3}; do
    timeout -k 10 200 python tools/ab.py --lib tools/var_$v.so --config $c --rounds ${AB_ROUNDS:-5} --steps 100 \
      --variants spec1_nt1,spec1,spec1_noobs >> gpurun_out/var.log 2>&1 || exit $?
  done
done
grep -v amdgpu.ids gpurun_out/var.log
