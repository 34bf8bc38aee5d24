#!/bin/bash
# Interleave-free A/B of library variants (tools/variants.py) on the GPU.
# VARS="p8d1:c3 p8d2:c3 ..." (variant:config pairs)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for vc in $VARS; do
  v=${vc%%:*}; c=${vc##*:}
  timeout -k 10 200 python tools/ab.py --lib tools/var_$v.so --config $c --rounds ${AB_ROUNDS:-5} --steps ${AB_STEPS:-100} --variants ${AB_VARIANTS:-spec1,spec1_noobs} >> gpurun_out/var.log 2>&1 || exit $?
done
grep -v amdgpu.ids gpurun_out/var.log
