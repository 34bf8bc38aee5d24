#!/bin/bash
# PMC instruction / wait counts of diagnostic variants (tools/pmc_quick.sh per variant).
set -u
cd "$(dirname "$0")/.."
for v in ${DIAG_VARS:-base noresp}; do
  DRL_LIB=$PWD/tools/var_$v.so TAG=_$v EXTRA="--obs-k ${OBSK:-0} --no-dqn --rollout-chunk 0 --loop-segments 0 --no-pmc-traffic --cached-steps 0" \
    bash tools/pmc_quick.sh > gpurun_out/pmc_$v.txt 2>&1 || exit $?
  echo "== $v"; cat gpurun_out/pmc_$v.txt
done
