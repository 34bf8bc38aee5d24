#!/bin/bash
# rocprofv3 passes for the bench workload (run on the GPU box).
#   1. kernel trace + stats (per-kernel durations)
#   2..n. one PMC pass per counter group (no trace domains mixed with --pmc)
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/prof}
CFG=${CFG:-c3}
ARGS="--config $CFG --steps ${STEPS:-200} --warmup ${WARMUP:-20} --no-cpu-baseline --no-reset-bench --no-dqn --rollout-chunk 0 --loop-segments 0 --no-pmc-traffic --cached-steps 0"
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py $ARGS > $OUT/trace.log 2>&1 || exit $?
PMC_ARGS="--config $CFG --steps 20 --warmup 2 --no-cpu-baseline --no-reset-bench --no-dqn --rollout-chunk 0 --loop-segments 0 --no-pmc-traffic --cached-steps 0"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT" \
           "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE" ${EXTRA_PMC:-}; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-include-regex "${KREGEX:-drl_step|drl_refill}" -d $OUT/pmc$i -o run --output-format csv -- python3 bench.py $PMC_ARGS > $OUT/pmc$i.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "pmc pass $i ($grp) rc=$rc"; tail -5 $OUT/pmc$i.log; fi
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
ls -R $OUT | head -50
