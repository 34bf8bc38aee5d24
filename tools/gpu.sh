#!/bin/bash
# tools/gpu.sh — the one GPU-box driver script (run through gpurun).
#
#   tools/gpu.sh TASK [TASK ...]
#
# Tasks run in order; each GPU step has its own time limit (timeout -k 10)
# and the script stops at the first crash, abort or time limit (pytest's rc 1
# = test failures only: the later tasks still run).  Output goes under
# gpurun_out/ (copy what should be kept to profiles/).
#
#   tests     pytest -m gpu                    PYTEST_K (-k expression), PYTEST_ARGS, T_TESTS (s)
#   smoke     __graft_entry__.smoke()
#   bench     python bench.py $BENCH_ARGS      -> gpurun_out/bench$TAG.json
#   configs   bench lines of CFGS (c4 c5)      -> gpurun_out/bench_<cfg>$TAG.json
#   profile   rocprofv3 kernel trace + stats, then one PMC pass per counter
#             group, of the bench step loop    CFG, STEPS, KREGEX, EXTRA_PMC
#   pmc       instruction / wait / byte PMC passes of PYCMD (default: the
#             bench step loop) summarised per wave   CFG, KREGEX, PYCMD, TAG
#   reset     tools/reset_rate.py              RR_CFGS, RR_VARIANTS, RR_ARGS
#   act       tools/time_act.py                ACT_ARGS
#   ab        tools/ab.py per variant library  VARS="name:cfg ...", AB_ROUNDS, AB_STEPS, AB_VARIANTS
#   loopprof  rocprofv3 kernel trace + stats of the graph-captured train loop (tools/loop_only.py) per config
#             of LCFGS (c3 c5)                 -> gpurun_out/loopprof_<cfg>$TAG/
#   run       any python command               CMD="tools/x.py ...", T_RUN (s), TAG
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-}

step() {  # step NAME SECONDS LOG CMD...: run one GPU step, stop the script on a crash / limit
  local name=$1 secs=$2 log=$3; shift 3
  timeout -k 10 "$secs" "$@" > "$log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; grep -v amdgpu.ids "$log" | tail -${TAIL:-4}
  if [ $rc -ne 0 ] && { [ "$name" != tests ] || [ $rc -ne 1 ]; }; then exit $rc; fi
}

pmc_passes() {  # pmc_passes OUT KREGEX GROUP... -- CMD...: one rocprofv3 --pmc run per counter group
  local out=$1 kre=$2; shift 2
  local groups=()
  while [ "$1" != "--" ]; do groups+=("$1"); shift; done
  shift
  local i=0
  for grp in "${groups[@]}"; do
    i=$((i+1))
    step "pmc$i" 240 "$out/pmc$i.log" rocprofv3 --pmc $grp --kernel-include-regex "$kre" -d "$out/pmc$i" -o run \
      --output-format csv -- "$@"
  done
}

LOOP_ONLY="--no-cpu-baseline --no-reset-bench --no-dqn --rollout-chunk 0 --loop-segments 0 --no-pmc-traffic --cached-steps 0 --c5-envs 0"

for task in "$@"; do
  case $task in
    tests)
      # PYTEST_K: a -k expression (spaces kept); PYTEST_ARGS="-k <expr>" is read the same way
      K=${PYTEST_K:-}; PA=${PYTEST_ARGS:-}
      if [ -z "$K" ] && [ "${PA#-k }" != "$PA" ]; then K=${PA#-k }; PA=; fi
      step tests "${T_TESTS:-900}" gpurun_out/pytest_gpu$TAG.log \
        python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread ${K:+-k "$K"} $PA ;;
    smoke)
      step smoke 300 gpurun_out/smoke$TAG.log python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)
      step bench "${T_BENCH:-600}" gpurun_out/bench$TAG.json python bench.py ${BENCH_ARGS:-} ;;
    configs)
      for c in ${CFGS:-c4 c5}; do
        step "bench-$c" 400 gpurun_out/bench_$c$TAG.json python bench.py --config $c --no-cpu-baseline --c5-envs 0 \
          ${BENCH_ARGS:-}
      done ;;
    profile)
      OUT=gpurun_out/prof$TAG; mkdir -p $OUT
      A="--config ${CFG:-c3} --steps ${STEPS:-200} --warmup 20 $LOOP_ONLY ${EXTRA:-}"
      step trace 300 $OUT/trace.log rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
        python3 bench.py $A
      pmc_passes $OUT "${KREGEX:-drl_step|drl_refill}" "FETCH_SIZE" "WRITE_SIZE" \
        "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
        "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT" \
        "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE" ${EXTRA_PMC:-} -- \
        python3 bench.py --config ${CFG:-c3} --steps 20 --warmup 2 $LOOP_ONLY ${EXTRA:-} ;;
    pmc)
      OUT=gpurun_out/pmcq$TAG; mkdir -p $OUT
      pmc_passes $OUT "${KREGEX:-drl_step}" \
        "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH" \
        "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU" \
        "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA" \
        ${EXTRA_PMC:-} -- python3 ${PYCMD:-bench.py --config ${CFG:-c3} --steps 20 --warmup 2 $LOOP_ONLY}
      python3 tools/summarize_profile.py --per-wave "$OUT" | tee $OUT/summary.txt ;;
    reset)
      step reset 400 gpurun_out/reset_rate$TAG.log python tools/reset_rate.py --configs ${RR_CFGS:-c3,c4,c5} \
        --variants ${RR_VARIANTS:-wave} ${RR_ARGS:-} ;;
    act)
      step act 300 gpurun_out/time_act$TAG.log python tools/time_act.py ${ACT_ARGS:-} ;;
    ab)
      for vc in ${VARS:?VARS=\"name:cfg ...\"}; do
        v=${vc%%:*}; c=${vc##*:}
        step "ab-$v" 300 gpurun_out/ab_$v$TAG.log python tools/ab.py --lib tools/var_$v.so --config $c \
          --rounds ${AB_ROUNDS:-5} --steps ${AB_STEPS:-100} --variants ${AB_VARIANTS:-spec1,spec1_noobs}
      done ;;
    loopprof)
      for c in ${LCFGS:-c3 c5}; do
        OUT=gpurun_out/loopprof_$c$TAG; mkdir -p $OUT
        step "loopprof-$c" 300 $OUT/trace.log rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv \
          -- python3 tools/loop_only.py --config $c --segments ${LSEG:-3} ${LARGS:-}
      done ;;
    run)
      step run "${T_RUN:-300}" gpurun_out/run$TAG.log python ${CMD:?CMD=\"tools/x.py ...\"} ;;
    *)
      echo "unknown task $task"; exit 2 ;;
  esac
done
echo done
