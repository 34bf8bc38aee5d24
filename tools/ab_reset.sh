#!/bin/bash
# reset A/B over variant libraries (tools/variants.py builds): tests on each, then interleaved rates.
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # run LOG SECONDS CMD...
  local log=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "$log" 2>&1
  local rc=$?
  echo "[$log] rc=$rc"; grep -v amdgpu.ids "$log" | tail -${TAIL:-3}
  if [ $rc -gt 1 ]; then exit $rc; fi
}
for v in ${VARS:?}; do
  DRL_LIB=$PWD/tools/var_$v.so run gpurun_out/rsab_tests_$v.log 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q \
    --timeout 120 --timeout-method thread -x -k "reset_matches_oracle or reset_states_fixture"
done
for r in 1 2; do
  TAIL=3 run gpurun_out/rsab_rate_default_$r.log 200 python tools/reset_rate.py --configs ${CFGS:-c4,c5} --variants wave
  for v in $VARS; do
    TAIL=3 DRL_LIB=$PWD/tools/var_$v.so run gpurun_out/rsab_rate_${v}_$r.log 200 python tools/reset_rate.py \
      --configs ${CFGS:-c4,c5} --variants wave
  done
done
