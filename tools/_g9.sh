#!/bin/bash
# round 4: code act v4 -- parity, timing vs v3, stamps, per-wave PMC of the v4 act at C3
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "code or qnet or dqn" > gpurun_out/g9_tests.log 2>&1; rc=$?
tail -5 gpurun_out/g9_tests.log
[ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  timeout -k 10 120 python tools/time_act.py --precision f32 --input code >> gpurun_out/g9_act.log 2>&1 || exit 1
  DRL_QN_CODE=3 timeout -k 10 120 python tools/time_act.py --precision f32 --input code >> gpurun_out/g9_act.log 2>&1 || exit 1
done
timeout -k 10 120 python tools/time_act.py --precision f32 --input code --envs 131072 >> gpurun_out/g9_act.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/g9_act.log
timeout -k 10 120 python tools/time_act.py --lib tools/var_qst4.so --precision f32 --input code --stamps > gpurun_out/g9_stamps.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/g9_stamps.log
KREGEX=drl_qnet_act_code4 PYCMD="tools/time_act.py --precision f32 --input code --iters 20" TAG=_g9act \
  EXTRA_PMC="SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT" bash tools/gpu.sh pmc > gpurun_out/g9_pmc.log 2>&1 || exit 1
tail -30 gpurun_out/g9_pmc.log
