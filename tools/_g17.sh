#!/bin/bash
# round 4: where the C5 step's 139.5 us go now that it is off the bandwidth wall -- per-phase stamps (C5, C3),
# per-wave PMC of the C5 step loop
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 300 python tools/stamps.py --prebuilt --config c5 --steps 8 > gpurun_out/g17_stamps_c5.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/g17_stamps_c5.log
timeout -k 10 300 python tools/stamps.py --prebuilt --config c3 --steps 8 > gpurun_out/g17_stamps_c3.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/g17_stamps_c3.log
CFG=c5 KREGEX=drl_step TAG=_g17c5 EXTRA_PMC="SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS" bash tools/gpu.sh pmc > gpurun_out/g17_pmc.log 2>&1 || exit 1
tail -28 gpurun_out/g17_pmc.log
