set -o pipefail
PYTEST_K="policy_code" tools/gpu.sh tests || exit 1
timeout -k 10 120 python tools/time_act.py --precision f32 --input code --synth > gpurun_out/act_code9.log 2>&1 || exit 1
timeout -k 10 120 python tools/time_act.py --precision f32 --input code >> gpurun_out/act_code9.log 2>&1 || exit 1
timeout -k 10 240 python3 tools/loop_only.py --input code >> gpurun_out/act_code9.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/act_code9.log
