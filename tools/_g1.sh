set -o pipefail
export TMPDIR=/tmp
PYTEST_K="policy_code or train_segment or replay" tools/gpu.sh tests || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/loopprof_code3 -o run --output-format csv -- python3 tools/loop_only.py --input code > gpurun_out/loop_code3.log 2>&1 || exit 1
grep us_per_step gpurun_out/loop_code3.log
