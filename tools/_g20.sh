#!/bin/bash
# round 4: kernel breakdown of the C3 and C5 f32 train loops on the policy code (rocprofv3 kernel trace)
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/prof_loop
for c in c3 c5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_loop/$c -o run --output-format csv -- python3 tools/loop_only.py --config $c --segments 3 > gpurun_out/prof_loop/$c.log 2>&1 || exit 1
  tail -2 gpurun_out/prof_loop/$c.log
done
