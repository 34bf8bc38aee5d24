# Round-end evidence, second half (after tools/gpu_check.sh ran in another
# call): C4/C5 bench lines, the parallel-branch loop line, and the rocprofv3
# trace + PMC passes of C3.
set -u
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in c4 c5; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err || exit $?
done
timeout -k 10 300 python bench.py --parallel-loop --no-cpu-baseline --no-reset-bench --rollout-chunk 0 > gpurun_out/bench_parloop.json 2> gpurun_out/bench_parloop.err || exit $?
OUT=gpurun_out/prof CFG=c3 bash tools/profile.sh > gpurun_out/profile.log 2>&1 || { tail -5 gpurun_out/profile.log; exit 1; }
echo done
