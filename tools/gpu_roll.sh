set -u
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 700 python -m pytest tests -m gpu -q -x -k "${PYTEST_K:-gpu or not gpu}" > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for c in ${CFGS:-c3 c5}; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --loop-segments 0 --no-dqn > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err || { tail -5 gpurun_out/bench_$c.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/bench_$c.json').read().strip().splitlines()[-1])
print('$c step', round(d['value']/1e9,3), 'G/s', round(d['roofline']['avg_launch_us'],2), 'us; rollout', json.dumps(d['rollout']))"
done
