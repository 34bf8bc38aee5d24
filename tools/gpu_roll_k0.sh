set -u
cd /root/repo
export TMPDIR=/tmp
for k in 0 1; do
  timeout -k 10 300 python bench.py --config c3 --obs-k $k --no-cpu-baseline --no-dqn --loop-segments 0 --no-reset-bench > gpurun_out/b_k$k.json 2>/dev/null || exit 1
  python3 -c "
import json; d=json.loads(open('gpurun_out/b_k$k.json').read().strip().splitlines()[-1])
print('K=$k step', round(d['roofline']['avg_launch_us'],2), 'us/launch; rollout', round(d['rollout']['ms_per_step']*1e3,2), 'us/step')"
done
