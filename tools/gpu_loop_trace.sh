set -u
cd /root/repo
export TMPDIR=/tmp
for c in ${CFGS:-c3 c5}; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/looptr_$c -o run --output-format csv -- python3 tools/loop_only.py --config $c > gpurun_out/looptr_$c.log 2>&1 || exit $?
  echo "== $c"; tail -1 gpurun_out/looptr_$c.log | cut -c1-200
  python3 tools/trace_gaps.py gpurun_out/looptr_$c 404
done
