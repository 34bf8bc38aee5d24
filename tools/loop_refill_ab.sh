for c in c3 c5; do for r in 1 2; do
timeout -k 10 200 python tools/loop_only.py --config $c --segments 5 --refill-branch >> gpurun_out/loopab_r06i.log 2>&1 || exit $?
echo "$c branch" >> gpurun_out/loopab_r06i.log
timeout -k 10 200 python tools/loop_only.py --config $c --segments 5 >> gpurun_out/loopab_r06i.log 2>&1 || exit $?
echo "$c inline" >> gpurun_out/loopab_r06i.log
done; done
