# A/B of TrainSegment(synth_branch=True) (synthetic actions beside the learner) against the fused act
mkdir -p gpurun_out
for c in c5 c3; do for r in 1 2; do
timeout -k 10 200 python tools/loop_only.py --config $c --segments 5 --synth-branch >> gpurun_out/loopsyn.log 2>&1 || exit $?
echo "$c synth-branch" >> gpurun_out/loopsyn.log
timeout -k 10 200 python tools/loop_only.py --config $c --segments 5 >> gpurun_out/loopsyn.log 2>&1 || exit $?
echo "$c fused" >> gpurun_out/loopsyn.log
done; done
