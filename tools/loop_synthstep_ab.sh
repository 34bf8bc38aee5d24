# A/B of TrainSegment(synth_in_step=True) (drl_step_code_replay_synth) against the act's synthetic columns
mkdir -p gpurun_out
for c in c5 c3; do for r in 1 2; do
timeout -k 10 200 python tools/loop_only.py --config $c --segments 5 >> gpurun_out/loopsynstep.log 2>&1 || exit $?
echo "$c synth-in-step" >> gpurun_out/loopsynstep.log
timeout -k 10 200 python tools/loop_only.py --config $c --segments 5 --synth-in-act >> gpurun_out/loopsynstep.log 2>&1 || exit $?
echo "$c synth-in-act" >> gpurun_out/loopsynstep.log
done; done
