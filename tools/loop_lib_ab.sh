# A/B of library variants (tools/variants.py) on the graph-captured train loop: LIBS="cur xcd ..." CFGS="c3 c5"
mkdir -p gpurun_out
for r in 1 2; do for c in ${CFGS:-c3 c5}; do for l in ${LIBS:-cur}; do
timeout -k 10 200 python tools/loop_only.py --config $c --segments 5 --lib tools/var_$l.so >> gpurun_out/looplib${TAG:-}.log 2>&1 || exit $?
echo "$c $l" >> gpurun_out/looplib${TAG:-}.log
done; done; done
