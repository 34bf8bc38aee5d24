set -u
cd /root/repo
bash tools/gpu_check.sh || exit $?
rm -f gpurun_out/ab.log
for c in c3 c4 c5; do timeout -k 10 200 python tools/ab.py --config $c --rounds 5 --steps 100 --variants ${AB_VARIANTS:-wpb1,wpb2,wpb4,wpb1_noobs} >> gpurun_out/ab.log 2>&1 || exit $?; done
cat gpurun_out/ab.log
