set -u
cd /root/repo
bash tools/gpu_check.sh || exit $?
for c in c3 c5; do timeout -k 10 200 python tools/ab.py --config $c --rounds 5 --steps 100 >> gpurun_out/ab.log 2>&1 || exit $?; done
cat gpurun_out/ab.log
