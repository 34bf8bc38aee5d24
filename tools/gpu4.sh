set -u
cd /root/repo
bash tools/gpu_check.sh || exit $?
rm -f gpurun_out/ab.log gpurun_out/stamps.log gpurun_out/scan.log
for c in c3 c4 c5; do timeout -k 10 200 python tools/ab.py --config $c --rounds 5 --steps 100 --variants ${AB_VARIANTS:-wpb1,wpb1_wide0,wpb1_noobs} >> gpurun_out/ab.log 2>&1 || exit $?; done
timeout -k 10 300 python tools/scan_envs.py --config c3 --obs 1 --envs 8192,49152,65536,131072,262144 > gpurun_out/scan.log 2>&1 || exit $?
for c in c3 c5; do timeout -k 10 200 python tools/stamps.py --config $c >> gpurun_out/stamps.log 2>&1 || exit $?; done
bash tools/pmc_quick.sh > gpurun_out/pmcq.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/ab.log gpurun_out/scan.log gpurun_out/stamps.log gpurun_out/pmcq.log
