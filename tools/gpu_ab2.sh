set -u
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 700 python -m pytest tests -m gpu -q -x -k "${PYTEST_K:-gpu or not gpu}" > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/ab.log
for c in ${CFGS:-c3 c4 c5}; do timeout -k 10 200 python tools/ab.py --config $c --rounds 5 --steps 100 --variants ${AB_VARIANTS} >> gpurun_out/ab.log 2>&1 || exit $?; done
grep -v amdgpu.ids gpurun_out/ab.log
