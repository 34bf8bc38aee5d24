# Reset kernels on the GPU: parity tests (all reset variants), resets/s A/B,
# then PMC counters of the wave reset kernel (continuing resets only).
set -u
cd /root/repo
export TMPDIR=/tmp
if [ -z "${SKIP_TESTS:-}" ]; then
timeout -k 10 700 python -m pytest tests -m gpu -q -x ${PYTEST_K:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 400 python tools/reset_rate.py --configs ${RR_CFGS:-c3,c4,c5} --variants ${RR_VARIANTS:-wave,lane} ${RR_ARGS:-} > gpurun_out/reset_rate.log 2>&1
rc=$?; cat gpurun_out/reset_rate.log; [ $rc -eq 0 ] || exit $rc
for c in ${PMC_CFGS:-c5 c3}; do
  TAG=_reset_$c KREGEX=drl_reset_wave PYCMD="tools/reset_rate.py --configs $c --variants wave --rounds 1 --reps 2" bash tools/pmc_quick.sh > gpurun_out/pmc_reset_$c.log 2>&1 || exit $?
  echo "== $c"; grep -v amdgpu.ids gpurun_out/pmc_reset_$c.log
done
