set -u
cd /root/repo
export TMPDIR=/tmp
rm -f gpurun_out/var.log
for v in base nt base nt; do
  for c in c3 c5; do
    timeout -k 10 200 python tools/ab.py --lib tools/var_$v.so --config $c --rounds 4 --steps 100 --variants spec1 >> gpurun_out/var.log 2>&1 || exit 1
    timeout -k 10 200 python tools/roll_buffers.py $c tools/var_$v.so >> gpurun_out/var.log 2>&1 || exit 1
  done
done
grep -v amdgpu.ids gpurun_out/var.log
