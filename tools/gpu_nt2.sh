set -u
cd /root/repo
export TMPDIR=/tmp
rm -f gpurun_out/var.log
for v in nt cached nt cached; do
  for c in c3 c5; do
    timeout -k 10 200 python tools/loop_only.py --lib tools/var_$v.so --config $c --segments 3 >> gpurun_out/var.log 2>&1 || exit 1
  done
done
grep -v amdgpu.ids gpurun_out/var.log
