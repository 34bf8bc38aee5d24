set -u
cd /root/repo
export TMPDIR=/tmp
OUT=gpurun_out/pmcq${TAG:-}; mkdir -p $OUT
A="--config ${CFG:-c3} --steps 20 --warmup 2 --no-cpu-baseline --no-reset-bench --no-pmc-traffic ${EXTRA:-}"
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU" "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA" ${EXTRA_PMC:-}; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $grp --kernel-include-regex ${KREGEX:-drl_step} -d $OUT/p$i -o run --output-format csv -- python3 ${PYCMD:-bench.py $A} > $OUT/p$i.log 2>&1
  rc=$?; if [ $rc -ne 0 ]; then echo "pass $i rc=$rc"; tail -3 $OUT/p$i.log; fi
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
OUT=$OUT python3 - <<'PY'
import csv, collections, glob, os
agg = collections.defaultdict(list)
for f in glob.glob(os.environ['OUT'] + '/p*/run_counter_collection.csv'):
    for r in csv.DictReader(open(f)):
        agg[r['Counter_Name']].append(float(r['Counter_Value']))
m = {k: sum(v)/len(v) for k, v in agg.items()}
w = m.get('SQ_WAVES', 1)
for k in sorted(m):
    print(f"{k:24s} {m[k]:16.1f}   per-wave {m[k]/w:10.1f}")
PY
