D=gpurun_out/$1
mkdir -p $D && export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_express.py -x -q > $D/t.log 2>&1; rc=$?; tail -3 $D/t.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python tools/expressbench.py || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/kt -o kt --output-format csv -- python3 tools/expressbench.py --reps 10 > $D/kt.log 2>&1 || exit 1
python - $D <<'PY'
import csv, collections, sys
rows = list(csv.DictReader(open(sys.argv[1] + '/kt/kt_kernel_trace.csv')))
d = collections.defaultdict(list)
for r in rows:
    d[r['Kernel_Name'][:40]].append((int(r['End_Timestamp'])-int(r['Start_Timestamp']), r['VGPR_Count'], r['SGPR_Count'], r['LDS_Block_Size']))
for k,v in d.items(): print(k, len(v), round(sum(x[0] for x in v)/len(v)/1e3, 2), 'us', v[0][1:])
PY
