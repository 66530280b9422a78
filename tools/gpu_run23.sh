set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
for impl in 1 0; do
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VMEM -d gpurun_out/pmc/a$impl -o run --output-format csv -- python tools/pool_probe.py $impl > gpurun_out/pmc/a$impl.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE WRITE_SIZE TCP_TOTAL_CACHE_ACCESSES_sum -d gpurun_out/pmc/b$impl -o run --output-format csv -- python tools/pool_probe.py $impl > gpurun_out/pmc/b$impl.log 2>&1
done
for f in $(find gpurun_out/pmc -name "*counter_collection.csv"); do echo "== $f"; python - "$f" <<'PY'
import csv,sys
from collections import defaultdict
rows=list(csv.DictReader(open(sys.argv[1])))
agg=defaultdict(float); n=defaultdict(int)
for r in rows:
    if 'maxpool' not in r['Kernel_Name']: continue
    agg[r['Counter_Name']]+=float(r['Counter_Value']); n[r['Counter_Name']]+=1
for k,v in agg.items(): print(k, v/ max(1,n[k]) * (1 if k in ('FETCH_SIZE','WRITE_SIZE') else 1), 'dispatch-avg-rows', n[k])
PY
done
