# Record several kernel-plan tables (independent tuning runs) and bench each from its table on the
# same box, twice, interleaved; the fastest table is the one to ship (tuning timings are noisy).
# bash tools/gpu/plan_pick.sh TAG [N]
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${1:-planpick}
N=${2:-3}
mkdir -p $D
for i in $(seq 1 $N); do
  MILNCE_PLAN_TABLE=0 timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --save_plan $D/t$i.json > $D/tune$i.log 2>&1 || { tail -5 $D/tune$i.log; exit 1; }
  echo "table $i: $(grep -o '"plan_hash": "[0-9a-f]*"' $D/tune$i.log)"
done
for r in 1 2; do
  for i in $(seq 1 $N); do
    MILNCE_PLAN_TABLE=$D/t$i.json timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $D/b$i-$r.log 2>&1 || { tail -5 $D/b$i-$r.log; exit 1; }
    echo "table $i round $r: $(grep -o '"value": [0-9.]*\|"plan_hash": "[0-9a-f]*"\|"table_status": "[a-z]*"' $D/b$i-$r.log | tr '\n' ' ')"
  done
done
