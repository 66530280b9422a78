# Same-box A/B of environment variants on ONE kernel plan: a tuning run records the plan table,
# then every variant runs bench.py from it (2 rounds, interleaved).
# bash tools/gpu/r6_ab.sh TAG "ENV_A" "ENV_B" ...   ("-" = no extra variables)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${1:-r6ab}
shift
mkdir -p $D
MILNCE_PLAN_TABLE=0 timeout -k 10 300 python bench.py --steps 5 --warmup 3 --save_plan $D/plan.json > $D/tune.log 2>&1 || { tail -20 $D/tune.log; exit 1; }
export MILNCE_PLAN_TABLE=$D/plan.json
for r in ${AB_ROUNDS:-1 2}; do
  for e in "$@"; do
    echo "== [$e] round $r"
    if [ "$e" = "-" ]; then timeout -k 10 300 python bench.py --steps 20 --warmup 5 | cut -c1-170
    else env $e timeout -k 10 300 python bench.py --steps 20 --warmup 5 | cut -c1-170; fi
  done
done > $D/bench.txt 2>&1
grep -v amdgpu.ids $D/bench.txt | sed -e 's/"metric.*"value": //' -e 's/, "unit.*ms_per_step"/ ms/' -e 's/, "hig.*//'
