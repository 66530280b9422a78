# Same-box A/B of tuner settings: every variant TUNES its own plan (MILNCE_PLAN_TABLE=0), rounds
# interleaved. bash tools/gpu/r6_tuned_ab.sh TAG "ENV_A" "ENV_B" ...   ("-" = no extra variables)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${1:-r6tab}
shift
mkdir -p $D
for r in ${AB_ROUNDS:-1 2}; do
  for e in "$@"; do
    echo "== [$e] round $r"
    if [ "$e" = "-" ]; then MILNCE_PLAN_TABLE=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 | cut -c1-170
    else env MILNCE_PLAN_TABLE=0 $e timeout -k 10 300 python bench.py --steps 20 --warmup 5 | cut -c1-170; fi
  done
done > $D/bench.txt 2>&1
grep -v amdgpu.ids $D/bench.txt | sed -e 's/"metric.*"value": //' -e 's/, "unit.*ms_per_step"/ ms/' -e 's/, "hig.*//'
