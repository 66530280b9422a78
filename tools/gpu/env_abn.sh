# Same-box comparison of several environments (2 rounds each):
# bash tools/gpu/env_abn.sh TAG "ENV_A" "ENV_B" ...   ("-" = no extra variables)
set -e
cd $GRAFT_REPO_ROOT
D=gpurun_out/${1:-envabn}
shift
mkdir -p $D
for r in 1 2; do
  for e in "$@"; do
    echo "== [$e] round $r"
    if [ "$e" = "-" ]; then timeout -k 10 300 python bench.py --steps 20 --warmup 5 | cut -c1-170
    else env $e timeout -k 10 300 python bench.py --steps 20 --warmup 5 | cut -c1-170; fi
  done
done > $D/bench.txt 2>&1
grep -v amdgpu.ids $D/bench.txt | sed -e 's/"metric.*"value": //' -e 's/, "unit.*ms_per_step"/ ms/' -e 's/, "hig.*//'
